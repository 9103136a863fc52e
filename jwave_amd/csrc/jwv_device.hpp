// jwv_device.hpp — shared device-side definitions for the gfx950 kernels.
//
// Data model ("axis view").  Every FWT/WPT kernel transforms signals that lie
// along the middle axis of a row-major [outer][len][inner] block:
//   element (o, i, c) lives at  base + off(o) + i*s_len + c      (inner stride 1)
//   off(o) = (o / pk) * s_outer + (o % pk) * s_pk
// where pk splits the outer index into (signal, packet) so that WPT passes can
// address the packets of a signal as independent signals.  1-D batches use
// inner = 1; 2-D columns use outer = 1, inner = cols; 3-D axes use all three.
//
// Math modes.  EXACT evaluates `acc + a*b` as two rounded operations in the
// reference's summation order (Wavelet.java:236-303, MODWTTransform.java:
// 677-716) — results are bit-identical to the JVM.  FMA uses fused
// multiply-add (one rounding), same order; ~2x fewer FP64 instructions.
// The translation unit is compiled with -ffp-contract=off so the compiler never
// fuses on its own.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace jwv {

constexpr int kMaxTaps = 64;

struct AxisView {
  int64_t s_outer;  // stride between signals (in doubles)
  int64_t s_pk;     // stride between packets inside a signal
  int64_t s_len;    // stride between consecutive samples of one signal
  int32_t pk;       // packets per signal (1 = plain signals)
  int32_t pad_;
};

__device__ __forceinline__ int64_t view_base(const AxisView& v, int64_t o) {
  if (v.pk == 1) return o * v.s_outer;
  return (o / v.pk) * v.s_outer + (o % v.pk) * v.s_pk;
}

// Filter bank passed by value in the kernel-argument segment: the compiler
// keeps the taps in SGPRs (VALU FP64 ops take one scalar 64-bit operand).
template <int L>
struct FwdTaps {
  double lo[L];
  double hi[L];
};
template <int L>
struct RevTaps {
  double lo_r[L];
  double hi_r[L];
};
// Runtime-L bank (L <= kMaxTaps) for odd / long / scaled wavelets.
struct AnyTaps {
  double lo[kMaxTaps];
  double hi[kMaxTaps];
  double lo_r[kMaxTaps];
  double hi_r[kMaxTaps];
  double scale;
  int32_t L;
  int32_t pad_;
};

template <bool FMA>
__device__ __forceinline__ double mac(double acc, double a, double b) {
  if constexpr (FMA) {
    return __builtin_fma(a, b, acc);
  } else {
    return acc + a * b;  // two roundings (-ffp-contract=off)
  }
}

}  // namespace jwv
