// modwt_nonfinite.hpp — MODWT outputs on non-finite input, as Java's DIRECT
// loops give them.
//
// circularConvolve / circularConvolveAdjoint (MODWTTransform.java:677-716)
// multiply EVERY tap of the upsampled filter, the 2^(j-1)-1 zeros between the
// L real taps included (upsample, :618-630).  For finite samples x*0.0 = +-0.0
// and adding it to a sum that started at +0.0 changes nothing, which is why
// the kernels sum only the L real taps.  For x = +-inf or NaN, x*0.0 is NaN:
// Java's output is NaN wherever the output's window (forward: positions
// n-m, inverse: n+m, m = 0 .. C = (L-1)*2^(j-1)) holds a non-finite value at
// a zero tap (m mod 2^(j-1) != 0).  Everywhere else the sparse sum is Java's
// sum bit for bit (a non-finite value at a real tap reaches the sparse sum
// through the same product).
//
// How the kernels reproduce it without slowing the finite case:
//  * Detection.  A non-finite value at any position of a level's window makes
//    some output of that level non-finite (each window position is a real tap
//    of some output of the tile, because a tile has at least 2^(j-1) outputs,
//    and x*c is non-finite for non-finite x and any c, 0 included), and a
//    non-finite value at window position q of level j is again one at q in
//    level j+1 (tap m = 0).  So a tile pass whose LAST level's outputs are all
//    finite read only finite values at every level: its sparse results are
//    Java's.  The fast pass checks just those outputs (register values it
//    stores anyway; one v_cmp_class per output of one level).
//  * Repair.  A block whose check fired runs its tile (or chunk) again in the
//    slow form: the same sums, plus, per level, the range [lo, hi] of
//    non-finite window positions (one LDS min/max per lane that saw one), and
//    for every output whose window meets that range a scan of the zero taps
//    in it; a hit stores NaN (W_j and V_j / the inverse's V_{j-1}).  Every
//    store of the repair comes from the lane that made the fast store to the
//    same address, so it lands last.  Overflow to inf in a finite signal also
//    fires the check; the repair then changes nothing it need not.
// NaN payloads are not reproduced (Java gives the JVM's NaN, the GPU its
// canonical quiet NaN); tests compare NaN positions.
#pragma once
#include "jwv_device.hpp"

namespace jwv {

// +-inf, signalling or quiet NaN: v_cmp_class_f64 with the class mask
// sNaN | qNaN | -inf | +inf
__device__ __forceinline__ bool nonfinite(double x) { return __builtin_amdgcn_class(x, 0x207); }
__device__ __forceinline__ double mod_nan() { return __builtin_nan(""); }

// Waves per SIMD the fast pass reaches when LDS is what limits it (the repair
// pass shares the kernel's register allocation; __launch_bounds__ with this
// keeps the repair from lowering the fast pass's occupancy).
constexpr int mod_lds_waves(long lds_bytes, int nt, int cap = 8) {
  const long blocks = (160 * 1024) / (lds_bytes + 64);
  const long w = blocks * (nt / 64) / 4;
  return w < 1 ? 1 : (w > cap ? cap : (int)w);
}

// Block-shared words: the end-of-pass "any non-finite" flag and the
// non-finite position ranges of up to two windows (V, W).
struct ModNf {
  int any[2];
  int lo[2];
  int hi[2];
};

__device__ __forceinline__ void nf_init(ModNf& f) {
  if (threadIdx.x == 0) {
    f.any[0] = f.any[1] = 0;
    f.lo[0] = f.lo[1] = 0x7fffffff;
    f.hi[0] = f.hi[1] = -0x7fffffff;
  }
}

// Block-wide OR of a per-lane flag (every lane must call it), for the gen-th
// time (gen = 1, 2, ...; nf_init before the pass's first barrier).  Slots
// alternate by gen, so a lane that runs ahead to the next call never
// overwrites the slot a slower lane is about to read.
__device__ __forceinline__ bool nf_any(ModNf& f, bool bad, int gen = 1) {
  if (bad) f.any[gen & 1] = gen;
  lds_barrier();
  return __builtin_amdgcn_readfirstlane(f.any[gen & 1]) == gen;
}

// Non-finite position range of NW windows over positions [q0, q1):
// win(k, q) reads position q of window k.  Every lane must call it; the
// result is block-uniform (lo > hi: none).
template <int NW, int NT, class Win>
__device__ __forceinline__ void nf_window(ModNf& f, int q0, int q1, Win win, int (&lo)[2],
                                          int (&hi)[2]) {
  lds_barrier();  // earlier readers of the range words are done
  if (threadIdx.x == 0)
    for (int k = 0; k < NW; ++k) {
      f.lo[k] = 0x7fffffff;
      f.hi[k] = -0x7fffffff;
    }
  lds_barrier();
  for (int k = 0; k < NW; ++k) {
    int a = 0x7fffffff, b = -0x7fffffff;
    for (int q = q0 + (int)threadIdx.x; q < q1; q += NT)
      if (nonfinite(win(k, q))) {
        a = q < a ? q : a;
        b = q;
      }
    if (a <= b) {
      atomicMin(&f.lo[k], a);
      atomicMax(&f.hi[k], b);
    }
  }
  lds_barrier();
  for (int k = 0; k < NW; ++k) {
    lo[k] = __builtin_amdgcn_readfirstlane(f.lo[k]);
    hi[k] = __builtin_amdgcn_readfirstlane(f.hi[k]);
  }
}

// Forward output at position e reads window positions e - m, m = 0 .. C:
// true if a zero tap (m mod st != 0) holds a non-finite value.  Only [lo, hi]
// can hold one.
template <class At>
__device__ __forceinline__ bool nf_fwd_zero(At at, int e, int st, int C, int lo, int hi) {
  if (st == 1) return false;
  const int a = e - C > lo ? e - C : lo, b = e < hi ? e : hi;
  for (int q = a; q <= b; ++q)
    if (((e - q) & (st - 1)) != 0 && nonfinite(at(q))) return true;
  return false;
}
// Inverse (adjoint) output at position p reads p + m, m = 0 .. C.
template <class At>
__device__ __forceinline__ bool nf_inv_zero(At at, int p, int st, int C, int lo, int hi) {
  if (st == 1) return false;
  const int a = p > lo ? p : lo, b = p + C < hi ? p + C : hi;
  for (int q = a; q <= b; ++q)
    if (((q - p) & (st - 1)) != 0 && nonfinite(at(q))) return true;
  return false;
}

}  // namespace jwv
