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

// Diagnostic phase stamps (separate build with -DJWV_STAMPS only): thread 0
// of block 0 records s_memrealtime (100 MHz) at numbered points.
#ifdef JWV_STAMPS
extern __device__ unsigned long long jwv_stamps[64];
extern __device__ unsigned long long jwv_clocks[64];
#define JWV_STAMP(k)                                                        \
  do {                                                                      \
    if (threadIdx.x == 0 && blockIdx.x == 0) {                              \
      jwv_stamps[(k)] = __builtin_amdgcn_s_memrealtime();                   \
      jwv_clocks[(k)] = __builtin_amdgcn_s_memtime();                       \
    }                                                                       \
  } while (0)
#else
#define JWV_STAMP(k) \
  do {               \
  } while (0)
#endif

namespace jwv {

constexpr int kMaxTaps = 64;

struct AxisView {
  int64_t s_outer;  // stride between signals (in doubles)
  int64_t s_pk;     // stride between packets inside a signal
  int64_t s_len;    // stride between consecutive samples of one signal
  int32_t pk;       // packets per signal (1 = plain signals)
  int32_t pad_;
};

// Segments of one AncientEgyptianDecomposition varlen launch (aed_kernels.hpp),
// passed by value in the kernel arguments.
struct VarSegs {
  static constexpr int kMax = 32;
  int count;
  int n[kMax];     // segment length (a power of two)
  int h0[kMax];    // FWT fwd: level input size; FWT/WPT rev: first synthesis size
  int nlev[kMax];  // levels (0 = copy)
  int64_t off[kMax];
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

// LDS-DMA of 16 B per lane issued through inline asm: the compiler's waitcnt
// analysis does not see it, so barriers elsewhere in the kernel do not get a
// conservative vmcnt(0) (which would make every wave drain its global
// stores).  The issuing wave must `s_waitcnt vmcnt(0)` itself (asm) before a
// barrier that publishes the data.  lds_dst must be wave-uniform.
__device__ __forceinline__ void dma16_asm(const void* g, double* lds_dst) {
  // wave-uniform by contract; readfirstlane lets the compiler keep it in an
  // SGPR even when it cannot prove the uniformity itself
  const unsigned lds_addr = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)((__attribute__((address_space(3))) double*)lds_dst));
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :
      : "v"(g), "s"(lds_addr)
      : "memory", "m0");
}

// Workgroup barrier that orders LDS only.  __syncthreads() is a workgroup
// fence on every address space: the compiler puts `s_waitcnt vmcnt(0)` in
// front of it, so each barrier would wait until the wave's global stores
// (detail coefficients already on their way to HBM) are acknowledged.  None
// of these kernels reads global memory written in the same launch, so an
// LDS-scoped fence (lgkmcnt only) is the complete requirement.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Wait for this wave's LDS-DMA loads, then a workgroup barrier: after it
// every wave sees every other wave's DMA'd rows in LDS.
__device__ __forceinline__ void dma_fence_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
}

// Load a window of W rows (C doubles each; row e from global src + rowoff(e),
// columns contiguous) into lds[e*C + c].
//  dma = 1: LDS-DMA, 16 B per lane (global_load_lds_dwordx4): every request in
//           flight at once, no VGPRs.  Requires src + rowoff(e) 16-B aligned for
//           even e (C=1) / every e (C>=2), C even or 1, and that for C=1 the
//           pair (e, e+1) is contiguous in global memory; reads one row past W
//           when W is odd (LDS must have room; global row must exist).
//  dma = 0: plain loads, all issued before the first LDS write (MAXU bound).
// Columns c0+c >= inner are zero-filled (register path) or skipped (dma path
// is only used when the slab is complete).  Caller issues dma_fence_barrier().
template <int C, int NT, int MAXU, typename RowOff>
__device__ __forceinline__ void load_window(double* lds, const double* __restrict__ src, int W,
                                            bool dma, int c0, int inner, RowOff rowoff) {
  const int tid = threadIdx.x;
  if (dma) {
    const int lane = tid & 63, wave = tid >> 6;
    constexpr int UPR = C == 1 ? 1 : C / 2;  // 16-B units per row (C >= 2)
    const int nunits = C == 1 ? (W + 1) >> 1 : W * UPR;
    for (int u0 = wave * 64; u0 < nunits; u0 += NT) {
      const int u = u0 + lane;
      if (u < nunits) {
        const double* g = C == 1 ? src + rowoff(2 * u) : src + rowoff(u / UPR) + (u % UPR) * 2;
        __builtin_amdgcn_global_load_lds(
            (const void*)g, (__attribute__((address_space(3))) void*)(lds + 2 * u0), 16, 0, 0);
      }
    }
    return;
  }
  const int total = W * C;
  double v[MAXU];
#pragma unroll
  for (int r = 0; r < MAXU; ++r) {
    const int q = tid + r * NT;
    v[r] = 0.0;
    if (q < total) {
      const int e = q / C, c = q % C;
      if (c0 + c < inner) v[r] = src[rowoff(e) + c];
    }
  }
#pragma unroll
  for (int r = 0; r < MAXU; ++r) {
    const int q = tid + r * NT;
    if (q < total) lds[q] = v[r];
  }
}

// Pair-slot iteration for a level with np pairs: slot r of this thread is
// pair p = tid + r*NT.  f(r, p, valid) must only store when `valid`.
// When R = ceil(np/NT) <= 4 the slots run branch-free (invalid slots compute
// on a clamped pair index) so the independent LDS reads / FP64 chains of all
// slots overlap; larger R keeps the MAXP-unrolled guarded form.
template <int R, int NT, typename F>
__device__ __forceinline__ void pairs_flat(int np, F& f) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int p0 = (int)threadIdx.x + r * NT;
    const bool v = p0 < np;
    f(r, v ? p0 : np - 1, v);
  }
}
template <int MAXP, int NT, typename F>
__device__ __forceinline__ void for_pairs(int np, F&& f) {
  const int R = (np + NT - 1) / NT;
  if (R <= 1) { pairs_flat<1, NT>(np, f); return; }
  if constexpr (MAXP >= 2) if (R == 2) { pairs_flat<2, NT>(np, f); return; }
  if constexpr (MAXP >= 3) if (R == 3) { pairs_flat<3, NT>(np, f); return; }
  if constexpr (MAXP >= 4) if (R == 4) { pairs_flat<4, NT>(np, f); return; }
#pragma unroll
  for (int r = 0; r < MAXP; ++r) {
    const int p0 = (int)threadIdx.x + r * NT;
    if (p0 < np) f(r, p0, true);
  }
}

// Wave-local LDS ordering: a wave's LDS ops execute in program order, so only
// the compiler has to be kept from moving them across this point.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// threadIdx.x through an empty asm: computations derived from it cannot be
// hoisted above this point.  The level functions of the compile-time-geometry
// kernels take their lane index this way; otherwise the compiler hoists every
// level's slot addresses to kernel entry and keeps them live (WPT L=16: ~200
// VGPRs instead of ~100).
__device__ __forceinline__ int opaque_tid() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// ---------------------------------------------------------------------------
// In-launch hand-off between workgroups (chained kernels, fwt1_chain.hpp).
// gfx950 L1s are per CU and never refreshed by other CUs' stores; the XCD L2s
// are kept coherent for hipMalloc memory only for write-through data.  The
// protocol (MI355X_MICROARCH.md, inter-workgroup visibility):
//   producer: handed-off bytes stored write-through (sc1) -> every storing
//             wave `s_waitcnt vmcnt(0)` -> workgroup barrier -> ONE lane
//             signals with an agent-scope atomic (counter add or flag store);
//   consumer: ONE lane polls relaxed (sc1 loads) or reads its add's return
//             value -> that lane's agent-scope acquire (buffer_inv sc1) ->
//             `s_waitcnt vmcnt(0)` -> workgroup barrier -> plain / LDS-DMA loads.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// Two adjacent doubles (16-B aligned p): one 16-B store, or two sc1 stores.
template <bool WT>
__device__ __forceinline__ void st2(double* p, double a, double b) {
  if constexpr (WT) {
    st_wt(p, a);
    st_wt(p + 1, b);
  } else {
    *reinterpret_cast<double2*>(p) = make_double2(a, b);
  }
}
// Cache policy of the 16-B output stores of the full-length passes (kernel
// argument, wave-uniform): 0 plain; 1 sc1 (write-through: the line leaves the
// XCD L2 with the store, so the launch ends with no dirty lines to write back
// and the next dependent launch starts without that write-back,
// MI355X_MICROARCH.md "boundary"); 2 nt.  base must be wave-uniform (it
// becomes the buffer descriptor); off in doubles, < 2^28.
typedef unsigned int jwv_u32x4 __attribute__((ext_vector_type(4)));
// Tile of this block in an XCD-chunked walk: consecutive blockIdx go to
// different XCDs, so XCD x takes the contiguous chunk x of the nblk tiles
// (its L2 keeps the halo rows); sp bit 2 walks every chunk last-to-first
// (the next pass then starts on the most recently written, MALL-resident
// end).  Clears the bit (st2_pol reads sp & 3).
// sp bit 3 selects the grouped walk instead: XCD x takes groups of G = 2^(sp
// bits 8..12) consecutive tiles and the 8 XCDs work side by side, so the grid
// sweeps memory as ONE front (the chunked walk runs 8 fronts exactly 1/8 of
// the array apart, which cold HBM serves more slowly).
__device__ __forceinline__ int tile_order(int nblk, int& sp) {
  const bool desc = (sp & 4) != 0;
  const bool grouped = (sp & 8) != 0;
  const int gs = (sp >> 8) & 31;
  sp &= 3;
  const int b = blockIdx.x;
  if (grouped && (nblk & ((8 << gs) - 1)) == 0) {
    const int x = b & 7, j = b >> 3;
    return ((j >> gs) << (gs + 3)) + (x << gs) + (j & ((1 << gs) - 1));
  }
  if ((nblk & 7) == 0) {
    const int per = nblk >> 3, j = b >> 3;
    return (b & 7) * per + (desc ? per - 1 - j : j);
  }
  return desc ? nblk - 1 - b : b;
}

__device__ __forceinline__ void st2_pol(double* base, int off, double a, double b, int sp) {
  sp &= 3;
  if (sp == 0) {
    *reinterpret_cast<double2*>(base + off) = make_double2(a, b);
    return;
  }
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7ffffff0, 0x00020000);
  const jwv_u32x4 v = __builtin_bit_cast(jwv_u32x4, make_double2(a, b));
  if (sp == 1) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off * 8, 0, 16);
  else __builtin_amdgcn_raw_buffer_store_b128(v, rs, off * 8, 0, 2);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ unsigned atomic_add_agent(unsigned* p, unsigned v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_agent(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned load_agent(const unsigned* p) {
  return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<unsigned long long*>(
                                                          const_cast<double*>(p)),
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// Window of W handed-off doubles (lds[e] = src[rowoff(e)]) read with sc1
// loads (L1 bypass) into registers, then LDS: with the producer's sc1 stores
// and the signal read before, no acquire is needed.  All MAXU loads are in
// flight at once.  Caller issues lds_barrier().
template <int NT, int MAXU, typename RowOff>
__device__ __forceinline__ void load_window_wt(double* lds, const double* src, int W,
                                               RowOff rowoff) {
  const int tid = threadIdx.x;
  double v[MAXU];
#pragma unroll
  for (int r = 0; r < MAXU; ++r) {
    const int e = tid + r * NT;
    if (e < W) v[r] = ld_wt(src + rowoff(e));
  }
#pragma unroll
  for (int r = 0; r < MAXU; ++r) {
    const int e = tid + r * NT;
    if (e < W) lds[e] = v[r];
  }
}
// Acquire for the whole workgroup: lane 0 invalidates this CU's L1, its wait
// holds the barrier until the invalidate has completed.
__device__ __forceinline__ void block_acquire() {
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}
// Bounded relaxed poll of one flag (one lane).  Never spins forever: after
// `lim` polls (host default 2^22) it records a timeout and gives up (results
// are then wrong; every host entry reads the timeout word and fails with
// JWV_ERR_DEVICE; the grid still drains).
__device__ __forceinline__ void poll_eq(const unsigned* f, unsigned v, unsigned* tmo,
                                        unsigned lim) {
  for (unsigned i = 0; i < lim; ++i) {
    if (load_agent(f) == v) return;
    __builtin_amdgcn_s_sleep(2);
  }
  store_agent(tmo, 1u);
}

// Wave-wide bounded poll until every flag f[0, n) equals v (one wave).
__device__ __forceinline__ void poll_all(const unsigned* f, int n, unsigned v, unsigned* tmo,
                                         unsigned lim) {
  const int lane = threadIdx.x & 63;
  for (unsigned i = 0; i < lim; ++i) {
    bool ok = true;
    for (int k = lane; k < n; k += 64) ok = ok && load_agent(f + k) == v;
    if (__all(ok)) return;
    __builtin_amdgcn_s_sleep(2);
  }
  if (lane == 0) store_agent(tmo, 1u);
}

// 16-B LDS read at a 16-B aligned address the compiler cannot prove aligned
// on its own (offsets built from runtime lane indices): without the
// assumption it splits the access into ds_read2_b64 (8 cycles, and 2-way
// bank-conflicted at a 16-B lane stride) instead of one ds_read_b128.
__device__ __forceinline__ double2 ld16(const double* p) {
  return *reinterpret_cast<const double2*>(__builtin_assume_aligned(p, 16));
}
__device__ __forceinline__ void st16(double* p, double a, double b) {
  *reinterpret_cast<double2*>(__builtin_assume_aligned(p, 16)) = make_double2(a, b);
}

// Materialise two results here: stops the compiler from sinking their
// computation into later exec-masked stores, where two independent FP64
// accumulation chains would run one after the other instead of interleaved
// (latency-bound tail levels: ~2x per level).
__device__ __forceinline__ void pin2(double& a, double& b) { asm volatile("" : "+v"(a), "+v"(b)); }

template <bool FMA>
__device__ __forceinline__ double mac(double acc, double a, double b) {
  if constexpr (FMA) {
    return __builtin_fma(a, b, acc);
  } else {
    return acc + a * b;  // two roundings (-ffp-contract=off)
  }
}

}  // namespace jwv
