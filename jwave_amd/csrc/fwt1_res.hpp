// fwt1_res.hpp — resident FWT kernels for contiguous signals (C = 1, stride
// 1, 16-B aligned rows) with a compiled-in tap count.  One block holds a
// whole level input (<= CAP samples) in LDS and runs the remaining levels:
// the deep tail of a long 1-D signal (one block, latency-bound) and batches of
// rows (one block per row).
//
// Latency rules for the tail, where one wave often works alone:
//  * every level issues all of its LDS reads before its first FP64 op (one
//    LDS round trip per level, not one per tap);
//  * the reverse array-head pairs (Wavelet.java:284-296 order, wave 0 only)
//    take their runtime-rotated order from LDS (inputs and an LDS copy of the
//    taps); interior pairs read their inputs without wrapping;
//  * barriers are LDS-only (lds_barrier), so the detail stores of the forward
//    levels stay in flight across them.
// Math and summation order are those of fwt_fwd_res / fwt_rev_res.
#pragma once
#include "fwt_kernels.hpp"

namespace jwv {

// a, d of pair p of a level of size h (mask msk = h-1) from LDS, wrap by mask.
template <int L, bool FMA>
__device__ __forceinline__ void fwd_pair_wrap(const FwdTaps<L>& tp, const double* in, int p,
                                              int msk, double& a, double& d) {
  double x[L];
#pragma unroll
  for (int j = 0; j < L; ++j) x[j] = in[(2 * p + j) & msk];
  fwd_pair<L, FMA>(tp, [&](int j) { return x[j]; }, a, d);
  pin2(a, d);
}

// Synthesis pair m of a level of size h >= L: a = lds[0, half), d =
// lds[half, h).  Interior pairs (m >= Q-1) sum q descending from registers;
// the array-head pairs (m < Q-1, lanes of wave 0) take rev_pair_head's order
// through rev_pair_rot_t (inputs and taps tl from LDS, no register select).
// rot (wave-uniform): every lane of the wave takes the rotated form (r = m
// for head pairs, Q-1 = the interior order otherwise), so a wave holding
// head pairs runs one path instead of both under divergence (the
// latency-bound single-wave levels, and wave 0 of the block-wide ones).
template <int L, bool FMA>
__device__ __forceinline__ void rev_pair_wrap(const RevTaps<L>& tp, const double* tl,
                                              const double* lds, int half, int m, double& xe,
                                              double& xo, bool rot = false) {
  constexpr int Q = (L + 1) / 2;
  const int hm = half - 1;
  if (rot) {
    rev_pair_rot_t<L, FMA>(tl, [=](int q) { return lds[(m - q) & hm]; },
                           [=](int q) { return lds[half + ((m - q) & hm)]; },
                           m < Q - 1 ? m : Q - 1, xe, xo);
  } else if (m >= Q - 1) {
    double av[Q], dv[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      av[q] = lds[m - q];
      dv[q] = lds[half + m - q];
    }
    rev_pair<L, FMA>(tp, av, dv, -1, xe, xo);  // A[-q * -1] = av[q] = a[m - q]
  } else {
    rev_pair_rot_t<L, FMA>(tl, [=](int q) { return lds[(m - q) & hm]; },
                           [=](int q) { return lds[half + ((m - q) & hm)]; }, m, xe, xo);
  }
  pin2(xe, xo);
}

// ====================================================================
// Forward, resident, C = 1.  src row: level input of length h0 (DMA-able);
// dst row: coefficient array (details of level size h at dst[h/2, h), final
// approximation at dst[0, h_end)).
// ====================================================================
// Levels of the resident forward on a level input already in lds[0, h0):
// details to y[h/2, h) per level, the final approximation to y[0, h_end).
template <int L, int NT, int CAP, bool FMA>
__device__ __forceinline__ void fwd_res1_levels(double* lds, double* __restrict__ y, int h0,
                                                int nlev, const FwdTaps<L>& tp) {
  constexpr int RM = CAP / 2 / NT > 0 ? CAP / 2 / NT : 1;
  const int tid = threadIdx.x;
  int h = h0, lev = 0;
  // block-wide levels: np = h/2 > 64 pairs, a power of two
  for (; lev < nlev && (h >> 1) > 64; ++lev, h >>= 1) {
    JWV_STAMP(2 + lev);
    const int half = h >> 1, msk = h - 1;
    double av[RM];
    auto slot = [&](int r) {
      const int p = tid + r * NT;
      double a, d;
      fwd_pair_wrap<L, FMA>(tp, lds, p, msk, a, d);
      av[r] = a;
      y[half + p] = d;
    };
    const int R = half / NT;  // 0 when half < NT
    if (R <= 1) {
      if (tid < half) slot(0);
    } else if (R == 2) {
#pragma unroll
      for (int r = 0; r < 2; ++r) slot(r);
    } else if (R == 4) {
#pragma unroll
      for (int r = 0; r < (RM < 4 ? RM : 4); ++r) slot(r);
    } else if (R == 8) {
#pragma unroll
      for (int r = 0; r < (RM < 8 ? RM : 8); ++r) slot(r);
    } else {
#pragma unroll
      for (int r = 0; r < (RM < 16 ? RM : 16); ++r) slot(r);
    }
    lds_barrier();
    if (R <= 1) {
      if (tid < half) lds[tid] = av[0];
    } else {
#pragma unroll
      for (int r = 0; r < RM; ++r)
        if (r < R) lds[tid + r * NT] = av[r];
    }
    lds_barrier();
  }
  // small levels: wave 0 alone (no block barriers)
  if (lev < nlev) {
    if (tid < 64) {
      int hh = h;
      for (int lv = lev; lv < nlev; ++lv, hh >>= 1) {
        JWV_STAMP(2 + lv);
        const int half = hh >> 1;
        const bool v = tid < half;
        const int p = v ? tid : half - 1;
        double a, d;
        fwd_pair_wrap<L, FMA>(tp, lds, p, hh - 1, a, d);
        if (v) y[half + p] = d;
        wave_lds_sync();
        if (v) lds[p] = a;
        wave_lds_sync();
      }
    }
    h >>= (nlev - lev);
    lds_barrier();
  }
  JWV_STAMP(40);
  for (int q = tid; q < h; q += NT) y[q] = lds[q];
  JWV_STAMP(42);
}

template <int L, int NT, int CAP, bool FMA>
__global__ __launch_bounds__(NT) void fwt_fwd_res1(const double* __restrict__ src, int64_t s_src,
                                                   double* __restrict__ dst, int64_t s_dst, int h0,
                                                   int nlev, FwdTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int64_t o = blockIdx.x;
  JWV_STAMP(0);
  load_window<1, NT, (CAP + NT - 1) / NT>(lds, src + o * s_src, h0, true, 0, 1,
                                          [&](int e) { return (int64_t)e; });
  dma_fence_barrier();
  JWV_STAMP(1);
  fwd_res1_levels<L, NT, CAP, FMA>(lds, dst + o * s_dst, h0, nlev, tp);
}

// ====================================================================
// Reverse, resident, C = 1.  src row: coefficient prefix [0, htop) with
// htop = h0 << (nlev-1) (h0 = first synthesis level size); dst row: [0, htop).
// ====================================================================
// Levels of the resident reverse on the coefficient prefix already in
// lds[0, htop), htop = h0 << (nlev-1); the result is left in lds[0, htop)
// (the caller stores it; ends with a block barrier).
template <int L, int NT, int CAP, bool FMA>
__device__ __forceinline__ void rev_res1_levels(double* lds, int h0, int nlev,
                                                const RevTaps<L>& tp) {
  constexpr int RM = CAP / 2 / NT > 0 ? CAP / 2 / NT : 1;
  const int tid = threadIdx.x;
  __shared__ __attribute__((aligned(16))) double tl[2 * L];
  stage_rev_taps<L>(tp, tl);
  lds_barrier();
  int h = h0, lev = 0;
  if (nlev > 0 && (h >> 1) <= 64) {  // small levels: wave 0 alone
    if (tid < 64) {
      int hh = h;
      for (; lev < nlev && (hh >> 1) <= 64; ++lev, hh <<= 1) {
        JWV_STAMP(2 + lev);
        const int half = hh >> 1;
        const bool v = tid < half;
        const int m = v ? tid : half - 1;
        double xe, xo;
        if (hh < L) {
          constexpr int HM = L / 2;
          double av[HM], dv[HM];
#pragma unroll
          for (int i = 0; i < HM; ++i) {
            av[i] = i < half ? lds[i] : 0.0;
            dv[i] = i < half ? lds[half + i] : 0.0;
          }
          rev_small_c<L, FMA>(tp, av, dv, 1, hh, m, xe, xo);  // h < L: compile-time h
        } else {
          rev_pair_wrap<L, FMA>(tp, tl, lds, half, m, xe, xo, true);
        }
        wave_lds_sync();
        if (v) *reinterpret_cast<double2*>(lds + 2 * m) = make_double2(xe, xo);
        wave_lds_sync();
      }
      h = hh;
    }
    // the other waves catch up on (h, lev); wave 0 has already advanced
    while ((h >> 1) <= 64 && lev < nlev) { ++lev; h <<= 1; }
    lds_barrier();
  }
  for (; lev < nlev; ++lev, h <<= 1) {
    JWV_STAMP(2 + lev);
    const int half = h >> 1;
    double xe[RM], xo[RM];
    auto slot = [&](int r) {
      rev_pair_wrap<L, FMA>(tp, tl, lds, half, tid + r * NT, xe[r], xo[r], r == 0 && tid < 64);
    };
    const int R = half / NT;
    if (R <= 1) {
      if (tid < half) slot(0);
    } else if (R == 2) {
#pragma unroll
      for (int r = 0; r < 2; ++r) slot(r);
    } else if (R == 4) {
#pragma unroll
      for (int r = 0; r < (RM < 4 ? RM : 4); ++r) slot(r);
    } else if (R == 8) {
#pragma unroll
      for (int r = 0; r < (RM < 8 ? RM : 8); ++r) slot(r);
    } else {
#pragma unroll
      for (int r = 0; r < (RM < 16 ? RM : 16); ++r) slot(r);
    }
    lds_barrier();
    if (R <= 1) {
      if (tid < half) *reinterpret_cast<double2*>(lds + 2 * tid) = make_double2(xe[0], xo[0]);
    } else {
#pragma unroll
      for (int r = 0; r < RM; ++r)
        if (r < R) {
          const int m = tid + r * NT;
          *reinterpret_cast<double2*>(lds + 2 * m) = make_double2(xe[r], xo[r]);
        }
    }
    lds_barrier();
  }
}

template <int L, int NT, int CAP, bool FMA>
__global__ __launch_bounds__(NT) void fwt_rev_res1(const double* __restrict__ src, int64_t s_src,
                                                   double* __restrict__ dst, int64_t s_dst, int h0,
                                                   int nlev, RevTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int64_t o = blockIdx.x;
  const int tid = threadIdx.x;
  const int htop = nlev > 0 ? (h0 << (nlev - 1)) : h0;
  JWV_STAMP(0);
  load_window<1, NT, (CAP + NT - 1) / NT>(lds, src + o * s_src, htop, true, 0, 1,
                                          [&](int e) { return (int64_t)e; });
  dma_fence_barrier();
  JWV_STAMP(1);
  rev_res1_levels<L, NT, CAP, FMA>(lds, h0, nlev, tp);
  JWV_STAMP(40);
  double* __restrict__ y = dst + o * s_dst;
  for (int q = 2 * tid; q < htop; q += 2 * NT)
    *reinterpret_cast<double2*>(y + q) = *reinterpret_cast<const double2*>(lds + q);
  JWV_STAMP(42);
}

}  // namespace jwv
