// fwt_colres.hpp — forward resident pass over 8-column slabs with
// compile-time geometry: the column tail of the 2-D forward transform
// (BasicTransform.forward(double[][]), BasicTransform.java:369-395; config 3:
// the [1024][8192] approximation block, 10 levels per column).  Same math,
// per-output order and outputs as fwt_fwd_res (fwt_kernels.hpp, through
// fwd_pair: Wavelet.java:236-260), so EXACT results stay bit-identical.
//
// What the compile-time form changes against the generic resident kernel
// (runtime h, per-tap (2i + j) & (h - 1) index math, one pair per lane, rows
// of 8 doubles: 2-way bank conflicts; SQ r06: FP64 48% of VALU, conflicts 46%
// of LDS cycles):
//  * a lane computes a couple (pairs 2k, 2k+1 of one column) from L+2 rows;
//    rows are stored at a pitch of 10 doubles (8 columns + 2 pad), so the
//    32 lanes of a ds_read_b64 group (8 columns x 4 couples, rows 4k+j) hit
//    bank segments 20(4k+j) mod 64 = 16k + 20j: conflict-free;
//  * every tap is an immediate offset from one per-lane base (interior
//    couples); only the couples whose window wraps (the last (L+2)/4 or so
//    per column) take the masked index;
//  * levels recurse at compile time; levels with at most 64 work items run
//    on wave 0 with wave-local LDS ordering (no block barriers).
// LDS-DMA lands the rows in the padded image directly (pad units read a
// valid address and are never used).
#pragma once
#include "fwt_kernels.hpp"

namespace jwv {

constexpr int kCresP = 10;  // LDS row pitch (doubles)

template <int L, int NT, int H, bool FMA, int h>
struct CresLevel {
  static_assert(h >= 2 && (h & (h - 1)) == 0, "power-of-two levels");
  static constexpr int P = h / 2;                   // pairs per column
  static constexpr bool kCouple = h >= 4;
  static constexpr int NI = (kCouple ? P / 2 : P) * 8;  // work items (couples or pairs)
  static constexpr bool kWave = NI <= 64;           // wave 0 alone
  static constexpr int R = kWave ? 1 : (NI + NT - 1) / NT;
  // first couple whose rows 4k .. 4k+L+1 wrap past h-1
  static constexpr int KW = h >= L + 2 ? (h - L - 2) / 4 + 1 : 0;

  // details of level h -> rows [P, h) of the column block; approximations
  // stay in LDS rows [0, P).  nlev: levels left including this one.
  __device__ __forceinline__ static void run(const FwdTaps<L>& tp, double* lds,
                                             double* __restrict__ y, int64_t sl, int nlev) {
    const int tid = opaque_tid();
    if (kWave && tid >= 64) {
      // the other waves skip to the final barrier below
    } else {
      double av[R][2];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int w = tid + r * NT;
        const bool ok = kWave ? w < NI : ((r + 1) * NT <= NI || w < NI);
        const int wc = ok ? w : NI - 1;
        const int c = wc & 7, k = wc >> 3;
        double a0, d0, a1 = 0.0, d1 = 0.0;
        if constexpr (kCouple) {
          double x[L + 2];
          if (k < KW) {  // interior: immediate offsets from one base
            const double* b = lds + 4 * k * kCresP + c;
#pragma unroll
            for (int j = 0; j < L + 2; ++j) x[j] = b[j * kCresP];
          } else {
#pragma unroll
            for (int j = 0; j < L + 2; ++j) x[j] = lds[((4 * k + j) & (h - 1)) * kCresP + c];
          }
          fwd_pair<L, FMA>(tp, [&](int j) { return x[j]; }, a0, d0);
          fwd_pair<L, FMA>(tp, [&](int j) { return x[j + 2]; }, a1, d1);
        } else {
          fwd_pair<L, FMA>(tp, [&](int j) { return lds[((2 * k + j) & (h - 1)) * kCresP + c]; },
                           a0, d0);
        }
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(d0), "+v"(d1) :: "memory");  // slot boundary
        if (ok) {
          const int i = kCouple ? 2 * k : k;
          y[(int64_t)(P + i) * sl + c] = d0;
          if constexpr (kCouple) y[(int64_t)(P + i + 1) * sl + c] = d1;
        }
        av[r][0] = a0;
        av[r][1] = a1;
      }
      if constexpr (kWave) wave_lds_sync(); else lds_barrier();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int w = tid + r * NT;
        const bool ok = kWave ? w < NI : ((r + 1) * NT <= NI || w < NI);
        if (ok) {
          const int c = w & 7, k = w >> 3;
          const int i = kCouple ? 2 * k : k;
          lds[i * kCresP + c] = av[r][0];
          if constexpr (kCouple) lds[(i + 1) * kCresP + c] = av[r][1];
        }
      }
    }
    if constexpr (kWave) {
      if (tid < 64) wave_lds_sync();
    } else {
      lds_barrier();
    }
    if constexpr (h > 2)
      if (nlev > 1) CresLevel<L, NT, H, FMA, h / 2>::run(tp, lds, y, sl, nlev - 1);
  }
};

// Grid: one block per 8-column slab (res_slab_block pairs the two halves of
// each 128-B row line on one XCD).  src rows [0, H) of the slab (row stride
// sv.s_len), nlev levels from H; details and the final approximations to dst
// as fwt_fwd_res writes them.  Needs inner % 8 == 0 and 16-B aligned rows.
template <int L, int NT, int H, bool FMA>
__global__ __launch_bounds__(NT) void fwt_fwd_cres8(const double* __restrict__ src, AxisView sv,
                                                    double* __restrict__ dst, AxisView dv, int nlev,
                                                    int inner, FwdTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  static_assert(kCresP == 10, "pad units: 4 data + 1 pad per row");
  const int ncb = inner >> 3;
  const int64_t bs = res_slab_block<8>(blockIdx.x);
  const int64_t o = bs / ncb;
  const int c0 = (int)(bs % ncb) * 8;
  const double* s = src + view_base(sv, o) + c0;
  double* y = dst + view_base(dv, o) + c0;
  // rows x (4 data + 1 pad) 16-B units, contiguous in LDS: unit u -> row u / 5
  {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int nunits = H * 5;
    for (int u0 = wave * 64; u0 < nunits; u0 += NT) {
      const int u = u0 + lane;
      if (u < nunits) {
        const int row = u / 5, sub = u - 5 * (u / 5);
        const double* g = s + (int64_t)row * sv.s_len + 2 * (sub < 4 ? sub : 0);
        __builtin_amdgcn_global_load_lds((const void*)g,
                                         (__attribute__((address_space(3))) void*)(lds + 2 * u0),
                                         16, 0, 0);
      }
    }
  }
  dma_fence_barrier();
  CresLevel<L, NT, H, FMA, H>::run(tp, lds, y, dv.s_len, nlev);
  lds_barrier();  // wave 0's last levels
  // the final approximations: rows [0, H >> nlev)
  const int hend = H >> nlev;
  for (int q = threadIdx.x; q < hend * 8; q += NT) {
    const int i = q >> 3, c = q & 7;
    y[(int64_t)i * dv.s_len + c] = lds[i * kCresP + c];
  }
}


// ------------------------------------------------------------------ reverse
// Reverse column tail with compile-time geometry (config 3: 8-column slabs,
// levels of output size 2 .. HTOP = 1024; BasicTransform.reverse(double[][])
// columns, Wavelet.reverse, Wavelet.java:277-303, through rev_pair /
// rev_pair_rot_t / rev_small_cH exactly as rev_small_levels takes them:
// EXACT results are bit-identical to fwt_rev_col16).
// Rows at a dense pitch of 8 doubles: work item w = (pair m = w >> 3, column
// c = w & 7), so the 32 lanes of a ds_read_b64 group read 4 consecutive rows
// = 256 contiguous bytes (conflict-free) at every tap.  Interior pairs
// (m >= Q-1) read a[m-q], d[m-q] at immediate offsets; the array-head pairs
// (m < Q-1) all sit in wave 0's first slot, which alone takes the rotated
// form (rev_small_levels runs the rotated form in slot 0 of every column's
// wave).  Levels with at most 64 items run on wave 0 with wave-local
// ordering; a level's outputs overwrite rows [0, hh) after its reads.
// Element (index i, column c) of the level arrays at lds[i * SI + c * SC]
// (dense rows of 8 columns: SI = 8, SC = 1).  The same levels over blocks of
// 8 rows (SI = 1, SC = a padded row pitch) measured no faster than the
// wave-per-row tail (r06, profiles/r06/ab_rev_tails_ct.txt) and are not built.
template <int L, int NT, bool FMA, int hh, int HTOP, int SI = 8, int SC = 1>
struct RevCresLevel {
  static constexpr int half = hh / 2, Q = L / 2;
  static constexpr int NI = half * 8;
  static constexpr bool kWave = NI <= 64;
  static constexpr int R = kWave ? 1 : (NI + NT - 1) / NT;
  __device__ __forceinline__ static void run(const RevTaps<L>& tp, const double* tl, double* lds,
                                             int h0) {
    if (hh >= h0) {  // block-uniform: the levels below the input size are skipped
      // the first block-wide level after wave 0's levels: publish them
      if constexpr (!kWave && hh > 2 && 2 * hh <= 64)
        if (hh > h0) lds_barrier();
      const int tid = opaque_tid();
      if (!kWave || tid < 64) {
        double xe[R], xo[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int w = tid + r * NT;
          const int wc = w < NI ? w : NI - 1;
          const int c = wc & 7, m = wc >> 3;
          if constexpr (hh < L) {
            rev_small_cH<L, FMA, hh>(tp, lds + c * SC, lds + half * SI + c * SC, SI, m, xe[r],
                                     xo[r]);
          } else {
            // wave-uniform: does this wave's slot hold array-head pairs?
            const int mb = (__builtin_amdgcn_readfirstlane(tid & ~63) + r * NT) >> 3;
            if (mb < Q - 1) {
              constexpr int hm = half - 1;
              rev_pair_rot_t<L, FMA>(
                  tl, [=](int q) { return lds[((m - q) & hm) * SI + c * SC]; },
                  [=](int q) { return lds[(half + ((m - q) & hm)) * SI + c * SC]; },
                  m < Q - 1 ? m : Q - 1, xe[r], xo[r]);
            } else {
              const double* A = lds + m * SI + c * SC;
              double av[Q], dv[Q];
#pragma unroll
              for (int q = 0; q < Q; ++q) {
                av[q] = A[-SI * q];
                dv[q] = A[half * SI - SI * q];
              }
              rev_pair<L, FMA>(tp, av, dv, -1, xe[r], xo[r]);
            }
          }
          pin2(xe[r], xo[r]);
        }
        if constexpr (kWave) wave_lds_sync(); else lds_barrier();
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int w = tid + r * NT;
          if ((r + 1) * NT <= NI || w < NI) {
            const int c = w & 7, m = w >> 3;
            lds[(2 * m) * SI + c * SC] = xe[r];
            lds[(2 * m + 1) * SI + c * SC] = xo[r];
          }
        }
      } else if constexpr (!kWave) {
        lds_barrier();
      }
      if constexpr (kWave) {
        if (tid < 64) wave_lds_sync();
      } else {
        lds_barrier();
      }
    }
    if constexpr (hh < HTOP) RevCresLevel<L, NT, FMA, 2 * hh, HTOP, SI, SC>::run(tp, tl, lds, h0);
  }
};

// Grid: one block per 8-column slab (res_slab_block pairs the halves of each
// 128-B line on one XCD).  Rows [0, HTOP) of the slab from src (coefficient
// prefix), levels of output size h0 .. HTOP, rows [0, HTOP) to dst.  Needs
// inner % 8 == 0 and 16-B aligned rows (the host checks).
template <int L, int NT, int HTOP, bool FMA>
__global__ __launch_bounds__(NT) void fwt_rev_cres8(const double* __restrict__ src, AxisView sv,
                                                    double* __restrict__ dst, AxisView dv, int h0,
                                                    int inner, RevTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ __attribute__((aligned(16))) double tl[2 * L];
  stage_rev_taps<L>(tp, tl);
  const int ncb = inner >> 3;
  const int64_t bs = res_slab_block<8>(blockIdx.x);
  const int64_t o = bs / ncb;
  const int c0 = (int)(bs % ncb) * 8;
  const double* s = src + view_base(sv, o) + c0;
  double* y = dst + view_base(dv, o) + c0;
  {  // rows x 4 16-B units, dense: unit u -> row u >> 2
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int nunits = HTOP * 4;
    for (int u0 = wave * 64; u0 < nunits; u0 += NT) {
      const int u = u0 + lane;
      const double* g = s + (int64_t)(u >> 2) * sv.s_len + 2 * (u & 3);
      __builtin_amdgcn_global_load_lds((const void*)g,
                                       (__attribute__((address_space(3))) void*)(lds + 2 * u0),
                                       16, 0, 0);
    }
  }
  dma_fence_barrier();  // also publishes tl
  RevCresLevel<L, NT, FMA, 2, HTOP>::run(tp, tl, lds, h0);
  for (int u = threadIdx.x; u < HTOP * 4; u += NT) {
    const int r = u >> 2, c = 2 * (u & 3);
    *reinterpret_cast<double2*>(y + (int64_t)r * dv.s_len + c) =
        *reinterpret_cast<const double2*>(lds + 8 * r + c);
  }
}


}  // namespace jwv
