// fwt1_row.hpp — batches of short contiguous rows (the resident tails of
// the 2-D row passes, config 3: 8192 rows of 512 / 1024 samples, and any
// batch of >= 64 rows up to kSmallH samples): one WAVE per row.
//
// The block-per-row resident kernels (fwt_fwd_res1 / fwt_rev_res1) spend
// these rows' deep levels on wave 0 while the other waves of the block wait
// at barriers; here a wave owns its row outright (no block barrier at all,
// wave-local LDS ordering only), kSmallRows rows per block, so a CU runs
// many of these latency chains side by side.  Per level, lane l takes pairs
// l, l + 64, ... (all reads of the level before any write: in place).
// Math and summation order are those of the resident kernels' wave-0 levels
// (fwd_res1_levels / rev_res1_levels, fwt1_res.hpp; Wavelet.java:236-303):
// EXACT results are bit-identical.
//
// Measured and not kept (round 3): one block per 8192-sample row with every
// level resident (64 KB of LDS per row; persistent double-buffered or two
// blocks per CU, 512 / 1024 threads): forward 274-288 us, reverse 372-406 us
// on config 3 against 221 + 44 / 296 + 88 us for the tile pass + resident
// tail it was meant to replace; the levels run at 1-2 blocks per CU with
// their barrier chains exposed (SQ: VALU ~54% of SIMD cycles).
#pragma once
#include "fwt1_res.hpp"

namespace jwv {

constexpr int kSmallRows = 2, kSmallH = 1024;

// One wave's forward levels over its row / column lds[0, h0) (h0 <= kSmallH):
// per level, lane l takes pairs l, l + 64, ...; all reads of a level before
// any write.  Details go to y[half + p].  Returns the final approximation
// length.
template <int L, bool FMA>
__device__ __forceinline__ int fwd_small_levels(const FwdTaps<L>& tp, double* lds, int lane, int h0,
                                                int nlev, double* __restrict__ y) {
  constexpr int RM = kSmallH / 128;  // pairs per lane at most
  int h = h0;
  for (int lv = 0; lv < nlev; ++lv, h >>= 1) {
    const int half = h >> 1, msk = h - 1;
    if (half <= 64) {
      const bool v = lane < half;
      const int p = v ? lane : half - 1;
      double a, d;
      fwd_pair_wrap<L, FMA>(tp, lds, p, msk, a, d);
      if (v) y[half + p] = d;
      wave_lds_sync();
      if (v) lds[p] = a;
    } else {
      double av[RM];
      auto slot = [&](int r) {
        const int p = lane + 64 * r;
        double a, d;
        fwd_pair_wrap<L, FMA>(tp, lds, p, msk, a, d);
        av[r] = a;
        y[half + p] = d;
      };
      const int R = half >> 6;  // 2, 4, ..., RM
#pragma unroll
      for (int r = 0; r < RM; ++r)
        if (r < R) slot(r);
      wave_lds_sync();
#pragma unroll
      for (int r = 0; r < RM; ++r)
        if (r < R) lds[lane + 64 * r] = av[r];
    }
    wave_lds_sync();
  }
  return h;
}

// Forward: rows of h0 <= kSmallH samples (src; read whole first) -> nlev
// levels -> dst (details per level, then the final approximation).
template <int L, bool FMA>
__global__ __launch_bounds__(64 * kSmallRows) void fwt_fwd_small1(const double* src, int64_t s_src,
                                                                   double* dst, int64_t s_dst,
                                                                   int h0, int nlev,
                                                                   int64_t nrows, FwdTaps<L> tp) {
  __shared__ __attribute__((aligned(16))) double sm[kSmallRows][kSmallH];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t row = (int64_t)blockIdx.x * kSmallRows + w;
  if (row >= nrows) return;  // wave-uniform; no block barrier below
  double* lds = sm[w];
  const double* s = src + row * s_src;
  double* __restrict__ y = dst + row * s_dst;
  for (int q = 2 * lane; q < h0; q += 128)
    *reinterpret_cast<double2*>(lds + q) = *reinterpret_cast<const double2*>(s + q);
  wave_lds_sync();
  const int h = fwd_small_levels<L, FMA>(tp, lds, lane, h0, nlev, y);
  for (int q = lane; q < h; q += 64) y[q] = lds[q];
}

// One wave's reverse levels of output size h0 .. h0 << (nlev-1) <= kSmallH,
// in place over lds (the coefficient prefix): all reads of a level before
// any write.  tl: the block's staged taps (stage_rev_taps).
template <int L, bool FMA>
__device__ __forceinline__ void rev_small_levels(const RevTaps<L>& tp, const double* tl, double* lds,
                                                 int lane, int h0, int nlev) {
  constexpr int RM = kSmallH / 128;
  int hh = h0;
  for (int lev = 0; lev < nlev; ++lev, hh <<= 1) {
    const int half = hh >> 1;
    if (half <= 64) {
      const bool v = lane < half;
      const int m = v ? lane : half - 1;
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
    } else {
      double xe[RM], xo[RM];
      const int R = half >> 6;
      // slot 0 holds the array-head pairs: the whole slot takes the rotated
      // form (r = m for head pairs, the interior order otherwise)
#pragma unroll
      for (int r = 0; r < RM; ++r)
        if (r < R) rev_pair_wrap<L, FMA>(tp, tl, lds, half, lane + 64 * r, xe[r], xo[r], r == 0);
      wave_lds_sync();
#pragma unroll
      for (int r = 0; r < RM; ++r)
        if (r < R)
          *reinterpret_cast<double2*>(lds + 2 * (lane + 64 * r)) = make_double2(xe[r], xo[r]);
    }
    wave_lds_sync();
  }
}

// Reverse: levels of output size h0 .. htop = h0 << (nlev-1) <= kSmallH of
// rows whose coefficient prefix [0, htop) is read from src; the level-htop
// outputs go to dst[0, htop).
template <int L, bool FMA>
__global__ __launch_bounds__(64 * kSmallRows) void fwt_rev_small1(const double* src, int64_t s_src,
                                                                   double* dst, int64_t s_dst,
                                                                   int h0, int nlev,
                                                                   int64_t nrows, RevTaps<L> tp) {
  __shared__ __attribute__((aligned(16))) double sm[kSmallRows][kSmallH];
  __shared__ __attribute__((aligned(16))) double tl[2 * L];
  stage_rev_taps<L>(tp, tl);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t row = (int64_t)blockIdx.x * kSmallRows + w;
  if (row >= nrows) return;
  double* lds = sm[w];
  const int htop = h0 << (nlev - 1);
  const double* s = src + row * s_src;
  for (int q = 2 * lane; q < htop; q += 128)
    *reinterpret_cast<double2*>(lds + q) = *reinterpret_cast<const double2*>(s + q);
  wave_lds_sync();
  rev_small_levels<L, FMA>(tp, tl, lds, lane, h0, nlev);
  double* __restrict__ y = dst + row * s_dst;
  for (int q = 2 * lane; q < htop; q += 128)
    *reinterpret_cast<double2*>(y + q) = *reinterpret_cast<const double2*>(lds + q);
}


// ---------------------------------------------------------------------------
// The reverse resident tails of the 2-D / 3-D COLUMN passes (config 3: 8192
// columns, 1 -> 1024 rows): one block per slab of CW columns, one wave per
// column.  The slab's rows [0, h) are loaded as whole 128-B lines
// (16-B pieces, 8 per row) and written transposed into LDS, column c at
// c * S (S = h + 2: 16-B aligned columns; the 16 lanes of a ds_write_b64
// group, 2 rows x 8 column pairs, land in distinct banks), so each wave runs
// the row kernels' wave-local levels (rev_small_levels, in place, no block
// barrier) on a contiguous column; then the slab goes back the same way.
// Same math and order as the block-per-slab resident kernel (fwt_rev_res):
// EXACT results are bit-identical.  That one moved 64-B row segments through
// 10 barrier-separated levels per block.
// CW = 8: a block holds half a slab (64 KB of LDS, two blocks per CU) and
// the two halves of every 128-B line go to blocks b and b + 8, which share
// an XCD (round-robin dealing) and start together, so the line is fetched
// from HBM once.
constexpr int kColW = 16;
__host__ __device__ constexpr int col16_stride(int h) { return h + 2; }

// slab column c0 of block b (CW = 8: pairs of half slabs on one XCD)
template <int CW>
__device__ __forceinline__ int64_t col_block(int64_t b, int nsl, int64_t& o) {
  if constexpr (CW == 16) {
    o = b / nsl;
    return (b - o * nsl) * 16;
  } else {
    const int nh = 2 * nsl;  // half slabs per outer
    const int64_t grp = b >> 4;
    const int64_t hs = ((grp << 3) + (b & 7)) * 2 + ((b >> 3) & 1);
    o = hs / nh;
    return (hs - o * nh) * 8;
  }
}

template <bool LOAD, int CW>
__device__ __forceinline__ void col16_move(double* sm, int S, double* g, int64_t s_len, int h) {
  const int tid = threadIdx.x;
  constexpr int PR = CW / 2;  // 16-B pieces per row
  for (int q = tid; q < PR * h; q += 64 * CW) {
    const int r = q / PR, c = 2 * (q % PR);
    double* gp = g + r * s_len + c;
    if constexpr (LOAD) {
      const double2 v = *reinterpret_cast<const double2*>(gp);
      sm[c * S + r] = v.x;
      sm[(c + 1) * S + r] = v.y;
    } else {
      *reinterpret_cast<double2*>(gp) = make_double2(sm[c * S + r], sm[(c + 1) * S + r]);
    }
  }
}

// Reverse: levels of output size h0 .. htop = h0 << (nlev-1) <= kSmallH
// over the slab rows [0, htop), written back to rows [0, htop).
template <int L, bool FMA, int CW>
__global__ __launch_bounds__(64 * CW) void fwt_rev_col16(const double* src, AxisView sv,
                                                         double* dst, AxisView dv, int h0,
                                                         int nlev, int inner, RevTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  __shared__ __attribute__((aligned(16))) double tl[2 * L];
  stage_rev_taps<L>(tp, tl);
  const int htop = h0 << (nlev - 1);
  const int S = col16_stride(htop);
  int64_t o;
  const int64_t c0 = col_block<CW>(blockIdx.x, inner / 16, o);
  col16_move<true, CW>(sm, S, const_cast<double*>(src) + view_base(sv, o) + c0, sv.s_len, htop);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  rev_small_levels<L, FMA>(tp, tl, sm + w * S, lane, h0, nlev);
  __syncthreads();
  col16_move<false, CW>(sm, S, dst + view_base(dv, o) + c0, dv.s_len, htop);
}

}  // namespace jwv
