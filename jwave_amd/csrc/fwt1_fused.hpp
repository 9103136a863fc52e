// fwt1_fused.hpp — the row passes of many contiguous rows (2-D row passes,
// batches; config 3: 8192 rows of 8192 samples) with their resident tail in
// the SAME launch.
//
// Forward (fwt_fwd_tile1r): the tile pass of fwt_fwd_tile1 (K levels per
// tile of T samples, ntile tiles per row), whose level-K approximations go
// out write-through; every tile then counts itself into its row's arrival
// counter (MI355X_MICROARCH.md hand-off protocol, jwv_device.hpp).  The
// block that completes a row's count is the row's last tile: its wave 0 reads
// the row's h >> K approximations back (sc1 loads: L2, the producers are
// its XCD neighbours in the grouped tile walk) and runs the remaining levels
// exactly as the wave-per-row tail kernel does (fwd_small_levels,
// fwt1_row.hpp), writing the row's coefficients [0, h >> K); the other waves
// leave.  The separate tail launch (and its kernel boundary) is gone; the
// tails run while other rows' tiles stream.  Counters: one per row, zero
// between launches (the last arriver re-zeroes it; a failed call re-zeroes
// them all, capi.cpp row_counters_resync).  Same math and summation order as
// tile pass + tail: EXACT results are bit-identical.
#pragma once
#include "fwt1_kernels.hpp"
#include "fwt1_row.hpp"

namespace jwv {

// which waves run a fused row tail / head: 0 wave 0; 1 wave (row mod 4), so
// the chains of a CU's blocks spread over its SIMDs; 2 the whole block
// (block-wide resident levels, a barrier per level)
#ifndef JWV_FWDR_MODE
#define JWV_FWDR_MODE 1
#endif
#ifndef JWV_REVH_MODE
#define JWV_REVH_MODE 1
#endif

template <int L, int NT, int T, int K, bool FMA>
__global__ __launch_bounds__(NT) void fwt_fwd_tile1r(const double* __restrict__ src,
                                                     int64_t s_src, double* __restrict__ dst,
                                                     int64_t s_dst, double* adst, int64_t s_adst,
                                                     int h, FwdTaps<L> tp, int sp,
                                                     unsigned* cnt, int levr) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int last;
  using G = Fwd1Geo<L, T, K>;
  constexpr int M0 = G::m(0);
  static_assert(G::lds_doubles() >= 2, "window");
  const int ntile = h / T;
  const int b = tile_order(gridDim.x, sp);
  const int t = b % ntile;
  const int64_t o = b / ntile;
  const double* s = src + o * s_src;
  const int msk = h - 1, base = t * T;
  load_window<1, NT, (M0 + NT - 1) / NT>(lds, s, M0, true, 0, 1,
                                          [&](int e) { return (int64_t)((base + e) & msk); });
  dma_fence_barrier();
  Fwd1Level<L, NT, T, K, FMA, 1, true>::run(tp, lds, dst + o * s_dst, h, t, adst + o * s_adst, sp);
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = atomic_add_agent(cnt + o, 1u);
    last = old == (unsigned)(ntile - 1);
    if (last) store_agent(cnt + o, 0u);
  }
  __syncthreads();
  if (!last) return;
  // the row's last tile: the resident levels (lds is free: every wave of
  // this block passed the barrier after its last window read)
  const int h0 = h >> K;
  const double* ap = adst + o * s_adst;
  double* __restrict__ y = dst + o * s_dst;
#if JWV_FWDR_MODE == 2
  load_window_wt<NT, (kSmallH + NT - 1) / NT>(lds, ap, h0, [](int e) { return e; });
  lds_barrier();
  fwd_res1_levels<L, NT, kSmallH, FMA>(lds, y, h0, levr, tp);
#else
  const int w = JWV_FWDR_MODE == 1 ? (int)(o & (NT / 64 - 1)) : 0;
  if ((int)(threadIdx.x >> 6) != w) return;
  const int lane = threadIdx.x & 63;
  constexpr int PR = kSmallH / 64;
  double v[PR];
#pragma unroll
  for (int r = 0; r < PR; ++r)
    if (lane + 64 * r < h0) v[r] = ld_wt(ap + lane + 64 * r);
#pragma unroll
  for (int r = 0; r < PR; ++r)
    if (lane + 64 * r < h0) lds[lane + 64 * r] = v[r];
  wave_lds_sync();
  const int hh = fwd_small_levels<L, FMA>(tp, lds, lane, h0, levr, y);
  for (int q = lane; q < hh; q += 64) y[q] = lds[q];
#endif
}

// Reverse (fwt_rev_tile1h): the first tile pass over many rows with the
// rows' resident head in the same launch.  Every tile recomputes its row's
// head itself (no inter-workgroup wait): wave 0 loads the coefficient
// prefix [0, hR) of its row (hR = h0 << (nres-1) <= kSmallH, the 4 tiles of
// a row are neighbours in the grouped tile walk, so 3 of the 4 reads hit
// L2) and runs the nres head levels exactly as the wave-per-row tail kernel
// does (rev_small_levels, fwt1_row.hpp), while the block's detail windows
// land by LDS-DMA; the tile's level-K approximation window is then taken
// from that LDS copy instead of a workspace row written by a separate launch.
// LDS: the tile's in-place windows, then the head (hR + 2), then the staged
// taps (2L).  Same math and order as tail + tile pass: EXACT results are
// bit-identical.
template <int L, int T, int K>
__host__ __device__ constexpr int rev1h_head_off() {
  return (Rev1Geo<L, T, K>::ip_lds_doubles() + 1) & ~1;
}
template <int L, int T, int K>
__host__ __device__ constexpr int rev1h_lds_doubles(int hR) {
  return rev1h_head_off<L, T, K>() + hR + 2 + 2 * L;
}

template <int L, int NT, int T, int K, bool FMA>
__global__ __launch_bounds__(NT) void fwt_rev_tile1h(const double* __restrict__ coef, int64_t s_c,
                                                     double* __restrict__ dst, int64_t s_d,
                                                     int hK, int h0, int nres, RevTaps<L> tp,
                                                     int sp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using G = Rev1Geo<L, T, K>;
  constexpr int MAXU = (G::len(1) + NT - 1) / NT;
  const int hR = hK >> K;
  double* head = lds + rev1h_head_off<L, T, K>();
  double* tl = head + hR + 2;
  const int ntile = hK / T;
  const int b = tile_order(gridDim.x, sp);
  const int t = b % ntile;
  const int64_t o = b / ntile;
  const double* sc = coef + o * s_c;
  // the head's wave: the row's coefficient prefix into registers first (its
  // loads then complete ahead of the DMA burst below), the staged taps
  constexpr int PR = kSmallH / 128;
#if JWV_REVH_MODE == 2
  const bool w0 = false;
#else
  const bool w0 = (int)(threadIdx.x >> 6) == (JWV_REVH_MODE == 1 ? (int)(o & (NT / 64 - 1)) : 0);
#endif
  const int lane = threadIdx.x & 63;
  double2 pre[PR];
  if (w0) {
#pragma unroll
    for (int r = 0; r < PR; ++r) {
      const int q = 2 * lane + 128 * r;
      if (q < hR) pre[r] = *reinterpret_cast<const double2*>(sc + q);
    }
    if (lane == 0) {  // stage_rev_taps' layout, by this wave
#pragma unroll
      for (int q = 0; q < L / 2; ++q) {
        *reinterpret_cast<double2*>(tl + 4 * q) = make_double2(tp.lo_r[2 * q], tp.lo_r[2 * q + 1]);
        *reinterpret_cast<double2*>(tl + 4 * q + 2) =
            make_double2(tp.hi_r[2 * q], tp.hi_r[2 * q + 1]);
      }
    }
  }
  // the detail windows in one DMA burst
#pragma unroll
  for (int l = K - 1; l >= 0; --l) {
    const int half = hK >> (l + 1), hm = half - 1;
    const int B = (t * T >> (l + 1)) - G::c(l + 1);
    load_window<1, NT, MAXU>(lds + G::ip_doff(l), sc, G::len(l + 1), true, 0, 1,
                             [&](int e) { return (int64_t)half + ((B + e) & hm); });
  }
#if JWV_REVH_MODE == 2
  for (int q = 2 * threadIdx.x; q < hR; q += 2 * NT)
    *reinterpret_cast<double2*>(head + q) = *reinterpret_cast<const double2*>(sc + q);
  dma_fence_barrier();
  rev_res1_levels<L, NT, kSmallH, FMA>(head, h0, nres, tp);  // ends with a block barrier
#else
  if (w0) {  // the head, wave-local (tl and head are this wave's writes)
#pragma unroll
    for (int r = 0; r < PR; ++r) {
      const int q = 2 * lane + 128 * r;
      if (q < hR) *reinterpret_cast<double2*>(head + q) = pre[r];
    }
    wave_lds_sync();
    rev_small_levels<L, FMA>(tp, tl, head, lane, h0, nres);
  }
  dma_fence_barrier();
#endif
  {
    const int BK = (t * T >> K) - G::c(K), am = hR - 1;
    for (int e = threadIdx.x; e < G::len(K); e += NT) lds[e] = head[(BK + e) & am];
  }
  lds_barrier();
  Rev1Level<L, NT, T, K, FMA, K - 1, false, true, true>::run(tp, lds, t, dst + o * s_d, sp);
}

}  // namespace jwv
