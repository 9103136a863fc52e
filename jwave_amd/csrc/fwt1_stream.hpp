// fwt1_stream.hpp — the full-length forward pass of long contiguous signals
// (C = 1, compile-time geometry) as a persistent, double-buffered grid.
//
// fwt_fwd_tile1 launches one block per tile: a block DMAs its window, waits
// for all of it, computes K levels, stores, exits.  Co-resident blocks tend to
// sit in the same phase, so the CU alternates between "everyone waits for
// HBM" and "everyone computes".  Here each block owns a strided run of tiles
// and a loader wave keeps ONE TILE AHEAD: while the NTC compute threads run
// the K levels of tile k out of LDS buffer k&1, the loader's LDS-DMA for tile
// k+1 fills the other buffer, so every block always has a window in flight.
//
//  * The loader issues the DMA through inline asm (dma16_asm) and never
//    stores, so the compiler adds no vmcnt wait to its barriers and its own
//    `s_waitcnt vmcnt(0)` waits for its DMA only; the compute waves' stores
//    are never waited on inside the loop (lds_barrier orders LDS only).
//  * The loader joins every block barrier of the level chain (kBarriers).
//  * Tile walk: XCD x (blocks b with b % 8 == x) takes the contiguous chunk x
//    of the tiles and its blocks walk it side by side, so a tile's halo is its
//    neighbour's head, already in that XCD's L2 (as tile_order()).
//
// Math, summation order and outputs are exactly fwt_fwd_tile1's (the level
// bodies are Fwd1Level), so EXACT results stay bit-identical
// (Wavelet.java:236-260 per level, FastWaveletTransform.java:90-97).
#pragma once
#include "fwt1_kernels.hpp"

namespace jwv {

template <int L, int T, int K>
struct Fwd1Stream {
  using G = Fwd1Geo<L, T, K>;
  static constexpr int M0 = G::m(0);
  static constexpr int kUnits = (M0 + 1) / 2;               // 16-B DMA units per window
  static constexpr int kBuf = (G::lds_doubles() + 1) & ~1;  // doubles per buffer (16-B aligned)
  // block barriers inside Fwd1Level<..,1>::run: one per level below K, plus
  // the in-place level 1's extra one
  static constexpr int kBarriers = K >= 2 ? K : 0;
};

template <int L, int NTC, int T, int K, bool FMA>
__global__ __launch_bounds__(NTC + 64) void fwt_fwd_stream1(const double* __restrict__ src,
                                                            int64_t s_src,
                                                            double* __restrict__ dst,
                                                            int64_t s_dst,
                                                            double* __restrict__ adst,
                                                            int64_t s_adst, int h, int64_t ntotal,
                                                            FwdTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using S = Fwd1Stream<L, T, K>;
  const int tid = threadIdx.x;
  const bool loader = tid >= NTC;
  const int lane = tid & 63;
  const int ntile = h / T;
  const int msk = h - 1;

  const int64_t nb = gridDim.x, b = blockIdx.x;
  int64_t first, stride, count;
  if ((nb & 7) == 0 && (ntotal & 7) == 0) {
    const int64_t nper = nb >> 3, chunk = ntotal >> 3;
    const int64_t x = b & 7, slot = b >> 3;
    first = x * chunk + slot;
    stride = nper;
    count = slot < chunk ? (chunk - slot + nper - 1) / nper : 0;
  } else {
    first = b;
    stride = nb;
    count = b < ntotal ? (ntotal - b + nb - 1) / nb : 0;
  }

  auto issue = [&](int64_t g, double* buf) {  // loader wave only
    const int64_t o = g / ntile;
    const int base = (int)(g % ntile) * T;
    const double* s = src + o * s_src;
#pragma unroll
    for (int u0 = 0; u0 < S::kUnits; u0 += 64) {
      const int u = u0 + lane;
      if (u < S::kUnits) dma16_asm((const void*)(s + ((base + 2 * u) & msk)), buf + 2 * u0);
    }
  };

  if (loader) {
    if (count > 0) issue(first, lds);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  lds_barrier();
  for (int64_t k = 0; k < count; ++k) {
    const int64_t g = first + k * stride;
    double* cur = lds + (k & 1) * S::kBuf;
    if (loader) {
      if (k + 1 < count) issue(g + stride, lds + ((k + 1) & 1) * S::kBuf);
#pragma unroll
      for (int i = 0; i < S::kBarriers; ++i) lds_barrier();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      const int64_t o = g / ntile;
      const int t = (int)(g % ntile);
      Fwd1Level<L, NTC, T, K, FMA, 1>::run(tp, cur, dst + o * s_dst, h, t, adst + o * s_adst, 0);
    }
    lds_barrier();  // next window landed; every wave is done with `cur`
  }
}

}  // namespace jwv
