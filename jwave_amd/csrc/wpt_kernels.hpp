// wpt_kernels.hpp — full-tree Wavelet Packet Transform kernels (fp64).
//
// Reference: WaveletPacketTransform.forward (WaveletPacketTransform.java:73-124)
// applies Wavelet.forward to every packet [p*h, (p+1)*h) at each level (h = n,
// n/2, ..), wrap inside the packet; reverse (:141-191) mirrors it with
// Wavelet.reverse from the smallest packets up.  After K levels a signal holds
// 2^K bands in natural (Paley) order: band b at [b*n/2^K, (b+1)*n/2^K).
//
// Shapes (same scheme as fwt_kernels.hpp):
//  * wpt_fwd_res / wpt_rev_res: a whole signal (or packet) of C columns in LDS,
//    every level in place (register-staged), wrap `& (h-1)` per packet.
//  * wpt_fwd_tile / wpt_rev_tile: K levels fused on a tile of T samples with
//    its halo.  By periodicity the band fragments a tile derives from the
//    mod-n extended input are exactly the packets' periodic extensions, so one
//    tile yields T/2^K samples of every one of the 2^K bands.
#pragma once
#include "fwt_kernels.hpp"

namespace jwv {

// ---------------------------------------------------------------- forward
template <int L, int C, int NT, int CAP, bool FMA>
__device__ __forceinline__ void wpt_fwd_res_blk(const double* __restrict__ s, AxisView sv,
    double* __restrict__ y, AxisView dv, int n, int nlev, int c0, int inner, int dma,
    const typename FB<L>::Fwd& tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int MAXP = (CAP / 2 * C + NT - 1) / NT;
  constexpr int MAXU = (CAP * C + NT - 1) / NT;
  const int tid = threadIdx.x;
  load_window<C, NT, MAXU>(lds, s, n, dma != 0, c0, inner,
                           [&](int e) { return (int64_t)e * sv.s_len; });
  dma_fence_barrier();
  const int np = (n >> 1) * C;
  int h = n;
  for (int lev = 0; lev < nlev; ++lev) {
    const int half = h >> 1, msk = h - 1;
    double av[MAXP], dv2[MAXP];
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) {
        const int pr = p / C, c = p % C;
        const int pk = pr / half, i = pr % half;
        const int pb = pk * h;
        fwd_pair<L, FMA>(tp, [&](int j) { return lds[(pb + ((2 * i + j) & msk)) * C + c]; },
                         av[r], dv2[r]);
      }
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) {
        const int pr = p / C, c = p % C;
        const int pk = pr / half, i = pr % half;
        lds[(pk * h + i) * C + c] = av[r];
        lds[(pk * h + half + i) * C + c] = dv2[r];
      }
    }
    lds_barrier();
    h = half;
  }
  for (int q = tid; q < n * C; q += NT) {
    const int i = q / C, c = q % C;
    if (c0 + c < inner) y[(int64_t)i * dv.s_len + c] = lds[q];
  }
}

template <int L, int C, int NT, int CAP, bool FMA>
__global__ __launch_bounds__(NT) void wpt_fwd_res(const double* __restrict__ src, AxisView sv,
    double* __restrict__ dst, AxisView dv, int n, int nlev, int inner, int dma,
    typename FB<L>::Fwd tp) {
  const int ncb = (inner + C - 1) / C;
  const int64_t o = blockIdx.x / ncb;
  const int c0 = (blockIdx.x % ncb) * C;
  const double* s = src + view_base(sv, o) + c0;
  double* y = dst + view_base(dv, o) + c0;
  wpt_fwd_res_blk<L, C, NT, CAP, FMA>(s, sv, y, dv, n, nlev, c0, inner, dma, tp);
}

// Tiled: signal (or packet) length h, tile t covers [tT, tT+T).  After level
// l the LDS holds 2^l fragments of m_l samples, fragment f at [f*m_l, ..).
template <int L, int C, int NT, int T, int KMAX, bool FMA>
__global__ __launch_bounds__(NT) void wpt_fwd_tile(const double* __restrict__ src, AxisView sv,
                                                   double* __restrict__ dst, AxisView dv, int h,
                                                   int K, int inner, int dma,
                                                   typename FB<L>::Fwd tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int LM = LMax<L>::v;
  constexpr int M0MAX = T + (LM - 2) * ((1 << KMAX) - 1);
  constexpr int MAXP = ((M0MAX - (LM - 2)) / 2 * C + NT - 1) / NT;
  constexpr int MAXU = (M0MAX * C + NT - 1) / NT;
  const int nL = FB<L>::n(tp);
  const int ntile = h / T;
  const int ncb = (inner + C - 1) / C;
  const int nblk = gridDim.x;
  int b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  const int t = b % ntile;
  const int rest = b / ntile;
  const int64_t o = rest / ncb;
  const int c0 = (rest % ncb) * C;
  const double* s = src + view_base(sv, o) + c0;
  double* y = dst + view_base(dv, o) + c0;
  const int tid = threadIdx.x;

  const int m0 = T + (nL - 2) * ((1 << K) - 1);
  const int msk = h - 1;
  load_window<C, NT, MAXU>(lds, s, m0, dma != 0, c0, inner,
                           [&](int e) { return (int64_t)((t * T + e) & msk) * sv.s_len; });
  dma_fence_barrier();
  int m = m0;
  for (int l = 1; l <= K; ++l) {
    const int mo = (m - (nL - 2)) >> 1;
    const int nfrag = 1 << (l - 1);
    const int np = nfrag * mo * C;
    double av[MAXP], dv2[MAXP];
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) {
        const int pr = p / C, c = p % C;
        const int f = pr / mo, i = pr % mo;
        const int fb = f * m;
        fwd_pair<L, FMA>(tp, [&](int j) { return lds[(fb + 2 * i + j) * C + c]; }, av[r],
                         dv2[r]);
      }
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) {
        const int pr = p / C, c = p % C;
        const int f = pr / mo, i = pr % mo;
        lds[((2 * f) * mo + i) * C + c] = av[r];
        lds[((2 * f + 1) * mo + i) * C + c] = dv2[r];
      }
    }
    lds_barrier();
    m = mo;
  }
  // 2^K bands, own part T>>K of each
  const int own = T >> K, nb = 1 << K, band = h >> K;
  for (int q = tid; q < nb * own * C; q += NT) {
    const int pr = q / C, c = q % C;
    const int f = pr / own, i = pr % own;
    if (c0 + c < inner)
      y[((int64_t)f * band + (int64_t)t * own + i) * dv.s_len + c] = lds[(f * m + i) * C + c];
  }
}

// ---------------------------------------------------------------- reverse
// Resident: signal/packet of length n; reverse levels with packet sizes
// h0, 2h0, .., h0 << (nlev-1) (<= n).  Every packet of size h is reversed in place.
template <int L, int C, int NT, int CAP, bool FMA>
__device__ __forceinline__ void wpt_rev_res_blk(const double* __restrict__ s, AxisView sv,
    double* __restrict__ y, AxisView dv, int n, int h0, int nlev, int c0, int inner,
    int dma, const typename FB<L>::Rev& tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int MAXP = (CAP / 2 * C + NT - 1) / NT;
  constexpr int MAXU = (CAP * C + NT - 1) / NT;
  const int nL = FB<L>::nr(tp);
  const int tid = threadIdx.x;
  load_window<C, NT, MAXU>(lds, s, n, dma != 0, c0, inner,
                           [&](int e) { return (int64_t)e * sv.s_len; });
  dma_fence_barrier();
  const int np = (n >> 1) * C;
  int h = h0;
  for (int lev = 0; lev < nlev; ++lev) {
    const int half = h >> 1, hm = half - 1;
    double xe[MAXP], xo[MAXP];
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) {
        const int pr = p / C, c = p % C;
        const int pk = pr / half, m = pr % half;
        const double* A = lds + (pk * h) * C + c;
        const double* D = lds + (pk * h + half) * C + c;
        if (h >= nL) {
          if (m >= ((nL + 1) >> 1) - 1) {
            rev_pair<L, FMA>(tp, A + m * C, D + m * C, C, xe[r], xo[r]);
          } else {
            rev_pair_head<L, FMA>(
                tp, m, [=](int q) { return A[((m - q) & hm) * C]; },
                [=](int q) { return D[((m - q) & hm) * C]; }, xe[r], xo[r]);
          }
        } else {
          xe[r] = rev_small<L, FMA>(tp, A, D, C, h, 2 * m);
          xo[r] = rev_small<L, FMA>(tp, A, D, C, h, 2 * m + 1);
        }
      }
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) {
        const int pr = p / C, c = p % C;
        const int pk = pr / half, m = pr % half;
        lds[(pk * h + 2 * m) * C + c] = xe[r];
        lds[(pk * h + 2 * m + 1) * C + c] = xo[r];
      }
    }
    lds_barrier();
    h <<= 1;
  }
  for (int q = tid; q < n * C; q += NT) {
    const int i = q / C, c = q % C;
    if (c0 + c < inner) y[(int64_t)i * dv.s_len + c] = lds[q];
  }
}

template <int L, int C, int NT, int CAP, bool FMA>
__global__ __launch_bounds__(NT) void wpt_rev_res(const double* __restrict__ src, AxisView sv,
    double* __restrict__ dst, AxisView dv, int n, int h0, int nlev, int inner, int dma,
    typename FB<L>::Rev tp) {
  const int ncb = (inner + C - 1) / C;
  const int64_t o = blockIdx.x / ncb;
  const int c0 = (blockIdx.x % ncb) * C;
  const double* s = src + view_base(sv, o) + c0;
  double* y = dst + view_base(dv, o) + c0;
  wpt_rev_res_blk<L, C, NT, CAP, FMA>(s, sv, y, dv, n, h0, nlev, c0, inner, dma, tp);
}

// Tiled reverse: K levels, packet sizes hK>>(K-1) .. hK (hK = signal/packet
// length of this pass).  Input: 2^K bands of length hK>>K.  Tile t writes
// dst[tT, tT+T).  Windows as in fwt_rev_tile; at coarse level l there are 2^l
// fragments of width W_l, fragment f at [f*W_l, ..).
template <int L, int C, int NT, int T, int KMAX, bool FMA>
__global__ __launch_bounds__(NT) void wpt_rev_tile(const double* __restrict__ src, AxisView sv,
                                                   double* __restrict__ dst, AxisView dv, int hK,
                                                   int K, int inner, int dma,
                                                   typename FB<L>::Rev tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int LM = LMax<L>::v;
  constexpr int QM = (LM + 1) / 2;
  constexpr int MAXP = ((T / 2 + (1 << KMAX) * (QM + 2)) * C + NT - 1) / NT;
  constexpr int MAXU = ((T + (1 << KMAX) * (2 * QM + 4)) * C + NT - 1) / NT;
  const int nL = FB<L>::nr(tp);
  const int Q = (nL + 1) >> 1;
  const int ntile = hK / T;
  const int ncb = (inner + C - 1) / C;
  const int nblk = gridDim.x;
  int b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  const int t = b % ntile;
  const int rest = b / ntile;
  const int64_t o = rest / ncb;
  const int c0 = (rest % ncb) * C;
  const double* s = src + view_base(sv, o) + c0;
  double* y = dst + view_base(dv, o) + c0;
  const int tid = threadIdx.x;
  auto win_b = [&](int l) {
    int bb = t * T;
    for (int k = 0; k < l; ++k) bb = ((bb >> 1) - (Q - 1)) & ~1;
    return bb;
  };
  auto win_e = [&](int l) { return (t * T + T) >> l; };

  {  // coarsest level: 2^K band windows
    const int BK = win_b(K), WK = win_e(K) - BK;
    const int band = hK >> K, bm = band - 1, nb = 1 << K;
    // the 2^K band windows, stacked: row e' = f*WK + e  (WK is even)
    load_window<C, NT, MAXU>(lds, s, nb * WK, dma != 0, c0, inner, [&](int r) {
      const int f = r / WK, e = r % WK;
      return ((int64_t)f * band + ((BK + e) & bm)) * sv.s_len;
    });
  }
  dma_fence_barrier();
  for (int l = K - 1; l >= 0; --l) {
    const int half = hK >> (l + 1), hm = half - 1;
    const int Bl = win_b(l), Bl1 = win_b(l + 1);
    const int Wl = win_e(l) - Bl, Wl1 = win_e(l + 1) - Bl1;
    const int pbase = Bl >> 1;
    const int off = pbase - Bl1;
    const int nfrag = 1 << l;
    const int pw = Wl >> 1;  // pairs per fragment
    const int np = nfrag * pw * C;
    double xe[MAXP], xo[MAXP];
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) {
        const int pr = p / C, c = p % C;
        const int f = pr / pw, ml = pr % pw;
        const int mg = (pbase + ml) & hm;
        const int li = off + ml;
        const double* A = lds + ((2 * f) * Wl1) * C + c;
        const double* D = lds + ((2 * f + 1) * Wl1) * C + c;
        if (mg >= Q - 1) {
          rev_pair<L, FMA>(tp, A + li * C, D + li * C, C, xe[r], xo[r]);
        } else {
          rev_pair_head<L, FMA>(
              tp, mg, [=](int q) { return A[(li - q) * C]; }, [=](int q) { return D[(li - q) * C]; },
              xe[r], xo[r]);
        }
      }
    }
    if (l == 0) {
#pragma unroll
      for (int r = 0; r < MAXP; ++r) {
        const int p = tid + r * NT;
        if (p < np) {
          const int ml = p / C, c = p % C;
          if (c0 + c < inner) {
            const int64_t k = (int64_t)t * T + 2 * ml;
            y[k * dv.s_len + c] = xe[r];
            y[(k + 1) * dv.s_len + c] = xo[r];
          }
        }
      }
    } else {
      lds_barrier();
#pragma unroll
      for (int r = 0; r < MAXP; ++r) {
        const int p = tid + r * NT;
        if (p < np) {
          const int pr = p / C, c = p % C;
          const int f = pr / pw, ml = pr % pw;
          lds[(f * Wl + 2 * ml) * C + c] = xe[r];
          lds[(f * Wl + 2 * ml + 1) * C + c] = xo[r];
        }
      }
      lds_barrier();
    }
  }
}

}  // namespace jwv
