// fwt_kernels.hpp — Mallat-pyramid FWT kernels for gfx950 (fp64).
//
// Reference semantics: one analysis level is Wavelet.forward(x, h)
// (transforms/wavelets/Wavelet.java:236-260):
//     a[i] = sum_j x[(2i+j) mod h] lo[j],  d[i] = sum_j x[(2i+j) mod h] hi[j]
// with [a | d] written over x[0..h); FastWaveletTransform.forward
// (FastWaveletTransform.java:71-101) repeats it on the shrinking prefix.
// One synthesis level is Wavelet.reverse (Wavelet.java:277-303), a scatter-add
// x[(2i+j) mod h] += a[i] loR[j] + d[i] hiR[j]; here it is a gather in which
// every output sums its terms in the order the scatter loop produces them
// (i ascending, then j ascending), so EXACT mode is bit-identical.
//
// Two kernel shapes per direction:
//  * *_res  ("resident"): the whole level-input of C signals sits in LDS and
//           all remaining levels run there (short signals, 2-D rows, the deep
//           tail of a long 1-D signal).  Wrap is `& (h-1)` inside LDS.
//  * *_tile ("tiled"): a long signal is cut into tiles of T samples; a block
//           loads its tile plus the halo the next K levels need, with global
//           indices taken mod h (periodic extension), and fuses K levels in
//           LDS.  Each level's details go straight to HBM; only the level-K
//           approximation (T/2^K per tile) is handed to the next pass.
//           HBM traffic ~ read once + write once per K levels.
#pragma once
#include "jwv_device.hpp"

namespace jwv {

// ---------------------------------------------------------------- tap access
template <int L>
struct FB {
  using Fwd = FwdTaps<L>;
  using Rev = RevTaps<L>;
  static constexpr bool kStatic = true;
  __device__ static constexpr int n(const Fwd&) { return L; }
  __device__ static constexpr int nr(const Rev&) { return L; }
  __device__ static double lo(const Fwd& t, int j) { return t.lo[j]; }
  __device__ static double hi(const Fwd& t, int j) { return t.hi[j]; }
  __device__ static double lor(const Rev& t, int j) { return t.lo_r[j]; }
  __device__ static double hir(const Rev& t, int j) { return t.hi_r[j]; }
  __device__ static double scale(double v, const Rev&) { return v; }
};
template <>
struct FB<0> {
  using Fwd = AnyTaps;
  using Rev = AnyTaps;
  static constexpr bool kStatic = false;
  __device__ static int n(const Fwd& t) { return t.L; }
  __device__ static int nr(const Rev& t) { return t.L; }
  __device__ static double lo(const Fwd& t, int j) { return t.lo[j]; }
  __device__ static double hi(const Fwd& t, int j) { return t.hi[j]; }
  __device__ static double lor(const Rev& t, int j) { return t.lo_r[j]; }
  __device__ static double hir(const Rev& t, int j) { return t.hi_r[j]; }
  // Haar1Orthogonal.reverse: term scaled by 0.5 (haar/Haar1Orthogonal.java:198-200);
  // x*1.0 == x exactly, so unscaled banks are unaffected.
  __device__ static double scale(double v, const Rev& t) { return t.scale * v; }
};

// Upper bound on taps used to size static register/LDS budgets.
template <int L>
struct LMax {
  static constexpr int v = L == 0 ? kMaxTaps : L;
};

// ------------------------------------------------------------ forward pair
// a = sum_j x[k_j] lo[j], d = sum_j x[k_j] hi[j], j ascending, from +0.0
// (Wavelet.java:244-253).  `at(j)` yields the LDS address of x[2i+j].
template <int L, bool FMA, typename At>
__device__ __forceinline__ void fwd_pair(const typename FB<L>::Fwd& tp, At at, double& a,
                                         double& d) {
  double sa = 0.0, sd = 0.0;
  if constexpr (FB<L>::kStatic) {
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const double v = at(j);
      sa = mac<FMA>(sa, v, FB<L>::lo(tp, j));
      sd = mac<FMA>(sd, v, FB<L>::hi(tp, j));
    }
  } else {
    const int n = FB<L>::n(tp);
    for (int j = 0; j < n; ++j) {
      const double v = at(j);
      sa = mac<FMA>(sa, v, FB<L>::lo(tp, j));
      sd = mac<FMA>(sd, v, FB<L>::hi(tp, j));
    }
  }
  a = sa;
  d = sd;
}

// ------------------------------------------------------------ reverse pair
// Outputs x[2m] (even taps j=2q) and x[2m+1] (odd taps j=2q+1) of one
// synthesis level of size h (half = h/2 pairs).  Term q reads a[m-q], d[m-q]
// (indices mod half).  Scatter order of Wavelet.reverse = i ascending: the
// non-wrapped terms (q <= mg) in q-descending order first, then the wrapped
// ones (q > mg) in q-descending order.  Valid for h >= L (at most one wrap);
// smaller levels use rev_level_small.  A(q)/D(q) return a[m-q], d[m-q].
template <int L, bool FMA, typename GetA, typename GetD>
__device__ __forceinline__ void rev_pair(const typename FB<L>::Rev& tp, int mg, GetA A, GetD D,
                                         double& xe, double& xo) {
  constexpr int LM = LMax<L>::v;
  constexpr int QM = (LM + 1) / 2;
  const int nt = FB<L>::nr(tp);
  const int qe = (nt + 1) >> 1;  // even taps
  const int qo = nt >> 1;        // odd taps
  double se = 0.0, so = 0.0;
  auto term_e = [&](int q) {
    const int j = 2 * q;
    double t = A(q) * FB<L>::lor(tp, j);
    t = mac<FMA>(t, D(q), FB<L>::hir(tp, j));
    return FB<L>::scale(t, tp);
  };
  auto term_o = [&](int q) {
    const int j = 2 * q + 1;
    double t = A(q) * FB<L>::lor(tp, j);
    t = mac<FMA>(t, D(q), FB<L>::hir(tp, j));
    return FB<L>::scale(t, tp);
  };
  if (mg >= QM - 1 || (!FB<L>::kStatic && mg >= qe - 1)) {
    // interior: plain q-descending order
    if constexpr (FB<L>::kStatic) {
#pragma unroll
      for (int q = QM - 1; q >= 0; --q) {
        if (q < qe) se += term_e(q);
        if (q < qo) so += term_o(q);
      }
    } else {
      for (int q = qe - 1; q >= 0; --q) {
        se += term_e(q);
        if (q < qo) so += term_o(q);
      }
    }
  } else {
    // array head: non-wrapped (q <= mg) first, then wrapped (q > mg)
    for (int q = qe - 1; q >= 0; --q)
      if (q <= mg) se += term_e(q);
    for (int q = qe - 1; q >= 0; --q)
      if (q > mg) se += term_e(q);
    for (int q = qo - 1; q >= 0; --q)
      if (q <= mg) so += term_o(q);
    for (int q = qo - 1; q >= 0; --q)
      if (q > mg) so += term_o(q);
  }
  xe = se;  // se started at +0.0 like arrTime[k] (Wavelet.java:282)
  xo = so;
}

// Levels with h < L wrap several times: emulate the scatter literally
// (i ascending, j ascending).  Only for tiny h (h < L <= 64), per output k.
template <int L, bool FMA>
__device__ double rev_small(const typename FB<L>::Rev& tp, const double* a, const double* d,
                            int stride, int h, int k) {
  const int half = h >> 1, nt = FB<L>::nr(tp);
  double x = 0.0;
  for (int i = 0; i < half; ++i)
    for (int j = 0; j < nt; ++j)
      if (((2 * i + j) & (h - 1)) == k) {
        double t = a[i * stride] * FB<L>::lor(tp, j);
        t = mac<FMA>(t, d[i * stride], FB<L>::hir(tp, j));
        x += FB<L>::scale(t, tp);
      }
  return x;
}

// ====================================================================
// Forward, resident.  Grid: one block per (outer o, column slab cb).
// src: level input of length h0 (view sv); dst: coefficient array (view dv):
// level of size h writes details to dst[h/2 .. h), the final approximation to
// dst[0 .. h_end).  nlev >= 0 levels; LDS = h0*C doubles.
// ====================================================================
template <int L, int C, int NT, int CAP, bool FMA>
__global__ __launch_bounds__(NT) void fwt_fwd_res(const double* __restrict__ src, AxisView sv,
                                                  double* __restrict__ dst, AxisView dv, int h0,
                                                  int nlev, int inner, int dma,
                                                  typename FB<L>::Fwd tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int MAXP = (CAP / 2 * C + NT - 1) / NT;
  constexpr int MAXU = (CAP * C + NT - 1) / NT;
  const int ncb = (inner + C - 1) / C;
  const int64_t o = blockIdx.x / ncb;
  const int c0 = (blockIdx.x % ncb) * C;
  const double* s = src + view_base(sv, o) + c0;
  double* y = dst + view_base(dv, o) + c0;
  const int tid = threadIdx.x;

  load_window<C, NT, MAXU>(lds, s, h0, dma != 0, c0, inner,
                           [&](int e) { return (int64_t)e * sv.s_len; });
  dma_fence_barrier();

  int h = h0;
  for (int lev = 0; lev < nlev; ++lev) {
    const int half = h >> 1, np = half * C, msk = h - 1;
    double av[MAXP];
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) {
        const int i = p / C, c = p % C;
        double a, d;
        fwd_pair<L, FMA>(tp, [&](int j) { return lds[((2 * i + j) & msk) * C + c]; }, a, d);
        av[r] = a;
        if (c0 + c < inner) y[(int64_t)(half + i) * dv.s_len + c] = d;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) lds[p] = av[r];
    }
    __syncthreads();
    h = half;
  }
  for (int q = tid; q < h * C; q += NT) {
    const int i = q / C, c = q % C;
    if (c0 + c < inner) y[(int64_t)i * dv.s_len + c] = lds[q];
  }
}

// ====================================================================
// Forward, tiled.  Grid: (outer * ncb) * (h / T) blocks; tile t covers level
// input [tT, tT+T).  Window m0 = T + (L-2)(2^K - 1) samples (periodic mod h).
// Level l (1..K, size h_l = h >> (l-1)) writes its own T>>l details to
// dst[h_l/2 + t*(T>>l) ..]; the K-th approximation (T>>K) goes to adst (view
// av, level-K array of length h>>K).  Blocks are ordered tile-fastest within
// an XCD group so that a tile and its halo neighbour share an L2.
// ====================================================================
template <int L, int C, int NT, int T, int KMAX, bool FMA>
__global__ __launch_bounds__(NT) void fwt_fwd_tile(const double* __restrict__ src, AxisView sv,
                                                   double* __restrict__ dst, AxisView dv,
                                                   double* __restrict__ adst, AxisView av_,
                                                   int h, int K, int inner, int dma,
                                                   typename FB<L>::Fwd tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int LM = LMax<L>::v;
  constexpr int M0MAX = T + (LM - 2) * ((1 << KMAX) - 1);
  constexpr int MAXP = ((M0MAX - (LM - 2)) / 2 * C + NT - 1) / NT;
  constexpr int MAXU = (M0MAX * C + NT - 1) / NT;
  const int nL = FB<L>::n(tp);
  const int ntile = h / T;
  const int ncb = (inner + C - 1) / C;
  // XCD-aware remap: consecutive blockIdx go to different XCDs; give each XCD
  // a contiguous run of tiles so halo re-reads hit its L2.
  const int nblk = gridDim.x;
  int b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  const int t = b % ntile;
  const int rest = b / ntile;
  const int64_t o = rest / ncb;
  const int c0 = (rest % ncb) * C;
  const double* s = src + view_base(sv, o) + c0;
  double* y = dst + view_base(dv, o) + c0;
  double* ya = adst + view_base(av_, o) + c0;
  const int tid = threadIdx.x;

  const int m0 = T + (nL - 2) * ((1 << K) - 1);
  const int msk = h - 1;
  const int base = t * T;
  load_window<C, NT, MAXU>(lds, s, m0, dma != 0, c0, inner,
                           [&](int e) { return (int64_t)((base + e) & msk) * sv.s_len; });
  dma_fence_barrier();

  int m = m0, hl = h;
  for (int l = 1; l <= K; ++l) {
    const int mo = (m - (nL - 2)) >> 1;
    const int own = T >> l;
    const int np = mo * C;
    const int64_t dbase = (int64_t)(hl >> 1) + (int64_t)t * own;
    double av[MAXP];
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) {
        const int i = p / C, c = p % C;
        double a, d;
        fwd_pair<L, FMA>(tp, [&](int j) { return lds[(2 * i + j) * C + c]; }, a, d);
        av[r] = a;
        if (i < own && c0 + c < inner) y[(dbase + i) * dv.s_len + c] = d;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) lds[p] = av[r];
    }
    __syncthreads();
    m = mo;
    hl >>= 1;
  }
  const int own = T >> K;
  for (int q = tid; q < own * C; q += NT) {
    const int i = q / C, c = q % C;
    if (c0 + c < inner) ya[((int64_t)t * own + i) * av_.s_len + c] = lds[q];
  }
}

// ====================================================================
// Reverse, resident.  src holds the coefficient prefix [0, htop) of each
// signal (htop = h0 << (nlev-1), or h0 when nlev == 0); levels of size h0,
// 2h0, .., htop run in LDS; the result [0, htop) goes to dst.
// ====================================================================
template <int L, int C, int NT, int CAP, bool FMA>
__global__ __launch_bounds__(NT) void fwt_rev_res(const double* __restrict__ src, AxisView sv,
                                                  double* __restrict__ dst, AxisView dv, int h0,
                                                  int nlev, int inner, int dma,
                                                  typename FB<L>::Rev tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int MAXP = (CAP / 2 * C + NT - 1) / NT;
  constexpr int MAXU = (CAP * C + NT - 1) / NT;
  const int nL = FB<L>::nr(tp);
  const int ncb = (inner + C - 1) / C;
  const int64_t o = blockIdx.x / ncb;
  const int c0 = (blockIdx.x % ncb) * C;
  const double* s = src + view_base(sv, o) + c0;
  double* y = dst + view_base(dv, o) + c0;
  const int tid = threadIdx.x;
  const int htop = nlev > 0 ? (h0 << (nlev - 1)) : h0;

  load_window<C, NT, MAXU>(lds, s, htop, dma != 0, c0, inner,
                           [&](int e) { return (int64_t)e * sv.s_len; });
  dma_fence_barrier();

  int h = h0;
  for (int lev = 0; lev < nlev; ++lev) {
    const int half = h >> 1, np = half * C, hm = half - 1;
    double xe[MAXP], xo[MAXP];
    if (h >= nL) {
#pragma unroll
      for (int r = 0; r < MAXP; ++r) {
        const int p = tid + r * NT;
        if (p < np) {
          const int m = p / C, c = p % C;
          rev_pair<L, FMA>(
              tp, m, [&](int q) { return lds[((m - q) & hm) * C + c]; },
              [&](int q) { return lds[(half + ((m - q) & hm)) * C + c]; }, xe[r], xo[r]);
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < MAXP; ++r) {
        const int p = tid + r * NT;
        if (p < np) {
          const int m = p / C, c = p % C;
          xe[r] = rev_small<L, FMA>(tp, lds + c, lds + half * C + c, C, h, 2 * m);
          xo[r] = rev_small<L, FMA>(tp, lds + c, lds + half * C + c, C, h, 2 * m + 1);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) {
        const int m = p / C, c = p % C;
        lds[(2 * m) * C + c] = xe[r];
        lds[(2 * m + 1) * C + c] = xo[r];
      }
    }
    __syncthreads();
    h <<= 1;
  }
  for (int q = tid; q < htop * C; q += NT) {
    const int i = q / C, c = q % C;
    if (c0 + c < inner) y[(int64_t)i * dv.s_len + c] = lds[q];
  }
}

// ====================================================================
// Reverse, tiled: K levels of sizes h1, 2h1, .., hK = h1 << (K-1).
// asrc: approximation of length h1/2 (view as); coef: coefficient array (view
// cv, details of level size h at coef[h/2 .. h)); dst: output of length hK.
// Tile t produces dst[tT, tT+T).  Windows (pair aligned) from fine to coarse:
//   B_0 = tT, E_0 = tT+T;  B_{l+1} = even_floor(B_l/2 - (Q-1)), E_{l+1} = E_l/2
// LDS: A window (<= T/2 + 2Q + 2) then D window (same bound), times C.
// ====================================================================
template <int L, int C, int NT, int T, int KMAX, bool FMA>
__global__ __launch_bounds__(NT) void fwt_rev_tile(const double* __restrict__ asrc, AxisView as,
                                                   const double* __restrict__ coef, AxisView cv,
                                                   double* __restrict__ dst, AxisView dv, int h1,
                                                   int K, int inner, int dma,
                                                   typename FB<L>::Rev tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int LM = LMax<L>::v;
  constexpr int QM = (LM + 1) / 2;
  constexpr int WMAX = T / 2 + 2 * QM + 4;  // max window (pairs*2) at level >= 1
  constexpr int MAXP = ((T / 2 + QM + 2) * C + NT - 1) / NT;
  constexpr int MAXU = (WMAX * C + NT - 1) / NT;
  const int nL = FB<L>::nr(tp);
  const int Q = (nL + 1) >> 1;
  const int hK = h1 << (K - 1);
  const int ntile = hK / T;
  const int ncb = (inner + C - 1) / C;
  const int nblk = gridDim.x;
  int b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  const int t = b % ntile;
  const int rest = b / ntile;
  const int64_t o = rest / ncb;
  const int c0 = (rest % ncb) * C;
  const double* sa = asrc + view_base(as, o) + c0;
  const double* sc = coef + view_base(cv, o) + c0;
  double* y = dst + view_base(dv, o) + c0;
  const int tid = threadIdx.x;
  double* abuf = lds;
  double* dbuf = lds + WMAX * C;

  // window bounds; B may be negative (periodic).  Recomputed on demand so no
  // runtime-indexed register array is needed.
  auto win_b = [&](int l) {
    int bb = t * T;
    for (int k = 0; k < l; ++k) bb = ((bb >> 1) - (Q - 1)) & ~1;  // even floor
    return bb;
  };
  auto win_e = [&](int l) { return (t * T + T) >> l; };
  // coarsest approximation window: a of length h1/2 = hK >> K
  {
    const int BK = win_b(K);
    const int W = win_e(K) - BK;
    const int am = (hK >> K) - 1;
    load_window<C, NT, MAXU>(abuf, sa, W, dma != 0, c0, inner,
                             [&](int e) { return (int64_t)((BK + e) & am) * as.s_len; });
  }
  for (int l = K - 1; l >= 0; --l) {
    // level with output size hl = hK >> l; inputs a,d of length half = hl/2
    const int half = hK >> (l + 1), hm = half - 1;
    const int Bl = win_b(l), Bl1 = win_b(l + 1);
    const int Wd = win_e(l + 1) - Bl1;
    load_window<C, NT, MAXU>(dbuf, sc, Wd, dma != 0, c0, inner, [&](int e) {
      return ((int64_t)half + ((Bl1 + e) & hm)) * cv.s_len;
    });
    dma_fence_barrier();
    const int pbase = Bl >> 1;                     // first pair (global, may be <0)
    const int np = ((win_e(l) - Bl) >> 1) * C;     // pairs in window
    const int off = pbase - Bl1;                   // local index of a[pbase]
    double xe[MAXP], xo[MAXP];
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < np) {
        const int ml = p / C, c = p % C;
        const int mg = (pbase + ml) & hm;
        const int li = off + ml;
        rev_pair<L, FMA>(
            tp, mg, [&](int q) { return abuf[(li - q) * C + c]; },
            [&](int q) { return dbuf[(li - q) * C + c]; }, xe[r], xo[r]);
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
      __syncthreads();
#pragma unroll
      for (int r = 0; r < MAXP; ++r) {
        const int p = tid + r * NT;
        if (p < np) {
          const int ml = p / C, c = p % C;
          abuf[(2 * ml) * C + c] = xe[r];
          abuf[(2 * ml + 1) * C + c] = xo[r];
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace jwv
