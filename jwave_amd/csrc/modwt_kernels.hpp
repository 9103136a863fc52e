// modwt_kernels.hpp — MODWT pyramid kernels (fp64, any signal length N).
//
// Reference: MODWTTransform.forwardMODWT (MODWTTransform.java:256-306) with
// DIRECT circular convolution (circularConvolve :677-690): for j = 1..J,
//   W_j[n] = sum_m V_{j-1}[(n-m) mod N] hU_j[m],  V_j[n] = ... gU_j[m]
// where hU_j/gU_j are the taps upsampled with 2^(j-1)-1 zeros (:618-630).
// Only the taps l at m = l*2^(j-1) are nonzero; for finite input, adding the
// +-0.0 products of the zero taps to a sum that started at +0.0 never changes
// it, so summing the L nonzero taps in ascending order reproduces the Java
// DIRECT result bit for bit (EXACT mode).  inverseMODWT (:337-375) uses the
// adjoint (circularConvolveAdjoint :703-716, index n+m) and adds the two sums.
//
// Tiled fusion: a tile of T outputs fuses levels j0..j1.  Forward needs a left
// halo S = (L-1)(2^j1 - 2^(j0-1)) of V_{j0-1}; inverse a right halo of the
// same size on V_j1 and on every W_j it reads.  Deep levels whose halo would
// not fit run per level with a direct global gather (modwt_*_level).
//
// Non-finite input: every kernel here runs a fast pass that checks its last
// level's outputs and, in a block whose check fired, a repair pass
// (SLOW = true) with Java's zero-tap NaNs (modwt_nonfinite.hpp).
#pragma once
#include "jwv_device.hpp"
#include "modwt_nonfinite.hpp"

namespace jwv {

template <int L>
struct ModwtTaps {
  double g[L];
  double h[L];
};
struct ModwtAnyTaps {
  double g[kMaxTaps];
  double h[kMaxTaps];
  int32_t L;
  int32_t pad_;
};
// L == 0: runtime tap count (odd / long banks).
template <int L>
struct MB {
  using Arg = ModwtTaps<L>;
  __device__ static constexpr int n(const Arg&) { return L; }
};
template <>
struct MB<0> {
  using Arg = ModwtAnyTaps;
  __device__ static int n(const Arg& a) { return a.L; }
};

__device__ __forceinline__ int64_t wrap_mod(int64_t g, int64_t N) {
  if (g >= 0 && g < N) return g;
  int64_t r = g % N;
  return r < 0 ? r + N : r;
}

// XCD-aware tile order.  Blocks b and b+8 share an XCD (round-robin dealing),
// so plain order puts a tile and the neighbour whose samples form its halo on
// different L2s: every halo is a second HBM read.  Here XCD group x = b % 8
// walks a contiguous run of tiles, [x*q + min(x, r), ...) with q = nblk/8,
// r = nblk%8, so neighbours run side by side on one L2.  Bijective for any
// grid size (N is not a multiple of the tile in general).
__device__ __forceinline__ int64_t xcd_tile() {
  const int nblk = gridDim.x, b = blockIdx.x;
  const int q = nblk >> 3, r = nblk & 7, x = b & 7;
  return (int64_t)x * q + (x < r ? x : r) + (b >> 3);
}

// Forward, tiled.  src = V_{j0-1} (length N); W_j -> wout + (j-1)*ldw;
// V_{j1} -> vout.  Grid: ceil(N/T) blocks.  LDS: (T + S) doubles.
template <int L, int NT, int T, int SMAX, bool FMA, bool SLOW>
__device__ __forceinline__ void modwt_fwd_tile_body(const double* __restrict__ src,
                                                    double* __restrict__ wout, int64_t ldw,
                                                    double* __restrict__ vout, int64_t N, int j0,
                                                    int j1, const typename MB<L>::Arg& tp,
                                                    double* lds, ModNf& nf, bool& bad) {
  constexpr int MAXP = (T + SMAX + NT - 1) / NT;
  const int nL = MB<L>::n(tp);
  const int S = (nL - 1) * ((1 << j1) - (1 << (j0 - 1)));
  const int64_t t0 = xcd_tile() * T;
  const int tid = threadIdx.x;
  const int W = T + S;
  load_window<1, NT, MAXP>(lds, src, W, false, 0, 1,
                           [&](int e) { return wrap_mod(t0 - S + e, N); });
  lds_barrier();
  int Sj = S;  // halo still carried by the level input
  for (int j = j0; j <= j1; ++j) {
    const int st = 1 << (j - 1);
    const int Sn = Sj - (nL - 1) * st;  // halo of this level's output
    const int e0 = S - Sn;              // first output (window index)
    const int nout = T + Sn;
    double* wrow = wout + (int64_t)(j - 1) * ldw;
    // repair: window positions [e0 - C, W) (C = Sj - Sn)
    int lo[2] = {1, 1}, hi[2] = {0, 0};
    if constexpr (SLOW)
      if (st > 1)
        nf_window<1, NT>(nf, e0 - (Sj - Sn), W, [&](int, int q) { return lds[q]; }, lo, hi);
    double vv[MAXP];
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < nout) {
        const int e = e0 + p;
        double sw = 0.0, sv = 0.0;
#pragma unroll
        for (int l = 0; l < MB<L>::n(tp); ++l) {
          const double v = lds[e - l * st];
          sw = mac<FMA>(sw, v, tp.h[l]);
          sv = mac<FMA>(sv, v, tp.g[l]);
        }
        if constexpr (SLOW)
          if (lo[0] <= hi[0] &&
              nf_fwd_zero([&](int q) { return lds[q]; }, e, st, Sj - Sn, lo[0], hi[0]))
            sw = sv = mod_nan();
        vv[r] = sv;
        const int64_t g = t0 + (e - S);
        if (e >= S && g < N) wrow[g] = sw;
      }
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < nout) lds[e0 + p] = vv[r];
    }
    lds_barrier();
    Sj = Sn;
  }
  for (int p = tid; p < T; p += NT) {
    const int64_t g = t0 + p;
    if (g < N) {
      const double v = lds[S + p];
      if constexpr (!SLOW) bad = bad || nonfinite(v);
      vout[g] = v;
    }
  }
}

// (bounds: the fast pass's own occupancy, so the repair pass cannot lower it)
template <int L, int NT, int T, int SMAX, bool FMA>
__global__ __launch_bounds__(NT, L == 16 ? 5 : 6) void modwt_fwd_tile(const double* __restrict__ src,
                                                     double* __restrict__ wout, int64_t ldw,
                                                     double* __restrict__ vout, int64_t N, int j0,
                                                     int j1, typename MB<L>::Arg tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ ModNf nf;
  nf_init(nf);
  bool bad = false;
  modwt_fwd_tile_body<L, NT, T, SMAX, FMA, false>(src, wout, ldw, vout, N, j0, j1, tp, lds, nf,
                                                  bad);
  if (nf_any(nf, bad))
    modwt_fwd_tile_body<L, NT, T, SMAX, FMA, true>(src, wout, ldw, vout, N, j0, j1, tp, lds, nf,
                                                   bad);
}

// Forward, one level, direct gather (deep levels).  A block walks chunks of
// B = max(256, st) consecutive outputs (grid-stride over chunks): the real taps
// of a chunk's outputs then cover every position of their windows, so a
// chunk whose outputs are all finite read only finite values, and the repair
// runs per chunk (its window, C + B positions, scanned from global memory).
__host__ __device__ inline int modwt_level_chunk(int j) {
  return j - 1 > 8 ? 1 << (j - 1) : 256;
}
template <int L, bool FMA, bool SLOW>
__device__ __forceinline__ void modwt_fwd_level_chunk(const double* __restrict__ src,
                                                      double* __restrict__ wrow,
                                                      double* __restrict__ vout, int64_t N, int j,
                                                      const typename MB<L>::Arg& tp, int64_t c0,
                                                      int B, ModNf& nf, bool& bad) {
  const int st = 1 << (j - 1);
  const int C = (MB<L>::n(tp) - 1) * st;
  auto at = [&](int q) { return src[wrap_mod(c0 + q, N)]; };
  int lo[2] = {1, 1}, hi[2] = {0, 0};
  if constexpr (SLOW) nf_window<1, 256>(nf, -C, B, [&](int, int q) { return at(q); }, lo, hi);
  for (int p = threadIdx.x; p < B && c0 + p < N; p += 256) {
    const int64_t n = c0 + p;
    double sw = 0.0, sv = 0.0;
#pragma unroll
    for (int l = 0; l < MB<L>::n(tp); ++l) {
      const double v = src[wrap_mod(n - (int64_t)l * st, N)];
      sw = mac<FMA>(sw, v, tp.h[l]);
      sv = mac<FMA>(sv, v, tp.g[l]);
    }
    if constexpr (SLOW)
      if (lo[0] <= hi[0] && nf_fwd_zero(at, p, st, C, lo[0], hi[0])) sw = sv = mod_nan();
    if constexpr (!SLOW) bad = bad || nonfinite(sv);
    wrow[n] = sw;
    vout[n] = sv;
  }
}
template <int L, bool FMA>
__global__ __launch_bounds__(256, L == 16 ? 6 : 8) void modwt_fwd_level(const double* __restrict__ src,
                                                       double* __restrict__ wrow,
                                                       double* __restrict__ vout, int64_t N,
                                                       int j, typename MB<L>::Arg tp) {
  __shared__ ModNf nf;
  nf_init(nf);
  const int B = modwt_level_chunk(j);
  int gen = 0;
  for (int64_t c0 = (int64_t)blockIdx.x * B; c0 < N; c0 += (int64_t)gridDim.x * B) {
    bool bad = false;
    modwt_fwd_level_chunk<L, FMA, false>(src, wrow, vout, N, j, tp, c0, B, nf, bad);
    if (j > 1 && nf_any(nf, bad, ++gen))
      modwt_fwd_level_chunk<L, FMA, true>(src, wrow, vout, N, j, tp, c0, B, nf, bad);
  }
}

// Inverse, tiled: levels j1 down to j0.  vsrc = V_{j1}; W_j at coef+(j-1)*ldw;
// output V_{j0-1} -> dst.  LDS: 2 * (T + R) doubles.  The W window of the
// next level is loaded into registers while the current level computes, so
// each block pays one exposed HBM latency instead of one per level.
template <int L, int NT, int T, int SMAX, bool FMA, bool SLOW>
__device__ __forceinline__ void modwt_inv_tile_body(const double* __restrict__ vsrc,
                                                    const double* __restrict__ coef, int64_t ldw,
                                                    double* __restrict__ dst, int64_t N, int j0,
                                                    int j1, const typename MB<L>::Arg& tp,
                                                    double* lds, ModNf& nf, bool& bad) {
  constexpr int MAXP = (T + SMAX + NT - 1) / NT;
  const int nL = MB<L>::n(tp);
  const int R = (nL - 1) * ((1 << j1) - (1 << (j0 - 1)));
  double* vb = lds;
  double* wb = lds + (T + R);
  const int64_t t0 = xcd_tile() * T;
  const int tid = threadIdx.x;
  // W window of level j (length T + Rj) -> registers (all loads in flight)
  double pw[MAXP];
  auto fetch_w = [&](int j, int W) {
    const double* wrow = coef + (int64_t)(j - 1) * ldw;
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int q = tid + r * NT;
      pw[r] = q < W ? wrow[wrap_mod(t0 + q, N)] : 0.0;
    }
  };
  load_window<1, NT, MAXP>(vb, vsrc, T + R, false, 0, 1,
                           [&](int e) { return wrap_mod(t0 + e, N); });
  fetch_w(j1, T + R);
  int Rj = R;
  for (int j = j1; j >= j0; --j) {
    const int st = 1 << (j - 1);
    const int Rn = Rj - (nL - 1) * st;
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int q = tid + r * NT;
      if (q < T + Rj) wb[q] = pw[r];
    }
    lds_barrier();
    if (j > j0) fetch_w(j - 1, T + Rn);  // next level's W, in flight during this level
    const int nout = T + Rn;
    // repair: V and W window positions [0, T + Rj)
    int lo[2] = {1, 1}, hi[2] = {0, 0};
    if constexpr (SLOW)
      if (st > 1)
        nf_window<2, NT>(nf, 0, T + Rj, [&](int k, int q) { return k ? wb[q] : vb[q]; }, lo, hi);
    double vv[MAXP];
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int p = tid + r * NT;
      if (p < nout) {
        double sa = 0.0, sd = 0.0;
#pragma unroll
        for (int l = 0; l < MB<L>::n(tp); ++l) {
          sa = mac<FMA>(sa, vb[p + l * st], tp.g[l]);
          sd = mac<FMA>(sd, wb[p + l * st], tp.h[l]);
        }
        vv[r] = sa + sd;
        if constexpr (SLOW)
          if ((lo[0] <= hi[0] &&
               nf_inv_zero([&](int q) { return vb[q]; }, p, st, Rj - Rn, lo[0], hi[0])) ||
              (lo[1] <= hi[1] &&
               nf_inv_zero([&](int q) { return wb[q]; }, p, st, Rj - Rn, lo[1], hi[1])))
            vv[r] = mod_nan();
      }
    }
    lds_barrier();
    if (j == j0) {
#pragma unroll
      for (int r = 0; r < MAXP; ++r) {
        const int p = tid + r * NT;
        if (p < T && t0 + p < N) {
          if constexpr (!SLOW) bad = bad || nonfinite(vv[r]);
          dst[t0 + p] = vv[r];
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < MAXP; ++r) {
        const int p = tid + r * NT;
        if (p < nout) vb[p] = vv[r];
      }
      // (the barrier at the top of the next level orders these writes)
    }
    Rj = Rn;
  }
}

template <int L, int NT, int T, int SMAX, bool FMA>
__global__ __launch_bounds__(NT, 4) void modwt_inv_tile(const double* __restrict__ vsrc,
                                                     const double* __restrict__ coef, int64_t ldw,
                                                     double* __restrict__ dst, int64_t N, int j0,
                                                     int j1, typename MB<L>::Arg tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ ModNf nf;
  nf_init(nf);
  bool bad = false;
  modwt_inv_tile_body<L, NT, T, SMAX, FMA, false>(vsrc, coef, ldw, dst, N, j0, j1, tp, lds, nf,
                                                  bad);
  if (nf_any(nf, bad))
    modwt_inv_tile_body<L, NT, T, SMAX, FMA, true>(vsrc, coef, ldw, dst, N, j0, j1, tp, lds, nf,
                                                   bad);
}

// Inverse, one level, direct gather, in chunks as modwt_fwd_level.
template <int L, bool FMA, bool SLOW>
__device__ __forceinline__ void modwt_inv_level_chunk(const double* __restrict__ vsrc,
                                                      const double* __restrict__ wrow,
                                                      double* __restrict__ dst, int64_t N, int j,
                                                      const typename MB<L>::Arg& tp, int64_t c0,
                                                      int B, ModNf& nf, bool& bad) {
  const int st = 1 << (j - 1);
  const int C = (MB<L>::n(tp) - 1) * st;
  int lo[2] = {1, 1}, hi[2] = {0, 0};
  if constexpr (SLOW)
    nf_window<2, 256>(nf, 0, B + C, [&](int k, int q) {
      const int64_t g = wrap_mod(c0 + q, N);
      return k ? wrow[g] : vsrc[g];
    }, lo, hi);
  for (int p = threadIdx.x; p < B && c0 + p < N; p += 256) {
    const int64_t n = c0 + p;
    double sa = 0.0, sd = 0.0;
#pragma unroll
    for (int l = 0; l < MB<L>::n(tp); ++l) {
      const int64_t k = wrap_mod(n + (int64_t)l * st, N);
      sa = mac<FMA>(sa, vsrc[k], tp.g[l]);
      sd = mac<FMA>(sd, wrow[k], tp.h[l]);
    }
    double v = sa + sd;
    if constexpr (SLOW)
      if ((lo[0] <= hi[0] && nf_inv_zero([&](int q) { return vsrc[wrap_mod(c0 + q, N)]; }, p, st,
                                         C, lo[0], hi[0])) ||
          (lo[1] <= hi[1] && nf_inv_zero([&](int q) { return wrow[wrap_mod(c0 + q, N)]; }, p, st,
                                         C, lo[1], hi[1])))
        v = mod_nan();
    if constexpr (!SLOW) bad = bad || nonfinite(v);
    dst[n] = v;
  }
}
template <int L, bool FMA>
__global__ __launch_bounds__(256, L == 16 ? 6 : 8) void modwt_inv_level(const double* __restrict__ vsrc,
                                                       const double* __restrict__ wrow,
                                                       double* __restrict__ dst, int64_t N, int j,
                                                       typename MB<L>::Arg tp) {
  __shared__ ModNf nf;
  nf_init(nf);
  const int B = modwt_level_chunk(j);
  int gen = 0;
  for (int64_t c0 = (int64_t)blockIdx.x * B; c0 < N; c0 += (int64_t)gridDim.x * B) {
    bool bad = false;
    modwt_inv_level_chunk<L, FMA, false>(vsrc, wrow, dst, N, j, tp, c0, B, nf, bad);
    if (j > 1 && nf_any(nf, bad, ++gen))
      modwt_inv_level_chunk<L, FMA, true>(vsrc, wrow, dst, N, j, tp, c0, B, nf, bad);
  }
}

// ---------------------------------------------------------------------------
// Inverse tile in class-major ("polyphase") LDS layout (compile-time L).
// At level j the taps of output p sit st = 2^(j-1) apart, so each residue
// class r = p mod st is an ordinary stride-1 convolution over m = p div st.
// Both windows of level j (V_j and W_j) are stored class by class: position
// q -> r*M_j + m, so a lane's taps are consecutive doubles at immediate
// offsets for every level (no per-tap address math, no per-level code), and a
// lane computes two outputs m = 2mb, 2mb+1 of one class from L+2 values read
// as (L+2)/2 16-B LDS reads.  Lanes walk classes fastest (u -> r = u mod st,
// mb = u div st) and M_j is padded so that each 16-lane phase of a 16-B read
// hits 16 distinct 16-B bank groups (M_j/2 odd for st >= 16, M_j/2 = 16/st
// mod 16 below).  Level j's outputs land directly in level j-1's layout
// (class r' = r mod st/2, m' = 2m + r div (st/2)).  Same math and order as
// modwt_inv_tile: each output sums its L taps of V and of W in ascending order
// from 0.0, then adds the two sums.
struct ModCm {
  // class length of level sh (input window Win, output window Wout)
  __host__ __device__ static int M(int Win, int Wout, int sh, int L) {
    const int st = 1 << sh;
    const int Min = (Win + st - 1) >> sh;
    const int nmb = (((Wout + st - 1) >> sh) + 1) >> 1;
    int m = Min > 2 * nmb + L ? Min : 2 * nmb + L;
    int h = (m + 1) >> 1;
    if (st >= 16) {
      h |= 1;
    } else {
      const int want = 16 / st;
      h += ((want - h) % 16 + 16) % 16;
    }
    return 2 * h;
  }
  __host__ __device__ static int nmb(int Wout, int sh) {
    return ((((Wout + (1 << sh) - 1) >> sh) + 1) >> 1);
  }
  // doubles per buffer over levels j0..j1 (host: LDS size)
  __host__ static int buf(int T, int L, int j0, int j1) {
    int b = 0;
    for (int j = j1; j >= j0; --j) {
      const int Rj = (L - 1) * ((1 << j) - (1 << (j0 - 1)));
      const int Rn = Rj - (L - 1) * (1 << (j - 1));
      const int v = (1 << (j - 1)) * M(T + Rj, T + Rn, j - 1, L);
      b = v > b ? v : b;
    }
    return (b + 1) & ~1;
  }
};

template <int L, int NT, int T, int SMAX, bool FMA, bool SLOW>
__device__ __forceinline__ void modwt_inv_tile_cm_body(const double* __restrict__ vsrc,
                                                       const double* __restrict__ coef,
                                                       int64_t ldw, double* __restrict__ dst,
                                                       int64_t N, int j0, int j1, int buf,
                                                       const ModwtTaps<L>& tp, double* lds,
                                                       ModNf& nf, bool& bad) {
  constexpr int MAXP = (T + SMAX + NT - 1) / NT;
  constexpr int MAXI = (T + SMAX) / (2 * NT) + 2;  // item slots: nmb*st <= W/2 + st
  const int R = (L - 1) * ((1 << j1) - (1 << (j0 - 1)));
  double* vb = lds;
  double* wb = lds + buf;
  const int64_t t0 = xcd_tile() * T;
  const int tid = threadIdx.x;
  const bool inside = t0 + T + R <= N;  // block-uniform: no wrap
  auto gidx = [&](int q) { return inside ? t0 + q : wrap_mod(t0 + q, N); };
  // the next level's W window, in flight in registers during a level
  double pw[MAXP];
  auto fetch = [&](const double* row, int W) {
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int q = tid + r * NT;
      if (q < W) pw[r] = row[gidx(q)];
    }
  };
  // registers -> class-major layout (sh, class length M)
  auto scatter = [&](double* b, int W, int sh, int M) {
    const int msk = (1 << sh) - 1;
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int q = tid + r * NT;
      if (q < W) b[(q & msk) * M + (q >> sh)] = pw[r];
    }
  };
  auto halo = [&](int j) { return (L - 1) * ((1 << j) - (1 << (j0 - 1))); };
  {
    fetch(vsrc, T + R);
    const int sh = j1 - 1;
    scatter(vb, T + R, sh, ModCm::M(T + R, T + halo(j1 - 1), sh, L));
  }
  fetch(coef + (int64_t)(j1 - 1) * ldw, T + R);
  for (int j = j1; j >= j0; --j) {
    const int sh = j - 1, st = 1 << sh;
    const int Win = T + halo(j), Wout = T + halo(j - 1);
    const int M = ModCm::M(Win, Wout, sh, L);
    scatter(wb, Win, sh, M);
    lds_barrier();
    if (j > j0) fetch(coef + (int64_t)(j - 2) * ldw, Wout);  // next level's W in flight
    const int nmb = ModCm::nmb(Wout, sh);
    const int nitems = nmb << sh;
    // repair: V and W window positions [0, Win), class-major
    const int msk = st - 1, C = (L - 1) * st;
    auto atv = [&](int q) { return vb[(q & msk) * M + (q >> sh)]; };
    auto atw = [&](int q) { return wb[(q & msk) * M + (q >> sh)]; };
    int lo[2] = {1, 1}, hi[2] = {0, 0};
    if constexpr (SLOW)
      if (st > 1)
        nf_window<2, NT>(nf, 0, Win, [&](int k, int q) { return k ? atw(q) : atv(q); }, lo, hi);
    auto nan_at = [&](int p) {
      return (lo[0] <= hi[0] && nf_inv_zero(atv, p, st, C, lo[0], hi[0])) ||
             (lo[1] <= hi[1] && nf_inv_zero(atw, p, st, C, lo[1], hi[1]));
    };
    double o0[MAXI], o1[MAXI];
#pragma unroll
    for (int k = 0; k < MAXI; ++k) {
      const int u = tid + k * NT;
      if ((k + 1) * NT <= nitems || u < nitems) {
        const int base = (u & (st - 1)) * M + 2 * (u >> sh);
        const double* va = vb + base;
        const double* wa = wb + base;
        double xv[L + 2], xw[L + 2];
#pragma unroll
        for (int e = 0; e < L + 2; e += 2) {
          const double2 a = *reinterpret_cast<const double2*>(va + e);
          const double2 w = *reinterpret_cast<const double2*>(wa + e);
          xv[e] = a.x;
          xv[e + 1] = a.y;
          xw[e] = w.x;
          xw[e + 1] = w.y;
        }
        double sa0 = 0.0, sd0 = 0.0, sa1 = 0.0, sd1 = 0.0;
#pragma unroll
        for (int l = 0; l < L; ++l) {
          sa0 = mac<FMA>(sa0, xv[l], tp.g[l]);
          sd0 = mac<FMA>(sd0, xw[l], tp.h[l]);
          sa1 = mac<FMA>(sa1, xv[l + 1], tp.g[l]);
          sd1 = mac<FMA>(sd1, xw[l + 1], tp.h[l]);
        }
        o0[k] = sa0 + sd0;
        o1[k] = sa1 + sd1;
        if constexpr (SLOW) {
          const int p = (u & (st - 1)) + ((2 * (u >> sh)) << sh);
          if (nan_at(p)) o0[k] = mod_nan();
          if (nan_at(p + st)) o1[k] = mod_nan();
        }
      }
    }
    lds_barrier();
    if (j == j0) {
#pragma unroll
      for (int k = 0; k < MAXI; ++k) {
        const int u = tid + k * NT;
        if ((k + 1) * NT <= nitems || u < nitems) {
          const int p = (u & (st - 1)) + ((2 * (u >> sh)) << sh);
          if (p < T && t0 + p < N) {
            if constexpr (!SLOW) bad = bad || nonfinite(o0[k]);
            dst[t0 + p] = o0[k];
          }
          if (p + st < T && t0 + p + st < N) {
            if constexpr (!SLOW) bad = bad || nonfinite(o1[k]);
            dst[t0 + p + st] = o1[k];
          }
        }
      }
    } else {
      // level j-1 layout: class r' = r mod st/2, m' = 2m + (r >= st/2)
      const int shn = sh - 1;
      const int Mn = ModCm::M(Wout, T + halo(j - 2), shn, L);
#pragma unroll
      for (int k = 0; k < MAXI; ++k) {
        const int u = tid + k * NT;
        if ((k + 1) * NT <= nitems || u < nitems) {
          const int r = u & (st - 1), m = 2 * (u >> sh);
          const int p = r + (m << sh);
          double* ob = vb + (r & ((st >> 1) - 1)) * Mn + 2 * m + (r >> shn);
          if (p < Wout) ob[0] = o0[k];
          if (p + st < Wout) ob[2] = o1[k];
        }
      }
      // (the barrier after the next level's W scatter orders these writes)
    }
  }
}

template <int L, int NT, int T, int SMAX, bool FMA>
__global__ __launch_bounds__(NT) void modwt_inv_tile_cm(const double* __restrict__ vsrc,
                                                        const double* __restrict__ coef,
                                                        int64_t ldw, double* __restrict__ dst,
                                                        int64_t N, int j0, int j1, int buf,
                                                        ModwtTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ ModNf nf;
  nf_init(nf);
  bool bad = false;
  modwt_inv_tile_cm_body<L, NT, T, SMAX, FMA, false>(vsrc, coef, ldw, dst, N, j0, j1, buf, tp,
                                                     lds, nf, bad);
  if (nf_any(nf, bad))
    modwt_inv_tile_cm_body<L, NT, T, SMAX, FMA, true>(vsrc, coef, ldw, dst, N, j0, j1, buf, tp,
                                                      lds, nf, bad);
}

}  // namespace jwv
