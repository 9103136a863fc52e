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
#pragma once
#include "jwv_device.hpp"

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

// Forward, tiled.  src = V_{j0-1} (length N); W_j -> wout + (j-1)*ldw;
// V_{j1} -> vout.  Grid: ceil(N/T) blocks.  LDS: (T + S) doubles.
template <int L, int NT, int T, int SMAX, bool FMA>
__global__ __launch_bounds__(NT) void modwt_fwd_tile(const double* __restrict__ src,
                                                     double* __restrict__ wout, int64_t ldw,
                                                     double* __restrict__ vout, int64_t N, int j0,
                                                     int j1, typename MB<L>::Arg tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int MAXP = (T + SMAX + NT - 1) / NT;
  const int nL = MB<L>::n(tp);
  const int S = (nL - 1) * ((1 << j1) - (1 << (j0 - 1)));
  const int64_t t0 = (int64_t)blockIdx.x * T;
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
    if (g < N) vout[g] = lds[S + p];
  }
}

// Forward, one level, direct gather (deep levels).  Grid-stride over N.
template <int L, bool FMA>
__global__ __launch_bounds__(256) void modwt_fwd_level(const double* __restrict__ src,
                                                       double* __restrict__ wrow,
                                                       double* __restrict__ vout, int64_t N,
                                                       int j, typename MB<L>::Arg tp) {
  const int64_t st = (int64_t)1 << (j - 1);
  for (int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x; n < N; n += (int64_t)gridDim.x * 256) {
    double sw = 0.0, sv = 0.0;
#pragma unroll
    for (int l = 0; l < MB<L>::n(tp); ++l) {
      const double v = src[wrap_mod(n - l * st, N)];
      sw = mac<FMA>(sw, v, tp.h[l]);
      sv = mac<FMA>(sv, v, tp.g[l]);
    }
    wrow[n] = sw;
    vout[n] = sv;
  }
}

// Inverse, tiled: levels j1 down to j0.  vsrc = V_{j1}; W_j at coef+(j-1)*ldw;
// output V_{j0-1} -> dst.  LDS: 2 * (T + R) doubles.  The W window of the
// next level is loaded into registers while the current level computes, so
// each block pays one exposed HBM latency instead of one per level.
template <int L, int NT, int T, int SMAX, bool FMA>
__global__ __launch_bounds__(NT) void modwt_inv_tile(const double* __restrict__ vsrc,
                                                     const double* __restrict__ coef, int64_t ldw,
                                                     double* __restrict__ dst, int64_t N, int j0,
                                                     int j1, typename MB<L>::Arg tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int MAXP = (T + SMAX + NT - 1) / NT;
  const int nL = MB<L>::n(tp);
  const int R = (nL - 1) * ((1 << j1) - (1 << (j0 - 1)));
  double* vb = lds;
  double* wb = lds + (T + R);
  const int64_t t0 = (int64_t)blockIdx.x * T;
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
      }
    }
    lds_barrier();
    if (j == j0) {
#pragma unroll
      for (int r = 0; r < MAXP; ++r) {
        const int p = tid + r * NT;
        if (p < T && t0 + p < N) dst[t0 + p] = vv[r];
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

// Inverse, one level, direct gather.
template <int L, bool FMA>
__global__ __launch_bounds__(256) void modwt_inv_level(const double* __restrict__ vsrc,
                                                       const double* __restrict__ wrow,
                                                       double* __restrict__ dst, int64_t N, int j,
                                                       typename MB<L>::Arg tp) {
  const int64_t st = (int64_t)1 << (j - 1);
  for (int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x; n < N; n += (int64_t)gridDim.x * 256) {
    double sa = 0.0, sd = 0.0;
#pragma unroll
    for (int l = 0; l < MB<L>::n(tp); ++l) {
      const int64_t k = wrap_mod(n + l * st, N);
      sa = mac<FMA>(sa, vsrc[k], tp.g[l]);
      sd = mac<FMA>(sd, wrow[k], tp.h[l]);
    }
    dst[n] = sa + sd;
  }
}

}  // namespace jwv
