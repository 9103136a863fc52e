// modwt1_kernels.hpp — MODWT tiles with compile-time geometry (tap count L,
// tile T, fused levels J0..J1 are template arguments).
//
// Same math, summation order and outputs as modwt_fwd_tile / modwt_inv_tile
// (MODWTTransform.java:256-375 with DIRECT circular convolution :677-716; see
// modwt_kernels.hpp), so EXACT results stay bit-identical.  What the
// compile-time form changes, level by level (template recursion over j):
//  * every tap of every output is an LDS read at an IMMEDIATE offset from one
//    per-slot address (taps st = 2^(j-1) apart are constants), so the runtime
//    kernels' per-tap address arithmetic (SALU shifts + VALU adds, ~5e7 SALU
//    instructions per config-5 launch) disappears;
//  * pair slots run branch-free (an invalid slot computes on a clamped index
//    and is masked only at its store), so the W and V accumulation chains of
//    a slot interleave and consecutive slots overlap — the runtime kernels
//    sank the W chain into the store branch and ran the slots one by one;
//  * a slot fence every kFence slots bounds how many slots' reads the
//    compiler hoists (registers), and the lane index is re-read per level
//    (opaque_tid) so no level's addresses are kept live across the others.
#pragma once
#include "modwt_kernels.hpp"

namespace jwv {

#ifndef JWV_MOD1_FENCE
#define JWV_MOD1_FENCE 2
#endif

// ---------------------------------------------------------------- forward
// Window: T outputs + left halo S of V_{J0-1}.  After level j the window
// still carries Sn(j) = (L-1)(2^J1 - 2^j) halo samples; level j's outputs are
// window indices [e0(j), S + T) with e0(j) = S - Sn(j).
template <int L, int T, int J0, int J1>
struct ModFwd1Geo {
  static constexpr int S = (L - 1) * ((1 << J1) - (1 << (J0 - 1)));
  static constexpr int W = T + S;
  static constexpr int Sn(int j) { return (L - 1) * ((1 << J1) - (1 << j)); }
  static constexpr int e0(int j) { return S - Sn(j); }
  static constexpr int nout(int j) { return T + Sn(j); }
  static constexpr int lds_doubles() { return W + 8; }  // + pad and one pair past the end
};

// P2: a lane computes two adjacent outputs (e, e+1) with e of the parity of
// e0(j) (= the parity of S for every level: Sn(j) is even), so the pairs
// tile each level's outputs exactly; the window sits at lds + kPad with kPad
// + e0 even, so every tap pair (e - l*st, e + 1 - l*st) is one 16-B LDS read
// (st = 1: the 10-value run e-8 .. e+1) at a 16-B lane stride, and the W
// pair (t0 - S + e even) is one 16-B store when the rows are 16-B aligned.
template <int L, int NT, int T, int J0, int J1, bool FMA, int j, bool P2>
struct ModFwd1Level {
  static constexpr int kPad = (ModFwd1Geo<L, T, J0, J1>::S & 1) ? 1 : 2;
  __device__ __forceinline__ static void run_p2(const ModwtTaps<L>& tp, double* lds,
                                                double* __restrict__ wout, int64_t ldw,
                                                int64_t t0, int64_t N) {
    using G = ModFwd1Geo<L, T, J0, J1>;
    constexpr int st = 1 << (j - 1);
    constexpr int e0 = G::e0(j), nout = G::nout(j);
    static_assert(((kPad + e0) & 1) == 0 && (nout & 1) == 0, "pairs must tile the outputs");
    constexpr int NP = nout / 2;
    constexpr int R = (NP + NT - 1) / NT;
    const int tid = opaque_tid();
    double* __restrict__ wrow = wout + (int64_t)(j - 1) * ldw + (t0 - G::S);
    // 16-B W stores: row base (j-1)*ldw + t0 - S + e is even for these e
    const bool w16 = (((uintptr_t)wrow + 8 * e0) & 15) == 0;
    double2 vv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = tid + r * NT;
      const bool full = (r + 1) * NT <= NP;
      const int kc = full ? k : (k < NP ? k : NP - 1);
      const int e = e0 + 2 * kc;
      const double* b = lds + kPad + e;  // window index e, 16-B aligned
      double x0[L], x1[L];  // x0[l] = win[e - l*st], x1[l] = win[e + 1 - l*st]
      if constexpr (st == 1) {
        double v[L + 2];
#pragma unroll
        for (int i = 0; i < L + 2; i += 2) {
          const double2 u = *reinterpret_cast<const double2*>(b - L + i);
          v[i] = u.x;
          v[i + 1] = u.y;
        }
#pragma unroll
        for (int l = 0; l < L; ++l) {
          x0[l] = v[L - l];
          x1[l] = v[L + 1 - l];
        }
      } else {
#pragma unroll
        for (int l = 0; l < L; ++l) {
          const double2 u = *reinterpret_cast<const double2*>(b - l * st);
          x0[l] = u.x;
          x1[l] = u.y;
        }
      }
      double sw0 = 0.0, sv0 = 0.0, sw1 = 0.0, sv1 = 0.0;
#pragma unroll
      for (int l = 0; l < L; ++l) {
        sw0 = mac<FMA>(sw0, x0[l], tp.h[l]);
        sv0 = mac<FMA>(sv0, x0[l], tp.g[l]);
        sw1 = mac<FMA>(sw1, x1[l], tp.h[l]);
        sv1 = mac<FMA>(sv1, x1[l], tp.g[l]);
      }
      pin2(sw0, sv0);
      pin2(sw1, sv1);
      vv[r] = make_double2(sv0, sv1);
      const int ee = e0 + 2 * k;  // S has e0's parity: a pair is all halo or all own
      if ((full || k < NP) && e0 + 2 * (r + 1) * NT > G::S && ee >= G::S) {
        const int64_t g = t0 + (ee - G::S);
        if (w16 && g + 1 < N) {
          *reinterpret_cast<double2*>(wrow + ee) = make_double2(sw0, sw1);
        } else {
          if (g < N) wrow[ee] = sw0;
          if (g + 1 < N) wrow[ee + 1] = sw1;
        }
      }
      if constexpr (JWV_MOD1_FENCE > 0)
        if ((r + 1) % JWV_MOD1_FENCE == 0)
          asm volatile("" : "+v"(vv[r].x), "+v"(vv[r].y) :: "memory");
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = tid + r * NT;
      if ((r + 1) * NT <= NP || k < NP)
        *reinterpret_cast<double2*>(lds + kPad + e0 + 2 * k) = vv[r];
    }
    lds_barrier();
    if constexpr (j < J1)
      ModFwd1Level<L, NT, T, J0, J1, FMA, j + 1, P2>::run(tp, lds, wout, ldw, t0, N);
  }
  __device__ __forceinline__ static void run(const ModwtTaps<L>& tp, double* lds,
                                             double* __restrict__ wout, int64_t ldw, int64_t t0,
                                             int64_t N) {
    if constexpr (P2) {
      run_p2(tp, lds, wout, ldw, t0, N);
      return;
    }
    using G = ModFwd1Geo<L, T, J0, J1>;
    constexpr int st = 1 << (j - 1);
    constexpr int e0 = G::e0(j), nout = G::nout(j);
    constexpr int R = (nout + NT - 1) / NT;
    const int tid = opaque_tid();
    // W_j[g] for window index e: g = t0 + e - S (stored only for e >= S)
    double* __restrict__ wrow = wout + (int64_t)(j - 1) * ldw + (t0 - G::S);
    double vv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int p = tid + r * NT;
      const bool full = (r + 1) * NT <= nout;  // compile-time per slot
      const bool v = full || p < nout;
      const int pc = full ? p : (v ? p : nout - 1);
      const double* b = lds + e0 + pc;
      double x[L];
#pragma unroll
      for (int l = 0; l < L; ++l) x[l] = b[-l * st];
      double sw = 0.0, sv = 0.0;
#pragma unroll
      for (int l = 0; l < L; ++l) {
        sw = mac<FMA>(sw, x[l], tp.h[l]);
        sv = mac<FMA>(sv, x[l], tp.g[l]);
      }
      pin2(sw, sv);
      vv[r] = sv;
      const int e = e0 + p;
      // outputs of the tile's own range: e >= S, inside the signal
      if (v && (e0 + (r + 1) * NT - 1 < G::S ? false : e >= G::S) && t0 + (e - G::S) < N)
        wrow[e] = sw;
      if constexpr (JWV_MOD1_FENCE > 0)
        if ((r + 1) % JWV_MOD1_FENCE == 0) asm volatile("" : "+v"(vv[r]) :: "memory");
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int p = tid + r * NT;
      if ((r + 1) * NT <= nout || p < nout) lds[e0 + p] = vv[r];
    }
    lds_barrier();
    if constexpr (j < J1)
      ModFwd1Level<L, NT, T, J0, J1, FMA, j + 1, P2>::run(tp, lds, wout, ldw, t0, N);
  }
};

// src = V_{J0-1} (length N); W_j -> wout + (j-1)*ldw; V_{J1} -> vout.
// Grid: ceil(N/T) blocks (XCD-aware order, xcd_tile).
template <int L, int NT, int T, int J0, int J1, bool FMA, bool P2 = false>
__global__ __launch_bounds__(NT) void modwt_fwd_tile1(const double* __restrict__ src,
                                                      double* __restrict__ wout, int64_t ldw,
                                                      double* __restrict__ vout, int64_t N,
                                                      ModwtTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using G = ModFwd1Geo<L, T, J0, J1>;
  constexpr int MAXP = (G::W + NT - 1) / NT;
  constexpr int pad = P2 ? ModFwd1Level<L, NT, T, J0, J1, FMA, J0, P2>::kPad : 0;
  const int64_t t0 = xcd_tile() * T;
  const bool inside = t0 - G::S >= 0 && t0 + T <= N;  // block-uniform: no wrap
  load_window<1, NT, MAXP>(lds + pad, src, G::W, false, 0, 1, [&](int e) {
    return inside ? t0 - G::S + e : wrap_mod(t0 - G::S + e, N);
  });
  lds_barrier();
  ModFwd1Level<L, NT, T, J0, J1, FMA, J0, P2>::run(tp, lds, wout, ldw, t0, N);
  const int tid = threadIdx.x;
#pragma unroll
  for (int r = 0; r < (T + NT - 1) / NT; ++r) {
    const int p = tid + r * NT;
    if (p < T && t0 + p < N) vout[t0 + p] = lds[pad + G::S + p];
  }
}

// ---------------------------------------------------------------- inverse
// Levels J1 down to J0.  Window of level j: T outputs + right halo Rin(j) =
// (L-1)(2^j - 2^(J0-1)); its outputs carry Rout(j) = Rin(j) - (L-1)2^(j-1).
// LDS: vb (V window, in place) and wb (this level's W window).  The next
// level's W window is fetched into registers while this level computes.
template <int L, int T, int J0, int J1>
struct ModInv1Geo {
  static constexpr int Rin(int j) { return (L - 1) * ((1 << j) - (1 << (J0 - 1))); }
  static constexpr int Rout(int j) { return Rin(j) - (L - 1) * (1 << (j - 1)); }
  static constexpr int Wmax = T + Rin(J1);
  static constexpr int buf() { return (Wmax + 4) & ~1; }  // + one pair read past the end (P2)
  static constexpr int lds_doubles() { return 2 * buf(); }
};

template <int L, int NT, int T, int J0, int J1, bool FMA, int j, bool P2 = false>
struct ModInv1Level {
  using G = ModInv1Geo<L, T, J0, J1>;
  static constexpr int MAXP = (G::Wmax + NT - 1) / NT;
  // fetch the W_j window [t0, t0 + T + Rin(j)) into registers
  __device__ __forceinline__ static void fetch(double (&pw)[MAXP], const double* __restrict__ coef,
                                               int64_t ldw, int64_t t0, int64_t N, bool inside) {
    constexpr int Wn = T + G::Rin(j);
    const double* row = coef + (int64_t)(j - 1) * ldw;
    const int tid = opaque_tid();
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int q = tid + r * NT;
      if (r * NT < Wn && ((r + 1) * NT <= Wn || q < Wn))
        pw[r] = row[inside ? t0 + q : wrap_mod(t0 + q, N)];
    }
  }
  __device__ __forceinline__ static void run(const ModwtTaps<L>& tp, double* vb, double* wb,
                                             double (&pw)[MAXP], const double* __restrict__ coef,
                                             int64_t ldw, double* __restrict__ dst, int64_t t0,
                                             int64_t N, bool inside) {
    constexpr int st = 1 << (j - 1);
    constexpr int Wn = T + G::Rin(j), nout = T + G::Rout(j);
    constexpr int R = (nout + NT - 1) / NT;
    const int tid = opaque_tid();
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int q = tid + r * NT;
      if (r * NT < Wn && ((r + 1) * NT <= Wn || q < Wn)) wb[q] = pw[r];
    }
    lds_barrier();
    if constexpr (j > J0)
      ModInv1Level<L, NT, T, J0, J1, FMA, j - 1, P2>::fetch(pw, coef, ldw, t0, N, inside);
    if constexpr (P2) {
      compute_p2(tp, vb, wb, pw, coef, ldw, dst, t0, N, inside);
      return;
    }
    double vv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int p = tid + r * NT;
      const bool full = (r + 1) * NT <= nout;
      const int pc = full ? p : (p < nout ? p : nout - 1);
      const double* a = vb + pc;
      const double* w = wb + pc;
      double xv[L], xw[L];
#pragma unroll
      for (int l = 0; l < L; ++l) {
        xv[l] = a[l * st];
        xw[l] = w[l * st];
      }
      double sa = 0.0, sd = 0.0;
#pragma unroll
      for (int l = 0; l < L; ++l) {
        sa = mac<FMA>(sa, xv[l], tp.g[l]);
        sd = mac<FMA>(sd, xw[l], tp.h[l]);
      }
      pin2(sa, sd);
      vv[r] = sa + sd;
      if constexpr (JWV_MOD1_FENCE > 0)
        if ((r + 1) % JWV_MOD1_FENCE == 0) asm volatile("" : "+v"(vv[r]) :: "memory");
    }
    lds_barrier();
    if constexpr (j == J0) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int p = tid + r * NT;
        if (r * NT < T && (p < T) && t0 + p < N) dst[t0 + p] = vv[r];
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int p = tid + r * NT;
        if ((r + 1) * NT <= nout || p < nout) vb[p] = vv[r];
      }
      // (the barrier after the next level's W write orders these)
      ModInv1Level<L, NT, T, J0, J1, FMA, j - 1, P2>::run(tp, vb, wb, pw, coef, ldw, dst, t0, N,
                                                          inside);
    }
  }
  // P2: a lane computes the adjacent outputs (p, p+1), p even: every tap pair
  // (p + l*st, p + 1 + l*st) of V and of W is one 16-B LDS read (st = 1: the
  // 10-value runs p .. p+9), 16-B lane stride.  An odd output count leaves
  // one extra output at index nout, past what the next level reads.
  __device__ __forceinline__ static void compute_p2(const ModwtTaps<L>& tp, double* vb, double* wb,
                                                    double (&pw)[MAXP],
                                                    const double* __restrict__ coef, int64_t ldw,
                                                    double* __restrict__ dst, int64_t t0,
                                                    int64_t N, bool inside) {
    constexpr int st = 1 << (j - 1);
    constexpr int nout = T + G::Rout(j);
    constexpr int NP = (nout + 1) / 2;
    constexpr int R = (NP + NT - 1) / NT;
    const int tid = opaque_tid();
    double2 vv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = tid + r * NT;
      const bool full = (r + 1) * NT <= NP;
      const int kc = full ? k : (k < NP ? k : NP - 1);
      const double* a = vb + 2 * kc;
      const double* w = wb + 2 * kc;
      double av0[L], av1[L], aw0[L], aw1[L];
      if constexpr (st == 1) {
        double va[L + 2], vw[L + 2];
#pragma unroll
        for (int i = 0; i < L + 2; i += 2) {
          const double2 u = *reinterpret_cast<const double2*>(a + i);
          const double2 z = *reinterpret_cast<const double2*>(w + i);
          va[i] = u.x;
          va[i + 1] = u.y;
          vw[i] = z.x;
          vw[i + 1] = z.y;
        }
#pragma unroll
        for (int l = 0; l < L; ++l) {
          av0[l] = va[l];
          av1[l] = va[l + 1];
          aw0[l] = vw[l];
          aw1[l] = vw[l + 1];
        }
      } else {
#pragma unroll
        for (int l = 0; l < L; ++l) {
          const double2 u = *reinterpret_cast<const double2*>(a + l * st);
          const double2 z = *reinterpret_cast<const double2*>(w + l * st);
          av0[l] = u.x;
          av1[l] = u.y;
          aw0[l] = z.x;
          aw1[l] = z.y;
        }
      }
      double sa0 = 0.0, sd0 = 0.0, sa1 = 0.0, sd1 = 0.0;
#pragma unroll
      for (int l = 0; l < L; ++l) {
        sa0 = mac<FMA>(sa0, av0[l], tp.g[l]);
        sd0 = mac<FMA>(sd0, aw0[l], tp.h[l]);
        sa1 = mac<FMA>(sa1, av1[l], tp.g[l]);
        sd1 = mac<FMA>(sd1, aw1[l], tp.h[l]);
      }
      pin2(sa0, sd0);
      pin2(sa1, sd1);
      vv[r] = make_double2(sa0 + sd0, sa1 + sd1);
      if constexpr (JWV_MOD1_FENCE > 0)
        if ((r + 1) % JWV_MOD1_FENCE == 0)
          asm volatile("" : "+v"(vv[r].x), "+v"(vv[r].y) :: "memory");
    }
    lds_barrier();
    if constexpr (j == J0) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        const int p = 2 * k;
        if (r * NT * 2 < T && p < T) {
          if (t0 + p + 1 < N && p + 1 < T) {
            *reinterpret_cast<double2*>(dst + t0 + p) = vv[r];
          } else {
            if (t0 + p < N) dst[t0 + p] = vv[r].x;
          }
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        if ((r + 1) * NT <= NP || k < NP) *reinterpret_cast<double2*>(vb + 2 * k) = vv[r];
      }
      ModInv1Level<L, NT, T, J0, J1, FMA, j - 1, P2>::run(tp, vb, wb, pw, coef, ldw, dst, t0, N,
                                                          inside);
    }
  }
};

// vsrc = V_{J1}; W_j at coef + (j-1)*ldw; output V_{J0-1} -> dst.
template <int L, int NT, int T, int J0, int J1, bool FMA, bool P2 = false>
__global__ __launch_bounds__(NT) void modwt_inv_tile1(const double* __restrict__ vsrc,
                                                      const double* __restrict__ coef, int64_t ldw,
                                                      double* __restrict__ dst, int64_t N,
                                                      ModwtTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using G = ModInv1Geo<L, T, J0, J1>;
  using Top = ModInv1Level<L, NT, T, J0, J1, FMA, J1, P2>;
  double* vb = lds;
  double* wb = lds + G::buf();
  const int64_t t0 = xcd_tile() * T;
  const bool inside = t0 + G::Wmax <= N;
  double pw[Top::MAXP];
  load_window<1, NT, Top::MAXP>(vb, vsrc, G::Wmax, false, 0, 1, [&](int e) {
    return inside ? t0 + e : wrap_mod(t0 + e, N);
  });
  Top::fetch(pw, coef, ldw, t0, N, inside);
  Top::run(tp, vb, wb, pw, coef, ldw, dst, t0, N, inside);
}

}  // namespace jwv
