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

// Couples with the products of G taps / terms issued ahead of their adds
// (fwd_couple_pipe, rev_couple_pipe; 0 = fwd_pair / rev_pair per pair, the
// multiply and its dependent add adjacent): the WPT tiles (config 4: 4.47-4.52
// -> 4.42-4.43 ms/step, r05j).  The same forms in the FWT tiles and the MODWT
// sums measured no change (r05l / r05k) and are not used there.
#ifndef JWV_WPT_FPIPE
#define JWV_WPT_FPIPE 2
#endif
#ifndef JWV_WPT_RPIPE
#define JWV_WPT_RPIPE 2
#endif
// ZS = false ("no zero start", EXACT only): a sum starts at its first
// product instead of adding it to +0.0.  The two folds differ only in the
// sign of a zero running sum (start +0.0: never -0 under round-to-nearest;
// first product: possibly -0), so every non-zero value is identical and a
// -0 can only stand where Java holds +0.  Products of such a zero are zeros
// again, so the same holds for every later level fed from it, and a level
// that starts from +0.0 (ZS = true) restores Java's sign.  Used for the WPT
// tiles' LDS-only levels; the level that writes HBM keeps ZS = true.
// A couple's four sums (pairs at x and x + 2, analysis lo / hi) with the
// products of G taps issued ahead of their adds: per group 4G independent
// multiplies, then the 4G adds in the per-output order (j ascending), so no
// add waits on the multiply issued just before it and the four chains
// alternate.  Same operations and order per output as fwd_pair (bit-exact).
template <int L, bool FMA, int G, bool ZS = true>
__device__ __forceinline__ void fwd_couple_pipe(const FwdTaps<L>& tp, const double* x,
                                                double& a0, double& d0, double& a1, double& d1) {
  static_assert(L % G == 0, "tap groups");
  double sa0 = 0.0, sd0 = 0.0, sa1 = 0.0, sd1 = 0.0;
#pragma unroll
  for (int j0 = 0; j0 < L; j0 += G) {
    double pa0[G], pd0[G], pa1[G], pd1[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      pa0[g] = x[j0 + g] * tp.lo[j0 + g];
      pd0[g] = x[j0 + g] * tp.hi[j0 + g];
      pa1[g] = x[j0 + g + 2] * tp.lo[j0 + g];
      pd1[g] = x[j0 + g + 2] * tp.hi[j0 + g];
    }
#pragma unroll
    for (int g = 0; g < G; ++g) asm volatile("" : "+v"(pa0[g]), "+v"(pd0[g]), "+v"(pa1[g]), "+v"(pd1[g]));
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if constexpr (FMA) {  // FMA mode keeps its fused form (its own order: fwd_pair's)
        sa0 = __builtin_fma(x[j0 + g], tp.lo[j0 + g], sa0);
        sd0 = __builtin_fma(x[j0 + g], tp.hi[j0 + g], sd0);
        sa1 = __builtin_fma(x[j0 + g + 2], tp.lo[j0 + g], sa1);
        sd1 = __builtin_fma(x[j0 + g + 2], tp.hi[j0 + g], sd1);
      } else if (!ZS && j0 == 0 && g == 0) {
        sa0 = pa0[0];
        sd0 = pd0[0];
        sa1 = pa1[0];
        sd1 = pd1[0];
      } else {
        sa0 = sa0 + pa0[g];
        sd0 = sd0 + pd0[g];
        sa1 = sa1 + pa1[g];
        sd1 = sd1 + pd1[g];
      }
    }
    asm volatile("" : "+v"(sa0), "+v"(sd0), "+v"(sa1), "+v"(sd1));
  }
  a0 = sa0;
  d0 = sd0;
  a1 = sa1;
  d1 = sd1;
}

// fwd_couple_pipe over three adjacent pairs (x, x + 2, x + 4; six sums): the
// WPT forward trio tiles (wpt1_kernels.hpp).  Same per-output operations and
// order as fwd_pair (bit-exact); FMA mode keeps its fused form.
template <int L, bool FMA, int G, bool ZS = true>
__device__ __forceinline__ void fwd_trio_pipe(const FwdTaps<L>& tp, const double* x, double* a,
                                              double* d) {
  static_assert(L % G == 0, "tap groups");
  double sa[3] = {0.0, 0.0, 0.0}, sd[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int j0 = 0; j0 < L; j0 += G) {
    double pa[3][G], pd[3][G];
    if constexpr (!FMA) {
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          pa[p][g] = x[j0 + g + 2 * p] * tp.lo[j0 + g];
          pd[p][g] = x[j0 + g + 2 * p] * tp.hi[j0 + g];
        }
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int p = 0; p < 3; ++p) asm volatile("" : "+v"(pa[p][g]), "+v"(pd[p][g]));
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        if constexpr (FMA) {
          sa[p] = __builtin_fma(x[j0 + g + 2 * p], tp.lo[j0 + g], sa[p]);
          sd[p] = __builtin_fma(x[j0 + g + 2 * p], tp.hi[j0 + g], sd[p]);
        } else if (!ZS && j0 == 0 && g == 0) {
          sa[p] = pa[p][0];
          sd[p] = pd[p][0];
        } else {
          sa[p] = sa[p] + pa[p][g];
          sd[p] = sd[p] + pd[p][g];
        }
      }
#pragma unroll
    for (int p = 0; p < 3; ++p) asm volatile("" : "+v"(sa[p]), "+v"(sd[p]));
  }
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    a[p] = sa[p];
    d[p] = sd[p];
  }
}

// A reverse couple (pairs m, m+1; A/D point at a[m], d[m]) with the products
// of G terms issued ahead of their adds:
// per group 8G independent multiplies (a*lor, d*hir of both pairs, even and
// odd outputs), then the 4G term sums a*lor + d*hir, then the 4G accumulator
// adds; each output keeps its order (q descending) and its operations
// (EXACT only; bit-exact with rev_pair / rev_couple_ilv; ZS as above).
template <int L, int G, bool ZS = true>
__device__ __forceinline__ void rev_couple_pipe(const RevTaps<L>& tp, const double* A,
                                                const double* D, double& e0, double& o0,
                                                double& e1, double& o1) {
  constexpr int Q = L / 2;
  static_assert(L % 2 == 0 && Q % G == 0, "even bank, whole term groups");
  double se0 = 0.0, so0 = 0.0, se1 = 0.0, so1 = 0.0;
#pragma unroll
  for (int q0 = Q - 1; q0 >= 0; q0 -= G) {
    double ta0[G], ua0[G], ta1[G], ua1[G], tb0[G], ub0[G], tb1[G], ub1[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int q = q0 - g;
      const double a0 = A[-q], d0 = D[-q], a1 = A[1 - q], d1 = D[1 - q];
      ta0[g] = a0 * tp.lo_r[2 * q];
      ua0[g] = d0 * tp.hi_r[2 * q];
      ta1[g] = a1 * tp.lo_r[2 * q];
      ua1[g] = d1 * tp.hi_r[2 * q];
      tb0[g] = a0 * tp.lo_r[2 * q + 1];
      ub0[g] = d0 * tp.hi_r[2 * q + 1];
      tb1[g] = a1 * tp.lo_r[2 * q + 1];
      ub1[g] = d1 * tp.hi_r[2 * q + 1];
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      asm volatile("" : "+v"(ta0[g]), "+v"(ua0[g]), "+v"(ta1[g]), "+v"(ua1[g]));
      asm volatile("" : "+v"(tb0[g]), "+v"(ub0[g]), "+v"(tb1[g]), "+v"(ub1[g]));
    }
    double ve0[G], ve1[G], vo0[G], vo1[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      ve0[g] = ta0[g] + ua0[g];
      ve1[g] = ta1[g] + ua1[g];
      vo0[g] = tb0[g] + ub0[g];
      vo1[g] = tb1[g] + ub1[g];
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (!ZS && q0 == Q - 1 && g == 0) {
        se0 = ve0[0];
        se1 = ve1[0];
        so0 = vo0[0];
        so1 = vo1[0];
      } else {
        se0 += ve0[g];
        se1 += ve1[g];
        so0 += vo0[g];
        so1 += vo1[g];
      }
    }
    asm volatile("" : "+v"(se0), "+v"(so0), "+v"(se1), "+v"(so1));
  }
  e0 = se0;
  o0 = so0;
  e1 = se1;
  o1 = so1;
}

// ------------------------------------------------------------ reverse pair
// Outputs x[2m] (even taps j=2q) and x[2m+1] (odd taps j=2q+1) of one
// synthesis level of size h (half = h/2 pairs).  Term q reads a[m-q], d[m-q]
// (indices mod half).  Scatter order of Wavelet.reverse = i ascending: the
// non-wrapped terms (q <= mg) in q-descending order first, then the wrapped
// ones (q > mg) in q-descending order.  Valid for h >= L (at most one wrap);
// smaller levels use rev_level_small.  A(q)/D(q) return a[m-q], d[m-q].
// Array-head case of rev_pair (mg < Q-1, only the first pairs of a level):
// non-wrapped terms (q <= mg) q-descending, then wrapped ones (q > mg).
// Kept out of line so the unrolled interior loops stay small.  A/D point at
// a[m], d[m] (stride `st`), so term q reads A[-q*st].
// A(q), D(q) return a[m-q], d[m-q] (wrapped by the caller).  Inlined with
// static tap indices (a call would need a stack frame = scratch).
template <int L, bool FMA, typename GA, typename GD>
__device__ __forceinline__ void rev_pair_head(const typename FB<L>::Rev& tp, int mg, GA A, GD D,
                                              double& xe, double& xo) {
  constexpr int QM = (LMax<L>::v + 1) / 2;
  const int nt = FB<L>::nr(tp);
  const int qe = (nt + 1) >> 1, qo = nt >> 1;
  double se = 0.0, so = 0.0;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int q = QM - 1; q >= 0; --q) {
      if (q >= qe || (q <= mg) != (pass == 0)) continue;
      double t = A(q) * FB<L>::lor(tp, 2 * q);
      t = mac<FMA>(t, D(q), FB<L>::hir(tp, 2 * q));
      se += FB<L>::scale(t, tp);
    }
  }
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int q = QM - 1; q >= 0; --q) {
      if (q >= qo || (q <= mg) != (pass == 0)) continue;
      double t = A(q) * FB<L>::lor(tp, 2 * q + 1);
      t = mac<FMA>(t, D(q), FB<L>::hir(tp, 2 * q + 1));
      so += FB<L>::scale(t, tp);
    }
  }
  xe = se;
  xo = so;
}

// Outputs x[2m] (even taps j=2q) and x[2m+1] (odd taps j=2q+1) of one
// synthesis level of size h >= L (at most one wrap).  Term q reads a[m-q],
// d[m-q] = A[-q*st], D[-q*st] (the caller's window already holds the periodic
// extension).  Scatter order of Wavelet.reverse = i ascending = q descending
// for interior pairs (mg >= Q-1, checked by the caller: head pairs go to
// rev_pair_head).
template <int L, bool FMA>
__device__ __forceinline__ void rev_pair(const typename FB<L>::Rev& tp, const double* A,
                                         const double* D, int st, double& xe, double& xo) {
  const int nt = FB<L>::nr(tp);
  const int qe = (nt + 1) >> 1;
  double se = 0.0, so = 0.0;
  if constexpr (FB<L>::kStatic) {
    constexpr int QE = (L + 1) / 2, QO = L / 2;
#pragma unroll
    for (int q = QE - 1; q >= 0; --q) {
      const double a = A[-q * st], d = D[-q * st];
      double t = a * FB<L>::lor(tp, 2 * q);
      se += mac<FMA>(t, d, FB<L>::hir(tp, 2 * q));
      if (q < QO) {
        double u = a * FB<L>::lor(tp, 2 * q + 1);
        so += mac<FMA>(u, d, FB<L>::hir(tp, 2 * q + 1));
      }
    }
  } else {
    const int qo = nt >> 1;
    for (int q = qe - 1; q >= 0; --q) {
      const double a = A[-q * st], d = D[-q * st];
      double t = a * FB<L>::lor(tp, 2 * q);
      se += FB<L>::scale(mac<FMA>(t, d, FB<L>::hir(tp, 2 * q)), tp);
      if (q < qo) {
        double u = a * FB<L>::lor(tp, 2 * q + 1);
        so += FB<L>::scale(mac<FMA>(u, d, FB<L>::hir(tp, 2 * q + 1)), tp);
      }
    }
  }
  xe = se;  // started at +0.0 like arrTime[k] (Wavelet.java:282)
  xo = so;
}

// Interior and array-head pairs in one branch-free form (compiled-in even L):
// rev_pair_head's order (q = mg..0, then Q-1..mg+1) is the interior order
// (q = Q-1..0) rotated, over the same per-term values.  r = mg for a head
// pair (mg < Q-1), r = Q-1 for every other pair; the rotation is a register
// select, so a wave holding both kinds of pair runs ONE path (rev_pair +
// rev_pair_head under divergence run both, and every level of a resident
// reverse has its head lanes in wave 0).  Results are bit-identical to
// rev_pair / rev_pair_head.
template <int L, bool FMA, typename GA, typename GD>
__device__ __forceinline__ void rev_pair_rot(const RevTaps<L>& tp, GA A, GD D, int r, double& xe,
                                             double& xo) {
  static_assert(L >= 2 && (L & 1) == 0, "compiled-in even banks only");
  constexpr int Q = L / 2;
  double te[Q], to[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const double a = A(q), d = D(q);
    te[q] = mac<FMA>(a * tp.lo_r[2 * q], d, tp.hi_r[2 * q]);
    to[q] = mac<FMA>(a * tp.lo_r[2 * q + 1], d, tp.hi_r[2 * q + 1]);
  }
  double se = 0.0, so = 0.0;
#pragma unroll
  for (int k = 0; k < Q; ++k) {
    const int q = (r - k) & (Q - 1);
    double ve = te[0], vo = to[0];
#pragma unroll
    for (int i = 1; i < Q; ++i) {
      ve = q == i ? te[i] : ve;
      vo = q == i ? to[i] : vo;
    }
    se += ve;
    so += vo;
  }
  xe = se;
  xo = so;
}

// The same rotated order with the per-term values computed in that order:
// q = (r - k) mod Q is a runtime index, so the inputs come from LDS (A, D)
// and the taps from an LDS copy tl (stage_rev_taps) instead of a Q x Q
// register select.  Bit-identical to rev_pair_rot.  For the array-head lanes
// only: interior pairs keep rev_pair.
template <int L, bool FMA, typename GA, typename GD>
__device__ __forceinline__ void rev_pair_rot_t(const double* tl, GA A, GD D, int r, double& xe,
                                               double& xo) {
  static_assert(L >= 2 && (L & 1) == 0, "compiled-in even banks only");
  constexpr int Q = L / 2;
  double se = 0.0, so = 0.0;
#pragma unroll
  for (int k = 0; k < Q; ++k) {
    const int q = (r - k) & (Q - 1);
    const double a = A(q), d = D(q);
    const double2 lo = *reinterpret_cast<const double2*>(tl + 4 * q);
    const double2 hi = *reinterpret_cast<const double2*>(tl + 4 * q + 2);
    se += mac<FMA>(a * lo.x, d, hi.x);
    so += mac<FMA>(a * lo.y, d, hi.y);
  }
  xe = se;
  xo = so;
}
// tl[4q .. 4q+3] = lo_r[2q], lo_r[2q+1], hi_r[2q], hi_r[2q+1] (2L doubles);
// thread 0 writes, the caller's next block barrier publishes.
template <int L>
__device__ __forceinline__ void stage_rev_taps(const RevTaps<L>& tp, double* tl) {
  if (threadIdx.x == 0) {
#pragma unroll
    for (int q = 0; q < L / 2; ++q) {
      *reinterpret_cast<double2*>(tl + 4 * q) = make_double2(tp.lo_r[2 * q], tp.lo_r[2 * q + 1]);
      *reinterpret_cast<double2*>(tl + 4 * q + 2) =
          make_double2(tp.hi_r[2 * q], tp.hi_r[2 * q + 1]);
    }
  }
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

// rev_small for compiled-in banks: all H outputs of a level of size H < L at
// compile-time H (Wavelet.reverse's scatter order, i then j ascending, each
// output a fixed chain), then the pair (2m, 2m+1) by register select.  A, D:
// the level's a and d values at stride `stride`.
template <int L, bool FMA, int H>
__device__ __forceinline__ void rev_small_cH(const RevTaps<L>& tp, const double* A,
                                             const double* D, int stride, int m, double& xe,
                                             double& xo) {
  double x[H];
#pragma unroll
  for (int k = 0; k < H; ++k) x[k] = 0.0;
#pragma unroll
  for (int i = 0; i < H / 2; ++i) {
    const double a = A[i * stride], d = D[i * stride];
#pragma unroll
    for (int j = 0; j < L; ++j) {
      double t = a * tp.lo_r[j];
      t = mac<FMA>(t, d, tp.hi_r[j]);
      x[(2 * i + j) & (H - 1)] += t;
    }
  }
  xe = x[0];
  xo = x[1];
#pragma unroll
  for (int q = 1; q < H / 2; ++q)
    if (m == q) {
      xe = x[2 * q];
      xo = x[2 * q + 1];
    }
}
template <int L, bool FMA>
__device__ __forceinline__ void rev_small_c(const RevTaps<L>& tp, const double* A, const double* D,
                                            int stride, int h, int m, double& xe, double& xo) {
  if constexpr (L > 2) if (h == 2) return rev_small_cH<L, FMA, 2>(tp, A, D, stride, m, xe, xo);
  if constexpr (L > 4) if (h == 4) return rev_small_cH<L, FMA, 4>(tp, A, D, stride, m, xe, xo);
  if constexpr (L > 8) if (h == 8) return rev_small_cH<L, FMA, 8>(tp, A, D, stride, m, xe, xo);
  if constexpr (L > 16) if (h == 16) return rev_small_cH<L, FMA, 16>(tp, A, D, stride, m, xe, xo);
  xe = xo = 0.0;  // unreachable: h < L, both powers of two
}

// ====================================================================
// Forward, resident.  Grid: one block per (outer o, column slab cb).
// src: level input of length h0 (view sv); dst: coefficient array (view dv):
// level of size h writes details to dst[h/2 .. h), the final approximation to
// dst[0 .. h_end).  nlev >= 0 levels; LDS = h0*C doubles.  Levels with more
// than 64 pairs run block-wide; the rest run on wave 0 alone (no block
// barriers: a deep tail is latency-bound).
// ====================================================================
template <int L, int C, int NT, int CAP, bool FMA>
__device__ __forceinline__ void fwt_fwd_res_blk(const double* __restrict__ s, AxisView sv,
    double* __restrict__ y, AxisView dv, int h0, int nlev, int c0, int inner, int dma,
    const typename FB<L>::Fwd& tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int MAXP = (CAP / 2 * C + NT - 1) / NT;
  constexpr int MAXU = (CAP * C + NT - 1) / NT;
  const int tid = threadIdx.x;
  JWV_STAMP(0);
  load_window<C, NT, MAXU>(lds, s, h0, dma != 0, c0, inner,
                           [&](int e) { return (int64_t)e * sv.s_len; });
  dma_fence_barrier();
  JWV_STAMP(1);

  int h = h0, lev = 0;
  for (; lev < nlev && (h >> 1) * C > 64; ++lev, h >>= 1) {
    JWV_STAMP(2 + lev);
    const int half = h >> 1, np = half * C, msk = h - 1;
    double av[MAXP];
    for_pairs<MAXP, NT>(np, [&](int r, int p, bool v) {
      const int i = p / C, c = p % C;
      double a, d;
      fwd_pair<L, FMA>(tp, [&](int j) { return lds[((2 * i + j) & msk) * C + c]; }, a, d);
      av[r] = a;
      if (v && c0 + c < inner) y[(int64_t)(half + i) * dv.s_len + c] = d;
    });
    lds_barrier();
    for_pairs<MAXP, NT>(np, [&](int r, int p, bool v) {
      if (v) lds[p] = av[r];
    });
    lds_barrier();
  }
  if (lev < nlev) {  // small levels: wave 0 only
    if (tid < 64) {
      int hh = h;
      for (int lv = lev; lv < nlev; ++lv, hh >>= 1) {
        const int half = hh >> 1, np = half * C, msk = hh - 1;
        const bool v = tid < np;
        const int p = v ? tid : np - 1;
        const int i = p / C, c = p % C;
        double a, d;
        fwd_pair<L, FMA>(tp, [&](int j) { return lds[((2 * i + j) & msk) * C + c]; }, a, d);
        if (v && c0 + c < inner) y[(int64_t)(half + i) * dv.s_len + c] = d;
        wave_lds_sync();
        if (v) lds[p] = a;
        wave_lds_sync();
      }
    }
    h >>= (nlev - lev);
    JWV_STAMP(40);
    lds_barrier();
  }
  JWV_STAMP(41);
  for (int q = tid; q < h * C; q += NT) {
    const int i = q / C, c = q % C;
    if (c0 + c < inner) y[(int64_t)i * dv.s_len + c] = lds[q];
  }
  JWV_STAMP(42);
}

// Slab of block b for the resident column passes: with 8-column slabs the
// two halves of every 128-B row line belong to slabs 2k and 2k+1; blocks b
// and b + 8 share an XCD (round-robin dealing) and start together, so they
// take a slab pair and the line is fetched from HBM once (bijective for
// grids of whole 16-block groups; otherwise the plain order).
template <int C>
__device__ __forceinline__ int64_t res_slab_block(int64_t b) {
  if constexpr (C == 8) {
    if ((gridDim.x & 15) == 0) return ((b >> 4) * 8 + (b & 7)) * 2 + ((b >> 3) & 1);
  }
  return b;
}

template <int L, int C, int NT, int CAP, bool FMA>
__global__ __launch_bounds__(NT) void fwt_fwd_res(const double* __restrict__ src, AxisView sv,
    double* __restrict__ dst, AxisView dv, int h0, int nlev, int inner, int dma,
    typename FB<L>::Fwd tp) {
  const int ncb = (inner + C - 1) / C;
  const int64_t bs = res_slab_block<C>(blockIdx.x);
  const int64_t o = bs / ncb;
  const int c0 = (int)(bs % ncb) * C;
  const double* s = src + view_base(sv, o) + c0;
  double* y = dst + view_base(dv, o) + c0;
  fwt_fwd_res_blk<L, C, NT, CAP, FMA>(s, sv, y, dv, h0, nlev, c0, inner, dma, tp);
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
    for_pairs<MAXP, NT>(np, [&](int r, int p, bool v) {
      const int i = p / C, c = p % C;
      double a, d;
      fwd_pair<L, FMA>(tp, [&](int j) { return lds[(2 * i + j) * C + c]; }, a, d);
      av[r] = a;
      if (v && i < own && c0 + c < inner) y[(dbase + i) * dv.s_len + c] = d;
    });
    lds_barrier();
    for_pairs<MAXP, NT>(np, [&](int r, int p, bool v) {
      if (v) lds[p] = av[r];
    });
    lds_barrier();
    m = mo;
    hl >>= 1;
  }
  const int own = T >> K;
  for (int q = tid; q < own * C; q += NT) {
    const int i = q / C, c = q % C;
    if (c0 + c < inner) ya[((int64_t)t * own + i) * av_.s_len + c] = lds[q];
  }
}

// One synthesis pair at global pair index m (m < qe-1: array head, whose
// terms are summed in scatter order by rev_pair_head).  A/D point at the LDS
// copies of a[m], d[m] (stride C); Aw(q)/Dw(q) give a[m-q]/d[m-q] wrapped.
// The interior formula is always evaluated (on a clamped index for head
// pairs) so that the common path stays branch-free.
template <int L, bool FMA, typename AW, typename DW>
__device__ __forceinline__ void rev_pair_any(const typename FB<L>::Rev& tp, int m, int qe,
                                             const double* A, const double* D, int C,
                                             AW Aw, DW Dw, double& xe, double& xo) {
  const int sh = m < qe - 1 ? (qe - 1 - m) : 0;  // clamp for head pairs
  rev_pair<L, FMA>(tp, A + sh * C, D + sh * C, C, xe, xo);
  if (sh) rev_pair_head<L, FMA>(tp, m, Aw, Dw, xe, xo);
}

// ====================================================================
// Reverse, resident.  src holds the coefficient prefix [0, htop) of each
// signal (htop = h0 << (nlev-1), or h0 when nlev == 0); levels of size h0,
// 2h0, .., htop run in LDS; the result [0, htop) goes to dst.  Levels with at
// most 64 pairs (the first ones) run on wave 0 alone.
// ====================================================================
template <int L, int C, int NT, int CAP, bool FMA>
__device__ __forceinline__ void fwt_rev_res_blk(const double* __restrict__ s, AxisView sv,
    double* __restrict__ y, AxisView dv, int h0, int nlev, int c0, int inner, int dma,
    const typename FB<L>::Rev& tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int MAXP = (CAP / 2 * C + NT - 1) / NT;
  constexpr int MAXU = (CAP * C + NT - 1) / NT;
  const int nL = FB<L>::nr(tp);
  const int qe = (nL + 1) >> 1;
  const int tid = threadIdx.x;
  const int htop = nlev > 0 ? (h0 << (nlev - 1)) : h0;

  __shared__ __attribute__((aligned(16))) double tl[2 * (L > 0 ? L : 2)];
  if constexpr (FB<L>::kStatic) stage_rev_taps<L>(tp, tl);
  JWV_STAMP(0);
  load_window<C, NT, MAXU>(lds, s, htop, dma != 0, c0, inner,
                           [&](int e) { return (int64_t)e * sv.s_len; });
  dma_fence_barrier();
  JWV_STAMP(1);

  // one synthesis pair of a level of size h >= L, from the LDS level image.
  // Compiled-in banks: interior pairs read without wrapping; the array-head
  // pairs (m < Q-1, rotated order, rev_pair_rot) sit in wave 0 at every
  // level, so only wave 0 runs both paths.
  auto pair_at = [&](int h, int p, double& xe, double& xo) {
    const int half = h >> 1, hm = half - 1;
    const int m = p / C, c = p % C;
    const double* lb = lds + c;
    if constexpr (FB<L>::kStatic) {
      constexpr int Q = L / 2;
      if (m >= Q - 1) {
        rev_pair<L, FMA>(tp, lb + m * C, lb + (half + m) * C, C, xe, xo);
      } else {
        rev_pair_rot_t<L, FMA>(tl, [=](int q) { return lb[((m - q) & hm) * C]; },
                               [=](int q) { return lb[(half + ((m - q) & hm)) * C]; }, m, xe, xo);
      }
    } else {
      rev_pair_any<L, FMA>(
          tp, m, qe, lb + m * C, lb + (half + m) * C, C,
          [=](int q) { return lb[((m - q) & hm) * C]; },
          [=](int q) { return lb[(half + ((m - q) & hm)) * C]; }, xe, xo);
    }
  };
  // levels with h < L wrap several times: literal scatter order (one site);
  // compiled-in banks evaluate all h outputs at compile-time h (rev_small_c)
  auto pair_small = [&](int h, int p, double& xe, double& xo) {
    const int half = h >> 1;
    const int m = p / C, c = p % C;
    const double* lb = lds + c;
    if constexpr (FB<L>::kStatic) {
      rev_small_c<L, FMA>(tp, lb, lb + half * C, C, h, m, xe, xo);
    } else {
      xe = rev_small<L, FMA>(tp, lb, lb + half * C, C, h, 2 * m);
      xo = rev_small<L, FMA>(tp, lb, lb + half * C, C, h, 2 * m + 1);
    }
  };

  int h = h0, lev = 0;
  if ((h >> 1) * C <= 64 && nlev > 0) {  // small levels: wave 0 only
    if (tid < 64) {
      int hh = h;
      for (int lv = 0; lv < nlev && (hh >> 1) * C <= 64; ++lv, hh <<= 1) {
        JWV_STAMP(16 + lv);
        const int np = (hh >> 1) * C;
        const bool v = tid < np;
        const int p = v ? tid : np - 1;
        double xe, xo;
        if (hh < nL) pair_small(hh, p, xe, xo); else pair_at(hh, p, xe, xo);
        wave_lds_sync();
        if (v) {
          const int m = p / C, c = p % C;
          lds[(2 * m) * C + c] = xe;
          lds[(2 * m + 1) * C + c] = xo;
        }
        wave_lds_sync();
      }
    }
    while (lev < nlev && (h >> 1) * C <= 64) { ++lev; h <<= 1; }
    lds_barrier();
  }
  JWV_STAMP(2);
  // block-wide levels that still wrap several times (runtime L with C = 8:
  // h < 64 so np <= 256 = 2 slots of NT >= 128; all read before any write)
  for (; lev < nlev && h < nL; ++lev, h <<= 1) {
    const int np = (h >> 1) * C;
    double xe[2] = {0.0, 0.0}, xo[2] = {0.0, 0.0};
#pragma unroll
    for (int r = 0; r < 2; ++r)
      if (tid + r * NT < np) pair_small(h, tid + r * NT, xe[r], xo[r]);
    lds_barrier();
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int p = tid + r * NT;
      if (p < np) {
        const int m = p / C, c = p % C;
        lds[(2 * m) * C + c] = xe[r];
        lds[(2 * m + 1) * C + c] = xo[r];
      }
    }
    lds_barrier();
  }
  for (; lev < nlev; ++lev, h <<= 1) {
    JWV_STAMP(3 + lev);
    const int np = (h >> 1) * C;
    double xe[MAXP], xo[MAXP];
    for_pairs<MAXP, NT>(np, [&](int r, int p, bool v) { pair_at(h, p, xe[r], xo[r]); });
    lds_barrier();
    for_pairs<MAXP, NT>(np, [&](int r, int p, bool v) {
      if (v) {
        const int m = p / C, c = p % C;
        lds[(2 * m) * C + c] = xe[r];
        lds[(2 * m + 1) * C + c] = xo[r];
      }
    });
    lds_barrier();
  }
  JWV_STAMP(30);
  for (int q = tid; q < htop * C; q += NT) {
    const int i = q / C, c = q % C;
    if (c0 + c < inner) y[(int64_t)i * dv.s_len + c] = lds[q];
  }
  JWV_STAMP(42);
}

template <int L, int C, int NT, int CAP, bool FMA>
__global__ __launch_bounds__(NT) void fwt_rev_res(const double* __restrict__ src, AxisView sv,
    double* __restrict__ dst, AxisView dv, int h0, int nlev, int inner, int dma,
    typename FB<L>::Rev tp) {
  const int ncb = (inner + C - 1) / C;
  const int64_t bs = res_slab_block<C>(blockIdx.x);
  const int64_t o = bs / ncb;
  const int c0 = (int)(bs % ncb) * C;
  const double* s = src + view_base(sv, o) + c0;
  double* y = dst + view_base(dv, o) + c0;
  fwt_rev_res_blk<L, C, NT, CAP, FMA>(s, sv, y, dv, h0, nlev, c0, inner, dma, tp);
}

// ====================================================================
// Reverse, tiled: K levels of sizes h1, 2h1, .., hK = h1 << (K-1).
// asrc: approximation of length h1/2 (view as); coef: coefficient array (view
// cv, details of level size h at coef[h/2 .. h)); dst: output of length hK.
// Tile t produces dst[tT, tT+T).  Windows (pair aligned) from fine to coarse:
//   B_0 = tT, E_0 = tT+T;  B_{l+1} = even_floor(B_l/2 - (Q-1)), E_{l+1} = E_l/2
// PREF = false: the detail window of each level is loaded just before that
// level; LDS = A window (<= T/2 + 2Q + 4) + one D window (same bound).
// PREF = true: all detail windows are fetched in one burst up front (one
// memory latency per block); LDS = A window + sum of D windows (<= T + K(2Q+4)).
// ====================================================================
template <int L, int C, int NT, int T, int KMAX, bool FMA, bool PREF>
__global__ __launch_bounds__(NT) void fwt_rev_tile(const double* __restrict__ asrc, AxisView as,
                                                   const double* __restrict__ coef, AxisView cv,
                                                   double* __restrict__ dst, AxisView dv, int h1,
                                                   int K, int inner, int dma,
                                                   typename FB<L>::Rev tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int LM = LMax<L>::v;
  constexpr int QM = (LM + 1) / 2;
  constexpr int WA = T / 2 + 2 * QM + 4;  // window bound (levels >= 1)
  constexpr int MAXP = ((T / 2 + QM + 2) * C + NT - 1) / NT;
  constexpr int MAXU = (WA * C + NT - 1) / NT;
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
  double* abuf = lds;
  double* dall = lds + WA * C;

  auto win_b = [&](int l) {
    int bb = t * T;
    for (int k = 0; k < l; ++k) bb = ((bb >> 1) - (Q - 1)) & ~1;  // even floor
    return bb;
  };
  auto win_e = [&](int l) { return (t * T + T) >> l; };
  auto load_d = [&](double* buf, int l) {
    const int half = hK >> (l + 1), hm = half - 1;
    const int Bl1 = win_b(l + 1);
    load_window<C, NT, MAXU>(buf, sc, win_e(l + 1) - Bl1, dma != 0, c0, inner, [&](int e) {
      return ((int64_t)half + ((Bl1 + e) & hm)) * cv.s_len;
    });
  };

  {
    const int BK = win_b(K);
    const int am = (hK >> K) - 1;
    load_window<C, NT, MAXU>(abuf, sa, win_e(K) - BK, dma != 0, c0, inner,
                             [&](int e) { return (int64_t)((BK + e) & am) * as.s_len; });
  }
  if constexpr (PREF) {
    int doff = 0;
    for (int l = K - 1; l >= 0; --l) {
      load_d(dall + doff * C, l);
      doff += win_e(l + 1) - win_b(l + 1);
    }
    dma_fence_barrier();
  }
  int doff = 0;
  for (int l = K - 1; l >= 0; --l) {
    // level with output size hK >> l; inputs a, d of length half
    const int half = hK >> (l + 1), hm = half - 1;
    const int Bl = win_b(l), Bl1 = win_b(l + 1);
    const int Wd = win_e(l + 1) - Bl1;
    const double* dbuf = PREF ? dall + doff * C : dall;
    doff += Wd;
    if constexpr (!PREF) {
      load_d(dall, l);
      dma_fence_barrier();
    }
    const int pbase = Bl >> 1;                  // first pair (global, may be <0)
    const int np = ((win_e(l) - Bl) >> 1) * C;  // pairs in window
    const int off = pbase - Bl1;                // local index of a[pbase]
    double xe[MAXP], xo[MAXP];
    for_pairs<MAXP, NT>(np, [&](int r, int p, bool v) {
      const int ml = p / C, c = p % C;
      const int mg = (pbase + ml) & hm;
      const int li = off + ml;
      const double* ab = abuf + c;
      const double* db = dbuf + c;
      // window indices never wrap (the halo holds the periodic extension)
      if (mg >= Q - 1) {
        rev_pair<L, FMA>(tp, ab + li * C, db + li * C, C, xe[r], xo[r]);
      } else {
        rev_pair_head<L, FMA>(
            tp, mg, [=](int q) { return ab[(li - q) * C]; },
            [=](int q) { return db[(li - q) * C]; }, xe[r], xo[r]);
      }
    });
    if (l == 0) {
      for_pairs<MAXP, NT>(np, [&](int r, int p, bool v) {
        const int ml = p / C, c = p % C;
        if (v && c0 + c < inner) {
          const int64_t k = (int64_t)t * T + 2 * ml;
          y[k * dv.s_len + c] = xe[r];
          y[(k + 1) * dv.s_len + c] = xo[r];
        }
      });
    } else {
      lds_barrier();
      for_pairs<MAXP, NT>(np, [&](int r, int p, bool v) {
        if (v) {
          const int ml = p / C, c = p % C;
          abuf[(2 * ml) * C + c] = xe[r];
          abuf[(2 * ml + 1) * C + c] = xo[r];
        }
      });
      lds_barrier();
    }
  }
}

}  // namespace jwv
