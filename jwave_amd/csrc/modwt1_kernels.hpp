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
//
// Non-finite input (modwt_nonfinite.hpp): each kernel runs its tile as a fast
// pass that checks its last level's outputs and, in a block whose check
// fired, again with SLOW = true (the Java zero-tap NaN repair).
#pragma once
#include "modwt_kernels.hpp"
#include "modwt_nonfinite.hpp"

namespace jwv {

#ifndef JWV_MOD1_FENCE
#define JWV_MOD1_FENCE 2
#endif

template <bool FMA>
__device__ __forceinline__ double mod_mac(double acc, double a, double b) {
  return mac<FMA>(acc, a, b);
}

// Buffer-resource access for tiles that do not wrap: the block-uniform base
// lives in SGPRs, a lane adds one 32-bit offset, slot offsets are scalar, so a
// load or store costs no per-access 64-bit address VALU.
__device__ __forceinline__ auto mod_rsrc(const double* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), 0, 0x7ffffff0, 0x00020000);
}
// lds[e] = src[e], e < W (no wrap), loads all in flight before the LDS writes
template <int NT, int MAXP>
__device__ __forceinline__ void mod_load_window(double* lds, const double* src, int W) {
  const int tid = threadIdx.x;
  const auto rs = mod_rsrc(src);
  double v[MAXP];
#pragma unroll
  for (int r = 0; r < MAXP; ++r)
    if ((r + 1) * NT <= W || tid + r * NT < W)
      v[r] = __builtin_bit_cast(double,
                                __builtin_amdgcn_raw_buffer_load_b64(rs, tid * 8, r * NT * 8, 0));
#pragma unroll
  for (int r = 0; r < MAXP; ++r)
    if ((r + 1) * NT <= W || tid + r * NT < W) lds[tid + r * NT] = v[r];
}
__device__ __forceinline__ void mod_store2(double* base, int off, double a, double b) {
  const jwv_u32x4 v = __builtin_bit_cast(jwv_u32x4, make_double2(a, b));
  __builtin_amdgcn_raw_buffer_store_b128(v, mod_rsrc(base), off * 8, 0, 0);
}

// Run form of a level (M > 1): a lane computes M output pairs whose slots
// (16-B units) are h = st/2 apart (st = 1: M adjacent pairs).  Pair slot s
// reads tap slots s + l*h (inverse) or s - l*h (forward), so the M pairs
// share all but M + L - 1 of their M*L 16-B LDS reads per operand (st = 1:
// M + L/2 reads).  Lanes take (block, residue) = (t / h, t % h), a block
// covering M*h slots: the 16 lanes of a ds_read_b128 group then sit at
// distinct slots mod 16 for odd M, so the reads stay conflict-free at every
// stride.  Summation order per output is the P2/one-output kernels' order.
template <int L, int M>
struct ModRun {
  static_assert((M & 1) == 1 && L % 2 == 0, "odd M, even L");
  template <int st>
  static constexpr int h() { return st >= 2 ? st / 2 : 1; }
  template <int st>
  static constexpr int nrd() { return st == 1 ? M + L / 2 : M + L - 1; }
  template <int st>
  __device__ __forceinline__ static int slot0(int t) {
    constexpr int H = h<st>();
    return (t / H) * (M * H) + (t % H);
  }
};

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
  // Run form (ModRun, M pairs per lane): level j reads up to window index
  // e0(j) + 2*NB*M*h (past its last output slot, NB run blocks of M*h slots)
  static constexpr int kPad = (S & 1) ? 1 : 2;
  static constexpr int run_reach(int j, int M) {
    const int st = 1 << (j - 1), h = st >= 2 ? st / 2 : 1;
    const int ns = nout(j) / 2, nb = (ns + M * h - 1) / (M * h);
    return kPad + e0(j) + 2 * nb * M * h;
  }
  static constexpr int lds_doubles(int M) {
    M %= 1000;
    int b = lds_doubles();
    if (M % 100 > 1)
      for (int j = J0; j <= J1; ++j) {
        const int r = run_reach(j, M % 100) + 2;
        if (r > b) b = r;
      }
    return b;
  }
};

// P2: a lane computes two adjacent outputs (e, e+1) with e of the parity of
// e0(j) (= the parity of S for every level: Sn(j) is even), so the pairs
// tile each level's outputs exactly; the window sits at lds + kPad with kPad
// + e0 even, so every tap pair (e - l*st, e + 1 - l*st) is one 16-B LDS read
// (st = 1: the 10-value run e-8 .. e+1) at a 16-B lane stride, and the W
// pair (t0 - S + e even) is one 16-B store when the rows are 16-B aligned.
template <int L, int NT, int T, int J0, int J1, bool FMA, int j, bool P2, int M = 1,
          bool SLOW = false>
struct ModFwd1Level {
  static constexpr int kPad = ModFwd1Geo<L, T, J0, J1>::kPad;
  // M = m + 100*jr: run form with m pairs per lane on levels j >= jr
  static constexpr int kM = M % 100, kJR = (M / 100) % 10;
  static constexpr bool kRun = kM > 1 && j >= kJR;
  __device__ __forceinline__ static void run_p2(const ModwtTaps<L>& tp, double* lds,
                                                double* __restrict__ wout, int64_t ldw,
                                                int64_t t0, int64_t N, ModNf& nf) {
    using G = ModFwd1Geo<L, T, J0, J1>;
    constexpr int st = 1 << (j - 1);
    constexpr int e0 = G::e0(j), nout = G::nout(j);
    static_assert(((kPad + e0) & 1) == 0 && (nout & 1) == 0, "pairs must tile the outputs");
    constexpr int NP = nout / 2;
    constexpr int R = (NP + NT - 1) / NT;
    // repair: window positions [e0 - C, S + T) at lds[kPad + q]
    constexpr int C = (L - 1) * st;
    int lo[2] = {1, 1}, hi[2] = {0, 0};
    auto at = [&](int q) { return lds[kPad + q]; };
    if constexpr (SLOW && j >= 2)
      nf_window<1, NT>(nf, e0 - C, G::W, [&](int, int q) { return at(q); }, lo, hi);
    const int tid = opaque_tid();
    double* __restrict__ wrow = wout + (int64_t)(j - 1) * ldw + (t0 - G::S);
    // 16-B W stores: row base (j-1)*ldw + t0 - S + e is even for these e
    const bool w16 = (((uintptr_t)wrow + 8 * e0) & 15) == 0;
    // the whole tile inside the signal and 16-B rows: buffer stores
    const bool wfast = w16 && t0 + T <= N;
    // repair mask (bit 2r + h: output e0 + 2k + h is Java's NaN), formed
    // before the sums so the scans hold no sum registers
    static_assert(2 * R <= 32, "repair mask bits");
    uint32_t nm = 0;
    if constexpr (SLOW && j >= 2)
      if (lo[0] <= hi[0]) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int k = tid + r * NT;
          const int e = e0 + 2 * ((r + 1) * NT <= NP ? k : (k < NP ? k : NP - 1));
          if (nf_fwd_zero(at, e, st, C, lo[0], hi[0])) nm |= 1u << (2 * r);
          if (nf_fwd_zero(at, e + 1, st, C, lo[0], hi[0])) nm |= 2u << (2 * r);
        }
        asm volatile("" : "+v"(nm)::"memory");
      }
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
        sw0 = mod_mac<FMA>(sw0, x0[l], tp.h[l]);
        sv0 = mod_mac<FMA>(sv0, x0[l], tp.g[l]);
        sw1 = mod_mac<FMA>(sw1, x1[l], tp.h[l]);
        sv1 = mod_mac<FMA>(sv1, x1[l], tp.g[l]);
      }
      if constexpr (SLOW) {
        if ((nm >> (2 * r)) & 1) sw0 = sv0 = mod_nan();
        if ((nm >> (2 * r)) & 2) sw1 = sv1 = mod_nan();
      }
      pin2(sw0, sv0);
      pin2(sw1, sv1);
      vv[r] = make_double2(sv0, sv1);
      const int ee = e0 + 2 * k;  // S has e0's parity: a pair is all halo or all own
      if ((full || k < NP) && e0 + 2 * (r + 1) * NT > G::S && ee >= G::S) {
        const int64_t g = t0 + (ee - G::S);
        if (wfast) {
          mod_store2(wrow, ee, sw0, sw1);
        } else if (w16 && g + 1 < N) {
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
      ModFwd1Level<L, NT, T, J0, J1, FMA, j + 1, P2, M, SLOW>::run(tp, lds, wout, ldw, t0, N, nf);
  }
  __device__ __forceinline__ static void run(const ModwtTaps<L>& tp, double* lds,
                                             double* __restrict__ wout, int64_t ldw, int64_t t0,
                                             int64_t N, ModNf& nf) {
    static_assert(P2 && M == 1, "forward: the P2 form");
    run_p2(tp, lds, wout, ldw, t0, N, nf);
  }
};

// One forward tile: window load, levels J0..J1, V_{J1} out.  The fast pass
// (SLOW = false) ORs "a V_{J1} output is not finite" into bad.
template <int L, int NT, int T, int J0, int J1, bool FMA, bool P2, int M, bool SLOW>
__device__ __forceinline__ void modwt_fwd_tile1_body(const double* __restrict__ src,
                                                     double* __restrict__ wout, int64_t ldw,
                                                     double* __restrict__ vout, int64_t N,
                                                     const ModwtTaps<L>& tp, double* lds,
                                                     ModNf& nf, bool& bad) {
  using G = ModFwd1Geo<L, T, J0, J1>;
  constexpr int MAXP = (G::W + NT - 1) / NT;
  constexpr int pad = (P2 || M % 100 > 1) ? G::kPad : 0;
  const int64_t t0 = xcd_tile() * T;
  const bool inside = t0 - G::S >= 0 && t0 + T <= N;  // block-uniform: no wrap
  if (inside)
    mod_load_window<NT, MAXP>(lds + pad, src + (t0 - G::S), G::W);
  else
    load_window<1, NT, MAXP>(lds + pad, src, G::W, false, 0, 1,
                             [&](int e) { return wrap_mod(t0 - G::S + e, N); });
  lds_barrier();
  ModFwd1Level<L, NT, T, J0, J1, FMA, J0, P2, M, SLOW>::run(tp, lds, wout, ldw, t0, N, nf);
  const int tid = threadIdx.x;
#pragma unroll
  for (int r = 0; r < (T + NT - 1) / NT; ++r) {
    const int p = tid + r * NT;
    if (p < T && t0 + p < N) {
      const double v = lds[pad + G::S + p];
      if constexpr (!SLOW) bad = bad || nonfinite(v);
      vout[t0 + p] = v;
    }
  }
}

// src = V_{J0-1} (length N); W_j -> wout + (j-1)*ldw; V_{J1} -> vout.
// Grid: ceil(N/T) blocks (XCD-aware order, xcd_tile).
template <int L, int NT, int T, int J0, int J1, bool FMA, bool P2 = false, int M = 1>
__global__ __launch_bounds__(NT, mod_lds_waves(ModFwd1Geo<L, T, J0, J1>::lds_doubles(M) * 8, NT))
void modwt_fwd_tile1(const double* __restrict__ src,
                                                      double* __restrict__ wout, int64_t ldw,
                                                      double* __restrict__ vout, int64_t N,
                                                      ModwtTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ ModNf nf;
  nf_init(nf);
  bool bad = false;
  modwt_fwd_tile1_body<L, NT, T, J0, J1, FMA, P2, M, false>(src, wout, ldw, vout, N, tp, lds, nf,
                                                            bad);
  if (nf_any(nf, bad))
    modwt_fwd_tile1_body<L, NT, T, J0, J1, FMA, P2, M, true>(src, wout, ldw, vout, N, tp, lds, nf,
                                                             bad);
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
  // Run form (M pairs per lane, ModRun): the last run block of level j reads
  // up to 2*NB*M*h + (L-1)*st doubles (st = 1: 2*NB*M + L) of each buffer.
  static constexpr int nout(int j) { return T + Rout(j); }
  static constexpr int run_reach(int j, int M) {
    const int st = 1 << (j - 1), h = st >= 2 ? st / 2 : 1;
    const int ns = (nout(j) + 1) / 2, nb = (ns + M * h - 1) / (M * h);
    return st == 1 ? 2 * nb * M + L : 2 * nb * M * h + (L - 1) * st;
  }
  static constexpr int run_buf(int M) {
    M %= 1000;
    int b = buf();
    for (int j = J0; j <= J1; ++j) {
      const int r = (run_reach(j, M % 100) + 3) & ~1;
      if (r > b) b = r;
    }
    return b;
  }
  static constexpr int lds_doubles(int M) {
    return M % 100 > 1 ? 2 * run_buf(M) : lds_doubles();
  }
};


template <int L, int NT, int T, int J0, int J1, bool FMA, int j, bool P2 = false, int M = 1,
          bool SLOW = false>
struct ModInv1Level {
  using G = ModInv1Geo<L, T, J0, J1>;
  // M = m + 100*jr: run form with m pairs per lane on levels j >= jr
  static constexpr int kM = M % 100, kJR = (M / 100) % 10;
  static constexpr bool kRun = kM > 1 && j >= kJR;
  static constexpr int MAXP = (G::Wmax + NT - 1) / NT;
  // fetch the W_j window [t0, t0 + T + Rin(j)) into registers
  __device__ __forceinline__ static void fetch(double (&pw)[MAXP], const double* __restrict__ coef,
                                               int64_t ldw, int64_t t0, int64_t N, bool inside) {
    constexpr int Wn = T + G::Rin(j);
    const double* row = coef + (int64_t)(j - 1) * ldw;
    const int tid = opaque_tid();
    if (inside) {
      // buffer loads: block-uniform base in SGPRs, one lane offset, the slot
      // offsets r*NT*8 as scalar offsets (no per-load 64-bit address VALU)
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(row + t0), 0,
                                                        0x7ffffff0, 0x00020000);
#pragma unroll
      for (int r = 0; r < MAXP; ++r) {
        const int q = tid + r * NT;
        if (r * NT < Wn && ((r + 1) * NT <= Wn || q < Wn))
          pw[r] = __builtin_bit_cast(
              double, __builtin_amdgcn_raw_buffer_load_b64(rs, tid * 8, r * NT * 8, 0));
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int q = tid + r * NT;
      if (r * NT < Wn && ((r + 1) * NT <= Wn || q < Wn)) pw[r] = row[wrap_mod(t0 + q, N)];
    }
  }
  using Next = ModInv1Level<L, NT, T, J0, J1, FMA, j - 1, P2, M, SLOW>;
  // Repair state of a level: non-finite ranges of the V (0) and W (1) windows
  struct Nf {
    ModNf& f;
    bool& bad;
    int lo[2] = {1, 1}, hi[2] = {0, 0};
  };
  static constexpr int kC = (L - 1) * (1 << (j - 1));
  // Java's NaN at output p (SLOW only; needs the level's windows intact)
  __device__ __forceinline__ static bool nf_out(const Nf& nf, const double* vb, const double* wb,
                                                int p) {
    constexpr int st = 1 << (j - 1);
    if constexpr (!SLOW || st == 1) {
      return false;
    } else {
      return (nf.lo[0] <= nf.hi[0] &&
              nf_inv_zero([&](int q) { return vb[q]; }, p, st, kC, nf.lo[0], nf.hi[0])) ||
             (nf.lo[1] <= nf.hi[1] &&
              nf_inv_zero([&](int q) { return wb[q]; }, p, st, kC, nf.lo[1], nf.hi[1]));
    }
  }
  __device__ __forceinline__ static void run(const ModwtTaps<L>& tp, double* vb, double* wb,
                                             double (&pw)[MAXP], const double* __restrict__ coef,
                                             int64_t ldw, double* __restrict__ dst, int64_t t0,
                                             int64_t N, bool inside, ModNf& f, bool& bad) {
    static_assert(P2, "inverse: the P2 or run form");
    constexpr int Wn = T + G::Rin(j);
    const int tid = opaque_tid();
#pragma unroll
    for (int r = 0; r < MAXP; ++r) {
      const int q = tid + r * NT;
      if (r * NT < Wn && ((r + 1) * NT <= Wn || q < Wn)) wb[q] = pw[r];
    }
    lds_barrier();
    if constexpr (j > J0) Next::fetch(pw, coef, ldw, t0, N, inside);
    Nf nf{f, bad};
    if constexpr (SLOW && j >= 2)
      nf_window<2, NT>(f, 0, Wn, [&](int k, int q) { return k ? wb[q] : vb[q]; }, nf.lo, nf.hi);
    if constexpr (kRun)
      compute_mr(tp, vb, wb, pw, coef, ldw, dst, t0, N, inside, nf);
    else
      compute_p2(tp, vb, wb, pw, coef, ldw, dst, t0, N, inside, nf);
  }
  // P2: a lane computes the adjacent outputs (p, p+1), p even: every tap pair
  // (p + l*st, p + 1 + l*st) of V and of W is one 16-B LDS read (st = 1: the
  // 10-value runs p .. p+9), 16-B lane stride.  An odd output count leaves
  // one extra output at index nout, past what the next level reads.
  __device__ __forceinline__ static void compute_p2(const ModwtTaps<L>& tp, double* vb, double* wb,
                                                    double (&pw)[MAXP],
                                                    const double* __restrict__ coef, int64_t ldw,
                                                    double* __restrict__ dst, int64_t t0,
                                                    int64_t N, bool inside, Nf& nf) {
    constexpr int st = 1 << (j - 1);
    constexpr int nout = T + G::Rout(j);
    constexpr int NP = (nout + 1) / 2;
    constexpr int R = (NP + NT - 1) / NT;
    const int tid = opaque_tid();
    // repair mask (bit 2r + h: output 2kc + h is Java's NaN), formed before
    // the sums so the scans hold no sum registers
    static_assert(2 * R <= 32, "repair mask bits");
    uint32_t nm = 0;
    if constexpr (SLOW) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        const int kc = (r + 1) * NT <= NP ? k : (k < NP ? k : NP - 1);
        if (nf_out(nf, vb, wb, 2 * kc)) nm |= 1u << (2 * r);
        if (nf_out(nf, vb, wb, 2 * kc + 1)) nm |= 2u << (2 * r);
      }
      asm volatile("" : "+v"(nm)::"memory");
    }
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
      // LDS-only levels (j > J0) start each sum at its first product (the
      // signed-zero argument of fwt_kernels.hpp, ZS): one dependent add less
      // per chain; the level that writes HBM starts from +0.0
      constexpr bool kZ = j == J0;
      double sa0 = 0.0, sd0 = 0.0, sa1 = 0.0, sd1 = 0.0;
      if constexpr (!kZ) {
        sa0 = av0[0] * tp.g[0];
        sd0 = aw0[0] * tp.h[0];
        sa1 = av1[0] * tp.g[0];
        sd1 = aw1[0] * tp.h[0];
      }
#pragma unroll
      for (int l = kZ ? 0 : 1; l < L; ++l) {
        sa0 = mod_mac<FMA>(sa0, av0[l], tp.g[l]);
        sd0 = mod_mac<FMA>(sd0, aw0[l], tp.h[l]);
        sa1 = mod_mac<FMA>(sa1, av1[l], tp.g[l]);
        sd1 = mod_mac<FMA>(sd1, aw1[l], tp.h[l]);
      }
      pin2(sa0, sd0);
      pin2(sa1, sd1);
      vv[r] = make_double2(sa0 + sd0, sa1 + sd1);
      if constexpr (SLOW) {
        if ((nm >> (2 * r)) & 1) vv[r].x = mod_nan();
        if ((nm >> (2 * r)) & 2) vv[r].y = mod_nan();
      }
      if constexpr (JWV_MOD1_FENCE > 0)
        if ((r + 1) % JWV_MOD1_FENCE == 0)
          asm volatile("" : "+v"(vv[r].x), "+v"(vv[r].y) :: "memory");
    }
    lds_barrier();
    if constexpr (j == J0) {
      const bool dfast = t0 + T <= N && (((uintptr_t)(dst + t0)) & 15) == 0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        const int p = 2 * k;
        if (r * NT * 2 < T && p < T) {
          if constexpr (!SLOW)
            nf.bad = nf.bad || nonfinite(vv[r].x) || (p + 1 < T && nonfinite(vv[r].y));
          if (dfast) {
            mod_store2(dst + t0, p, vv[r].x, vv[r].y);
          } else if (t0 + p + 1 < N && p + 1 < T) {
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
      Next::run(tp, vb, wb, pw, coef, ldw, dst, t0, N, inside, nf.f, nf.bad);
    }
  }
  // Run form (ModRun): output pair slot s = s0 + m*h, m < M, reads tap slots
  // s0 + k*h, k < M + L - 1 (st = 1: doubles 2*s0 .. 2*s0 + 2M + L - 1).
  // V taps first, then W taps (registers: one operand's run at a time).
  template <bool ISW>
  __device__ __forceinline__ static void run_sums(const ModwtTaps<L>& tp, const double* base,
                                                  double (&acc)[kM][2]) {
    constexpr int st = 1 << (j - 1);
    constexpr int H = ModRun<L, kM>::template h<st>();
    constexpr int NRD = ModRun<L, kM>::template nrd<st>();
    double v[2 * NRD];
#pragma unroll
    for (int k = 0; k < NRD; ++k) {
      const double2 u = *reinterpret_cast<const double2*>(base + 2 * k * H);
      v[2 * k] = u.x;
      v[2 * k + 1] = u.y;
    }
#pragma unroll
    for (int m = 0; m < kM; ++m) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        double s = 0.0;
        constexpr bool kZ = j == J0;  // as in compute_p2
#pragma unroll
        for (int l = 0; l < L; ++l) {
          // st = 1: output 2(s0+m)+q, tap l -> double 2m + q + l of the run;
          // st >= 2: slot m + l of the run, half q
          const double x = st == 1 ? v[2 * m + q + l] : v[2 * (m + l) + q];
          if (!kZ && l == 0)
            s = x * (ISW ? tp.h[0] : tp.g[0]);
          else
            s = mod_mac<FMA>(s, x, ISW ? tp.h[l] : tp.g[l]);
        }
        acc[m][q] = s;
      }
    }
  }
  __device__ __forceinline__ static void compute_mr(const ModwtTaps<L>& tp, double* vb, double* wb,
                                                    double (&pw)[MAXP],
                                                    const double* __restrict__ coef, int64_t ldw,
                                                    double* __restrict__ dst, int64_t t0,
                                                    int64_t N, bool inside, Nf& nf) {
    constexpr int st = 1 << (j - 1);
    constexpr int H = ModRun<L, kM>::template h<st>();
    constexpr int nout = G::nout(j);
    constexpr int NS = (nout + 1) / 2;  // output pair slots
    constexpr int NB = (NS + kM * H - 1) / (kM * H);
    constexpr int NTASK = NB * H;
    constexpr int R = (NTASK + NT - 1) / NT;
    static_assert(G::run_reach(j, kM) <= G::run_buf(M), "run reads past the buffer");
    const int tid = opaque_tid();
    // repair mask (bit 2(r kM + m) + h), formed before the sums
    static_assert(2 * R * kM <= 32, "repair mask bits");
    uint32_t nm = 0;
    if constexpr (SLOW) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int t = tid + r * NT;
        const int s0 = ModRun<L, kM>::template slot0<st>(t < NTASK ? t : NTASK - 1);
#pragma unroll
        for (int m = 0; m < kM; ++m) {
          const int s = s0 + m * H;
          if (nf_out(nf, vb, wb, 2 * s)) nm |= 1u << (2 * (r * kM + m));
          if (nf_out(nf, vb, wb, 2 * s + 1)) nm |= 2u << (2 * (r * kM + m));
        }
      }
      asm volatile("" : "+v"(nm)::"memory");
    }
    double2 vv[R][kM];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int t = tid + r * NT;
      const bool full = (r + 1) * NT <= NTASK;
      // a wave whose tasks all lie past NTASK skips the slot (scalar branch)
      if (!full && __builtin_amdgcn_readfirstlane((tid & ~63) + r * NT) >= NTASK) continue;
      const int tc = full ? t : (t < NTASK ? t : NTASK - 1);
      const int s0 = ModRun<L, kM>::template slot0<st>(tc);
      double sa[kM][2], sd[kM][2];
      run_sums<false>(tp, vb + 2 * s0, sa);
      run_sums<true>(tp, wb + 2 * s0, sd);
#pragma unroll
      for (int m = 0; m < kM; ++m) {
        pin2(sa[m][0], sd[m][0]);
        pin2(sa[m][1], sd[m][1]);
        vv[r][m] = make_double2(sa[m][0] + sd[m][0], sa[m][1] + sd[m][1]);
        if constexpr (SLOW) {
          if ((nm >> (2 * (r * kM + m))) & 1) vv[r][m].x = mod_nan();
          if ((nm >> (2 * (r * kM + m))) & 2) vv[r][m].y = mod_nan();
        }
      }
      asm volatile("" ::: "memory");  // slot fence
    }
    lds_barrier();
    // final level, whole tile inside the signal, 16-B aligned output: buffer stores
    const bool dfast = j == J0 && t0 + T <= N && (((uintptr_t)(dst + t0)) & 15) == 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int t = tid + r * NT;
      const bool ok = (r + 1) * NT <= NTASK || t < NTASK;
      const int s0 = ModRun<L, kM>::template slot0<st>(ok ? t : 0);
#pragma unroll
      for (int m = 0; m < kM; ++m) {
        const int s = s0 + m * H;
        if constexpr (j == J0) {
          const int p = 2 * s;
          if (ok && p < T) {
            if constexpr (!SLOW)
              nf.bad = nf.bad || nonfinite(vv[r][m].x) || (p + 1 < T && nonfinite(vv[r][m].y));
            if (dfast) {
              mod_store2(dst + t0, p, vv[r][m].x, vv[r][m].y);
            } else if (t0 + p + 1 < N && p + 1 < T) {
              *reinterpret_cast<double2*>(dst + t0 + p) = vv[r][m];
            } else if (t0 + p < N) {
              dst[t0 + p] = vv[r][m].x;
            }
          }
        } else {
          if (ok && s < NS) *reinterpret_cast<double2*>(vb + 2 * s) = vv[r][m];
        }
      }
    }
    if constexpr (j > J0) Next::run(tp, vb, wb, pw, coef, ldw, dst, t0, N, inside, nf.f, nf.bad);
  }
};

// One inverse tile (fast pass: SLOW = false, ORs "an output is not finite"
// into bad).
template <int L, int NT, int T, int J0, int J1, bool FMA, bool P2, int M, bool SLOW>
__device__ __forceinline__ void modwt_inv_tile1_body(const double* __restrict__ vsrc,
                                                     const double* __restrict__ coef, int64_t ldw,
                                                     double* __restrict__ dst, int64_t N,
                                                     const ModwtTaps<L>& tp, double* lds,
                                                     ModNf& nf, bool& bad) {
  using G = ModInv1Geo<L, T, J0, J1>;
  using Top = ModInv1Level<L, NT, T, J0, J1, FMA, J1, P2, M, SLOW>;
  double* vb = lds;
  double* wb = lds + (M % 100 > 1 ? G::run_buf(M) : G::buf());
  const int64_t t0 = xcd_tile() * T;
  const bool inside = t0 + G::Wmax <= N;
  double pw[Top::MAXP];
  if (inside)
    mod_load_window<NT, Top::MAXP>(vb, vsrc + t0, G::Wmax);
  else
    load_window<1, NT, Top::MAXP>(vb, vsrc, G::Wmax, false, 0, 1,
                                  [&](int e) { return wrap_mod(t0 + e, N); });
  Top::fetch(pw, coef, ldw, t0, N, inside);
  Top::run(tp, vb, wb, pw, coef, ldw, dst, t0, N, inside, nf, bad);
}

// vsrc = V_{J1}; W_j at coef + (j-1)*ldw; output V_{J0-1} -> dst.
template <int L, int NT, int T, int J0, int J1, bool FMA, bool P2 = false, int M = 1>
// (the fast pass alone needs up to 80 VGPRs from J1 = 3 on: 6 waves per SIMD)
__global__ __launch_bounds__(NT, mod_lds_waves(ModInv1Geo<L, T, J0, J1>::lds_doubles(M) * 8, NT,
                                               J1 - J0 >= 2 ? 6 : 8))
void modwt_inv_tile1(const double* __restrict__ vsrc,
                                                      const double* __restrict__ coef, int64_t ldw,
                                                      double* __restrict__ dst, int64_t N,
                                                      ModwtTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ ModNf nf;
  nf_init(nf);
  bool bad = false;
  modwt_inv_tile1_body<L, NT, T, J0, J1, FMA, P2, M, false>(vsrc, coef, ldw, dst, N, tp, lds, nf,
                                                            bad);
  if (nf_any(nf, bad))
    modwt_inv_tile1_body<L, NT, T, J0, J1, FMA, P2, M, true>(vsrc, coef, ldw, dst, N, tp, lds, nf,
                                                             bad);
}

}  // namespace jwv
