// fwt1_kernels.hpp — FWT tile kernels for contiguous signals (C = 1,
// sample stride 1, every base pointer 16-B aligned) with compile-time
// geometry: tap count L, tile T and fused level count K are template
// arguments, so every level's window size, slot count and store guard is a
// constant and the level loop unrolls into straight-line code.
//
// Same math and summation order as fwt_fwd_tile / fwt_rev_tile
// (Wavelet.java:236-303; see fwt_kernels.hpp), so EXACT results stay
// bit-identical.  Differences are structural only:
//  * reverse levels ping-pong between two LDS buffers (one barrier per
//    level); the forward runs level 1 in place and ping-pongs the rest inside
//    the level-0 window (LDS = one window);
//  * detail / output stores use an SGPR base + 32-bit lane offset; the final
//    synthesis level stores (x[2m], x[2m+1]) as one 16-B store;
//  * reverse: the array-head pairs (Wavelet.java:284-296 wrap order) exist
//    only in the first tiles' windows; every other block skips the head test.
#pragma once
#include "fwt_kernels.hpp"

namespace jwv {

// ---------------------------------------------------------------- forward
// Window after l fused levels: T/2^l own samples + (L-2)(2^(K-l) - 1) halo.
// LDS holds only the level-0 window: level 1 runs in place (its results wait
// in registers across one extra barrier), then levels alternate between
// offset 0 (odd l) and offset o2 = even(m(1)) (even l) inside that window.
template <int L, int T, int K>
struct Fwd1Geo {
  static constexpr int m(int l) { return (T >> l) + (L - 2) * ((1 << (K - l)) - 1); }
  static constexpr int o2() { return (m(1) + 1) & ~1; }
  static_assert((L & 1) == 0 && ((T >> K) & 1) == 0, "pair couples need even windows");
  static constexpr int off(int l) { return (l & 1) ? 0 : o2(); }  // level-l output (l >= 1)
  static constexpr int lds_doubles() {
    return (m(0) + 2 > o2() + m(2 <= K ? 2 : 1)) ? m(0) + 2 : o2() + m(2 <= K ? 2 : 1);
  }
};

#ifndef JWV_FWD_SLOT_FENCE
#define JWV_FWD_SLOT_FENCE 1
#endif
#ifndef JWV_FWD_FENCE_MINL
#define JWV_FWD_FENCE_MINL 12
#endif
// A lane computes two adjacent pairs ("a couple", L+2 window values read as
// 16-B LDS reads at a 32-B lane stride).
template <int L, int NT, int T, int K, bool FMA, int l, bool WT = false>
struct Fwd1Level {
  // level l reads the level-(l-1) window at lds + off(l-1) (l = 1: lds) and
  // writes its approximations at lds + off(l) (the last level: ya).
  // yd0: the signal's coefficient row; ya: its level-K approximation row.
  // Each lane computes two adjacent pairs (p, p+1): one 16-B store per lane
  // for the details and approximations, L+2 window reads for two pairs.
  // Segmented rows (lsw < 31): sample i of the row lives at
  // yd0 + (i >> lsw) * ss + (i & (2^lsw - 1)) -- the [W][rows][cols/W] send
  // layout of the sharded 2-D transform (distributed.py); a level's detail
  // range of one tile (T >> l samples, aligned) never straddles a segment
  // (host: 2^lsw >= T / 2).
  __device__ __forceinline__ static void run(const FwdTaps<L>& tp, double* lds,
                                             double* __restrict__ yd0, int hl, int t,
                                             double* __restrict__ ya, int sp = 0, int lsw = 31,
                                             int64_t ss = 0) {
    using G = Fwd1Geo<L, T, K>;
    JWV_STAMP(10 + l);
    constexpr int mo = G::m(l);      // even
    constexpr int own = T >> l;      // even
    constexpr int NP2 = mo / 2;      // pair couples
    constexpr int R = (NP2 + NT - 1) / NT;
    const double* in = lds + (l == 1 ? 0 : G::off(l - 1));
    double* out = lds + G::off(l);
    const int tid = opaque_tid();  // per-level: keeps address math out of the prologue
    const int i0 = (hl >> 1) + t * own;
    double* __restrict__ yd =
        yd0 + (int64_t)(i0 >> lsw) * ss + (i0 & (int)((1u << (lsw & 31)) - 1u));
    double2 av[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int q = tid + r * NT;  // couple index: pairs 2q, 2q+1
      if ((r + 1) * NT <= NP2 || q < NP2) {
        double x[L + 2];
#pragma unroll
        for (int j = 0; j < L + 2; j += 2) {
          const double2 v = *reinterpret_cast<const double2*>(in + 4 * q + j);
          x[j] = v.x;
          x[j + 1] = v.y;
        }
        double a0, d0, a1, d1;
        fwd_pair<L, FMA>(tp, [&](int j) { return x[j]; }, a0, d0);
        fwd_pair<L, FMA>(tp, [&](int j) { return x[j + 2]; }, a1, d1);
        // long banks: a slot boundary keeps the compiler from hoisting every
        // slot's L+2 window reads at once (L = 16: 118 -> 54 VGPRs, 8 waves
        // per SIMD).  L = 8 (68 -> 40 VGPRs) measured 1.5% slower on config 2,
        // so the fence starts at JWV_FWD_FENCE_MINL = 12.
        if constexpr (L >= JWV_FWD_FENCE_MINL && JWV_FWD_SLOT_FENCE)
          asm volatile("" : "+v"(a0), "+v"(a1), "+v"(d0), "+v"(d1) :: "memory");
        const int p = 2 * q;
        if constexpr (l == K) {  // WT: handed to another workgroup of this launch
          st2<WT>(ya + (int64_t)t * own + p, a0, a1);
        } else if constexpr (l == 1) {
          av[r] = make_double2(a0, a1);  // in place: written after every wave has read
        } else {
          *reinterpret_cast<double2*>(out + p) = make_double2(a0, a1);
        }
        if (2 * r * NT < own && (2 * (r + 1) * NT <= own || p < own))
          st2_pol(yd, p, d0, d1, sp);
      }
    }
    if constexpr (l < K) {
      if constexpr (l == 1) {
        lds_barrier();
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int q = tid + r * NT;
          if ((r + 1) * NT <= NP2 || q < NP2) *reinterpret_cast<double2*>(out + 2 * q) = av[r];
        }
      }
      lds_barrier();
      Fwd1Level<L, NT, T, K, FMA, l + 1, WT>::run(tp, lds, yd0, hl >> 1, t, ya, sp, lsw, ss);
    }
  }
};

// Grid: nouter * (h / T) blocks, tile-fastest, XCD-remapped like fwt_fwd_tile.
// src: level input (length h, stride 1); dst: coefficient array of the
// signal (details of level size hl at dst[hl/2 ..]); adst: level-K output.
template <int L, int NT, int T, int K, bool FMA>
__global__ __launch_bounds__(NT) void fwt_fwd_tile1(const double* __restrict__ src,
                                                    int64_t s_src, double* __restrict__ dst,
                                                    int64_t s_dst, double* __restrict__ adst,
                                                    int64_t s_adst, int h, FwdTaps<L> tp,
                                                    int sp, int lsw, int64_t ss) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using G = Fwd1Geo<L, T, K>;
  constexpr int M0 = G::m(0);
  const int ntile = h / T;
  const int b = tile_order(gridDim.x, sp);
  const int t = b % ntile;
  const int64_t o = b / ntile;
  const double* s = src + o * s_src;
  const int msk = h - 1, base = t * T;
  JWV_STAMP(0);
  load_window<1, NT, (M0 + NT - 1) / NT>(lds, s, M0, true, 0, 1,
                                          [&](int e) { return (int64_t)((base + e) & msk); });
  dma_fence_barrier();
  JWV_STAMP(1);
  Fwd1Level<L, NT, T, K, FMA, 1, false>::run(tp, lds, dst + o * s_dst, h, t, adst + o * s_adst,
                                                 sp, lsw, ss);
}

// ---------------------------------------------------------------- reverse
// Window of the level-l array (l = 0: the output): [tT/2^l - c_l, (t+1)T/2^l),
// c_0 = 0, c_{l+1} = ceil_even(c_l/2 + Q-1) (fwt_rev_tile's B_{l+1} recursion
// with every tile boundary even).  Needs T/2^K even.
template <int L, int T, int K>
struct Rev1Geo {
  static constexpr int Q = L / 2;
  static constexpr int c(int l) {
    int cc = 0;
    for (int k = 0; k < l; ++k) cc = ((cc / 2 + (Q - 1)) + 1) & ~1;
    return cc;
  }
  static constexpr int len(int l) { return (T >> l) + c(l); }
  // LDS: detail windows of levels K-1 .. 0 (each len(l+1)), then two
  // approximation buffers: buf[1] (len(1)), buf[0] (len(2)).  Level l reads
  // buf[(l+1)&1] and writes buf[l&1]; the initial level-K window goes to buf[K&1].
  static constexpr int doff(int l) {  // offset of level l's detail window
    int o = 0;
    for (int k = K - 1; k > l; --k) o += len(k + 1);
    return o;
  }
  static constexpr int dtotal() { return doff(-1); }
  static constexpr int buf1() { return dtotal(); }
  static constexpr int buf0() { return dtotal() + len(1); }
  // + 4: a couple of Rev1Level reads up to 3 values past its window
  static constexpr int lds_doubles() {
    return dtotal() + len(1) + (K >= 2 ? (len(2) > len(K) ? len(2) : len(K)) : 0) + 4;
  }
  // In-place layout (IP): [a_K | d_{K-1} | ... | d_0].  Every level reads its
  // approximations at 0 and writes its outputs over [0, len(l)) once every
  // lane has read (a second barrier per level), so LDS holds the input
  // windows only: rows of config 3 (T = 2048, K = 3) 27 -> 17 KB, 16-column
  // slabs (T = 256) 61 -> 39 KB, i.e. 5 -> 7 and 2 -> 4 blocks per CU.
  static constexpr int ip_doff(int l) {
    int o = len(K);
    for (int k = K - 1; k > l; --k) o += len(k + 1);
    return o;
  }
  static constexpr int ip_lds_doubles() { return ip_doff(-1) + 4; }
  static constexpr bool ip_fits() {  // level l's outputs end before d_{l-1}
    for (int l = 1; l < K; ++l)
      if (len(l) > ip_doff(l - 1)) return false;
    return true;
  }
  static_assert(((T >> K) & 1) == 0, "T/2^K must be even");
  static_assert(ip_fits(), "in-place level outputs must not reach unread windows");
};

// Each lane synthesises two adjacent pairs (ml, ml+1) of one level ("a
// couple"): they share Q-1 of their Q a/d inputs, so the lane reads Q+1 (+1
// for alignment) values per operand with 16-B LDS reads at a 16-B lane stride
// (conflict-free), instead of 2Q 8-B reads per pair.
#ifndef JWV_REV_COUPLE0
#define JWV_REV_COUPLE0 1
#endif
template <int L, int NT, int T, int K, bool FMA, int l, bool WT = false, bool CP = false,
          bool IP = false>
struct Rev1Level {
  // tl: the taps staged in LDS (stage_rev_taps; couples only): the array-head
  // pairs' rotated order reads them at a runtime index
  __device__ __forceinline__ static void run(const RevTaps<L>& tp, double* lds, int t,
                                             double* __restrict__ y, int sp = 0,
                                             const double* tl = nullptr) {
    using G = Rev1Geo<L, T, K>;
    JWV_STAMP(20 + l);
    constexpr int Q = G::Q;
    constexpr int np = G::len(l) / 2;               // pairs of this level's window
    constexpr int NC = (np + 1) / 2;                // couples
    constexpr int off = G::c(l + 1) - G::c(l) / 2;  // local index of a[pair 0]
    constexpr int sh = (off - (Q - 1)) & 1;         // 1: reads start one lower (even)
    constexpr int NR = (Q + 3) & ~1;                // values read per operand (even, >= Q+2)
    constexpr int R = (NC + NT - 1) / NT;
    constexpr int RS = (np + NT - 1) / NT;
    // CP: couples (throughput-bound tile passes; the latency-bound head and
    // chain kernels keep one pair per lane: twice the lanes per level).
    // Short banks (L <= 8: 2Q <= 8 reads per pair) measured slower with
    // couples on the HBM-bound 1D pass (config 2, +1.7 us/step); L = 16 rows
    // of config 3 gain 11% on the reverse tile at l > 0, and level 0 (the
    // global stores, two 16-B stores at a 32-B lane stride) another ~4%
    // (config 3 rev tiles 362 -> 341 us, 1.418 -> 1.402 ms/step over three
    // alternating runs on one box; JWV_REV_COUPLE0=0 restores one pair per
    // lane at level 0).
    constexpr bool kCouple = CP && L >= 12 && (l > 0 || JWV_REV_COUPLE0);
    static_assert(Q - 2 + G::c(l) / 2 < NT, "array-head pairs must sit in slot 0");
    const double* ab = lds + (IP ? 0 : (((l + 1) & 1) != 0) ? G::buf1() : G::buf0());
    const double* db = lds + (IP ? G::ip_doff(l) : G::doff(l));
    double* ob = lds + (IP ? 0 : ((l & 1) != 0) ? G::buf1() : G::buf0());
    const int tid = opaque_tid();  // per-level: keeps address math out of the prologue
    const int pbase = t * (T >> (l + 1)) - G::c(l) / 2;  // global index of window pair 0
    auto is_head = [&](int ml) { return pbase + ml >= 0 && pbase + ml < Q - 1; };
    auto put_now = [&](int ml, double xe, double xo) {
      if constexpr (l == 0) {  // WT: handed to another workgroup of this launch
        if constexpr (WT) st2<true>(y + (int64_t)t * T + 2 * ml, xe, xo);
        else st2_pol(y + (int64_t)t * T, 2 * ml, xe, xo, sp);
      } else {
        *reinterpret_cast<double2*>(ob + 2 * ml) = make_double2(xe, xo);
      }
    };
    // IP, l > 0: the outputs overwrite this level's inputs, so they wait in
    // registers (slot i of a compile-time index; ml < 0: nothing to write)
    // until every lane has read.
    constexpr bool DEF = IP && l > 0;
    constexpr int NPUT = DEF ? (kCouple ? 2 * R + 1 : RS) : 1;
    double2 dres[NPUT];
    int dml[NPUT];
#pragma unroll
    for (int i = 0; i < NPUT; ++i) dml[i] = -1;
    auto put = [&](int i, int ml, double xe, double xo, bool w) {
      if constexpr (DEF) {
        // slot fence: the next slot's window reads stay below this one
        asm volatile("" : "+v"(xe), "+v"(xo)::"memory");
        dres[i] = make_double2(xe, xo);
        dml[i] = w ? ml : -1;
      } else if (w) {
        put_now(ml, xe, xo);
      }
    };
    if constexpr (kCouple) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        if ((r + 1) * NT <= NC || k < NC) {
          const int ml = 2 * k;
          const int st = off + ml - (Q - 1) - sh;  // even
          double av[NR], dv[NR];
#pragma unroll
          for (int j = 0; j < NR; j += 2) {
            const double2 u = *reinterpret_cast<const double2*>(ab + st + j);
            const double2 w = *reinterpret_cast<const double2*>(db + st + j);
            av[j] = u.x;
            av[j + 1] = u.y;
            dv[j] = w.x;
            dv[j + 1] = w.y;
          }
          // window in registers here (else the loads sink into rev_pair's
          // term loop as ds_read2_b64 at odd offsets, see wpt1_kernels.hpp)
#pragma unroll
          for (int j = 0; j < NR; ++j) asm volatile("" : "+v"(av[j]), "+v"(dv[j]));
          // pair ml reads a[li - q] = av[(Q-1) + sh - q]; pair ml+1 one further
          double x0e, x0o, x1e, x1o;
          rev_pair<L, FMA>(tp, av + (Q - 1) + sh, dv + (Q - 1) + sh, 1, x0e, x0o);
          rev_pair<L, FMA>(tp, av + Q + sh, dv + Q + sh, 1, x1e, x1o);
          // array-head pairs are left to the fix-up below (block-uniform test)
          bool w0 = true, w1 = (np % 2 == 0) || ml + 1 < np;  // odd np: last couple single
          if (r == 0 && pbase < Q - 1) {
            w0 = !is_head(ml);
            w1 = w1 && !is_head(ml + 1);
          }
          put(2 * r, ml, x0e, x0o, w0);
          put(2 * r + 1, ml + 1, x1e, x1o, w1);
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < RS; ++r) {
        const int ml = tid + r * NT;
        if ((r + 1) * NT <= np || ml < np) {
          const int li = off + ml;
          double xe, xo;
          // array-head tiles (block-uniform): the rotated form for every pair
          // of the slot, r = Q-1 (the interior order) for non-head pairs
          if (r == 0 && pbase < Q - 1) {
            const int mg = pbase + ml;
            rev_pair_rot<L, FMA>(tp, [=](int q) { return ab[li - q]; },
                                 [=](int q) { return db[li - q]; }, is_head(ml) ? mg : Q - 1,
                                 xe, xo);
          } else {
            rev_pair<L, FMA>(tp, ab + li, db + li, 1, xe, xo);
          }
          put(r, ml, xe, xo, true);
        }
      }
    }
    // Couples: array-head pairs (global pair index mg < Q-1,
    // Wavelet.java:284-296 order = the interior order rotated, rev_pair_rot)
    // only in the first tiles of a row, one lane each, after the interior pass
    // so the rotation's registers are never live beside a couple's.
    if (kCouple && pbase < Q - 1 && tid < Q - 1) {
      const int ml = tid - pbase;
      if (ml >= 0 && ml < np) {
        const int li = off + ml;
        double xe, xo;
        // rotation r = mg = tid at a runtime index: taps from LDS, not a
        // Q x Q register select (~230 v_cndmask per level in wave 0 of every
        // head tile: a quarter of config 3's row tiles)
        rev_pair_rot_t<L, FMA>(tl, [=](int q) { return ab[li - q]; },
                               [=](int q) { return db[li - q]; }, tid, xe, xo);
        put(NPUT - 1, ml, xe, xo, true);
      }
    }
    if constexpr (DEF) {
      lds_barrier();
#pragma unroll
      for (int i = 0; i < NPUT; ++i)
        if (dml[i] >= 0) put_now(dml[i], dres[i].x, dres[i].y);
    }
    if constexpr (l > 0) {
      lds_barrier();
      Rev1Level<L, NT, T, K, FMA, l - 1, WT, CP, IP>::run(tp, lds, t, y, sp, tl);
    }
  }
};

// Grid: nouter * (hK / T) blocks.  asrc: level-K approximation (length
// h1/2 = hK >> K); coef: the coefficient array (details of level size h at
// coef[h/2 ..)); dst: output of length hK.
template <int L, int T, int K, bool IP>
__host__ __device__ constexpr int rev1_lds_doubles() {
  return IP ? Rev1Geo<L, T, K>::ip_lds_doubles() : Rev1Geo<L, T, K>::lds_doubles();
}

template <int L, int NT, int T, int K, bool FMA, bool IP>
__global__ __launch_bounds__(NT) void fwt_rev_tile1(const double* __restrict__ asrc,
                                                    int64_t s_a, const double* __restrict__ coef,
                                                    int64_t s_c, double* __restrict__ dst,
                                                    int64_t s_d, int hK, RevTaps<L> tp,
                                                    int sp, int lsw, int64_t ss) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ __attribute__((aligned(16))) double tl[2 * L];
  using G = Rev1Geo<L, T, K>;
  constexpr int MAXU = (G::len(1) + NT - 1) / NT;
  const int ntile = hK / T;
  const int b = tile_order(gridDim.x, sp);
  const int t = b % ntile;
  const int64_t o = b / ntile;
  const double* sa = asrc + o * s_a;
  const double* sc = coef + o * s_c;
  // every window in one burst: level-K approximation, then the details
  {
    const int BK = (t * T >> K) - G::c(K);
    const int am = (hK >> K) - 1;
    load_window<1, NT, MAXU>(lds + (IP ? 0 : (K & 1) ? G::buf1() : G::buf0()), sa, G::len(K),
                             true, 0, 1, [&](int e) { return (int64_t)((BK + e) & am); });
  }
#pragma unroll
  for (int l = K - 1; l >= 0; --l) {
    const int half = hK >> (l + 1), hm = half - 1;
    const int B = (t * T >> (l + 1)) - G::c(l + 1);
    // segmented coefficient rows (lsw < 31, see Fwd1Level): a 16-B piece
    // (e even, segments of even length) never straddles a segment
    const int sm = (int)((1u << (lsw & 31)) - 1u);
    load_window<1, NT, MAXU>(lds + (IP ? G::ip_doff(l) : G::doff(l)), sc, G::len(l + 1), true, 0,
                             1, [&](int e) {
                               const int i = half + ((B + e) & hm);
                               return (int64_t)(i >> lsw) * ss + (i & sm);
                             });
  }
  stage_rev_taps<L>(tp, tl);  // published by the barrier below
  dma_fence_barrier();
  Rev1Level<L, NT, T, K, FMA, K - 1, false, true, IP>::run(tp, lds, t, dst + o * s_d, sp, tl);
}

}  // namespace jwv
