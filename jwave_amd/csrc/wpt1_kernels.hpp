// wpt1_kernels.hpp — Wavelet Packet Transform tile kernels for contiguous
// packets (C = 1, stride 1, 16-B aligned rows) with compile-time geometry
// (tap count L, tile T, fused levels K).
//
// Reference: WaveletPacketTransform.forward (WaveletPacketTransform.java:73-124)
// transforms every packet of a level with Wavelet.forward (wrap inside the
// packet), output per packet [a | d], packet p of level l splitting into
// packets 2p (a) and 2p+1 (d) of level l+1; reverse (:141-191) undoes it
// level by level.  Math and summation order are those of Wavelet.forward /
// Wavelet.reverse (Wavelet.java:236-303), as in fwt_kernels.hpp.
//
// A block owns T consecutive samples (tile t) of one row (a packet of size h
// at the pass start) and runs K levels in LDS; only the last level touches
// HBM, so one pass reads and writes the array once.
//  forward: level-0 window [tT, tT + T + (L-2)(2^K-1)) mod h; level l holds
//           2^l sub-windows (one per packet) of m_l = T/2^l + (L-2)(2^(K-l)-1)
//           samples; periodicity of the row carries over to every packet.
//  reverse: level-l windows [tT/2^l - c_l, (t+1)T/2^l) of all 2^l packets
//           (c_l as in fwt1_kernels.hpp); level 0 = the T outputs.
// Levels run in place: every lane computes its pairs into registers, a
// barrier, then writes (two LDS-only barriers per level).
#pragma once
#include "fwt1_kernels.hpp"

// Round 5 (profiles/r05o, r05p, r05u, r05v): unsigned slot
// division, unpredicated reverse couple stores with the head pairs rewritten
// after a head-tile barrier, head pairs from LDS-staged taps, LDS-only levels
// without the +0.0 start (fwt_kernels.hpp ZS), FMA mode's reverse terms as two
// FMAs.

namespace jwv {

// ---------------------------------------------------------------- forward
template <int L, int T, int K>
struct Wpt1FwdGeo {
  static constexpr int m(int l) { return (T >> l) + (L - 2) * ((1 << (K - l)) - 1); }
  static constexpr int lds_doubles() { return m(0) + 2; }
  static_assert((L & 1) == 0 && ((T >> K) & 1) == 0, "even windows");
};

template <int L, int NT, int T, int K, bool FMA, int l>
struct Wpt1FwdLevel {
  // lds: 2^(l-1) input sub-windows of m(l-1) samples (stride m(l-1)).
  __device__ __forceinline__ static void run(const FwdTaps<L>& tp, double* lds, int h, int t,
                                             double* __restrict__ y) {
    using G = Wpt1FwdGeo<L, T, K>;
    constexpr int mi = G::m(l - 1), mo = G::m(l);
    constexpr int NC = (1 << (l - 1)) * (mo / 2);  // pair couples (2 adjacent pairs)
    constexpr int R = (NC + NT - 1) / NT;
    const int tid = opaque_tid();  // per-level: keeps address math out of the prologue
    double2 ra[R], rd[R];
    int wo[R];  // write-back offset (2s)*mo + i, kept from the read phase
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int q = tid + r * NT;
      if ((r + 1) * NT <= NC || q < NC) {
        const int s = (int)((unsigned)q / (unsigned)(mo / 2));       // sub-window
        const int i = (int)(2u * ((unsigned)q % (unsigned)(mo / 2)));  // first pair
        wo[r] = (2 * s) * mo + i;
        const double* in = lds + s * mi + 2 * i;
        double x[L + 2];
#pragma unroll
        for (int j = 0; j < L + 2; j += 2) {
          const double2 v = *reinterpret_cast<const double2*>(in + j);
          x[j] = v.x;
          x[j + 1] = v.y;
        }
        double a0, d0, a1, d1;
        if constexpr (JWV_WPT_FPIPE > 0 && !FMA) {
          fwd_couple_pipe<L, FMA, (JWV_WPT_FPIPE < L ? JWV_WPT_FPIPE : L), l == K>(
              tp, x, a0, d0, a1, d1);
        } else {
          fwd_pair<L, FMA>(tp, [&](int j) { return x[j]; }, a0, d0);
          fwd_pair<L, FMA>(tp, [&](int j) { return x[j + 2]; }, a1, d1);
        }
        // slot boundary: results exist here and later slots' LDS reads stay
        // below, so the compiler cannot hoist all slots' windows at once
        // (L = 16: ~190 VGPRs, 2 waves/SIMD -> ~80 VGPRs)
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(d0), "+v"(d1) :: "memory");
        if constexpr (l == K) {
          // packets 2s (a) and 2s+1 (d) of size h/2^K; own range t*T/2^K + i
          const int hp = h >> K;
          double* pa = y + (int64_t)(2 * s) * hp + t * (T >> K) + i;
          *reinterpret_cast<double2*>(pa) = make_double2(a0, a1);
          *reinterpret_cast<double2*>(pa + hp) = make_double2(d0, d1);
        } else {
          ra[r] = make_double2(a0, a1);
          rd[r] = make_double2(d0, d1);
        }
      }
    }
    if constexpr (l < K) {
      lds_barrier();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int q = tid + r * NT;
        if ((r + 1) * NT <= NC || q < NC) {
          *reinterpret_cast<double2*>(lds + wo[r]) = ra[r];
          *reinterpret_cast<double2*>(lds + wo[r] + mo) = rd[r];
        }
      }
      lds_barrier();
      Wpt1FwdLevel<L, NT, T, K, FMA, l + 1>::run(tp, lds, h, t, y);
    }
  }
};

// Trio form of the forward tile: a lane computes three adjacent pairs
// (3k .. 3k+2 of a sub-window) from L + 4 samples.  Couples start 4 doubles
// (two 16-B units) apart, so the 16 lanes of a ds_read_b128 group land on 8
// of the 16 unit slots of a bank row (2-way conflicts on every window read,
// SQ r06: 41.6% of LDS-active cycles); trios start 3 units apart and 3 is
// odd, so the group covers all 16 slots.  A trio also reads 10 units for 6
// outputs instead of 9 for 4 and spreads the per-slot address work over 6.
// Sub-windows are padded to whole trios (stride st(l), even): the trio that
// runs past a sub-window's last pair reads the next window's start (or the
// tail pad) and writes its surplus pairs into the padding, so only the level
// that stores to HBM needs a per-pair predicate.
template <int L, int T, int K>
struct Wpt3FwdGeo {
  static constexpr int m(int l) { return Wpt1FwdGeo<L, T, K>::m(l); }
  static constexpr int trios(int l) { return (m(l) + 2) / 3; }  // per sub-window of level l
  static constexpr int st(int l) { return l == 0 ? m(0) : (3 * trios(l) + 1) & ~1; }
  static constexpr int lds_doubles() {
    int n = m(0);
    for (int l = 1; l <= K; ++l) {
      const int rd = ((1 << (l - 1)) - 1) * st(l - 1) + 6 * (trios(l) - 1) + L + 4;
      n = rd > n ? rd : n;
      const int wr = l < K ? (1 << l) * st(l) : 0;
      n = wr > n ? wr : n;
    }
    return (n + 1) & ~1;
  }
};

template <int L, int NT, int T, int K, bool FMA, int l>
struct Wpt3FwdLevel {
  // lds: 2^(l-1) input sub-windows (stride st(l-1)); writes 2^l sub-windows
  // of m(l) samples at stride st(l) (a: 2s, d: 2s + 1)
  __device__ __forceinline__ static void run(const FwdTaps<L>& tp, double* lds, int h, int t,
                                             double* __restrict__ y) {
    using G = Wpt3FwdGeo<L, T, K>;
    constexpr int mi = G::st(l - 1), mo = G::m(l), so = G::st(l), M = G::trios(l);
    constexpr int NC = (1 << (l - 1)) * M;
    constexpr int R = (NC + NT - 1) / NT;
    const int tid = opaque_tid();
    double ra[R][3], rd[R][3];
    int wo[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int q = tid + r * NT;
      if ((r + 1) * NT <= NC || q < NC) {
        const int s = (int)((unsigned)q / (unsigned)M);  // sub-window
        const int k = q - s * M;                          // trio
        wo[r] = (2 * s) * so + 3 * k;
        const double* in = lds + s * mi + 6 * k;
        double x[L + 4];
#pragma unroll
        for (int j = 0; j < L + 4; j += 2) {
          const double2 v = *reinterpret_cast<const double2*>(in + j);
          x[j] = v.x;
          x[j + 1] = v.y;
        }
        double a[3], d[3];
        fwd_trio_pipe<L, FMA, 2, l == K>(tp, x, a, d);
        asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(d[0]), "+v"(d[1]),
                     "+v"(d[2]) :: "memory");  // slot boundary
        if constexpr (l == K) {
          // packets 2s (a) and 2s+1 (d) of size h/2^K; own range t*T/2^K + 3k
          const int hp = h >> K;
          double* pa = y + (int64_t)(2 * s) * hp + t * (T >> K) + 3 * k;
          double* pd = pa + hp;
#pragma unroll
          for (int p = 0; p < 3; ++p)
            if (mo % 3 == 0 || 3 * k + p < mo) {
              pa[p] = a[p];
              pd[p] = d[p];
            }
        } else {
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            ra[r][p] = a[p];
            rd[r][p] = d[p];
          }
        }
      }
    }
    if constexpr (l < K) {
      lds_barrier();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int q = tid + r * NT;
        if ((r + 1) * NT <= NC || q < NC) {
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            lds[wo[r] + p] = ra[r][p];
            lds[wo[r] + so + p] = rd[r][p];
          }
        }
      }
      lds_barrier();
      Wpt3FwdLevel<L, NT, T, K, FMA, l + 1>::run(tp, lds, h, t, y);
    }
  }
};

// Grid and window as wpt_fwd_tile1; the levels in trio form.
template <int L, int NT, int T, int K, bool FMA>
__global__ __launch_bounds__(NT) void wpt_fwd_tile3(const double* __restrict__ src, AxisView sv,
                                                    double* __restrict__ dst, AxisView dv, int h,
                                                    FwdTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int M0 = Wpt3FwdGeo<L, T, K>::m(0);
  const int ntile = h / T;
  const int nblk = gridDim.x;
  int b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  const int t = b % ntile;
  const int64_t o = b / ntile;
  const double* s = src + view_base(sv, o);
  const int msk = h - 1, base = t * T;
  load_window<1, NT, (M0 + NT - 1) / NT>(lds, s, M0, true, 0, 1,
                                          [&](int e) { return (int64_t)((base + e) & msk); });
  dma_fence_barrier();
  Wpt3FwdLevel<L, NT, T, K, FMA, 1>::run(tp, lds, h, t, dst + view_base(dv, o));
}

// Grid: rows * (h / T) blocks; row o = packet o of the pass input (view sv,
// packets addressed through view_base); output rows likewise (view dv).
template <int L, int NT, int T, int K, bool FMA>
__global__ __launch_bounds__(NT) void wpt_fwd_tile1(const double* __restrict__ src, AxisView sv,
                                                    double* __restrict__ dst, AxisView dv, int h,
                                                    FwdTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using G = Wpt1FwdGeo<L, T, K>;
  constexpr int M0 = G::m(0);
  const int ntile = h / T;
  const int nblk = gridDim.x;
  int b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  const int t = b % ntile;
  const int64_t o = b / ntile;
  const double* s = src + view_base(sv, o);
  const int msk = h - 1, base = t * T;
  load_window<1, NT, (M0 + NT - 1) / NT>(lds, s, M0, true, 0, 1,
                                          [&](int e) { return (int64_t)((base + e) & msk); });
  dma_fence_barrier();
  Wpt1FwdLevel<L, NT, T, K, FMA, 1>::run(tp, lds, h, t, dst + view_base(dv, o));
}

// ---------------------------------------------------------------- reverse
template <int L, int T, int K>
struct Wpt1RevGeo {
  using R = Rev1Geo<L, T, K>;
  static constexpr int len(int l) { return R::len(l); }
  static constexpr int c(int l) { return R::c(l); }
  // + 4: the odd-window couple tail reads up to two samples past a window
  static constexpr int lds_doubles() { return (1 << K) * len(K) + 4; }
};

// Couple (pairs m, m+1) of rev_pair with the term loop shared: A/D point at
// a[m], d[m]; the four sums keep rev_pair's per-output order (q descending),
// and are materialised after every term so the compiler cannot schedule the
// four dependent add chains one after the other (it does for two rev_pair
// calls: each add then waits on its predecessor).  Compiled-in L only.
template <int L, bool FMA>
__device__ __forceinline__ void rev_couple_ilv(const RevTaps<L>& tp, const double* A,
                                               const double* D, double& e0, double& o0,
                                               double& e1, double& o1) {
  constexpr int QE = (L + 1) / 2, QO = L / 2;
  double se0 = 0.0, so0 = 0.0, se1 = 0.0, so1 = 0.0;
  if constexpr (FMA) {
    // FMA mode: each term's two products go into the running sum as two
    // fused multiply-adds (2 instructions per term instead of mul, fma, add;
    // same terms, same term order, within FMA mode's 1e-12 contract)
#pragma unroll
    for (int q = QE - 1; q >= 0; --q) {
      const double a0 = A[-q], d0 = D[-q], a1 = A[1 - q], d1 = D[1 - q];
      se0 = __builtin_fma(a0, tp.lo_r[2 * q], se0);
      se1 = __builtin_fma(a1, tp.lo_r[2 * q], se1);
      if (q < QO) {
        so0 = __builtin_fma(a0, tp.lo_r[2 * q + 1], so0);
        so1 = __builtin_fma(a1, tp.lo_r[2 * q + 1], so1);
      }
      se0 = __builtin_fma(d0, tp.hi_r[2 * q], se0);
      se1 = __builtin_fma(d1, tp.hi_r[2 * q], se1);
      if (q < QO) {
        so0 = __builtin_fma(d0, tp.hi_r[2 * q + 1], so0);
        so1 = __builtin_fma(d1, tp.hi_r[2 * q + 1], so1);
      }
    }
    e0 = se0;
    o0 = so0;
    e1 = se1;
    o1 = so1;
    return;
  }
#pragma unroll
  for (int q = QE - 1; q >= 0; --q) {
    const double a0 = A[-q], d0 = D[-q], a1 = A[1 - q], d1 = D[1 - q];
    se0 += mac<FMA>(a0 * FB<L>::lor(tp, 2 * q), d0, FB<L>::hir(tp, 2 * q));
    se1 += mac<FMA>(a1 * FB<L>::lor(tp, 2 * q), d1, FB<L>::hir(tp, 2 * q));
    if (q < QO) {
      so0 += mac<FMA>(a0 * FB<L>::lor(tp, 2 * q + 1), d0, FB<L>::hir(tp, 2 * q + 1));
      so1 += mac<FMA>(a1 * FB<L>::lor(tp, 2 * q + 1), d1, FB<L>::hir(tp, 2 * q + 1));
    }
    asm volatile("" : "+v"(se0), "+v"(so0), "+v"(se1), "+v"(so1));
  }
  e0 = se0;
  o0 = so0;
  e1 = se1;
  o1 = so1;
}

template <int L, int NT, int T, int K, bool FMA, int l, bool ILV = false>
struct Wpt1RevLevel {
  // lds: 2^l packet windows of len(l) (stride len(l)); produces 2^(l-1)
  // windows of len(l-1) (level 1: the T outputs, to y).  Each lane computes
  // two adjacent pairs (ml, ml+1) from Q+2 registers per operand read with
  // (Q+2)/2 conflict-free 16-B LDS reads (lane stride 16 B).
  // Array-head pairs (global pair index < Q-1, Wavelet.java:284-296 order)
  // occur only in the first tiles: there, lanes tid < 2^(l-1)(Q-1) compute one
  // head pair each, and the couples skip storing them (one copy of the head
  // code per level instead of one per unrolled slot).
  // tl: the taps staged in LDS (the head pairs' rotated order reads them at a
  // runtime index, rev_pair_rot_t)
  __device__ __forceinline__ static void run(const RevTaps<L>& tp, double* lds, int t,
                                             double* __restrict__ y, const double* tl) {
    using G = Wpt1RevGeo<L, T, K>;
    constexpr int Q = L / 2;
    constexpr int li_ = G::len(l), lo_ = G::len(l - 1);  // window strides in LDS
    constexpr int NW = 1 << (l - 1);                // output windows
    constexpr int NPW = G::len(l - 1) / 2;          // pairs per output window
    constexpr int NCW = (NPW + 1) / 2;              // couples per output window
    constexpr int NC = NW * NCW;                    // couples of the level
    constexpr int off = G::c(l) - G::c(l - 1) / 2;  // local index of a[pair 0]
    // couple k reads a[off + 2k - (Q-1) .. off + 2k + 1] from an even start
    constexpr int sh = (off - (Q - 1)) & 1;         // 1: start one lower
    constexpr int NR = (Q + 3) & ~1;                // registers per operand (even, >= Q+2)
    constexpr int R = (NC + NT - 1) / NT;
    static_assert(NW * (Q - 1) <= NT, "one head pair per lane");
    const int tid = opaque_tid();  // per-level: keeps address math out of the prologue
    const int pbase = t * (T >> l) - G::c(l - 1) / 2;  // global index of pair 0
    const bool head_tile = pbase < Q - 1;              // block-uniform
    double4 rx[R];
    int wo[R];  // write-back: (s*lo_ + 2*ml) << 2 | w1 << 1 | w0, kept from the read phase
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = tid + r * NT;
      if ((r + 1) * NT <= NC || k < NC) {
        const int s = (int)((unsigned)k / (unsigned)NCW);
        const int ml = (int)(2u * ((unsigned)k % (unsigned)NCW));
        const double* ab = lds + (2 * s) * li_;
        const double* db = ab + li_;
        const int st = off + ml - (Q - 1) - sh;  // even
        double av[NR], dv[NR];
#pragma unroll
        for (int j = 0; j < NR; j += 2) {
          const double2 u = ld16(ab + st + j);
          const double2 w = ld16(db + st + j);
          av[j] = u.x; av[j + 1] = u.y;
          dv[j] = w.x; dv[j + 1] = w.y;
        }
        // the window in registers here: left to itself the compiler sinks
        // the loads into the term loop as per-term ds_read2_b64 at odd
        // offsets (8 cycles each, 2-way conflicted), not 16-B ds_read_b128
#pragma unroll
        for (int j = 0; j < NR; ++j) asm volatile("" : "+v"(av[j]), "+v"(dv[j]));
        // pair ml: a[li - q] = av[(Q-1) + sh - q]; pair ml+1: one further
        double x0e, x0o, x1e, x1o;
        if constexpr (ILV && !FMA && JWV_WPT_RPIPE > 0 && (L / 2) % JWV_WPT_RPIPE == 0) {
          rev_couple_pipe<L, JWV_WPT_RPIPE, l == 1>(tp, av + (Q - 1) + sh, dv + (Q - 1) + sh, x0e, x0o,
                                            x1e, x1o);
        } else if constexpr (ILV) {
          rev_couple_ilv<L, FMA>(tp, av + (Q - 1) + sh, dv + (Q - 1) + sh, x0e, x0o, x1e, x1o);
        } else {
          rev_pair<L, FMA>(tp, av + (Q - 1) + sh, dv + (Q - 1) + sh, 1, x0e, x0o);
          rev_pair<L, FMA>(tp, av + Q + sh, dv + Q + sh, 1, x1e, x1o);
        }
        asm volatile("" : "+v"(x0e), "+v"(x0o), "+v"(x1e), "+v"(x1o) :: "memory");  // slot boundary
        // array-head pairs are stored like the others and overwritten by the
        // head lanes after one more barrier (head tiles only, below)
        const bool w0 = true;
        const bool w1 = (NPW % 2 == 0) || ml + 1 < NPW;
        if constexpr (l == 1) {
          double* yo = y + (int64_t)t * T + 2 * ml;
          if (w0) *reinterpret_cast<double2*>(yo) = make_double2(x0e, x0o);
          if (w1) *reinterpret_cast<double2*>(yo + 2) = make_double2(x1e, x1o);
        } else {
          rx[r] = make_double4(x0e, x0o, x1e, x1o);
          wo[r] = ((s * lo_ + 2 * ml) << 2) | (w1 ? 2 : 0) | (w0 ? 1 : 0);
        }
      }
    }
    // head pairs: lane -> (window hs, global pair hm)
    int hs = -1, hml = 0;
    double hxe = 0.0, hxo = 0.0;
    if (Q > 1 && head_tile && tid < NW * (Q - 1)) {
      constexpr int Q1 = Q > 1 ? Q - 1 : 1;  // Haar (Q = 1) has no head pairs
      const int s = tid / Q1, m = tid % Q1, ml = m - pbase;
      if (ml >= 0 && ml < NPW) {
        const double* ab = lds + (2 * s) * li_;
        const double* db = ab + li_;
        const int li = off + ml;
        rev_pair_rot_t<L, FMA>(tl, [=](int q) { return ab[li - q]; },
                               [=](int q) { return db[li - q]; }, m, hxe, hxo);
        hs = s;
        hml = ml;
      }
    }
    if constexpr (l == 1) {
      if (head_tile) {
        __syncthreads();  // the couples' stores of the head pairs first (workgroup order)
        if (hs >= 0) *reinterpret_cast<double2*>(y + (int64_t)t * T + 2 * hml) = make_double2(hxe, hxo);
      }
    } else {
      lds_barrier();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        if ((r + 1) * NT <= NC || k < NC) {
          double* ob = lds + (wo[r] >> 2);
          if (wo[r] & 1) *reinterpret_cast<double2*>(ob) = make_double2(rx[r].x, rx[r].y);
          if (wo[r] & 2) *reinterpret_cast<double2*>(ob + 2) = make_double2(rx[r].z, rx[r].w);
        }
      }
      if (head_tile) {
        lds_barrier();
        if (hs >= 0) *reinterpret_cast<double2*>(lds + hs * lo_ + 2 * hml) = make_double2(hxe, hxo);
      }
      lds_barrier();
      Wpt1RevLevel<L, NT, T, K, FMA, l - 1, ILV>::run(tp, lds, t, y, tl);
    }
  }
};

// Grid: rows * (h / T) blocks; h = output packet size of the pass; input
// row o holds 2^K packets of h/2^K (view sv), output row o (view dv).
template <int L, int NT, int T, int K, bool FMA, bool ILV = false>
__global__ __launch_bounds__(NT) void wpt_rev_tile1(const double* __restrict__ src, AxisView sv,
                                                    double* __restrict__ dst, AxisView dv, int h,
                                                    RevTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ __attribute__((aligned(16))) double tl[2 * L];
  using G = Wpt1RevGeo<L, T, K>;
  constexpr int LK = G::len(K);
  constexpr int NW = 1 << K;
  const int ntile = h / T;
  const int nblk = gridDim.x;
  int b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  const int t = b % ntile;
  const int64_t o = b / ntile;
  const double* s = src + view_base(sv, o);
  const int hp = h >> K, pm = hp - 1;
  const int BK = t * (T >> K) - G::c(K);
  // all 2^K packet windows in one burst: window w -> lds[w * LK ..)
  load_window<1, NT, (NW * LK + NT - 1) / NT>(
      lds, s, NW * LK, true, 0, 1, [&](int e) {
        const int w = e / LK, k = e - w * LK;
        return (int64_t)w * hp + ((BK + k) & pm);
      });
  stage_rev_taps<L>(tp, tl);  // published by the barrier below
  dma_fence_barrier();
  Wpt1RevLevel<L, NT, T, K, FMA, K, ILV>::run(tp, lds, t, dst + view_base(dv, o), tl);
}

}  // namespace jwv
