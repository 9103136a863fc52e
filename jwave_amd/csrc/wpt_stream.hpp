// wpt_stream.hpp — WaveletPacketTransform forward (WaveletPacketTransform.java:
// 73-124) over rows of packets as a stream of tiles with carried halos
// (compile-time L, T, K; contiguous 16-B aligned rows, even K).
//
// Same math and summation order as wpt_fwd_tile1 (Wavelet.forward,
// Wavelet.java:236-255, wrap inside every packet): EXACT results are
// bit-identical.  What changes is the right halo.  The tile kernel owns T
// samples of a row and recomputes (L-2)(2^(K-l)-1) halo samples per packet
// at every level l (config 4, T = 8192: 7.3% extra FP64, and 72 KB of LDS
// per block).  Here a block owns a run of consecutive tiles (one or more row
// segments) and walks each segment from the right: the halo of tile t's
// level-l input packet, its first L-2 samples right of the tile, is the head
// of that packet in tile t+1, which the block saved (the carry) when it ran
// tile t+1.  Every level then computes exactly T/2 pairs (T/4 couples, an
// exact multiple of the block), the input of level l sits in one of two
// parity buffers (one barrier per level), and the row window of the NEXT
// tile comes in through registers while this tile runs.  A segment's
// rightmost tile takes its carries from a prologue that runs the halo
// recursion once (at most one per row per block).
#pragma once
#include <cstddef>
#include "wpt1_kernels.hpp"

namespace jwv {

// The streamed kernels' single argument.  Their tile loop keeps more scalar
// state live than the one-tile kernels, and with the 32 FP64 taps (64 SGPRs)
// held across it the compiler spilled SGPRs to VGPR lanes (one v_readlane
// per tap use in the reverse: 2.6 readlanes per FP64 instruction).  So every
// level reloads the taps from the kernel-argument segment (scalar loads,
// K$ hits) and they live only inside the level.
template <typename Taps>
struct WptStreamArgs {
  const double* src;
  AxisView sv;
  double* dst;
  AxisView dv;
  int64_t ntile;
  int h;
  int pad_;
  Taps tp;
};
template <typename Taps>
__device__ __forceinline__ Taps stream_taps() {
  using CD = const __attribute__((address_space(4))) double;
  constexpr int n = sizeof(Taps) / sizeof(double);
  static_assert(offsetof(WptStreamArgs<Taps>, tp) % 8 == 0, "taps at a double boundary");
  CD* p = (CD*)((const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() +
                offsetof(WptStreamArgs<Taps>, tp));
  asm volatile("" : "+s"(p));  // a fresh pointer per level: loads stay in the level
  Taps t;
  double* d = reinterpret_cast<double*>(&t);
#pragma unroll
  for (int i = 0; i < n; ++i) d[i] = p[i];
  return t;
}

template <int L, int T, int K>
struct WptFStreamGeo {
  static constexpr int Q0 = L - 2;                              // halo per packet
  static constexpr int Tl(int l) { return T >> (l - 1); }       // own samples / packet, level-l input
  static constexpr int np(int l) { return 1 << (l - 1); }       // packets, level-l input
  static constexpr int m(int l) { return Tl(l) + Q0; }          // packet stride in LDS
  static constexpr int isz(int l) { return np(l) * m(l); }
  static constexpr int bsize(int p) {
    int b = 0;
    for (int l = 1; l <= K; ++l)
      if ((l & 1) == p && isz(l) + 2 > b) b = isz(l) + 2;
    return (b + 1) & ~1;
  }
  static constexpr int buf(int p) { return p ? bsize(0) : 0; }
  // carry of level l's outputs (1 <= l < K): 2^l packets x Q0
  static constexpr int coff(int l) { return Q0 * ((1 << l) - 2); }
  static constexpr int carry0() { return bsize(0) + bsize(1); }
  static constexpr int lds_doubles() { return carry0() + coff(K); }
  // prologue: E(l) = outputs per packet of level l needed left-aligned at the
  // segment's right end (E(K-1) = Q0: the carry; E(0) = the row window)
  static constexpr int E(int l) { return l >= K - 1 ? Q0 : 2 * E(l + 1) + Q0; }
  static constexpr int pin(int l) { return np(l) * E(l - 1); }  // prologue input of level l
  static constexpr int preg(int p) { return p ? ((pin(1) + 3) & ~1) : 0; }
  static_assert(preg(1) + pin(2) + 2 <= bsize(0), "prologue regions inside buffer 0");
  static_assert((K & 1) == 0 && K >= 2, "even K: the row window goes in during level K");
  static_assert((Tl(K) & 3) == 0 && (Q0 & 1) == 0, "couples tile every packet");
};

template <int L, int NT, int T, int K, bool FMA>
struct WptFStream {
  using G = WptFStreamGeo<L, T, K>;
  static constexpr int Q0 = G::Q0;
  static constexpr int nq(int n) { return ((n + 1) / 2 + NT - 1) / NT; }
  static constexpr int kQX = nq(G::m(1));
  static constexpr int kQP = nq(G::E(0));

  // row samples [s0, s0 + n) mod h (s0, h even: a 16-B piece never straddles
  // the wrap) into registers: one buffer load per piece on every path
  template <int n, int Q>
  __device__ __forceinline__ static void fetch(double2 (&r)[Q], const double* __restrict__ row,
                                               int s0, int h) {
    constexpr int n2 = (n + 1) / 2;
    static_assert(nq(n) <= Q, "window pieces");
    const int tid = opaque_tid();
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(row), 0, h * 8, 0x00020000);
#pragma unroll
    for (int q = 0; q < nq(n); ++q) {
      int e = 2 * (tid + q * NT);
      if ((q + 1) * NT > n2) e = e < 2 * n2 ? e : 2 * (n2 - 1);
      int g = s0 + e;
      g = g >= h ? g - h : g;
      r[q] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, g * 8, 0, 0));
    }
  }
  template <int n, int Q>
  __device__ __forceinline__ static void put(double* lds, const double2 (&r)[Q]) {
    constexpr int n2 = (n + 1) / 2;
    const int tid = opaque_tid();
#pragma unroll
    for (int q = 0; q < nq(n); ++q)
      if ((q + 1) * NT <= n2 || tid + q * NT < n2) st16(lds + 2 * (tid + q * NT), r[q].x, r[q].y);
  }

  // ---- prologue: carries of the tile right of the segment (row position c1)
  // Level l turns np(l) packets of E(l-1) samples into 2 np(l) packets of
  // E(l); the first Q0 of every output packet are the carry of level l.
  template <int l>
  __device__ __forceinline__ static void pro_level(double* lds) {
    if constexpr (l < K) {
      const FwdTaps<L> tp = stream_taps<FwdTaps<L>>();
      constexpr int mi = G::E(l - 1), mo = G::E(l), npk = G::np(l);
      constexpr int NPR = npk * mo, R = (NPR + NT - 1) / NT;  // pairs
      const int tid = opaque_tid();
      const double* in = lds + G::preg((l - 1) & 1);
      double* out = lds + G::preg(l & 1);
      double* cw = lds + G::carry0() + G::coff(l);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        if ((r + 1) * NT <= NPR || k < NPR) {
          const int s = k / mo, i = k - s * mo;
          const double* x = in + s * mi + 2 * i;
          double v[L];
#pragma unroll
          for (int j = 0; j < L; j += 2) {
            const double2 u = ld16(x + j);
            v[j] = u.x;
            v[j + 1] = u.y;
          }
          double a, d;
          fwd_pair<L, FMA>(tp, [&](int j) { return v[j]; }, a, d);
          if constexpr (l < K - 1) {
            out[(2 * s) * mo + i] = a;
            out[(2 * s + 1) * mo + i] = d;
          }
          if (i < Q0) {
            cw[(2 * s) * Q0 + i] = a;
            cw[(2 * s + 1) * Q0 + i] = d;
          }
        }
      }
      lds_barrier();
      pro_level<l + 1>(lds);
    }
  }

  // ---- main loop: level l of tile t of the row at y
  template <int l>
  __device__ __forceinline__ static void level(double* lds, double* __restrict__ y, int h, int t,
                                               const double* __restrict__ rown, int sn,
                                               double2 (&rx)[kQX]) {
    constexpr int mi = G::m(l), Tli = G::Tl(l);
    constexpr int NC = T / 4, R = NC / NT, CPP = Tli / 4;  // couples, per lane, per packet
    static_assert(R * NT == NC, "T = 4 NT R");
    const int tid = opaque_tid();
    const FwdTaps<L> tp = stream_taps<FwdTaps<L>>();
    const double* in = lds + G::buf(l & 1);
    // carry traffic in registers (read before the sums, written after):
    // the tails of this level's output packets (heads of tile t+1's) and the
    // heads of this level's input packets (for tile t-1)
    constexpr int CT = l < K ? (1 << l) * Q0 : 0, CS = l >= 2 ? G::np(l) * Q0 : 0;
    constexpr int RT = (CT + NT - 1) / NT, RS = (CS + NT - 1) / NT;
    double tv[RT > 0 ? RT : 1], hv[RS > 0 ? RS : 1];
    if constexpr (CT > 0) {
      const double* cr = lds + G::carry0() + G::coff(l);
#pragma unroll
      for (int r = 0; r < RT; ++r)
        if ((r + 1) * NT <= CT || tid + r * NT < CT) tv[r] = cr[tid + r * NT];
    }
#pragma unroll
    for (int r = 0; r < RS; ++r) {
      const int v = tid + r * NT;
      if ((r + 1) * NT <= CS || v < CS) hv[r] = in[(v / Q0) * mi + v % Q0];
    }
    double2 ra[R], rd[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = tid + r * NT;
      const int s = k / CPP, i = 2 * (k - s * CPP);  // packet, first pair
      const double* x = in + s * mi + 2 * i;
      double xv[L + 2];
#pragma unroll
      for (int j = 0; j < L + 2; j += 2) {
        const double2 u = ld16(x + j);
        xv[j] = u.x;
        xv[j + 1] = u.y;
      }
#pragma unroll
      for (int j = 0; j < L + 2; ++j) asm volatile("" : "+v"(xv[j]));
      double a0, d0, a1, d1;
      fwd_pair<L, FMA>(tp, [&](int j) { return xv[j]; }, a0, d0);
      fwd_pair<L, FMA>(tp, [&](int j) { return xv[j + 2]; }, a1, d1);
      asm volatile("" : "+v"(a0), "+v"(a1), "+v"(d0), "+v"(d1) :: "memory");
      ra[r] = make_double2(a0, a1);
      rd[r] = make_double2(d0, d1);
    }
    if constexpr (CS > 0) {
      double* cw = lds + G::carry0() + G::coff(l - 1);
#pragma unroll
      for (int r = 0; r < RS; ++r)
        if ((r + 1) * NT <= CS || tid + r * NT < CS) cw[tid + r * NT] = hv[r];
    }
    if constexpr (l < K) {
      constexpr int mo = G::m(l + 1), Tlo = G::Tl(l + 1);
      double* out = lds + G::buf((l + 1) & 1);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        const int s = k / CPP, i = 2 * (k - s * CPP);
        st16(out + (2 * s) * mo + i, ra[r].x, ra[r].y);
        st16(out + (2 * s + 1) * mo + i, rd[r].x, rd[r].y);
      }
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const int v = tid + r * NT;
        if ((r + 1) * NT <= CT || v < CT) out[(v / Q0) * mo + Tlo + v % Q0] = tv[r];
      }
    } else {
      // packets 2s (a) and 2s+1 (d) of size h/2^K; own range t*T/2^K + i
      const int hp = h >> K;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        const int s = k / CPP, i = 2 * (k - s * CPP);
        double* pa = y + (int64_t)(2 * s) * hp + t * (T >> K) + i;
        st16(pa, ra[r].x, ra[r].y);
        st16(pa + hp, rd[r].x, rd[r].y);
      }
      // the next tile's row window into the level-1 buffer (level K reads
      // the other parity), then its registers take the tile after that
      put<G::m(1)>(lds + G::buf(1), rx);
      fetch<G::m(1)>(rx, rown, sn, h);
    }
    lds_barrier();
    if constexpr (l < K) level<l + 1>(lds, y, h, t, rown, sn, rx);
  }
};

// Grid: blocks share the rows * (h/T) tiles (global index g = row * (h/T) +
// tile) in contiguous runs; a block walks its run from the top.  src / dst
// rows as in wpt_fwd_tile1 (16-B aligned rows, h a multiple of T).
template <int L, int NT, int T, int K, bool FMA>
__global__ __launch_bounds__(NT) void wpt_fwd_stream(WptStreamArgs<FwdTaps<L>> args) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const double* __restrict__ src = args.src;
  double* __restrict__ dst = args.dst;
  const AxisView sv = args.sv, dv = args.dv;
  const int h = args.h;
  const int64_t ntile = args.ntile;
  using S = WptFStream<L, NT, T, K, FMA>;
  using G = WptFStreamGeo<L, T, K>;
  const int64_t b = blockIdx.x, nb = gridDim.x;
  const int64_t ga = b * ntile / nb, gb = (b + 1) * ntile / nb;
  if (ga >= gb) return;  // block-uniform (never with nb <= ntile)
  const int ntr = h / T;
  // the tile after g in walk order (downwards; past the run: g itself)
  const auto next_of = [&](int64_t g) { return g - 1 >= ga ? g - 1 : g; };
  double2 rx[S::kQX];
  {
    // the first tile's row window into the level-1 buffer, then the
    // registers take the next one's
    const int64_t o = (gb - 1) / ntr;
    S::template fetch<G::m(1)>(rx, src + view_base(sv, o), (int)((gb - 1) - o * ntr) * T, h);
    S::template put<G::m(1)>(lds + G::buf(1), rx);
    const int64_t gn = next_of(gb - 1), on = gn / ntr;
    S::template fetch<G::m(1)>(rx, src + view_base(sv, on), (int)(gn - on * ntr) * T, h);
  }
  for (int64_t g = gb - 1; g >= ga; --g) {
    const int64_t o = g / ntr;
    const int t = (int)(g - o * ntr);
    if (g == gb - 1 || t == ntr - 1) {
      // a row segment starts: the carries at the row position right of tile
      // t (prologue regions in buffer 0; buffer 1 holds tile t's window)
      const int c1 = t + 1 < ntr ? (t + 1) * T : 0;
      double2 px[S::kQP];
      S::template fetch<G::E(0)>(px, src + view_base(sv, o), c1, h);
      S::template put<G::E(0)>(lds + G::preg(0), px);
      lds_barrier();
      S::template pro_level<1>(lds);
    }
    const int64_t gn = next_of(next_of(g)), on = gn / ntr;
    S::template level<1>(lds, dst + view_base(dv, o), h, t, src + view_base(sv, on),
                         (int)(gn - on * ntr) * T, rx);
  }
}


// ---------------------------------------------------------------- reverse
// WaveletPacketTransform.reverse (WaveletPacketTransform.java:141-191) as a
// left-to-right stream: level l (K .. 1) merges packets 2s (a) and 2s+1 (d)
// of level-l data into packet s of level l-1; output pair m reads a[m-q],
// d[m-q], q < Q = L/2 (Wavelet.reverse, Wavelet.java:270-303), so the halo
// is the Q-1 values LEFT of the tile in every input packet: the tail of that
// packet in tile t-1, carried.  Level-l data sit in the buffer of the parity
// of l, every packet as [pad | Q-1 halo | T/2^l own] (stride T/2^l + Q), so a
// couple's reads are 16-B aligned.  Level K's bands come from HBM with their
// halo (one tile ahead, through registers); level 1 writes the row.  A row's
// tile 0 holds the array-head pairs (m < Q-1), summed in the scatter order
// of rev_pair_head over the wrapped halo, as in wpt_rev_tile1.
template <int L, int T, int K>
struct WptRStreamGeo {
  static constexpr int Q = L / 2, H = Q - 1;
  static constexpr int Tl(int l) { return T >> l; }          // own values per packet, level-l data
  static constexpr int np(int l) { return 1 << l; }           // packets of level-l data
  static constexpr int m(int l) { return Tl(l) + Q; }         // packet stride
  static constexpr int isz(int l) { return np(l) * m(l); }
  static constexpr int bsize(int p) {
    int b = 0;
    for (int l = 1; l <= K; ++l)
      if ((l & 1) == p && isz(l) + 4 > b) b = isz(l) + 4;
    return (b + 1) & ~1;
  }
  static constexpr int buf(int p) { return p ? bsize(0) : 0; }
  // carry of level-l data (1 <= l < K): np(l) packets x H
  static constexpr int coff(int l) { return H * ((1 << l) - 2); }
  static constexpr int carry0() { return bsize(0) + bsize(1); }
  static constexpr int lds_doubles() { return carry0() + coff(K); }
  // prologue: level l (K .. 2) computes P(l) trailing pairs per output packet
  // from D(l) = P(l) + H trailing values per input packet; D(1) = H (carry)
  static constexpr int D(int l) { return l <= 1 ? H : P(l) + H; }
  static constexpr int P(int l) { return (D(l - 1) + 1) / 2; }
  static constexpr int pin(int l) { return np(l) * D(l); }
  static constexpr int pout(int l) { return np(l - 1) * 2 * P(l); }
  static constexpr int preg(int p) { return p ? ((pin(K) + 3) & ~1) : 0; }
  static_assert(preg(1) + pout(K) + 2 <= bsize((K - 1) & 1) && pin(K - 1) <= pout(K),
                "prologue regions");
  static_assert((K & 1) == 0 && K >= 2 && (Tl(K) & 1) == 0 && Tl(K) >= Q, "geometry");
};

template <int L, int NT, int T, int K, bool FMA>
struct WptRStream {
  using G = WptRStreamGeo<L, T, K>;
  static constexpr int Q = G::Q, H = G::H;
  static constexpr int kNB = G::np(K) * G::m(K);  // band window doubles
  static constexpr int kQB = (kNB / 2 + NT - 1) / NT;

  // level-K bands of tile t: packet p, values [t Tl(K) - Q, (t+1) Tl(K)) mod
  // hp, into registers; one buffer load per 16-B piece on every path
  __device__ __forceinline__ static void fetch(double2 (&r)[kQB], const double* __restrict__ row,
                                               int t, int h) {
    constexpr int n2 = kNB / 2, PP = G::m(K) / 2;  // pieces per packet window
    const int tid = opaque_tid();
    const int hp = h >> K;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(row), 0, h * 8, 0x00020000);
    const int b0 = t * G::Tl(K) - Q;
#pragma unroll
    for (int q = 0; q < kQB; ++q) {
      int e = tid + q * NT;
      if ((q + 1) * NT > n2) e = e < n2 ? e : n2 - 1;
      const int p = e / PP;
      int x = b0 + 2 * (e - p * PP);
      x = x < 0 ? x + hp : x;
      r[q] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(
                                             rs, (p * hp + x) * 8, 0, 0));
    }
  }
  __device__ __forceinline__ static void put(double* lds, const double2 (&r)[kQB]) {
    constexpr int n2 = kNB / 2;
    const int tid = opaque_tid();
#pragma unroll
    for (int q = 0; q < kQB; ++q)
      if ((q + 1) * NT <= n2 || tid + q * NT < n2) st16(lds + 2 * (tid + q * NT), r[q].x, r[q].y);
  }

  // ---- prologue: carries of the tile left of the segment (tile t0 - 1).
  // Prologue level l holds np(l) packets of D(l) trailing values (stride
  // D(l) + 1 for l = K: the band load; else 2 P(l+1)), and writes np(l-1)
  // packets of 2 P(l) values; every level-l data tail (H) is a carry.
  template <int l>
  __device__ __forceinline__ static void pro_level(double* lds, double* pb) {
    if constexpr (l >= 2) {
      const RevTaps<L> tp = stream_taps<RevTaps<L>>();
      constexpr int si = l == K ? G::D(K) : 2 * G::P(l + 1);  // input packet stride
      constexpr int bi = si - G::D(l);                          // first used value
      constexpr int pl = G::P(l), so = 2 * pl, nw = G::np(l - 1);
      constexpr int NPR = nw * pl, R = (NPR + NT - 1) / NT;
      const int tid = opaque_tid();
      const double* in = pb + G::preg((K - l) & 1);
      double* out = pb + G::preg((K - l + 1) & 1);
      // the carry of level-l data itself (l < K): the input packets' tails
      if constexpr (l < K) {
        double* cl = lds + G::carry0() + G::coff(l);
        for (int v = tid; v < G::np(l) * H; v += NT)
          cl[v] = in[(v / H) * si + si - H + v % H];
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        if ((r + 1) * NT <= NPR || k < NPR) {
          const int s = k / pl, j = k - s * pl;
          const double* ab = in + (2 * s) * si + bi;
          const double* db = ab + si;
          double av[Q], dv[Q];
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            av[q] = ab[H + j - q];
            dv[q] = db[H + j - q];
          }
          double xe, xo;
          rev_pair<L, FMA>(tp, av + 0, dv + 0, -1, xe, xo);  // A[-q*st] = av[q]
          out[s * so + 2 * j] = xe;
          out[s * so + 2 * j + 1] = xo;
        }
      }
      lds_barrier();
      if constexpr (l == 2) {  // level-1 data: its tail is the last carry
        double* c1 = lds + G::carry0() + G::coff(1);
        for (int v = tid; v < G::np(1) * H; v += NT) c1[v] = out[(v / H) * so + so - H + v % H];
        lds_barrier();
      }
      pro_level<l - 1>(lds, pb);
    }
  }

  // ---- main loop: level l of tile t (row output y)
  template <int l>
  __device__ __forceinline__ static void level(double* lds, double* __restrict__ y, int t, bool head,
                                               const double* __restrict__ rown, int tn, int h,
                                               double2 (&rb)[kQB]) {
    constexpr int mi = G::m(l), Tli = G::Tl(l);
    constexpr int NC = T / 4, R = NC / NT, NCW = Tli / 2;  // couples, per lane, per packet
    static_assert(R * NT == NC, "T = 4 NT R");
    const int tid = opaque_tid();
    const RevTaps<L> tp = stream_taps<RevTaps<L>>();
    const double* in = lds + G::buf(l & 1);
    // carries in registers: the halo of level-(l-1) data (l >= 2) and the
    // tails of this level's input packets (l < K) for the next tile
    constexpr int CH = l >= 2 ? G::np(l - 1) * H : 0, CS = l < K ? G::np(l) * H : 0;
    constexpr int RH = (CH + NT - 1) / NT, RS = (CS + NT - 1) / NT;
    double hv[RH > 0 ? RH : 1], sv[RS > 0 ? RS : 1];
    if constexpr (CH > 0) {
      const double* cr = lds + G::carry0() + G::coff(l - 1);
#pragma unroll
      for (int r = 0; r < RH; ++r)
        if ((r + 1) * NT <= CH || tid + r * NT < CH) hv[r] = cr[tid + r * NT];
    }
#pragma unroll
    for (int r = 0; r < RS; ++r) {
      const int v = tid + r * NT;
      if ((r + 1) * NT <= CS || v < CS) sv[r] = in[(v / H) * mi + Q + Tli - H + v % H];
    }
    double4 rx[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = tid + r * NT;
      const int s = k / NCW, ml = 2 * (k - s * NCW);
      const double* ab = in + (2 * s) * mi + ml;  // a[ml - H - 1 ..], 16-B aligned
      const double* db = ab + mi;
      double av[10], dv[10];
      static_assert(Q + 2 <= 10, "couple registers");
#pragma unroll
      for (int j = 0; j < Q + 2; j += 2) {
        const double2 u = ld16(ab + j), w = ld16(db + j);
        av[j] = u.x; av[j + 1] = u.y;
        dv[j] = w.x; dv[j + 1] = w.y;
      }
#pragma unroll
      for (int j = 0; j < Q + 2; ++j) asm volatile("" : "+v"(av[j]), "+v"(dv[j]));
      // pair ml: A[-q] = a[ml - q] = av[Q - q]; pair ml + 1 one further
      double x0e, x0o, x1e, x1o;
      rev_couple_ilv<L, FMA>(tp, av + Q, dv + Q, x0e, x0o, x1e, x1o);
      asm volatile("" : "+v"(x0e), "+v"(x0o), "+v"(x1e), "+v"(x1o) :: "memory");
      rx[r] = make_double4(x0e, x0o, x1e, x1o);
    }
    if constexpr (CS > 0) {
      double* cw = lds + G::carry0() + G::coff(l);
#pragma unroll
      for (int r = 0; r < RS; ++r)
        if ((r + 1) * NT <= CS || tid + r * NT < CS) cw[tid + r * NT] = sv[r];
    }
    // array-head pairs of a row's tile 0 (block-uniform): the couples'
    // values for pairs m < H are replaced by rev_pair_head's
    double hxe = 0.0, hxo = 0.0;
    const bool hl = head && tid < G::np(l - 1) * H;
    const int hs = tid / H, hm = tid - hs * H;
    if (hl) {
      const double* ab = in + (2 * hs) * mi + Q + hm;  // a[hm]
      const double* db = ab + mi;
      rev_pair_head<L, FMA>(
          tp, hm, [=](int q) { return ab[-q]; }, [=](int q) { return db[-q]; }, hxe, hxo);
    }
    if constexpr (l > 1) {
      constexpr int mo = G::m(l - 1);
      double* out = lds + G::buf((l - 1) & 1);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        const int s = k / NCW, ml = 2 * (k - s * NCW);
        double* o = out + s * mo + Q + 2 * ml;
        if (!head || ml >= H) st16(o, rx[r].x, rx[r].y);
        if (!head || ml + 1 >= H) st16(o + 2, rx[r].z, rx[r].w);
      }
      if (hl) st16(out + hs * mo + Q + 2 * hm, hxe, hxo);
#pragma unroll
      for (int r = 0; r < RH; ++r) {
        const int v = tid + r * NT;
        if ((r + 1) * NT <= CH || v < CH) out[(v / H) * mo + 1 + v % H] = hv[r];
      }
    } else {
      double* yo = y + (int64_t)t * T;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int ml = 2 * (tid + r * NT);
        if (!head || ml >= H) st16(yo + 2 * ml, rx[r].x, rx[r].y);
        if (!head || ml + 1 >= H) st16(yo + 2 * ml + 2, rx[r].z, rx[r].w);
      }
      if (hl) st16(yo + 2 * hm, hxe, hxo);
      // the next tile's bands into the level-K buffer (level 1 reads the
      // other parity), then the registers take the tile after that
      put(lds + G::buf(K & 1), rb);
      fetch(rb, rown, tn, h);
    }
    lds_barrier();
    if constexpr (l > 1) level<l - 1>(lds, y, t, head, rown, tn, h, rb);
  }
};

// Grid: blocks share the rows * (h/T) tiles (g = row * (h/T) + tile) in
// contiguous runs, walked upwards.  src: rows of 2^K bands (packets of h/2^K),
// dst: rows of h samples (16-B aligned rows, h a multiple of T).
template <int L, int NT, int T, int K, bool FMA>
__global__ __launch_bounds__(NT) void wpt_rev_stream(WptStreamArgs<RevTaps<L>> args) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const double* __restrict__ src = args.src;
  double* __restrict__ dst = args.dst;
  const AxisView sv = args.sv, dv = args.dv;
  const int h = args.h;
  const int64_t ntile = args.ntile;
  using S = WptRStream<L, NT, T, K, FMA>;
  using G = WptRStreamGeo<L, T, K>;
  const int64_t b = blockIdx.x, nb = gridDim.x;
  const int64_t ga = b * ntile / nb, gb = (b + 1) * ntile / nb;
  if (ga >= gb) return;  // block-uniform (never with nb <= ntile)
  const int ntr = h / T;
  const auto next_of = [&](int64_t g) { return g + 1 < gb ? g + 1 : g; };
  double2 rb[S::kQB];
  {
    const int64_t o = ga / ntr;
    S::fetch(rb, src + view_base(sv, o), (int)(ga - o * ntr), h);
    S::put(lds + G::buf(K & 1), rb);
    const int64_t gn = next_of(ga), on = gn / ntr;
    S::fetch(rb, src + view_base(sv, on), (int)(gn - on * ntr), h);
  }
  for (int64_t g = ga; g < gb; ++g) {
    const int64_t o = g / ntr;
    const int t = (int)(g - o * ntr);
    if (g == ga || t == 0) {
      // a row segment starts: the carries of the tile left of tile t (the
      // prologue works in the buffer of parity K-1: the other one holds this
      // tile's bands)
      const int t0 = t > 0 ? t - 1 : ntr - 1;
      const double* row = src + view_base(sv, o);
      const int hp = h >> K;
      double* pb = lds + G::buf((K - 1) & 1);
      double* pin = pb + G::preg(0);
      const int tid = threadIdx.x;
      for (int v = tid; v < G::pin(K); v += NT) {
        const int p = v / G::D(K), i = v - p * G::D(K);
        int x = (t0 + 1) * G::Tl(K) - G::D(K) + i;
        x = x >= hp ? x - hp : x;
        pin[v] = row[(int64_t)p * hp + x];
      }
      lds_barrier();
      S::template pro_level<K>(lds, pb);
    }
    const int64_t gn = next_of(next_of(g)), on = gn / ntr;
    S::template level<K>(lds, dst + view_base(dv, o), t, t == 0, src + view_base(sv, on),
                         (int)(gn - on * ntr), h, rb);
  }
}

}  // namespace jwv
