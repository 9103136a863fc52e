// modwt_stream.hpp — forwardMODWT as a left-to-right stream of tiles with
// carried halos (compile-time L, T, J1; levels 1 .. J1, J1 even).
//
// Same math and per-output summation order as modwt_fwd_tile1
// (MODWTTransform.java:256-306, DIRECT circular convolution :677-690): level
// j computes W_j[p] = sum_l h[l] V_{j-1}[p - l st] and V_j[p] = sum_l g[l]
// V_{j-1}[p - l st], st = 2^(j-1), l ascending, so EXACT results are
// bit-identical to the tile kernels.
//
// What changes is where the LEFT halo comes from.  A tile kernel that owns
// outputs [p0, p0 + T) recomputes V_j on [p0 - (L-1)(2^J1 - 2^j), p0) at
// every level (config 5, T = 8192: 16% extra FP64) and keeps one window of
// T + 1785 doubles per block.  Here a block owns a chunk of consecutive tiles
// and walks it from the left: the halo of tile t at level j+1, V_j[p0 -
// (L-1) 2^j, p0), is the tail of tile t-1's V_j, which the block saved (the
// carry) when it ran tile t-1.  Every level computes exactly T outputs; the
// chunk's first tile takes its carries from a prologue that runs the halo
// recursion once.  Level j's input sits in one of two parity buffers (one
// barrier per level), W_j and V_J1 go straight to HBM, and the signal window
// of the next tile comes in through registers while this tile runs (one
// buffer load per 16-B piece on every path, so the compiler's vmcnt waits
// stay counted).
//
// Measured and not kept (r04e/r04f, one box each): the same stream for the
// inverse (right to left; 256 x 512 and 512 x 1024 tiles: 239-251 us against
// 228-232 for modwt_inv_tile1) and for the WPT forward and reverse (carried
// packet halos; every geometry 5-20% slower than wpt_fwd_tile1 /
// wpt_rev_tile1).
//
// Non-finite input (modwt_nonfinite.hpp): the fast pass checks V_J1; a block
// whose chunk saw a non-finite value runs the chunk again with SLOW = true,
// which repairs the outputs Java's zero taps make NaN (prologue levels
// included: their V values become the carries).
#pragma once
#include "modwt1_kernels.hpp"
#include "modwt_nonfinite.hpp"

namespace jwv {

// Level j's input window [p0 - (L-1) st, p0 + T) sits in the buffer of the
// parity of j with its own part at H(j) (level 1: one pad double in front so
// every tap pair is a 16-B read).
template <int L, int T, int J1>
struct ModFStreamGeo {
  static constexpr int st(int j) { return 1 << (j - 1); }
  static constexpr int C(int j) { return (L - 1) * st(j); }       // left halo of level j
  static constexpr int H(int j) { return C(j) + (C(j) & 1); }     // own part of level j's input
  static constexpr int Wn(int j) { return T + H(j); }              // level j's input window
  // carry of V_j (1 <= j < J1): its last C(j+1) values, at coff(j)
  static constexpr int coff(int j) { return (L - 1) * (2 * st(j) - 2); }
  static constexpr int ncarry() { return coff(J1); }
  static constexpr int bsize(int p) {
    int b = 0;
    for (int j = 1; j <= J1; ++j)
      if ((j & 1) == p && Wn(j) + 2 > b) b = Wn(j) + 2;
    return (b + 1) & ~1;
  }
  static constexpr int buf(int p) { return p ? bsize(0) : 0; }
  // prologue: V_j on [c0 - D(j), c0), D(J1-1) = C(J1), D(j) = D(j+1) + C(j+1);
  // x on [c0 - D(0) - pad, c0).  Regions: Q(odd j) at 0, Q(even j) after it,
  // both below the carries (which the prologue writes level by level); X at
  // the end, over the carries (it is read only before level 1's barrier)
  static constexpr int D(int j) {
    int d = 0;
    for (int i = j + 1; i <= J1; ++i) d += C(i);
    return d;
  }
  static constexpr int XP() { return D(0) + (D(0) & 1); }  // padded x extent (even)
  static constexpr int q(int p) { return p ? ((D(1) + 3) & ~1) : 0; }
  static constexpr int qend() { return (q(1) + D(2) + 3) & ~1; }
  static constexpr int carry0() {
    return bsize(0) + bsize(1) > qend() ? bsize(0) + bsize(1) : qend();
  }
  static constexpr int lds_doubles() { return carry0() + ncarry(); }
  static constexpr int qx() { return lds_doubles() - ((XP() + 3) & ~1); }
  static_assert(q(0) + D(1) + 2 <= q(1) && qend() <= carry0() && qx() >= 0, "prologue regions");
  static_assert(T % 2 == 0 && (J1 & 1) == 0 && C(J1) <= T, "geometry");
};

template <int L, int NT, int T, int J1, bool FMA>
struct ModFStream {
  using G = ModFStreamGeo<L, T, J1>;
  static constexpr int nq(int n) { return ((n + 1) / 2 + NT - 1) / NT; }
  static constexpr int kQX = nq(G::Wn(1));
  static constexpr int kQP = nq(G::XP());

  // x on [p0 - H(1) ..) (n doubles, 16-B pieces; p0 - H(1) even) into
  // registers, every position wrapped into [0, N): one buffer load per piece
  // on every path
  template <int n, int Q>
  __device__ __forceinline__ static void fetch(double2 (&r)[Q], const double* __restrict__ src,
                                               int64_t s0, int64_t N) {
    constexpr int n2 = (n + 1) / 2;
    static_assert(nq(n) <= Q, "window pieces");
    const int tid = opaque_tid();
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(src), 0,
                                                      (int)(N * 8), 0x00020000);
    const int is0 = (int)s0, iN = (int)N;
#pragma unroll
    for (int q = 0; q < nq(n); ++q) {
      int e = 2 * (tid + q * NT);
      if ((q + 1) * NT > n2) e = e < 2 * n2 ? e : 2 * (n2 - 1);
      int g = is0 + e;
      g = g < 0 ? g + iN : (g >= iN ? g - iN : g);
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
  // outputs (e, e+1), e even, of level j from the input window at b (own
  // part of the outputs' positions at b + e): W pair in w, V pair in v
  template <int j>
  __device__ __forceinline__ static void pair(const ModwtTaps<L>& tp, const double* b, int e,
                                              double2& w, double2& v) {
    constexpr int st = 1 << (j - 1);
    double x0[L], x1[L];  // x0[l] = in[e - l st], x1[l] = in[e + 1 - l st]
    if constexpr (st == 1) {
      double u[L + 2];
#pragma unroll
      for (int i = 0; i < L + 2; i += 2) {
        const double2 z = ld16(b + e - L + i);
        u[i] = z.x;
        u[i + 1] = z.y;
      }
#pragma unroll
      for (int i = 0; i < L + 2; ++i) asm volatile("" : "+v"(u[i]));
#pragma unroll
      for (int l = 0; l < L; ++l) {
        x0[l] = u[L - l];
        x1[l] = u[L + 1 - l];
      }
    } else {
#pragma unroll
      for (int l = 0; l < L; ++l) {
        const double2 z = ld16(b + e - l * st);
        x0[l] = z.x;
        x1[l] = z.y;
      }
#pragma unroll
      for (int l = 0; l < L; ++l) asm volatile("" : "+v"(x0[l]), "+v"(x1[l]));
    }
    // V below the top level is LDS-only: its sums start at the first product
    // (the signed-zero argument of fwt_kernels.hpp, ZS); W and V_J1 are
    // outputs and start from +0.0
    constexpr bool kZv = j == J1;
    double sw0 = 0.0, sv0 = 0.0, sw1 = 0.0, sv1 = 0.0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      sw0 = mod_mac<FMA>(sw0, x0[l], tp.h[l]);
      sw1 = mod_mac<FMA>(sw1, x1[l], tp.h[l]);
      if (!kZv && l == 0) {
        sv0 = x0[0] * tp.g[0];
        sv1 = x1[0] * tp.g[0];
      } else {
        sv0 = mod_mac<FMA>(sv0, x0[l], tp.g[l]);
        sv1 = mod_mac<FMA>(sv1, x1[l], tp.g[l]);
      }
    }
    pin2(sw0, sv0);
    pin2(sw1, sv1);
    w = make_double2(sw0, sw1);
    v = make_double2(sv0, sv1);
  }

  // ---- prologue: the carries left of the chunk (positions .. c0)
  template <int j, bool SLOW>
  __device__ __forceinline__ static void pro_level(const ModwtTaps<L>& tp, double* lds, ModNf& nf) {
    if constexpr (j < J1) {
      constexpr int nout = G::D(j), np = nout / 2, R = (np + NT - 1) / NT;
      static_assert(nout % 2 == 0, "even prologue extents");
      // input V_{j-1} on [c0 - D(j-1), c0): output e reads index C(j) + e
      // (level 1: the x region, padded by one, so index 1 + C(1) + e = H(1) + e)
      const double* in = j == 1 ? lds + G::qx() : lds + G::q(j & 1 ? 1 : 0);
      constexpr int base = j == 1 ? G::H(1) : G::C(j);
      // repair: window positions [-C(j), nout) at in[base + q]
      int lo[2] = {1, 1}, hi[2] = {0, 0};
      auto at = [&](int q) { return in[base + q]; };
      if constexpr (SLOW && j >= 2)
        nf_window<1, NT>(nf, -G::C(j), nout, [&](int, int q) { return at(q); }, lo, hi);
      const int tid = opaque_tid();
      double* out = lds + G::q(j & 1 ? 0 : 1);
      double2 o[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        const int kc = (r + 1) * NT <= np ? k : (k < np ? k : np - 1);
        double2 w;
        pair<j>(tp, in, base + 2 * kc, w, o[r]);
        if constexpr (SLOW && j >= 2)
          if (lo[0] <= hi[0]) {
            if (nf_fwd_zero(at, 2 * kc, 1 << (j - 1), G::C(j), lo[0], hi[0])) o[r].x = mod_nan();
            if (nf_fwd_zero(at, 2 * kc + 1, 1 << (j - 1), G::C(j), lo[0], hi[0])) o[r].y = mod_nan();
          }
      }
      lds_barrier();  // the input is dead (level 1: x overlaps the carries)
      constexpr int CS = G::C(j + 1);  // carry of V_j: its last C(j+1) values
      double* cw = lds + G::carry0() + G::coff(j);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        if ((r + 1) * NT <= np || k < np) {
          st16(out + 2 * k, o[r].x, o[r].y);
          const int c = 2 * k - (nout - CS);
          if (c >= 0) st16(cw + c, o[r].x, o[r].y);  // CS, nout even
        }
      }
      lds_barrier();
      pro_level<j + 1, SLOW>(tp, lds, nf);
    }
  }

  // ---- main loop, level j of tile p0
  template <int j, bool SLOW>
  __device__ __forceinline__ static void level(const ModwtTaps<L>& tp, double* lds,
                                               const double* __restrict__ src,
                                               double* __restrict__ wout, int64_t ldw,
                                               double* __restrict__ vout, int64_t p0, int64_t pn,
                                               int64_t N, double2 (&rx)[kQX], ModNf& nf,
                                               bool& bad) {
    constexpr int R = T / 2 / NT;
    static_assert(R * 2 * NT == T, "T = 2 NT R");
    const double* in = lds + G::buf(j & 1);
    // repair: window positions [-C(j), T) at in[H(j) + q]
    int lo[2] = {1, 1}, hi[2] = {0, 0};
    auto at = [&](int q) { return in[G::H(j) + q]; };
    if constexpr (SLOW && j >= 2)
      nf_window<1, NT>(nf, -G::C(j), T, [&](int, int q) { return at(q); }, lo, hi);
    const int tid = opaque_tid();
    // carries: the head of V_j's buffer (V_j tail of the tile to the left)
    // and the tail of this level's input V_{j-1} (j >= 2) for the tile to
    // the right, read before the sums, written after them
    constexpr int CH = j < J1 ? G::C(j + 1) : 0, CS = j >= 2 ? G::C(j) : 0;
    constexpr int RH = (CH + NT - 1) / NT, RS = (CS + NT - 1) / NT;
    double hv[RH > 0 ? RH : 1], sv[RS > 0 ? RS : 1];
    if constexpr (CH > 0) {
      const double* cr = lds + G::carry0() + G::coff(j);
#pragma unroll
      for (int r = 0; r < RH; ++r)
        if ((r + 1) * NT <= CH || tid + r * NT < CH) hv[r] = cr[tid + r * NT];
    }
#pragma unroll
    for (int r = 0; r < RS; ++r)
      if ((r + 1) * NT <= CS || tid + r * NT < CS) sv[r] = in[G::H(j) + T - CS + tid + r * NT];
    double2 w[R], v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) pair<j>(tp, in, G::H(j) + 2 * (tid + r * NT), w[r], v[r]);
    if constexpr (!SLOW && j == J1) {
#pragma unroll
      for (int r = 0; r < R; ++r) bad = bad || nonfinite(v[r].x) || nonfinite(v[r].y);
    }
    if constexpr (SLOW && j >= 2)
      if (lo[0] <= hi[0]) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            if (nf_fwd_zero(at, 2 * (tid + r * NT) + h, 1 << (j - 1), G::C(j), lo[0], hi[0])) {
              (h ? w[r].y : w[r].x) = mod_nan();
              (h ? v[r].y : v[r].x) = mod_nan();
            }
      }
    if constexpr (CS > 0) {
      double* cw = lds + G::carry0() + G::coff(j - 1);
#pragma unroll
      for (int r = 0; r < RS; ++r)
        if ((r + 1) * NT <= CS || tid + r * NT < CS) cw[tid + r * NT] = sv[r];
    }
    // W_j pairs to HBM: pairs past N (ragged last tile; N even) are dropped
    {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(wout + (int64_t)(j - 1) * ldw, 0,
                                                        (int)(N * 8), 0x00020000);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int p = (int)p0 + 2 * (tid + r * NT);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(jwv_u32x4, w[r]), rs, p * 8, 0, 0);
      }
    }
    if constexpr (j < J1) {
      double* vo = lds + G::buf((j + 1) & 1);
#pragma unroll
      for (int r = 0; r < R; ++r) st16(vo + G::H(j + 1) + 2 * (tid + r * NT), v[r].x, v[r].y);
#pragma unroll
      for (int r = 0; r < RH; ++r)
        if ((r + 1) * NT <= CH || tid + r * NT < CH) vo[tid + r * NT] = hv[r];
    } else {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(vout, 0, (int)(N * 8), 0x00020000);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int p = (int)p0 + 2 * (tid + r * NT);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(jwv_u32x4, v[r]), rs, p * 8, 0, 0);
      }
      // the next tile's signal window into the level-1 buffer (free since
      // level 2 read... level J1 reads the other parity), then its registers
      // take the tile after that
      static_assert(((J1 + 1) & 1) == 1, "level 1 input buffer is not the one level J1 reads");
      put<G::Wn(1)>(lds + G::buf(1), rx);
      fetch<G::Wn(1)>(rx, src, pn - G::H(1), N);
    }
    lds_barrier();
    if constexpr (j < J1) level<j + 1, SLOW>(tp, lds, src, wout, ldw, vout, p0, pn, N, rx, nf, bad);
  }

  // the chunk of tiles [ta, tb): prologue, then the tiles left to right
  template <bool SLOW>
  __device__ __forceinline__ static void chunk(const ModwtTaps<L>& tp, double* lds,
                                               const double* __restrict__ src,
                                               double* __restrict__ wout, int64_t ldw,
                                               double* __restrict__ vout, int64_t N, int64_t ta,
                                               int64_t tb, ModNf& nf, bool& bad) {
    double2 rx[kQX];
    {
      // prologue: x on [c0 - XP, c0) (XP even), then V_1 .. V_{J1-1} heads
      const int64_t c0 = ta * T;
      double2 px[kQP];
      fetch<G::XP()>(px, src, c0 - G::XP(), N);
      fetch<G::Wn(1)>(rx, src, c0 - G::H(1), N);  // the first tile's window
      put<G::XP()>(lds + G::qx(), px);
      lds_barrier();
      pro_level<1, SLOW>(tp, lds, nf);
    }
    put<G::Wn(1)>(lds + G::buf(1), rx);
    {
      const int64_t pn = (ta + 1 < tb ? ta + 1 : ta) * T;
      fetch<G::Wn(1)>(rx, src, pn - G::H(1), N);
    }
    lds_barrier();
    for (int64_t t = ta; t < tb; ++t) {
      // the window loaded during tile t is tile t+2's (past the chunk end: a
      // tile of the chunk, never used)
      const int64_t pn = (t + 2 < tb ? t + 2 : t) * T;
      level<1, SLOW>(tp, lds, src, wout, ldw, vout, t * T, pn, N, rx, nf, bad);
    }
  }
};

// Grid: one block per chunk of consecutive T-sample tiles.  src = V_0 (the
// signal, length N even); W_j -> wout + (j-1)*ldw (ldw even, 16-B aligned);
// V_J1 -> vout.
template <int L, int NT, int T, int J1, bool FMA>
__global__ __launch_bounds__(NT) void modwt_fwd_stream(const double* __restrict__ src,
                                                       double* __restrict__ wout, int64_t ldw,
                                                       double* __restrict__ vout, int64_t N,
                                                       int64_t ntile, ModwtTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ ModNf nf;
  using S = ModFStream<L, NT, T, J1, FMA>;
  const int64_t b = blockIdx.x, nb = gridDim.x;
  const int64_t ta = b * ntile / nb, tb = (b + 1) * ntile / nb;
  if (ta >= tb) return;  // block-uniform (never with nb <= ntile)
  nf_init(nf);
  bool bad = false;
  S::template chunk<false>(tp, lds, src, wout, ldw, vout, N, ta, tb, nf, bad);
  if (nf_any(nf, bad)) S::template chunk<true>(tp, lds, src, wout, ldw, vout, N, ta, tb, nf, bad);
}

}  // namespace jwv
