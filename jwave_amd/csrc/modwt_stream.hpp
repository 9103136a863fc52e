// modwt_stream.hpp — MODWT inverse as a right-to-left stream of tiles with
// carried halos (compile-time L, T, J1; levels J1 .. 1).
//
// Same math and per-output summation order as modwt_inv_tile1's P2 form
// (MODWTTransform.java:337-375, DIRECT circular convolution :703-716): output
// p of level j is sum_l g[l] V_j[p + l st] + sum_l h[l] W_j[p + l st] with
// st = 2^(j-1), the two sums accumulated in l order, then added.  EXACT
// results are bit-identical to the tile kernels.
//
// What changes is where the right halo comes from.  A tile kernel that owns
// outputs [p0, p0 + T) recomputes V_j on [p0 + T, p0 + T + (L-1)(2^j - 1))
// at every level (config 5, T = 2048: 10.5% extra FP64, 48% extra window
// reads) and keeps two windows of T + 1785 doubles in LDS (2 blocks per CU).
// Here a block owns a chunk of consecutive tiles and walks it from the right:
// the halo of tile t at level j, V_j[p0 + T, p0 + T + (L-1) st), is the head
// of tile t+1's V_j, which the block saved (the carry) when it ran tile t+1.
// So every level computes exactly T outputs, each V value is computed once
// (a chunk's rightmost tile takes its carries from a short prologue that runs
// the halo recursion once per chunk), and the LDS holds two V and two W
// windows of T + (L-1) st: one barrier per level (ping-pong by level
// parity), T = 512 at 3 blocks per CU.
//
// Every W window (and the top V window) of the NEXT tile is loaded into
// registers while this tile runs: a window's registers are written to LDS one
// level before it is read and refilled at once with the next tile's window,
// so each load has a whole tile (J1 levels) to arrive, and the loads leave in
// the order they are consumed (in-order vmcnt).
#pragma once
#include "modwt1_kernels.hpp"

namespace jwv {

template <int L, int T, int J1>
struct ModStreamGeo {
  static constexpr int st(int j) { return 1 << (j - 1); }
  // window of V_j / W_j in the main loop: T outputs + (L-1) st halo
  static constexpr int Wn(int j) { return T + (L - 1) * st(j); }
  // carried head of V_j (j < J1) and its offset in the carry area
  static constexpr int C(int j) { return (L - 1) * st(j); }
  static constexpr int coff(int j) { return (L - 1) * (st(j) - 1); }
  static constexpr int ncarry() { return coff(J1); }
  // prologue extent of V_j / W_j: (L-1)(2^j - 1)
  static constexpr int E(int j) { return (L - 1) * ((1 << j) - 1); }
  // parity buffers (+2: the st = 1 pair reads one double past a window)
  static constexpr int bsize(int p) {
    int b = 0;
    for (int j = 1; j <= J1; ++j)
      if ((j & 1) == p && Wn(j) + 2 > b) b = Wn(j) + 2;
    return (b + 1) & ~1;
  }
  // [V parity 0 | V parity 1 | W parity 0 | W parity 1 | carries]
  static constexpr int vbuf(int p) { return p ? bsize(0) : 0; }
  static constexpr int wbuf(int p) { return bsize(0) + bsize(1) + (p ? bsize(0) : 0); }
  static constexpr int carry0() { return 2 * bsize(0) + 2 * bsize(1); }
  static constexpr int lds_doubles() { return carry0() + ncarry(); }
  // prologue regions inside the four buffers
  static constexpr int pv(int p) { return p == (J1 & 1) ? 0 : ((E(J1) + 3) & ~1); }
  static constexpr int pw() { return ((E(J1) + 3) & ~1) + ((E(J1 - 1) + 3) & ~1); }
  static_assert(pw() + E(J1) + 2 <= carry0(), "prologue fits the tile buffers");
  static_assert(T % 2 == 0 && J1 >= 2, "geometry");
  static_assert(vbuf(1) + bsize(1) <= wbuf(0) && wbuf(0) + bsize(0) <= wbuf(1) &&
                    wbuf(1) + bsize(1) <= carry0(),
                "buffers are disjoint");
};

template <int L, int NT, int T, int J1, bool FMA>
struct ModStream {
  using G = ModStreamGeo<L, T, J1>;
  // 16-B pieces per lane of a window of n doubles
  static constexpr int nq(int n) { return ((n + 1) / 2 + NT - 1) / NT; }
  static constexpr int kQV = nq(G::Wn(J1));
  static constexpr int kQW = nq(G::Wn(J1));  // every W window fits the top one's pieces
  static constexpr int kQP = nq(G::E(J1));   // prologue windows
  static_assert(G::C(J1 - 1) <= T, "a carry is a head of one tile");
  // Loads per tile in the steady state: the top V window and W_J1 .. W_1.
  static constexpr int nloads() {
    int n = nq(G::Wn(J1));
    for (int j = 1; j <= J1; ++j) n += nq(G::Wn(j));
    return n;
  }
  // Wait until the loads of a window are in: vmcnt(N) with N = the loads
  // issued after them (a window is put one tile cycle after its fetch, so N
  // = nloads() minus the window and what was fetched with it before it).
  // The compiler's own waits also count the V_0 stores issued after those
  // loads, and a store can retire before an older load: with them alone
  // the window could be read stale (seen on hardware).  Counting loads only
  // is safe, since loads retire in order.
  template <int N>
  __device__ __forceinline__ static void vm_wait() {
    static_assert(N >= 0 && N < 63, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  }

  // One window of n doubles at src[p0 ..) (16-B pieces) into registers, as
  // exactly nq(n) buffer loads per lane on every path: no branch, so the
  // compiler can wait for each window with a counted vmcnt while the loads
  // issued after it stay in flight.  Positions wrap at N (at most once: the
  // host guarantees n + 2 < N); N and p0 are even, so a 16-B piece never
  // straddles the wrap.  Lanes past the window's end load a valid piece.
  template <int n, int Q>
  __device__ __forceinline__ static void fetch(double2 (&r)[Q], const double* __restrict__ src,
                                               int64_t p0, int64_t N) {
    constexpr int n2 = (n + 1) / 2;
    static_assert(nq(n) <= Q, "window pieces");
    const int tid = opaque_tid();
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(src), 0,
                                                      (int)(N * 8), 0x00020000);
    const int np = (int)(N - p0), ip0 = (int)p0;
#pragma unroll
    for (int q = 0; q < nq(n); ++q) {
      int e = 2 * (tid + q * NT);
      if ((q + 1) * NT > n2) e = e < 2 * n2 ? e : 2 * (n2 - 1);
      const int g = e < np ? ip0 + e : e - np;
      r[q] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, g * 8, 0, 0));
    }
  }
  template <int n, int Q>
  __device__ __forceinline__ static void put(double* lds, const double2 (&r)[Q]) {
    constexpr int n2 = (n + 1) / 2;
    static_assert(nq(n) <= Q, "window pieces");
    const int tid = opaque_tid();
#pragma unroll
    for (int q = 0; q < nq(n); ++q)
      if ((q + 1) * NT <= n2 || tid + q * NT < n2) st16(lds + 2 * (tid + q * NT), r[q].x, r[q].y);
  }

  // sum_l c[l] x[2k + l st] and sum_l c[l] x[2k + 1 + l st] (l ascending)
  template <int j, bool ISW>
  __device__ __forceinline__ static void sums(const ModwtTaps<L>& tp, const double* x, int k,
                                              double& s0, double& s1) {
    constexpr int st = 1 << (j - 1);
    const double* a = x + 2 * k;
    double v0[L], v1[L];
    if constexpr (st == 1) {
      double v[L + 2];
#pragma unroll
      for (int i = 0; i < L + 2; i += 2) {
        const double2 u = ld16(a + i);
        v[i] = u.x;
        v[i + 1] = u.y;
      }
#pragma unroll
      for (int i = 0; i < L + 2; ++i) asm volatile("" : "+v"(v[i]));
#pragma unroll
      for (int l = 0; l < L; ++l) {
        v0[l] = v[l];
        v1[l] = v[l + 1];
      }
    } else {
#pragma unroll
      for (int l = 0; l < L; ++l) {
        const double2 u = ld16(a + l * st);
        v0[l] = u.x;
        v1[l] = u.y;
      }
#pragma unroll
      for (int l = 0; l < L; ++l) asm volatile("" : "+v"(v0[l]), "+v"(v1[l]));
    }
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      a0 = mod_mac<FMA>(a0, v0[l], ISW ? tp.h[l] : tp.g[l]);
      a1 = mod_mac<FMA>(a1, v1[l], ISW ? tp.h[l] : tp.g[l]);
    }
    s0 = a0;
    s1 = a1;
  }
  // outputs (2k, 2k+1) of level j from the V / W windows at vb / wb: the V
  // sums, then the W sums (one operand's taps in registers at a time)
  template <int j>
  __device__ __forceinline__ static double2 pair(const ModwtTaps<L>& tp, const double* vb,
                                                 const double* wb, int k) {
    double sa0, sa1, sd0, sd1;
    sums<j, false>(tp, vb, k, sa0, sa1);
    sums<j, true>(tp, wb, k, sd0, sd1);
    pin2(sa0, sd0);
    pin2(sa1, sd1);
    return make_double2(sa0 + sd0, sa1 + sd1);
  }

  // ---- prologue: carries of the tile right of the chunk (positions c1 ..)
  // Level j computes V_{j-1} on [c1, c1 + E(j-1)) from V_j, W_j on
  // [c1, c1 + E(j)); the head C(j-1) of every V_{j-1} is a carry.  Its W
  // windows are all in registers (pw[j-1]) before it starts; after level J1
  // (whose windows are the big ones) the first tile's windows are issued.
  template <int j>
  __device__ __forceinline__ static void pro_fetch(double2 (&pw)[J1][kQP],
                                                   const double* __restrict__ coef, int64_t ldw,
                                                   int64_t c1, int64_t N) {
    fetch<G::E(j)>(pw[j - 1], coef + (int64_t)(j - 1) * ldw, c1, N);
    if constexpr (j > 2) pro_fetch<j - 1>(pw, coef, ldw, c1, N);
  }
  template <int j>
  __device__ __forceinline__ static void fetch_all(double2 (&rw)[J1][kQW],
                                                   const double* __restrict__ coef, int64_t ldw,
                                                   int64_t p0, int64_t N) {
    fetch<G::Wn(j)>(rw[j - 1], coef + (int64_t)(j - 1) * ldw, p0, N);
    if constexpr (j > 1) fetch_all<j - 1>(rw, coef, ldw, p0, N);
  }
  template <int j>
  __device__ __forceinline__ static void pro_level(const ModwtTaps<L>& tp, double* lds,
                                                   double2 (&pw)[J1][kQP],
                                                   const double* __restrict__ vsrc,
                                                   const double* __restrict__ coef, int64_t ldw,
                                                   int64_t p0, int64_t N, double2 (&rv)[kQV],
                                                   double2 (&rw)[J1][kQW]) {
    if constexpr (j >= 2) {
      constexpr int nout = G::E(j - 1), np = (nout + 1) / 2, R = (np + NT - 1) / NT;
      const int tid = opaque_tid();
      const double* vin = lds + G::pv(j & 1);
      double* vout = lds + G::pv((j - 1) & 1);
      double* wb = lds + G::pw();
      put<G::E(j)>(wb, pw[j - 1]);
      lds_barrier();
      double2 o[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        const int kc = (r + 1) * NT <= np ? k : (k < np ? k : np - 1);
        o[r] = pair<j>(tp, vin, wb, kc);
      }
      if constexpr (j == J1) {
        fetch<G::Wn(J1)>(rv, vsrc, p0, N);
        fetch_all<J1>(rw, coef, ldw, p0, N);
      }
      double* carry = lds + G::carry0() + G::coff(j - 1);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        if ((r + 1) * NT <= np || k < np) {
          st16(vout + 2 * k, o[r].x, o[r].y);
          if (2 * k < G::C(j - 1)) carry[2 * k] = o[r].x;
          if (2 * k + 1 < G::C(j - 1)) carry[2 * k + 1] = o[r].y;
        }
      }
      lds_barrier();
      pro_level<j - 1>(tp, lds, pw, vsrc, coef, ldw, p0, N, rv, rw);
    }
  }

  // the top windows (V_J1, W_J1: fetched in that order) into the buffers of
  // the parity of J1
  __device__ __forceinline__ static void put_top(double* lds, const double2 (&rv)[kQV],
                                                 const double2 (&rw)[J1][kQW]) {
    vm_wait<nloads() - nq(G::Wn(J1))>();
    put<G::Wn(J1)>(lds + G::vbuf(J1 & 1), rv);
    vm_wait<nloads() - 2 * nq(G::Wn(J1))>();
    put<G::Wn(J1)>(lds + G::wbuf(J1 & 1), rw[J1 - 1]);
  }

  // ---- main loop, level j of tile p0: V_{j-1} <- (V_j, W_j)
  template <int j>
  __device__ __forceinline__ static void level(const ModwtTaps<L>& tp, double* lds,
                                               const double* __restrict__ vsrc,
                                               const double* __restrict__ coef, int64_t ldw,
                                               double* __restrict__ dst, int64_t p0, int64_t pn,
                                               int64_t pt, int64_t N, double2 (&rv)[kQV],
                                               double2 (&rw)[J1][kQW]) {
    constexpr int R = T / 2 / NT;
    static_assert(R * 2 * NT == T, "T = 2 NT R");
    const int tid = opaque_tid();
    const double* vb = lds + G::vbuf(j & 1);
    const double* wb = lds + G::wbuf(j & 1);
    // carry traffic in registers, read before the level's sums and written
    // after them (off the phase's latency chain): the tail of V_{j-1} (the
    // carry of the tile to the right) and the head of V_j (the carry of the
    // tile to the left)
    constexpr int CT = j > 1 ? G::C(j - 1) : 0, CS = j < J1 ? G::C(j) : 0;
    constexpr int RT = (CT + NT - 1) / NT, RS = (CS + NT - 1) / NT;
    double tv[RT > 0 ? RT : 1], hv[RS > 0 ? RS : 1];
    if constexpr (CT > 0) {
      const double* cr = lds + G::carry0() + G::coff(j - 1);
#pragma unroll
      for (int r = 0; r < RT; ++r)
        if ((r + 1) * NT <= CT || tid + r * NT < CT) tv[r] = cr[tid + r * NT];
    }
#pragma unroll
    for (int r = 0; r < RS; ++r)
      if ((r + 1) * NT <= CS || tid + r * NT < CS) hv[r] = vb[tid + r * NT];
    double2 o[R];
#pragma unroll
    for (int r = 0; r < R; ++r) o[r] = pair<j>(tp, vb, wb, tid + r * NT);
    if constexpr (CS > 0) {
      double* cw = lds + G::carry0() + G::coff(j);
#pragma unroll
      for (int r = 0; r < RS; ++r)
        if ((r + 1) * NT <= CS || tid + r * NT < CS) cw[tid + r * NT] = hv[r];
    }
    if constexpr (j > 1) {
      double* vo = lds + G::vbuf((j - 1) & 1);
#pragma unroll
      for (int r = 0; r < R; ++r) st16(vo + 2 * (tid + r * NT), o[r].x, o[r].y);
#pragma unroll
      for (int r = 0; r < RT; ++r)
        if ((r + 1) * NT <= CT || tid + r * NT < CT) vo[T + tid + r * NT] = tv[r];
      // W_{j-1} into LDS, then its registers take the next tile's W_{j-1}
      vm_wait<nloads() - nq(G::Wn(j - 1))>();
      put<G::Wn(j - 1)>(lds + G::wbuf((j - 1) & 1), rw[j - 2]);
      fetch<G::Wn(j - 1)>(rw[j - 2], coef + (int64_t)(j - 2) * ldw, pn, N);
    } else {
      // V_0 stores: one buffer store per pair on every tile; pairs past N
      // (ragged last tile; N even) fall outside the resource and are dropped
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)(N * 8), 0x00020000);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int p = (int)p0 + 2 * (tid + r * NT);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(jwv_u32x4, o[r]), rs, p * 8, 0, 0);
      }
      // the next tile's top windows (parity of J1, not read at level 1)
      static_assert((J1 & 1) == 0, "top windows written during level 1");
      put_top(lds, rv, rw);
      fetch<G::Wn(J1)>(rv, vsrc, pt, N);
      fetch<G::Wn(J1)>(rw[J1 - 1], coef + (int64_t)(J1 - 1) * ldw, pt, N);
    }
    lds_barrier();
    if constexpr (j > 1)
      level<j - 1>(tp, lds, vsrc, coef, ldw, dst, p0, pn, pt, N, rv, rw);
  }
};

// Grid: one block per chunk of consecutive T-output tiles (ntile tiles in
// all, chunks as even as integers allow).  vsrc = V_{J1}; W_j at coef +
// (j-1)*ldw (ldw even, 16-B aligned rows); output V_0 -> dst.
template <int L, int NT, int T, int J1, bool FMA>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT >= 512 ? 4 : 3))) void modwt_inv_stream(const double* __restrict__ vsrc,
                                                       const double* __restrict__ coef,
                                                       int64_t ldw, double* __restrict__ dst,
                                                       int64_t N, int64_t ntile,
                                                       ModwtTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using S = ModStream<L, NT, T, J1, FMA>;
  using G = ModStreamGeo<L, T, J1>;
  const int64_t b = blockIdx.x, nb = gridDim.x;
  const int64_t ta = b * ntile / nb, tb = (b + 1) * ntile / nb;
  if (ta >= tb) return;  // block-uniform (never with nb <= ntile)
  double2 rv[S::kQV];
  double2 rw[J1][S::kQW];
  {
    // prologue windows (registers): V_J1 and W_J1 .. W_2 at c1 = the chunk end
    const int64_t c1 = tb * T >= N ? tb * T - N : tb * T;
    double2 pv[S::kQP];
    double2 pw[J1][S::kQP];
    S::template fetch<G::E(J1)>(pv, vsrc, c1, N);
    S::template pro_fetch<J1>(pw, coef, ldw, c1, N);
    S::template put<G::E(J1)>(lds + G::pv(J1 & 1), pv);
    // the rightmost tile's windows are issued inside level J1 of the prologue
    S::template pro_level<J1>(tp, lds, pw, vsrc, coef, ldw, (tb - 1) * T, N, rv, rw);
  }
  // the rightmost tile's top windows, then the top registers take tile tb-2's
  S::put_top(lds, rv, rw);
  {
    const int64_t pt = (tb - 2 >= ta ? tb - 2 : tb - 1) * T;
    S::template fetch<G::Wn(J1)>(rv, vsrc, pt, N);
    S::template fetch<G::Wn(J1)>(rw[J1 - 1], coef + (int64_t)(J1 - 1) * ldw, pt, N);
  }
  lds_barrier();
  for (int64_t t = tb - 1; t >= ta; --t) {
    // loads issued during tile t: W_{J1-1} .. W_1 of tile t-1, the top
    // windows of tile t-2; past the chunk start a tile of the chunk is
    // re-read instead (never used)
    const int64_t pn = (t - 1 >= ta ? t - 1 : t) * T;
    const int64_t pt = (t - 2 >= ta ? t - 2 : t) * T;
    S::template level<J1>(tp, lds, vsrc, coef, ldw, dst, t * T, pn, pt, N, rv, rw);
  }
}


// ---------------------------------------------------------------- forward
// The same stream for forwardMODWT (MODWTTransform.java:256-306, DIRECT
// :677-690): level j computes W_j[p] = sum_l h[l] V_{j-1}[p - l st] and
// V_j[p] = sum_l g[l] V_{j-1}[p - l st] (l ascending, the order of
// modwt_fwd_tile1), so the halo is on the LEFT: a block walks its chunk from
// the left and carries the tail of every V_j (j < J1) into the next tile.
// Level j's input window [p0 - (L-1) st, p0 + T) sits in the buffer of the
// parity of j with its own part at H(j) (level 1: one pad double in front so
// every tap pair is a 16-B read).  W_j and V_J1 go straight to HBM; only the
// signal window is loaded (one tile ahead, into registers).
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
    double sw0 = 0.0, sv0 = 0.0, sw1 = 0.0, sv1 = 0.0;
#pragma unroll
    for (int l = 0; l < L; ++l) {
      sw0 = mod_mac<FMA>(sw0, x0[l], tp.h[l]);
      sv0 = mod_mac<FMA>(sv0, x0[l], tp.g[l]);
      sw1 = mod_mac<FMA>(sw1, x1[l], tp.h[l]);
      sv1 = mod_mac<FMA>(sv1, x1[l], tp.g[l]);
    }
    pin2(sw0, sv0);
    pin2(sw1, sv1);
    w = make_double2(sw0, sw1);
    v = make_double2(sv0, sv1);
  }

  // ---- prologue: the carries left of the chunk (positions .. c0)
  template <int j>
  __device__ __forceinline__ static void pro_level(const ModwtTaps<L>& tp, double* lds) {
    if constexpr (j < J1) {
      constexpr int nout = G::D(j), np = nout / 2, R = (np + NT - 1) / NT;
      static_assert(nout % 2 == 0, "even prologue extents");
      const int tid = opaque_tid();
      // input V_{j-1} on [c0 - D(j-1), c0): output e reads index C(j) + e
      // (level 1: the x region, padded by one, so index 1 + C(1) + e = H(1) + e)
      const double* in = j == 1 ? lds + G::qx() : lds + G::q(j & 1 ? 1 : 0);
      constexpr int base = j == 1 ? G::H(1) : G::C(j);
      double* out = lds + G::q(j & 1 ? 0 : 1);
      double2 o[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = tid + r * NT;
        const int kc = (r + 1) * NT <= np ? k : (k < np ? k : np - 1);
        double2 w;
        pair<j>(tp, in, base + 2 * kc, w, o[r]);
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
      pro_level<j + 1>(tp, lds);
    }
  }

  // ---- main loop, level j of tile p0
  template <int j>
  __device__ __forceinline__ static void level(const ModwtTaps<L>& tp, double* lds,
                                               const double* __restrict__ src,
                                               double* __restrict__ wout, int64_t ldw,
                                               double* __restrict__ vout, int64_t p0, int64_t pn,
                                               int64_t N, double2 (&rx)[kQX]) {
    constexpr int R = T / 2 / NT;
    static_assert(R * 2 * NT == T, "T = 2 NT R");
    const int tid = opaque_tid();
    const double* in = lds + G::buf(j & 1);
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
    if constexpr (j < J1) level<j + 1>(tp, lds, src, wout, ldw, vout, p0, pn, N, rx);
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
  using S = ModFStream<L, NT, T, J1, FMA>;
  using G = ModFStreamGeo<L, T, J1>;
  const int64_t b = blockIdx.x, nb = gridDim.x;
  const int64_t ta = b * ntile / nb, tb = (b + 1) * ntile / nb;
  if (ta >= tb) return;  // block-uniform (never with nb <= ntile)
  double2 rx[S::kQX];
  {
    // prologue: x on [c0 - XP, c0) (XP even), then V_1 .. V_{J1-1} heads
    const int64_t c0 = ta * T;
    double2 px[S::kQP];
    S::template fetch<G::XP()>(px, src, c0 - G::XP(), N);
    S::template fetch<G::Wn(1)>(rx, src, c0 - G::H(1), N);  // the first tile's window
    S::template put<G::XP()>(lds + G::qx(), px);
    lds_barrier();
    S::template pro_level<1>(tp, lds);
  }
  S::template put<G::Wn(1)>(lds + G::buf(1), rx);
  {
    const int64_t pn = (ta + 1 < tb ? ta + 1 : ta) * T;
    S::template fetch<G::Wn(1)>(rx, src, pn - G::H(1), N);
  }
  lds_barrier();
  for (int64_t t = ta; t < tb; ++t) {
    // the window loaded during tile t is tile t+2's (past the chunk end: a
    // tile of the chunk, never used)
    const int64_t pn = (t + 2 < tb ? t + 2 : t) * T;
    S::template level<1>(tp, lds, src, wout, ldw, vout, t * T, pn, N, rx);
  }
}

}  // namespace jwv
