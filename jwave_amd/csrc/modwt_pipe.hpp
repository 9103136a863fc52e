// modwt_pipe.hpp — pipelined MODWT inverse: one persistent 1024-thread block
// per CU, every LDS window landed by LDS-DMA seven level-steps before it is
// read.
//
// Math, order and outputs are those of modwt_inv_tile1 (MODWTTransform.java:
// 337-375 with circularConvolveAdjoint :703-716): for j = J1 .. 1,
//   V_{j-1}[p] = (sum_l g[l] V_j[p + l*st]) + (sum_l h[l] W_j[p + l*st]),
// st = 2^(j-1), each sum in ascending l from +0.0 (EXACT: two roundings per
// term), so results are bit-identical to the oracle.
//
// Why a pipeline.  A tile of T outputs needs, per level, a window of W_j from
// HBM.  The one-tile-per-block kernel fetched level j-1's window while level j
// computed: one level of compute (~0.5 us per block) against a loaded-HBM
// latency of several us, eight times per tile (SQ_WAIT_ANY 49% of wave
// cycles, VALU issue 95 of 228 us).  Here a block keeps ALL windows of its
// tile in LDS (V_J1 and W_1 .. W_J1, ~150 KB at T = 1024) and walks the tiles
// of its XCD's chunk.  A level-step (k, j) starts with one counted vmcnt wait
// and one barrier, which also frees the buffers the previous step read; the
// step then re-fills them by LDS-DMA with the NEXT tile's windows:
//   step (k, j), j < J1:  W_{j+1}(k+1) -> WB[j+1]
//   step (k, J1):         V_J1(k+1) -> the idle big V buffer, W_1(k) -> WB[1]
// so every window is issued seven steps before the step that reads it, and
// the counted wait (own DMAs only, no VGPRs held) never drains the newer ones.
// The V chain alternates between a big buffer (V_J1, V_J1-2, ..) and a small
// one (V_J1-1, ..): a level writes a buffer nobody reads any more, so ONE
// barrier per level suffices.
//
// Tiles whose windows would wrap or run past the signal end (the last few)
// run in a second, plain launch (modwt_inv_pipe_edge): wrapped register loads,
// same LDS layout, same level code.
#pragma once
#include "modwt1_kernels.hpp"

namespace jwv {

template <int L, int T, int J1>
struct InvPipeGeo {
  static_assert(J1 >= 2 && J1 <= 8 && (T % 2) == 0, "pipe geometry");
  static constexpr int Rin(int j) { return j <= 0 ? 0 : (L - 1) * ((1 << j) - 1); }
  static constexpr int Wn(int j) { return T + Rin(j); }         // V_j / W_j window
  static constexpr int nout(int j) { return T + Rin(j - 1); }   // outputs of level j
  static constexpr int NS(int j) { return (nout(j) + 1) / 2; }  // output pair slots
  static constexpr int st(int j) { return 1 << (j - 1); }
  // doubles a level-j step reads from its inputs (pair slots clamped to NS-1)
  static constexpr int reach(int j) { return j == 1 ? 2 * NS(1) + L : 2 * NS(j) + (L - 1) * st(j); }
  static constexpr int units(int j) { return (Wn(j) + 1) / 2; }  // 16-B DMA units
  static constexpr int mx(int a, int b) { return a > b ? a : b; }
  static constexpr int ev(int a) { return (a + 1) & ~1; }
  static constexpr int wsize(int j) { return ev(mx(2 * units(j), reach(j))); }
  // big V buffer: V_J1 (DMA) and V_j for j = J1-2, J1-4, .. (written by level j+1)
  static constexpr int vbig() {
    int b = mx(2 * units(J1), reach(J1));
    for (int j = J1 - 2; j >= 1; j -= 2) b = mx(b, mx(2 * NS(j + 1), reach(j)));
    return ev(b);
  }
  static constexpr int vsmall() {
    int b = 2;
    for (int j = J1 - 1; j >= 1; j -= 2) b = mx(b, mx(2 * NS(j + 1), reach(j)));
    return ev(b);
  }
  static constexpr int woff(int j) {  // WB[j]
    int o = 2 * vbig() + vsmall();
    for (int i = 1; i < j; ++i) o += wsize(i);
    return o;
  }
  static constexpr int lds_doubles() { return woff(J1 + 1); }
};

// DMA of one window: units [0, U) of 16 B from g to lds (both 16-B aligned)
// as P one-KB pieces (one wave instruction each).  The pieces of consecutive
// windows are dealt round-robin over the NW waves, continuing from the deal
// position `off` (block-uniform), so any run of S consecutive pieces gives
// every wave floor(S/NW) or ceil(S/NW) of them: a wave that waits for all but
// floor(S/NW) of its DMAs has the window before those S pieces in LDS.
template <int NT, int U>
struct PipeDma {
  static constexpr int NW = NT / 64, P = (U + 63) / 64;
  static_assert((NW & (NW - 1)) == 0, "waves per block: a power of two");
  __device__ __forceinline__ static void issue(double* lds, const double* g, int& off) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int p = (wave - off) & (NW - 1); p < P; p += NW) {
      const int u = p * 64 + lane;
      if (u < U) dma16_asm(g + 2 * u, lds + 128 * p);
    }
    off = (off + P) & (NW - 1);
  }
};

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N < 63 ? N : 63) : "memory");
}

template <int L, int NT, int T, int J1, bool FMA>
struct InvPipe {
  using G = InvPipeGeo<L, T, J1>;
  // Counted wait before step j: the pieces dealt after the window step j
  // needs (see the file comment for the issue order), per wave at least
  // floor(S / NW).
  static constexpr int pc(int j) { return (G::units(j) + 63) / 64; }
  template <int j>
  static constexpr int nwait() {
    int n = 0;
    if (j == J1) {
      for (int i = 2; i <= J1 - 1; ++i) n += pc(i);
    } else if (j == 1) {
      for (int i = 3; i <= J1; ++i) n += pc(i);
    } else {
      for (int i = 2; i <= j - 1; ++i) n += pc(i);
      n += pc(J1) /* V_J1: W_J1's window length */ + pc(1);
      for (int i = j + 2; i <= J1; ++i) n += pc(i);
    }
    return n / (NT / 64);
  }

  // One level: reads X (V_j) and W (W_j), writes V_{j-1} pairs to Y, or, at
  // j = 1, the tile's T outputs to dst + t0 (EDGE: guarded, wrap-free
  // signal end; else 16-B buffer stores, dst + t0 16-B aligned).
  template <int j, bool EDGE>
  __device__ __forceinline__ static void level(const ModwtTaps<L>& tp, const double* X,
                                               const double* W, double* Y, double* dst,
                                               int64_t t0, int64_t N) {
    constexpr int st = G::st(j), ns = G::NS(j);
    constexpr int R = (ns + NT - 1) / NT;
    const int tid = opaque_tid();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int t = tid + r * NT;
      const bool full = (r + 1) * NT <= ns;
      if (!full && __builtin_amdgcn_readfirstlane((tid & ~63) + r * NT) >= ns) continue;
      const int s = full ? t : (t < ns ? t : ns - 1);
      const double* a = X + 2 * s;
      const double* w = W + 2 * s;
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
#pragma unroll
      for (int l = 0; l < L; ++l)
        asm volatile("" : "+v"(av0[l]), "+v"(av1[l]), "+v"(aw0[l]), "+v"(aw1[l]));
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
      const double o0 = sa0 + sd0, o1 = sa1 + sd1;
      if constexpr (j > 1) {
        if (full || t < ns) *reinterpret_cast<double2*>(Y + 2 * s) = make_double2(o0, o1);
      } else {
        const int p = 2 * s;  // nout(1) = T: every pair lies in the tile
        if (full || t < ns) {
          if constexpr (EDGE) {
            if (t0 + p < N) dst[t0 + p] = o0;
            if (t0 + p + 1 < N) dst[t0 + p + 1] = o1;
          } else {
            mod_store2(dst + t0, p, o0, o1);
          }
        }
      }
      asm volatile("" ::: "memory");  // slot fence
    }
  }

  // X_j: the big buffer of the tile for (J1 - j) even, else the small one.
  __device__ __forceinline__ static double* xbuf(double* lds, int cur, int j) {
    return ((J1 - j) & 1) ? lds + 2 * G::vbig() : lds + cur * G::vbig();
  }

  // Level-steps J1 .. 1 of the tile at t0 (interior).  tn >= 0: the next
  // tile of this block, whose windows are issued here.
  template <int j>
  __device__ __forceinline__ static void steps(const ModwtTaps<L>& tp, double* lds, int cur,
                                               const double* vsrc, const double* coef,
                                               int64_t ldw, double* dst, int64_t t0, int64_t tn,
                                               int64_t N, int& off) {
    if (j == J1 || tn >= 0)
      vm_wait<nwait<j>()>();
    else
      vm_wait<0>();  // last tile: the DMAs counted above were not issued
    lds_barrier();
    if constexpr (j == J1) {
      if (tn >= 0)
        PipeDma<NT, G::units(J1)>::issue(lds + (cur ^ 1) * G::vbig(), vsrc + tn, off);
      PipeDma<NT, G::units(1)>::issue(lds + G::woff(1), coef + t0, off);
    } else {
      if (tn >= 0)
        PipeDma<NT, G::units(j + 1)>::issue(lds + G::woff(j + 1), coef + (int64_t)j * ldw + tn, off);
    }
    level<j, false>(tp, xbuf(lds, cur, j), lds + G::woff(j), j > 1 ? xbuf(lds, cur, j - 1) : nullptr,
                    dst, t0, N);
    if constexpr (j > 1) steps<j - 1>(tp, lds, cur, vsrc, coef, ldw, dst, t0, tn, N, off);
  }

  template <int j>
  __device__ __forceinline__ static void prologue(double* lds, const double* coef, int64_t ldw,
                                                  int64_t t0, int& off) {
    PipeDma<NT, G::units(j)>::issue(lds + G::woff(j), coef + (int64_t)(j - 1) * ldw + t0, off);
    if constexpr (j > 2) prologue<j - 1>(lds, coef, ldw, t0, off);
  }

  // Edge tiles: every window loaded with wrapped plain loads, then the levels.
  template <int j>
  __device__ __forceinline__ static void edge_steps(const ModwtTaps<L>& tp, double* lds,
                                                    double* dst, int64_t t0, int64_t N) {
    lds_barrier();
    level<j, true>(tp, xbuf(lds, 0, j), lds + G::woff(j), j > 1 ? xbuf(lds, 0, j - 1) : nullptr,
                   dst, t0, N);
    if constexpr (j > 1) edge_steps<j - 1>(tp, lds, dst, t0, N);
  }
  template <int j>
  __device__ __forceinline__ static void edge_load(double* lds, const double* coef, int64_t ldw,
                                                   int64_t t0, int64_t N) {
    const double* row = coef + (int64_t)(j - 1) * ldw;
    double* b = lds + G::woff(j);
    for (int e = threadIdx.x; e < 2 * G::units(j); e += NT) b[e] = row[wrap_mod(t0 + e, N)];
    if constexpr (j > 1) edge_load<j - 1>(lds, coef, ldw, t0, N);
  }
};

// Interior tiles [0, ninner): persistent grid of 8 * (blocks per XCD); XCD x
// = blockIdx % 8 walks the contiguous chunk x of the tiles (a tile's halo is
// its neighbour's window in the same L2).  vsrc = V_J1 (length N, 16-B
// aligned), W_j at coef + (j-1)*ldw (ldw even), dst 16-B aligned.
template <int L, int NT, int T, int J1, bool FMA>
__global__ __launch_bounds__(NT) void modwt_inv_pipe(const double* __restrict__ vsrc,
                                                     const double* __restrict__ coef, int64_t ldw,
                                                     double* __restrict__ dst, int64_t N,
                                                     int64_t ninner, ModwtTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using P = InvPipe<L, NT, T, J1, FMA>;
  using G = InvPipeGeo<L, T, J1>;
  const int x = blockIdx.x & 7, nbx = gridDim.x >> 3, bx = blockIdx.x >> 3;
  const int64_t q = ninner >> 3, rr = ninner & 7;
  const int64_t c0 = x * q + (x < rr ? x : rr), c1 = c0 + q + (x < rr ? 1 : 0);
  int64_t tile = c0 + bx;
  if (tile >= c1) return;  // block-uniform
  // prologue: V_J1, W_J1 .. W_2 of the first tile (W_1 is issued by step J1)
  int off = 0, cur = 0;
  PipeDma<NT, G::units(J1)>::issue(lds, vsrc + tile * T, off);
  P::template prologue<J1>(lds, coef, ldw, tile * T, off);
  for (;;) {
    const int64_t t0 = tile * T;
    const int64_t nt = tile + nbx;
    const int64_t tn = nt < c1 ? nt * T : -1;
    P::template steps<J1>(tp, lds, cur, vsrc, coef, ldw, dst, t0, tn, N, off);
    if (tn < 0) break;
    tile = nt;
    cur ^= 1;
  }
}

// Tiles [ninner, ntile): one block each, wrapped loads, same levels.
template <int L, int NT, int T, int J1, bool FMA>
__global__ __launch_bounds__(NT) void modwt_inv_pipe_edge(const double* __restrict__ vsrc,
                                                          const double* __restrict__ coef,
                                                          int64_t ldw, double* __restrict__ dst,
                                                          int64_t N, int64_t ninner,
                                                          ModwtTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using P = InvPipe<L, NT, T, J1, FMA>;
  using G = InvPipeGeo<L, T, J1>;
  const int64_t t0 = (ninner + blockIdx.x) * T;
  for (int e = threadIdx.x; e < 2 * G::units(J1); e += NT) lds[e] = vsrc[wrap_mod(t0 + e, N)];
  P::template edge_load<J1>(lds, coef, ldw, t0, N);
  P::template edge_steps<J1>(tp, lds, dst, t0, N);
}


// ---------------------------------------------------------------- forward
// Pipelined forward (MODWTTransform.java:256-306 with circularConvolve
// :677-690; same levels, order and outputs as modwt_fwd_tile1's P2 form).
// One persistent 1024-thread block per CU keeps TWO windows of T + S samples
// in LDS (T = 8192: 2 x 78 KB): while a tile's levels run in place in one
// window, the next tile's window lands in the other by LDS-DMA.  Every W
// store is issued unconditionally (lanes with nothing to store point their
// buffer offset past the descriptor's range, which the hardware drops), so
// each wave issues the same compile-time number of stores per tile and the
// next tile's wait is one exact vmcnt: the window, never the stores.
namespace pipe {
constexpr unsigned kOOB = 0x80000000u;  // buffer offset past num_records: dropped
__device__ __forceinline__ void st2_oob(const __amdgpu_buffer_rsrc_t rs, unsigned off, double a,
                                        double b) {
  const jwv_u32x4 v = __builtin_bit_cast(jwv_u32x4, make_double2(a, b));
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);
}
}  // namespace pipe

template <int L, int T, int J1>
struct FwdPipeGeo {
  static_assert(J1 >= 1 && J1 <= 8 && (T % 2) == 0, "pipe geometry");
  static constexpr int S = (L - 1) * ((1 << J1) - 1);  // left halo of V_0
  static constexpr int W = T + S;
  static constexpr int Sn(int j) { return (L - 1) * ((1 << J1) - (1 << j)); }
  static constexpr int e0(int j) { return S - Sn(j); }
  static constexpr int NP(int j) { return (T + Sn(j)) / 2; }  // output pairs of level j
  static constexpr int kPad = (S & 1) ? 1 : 2;  // window index e at buffer kPad + e
  // the DMA starts on the even global index t0 - S - (S & 1), at buffer kPad - (S & 1)
  static constexpr int dma_lds() { return kPad - (S & 1); }
  static constexpr int units() { return (W + (S & 1) + 1) / 2; }
  static constexpr int buf() { return (kPad + W + 9) & ~1; }  // + one pair read past the end
  static constexpr int lds_doubles() { return 2 * buf(); }
};

template <int L, int NT, int T, int J1, bool FMA>
struct FwdPipe {
  using G = FwdPipeGeo<L, T, J1>;
  template <int j>
  static constexpr int R() { return (G::NP(j) + NT - 1) / NT; }
  static constexpr int nstores() {  // per wave per interior tile
    int n = T / 2 / NT;  // V_J1
    for (int j = 1; j <= J1; ++j) n += (G::NP(j) + NT - 1) / NT;
    return n;
  }
  static_assert(T / 2 % NT == 0, "V output pairs per lane");

  // Level j in place in the window b (window index e at b[kPad + e]).
  // EDGE: guarded stores for tiles at the signal's ends; else every slot
  // stores (OOB-masked), wrow 16-B aligned.
  template <int j, bool EDGE>
  __device__ __forceinline__ static void level(const ModwtTaps<L>& tp, double* b,
                                               double* __restrict__ wout, int64_t ldw, int64_t t0,
                                               int64_t N) {
    constexpr int st = 1 << (j - 1), e0 = G::e0(j), NP = G::NP(j), RR = R<j>();
    constexpr int kPad = G::kPad;
    static_assert(((kPad + e0) & 1) == 0, "16-B pair reads");
    const int tid = opaque_tid();
    double* __restrict__ wrow = wout + (int64_t)(j - 1) * ldw + (t0 - G::S);
    const auto rs = mod_rsrc(wrow);
    double2 vv[RR];
#pragma unroll
    for (int r = 0; r < RR; ++r) {
      const int k = tid + r * NT;
      const bool full = (r + 1) * NT <= NP;
      const bool valid = full || k < NP;
      const int kc = valid ? k : NP - 1;
      const int e = e0 + 2 * kc;
      const double* p = b + kPad + e;
      double x0[L], x1[L];
      if constexpr (st == 1) {
        double v[L + 2];
#pragma unroll
        for (int i = 0; i < L + 2; i += 2) {
          const double2 u = *reinterpret_cast<const double2*>(p - L + i);
          v[i] = u.x;
          v[i + 1] = u.y;
        }
#pragma unroll
        for (int i = 0; i < L + 2; ++i) asm volatile("" : "+v"(v[i]));
#pragma unroll
        for (int l = 0; l < L; ++l) {
          x0[l] = v[L - l];
          x1[l] = v[L + 1 - l];
        }
      } else {
#pragma unroll
        for (int l = 0; l < L; ++l) {
          const double2 u = *reinterpret_cast<const double2*>(p - l * st);
          x0[l] = u.x;
          x1[l] = u.y;
        }
      }
      // operands in registers here (16-B ds_read_b128, not per-use reads)
#pragma unroll
      for (int l = 0; l < L; ++l) asm volatile("" : "+v"(x0[l]), "+v"(x1[l]));
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
      const bool own = valid && e >= G::S;  // a pair is all halo or all own
      if constexpr (EDGE) {
        if (own) {
          const int64_t g = t0 + (e - G::S);
          if (g < N) wrow[e] = sw0;
          if (g + 1 < N) wrow[e + 1] = sw1;
        }
      } else {
        pipe::st2_oob(rs, own ? (unsigned)e * 8u : pipe::kOOB, sw0, sw1);
      }
      asm volatile("" ::: "memory");  // slot fence
    }
    lds_barrier();
#pragma unroll
    for (int r = 0; r < RR; ++r) {
      const int k = tid + r * NT;
      if ((r + 1) * NT <= NP || k < NP) *reinterpret_cast<double2*>(b + kPad + e0 + 2 * k) = vv[r];
    }
    lds_barrier();
    if constexpr (j < J1) level<j + 1, EDGE>(tp, b, wout, ldw, t0, N);
  }

  // V_J1 = window [S, S + T) -> vout + t0
  template <bool EDGE>
  __device__ __forceinline__ static void vstore(const double* b, double* __restrict__ vout,
                                                int64_t t0, int64_t N) {
    const int tid = threadIdx.x;
    const double* v = b + G::kPad + G::S;  // even: 16-B pairs
    const auto rs = mod_rsrc(vout + t0);
#pragma unroll
    for (int r = 0; r < T / 2 / NT; ++r) {
      const int q = tid + r * NT;
      const double2 u = *reinterpret_cast<const double2*>(v + 2 * q);
      if constexpr (EDGE) {
        if (t0 + 2 * q < N) vout[t0 + 2 * q] = u.x;
        if (t0 + 2 * q + 1 < N) vout[t0 + 2 * q + 1] = u.y;
      } else {
        pipe::st2_oob(rs, (unsigned)q * 16u, u.x, u.y);
      }
    }
  }
};

// Interior tiles [1, nfull): window [t0 - S - (S&1), t0 + T) inside the
// signal.  Persistent grid of 8 * (blocks per XCD), XCD x walks chunk x.
// src (V_0), wout rows (ldw even) and vout 16-B aligned.
template <int L, int NT, int T, int J1, bool FMA>
__global__ __launch_bounds__(NT) void modwt_fwd_pipe(const double* __restrict__ src,
                                                     double* __restrict__ wout, int64_t ldw,
                                                     double* __restrict__ vout, int64_t N,
                                                     int64_t ti0, int64_t ti1, ModwtTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using P = FwdPipe<L, NT, T, J1, FMA>;
  using G = FwdPipeGeo<L, T, J1>;
  const int64_t nt = ti1 - ti0;
  const int x = blockIdx.x & 7, nbx = gridDim.x >> 3, bx = blockIdx.x >> 3;
  const int64_t q = nt >> 3, rr = nt & 7;
  const int64_t c0 = ti0 + x * q + (x < rr ? x : rr), c1 = c0 + q + (x < rr ? 1 : 0);
  int64_t tile = c0 + bx;
  if (tile >= c1) return;  // block-uniform
  int off = 0, cur = 0;
  auto window = [&](int64_t t) { return src + (t * T - G::S - (G::S & 1)); };
  PipeDma<NT, G::units()>::issue(lds + G::dma_lds(), window(tile), off);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (;;) {
    lds_barrier();  // this tile's window (every wave waited for its pieces)
    const int64_t t0 = tile * T;
    const int64_t tn = tile + nbx;
    double* b = lds + cur * G::buf();
    if (tn < c1) PipeDma<NT, G::units()>::issue(lds + (cur ^ 1) * G::buf() + G::dma_lds(), window(tn), off);
    P::template level<1, false>(tp, b, wout, ldw, t0, N);
    P::template vstore<false>(b, vout, t0, N);
    if (tn >= c1) break;
    vm_wait<P::nstores()>();  // the next window; this tile's stores stay in flight
    tile = tn;
    cur ^= 1;
  }
}

// Tiles whose window wraps or runs past the end: one block each (tile index
// from the list {0} + [ti1, ntile)), wrapped plain loads, guarded stores.
template <int L, int NT, int T, int J1, bool FMA>
__global__ __launch_bounds__(NT) void modwt_fwd_pipe_edge(const double* __restrict__ src,
                                                          double* __restrict__ wout, int64_t ldw,
                                                          double* __restrict__ vout, int64_t N,
                                                          int64_t ti0, int64_t ti1,
                                                          ModwtTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using P = FwdPipe<L, NT, T, J1, FMA>;
  using G = FwdPipeGeo<L, T, J1>;
  const int64_t tile = (int64_t)blockIdx.x < ti0 ? blockIdx.x : ti1 + (blockIdx.x - ti0);
  const int64_t t0 = tile * T;
  for (int e = threadIdx.x; e < G::W; e += NT) lds[G::kPad + e] = src[wrap_mod(t0 - G::S + e, N)];
  lds_barrier();
  P::template level<1, true>(tp, lds, wout, ldw, t0, N);
  P::template vstore<true>(lds, vout, t0, N);
}

}  // namespace jwv
