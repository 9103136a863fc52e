// fwt1_chain.hpp — a whole FastWaveletTransform of a long contiguous signal
// in ONE launch per direction (C = 1, compiled-in tap count).
//
// The multi-launch plan (fwt1_kernels.hpp + fwt1_res.hpp) pays, per
// direction, two kernel boundaries and two latency-bound tail kernels whose
// blocks start only after the previous grid has drained.  Here the stages of
// that plan are roles inside one grid and hand their level approximations to
// each other through HBM/L2 with the agent-scope protocol of jwv_device.hpp
// (write-through stores, one atomic per workgroup, write-through loads of the
// handed-off bytes after the signal — no acquire, no L2 write-back):
//
// Forward (fwt_fwd_chain1), roles by arrival — no workgroup ever waits:
//   A  every block: a tile of TA level-0 samples, KA levels (the big pass);
//      its TA>>KA approximations go write-through to wsA, then it counts
//      itself into the counter of every B unit whose window it feeds;
//   B  the block that completes a unit's counter: TB level-KA samples (a
//      window of wsA), KB more levels, approximations write-through to wsB,
//      then counts into the C counter;
//   C  the block that completes the C counter: the remaining levels of the
//      whole wsB array resident in LDS (fwd_res1_levels).
// Reverse (fwt_rev_chain1), a persistent grid of co-resident blocks with
// static roles (no ticket counter: one atomic word serialises block starts):
//   block 0         R: resident synthesis of the coefficient prefix up to hR
//                      samples, written through to wsR, then a flag;
//   blocks 1..nM    M: a tile of TM outputs, KM levels, from wsR + details;
//                      written through to wsM, then the unit's flag;
//   every block     A: tiles of TA outputs, KA levels, from wsM + details.
//   M and A blocks load their first detail windows before they wait (no
//   dependency).  Waits are bounded polls, so the grid drains even if it
//   were not co-resident (the timeout word then reports the failure).
//
// Math, summation order and the array-head handling are exactly those of
// the per-level reference loops (Wavelet.java:236-303) as implemented by
// Fwd1Level / Rev1Level / *_res1_levels, so EXACT results stay bit-identical.
//
// Counters: cnt[0, nU) B-unit arrivals, cnt[nU] C arrivals (forward); every
// counter is reset to 0 by the block that completes it, so a buffer zeroed
// once at allocation is ready for every call.  Reverse: ctl[0] timeout word,
// ctl[1] R flag, ctl[2 + u] M-unit flags; flags carry the call's epoch
// (never 0), so they need no reset.
#pragma once
#include "fwt1_kernels.hpp"
#include "fwt1_res.hpp"

namespace jwv {

template <int L, int NT, int TA, int KA, int TB, int KB, int CAPC>
struct FwdChain {
  using GA = Fwd1Geo<L, TA, KA>;
  using GB = Fwd1Geo<L, TB, KB>;
  // LDS of the tile roles; the launch adds room for the resident role's
  // hC + 2 doubles (ctl_off) and 16 B of control words after that.
  static constexpr int lds_tiles() {
    return GA::lds_doubles() > GB::lds_doubles() ? GA::lds_doubles() : GB::lds_doubles();
  }
  __host__ __device__ static int ctl_off(int hC) {
    const int m = lds_tiles();
    return ((hC + 2 > m ? hC + 2 : m) + 1) & ~1;
  }
  static constexpr int oA = TA >> KA;
  static_assert(TB % oA == 0, "B units must start on A-tile boundaries");
};

// Forward tail LDS: the B window, the resident C array, 16 B of control.
template <int L, int TB, int KB>
__host__ __device__ inline int tail_ctl_off(int hC) {
  const int m = Fwd1Geo<L, TB, KB>::lds_doubles();
  return ((hC + 2 > m ? hC + 2 : m) + 1) & ~1;
}

template <int L, int NT, int TA, int KA, int TB, int KB, int CAPC, bool FMA, int MINW = 1>
__global__ __launch_bounds__(NT, MINW) void fwt_fwd_chain1(const double* __restrict__ src,
                                                     double* __restrict__ dst, double* wsA,
                                                     double* wsB, unsigned* cnt, int h, int levC,
                                                     FwdTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using CH = FwdChain<L, NT, TA, KA, TB, KB, CAPC>;
  using GA = typename CH::GA;
  using GB = typename CH::GB;
  const int tid = threadIdx.x;
  const int ntA = h / TA;
  const int hB = h >> KA, nU = hB / TB;
  int* ctl = reinterpret_cast<int*>(lds + CH::ctl_off(hB >> KB));  // [0,1] units completed, [3] count / C flag
  // B unit u reads wsA[u*TB, u*TB + mB) (mod hB): A tiles [u*g, u*g + need)
  constexpr int g = TB / CH::oA;
  constexpr int need = (GB::m(0) + CH::oA - 1) / CH::oA;

  // ---- A: the big pass (tile t, KA levels)
  int b = blockIdx.x;
  if ((ntA & 7) == 0) b = (b & 7) * (ntA >> 3) + (b >> 3);
  const int t = b;
  {
    const int msk = h - 1, base = t * TA;
    load_window<1, NT, (GA::m(0) + NT - 1) / NT>(
        lds, src, GA::m(0), true, 0, 1, [&](int e) { return (int64_t)((base + e) & msk); });
    dma_fence_barrier();
    Fwd1Level<L, NT, TA, KA, FMA, 1, true>::run(tp, lds, dst, h, t, wsA);
  }
  drain_stores();
  __syncthreads();
  if (tid == 0) {
    int n = 0;
    const int u0 = t / g;
    const int ncand = (need - 1) / g + 2 < nU ? (need - 1) / g + 2 : nU;
    for (int j = 0; j < ncand; ++j) {
      const int u = (u0 - j + nU) % nU;
      int d = t - u * g;
      if (d < 0) d += ntA;
      if (d < need) {
        const unsigned old = atomic_add_agent(cnt + u, 1u);
        if (old == (unsigned)need - 1) {
          store_agent(cnt + u, 0u);
          ctl[n++] = u;
        }
      }
    }
    ctl[3] = n;
  }
  __syncthreads();
  const int nb = ctl[3];
  if (nb == 0) return;

  // ---- B: units this block completed (KB levels on a window of wsA)
  for (int k = 0; k < nb; ++k) {
    const int u = ctl[k];
    const int msk = hB - 1, base = u * TB;
    load_window_wt<NT, (GB::m(0) + NT - 1) / NT>(lds, wsA, GB::m(0),
                                                  [&](int e) { return (base + e) & msk; });
    lds_barrier();
    Fwd1Level<L, NT, TB, KB, FMA, 1, true>::run(tp, lds, dst, hB, u, wsB);
    drain_stores();
    __syncthreads();
    if (tid == 0) {
      const unsigned old = atomic_add_agent(cnt + nU, 1u);
      const int last = old == (unsigned)nU - 1;
      if (last) store_agent(cnt + nU, 0u);
      ctl[3] = last;  // nb is already in registers (nb <= 2: a tile feeds <= 2 units)
    }
    __syncthreads();
    if (ctl[3]) {
      // ---- C: the remaining levels of wsB, resident
      const int hC = hB >> KB;
      load_window_wt<NT, (CAPC + NT - 1) / NT>(lds, wsB, hC, [](int e) { return e; });
      lds_barrier();
      fwd_res1_levels<L, NT, CAPC, FMA>(lds, dst, hC, levC, tp);
      return;
    }
    __syncthreads();  // LDS reuse by the next unit
  }
}

// ---------------------------------------------------------------- reverse
template <int L, int NT, int CAPR, int TM, int KM, int TA, int KA>
struct RevChain {
  using GM = Rev1Geo<L, TM, KM>;
  using GA = Rev1Geo<L, TA, KA>;
  static constexpr int lds_tiles() {
    return GM::lds_doubles() > GA::lds_doubles() ? GM::lds_doubles() : GA::lds_doubles();
  }
  static int lds_doubles(int hR) { return hR + 2 > lds_tiles() ? hR + 2 : lds_tiles(); }
};

// Detail windows of a rev tile (levels K-1..0) into LDS, as fwt_rev_tile1.
template <int L, int NT, int T, int K>
__device__ __forceinline__ void rev1_load_details(double* lds, const double* __restrict__ coef,
                                                  int hK, int t) {
  using G = Rev1Geo<L, T, K>;
  constexpr int MAXU = (G::len(1) + NT - 1) / NT;
#pragma unroll
  for (int l = K - 1; l >= 0; --l) {
    const int half = hK >> (l + 1), hm = half - 1;
    const int B = (t * T >> (l + 1)) - G::c(l + 1);
    load_window<1, NT, MAXU>(lds + G::doff(l), coef, G::len(l + 1), true, 0, 1,
                             [&](int e) { return (int64_t)half + ((B + e) & hm); });
  }
}
// Level-K approximation window (handed off by another workgroup): sc1 loads.
template <int L, int NT, int T, int K>
__device__ __forceinline__ void rev1_load_approx(double* lds, const double* asrc, int hK, int t) {
  using G = Rev1Geo<L, T, K>;
  constexpr int MAXU = (G::len(K) + NT - 1) / NT;
  const int BK = (t * T >> K) - G::c(K);
  const int am = (hK >> K) - 1;
  load_window_wt<NT, MAXU>(lds + ((K & 1) ? G::buf1() : G::buf0()), asrc, G::len(K),
                           [&](int e) { return (BK + e) & am; });
}

// h: output length; hR = h0R << (nR-1): resident part's output (wsR);
// hM = hR << KM (wsM); h = hM << KA.
// Persistent grid of G co-resident blocks (G >= 1 + nM, sized by the host
// from the occupancy query): block 0 runs R, blocks 1..nM run the M units,
// then every block takes A tiles b, b + G, ...  ctl: [0] timeout word (set
// by a wait that gave up; read and cleared by the host after the call), [1] R
// flag, [2 + u] M flags.  Waits are bounded (poll_eq/poll_all).
template <int L, int NT, int CAPR, int TM, int KM, int TA, int KA, bool FMA, int MINW>
__global__ __launch_bounds__(NT, MINW) void fwt_rev_chain1(const double* __restrict__ coef,
                                                           double* __restrict__ dst, double* wsR,
                                                           double* wsM, unsigned* ctlg, int h,
                                                           int h0R, int nR, unsigned epoch,
                                                           unsigned spins, RevTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x, b = blockIdx.x, G = gridDim.x;
  const int hR = h0R << (nR - 1), hM = hR << KM;
  const int nM = hM / TM, nA = h / TA;
  unsigned* tmo = ctlg;
  unsigned* rflag = ctlg + 1;
  unsigned* mflag = ctlg + 2;

  if (b == 0) {  // ---- R: resident deep levels
    load_window<1, NT, (CAPR + NT - 1) / NT>(lds, coef, hR, true, 0, 1,
                                              [&](int e) { return (int64_t)e; });
    dma_fence_barrier();
    rev_res1_levels<L, NT, CAPR, FMA>(lds, h0R, nR, tp);
    for (int q = 2 * tid; q < hR; q += 2 * NT) st2<true>(wsR + q, lds[q], lds[q + 1]);
    drain_stores();
    __syncthreads();
    if (tid == 0) store_agent(rflag, epoch);
  } else if (b <= nM) {  // ---- M: unit u, KM levels from wsR
    const int u = b - 1;
    rev1_load_details<L, NT, TM, KM>(lds, coef, hM, u);
    if (tid == 0) poll_eq(rflag, epoch, tmo, spins);
    __syncthreads();
    rev1_load_approx<L, NT, TM, KM>(lds, wsR, hM, u);
    dma_fence_barrier();  // the detail DMA and the approximation window
    Rev1Level<L, NT, TM, KM, FMA, KM - 1, true>::run(tp, lds, u, wsM);
    drain_stores();
    __syncthreads();
    if (tid == 0) store_agent(mflag + u, epoch);
  }
  // ---- A: tiles b, b + G, ...; KA levels from wsM.  The first tile's
  // details are fetched while the M units finish; after every M flag has been
  // seen once, each tile is one load burst (details DMA + sc1 approximation).
  int t = b;
  if (t >= nA) return;
  if (b > nM) rev1_load_details<L, NT, TA, KA>(lds, coef, h, t);
  else __syncthreads();  // R / M role done with LDS
  if (tid < 64) poll_all(mflag, nM, epoch, tmo, spins);
  __syncthreads();
  for (bool first = b > nM;; first = false) {
    if (!first) rev1_load_details<L, NT, TA, KA>(lds, coef, h, t);
    rev1_load_approx<L, NT, TA, KA>(lds, wsM, h, t);
    dma_fence_barrier();
    Rev1Level<L, NT, TA, KA, FMA, KA - 1>::run(tp, lds, t, dst);
    t += G;
    if (t >= nA) break;
    lds_barrier();  // LDS reuse by the next tile
  }
}

// ====================================================================
// Head / tail kernels: the latency-bound ends of the multi-launch plan fused
// into one launch each, the big pass staying a standalone tile kernel
// (fwt_fwd_tile1 / fwt_rev_tile1: its own occupancy, fresh blocks, no
// hand-off work).  Measured on config 2 this beats both the three-launch plan
// and the whole-transform chains above when the data is MALL-warm.
// ====================================================================

// Forward tail: B units (tiles of TB level-input samples, KB levels; input =
// the big pass's approximation, written by the previous launch) and, in the
// block that completes the counter, the resident C levels.  Grid: hB / TB.
// cnt[0]: arrival counter, never reset; the block whose add returns last_old
// is the last arriver (jwv_epoch.hpp).
template <int L, int NT, int TB, int KB, int CAPC, bool FMA>
__global__ __launch_bounds__(NT) void fwt_fwd_tail1(const double* __restrict__ src,
                                                    double* __restrict__ dst, double* wsB,
                                                    unsigned* cnt, unsigned last_old, int hB,
                                                    int levC, FwdTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using GB = Fwd1Geo<L, TB, KB>;
  // XCD x (blocks b = x mod 8) takes the contiguous units [x nU/8, (x+1) nU/8):
  // a unit's halo (up to (L-2)(2^KB - 1) samples past its TB own ones, 1.5 x
  // TB at L = 8, KB = 9) is its neighbours' input, fetched into the same L2
  // (round-robin dealing put every neighbour on another XCD: 2.6 x the input
  // from the fabric, r05g)
  const int tid = threadIdx.x, nU = gridDim.x;
  const int u = (nU & 7) == 0 ? (blockIdx.x & 7) * (nU >> 3) + (blockIdx.x >> 3)
                              : (int)blockIdx.x;
  int* ctl = reinterpret_cast<int*>(lds + tail_ctl_off<L, TB, KB>(hB >> KB));
  {
    const int msk = hB - 1, base = u * TB;
    load_window<1, NT, (GB::m(0) + NT - 1) / NT>(
        lds, src, GB::m(0), true, 0, 1, [&](int e) { return (int64_t)((base + e) & msk); });
    dma_fence_barrier();
    Fwd1Level<L, NT, TB, KB, FMA, 1, true>::run(tp, lds, dst, hB, u, wsB);
  }
  drain_stores();
  __syncthreads();
  if (tid == 0) {
    ctl[0] = atomic_add_agent(cnt, 1u) == last_old;
  }
  __syncthreads();
  if (!ctl[0]) return;
  const int hC = hB >> KB;
  load_window_wt<NT, (CAPC + NT - 1) / NT>(lds, wsB, hC, [](int e) { return e; });
  lds_barrier();
  fwd_res1_levels<L, NT, CAPC, FMA>(lds, dst, hC, levC, tp);
}

// Reverse head: the resident deep levels (R) and the first tiled pass (M
// units) in one launch with NO inter-workgroup dependency.  Every block is an
// M unit that synthesises the coefficient prefix [0, hR) itself (R, resident
// in its own LDS region: 8 KB of L2-served reads and ~10 latency-bound levels
// per block, overlapped with its detail-window DMA), takes its level-K
// approximation window from that LDS copy, and runs KM levels; the hR << KM
// outputs go to wsM (plain stores, read by the next launch).  The R result is
// identical in every block (same code, same inputs), so the output equals the
// one-producer hand-off it replaces, without a flag, a poll or a timeout path.
// Grid hM / TM blocks.
template <int L, int TM, int KM>
struct RevHeadGeo {
  using G = Rev1Geo<L, TM, KM>;
  static constexpr int roff() { return (G::lds_doubles() + 1) & ~1; }  // R region (16-B aligned)
  __host__ __device__ static int lds_doubles(int hR) { return roff() + hR + 2; }
};

template <int L, int NT, int CAPR, int TM, int KM, bool FMA>
__global__ __launch_bounds__(NT) void fwt_rev_head1(const double* __restrict__ coef,
                                                    double* __restrict__ wsM, int h0R, int nR,
                                                    RevTaps<L> tp) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using G = Rev1Geo<L, TM, KM>;
  const int tid = threadIdx.x, u = blockIdx.x;
  const int hR = h0R << (nR - 1), hM = hR << KM;
  double* rl = lds + RevHeadGeo<L, TM, KM>::roff();
  JWV_STAMP(0);
  // one DMA burst: this unit's detail windows and the coefficient prefix
  rev1_load_details<L, NT, TM, KM>(lds, coef, hM, u);
  load_window<1, NT, (CAPR + NT - 1) / NT>(rl, coef, hR, true, 0, 1,
                                            [&](int e) { return (int64_t)e; });
  dma_fence_barrier();
  JWV_STAMP(1);
  rev_res1_levels<L, NT, CAPR, FMA>(rl, h0R, nR, tp);  // ends with a block barrier
  JWV_STAMP(30);
  {
    const int BK = (u * TM >> KM) - G::c(KM), am = hR - 1;
    double* aw = lds + ((KM & 1) ? G::buf1() : G::buf0());
    for (int e = tid; e < G::len(KM); e += NT) aw[e] = rl[(BK + e) & am];
  }
  lds_barrier();
  Rev1Level<L, NT, TM, KM, FMA, KM - 1>::run(tp, lds, u, wsM);
  JWV_STAMP(31);
}

}  // namespace jwv
