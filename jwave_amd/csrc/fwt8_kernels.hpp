// fwt8_kernels.hpp — FWT tile kernels for 8-column slabs with compile-time
// geometry (tap count L, tile T rows, fused levels K): the C = 8 counterpart
// of fwt1_kernels.hpp.  They run the column passes of a row-major matrix
// (BasicTransform.forward/reverse(double[][]), BasicTransform.java:361-474)
// and the strided axes of 3-D volumes (BasicTransform.java:509-659).
//
// Same math and summation order as fwt_fwd_tile / fwt_rev_tile
// (Wavelet.java:236-303, see fwt_kernels.hpp), so EXACT results stay
// bit-identical.  Differences from the generic C = 8 kernels are structural:
//  * forward: a lane computes two adjacent pairs (2q, 2q+1) of one column
//    from L+2 window rows instead of 2L reads for two separate pairs.  The
//    window sits in LDS with one pad row per 16 rows (row r at 8*(r + r/16)
//    doubles): the 32 lanes of a ds_read_b64 group hold 8 columns x 4 couples
//    16 rows apart, whose addresses then differ by 136 doubles = 16 banks, so
//    the group is conflict-free (unpadded, rows 4 apart share all 16 banks:
//    4-way).  A wave's couples share their row phase mod 16, so the window
//    loads are immediate offsets from one address (item8_couple).  LDS-DMA
//    fills the padded layout directly: one wave instruction moves 64 x 16 B =
//    16 rows.  Levels run in place (results wait in
//    registers across one barrier);
//  * reverse: one pair per lane, consecutive lanes on consecutive columns then
//    pairs (a 256-B conflict-free span per 32 lanes); every window of the tile
//    (level-K approximation + K detail windows) arrives in one LDS-DMA burst
//    instead of one HBM round trip per level; levels ping-pong between two
//    buffers with one barrier per level (Rev1Geo layout, rows of 8).
#pragma once
#include "fwt1_kernels.hpp"

namespace jwv {

// padded LDS row offset (doubles) of window row r
__host__ __device__ constexpr int prow8(int r) { return 8 * (r + (r >> 4)); }

// forward work item w -> column c = w & 7, couple q = 32*qg + 4*qa + qb with
// qa = (w >> 3) & 7, qb = (w >> 6) & 3 (one value per wave), qg = w >> 8.  The
// 32 items of one ds_read group sit at couples 4 apart (rows 16 apart: 17
// padded rows = 136 doubles = 8 banks-of-8-B apart, conflict-free), and since
// qb is wave-uniform the pad rows a couple's L+2 window crosses are too: the
// window loads become compile-time offsets from one address (load_couple8).
__device__ __forceinline__ int item8_couple(int w) {
  return ((w >> 8) << 5) + (((w >> 3) & 7) << 2) + ((w >> 6) & 3);
}

// x[j] = window row 4q + j of column c; xb = lds + 8*(4q + (4q >> 4)) + c with
// 4q = 16m + 4*QB, so row 4q + j sits (j + ((4*QB + j) >> 4)) padded rows on
template <int N, int QB>
__device__ __forceinline__ void load_couple8_qb(const double* xb, double* x) {
#pragma unroll
  for (int j = 0; j < N; ++j) x[j] = xb[8 * (j + ((4 * QB + j) >> 4))];
}
template <int N>
__device__ __forceinline__ void load_couple8(const double* xb, int qb, double* x) {
  switch (__builtin_amdgcn_readfirstlane(qb)) {  // wave-uniform: a scalar branch
    case 0: load_couple8_qb<N, 0>(xb, x); break;
    case 1: load_couple8_qb<N, 1>(xb, x); break;
    case 2: load_couple8_qb<N, 2>(xb, x); break;
    default: load_couple8_qb<N, 3>(xb, x); break;
  }
}

// W rows x 8 columns -> padded LDS rows by LDS-DMA (16 B per lane).
// rowoff(e): offset of row e's first column (16-B aligned in global memory).
template <int NT, typename RowOff>
__device__ __forceinline__ void load_rows8_padded(double* lds, const double* __restrict__ src,
                                                  int W, RowOff rowoff) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nunits = W * 4;
  for (int u0 = wave * 64; u0 < nunits; u0 += NT) {
    const int u = u0 + lane;
    if (u < nunits)
      __builtin_amdgcn_global_load_lds(
          (const void*)(src + rowoff(u >> 2) + 2 * (u & 3)),
          (__attribute__((address_space(3))) void*)(lds + 136 * (u0 >> 6)), 16, 0, 0);
  }
}

template <int L, int T, int K>
struct Fwd8Geo {
  using G = Fwd1Geo<L, T, K>;
  static constexpr int lds_doubles() { return prow8(G::m(0)) + 16; }
};

template <int L, int NT, int T, int K, bool FMA, int l>
struct Fwd8Level {
  // In place: level l reads window rows [0, m(l-1)) and leaves its m(l)
  // approximation rows at [0, m(l)).  y: detail rows of the slab (row i at
  // y + i*sl), ya: level-K approximation rows (row i at ya + i*sa).
  __device__ __forceinline__ static void run(const FwdTaps<L>& tp, double* lds,
                                             double* __restrict__ y, int64_t sl, int hl, int t,
                                             double* __restrict__ ya, int64_t sa) {
    using G = Fwd1Geo<L, T, K>;
    constexpr int mo = G::m(l);  // even
    constexpr int own = T >> l;  // even
    constexpr int NCQ = mo / 2;  // couples per column
    constexpr int NI = ((NCQ + 31) / 32) * 256;
    static_assert(NT % 64 == 0, "qb must be wave-uniform");
    constexpr int R = (NI + NT - 1) / NT;
    const int tid = opaque_tid();  // per-level: keeps address math out of the prologue
    double2 av[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int w = tid + r * NT;
      const int c = w & 7, q = item8_couple(w);
      if (((r + 1) * NT <= NI || w < NI) && q < NCQ) {
        double x[L + 2];
        load_couple8<L + 2>(lds + prow8(4 * q) + c, (w >> 6) & 3, x);
        double a0, d0, a1, d1;
        fwd_pair<L, FMA>(tp, [&](int j) { return x[j]; }, a0, d0);
        fwd_pair<L, FMA>(tp, [&](int j) { return x[j + 2]; }, a1, d1);
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(d0), "+v"(d1) :: "memory");  // slot boundary
        const int p = 2 * q;
        if (p < own) {
          double* yd = y + ((int64_t)(hl >> 1) + (int64_t)t * own + p) * sl + c;
          yd[0] = d0;
          yd[sl] = d1;
          if constexpr (l == K) {
            double* yo = ya + ((int64_t)t * own + p) * sa + c;
            yo[0] = a0;
            yo[sa] = a1;
          }
        }
        if constexpr (l < K) av[r] = make_double2(a0, a1);
      }
    }
    if constexpr (l < K) {
      lds_barrier();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int w = tid + r * NT;
        const int c = w & 7, q = item8_couple(w);
        if (((r + 1) * NT <= NI || w < NI) && q < NCQ) {
          lds[prow8(2 * q) + c] = av[r].x;
          lds[prow8(2 * q + 1) + c] = av[r].y;
        }
      }
      lds_barrier();
      Fwd8Level<L, NT, T, K, FMA, l + 1>::run(tp, lds, y, sl, hl >> 1, t, ya, sa);
    }
  }
};

// Grid: nouter * (inner/8) * (h/T) blocks, tile-fastest, XCD-remapped like
// fwt_fwd_tile.  Views as fwt_fwd_tile: row i of slab (o, c0) of the level
// input is src + view_base(sv, o) + c0 + i*sv.s_len.  Needs inner % 8 == 0
// and 16-B aligned row segments (host: dma_view).
template <int L, int NT, int T, int K, bool FMA>
__global__ __launch_bounds__(NT) void fwt_fwd_tile8(const double* __restrict__ src, AxisView sv,
                                                    double* __restrict__ dst, AxisView dv,
                                                    double* __restrict__ adst, AxisView av_, int h,
                                                    int inner, FwdTaps<L> tp, int order) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using G = Fwd1Geo<L, T, K>;
  const int ntile = h / T, ncb = inner >> 3;
  const int nblk = gridDim.x;
  int b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  // order 0: tile-fastest (a slab's tiles run side by side: halo rows in the
  // same L2); order 1: slab-fastest (concurrent blocks cover whole matrix
  // rows: contiguous DRAM rows, both 64-B halves of each 128-B line at once)
  const int nsl = nblk / ntile;
  const int t = order ? b / nsl : b % ntile;
  const int rest = order ? b % nsl : b / ntile;
  const int64_t o = rest / ncb;
  const int c0 = (rest % ncb) * 8;
  const double* s = src + view_base(sv, o) + c0;
  const int msk = h - 1, base = t * T;
  const int64_t ssl = sv.s_len;
  load_rows8_padded<NT>(lds, s, G::m(0),
                        [&](int e) { return (int64_t)((base + e) & msk) * ssl; });
  dma_fence_barrier();
  Fwd8Level<L, NT, T, K, FMA, 1>::run(tp, lds, dst + view_base(dv, o) + c0, dv.s_len, h, t,
                                       adst + view_base(av_, o) + c0, av_.s_len);
}

// ---------------------------------------------------------------- reverse
template <int L, int T, int K>
struct Rev8Geo {
  using G = Rev1Geo<L, T, K>;
  static constexpr int lds_doubles() { return 8 * G::lds_doubles(); }
};

template <int L, int NT, int T, int K, bool FMA, int l>
struct Rev8Level {
  __device__ __forceinline__ static void run(const RevTaps<L>& tp, double* lds, int t,
                                             double* __restrict__ y, int64_t sl) {
    using G = Rev1Geo<L, T, K>;
    constexpr int Q = G::Q;
    constexpr int np = G::len(l) / 2;               // pairs per column of this level
    constexpr int off = G::c(l + 1) - G::c(l) / 2;  // local row of a[pair 0]
    constexpr int NI = np * 8;
    constexpr int R = (NI + NT - 1) / NT;
    // head pairs (global pair index < Q-1) exist only in the first tiles, and
    // there only in slot 0: ml < Q-1 + c(l)/2
    static_assert(8 * (Q - 1 + G::c(l) / 2) <= NT, "head pairs must sit in slot 0");
    const double* ab = lds + 8 * ((((l + 1) & 1) != 0) ? G::buf1() : G::buf0());
    const double* db = lds + 8 * G::doff(l);
    double* ob = lds + 8 * (((l & 1) != 0) ? G::buf1() : G::buf0());
    const int tid = opaque_tid();  // per-level: keeps address math out of the prologue
    const int pbase = t * (T >> (l + 1)) - G::c(l) / 2;  // global index of window pair 0
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int w = tid + r * NT;
      if ((r + 1) * NT <= NI || w < NI) {
        const int c = w & 7, ml = w >> 3;
        const int li = off + ml;
        const double* ac = ab + c;
        const double* dc = db + c;
        double xe, xo;
        rev_pair<L, FMA>(tp, ac + li * 8, dc + li * 8, 8, xe, xo);
        if (r == 0 && pbase < Q - 1) {
          const int mg = pbase + ml;
          if (mg >= 0 && mg < Q - 1)
            rev_pair_head<L, FMA>(
                tp, mg, [=](int q) { return ac[(li - q) * 8]; },
                [=](int q) { return dc[(li - q) * 8]; }, xe, xo);
        }
        if constexpr (l == 0) {
          double* yo = y + ((int64_t)t * T + 2 * ml) * sl + c;
          yo[0] = xe;
          yo[sl] = xo;
        } else {
          ob[(2 * ml) * 8 + c] = xe;
          ob[(2 * ml + 1) * 8 + c] = xo;
        }
      }
    }
    if constexpr (l > 0) {
      lds_barrier();
      Rev8Level<L, NT, T, K, FMA, l - 1>::run(tp, lds, t, y, sl);
    }
  }
};

// Grid: nouter * (inner/8) * (hK/T) blocks.  asrc: level-K approximation
// (view as, length hK >> K); coef: coefficient array (view cv, details of
// level size h at rows [h/2, h)); dst: output rows [0, hK) (view dv).
template <int L, int NT, int T, int K, bool FMA>
__global__ __launch_bounds__(NT) void fwt_rev_tile8(const double* __restrict__ asrc, AxisView as,
                                                    const double* __restrict__ coef, AxisView cv,
                                                    double* __restrict__ dst, AxisView dv, int hK,
                                                    int inner, RevTaps<L> tp, int order) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using G = Rev1Geo<L, T, K>;
  const int ntile = hK / T, ncb = inner >> 3;
  const int nblk = gridDim.x;
  int b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  // order 0: tile-fastest (a slab's tiles run side by side: halo rows in the
  // same L2); order 1: slab-fastest (concurrent blocks cover whole matrix
  // rows: contiguous DRAM rows, both 64-B halves of each 128-B line at once)
  const int nsl = nblk / ntile;
  const int t = order ? b / nsl : b % ntile;
  const int rest = order ? b % nsl : b / ntile;
  const int64_t o = rest / ncb;
  const int c0 = (rest % ncb) * 8;
  const double* sa = asrc + view_base(as, o) + c0;
  const double* sc = coef + view_base(cv, o) + c0;
  const int64_t asl = as.s_len, csl = cv.s_len;
  // every window in one burst: level-K approximation, then the details
  {
    const int BK = (t * T >> K) - G::c(K);
    const int am = (hK >> K) - 1;
    load_window<8, NT, 1>(lds + 8 * ((K & 1) ? G::buf1() : G::buf0()), sa, G::len(K), true, 0,
                          inner, [&](int e) { return (int64_t)((BK + e) & am) * asl; });
  }
#pragma unroll
  for (int l = K - 1; l >= 0; --l) {
    const int half = hK >> (l + 1), hm = half - 1;
    const int B = (t * T >> (l + 1)) - G::c(l + 1);
    load_window<8, NT, 1>(lds + 8 * G::doff(l), sc, G::len(l + 1), true, 0, inner, [&](int e) {
      return ((int64_t)half + ((B + e) & hm)) * csl;
    });
  }
  dma_fence_barrier();
  Rev8Level<L, NT, T, K, FMA, K - 1>::run(tp, lds, t, dst + view_base(dv, o) + c0, dv.s_len);
}

}  // namespace jwv
