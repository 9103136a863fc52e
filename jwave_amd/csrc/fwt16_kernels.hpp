// fwt16_kernels.hpp — FWT tile kernels for 16-column slabs (the column passes
// of a row-major matrix, BasicTransform.forward/reverse(double[][]),
// BasicTransform.java:361-474, and the strided axes of 3-D volumes,
// :509-659).  Same math, order and outputs as fwt8_kernels.hpp (Wavelet.java:
// 236-303 through fwd_pair / rev_pair), so EXACT results stay bit-identical.
//
// Why 16 columns: a slab row is then 128 B, one whole cache line.  With
// 8-column slabs every row segment a block loads or stores is half a line,
// and the other half belongs to another block (another slab); the column
// tiles ran at 3.3-3.5 TB/s against 4.7 for the row tiles of the same bytes.
// Here every global load and store of a tile covers whole 128-B lines.
//
//  * forward: a lane computes a couple (pairs 2q, 2q+1) of one column from
//    L+2 window rows; lanes 0-15 / 16-31 of a ds_read_b64 group (256 B per
//    LDS cycle) hold couples q and q+1, i.e. rows 4q+j and 4q+4+j.  Rows are
//    stored two per 256-B line with the half swizzled, h(r) = (r & 1) ^
//    ((r >> 2) & 1), so those two rows always sit in opposite halves: the
//    group is conflict-free without padding (unswizzled they share one half:
//    2-way).  The swizzle turns each window read into an immediate offset from
//    one of two per-lane bases.  LDS-DMA writes the swizzled image directly
//    (each lane computes the row of its 16-B destination).
//  * reverse: one pair per lane, lanes 0-15 / 16-31 on pairs ml / ml+1: rows
//    li and li+1 of a plain 128-B-row layout, 256 contiguous bytes,
//    conflict-free; every window of the tile arrives in one LDS-DMA burst and
//    levels ping-pong between two buffers (Rev1Geo layout, rows of 16).
#pragma once
#include "fwt8_kernels.hpp"

namespace jwv {

// swizzled LDS offset (doubles) of window row r, column 0
__host__ __device__ constexpr int srow16(int r) {
  return 32 * (r >> 1) + 16 * ((r & 1) ^ ((r >> 2) & 1));
}

template <int L, int T, int K>
struct Fwd16Geo {
  using G = Fwd1Geo<L, T, K>;
  static constexpr int rows() { return (G::m(0) + 1) & ~1; }  // whole lines
  static constexpr int lds_doubles() { return 16 * rows() + 32; }
};

// W rows (W even) x 16 columns -> swizzled LDS by LDS-DMA.  Unit u (16 B)
// lands at lds + 2u: line u >> 4, half (u >> 3) & 1, columns 2(u & 7) + {0,1};
// that half holds row r = 2*line + (half ^ (line >> 1 & 1)).  rowoff(r): the
// offset of row r's first column (16-B aligned in global memory).
template <int NT, typename RowOff>
__device__ __forceinline__ void load_rows16_swz(double* lds, const double* __restrict__ src, int W,
                                                RowOff rowoff) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nunits = W * 8;
  for (int u0 = wave * 64; u0 < nunits; u0 += NT) {
    const int u = u0 + lane;
    if (u < nunits) {
      const int line = u >> 4, half = (u >> 3) & 1;
      const int r = 2 * line + (half ^ ((line >> 1) & 1));
      __builtin_amdgcn_global_load_lds((const void*)(src + rowoff(r) + 2 * (u & 7)),
                                       (__attribute__((address_space(3))) void*)(lds + 2 * u0), 16,
                                       0, 0);
    }
  }
}

template <int L, int NT, int T, int K, bool FMA, int l>
struct Fwd16Level {
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
    constexpr int NI = NCQ * 16;
    constexpr int R = (NI + NT - 1) / NT;
    const int tid = opaque_tid();  // per-level: keeps address math out of the prologue
    double2 av[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int w = tid + r * NT;
      const bool full = (r + 1) * NT <= NI;
      if (!full && __builtin_amdgcn_readfirstlane((tid & ~63) + r * NT) >= NI) continue;
      const int c = w & 15, qq = w >> 4;
      const int q = full || qq < NCQ ? qq : NCQ - 1;
      // row 4q + j: line 2q + (j >> 1), half k(j) ^ (q & 1), k(j) = (j&1)^((j>>2)&1)
      const int p = q & 1;
      const double* b0 = lds + 64 * q + 16 * p + c;        // k(j) = 0
      const double* b1 = lds + 64 * q + 16 * (p ^ 1) + c;  // k(j) = 1
      double x[L + 2];
#pragma unroll
      for (int j = 0; j < L + 2; ++j) {
        const int kj = (j & 1) ^ ((j >> 2) & 1);
        x[j] = (kj ? b1 : b0)[32 * (j >> 1)];
      }
      double a0, d0, a1, d1;
      fwd_pair<L, FMA>(tp, [&](int j) { return x[j]; }, a0, d0);
      fwd_pair<L, FMA>(tp, [&](int j) { return x[j + 2]; }, a1, d1);
      asm volatile("" : "+v"(a0), "+v"(a1), "+v"(d0), "+v"(d1) :: "memory");  // slot boundary
      if (full || qq < NCQ) {
        const int pp = 2 * q;
        if (pp < own) {
          double* yd = y + ((int64_t)(hl >> 1) + (int64_t)t * own + pp) * sl + c;
          yd[0] = d0;
          yd[sl] = d1;
          if constexpr (l == K) {
            double* yo = ya + ((int64_t)t * own + pp) * sa + c;
            yo[0] = a0;
            yo[sa] = a1;
          }
        }
      }
      if constexpr (l < K) av[r] = make_double2(a0, a1);
    }
    if constexpr (l < K) {
      lds_barrier();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int w = tid + r * NT;
        const int c = w & 15, q = w >> 4;
        if (((r + 1) * NT <= NI || w < NI)) {
          // rows 2q, 2q+1: line q, halves (q >> 1) & 1 and its complement
          const int h = (q >> 1) & 1;
          lds[32 * q + 16 * h + c] = av[r].x;
          lds[32 * q + 16 * (h ^ 1) + c] = av[r].y;
        }
      }
      lds_barrier();
      Fwd16Level<L, NT, T, K, FMA, l + 1>::run(tp, lds, y, sl, hl >> 1, t, ya, sa);
    }
  }
};

// Grid: nouter * (inner/16) * (h/T) blocks, slab order as fwt_fwd_tile8.
// Needs inner % 16 == 0 and 16-B aligned row segments (host: dma_view).
template <int L, int NT, int T, int K, bool FMA>
__global__ __launch_bounds__(NT) void fwt_fwd_tile16(const double* __restrict__ src, AxisView sv,
                                                     double* __restrict__ dst, AxisView dv,
                                                     double* __restrict__ adst, AxisView av_,
                                                     int h, int inner, FwdTaps<L> tp, int order) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using FG = Fwd16Geo<L, T, K>;
  const int ntile = h / T, ncb = inner >> 4;
  const int nblk = gridDim.x;
  int b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  const int nsl = nblk / ntile;
  const int t = order ? b / nsl : b % ntile;
  const int rest = order ? b % nsl : b / ntile;
  const int64_t o = rest / ncb;
  const int c0 = (rest % ncb) * 16;
  const double* s = src + view_base(sv, o) + c0;
  const int msk = h - 1, base = t * T;
  const int64_t ssl = sv.s_len;
  // rows() may exceed m(0) by one: that row is read (wrapped) and never used
  load_rows16_swz<NT>(lds, s, FG::rows(),
                      [&](int e) { return (int64_t)((base + e) & msk) * ssl; });
  dma_fence_barrier();
  Fwd16Level<L, NT, T, K, FMA, 1>::run(tp, lds, dst + view_base(dv, o) + c0, dv.s_len, h, t,
                                        adst + view_base(av_, o) + c0, av_.s_len);
}

// ---------------------------------------------------------------- reverse
template <int L, int T, int K, bool IP>
struct Rev16Geo {
  using G = Rev1Geo<L, T, K>;
  static constexpr int lds_doubles() { return 16 * (IP ? G::ip_lds_doubles() : G::lds_doubles()); }
};

// IP: Rev1Geo's in-place layout (rows of 16); a level's outputs wait in
// registers until every lane has read its inputs (second barrier).
template <int L, int NT, int T, int K, bool FMA, int l, bool IP>
struct Rev16Level {
  __device__ __forceinline__ static void run(const RevTaps<L>& tp, double* lds, int t,
                                             double* __restrict__ y, int64_t sl) {
    using G = Rev1Geo<L, T, K>;
    constexpr int Q = G::Q;
    constexpr int np = G::len(l) / 2;               // pairs per column of this level
    constexpr int off = G::c(l + 1) - G::c(l) / 2;  // local row of a[pair 0]
    constexpr int NI = np * 16;
    constexpr int R = (NI + NT - 1) / NT;
    // head pairs (global pair index < Q-1) exist only in the first tiles, and
    // there only in slot 0: ml < Q-1 + c(l)/2
    static_assert(16 * (Q - 1 + G::c(l) / 2) <= NT, "head pairs must sit in slot 0");
    const double* ab = lds + 16 * (IP ? 0 : (((l + 1) & 1) != 0) ? G::buf1() : G::buf0());
    const double* db = lds + 16 * (IP ? G::ip_doff(l) : G::doff(l));
    double* ob = lds + 16 * (IP ? 0 : ((l & 1) != 0) ? G::buf1() : G::buf0());
    constexpr bool DEF = IP && l > 0;
    double2 dres[DEF ? R : 1];
    const int tid = opaque_tid();  // per-level: keeps address math out of the prologue
    const int pbase = t * (T >> (l + 1)) - G::c(l) / 2;  // global index of window pair 0
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int w = tid + r * NT;
      if ((r + 1) * NT <= NI || w < NI) {
        const int c = w & 15, ml = w >> 4;
        const int li = off + ml;
        const double* ac = ab + c;
        const double* dc = db + c;
        double xe, xo;
        rev_pair<L, FMA>(tp, ac + li * 16, dc + li * 16, 16, xe, xo);
        if (r == 0 && pbase < Q - 1) {
          const int mg = pbase + ml;
          if (mg >= 0 && mg < Q - 1)
            rev_pair_head<L, FMA>(
                tp, mg, [=](int q) { return ac[(li - q) * 16]; },
                [=](int q) { return dc[(li - q) * 16]; }, xe, xo);
        }
        if constexpr (l == 0) {
          double* yo = y + ((int64_t)t * T + 2 * ml) * sl + c;
          yo[0] = xe;
          yo[sl] = xo;
        } else if constexpr (DEF) {
          // slot fence: the next slot's window reads stay below this one
          asm volatile("" : "+v"(xe), "+v"(xo)::"memory");
          dres[r] = make_double2(xe, xo);
        } else {
          ob[(2 * ml) * 16 + c] = xe;
          ob[(2 * ml + 1) * 16 + c] = xo;
        }
      }
    }
    if constexpr (DEF) {
      lds_barrier();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int w = tid + r * NT;
        if ((r + 1) * NT <= NI || w < NI) {
          const int c = w & 15, ml = w >> 4;
          ob[(2 * ml) * 16 + c] = dres[r].x;
          ob[(2 * ml + 1) * 16 + c] = dres[r].y;
        }
      }
    }
    if constexpr (l > 0) {
      lds_barrier();
      Rev16Level<L, NT, T, K, FMA, l - 1, IP>::run(tp, lds, t, y, sl);
    }
  }
};

// Grid: nouter * (inner/16) * (hK/T) blocks.  asrc: level-K approximation
// (view as, length hK >> K); coef: coefficient array (view cv, details of
// level size h at rows [h/2, h)); dst: output rows [0, hK) (view dv).
template <int L, int NT, int T, int K, bool FMA, bool IP>
__global__ __launch_bounds__(NT) void fwt_rev_tile16(const double* __restrict__ asrc, AxisView as,
                                                     const double* __restrict__ coef, AxisView cv,
                                                     double* __restrict__ dst, AxisView dv, int hK,
                                                     int inner, RevTaps<L> tp, int order) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using G = Rev1Geo<L, T, K>;
  const int ntile = hK / T, ncb = inner >> 4;
  const int nblk = gridDim.x;
  int b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  const int nsl = nblk / ntile;
  const int t = order ? b / nsl : b % ntile;
  const int rest = order ? b % nsl : b / ntile;
  const int64_t o = rest / ncb;
  const int c0 = (rest % ncb) * 16;
  const double* sa = asrc + view_base(as, o) + c0;
  const double* sc = coef + view_base(cv, o) + c0;
  const int64_t asl = as.s_len, csl = cv.s_len;
  // every window in one burst: level-K approximation, then the details
  {
    const int BK = (t * T >> K) - G::c(K);
    const int am = (hK >> K) - 1;
    load_window<16, NT, 1>(lds + 16 * (IP ? 0 : (K & 1) ? G::buf1() : G::buf0()), sa, G::len(K),
                           true, 0,
                           inner, [&](int e) { return (int64_t)((BK + e) & am) * asl; });
  }
#pragma unroll
  for (int l = K - 1; l >= 0; --l) {
    const int half = hK >> (l + 1), hm = half - 1;
    const int B = (t * T >> (l + 1)) - G::c(l + 1);
    load_window<16, NT, 1>(lds + 16 * (IP ? G::ip_doff(l) : G::doff(l)), sc, G::len(l + 1), true,
                           0, inner, [&](int e) {
      return ((int64_t)half + ((B + e) & hm)) * csl;
    });
  }
  dma_fence_barrier();
  Rev16Level<L, NT, T, K, FMA, K - 1, IP>::run(tp, lds, t, dst + view_base(dv, o) + c0, dv.s_len);
}

}  // namespace jwv
