// aed_kernels.hpp — AncientEgyptianDecomposition's small sub-transforms in ONE
// launch (AncientEgyptianDecomposition.java:97-184).
//
// The reference splits an array of any length into power-of-two pieces
// (MathToolKit.decompose, largest first, MathToolKit.java:57-80) and runs the
// wrapped transform's full-depth forward / reverse on each.  Every piece that
// fits one workgroup's LDS (<= the resident cap) becomes one block of this
// varlen launch: block i transforms segment i (its own offset, length and
// level plan) with the same resident bodies as the batched kernels
// (fwt_fwd_res_blk, ..), so the results are bit-identical to separate calls.
// Larger pieces (HBM-bound) keep their own multi-pass plans.
#pragma once
#include "wpt_kernels.hpp"

namespace jwv {

// OP: 0 FWT forward, 1 FWT reverse, 2 WPT forward, 3 WPT reverse.  Contiguous
// 1-D segments, register-path loads (segment offsets may be odd).
template <int L, int NT, int CAP, bool FMA, int OP, typename TP>
__global__ __launch_bounds__(NT) void res_varlen(const double* __restrict__ src,
                                                 double* __restrict__ dst, VarSegs sg, TP tp) {
  const int i = blockIdx.x;
  AxisView v{};
  v.s_len = 1;
  v.pk = 1;
  const double* s = src + sg.off[i];
  double* y = dst + sg.off[i];
  if constexpr (OP == 0)
    fwt_fwd_res_blk<L, 1, NT, CAP, FMA>(s, v, y, v, sg.h0[i], sg.nlev[i], 0, 1, 0, tp);
  else if constexpr (OP == 1)
    fwt_rev_res_blk<L, 1, NT, CAP, FMA>(s, v, y, v, sg.h0[i], sg.nlev[i], 0, 1, 0, tp);
  else if constexpr (OP == 2)
    wpt_fwd_res_blk<L, 1, NT, CAP, FMA>(s, v, y, v, sg.n[i], sg.nlev[i], 0, 1, 0, tp);
  else
    wpt_rev_res_blk<L, 1, NT, CAP, FMA>(s, v, y, v, sg.n[i], sg.h0[i], sg.nlev[i], 0, 1, 0, tp);
}

}  // namespace jwv
