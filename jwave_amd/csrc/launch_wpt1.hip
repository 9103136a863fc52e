// launch_wpt1.hip — dispatch of the C = 1 compile-time-geometry WPT tiles
// (wpt1_kernels.hpp) for one math mode (compiled twice).
#include "wpt1_kernels.hpp"
#include "jwv_launch.hpp"

#ifndef JWV_FMA
#error "JWV_FMA must be 0 or 1"
#endif
#if JWV_FMA
#define JWV_NS fused
#else
#define JWV_NS exact
#endif

namespace jwv {
namespace {
constexpr bool kFMA = JWV_FMA != 0;

template <typename Kern>
hipError_t prep1(Kern kernel, size_t lds) {
  if (lds > 65536)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  return hipSuccess;
}
// ---- WPT
constexpr int kWptT = Geo::kWpt1T;
template <int L, int K>
hipError_t wfwd1_k(const Bank& b, const TileArgs& a, hipStream_t s) {
  auto k = wpt_fwd_tile1<L, 256, kWptT, K, kFMA>;
  const size_t lds = (size_t)Wpt1FwdGeo<L, kWptT, K>::lds_doubles() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  FwdTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = b.lo[j]; tp.hi[j] = b.hi[j]; }
  const dim3 grid((unsigned)(a.nouter * (a.h / kWptT)));
  JWV_LAUNCH(k, grid, dim3(256), lds, s, a.src, a.sv, a.dst, a.dv, a.h, tp);
  return hipGetLastError();
}
// The reverse tiles' couples as four interleaved sums (rev_couple_ilv) for
// L >= 8: config 4 reverse 2728-2752 -> 2702-2708 us.
template <int L, int K>
hipError_t wrev1_k(const Bank& b, const TileArgs& a, hipStream_t s) {
  constexpr bool ILV = L >= 8;
  auto k = wpt_rev_tile1<L, 256, kWptT, K, kFMA, ILV>;
  const size_t lds = (size_t)Wpt1RevGeo<L, kWptT, K>::lds_doubles() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  RevTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo_r[j] = b.lo_r[j]; tp.hi_r[j] = b.hi_r[j]; }
  const dim3 grid((unsigned)(a.nouter * (a.h / kWptT)));
  JWV_LAUNCH(k, grid, dim3(256), lds, s, a.src, a.sv, a.dst, a.dv, a.h, tp);
  return hipGetLastError();
}
// 8192-sample forward WPT tiles, 512 threads: half the halo recompute of the
// 4096 tile (14.7% -> 7.4% extra pairs) at the same waves per CU.  Config 4
// forward 2597 -> 2468 us; the reverse (halo ~7% at 4096) measured no gain
// and keeps 4096.  Levels in trio form (wpt_fwd_tile3, r06: EXACT forward
// -0.7%, FMA forward -4.3%, profiles/r06/ab_trio_wpt_fwt.txt).
template <int L>
hipError_t wpt8k_fwd(const Bank& b, const TileArgs& a, hipStream_t s) {
  constexpr int TT = 8192, K = 6;
  const dim3 grid((unsigned)(a.nouter * (a.h / TT)));
  auto k = wpt_fwd_tile3<L, 512, TT, K, kFMA>;
  const size_t lds = (size_t)Wpt3FwdGeo<L, TT, K>::lds_doubles() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  FwdTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = b.lo[j]; tp.hi[j] = b.hi[j]; }
  JWV_LAUNCH(k, grid, dim3(512), lds, s, a.src, a.sv, a.dst, a.dv, a.h, tp);
  return hipGetLastError();
}
template <int L>
hipError_t wpt1_l(const Bank& b, const TileArgs& a, hipStream_t s, bool fwd) {
  if (fwd && a.K == 6 && a.h % 8192 == 0) return wpt8k_fwd<L>(b, a, s);
  switch (a.K) {
    case 1: return fwd ? wfwd1_k<L, 1>(b, a, s) : wrev1_k<L, 1>(b, a, s);
    case 2: return fwd ? wfwd1_k<L, 2>(b, a, s) : wrev1_k<L, 2>(b, a, s);
    case 3: return fwd ? wfwd1_k<L, 3>(b, a, s) : wrev1_k<L, 3>(b, a, s);
    case 4: return fwd ? wfwd1_k<L, 4>(b, a, s) : wrev1_k<L, 4>(b, a, s);
    case 5: return fwd ? wfwd1_k<L, 5>(b, a, s) : wrev1_k<L, 5>(b, a, s);
    default: return fwd ? wfwd1_k<L, 6>(b, a, s) : wrev1_k<L, 6>(b, a, s);
  }
}

// packet views: stride-1 samples, even strides (16-B aligned packet rows)
bool pk_ok(const AxisView& v) {
  return v.s_len == 1 && (v.s_outer & 1) == 0 && (v.pk == 1 || (v.s_pk & 1) == 0);
}
}  // namespace

namespace JWV_NS {
bool wpt_tile1(const Bank& b, const TileArgs& a, hipStream_t s, bool fwd, hipError_t& err) {
  if (!Geo::fwt1() || !a.dma || a.inner != 1 || (!fwd && b.scale != 1.0)) return false;
  if (!pk_ok(a.sv) || !pk_ok(a.dv) || a.K < 1 || a.K > Geo::kWpt1KMax) return false;
  if (((uintptr_t)a.dst & 15) || ((uintptr_t)a.src & 15) || a.h < kWptT || a.h % kWptT) return false;
  switch (b.L) {
    case 2: err = wpt1_l<2>(b, a, s, fwd); return true;
    case 4: err = wpt1_l<4>(b, a, s, fwd); return true;
    case 8: err = wpt1_l<8>(b, a, s, fwd); return true;
    case 16: err = wpt1_l<16>(b, a, s, fwd); return true;
    default: return false;
  }
}
}  // namespace JWV_NS
}  // namespace jwv
