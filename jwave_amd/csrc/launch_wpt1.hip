// launch_wpt1.hip — dispatch of the C = 1 compile-time-geometry WPT tiles
// (wpt1_kernels.hpp) for one math mode (compiled twice).
#include "wpt1_kernels.hpp"
#include "wpt_stream.hpp"

#include <cstdlib>
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
  hipLaunchKernelGGL(k, grid, dim3(256), lds, s, a.src, a.sv, a.dst, a.dv, a.h, tp);
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
  hipLaunchKernelGGL(k, grid, dim3(256), lds, s, a.src, a.sv, a.dst, a.dv, a.h, tp);
  return hipGetLastError();
}
// 8192-sample forward WPT tiles, 512 threads: half the halo recompute of the
// 4096 tile (14.7% -> 7.4% extra pairs) at the same waves per CU.  Config 4
// forward 2597 -> 2468 us; the reverse (halo ~7% at 4096) measured no gain
// and keeps 4096.
template <int L>
hipError_t wpt8k_fwd(const Bank& b, const TileArgs& a, hipStream_t s) {
  constexpr int TT = 8192, K = 6;
  const dim3 grid((unsigned)(a.nouter * (a.h / TT)));
  auto k = wpt_fwd_tile1<L, 512, TT, K, kFMA>;
  const size_t lds = (size_t)Wpt1FwdGeo<L, TT, K>::lds_doubles() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  FwdTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = b.lo[j]; tp.hi[j] = b.hi[j]; }
  hipLaunchKernelGGL(k, grid, dim3(512), lds, s, a.src, a.sv, a.dst, a.dv, a.h, tp);
  return hipGetLastError();
}
// Streamed forward (wpt_stream.hpp): runs of tiles per resident block with
// carried halos.  env JWV_WPT_FSTREAM=1 (256 x 2048), 2 (512 x 2048),
// 3 (256 x 4096) (A/B this round).
int wfstream_env() {
  static const int v = [] {
    const char* e = std::getenv("JWV_WPT_FSTREAM");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}
int cu_count() {
  static const int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
    return n;
  }();
  return v;
}
template <int L, int NT, int T>
hipError_t wfs_k(const Bank& b, const TileArgs& a, hipStream_t s) {
  constexpr int K = 6;
  using G = WptFStreamGeo<L, T, K>;
  auto k = wpt_fwd_stream<L, NT, T, K, kFMA>;
  const size_t lds = (size_t)G::lds_doubles() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  int per = 0;
  if (hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, NT, lds)) return e;
  if (per < 1) per = 1;
  const int64_t ntile = a.nouter * (a.h / T);
  int64_t nb = (int64_t)per * cu_count();
  if (nb > ntile) nb = ntile;
  WptStreamArgs<FwdTaps<L>> args{a.src, a.sv, a.dst, a.dv, ntile, a.h, 0, {}};
  for (int j = 0; j < L; ++j) { args.tp.lo[j] = b.lo[j]; args.tp.hi[j] = b.hi[j]; }
  hipLaunchKernelGGL(k, dim3((unsigned)nb), dim3(NT), lds, s, args);
  return hipGetLastError();
}
template <int L>
bool wpt_fstream(const Bank& b, const TileArgs& a, hipStream_t s, hipError_t& err) {
  if constexpr (L != 16) {
    return false;
  } else {
    const int v = wfstream_env();
    // contiguous rows of whole packets (pk == 1), 6 levels, rows fit int offsets
    if (!v || a.K != 6 || a.sv.pk != 1 || a.dv.pk != 1 || a.h % 4096 || a.h < 8192 ||
        (int64_t)a.h * 8 >= (int64_t(1) << 31))
      return false;
    if (v == 1) err = wfs_k<L, 256, 2048>(b, a, s);
    else if (v == 2) err = wfs_k<L, 512, 2048>(b, a, s);
    else err = wfs_k<L, 256, 4096>(b, a, s);
    return true;
  }
}
// Streamed reverse (wpt_stream.hpp).  env JWV_WPT_RSTREAM=1 (256 x 2048),
// 2 (512 x 2048), 3 (256 x 4096) (A/B this round).
int wrstream_env() {
  static const int v = [] {
    const char* e = std::getenv("JWV_WPT_RSTREAM");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}
template <int L, int NT, int T>
hipError_t wrs_k(const Bank& b, const TileArgs& a, hipStream_t s) {
  constexpr int K = 6;
  using G = WptRStreamGeo<L, T, K>;
  auto k = wpt_rev_stream<L, NT, T, K, kFMA>;
  const size_t lds = (size_t)G::lds_doubles() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  int per = 0;
  if (hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, NT, lds)) return e;
  if (per < 1) per = 1;
  const int64_t ntile = a.nouter * (a.h / T);
  int64_t nb = (int64_t)per * cu_count();
  if (nb > ntile) nb = ntile;
  WptStreamArgs<RevTaps<L>> args{a.src, a.sv, a.dst, a.dv, ntile, a.h, 0, {}};
  for (int j = 0; j < L; ++j) { args.tp.lo_r[j] = b.lo_r[j]; args.tp.hi_r[j] = b.hi_r[j]; }
  hipLaunchKernelGGL(k, dim3((unsigned)nb), dim3(NT), lds, s, args);
  return hipGetLastError();
}
template <int L>
bool wpt_rstream(const Bank& b, const TileArgs& a, hipStream_t s, hipError_t& err) {
  if constexpr (L != 16) {
    return false;
  } else {
    const int v = wrstream_env();
    if (!v || a.K != 6 || a.sv.pk != 1 || a.dv.pk != 1 || a.h % 4096 || a.h < 8192 ||
        (int64_t)a.h * 8 >= (int64_t(1) << 31))
      return false;
    if (v == 1) err = wrs_k<L, 256, 2048>(b, a, s);
    else if (v == 2) err = wrs_k<L, 512, 2048>(b, a, s);
    else err = wrs_k<L, 256, 4096>(b, a, s);
    return true;
  }
}
template <int L>
hipError_t wpt1_l(const Bank& b, const TileArgs& a, hipStream_t s, bool fwd) {
  {
    hipError_t e = hipSuccess;
    if (fwd ? wpt_fstream<L>(b, a, s, e) : wpt_rstream<L>(b, a, s, e)) return e;
  }
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
