// launch_fwt1.hip — dispatch of the C = 1 compile-time-geometry FWT tile
// kernels (fwt1_kernels.hpp) for one math mode (compiled twice, like
// launch_fwt_wpt.hip).  Used for contiguous, 16-B aligned signals with a
// compiled-in tap count; every other case keeps the generic tile kernels.
#include "fwt1_kernels.hpp"
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

template <int L, int NT, int T, int K>
hipError_t fwd1_k(const Bank& b, const TileArgs& a, hipStream_t s) {
  auto k = fwt_fwd_tile1<L, NT, T, K, kFMA>;
  const size_t lds = (size_t)Fwd1Geo<L, T, K>::lds_doubles() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  FwdTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = b.lo[j]; tp.hi[j] = b.hi[j]; }
  const dim3 grid((unsigned)(a.nouter * (a.h / T)));
  hipLaunchKernelGGL(k, grid, dim3(NT), lds, s, a.src, a.sv.s_outer, a.dst, a.dv.s_outer, a.adst,
                     a.av.s_outer, a.h, tp);
  return hipGetLastError();
}
template <int L, int NT, int T>
hipError_t fwd1_t(const Bank& b, const TileArgs& a, hipStream_t s) {
  switch (a.K) {
    case 1: return fwd1_k<L, NT, T, 1>(b, a, s);
    case 2: return fwd1_k<L, NT, T, 2>(b, a, s);
    case 3: return fwd1_k<L, NT, T, 3>(b, a, s);
    case 4: return fwd1_k<L, NT, T, 4>(b, a, s);
    case 5: return fwd1_k<L, NT, T, 5>(b, a, s);
    default: return fwd1_k<L, NT, T, 6>(b, a, s);
  }
}
template <int L>
hipError_t fwd1_l(const Bank& b, const TileArgs& a, hipStream_t s) {
  if constexpr (L == 8) {  // geometry variants for tuning (env JWV_FWD1_T / JWV_FWD1_NT)
    if (Geo::fwd1_t() == 2048) return fwd1_t<L, 256, 2048>(b, a, s);
    if (Geo::fwd1_nt() == 512) return fwd1_t<L, 512, 4096>(b, a, s);
  }
  return fwd1_t<L, 256, 4096>(b, a, s);
}

template <int L, int NT, int T, int K>
hipError_t rev1_k(const Bank& b, const TileArgs& a, hipStream_t s) {
  auto k = fwt_rev_tile1<L, NT, T, K, kFMA>;
  const size_t lds = (size_t)Rev1Geo<L, T, K>::lds_doubles() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  RevTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo_r[j] = b.lo_r[j]; tp.hi_r[j] = b.hi_r[j]; }
  const int hK = a.h << (a.K - 1);
  const dim3 grid((unsigned)(a.nouter * (hK / T)));
  hipLaunchKernelGGL(k, grid, dim3(NT), lds, s, a.src, a.sv.s_outer, a.coef, a.cv.s_outer, a.dst,
                     a.dv.s_outer, hK, tp);
  return hipGetLastError();
}
template <int L, int NT, int T>
hipError_t rev1_t(const Bank& b, const TileArgs& a, hipStream_t s) {
  switch (a.K) {
    case 1: return rev1_k<L, NT, T, 1>(b, a, s);
    case 2: return rev1_k<L, NT, T, 2>(b, a, s);
    case 3: return rev1_k<L, NT, T, 3>(b, a, s);
    case 4: return rev1_k<L, NT, T, 4>(b, a, s);
    case 5: return rev1_k<L, NT, T, 5>(b, a, s);
    default: return rev1_k<L, NT, T, 6>(b, a, s);
  }
}
template <int L>
hipError_t rev1_l(const Bank& b, const TileArgs& a, hipStream_t s) {
  if constexpr (L == 8) {  // env JWV_REV1_T / JWV_REV1_NT
    if (Geo::rev1_t() == 4096) return rev1_t<L, 256, 4096>(b, a, s);
    if (Geo::rev1_nt() == 128) return rev1_t<L, 128, 2048>(b, a, s);
  }
  return rev1_t<L, 256, 2048>(b, a, s);
}

bool plain(const AxisView& v) { return v.pk == 1 && v.s_len == 1; }
bool even_rows(const AxisView& v, int64_t nouter) { return nouter == 1 || (v.s_outer & 1) == 0; }
}  // namespace

namespace JWV_NS {
// Returns false (and launches nothing) when the case is not covered.
bool fwt_fwd_tile1(const Bank& b, const TileArgs& a, hipStream_t s, hipError_t& err) {
  if (!Geo::fwt1() || !a.dma || a.inner != 1 || b.scale != 1.0) return false;
  if (!plain(a.sv) || !plain(a.dv) || !plain(a.av) || a.K < 1 || a.K > 6) return false;
  if (a.h % 4096) return false;
  switch (b.L) {
    case 2: err = fwd1_l<2>(b, a, s); return true;
    case 4: err = fwd1_l<4>(b, a, s); return true;
    case 8: err = fwd1_l<8>(b, a, s); return true;
    case 16: err = fwd1_l<16>(b, a, s); return true;
    default: return false;
  }
}
bool fwt_rev_tile1(const Bank& b, const TileArgs& a, hipStream_t s, hipError_t& err) {
  if (!Geo::fwt1() || !a.dma || a.inner != 1 || b.scale != 1.0) return false;
  if (!plain(a.sv) || !plain(a.cv) || !plain(a.dv) || a.K < 1 || a.K > 6) return false;
  if (((uintptr_t)a.dst & 15) || !even_rows(a.dv, a.nouter)) return false;
  if ((a.h << (a.K - 1)) % 4096) return false;
  switch (b.L) {
    case 2: err = rev1_l<2>(b, a, s); return true;
    case 4: err = rev1_l<4>(b, a, s); return true;
    case 8: err = rev1_l<8>(b, a, s); return true;
    case 16: err = rev1_l<16>(b, a, s); return true;
    default: return false;
  }
}
}  // namespace JWV_NS
}  // namespace jwv
