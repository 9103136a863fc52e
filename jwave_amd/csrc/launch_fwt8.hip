// launch_fwt8.hip — dispatch of the C = 8 column-slab tiles
// (fwt8_kernels.hpp) for one math mode (compiled twice).
#include "fwt16_kernels.hpp"
#include "fwt1_row.hpp"
#include "fwt_colres.hpp"
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
// ---- C = 8 column slabs (fwt8_kernels.hpp); tile rows = the generic C = 8
// tile the planner sizes grids and workspaces for
constexpr int kT8 = Geo::kFwtT8;
template <int L, int K>
hipError_t fwd8_k(const Bank& b, const TileArgs& a, hipStream_t s) {
  auto k = fwt_fwd_tile8<L, 256, kT8, K, kFMA>;
  const size_t lds = (size_t)Fwd8Geo<L, kT8, K>::lds_doubles() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  FwdTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = b.lo[j]; tp.hi[j] = b.hi[j]; }
  const dim3 grid((unsigned)(a.nouter * (a.inner / 8) * (a.h / kT8)));
  JWV_LAUNCH(k, grid, dim3(256), lds, s, a.src, a.sv, a.dst, a.dv, a.adst, a.av, a.h,
                     a.inner, tp, Geo::slab_order());
  return hipGetLastError();
}
template <int L, int K>
hipError_t rev8_k(const Bank& b, const TileArgs& a, hipStream_t s) {
  auto k = fwt_rev_tile8<L, 256, kT8, K, kFMA>;
  const size_t lds = (size_t)Rev8Geo<L, kT8, K>::lds_doubles() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  RevTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo_r[j] = b.lo_r[j]; tp.hi_r[j] = b.hi_r[j]; }
  const int hK = a.h << (a.K - 1);
  const dim3 grid((unsigned)(a.nouter * (a.inner / 8) * (hK / kT8)));
  JWV_LAUNCH(k, grid, dim3(256), lds, s, a.src, a.sv, a.coef, a.cv, a.dst, a.dv, hK,
                     a.inner, tp, Geo::slab_order());
  return hipGetLastError();
}
// ---- C = 16 column slabs (fwt16_kernels.hpp): whole 128-B row lines.
// Forward 512-row tiles (78 KB of LDS at L = 16: 2 blocks per CU), reverse
// 256-row tiles (every window in LDS: 61 KB).  Config 3 against the C = 8
// tiles (r04b, one box, two rounds): 1.368 / 1.371 -> 1.341 / 1.334 ms/step.
// r06 (profiles/r06/ab_col16_geometry.txt): forward blocks of 512 threads
// (4 waves per SIMD at 2 blocks per CU) -8.8 us per column pass against 256;
// 256-row tiles (3 blocks per CU, 38% halo) and 1024-row tiles (1 block of
// 1024 threads) slower.
constexpr int kT16F = 512, kT16R = 256, kNT16F = 512;
constexpr bool kRev16IP = true;  // Rev1Geo in-place layout: 61 -> 39 KB, 2 -> 4 blocks per CU
template <int L, int K>
hipError_t fwd16_k(const Bank& b, const TileArgs& a, hipStream_t s) {
  auto k = fwt_fwd_tile16<L, kNT16F, kT16F, K, kFMA>;
  const size_t lds = (size_t)Fwd16Geo<L, kT16F, K>::lds_doubles() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  FwdTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = b.lo[j]; tp.hi[j] = b.hi[j]; }
  const dim3 grid((unsigned)(a.nouter * (a.inner / 16) * (a.h / kT16F)));
  JWV_LAUNCH(k, grid, dim3(kNT16F), lds, s, a.src, a.sv, a.dst, a.dv, a.adst, a.av, a.h,
                     a.inner, tp, Geo::slab_order());
  return hipGetLastError();
}
template <int L, int K>
hipError_t rev16_k(const Bank& b, const TileArgs& a, hipStream_t s) {
  auto k = fwt_rev_tile16<L, 256, kT16R, K, kFMA, kRev16IP>;
  const size_t lds = (size_t)Rev16Geo<L, kT16R, K, kRev16IP>::lds_doubles() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  RevTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo_r[j] = b.lo_r[j]; tp.hi_r[j] = b.hi_r[j]; }
  const int hK = a.h << (a.K - 1);
  const dim3 grid((unsigned)(a.nouter * (a.inner / 16) * (hK / kT16R)));
  JWV_LAUNCH(k, grid, dim3(256), lds, s, a.src, a.sv, a.coef, a.cv, a.dst, a.dv, hK,
                     a.inner, tp, Geo::slab_order());
  return hipGetLastError();
}
template <int L>
hipError_t tile16_l(const Bank& b, const TileArgs& a, hipStream_t s, bool fwd) {
  switch (a.K) {
    case 1: return fwd ? fwd16_k<L, 1>(b, a, s) : rev16_k<L, 1>(b, a, s);
    case 2: return fwd ? fwd16_k<L, 2>(b, a, s) : rev16_k<L, 2>(b, a, s);
    default: return fwd ? fwd16_k<L, 3>(b, a, s) : rev16_k<L, 3>(b, a, s);
  }
}
template <int L>
hipError_t tile8_l(const Bank& b, const TileArgs& a, hipStream_t s, bool fwd) {
  if (a.inner % 16 == 0) {
    const int64_t hT = fwd ? (int64_t)a.h : ((int64_t)a.h << (a.K - 1));
    if (hT % (fwd ? kT16F : kT16R) == 0) return tile16_l<L>(b, a, s, fwd);
  }
  switch (a.K) {
    case 1: return fwd ? fwd8_k<L, 1>(b, a, s) : rev8_k<L, 1>(b, a, s);
    case 2: return fwd ? fwd8_k<L, 2>(b, a, s) : rev8_k<L, 2>(b, a, s);
    default: return fwd ? fwd8_k<L, 3>(b, a, s) : rev8_k<L, 3>(b, a, s);
  }
}

template <int L, int CW>
hipError_t res16_cw(const Bank& b, const ResArgs& a, hipStream_t s) {
  const int htop = a.n << (a.nlev - 1);
  const size_t lds = (size_t)CW * col16_stride(htop) * sizeof(double);
  const dim3 grid((unsigned)(a.nouter * (a.inner / CW)));
  auto k = fwt_rev_col16<L, kFMA, CW>;
  if (hipError_t e = prep1(k, lds)) return e;
  RevTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo_r[j] = b.lo_r[j]; tp.hi_r[j] = b.hi_r[j]; }
  JWV_LAUNCH(k, grid, dim3(64 * CW), lds, s, a.src, a.sv, a.dst, a.dv, a.n, a.nlev,
                     a.inner, tp);
  return hipGetLastError();
}
// forward column tails with compile-time geometry (fwt_colres.hpp); r06 A/B
// (profiles/r06/ab_col_tail_cres.txt): config 3 forward column tail 51.7 us
// (fwt_fwd_res) -> 46.7 (256 threads) / 45.5 us (512 threads)
constexpr int kCresH = 1024, kCresNT = 512;
template <int L>
hipError_t cres8_l(const Bank& b, const ResArgs& a, hipStream_t s) {
  auto k = fwt_fwd_cres8<L, kCresNT, kCresH, kFMA>;
  const size_t lds = (size_t)kCresH * kCresP * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  FwdTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = b.lo[j]; tp.hi[j] = b.hi[j]; }
  const dim3 grid((unsigned)(a.nouter * (a.inner / 8)));
  JWV_LAUNCH(k, grid, dim3(kCresNT), lds, s, a.src, a.sv, a.dst, a.dv, a.nlev, a.inner, tp);
  return hipGetLastError();
}
template <int L>
hipError_t rcres8_l(const Bank& b, const ResArgs& a, hipStream_t s) {
  auto k = fwt_rev_cres8<L, kCresNT, kCresH, kFMA>;
  const size_t lds = (size_t)kCresH * 8 * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  RevTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo_r[j] = b.lo_r[j]; tp.hi_r[j] = b.hi_r[j]; }
  const dim3 grid((unsigned)(a.nouter * (a.inner / 8)));
  JWV_LAUNCH(k, grid, dim3(kCresNT), lds, s, a.src, a.sv, a.dst, a.dv, a.n, a.inner, tp);
  return hipGetLastError();
}
template <int L>
hipError_t res16_l(const Bank& b, const ResArgs& a, hipStream_t s, bool fwd) {
  // the half-slab pairing is a bijection for whole groups of 16 blocks
  const bool half = (a.nouter * (a.inner / 8)) % 16 == 0;
  return half ? res16_cw<L, 8>(b, a, s) : res16_cw<L, 16>(b, a, s);
}
}  // namespace

namespace JWV_NS {
// Reverse resident tails of column passes with one wave per column
// (fwt1_row.hpp): XCD-paired half slabs, 16-B aligned row segments, a
// compiled-in tap count, at most kSmallH rows.  Config 3 reverse column tail
// 74-75 -> 60-61 us (r04h: 16-column blocks 69 us).  Tails of 1024 rows take
// the compile-time block-per-slab kernels (fwt_colres.hpp: forward r06
// 51.7 -> 45.5 us, reverse -5.8 us against the wave-per-column kernel, which
// keeps the other heights); other forward heights fall back to the generic
// fwt_fwd_res.
bool fwt_res16(const Bank& b, const ResArgs& a, hipStream_t s, bool fwd, hipError_t& err) {
  if (fwd) {
    // forward column tails of 1024 rows, 8-column slabs (config 3)
    if (!a.dma || a.inner % 8 || a.n != kCresH || a.nlev < 1 || a.nlev > 10 ||
        a.sv.pk != 1 || a.dv.pk != 1 || (a.sv.s_len & 1) || (a.dv.s_len & 1) ||
        (a.sv.s_outer & 1) || (a.dv.s_outer & 1) || (((uintptr_t)a.src | (uintptr_t)a.dst) & 15))
      return false;
    switch (b.L) {
      case 8: err = cres8_l<8>(b, a, s); return true;
      case 16: err = cres8_l<16>(b, a, s); return true;
      default: return false;
    }
  }
  if (!fwd && a.dma && b.scale == 1.0 && a.inner % 8 == 0 && a.n >= 2 &&
      a.nlev >= 1 && ((int64_t)a.n << (a.nlev - 1)) == kCresH && a.sv.pk == 1 && a.dv.pk == 1 &&
      !(a.sv.s_len & 1) && !(a.dv.s_len & 1) && !(a.sv.s_outer & 1) && !(a.dv.s_outer & 1) &&
      !(((uintptr_t)a.src | (uintptr_t)a.dst) & 15)) {
    // reverse column tails of 1024 rows, 8-column slabs (config 3)
    switch (b.L) {
      case 8: err = rcres8_l<8>(b, a, s); return true;
      case 16: err = rcres8_l<16>(b, a, s); return true;
      default: break;
    }
  }
  if (!a.dma || a.inner % kColW || a.nlev < 1 || a.sv.pk != 1 || a.dv.pk != 1) return false;
  if (!fwd && b.scale != 1.0) return false;
  if ((a.sv.s_len & 1) || (a.dv.s_len & 1) || (a.sv.s_outer & 1) || (a.dv.s_outer & 1) ||
      (((uintptr_t)a.src | (uintptr_t)a.dst) & 15))
    return false;
  const int64_t htop = fwd ? a.n : ((int64_t)a.n << (a.nlev - 1));
  if (htop > kSmallH || htop < 2) return false;
  switch (b.L) {
    case 2: err = res16_l<2>(b, a, s, fwd); return true;
    case 4: err = res16_l<4>(b, a, s, fwd); return true;
    case 8: err = res16_l<8>(b, a, s, fwd); return true;
    case 16: err = res16_l<16>(b, a, s, fwd); return true;
    default: return false;
  }
}
// C = 8 slabs: every row segment 16-B aligned (a.dma), whole slabs, a
// compiled-in tap count, at most Geo::kFwtK8 levels (the generic bound).
bool fwt_tile8(const Bank& b, const TileArgs& a, hipStream_t s, bool fwd, hipError_t& err) {
  if (!Geo::fwt8() || !a.dma || a.inner % 8 || a.K < 1 || a.K > 3 || a.K > Geo::kFwtK8)
    return false;
  if (!fwd && b.scale != 1.0) return false;
  const int64_t hT = fwd ? (int64_t)a.h : ((int64_t)a.h << (a.K - 1));
  if (hT < kT8 || hT % kT8) return false;
  switch (b.L) {
    case 2: err = tile8_l<2>(b, a, s, fwd); return true;
    case 4: err = tile8_l<4>(b, a, s, fwd); return true;
    case 8: err = tile8_l<8>(b, a, s, fwd); return true;
    case 16: err = tile8_l<16>(b, a, s, fwd); return true;
    default: return false;
  }
}
}  // namespace JWV_NS
}  // namespace jwv
