// launch_fwt1.hip — dispatch of the C = 1 compile-time-geometry FWT kernels
// (tiles fwt1_kernels.hpp, resident fwt1_res.hpp, wave-per-row fwt1_row.hpp)
// for one math mode (compiled twice, like launch_fwt_wpt.hip; the WPT and
// column-slab tiles live in launch_wpt1.hip / launch_fwt8.hip).  Used for contiguous, 16-B aligned signals with a
// compiled-in tap count; every other case keeps the generic tile kernels.
#include "fwt1_kernels.hpp"
#include <cstdlib>
#include "fwt1_res.hpp"
#include "fwt1_row.hpp"
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
constexpr int kFwdT = Geo::kFwt1T, kRevT = Geo::kRev1T;

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
  JWV_LAUNCH(k, grid, dim3(NT), lds, s, a.src, a.sv.s_outer, a.dst, a.dv.s_outer, a.adst,
                     a.av.s_outer, a.h, tp, a.sp, a.lsw, a.ss);
  return hipGetLastError();
}
template <int L>
hipError_t fwd1_l(const Bank& b, const TileArgs& a, hipStream_t s) {
  constexpr int NT = 256, T = kFwdT;
  if (a.t1 == 1024) {  // first pass of a long signal (Geo::fwd1_first_t)
    switch (a.K) {
      case 4: return fwd1_k<L, NT, 1024, 4>(b, a, s);
      case 5: return fwd1_k<L, NT, 1024, 5>(b, a, s);
      case 6: return fwd1_k<L, NT, 1024, 6>(b, a, s);
      default: return hipErrorInvalidValue;
    }
  }
  switch (a.K) {
    case 1: return fwd1_k<L, NT, T, 1>(b, a, s);
    case 2: return fwd1_k<L, NT, T, 2>(b, a, s);
    case 3: return fwd1_k<L, NT, T, 3>(b, a, s);
    case 4: return fwd1_k<L, NT, T, 4>(b, a, s);
    case 5: return fwd1_k<L, NT, T, 5>(b, a, s);
    case 6: return fwd1_k<L, NT, T, 6>(b, a, s);
    // deep passes (latency-bound, few blocks): 512 threads halve the pair
    // slots of the wide levels (config 2: 0.6 us per call)
    case 7: return fwd1_k<L, 512, T, 7>(b, a, s);
    case 8: return fwd1_k<L, 512, T, 8>(b, a, s);
    default: return fwd1_k<L, 512, T, 9>(b, a, s);
  }
}

template <int L, int NT, int T, int K>
hipError_t rev1_k(const Bank& b, const TileArgs& a, hipStream_t s) {
  constexpr bool IP = true;  // Rev1Geo in-place layout (r04s: rev tiles 269 -> 247 us, config 3)
  auto k = fwt_rev_tile1<L, NT, T, K, kFMA, IP>;
  const size_t lds = (size_t)rev1_lds_doubles<L, T, K, IP>() * sizeof(double);
  if (hipError_t e = prep1(k, lds)) return e;
  RevTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo_r[j] = b.lo_r[j]; tp.hi_r[j] = b.hi_r[j]; }
  const int hK = a.h << (a.K - 1);
  const dim3 grid((unsigned)(a.nouter * (hK / T)));
  JWV_LAUNCH(k, grid, dim3(NT), lds, s, a.src, a.sv.s_outer, a.coef, a.cv.s_outer, a.dst,
                     a.dv.s_outer, hK, tp, a.sp, a.lsw, a.ss);
  return hipGetLastError();
}
template <int L>
hipError_t rev1_l(const Bank& b, const TileArgs& a, hipStream_t s) {
  constexpr int NT = 256, T = kRevT;
  switch (a.K) {
    case 1: return rev1_k<L, NT, T, 1>(b, a, s);
    case 2: return rev1_k<L, NT, T, 2>(b, a, s);
    case 3: return rev1_k<L, NT, T, 3>(b, a, s);
    case 4: return rev1_k<L, NT, T, 4>(b, a, s);
    case 5: return rev1_k<L, NT, T, 5>(b, a, s);
    case 6: return rev1_k<L, NT, T, 6>(b, a, s);
    case 7: return rev1_k<L, NT, T, 7>(b, a, s);
    case 8: return rev1_k<L, NT, T, 8>(b, a, s);
    default: return rev1_k<L, NT, T, 9>(b, a, s);
  }
}

// resident kernels for a handful of rows (latency-bound tail): 1024 threads;
// many short rows (the tail under the C = 1 row tile passes): 256 threads,
// slot loops sized for kRowCap
constexpr int kCap = Geo::kResCap1;
constexpr int kRowCap = 1024;
template <int L, int NTX, int CAPX>
hipError_t fwd_res1_l(const Bank& b, const ResArgs& a, hipStream_t s) {
  FwdTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = b.lo[j]; tp.hi[j] = b.hi[j]; }
  const size_t lds = (size_t)(a.n + 2) * sizeof(double);
  const dim3 grid((unsigned)a.nouter);
  auto k = fwt_fwd_res1<L, NTX, CAPX, kFMA>;
  if (hipError_t e = prep1(k, lds)) return e;
  JWV_LAUNCH(k, grid, dim3(NTX), lds, s, a.src, a.sv.s_outer, a.dst, a.dv.s_outer, a.n,
                     a.nlev, tp);
  return hipGetLastError();
}
template <int L, int NTX, int CAPX>
hipError_t rev_res1_l(const Bank& b, const ResArgs& a, hipStream_t s) {
  RevTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo_r[j] = b.lo_r[j]; tp.hi_r[j] = b.hi_r[j]; }
  const int htop = a.nlev > 0 ? (a.n << (a.nlev - 1)) : a.n;
  const size_t lds = (size_t)(htop + 2) * sizeof(double);
  const dim3 grid((unsigned)a.nouter);
  auto k = fwt_rev_res1<L, NTX, CAPX, kFMA>;
  if (hipError_t e = prep1(k, lds)) return e;
  JWV_LAUNCH(k, grid, dim3(NTX), lds, s, a.src, a.sv.s_outer, a.dst, a.dv.s_outer, a.n,
                     a.nlev, tp);
  return hipGetLastError();
}

bool plain(const AxisView& v) { return v.pk == 1 && v.s_len == 1; }
// packet views: stride-1 samples, even strides (16-B aligned packet rows)
bool pk_ok(const AxisView& v) {
  return v.s_len == 1 && (v.s_outer & 1) == 0 && (v.pk == 1 || (v.s_pk & 1) == 0);
}
bool even_rows(const AxisView& v, int64_t nouter) { return nouter == 1 || (v.s_outer & 1) == 0; }
}  // namespace

namespace JWV_NS {
// Returns false (and launches nothing) when the case is not covered.
bool fwt_fwd_tile1(const Bank& b, const TileArgs& a, hipStream_t s, hipError_t& err) {
  if (!Geo::fwt1() || !a.dma || a.inner != 1) return false;  // (scale: synthesis only)
  if (!plain(a.sv) || !plain(a.dv) || !plain(a.av) || a.K < 1 || a.K > Geo::kFwt1KMax) return false;
  if (((uintptr_t)a.dst & 15) || ((uintptr_t)a.adst & 15) || !even_rows(a.dv, a.nouter) ||
      !even_rows(a.av, a.nouter))
    return false;
  if (a.t1 != 0 && (a.t1 != 1024 || a.K < 4 || a.K > 6)) return false;
  if (a.h % (a.t1 ? a.t1 : kFwdT)) return false;
  switch (b.L) {
    case 2: err = fwd1_l<2>(b, a, s); return true;
    case 4: err = fwd1_l<4>(b, a, s); return true;
    case 8: err = fwd1_l<8>(b, a, s); return true;
    case 16: err = fwd1_l<16>(b, a, s); return true;
    default: return false;
  }
}
// A handful of signals (the latency-bound tail of long 1-D signals): 1024
// threads; batches of rows up to kRowCap: 256 threads (res1_rows).
// Batches of short rows (<= kRowCap) also take the compiled-in kernels with
// 256 threads.  Config 3 row tails:
// fwd 51 -> 41 us, rev ~100 -> 90 us.
bool res1_rows() { return true; }
// Batches of >= 64 rows up to kSmallH samples (the row passes' resident
// tails, config 3): one wave per row (fwt1_row.hpp) instead of the
// block-per-row kernels above.  Config 3 tails (8192 rows, one box):
// forward 45.8 -> 40.1 us, reverse 79.0 -> 73.9 us.
bool small1() { return true; }
template <int L>
hipError_t fwd_small1_l(const Bank& b, const ResArgs& a, hipStream_t s) {
  FwdTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = b.lo[j]; tp.hi[j] = b.hi[j]; }
  auto k = fwt_fwd_small1<L, kFMA>;
  JWV_LAUNCH(k, dim3((unsigned)((a.nouter + kSmallRows - 1) / kSmallRows)),
                     dim3(64 * kSmallRows), 0, s, a.src, a.sv.s_outer, a.dst, a.dv.s_outer, a.n,
                     a.nlev, a.nouter, tp);
  return hipGetLastError();
}
template <int L>
hipError_t rev_small1_l(const Bank& b, const ResArgs& a, hipStream_t s) {
  RevTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo_r[j] = b.lo_r[j]; tp.hi_r[j] = b.hi_r[j]; }
  auto k = fwt_rev_small1<L, kFMA>;
  JWV_LAUNCH(k, dim3((unsigned)((a.nouter + kSmallRows - 1) / kSmallRows)),
                     dim3(64 * kSmallRows), 0, s, a.src, a.sv.s_outer, a.dst, a.dv.s_outer, a.n,
                     a.nlev, a.nouter, tp);
  return hipGetLastError();
}
// rows the wave-per-row kernels take (level input n / reverse top htop)
bool small1_case(const ResArgs& a, int64_t htop) {
  return small1() && a.nouter >= 64 && htop <= kSmallH && a.nlev >= 1;
}

template <int L>
hipError_t fwd_res1_pick(const Bank& b, const ResArgs& a, hipStream_t s) {
  if (small1_case(a, a.n)) return fwd_small1_l<L>(b, a, s);
  if (a.nouter >= 64) return fwd_res1_l<L, 256, kRowCap>(b, a, s);
  return fwd_res1_l<L, 1024, kCap>(b, a, s);
}
template <int L>
hipError_t rev_res1_pick(const Bank& b, const ResArgs& a, hipStream_t s) {
  if (a.nlev > 0 && small1_case(a, (int64_t)a.n << (a.nlev - 1))) return rev_small1_l<L>(b, a, s);
  if (a.nouter >= 64) return rev_res1_l<L, 256, kRowCap>(b, a, s);
  return rev_res1_l<L, 1024, kCap>(b, a, s);
}
bool fwt_fwd_res1(const Bank& b, const ResArgs& a, hipStream_t s, hipError_t& err) {
  if (!Geo::fwt1() || !a.dma || a.inner != 1 || !plain(a.sv) || !plain(a.dv)) return false;
  if (a.nouter >= 64 && !(res1_rows() && a.n <= kRowCap)) return false;
  if (a.n > kCap || a.n < 2) return false;
  switch (b.L) {
    case 2: err = fwd_res1_pick<2>(b, a, s); return true;
    case 4: err = fwd_res1_pick<4>(b, a, s); return true;
    case 8: err = fwd_res1_pick<8>(b, a, s); return true;
    case 16: err = fwd_res1_pick<16>(b, a, s); return true;
    default: return false;
  }
}
bool fwt_rev_res1(const Bank& b, const ResArgs& a, hipStream_t s, hipError_t& err) {
  if (!Geo::fwt1() || !a.dma || a.inner != 1 || b.scale != 1.0) return false;
  if (!plain(a.sv) || !plain(a.dv)) return false;
  if (((uintptr_t)a.dst & 15) || !even_rows(a.dv, a.nouter)) return false;
  const int64_t htop = a.nlev > 0 ? ((int64_t)a.n << (a.nlev - 1)) : a.n;
  if (a.nouter >= 64 && !(res1_rows() && htop <= kRowCap)) return false;
  if (htop > kCap || htop < 2) return false;
  switch (b.L) {
    case 2: err = rev_res1_pick<2>(b, a, s); return true;
    case 4: err = rev_res1_pick<4>(b, a, s); return true;
    case 8: err = rev_res1_pick<8>(b, a, s); return true;
    case 16: err = rev_res1_pick<16>(b, a, s); return true;
    default: return false;
  }
}
bool fwt_rev_tile1(const Bank& b, const TileArgs& a, hipStream_t s, hipError_t& err) {
  if (!Geo::fwt1() || !a.dma || a.inner != 1 || b.scale != 1.0) return false;
  if (!plain(a.sv) || !plain(a.cv) || !plain(a.dv) || a.K < 1 || a.K > Geo::kFwt1KMax) return false;
  if (((uintptr_t)a.dst & 15) || !even_rows(a.dv, a.nouter)) return false;
  if ((a.h << (a.K - 1)) % kRevT) return false;
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
