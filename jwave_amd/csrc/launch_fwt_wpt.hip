// launch_fwt_wpt.hip — instantiates the FWT / WPT kernels for one math mode.
// Compiled twice: -DJWV_FMA=0 (namespace jwv::exact) and -DJWV_FMA=1
// (namespace jwv::fused).  Grid/LDS geometry comes from jwv::Geo.
#include "jwv_launch.hpp"
#include "aed_kernels.hpp"
#include <type_traits>

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
constexpr int NT = Geo::NT;

template <int L>
FwdTaps<L> fwd_taps_s(const Bank& b) {
  FwdTaps<L> t;
  for (int j = 0; j < L; ++j) { t.lo[j] = b.lo[j]; t.hi[j] = b.hi[j]; }
  return t;
}
template <int L>
RevTaps<L> rev_taps_s(const Bank& b) {
  RevTaps<L> t;
  for (int j = 0; j < L; ++j) { t.lo_r[j] = b.lo_r[j]; t.hi_r[j] = b.hi_r[j]; }
  return t;
}
AnyTaps any_taps(const Bank& b) {
  AnyTaps t{};
  for (int j = 0; j < b.L; ++j) {
    t.lo[j] = b.lo[j]; t.hi[j] = b.hi[j]; t.lo_r[j] = b.lo_r[j]; t.hi_r[j] = b.hi_r[j];
  }
  t.scale = b.scale;
  t.L = b.L;
  return t;
}
template <int L>
typename FB<L>::Fwd fwd_taps(const Bank& b) {
  if constexpr (L == 0) return any_taps(b); else return fwd_taps_s<L>(b);
}
template <int L>
typename FB<L>::Rev rev_taps(const Bank& b) {
  if constexpr (L == 0) return any_taps(b); else return rev_taps_s<L>(b);
}

template <typename K>
hipError_t prep(K kernel, size_t lds) {
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <int C> constexpr int cap() { return C == 1 ? Geo::kResCap1 : Geo::kResCap8; }
template <int C> constexpr int fwt_T() { return C == 1 ? Geo::kFwtT1 : Geo::kFwtT8; }
template <int C> constexpr int fwt_K() { return C == 1 ? Geo::kFwtK1 : Geo::kFwtK8; }
template <int C> constexpr int wpt_T() { return C == 1 ? Geo::kWptT1 : Geo::kWptT8; }
template <int C> constexpr int wpt_K() { return C == 1 ? Geo::kWptK1 : Geo::kWptK8; }
inline unsigned ncb(int inner, int C) { return (unsigned)((inner + C - 1) / C); }

// ------------------------------------------------------------- FWT
// A single-signal tail (few blocks) is latency-bound: give it 1024 threads.
constexpr int kBigNT = 1024;
inline bool few_blocks(const ResArgs& a, int C) { return C == 1 && a.nouter * ncb(a.inner, C) < 64; }

// Short rows of a batch (the resident tail under the C = 1 row tile passes)
// take a CAP = kShortCap instantiation: its slot loops are sized for the row,
// not for 8192 elements (config 3 row tails: ~4x faster).
constexpr int kShortCap = 1024;

template <int L, int C, int NTX, int CAPX = cap<C>()>
hipError_t fwt_fwd_res_nt(const Bank& b, const ResArgs& a, hipStream_t s) {
  auto k = fwt_fwd_res<L, C, NTX, CAPX, kFMA>;
  const size_t lds = (size_t)(a.n + 2) * C * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)(a.nouter * ncb(a.inner, C)));
  JWV_LAUNCH(k, grid, dim3(NTX), lds, s, a.src, a.sv, a.dst, a.dv, a.n, a.nlev, a.inner,
                     a.dma, fwd_taps<L>(b));
  return hipGetLastError();
}
template <int L, int C>
hipError_t fwt_fwd_res_go(const Bank& b, const ResArgs& a, hipStream_t s) {
  if constexpr (C == 1) {
    if (few_blocks(a, C)) return fwt_fwd_res_nt<L, C, kBigNT>(b, a, s);
    if (a.n <= kShortCap) return fwt_fwd_res_nt<L, C, NT, kShortCap>(b, a, s);
  }
  return fwt_fwd_res_nt<L, C, NT>(b, a, s);
}
template <int L, int C, int NTX, int CAPX = cap<C>()>
hipError_t fwt_rev_res_nt(const Bank& b, const ResArgs& a, hipStream_t s) {
  auto k = fwt_rev_res<L, C, NTX, CAPX, kFMA>;
  const int htop = a.nlev > 0 ? (a.n << (a.nlev - 1)) : a.n;
  const size_t lds = (size_t)(htop + 2) * C * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)(a.nouter * ncb(a.inner, C)));
  JWV_LAUNCH(k, grid, dim3(NTX), lds, s, a.src, a.sv, a.dst, a.dv, a.n, a.nlev, a.inner,
                     a.dma, rev_taps<L>(b));
  return hipGetLastError();
}
template <int L, int C>
hipError_t fwt_rev_res_go(const Bank& b, const ResArgs& a, hipStream_t s) {
  if constexpr (C == 1) {
    if (few_blocks(a, C)) return fwt_rev_res_nt<L, C, kBigNT>(b, a, s);
    const int htop = a.nlev > 0 ? (a.n << (a.nlev - 1)) : a.n;
    if (htop <= kShortCap) return fwt_rev_res_nt<L, C, NT, kShortCap>(b, a, s);
  }
  return fwt_rev_res_nt<L, C, NT>(b, a, s);
}
template <int L, int C, int T>
hipError_t fwt_fwd_tile_t(const Bank& b, const TileArgs& a, hipStream_t s) {
  constexpr int KM = fwt_K<C>();
  auto k = fwt_fwd_tile<L, C, NT, T, KM, kFMA>;
  const int m0 = T + (b.L - 2) * ((1 << a.K) - 1);
  const size_t lds = (size_t)(m0 + 2) * C * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)(a.nouter * ncb(a.inner, C) * (a.h / T)));
  JWV_LAUNCH(k, grid, dim3(NT), lds, s, a.src, a.sv, a.dst, a.dv, a.adst, a.av, a.h, a.K,
                     a.inner, a.dma, fwd_taps<L>(b));
  return hipGetLastError();
}
template <int L, int C>
hipError_t fwt_fwd_tile_go(const Bank& b, const TileArgs& a, hipStream_t s) {
  return fwt_fwd_tile_t<L, C, fwt_T<C>()>(b, a, s);
}
template <int L, int C, int T, bool PREF>
hipError_t fwt_rev_tile_t(const Bank& b, const TileArgs& a, hipStream_t s) {
  constexpr int KM = fwt_K<C>();
  constexpr int QM = (LMax<L>::v + 1) / 2;
  auto k = fwt_rev_tile<L, C, NT, T, KM, kFMA, PREF>;
  const size_t lds = (size_t)((T / 2 + 2 * QM + 4) +
                              (PREF ? (T + a.K * (2 * QM + 4)) : (T / 2 + 2 * QM + 4))) *
                     C * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const int hK = a.h << (a.K - 1);
  const dim3 grid((unsigned)(a.nouter * ncb(a.inner, C) * (hK / T)));
  JWV_LAUNCH(k, grid, dim3(NT), lds, s, a.src, a.sv, a.coef, a.cv, a.dst, a.dv, a.h, a.K,
                     a.inner, a.dma, rev_taps<L>(b));
  return hipGetLastError();
}
template <int L, int C>
hipError_t fwt_rev_tile_go(const Bank& b, const TileArgs& a, hipStream_t s) {
  return fwt_rev_tile_t<L, C, fwt_T<C>(), false>(b, a, s);
}

// ------------------------------------------------------------- WPT
template <int L, int C>
hipError_t wpt_fwd_res_go(const Bank& b, const ResArgs& a, hipStream_t s) {
  auto k = wpt_fwd_res<L, C, NT, cap<C>(), kFMA>;
  const size_t lds = (size_t)(a.n + 2) * C * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)(a.nouter * ncb(a.inner, C)));
  JWV_LAUNCH(k, grid, dim3(NT), lds, s, a.src, a.sv, a.dst, a.dv, a.n, a.nlev, a.inner,
                     a.dma, fwd_taps<L>(b));
  return hipGetLastError();
}
template <int L, int C>
hipError_t wpt_rev_res_go(const Bank& b, const ResArgs& a, hipStream_t s) {
  auto k = wpt_rev_res<L, C, NT, cap<C>(), kFMA>;
  const size_t lds = (size_t)(a.n + 2) * C * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)(a.nouter * ncb(a.inner, C)));
  JWV_LAUNCH(k, grid, dim3(NT), lds, s, a.src, a.sv, a.dst, a.dv, a.n, a.h0, a.nlev,
                     a.inner, a.dma, rev_taps<L>(b));
  return hipGetLastError();
}
template <int L, int C>
hipError_t wpt_fwd_tile_go(const Bank& b, const TileArgs& a, hipStream_t s) {
  constexpr int T = wpt_T<C>(), KM = wpt_K<C>();
  auto k = wpt_fwd_tile<L, C, NT, T, KM, kFMA>;
  const int m0 = T + (b.L - 2) * ((1 << a.K) - 1);
  const size_t lds = (size_t)(m0 + 2) * C * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)(a.nouter * ncb(a.inner, C) * (a.h / T)));
  JWV_LAUNCH(k, grid, dim3(NT), lds, s, a.src, a.sv, a.dst, a.dv, a.h, a.K, a.inner,
                     a.dma, fwd_taps<L>(b));
  return hipGetLastError();
}
template <int L, int C>
hipError_t wpt_rev_tile_go(const Bank& b, const TileArgs& a, hipStream_t s) {
  constexpr int T = wpt_T<C>(), KM = wpt_K<C>();
  constexpr int QM = (LMax<L>::v + 1) / 2;
  auto k = wpt_rev_tile<L, C, NT, T, KM, kFMA>;
  const size_t lds = (size_t)(T + (1 << KM) * (2 * QM + 4)) * C * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)(a.nouter * ncb(a.inner, C) * (a.h / T)));
  JWV_LAUNCH(k, grid, dim3(NT), lds, s, a.src, a.sv, a.dst, a.dv, a.h, a.K, a.inner,
                     a.dma, rev_taps<L>(b));
  return hipGetLastError();
}

// ------------------------------------------------------------- AED varlen
template <int L, int OP>
hipError_t res_var_go(const Bank& b, const VarArgs& a, hipStream_t s) {
  constexpr bool fwd = OP == 0 || OP == 2;
  using TP = typename std::conditional<fwd, typename FB<L>::Fwd, typename FB<L>::Rev>::type;
  auto k = res_varlen<L, NT, cap<1>(), kFMA, OP, TP>;
  int mx = 0;
  for (int i = 0; i < a.seg.count; ++i) mx = a.seg.n[i] > mx ? a.seg.n[i] : mx;
  const size_t lds = (size_t)(mx + 2) * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  TP tp;
  if constexpr (fwd) tp = fwd_taps<L>(b); else tp = rev_taps<L>(b);
  JWV_LAUNCH(k, dim3((unsigned)a.seg.count), dim3(NT), lds, s, a.src, a.dst, a.seg, tp);
  return hipGetLastError();
}
template <int OP>
hipError_t res_var_l(const Bank& b, const VarArgs& a, hipStream_t s) {
  const bool rev = OP == 1 || OP == 3;
  switch ((rev && b.scale != 1.0) ? 0 : static_l(b.L)) {
    case 2: return res_var_go<2, OP>(b, a, s);
    case 4: return res_var_go<4, OP>(b, a, s);
    case 8: return res_var_go<8, OP>(b, a, s);
    case 16: return res_var_go<16, OP>(b, a, s);
    default: return res_var_go<0, OP>(b, a, s);
  }
}

}  // namespace

// L dispatch: compiled-in tap counts, else the runtime-L kernels.  A scaled
// synthesis bank (Haar1Orthogonal) always takes the runtime-L reverse path.
#define JWV_DISPATCH(GO, b, C, a, s, rev)                                   \
  do {                                                                      \
    const int L_ = ((rev) && (b).scale != 1.0) ? 0 : static_l((b).L);       \
    if ((C) == 1) {                                                         \
      switch (L_) {                                                         \
        case 2: return GO<2, 1>(b, a, s);                                   \
        case 4: return GO<4, 1>(b, a, s);                                   \
        case 8: return GO<8, 1>(b, a, s);                                   \
        case 16: return GO<16, 1>(b, a, s);                                 \
        default: return GO<0, 1>(b, a, s);                                  \
      }                                                                     \
    }                                                                       \
    switch (L_) {                                                           \
      case 2: return GO<2, 8>(b, a, s);                                     \
      case 4: return GO<4, 8>(b, a, s);                                     \
      case 8: return GO<8, 8>(b, a, s);                                     \
      case 16: return GO<16, 8>(b, a, s);                                   \
      default: return GO<0, 8>(b, a, s);                                    \
    }                                                                       \
  } while (0)

namespace JWV_NS {
hipError_t fwt_fwd_res(const Bank& b, int C, const ResArgs& a, hipStream_t s) {
  JWV_DISPATCH(fwt_fwd_res_go, b, C, a, s, false);
}
hipError_t fwt_rev_res(const Bank& b, int C, const ResArgs& a, hipStream_t s) {
  JWV_DISPATCH(fwt_rev_res_go, b, C, a, s, true);
}
hipError_t fwt_fwd_tile(const Bank& b, int C, const TileArgs& a, hipStream_t s) {
  JWV_DISPATCH(fwt_fwd_tile_go, b, C, a, s, false);
}
hipError_t fwt_rev_tile(const Bank& b, int C, const TileArgs& a, hipStream_t s) {
  JWV_DISPATCH(fwt_rev_tile_go, b, C, a, s, true);
}
hipError_t wpt_fwd_res(const Bank& b, int C, const ResArgs& a, hipStream_t s) {
  JWV_DISPATCH(wpt_fwd_res_go, b, C, a, s, false);
}
hipError_t wpt_rev_res(const Bank& b, int C, const ResArgs& a, hipStream_t s) {
  JWV_DISPATCH(wpt_rev_res_go, b, C, a, s, true);
}
hipError_t wpt_fwd_tile(const Bank& b, int C, const TileArgs& a, hipStream_t s) {
  JWV_DISPATCH(wpt_fwd_tile_go, b, C, a, s, false);
}
hipError_t wpt_rev_tile(const Bank& b, int C, const TileArgs& a, hipStream_t s) {
  JWV_DISPATCH(wpt_rev_tile_go, b, C, a, s, true);
}
hipError_t res_varlen(const Bank& b, bool wpt, bool fwd, const VarArgs& a, hipStream_t s) {
  if (a.seg.count < 1 || a.seg.count > VarSegs::kMax) return hipErrorInvalidValue;
  if (!wpt) return fwd ? res_var_l<0>(b, a, s) : res_var_l<1>(b, a, s);
  return fwd ? res_var_l<2>(b, a, s) : res_var_l<3>(b, a, s);
}
}  // namespace JWV_NS

}  // namespace jwv
