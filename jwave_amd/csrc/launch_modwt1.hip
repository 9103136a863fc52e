// launch_modwt1.hip — the compile-time-geometry MODWT tiles
// (modwt1_kernels.hpp) for one math mode (compiled twice, like
// launch_modwt.hip).  Covered: tap count L = 8, fused levels 1..j1 with
// j1 <= 8 (config 5: Daubechies4, J = 8, one launch per direction); every
// other case keeps the runtime-geometry tiles.
#include "modwt1_kernels.hpp"
#include "jwv_modwt1.hpp"

#include <cstdlib>

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
constexpr int kNT = 512, kTF = 4096, kTI = 2048;

template <typename K>
hipError_t prep(K kernel, size_t lds) {
  if (lds > 65536)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  return hipSuccess;
}
template <int L>
ModwtTaps<L> taps(const Bank& b) {
  ModwtTaps<L> t{};
  for (int j = 0; j < L; ++j) { t.g[j] = b.lo[j]; t.h[j] = b.hi[j]; }
  return t;
}

// env JWV_MODWT_P2 (default 3): bit 0 forward, bit 1 inverse — two adjacent
// outputs per lane (16-B LDS reads); a clear bit = one output per lane
int p2_bits() {
  static const int v = [] {
    const char* e = std::getenv("JWV_MODWT_P2");
    return e ? std::atoi(e) : 3;
  }();
  return v;
}

template <int L, int J1, bool P2, int NT = kNT, int TF = kTF>
hipError_t fwd_kp(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  auto k = modwt_fwd_tile1<L, NT, TF, 1, J1, kFMA, P2>;
  const size_t lds = (size_t)ModFwd1Geo<L, TF, 1, J1>::lds_doubles() * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)((a.N + TF - 1) / TF));
  hipLaunchKernelGGL(k, grid, dim3(NT), lds, s, a.src, a.wout, a.ldw, a.vout, a.N, taps<L>(b));
  return hipGetLastError();
}
// tile geometry of the full-depth (J1 = 8) launches: env JWV_MODWT_GF (forward)
// / JWV_MODWT_GI (inverse) = 0 default, 1.. the alternatives below
int geo_env(const char* name) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : 0;
}
int geo_f() { static const int v = geo_env("JWV_MODWT_GF"); return v; }
int geo_i() { static const int v = geo_env("JWV_MODWT_GI"); return v; }
template <int L, int J1, bool P2, int NT = kNT, int TI = kTI>
hipError_t inv_kp(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  auto k = modwt_inv_tile1<L, NT, TI, 1, J1, kFMA, P2>;
  const size_t lds = (size_t)ModInv1Geo<L, TI, 1, J1>::lds_doubles() * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)((a.N + TI - 1) / TI));
  hipLaunchKernelGGL(k, grid, dim3(NT), lds, s, a.src, a.coef, a.ldw, a.vout, a.N, taps<L>(b));
  return hipGetLastError();
}
// Full-depth forward (J1 = 8, config 5): 1024 x 8192 tiles (half the halo
// recompute of 4096-sample tiles; 16 waves per CU either way): 186-188 ->
// 173-176 us per launch (two runs, one box); 512 x 8192 (200 us) and
// 256 x 4096 (214 us) measured slower.  JWV_MODWT_GF selects the others.
template <int L, int J1>
hipError_t fwd_k(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  if constexpr (J1 == 8) {
    switch (geo_f()) {
      case 1: return fwd_kp<L, J1, true, 512, 8192>(b, a, s);
      case 3: return fwd_kp<L, J1, true, 256, 4096>(b, a, s);
      case 4: return fwd_kp<L, J1, true, 512, 4096>(b, a, s);
      case 5: return fwd_kp<L, J1, true, 1024, 16384>(b, a, s);
      default:
        if (p2_bits() & 1) return fwd_kp<L, J1, true, 1024, 8192>(b, a, s);
        break;
    }
  }
  return (p2_bits() & 1) ? fwd_kp<L, J1, true>(b, a, s) : fwd_kp<L, J1, false>(b, a, s);
}
template <int L, int J1>
hipError_t inv_k(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  if constexpr (J1 == 8) {
    switch (geo_i()) {
      case 1: return inv_kp<L, J1, true, 512, 1024>(b, a, s);
      case 2: return inv_kp<L, J1, true, 256, 1024>(b, a, s);
      case 3: return inv_kp<L, J1, true, 1024, 4096>(b, a, s);
      case 4: return inv_kp<L, J1, true, 256, 2048>(b, a, s);
      default: break;
    }
  }
  return (p2_bits() & 2) ? inv_kp<L, J1, true>(b, a, s) : inv_kp<L, J1, false>(b, a, s);
}
template <int L, bool FWD>
hipError_t go(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  switch (a.j1) {
    case 1: return FWD ? fwd_k<L, 1>(b, a, s) : inv_k<L, 1>(b, a, s);
    case 2: return FWD ? fwd_k<L, 2>(b, a, s) : inv_k<L, 2>(b, a, s);
    case 3: return FWD ? fwd_k<L, 3>(b, a, s) : inv_k<L, 3>(b, a, s);
    case 4: return FWD ? fwd_k<L, 4>(b, a, s) : inv_k<L, 4>(b, a, s);
    case 5: return FWD ? fwd_k<L, 5>(b, a, s) : inv_k<L, 5>(b, a, s);
    case 6: return FWD ? fwd_k<L, 6>(b, a, s) : inv_k<L, 6>(b, a, s);
    case 7: return FWD ? fwd_k<L, 7>(b, a, s) : inv_k<L, 7>(b, a, s);
    default: return FWD ? fwd_k<L, 8>(b, a, s) : inv_k<L, 8>(b, a, s);
  }
}
bool covered(const Bank& b, const ModwtArgs& a) {
  return b.L == 8 && a.j0 == 1 && a.j1 >= 1 && a.j1 <= 8 && a.N >= 1;
}
}  // namespace

namespace JWV_NS {
bool modwt_fwd1(const Bank& b, const ModwtArgs& a, hipStream_t s, hipError_t& err) {
  if (!covered(b, a)) return false;
  err = go<8, true>(b, a, s);
  return true;
}
bool modwt_inv1(const Bank& b, const ModwtArgs& a, hipStream_t s, hipError_t& err) {
  if (!covered(b, a)) return false;
  err = go<8, false>(b, a, s);
  return true;
}
}  // namespace JWV_NS
}  // namespace jwv
