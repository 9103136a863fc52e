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

template <int L, int J1, bool P2, int NT = kNT, int TF = kTF, int M = 1>
hipError_t fwd_kp(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  auto k = modwt_fwd_tile1<L, NT, TF, 1, J1, kFMA, P2, M>;
  const size_t lds = (size_t)ModFwd1Geo<L, TF, 1, J1>::lds_doubles(M) * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)((a.N + TF - 1) / TF));
  hipLaunchKernelGGL(k, grid, dim3(NT), lds, s, a.src, a.wout, a.ldw, a.vout, a.N, taps<L>(b));
  return hipGetLastError();
}
// Persistent tiles (modwt_fwd_tile1p / modwt_inv_tile1p): blocks per CU x
// CUs, a multiple of 8 (XCDs); env JWV_MODWT_PF bit 0 forward, bit 1 inverse
// (a clear bit keeps the one-tile-per-block grid).  Off by default: r03, one
// box, two rounds: forward 169.2 / 169.6 us one tile per block vs 200.3 /
// 201.3 persistent; inverse (303) 225.0 / 226.8 vs 243.2 / 246.6.
int pf_env() {
  static const int v = [] {
    const char* e = std::getenv("JWV_MODWT_PF");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}
int cu_count() {
  static const int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 8)
      n = 256;
    return n;
  }();
  return v;
}
template <int L, int J1, int NT, int TF, int M = 1>
hipError_t fwd_kpp(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  auto k = modwt_fwd_tile1p<L, NT, TF, 1, J1, kFMA, true, M>;
  const size_t lds = (size_t)ModFwd1Geo<L, TF, 1, J1>::lds_doubles(M) * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const int64_t ntile = (a.N + TF - 1) / TF;
  const int per_cu = lds > 81920 ? 1 : 2;
  int64_t nb = (int64_t)(cu_count() / 8) * per_cu;  // blocks per XCD
  const int64_t need = (ntile + 7) / 8;            // tiles per XCD chunk
  if (nb > need) nb = need;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL(k, dim3((unsigned)(8 * nb)), dim3(NT), lds, s, a.src, a.wout, a.ldw, a.vout,
                     a.N, taps<L>(b));
  return hipGetLastError();
}
template <int L, int J1, int NT, int TI, int M = 1>
hipError_t inv_kpp(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  auto k = modwt_inv_tile1p<L, NT, TI, 1, J1, kFMA, true, M>;
  const size_t lds = (size_t)ModInv1Geo<L, TI, 1, J1>::lds_doubles(M) * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const int64_t ntile = (a.N + TI - 1) / TI;
  const int per_cu = (int)(163840 / (lds + 1024));  // LDS-bound blocks per CU
  int64_t nb = (int64_t)(cu_count() / 8) * (per_cu < 1 ? 1 : per_cu);
  const int64_t need = (ntile + 7) / 8;
  if (nb > need) nb = need;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL(k, dim3((unsigned)(8 * nb)), dim3(NT), lds, s, a.src, a.coef, a.ldw, a.vout,
                     a.N, taps<L>(b));
  return hipGetLastError();
}
// tile geometry of the full-depth (J1 = 8) launches: env JWV_MODWT_GF (forward)
// / JWV_MODWT_GI (inverse) = 0 default, 1.. the alternatives below
int geo_env(const char* name) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : 0;
}
int geo_f() { static const int v = geo_env("JWV_MODWT_GF"); return v; }
// Run form (ModRun) of the full-depth launches: env JWV_MODWT_RUN (inverse) /
// JWV_MODWT_RUNF (forward) = m + 100*jr, m pairs per lane on levels j >= jr
// (3, 303, 503; 1 = the two-output P2 form on every level)
int run_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}
// inverse: 303 (r03, one box, two rounds: 235.3 / 236.8 us against 250.0 /
// 252.1 for the P2 form, 243.5 / 239.7 for 3, 239.1 / 237.9 for 503)
int run_m() { static const int v = run_env("JWV_MODWT_RUN", 303); return v; }
// forward (env JWV_MODWT_RUNF): 1, the P2 form (r03: 176.3 / 174.4 us against
// 207.9 / 209.4 for 3, 203.6 / 203.0 for 303, 206.0 / 205.1 for 503 — the run
// form's W stores leave the wave as H-slot runs M*H slots apart)
int run_f() { static const int v = run_env("JWV_MODWT_RUNF", 1); return v; }
int geo_i() { static const int v = geo_env("JWV_MODWT_GI"); return v; }
template <int L, int J1, bool P2, int NT = kNT, int TI = kTI, int M = 1>
hipError_t inv_kp(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  auto k = modwt_inv_tile1<L, NT, TI, 1, J1, kFMA, P2, M>;
  const size_t lds = (size_t)ModInv1Geo<L, TI, 1, J1>::lds_doubles(M) * sizeof(double);
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
        if (p2_bits() & 1) {
          if ((pf_env() & 1) && run_f() == 1) return fwd_kpp<L, J1, 1024, 8192>(b, a, s);
          switch (run_f()) {
            case 3: return fwd_kp<L, J1, true, 1024, 8192, 3>(b, a, s);
            case 303: return fwd_kp<L, J1, true, 1024, 8192, 303>(b, a, s);
            case 503: return fwd_kp<L, J1, true, 1024, 8192, 503>(b, a, s);
            default: break;
          }
          return fwd_kp<L, J1, true, 1024, 8192>(b, a, s);
        }
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
      case 5: return inv_kp<L, J1, true, 1024, 4096, 303>(b, a, s);
      case 6: return inv_kp<L, J1, true, 512, 1536, 303>(b, a, s);
      case 7: return inv_kp<L, J1, true, 256, 1024, 303>(b, a, s);
      default:
        if (p2_bits() & 2) {
          if (pf_env() & 2) {
            if (run_m() == 303) return inv_kpp<L, J1, kNT, kTI, 303>(b, a, s);
            if (run_m() == 1303) return inv_kpp<L, J1, kNT, kTI, 1303>(b, a, s);
            if (run_m() == 1) return inv_kpp<L, J1, kNT, kTI>(b, a, s);
          }
          switch (run_m()) {
            case 3: return inv_kp<L, J1, true, kNT, kTI, 3>(b, a, s);
            case 303: return inv_kp<L, J1, true, kNT, kTI, 303>(b, a, s);
            case 1303: return inv_kp<L, J1, true, kNT, kTI, 1303>(b, a, s);
            case 503: return inv_kp<L, J1, true, kNT, kTI, 503>(b, a, s);
            default: break;
          }
        }
        break;
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
