// launch_modwt1.hip — the compile-time-geometry MODWT kernels
// (modwt1_kernels.hpp) for one math mode (compiled twice, like
// launch_modwt.hip).  Covered: tap count L = 8, fused levels 1..j1 with
// j1 <= 8 (config 5: Daubechies4, J = 8, one launch per direction); every
// other case keeps the runtime-geometry tiles.
#include "modwt1_kernels.hpp"
#include "modwt_stream.hpp"
#include "jwv_modwt1.hpp"


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
  if (lds + sizeof(ModNf) > 65536)  // + the static repair words (modwt_nonfinite.hpp)
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
// One tile per block (modwt1_kernels.hpp), two outputs per lane (P2).  Full
// depth (J1 = 8, config 5): forward 1024 x 8192 tiles (half the halo
// recompute of 4096-sample tiles; 512 x 8192: 200 us, 256 x 4096: 214 us,
// against 173-176), inverse 512 x 2048 in the run form from level 3 (M = 303:
// 235 us against 250 for P2 on every level).  Measured and removed (r04b):
// persistent 1024-thread blocks with every window by LDS-DMA one level ahead
// and one barrier per level: forward 227-230 + 42 us (edge tiles), inverse
// 283-294 + 17 us, against 173-175 / 230-232 us.
template <int L, int J1, int NT, int TF>
hipError_t fwd_kp(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  auto k = modwt_fwd_tile1<L, NT, TF, 1, J1, kFMA, true, 1>;
  const size_t lds = (size_t)ModFwd1Geo<L, TF, 1, J1>::lds_doubles(1) * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)((a.N + TF - 1) / TF));
  JWV_LAUNCH(k, grid, dim3(NT), lds, s, a.src, a.wout, a.ldw, a.vout, a.N, taps<L>(b));
  return hipGetLastError();
}
template <int L, int J1, int M>
hipError_t inv_kp(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  auto k = modwt_inv_tile1<L, kNT, kTI, 1, J1, kFMA, true, M>;
  const size_t lds = (size_t)ModInv1Geo<L, kTI, 1, J1>::lds_doubles(M) * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)((a.N + kTI - 1) / kTI));
  JWV_LAUNCH(k, grid, dim3(kNT), lds, s, a.src, a.coef, a.ldw, a.vout, a.N, taps<L>(b));
  return hipGetLastError();
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
// Streamed forward (modwt_stream.hpp): chunks of 1024-sample tiles walked
// left to right with carried halos, one chunk per resident block (512
// threads, 3 blocks per CU).  Config 5 forward 172-175 -> 164-165 us
// (r04e/r04f, one box each, two rounds; 256 x 1024: 173-175, 1024 x 2048:
// 188, 512 x 2048: 172-173).  Needs N and ldw even and 16-B aligned rows;
// else the tile kernel.
template <int L, int J1, int NT, int T>
bool fwd_stream_g(const Bank& b, const ModwtArgs& a, hipStream_t s, hipError_t& err) {
  if constexpr ((J1 & 1) != 0) {
    return false;
  } else {
    using G = ModFStreamGeo<L, T, J1>;
    if ((a.N & 1) || (a.ldw & 1) ||
        (((uintptr_t)a.wout | (uintptr_t)a.src | (uintptr_t)a.vout) & 15) ||
        a.N < 2 * (G::XP() + G::Wn(1)) || a.N * 8 >= (int64_t(1) << 31))
      return false;
    auto k = modwt_fwd_stream<L, NT, T, J1, kFMA>;
    const size_t lds = (size_t)G::lds_doubles() * sizeof(double);
    if ((err = prep(k, lds))) return true;
    int per = 0;
    if ((err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, NT, lds))) return true;
    if (per < 1) per = 1;
    const int64_t ntile = (a.N + T - 1) / T;
    int64_t nb = (int64_t)per * cu_count();
    if (nb > ntile) nb = ntile;
    JWV_LAUNCH(k, dim3((unsigned)nb), dim3(NT), lds, s, a.src, a.wout, a.ldw, a.vout,
                       a.N, ntile, taps<L>(b));
    err = hipGetLastError();
    return true;
  }
}
template <int L, int J1>
bool fwd_stream(const Bank& b, const ModwtArgs& a, hipStream_t s, hipError_t& err) {
  return fwd_stream_g<L, J1, 512, 1024>(b, a, s, err);
}

template <int L, int J1>
hipError_t fwd_k(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  if constexpr (J1 == 8) {
    hipError_t e = hipSuccess;
    if (fwd_stream<L, J1>(b, a, s, e)) return e;
    return fwd_kp<L, J1, 1024, 8192>(b, a, s);
  }
  return fwd_kp<L, J1, kNT, kTF>(b, a, s);
}
template <int L, int J1>
hipError_t inv_k(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  if constexpr (J1 == 8) return inv_kp<L, J1, 303>(b, a, s);
  return inv_kp<L, J1, 1>(b, a, s);
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
