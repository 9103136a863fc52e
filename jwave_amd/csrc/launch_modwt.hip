// launch_modwt.hip — instantiates the MODWT kernels for one math mode
// (compiled with -DJWV_FMA=0 and -DJWV_FMA=1), plus the strided copy kernel
// used for level-0 transforms (exact build only).
#include "jwv_launch.hpp"
#include "modwt_kernels.hpp"

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
constexpr int NT = 256;
constexpr int TI = Geo::kModTInv;  // inverse: two windows in LDS, smaller tile
constexpr int SMAX = Geo::kModS;

// Bank.lo / Bank.hi carry the MODWT g / h filters here (see capi.cpp).
template <int L>
typename MB<L>::Arg mtaps(const Bank& b) {
  typename MB<L>::Arg t{};
  if constexpr (L == 0) t.L = b.L;
  for (int j = 0; j < b.L; ++j) { t.g[j] = b.lo[j]; t.h[j] = b.hi[j]; }
  return t;
}

template <typename K>
hipError_t prep(K kernel, size_t lds) {
  if (lds + sizeof(ModNf) > 65536)  // + the static repair words (modwt_nonfinite.hpp)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  return hipSuccess;
}

// blocks for a one-level kernel: chunks of modwt_level_chunk(j) outputs
unsigned level_grid(int64_t N, int j) {
  const int64_t B = modwt_level_chunk(j);
  int64_t g = (N + B - 1) / B;
  return (unsigned)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

// Runtime-geometry tiles (banks the compile-time kernels do not cover):
// forward 512 x 4096 (config 5 228 -> 203 us against 256 x 1024), inverse in
// the class-major layout, 512 x 2048 (386 -> 285 us); register-blocked and
// two-deep-prefetch variants measured no better and were removed.
template <int L, int NTX, int TX>
hipError_t fwd_tile_go(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  const auto tp = mtaps<L>(b);
  auto k = modwt_fwd_tile<L, NTX, TX, SMAX, kFMA>;
  const int S = (b.L - 1) * ((1 << a.j1) - (1 << (a.j0 - 1)));
  const size_t lds = (size_t)(TX + S) * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)((a.N + TX - 1) / TX));
  JWV_LAUNCH(k, grid, dim3(NTX), lds, s, a.src, a.wout, a.ldw, a.vout, a.N, a.j0, a.j1,
                     tp);
  return hipGetLastError();
}

template <int L>
hipError_t fwd_go(const Bank& b, bool tiled, const ModwtArgs& a, hipStream_t s) {
  if (tiled) {
    return fwd_tile_go<L, 512, 4096>(b, a, s);
  }
  const auto tp = mtaps<L>(b);
  auto k = modwt_fwd_level<L, kFMA>;
  JWV_LAUNCH(k, dim3(level_grid(a.N, a.j0)), dim3(256), 0, s, a.src,
                     a.wout + (int64_t)(a.j0 - 1) * a.ldw, a.vout, a.N, a.j0, tp);
  return hipGetLastError();
}

template <int L, int NTX, int TX>
hipError_t inv_tile_go(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  const auto tp = mtaps<L>(b);
  auto k = modwt_inv_tile<L, NTX, TX, SMAX, kFMA>;
  const int R = (b.L - 1) * ((1 << a.j1) - (1 << (a.j0 - 1)));
  const size_t lds = (size_t)2 * (TX + R) * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)((a.N + TX - 1) / TX));
  JWV_LAUNCH(k, grid, dim3(NTX), lds, s, a.src, a.coef, a.ldw, a.vout, a.N, a.j0, a.j1,
                     tp);
  return hipGetLastError();
}

template <int L, int NTX, int TX>
hipError_t inv_tile_cm_go(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  if constexpr (L == 0) {
    return inv_tile_go<L, NT, TI>(b, a, s);
  } else {
    const auto tp = mtaps<L>(b);
    auto k = modwt_inv_tile_cm<L, NTX, TX, SMAX, kFMA>;
    const int buf = ModCm::buf(TX, b.L, a.j0, a.j1);
    const size_t lds = (size_t)2 * buf * sizeof(double);
    // The class padding grows with the stride: a deep level alone (Haar1 at
    // j = 12: st = 2048, 6 doubles per class) needs more than a CU's LDS in
    // this layout; the plain-layout tile needs 2 (T + R) doubles.
    if (lds + sizeof(ModNf) > 160 * 1024) return inv_tile_go<L, NT, TI>(b, a, s);
    if (hipError_t e = prep(k, lds)) return e;
    const dim3 grid((unsigned)((a.N + TX - 1) / TX));
    JWV_LAUNCH(k, grid, dim3(NTX), lds, s, a.src, a.coef, a.ldw, a.vout, a.N, a.j0,
                       a.j1, buf, tp);
    return hipGetLastError();
  }
}

template <int L>
hipError_t inv_go(const Bank& b, bool tiled, const ModwtArgs& a, hipStream_t s) {
  if (tiled) {
    return inv_tile_cm_go<L, 512, 2048>(b, a, s);
  }
  const auto tp = mtaps<L>(b);
  auto k = modwt_inv_level<L, kFMA>;
  JWV_LAUNCH(k, dim3(level_grid(a.N, a.j0)), dim3(256), 0, s, a.src,
                     a.coef + (int64_t)(a.j0 - 1) * a.ldw, a.vout, a.N, a.j0, tp);
  return hipGetLastError();
}

#if !JWV_FMA
__global__ __launch_bounds__(256) void copy_axis_kernel(const double* __restrict__ src,
                                                        AxisView sv, double* __restrict__ dst,
                                                        AxisView dv, int64_t nouter, int len,
                                                        int inner) {
  const int64_t total = nouter * (int64_t)len * inner;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * 256) {
    const int c = (int)(q % inner);
    const int64_t r = q / inner;
    const int i = (int)(r % len);
    const int64_t o = r / len;
    dst[view_base(dv, o) + i * dv.s_len + c] = src[view_base(sv, o) + i * sv.s_len + c];
  }
}
#endif
}  // namespace

namespace JWV_NS {
hipError_t modwt_fwd(const Bank& b, bool tiled, const ModwtArgs& a, hipStream_t s) {
  switch (b.L) {
    case 2: return fwd_go<2>(b, tiled, a, s);
    case 4: return fwd_go<4>(b, tiled, a, s);
    case 8: return fwd_go<8>(b, tiled, a, s);
    case 16: return fwd_go<16>(b, tiled, a, s);
    default: return fwd_go<0>(b, tiled, a, s);
  }
}
hipError_t modwt_inv(const Bank& b, bool tiled, const ModwtArgs& a, hipStream_t s) {
  switch (b.L) {
    case 2: return inv_go<2>(b, tiled, a, s);
    case 4: return inv_go<4>(b, tiled, a, s);
    case 8: return inv_go<8>(b, tiled, a, s);
    case 16: return inv_go<16>(b, tiled, a, s);
    default: return inv_go<0>(b, tiled, a, s);
  }
}
}  // namespace JWV_NS

#if !JWV_FMA
hipError_t launch_copy_axis(const double* src, AxisView sv, double* dst, AxisView dv,
                            int64_t nouter, int len, int inner, hipStream_t s) {
  const int64_t total = nouter * (int64_t)len * inner;
  if (total == 0) return hipSuccess;
  int64_t g = (total + 255) / 256;
  if (g > 16384) g = 16384;
  JWV_LAUNCH(copy_axis_kernel, dim3((unsigned)g), dim3(256), 0, s, src, sv, dst, dv,
                     nouter, len, inner);
  return hipGetLastError();
}
#endif

}  // namespace jwv
