// launch_modwt1.hip — the compile-time-geometry MODWT kernels (modwt_pipe.hpp,
// modwt1_kernels.hpp) for one math mode (compiled twice, like
// launch_modwt.hip).  Covered: tap count L = 8, fused levels 1..j1 with
// j1 <= 8 (config 5: Daubechies4, J = 8, one launch per direction); every
// other case keeps the runtime-geometry tiles.
#include "modwt1_kernels.hpp"
#include "modwt_pipe.hpp"
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

// One tile per block (modwt1_kernels.hpp): the fallback of the pipelined
// kernels for rows or outputs that are not 16-B aligned.  Two outputs per
// lane (P2).  Full depth (J1 = 8, config 5): forward 1024 x 8192 tiles (half
// the halo recompute of 4096-sample tiles; 512 x 8192: 200 us, 256 x 4096:
// 214 us, against 173-176), inverse 512 x 2048 in the run form from level 3
// (M = 303: 235 us against 250 for P2 on every level).
template <int L, int J1, int NT, int TF>
hipError_t fwd_kp(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  auto k = modwt_fwd_tile1<L, NT, TF, 1, J1, kFMA, true, 1>;
  const size_t lds = (size_t)ModFwd1Geo<L, TF, 1, J1>::lds_doubles(1) * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)((a.N + TF - 1) / TF));
  hipLaunchKernelGGL(k, grid, dim3(NT), lds, s, a.src, a.wout, a.ldw, a.vout, a.N, taps<L>(b));
  return hipGetLastError();
}
template <int L, int J1, int M>
hipError_t inv_kp(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  auto k = modwt_inv_tile1<L, kNT, kTI, 1, J1, kFMA, true, M>;
  const size_t lds = (size_t)ModInv1Geo<L, kTI, 1, J1>::lds_doubles(M) * sizeof(double);
  if (hipError_t e = prep(k, lds)) return e;
  const dim3 grid((unsigned)((a.N + kTI - 1) / kTI));
  hipLaunchKernelGGL(k, grid, dim3(kNT), lds, s, a.src, a.coef, a.ldw, a.vout, a.N, taps<L>(b));
  return hipGetLastError();
}

// Pipelined inverse / forward (modwt_pipe.hpp): persistent 1024-thread blocks,
// one per CU, windows by LDS-DMA; tiles 1024 (inverse) / 8192 (forward).
// Need 16-B aligned rows (ldw even) and outputs.  env JWV_MODWT_PIPE: bit 0
// inverse, bit 1 forward (A/B this round; default off until measured).
constexpr int kPipeT = 1024, kPipeNT = 1024, kPipeTF = 8192;
int pipe_env() {
  static const int v = [] {
    const char* e = std::getenv("JWV_MODWT_PIPE");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}
template <int L, int J1>
bool fwd_pipe(const Bank& b, const ModwtArgs& a, hipStream_t s, hipError_t& err) {
  using G = FwdPipeGeo<L, kPipeTF, J1>;
  if (!(pipe_env() & 2) || (a.ldw & 1) ||
      (((uintptr_t)a.wout | (uintptr_t)a.src | (uintptr_t)a.vout) & 15))
    return false;
  const size_t lds = (size_t)G::lds_doubles() * sizeof(double);
  static_assert(G::lds_doubles() * 8 <= 163840, "pipe LDS");
  const int64_t ntile = (a.N + kPipeTF - 1) / kPipeTF;
  int64_t ti0 = (G::S + (G::S & 1) + kPipeTF - 1) / kPipeTF;
  int64_t ti1 = a.N / kPipeTF;
  if (ti1 < ti0) ti1 = ti0 = 0;  // no interior tile: every tile takes the edge kernel
  const ModwtTaps<L> tp = taps<L>(b);
  if (ti1 > ti0) {
    auto k = modwt_fwd_pipe<L, kPipeNT, kPipeTF, J1, kFMA>;
    if ((err = prep(k, lds))) return true;
    int64_t per = cu_count() / 8;
    const int64_t need = (ti1 - ti0 + 7) / 8;
    if (per > need) per = need;
    if (per < 1) per = 1;
    hipLaunchKernelGGL(k, dim3((unsigned)(8 * per)), dim3(kPipeNT), lds, s, a.src, a.wout, a.ldw,
                       a.vout, a.N, ti0, ti1, tp);
    if ((err = hipGetLastError())) return true;
  }
  const int64_t nedge = ti0 + (ntile - ti1);
  if (nedge > 0) {
    auto k = modwt_fwd_pipe_edge<L, kPipeNT, kPipeTF, J1, kFMA>;
    if ((err = prep(k, lds))) return true;
    hipLaunchKernelGGL(k, dim3((unsigned)nedge), dim3(kPipeNT), lds, s, a.src, a.wout, a.ldw,
                       a.vout, a.N, ti0, ti1, tp);
    err = hipGetLastError();
  }
  return true;
}
template <int L, int J1>
bool inv_pipe(const Bank& b, const ModwtArgs& a, hipStream_t s, hipError_t& err) {
  if constexpr (J1 < 2) {
    return false;
  } else {
    using G = InvPipeGeo<L, kPipeT, J1>;
    if (!(pipe_env() & 1) || (a.ldw & 1) ||
        (((uintptr_t)a.coef | (uintptr_t)a.src | (uintptr_t)a.vout) & 15))
      return false;
    const size_t lds = (size_t)G::lds_doubles() * sizeof(double);
    static_assert(G::lds_doubles() * 8 <= 163840, "pipe LDS");
    const int64_t u2 = 2 * G::units(J1);
    const int64_t ntile = (a.N + kPipeT - 1) / kPipeT;
    const int64_t ninner = a.N >= u2 ? (a.N - u2) / kPipeT + 1 : 0;
    const ModwtTaps<L> tp = taps<L>(b);
    if (ninner > 0) {
      auto k = modwt_inv_pipe<L, kPipeNT, kPipeT, J1, kFMA>;
      if ((err = prep(k, lds))) return true;
      int64_t per = cu_count() / 8;
      const int64_t need = (ninner + 7) / 8;
      if (per > need) per = need;
      if (per < 1) per = 1;
      hipLaunchKernelGGL(k, dim3((unsigned)(8 * per)), dim3(kPipeNT), lds, s, a.src, a.coef, a.ldw,
                         a.vout, a.N, ninner, tp);
      if ((err = hipGetLastError())) return true;
    }
    if (ntile > ninner) {
      auto k = modwt_inv_pipe_edge<L, kPipeNT, kPipeT, J1, kFMA>;
      if ((err = prep(k, lds))) return true;
      hipLaunchKernelGGL(k, dim3((unsigned)(ntile - ninner)), dim3(kPipeNT), lds, s, a.src, a.coef,
                         a.ldw, a.vout, a.N, ninner, tp);
      err = hipGetLastError();
    }
    return true;
  }
}
template <int L, int J1>
hipError_t fwd_k(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (fwd_pipe<L, J1>(b, a, s, e)) return e;
  if constexpr (J1 == 8) return fwd_kp<L, J1, 1024, 8192>(b, a, s);
  return fwd_kp<L, J1, kNT, kTF>(b, a, s);
}
template <int L, int J1>
hipError_t inv_k(const Bank& b, const ModwtArgs& a, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (inv_pipe<L, J1>(b, a, s, e)) return e;
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
