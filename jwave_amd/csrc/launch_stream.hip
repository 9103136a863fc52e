// launch_stream.hip — launches of the persistent tile passes
// (fwt1_stream.hpp) for one math mode (compiled twice, like launch_fwt1.hip).
#include "fwt1_chain.hpp"
#include "fwt1_stream.hpp"
#include "jwv_stream.hpp"

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
constexpr int kT = Geo::kFwt1T;

// Blocks per CU the kernel can hold (occupancy query, cached per kernel).
template <typename Kern>
int resident_blocks(Kern k, int threads, size_t lds) {
  static int occ = 0, ncu = 0;
  if (!occ) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, threads, lds) != hipSuccess || occ <= 0)
      occ = 1;
  }
  return occ * ncu;
}

template <int L, int NTC, int T, int K>
hipError_t fwd_k(const Bank& b, const TileArgs& a, hipStream_t s) {
  auto k = fwt_fwd_stream1<L, NTC, T, K, kFMA>;
  const size_t lds = (size_t)2 * Fwd1Stream<L, T, K>::kBuf * sizeof(double);
  if (lds > 65536)
    if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds))
      return e;
  FwdTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = b.lo[j]; tp.hi[j] = b.hi[j]; }
  const int64_t ntotal = a.nouter * (int64_t)(a.h / T);
  int64_t grid = resident_blocks(k, NTC + 64, lds);
  grid &= ~(int64_t)7;  // whole XCD groups (the chunked walk needs nb % 8 == 0)
  if (grid > ntotal) grid = (ntotal + 7) & ~(int64_t)7;
  if (grid < 8) grid = 8;
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(NTC + 64), lds, s, a.src, a.sv.s_outer, a.dst,
                     a.dv.s_outer, a.adst, a.av.s_outer, a.h, ntotal, tp);
  return hipGetLastError();
}
template <int L>
hipError_t fwd_l(const Bank& b, const TileArgs& a, hipStream_t s) {
  switch (a.K) {
    case 1: return fwd_k<L, 256, kT, 1>(b, a, s);
    case 2: return fwd_k<L, 256, kT, 2>(b, a, s);
    case 3: return fwd_k<L, 256, kT, 3>(b, a, s);
    case 4: return fwd_k<L, 256, kT, 4>(b, a, s);
    case 5: return fwd_k<L, 256, kT, 5>(b, a, s);
    default: return fwd_k<L, 256, kT, 6>(b, a, s);
  }
}
// fused forward tail: kTailTB x kTailKB units, 512 threads (the deep pass's
// geometry), the last arriver runs the resident levels (<= kTailCap samples)
template <int L, int KB>
hipError_t tail_k(const Bank& b, const TailArgs& a, hipStream_t s) {
  constexpr int NT = 512;
  auto k = fwt_fwd_tail1<L, NT, kTailTB, KB, kTailCap, kFMA>;
  const int hC = a.hB >> KB;
  if (a.hB % kTailTB || hC > kTailCap || hC < 1) return hipErrorInvalidValue;
  const size_t lds = ((size_t)tail_ctl_off<L, kTailTB, KB>(hC) + 2) * sizeof(double);
  if (lds > 65536)
    if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds))
      return e;
  FwdTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = b.lo[j]; tp.hi[j] = b.hi[j]; }
  hipLaunchKernelGGL(k, dim3((unsigned)(a.hB / kTailTB)), dim3(NT), lds, s, a.src, a.dst, a.wsB,
                     a.cnt, a.hB, a.levC, tp);
  return hipGetLastError();
}
template <int L>
hipError_t tail_l(const Bank& b, const TailArgs& a, hipStream_t s) {
  switch (a.KB) {
    case 6: return tail_k<L, 6>(b, a, s);
    case 7: return tail_k<L, 7>(b, a, s);
    case 8: return tail_k<L, 8>(b, a, s);
    case 9: return tail_k<L, 9>(b, a, s);
    default: return hipErrorInvalidValue;
  }
}
bool plain(const AxisView& v) { return v.pk == 1 && v.s_len == 1; }
bool even_rows(const AxisView& v, int64_t nouter) { return nouter == 1 || (v.s_outer & 1) == 0; }
}  // namespace

namespace JWV_NS {
bool fwt_fwd_stream1(const Bank& b, const TileArgs& a, hipStream_t s, hipError_t& err) {
  if (!a.dma || a.inner != 1 || a.t1 != 0 || a.sp != 0) return false;
  if (!plain(a.sv) || !plain(a.dv) || !plain(a.av) || a.K < 1 || a.K > 6) return false;
  if (((uintptr_t)a.src & 15) || ((uintptr_t)a.dst & 15) || ((uintptr_t)a.adst & 15)) return false;
  if (!even_rows(a.sv, a.nouter) || !even_rows(a.dv, a.nouter) || !even_rows(a.av, a.nouter))
    return false;
  if (a.h < kT || a.h % kT) return false;
  switch (b.L) {
    case 2: err = fwd_l<2>(b, a, s); return true;
    case 4: err = fwd_l<4>(b, a, s); return true;
    case 8: err = fwd_l<8>(b, a, s); return true;
    case 16: err = fwd_l<16>(b, a, s); return true;
    default: return false;
  }
}
hipError_t fwt_fwd_tail(const Bank& b, const TailArgs& a, hipStream_t s) {
  switch (b.L) {
    case 2: return tail_l<2>(b, a, s);
    case 4: return tail_l<4>(b, a, s);
    case 8: return tail_l<8>(b, a, s);
    case 16: return tail_l<16>(b, a, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace JWV_NS
}  // namespace jwv
