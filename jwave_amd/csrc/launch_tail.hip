// launch_tail.hip — launches of the fused forward tail (fwt_fwd_tail1,
// fwt1_chain.hpp) for one math mode (compiled twice, like launch_fwt1.hip).
#include "fwt1_chain.hpp"
#include "jwv_tail.hpp"

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
  JWV_LAUNCH(k, dim3((unsigned)(a.hB / kTailTB)), dim3(NT), lds, s, a.src, a.dst, a.wsB,
                     a.cnt, a.last_old, a.hB, a.levC, tp);
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
}  // namespace

namespace JWV_NS {
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
