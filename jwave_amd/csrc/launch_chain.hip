// launch_chain.hip — launches of the single-launch FWT chains
// (fwt1_chain.hpp) for one math mode (compiled twice, like launch_fwt1.hip).
#include "fwt1_chain.hpp"
#include "jwv_launch.hpp"

#include <algorithm>

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
using CG = ChainGeo;

template <typename Kern>
hipError_t prep_c(Kern kernel, size_t lds) {
  if (lds > 65536)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  return hipSuccess;
}

template <int L>
hipError_t fwd_l(const Bank& b, const ChainFwdArgs& a, hipStream_t s) {
  using CH = FwdChain<L, NT, CG::kTAf, CG::kKA, CG::kTB, CG::kKB, CG::kCap>;
  auto k = fwt_fwd_chain1<L, NT, CG::kTAf, CG::kKA, CG::kTB, CG::kKB, CG::kCap, kFMA, 4>;
  const int hC = (a.h >> CG::kKA) >> CG::kKB;
  const size_t lds = ((size_t)CH::ctl_off(hC) + 2) * sizeof(double);
  if (hipError_t e = prep_c(k, lds)) return e;
  FwdTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = b.lo[j]; tp.hi[j] = b.hi[j]; }
  JWV_LAUNCH(k, dim3((unsigned)(a.h / CG::kTAf)), dim3(NT), lds, s, a.src, a.dst, a.wsA,
                     a.wsB, a.cnt, a.h, a.levC, tp);
  return hipGetLastError();
}

// Reverse: persistent grid of co-resident blocks (static roles, bounded
// waits): CUs x (occupancy - 1) blocks, the margin the occupancy query needs
// (MI355X_MICROARCH.md: it can report one block per CU too many).
constexpr int kRevMinW = 5;
template <int L>
hipError_t rev_l(const Bank& b, const ChainRevArgs& a, hipStream_t s) {
  using CH = RevChain<L, NT, CG::kCap, CG::kTM, CG::kKM, CG::kTA, CG::kKAr>;
  auto k = fwt_rev_chain1<L, NT, CG::kCap, CG::kTM, CG::kKM, CG::kTA, CG::kKAr, kFMA, kRevMinW>;
  const int hR = a.h0R << (a.nR - 1);
  const size_t lds = (size_t)CH::lds_doubles(hR) * sizeof(double);
  if (hipError_t e = prep_c(k, lds)) return e;
  int dev = 0, ncu = 0, occ = 0;
  if (hipError_t e = hipGetDevice(&dev)) return e;
  if (hipError_t e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev))
    return e;
  if (hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, NT, lds)) return e;
  const int hM = hR << CG::kKM, nM = hM / CG::kTM, nA = a.h / CG::kTA;
  const long G = std::min<long>((long)ncu * std::max(1, std::min(occ - 1, 4)), 1L + nM + nA);
  if (G < 1 + nM) return hipErrorLaunchOutOfResources;  // M roles must all be co-resident
  RevTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo_r[j] = b.lo_r[j]; tp.hi_r[j] = b.hi_r[j]; }
  JWV_LAUNCH(k, dim3((unsigned)G), dim3(NT), lds, s, a.coef, a.dst, a.wsR, a.wsM, a.ctl,
                     a.h, a.h0R, a.nR, a.epoch, a.spins, tp);
  return hipGetLastError();
}
#ifndef JWV_HEAD_NT
#define JWV_HEAD_NT 512
#endif
template <int L>
hipError_t head_l(const Bank& b, const RevHeadArgs& a, hipStream_t s) {
  // 512 threads: the wide levels of R and M take half the pair slots
  constexpr int NTH = JWV_HEAD_NT;
  auto k = fwt_rev_head1<L, NTH, CG::kCap, CG::kTM, CG::kKM, kFMA>;
  const int hR = a.h0R << (a.nR - 1), nM = (hR << CG::kKM) / CG::kTM;
  if (hR > CG::kCap || nM < 1) return hipErrorInvalidValue;
  const size_t lds = (size_t)RevHeadGeo<L, CG::kTM, CG::kKM>::lds_doubles(hR) * sizeof(double);
  if (hipError_t e = prep_c(k, lds)) return e;
  RevTaps<L> tp;
  for (int j = 0; j < L; ++j) { tp.lo_r[j] = b.lo_r[j]; tp.hi_r[j] = b.hi_r[j]; }
  JWV_LAUNCH(k, dim3((unsigned)nM), dim3(NTH), lds, s, a.coef, a.wsM, a.h0R, a.nR, tp);
  return hipGetLastError();
}
}  // namespace

namespace JWV_NS {
hipError_t fwt_rev_head(const Bank& b, const RevHeadArgs& a, hipStream_t s) {
  switch (b.L) {
    case 2: return head_l<2>(b, a, s);
    case 4: return head_l<4>(b, a, s);
    case 8: return head_l<8>(b, a, s);
    case 16: return head_l<16>(b, a, s);
    default: return hipErrorInvalidValue;
  }
}
hipError_t fwt_fwd_chain(const Bank& b, const ChainFwdArgs& a, hipStream_t s) {
  switch (b.L) {
    case 2: return fwd_l<2>(b, a, s);
    case 4: return fwd_l<4>(b, a, s);
    case 8: return fwd_l<8>(b, a, s);
    case 16: return fwd_l<16>(b, a, s);
    default: return hipErrorInvalidValue;
  }
}
hipError_t fwt_rev_chain(const Bank& b, const ChainRevArgs& a, hipStream_t s) {
  switch (b.L) {
    case 2: return rev_l<2>(b, a, s);
    case 4: return rev_l<4>(b, a, s);
    case 8: return rev_l<8>(b, a, s);
    case 16: return rev_l<16>(b, a, s);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace JWV_NS
}  // namespace jwv
