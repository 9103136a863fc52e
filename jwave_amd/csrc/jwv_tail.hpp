// jwv_tail.hpp — host entry points of launch_tail.hip, one per math mode:
// the fused forward tail (fwt_fwd_tail1, fwt1_chain.hpp).
#pragma once
#include "jwv_epoch.hpp"
#include "jwv_launch.hpp"

namespace jwv {
// Forward tail of one long contiguous signal in ONE launch: B units of
// kTailTB level-input samples run KB (kTailKMin..kTailKMax) levels each (the
// deep tile pass);
// the unit that completes the arrival counter runs the remaining levC levels
// resident (the resident pass), so the two latency-bound launches and the
// boundary between them become one.
struct TailArgs {
  const double* src;   // level input, length hB (the first pass's approximation)
  double* dst;         // the signal's coefficient array
  double* wsB;         // hB >> kTailKB doubles (handed to the last unit)
  unsigned* cnt;       // arrival counter (never reset, jwv_epoch.hpp)
  unsigned last_old;   // tail_last_old(counter value at launch, hB / kTailTB)
  int hB, KB, levC;
};
constexpr int kTailTB = 2048, kTailKMin = 6, kTailKMax = 9, kTailCap = 1024;
namespace exact {
hipError_t fwt_fwd_tail(const Bank&, const TailArgs&, hipStream_t);
}
namespace fused {
hipError_t fwt_fwd_tail(const Bank&, const TailArgs&, hipStream_t);
}
}  // namespace jwv
