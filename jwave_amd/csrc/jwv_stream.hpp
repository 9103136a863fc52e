// jwv_stream.hpp — host entry points of launch_stream.hip, one per math mode:
// the persistent (streaming) forward pass (fwt1_stream.hpp) and the fused
// forward tail (fwt_fwd_tail1, fwt1_chain.hpp).
#pragma once
#include "jwv_launch.hpp"

namespace jwv {
// Full-length forward pass of contiguous signals as a persistent,
// double-buffered grid.  Returns false (nothing launched) when the case is not
// covered; the caller then launches fwt_fwd_tile1.
//
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
  unsigned* cnt;       // one word, zero between calls (reset by the last unit)
  int hB, KB, levC;
};
constexpr int kTailTB = 2048, kTailKMin = 6, kTailKMax = 9, kTailCap = 1024;
namespace exact {
bool fwt_fwd_stream1(const Bank&, const TileArgs&, hipStream_t, hipError_t& err);
hipError_t fwt_fwd_tail(const Bank&, const TailArgs&, hipStream_t);
}
namespace fused {
bool fwt_fwd_stream1(const Bank&, const TileArgs&, hipStream_t, hipError_t& err);
hipError_t fwt_fwd_tail(const Bank&, const TailArgs&, hipStream_t);
}
}  // namespace jwv
