// jwv_epoch.hpp — arithmetic of the fused forward tail's arrival counter
// (fwt_fwd_tail1, fwt1_chain.hpp; host side in capi.cpp).  No HIP types, so
// the CPU tests compile it with gcc (tests/test_epoch.py).
//
// The counter is never reset: it only grows (mod 2^32).  The host knows the
// value it holds when a launch starts (`base`: every enqueued launch of nU
// blocks adds exactly nU), and passes the value the LAST arriver's atomic add
// returns, base + nU - 1.  Exactly one block of the launch sees it, whatever
// the value of base, including across the 2^32 wrap.  A launch that did not
// complete leaves the counter at an unknown value; the host's error path
// re-zeroes the counter and its base together (capi.cpp tail_resync), so the
// next call cannot fire its resident levels early or never.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define JWV_EPOCH_HD __host__ __device__
#else
#define JWV_EPOCH_HD
#endif

namespace jwv {
// value the last of nU arrivals reads when the launch starts at `base`
JWV_EPOCH_HD constexpr uint32_t tail_last_old(uint32_t base, uint32_t nU) { return base + nU - 1u; }
// counter value after a completed launch of nU blocks
JWV_EPOCH_HD constexpr uint32_t tail_next_base(uint32_t base, uint32_t nU) { return base + nU; }
}  // namespace jwv
