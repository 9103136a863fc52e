// jwv_modwt1.hpp — host entry points of launch_modwt1.hip (compile-time-
// geometry MODWT tiles), one per math mode.  Each returns false (nothing
// launched) when the case is not covered.
#pragma once
#include "jwv_launch.hpp"

namespace jwv {
namespace exact {
bool modwt_fwd1(const Bank&, const ModwtArgs&, hipStream_t, hipError_t& err);
bool modwt_inv1(const Bank&, const ModwtArgs&, hipStream_t, hipError_t& err);
}  // namespace exact
namespace fused {
bool modwt_fwd1(const Bank&, const ModwtArgs&, hipStream_t, hipError_t& err);
bool modwt_inv1(const Bank&, const ModwtArgs&, hipStream_t, hipError_t& err);
}  // namespace fused
}  // namespace jwv
