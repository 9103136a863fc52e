// jwv_stream.hpp — host entry points of the persistent (streaming) tile
// passes (fwt1_stream.hpp, launch_stream.hip), one per math mode.
#pragma once
#include "jwv_launch.hpp"

namespace jwv {
// Full-length forward pass of contiguous signals as a persistent,
// double-buffered grid.  Returns false (nothing launched) when the case is not
// covered; the caller then launches fwt_fwd_tile1.
namespace exact {
bool fwt_fwd_stream1(const Bank&, const TileArgs&, hipStream_t, hipError_t& err);
}
namespace fused {
bool fwt_fwd_stream1(const Bank&, const TileArgs&, hipStream_t, hipError_t& err);
}
}  // namespace jwv
