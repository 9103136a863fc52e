// jwv_launch.hpp — host-side launch interface between the C-ABI planner
// (capi.cpp) and the kernel translation units (launch_*.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include "jwv_device.hpp"

namespace jwv {

// Kernel timing for the planner's profiled pass (capi.cpp ProfScope): while
// a scope is open, the first kernel launched through JWV_LAUNCH carries the
// scope's start / stop events in its own dispatch packet
// (hipExtLaunchKernelGGL), so the elapsed time is the kernel's execution
// alone, as rocprofv3 reports it (events recorded as separate commands
// around the launch added ~6 us per launch of queue latency).
struct LaunchEvents {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int launches = 0;
};
extern thread_local LaunchEvents g_launch_ev;
#define JWV_LAUNCH(kernel, grid, block, lds, stream, ...)                                      \
  do {                                                                                        \
    if (::jwv::g_launch_ev.e0 && ::jwv::g_launch_ev.launches++ == 0)                          \
      hipExtLaunchKernelGGL(kernel, grid, block, lds, stream, ::jwv::g_launch_ev.e0,           \
                            ::jwv::g_launch_ev.e1, 0, __VA_ARGS__);                           \
    else                                                                                      \
      hipLaunchKernelGGL(kernel, grid, block, lds, stream, __VA_ARGS__);                     \
  } while (0)

// Host copy of a filter bank (Wavelet getters, Wavelet.java:152-219).
struct Bank {
  int L = 0;
  int tw = 2;
  double lo[kMaxTaps] = {};
  double hi[kMaxTaps] = {};
  double lo_r[kMaxTaps] = {};
  double hi_r[kMaxTaps] = {};
  double scale = 1.0;  // Haar1Orthogonal reverse factor
};

// Tap counts with compiled-in (unrolled, SGPR-resident) kernels; every other
// bank runs the runtime-L kernels (L=0 instantiation).
inline int static_l(int L) {
  switch (L) {
    case 2: case 4: case 8: case 16: return L;
    default: return 0;
  }
}

struct ResArgs {  // resident FWT/WPT kernels
  const double* src; AxisView sv;
  double* dst; AxisView dv;
  int n;       // FWT fwd: h0 (level input length); FWT rev: h0; WPT: signal/packet length
  int h0;      // WPT rev: first packet size
  int nlev;
  int64_t nouter;
  int inner;
  int dma;     // 1: windows may be loaded with LDS-DMA (alignment checked by host)
};
struct TileArgs {  // tiled FWT/WPT kernels
  const double* src; AxisView sv;   // level input (fwd) / approximation (FWT rev) / bands (WPT rev)
  const double* coef; AxisView cv;  // FWT rev: coefficient array
  double* dst; AxisView dv;
  double* adst; AxisView av;        // FWT fwd: level-K approximation
  int h;       // FWT/WPT fwd: level input length; FWT rev: h1; WPT rev: hK
  int K;
  int64_t nouter;
  int inner;
  int dma;
  int sp = 0;  // cache policy of the full-length output stores (st2_pol), C = 1 kernels
  int t1 = 0;  // C = 1 forward tile: 0 = Geo::kFwt1T, or 1024 (first pass of a long signal)
  // C = 1 tiles: segmented rows of the coefficient array (forward dst /
  // reverse coef): sample i at row + (i >> lsw) * ss + (i mod 2^lsw); 31 = plain
  int lsw = 31;
  int64_t ss = 0;
};
// AncientEgyptianDecomposition varlen launch (aed_kernels.hpp): contiguous
// 1-D segments of src / dst, one block each.
struct VarArgs {
  const double* src;
  double* dst;
  const VarSegs& seg;
};
struct ModwtArgs {
  const double* src;  // fwd: V_{j0-1}; inv: V_{j1}
  const double* coef; // inv: W rows base
  double* wout;       // fwd: W rows base
  double* vout;       // fwd: V_{j1}; inv: V_{j0-1}
  int64_t ldw;
  int64_t N;
  int j0, j1;
};

// Geometry of the compiled kernels (must match the template arguments used
// in launch_*.hip).  C = column slab: 1 for contiguous signals, 8 otherwise.
struct Geo {
  static constexpr int NT = 256;
  static constexpr int kResCap1 = 8192;  // resident elements per column, C = 1
  static constexpr int kResCap8 = 1024;  // C = 8
  static constexpr int kFwtT1 = 4096, kFwtK1 = 6;
  static constexpr int kFwtT8 = 512, kFwtK8 = 3;
  static constexpr int kWptT1 = 8192, kWptK1 = 6;
  static constexpr int kWptT8 = 512, kWptK8 = 3;
  static constexpr int kModT = 4096, kModTInv = 1024, kModS = 2048;
  static int res_cap(int C) { return C == 1 ? kResCap1 : kResCap8; }
  // tile of the C = 1 FWT passes (4096)
  static int fwd_t1();
  static int rev_t1();
  static bool rev_pref();  // reverse detail prefetch-all (off)
  // C = 1 compile-time-geometry kernels (fwt1_kernels.hpp, fwt1_res.hpp):
  // on.  Tiles: forward T = 4096, reverse T = 2048, up
  // to kFwt1KMax fused levels; the planner lets the last forward tile pass run
  // down to kFwt1Tail samples and starts the reverse tile passes above
  // kFwt1Tail * 2, so the single-block tails stay short.
  static bool fwt1();
  // C = 8 compile-time-geometry column-slab tiles (fwt8_kernels.hpp): on
  static bool fwt8();
  // block order of the C = 8 slab tiles: 1 slab-fastest
  static int slab_order();
  // st2_pol policy of the full-length output passes (0 plain)
  static int store_pol();
  static int tile_desc(int rev);  // sp bit 2 for the big pass (0)
  // sp bits of the C = 1 tile walk (tile_order): the grouped one-front walk
  // with G = 64 tiles per XCD group
  static int tile_walk();
  // First (full-length) forward pass of one long contiguous signal: tile
  // and fused levels; the last forward tile pass runs down to fwd1_tail()
  // samples.
  static int fwd1_first_t();
  static int fwd1_first_k();
  static int fwd1_tail();
  static constexpr int kFwt1T = 2048, kRev1T = 2048, kFwt1KMax = 9;
  static constexpr int kFwt1FwdTail = 512, kFwt1RevTail = 1024;
  static constexpr int kWpt1T = 4096, kWpt1KMax = 6;  // WPT tiles (wpt1_kernels.hpp)
  static int fwt_t(int C) { return C == 1 ? kFwtT1 : kFwtT8; }
  static int fwt_k(int C) { return C == 1 ? kFwtK1 : kFwtK8; }
  static int wpt_t(int C) { return C == 1 ? kWptT1 : kWptT8; }
  static int wpt_k(int C) { return C == 1 ? kWptK1 : kWptK8; }
};

// Single-launch FWT chains (fwt1_chain.hpp): geometry of the compiled roles.
// Forward: A tiles (kTAf, kKA) -> B units (kTB, kKB) -> resident C (<= kCap).
// Reverse: resident R (<= kCap) -> M units (kTM, kKM) -> A tiles (kTA, kKAr).
struct ChainGeo {
  static constexpr int kTAf = 4096, kKA = 6, kTB = 2048, kKB = 7, kCap = 2048;
  static constexpr int kTA = 2048;
  static constexpr int kTM = 2048, kKM = 9, kKAr = 5;
  static constexpr int kWords = 4096;  // sync words per direction (ctx buffer: 2x)
  static int default_plan();          // JWV_PLAN_* bits: REV_HEAD | FWD_TAIL
};
struct ChainFwdArgs {
  const double* src; double* dst;
  double* wsA; double* wsB;   // h >> kKA, h >> (kKA + kKB) doubles
  unsigned* cnt;              // >= nU + 1 words, zero between calls
  int h, levC;
};
struct ChainRevArgs {
  const double* coef; double* dst;
  double* wsR; double* wsM;   // hR, hR << kKM doubles
  unsigned* ctl;              // >= 2 + nM words
  int h, h0R, nR;
  unsigned epoch;             // != 0, new per call
  unsigned spins;             // poll bound of each in-kernel wait
};
struct RevHeadArgs {  // fwt_rev_head1: R (redundant per block) + M units in one launch
  const double* coef;
  double* wsM;                // hR << kKM doubles (read by the next launch)
  int h0R, nR;
};
hipError_t launch_fwt_rev_head(const Bank&, bool fma, const RevHeadArgs&, hipStream_t);
hipError_t launch_fwt_fwd_chain(const Bank&, bool fma, const ChainFwdArgs&, hipStream_t);
hipError_t launch_fwt_rev_chain(const Bank&, bool fma, const ChainRevArgs&, hipStream_t);

// Each returns hipSuccess or the launch error.  `fma` selects the math mode.
hipError_t launch_fwt_fwd_res(const Bank&, bool fma, int C, const ResArgs&, hipStream_t);
hipError_t launch_fwt_rev_res(const Bank&, bool fma, int C, const ResArgs&, hipStream_t);
hipError_t launch_fwt_fwd_tile(const Bank&, bool fma, int C, const TileArgs&, hipStream_t);
hipError_t launch_fwt_rev_tile(const Bank&, bool fma, int C, const TileArgs&, hipStream_t);
hipError_t launch_wpt_fwd_res(const Bank&, bool fma, int C, const ResArgs&, hipStream_t);
hipError_t launch_wpt_rev_res(const Bank&, bool fma, int C, const ResArgs&, hipStream_t);
hipError_t launch_wpt_fwd_tile(const Bank&, bool fma, int C, const TileArgs&, hipStream_t);
hipError_t launch_wpt_rev_tile(const Bank&, bool fma, int C, const TileArgs&, hipStream_t);
hipError_t launch_modwt_fwd(const Bank& modwt_gh, bool fma, bool tiled, const ModwtArgs&,
                            hipStream_t);
hipError_t launch_modwt_inv(const Bank& modwt_gh, bool fma, bool tiled, const ModwtArgs&,
                            hipStream_t);
hipError_t launch_res_varlen(const Bank&, bool fma, bool wpt, bool fwd, const VarArgs&,
                             hipStream_t);
hipError_t launch_copy_axis(const double* src, AxisView sv, double* dst, AxisView dv,
                            int64_t nouter, int len, int inner, hipStream_t);

// CompressorMagnitude (launch_compress.hip): y = c with |c| < mean|c| *
// threshold zeroed, decisions identical to Java's left-to-right magnitude;
// scratch holds compress_scratch(n) doubles (the magnitude lands in
// scratch[compress_partials(n) + 1]).
int compress_partials(int64_t n);
int compress_scratch(int64_t n);
hipError_t launch_compress_magnitude(const double* c, double* y, int64_t n, double threshold,
                                     double* scratch, hipStream_t s);

// Per-mode entry points implemented by launch_{fwt,wpt,modwt}.hip compiled
// twice (JWV_FMA=0 / 1).
namespace exact {
hipError_t fwt_rev_head(const Bank&, const RevHeadArgs&, hipStream_t);
hipError_t fwt_fwd_chain(const Bank&, const ChainFwdArgs&, hipStream_t);
hipError_t fwt_rev_chain(const Bank&, const ChainRevArgs&, hipStream_t);
// fwt1 kernels: return false when the case is not covered (nothing launched)
bool wpt_tile1(const Bank&, const TileArgs&, hipStream_t, bool fwd, hipError_t& err);
bool fwt_fwd_res1(const Bank&, const ResArgs&, hipStream_t, hipError_t& err);
bool fwt_rev_res1(const Bank&, const ResArgs&, hipStream_t, hipError_t& err);
bool fwt_fwd_tile1(const Bank&, const TileArgs&, hipStream_t, hipError_t& err);
bool fwt_rev_tile1(const Bank&, const TileArgs&, hipStream_t, hipError_t& err);
bool fwt_tile8(const Bank&, const TileArgs&, hipStream_t, bool fwd, hipError_t& err);
bool fwt_res16(const Bank&, const ResArgs&, hipStream_t, bool fwd, hipError_t& err);
hipError_t fwt_fwd_res(const Bank&, int C, const ResArgs&, hipStream_t);
hipError_t fwt_rev_res(const Bank&, int C, const ResArgs&, hipStream_t);
hipError_t fwt_fwd_tile(const Bank&, int C, const TileArgs&, hipStream_t);
hipError_t fwt_rev_tile(const Bank&, int C, const TileArgs&, hipStream_t);
hipError_t wpt_fwd_res(const Bank&, int C, const ResArgs&, hipStream_t);
hipError_t wpt_rev_res(const Bank&, int C, const ResArgs&, hipStream_t);
hipError_t wpt_fwd_tile(const Bank&, int C, const TileArgs&, hipStream_t);
hipError_t wpt_rev_tile(const Bank&, int C, const TileArgs&, hipStream_t);
hipError_t modwt_fwd(const Bank&, bool tiled, const ModwtArgs&, hipStream_t);
hipError_t modwt_inv(const Bank&, bool tiled, const ModwtArgs&, hipStream_t);
hipError_t res_varlen(const Bank&, bool wpt, bool fwd, const VarArgs&, hipStream_t);
}  // namespace exact
namespace fused {
hipError_t fwt_rev_head(const Bank&, const RevHeadArgs&, hipStream_t);
hipError_t fwt_fwd_chain(const Bank&, const ChainFwdArgs&, hipStream_t);
hipError_t fwt_rev_chain(const Bank&, const ChainRevArgs&, hipStream_t);
// fwt1 kernels: return false when the case is not covered (nothing launched)
bool wpt_tile1(const Bank&, const TileArgs&, hipStream_t, bool fwd, hipError_t& err);
bool fwt_fwd_res1(const Bank&, const ResArgs&, hipStream_t, hipError_t& err);
bool fwt_rev_res1(const Bank&, const ResArgs&, hipStream_t, hipError_t& err);
bool fwt_fwd_tile1(const Bank&, const TileArgs&, hipStream_t, hipError_t& err);
bool fwt_rev_tile1(const Bank&, const TileArgs&, hipStream_t, hipError_t& err);
bool fwt_tile8(const Bank&, const TileArgs&, hipStream_t, bool fwd, hipError_t& err);
bool fwt_res16(const Bank&, const ResArgs&, hipStream_t, bool fwd, hipError_t& err);
hipError_t fwt_fwd_res(const Bank&, int C, const ResArgs&, hipStream_t);
hipError_t fwt_rev_res(const Bank&, int C, const ResArgs&, hipStream_t);
hipError_t fwt_fwd_tile(const Bank&, int C, const TileArgs&, hipStream_t);
hipError_t fwt_rev_tile(const Bank&, int C, const TileArgs&, hipStream_t);
hipError_t wpt_fwd_res(const Bank&, int C, const ResArgs&, hipStream_t);
hipError_t wpt_rev_res(const Bank&, int C, const ResArgs&, hipStream_t);
hipError_t wpt_fwd_tile(const Bank&, int C, const TileArgs&, hipStream_t);
hipError_t wpt_rev_tile(const Bank&, int C, const TileArgs&, hipStream_t);
hipError_t modwt_fwd(const Bank&, bool tiled, const ModwtArgs&, hipStream_t);
hipError_t modwt_inv(const Bank&, bool tiled, const ModwtArgs&, hipStream_t);
hipError_t res_varlen(const Bank&, bool wpt, bool fwd, const VarArgs&, hipStream_t);
}  // namespace fused

}  // namespace jwv
