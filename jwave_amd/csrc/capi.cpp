// capi.cpp — C ABI of libjwave_hip.so: validation (reference messages), the
// pass planner, device workspace and host<->device staging.
//
// Every FWT / WPT transform is an "axis transform" over a [outer][len][inner]
// block (see jwv_device.hpp); the planner splits the reference's level loop
// into device passes:
//   forward : tiled passes of K fused levels while the level input is longer
//             than one block's LDS can hold, then one resident pass for the
//             rest (FastWaveletTransform.java:90-97, WaveletPacketTransform.java:95-121);
//   reverse : a resident pass for the small levels, then tiled passes
//             (FastWaveletTransform.java:137-149, WaveletPacketTransform.java:163-188).
// 2-D / 3-D transforms are sequences of axis transforms in the order of
// BasicTransform.java:361-474 / 509-659.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <sched.h>
#include <thread>
#include <string>
#include <vector>

#ifndef __HIP_DEVICE_COMPILE__
#include <immintrin.h>  // host staging copies (nt_copy)
#endif

#include "../../include/jwave_hip.h"
#include "jwv_launch.hpp"
#include "jwv_modwt1.hpp"
#include "jwv_tail.hpp"

using jwv::AxisView;
using jwv::Bank;
using jwv::Geo;

namespace jwv {
thread_local LaunchEvents g_launch_ev;  // jwv_launch.hpp
}

namespace {

thread_local std::string g_tls_error;

struct DevBuf {
  double* p = nullptr;
  size_t n = 0;  // doubles
};

// Host staging of the host-pointer entry points (Transform.forward(double[])
// semantics: host array in, host array out).  Pageable caller memory goes
// through a ring of pinned chunks: host threads copy chunk k into a pinned
// slot while the DMA engine moves chunk k-1 to the device (and the reverse
// on the way out), so the PCIe transfer runs at the pinned rate instead of
// the driver's pageable path.  Pinned caller memory (hipHostMalloc /
// jwv_host_alloc / hipHostRegister) is DMA'd directly.
constexpr size_t kPinChunk = size_t(32) << 20;  // bytes per slot
constexpr int kPinSlots = 4;

#ifndef __HIP_DEVICE_COMPILE__
// Staging copy with non-temporal stores.  Its destination (a pinned slot on
// the way in, the caller's array on the way out) is written once and not read
// again by this core, so streaming stores skip the read-for-ownership a plain
// store pays: 2 DRAM transfers per byte instead of 3.  Ends and short copies
// go through memcpy; the sfence makes the streamed bytes visible before the
// copy is reported done (and the DMA engine reads them).
__attribute__((target("avx512f"))) static void nt_copy512(char* d, const char* s, size_t n) {
  size_t head = (64 - ((uintptr_t)d & 63)) & 63;
  head = std::min(head, n);
  std::memcpy(d, s, head);
  d += head, s += head, n -= head;
  size_t i = 0;
  for (; i + 256 <= n; i += 256) {
    const __m512i a = _mm512_loadu_si512(s + i), b = _mm512_loadu_si512(s + i + 64),
                  c = _mm512_loadu_si512(s + i + 128), e = _mm512_loadu_si512(s + i + 192);
    _mm512_stream_si512((__m512i*)(d + i), a);
    _mm512_stream_si512((__m512i*)(d + i + 64), b);
    _mm512_stream_si512((__m512i*)(d + i + 128), c);
    _mm512_stream_si512((__m512i*)(d + i + 192), e);
  }
  for (; i + 64 <= n; i += 64) _mm512_stream_si512((__m512i*)(d + i), _mm512_loadu_si512(s + i));
  std::memcpy(d + i, s + i, n - i);
  _mm_sfence();
}
__attribute__((target("avx2"))) static void nt_copy256(char* d, const char* s, size_t n) {
  size_t head = (32 - ((uintptr_t)d & 31)) & 31;
  head = std::min(head, n);
  std::memcpy(d, s, head);
  d += head, s += head, n -= head;
  size_t i = 0;
  for (; i + 128 <= n; i += 128)
    for (int k = 0; k < 128; k += 32)
      _mm256_stream_si256((__m256i*)(d + i + k), _mm256_loadu_si256((const __m256i*)(s + i + k)));
  std::memcpy(d + i, s + i, n - i);
  _mm_sfence();
}
void nt_copy(void* dst, const void* src, size_t n) {
  static const int isa = __builtin_cpu_supports("avx512f") ? 2 : __builtin_cpu_supports("avx2") ? 1 : 0;
  if (n < (size_t(64) << 10) || isa == 0) std::memcpy(dst, src, n);
  else if (isa == 2) nt_copy512((char*)dst, (const char*)src, n);
  else nt_copy256((char*)dst, (const char*)src, n);
}
#else
void nt_copy(void*, const void*, size_t) {}  // the device pass never runs host code
#endif

// Host threads for the pageable <-> pinned copies (one core's memcpy is
// several times slower than the PCIe link).  One pool per process, shared by
// every context (Java keeps a context per thread; a multi-device batch runs
// one thread per device): each copy() waits only for its own parts.
class CopyPool {
 public:
  explicit CopyPool(int n) { grow(n); }
  int size() {
    std::lock_guard<std::mutex> lk(mu_);
    return (int)th_.size() + 1;
  }
  // at least n worker threads (never shrinks; threads sleep when idle)
  void grow(int n) {
    std::lock_guard<std::mutex> lk(mu_);
    while ((int)th_.size() < n) th_.emplace_back([this] { loop(); });
  }
  // memcpy split over the pool's threads and the caller; returns when done
  void copy(void* dst, const void* src, size_t bytes) {
    const int parts = bytes >= (size_t(1) << 20) ? size() : 1;
    if (parts == 1) {
      nt_copy(dst, src, bytes);
      return;
    }
    const size_t per = ((bytes + parts - 1) / parts + 63) & ~size_t(63);
    Group g;
    std::unique_lock<std::mutex> lk(mu_);
    for (int i = 1; i < parts; ++i) {
      const size_t off = per * i;
      if (off >= bytes) break;
      ++g.pending;
      jobs_.push_back({&g, (char*)dst + off, (const char*)src + off, std::min(per, bytes - off),
                       0, 0, 1});
    }
    lk.unlock();
    cv_.notify_all();
    nt_copy(dst, src, std::min(per, bytes));
    lk.lock();
    done_.wait(lk, [&g] { return g.pending == 0; });
  }
  // nrows rows of w bytes, at pitches dp / sp bytes; rows split over the pool
  void copy2d(void* dst, size_t dp, const void* src, size_t sp, size_t w, size_t nrows) {
    const size_t bytes = w * nrows;
    const int parts = (int)std::min<size_t>(bytes >= (size_t(1) << 20) ? size() : 1, nrows);
    const size_t per = (nrows + parts - 1) / parts;
    Group g;
    std::unique_lock<std::mutex> lk(mu_);
    for (int i = 1; i < parts; ++i) {
      const size_t r0 = per * i;
      if (r0 >= nrows) break;
      ++g.pending;
      jobs_.push_back({&g, (char*)dst + r0 * dp, (const char*)src + r0 * sp, w, dp, sp,
                       std::min(per, nrows - r0)});
    }
    lk.unlock();
    cv_.notify_all();
    for (size_t r = 0; r < std::min(per, nrows); ++r)
      nt_copy((char*)dst + r * dp, (const char*)src + r * sp, w);
    lk.lock();
    done_.wait(lk, [&g] { return g.pending == 0; });
  }

 private:
  struct Group {
    int pending = 0;
  };
  struct Job {
    Group* g;
    char* d;
    const char* s;
    size_t n;            // bytes per row
    size_t dp, sp, rows; // row pitches (bytes) and row count (1: one contiguous run)
  };
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [this] { return !jobs_.empty(); });
      const Job job = jobs_.front();
      jobs_.pop_front();
      lk.unlock();
      for (size_t r = 0; r < job.rows; ++r) nt_copy(job.d + r * job.dp, job.s + r * job.sp, job.n);
      lk.lock();
      if (--job.g->pending == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::deque<Job> jobs_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
};

// The process's CPU share (sched affinity).
int affinity_cpus() {
  cpu_set_t cs;
  int hw = (int)std::thread::hardware_concurrency();
  if (sched_getaffinity(0, sizeof(cs), &cs) == 0) hw = CPU_COUNT(&cs);
  return std::max(1, hw);
}
// The process's pool: its CPU share, at most 16 threads per GPU in use (the
// GPU box's share per GPU), counting the caller: 16 for single-device
// contexts, grown by jwv_mctx_create to 16 per listed device.  Never
// destroyed (its threads sleep until process exit).
CopyPool& copy_pool() {
  static CopyPool* pool = new CopyPool(std::min(affinity_cpus(), 16) - 1);
  return *pool;
}

struct PinRing {
  char* p[kPinSlots] = {};
  hipEvent_t ev[kPinSlots] = {};
  double stat[6] = {};  // jwv_ctx_stage_stats
};
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct jwv_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  int math = JWV_MATH_EXACT;
  std::string err;
  std::mutex mu;
  DevBuf ws[2];  // small ping-pong scratch (level approximations)
  DevBuf big;    // full-size intermediate between 2-D/3-D axes
  DevBuf big2;   // full-size intermediate between multi-pass WPT passes
  DevBuf red;    // reduction scratch (CompressorMagnitude)
  DevBuf hin, hout;  // device buffers of the host-pointer entry points
  PinRing pin;       // their pinned host staging (allocated on first use)
  unsigned tail_base = 0;    // fused forward tail: counter value before the next launch
  bool tail_dirty = false;   // a tail launch was enqueued by the call in progress
  // single-launch FWT chains: [0, kWords) forward counters, [kWords, 2 kWords)
  // reverse ticket/flags; zeroed once, left zero by every completed launch
  unsigned* sync = nullptr;
  unsigned epoch = 0;  // reverse flag value of the last call (never 0)
  unsigned poll_limit = 1u << 22;  // bound of every in-kernel wait (chained reverse)
  bool waited = false;  // a launch with an in-kernel wait is queued, timeout word unchecked
  hipEvent_t switch_ev = nullptr;  // orders a stream switch after the old stream's work
  int plan = -1;       // JWV_PLAN_* bits; -1 = env defaults
  // profiling: hipEvent pairs around every kernel launch on the launch stream
  bool prof = false;
  int prof_only = -1;  // -1: every kind; else one KernelKind
  struct Rec { int kind; double bytes; hipEvent_t e0, e1; };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> ev_pool;
};

struct jwv_mctx {
  std::vector<jwv_ctx*> ctx;  // one per listed device
  std::string err;
  std::mutex mu;
  // multi-device 2-D (jwv_m_fwt2d_*): per device three block buffers, a
  // packing scratch, and the event that ends its first phase
  std::vector<DevBuf> a, b, c, t;
  std::vector<hipEvent_t> ev;
};

namespace {

struct Fail {
  int code;
  std::string msg;
};

int set_err(jwv_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg; else g_tls_error = msg;
  return code;
}

#define HIPCHK(expr)                                                                \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess)                                                           \
      throw Fail{JWV_ERR_DEVICE, std::string("HIP error: ") + hipGetErrorString(e_) + \
                                     " at " #expr};                                 \
  } while (0)

// MathToolKit.isBinary — tools/MathToolKit.java:185-188
bool is_binary(int64_t n) { return n > 0 && (n & (n - 1)) == 0; }
// BasicTransform.calcExponent / MathToolKit.getExponent (:202-206) — exact
// for powers of two in int range.
int exponent(int64_t n) {
  int e = 0;
  while ((int64_t(1) << (e + 1)) <= n) ++e;
  return e;
}

Bank make_bank(const jwv_taps* t) {
  if (!t) throw Fail{JWV_ERR_BAD_CALL, "jwv_taps is NULL"};
  if (t->mother_wavelength < 1 || t->mother_wavelength > JWV_MAX_TAPS)
    throw Fail{JWV_ERR_BAD_CALL, "mother_wavelength must be in [1, 64]"};
  if (t->transform_wavelength < 1)
    throw Fail{JWV_ERR_BAD_CALL, "transform_wavelength must be >= 1"};
  if (!t->lo || !t->hi || !t->lo_r || !t->hi_r)
    throw Fail{JWV_ERR_BAD_CALL, "tap pointer is NULL"};
  Bank b;
  b.L = t->mother_wavelength;
  b.tw = t->transform_wavelength;
  for (int j = 0; j < b.L; ++j) {
    b.lo[j] = t->lo[j]; b.hi[j] = t->hi[j]; b.lo_r[j] = t->lo_r[j]; b.hi_r[j] = t->hi_r[j];
  }
  b.scale = t->reverse_scale;
  return b;
}

AxisView cview(int64_t len, int64_t inner) {
  AxisView v{};
  v.s_outer = len * inner;
  v.s_pk = 0;
  v.s_len = inner;
  v.pk = 1;
  return v;
}

AxisView with_packets(AxisView v, int pk, int h) {
  v.pk = pk;
  v.s_pk = (int64_t)h * v.s_len;
  return v;
}

// grow-only device buffer; synchronises the stream before freeing (a queued
// kernel may still use the old buffer).
double* grow(jwv_ctx* c, DevBuf& b, size_t n) {
  if (b.n >= n) return b.p;
  HIPCHK(hipStreamSynchronize(c->stream));
  if (b.p) HIPCHK(hipFree(b.p));
  b.p = nullptr;
  b.n = 0;
  HIPCHK(hipMalloc(&b.p, std::max<size_t>(n, 1) * sizeof(double)));
  b.n = n;
  return b.p;
}

void hipchk(hipError_t e, const char* what) {
  if (e != hipSuccess)
    throw Fail{JWV_ERR_DEVICE, std::string("HIP error: ") + hipGetErrorString(e) + " in " + what};
}

enum KernelKind {
  K_FWT_FWD_TILE, K_FWT_FWD_RES, K_FWT_REV_TILE, K_FWT_REV_RES, K_WPT_FWD_TILE, K_WPT_FWD_RES,
  K_WPT_REV_TILE, K_WPT_REV_RES, K_MODWT_FWD_TILE, K_MODWT_FWD_LEVEL, K_MODWT_INV_TILE,
  K_MODWT_INV_LEVEL, K_COPY, K_FWT_FWD_CHAIN, K_FWT_REV_CHAIN, K_FWT_REV_HEAD,
  K_FWT_FWD_TILE_DEEP, K_FWT_REV_TILE_DEEP, K_AED_VARLEN, K_FWT_FWD_TAIL, K_NKINDS
};
// *_tile: the tiled pass that reads (forward) or writes (reverse) the full-length
// axis — the HBM-bound launch; *_tile_deep: tiled passes over an intermediate
// approximation (1/2^K of the bytes or less; latency-bound).  They are separate
// kernel instantiations (different fused level counts), as in rocprofv3.
const char* const kKindNames[K_NKINDS] = {
    "fwt_fwd_tile", "fwt_fwd_res", "fwt_rev_tile", "fwt_rev_res", "wpt_fwd_tile", "wpt_fwd_res",
    "wpt_rev_tile", "wpt_rev_res", "modwt_fwd_tile", "modwt_fwd_level", "modwt_inv_tile",
    "modwt_inv_level", "copy_axis", "fwt_fwd_chain", "fwt_rev_chain", "fwt_rev_head",
    "fwt_fwd_tile_deep", "fwt_rev_tile_deep", "aed_varlen", "fwt_fwd_tail"};

hipEvent_t take_event(jwv_ctx* c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  // timing-only events: no system-scope release when the event completes.
  // The default event writes back and invalidates the caches after the
  // bracketed kernel (~6 us per 2^24 pass on config 2), which the kernel's
  // own time does not include (rocprofv3 durations).
  hipEvent_t e;
  hipchk(hipEventCreateWithFlags(&e, hipEventDisableSystemFence), "hipEventCreate");
  return e;
}

// Brackets one kernel launch with events when profiling is on.  `bytes` is the
// launch's algorithmic HBM traffic (compulsory reads + writes).
struct ProfScope {
  jwv_ctx* c;
  bool on;
  size_t idx = 0;
  ProfScope(jwv_ctx* c_, int kind, double bytes)
      : c(c_), on(c_->prof && (c_->prof_only < 0 || c_->prof_only == kind)) {
    // env JWV_LAUNCH_LOG=1: one stderr line per launch, in launch order, so a
    // rocprofv3 --pmc run can attribute its dispatches to the planner's
    // kernel kinds (tools/pmc_traffic.py)
    static const bool log = [] {
      const char* v = std::getenv("JWV_LAUNCH_LOG");
      return v && *v == '1';
    }();
    if (log) std::fprintf(stderr, "JWV_LAUNCH %s %.0f\n", kKindNames[kind], bytes);
    if (!on) return;
    jwv_ctx::Rec r{kind, bytes, take_event(c), take_event(c)};
    c->recs.push_back(r);
    idx = c->recs.size() - 1;
    // the scope's first JWV_LAUNCH records both events in its dispatch packet
    jwv::g_launch_ev = {r.e0, r.e1, 0};
  }
  ~ProfScope() {
    if (!on) return;
    const int n = jwv::g_launch_ev.launches;
    jwv::g_launch_ev = {};
    const jwv_ctx::Rec& r = c->recs[idx];
    if (n == 0) {  // nothing launched (a copy): an empty span
      (void)hipEventRecord(r.e0, c->stream);
      (void)hipEventRecord(r.e1, c->stream);
    } else if (n > 1) {  // several launches: first start to last end
      (void)hipEventRecord(r.e1, c->stream);
    }
  }
};

struct Axis {
  const double* src;
  AxisView sv;
  double* dst;
  AxisView dv;
  int64_t outer;
  int len;
  int inner;
  // segmented coefficient rows (C = 1 row passes only; forward: dst, reverse:
  // src): sample i of row o at base + o * s_outer + (i >> lsw) * ss + (i mod
  // 2^lsw), the sharded 2-D transform's all-to-all layout; 31 = plain
  int lsw = 31;
  int64_t ss = 0;
};

bool use_fma(jwv_ctx* c) { return c->math == JWV_MATH_FMA; }

void copy_axis(jwv_ctx* c, const Axis& a) {
  { ProfScope ps_(c, K_COPY, 16.0 * a.outer * a.len * a.inner);
    hipchk(jwv::launch_copy_axis(a.src, a.sv, a.dst, a.dv, a.outer, a.len, a.inner, c->stream),
         "copy"); }
}

int col_slab(int inner) { return inner == 1 ? 1 : 8; }

// LDS-DMA (16 B per lane) needs 16-B aligned rows / row pairs.
bool dma_view(const double* base, const AxisView& v, int C, int inner) {
  if (((uintptr_t)base & 15) != 0) return false;
  if ((v.s_outer & 1) || (v.pk > 1 && (v.s_pk & 1))) return false;
  if (C == 1) return v.s_len == 1;
  return (v.s_len & 1) == 0 && inner % C == 0;
}

// Number of levels FastWaveletTransform / WaveletPacketTransform.forward runs
// (FastWaveletTransform.java:90: while h >= transformWavelength && l < level).
int fwd_levels(int len, int tw, int level) {
  int h = len, l = 0;
  while (h >= tw && l < level) { h >>= 1; ++l; }
  return l;
}
// First reverse level size (FastWaveletTransform.java:137-141); 0 = none.
int rev_first(int len, int tw, int level) {
  const int steps = exponent(len);
  int64_t h = tw;
  for (int l = level; l < steps; ++l) h <<= 1;
  return (h <= len && h >= tw) ? (int)h : 0;
}

// ------------------------------------------------------------------ FWT axis
// True when the C = 1 compile-time-geometry kernels (launch_fwt1.hip) take
// every tiled pass of this axis transform: contiguous 16-B aligned rows, a
// compiled-in tap count, an unscaled synthesis bank.  The planner then uses
// their deeper passes (up to Geo::kFwt1KMax levels) and short tails.
bool fast1(const Bank& b, const Axis& a, bool rev) {
  if (!Geo::fwt1() || a.inner != 1 || jwv::static_l(b.L) == 0) return false;
  if (rev && b.scale != 1.0) return false;
  if (a.sv.pk != 1 || a.dv.pk != 1 || a.sv.s_len != 1 || a.dv.s_len != 1) return false;
  if (!dma_view(a.src, a.sv, 1, 1)) return false;
  // 16-B output stores (both directions)
  if (((uintptr_t)a.dst & 15) || (a.outer > 1 && (a.dv.s_outer & 1))) return false;
  return true;
}

// ----------------------------------------------------------- FWT chains
// One launch per direction for a single long contiguous signal
// (fwt1_chain.hpp): the planner's tiled passes and resident tail become roles
// of one grid.  Only where the compiled role geometry (jwv::ChainGeo) covers
// the whole level plan; everything else takes the multi-launch plan below.
using jwv::ChainGeo;

// [0, kWords) forward chain, [kWords, 2 kWords) reverse chain, then the
// arrival counter of the fused forward tail (jwv_epoch.hpp: never reset; the
// context keeps the value it holds between launches in tail_base).  Like the
// workspace, it belongs to the context's launch stream: a context runs one
// transform at a time (its mutex), and a launch in flight on one stream must
// complete before the context is pointed at another (jwave_hip.h).
constexpr size_t kSyncWords = 2 * ChainGeo::kWords + 16 + 1;
unsigned* sync_words(jwv_ctx* c) {
  if (!c->sync) {
    HIPCHK(hipMalloc(&c->sync, kSyncWords * sizeof(unsigned)));
    HIPCHK(hipMemsetAsync(c->sync, 0, kSyncWords * sizeof(unsigned), c->stream));
  }
  return c->sync;
}
unsigned* tail_counter(jwv_ctx* c) { return sync_words(c) + 2 * ChainGeo::kWords + 16; }
// Error path: a failed call may have left a tail launch part-way, so the
// counter's value is unknown.  Drain the stream, zero the counter on it and
// drain again, then zero the base.  tail_dirty is cleared only when all of
// that succeeded; otherwise the next call of the context retries first
// (guarded), so no launch ever runs against a stale base.
bool tail_resync(jwv_ctx* c) {
  if (!c->sync || !c->tail_dirty) return true;
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess || (prev != c->device && hipSetDevice(c->device) != hipSuccess))
    return false;
  const bool ok = hipStreamSynchronize(c->stream) == hipSuccess &&
                  hipMemsetAsync(tail_counter(c), 0, sizeof(unsigned), c->stream) == hipSuccess &&
                  hipStreamSynchronize(c->stream) == hipSuccess;
  if (ok) {
    c->tail_base = 0;
    c->tail_dirty = false;
  }
  if (prev != c->device) (void)hipSetDevice(prev);
  return ok;
}

int plan_of(jwv_ctx* c) { return c->plan >= 0 ? c->plan : ChainGeo::default_plan(); }

// A planned launch of an axis transform.  The planner turns the reference's
// level loop into steps (tiled passes, the resident pass) before anything is
// launched; every workspace a plan uses is allocated while it is built
// (grow() synchronises the launch stream).  Round 5 measured a 2-D schedule
// that ran the resident steps on side streams beside the tile passes of
// independent column groups: slower, removed.
struct Step {
  bool res = false;  // the resident pass (fwt_fwd_res / fwt_rev_res)
  int h = 0;         // res: forward input length / reverse output length
  std::function<void()> go;
};
using Plan = std::vector<Step>;

void run_plan(const Plan& p) {
  for (const Step& s : p) s.go();
}

// One launch per direction (fwt1_chain.hpp) where the compiled geometry covers
// the plan; an empty function otherwise.
std::function<void()> fwd_chain_step(jwv_ctx* c, const Bank& b, const Axis& a, int nlev) {
  if (!(plan_of(c) & JWV_PLAN_CHAIN_FWD) || a.outer != 1 || !fast1(b, a, false)) return {};
  const int64_t h = a.len, hB = h >> ChainGeo::kKA, hC = hB >> ChainGeo::kKB;
  const int64_t mB = ChainGeo::kTB + (int64_t)(b.L - 2) * ((1 << ChainGeo::kKB) - 1);
  const int levC = nlev - ChainGeo::kKA - ChainGeo::kKB;
  if (levC < 0 || h % ChainGeo::kTAf || hB % ChainGeo::kTB || mB > hB || hC > ChainGeo::kCap)
    return {};
  if (hB / ChainGeo::kTB + 1 > ChainGeo::kWords) return {};
  double* wsA = grow(c, c->ws[0], (size_t)hB);
  double* wsB = grow(c, c->ws[1], (size_t)hC);
  const jwv::ChainFwdArgs ca{a.src, a.dst, wsA, wsB, sync_words(c), (int)h, levC};
  return [c, &b, ca, h] {
    ProfScope ps_(c, K_FWT_FWD_CHAIN, 16.0 * h);
    hipchk(jwv::launch_fwt_fwd_chain(b, use_fma(c), ca, c->stream), "fwt_fwd_chain");
  };
}

std::function<void()> rev_chain_step(jwv_ctx* c, const Bank& b, const Axis& a, int h0) {
  if (!(plan_of(c) & JWV_PLAN_CHAIN_REV) || a.outer != 1 || !fast1(b, a, true)) return {};
  const int64_t h = a.len, hM = h >> ChainGeo::kKAr, hR = hM >> ChainGeo::kKM;
  if (hM % ChainGeo::kTM || hR < 64 || hR > ChainGeo::kCap || h0 > hR) return {};
  if (2 + hM / ChainGeo::kTM > ChainGeo::kWords) return {};
  const int nR = exponent(hR / h0) + 1;
  double* wsR = grow(c, c->ws[0], (size_t)hR);
  double* wsM = grow(c, c->ws[1], (size_t)hM);
  return [c, &b, wsR, wsM, a, h, h0, nR] {
    if (++c->epoch == 0) c->epoch = 1;
    const jwv::ChainRevArgs ca{a.src, a.dst, wsR, wsM, sync_words(c) + ChainGeo::kWords, (int)h,
                               h0, nR, c->epoch, c->poll_limit};
    c->waited = true;
    ProfScope ps_(c, K_FWT_REV_CHAIN, 16.0 * h);
    hipchk(jwv::launch_fwt_rev_chain(b, use_fma(c), ca, c->stream), "fwt_rev_chain");
  };
}

// Resident-pass cap of an FWT axis transform.  Many contiguous signals (2-D
// rows, batches) can instead run their top levels through the C = 1 tile
// kernels and only a short tail resident (config 3 rows: 2.21 -> 1.99 ms per
// step at 2048).
// Resident reverse cap of row batches on the fwt1 path: the tile pass above
// it takes the remaining levels (1024; 256 and 512 measured slower).
int rev_row_tail() { return Geo::kFwt1RevTail; }

int fwt_res_cap(int C, int64_t outer) {
  constexpr int rowcap = 2048;
  if (C == 1 && outer >= 64 && rowcap >= 64 && rowcap < Geo::kResCap1) return rowcap;
  return Geo::res_cap(C);
}

// Cache policy of the full-length output stores of the forward (rev = 0) and
// reverse (rev = 1) big passes (st2_pol: 0 plain, 1 sc1, 2 nt): env
// JWV_STPOL_F / JWV_STPOL_R, else JWV_STPOL.  Default: the reverse of one
// 1-D signal (`final`: its output is the caller's result, not an
// intermediate another pass reads next) stores non-temporal, so it does not
// evict the coefficients a following reverse/forward pair streams from the
// Infinity Cache (config 2 steady state over 3 alternating runs: 111.3-113.5
// -> 109.0-111.3 us/step); forward outputs stay cacheable (nt on them: the
// reverse that reads them next took 123 us/step).
int store_pol_dir(int rev, bool final = false) { return rev && final ? 2 : 0; }

// FastWaveletTransform.forward's level loop (FastWaveletTransform.java:90-97)
// as device passes.  ws: the ping-pong pair for the level approximations.
Plan fwt_fwd_plan(jwv_ctx* c, const Bank& b, const Axis& a, int level, DevBuf* ws) {
  Plan p;
  const int nlev = fwd_levels(a.len, b.tw, level);
  if (nlev == 0 && a.lsw < 31) return {};  // a copy into segments: the caller's pack
  if (nlev == 0) {
    p.push_back({false, 0, [c, a] { copy_axis(c, a); }});
    return p;
  }
  if (auto f = fwd_chain_step(c, b, a, nlev)) {
    p.push_back({false, 0, f});
    return p;
  }
  const int C = col_slab(a.inner), cap = fwt_res_cap(C, a.outer), KM = Geo::fwt_k(C);
  const bool f1 = fast1(b, a, false);
  const bool seg = a.lsw < 31;
  const int sw = seg ? 1 << a.lsw : 0;
  // segmented output: C = 1 tile kernels only, every tile's per-level detail
  // range (T >> l <= T/2 samples, aligned) and every range written from the
  // start of the row inside one segment; else an empty plan (the caller
  // falls back to a plain pass + a pack)
  if (seg && (!f1 || a.outer < 2 || sw < Geo::kFwt1T / 2)) return {};
  // levels of the tiled pass at level-input size h: KM, except that on the
  // fwt1 path the pass that ends the tiled part runs on down to kFwt1FwdTail
  // the first pass of one long signal may use its own tile / level count
  const bool first1 = f1 && a.outer == 1 && a.len > cap &&
                      (a.len >> Geo::fwd1_first_k()) > cap && a.len % Geo::fwd1_first_t() == 0;
  auto pick_k = [&](int h, int rem) {
    if (first1 && h == a.len) return std::min(rem, Geo::fwd1_first_k());
    int K = std::min(rem, KM);
    if (f1 && (h >> K) <= cap)
      K = std::min(rem, std::min(exponent(h) - exponent(Geo::fwd1_tail()), Geo::kFwt1KMax));
    return K;
  };
  // workspace: the largest intermediate approximation
  {
    int h = a.len, rem = nlev;
    size_t need = 0;
    while (rem > 0 && h > cap) {
      const int K = pick_k(h, rem);
      if (K < rem) need = std::max(need, (size_t)a.outer * (size_t)(h >> K) * a.inner);
      h >>= K;
      rem -= K;
    }
    if (need) { grow(c, ws[0], need); grow(c, ws[1], need); }
  }
  const double* cur = a.src;
  AxisView cv = a.sv;
  int h = a.len, rem = nlev, pp = 0;
  while (rem > 0 && h > cap) {
    const int K = pick_k(h, rem);
    // JWV_PLAN_FWD_TAIL: this deep pass and the resident remainder in one
    // launch (fwt_fwd_tail1)
    if (f1 && a.outer == 1 && h < a.len && (plan_of(c) & JWV_PLAN_FWD_TAIL) &&
        K >= jwv::kTailKMin && K <= jwv::kTailKMax && rem > K && h % jwv::kTailTB == 0 &&
        (h >> K) <= jwv::kTailCap && ((uintptr_t)cur & 15) == 0) {
      double* wsB = ws[pp].p;
      unsigned* cnt = tail_counter(c);
      const int hh = h, lc = rem - K;
      p.push_back({false, 0, [c, &b, cur, a, wsB, cnt, hh, K, lc] {
        const unsigned nU = (unsigned)(hh / jwv::kTailTB);
        const jwv::TailArgs ta{cur, a.dst, wsB, cnt, jwv::tail_last_old(c->tail_base, nU),
                               hh, K, lc};
        c->tail_dirty = true;
        ProfScope ps_(c, K_FWT_FWD_TAIL, 16.0 * hh);
        hipchk(use_fma(c) ? jwv::fused::fwt_fwd_tail(b, ta, c->stream)
                          : jwv::exact::fwt_fwd_tail(b, ta, c->stream), "fwt_fwd_tail");
        c->tail_base = jwv::tail_next_base(c->tail_base, nU);
      }});
      return p;
    }
    const bool last = K == rem;
    if (seg && last && (h >> K) > sw) return {};
    double* ad = last ? a.dst : ws[pp].p;
    const AxisView av = last ? a.dv : cview(h >> K, a.inner);
    jwv::TileArgs t{cur, cv, nullptr, {}, a.dst, a.dv, ad, av, h, K, a.outer, a.inner,
                    dma_view(cur, cv, C, a.inner),
                    Geo::tile_walk(),
                    first1 && h == a.len && Geo::fwd1_first_t() != Geo::kFwt1T
                        ? Geo::fwd1_first_t() : 0};
    t.lsw = a.lsw;
    t.ss = a.ss;
    const int kind = h == a.len ? K_FWT_FWD_TILE : K_FWT_FWD_TILE_DEEP;
    const double bytes = 16.0 * a.outer * h * a.inner;
    p.push_back({false, 0, [c, &b, C, t, kind, bytes] {
      ProfScope ps_(c, kind, bytes);
      hipchk(jwv::launch_fwt_fwd_tile(b, use_fma(c), C, t, c->stream), "fwt_fwd_tile");
    }});
    cur = ad;
    cv = av;
    h >>= K;
    rem -= K;
    pp ^= 1;
  }
  if (rem > 0) {
    if (seg && h > sw) return {};
    const jwv::ResArgs r{cur, cv, a.dst, a.dv, h, 0, rem, a.outer, a.inner,
                         dma_view(cur, cv, C, a.inner)};
    const double bytes = 16.0 * a.outer * h * a.inner;
    p.push_back({true, h, [c, &b, C, r, bytes] {
      ProfScope ps_(c, K_FWT_FWD_RES, bytes);
      hipchk(jwv::launch_fwt_fwd_res(b, use_fma(c), C, r, c->stream), "fwt_fwd_res");
    }});
  }
  return p;
}

void fwt_fwd_axis(jwv_ctx* c, const Bank& b, const Axis& a, int level) {
  run_plan(fwt_fwd_plan(c, b, a, level, c->ws));
}

// FastWaveletTransform.reverse's level loop (FastWaveletTransform.java:137-149).
Plan fwt_rev_plan(jwv_ctx* c, const Bank& b, const Axis& a, int level, DevBuf* ws) {
  Plan p;
  const int h = rev_first(a.len, b.tw, level);
  if (h == 0 && a.lsw < 31) return {};
  if (h == 0) {
    p.push_back({false, 0, [c, a] { copy_axis(c, a); }});
    return p;
  }
  if (auto f = rev_chain_step(c, b, a, h)) {
    p.push_back({false, 0, f});
    return p;
  }
  const int C = col_slab(a.inner);
  // fwt1 path, signal longer than one resident block: the resident tail stops
  // at kFwt1RevTail and the tiled passes take up to kFwt1KMax levels
  const bool f1 = fast1(b, a, true) && a.len > fwt_res_cap(C, a.outer);
  // segmented input (see fwt_fwd_plan): C = 1 tiles, the resident part's
  // prefix inside the first segment; else an empty plan
  const bool seg = a.lsw < 31;
  const int sw = seg ? 1 << a.lsw : 0;
  if (seg && (!f1 || a.outer < 2)) return {};
  // batches of rows: the resident part stops at rev_row_tail(), one long
  // signal at kFwt1RevTail (the REV_HEAD plan)
  const int cap = f1 ? (a.outer > 1 ? rev_row_tail() : Geo::kFwt1RevTail) : Geo::res_cap(C);
  const int KM = f1 ? Geo::kFwt1KMax : Geo::fwt_k(C);
  // workspace sizing
  {
    size_t need = 0;
    int h1;
    if (h <= cap) {
      const int hres = std::min(a.len, cap);
      if (hres < a.len) need = (size_t)a.outer * hres * a.inner;
      h1 = hres * 2;
    } else {
      h1 = h;
    }
    while (h1 <= a.len) {
      const int K = std::min(exponent(a.len / h1) + 1, KM);
      const int hK = h1 << (K - 1);
      if (hK < a.len) need = std::max(need, (size_t)a.outer * hK * a.inner);
      h1 = hK * 2;
    }
    if (need) { grow(c, ws[0], need); grow(c, ws[1], need); }
  }
  const double* acur;
  AxisView acv;
  int h1, pp = 0;
  // JWV_PLAN_REV_HEAD: the resident pass and the first tiled pass (kFwt1KMax
  // levels, fwt1 geometry) fused into one launch (fwt_rev_head1); the
  // remaining tiled passes follow as below.
  if (f1 && h <= cap && a.outer == 1 && (plan_of(c) & JWV_PLAN_REV_HEAD) &&
      cap == Geo::kFwt1RevTail && Geo::kFwt1KMax == ChainGeo::kKM &&
      ((int64_t)cap << ChainGeo::kKM) <= a.len) {
    const int hM = cap << ChainGeo::kKM;
    const bool last = hM == a.len;
    double* out = last ? a.dst : ws[1].p;
    const jwv::RevHeadArgs ra{a.src, out, h, exponent(cap / h) + 1};
    p.push_back({false, 0, [c, &b, ra, hM] {
      ProfScope ps_(c, K_FWT_REV_HEAD, 16.0 * hM);
      hipchk(jwv::launch_fwt_rev_head(b, use_fma(c), ra, c->stream), "fwt_rev_head");
    }});
    if (last) return p;
    acur = out;
    acv = cview(hM, 1);
    h1 = hM * 2;
  } else if (h <= cap) {
    const int hres = std::min(a.len, cap);
    const int nres = exponent(hres / h) + 1;
    const bool last = hres == a.len;
    if (seg && hres > sw) return {};
    double* out = last ? a.dst : ws[pp].p;
    const AxisView ov = last ? a.dv : cview(hres, a.inner);
    const jwv::ResArgs r{a.src, a.sv, out, ov, h, 0, nres, a.outer, a.inner,
                         dma_view(a.src, a.sv, C, a.inner)};
    const double bytes = 16.0 * a.outer * hres * a.inner;
    p.push_back({true, hres, [c, &b, C, r, bytes] {
      ProfScope ps_(c, K_FWT_REV_RES, bytes);
      hipchk(jwv::launch_fwt_rev_res(b, use_fma(c), C, r, c->stream), "fwt_rev_res");
    }});
    if (last) return p;
    acur = out;
    acv = ov;
    h1 = hres * 2;
    pp ^= 1;
  } else {
    if (seg) return {};  // the first tile pass would read approximations from src
    acur = a.src;
    acv = a.sv;
    h1 = h;
  }
  while (h1 <= a.len) {
    const int K = std::min(exponent(a.len / h1) + 1, KM);
    const int hK = h1 << (K - 1);
    const bool last = hK == a.len;
    double* out = last ? a.dst : ws[pp].p;
    const AxisView ov = last ? a.dv : cview(hK, a.inner);
    jwv::TileArgs t{acur, acv, a.src, a.sv, out, ov, nullptr, {}, h1, K, a.outer, a.inner,
                    dma_view(acur, acv, C, a.inner) && dma_view(a.src, a.sv, C, a.inner),
                    (last ? store_pol_dir(1, a.outer == 1 && a.inner == 1) : 0) |
                        Geo::tile_walk()};
    t.lsw = a.lsw;
    t.ss = a.ss;
    const int kind = last ? K_FWT_REV_TILE : K_FWT_REV_TILE_DEEP;
    const double bytes = 16.0 * a.outer * hK * a.inner;
    p.push_back({false, 0, [c, &b, C, t, kind, bytes] {
      ProfScope ps_(c, kind, bytes);
      hipchk(jwv::launch_fwt_rev_tile(b, use_fma(c), C, t, c->stream), "fwt_rev_tile");
    }});
    acur = out;
    acv = ov;
    h1 = hK * 2;
    pp ^= 1;
  }
  return p;
}

void fwt_rev_axis(jwv_ctx* c, const Bank& b, const Axis& a, int level) {
  run_plan(fwt_rev_plan(c, b, a, level, c->ws));
}

// ------------------------------------------------------------------ WPT axis
struct WPass {
  bool tiled;
  int h;    // fwd: packet length at pass start; rev: packet length the pass works on
  int h0;   // rev resident: first packet size
  int nlev; // levels (K for tiled)
  int pk;   // packets per signal
};

void run_wpt_passes(jwv_ctx* c, const Bank& b, const Axis& a, bool fwd,
                    const std::vector<WPass>& ps) {
  const int C = col_slab(a.inner);
  const int P = (int)ps.size();
  if (P > 1) grow(c, c->big2, (size_t)a.outer * a.len * a.inner);
  const double* cur = a.src;
  AxisView cv = a.sv;
  for (int i = 0; i < P; ++i) {
    const WPass& p = ps[i];
    const bool to_dst = ((P - 1 - i) % 2) == 0;
    double* out = to_dst ? a.dst : c->big2.p;
    const AxisView ov = to_dst ? a.dv : cview(a.len, a.inner);
    const AxisView sv = with_packets(cv, p.pk, p.h), dv = with_packets(ov, p.pk, p.h);
    const int64_t nouter = a.outer * p.pk;
    if (p.tiled) {
      jwv::TileArgs t{cur, sv, nullptr, {}, out, dv, nullptr, {}, p.h, p.nlev, nouter, a.inner,
                      dma_view(cur, sv, C, a.inner)};
      ProfScope ps_(c, fwd ? K_WPT_FWD_TILE : K_WPT_REV_TILE, 16.0 * a.outer * a.len * a.inner);
      hipchk(fwd ? jwv::launch_wpt_fwd_tile(b, use_fma(c), C, t, c->stream)
                 : jwv::launch_wpt_rev_tile(b, use_fma(c), C, t, c->stream),
             "wpt_tile");
    } else {
      jwv::ResArgs r{cur, sv, out, dv, p.h, p.h0, p.nlev, nouter, a.inner,
                     dma_view(cur, sv, C, a.inner)};
      ProfScope ps_(c, fwd ? K_WPT_FWD_RES : K_WPT_REV_RES, 16.0 * a.outer * a.len * a.inner);
      hipchk(fwd ? jwv::launch_wpt_fwd_res(b, use_fma(c), C, r, c->stream)
                 : jwv::launch_wpt_rev_res(b, use_fma(c), C, r, c->stream),
             "wpt_res");
    }
    cur = out;
    cv = ov;
  }
}

void wpt_fwd_axis(jwv_ctx* c, const Bank& b, const Axis& a, int level) {
  const int nlev = fwd_levels(a.len, b.tw, level);
  if (nlev == 0) return copy_axis(c, a);
  const int C = col_slab(a.inner), cap = Geo::res_cap(C), KM = Geo::wpt_k(C);
  std::vector<WPass> ps;
  int h = a.len, pk = 1, rem = nlev;
  while (rem > 0) {
    if (h <= cap) {
      ps.push_back({false, h, 0, rem, pk});
      break;
    }
    const int K = std::min(rem, KM);
    ps.push_back({true, h, 0, K, pk});
    h >>= K;
    pk <<= K;
    rem -= K;
  }
  run_wpt_passes(c, b, a, true, ps);
}

// wpt1 kernels (launch_fwt1.hip) take every tiled WPT pass of this axis:
// contiguous 16-B aligned rows and packets, compiled-in tap count, unscaled
// synthesis bank (mirrors wpt_tile1's checks).
bool fastw(const Bank& b, const Axis& a, bool rev) {
  if (!Geo::fwt1() || a.inner != 1 || jwv::static_l(b.L) == 0) return false;
  if (rev && b.scale != 1.0) return false;
  if (a.sv.s_len != 1 || a.dv.s_len != 1 || (a.sv.s_outer & 1) || (a.dv.s_outer & 1)) return false;
  if (((uintptr_t)a.src & 15) || ((uintptr_t)a.dst & 15)) return false;
  return true;
}

void wpt_rev_axis(jwv_ctx* c, const Bank& b, const Axis& a, int level) {
  const int h = rev_first(a.len, b.tw, level);
  if (h == 0) return copy_axis(c, a);
  const int C = col_slab(a.inner), cap = Geo::res_cap(C), KM = Geo::wpt_k(C);
  std::vector<WPass> ps;
  if (fastw(b, a, true) && a.len >= Geo::kWpt1T) {
    // passes from the top: K = min(levels left, kWpt1KMax) ending at packet
    // size hK while hK >= the tile; the rest (packets < tile <= cap) resident
    std::vector<WPass> top;
    int nl = exponent(a.len / h) + 1, hK = a.len;
    while (nl > 0) {
      if (hK < Geo::kWpt1T) {
        top.push_back({false, hK, h, nl, a.len / hK});
        break;
      }
      const int K = std::min(nl, Geo::kWpt1KMax);
      top.push_back({true, hK, 0, K, a.len / hK});
      nl -= K;
      hK >>= K;
    }
    ps.assign(top.rbegin(), top.rend());
    return run_wpt_passes(c, b, a, false, ps);
  }
  int h1;
  if (h <= cap) {
    const int hres = std::min(a.len, cap);
    ps.push_back({false, hres, h, exponent(hres / h) + 1, a.len / hres});
    h1 = hres * 2;
  } else {
    h1 = h;
  }
  while (h1 <= a.len) {
    const int K = std::min(exponent(a.len / h1) + 1, KM);
    const int hK = h1 << (K - 1);
    ps.push_back({true, hK, 0, K, a.len / hK});
    h1 = hK * 2;
  }
  run_wpt_passes(c, b, a, false, ps);
}

// ------------------------------------------------------------- validation
enum class Kind { FWT, WPT };

void check_1d(Kind k, bool fwd, int64_t n, int level) {
  if (n > (int64_t(1) << 30))
    throw Fail{JWV_ERR_BAD_CALL, "signal length exceeds the Java int array range (2^30)"};
  const char* who = k == Kind::FWT ? (fwd ? "FastWaveletTransform#forward - "
                                          : "FastWaveletTransform#reverse - ")
                                   : "";
  if (!is_binary(n))
    throw Fail{JWV_ERR_FAILURE,
               std::string(who) +
                   "given array length is not 2^p | p E N ... = 1, 2, 4, 8, 16, 32, .. "
                   "please use the Ancient Egyptian Decomposition for any other array length!"};
  const int levels = exponent(n);
  if (level < 0 || level > levels) {
    if (k == Kind::FWT)
      throw Fail{JWV_ERR_FAILURE, std::string(who) + "given level is out of range for given array"};
    throw Fail{JWV_ERR_FAILURE, std::string("WaveletPacketTransform#") +
                                    (fwd ? "forward" : "reverse") +
                                    " - given level is out of range for given array"};
  }
}

void check_ptrs(const void* x, const void* y) {
  if (!x || !y) throw Fail{JWV_ERR_BAD_CALL, "NULL data pointer"};
}

void check_overlap(const double* x, size_t nx, const double* y, size_t ny) {
  const char* xa = (const char*)x;
  const char* ya = (const char*)y;
  if (xa < ya + ny * sizeof(double) && ya < xa + nx * sizeof(double))
    throw Fail{JWV_ERR_BAD_CALL, "output buffer overlaps input buffer"};
}

// The calling thread's current device, restored when the entry returns: a
// caller (torch, another library) working on another device is not silently
// re-pointed at the context's.
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) hipchk(hipSetDevice(dev), "hipSetDevice");
  }
  ~DeviceScope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

template <typename F>
int guarded(jwv_ctx* c, F&& f) {
  if (!c) return set_err(nullptr, JWV_ERR_BAD_CALL, "jwv_ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  try {
    c->err.clear();
    DeviceScope ds(c->device);
    if (c->tail_dirty && !tail_resync(c))  // an earlier failure's reset did not complete
      throw Fail{JWV_ERR_DEVICE, "context unusable: resetting the fused-tail counter failed"};
    f();
    c->tail_dirty = false;
    return JWV_OK;
  } catch (const Fail& e) {
    tail_resync(c);
    return set_err(c, e.code, e.msg);
  } catch (const std::exception& e) {
    tail_resync(c);
    return set_err(c, JWV_ERR_DEVICE, e.what());
  }
}

// After the stream has drained: a launch whose bounded in-kernel wait gave up
// (fwt_rev_chain1, only if its grid was not co-resident) left its timeout word
// set; its results are invalid -> JWV_ERR_DEVICE (JWaveError), word cleared.
void check_waits(jwv_ctx* c) {
  if (!c->waited || !c->sync) return;
  c->waited = false;
  unsigned* tmo = c->sync + ChainGeo::kWords;
  unsigned v = 0;
  hipchk(hipMemcpy(&v, tmo, sizeof(v), hipMemcpyDeviceToHost), "timeout word");
  if (v) {
    hipchk(hipMemset(tmo, 0, sizeof(v)), "timeout word");
    throw Fail{JWV_ERR_DEVICE, "chained reverse FWT: an in-kernel wait timed out (grid not "
                               "co-resident?); results of that call are invalid"};
  }
}

// Page-locked host memory (hipHostMalloc / hipHostRegister): DMA-able as is.
bool host_pinned(const void* p) {
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // plain pageable memory
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

PinRing& pin_ring(jwv_ctx* c) {
  PinRing& r = c->pin;
  if (!r.p[0]) {
    for (int i = 0; i < kPinSlots; ++i) {
      hipchk(hipHostMalloc((void**)&r.p[i], kPinChunk, hipHostMallocDefault), "hipHostMalloc");
      if (!r.ev[i])
        hipchk(hipEventCreateWithFlags(&r.ev[i], hipEventDisableTiming), "hipEventCreate");
    }
  }
  return r;
}

// Chunks of a staged transfer.  Only the first inbound copy (nothing to
// overlap it yet) and the last outbound copy (its DMA was the last one) are
// exposed, so the ends ramp: 4, 8, 16 MiB, then 32 MiB slots (ramp_up), and
// the mirror image on the way out.  With the streaming-store copies running
// faster than the link (~74 vs ~56 GB/s), those ends were ~0.9 ms of a
// 2 x 128 MiB call.
struct Chunk {
  size_t off, len;
};
std::vector<Chunk> stage_chunks(size_t bytes, bool ramp_up) {
  std::vector<size_t> len;
  size_t left = bytes, want = kPinChunk >> 3;
  while (left > 0) {
    const size_t l = std::min(left, want);
    len.push_back(l);
    left -= l;
    want = std::min(kPinChunk, want * 2);
  }
  if (!ramp_up) std::reverse(len.begin(), len.end());
  std::vector<Chunk> out;
  size_t off = 0;
  for (size_t l : len) {
    out.push_back({off, l});
    off += l;
  }
  return out;
}

// host x -> device dx (queued on the stream; returns when x may be reused)
void copy_in(jwv_ctx* c, const double* x, double* dx, size_t n) {
  const size_t bytes = n * sizeof(double);
  if (host_pinned(x)) {
    hipchk(hipMemcpyAsync(dx, x, bytes, hipMemcpyHostToDevice, c->stream), "H2D");
    return;
  }
  PinRing& r = pin_ring(c);
  const std::vector<Chunk> ch = stage_chunks(bytes, true);
  for (size_t k = 0; k < ch.size(); ++k) {
    const int s = (int)(k % kPinSlots);
    const size_t off = ch[k].off, len = ch[k].len;
    const double t0 = now_s();
    hipchk(hipEventSynchronize(r.ev[s]), "staging slot");  // its previous DMA is done
    const double t1 = now_s();
    copy_pool().copy(r.p[s], (const char*)x + off, len);
    r.stat[1] += t1 - t0;
    r.stat[0] += now_s() - t1;
    hipchk(hipMemcpyAsync((char*)dx + off, r.p[s], len, hipMemcpyHostToDevice, c->stream), "H2D");
    hipchk(hipEventRecord(r.ev[s], c->stream), "hipEventRecord");
  }
  r.stat[4] += (double)bytes;
}

// device dy -> host y, after the queued work; returns when y is complete
void copy_out(jwv_ctx* c, const double* dy, double* y, size_t n) {
  const size_t bytes = n * sizeof(double);
  if (host_pinned(y)) {
    hipchk(hipMemcpyAsync(y, dy, bytes, hipMemcpyDeviceToHost, c->stream), "D2H");
    hipchk(hipStreamSynchronize(c->stream), "sync");
    return;
  }
  PinRing& r = pin_ring(c);
  const std::vector<Chunk> ch = stage_chunks(bytes, false);
  const size_t nk = ch.size();
  auto issue = [&](size_t k) {
    const int s = (int)(k % kPinSlots);
    const size_t off = ch[k].off, len = ch[k].len;
    hipchk(hipMemcpyAsync(r.p[s], (const char*)dy + off, len, hipMemcpyDeviceToHost, c->stream),
           "D2H");
    hipchk(hipEventRecord(r.ev[s], c->stream), "hipEventRecord");
  };
  for (size_t k = 0; k < std::min<size_t>(nk, kPinSlots); ++k) issue(k);
  for (size_t k = 0; k < nk; ++k) {
    const int s = (int)(k % kPinSlots);
    const size_t off = ch[k].off, len = ch[k].len;
    const double t0 = now_s();
    hipchk(hipEventSynchronize(r.ev[s]), "staging slot");
    const double t1 = now_s();
    copy_pool().copy((char*)y + off, r.p[s], len);
    r.stat[2] += t1 - t0;
    r.stat[3] += now_s() - t1;
    if (k + kPinSlots < nk) issue(k + kPinSlots);
  }
  r.stat[5] += (double)bytes;
  hipchk(hipStreamSynchronize(c->stream), "sync");
}

// Row-strided host side (a column slab of a row-major host matrix): nrows
// rows of w doubles at a pitch of `pitch` doubles <-> a contiguous [nrows][w]
// device block.  Same pinned ring and ramped ends as copy_in / copy_out, in
// whole rows per chunk.
std::vector<Chunk> stage_row_chunks(size_t nrows, size_t w, bool ramp_up) {
  const size_t rb = w * sizeof(double);
  const size_t full = std::max<size_t>(1, kPinChunk / rb);
  size_t want = std::max<size_t>(1, full >> 3), left = nrows;
  std::vector<size_t> len;
  while (left > 0) {
    const size_t l = std::min(left, want);
    len.push_back(l);
    left -= l;
    want = std::min(full, want * 2);
  }
  if (!ramp_up) std::reverse(len.begin(), len.end());
  std::vector<Chunk> out;
  size_t r0 = 0;
  for (size_t l : len) {
    out.push_back({r0, l});
    r0 += l;
  }
  return out;
}
void copy_in2d(jwv_ctx* c, const double* x, size_t pitch, size_t nrows, size_t w, double* dx) {
  const size_t rb = w * sizeof(double);
  if (host_pinned(x)) {
    hipchk(hipMemcpy2DAsync(dx, rb, x, pitch * sizeof(double), rb, nrows, hipMemcpyHostToDevice,
                            c->stream), "H2D 2D");
    return;
  }
  if (rb > kPinChunk) {  // rows longer than a slot: row by row
    for (size_t r = 0; r < nrows; ++r) copy_in(c, x + r * pitch, dx + r * w, w);
    return;
  }
  PinRing& r = pin_ring(c);
  const std::vector<Chunk> ch = stage_row_chunks(nrows, w, true);
  for (size_t k = 0; k < ch.size(); ++k) {
    const int s = (int)(k % kPinSlots);
    const double t0 = now_s();
    hipchk(hipEventSynchronize(r.ev[s]), "staging slot");
    const double t1 = now_s();
    copy_pool().copy2d(r.p[s], rb, x + ch[k].off * pitch, pitch * sizeof(double), rb, ch[k].len);
    r.stat[1] += t1 - t0;
    r.stat[0] += now_s() - t1;
    hipchk(hipMemcpyAsync(dx + ch[k].off * w, r.p[s], ch[k].len * rb, hipMemcpyHostToDevice,
                          c->stream), "H2D");
    hipchk(hipEventRecord(r.ev[s], c->stream), "hipEventRecord");
  }
  r.stat[4] += (double)(rb * nrows);
}
void copy_out2d(jwv_ctx* c, const double* dy, size_t nrows, size_t w, double* y, size_t pitch) {
  const size_t rb = w * sizeof(double);
  if (host_pinned(y)) {
    hipchk(hipMemcpy2DAsync(y, pitch * sizeof(double), dy, rb, rb, nrows, hipMemcpyDeviceToHost,
                            c->stream), "D2H 2D");
    hipchk(hipStreamSynchronize(c->stream), "sync");
    return;
  }
  if (rb > kPinChunk) {
    for (size_t r = 0; r < nrows; ++r) copy_out(c, dy + r * w, y + r * pitch, w);
    return;
  }
  PinRing& r = pin_ring(c);
  const std::vector<Chunk> ch = stage_row_chunks(nrows, w, false);
  const size_t nk = ch.size();
  auto issue = [&](size_t k) {
    const int s = (int)(k % kPinSlots);
    hipchk(hipMemcpyAsync(r.p[s], dy + ch[k].off * w, ch[k].len * rb, hipMemcpyDeviceToHost,
                          c->stream), "D2H");
    hipchk(hipEventRecord(r.ev[s], c->stream), "hipEventRecord");
  };
  for (size_t k = 0; k < std::min<size_t>(nk, kPinSlots); ++k) issue(k);
  for (size_t k = 0; k < nk; ++k) {
    const int s = (int)(k % kPinSlots);
    const double t0 = now_s();
    hipchk(hipEventSynchronize(r.ev[s]), "staging slot");
    const double t1 = now_s();
    copy_pool().copy2d(y + ch[k].off * pitch, pitch * sizeof(double), r.p[s], rb, rb, ch[k].len);
    r.stat[2] += t1 - t0;
    r.stat[3] += now_s() - t1;
    if (k + kPinSlots < nk) issue(k + kPinSlots);
  }
  r.stat[5] += (double)(rb * nrows);
  hipchk(hipStreamSynchronize(c->stream), "sync");
}

// Host-pointer wrapper: stage in / run device body / stage out, synchronous.
template <typename Body>
void staged(jwv_ctx* c, const double* x, size_t nx, double* y, size_t ny, Body&& body) {
  double* dx = grow(c, c->hin, nx);
  double* dy = grow(c, c->hout, ny);
  copy_in(c, x, dx, nx);
  body(dx, dy);
  copy_out(c, dy, y, ny);
  check_waits(c);
}

// ----------------------------------------------------------------- bodies
void body_1d(jwv_ctx* c, Kind k, bool fwd, const Bank& b, const double* x, double* y,
             int64_t batch, int64_t n, int64_t ld, int level) {
  if (batch == 0 || n == 0) return;
  AxisView v{};
  v.s_outer = ld;
  v.s_len = 1;
  v.pk = 1;
  Axis a{x, v, y, v, batch, (int)n, 1};
  if (k == Kind::FWT) (fwd ? fwt_fwd_axis : fwt_rev_axis)(c, b, a, level);
  else (fwd ? wpt_fwd_axis : wpt_rev_axis)(c, b, a, level);
}

using AxisFn = void (*)(jwv_ctx*, const Bank&, const Axis&, int);

AxisFn axis_fn(Kind k, bool fwd) {
  if (k == Kind::FWT) return fwd ? fwt_fwd_axis : fwt_rev_axis;
  return fwd ? wpt_fwd_axis : wpt_rev_axis;
}

// BasicTransform.java:361-399 (forward: rows lvlN -> columns lvlM) and
// :436-474 (reverse: columns lvlM -> rows lvlN).
void body_2d(jwv_ctx* c, Kind k, bool fwd, const Bank& b, const double* x, double* y,
             int64_t rows, int64_t cols, int lvl_m, int lvl_n) {
  if (rows == 0 || cols == 0) return;
  double* tmp = grow(c, c->big, (size_t)(rows * cols));
  const AxisView rv = cview(cols, 1), cvw = cview(rows, cols);
  AxisFn f = axis_fn(k, fwd);
  if (fwd) {
    f(c, b, Axis{x, rv, tmp, rv, rows, (int)cols, 1}, lvl_n);
    f(c, b, Axis{tmp, cvw, y, cvw, 1, (int)rows, (int)cols}, lvl_m);
  } else {
    f(c, b, Axis{x, cvw, tmp, cvw, 1, (int)rows, (int)cols}, lvl_m);
    f(c, b, Axis{tmp, rv, y, rv, rows, (int)cols, 1}, lvl_n);
  }
}

// BasicTransform.java:509-560 / 602-659: slice 2-D transform with (lvlP on the
// Q axis, lvlQ on the R axis), then the P axis with lvlR.  pt: the reverse in
// ParallelTransform's order (ParallelTransform.java:183-216): the P axis
// first, then the slices.
void body_3d(jwv_ctx* c, Kind k, bool fwd, const Bank& b, const double* x, double* y, int64_t P,
             int64_t Q, int64_t R, int lvl_p, int lvl_q, int lvl_r, bool pt = false) {
  if (P == 0 || Q == 0 || R == 0) return;
  double* tmp = grow(c, c->big, (size_t)(P * Q * R));
  const AxisView vr = cview(R, 1), vq = cview(Q, R), vp = cview(P, Q * R);
  AxisFn f = axis_fn(k, fwd);
  if (fwd) {
    f(c, b, Axis{x, vr, y, vr, P * Q, (int)R, 1}, lvl_q);          // rows of each slice
    f(c, b, Axis{y, vq, tmp, vq, P, (int)Q, (int)R}, lvl_p);       // columns of each slice
    f(c, b, Axis{tmp, vp, y, vp, 1, (int)P, (int)(Q * R)}, lvl_r); // along i
  } else if (!pt) {
    f(c, b, Axis{x, vq, y, vq, P, (int)Q, (int)R}, lvl_p);         // slice columns
    f(c, b, Axis{y, vr, tmp, vr, P * Q, (int)R, 1}, lvl_q);        // slice rows
    f(c, b, Axis{tmp, vp, y, vp, 1, (int)P, (int)(Q * R)}, lvl_r); // along i
  } else {
    f(c, b, Axis{x, vp, y, vp, 1, (int)P, (int)(Q * R)}, lvl_r);   // along i
    f(c, b, Axis{y, vq, tmp, vq, P, (int)Q, (int)R}, lvl_p);       // slice columns
    f(c, b, Axis{tmp, vr, y, vr, P * Q, (int)R, 1}, lvl_q);        // slice rows
  }
}

// ------------------------------------------------ AncientEgyptianDecomposition
// AncientEgyptianDecomposition.forward / reverse (AncientEgyptianDecomposition.
// java:97-184): pieces of 2^p (MathToolKit.decompose, largest first,
// MathToolKit.java:57-80), each through the wrapped transform's full-depth
// forward / reverse (level p = calcExponent(2^p)).  Pieces up to the resident
// cap go into ONE varlen launch (aed_kernels.hpp); larger ones take their own
// pass plans.
void check_aed(int64_t n) {
  if (n < 1)  // MathToolKit.decompose (:61-64)
    throw Fail{JWV_ERR_FAILURE, "the supported number for decomposition is smaller than one"};
  if (n > 0x7fffffffLL) throw Fail{JWV_ERR_BAD_CALL, "array length exceeds the Java int range"};
}

void body_aed(jwv_ctx* c, Kind k, bool fwd, const Bank& b, const double* x, double* y,
              int64_t n) {
  jwv::VarSegs sg{};
  int64_t off = 0;
  for (int p = 62; p >= 0 && off < n; --p) {
    const int64_t m = int64_t(1) << p;
    if (((n - off) & m) == 0) continue;
    if (m > Geo::kResCap1) {
      body_1d(c, k, fwd, b, x + off, y + off, 1, m, m, p);
    } else {
      const int i = sg.count++;
      sg.n[i] = (int)m;
      sg.off[i] = off;
      if (fwd) {
        sg.h0[i] = (int)m;
        sg.nlev[i] = fwd_levels((int)m, b.tw, p);
      } else {
        const int h = rev_first((int)m, b.tw, p);
        sg.h0[i] = h ? h : (int)m;
        sg.nlev[i] = h ? exponent(m / h) + 1 : 0;
      }
    }
    off += m;
  }
  if (sg.count == 0) return;
  jwv::VarArgs va{x, y, sg};
  { ProfScope ps_(c, K_AED_VARLEN, 16.0 * (double)(n - (sg.count ? sg.off[0] : n)));
    hipchk(jwv::launch_res_varlen(b, use_fma(c), k == Kind::WPT, fwd, va, c->stream),
           "aed_varlen"); }
}

// WaveletTransform.decompose (WaveletTransform.java:136-145): row p =
// forward(x, p), p = 0..log2 n.  Row p is row p-1 with ONE more level applied
// (to the head [0, n >> (p-1)) for the FWT, to every packet of that size for
// the WPT), so each row costs one level plus a copy of the untouched tail —
// the same doubles as p separate forwards.
void body_decompose(jwv_ctx* c, Kind k, const Bank& b, const double* x, double* mat, int64_t n) {
  const int P = exponent(n);
  hipchk(hipMemcpyAsync(mat, x, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, c->stream),
         "decompose row 0");
  for (int p = 1; p <= P; ++p) {
    const int64_t h = n >> (p - 1);
    const double* prev = mat + (int64_t)(p - 1) * n;
    double* cur = mat + (int64_t)p * n;
    if (k == Kind::FWT) {
      body_1d(c, Kind::FWT, true, b, prev, cur, 1, h, h, 1);
      if (h < n)
        hipchk(hipMemcpyAsync(cur + h, prev + h, (size_t)(n - h) * sizeof(double),
                              hipMemcpyDeviceToDevice, c->stream), "decompose tail");
    } else {
      body_1d(c, Kind::FWT, true, b, prev, cur, n / h, h, h, 1);  // Wavelet.forward per packet
    }
  }
}

// ------------------------------------------------------------------ MODWT
// MODWTTransform.initializeFilterCache / normalize (MODWTTransform.java:452-484,
// 599-606); evaluated in the same order, compiled with -ffp-contract=off.
void modwt_filters(const Bank& b, double* g, double* h) {
  auto normalize = [](double* f, int n) {
    double energy = 0.0;
    for (int i = 0; i < n; ++i) energy += f[i] * f[i];
    const double norm = std::sqrt(energy);
    if (norm > 1e-12)
      for (int i = 0; i < n; ++i) f[i] /= norm;
  };
  for (int i = 0; i < b.L; ++i) { g[i] = b.lo[i]; h[i] = b.hi[i]; }
  normalize(g, b.L);
  normalize(h, b.L);
  const double s = std::sqrt(2.0);
  for (int i = 0; i < b.L; ++i) { g[i] = g[i] / s; h[i] = h[i] / s; }
}

Bank modwt_bank(const Bank& b) {
  Bank m;
  m.L = b.L;
  modwt_filters(b, m.lo, m.hi);
  return m;
}

void check_modwt(int64_t n, int J) {
  // MODWTTransform.forwardMODWT checks, :257-282
  if (J < 1)
    throw Fail{JWV_ERR_ILLEGAL_ARGUMENT,
               "MODWTTransform#forwardMODWT - decomposition level must be at least 1, requested: " +
                   std::to_string(J)};
  if (J > 13)
    throw Fail{JWV_ERR_ILLEGAL_ARGUMENT,
               "MODWTTransform#forwardMODWT - maximum supported decomposition level is 13, "
               "requested: " + std::to_string(J)};
  if (n > 0x7fffffffLL) throw Fail{JWV_ERR_BAD_CALL, "signal length exceeds int range"};
  if (n > 0) {
    int theo = 0;
    while ((int64_t(1) << (theo + 1)) <= n) ++theo;
    if (J > theo)
      throw Fail{JWV_ERR_ILLEGAL_ARGUMENT, "Decomposition level " + std::to_string(J) +
                                               " exceeds theoretical limit " +
                                               std::to_string(theo) + " for signal length " +
                                               std::to_string(n)};
  }
}

// The compile-time-geometry MODWT tiles (modwt1_kernels.hpp)
// where they cover the case, else the runtime tiles.
bool modwt_ct() { return true; }

int64_t modwt_halo(int L, int j0, int j1) {
  return (int64_t)(L - 1) * ((int64_t(1) << j1) - (int64_t(1) << (j0 - 1)));
}

// wv rows (W_1 .. W_J, V_J) at stride ldw >= N doubles (ldw = N: the packed
// [J+1][N] layout of the reference's double[][]).
void body_modwt_fwd(jwv_ctx* c, const Bank& b, const double* x, double* wv, int64_t N, int J,
                    int64_t ldw) {
  if (N == 0) return;
  const Bank m = modwt_bank(b);
  grow(c, c->ws[0], (size_t)N);
  grow(c, c->ws[1], (size_t)N);
  const double* vin = x;
  int pp = 0, j0 = 1;
  while (j0 <= J) {
    int j1 = j0 - 1;
    while (j1 + 1 <= J && modwt_halo(m.L, j0, j1 + 1) <= Geo::kModS) ++j1;
    const bool tiled = j1 >= j0;
    if (!tiled) j1 = j0;
    double* vout = (j1 == J) ? wv + (int64_t)J * ldw : c->ws[pp].p;
    jwv::ModwtArgs a{vin, nullptr, wv, vout, ldw, N, j0, j1};
    {
      ProfScope ps_(c, tiled ? K_MODWT_FWD_TILE : K_MODWT_FWD_LEVEL,
                    8.0 * N * (1 + (j1 - j0 + 1) + 1));
      hipError_t e = hipSuccess;
      const bool ct = tiled && modwt_ct() &&
                      (use_fma(c) ? jwv::fused::modwt_fwd1(m, a, c->stream, e)
                                  : jwv::exact::modwt_fwd1(m, a, c->stream, e));
      if (!ct) e = jwv::launch_modwt_fwd(m, use_fma(c), tiled, a, c->stream);
      hipchk(e, "modwt_fwd");
    }
    vin = vout;
    pp ^= 1;
    j0 = j1 + 1;
  }
}

void body_modwt_inv(jwv_ctx* c, const Bank& b, const double* wv, double* x, int64_t N, int J,
                    int64_t ldw) {
  if (N == 0 || J < 1) return;
  const Bank m = modwt_bank(b);
  grow(c, c->ws[0], (size_t)N);
  grow(c, c->ws[1], (size_t)N);
  const double* vin = wv + (int64_t)J * ldw;
  int pp = 0, j1 = J;
  while (j1 >= 1) {
    int j0 = j1 + 1;
    while (j0 - 1 >= 1 && modwt_halo(m.L, j0 - 1, j1) <= Geo::kModS) --j0;
    const bool tiled = j0 <= j1;
    if (!tiled) j0 = j1;
    double* vout = (j0 == 1) ? x : c->ws[pp].p;
    jwv::ModwtArgs a{vin, wv, nullptr, vout, ldw, N, j0, j1};
    {
      ProfScope ps_(c, tiled ? K_MODWT_INV_TILE : K_MODWT_INV_LEVEL,
                    8.0 * N * (1 + (j1 - j0 + 1) + 1));
      hipError_t e = hipSuccess;
      const bool ct = tiled && modwt_ct() &&
                      (use_fma(c) ? jwv::fused::modwt_inv1(m, a, c->stream, e)
                                  : jwv::exact::modwt_inv1(m, a, c->stream, e));
      if (!ct) e = jwv::launch_modwt_inv(m, use_fma(c), tiled, a, c->stream);
      hipchk(e, "modwt_inv");
    }
    vin = vout;
    pp ^= 1;
    j1 = j0 - 1;
  }
}

// A _dev entry's pointers must be device memory of the context's device: a
// kernel launched on device N must never be handed device M's buffers (nor
// host memory).
void check_dev_ptr(jwv_ctx* c, const void* p) {
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    throw Fail{JWV_ERR_BAD_CALL, "_dev entry point: not a HIP device pointer"};
  }
  if (at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeManaged)
    throw Fail{JWV_ERR_BAD_CALL, "_dev entry point given a host pointer"};
  if (at.device != c->device)
    throw Fail{JWV_ERR_BAD_CALL, "device pointer belongs to device " + std::to_string(at.device) +
                                     ", the context to device " + std::to_string(c->device)};
}
void need_device_ptrs(jwv_ctx* c, const double* x, const double* y) {
  check_ptrs(x, y);
  check_dev_ptr(c, x);
  check_dev_ptr(c, y);
}

}  // namespace

// dispatch shims for the two math modes
namespace jwv {
// Plan geometry: the measured defaults.  The alternatives
// these once selected through environment variables were measured slower
// and removed (git history keeps them).
int Geo::fwd_t1() { return kFwtT1; }
int Geo::rev_t1() { return kFwtT1; }
bool Geo::fwt1() { return true; }
// slab-fastest walk of the C = 8 tiles (config 3: 1.76 -> 1.58 ms/step)
int Geo::slab_order() { return 1; }
int Geo::store_pol() { return 0; }
int Geo::tile_desc(int) { return 0; }
// Grouped one-front walk, G = 64 (config 2, one MI355X, alternating runs on
// one box: forward big pass 53.7 -> 46.0 us by rocprofv3, 0.1231-0.1256 ->
// 0.1146-0.1182 ms/step; G = 32 / 128 within noise of 64).
int Geo::tile_walk() { return 8 | (6 << 8); }
int Geo::fwd1_first_t() { return kFwt1T; }
int Geo::fwd1_first_k() { return std::max(1, std::min(kFwt1KMax, kFwtK1)); }
int Geo::fwd1_tail() { return kFwt1FwdTail; }
bool Geo::fwt8() { return true; }
bool Geo::rev_pref() { return false; }
#define JWV_MODE2(name, ...) \
  return fma ? fused::name(__VA_ARGS__) : exact::name(__VA_ARGS__)
int ChainGeo::default_plan() { return JWV_PLAN_REV_HEAD | JWV_PLAN_FWD_TAIL; }
hipError_t launch_fwt_rev_head(const Bank& b, bool fma, const RevHeadArgs& a, hipStream_t s) {
  JWV_MODE2(fwt_rev_head, b, a, s);
}
hipError_t launch_fwt_fwd_chain(const Bank& b, bool fma, const ChainFwdArgs& a, hipStream_t s) {
  JWV_MODE2(fwt_fwd_chain, b, a, s);
}
hipError_t launch_fwt_rev_chain(const Bank& b, bool fma, const ChainRevArgs& a, hipStream_t s) {
  JWV_MODE2(fwt_rev_chain, b, a, s);
}
hipError_t launch_fwt_fwd_res(const Bank& b, bool fma, int C, const ResArgs& a, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (C == 1 && (fma ? fused::fwt_fwd_res1(b, a, s, e) : exact::fwt_fwd_res1(b, a, s, e)))
    return e;
  if (C == 8 && (fma ? fused::fwt_res16(b, a, s, true, e) : exact::fwt_res16(b, a, s, true, e)))
    return e;
  JWV_MODE2(fwt_fwd_res, b, C, a, s);
}
hipError_t launch_fwt_rev_res(const Bank& b, bool fma, int C, const ResArgs& a, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (C == 1 && (fma ? fused::fwt_rev_res1(b, a, s, e) : exact::fwt_rev_res1(b, a, s, e)))
    return e;
  if (C == 8 && (fma ? fused::fwt_res16(b, a, s, false, e) : exact::fwt_res16(b, a, s, false, e)))
    return e;
  JWV_MODE2(fwt_rev_res, b, C, a, s);
}
hipError_t launch_fwt_fwd_tile(const Bank& b, bool fma, int C, const TileArgs& a, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (C == 1 && (fma ? fused::fwt_fwd_tile1(b, a, s, e) : exact::fwt_fwd_tile1(b, a, s, e)))
    return e;
  if (a.lsw < 31) return hipErrorInvalidValue;  // segmented rows: C = 1 tiles only
  if (C == 8 && (fma ? fused::fwt_tile8(b, a, s, true, e) : exact::fwt_tile8(b, a, s, true, e)))
    return e;
  // the generic kernels are compiled for at most fwt_k(C) fused levels
  if (a.K > Geo::fwt_k(C)) return hipErrorInvalidValue;
  JWV_MODE2(fwt_fwd_tile, b, C, a, s);
}
hipError_t launch_fwt_rev_tile(const Bank& b, bool fma, int C, const TileArgs& a, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (C == 1 && (fma ? fused::fwt_rev_tile1(b, a, s, e) : exact::fwt_rev_tile1(b, a, s, e)))
    return e;
  if (a.lsw < 31) return hipErrorInvalidValue;  // segmented rows: C = 1 tiles only
  if (C == 8 && (fma ? fused::fwt_tile8(b, a, s, false, e) : exact::fwt_tile8(b, a, s, false, e)))
    return e;
  if (a.K > Geo::fwt_k(C)) return hipErrorInvalidValue;
  JWV_MODE2(fwt_rev_tile, b, C, a, s);
}
hipError_t launch_wpt_fwd_res(const Bank& b, bool fma, int C, const ResArgs& a, hipStream_t s) {
  JWV_MODE2(wpt_fwd_res, b, C, a, s);
}
hipError_t launch_wpt_rev_res(const Bank& b, bool fma, int C, const ResArgs& a, hipStream_t s) {
  JWV_MODE2(wpt_rev_res, b, C, a, s);
}
hipError_t launch_wpt_fwd_tile(const Bank& b, bool fma, int C, const TileArgs& a, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (C == 1 && (fma ? fused::wpt_tile1(b, a, s, true, e) : exact::wpt_tile1(b, a, s, true, e)))
    return e;
  if (a.K > Geo::wpt_k(C) || a.h < Geo::wpt_t(C)) return hipErrorInvalidValue;
  JWV_MODE2(wpt_fwd_tile, b, C, a, s);
}
hipError_t launch_wpt_rev_tile(const Bank& b, bool fma, int C, const TileArgs& a, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (C == 1 && (fma ? fused::wpt_tile1(b, a, s, false, e) : exact::wpt_tile1(b, a, s, false, e)))
    return e;
  if (a.K > Geo::wpt_k(C) || a.h < Geo::wpt_t(C)) return hipErrorInvalidValue;
  JWV_MODE2(wpt_rev_tile, b, C, a, s);
}
hipError_t launch_res_varlen(const Bank& b, bool fma, bool wpt, bool fwd, const VarArgs& a,
                             hipStream_t s) {
  JWV_MODE2(res_varlen, b, wpt, fwd, a, s);
}
hipError_t launch_modwt_fwd(const Bank& b, bool fma, bool tiled, const ModwtArgs& a,
                            hipStream_t s) {
  JWV_MODE2(modwt_fwd, b, tiled, a, s);
}
hipError_t launch_modwt_inv(const Bank& b, bool fma, bool tiled, const ModwtArgs& a,
                            hipStream_t s) {
  JWV_MODE2(modwt_inv, b, tiled, a, s);
}
}  // namespace jwv

// =================================================================== C ABI
extern "C" {

int jwv_version(void) { return 100; }

int jwv_ctx_create(int device, jwv_ctx** out) {
  if (!out) return set_err(nullptr, JWV_ERR_BAD_CALL, "out is NULL");
  *out = nullptr;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count == 0)
    return set_err(nullptr, JWV_ERR_DEVICE,
                   std::string("no HIP device available: ") + hipGetErrorString(e));
  if (device < 0 || device >= count)
    return set_err(nullptr, JWV_ERR_BAD_CALL, "device index out of range");
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  if ((e = hipSetDevice(device)) != hipSuccess)
    return set_err(nullptr, JWV_ERR_DEVICE, hipGetErrorString(e));
  jwv_ctx* c = new jwv_ctx();
  c->device = device;
  e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);  // the caller's device
  if (e != hipSuccess) {
    delete c;
    return set_err(nullptr, JWV_ERR_DEVICE, hipGetErrorString(e));
  }
  c->stream = c->own;
  *out = c;
  return JWV_OK;
}

int jwv_host_alloc(jwv_ctx* c, int64_t bytes, void** p) {
  return guarded(c, [&] {
    if (!p || bytes < 0) throw Fail{JWV_ERR_BAD_CALL, "jwv_host_alloc: bad arguments"};
    *p = nullptr;
    hipchk(hipHostMalloc(p, (size_t)std::max<int64_t>(bytes, 1), hipHostMallocDefault),
           "hipHostMalloc");
  });
}

int jwv_host_free(jwv_ctx* c, void* p) {
  return guarded(c, [&] {
    if (p) hipchk(hipHostFree(p), "hipHostFree");
  });
}

int jwv_ctx_stage_stats(jwv_ctx* c, double* out, int reset) {
  if (!c || !out) return set_err(c, JWV_ERR_BAD_CALL, "jwv_ctx_stage_stats: NULL argument");
  for (int i = 0; i < 6; ++i) out[i] = c->pin.stat[i];
  if (reset)
    for (int i = 0; i < 6; ++i) c->pin.stat[i] = 0.0;
  return JWV_OK;
}

int jwv_ctx_destroy(jwv_ctx* c) {
  if (!c) return JWV_OK;
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (DevBuf* b : {&c->ws[0], &c->ws[1], &c->big, &c->big2, &c->red, &c->hin, &c->hout})
    if (b->p) (void)hipFree(b->p);
  if (c->sync) (void)hipFree(c->sync);
  for (auto& r : c->recs) { (void)hipEventDestroy(r.e0); (void)hipEventDestroy(r.e1); }
  for (auto e : c->ev_pool) (void)hipEventDestroy(e);
  if (c->switch_ev) (void)hipEventDestroy(c->switch_ev);
  for (int i = 0; i < kPinSlots; ++i) {
    if (c->pin.p[i]) (void)hipHostFree(c->pin.p[i]);
    if (c->pin.ev[i]) (void)hipEventDestroy(c->pin.ev[i]);
  }
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
  if (prev >= 0) (void)hipSetDevice(prev);
  return JWV_OK;
}

const char* jwv_last_error(const jwv_ctx* c) { return c ? c->err.c_str() : g_tls_error.c_str(); }

// Work a context queued on its old stream (workspace reads and writes, the
// fused tail's arrival counter) must finish before anything it queues on the
// new one: the new stream waits on an event recorded on the old one, so
// alternating streams from one context is ordered without a host sync.
static int switch_stream(jwv_ctx* c, hipStream_t s) {
  if (s == c->stream) return JWV_OK;
  return guarded(c, [&] {
    if (!c->switch_ev) HIPCHK(hipEventCreateWithFlags(&c->switch_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(c->switch_ev, c->stream));
    HIPCHK(hipStreamWaitEvent(s, c->switch_ev, 0));
    c->stream = s;
  });
}

int jwv_ctx_set_stream(jwv_ctx* c, void* s) {
  if (!c) return set_err(nullptr, JWV_ERR_BAD_CALL, "jwv_ctx is NULL");
  return switch_stream(c, (hipStream_t)s);  // NULL = the legacy default stream
}

int jwv_ctx_reset_stream(jwv_ctx* c) {
  if (!c) return set_err(nullptr, JWV_ERR_BAD_CALL, "jwv_ctx is NULL");
  return switch_stream(c, c->own);
}

void* jwv_ctx_get_stream(const jwv_ctx* c) { return c ? (void*)c->stream : nullptr; }

int jwv_ctx_set_math(jwv_ctx* c, int mode) {
  if (!c) return set_err(nullptr, JWV_ERR_BAD_CALL, "jwv_ctx is NULL");
  if (mode != JWV_MATH_EXACT && mode != JWV_MATH_FMA)
    return set_err(c, JWV_ERR_BAD_CALL, "unknown math mode");
  c->math = mode;
  return JWV_OK;
}

int jwv_ctx_set_plan(jwv_ctx* c, int flags) {
  if (!c) return set_err(nullptr, JWV_ERR_BAD_CALL, "ctx is NULL");
  if (flags & ~(JWV_PLAN_CHAIN_REV | JWV_PLAN_CHAIN_FWD | JWV_PLAN_REV_HEAD | JWV_PLAN_FWD_TAIL))
    return set_err(c, JWV_ERR_BAD_CALL, "unknown plan flag");
  c->plan = flags;
  return JWV_OK;
}

int jwv_ctx_synchronize(jwv_ctx* c) {
  return guarded(c, [&] {
    hipchk(hipStreamSynchronize(c->stream), "sync");
    check_waits(c);
  });
}

int jwv_ctx_set_poll_limit(jwv_ctx* c, unsigned spins) {
  if (!c) return set_err(nullptr, JWV_ERR_BAD_CALL, "jwv_ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  c->poll_limit = spins ? spins : (1u << 22);
  return JWV_OK;
}

int jwv_ctx_profile_enable(jwv_ctx* c, int on) {
  if (!c) return set_err(nullptr, JWV_ERR_BAD_CALL, "jwv_ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  c->prof = on != 0;
  return JWV_OK;
}

int jwv_ctx_profile_select(jwv_ctx* c, const char* kind) {
  if (!c) return set_err(nullptr, JWV_ERR_BAD_CALL, "jwv_ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  c->prof_only = -1;
  if (kind && *kind) {
    for (int k = 0; k < K_NKINDS; ++k)
      if (std::strcmp(kind, kKindNames[k]) == 0) c->prof_only = k;
    if (c->prof_only < 0) return set_err(c, JWV_ERR_BAD_CALL, std::string("unknown kernel kind ") + kind);
  }
  return JWV_OK;
}

int jwv_ctx_profile_read(jwv_ctx* c, jwv_kernel_stat* out, int max_out, int* n_out) {
  return guarded(c, [&] {
    hipchk(hipStreamSynchronize(c->stream), "sync");
    jwv_kernel_stat acc[K_NKINDS];
    std::memset(acc, 0, sizeof(acc));
    for (auto& r : c->recs) {
      float ms = 0.f;
      hipchk(hipEventElapsedTime(&ms, r.e0, r.e1), "hipEventElapsedTime");
      acc[r.kind].launches += 1;
      acc[r.kind].total_ms += ms;
      acc[r.kind].bytes += r.bytes;
      c->ev_pool.push_back(r.e0);
      c->ev_pool.push_back(r.e1);
    }
    c->recs.clear();
    int n = 0;
    for (int k = 0; k < K_NKINDS; ++k) {
      if (acc[k].launches == 0) continue;
      std::snprintf(acc[k].name, sizeof(acc[k].name), "%s", kKindNames[k]);
      if (out && n < max_out) out[n] = acc[k];
      ++n;
    }
    if (n_out) *n_out = n;
  });
}

int jwv_ctx_trim(jwv_ctx* c) {
  return guarded(c, [&] {
    hipchk(hipStreamSynchronize(c->stream), "sync");
    for (DevBuf* b : {&c->ws[0], &c->ws[1], &c->big, &c->big2, &c->red, &c->hin, &c->hout}) {
      if (b->p) hipchk(hipFree(b->p), "free");
      b->p = nullptr;
      b->n = 0;
    }
    for (int i = 0; i < kPinSlots; ++i)
      if (c->pin.p[i]) {
        hipchk(hipHostFree(c->pin.p[i]), "hipHostFree");
        c->pin.p[i] = nullptr;
      }
  });
}

// ---- 1-D FWT / WPT ----------------------------------------------------------
#define JWV_1D(NAME, KIND, FWD)                                                                \
  int NAME(const double* x, double* y, int64_t n, int level, const jwv_taps* t, jwv_ctx* c) { \
    return guarded(c, [&] {                                                                    \
      const Bank b = make_bank(t);                                                             \
      check_1d(KIND, FWD, n, level);                                                           \
      check_ptrs(x, y);                                                                        \
      staged(c, x, (size_t)n, y, (size_t)n, [&](const double* dx, double* dy) {               \
        body_1d(c, KIND, FWD, b, dx, dy, 1, n, n, level);                                      \
      });                                                                                      \
    });                                                                                        \
  }                                                                                            \
  int NAME##_dev(const double* x, double* y, int64_t n, int level, const jwv_taps* t,          \
                 jwv_ctx* c) {                                                                 \
    return guarded(c, [&] {                                                                    \
      const Bank b = make_bank(t);                                                             \
      check_1d(KIND, FWD, n, level);                                                           \
      need_device_ptrs(c, x, y);                                                                  \
      check_overlap(x, (size_t)n, y, (size_t)n);                                               \
      body_1d(c, KIND, FWD, b, x, y, 1, n, n, level);                                          \
    });                                                                                        \
  }
JWV_1D(jwv_fwt_fwd_f64, Kind::FWT, true)
JWV_1D(jwv_fwt_rev_f64, Kind::FWT, false)
JWV_1D(jwv_wpt_fwd_f64, Kind::WPT, true)
JWV_1D(jwv_wpt_rev_f64, Kind::WPT, false)

#define JWV_BATCH(NAME, KIND, FWD)                                                              \
  int NAME(const double* x, double* y, int64_t batch, int64_t n, int64_t ld, int level,         \
           const jwv_taps* t, jwv_ctx* c) {                                                     \
    return guarded(c, [&] {                                                                     \
      const Bank b = make_bank(t);                                                              \
      if (batch < 0 || ld < n) throw Fail{JWV_ERR_BAD_CALL, "batch < 0 or ld < n"};             \
      check_1d(KIND, FWD, n, level);                                                            \
      if (batch == 0) return;                                                                   \
      check_ptrs(x, y);                                                                         \
      const size_t tot = (size_t)((batch - 1) * ld + n);                                        \
      staged(c, x, tot, y, tot, [&](const double* dx, double* dy) {                            \
        body_1d(c, KIND, FWD, b, dx, dy, batch, n, ld, level);                                  \
      });                                                                                       \
    });                                                                                         \
  }                                                                                             \
  int NAME##_dev(const double* x, double* y, int64_t batch, int64_t n, int64_t ld, int level,   \
                 const jwv_taps* t, jwv_ctx* c) {                                               \
    return guarded(c, [&] {                                                                     \
      const Bank b = make_bank(t);                                                              \
      if (batch < 0 || ld < n) throw Fail{JWV_ERR_BAD_CALL, "batch < 0 or ld < n"};             \
      check_1d(KIND, FWD, n, level);                                                            \
      if (batch == 0) return;                                                                   \
      need_device_ptrs(c, x, y);                                                                   \
      const size_t tot = (size_t)((batch - 1) * ld + n);                                        \
      check_overlap(x, tot, y, tot);                                                            \
      body_1d(c, KIND, FWD, b, x, y, batch, n, ld, level);                                      \
    });                                                                                         \
  }
JWV_BATCH(jwv_fwt_fwd_batch_f64, Kind::FWT, true)
JWV_BATCH(jwv_fwt_rev_batch_f64, Kind::FWT, false)
JWV_BATCH(jwv_wpt_fwd_batch_f64, Kind::WPT, true)
JWV_BATCH(jwv_wpt_rev_batch_f64, Kind::WPT, false)

// ---- segmented row passes (sharded 2-D transform) ----------------------------------
// The row pass of BasicTransform.java:369-378 (forward) / :461-470 (reverse)
// over a [rows][cols] block whose coefficient side is in the all-to-all layout
// [cols/seg][rows][seg] (chunk j = columns [j seg, (j+1) seg) of every row),
// so the sharded 2-D transform's exchange needs no pack / unpack pass
// (jwave_amd/distributed.py).  Where the row kernels cannot address the
// segments (short rows, seg < 1024, ...) the entry runs the plain row pass
// and packs / unpacks with one copy.
static void check_seg(int64_t rows, int64_t cols, int64_t seg) {
  if (rows < 0 || cols < 0) throw Fail{JWV_ERR_BAD_CALL, "negative dimension"};
  if (seg < 2 || (seg & (seg - 1)) || (cols && cols % seg) || seg > (int64_t(1) << 30))
    throw Fail{JWV_ERR_BAD_CALL, "seg must be a power of two >= 2 dividing cols"};
  if (rows > (int64_t(1) << 30) || rows * cols > (int64_t(1) << 33))
    throw Fail{JWV_ERR_BAD_CALL, "matrix too large"};
}
// [rows][cols] view <-> [cols/seg][rows][seg] copy: outer = chunk, len = row
static Axis seg_pack_axis(const double* plain, double* segd, int64_t rows, int64_t cols,
                          int64_t seg, bool pack) {
  AxisView pv{}, sv{};
  pv.s_outer = seg; pv.s_len = cols; pv.pk = 1;
  sv.s_outer = rows * seg; sv.s_len = seg; sv.pk = 1;
  if (pack) return Axis{plain, pv, segd, sv, cols / seg, (int)rows, (int)seg};
  return Axis{segd, sv, const_cast<double*>(plain), pv, cols / seg, (int)rows, (int)seg};
}

extern "C" int jwv_fwt_rows_seg_fwd_f64_dev(const double* x, double* y, int64_t rows,
                                            int64_t cols, int level, int64_t seg,
                                            const jwv_taps* t, jwv_ctx* c) {
  return guarded(c, [&] {
    const Bank b = make_bank(t);
    check_seg(rows, cols, seg);
    check_1d(Kind::FWT, true, cols, level);
    if (rows == 0 || cols == 0) return;
    need_device_ptrs(c, x, y);
    check_overlap(x, (size_t)(rows * cols), y, (size_t)(rows * cols));
    const AxisView rv = cview(cols, 1);
    AxisView ov = rv;
    ov.s_outer = seg;
    Axis a{x, rv, y, ov, rows, (int)cols, 1};
    a.lsw = exponent(seg);
    a.ss = rows * seg;
    Plan p = fwt_fwd_plan(c, b, a, level, c->ws);
    if (!p.empty()) return run_plan(p);
    double* tmp = grow(c, c->big, (size_t)(rows * cols));
    fwt_fwd_axis(c, b, Axis{x, rv, tmp, rv, rows, (int)cols, 1}, level);
    copy_axis(c, seg_pack_axis(tmp, y, rows, cols, seg, true));
  });
}

extern "C" int jwv_fwt_rows_seg_rev_f64_dev(const double* y, double* x, int64_t rows,
                                            int64_t cols, int level, int64_t seg,
                                            const jwv_taps* t, jwv_ctx* c) {
  return guarded(c, [&] {
    const Bank b = make_bank(t);
    check_seg(rows, cols, seg);
    check_1d(Kind::FWT, false, cols, level);
    if (rows == 0 || cols == 0) return;
    need_device_ptrs(c, y, x);
    check_overlap(y, (size_t)(rows * cols), x, (size_t)(rows * cols));
    const AxisView rv = cview(cols, 1);
    AxisView iv = rv;
    iv.s_outer = seg;
    Axis a{y, iv, x, rv, rows, (int)cols, 1};
    a.lsw = exponent(seg);
    a.ss = rows * seg;
    Plan p = fwt_rev_plan(c, b, a, level, c->ws);
    if (!p.empty()) return run_plan(p);
    double* tmp = grow(c, c->big, (size_t)(rows * cols));
    copy_axis(c, seg_pack_axis(tmp, const_cast<double*>(y), rows, cols, seg, false));
    fwt_rev_axis(c, b, Axis{tmp, rv, x, rv, rows, (int)cols, 1}, level);
  });
}

// ---- 2-D / 3-D -------------------------------------------------------------------
static void check_2d(Kind k, bool fwd, int64_t rows, int64_t cols, int lvl_m, int lvl_n) {
  if (rows < 0 || cols < 0) throw Fail{JWV_ERR_BAD_CALL, "negative dimension"};
  if (rows == 0 || cols == 0) return;
  // forward validates rows first (row pass), reverse the columns first
  if (fwd) { check_1d(k, true, cols, lvl_n); check_1d(k, true, rows, lvl_m); }
  else { check_1d(k, false, rows, lvl_m); check_1d(k, false, cols, lvl_n); }
  if (rows > (int64_t(1) << 30) || rows * cols > (int64_t(1) << 33))
    throw Fail{JWV_ERR_BAD_CALL, "matrix too large"};
}

#define JWV_2D(NAME, KIND, FWD)                                                                  \
  int NAME(const double* x, double* y, int64_t rows, int64_t cols, int lvl_m, int lvl_n,         \
           const jwv_taps* t, jwv_ctx* c) {                                                      \
    return guarded(c, [&] {                                                                      \
      const Bank b = make_bank(t);                                                               \
      check_2d(KIND, FWD, rows, cols, lvl_m, lvl_n);                                             \
      if (rows == 0 || cols == 0) return;                                                        \
      check_ptrs(x, y);                                                                          \
      const size_t tot = (size_t)(rows * cols);                                                  \
      staged(c, x, tot, y, tot, [&](const double* dx, double* dy) {                              \
        body_2d(c, KIND, FWD, b, dx, dy, rows, cols, lvl_m, lvl_n);                              \
      });                                                                                        \
    });                                                                                          \
  }
#define JWV_2D_DEV(NAME, KIND, FWD)                                                              \
  int NAME(const double* x, double* y, int64_t rows, int64_t cols, int lvl_m, int lvl_n,         \
           const jwv_taps* t, jwv_ctx* c) {                                                      \
    return guarded(c, [&] {                                                                      \
      const Bank b = make_bank(t);                                                               \
      check_2d(KIND, FWD, rows, cols, lvl_m, lvl_n);                                             \
      if (rows == 0 || cols == 0) return;                                                        \
      need_device_ptrs(c, x, y);                                                                    \
      check_overlap(x, (size_t)(rows * cols), y, (size_t)(rows * cols));                         \
      body_2d(c, KIND, FWD, b, x, y, rows, cols, lvl_m, lvl_n);                                  \
    });                                                                                          \
  }
// One axis of a contiguous [outer][len][inner] block: the per-dimension pass of
// BasicTransform.java:369-395 (rows: inner = 1; columns: outer = 1).  The
// sharded 2-D transform runs its column pass on a [rows][cols/W] slab with it.
#define JWV_AXIS_DEV(NAME, KIND, FWD)                                                            \
  int NAME(const double* x, double* y, int64_t outer, int64_t len, int64_t inner, int level,    \
           const jwv_taps* t, jwv_ctx* c) {                                                      \
    return guarded(c, [&] {                                                                      \
      const Bank b = make_bank(t);                                                               \
      if (outer < 0 || inner < 0) throw Fail{JWV_ERR_BAD_CALL, "negative dimension"};           \
      check_1d(KIND, FWD, len, level);                                                           \
      if (outer == 0 || len == 0 || inner == 0) return;                                          \
      if (inner > (int64_t(1) << 30)) throw Fail{JWV_ERR_BAD_CALL, "inner dimension too large"}; \
      need_device_ptrs(c, x, y);                                                                    \
      const size_t tot = (size_t)(outer * len * inner);                                          \
      check_overlap(x, tot, y, tot);                                                             \
      const AxisView v = cview(len, inner);                                                      \
      axis_fn(KIND, FWD)(c, b, Axis{x, v, y, v, outer, (int)len, (int)inner}, level);           \
    });                                                                                          \
  }
JWV_AXIS_DEV(jwv_fwt_axis_fwd_f64_dev, Kind::FWT, true)
JWV_AXIS_DEV(jwv_fwt_axis_rev_f64_dev, Kind::FWT, false)
JWV_AXIS_DEV(jwv_wpt_axis_fwd_f64_dev, Kind::WPT, true)
JWV_AXIS_DEV(jwv_wpt_axis_rev_f64_dev, Kind::WPT, false)

JWV_2D(jwv_fwt2d_fwd_f64, Kind::FWT, true)
JWV_2D(jwv_fwt2d_rev_f64, Kind::FWT, false)
JWV_2D_DEV(jwv_fwt2d_fwd_f64_dev, Kind::FWT, true)
JWV_2D_DEV(jwv_fwt2d_rev_f64_dev, Kind::FWT, false)
JWV_2D(jwv_wpt2d_fwd_f64, Kind::WPT, true)
JWV_2D(jwv_wpt2d_rev_f64, Kind::WPT, false)
JWV_2D_DEV(jwv_wpt2d_fwd_f64_dev, Kind::WPT, true)
JWV_2D_DEV(jwv_wpt2d_rev_f64_dev, Kind::WPT, false)

static void check_3d(Kind k, bool fwd, int64_t P, int64_t Q, int64_t R, int lp, int lq, int lr,
                     bool pt = false) {
  if (P < 0 || Q < 0 || R < 0) throw Fail{JWV_ERR_BAD_CALL, "negative dimension"};
  if (P == 0 || Q == 0 || R == 0) return;
  if (pt) {  // ParallelTransform reverse: P axis, then slice columns, slice rows
    check_1d(k, false, P, lr);
    check_1d(k, false, Q, lp);
    check_1d(k, false, R, lq);
  } else if (fwd) {
    check_1d(k, true, R, lq);
    check_1d(k, true, Q, lp);
    check_1d(k, true, P, lr);
  } else {
    check_1d(k, false, Q, lp);
    check_1d(k, false, R, lq);
    check_1d(k, false, P, lr);
  }
  if (P * Q * R > (int64_t(1) << 33)) throw Fail{JWV_ERR_BAD_CALL, "volume too large"};
}

#define JWV_3D(NAME, KIND, FWD, DEV) JWV_3DX(NAME, KIND, FWD, DEV, false)
#define JWV_3DX(NAME, KIND, FWD, DEV, PT)                                                         \
  int NAME(const double* x, double* y, int64_t P, int64_t Q, int64_t R, int lp, int lq, int lr,   \
           const jwv_taps* t, jwv_ctx* c) {                                                       \
    return guarded(c, [&] {                                                                       \
      const Bank b = make_bank(t);                                                                \
      check_3d(KIND, FWD, P, Q, R, lp, lq, lr, PT);                                               \
      if (P == 0 || Q == 0 || R == 0) return;                                                     \
      check_ptrs(x, y);                                                                           \
      const size_t tot = (size_t)(P * Q * R);                                                     \
      if (DEV) {                                                                                  \
        need_device_ptrs(c, x, y);                                                                \
        check_overlap(x, tot, y, tot);                                                            \
        body_3d(c, KIND, FWD, b, x, y, P, Q, R, lp, lq, lr, PT);                                  \
      } else {                                                                                    \
        staged(c, x, tot, y, tot, [&](const double* dx, double* dy) {                             \
          body_3d(c, KIND, FWD, b, dx, dy, P, Q, R, lp, lq, lr, PT);                              \
        });                                                                                       \
      }                                                                                           \
    });                                                                                           \
  }
JWV_3D(jwv_fwt3d_fwd_f64, Kind::FWT, true, false)
JWV_3D(jwv_fwt3d_rev_f64, Kind::FWT, false, false)
JWV_3D(jwv_fwt3d_fwd_f64_dev, Kind::FWT, true, true)
JWV_3D(jwv_fwt3d_rev_f64_dev, Kind::FWT, false, true)
JWV_3D(jwv_wpt3d_fwd_f64, Kind::WPT, true, false)
JWV_3D(jwv_wpt3d_rev_f64, Kind::WPT, false, false)
JWV_3DX(jwv_fwt3d_rev_pt_f64, Kind::FWT, false, false, true)
JWV_3DX(jwv_fwt3d_rev_pt_f64_dev, Kind::FWT, false, true, true)
JWV_3DX(jwv_wpt3d_rev_pt_f64, Kind::WPT, false, false, true)

// ---- CompressorMagnitude / denoise ---------------------------------------------------
namespace {
// Compressor(double threshold) (compressions/Compressor.java:66-80): a
// threshold <= 0 is reported and replaced by the default 1.0.
double compressor_threshold(double t) { return t > 0.0 ? t : 1.0; }

// y = CompressorMagnitude.compress(c) (CompressorMagnitude.java:73-84) on the
// device; the magnitude is copied to *mag (host) when mag != NULL (syncs).
void body_compress(jwv_ctx* c, const double* x, double* y, int64_t n, double threshold,
                   double* mag) {
  if (n == 0) return;
  const int np = jwv::compress_partials(n);
  double* scratch = grow(c, c->red, (size_t)jwv::compress_scratch(n));
  hipchk(jwv::launch_compress_magnitude(x, y, n, compressor_threshold(threshold), scratch,
                                        c->stream),
         "compress_magnitude");
  if (mag) {
    hipchk(hipMemcpyAsync(mag, scratch + np + 1, sizeof(double), hipMemcpyDeviceToHost, c->stream),
           "D2H");
    hipchk(hipStreamSynchronize(c->stream), "sync");
  }
}

// forward (level) -> CompressorMagnitude(threshold) -> reverse (level), all on
// the device: the usual denoising use of Transform + Compressor.
void body_denoise(jwv_ctx* c, const Bank& b, const double* x, double* y, int64_t n, int level,
                  double threshold) {
  if (n == 0) return;
  double* coef = grow(c, c->big, (size_t)n);
  body_1d(c, Kind::FWT, true, b, x, coef, 1, n, n, level);
  body_compress(c, coef, coef, n, threshold, nullptr);
  body_1d(c, Kind::FWT, false, b, coef, y, 1, n, n, level);
}
}  // namespace

int jwv_compress_magnitude_f64(const double* x, double* y, int64_t n, double threshold,
                               double* magnitude, jwv_ctx* c) {
  return guarded(c, [&] {
    if (n < 0) throw Fail{JWV_ERR_BAD_CALL, "n < 0"};
    if (n == 0) return;
    check_ptrs(x, y);
    staged(c, x, (size_t)n, y, (size_t)n,
           [&](const double* dx, double* dy) { body_compress(c, dx, dy, n, threshold, nullptr); });
    if (magnitude) {
      const int np = jwv::compress_partials(n);
      hipchk(hipMemcpy(magnitude, c->red.p + np + 1, sizeof(double), hipMemcpyDeviceToHost), "D2H");
    }
  });
}
int jwv_compress_magnitude_f64_dev(const double* x, double* y, int64_t n, double threshold,
                                   double* magnitude, jwv_ctx* c) {
  return guarded(c, [&] {
    if (n < 0) throw Fail{JWV_ERR_BAD_CALL, "n < 0"};
    if (n == 0) return;
    need_device_ptrs(c, x, y);
    // exact aliasing takes the in-place (classify-first) path; any partial
    // overlap would let the first pass's stores reach inputs of later passes
    if (x != y) check_overlap(x, (size_t)n, y, (size_t)n);
    body_compress(c, x, y, n, threshold, magnitude);
  });
}
int jwv_fwt_denoise_f64(const double* x, double* y, int64_t n, int level, double threshold,
                        const jwv_taps* t, jwv_ctx* c) {
  return guarded(c, [&] {
    const Bank b = make_bank(t);
    check_1d(Kind::FWT, true, n, level);
    if (n == 0) return;
    check_ptrs(x, y);
    staged(c, x, (size_t)n, y, (size_t)n,
           [&](const double* dx, double* dy) { body_denoise(c, b, dx, dy, n, level, threshold); });
  });
}
int jwv_fwt_denoise_f64_dev(const double* x, double* y, int64_t n, int level, double threshold,
                            const jwv_taps* t, jwv_ctx* c) {
  return guarded(c, [&] {
    const Bank b = make_bank(t);
    check_1d(Kind::FWT, true, n, level);
    if (n == 0) return;
    need_device_ptrs(c, x, y);
    body_denoise(c, b, x, y, n, level, threshold);
  });
}

// ---- AncientEgyptianDecomposition / decompose ------------------------------------
static Kind kind_of_transform(int transform) {
  if (transform == JWV_TRANSFORM_FWT) return Kind::FWT;
  if (transform == JWV_TRANSFORM_WPT) return Kind::WPT;
  throw Fail{JWV_ERR_BAD_CALL, "unknown transform (JWV_TRANSFORM_FWT | JWV_TRANSFORM_WPT)"};
}
#define JWV_AED(NAME, FWD, DEV)                                                                 \
  int NAME(const double* x, double* y, int64_t n, int transform, const jwv_taps* t,           \
           jwv_ctx* c) {                                                                       \
    return guarded(c, [&] {                                                                    \
      const Bank b = make_bank(t);                                                             \
      const Kind k = kind_of_transform(transform);                                             \
      check_aed(n);                                                                            \
      if (DEV) {                                                                               \
        need_device_ptrs(c, x, y);                                                             \
        check_overlap(x, (size_t)n, y, (size_t)n);                                             \
        body_aed(c, k, FWD, b, x, y, n);                                                       \
      } else {                                                                                 \
        check_ptrs(x, y);                                                                      \
        staged(c, x, (size_t)n, y, (size_t)n,                                                  \
               [&](const double* dx, double* dy) { body_aed(c, k, FWD, b, dx, dy, n); });      \
      }                                                                                        \
    });                                                                                        \
  }
JWV_AED(jwv_aed_fwd_f64, true, false)
JWV_AED(jwv_aed_rev_f64, false, false)
JWV_AED(jwv_aed_fwd_f64_dev, true, true)
JWV_AED(jwv_aed_rev_f64_dev, false, true)

// BasicTransform#calcExponent's check (BasicTransform.java:688-697)
static void check_decompose(int64_t n) {
  if (!is_binary(n))
    throw Fail{JWV_ERR_FAILURE, "BasicTransform#calcExponent - given number is not binary: "
                                "2^p | pEN .. = 1, 2, 4, 8, 16, 32, .. "};
  if (n > (int64_t(1) << 30))
    throw Fail{JWV_ERR_BAD_CALL, "signal length exceeds the Java int array range (2^30)"};
}
#define JWV_DECOMP(NAME, DEV)                                                                   \
  int NAME(const double* x, double* mat, int64_t n, int transform, const jwv_taps* t,         \
           jwv_ctx* c) {                                                                       \
    return guarded(c, [&] {                                                                    \
      const Bank b = make_bank(t);                                                             \
      const Kind k = kind_of_transform(transform);                                             \
      check_decompose(n);                                                                      \
      const size_t rows = (size_t)exponent(n) + 1;                                             \
      if (DEV) {                                                                               \
        need_device_ptrs(c, x, mat);                                                           \
        check_overlap(x, (size_t)n, mat, rows * (size_t)n);                                    \
        body_decompose(c, k, b, x, mat, n);                                                    \
      } else {                                                                                 \
        check_ptrs(x, mat);                                                                    \
        staged(c, x, (size_t)n, mat, rows * (size_t)n,                                         \
               [&](const double* dx, double* dy) { body_decompose(c, k, b, dx, dy, n); });     \
      }                                                                                        \
    });                                                                                        \
  }
JWV_DECOMP(jwv_decompose_f64, false)
JWV_DECOMP(jwv_decompose_f64_dev, true)

// ---- MODWT -------------------------------------------------------------------------
int jwv_modwt_filters(const jwv_taps* t, double* g, double* h) {
  try {
    const Bank b = make_bank(t);
    if (!g || !h) throw Fail{JWV_ERR_BAD_CALL, "NULL output"};
    modwt_filters(b, g, h);
    return JWV_OK;
  } catch (const Fail& e) {
    return set_err(nullptr, e.code, e.msg);
  }
}

int jwv_modwt_fwd_f64(const double* x, double* wv, int64_t n, int J, const jwv_taps* t,
                      jwv_ctx* c) {
  return guarded(c, [&] {
    const Bank b = make_bank(t);
    check_modwt(n, J);
    if (n == 0) return;
    check_ptrs(x, wv);
    staged(c, x, (size_t)n, wv, (size_t)n * (J + 1),
           [&](const double* dx, double* dy) { body_modwt_fwd(c, b, dx, dy, n, J, n); });
  });
}
int jwv_modwt_fwd_f64_dev(const double* x, double* wv, int64_t n, int J, const jwv_taps* t,
                          jwv_ctx* c) {
  return guarded(c, [&] {
    const Bank b = make_bank(t);
    check_modwt(n, J);
    if (n == 0) return;
    need_device_ptrs(c, x, wv);
    check_overlap(x, (size_t)n, wv, (size_t)n * (J + 1));
    body_modwt_fwd(c, b, x, wv, n, J, n);
  });
}
// MODWTTransform.inverseMODWT: coefficients.length <= 1 -> empty (:338-346).
int jwv_modwt_inv_f64(const double* wv, double* x, int64_t n, int J, const jwv_taps* t,
                      jwv_ctx* c) {
  return guarded(c, [&] {
    const Bank b = make_bank(t);
    if (J < 1 || n == 0) return;
    if (J > 13 || n > 0x7fffffffLL) throw Fail{JWV_ERR_BAD_CALL, "J > 13 or n too large"};
    check_ptrs(wv, x);
    staged(c, wv, (size_t)n * (J + 1), x, (size_t)n,
           [&](const double* dx, double* dy) { body_modwt_inv(c, b, dx, dy, n, J, n); });
  });
}
int jwv_modwt_inv_f64_dev(const double* wv, double* x, int64_t n, int J, const jwv_taps* t,
                          jwv_ctx* c) {
  return guarded(c, [&] {
    const Bank b = make_bank(t);
    if (J < 1 || n == 0) return;
    if (J > 13 || n > 0x7fffffffLL) throw Fail{JWV_ERR_BAD_CALL, "J > 13 or n too large"};
    need_device_ptrs(c, wv, x);
    check_overlap(wv, (size_t)n * (J + 1), x, (size_t)n);
    body_modwt_inv(c, b, wv, x, n, J, n);
  });
}

int jwv_modwt_fwd_ld_f64_dev(const double* x, double* wv, int64_t ldw, int64_t n, int J,
                             const jwv_taps* t, jwv_ctx* c) {
  return guarded(c, [&] {
    const Bank b = make_bank(t);
    check_modwt(n, J);
    if (n == 0) return;
    if (ldw < n) throw Fail{JWV_ERR_BAD_CALL, "ldw < n"};
    need_device_ptrs(c, x, wv);
    check_overlap(x, (size_t)n, wv, (size_t)(J * ldw + n));
    body_modwt_fwd(c, b, x, wv, n, J, ldw);
  });
}
int jwv_modwt_inv_ld_f64_dev(const double* wv, int64_t ldw, double* x, int64_t n, int J,
                             const jwv_taps* t, jwv_ctx* c) {
  return guarded(c, [&] {
    const Bank b = make_bank(t);
    if (J < 1 || n == 0) return;
    if (J > 13 || n > 0x7fffffffLL) throw Fail{JWV_ERR_BAD_CALL, "J > 13 or n too large"};
    if (ldw < n) throw Fail{JWV_ERR_BAD_CALL, "ldw < n"};
    need_device_ptrs(c, wv, x);
    check_overlap(wv, (size_t)(J * ldw + n), x, (size_t)n);
    body_modwt_inv(c, b, wv, x, n, J, ldw);
  });
}

// ---- multi-device batches ----------------------------------------------------
int jwv_batch_split(int64_t batch, int n, int i, int64_t* start, int64_t* count) {
  if (batch < 0 || n < 1 || i < 0 || i >= n || !start || !count)
    return set_err(nullptr, JWV_ERR_BAD_CALL, "jwv_batch_split: bad arguments");
  // floor(batch * k / n) without overflow: (batch / n) * k + (batch % n) * k / n
  auto at = [&](int64_t k) { return (batch / n) * k + (batch % n) * k / n; };
  *start = at(i);
  *count = at(i + 1) - *start;
  return JWV_OK;
}

int jwv_mctx_create(const int* devices, int n, jwv_mctx** out) {
  if (!out) return set_err(nullptr, JWV_ERR_BAD_CALL, "out is NULL");
  *out = nullptr;
  if (!devices || n < 1) return set_err(nullptr, JWV_ERR_BAD_CALL, "no devices given");
  jwv_mctx* m = new jwv_mctx();
  for (int i = 0; i < n; ++i) {
    jwv_ctx* c = nullptr;
    const int rc = jwv_ctx_create(devices[i], &c);
    if (rc != JWV_OK) {
      const std::string why = g_tls_error;
      jwv_mctx_destroy(m);
      return set_err(nullptr, rc, "device " + std::to_string(devices[i]) + ": " + why);
    }
    m->ctx.push_back(c);
  }
  // one staging thread per device shares the process-wide copy pool: size it
  // by the devices in use (16 threads each, within the CPU share)
  copy_pool().grow(std::min(affinity_cpus(), 16 * n) - 1);
  // direct xGMI peer copies for the 2-D exchange where the pair allows it
  // (otherwise hipMemcpyPeerAsync stages through the host)
  int prev = -1;
  if (hipGetDevice(&prev) == hipSuccess) {
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        int can = 0;
        if (devices[i] == devices[j] ||
            hipDeviceCanAccessPeer(&can, devices[i], devices[j]) != hipSuccess || !can)
          continue;
        if (hipSetDevice(devices[i]) == hipSuccess &&
            hipDeviceEnablePeerAccess(devices[j], 0) != hipSuccess)
          (void)hipGetLastError();  // already enabled
      }
    (void)hipSetDevice(prev);
  }
  *out = m;
  return JWV_OK;
}

int jwv_host_copy_threads(void) { return copy_pool().size(); }

int jwv_mctx_destroy(jwv_mctx* m) {
  if (!m) return JWV_OK;
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  for (size_t i = 0; i < m->a.size(); ++i) {
    if (hipSetDevice(m->ctx[i]->device) != hipSuccess) continue;
    (void)hipStreamSynchronize(m->ctx[i]->stream);
    for (DevBuf* d : {&m->a[i], &m->b[i], &m->c[i], &m->t[i]})
      if (d->p) (void)hipFree(d->p);
    if (m->ev[i]) (void)hipEventDestroy(m->ev[i]);
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  for (jwv_ctx* c : m->ctx) jwv_ctx_destroy(c);
  delete m;
  return JWV_OK;
}

const char* jwv_mctx_last_error(const jwv_mctx* m) {
  return m ? m->err.c_str() : g_tls_error.c_str();
}

int jwv_mctx_size(const jwv_mctx* m) { return m ? (int)m->ctx.size() : 0; }

jwv_ctx* jwv_mctx_ctx(jwv_mctx* m, int i) {
  return (m && i >= 0 && i < (int)m->ctx.size()) ? m->ctx[i] : nullptr;
}

int jwv_mctx_set_math(jwv_mctx* m, int mode) {
  if (!m) return set_err(nullptr, JWV_ERR_BAD_CALL, "jwv_mctx is NULL");
  for (jwv_ctx* c : m->ctx) {
    const int rc = jwv_ctx_set_math(c, mode);
    if (rc != JWV_OK) {
      m->err = jwv_last_error(c);
      return rc;
    }
  }
  return JWV_OK;
}

namespace {
using BatchFn = int (*)(const double*, double*, int64_t, int64_t, int64_t, int, const jwv_taps*,
                        jwv_ctx*);
int mbatch(Kind k, bool fwd, BatchFn fn, const double* x, double* y, int64_t batch, int64_t n,
           int64_t ld, int level, const jwv_taps* t, jwv_mctx* m) {
  if (!m) return set_err(nullptr, JWV_ERR_BAD_CALL, "jwv_mctx is NULL");
  std::lock_guard<std::mutex> lk(m->mu);
  m->err.clear();
  try {  // once, with the single-device entries' checks and messages
    (void)make_bank(t);
    if (batch < 0 || ld < n) throw Fail{JWV_ERR_BAD_CALL, "batch < 0 or ld < n"};
    check_1d(k, fwd, n, level);
    if (batch == 0) return JWV_OK;
    check_ptrs(x, y);
  } catch (const Fail& e) {
    m->err = e.msg;
    return e.code;
  }
  const int D = (int)m->ctx.size();
  std::vector<int> rc(D, JWV_OK);
  auto work = [&](int i) {
    int64_t s0 = 0, cnt = 0;
    jwv_batch_split(batch, D, i, &s0, &cnt);
    if (cnt > 0) rc[i] = fn(x + s0 * ld, y + s0 * ld, cnt, n, ld, level, t, m->ctx[i]);
  };
  std::vector<std::thread> th;
  for (int i = 1; i < D; ++i) th.emplace_back(work, i);
  work(0);
  for (auto& h : th) h.join();
  for (int i = 0; i < D; ++i)
    if (rc[i] != JWV_OK) {
      m->err = "device " + std::to_string(m->ctx[i]->device) + ": " + jwv_last_error(m->ctx[i]);
      return rc[i];
    }
  return JWV_OK;
}
}  // namespace

#define JWV_MBATCH(NAME, SINGLE, KIND, FWD)                                                    \
  int NAME(const double* x, double* y, int64_t batch, int64_t n, int64_t ld, int level,         \
           const jwv_taps* t, jwv_mctx* m) {                                                    \
    return mbatch(KIND, FWD, SINGLE, x, y, batch, n, ld, level, t, m);                          \
  }
JWV_MBATCH(jwv_m_fwt_fwd_batch_f64, jwv_fwt_fwd_batch_f64, Kind::FWT, true)
JWV_MBATCH(jwv_m_fwt_rev_batch_f64, jwv_fwt_rev_batch_f64, Kind::FWT, false)
JWV_MBATCH(jwv_m_wpt_fwd_batch_f64, jwv_wpt_fwd_batch_f64, Kind::WPT, true)
JWV_MBATCH(jwv_m_wpt_rev_batch_f64, jwv_wpt_rev_batch_f64, Kind::WPT, false)

// ---- multi-device 2-D ------------------------------------------------------------
// ParallelTransform.forward / reverse(double[][]) (ParallelTransform.java:70-126:
// rows split over threads, join, columns split over threads) over D GPUs of one
// process.  Device i holds rows [i rw, (i+1) rw) and, after one exchange,
// columns [i cw, (i+1) cw) (rw = rows/D, cw = cols/D):
//   forward  H2D row block -> row pass writing the exchange layout [D][rw][cw]
//            (jwv_fwt_rows_seg_*) -> every device pulls chunk i of every
//            device's block (hipMemcpyPeerAsync, xGMI; each waits on the
//            owners' phase-1 events) -> the received [rows][cw] slab's column
//            pass -> D2H into the columns of the host matrix (row-strided).
//   reverse  H2D column slab (row-strided) -> column pass -> exchange -> row
//            pass reading the chunks -> D2H of the row block.
// Each device's PCIe link carries 1/D of the bytes, each of its host copies
// runs on the process pool (grown to 16 threads per device).  D is the
// largest power of two <= the listed devices that divides rows with cw >= 2;
// 1 runs the single-device entry on the first device.  Results are the
// single-device entries' bits: the row and column passes are the same kernels
// on the same lines in the same order.
namespace {
class HostBarrier {
 public:
  explicit HostBarrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    const int g = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
      return;
    }
    cv_.wait(lk, [&] { return gen_ != g; });
  }

 private:
  int n_, count_ = 0, gen_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
};

int m2d_devices(int D, int64_t rows, int64_t cols) {
  int d = 1;
  while (d * 2 <= D) d *= 2;
  while (d > 1 && (rows % d || cols % d || cols / d < 2)) d /= 2;
  return d;
}

// row pass of `rows` rows into the exchange layout [cols/seg][rows][seg]
void rows_to_chunks(jwv_ctx* c, Kind k, const Bank& b, const double* x, double* y, int64_t rows,
                    int64_t cols, int level, int64_t seg, DevBuf& tmp) {
  const AxisView rv = cview(cols, 1);
  if (k == Kind::FWT) {
    AxisView ov = rv;
    ov.s_outer = seg;
    Axis a{x, rv, y, ov, rows, (int)cols, 1};
    a.lsw = exponent(seg);
    a.ss = rows * seg;
    Plan p = fwt_fwd_plan(c, b, a, level, c->ws);
    if (!p.empty()) return run_plan(p);
  }
  double* t = grow(c, tmp, (size_t)(rows * cols));
  axis_fn(k, true)(c, b, Axis{x, rv, t, rv, rows, (int)cols, 1}, level);
  copy_axis(c, seg_pack_axis(t, y, rows, cols, seg, true));
}
// reverse row pass reading the exchange layout
void chunks_to_rows(jwv_ctx* c, Kind k, const Bank& b, const double* y, double* x, int64_t rows,
                    int64_t cols, int level, int64_t seg, DevBuf& tmp) {
  const AxisView rv = cview(cols, 1);
  if (k == Kind::FWT) {
    AxisView iv = rv;
    iv.s_outer = seg;
    Axis a{y, iv, x, rv, rows, (int)cols, 1};
    a.lsw = exponent(seg);
    a.ss = rows * seg;
    Plan p = fwt_rev_plan(c, b, a, level, c->ws);
    if (!p.empty()) return run_plan(p);
  }
  double* t = grow(c, tmp, (size_t)(rows * cols));
  copy_axis(c, seg_pack_axis(t, const_cast<double*>(y), rows, cols, seg, false));
  axis_fn(k, false)(c, b, Axis{t, rv, x, rv, rows, (int)cols, 1}, level);
}

using Single2d = int (*)(const double*, double*, int64_t, int64_t, int, int, const jwv_taps*,
                         jwv_ctx*);
int m2d(Kind k, bool fwd, Single2d single, const double* in, double* out, int64_t rows,
        int64_t cols, int lvl_m, int lvl_n, const jwv_taps* t, jwv_mctx* m) {
  if (!m) return set_err(nullptr, JWV_ERR_BAD_CALL, "jwv_mctx is NULL");
  std::lock_guard<std::mutex> lk(m->mu);
  m->err.clear();
  Bank b;
  try {  // once, with the single-device entries' checks and messages
    b = make_bank(t);
    check_2d(k, fwd, rows, cols, lvl_m, lvl_n);
    if (rows == 0 || cols == 0) return JWV_OK;
    check_ptrs(in, out);
  } catch (const Fail& e) {
    m->err = e.msg;
    return e.code;
  }
  const int D = m2d_devices((int)m->ctx.size(), rows, cols);
  if (D == 1) {
    const int rc = single(in, out, rows, cols, lvl_m, lvl_n, t, m->ctx[0]);
    if (rc != JWV_OK) m->err = jwv_last_error(m->ctx[0]);
    return rc;
  }
  const size_t nd = m->ctx.size();
  if (m->a.size() < nd) {
    m->a.resize(nd), m->b.resize(nd), m->c.resize(nd), m->t.resize(nd);
    m->ev.resize(nd, nullptr);
  }
  const int64_t rw = rows / D, cw = cols / D;
  const size_t blk = (size_t)(rw * cols), chunk = (size_t)(rw * cw);
  std::vector<int> rc1(D, JWV_OK), rc2(D, JWV_OK);
  HostBarrier bar(D);
  auto work = [&](int i) {
    jwv_ctx* c = m->ctx[i];
    const AxisView sv = cview(rows, cw);  // a [rows][cw] slab, lines along rows
    rc1[i] = guarded(c, [&] {
      double* A = grow(c, m->a[i], blk);
      double* B = grow(c, m->b[i], blk);
      if (fwd) {
        copy_in(c, in + i * blk, A, blk);
        rows_to_chunks(c, k, b, A, B, rw, cols, lvl_n, cw, m->c[i]);
      } else {
        copy_in2d(c, in + i * cw, (size_t)cols, (size_t)rows, (size_t)cw, A);
        axis_fn(k, false)(c, b, Axis{A, sv, B, sv, 1, (int)rows, (int)cw}, lvl_m);
      }
      if (!m->ev[i]) HIPCHK(hipEventCreateWithFlags(&m->ev[i], hipEventDisableTiming));
      HIPCHK(hipEventRecord(m->ev[i], c->stream));
    });
    bar.wait();  // every device's phase-1 work is queued (or has failed)
    for (int d = 0; d < D; ++d)
      if (rc1[d] != JWV_OK) return;
    rc2[i] = guarded(c, [&] {
      double* A = m->a[i].p;
      double* C = grow(c, m->c[i], blk);
      // chunk i of every device's exchange block -> my slab (forward) / row
      // block's chunks (reverse)
      for (int d = 0; d < D; ++d) {
        HIPCHK(hipStreamWaitEvent(c->stream, m->ev[d], 0));
        HIPCHK(hipMemcpyPeerAsync(A + d * chunk, c->device, m->b[d].p + i * chunk,
                                  m->ctx[d]->device, chunk * sizeof(double), c->stream));
      }
      if (fwd) {
        axis_fn(k, true)(c, b, Axis{A, sv, C, sv, 1, (int)rows, (int)cw}, lvl_m);
        copy_out2d(c, C, (size_t)rows, (size_t)cw, out + i * cw, (size_t)cols);
      } else {
        chunks_to_rows(c, k, b, A, C, rw, cols, lvl_n, cw, m->t[i]);
        copy_out(c, C, out + i * blk, blk);
      }
      check_waits(c);
    });
  };
  std::vector<std::thread> th;
  for (int i = 1; i < D; ++i) th.emplace_back(work, i);
  work(0);
  for (auto& h : th) h.join();
  for (auto* rc : {&rc1, &rc2})
    for (int i = 0; i < D; ++i)
      if ((*rc)[i] != JWV_OK) {
        m->err = "device " + std::to_string(m->ctx[i]->device) + ": " + jwv_last_error(m->ctx[i]);
        return (*rc)[i];
      }
  return JWV_OK;
}
}  // namespace

int jwv_m_fwt2d_fwd_f64(const double* x, double* y, int64_t rows, int64_t cols, int lvl_m,
                        int lvl_n, const jwv_taps* t, jwv_mctx* m) {
  return m2d(Kind::FWT, true, jwv_fwt2d_fwd_f64, x, y, rows, cols, lvl_m, lvl_n, t, m);
}
int jwv_m_fwt2d_rev_f64(const double* y, double* x, int64_t rows, int64_t cols, int lvl_m,
                        int lvl_n, const jwv_taps* t, jwv_mctx* m) {
  return m2d(Kind::FWT, false, jwv_fwt2d_rev_f64, y, x, rows, cols, lvl_m, lvl_n, t, m);
}
int jwv_m_wpt2d_fwd_f64(const double* x, double* y, int64_t rows, int64_t cols, int lvl_m,
                        int lvl_n, const jwv_taps* t, jwv_mctx* m) {
  return m2d(Kind::WPT, true, jwv_wpt2d_fwd_f64, x, y, rows, cols, lvl_m, lvl_n, t, m);
}
int jwv_m_wpt2d_rev_f64(const double* y, double* x, int64_t rows, int64_t cols, int lvl_m,
                        int lvl_n, const jwv_taps* t, jwv_mctx* m) {
  return m2d(Kind::WPT, false, jwv_wpt2d_rev_f64, y, x, rows, cols, lvl_m, lvl_n, t, m);
}

// ---- MODWT batches -----------------------------------------------------------------
// forwardMODWT / inverseMODWT of `batch` signals of length n: x [batch][n],
// coefficients [batch][J+1][n] (each signal's double[J+1][n], packed).  One
// device: the signals one after another through the single-signal plan.
// jwv_m_*: contiguous blocks of signals per device (jwv_batch_split), one
// host thread per device, as the FWT/WPT batches.
int jwv_modwt_fwd_batch_f64(const double* x, double* wv, int64_t batch, int64_t n, int J,
                            const jwv_taps* t, jwv_ctx* c) {
  return guarded(c, [&] {
    const Bank b = make_bank(t);
    if (batch < 0) throw Fail{JWV_ERR_BAD_CALL, "batch < 0"};
    check_modwt(n, J);
    if (n == 0 || batch == 0) return;
    check_ptrs(x, wv);
    const int64_t out = (int64_t)(J + 1) * n;
    for (int64_t s = 0; s < batch; ++s)
      staged(c, x + s * n, (size_t)n, wv + s * out, (size_t)out,
             [&](const double* dx, double* dy) { body_modwt_fwd(c, b, dx, dy, n, J, n); });
  });
}
int jwv_modwt_inv_batch_f64(const double* wv, double* x, int64_t batch, int64_t n, int J,
                            const jwv_taps* t, jwv_ctx* c) {
  return guarded(c, [&] {
    const Bank b = make_bank(t);
    if (batch < 0) throw Fail{JWV_ERR_BAD_CALL, "batch < 0"};
    if (J < 1 || n == 0 || batch == 0) return;
    check_ptrs(wv, x);
    const int64_t in = (int64_t)(J + 1) * n;
    for (int64_t s = 0; s < batch; ++s)
      staged(c, wv + s * in, (size_t)in, x + s * n, (size_t)n,
             [&](const double* dx, double* dy) { body_modwt_inv(c, b, dx, dy, n, J, n); });
  });
}
namespace {
using ModwtBatchFn = int (*)(const double*, double*, int64_t, int64_t, int, const jwv_taps*,
                             jwv_ctx*);
int mmodwt(bool fwd, ModwtBatchFn fn, const double* in, double* out, int64_t batch, int64_t n,
           int J, const jwv_taps* t, jwv_mctx* m) {
  if (!m) return set_err(nullptr, JWV_ERR_BAD_CALL, "jwv_mctx is NULL");
  std::lock_guard<std::mutex> lk(m->mu);
  m->err.clear();
  try {
    (void)make_bank(t);
    if (batch < 0) throw Fail{JWV_ERR_BAD_CALL, "batch < 0"};
    if (fwd) check_modwt(n, J);
    if (n == 0 || batch == 0 || J < 1) return JWV_OK;
    check_ptrs(in, out);
  } catch (const Fail& e) {
    m->err = e.msg;
    return e.code;
  }
  const int64_t big = (int64_t)(J + 1) * n;
  const int64_t sin = fwd ? n : big, sout = fwd ? big : n;
  const int D = (int)m->ctx.size();
  std::vector<int> rc(D, JWV_OK);
  auto work = [&](int i) {
    int64_t s0 = 0, cnt = 0;
    jwv_batch_split(batch, D, i, &s0, &cnt);
    if (cnt > 0) rc[i] = fn(in + s0 * sin, out + s0 * sout, cnt, n, J, t, m->ctx[i]);
  };
  std::vector<std::thread> th;
  for (int i = 1; i < D; ++i) th.emplace_back(work, i);
  work(0);
  for (auto& h : th) h.join();
  for (int i = 0; i < D; ++i)
    if (rc[i] != JWV_OK) {
      m->err = "device " + std::to_string(m->ctx[i]->device) + ": " + jwv_last_error(m->ctx[i]);
      return rc[i];
    }
  return JWV_OK;
}
}  // namespace
int jwv_m_modwt_fwd_batch_f64(const double* x, double* wv, int64_t batch, int64_t n, int J,
                              const jwv_taps* t, jwv_mctx* m) {
  return mmodwt(true, jwv_modwt_fwd_batch_f64, x, wv, batch, n, J, t, m);
}
int jwv_m_modwt_inv_batch_f64(const double* wv, double* x, int64_t batch, int64_t n, int J,
                              const jwv_taps* t, jwv_mctx* m) {
  return mmodwt(false, jwv_modwt_inv_batch_f64, wv, x, batch, n, J, t, m);
}

}  // extern "C"
