// launch_compress.hip — CompressorMagnitude on the device
// (compressions/CompressorMagnitude.java:73-84, Compressor.java:96-110):
//   magnitude = (sum_i |c_i|) / n;  c_i kept if |c_i| >= magnitude * threshold,
//   else 0.
// The output is identical to Java's for every input although the sum is not
// taken left to right:
//  1. a fixed two-level tree gives S_t (fast, deterministic);
//  2. every term is >= 0, so Java's left-to-right sum S_j and S_t both lie
//     within (n + depth) * eps * S of the exact sum: S_j is in [S_lo, S_hi].
//     fl(fl(S/n) * thr) is monotone in S, so Java's cut lies in
//     [cut_lo, cut_hi];
//  3. the apply pass decides every |c| outside [cut_lo, cut_hi) as Java does
//     and raises a flag if any |c| falls inside (rare: a band of ~n*eps
//     relative width);
//  4. only then does one wave form S_j in Java's order and the decisions are
//     redone with Java's cut.  Steps 3-4 need no host round trip: the serial
//     and fix-up kernels return at once when the flag is clear.
// The magnitude handed back is S_t / n unless step 4 ran (then Java's).
#include "jwv_launch.hpp"

namespace jwv {
namespace {
constexpr int kRB = 256;        // threads per reduction block
constexpr int kRMaxBlocks = 1024;
// scratch after the partials: [0] cut used by the apply pass, [1] magnitude,
// [2] cut_lo, [3] cut_hi, [4] flag word (low 32 bits)
constexpr int kOut = 5;

__device__ double block_sum(double v) {
  __shared__ double red[kRB];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = kRB / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  return red[0];
}

// partial[b] = sum of |c| over a fixed grid-stride slice (order fixed by n, grid)
__global__ __launch_bounds__(kRB) void abs_sum_partial(const double* __restrict__ c, int64_t n,
                                                       double* __restrict__ partial) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kRB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kRB)
    s += fabs(c[i]);
  const double b = block_sum(s);
  if (threadIdx.x == 0) partial[blockIdx.x] = b;
}

__device__ __forceinline__ double cut_of(double S, int64_t n, double thr) {
  return (S / (double)n) * thr;  // CompressorMagnitude.java:82, Compressor.java:103
}

// S_t, its band [S_lo, S_hi] and the cuts of both ends; clears the flag (or
// sets it when the band is not finite: overflow decides nothing here).
__global__ __launch_bounds__(kRB) void abs_sum_final(const double* __restrict__ partial, int np,
                                                     int64_t n, double threshold,
                                                     double* __restrict__ out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += kRB) s += partial[i];
  const double tot = block_sum(s);
  if (threadIdx.x == 0) {
    // |S_j - S_t| <= (gamma_{n-1} + gamma_depth) * S; depth <= n/(np*kRB) + np/kRB + 16
    const double rel = 2.0 * ((double)n + 64.0) * 0x1p-53 * 1.01;
    const double band = tot * rel + ((double)n + 1.0) * 0x1p-1074;
    const double lo = fmax(nextafter(tot - band, 0.0), 0.0);
    const double hi = nextafter(tot + band, INFINITY);
    out[0] = cut_of(tot, n, threshold);
    out[1] = tot / (double)n;
    out[2] = cut_of(lo, n, threshold);
    out[3] = cut_of(hi, n, threshold);
    // NaN sums: every order gives NaN, every comparison is false (no band)
    const bool open = !isnan(tot) && !isfinite(hi);
    reinterpret_cast<unsigned*>(out + 4)[0] = open ? 1u : 0u;
    reinterpret_cast<unsigned*>(out + 4)[1] = 0u;
  }
}

// MODE 0: decide outside the band, copy inside it and raise the flag (x != y).
// MODE 1: classify only (in place: nothing is written before Java's cut is known).
// MODE 2: y = |x| >= cut_hi ? x : 0 (after a classify pass; cut_hi is Java's
//         cut when the serial pass ran, else no |x| lies in the band).
// MODE 3: as 2 but only when the flag is set (fix-up after MODE 0).
template <int MODE>
__global__ __launch_bounds__(256) void apply_cut(const double* c, double* y, int64_t n,
                                                 double* __restrict__ out) {
  unsigned* flag = reinterpret_cast<unsigned*>(out + 4);
  if (MODE == 3 && *flag == 0u) return;
  const double lo = out[2], hi = out[3];
  bool amb = false;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double v = c[i], a = fabs(v);
    if (MODE >= 2) {
      y[i] = a >= hi ? v : 0.0;
    } else {
      const bool in = a >= lo && a < hi;
      amb |= in;
      if (MODE == 0) y[i] = (a >= hi || in) ? v : 0.0;
    }
  }
  if (MODE <= 1 && __ballot(amb) != 0ull && (threadIdx.x & 63) == 0)
    __hip_atomic_fetch_or(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double lane_value(double v, int l) {
  const unsigned long long b = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Java's left-to-right sum (CompressorMagnitude.java:78-79) by one wave when
// the flag is set: lanes fetch 64 consecutive terms per step (U steps in
// flight), every lane adds all 64 of them in index order (wave-uniform sum).
__global__ __launch_bounds__(64) void abs_sum_serial(const double* __restrict__ c, int64_t n,
                                                     double threshold, double* __restrict__ out) {
  if (*reinterpret_cast<const unsigned*>(out + 4) == 0u) return;
  constexpr int U = 8;
  const int lane = threadIdx.x;
  double s = 0.0;
  int64_t i0 = 0;
  for (; i0 + 64 * U <= n; i0 += 64 * U) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = fabs(c[i0 + u * 64 + lane]);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int l = 0; l < 64; ++l) s += lane_value(v[u], l);
  }
  for (; i0 < n; i0 += 64) {
    const int64_t i = i0 + lane;
    const double v = i < n ? fabs(c[i]) : 0.0;
    const int m = n - i0 < 64 ? (int)(n - i0) : 64;
    for (int l = 0; l < m; ++l) s += __shfl(v, l);
  }
  if (lane == 0) {
    const double cut = cut_of(s, n, threshold);
    out[0] = cut;
    out[1] = s / (double)n;
    out[2] = cut;
    out[3] = cut;
  }
}

unsigned grid_of(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (unsigned)g;
}
}  // namespace

int compress_partials(int64_t n) {
  int64_t b = (n + kRB * 8 - 1) / (kRB * 8);
  return (int)(b < 1 ? 1 : (b > kRMaxBlocks ? kRMaxBlocks : b));
}
int compress_scratch(int64_t n) { return compress_partials(n) + kOut; }

hipError_t launch_compress_magnitude(const double* c, double* y, int64_t n, double threshold,
                                     double* scratch, hipStream_t s) {
  // scratch: compress_scratch(n) doubles; the magnitude ends at scratch[np + 1]
  const int np = compress_partials(n);
  double* out = scratch + np;
  const unsigned g = grid_of(n);
  JWV_LAUNCH(abs_sum_partial, dim3(np), dim3(kRB), 0, s, c, n, scratch);
  JWV_LAUNCH(abs_sum_final, dim3(1), dim3(kRB), 0, s, scratch, np, n, threshold, out);
  if (c != y) {
    JWV_LAUNCH(apply_cut<0>, dim3(g), dim3(256), 0, s, c, y, n, out);
    JWV_LAUNCH(abs_sum_serial, dim3(1), dim3(64), 0, s, c, n, threshold, out);
    JWV_LAUNCH(apply_cut<3>, dim3(g), dim3(256), 0, s, c, y, n, out);
  } else {
    JWV_LAUNCH(apply_cut<1>, dim3(g), dim3(256), 0, s, c, y, n, out);
    JWV_LAUNCH(abs_sum_serial, dim3(1), dim3(64), 0, s, c, n, threshold, out);
    JWV_LAUNCH(apply_cut<2>, dim3(g), dim3(256), 0, s, c, y, n, out);
  }
  return hipGetLastError();
}
}  // namespace jwv
