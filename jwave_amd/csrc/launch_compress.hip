// launch_compress.hip — CompressorMagnitude on the device
// (compressions/CompressorMagnitude.java:73-84, Compressor.java:96-110):
//   magnitude = (sum_i |c_i|) / n;  c_i kept if |c_i| >= magnitude * threshold,
//   else 0.
// The sum is a fixed two-level tree (per-block partial sums in a fixed order,
// then one block sums the partials in index order): deterministic, but not
// Java's left-to-right order, so `magnitude` can differ from the JVM's in the
// last bits; a coefficient lands on the other side of the threshold only if
// |c_i| is within ~n*eps of magnitude*threshold.
#include "jwv_launch.hpp"

namespace jwv {
namespace {
constexpr int kRB = 256;        // threads per reduction block
constexpr int kRMaxBlocks = 1024;

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

// cut = (sum(partial) / n) * threshold, written to out[0] (magnitude to out[1])
__global__ __launch_bounds__(kRB) void abs_sum_final(const double* __restrict__ partial, int np,
                                                     int64_t n, double threshold,
                                                     double* __restrict__ out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += kRB) s += partial[i];
  const double tot = block_sum(s);
  if (threadIdx.x == 0) {
    const double mag = tot / (double)n;  // CompressorMagnitude.java:82
    out[0] = mag * threshold;            // Compressor.java:103 (magnitude * _threshold)
    out[1] = mag;
  }
}

__global__ __launch_bounds__(256) void apply_cut(const double* __restrict__ c,
                                                 double* __restrict__ y, int64_t n,
                                                 const double* __restrict__ cut) {
  const double k = cut[0];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const double v = c[i];
    y[i] = fabs(v) >= k ? v : 0.0;
  }
}
}  // namespace

int compress_partials(int64_t n) {
  int64_t b = (n + kRB * 8 - 1) / (kRB * 8);
  return (int)(b < 1 ? 1 : (b > kRMaxBlocks ? kRMaxBlocks : b));
}

hipError_t launch_compress_magnitude(const double* c, double* y, int64_t n, double threshold,
                                     double* scratch, hipStream_t s) {
  // scratch: compress_partials(n) + 2 doubles
  const int np = compress_partials(n);
  double* out = scratch + np;
  hipLaunchKernelGGL(abs_sum_partial, dim3(np), dim3(kRB), 0, s, c, n, scratch);
  hipLaunchKernelGGL(abs_sum_final, dim3(1), dim3(kRB), 0, s, scratch, np, n, threshold, out);
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(apply_cut, dim3((unsigned)g), dim3(256), 0, s, c, y, n, out);
  return hipGetLastError();
}
}  // namespace jwv
