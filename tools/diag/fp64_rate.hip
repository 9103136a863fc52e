// Diagnostic: what FP64 issue rate the WPT couple's instruction shape reaches
// on one MI355X, independent of any transform.  Each lane runs the forward
// couple of wpt1_kernels.hpp (two pairs, 16 taps, EXACT: separate mul and add,
// four dependent add chains) over values it keeps in registers (R) or reads
// as 9 ds_read_b128 from a 4-KB LDS ring (LDS), many times, at several
// waves-per-SIMD counts.  Reports FP64 wave-instructions/s against the
// 1024-SIMD x 2.4 GHz / 4-cycle peak.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 fp64_rate.hip -o fp64_rate
// Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int L = 16;
struct Taps { double lo[L], hi[L]; };

template <bool USE_LDS, int ITERS>
__global__ void couple_kernel(const Taps tp, double* out, int seed) {
  __shared__ __attribute__((aligned(16))) double ring[512 + 32];
  const int tid = threadIdx.x;
  for (int i = tid; i < 512 + 32; i += blockDim.x) ring[i] = 1.0 + 1e-3 * ((i + seed) & 63);
  __syncthreads();
  double x[L + 2];
#pragma unroll
  for (int j = 0; j < L + 2; ++j) x[j] = 1.0 + 1e-4 * (j + tid);
  double acc = 0.0;
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (USE_LDS) {
      const double* in = ring + ((tid * 4 + it * 2) & 511);
#pragma unroll
      for (int j = 0; j < L + 2; j += 2) {
        const double2 v = *reinterpret_cast<const double2*>(in + j);
        x[j] = v.x;
        x[j + 1] = v.y;
      }
    }
    double a0 = 0.0, d0 = 0.0, a1 = 0.0, d1 = 0.0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      a0 = a0 + x[j] * tp.lo[j];
      d0 = d0 + x[j] * tp.hi[j];
      a1 = a1 + x[j + 2] * tp.lo[j];
      d1 = d1 + x[j + 2] * tp.hi[j];
    }
    asm volatile("" : "+v"(a0), "+v"(a1), "+v"(d0), "+v"(d1));
    acc += a0 - d0 + a1 - d1;
    if constexpr (!USE_LDS) {
#pragma unroll
      for (int j = 0; j < L + 2; ++j) asm volatile("" : "+v"(x[j]));
    }
  }
  if (acc == 12345.678) out[blockIdx.x * blockDim.x + tid] = acc;
}

template <bool USE_LDS>
void run(const char* name, int threads, int blocks_per_cu) {
  constexpr int ITERS = 2000;
  Taps tp;
  for (int j = 0; j < L; ++j) { tp.lo[j] = 0.01 * (j + 1); tp.hi[j] = -0.02 * (j + 1); }
  double* out;
  hipMalloc(&out, 1 << 24);
  const int grid = 256 * blocks_per_cu * 4;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((couple_kernel<USE_LDS, ITERS>), dim3(grid), dim3(threads), 0, 0, tp, out, 1);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL((couple_kernel<USE_LDS, ITERS>), dim3(grid), dim3(threads), 0, 0, tp, out,
                       r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double waves = 5.0 * grid * (threads / 64);
  const double fp64 = waves * ITERS * (4.0 * L * 2);  // mul + add per tap per chain
  const double rate = fp64 / (ms * 1e-3);
  const double peak = 1024.0 * 2.4e9 / 4.0;
  std::printf("%-4s threads %4d blocks/CU(launched) %d  %.3f ms  %.3e FP64 wave-instr/s  = %.3f of peak\n",
              name, threads, blocks_per_cu, ms, rate, rate / peak);
  hipFree(out);
}

int main() {
  for (int t : {256, 512, 1024})
    for (int b : {1, 2, 4}) {
      run<false>("REG", t, b);
      run<true>("LDS", t, b);
    }
  return 0;
}
