// Diagnostic: time the C = 1 FWT tile kernels (fwt1_kernels.hpp) on the
// config-2 big pass (D4, h = 2^24) for several (T, K) geometries, next to a
// 16-B copy kernel.  hipEvents around REPS back-to-back launches.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17
// Not part of the library.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../jwave_amd/csrc/fwt1_kernels.hpp"
using namespace jwv;

__global__ void copy16(const double2* __restrict__ s, double2* __restrict__ d, long n2) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long st = (long)gridDim.x * blockDim.x;
  for (; i < n2; i += st) d[i] = s[i];
}

static const int H = 1 << 24, REPS = 24;
static int NB = 6;  // NB buffer sets rotate: 6 x 512 MB > MALL (argv[1] = 1: MALL-warm)
static double *xs[8], *ys[8], *as_[8], *zs[8];
static double *x, *y, *a, *z;
static int rot = 0;
static void next() { rot = (rot + 1) % NB; x = xs[rot]; y = ys[rot]; a = as_[rot]; z = zs[rot]; }
static hipEvent_t e0, e1;

template <typename F>
static float timeit(F f) {
  for (int i = 0; i < 3; ++i) { next(); f(); }
  hipEventRecord(e0);
  for (int i = 0; i < REPS; ++i) { next(); f(); }
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / REPS;
}

template <int T, int K, int NT = 256>
static void fwd() {
  FwdTaps<8> tp;
  for (int j = 0; j < 8; ++j) { tp.lo[j] = 0.1 * j; tp.hi[j] = -0.1 * j; }
  auto k = fwt_fwd_tile1<8, NT, T, K, false>;
  const size_t lds = (size_t)Fwd1Geo<8, T, K>::lds_doubles() * 8;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const float us = timeit([&] {
    hipLaunchKernelGGL(k, dim3(H / T), dim3(NT), lds, 0, x, 0, y, 0, a, 0, H, tp, 0);
  });
  printf("fwd T=%5d K=%d NT=%d lds=%6zu B  %7.2f us  %6.0f GB/s (alg 16N)\n", T, K, NT, lds, us,
         16.0 * H / us / 1e3);
}

template <int T, int K, int NT = 256>
static void rev() {
  RevTaps<8> tp;
  for (int j = 0; j < 8; ++j) { tp.lo_r[j] = 0.1 * j; tp.hi_r[j] = -0.2 * j; }
  auto k = fwt_rev_tile1<8, NT, T, K, false>;
  const size_t lds = (size_t)Rev1Geo<8, T, K>::lds_doubles() * 8;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const float us = timeit([&] {
    hipLaunchKernelGGL(k, dim3(H / T), dim3(NT), lds, 0, a, 0, y, 0, z, 0, H, tp, 0);
  });
  printf("rev T=%5d K=%d NT=%d lds=%6zu B  %7.2f us  %6.0f GB/s (alg 16N)\n", T, K, NT, lds, us,
         16.0 * H / us / 1e3);
}

int main(int argc, char** argv) {
  if (argc > 1) NB = atoi(argv[1]);
  for (int i = 0; i < NB; ++i) {
    hipMalloc(&xs[i], (size_t)H * 8);
    hipMalloc(&ys[i], (size_t)H * 8);
    hipMalloc(&zs[i], (size_t)H * 8);
    hipMalloc(&as_[i], (size_t)H * 8);
    hipMemset(xs[i], 0, (size_t)H * 8);
    hipMemset(ys[i], 0, (size_t)H * 8);
    hipMemset(as_[i], 0, (size_t)H * 8);
  }
  next();
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int g : {1024, 2048, 4096, 8192, 32768}) {
    const float us = timeit([&] {
      hipLaunchKernelGGL(copy16, dim3(g), dim3(256), 0, 0, (const double2*)x, (double2*)z, (long)H / 2);
    });
    printf("copy16 grid=%d  %7.2f us  %6.0f GB/s\n", g, us, 16.0 * H / us / 1e3);
  }
  fwd<2048, 6>();
  fwd<2048, 5>();
  fwd<2048, 4>();
  fwd<2048, 3>();
  fwd<4096, 6>();
  fwd<4096, 5>();
  fwd<1024, 5>();
  fwd<1024, 4>();
  fwd<2048, 6, 512>();
  fwd<4096, 6, 512>();
  rev<2048, 5>();
  rev<2048, 6>();
  rev<2048, 4>();
  rev<4096, 5>();
  rev<4096, 6>();
  rev<1024, 5>();
  rev<2048, 5, 512>();
  return 0;
}
