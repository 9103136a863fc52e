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

// Structure only: the forward tile's window DMA (T + halo, as fwt_fwd_tile1),
// one barrier, then T outputs stored from LDS as 16-B stores — no levels.
template <int T, int M0, int NT>
__global__ __launch_bounds__(NT) void dma_store(const double* __restrict__ src, double* __restrict__ dst,
                                                int h) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  int sp = 0;
  const int t = tile_order(gridDim.x, sp);
  const int msk = h - 1, base = t * T;
  load_window<1, NT, (M0 + NT - 1) / NT>(lds, src, M0, true, 0, 1,
                                         [&](int e) { return (int64_t)((base + e) & msk); });
  dma_fence_barrier();
#pragma unroll
  for (int q = threadIdx.x; q < T / 2; q += NT)
    *reinterpret_cast<double2*>(dst + base + 2 * q) = *reinterpret_cast<const double2*>(lds + 2 * q + 7);
}
// Tile walks: 0 plain (t = b), 1 XCD-chunked (tile_order), G > 1: XCD x
// takes groups of G consecutive tiles, the 8 XCDs side by side (one front)
template <int ORD>  // ORD: 0, 1 or a power of two dividing nblk / 8
__device__ __forceinline__ int walk(int nblk) {
  const int b = blockIdx.x;
  if constexpr (ORD == 0) return b;
  if constexpr (ORD == 1) { int sp = 0; return tile_order(nblk, sp); }
  const int x = b & 7, j = b >> 3;
  return (j / ORD) * 8 * ORD + x * ORD + (j % ORD);
}
template <int T, int M0, int NT, int ORD>
__global__ __launch_bounds__(NT) void dma_store_o(const double* __restrict__ src, double* __restrict__ dst,
                                                  int h) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int t = walk<ORD>(gridDim.x);
  const int msk = h - 1, base = t * T;
  load_window<1, NT, (M0 + NT - 1) / NT>(lds, src, M0, true, 0, 1,
                                         [&](int e) { return (int64_t)((base + e) & msk); });
  dma_fence_barrier();
#pragma unroll
  for (int q = threadIdx.x; q < T / 2; q += NT)
    *reinterpret_cast<double2*>(dst + base + 2 * q) = *reinterpret_cast<const double2*>(lds + 2 * q + 7);
}
template <int T, int NT, int ORD>
__global__ __launch_bounds__(NT) void tile_copy_o(const double* __restrict__ src, double* __restrict__ dst) {
  const int t = walk<ORD>(gridDim.x);
  const double2* s = reinterpret_cast<const double2*>(src + (int64_t)t * T);
  double2* d = reinterpret_cast<double2*>(dst + (int64_t)t * T);
  double2 v[T / 2 / NT];
#pragma unroll
  for (int r = 0; r < T / 2 / NT; ++r) v[r] = s[threadIdx.x + r * NT];
#pragma unroll
  for (int r = 0; r < T / 2 / NT; ++r) d[threadIdx.x + r * NT] = v[r];
}
template <int ORD>
static void orders();
// Plain-load copy with the tile walk (no LDS)
template <int T, int NT>
__global__ __launch_bounds__(NT) void tile_copy(const double* __restrict__ src, double* __restrict__ dst) {
  int sp = 0;
  const int t = tile_order(gridDim.x, sp);
  const double2* s = reinterpret_cast<const double2*>(src + (int64_t)t * T);
  double2* d = reinterpret_cast<double2*>(dst + (int64_t)t * T);
  double2 v[T / 2 / NT];
#pragma unroll
  for (int r = 0; r < T / 2 / NT; ++r) v[r] = s[threadIdx.x + r * NT];
#pragma unroll
  for (int r = 0; r < T / 2 / NT; ++r) d[threadIdx.x + r * NT] = v[r];
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

template <int T, int K, int NT = 256, int SP = 0>
static void fwd() {
  FwdTaps<8> tp;
  for (int j = 0; j < 8; ++j) { tp.lo[j] = 0.1 * j; tp.hi[j] = -0.1 * j; }
  auto k = fwt_fwd_tile1<8, NT, T, K, false>;
  const size_t lds = (size_t)Fwd1Geo<8, T, K>::lds_doubles() * 8;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const float us = timeit([&] {
    hipLaunchKernelGGL(k, dim3(H / T), dim3(NT), lds, 0, x, 0, y, 0, a, 0, H, tp, SP);
  });
  printf("fwd T=%5d K=%d NT=%d sp=%4d lds=%6zu B  %7.2f us  %6.0f GB/s (alg 16N)\n", T, K, NT, SP,
         lds, us, 16.0 * H / us / 1e3);
}

// reverse structure only: every window of fwt_rev_tile1 by DMA in one burst,
// one barrier, T outputs stored from LDS (grouped walk, G = 64)
template <int T, int K, int NT>
__global__ __launch_bounds__(NT) void rev_dma_store(const double* __restrict__ asrc,
                                                    const double* __restrict__ coef,
                                                    double* __restrict__ dst, int hK) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using G = Rev1Geo<8, T, K>;
  constexpr int MAXU = (G::len(1) + NT - 1) / NT;
  int sp = 8 | (6 << 8);
  const int t = tile_order(gridDim.x, sp);
  {
    const int BK = (t * T >> K) - G::c(K);
    const int am = (hK >> K) - 1;
    load_window<1, NT, MAXU>(lds + ((K & 1) ? G::buf1() : G::buf0()), asrc, G::len(K), true, 0, 1,
                             [&](int e) { return (int64_t)((BK + e) & am); });
  }
#pragma unroll
  for (int l = K - 1; l >= 0; --l) {
    const int half = hK >> (l + 1), hm = half - 1;
    const int B = (t * T >> (l + 1)) - G::c(l + 1);
    load_window<1, NT, MAXU>(lds + G::doff(l), coef, G::len(l + 1), true, 0, 1,
                             [&](int e) { return (int64_t)half + ((B + e) & hm); });
  }
  dma_fence_barrier();
  for (int q = threadIdx.x; q < T / 2; q += NT) {
    const double2 a = *reinterpret_cast<const double2*>(lds + G::doff(0) + 2 * (q & 511));
    *reinterpret_cast<double2*>(dst + (int64_t)t * T + 2 * q) = a;
  }
}

template <int T, int K, int NT = 256, int SP = 0>
static void rev() {
  RevTaps<8> tp;
  for (int j = 0; j < 8; ++j) { tp.lo_r[j] = 0.1 * j; tp.hi_r[j] = -0.2 * j; }
  auto k = fwt_rev_tile1<8, NT, T, K, false>;
  const size_t lds = (size_t)Rev1Geo<8, T, K>::lds_doubles() * 8;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const float us = timeit([&] {
    hipLaunchKernelGGL(k, dim3(H / T), dim3(NT), lds, 0, a, 0, y, 0, z, 0, H, tp, SP);
  });
  printf("rev T=%5d K=%d NT=%d sp=%4d lds=%6zu B  %7.2f us  %6.0f GB/s (alg 16N)\n", T, K, NT, SP,
         lds, us, 16.0 * H / us / 1e3);
}

template <int ORD>
static void orders() {
  constexpr int T = 2048, M0 = 2048 + 6 * 63;
  const float a = timeit([&] {
    hipLaunchKernelGGL((tile_copy_o<T, 256, ORD>), dim3(H / T), dim3(256), 0, 0, x, z);
  });
  const float b = timeit([&] {
    hipLaunchKernelGGL((dma_store_o<T, M0, 256, ORD>), dim3(H / T), dim3(256), (M0 + 2) * 8, 0, x, z, H);
  });
  printf("order %4d: tile_copy %7.2f us  dma_store %7.2f us\n", ORD, a, b);
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
  orders<0>();
  orders<1>();
  orders<2>();
  orders<4>();
  orders<16>();
  orders<64>();
  if (argc > 2) {
    constexpr int G64 = 8 | (6 << 8);
    fwd<2048, 6, 256, G64>();
    fwd<2048, 6, 512, G64>();
    fwd<4096, 6, 512, G64>();
    rev<2048, 5, 256, G64>();
    rev<2048, 5, 512, G64>();
    rev<2048, 6, 256, G64>();
    rev<2048, 4, 256, G64>();
    rev<1024, 5, 256, G64>();
    rev<4096, 5, 512, G64>();
    {
      using RG = Rev1Geo<8, 2048, 5>;
      const size_t lds = (size_t)RG::lds_doubles() * 8;
      auto k = rev_dma_store<2048, 5, 256>;
      const float us = timeit([&] {
        hipLaunchKernelGGL(k, dim3(H / 2048), dim3(256), lds, 0, a, y, z, H);
      });
      printf("rev_dma_store T=2048 K=5 (windows, no levels)  %7.2f us\n", us);
    }
    return 0;
  }
  {
    constexpr int T = 2048, M0 = 2048 + 6 * 63;
    auto k = dma_store<T, M0, 256>;
    const float us = timeit([&] {
      hipLaunchKernelGGL(k, dim3(H / T), dim3(256), (M0 + 2) * 8, 0, x, z, H);
    });
    printf("dma_store T=%d (window %d, no levels)  %7.2f us  %6.0f GB/s\n", T, M0, us, 16.0 * H / us / 1e3);
    auto k2 = tile_copy<T, 256>;
    const float us2 = timeit([&] { hipLaunchKernelGGL(k2, dim3(H / T), dim3(256), 0, 0, x, z); });
    printf("tile_copy T=%d (registers, tile walk)  %7.2f us  %6.0f GB/s\n", T, us2, 16.0 * H / us2 / 1e3);
  }
  fwd<2048, 1>();
  fwd<2048, 2>();
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
