// Diagnostic: where the config-5 MODWT tiles spend their time.  Times the
// library's modwt_inv_tile1 / modwt_fwd_tile1 (config 5: Daubechies4-sized
// L = 8, J = 8, N = 10^7) with hipEvents, best and median of 20 launches.
// Built several times with the compile-time diagnostic switches of
// modwt1_kernels.hpp (JWV_EXP_MOD_NOBAR / NOWF / NOFP: wrong results by
// design) to split the launch into barrier, W-fetch and FP64 shares.
// Build: tools/diag/build_diag_modwt.sh.  Not part of the library.
#include <algorithm>
#include <cstdio>
#include <vector>
#include "../../jwave_amd/csrc/modwt1_kernels.hpp"
using namespace jwv;

#ifndef TAG
#define TAG "base"
#endif

template <typename F>
static void timed(const char* what, F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<float> t;
  for (int rep = 0; rep < 25; ++rep) {
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    if (rep >= 5) t.push_back(ms * 1e3f);
  }
  std::sort(t.begin(), t.end());
  std::printf("%-6s %-40s best %7.1f  median %7.1f us\n", TAG, what, t[0], t[t.size() / 2]);
}

int main() {
  const int64_t N = 10000000, ldw = N;
  double *x, *w, *v, *y;
  hipMalloc(&x, N * 8);
  hipMalloc(&w, 8 * N * 8);
  hipMalloc(&v, N * 8);
  hipMalloc(&y, N * 8);
  std::vector<double> h(N);
  for (int64_t i = 0; i < N; ++i) h[i] = ((i * 37) % 101) * 0.01 - 0.5;
  hipMemcpy(x, h.data(), N * 8, hipMemcpyHostToDevice);
  ModwtTaps<8> tp;
  for (int j = 0; j < 8; ++j) { tp.g[j] = 0.11 * (j + 1); tp.h[j] = -0.07 * (j + 1); }
  {
    auto k = modwt_fwd_tile1<8, 1024, 8192, 1, 8, false, true, 1>;
    const size_t lds = (size_t)ModFwd1Geo<8, 8192, 1, 8>::lds_doubles(1) * 8;
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    timed("fwd 1024x8192", [&] {
      hipLaunchKernelGGL(k, dim3((N + 8191) / 8192), dim3(1024), lds, 0, x, w, ldw, v, N, tp);
    });
  }
  {
    auto k = modwt_inv_tile1<8, 512, 2048, 1, 8, false, true, 303>;
    const size_t lds = (size_t)ModInv1Geo<8, 2048, 1, 8>::lds_doubles(303) * 8;
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    timed("inv 512x2048 run303", [&] {
      hipLaunchKernelGGL(k, dim3((N + 2047) / 2048), dim3(512), lds, 0, v, w, ldw, y, N, tp);
    });
  }
  {
    auto k = modwt_inv_tile1<8, 512, 2048, 1, 8, true, true, 303>;
    const size_t lds = (size_t)ModInv1Geo<8, 2048, 1, 8>::lds_doubles(303) * 8;
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    timed("inv 512x2048 run303 FMA", [&] {
      hipLaunchKernelGGL(k, dim3((N + 2047) / 2048), dim3(512), lds, 0, v, w, ldw, y, N, tp);
    });
  }
  return 0;
}
