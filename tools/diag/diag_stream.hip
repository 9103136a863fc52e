// Diagnostic: per-tile phase stamps of fwt_fwd_stream (block 0) on 2^24 D4.
#include <cstdio>
#include <vector>
#include "../../jwave_amd/csrc/fwt_kernels.hpp"
__device__ unsigned long long jwv_stamps[64];
__device__ unsigned long long jwv_clocks[64];
using namespace jwv;
int main(int argc, char** argv) {
  const int n = 1 << 24, T = 2048, K = 6, L = 8;
  const int bpc = argc > 1 ? atoi(argv[1]) : 2;
  double *x, *y, *a;
  hipMalloc(&x, (size_t)n * 8); hipMalloc(&y, (size_t)n * 8); hipMalloc(&a, (size_t)n / 64 * 8);
  hipMemset(x, 0, (size_t)n * 8);
  FwdTaps<8> tp; for (int j = 0; j < 8; ++j) { tp.lo[j] = 0.1 * j; tp.hi[j] = -0.1 * j; }
  AxisView v{n, 0, 1, 1, 0}, va{n / 64, 0, 1, 1, 0};
  auto k = fwt_fwd_stream<8, 256, 2048, 6, false>;
  const int M0MAX = T + 6 * 63, WBUF = (M0MAX + 3) & ~1;
  size_t lds = 2 * WBUF * 8;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  for (int rep = 0; rep < 4; ++rep) {
    unsigned long long z[64] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(jwv_stamps), z, sizeof(z));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(256 * bpc), dim3(320), lds, 0, x, v, y, v, a, va, n, K, (long)(n / T), tp);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long st[64];
    hipMemcpyFromSymbol(st, HIP_SYMBOL(jwv_stamps), sizeof(st));
    printf("bpc %d rep %d: %.1f us | per tile (compute, wait+barrier) us:", bpc, rep, ms * 1e3);
    for (int t = 0; t < 10; ++t)
      if (st[3 * t + 2]) printf(" (%.2f, %.2f)", (st[3 * t + 1] - st[3 * t]) / 100.0, (st[3 * t + 2] - st[3 * t + 1]) / 100.0);
    printf("\n");
  }
  return 0;
}
