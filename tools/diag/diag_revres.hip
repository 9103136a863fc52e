// Diagnostic: phase stamps of the resident forward kernel on a single 4096
// signal (D4).  Build: hipcc -DJWV_STAMPS ...  Not part of the library.
#include <cstdio>
#include <vector>
#include "../../jwave_amd/csrc/fwt_kernels.hpp"
__device__ unsigned long long jwv_stamps[64];
__device__ unsigned long long jwv_clocks[64];
__global__ void spin(double* p, int n) {  // keep the chip busy / clocks up
  double v = p[threadIdx.x];
  for (int i = 0; i < n; ++i) v = v * 1.0000001 + 1e-9;
  p[threadIdx.x] = v;
}
using namespace jwv;
int main() {
  const int n = 8192;
  double *x, *y;
  hipMalloc(&x, n * 8); hipMalloc(&y, n * 8);
  std::vector<double> hx(n, 1.0); hipMemcpy(x, hx.data(), n * 8, hipMemcpyHostToDevice);
  RevTaps<8> tp; for (int j = 0; j < 8; ++j) { tp.lo_r[j] = 0.1 * j; tp.hi_r[j] = -0.1 * j; }
  AxisView v{n, 0, 1, 1, 0};
  for (int rep = 0; rep < 6; ++rep) {
    unsigned long long z[64] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(jwv_stamps), z, sizeof(z));
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    if (rep >= 3) hipLaunchKernelGGL(spin, dim3(4096), dim3(256), 0, 0, y, 200000);
    hipEventRecord(a);
    hipLaunchKernelGGL((fwt_rev_res<8, 1, 1024, 8192, false>), dim3(1), dim3(1024), (n + 2) * 8, 0,
                       x, v, y, v, 2, 13, 1, 1, tp);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    unsigned long long st[64];
    hipMemcpyFromSymbol(st, HIP_SYMBOL(jwv_stamps), sizeof(st));
    printf("rep %d event %.2f us | stamps(us from start):", rep, ms * 1e3);
    for (int k = 0; k < 64; ++k) if (st[k]) printf(" [%d]%.2f", k, (st[k] - st[0]) / 100.0);
    unsigned long long ck[64];
    hipMemcpyFromSymbol(ck, HIP_SYMBOL(jwv_clocks), sizeof(ck));
    printf("  clock %.0f MHz\n", 100.0 * (double)(ck[42] - ck[0]) / (double)(st[42] - st[0]));
  }
  return 0;
}
