// Diagnostic: phase stamps of the C = 1 resident kernels (fwt1_res.hpp) on the
// config-2 tails (D4): forward 4096 -> 1 (12 levels), reverse 2 -> 8192 (13).
// Build: hipcc -DJWV_STAMPS ...  Not part of the library.
#include <cstdio>
#include <vector>
#include "../../jwave_amd/csrc/fwt1_res.hpp"
__device__ unsigned long long jwv_stamps[64];
__device__ unsigned long long jwv_clocks[64];
using namespace jwv;
static void show(const char* what, float ms) {
  unsigned long long st[64];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(jwv_stamps), sizeof(st));
  printf("%s event %.2f us | stamps:", what, ms * 1e3);
  for (int k = 0; k < 64; ++k) if (st[k]) printf(" [%d]%.2f", k, (st[k] - st[0]) / 100.0);
  printf("\n");
}
int main() {
  const int n = 8192;
  double *x, *y;
  hipMalloc(&x, n * 8); hipMalloc(&y, n * 8);
  std::vector<double> hx(n, 1.0); hipMemcpy(x, hx.data(), n * 8, hipMemcpyHostToDevice);
  FwdTaps<8> tf; RevTaps<8> tr;
  for (int j = 0; j < 8; ++j) { tf.lo[j] = 0.1 * j; tf.hi[j] = -0.1 * j; tr.lo_r[j] = 0.1 * j; tr.hi_r[j] = -0.2 * j; }
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int rep = 0; rep < 4; ++rep) {
    unsigned long long z[64] = {0};
    float ms;
    hipMemcpyToSymbol(HIP_SYMBOL(jwv_stamps), z, sizeof(z));
    hipEventRecord(a);
    hipLaunchKernelGGL((fwt_fwd_res1<8, 1024, 8192, false>), dim3(1), dim3(1024), 512 * 8 + 16, 0, x, 0, y, 0, 512, 9, tf);
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    if (rep >= 2) show("fwd_res1 512/9", ms);
    hipMemcpyToSymbol(HIP_SYMBOL(jwv_stamps), z, sizeof(z));
    hipEventRecord(a);
    hipLaunchKernelGGL((fwt_rev_res1<8, 1024, 8192, false>), dim3(1), dim3(1024), 1024 * 8 + 16, 0, x, 0, y, 0, 2, 10, tr);
    hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
    if (rep >= 2) show("rev_res1 2/10   ", ms);
  }
  return 0;
}
