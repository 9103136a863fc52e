// Diagnostic: the config-2 big forward pass (fwt_fwd_tile1, D4, 2^24, K=6) in
// isolation, timed with events; variants by -D (see fwt1_kernels.hpp):
//   JWV_EXP_NOSTORE_DEEP  details of levels >= 2 not stored
// and an LDS-DMA window copy kernel of the same grid (load + store only).
#include <cstdio>
#include <cstdlib>
#include "../../jwave_amd/csrc/fwt1_kernels.hpp"
using namespace jwv;
template <int NT, int T, int M0>
__global__ __launch_bounds__(NT) void copy_win(const double* __restrict__ src, double* __restrict__ dst, int h) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int nblk = gridDim.x;
  int b = blockIdx.x;
  if ((nblk & 7) == 0) b = (b & 7) * (nblk >> 3) + (b >> 3);
  const int t = b, msk = h - 1, base = t * T;
  load_window<1, NT, (M0 + NT - 1) / NT>(lds, src, M0, true, 0, 1, [&](int e) { return (int64_t)((base + e) & msk); });
  dma_fence_barrier();
  for (int q = threadIdx.x; q < T / 2; q += NT)
    *reinterpret_cast<double2*>(dst + base + 2 * q) = *reinterpret_cast<const double2*>(lds + 2 * q);
}
int main() {
  const int n = 1 << 24;
  double *x, *y, *a;
  hipMalloc(&x, n * 8); hipMalloc(&y, n * 8); hipMalloc(&a, n * 8);
  {
    double* hx = (double*)malloc((size_t)n * 8);
    unsigned long long st = 42;
    for (int i = 0; i < n; ++i) { st = st * 6364136223846793005ULL + 1442695040888963407ULL; hx[i] = (double)(st >> 11) * (1.0 / 9007199254740992.0); }
    hipMemcpy(x, hx, (size_t)n * 8, hipMemcpyHostToDevice);
    free(hx);
  }
  FwdTaps<8> tp; for (int j = 0; j < 8; ++j) { tp.lo[j] = 0.1 * j; tp.hi[j] = -0.1 * j; }
  constexpr int T = 2048, K = 6;
  using G = Fwd1Geo<8, T, K>;
  const size_t lds = G::lds_doubles() * 8;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 8; ++rep) {
    float ms1, ms2;
    hipEventRecord(e0);
    hipLaunchKernelGGL((fwt_fwd_tile1<8, 256, T, K, false>), dim3(n / T), dim3(256), lds, 0, x, 0, y, 0, a, 0, n, tp);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms1, e0, e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((copy_win<256, T, G::m(0)>), dim3(n / T), dim3(256), lds, 0, x, y, n);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms2, e0, e1);
    if (rep >= 4) printf("fwd_tile1 %.2f us   copy_win(same grid/LDS) %.2f us\n", ms1 * 1e3, ms2 * 1e3);
  }
  for (int rep = 0; rep < 6; ++rep) {  // back to back, no other kernel between
    float ms1;
    hipEventRecord(e0);
    for (int k = 0; k < 10; ++k)
      hipLaunchKernelGGL((fwt_fwd_tile1<8, 256, T, K, false>), dim3(n / T), dim3(256), lds, 0, x, 0, y, 0, a, 0, n, tp);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms1, e0, e1);
    printf("fwd_tile1 x10 back-to-back: %.2f us each\n", ms1 * 1e2);
  }
  return 0;
}
