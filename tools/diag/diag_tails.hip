// Diagnostic: phase stamps (block 0) of the config-2 latency-bound launches:
// forward deep pass fwt_fwd_tile1<8,256,T,K> on a 2^18 / 2^19 input, the
// resident forward tail fwt_fwd_res1 (512 / 1024 / 2048 -> 1), and the
// reverse head fwt_rev_head1 (hR = 1024, KM = 9).  Event time per launch too.
// Build: hipcc -DJWV_STAMPS -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950
#include <cstdio>
#include <vector>
#include "../../jwave_amd/csrc/fwt1_chain.hpp"
__device__ unsigned long long jwv_stamps[64];
__device__ unsigned long long jwv_clocks[64];
using namespace jwv;
static hipEvent_t ea, eb;
template <typename F>
static void timed(const char* what, F f) {
  float best = 1e9, ms;
  for (int rep = 0; rep < 6; ++rep) {
    unsigned long long z[64] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(jwv_stamps), z, sizeof(z));
    hipEventRecord(ea);
    f();
    hipEventRecord(eb); hipEventSynchronize(eb); hipEventElapsedTime(&ms, ea, eb);
    if (ms < best) best = ms;
  }
  unsigned long long st[64];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(jwv_stamps), sizeof(st));
  printf("%-34s event(best) %6.2f us | stamps:", what, best * 1e3);
  for (int k = 1; k < 64; ++k) if (st[k]) printf(" [%d]%.2f", k, (st[k] - st[0]) / 100.0);
  printf("\n");
}
template <int T, int K, int NT = 256>
static void deep(double* x, double* y, double* a, int h, const FwdTaps<8>& tp) {
  const size_t lds = (size_t)Fwd1Geo<8, T, K>::lds_doubles() * 8;
  auto k = fwt_fwd_tile1<8, NT, T, K, false>;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  char nm[64]; snprintf(nm, 64, "fwd deep T=%d K=%d h=%d NT=%d", T, K, h, NT);
  timed(nm, [&] { hipLaunchKernelGGL(k, dim3(h / T), dim3(NT), lds, 0, x, 0, y, 0, a, 0, h, tp, 0); });
}
template <int NT, int TM, int KM>
static void head(double* x, double* y, int hR, const RevTaps<8>& tr) {
  const int h0 = 2, nR = 31 - __builtin_clz(hR), nM = (hR << KM) / TM;
  const size_t lds = (size_t)RevHeadGeo<8, TM, KM>::lds_doubles(hR) * 8;
  auto k = fwt_rev_head1<8, NT, 2048, TM, KM, false>;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  char nm[64]; snprintf(nm, 64, "rev head NT=%d TM=%d KM=%d hR=%d", NT, TM, KM, hR);
  timed(nm, [&] { hipLaunchKernelGGL(k, dim3(nM), dim3(NT), lds, 0, x, y, h0, nR, tr); });
}
template <int NT>
static void res(double* x, double* y, int h, int nl, const FwdTaps<8>& tp) {
  char nm[64]; snprintf(nm, 64, "fwd res NT=%d h=%d", NT, h);
  timed(nm, [&] { hipLaunchKernelGGL((fwt_fwd_res1<8, NT, 8192, false>), dim3(1), dim3(NT), (h + 2) * 8, 0, x, 0, y, 0, h, nl, tp); });
}
int main() {
  const int n = 1 << 20;
  double *x, *y, *a;
  hipMalloc(&x, n * 8); hipMalloc(&y, n * 8); hipMalloc(&a, n * 8);
  std::vector<double> hx(n); for (int i = 0; i < n; ++i) hx[i] = (i * 37 % 101) * 0.01;
  hipMemcpy(x, hx.data(), n * 8, hipMemcpyHostToDevice);
  hipEventCreate(&ea); hipEventCreate(&eb);
  FwdTaps<8> tf; RevTaps<8> tr;
  for (int j = 0; j < 8; ++j) { tf.lo[j] = 0.1 * j; tf.hi[j] = -0.1 * j; tr.lo_r[j] = 0.1 * j; tr.hi_r[j] = -0.2 * j; }
  deep<2048, 9>(x, y, a, 1 << 18, tf);
  deep<2048, 9, 512>(x, y, a, 1 << 18, tf);
  deep<2048, 9, 1024>(x, y, a, 1 << 18, tf);
  head<256, 2048, 9>(x, y, 1024, tr);
  head<512, 2048, 9>(x, y, 1024, tr);
  head<1024, 2048, 9>(x, y, 1024, tr);
  head<256, 1024, 9>(x, y, 512, tr);
  head<512, 4096, 9>(x, y, 1024, tr);
  deep<1024, 8>(x, y, a, 1 << 18, tf);
  deep<1024, 9>(x, y, a, 1 << 19, tf);
  deep<1024, 8>(x, y, a, 1 << 19, tf);
  deep<512, 7>(x, y, a, 1 << 18, tf);
  deep<512, 8>(x, y, a, 1 << 19, tf);
  res<1024>(x, y, 512, 9, tf);
  res<1024>(x, y, 1024, 10, tf);
  res<1024>(x, y, 2048, 11, tf);
  res<256>(x, y, 512, 9, tf);
  res<512>(x, y, 1024, 10, tf);
  {
    const int hR = 1024, h0 = 2, nR = 10, nM = (hR << 9) / 2048;
    const size_t lds = (size_t)RevHeadGeo<8, 2048, 9>::lds_doubles(hR) * 8;
    auto k = fwt_rev_head1<8, 256, 2048, 2048, 9, false>;
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    timed("rev head hR=1024 KM=9", [&] { hipLaunchKernelGGL(k, dim3(nM), dim3(256), lds, 0, x, y, h0, nR, tr); });
  }
  {
    auto k = fwt_rev_res1<8, 1024, 8192, false>;
    timed("rev res NT=1024 2->1024", [&] { hipLaunchKernelGGL(k, dim3(1), dim3(1024), 1026 * 8, 0, x, 0, y, 0, 2, 10, tr); });
  }
  return 0;
}
