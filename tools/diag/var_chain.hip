// Diagnostic: single-launch FWT chains (fwt1_chain.hpp) vs the multi-launch
// plan on config 2 (D4, N = 2^24, full depth), buffer sets rotated so every
// launch streams from HBM (2.3 GB > MALL).  Outputs are compared bitwise with
// the multi-launch results.  Not part of the library.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17
#include <cstdio>
#include <algorithm>
#include <functional>
#include <cstring>
#include <vector>
#include "../../jwave_amd/csrc/fwt1_chain.hpp"
using namespace jwv;

static const int H = 1 << 24, REPS = 24, NB = 6;
static double *xs[NB], *ys[NB], *zs[NB];
static double *wa, *wb, *yref, *zref;
static unsigned* sync_;
static double *x, *y, *z;
static int rot = 0;
static unsigned epoch = 0;
static void next() { rot = (rot + 1) % NB; x = xs[rot]; y = ys[rot]; z = zs[rot]; }
static hipEvent_t e0, e1;
static FwdTaps<8> tf;
static RevTaps<8> tr;

__global__ void fill(double* p, long n, unsigned seed) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += gridDim.x * 256L) {
    unsigned long long v = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    v ^= v >> 31; v *= 0xBF58476D1CE4E5B9ull; v ^= v >> 29;
    p[i] = (double)(v >> 11) * (1.0 / 9007199254740992.0);
  }
}

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
template <typename K>
static void big_lds(K k, size_t lds) {
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}
static bool same(const double* a, const double* b, long n) {
  std::vector<double> ha(n), hb(n);
  hipMemcpy(ha.data(), a, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(hb.data(), b, n * 8, hipMemcpyDeviceToHost);
  return std::memcmp(ha.data(), hb.data(), n * 8) == 0;
}

// ---- multi-launch plan (as the library: tile K=6, tile K=9, res 512 -> 1)
static void fwd_multi() {
  auto k1 = fwt_fwd_tile1<8, 256, 2048, 6, false>;
  auto k2 = fwt_fwd_tile1<8, 256, 2048, 9, false>;
  auto k3 = fwt_fwd_res1<8, 1024, 8192, false>;
  const size_t l1 = Fwd1Geo<8, 2048, 6>::lds_doubles() * 8, l2 = Fwd1Geo<8, 2048, 9>::lds_doubles() * 8;
  big_lds(k2, l2);
  hipLaunchKernelGGL(k1, dim3(H / 2048), dim3(256), l1, 0, x, 0, y, 0, wa, 0, H, tf);
  hipLaunchKernelGGL(k2, dim3((H >> 6) / 2048), dim3(256), l2, 0, wa, 0, y, 0, wb, 0, H >> 6, tf);
  hipLaunchKernelGGL(k3, dim3(1), dim3(1024), (512 + 2) * 8, 0, wb, 0, y, 0, 512, 9, tf);
}
static void rev_multi() {
  auto k1 = fwt_rev_res1<8, 1024, 8192, false>;
  auto k2 = fwt_rev_tile1<8, 256, 2048, 9, false>;
  auto k3 = fwt_rev_tile1<8, 256, 2048, 5, false>;
  const size_t l2 = Rev1Geo<8, 2048, 9>::lds_doubles() * 8, l3 = Rev1Geo<8, 2048, 5>::lds_doubles() * 8;
  hipLaunchKernelGGL(k1, dim3(1), dim3(1024), (1024 + 2) * 8, 0, y, 0, wa, 0, 2, 10, tr);
  hipLaunchKernelGGL(k2, dim3((1 << 19) / 2048), dim3(256), l2, 0, wa, 0, y, 0, wb, 0, 1 << 19, tr);
  hipLaunchKernelGGL(k3, dim3(H / 2048), dim3(256), l3, 0, wb, 0, y, 0, z, 0, H, tr);
}

template <int TA, int MINW>
static void fwd_chain() {
  using CH = FwdChain<8, 256, TA, 6, 2048, 7, 2048>;
  auto k = fwt_fwd_chain1<8, 256, TA, 6, 2048, 7, 2048, false, MINW>;
  const int hC = (H >> 6) >> 7;
  const size_t lds = ((size_t)CH::ctl_off(hC) + 2) * 8;
  big_lds(k, lds);
  hipLaunchKernelGGL(k, dim3(H / TA), dim3(256), lds, 0, x, y, wa, wb, sync_, H, 24 - 13, tf);
}
template <int MINW>
static void rev_chain(int G) {
  using CH = RevChain<8, 256, 2048, 2048, 9, 2048, 5>;
  auto k = fwt_rev_chain1<8, 256, 2048, 2048, 9, 2048, 5, false, MINW>;
  const size_t lds = (size_t)CH::lds_doubles(1024) * 8;
  big_lds(k, lds);
  if (++epoch == 0) epoch = 1;
  hipLaunchKernelGGL(k, dim3(G), dim3(256), lds, 0, y, z, wa, wb, sync_ + 4096, H, 2, 10, epoch, tr);
}

template <int KB>
static void fwd_split() {
  auto k1 = fwt_fwd_tile1<8, 256, 2048, 6, false>;
  constexpr int CAPC = (1 << 18) >> KB;
  auto k2 = fwt_fwd_tail1<8, 256, 2048, KB, CAPC, false>;
  const size_t l1 = Fwd1Geo<8, 2048, 6>::lds_doubles() * 8;
  const size_t l2 = ((size_t)tail_ctl_off<8, 2048, KB>(CAPC) + 2) * 8;
  big_lds(k2, l2);
  hipLaunchKernelGGL(k1, dim3(H / 2048), dim3(256), l1, 0, x, 0, y, 0, wa, 0, H, tf);
  static unsigned base = 0;  // arrival counter value (jwv_epoch.hpp)
  const unsigned nU = (H >> 6) / 2048;
  hipLaunchKernelGGL(k2, dim3(nU), dim3(256), l2, 0, wa, y, wb, sync_ + 8000, base + nU - 1,
                     H >> 6, 24 - 6 - KB, tf);
  base += nU;
}
static double* wr;
static void rev_split() {
  auto k1 = fwt_rev_head1<8, 256, 1024, 2048, 9, false>;
  auto k2 = fwt_rev_tile1<8, 256, 2048, 5, false>;
  const size_t l1 = std::max<size_t>(Rev1Geo<8, 2048, 9>::lds_doubles(), 1026) * 8;
  const size_t l2 = Rev1Geo<8, 2048, 5>::lds_doubles() * 8;
  if (++epoch == 0) epoch = 1;
  hipLaunchKernelGGL(k1, dim3(1 + 256), dim3(256), l1, 0, y, wb, wr, sync_ + 7000, 2, 10, epoch, tr);
  hipLaunchKernelGGL(k2, dim3(H / 2048), dim3(256), l2, 0, wb, 0, y, 0, z, 0, H, tr);
}

int main() {
  for (int j = 0; j < 8; ++j) {
    tf.lo[j] = 0.1 * (j + 1) - 0.35; tf.hi[j] = -0.07 * j + 0.2;
    tr.lo_r[j] = 0.11 * j - 0.3; tr.hi_r[j] = -0.2 * j + 0.5;
  }
  for (int i = 0; i < NB; ++i) {
    hipMalloc(&xs[i], (size_t)H * 8); hipMalloc(&ys[i], (size_t)H * 8); hipMalloc(&zs[i], (size_t)H * 8);
    hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, xs[i], (long)H, 17u + i);
    hipLaunchKernelGGL(fill, dim3(2048), dim3(256), 0, 0, ys[i], (long)H, 91u + i);
  }
  hipMalloc(&wa, (size_t)H / 8 * 8); hipMalloc(&wb, (size_t)H / 8 * 8);
  hipMalloc(&yref, (size_t)H * 8); hipMalloc(&zref, (size_t)H * 8);
  hipMalloc(&sync_, 8192 * 4); hipMemset(sync_, 0, 8192 * 4);
  hipMalloc(&wr, 1 << 16);
  hipEventCreate(&e0); hipEventCreate(&e1);
  int dev; hipGetDevice(&dev);
  hipDeviceProp_t pr; hipGetDeviceProperties(&pr, dev);
  const int ncu = pr.multiProcessorCount;

  // references (buffer set 0)
  rot = NB - 1; next();
  fwd_multi(); hipMemcpy(yref, y, (size_t)H * 8, hipMemcpyDeviceToDevice);
  rev_multi(); hipMemcpy(zref, z, (size_t)H * 8, hipMemcpyDeviceToDevice);
  hipDeviceSynchronize();
  auto chk_fwd = [&](const char* nm, auto fn) {
    rot = NB - 1; next(); fn(); hipDeviceSynchronize();
    printf("  %s fwd bit-exact: %s\n", nm, same(y, yref, H) ? "yes" : "NO");
  };
  printf("fwd multi   %7.2f us\n", timeit(fwd_multi));
  printf("fwd split K9 %7.2f us\n", timeit(fwd_split<9>)); chk_fwd("splitK9", fwd_split<9>);
  printf("fwd split K7 %7.2f us\n", timeit(fwd_split<7>)); chk_fwd("splitK7", fwd_split<7>);
  printf("fwd chain T2048 W1  %7.2f us\n", timeit(fwd_chain<2048, 1>)); chk_fwd("T2048W1", fwd_chain<2048, 1>);
  printf("fwd chain T2048 W6  %7.2f us\n", timeit(fwd_chain<2048, 6>)); chk_fwd("T2048W6", fwd_chain<2048, 6>);
  printf("fwd chain T2048 W8  %7.2f us\n", timeit(fwd_chain<2048, 8>));
  printf("fwd chain T4096 W1  %7.2f us\n", timeit(fwd_chain<4096, 1>)); chk_fwd("T4096W1", fwd_chain<4096, 1>);
  printf("fwd chain T4096 W4  %7.2f us\n", timeit(fwd_chain<4096, 4>));
  // reverse: restore y (coefficients) of set 0 for the check
  rot = NB - 1; next(); fwd_multi(); hipDeviceSynchronize();
  printf("rev multi   %7.2f us\n", timeit(rev_multi));
  printf("rev split   %7.2f us\n", timeit(rev_split));
  rot = NB - 1; next(); fwd_multi(); rev_split(); hipDeviceSynchronize();
  printf("  rev split bit-exact: %s\n", same(z, zref, H) ? "yes" : "NO");
  // warm: one buffer set, fwd then rev per step (the bench's pattern);
  // configurations interleaved over 7 rounds, median reported
  {
    struct Cfg { const char* nm; std::function<void()> f, r; std::vector<float> t; };
    std::vector<Cfg> cf = {
        {"multi+multi", fwd_multi, rev_multi, {}},
        {"multi+split", fwd_multi, rev_split, {}},
        {"splitK9+multi", fwd_split<9>, rev_multi, {}},
        {"splitK7+multi", fwd_split<7>, rev_multi, {}},
        {"splitK9+split", fwd_split<9>, rev_split, {}},
        {"splitK7+split", fwd_split<7>, rev_split, {}},
        {"multi+chainG1024", fwd_multi, [&] { rev_chain<5>(ncu * 4); }, {}},
    };
    for (int round = 0; round < 7; ++round)
      for (auto& c : cf) {
        rot = NB - 1; next();
        for (int i = 0; i < 3; ++i) { c.f(); c.r(); }
        hipEventRecord(e0);
        for (int i = 0; i < REPS; ++i) { c.f(); c.r(); }
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        c.t.push_back(ms * 1e3f / REPS);
      }
    for (auto& c : cf) {
      std::sort(c.t.begin(), c.t.end());
      printf("warm step %-20s median %7.2f us  (min %7.2f max %7.2f)\n", c.nm, c.t[3], c.t[0], c.t[6]);
    }
  }
  for (int bpc : {2, 3, 4, 5}) {
    int occ1 = 0, occ4 = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ1, fwt_rev_chain1<8, 256, 2048, 2048, 9, 2048, 5, false, 1>, 256,
                                                 RevChain<8, 256, 2048, 2048, 9, 2048, 5>::lds_doubles(1024) * 8);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ4, fwt_rev_chain1<8, 256, 2048, 2048, 9, 2048, 5, false, 5>, 256,
                                                 RevChain<8, 256, 2048, 2048, 9, 2048, 5>::lds_doubles(1024) * 8);
    const int G = ncu * bpc;
    if (bpc <= occ1 - 1 || bpc <= 2) {
      printf("rev chain W1 G=%d (occ %d)  %7.2f us\n", G, occ1, timeit([&] { rev_chain<1>(G); }));
      rot = NB - 1; next(); fwd_multi(); rev_chain<1>(G); hipDeviceSynchronize();
      printf("  bit-exact: %s\n", same(z, zref, H) ? "yes" : "NO");
    }
    if (bpc <= occ4 - 1) printf("rev chain W5 G=%d (occ %d)  %7.2f us\n", G, occ4, timeit([&] { rev_chain<5>(G); }));
  }
  unsigned w[8192];
  hipMemcpy(w, sync_, sizeof(w), hipMemcpyDeviceToHost);
  int nz = 0; for (int i = 0; i < 4096; ++i) nz += w[i] != 0;
  printf("fwd counters nonzero after runs: %d; rev timeout word %u\n", nz, w[4096 + 1 + 256]);
  return 0;
}
