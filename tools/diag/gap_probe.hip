// gap_probe.hip — what sets the idle gap after a 128 MB streaming kernel?
// copy / read-only / write-only kernels with each load/store cache policy,
// each followed by a 1-block kernel; run under rocprofv3 --kernel-trace and
// read the gap (tiny start - big end) per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int LP, int SP, int MODE>  // MODE 0 copy, 1 read-only, 2 write-only
__global__ __launch_bounds__(256) void big(const double* src, double* dst, double* sink, int n2) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // 16-B unit
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7ffffff0, 0x00020000);
  const auto rd = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7ffffff0, 0x00020000);
  if (i >= n2) return;
  u4 v = {1u, 2u, 3u, 4u};
  if (MODE != 2) v = __builtin_amdgcn_raw_buffer_load_b128(rs, i * 16, 0, LP);
  if (MODE != 1) __builtin_amdgcn_raw_buffer_store_b128(v, rd, i * 16, 0, SP);
  else if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) sink[0] = 1.0;
}
__global__ void tiny(double* p) { if (threadIdx.x == 0) p[0] += 1.0; }

int main() {
  const int n = 1 << 24, n2 = n / 2;
  double *x, *y, *s;
  hipMalloc(&x, n * 8); hipMalloc(&y, n * 8); hipMalloc(&s, 64);
  hipMemset(x, 0, n * 8); hipMemset(y, 0, n * 8);
  const dim3 g(n2 / 256), b(256);
#define RUN(K) for (int r = 0; r < 6; ++r) { hipLaunchKernelGGL(K, g, b, 0, 0, x, y, s, n2); hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, 0, s); }
  RUN((big<0, 0, 0>)) RUN((big<0, 16, 0>)) RUN((big<0, 2, 0>)) RUN((big<2, 16, 0>)) RUN((big<16, 16, 0>)) RUN((big<17, 17, 0>))
  RUN((big<0, 0, 1>)) RUN((big<2, 0, 1>)) RUN((big<16, 0, 1>)) RUN((big<17, 0, 1>))
  RUN((big<0, 0, 2>)) RUN((big<0, 16, 2>)) RUN((big<0, 2, 2>)) RUN((big<0, 17, 2>))
  hipDeviceSynchronize();
  printf("done\n");
  return 0;
}
