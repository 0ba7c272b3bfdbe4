// Dependent-chain latency of the instructions on the EVD's critical path
// (one wave, gfx950).  Development aid: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN(name, init, body)                                                   \
  __global__ void k_##name(float* out, unsigned long long* cyc, int n) {          \
    float x = init + threadIdx.x * 1e-7f;                                         \
    double d = (double)x;                                                         \
    (void)d;                                                                      \
    __shared__ float lds[256];                                                    \
    lds[threadIdx.x] = 0.f;                                                       \
    __syncthreads();                                                              \
    unsigned long long t0 = clock64();                                            \
    for (int i = 0; i < n; ++i) { body; }                                         \
    unsigned long long t1 = clock64();                                            \
    out[threadIdx.x] = x + (float)d;                                              \
    if (threadIdx.x == 0) *cyc = t1 - t0;                                         \
  }

CHAIN(rcp, 1.5f, x = __builtin_amdgcn_rcpf(x) + 0.25f)
CHAIN(sqrt, 1.5f, x = __builtin_amdgcn_sqrtf(x) + 0.25f)
CHAIN(rsq, 1.5f, x = __builtin_amdgcn_rsqf(x) + 0.25f)
CHAIN(fma, 1.5f, x = fmaf(x, 0.999f, 0.001f))
CHAIN(fma64, 1.5f, d = fma(d, 0.999, 0.001))
CHAIN(lds, 1.5f, x = lds[(int)x & 63] + x)
CHAIN(ieee_sqrt, 1.5f, x = sqrtf(x) + 0.25f)
CHAIN(ieee_div, 1.5f, x = 1.0f / x + 0.25f)

int main() {
  float* out;
  unsigned long long *dc, hc;
  hipMalloc(&out, 256 * sizeof(float));
  hipMalloc(&dc, sizeof(unsigned long long));
  const int n = 4096;
#define RUN(name)                                                                 \
  hipLaunchKernelGGL(k_##name, dim3(1), dim3(64), 0, 0, out, dc, n);              \
  hipLaunchKernelGGL(k_##name, dim3(1), dim3(64), 0, 0, out, dc, n);              \
  hipMemcpy(&hc, dc, sizeof(hc), hipMemcpyDeviceToHost);                          \
  printf("%-10s %6.1f cycles per dependent op (incl. loop)\n", #name, (double)hc / n);
  RUN(rcp) RUN(sqrt) RUN(rsq) RUN(fma) RUN(fma64) RUN(lds) RUN(ieee_sqrt) RUN(ieee_div)
  return 0;
}
