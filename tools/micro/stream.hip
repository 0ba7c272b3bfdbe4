// HBM ceilings of the shapes the solver moves (development aid, round 5).
//  * copy    : out <- in, contiguous, 16 B per lane (the device copy ceiling);
//  * inplace : x <- x * c in place, contiguous (read + write of one buffer);
//  * tiles S : the quad apply's shape -- a column-major matrix (ld = 32768
//              floats: A's 16384 rows and V's stacked), 256 workgroups, each
//              owning 256 columns (a quad) and a quarter of the rows, walking
//              tiles of S rows x 256 columns in place, two tiles in flight.
//              S * 4 bytes is the contiguous run per column and tile.
// Prints one JSON line per case: bytes moved (read + write) over the best of
// 5 runs.  Build: hipcc --offload-arch=gfx950 -O3 stream.hip -o stream
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void copy_k(const f32x4* __restrict__ in, f32x4* __restrict__ out,
                                              size_t n4) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += 4 * stride) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < n4) v[u] = in[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < n4) out[i + u * stride] = v[u];
  }
}

__global__ __launch_bounds__(256) void inplace_k(f32x4* __restrict__ x, size_t n4, float c) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += 4 * stride) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < n4) v[u] = x[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * stride < n4) x[i + u * stride] = v[u] * c;
  }
}

// 512 threads; workgroup w: columns (w / SL) * 256 .. + 255, rows of slice w % SL
template <int S>
__global__ __launch_bounds__(512) void tiles_k(float* __restrict__ X, int ld, int rows, int SL, float c) {
  constexpr int LPC = S / 4;                 // lanes per column run
  constexpr int CPI = 64 / LPC;              // columns per wave instruction
  constexpr int NI = 256 / (8 * CPI);        // instructions per wave per tile
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.x / SL, sl = blockIdx.x % SL;
  const int r0 = sl * (rows / SL), r1 = r0 + rows / SL;
  float* base = X + (size_t)q * 256 * ld;
  const int lc = lane / LPC, lr = (lane % LPC) * 4;
  f32x4 a[NI], b[NI];
  auto ld_tile = [&](int r, f32x4 (&v)[NI]) {
#pragma unroll
    for (int j = 0; j < NI; ++j)
      v[j] = *reinterpret_cast<const f32x4*>(base + (size_t)((wave * NI + j) * CPI + lc) * ld + r + lr);
  };
  auto st_tile = [&](int r, f32x4 (&v)[NI]) {
#pragma unroll
    for (int j = 0; j < NI; ++j)
      *reinterpret_cast<f32x4*>(base + (size_t)((wave * NI + j) * CPI + lc) * ld + r + lr) = v[j] * c;
  };
  ld_tile(r0, a);
  for (int r = r0; r < r1; r += 2 * S) {
    if (r + S < r1) ld_tile(r + S, b);
    st_tile(r, a);
    if (r + S < r1) {
      if (r + 2 * S < r1) ld_tile(r + 2 * S, a);
      st_tile(r + S, b);
    }
  }
}

// The quad apply's exact load path: each of 8 waves LDS-DMAs its own 32
// columns of a 32-row tile (global_load_lds_dwordx4, 4 instructions, two
// tiles ahead), reads them back from LDS and stores the tile in place.
template <int AHEAD>
__global__ __launch_bounds__(512) void tiles_dma_k(float* __restrict__ X, int ld, int rows, int SL, float c) {
  __shared__ __attribute__((aligned(16))) char lds[AHEAD * 8 * 4096];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.x / SL, sl = blockIdx.x % SL;
  const int t0 = sl * (rows / SL) / 32, t1 = t0 + rows / SL / 32;
  float* own = X + ((size_t)q * 256 + wave * 32) * ld;
  auto dma = [&](int t) {
    char* dst = lds + ((t - t0) % AHEAD) * 8 * 4096 + wave * 4096;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds(own + (size_t)(8 * i + (lane >> 3)) * ld + t * 32 + (lane & 7) * 4,
                                       dst + i * 1024, 16, 0, 0);
  };
  for (int a = 0; a < AHEAD && t0 + a < t1; ++a) dma(t0 + a);
  for (int t = t0; t < t1; ++t) {
    // AHEAD == 2: exactly the apply's wait (younger: DMA of t + 1, stores of
    // t - 1); otherwise everything (conservative)
    const int younger = AHEAD == 2 ? (t + 1 < t1 ? 4 : 0) + (t > t0 ? 16 : 0) : 0;
    if (younger == 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if (younger == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (younger == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const float* R = reinterpret_cast<const float*>(lds + ((t - t0) % AHEAD) * 8 * 4096 + wave * 4096);
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = R[(2 * j + (lane >> 5)) * 32 + (lane & 31)];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (t + AHEAD < t1) dma(t + AHEAD);
#pragma unroll
    for (int j = 0; j < 16; ++j) own[(size_t)(2 * j + (lane >> 5)) * ld + t * 32 + (lane & 31)] = v[j] * c;
  }
}

// Same walk, loads into registers with the DMA's lane map, two tiles in flight
__global__ __launch_bounds__(512) void tiles_reg_k(float* __restrict__ X, int ld, int rows, int SL, float c) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = blockIdx.x / SL, sl = blockIdx.x % SL;
  const int t0 = sl * (rows / SL) / 32, t1 = t0 + rows / SL / 32;
  float* own = X + ((size_t)q * 256 + wave * 32) * ld;
  f32x4 a[4], b[4];
  auto ld4 = [&](int t, f32x4 (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      v[i] = *reinterpret_cast<const f32x4*>(own + (size_t)(8 * i + (lane >> 3)) * ld + t * 32 + (lane & 7) * 4);
  };
  auto st4 = [&](int t, f32x4 (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<f32x4*>(own + (size_t)(8 * i + (lane >> 3)) * ld + t * 32 + (lane & 7) * 4) = v[i] * c;
  };
  ld4(t0, a);
  for (int t = t0; t < t1; t += 2) {
    if (t + 1 < t1) ld4(t + 1, b);
    st4(t, a);
    if (t + 1 < t1) {
      if (t + 2 < t1) ld4(t + 2, a);
      st4(t + 1, b);
    }
  }
}

template <typename F>
static float best_ms(F launch) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 6; ++rep) {
    CHECK(hipEventRecord(e0));
    launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;  // rep 0 warms up
  }
  return best;
}

template <int S>
static void run_tiles(float* X, int ld, int rows, int ncol, int SL) {
  const int nq = ncol / 256;
  const float ms = best_ms([&] {
    hipLaunchKernelGGL((tiles_k<S>), dim3(nq * SL), dim3(512), 0, 0, X, ld, rows, SL, 1.0f);
  });
  const double bytes = 2.0 * ncol * (double)rows * 4;
  printf("{\"case\": \"tiles\", \"S_rows\": %d, \"run_B\": %d, \"workgroups\": %d, \"ms\": %.3f, \"TB_s\": %.3f}\n",
         S, S * 4, nq * SL, ms, bytes / ms / 1e9);
}

int main() {
  const int ld = 32768, rows = 32768, ncol = 16384;  // 2 GiB, the 16384^2 quad step's A and V
  const size_t n = (size_t)ld * ncol;
  float *X, *Y;
  CHECK(hipMalloc(&X, n * 4));
  CHECK(hipMalloc(&Y, n * 4));
  CHECK(hipMemset(X, 0, n * 4));
  CHECK(hipMemset(Y, 0, n * 4));
  const size_t n4 = n / 4;
  for (int grid : {1024, 4096}) {
    float ms = best_ms([&] {
      hipLaunchKernelGGL(copy_k, dim3(grid), dim3(256), 0, 0, (const f32x4*)X, (f32x4*)Y, n4);
    });
    printf("{\"case\": \"copy\", \"workgroups\": %d, \"ms\": %.3f, \"TB_s\": %.3f}\n", grid, ms,
           2.0 * n * 4 / ms / 1e9);
    ms = best_ms([&] { hipLaunchKernelGGL(inplace_k, dim3(grid), dim3(256), 0, 0, (f32x4*)X, n4, 1.0f); });
    printf("{\"case\": \"inplace\", \"workgroups\": %d, \"ms\": %.3f, \"TB_s\": %.3f}\n", grid, ms,
           2.0 * n * 4 / ms / 1e9);
  }
  for (int SL : {4, 8}) {
    run_tiles<32>(X, ld, rows, ncol, SL);
    run_tiles<64>(X, ld, rows, ncol, SL);
    run_tiles<128>(X, ld, rows, ncol, SL);
  }
  const int nq = ncol / 256;
  const double bytes = 2.0 * ncol * (double)rows * 4;
  for (int SL : {4, 8}) {
    float ms = best_ms([&] {
      hipLaunchKernelGGL(tiles_reg_k, dim3(nq * SL), dim3(512), 0, 0, X, ld, rows, SL, 1.0f);
    });
    printf("{\"case\": \"tiles_reg_applymap\", \"workgroups\": %d, \"ms\": %.3f, \"TB_s\": %.3f}\n", nq * SL, ms, bytes / ms / 1e9);
    ms = best_ms([&] {
      hipLaunchKernelGGL((tiles_dma_k<2>), dim3(nq * SL), dim3(512), 0, 0, X, ld, rows, SL, 1.0f);
    });
    printf("{\"case\": \"tiles_dma2\", \"workgroups\": %d, \"ms\": %.3f, \"TB_s\": %.3f}\n", nq * SL, ms, bytes / ms / 1e9);
    ms = best_ms([&] {
      hipLaunchKernelGGL((tiles_dma_k<1>), dim3(nq * SL), dim3(512), 0, 0, X, ld, rows, SL, 1.0f);
    });
    printf("{\"case\": \"tiles_dma1_drain\", \"workgroups\": %d, \"ms\": %.3f, \"TB_s\": %.3f}\n", nq * SL, ms, bytes / ms / 1e9);
  }
  CHECK(hipFree(X));
  CHECK(hipFree(Y));
  return 0;
}
