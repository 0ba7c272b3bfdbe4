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
  CHECK(hipFree(X));
  CHECK(hipFree(Y));
  return 0;
}
