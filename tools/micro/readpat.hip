// Read bandwidth of the block kernels' access shape (development aid).
// A column-major fp32 matrix (column stride ld floats) is read in slabs of S rows
// x 128 columns per workgroup, 16 B per lane, S/4 lanes per column segment, as the
// cross Gram reads its pair; the question is how the per-column segment length S*4
// bytes sets the achieved HBM read bandwidth.
// Build: hipcc --offload-arch=gfx950 -O3 readpat.hip -o readpat ; run: ./readpat
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

// grid: (ncolgroups, nchunks); workgroup (g, ch) reads columns 128 g .. +127,
// rows ch*rows_per_chunk .. +rows_per_chunk, S rows per slab
template <int S>
__global__ __launch_bounds__(256) void readpat(const float* __restrict__ A, int ld, int rows_per_chunk,
                                               float* __restrict__ out) {
  constexpr int LPC = S / 4;          // lanes per column segment
  constexpr int CPI = 64 / LPC;       // columns per wave instruction (>= 1)
  constexpr int NI = 128 / CPI / 4;   // instructions per wave per slab (4 waves)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lc = lane / LPC, lr = (lane % LPC) * 4;
  const float* base = A + (size_t)blockIdx.x * 128 * ld;
  const int r0 = blockIdx.y * rows_per_chunk;
  // U slabs per iteration: 32 loads (32 KB per wave) in flight for every S
  constexpr int U = 32 / NI;
  f32x4 acc = {0, 0, 0, 0};
  f32x4 v[U][NI];
  for (int r = r0; r < r0 + rows_per_chunk; r += U * S) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = (wave * NI + j) * CPI + lc;
        v[u][j] = *reinterpret_cast<const f32x4*>(base + (size_t)col * ld + r + u * S + lr);
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc += v[u][j];
  }
  const float s = acc[0] + acc[1] + acc[2] + acc[3];
  if (s == 12345.678f) out[blockIdx.x] = s;  // keep the loads
}

template <int S>
static void run(const float* A, int ld, int ncol, int rows, float* out, int nchunks) {
  const int groups = ncol / 128;
  const int rpc = rows / nchunks;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((readpat<S>), dim3(groups, nchunks), dim3(256), 0, 0, A, ld, rpc, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double bytes = (double)ncol * rows * 4;
  printf("{\"S_rows\": %d, \"segment_B\": %d, \"workgroups\": %d, \"rows_per_wg\": %d, \"ms\": %.3f, \"TB_s\": %.3f}\n",
         S, S * 4, groups * nchunks, rpc, best, bytes / best / 1e9);
}

int main() {
  const int rows = 16384, ld = 16384, ncol = 8192;  // 512 MB: one 64-pair step's Gram read
  float *A, *out;
  CHECK(hipMalloc(&A, (size_t)ld * ncol * 4));
  CHECK(hipMalloc(&out, 1 << 20));
  CHECK(hipMemset(A, 0, (size_t)ld * ncol * 4));
  for (int nch : {4, 8, 16}) {
    run<32>(A, ld, ncol, rows, out, nch);
    run<64>(A, ld, ncol, rows, out, nch);
    run<128>(A, ld, ncol, rows, out, nch);
    run<256>(A, ld, ncol, rows, out, nch);
  }
  CHECK(hipFree(A));
  CHECK(hipFree(out));
  return 0;
}
