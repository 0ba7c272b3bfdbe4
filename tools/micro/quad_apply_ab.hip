// Ablations of the quad apply (apply_quad_ts_kernel, csrc/hip/block.hip) at the
// headline geometry (development aid, round 6): 16384 rows of A and 16384 of V,
// 64 active quads (a merged 128-pair quad step of the 16384^2 solve), realistic
// T - I (entries ~U(-0.01, 0.01), split into 3 RNE bf16 parts).  Variants by the
// kernel's ABL flags:
//   0 production; 1 one MFMA per k block (B fragments still read);
//   2 no global memory; 3 = 1 + 2; 4 no MFMA loop (DMA, split, epilogue);
//   6 = 4 + 2 (split and epilogue only); 8 never the cheap k-half form; the
//   production form on small T - I (every k half cheap); and the NP = 2 (3-MFMA) form.
// Then the quad Gram (gram_quad_kernel) on the same A: production, one MFMA
// per tile and k step, no global reads, both.
// Prints one JSON line per variant: best and median of 12 timed launches.
// Build (post.o: the library's helpers it links against):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I svd-jacobi-mpi-cuda_amd/csrc/include
//     -I svd-jacobi-mpi-cuda_amd/csrc/hip -c tools/micro/quad_apply_ab.hip -o qab.o
//   hipcc --offload-arch=gfx950 qab.o svd-jacobi-mpi-cuda_amd/lib/obj/post.o -o tools/micro/quad_apply_ab
#include "block.hip"

#include <algorithm>
#include <cstdio>
#include <vector>


using namespace svdj;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__global__ void fill_uniform(float* p, size_t n, uint32_t seed, float lo, float hi) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = lo + (hi - lo) * (float)(x & 0xffffff) / 16777216.0f;
  }
}

// Ts[q][kb][ct][part][lane] from an fp32 T - I image of the same layout
template <int NP>
__global__ void split_ts(const float* __restrict__ src, bf16x8* __restrict__ Ts, int nfrag) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= nfrag) return;
  bf16x8 parts[NP];
  for (int e = 0; e < 8; ++e) {
    __bf16 p[NP];
    split_bf16<NP>(src[(size_t)f * 8 + e], p);
    for (int i = 0; i < NP; ++i) parts[i][e] = p[i];
  }
  const int lane = f % SVDJ_WAVE, rest = f / SVDJ_WAVE;
  for (int i = 0; i < NP; ++i) Ts[((size_t)rest * NP + i) * SVDJ_WAVE + lane] = parts[i];
}

template <int NP, int ABL>
static int run(const char* name, float* A, float* V, int m, int nq, const int32_t* pairs,
               const bf16x8* Ts, const int32_t* skip, double bytes) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> t;
  for (int it = 0; it < 14; ++it) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((apply_quad_ts_kernel<NP, ABL>), dim3(kQuadTsGrid), dim3(kQuadTsThreads), 0, 0,
                       A, m, m / 32, V, m, m / 32, pairs, nq, Ts, skip, skip);
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it >= 2) t.push_back(ms * 1e3f);
  }
  std::sort(t.begin(), t.end());
  printf("{\"variant\": \"%s\", \"np\": %d, \"abl\": %d, \"best_us\": %.1f, \"median_us\": %.1f, "
         "\"TB_s_at_best\": %.3f}\n", name, NP, ABL, t[0], t[t.size() / 2], bytes / (t[0] * 1e-6) / 1e12);
  fflush(stdout);
  return 0;
}

template <int ABL>
static int run_gram(const char* name, const float* A, int m, int nq, const int32_t* pairs,
                    float* slabs, int gch) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> t;
  const int rows = m / gch;
  for (int it = 0; it < 14; ++it) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(gram_quad_kernel<ABL>, dim3(nq, gch), dim3(kGramQThreads), 0, 0, A, m, m, pairs,
                       2 * nq, rows, slabs);
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (it >= 2) t.push_back(ms * 1e3f);
  }
  std::sort(t.begin(), t.end());
  const double bytes = (double)nq * 256 * m * 4;
  printf("{\"kernel\": \"gram_quad\", \"variant\": \"%s\", \"abl\": %d, \"chunks\": %d, "
         "\"best_us\": %.1f, \"median_us\": %.1f, \"read_TB_s_at_best\": %.3f}\n",
         name, ABL, gch, t[0], t[t.size() / 2], bytes / (t[0] * 1e-6) / 1e12);
  fflush(stdout);
  return 0;
}

int main() {
  const int m = 16384, nblk = 256, nq = nblk / 4;
  const size_t nA = (size_t)nblk * 64 * m;
  float *A, *V, *Tf;
  bf16x8* Ts;
  int32_t *pairs, *skip;
  const int nfrag = nq * 16 * 8 * SVDJ_WAVE;  // fragments of 8 values per part
  CK(hipMalloc(&A, nA * 4));
  CK(hipMalloc(&V, nA * 4));
  CK(hipMalloc(&Tf, (size_t)nfrag * 8 * 4));
  CK(hipMalloc(&Ts, (size_t)nfrag * 3 * 16));
  CK(hipMalloc(&pairs, nq * 4 * 4));
  CK(hipMalloc(&skip, nq * 2 * 4));
  CK(hipMemset(skip, 0, nq * 2 * 4));
  std::vector<int32_t> hp(nq * 4);
  for (int q = 0; q < nq; ++q) {  // quad blocks (a, b, c, d) = 4q .. 4q + 3: pairs (a, c), (b, d)
    hp[4 * q] = 4 * q; hp[4 * q + 1] = 4 * q + 2; hp[4 * q + 2] = 4 * q + 1; hp[4 * q + 3] = 4 * q + 3;
  }
  CK(hipMemcpy(pairs, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fill_uniform, dim3(4096), dim3(256), 0, 0, A, nA, 1u, 0.0f, 1.0f);
  hipLaunchKernelGGL(fill_uniform, dim3(4096), dim3(256), 0, 0, V, nA, 2u, -0.02f, 0.02f);
  hipLaunchKernelGGL(fill_uniform, dim3(4096), dim3(256), 0, 0, Tf, (size_t)nfrag * 8, 3u, -0.01f, 0.01f);
  CK(hipGetLastError());
  const double bytes = 2.0 * 2.0 * nA * 4;  // A and V read and written
  hipLaunchKernelGGL(split_ts<3>, dim3((nfrag + 255) / 256), dim3(256), 0, 0, Tf, Ts, nfrag);
  CK(hipDeviceSynchronize());
  if (run<3, 0>("production", A, V, m, nq, pairs, Ts, skip, bytes)) return 1;
  if (run<3, 1>("one_mfma_per_kb", A, V, m, nq, pairs, Ts, skip, bytes)) return 1;
  if (run<3, 2>("no_global_memory", A, V, m, nq, pairs, Ts, skip, bytes)) return 1;
  if (run<3, 3>("one_mfma_no_memory", A, V, m, nq, pairs, Ts, skip, bytes)) return 1;
  if (run<3, 4>("no_mfma_loop", A, V, m, nq, pairs, Ts, skip, bytes)) return 1;
  if (run<3, 6>("split_epilogue_only", A, V, m, nq, pairs, Ts, skip, bytes)) return 1;
  if (run<3, 8>("never_cheap", A, V, m, nq, pairs, Ts, skip, bytes)) return 1;
  // small T - I (~U(-0.001, 0.001)): every k half below 2^-9, the cheap form
  hipLaunchKernelGGL(fill_uniform, dim3(4096), dim3(256), 0, 0, Tf, (size_t)nfrag * 8, 3u, -0.001f, 0.001f);
  hipLaunchKernelGGL(split_ts<3>, dim3((nfrag + 255) / 256), dim3(256), 0, 0, Tf, Ts, nfrag);
  CK(hipDeviceSynchronize());
  if (run<3, 0>("production_all_cheap", A, V, m, nq, pairs, Ts, skip, bytes)) return 1;
  if (run<3, 2>("all_cheap_no_global_memory", A, V, m, nq, pairs, Ts, skip, bytes)) return 1;
  if (run<3, 8>("never_cheap_small_t", A, V, m, nq, pairs, Ts, skip, bytes)) return 1;
  hipLaunchKernelGGL(fill_uniform, dim3(4096), dim3(256), 0, 0, Tf, (size_t)nfrag * 8, 3u, -0.01f, 0.01f);
  hipLaunchKernelGGL(split_ts<2>, dim3((nfrag + 255) / 256), dim3(256), 0, 0, Tf, Ts, nfrag);
  CK(hipDeviceSynchronize());
  if (run<2, 0>("production_np2", A, V, m, nq, pairs, Ts, skip, bytes)) return 1;
  if (run<2, 2>("np2_no_global_memory", A, V, m, nq, pairs, Ts, skip, bytes)) return 1;
  // the quad Gram at the same geometry (4 row chunks per quad, as the merged step)
  float* slabs;
  CK(hipMalloc(&slabs, (size_t)3 * 2 * nq * 4 * 64 * 64 * 4));
  if (run_gram<0>("production", A, m, nq, pairs, slabs, 4)) return 1;
  if (run_gram<1>("one_mfma", A, m, nq, pairs, slabs, 4)) return 1;
  if (run_gram<2>("no_global_memory", A, m, nq, pairs, slabs, 4)) return 1;
  if (run_gram<3>("one_mfma_no_memory", A, m, nq, pairs, slabs, 4)) return 1;
  return 0;
}
