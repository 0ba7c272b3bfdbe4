// EVD kernel micro-benchmark (development aid): times one cross-step EVD
// launch of P pairs (the block step's middle kernel) in isolation, for the
// bipartite LDS kernel (mode 2) and the cross-only kernel (mode 3).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I<csrc/include> -I<csrc/hip> \
//         -c tools/micro/evd_bench.hip -o evd_bench.o
//   hipcc --offload-arch=gfx950 evd_bench.o <lib/obj/post.o> -o evd_bench
//   ./evd_bench P nchunk reps      (prints microseconds per launch)
#include "block.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>


template <typename K>
static double time_it(K launch, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a, nullptr);
  for (int r = 0; r < reps; ++r) launch();
  (void)hipEventRecord(b, nullptr);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1e3 / reps;
}

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 8, nchunk = argc > 2 ? atoi(argv[2]) : 1;
  const int reps = argc > 3 ? atoi(argv[3]) : 50;
  constexpr int W = 64;
  std::vector<int32_t> hp(2 * P);
  for (int p = 0; p < P; ++p) hp[2 * p] = 2 * p, hp[2 * p + 1] = 2 * p + 1;
  std::vector<float> hs((size_t)P * nchunk * W * W), hd((size_t)2 * P * W);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) * (1.0f / 16777216.0f); };
  for (auto& x : hs) x = (rnd() - 0.5f) * 0.2f / nchunk;
  for (auto& x : hd) x = 1.0f + rnd();
  int32_t *dp, *dsk, *dns;
  float *dsl, *dD, *dQ;
  uint32_t* dm;
  float* drec;
  (void)hipMalloc(&drec, (size_t)P * svdj::kCrossMaxInner * W * W * sizeof(*drec));
  (void)hipMalloc(&dns, P * 4);
  (void)hipMalloc(&dp, hp.size() * 4);
  (void)hipMalloc(&dsl, hs.size() * 4);
  (void)hipMalloc(&dD, hd.size() * 4);
  (void)hipMalloc(&dQ, (size_t)P * 4 * W * W * 4);
  (void)hipMalloc(&dsk, P * 4);
  (void)hipMalloc(&dm, 8);
  (void)hipMemcpy(dp, hp.data(), hp.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dsl, hs.data(), hs.size() * 4, hipMemcpyHostToDevice);
  auto reset = [&]() { (void)hipMemcpy(dD, hd.data(), hd.size() * 4, hipMemcpyHostToDevice); };
  reset();
  const double tb = time_it([&]() {
    hipLaunchKernelGGL((svdj::evd_kernel<float, W, svdj::EVD_BIP>), dim3(P), dim3(svdj::evd_threads(W)), 0,
                       nullptr, dp, 0, dsl, nchunk, dD, dQ, dsk, 1e-6f, 0, 1, dm);
  }, reps);
  reset();
  const double tc = time_it([&]() {
    hipLaunchKernelGGL((svdj::evd_cross_kernel<float, W>), dim3(P), dim3(svdj::cross_threads<W>()), 0,
                       nullptr, dp, dsl, nchunk, dD, drec, dns, dsk, 1e-6f, 0, 1, dm);
  }, reps);
  reset();
  const double tq = time_it([&]() {
    hipLaunchKernelGGL((svdj::evd_cross_kernel<float, W>), dim3(P), dim3(svdj::cross_threads<W>()), 0,
                       nullptr, dp, dsl, nchunk, dD, drec, dns, dsk, 1e-6f, 0, 1, dm);
    if (P >= 32)
      hipLaunchKernelGGL((svdj::qbuild_kernel<float, W, 16>), dim3(P, svdj::qbuild_blocks<W, 16>()),
                         dim3(svdj::kQbThreads), 0, nullptr, drec, dns, dsk, dQ);
    else
      hipLaunchKernelGGL((svdj::qbuild_kernel<float, W, 4>), dim3(P, svdj::qbuild_blocks<W, 4>()),
                         dim3(svdj::kQbThreads), 0, nullptr, drec, dns, dsk, dQ);
  }, reps);
  std::printf("P %d nchunk %d: bipartite %.2f us  cross evd %.2f us  cross evd+qbuild %.2f us\n",
              P, nchunk, tb, tc, tq);
#ifdef EVD_ABL
  // evd_cross_kernel ablations (its ABL flags): where a step's time goes
  auto abl = [&](auto ablc, const char* what) {
    constexpr int A = decltype(ablc)::value;
    reset();
    const double t = time_it([&]() {
      hipLaunchKernelGGL((svdj::evd_cross_kernel<float, W, A>), dim3(P), dim3(svdj::cross_threads<W>()), 0,
                         nullptr, dp, dsl, nchunk, dD, drec, dns, dsk, 1e-6f, 0, 1, dm);
    }, reps);
    std::printf("  abl %2d %-44s %.2f us\n", A, what, t);
  };
  abl(std::integral_constant<int, 1>{}, "no fp64 records");
  abl(std::integral_constant<int, 2>{}, "waves >= 1 idle");
  abl(std::integral_constant<int, 4>{}, "no rotation solve");
  abl(std::integral_constant<int, 8>{}, "solver lane: no LDS coupling traffic");
  abl(std::integral_constant<int, 3>{}, "records off, waves >= 1 idle");
  abl(std::integral_constant<int, 7>{}, "records off, idle, no solve");
  abl(std::integral_constant<int, 15>{}, "all off (barriers, DPP, bookkeeping)");
  abl(std::integral_constant<int, 16>{}, "no steps (assembly, launch, epilogue)");
  // diagonals per wave >= 1 (fewer waves at each step's barrier, more LDS work per wave)
  auto dpw = [&](auto dc) {
    constexpr int D = decltype(dc)::value;
    reset();
    const double t = time_it([&]() {
      hipLaunchKernelGGL((svdj::evd_cross_kernel<float, W, 0, D>), dim3(P),
                         dim3(svdj::cross_threads<W, D>()), 0, nullptr, dp, dsl, nchunk, dD, drec,
                         dns, dsk, 1e-6f, 0, 1, dm);
    }, reps);
    std::printf("  dpw %2d (%4d threads)                           %.2f us\n", D,
                svdj::cross_threads<W, D>(), t);
  };
  dpw(std::integral_constant<int, 2>{});
  dpw(std::integral_constant<int, 3>{});
  dpw(std::integral_constant<int, 4>{});
  dpw(std::integral_constant<int, 5>{});
  dpw(std::integral_constant<int, 6>{});
  dpw(std::integral_constant<int, 8>{});
  dpw(std::integral_constant<int, 10>{});
  dpw(std::integral_constant<int, 15>{});
#endif
  return 0;
}
