// Column-pair / block-pair schedules (host C++).
//
// Reference parity: the Sameh 1971 ordering used by the reference for its
// scalar sweep (reference main.cu:500-538 first half, main.cu:945-983 second
// half).  The reference recomputes this every step
// inside an OpenMP loop whose thread id doubles as the MPI rank
// (main.cu:525-554); here it is a pure function evaluated once per solve and
// uploaded to the GPU as a table.
//
// MI355X-native additions: the circle-method round robin used for block
// pairs inside one GPU, the bipartite "cross" schedule between two resident
// super-blocks, and the multi-GPU super-block tournament in which every GPU
// exchanges exactly ONE super-block per round (one xGMI send + one recv),
// instead of the reference's root-centred scatter/gather of every column set
// every step (main.cu:582-680, 854-936).
#include "svdj_cpu.h"

#include <cstddef>
#include <vector>

extern "C" int svdj_sameh_num_steps(int n) {
  if (n < 2) return 0;
  return (n % 2 == 0) ? n - 1 : n;
}

extern "C" int svdj_sameh_schedule(int n, int32_t* out) {
  if (n < 2 || out == nullptr) return 0;
  const long M = (n + 1) / 2;  // m_ordering
  const int steps = svdj_sameh_num_steps(n);
  const int half = n / 2;
  for (long i = 0; i < (long)steps * half * 2; ++i) out[i] = -1;
  int step = 0;
  // First half: k = 1 .. M-1, q = M-k+1 .. n-k (1-based).
  for (long k = 1; k < M; ++k, ++step) {
    int slot = 0;
    for (long q = M - k + 1; q <= n - k; ++q) {
      long p;
      if (q <= 2 * M - 2 * k) {
        p = 2 * M - 2 * k + 1 - q;
      } else if (q <= 2 * M - k - 1) {
        p = 4 * M - 2 * k - q;
      } else {
        p = n;
      }
      if (slot < half) {
        out[((long)step * half + slot) * 2 + 0] = (int32_t)(p - 1);
        out[((long)step * half + slot) * 2 + 1] = (int32_t)(q - 1);
      }
      ++slot;
    }
  }
  // Second half: k = M .. 2M-1, q = 4M-n-k .. 3M-k-1 (1-based).
  for (long k = M; k < 2 * M; ++k, ++step) {
    int slot = 0;
    for (long q = 4 * M - n - k; q < 3 * M - k; ++q) {
      long p;
      if (q < 2 * M - k + 1) {
        p = n;
      } else if (q <= 4 * M - 2 * k - 1) {
        p = 4 * M - 2 * k - q;
      } else {
        p = 6 * M - 2 * k - 1 - q;
      }
      if (slot < half) {
        out[((long)step * half + slot) * 2 + 0] = (int32_t)(p - 1);
        out[((long)step * half + slot) * 2 + 1] = (int32_t)(q - 1);
      }
      ++slot;
    }
  }
  return step;
}

extern "C" int svdj_round_robin(int nb, int32_t* out) {
  if (nb < 2 || (nb % 2) != 0 || out == nullptr) return -1;
  const int rounds = nb - 1;
  const int half = nb / 2;
  for (int r = 0; r < rounds; ++r) {
    int32_t* o = out + (long)r * half * 2;
    o[0] = r;
    o[1] = nb - 1;
    for (int k = 1; k < half; ++k) {
      int a = (r + k) % (nb - 1);
      int b = (r - k + (nb - 1)) % (nb - 1);
      if (a > b) { int t = a; a = b; b = t; }
      o[2 * k + 0] = a;
      o[2 * k + 1] = b;
    }
  }
  return rounds;
}

extern "C" int svdj_bipartite(int k, int32_t* out) {
  if (k < 1 || out == nullptr) return -1;
  for (int t = 0; t < k; ++t)
    for (int a = 0; a < k; ++a) {
      out[((long)t * k + a) * 2 + 0] = a;
      out[((long)t * k + a) * 2 + 1] = k + (a + t) % k;
    }
  return k;
}

// Quad orders (csrc/hip/block.hip "quad step"; parallel/schedule.py twins):
// two consecutive steps fuse over the four blocks (a, b, c, d) of a
// super-block pair {a, b} x {c, d}: step s pairs (a, c), (b, d), step s+1
// (a, d), (b, c), as pairs 2q, 2q+1 of quad q.
extern "C" int svdj_quad_round_robin(int nb, int32_t* out) {
  if (nb < 4 || nb % 4 || out == nullptr) return -1;
  const int K = nb / 2;  // super-blocks (2i, 2i+1)
  for (int i = 0; i < K; ++i) {  // step 0: within every super-block (the full-Gram step)
    out[2 * i] = 2 * i;
    out[2 * i + 1] = 2 * i + 1;
  }
  std::vector<int32_t> srr((size_t)(K - 1) * (K / 2) * 2);
  svdj_round_robin(K, srr.data());
  for (int t = 0; t < K - 1; ++t)
    for (int q = 0; q < K / 2; ++q) {
      const int I = srr[((size_t)t * (K / 2) + q) * 2], J = srr[((size_t)t * (K / 2) + q) * 2 + 1];
      const int a = 2 * I, b = 2 * I + 1, c = 2 * J, d = 2 * J + 1;
      int32_t* s1 = out + (size_t)(1 + 2 * t) * K * 2 + 4 * q;
      int32_t* s2 = out + (size_t)(2 + 2 * t) * K * 2 + 4 * q;
      s1[0] = a, s1[1] = c, s1[2] = b, s1[3] = d;
      s2[0] = a, s2[1] = d, s2[2] = b, s2[3] = c;
    }
  return nb - 1;
}

extern "C" int svdj_quad_bipartite(int h, const int32_t* xs, const int32_t* ys, int32_t* out) {
  if (h < 2 || h % 2 || !xs || !ys || !out) return -1;
  const int H = h / 2;
  for (int t = 0; t < H; ++t)
    for (int i = 0; i < H; ++i) {
      const int j = (i + t) % H;
      const int a = xs[2 * i], b = xs[2 * i + 1], c = ys[2 * j], d = ys[2 * j + 1];
      int32_t* s1 = out + (size_t)(2 * t) * h * 2 + 4 * i;
      int32_t* s2 = out + (size_t)(2 * t + 1) * h * 2 + 4 * i;
      s1[0] = a, s1[1] = c, s1[2] = b, s1[3] = d;
      s2[0] = a, s2[1] = d, s2[2] = b, s2[3] = c;
    }
  return h;
}

extern "C" int svdj_tournament(int P, int32_t* held, int32_t* xslot,
                               int32_t* send_to, int32_t* recv_from) {
  if (P < 1 || held == nullptr) return -1;
  const int nb = 2 * P;
  const int rounds = nb - 1;
  std::vector<int32_t> rr((size_t)rounds * P * 2);
  svdj_round_robin(nb, rr.data());
  auto H = [&](int r, int g, int s) -> int32_t& { return held[((long)r * P + g) * 2 + s]; };
  for (int r = 0; r < rounds; ++r)
    for (int g = 0; g < P; ++g) {
      if (xslot) xslot[(long)r * P + g] = -1;
      if (send_to) send_to[(long)r * P + g] = -1;
      if (recv_from) recv_from[(long)r * P + g] = -1;
    }
  for (int g = 0; g < P; ++g) {
    H(0, g, 0) = rr[2 * g + 0];
    H(0, g, 1) = rr[2 * g + 1];
  }
  std::vector<int> gpu_of(nb), slot_of(nb), partner(nb);
  std::vector<char> done(P);
  for (int r = 1; r < rounds; ++r) {
    for (int g = 0; g < P; ++g) {
      gpu_of[H(r - 1, g, 0)] = g; slot_of[H(r - 1, g, 0)] = 0;
      gpu_of[H(r - 1, g, 1)] = g; slot_of[H(r - 1, g, 1)] = 1;
    }
    const int32_t* m = rr.data() + (size_t)r * P * 2;
    for (int e = 0; e < P; ++e) { partner[m[2 * e]] = m[2 * e + 1]; partner[m[2 * e + 1]] = m[2 * e]; }
    for (int g = 0; g < P; ++g) done[g] = 0;
    for (int g0 = 0; g0 < P; ++g0) {
      if (done[g0]) continue;
      int g = g0, keep = 1;
      for (int guard = 0; guard <= P; ++guard) {
        const int kept = H(r - 1, g, keep);
        const int other = partner[kept];
        H(r, g, keep) = kept;
        H(r, g, 1 - keep) = other;
        done[g] = 1;
        const int h = gpu_of[other];
        if (xslot) xslot[(long)r * P + g] = 1 - keep;
        if (recv_from) recv_from[(long)r * P + g] = h;
        if (send_to) send_to[(long)r * P + h] = g;
        if (h == g0) break;
        keep = 1 - slot_of[other];
        g = h;
      }
    }
  }
  return rounds;
}
