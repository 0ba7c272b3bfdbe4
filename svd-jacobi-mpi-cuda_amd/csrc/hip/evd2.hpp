// Two-level EVD of the 64 x 64 pair Gram (W = 32) -- included by block.hip.
//
// The flat kernel (evd_kernel) runs 63 parallel Jacobi steps per sweep, each
// a workgroup-wide barrier pair around a few thousand tiny LDS updates: it
// is latency-bound (~2.3k cycles/step measured).  Here the 64 indices are cut
// into 8 sub-blocks of 8; a sweep is 7 super-steps of a round robin over the
// sub-blocks.  In a super-step each of the 4 waves owns one 16-index
// sub-problem (two sub-blocks) and runs a full 15-step Jacobi sweep on its
// 16 x 16 principal submatrix ENTIRELY INSIDE THE WAVE (wave-private LDS,
// no workgroup barrier; rotations re-solved redundantly per lane; the 16 x 16
// rotation J_x accumulated in fp64 registers with the same DPP round robin as
// the flat kernel).  Then the whole G and Q are updated with matrix cores:
//   G[I_x, I_y] <- J_x^T G[I_x, I_y] J_y   (v_mfma_f32_16x16x4f32 / _f64, the
//                                            first product's accumulator is
//                                            the second product's B operand),
//   Q[:, I_x]   <- Q[:, I_x] J_x           (v_mfma_f64_16x16x4f64, Q in fp64).
// Two workgroup barriers per super-step instead of two per Jacobi step.
#pragma once

namespace svdj {

constexpr int kEvd2Threads = 256;  // 4 waves = 4 sub-problems per super-step

// Position-form circle method (see evd_kernel): slot a of step st pairs
// (player at pos a, player at pos NN-1-a); player NN-1 is fixed.
template <int NN>
__device__ __forceinline__ void circle_pair(int st, int a, int& p, int& q) {
  constexpr int M = NN - 1;
  if (a == 0) {
    p = NN - 1;
    q = (M - (st % M)) % M;
  } else {
    p = (a - (st % M) + M) % M;
    q = (M - a - (st % M) + M) % M;
  }
}

template <typename T>
struct Mfma16;
template <>
struct Mfma16<float> {  // v_mfma_f32_16x16x4_f32: D row = 4*(l>>4) + e
  using acc_t = f32x4;
  __device__ static __forceinline__ acc_t mfma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ int row(int e, int l) { return 4 * (l >> 4) + e; }
};
template <>
struct Mfma16<double> {  // v_mfma_f64_16x16x4_f64: D row = (l>>4) + 4*e
  using acc_t = f64x4;
  __device__ static __forceinline__ acc_t mfma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ int row(int e, int l) { return (l >> 4) + 4 * e; }
};

template <typename T>
__device__ __forceinline__ typename Mfma16<T>::acc_t zero16() {
  typename Mfma16<T>::acc_t z;
  z[0] = z[1] = z[2] = z[3] = T(0);
  return z;
}

template <typename T>
__global__ __launch_bounds__(kEvd2Threads) void evd2_kernel(
    const int32_t* __restrict__ pairs, int full, const T* __restrict__ slabs, int nchunk,
    T* __restrict__ D, T* __restrict__ Qout, int32_t* __restrict__ skip, T tol,
    int max_inner, uint32_t* __restrict__ metric) {
  constexpr int W = 32, N = 64, LD = N + 1;
  constexpr int SB = 8, NSB = N / SB;     // sub-blocks
  constexpr int NS = 2 * SB;              // sub-problem size (16)
  constexpr int LH = NS + 1;              // padded H row
  constexpr int LQ = N + 1;               // padded Q row (fp64)
  using MF = Mfma16<T>;
  using MD = Mfma16<double>;

  __shared__ T G[N * LD];
  __shared__ double Q[N * LQ];
  __shared__ T Hb[4][2][NS * LH];
  __shared__ double Jb[4][NS * NS];
  __shared__ int sweep_rot;
  __shared__ float wmax[kEvd2Threads / SVDJ_WAVE];

  const int pair = blockIdx.x;
  const int bi = pairs[2 * pair], bj = pairs[2 * pair + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // ---- assemble G (full symmetric storage), Q = I
  if (full) {
    const T* s0 = slabs + (size_t)pair * nchunk * (4 * W * W);
    for (int i = tid; i < N * N; i += kEvd2Threads) {
      T acc = 0;
#pragma unroll 4
      for (int c = 0; c < nchunk; ++c) acc += s0[(size_t)c * 4 * W * W + i];
      G[(i / N) * LD + (i % N)] = acc;
    }
  } else {
    const T* s0 = slabs + (size_t)pair * nchunk * (W * W);
    for (int i = tid; i < N * N; i += kEvd2Threads) G[(i / N) * LD + (i % N)] = T(0);
    __syncthreads();
    for (int i = tid; i < W * W; i += kEvd2Threads) {
      T acc = 0;
#pragma unroll 4
      for (int c = 0; c < nchunk; ++c) acc += s0[(size_t)c * W * W + i];
      const int a = i / W, b = i % W;
      G[a * LD + W + b] = acc;
      G[(W + b) * LD + a] = acc;
    }
    for (int a = tid; a < W; a += kEvd2Threads) {
      G[a * LD + a] = D[bi * W + a];
      G[(W + a) * LD + W + a] = D[bj * W + a];
    }
  }
  for (int i = tid; i < N * N; i += kEvd2Threads) Q[(i / N) * LQ + (i % N)] = (i / N == i % N) ? 1.0 : 0.0;
  if (tid == 0) sweep_rot = 0;
  __syncthreads();

  // ---- convergence value before any rotation
  {
    float mx = 0.0f;
    for (int i = tid; i < N * N; i += kEvd2Threads) {
      const int r = i / N, c = i % N;
      const bool use = full ? (r < c) : (r < W && c >= W);
      if (!use) continue;
      const T d = sqrt(G[r * LD + r]) * sqrt(G[c * LD + c]);
      if (d > T(0)) {
        const float v = (float)(fabs(G[r * LD + c]) / d);
        mx = v > mx ? v : mx;
      }
    }
    mx = wave_max(mx);
    if (lane == 0) wmax[wave] = mx;
    __syncthreads();
    if (tid == 0) {
      float m2 = 0.0f;
      for (int w = 0; w < kEvd2Threads / SVDJ_WAVE; ++w) m2 = wmax[w] > m2 ? wmax[w] : m2;
      atomic_max_pos(&metric[0], m2);
    }
  }

  // ---- per-lane roles inside the wave's 16 x 16 sub-problem
  const int slot = lane & 7;   // rotation slot (8 per sub-sweep step)
  const int grp = lane >> 3;   // 8 groups: J rows 2*grp, 2*grp+1; block offset d = grp
  const int dblk = grp;
  const bool own_blk = dblk < 4 || (dblk == 4 && slot < 4);
  const int bslot = (slot + dblk) & 7;
  int jp0, jq0;
  circle_pair<NS>(0, slot, jp0, jq0);

  bool any = false;
  for (int sw = 0; sw < max_inner; ++sw) {
    for (int ss = 0; ss < NSB - 1; ++ss) {
      // ===== phase A: wave x solves sub-problem x (sub-blocks alpha, beta)
      int alpha, beta;
      circle_pair<NSB>(ss, wave, alpha, beta);
      auto gidx = [&](int i) { return i < SB ? alpha * SB + i : beta * SB + (i - SB); };
      T* H0 = Hb[wave][0];
      T* H1 = Hb[wave][1];
      for (int e = lane; e < NS * NS; e += 64) {
        const int r = e / NS, c = e % NS;
        H0[r * LH + c] = G[gidx(r) * LD + gidx(c)];
      }
      double jf[2], js[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int k = 2 * grp + i;
        jf[i] = (k == jp0) ? 1.0 : 0.0;
        js[i] = (k == jq0) ? 1.0 : 0.0;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bool wrot = false;
      int cur = 0;
      for (int st = 0; st < NS - 1; ++st) {
        const T* Hc = cur ? H1 : H0;
        T* Hn = cur ? H0 : H1;
        int p, q;
        circle_pair<NS>(st, slot, p, q);
        T ca, sa, ta;
        const T hpp = Hc[p * LH + p], hqq = Hc[q * LH + q], hpq = Hc[p * LH + q];
        const bool rot = rotation_fast(hpp, hqq, hpq, tol, ca, sa, ta);
        if (!rot) { ca = T(1); sa = T(0); ta = T(0); }
        if (own_blk) {
          if (dblk == 0) {
            Hn[p * LH + p] = hpp - ta * hpq;
            Hn[q * LH + q] = hqq + ta * hpq;
            const T v = rot ? T(0) : hpq;
            Hn[p * LH + q] = v;
            Hn[q * LH + p] = v;
          } else {
            int r, u;
            circle_pair<NS>(st, bslot, r, u);
            T cb, sb, tb;
            if (!rotation_fast(Hc[r * LH + r], Hc[u * LH + u], Hc[r * LH + u], tol, cb, sb, tb)) {
              cb = T(1);
              sb = T(0);
            }
            const T g00 = Hc[p * LH + r], g01 = Hc[p * LH + u];
            const T g10 = Hc[q * LH + r], g11 = Hc[q * LH + u];
            const T h00 = ca * g00 - sa * g10, h01 = ca * g01 - sa * g11;
            const T h10 = sa * g00 + ca * g10, h11 = sa * g01 + ca * g11;
            const T n00 = cb * h00 - sb * h01, n01 = sb * h00 + cb * h01;
            const T n10 = cb * h10 - sb * h11, n11 = sb * h10 + cb * h11;
            Hn[p * LH + r] = n00; Hn[r * LH + p] = n00;
            Hn[p * LH + u] = n01; Hn[u * LH + p] = n01;
            Hn[q * LH + r] = n10; Hn[r * LH + q] = n10;
            Hn[q * LH + u] = n11; Hn[u * LH + q] = n11;
          }
        }
        if (rot) {
          wrot = true;
          double c64, s64;
          if constexpr (sizeof(T) == 8) {
            c64 = ca;
            s64 = sa;
          } else {
            const double td = (double)ta;
            c64 = rsqrt64(1.0 + td * td);
            s64 = td * c64;
          }
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const double x = jf[i], y = js[i];
            jf[i] = c64 * x - s64 * y;
            js[i] = s64 * x + c64 * y;
          }
        }
        // this wave's LDS writes must land before its next step reads them
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        cur ^= 1;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const double f_r = dpp_shr1(jf[i]), s_r = dpp_shr1(js[i]), s_l = dpp_shl1(js[i]);
          const double nf = slot == 0 ? jf[i] : (slot == 1 ? s_r : f_r);
          const double ns = slot == 7 ? jf[i] : s_l;
          jf[i] = nf;
          js[i] = ns;
        }
      }
      // J_x (16 x 16, fp64): after 15 steps the circle is back at step 0
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int k = 2 * grp + i;
        Jb[wave][k * NS + jp0] = jf[i];
        Jb[wave][k * NS + jq0] = js[i];
      }
      const bool wany = __any(wrot);
      if (wany && lane == 0) sweep_rot = 1;
      __syncthreads();

      // ===== phase B: G[I_x, I_y] <- J_x^T G[I_x, I_y] J_y (y >= x), mirror
      for (int y = wave; y < 4; ++y) {
        int ay, by_;
        circle_pair<NSB>(ss, y, ay, by_);
        auto gy = [&](int i) { return i < SB ? ay * SB + i : by_ * SB + (i - SB); };
        const double* Jy = Jb[y];
        const double* Jx = Jb[wave];
        const int li = lane & 15, lk = lane >> 4;
        // stage 1: T1 = G[I_x, I_y] J_y ; lane: A[i=li][k=lk+4kk], B[k][j=li]
        typename MF::acc_t t1 = zero16<T>();
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int k = 4 * kk + lk;
          t1 = MF::mfma(G[gidx(li) * LD + gy(k)], (T)Jy[k * NS + li], t1);
        }
        // stage 2: G' = J_x^T T1 with T1's accumulator as the B operand:
        // k-step kk uses k = MF::row(kk, lane) so B = t1[kk] (same lane)
        typename MF::acc_t g2 = zero16<T>();
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int k = MF::row(kk, lane);
          g2 = MF::mfma((T)Jx[k * NS + li], t1[kk], g2);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = MF::row(e, lane);
          G[gidx(r) * LD + gy(li)] = g2[e];
          if (y != wave) G[gy(li) * LD + gidx(r)] = g2[e];
        }
      }
      // ===== Q[:, I_x] <- Q[:, I_x] J_x  (fp64 MFMA), 4 row tiles of 16
      {
        const double* Jx = Jb[wave];
        const int li = lane & 15, lk = lane >> 4;
        for (int kt = 0; kt < N / 16; ++kt) {
          double a[4];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) a[kk] = Q[(kt * 16 + li) * LQ + gidx(4 * kk + lk)];
          typename MD::acc_t acc = zero16<double>();
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) acc = MD::mfma(a[kk], Jx[(4 * kk + lk) * NS + li], acc);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int e = 0; e < 4; ++e) Q[(kt * 16 + MD::row(e, lane)) * LQ + gidx(li)] = acc[e];
        }
      }
      __syncthreads();
    }
    const int rot = sweep_rot;
    __syncthreads();
    if (tid == 0) sweep_rot = 0;
    if (!rot) break;
    any = true;
    __syncthreads();
  }

  if (tid == 0) {
    skip[pair] = any ? 0 : 1;
    if (any) atomicAdd(&metric[1], 1u);
  }
  if (!any && !full) return;
  if (any) {
    T* qo = Qout + (size_t)pair * N * N;
    for (int i = tid; i < N * N; i += kEvd2Threads) qo[i] = (T)Q[(i / N) * LQ + (i % N)];
  }
  for (int c = tid; c < N; c += kEvd2Threads) {
    const int col = (c < W ? bi * W + c : bj * W + (c - W));
    D[col] = G[c * LD + c];
  }
}

}  // namespace svdj
