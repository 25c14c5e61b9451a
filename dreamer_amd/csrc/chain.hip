// Fused per-step kernels of the imagination chain (Dreamer.py:158-164).
#include "chain.h"

#include <algorithm>

// ---------------------------------------------------------------------------
// k_actor_tail: the actor of one imagined step in one launch (chain.h).  It
// replaces three launches of the round-3 chain -- the one-hot z-gather of
// base_net.0 (k_zgather_add), the LN-SiLU + base_net.3 product and the
// LN-SiLU + stacked-heads product with the rsample epilogue (two skinny GEMMs):
// 5.3 + 6.2 + 8.2 us at B = 256.  A workgroup owns AT_ROWS batch rows and all
// of their columns, so both LayerNorms are local:
//   P1  indices / straight-through values of the rows and the two heads'
//       weights into LDS, the rows' h-parts into registers;
//   P2  the gather: thread (row, 4 columns) reads the R sampled rows of the
//       transposed z-columns (every load issued before the first add) and adds
//       them in group order, as k_zgather_add;
//   P3  base_net.3's rows are requested (thread (output j, half of K) holds its
//       half row in registers) while wave r normalises row r (LN + SiLU);
//   P4  pre2 = x1 W3^T + b3: each thread 2 x AT_ROWS dot products over its
//       half of K against x1 broadcast from LDS, the halves met by a lane swap;
//   P5  wave r: LN + SiLU of pre2, then the 2A head dot products (DPP sums);
//   P6  lanes i < A: clamp, softplus, tanh(mu + eps sigma) (EPI_ACTOR's math).
// ---------------------------------------------------------------------------
#define AT_ROWS 8
#define AT_NT 512
#define AT_MAXR 32     // latent groups
#define AT_KH4 25      // float4 per half row of base_net.3 (a1 <= 200)
#define AT_MAXW 256    // a1, a2 <= 256 (one float4 per lane)
#define AT_MAXH 16     // 2A <= 16

__device__ __forceinline__ float4 at_ln_silu(float4 x, bool ok, int K, float4 gv, float4 bv) {
  const float mean = wave_sum(ok ? (x.x + x.y) + (x.z + x.w) : 0.f) / (float)K;
  float sq = 0.f;
  if (ok) {
    const float dx = x.x - mean, dy = x.y - mean, dz = x.z - mean, dw = x.w - mean;
    sq = (dx * dx + dy * dy) + (dz * dz + dw * dw);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(sq) / (float)K + 1e-5f);
  if (!ok) return make_float4(0.f, 0.f, 0.f, 0.f);
  return make_float4(dr_silu_fast((x.x - mean) * rstd * gv.x + bv.x), dr_silu_fast((x.y - mean) * rstd * gv.y + bv.y),
                     dr_silu_fast((x.z - mean) * rstd * gv.z + bv.z), dr_silu_fast((x.w - mean) * rstd * gv.w + bv.w));
}

__global__ __launch_bounds__(AT_NT) void k_actor_tail(ActorTailArgs aa) {
  __shared__ ActorTailArgs a;
  dr_stage_args(aa, a, threadIdx.x);
  __shared__ int s_idx[AT_ROWS][AT_MAXR];
  __shared__ float s_zv[AT_ROWS][AT_MAXR];
  __shared__ __attribute__((aligned(16))) float s_x[AT_ROWS][AT_MAXW];   // pre1, then x1
  __shared__ __attribute__((aligned(16))) float s_p2[AT_ROWS][AT_MAXW];
  __shared__ __attribute__((aligned(16))) float s_wst[AT_MAXH][AT_MAXW];
  const int M = dr_uni(a.M), A = dr_uni(a.A), a1 = dr_uni(a.a1), a2 = dr_uni(a.a2);
  const int R = dr_uni(a.R), C = dr_uni(a.C);
  const int m0 = blockIdx.x * AT_ROWS;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int c4n = a1 >> 2;  // float4 columns of base_net.0
  // ---- P1: indices / values, stacked heads -> LDS; h-part -> registers ----
  for (int x = tid; x < AT_ROWS * AT_MAXR; x += AT_NT) {
    const int ml = x / AT_MAXR, u = x - ml * AT_MAXR, m = m0 + ml;
    const bool ok = m < M && u < R;
    s_idx[ml][u] = ok ? dr_g(a.idx)[m * R + u] : 0;
    s_zv[ml][u] = ok ? dr_g(a.zval)[m * R + u] : 0.f;
  }
  const float* wmu = dr_uni(a.wmu);
  const float* wls = dr_uni(a.wls);
  for (int x = tid; x < 2 * A * (a2 >> 2); x += AT_NT) {
    const int o = x / (a2 >> 2), k4 = x - o * (a2 >> 2);
    const float* src = o < A ? wmu : wls;
    const int oo = o < A ? o : o - A;
    *reinterpret_cast<float4*>(&s_wst[o][4 * k4]) = dr_ld4(src, (unsigned)(oo * a2 + 4 * k4));
  }
  const bool gthr = tid < AT_ROWS * c4n;
  const int gr = gthr ? tid / c4n : 0, gc = gthr ? tid - gr * c4n : 0, gm = m0 + gr;
  const bool glive = gthr && gm < M;
  const float4 hp = dr_ld4(dr_uni(a.hpart), glive ? (unsigned)(gm * (int)a.ldh + 4 * gc) : 0u);
  __syncthreads();
  // ---- P2: pre1 = hpart + sum_u zval[u] * wzt[u*C + idx[u]] ----
  {
    const float* wzt = dr_uni(a.wzt);
    const int ldw = dr_uni((int)a.ldw);
    float4 w[AT_MAXR];
#pragma unroll
    for (int u = 0; u < AT_MAXR; ++u) {
      const int iv = s_idx[gr][u];
      const bool ok = glive && u < R && iv >= 0;
      w[u] = dr_ld4(wzt, ok ? (unsigned)((u * C + iv) * ldw + 4 * gc) : 0u);
    }
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    bool dense = false;
#pragma unroll
    for (int u = 0; u < AT_MAXR; ++u) {
      if (u < R) {
        const float zv = s_zv[gr][u];
        dense = dense || s_idx[gr][u] < 0;
        v.x = fmaf(w[u].x, zv, v.x);
        v.y = fmaf(w[u].y, zv, v.y);
        v.z = fmaf(w[u].z, zv, v.z);
        v.w = fmaf(w[u].w, zv, v.w);
      }
    }
    if (dense && glive) {  // groups with several non-zero classes: every class
      const float* zr = a.z + (long long)gm * a.ldz;
      for (int u = 0; u < R; ++u) {
        if (s_idx[gr][u] >= 0) continue;
        for (int c = 0; c < C; ++c) {
          const float zc = zr[u * C + c];
          const float4 wc = dr_ld4(wzt, (unsigned)((u * C + c) * ldw + 4 * gc));
          v.x = fmaf(wc.x, zc, v.x);
          v.y = fmaf(wc.y, zc, v.y);
          v.z = fmaf(wc.z, zc, v.z);
          v.w = fmaf(wc.w, zc, v.w);
        }
      }
    }
    if (gthr) {
      const float4 p = make_float4(hp.x + v.x, hp.y + v.y, hp.z + v.z, hp.w + v.w);
      *reinterpret_cast<float4*>(&s_x[gr][4 * gc]) = p;
      if (glive) dr_st4(a.pre1, (unsigned)(gm * (int)a.ld1 + 4 * gc), p);
    }
  }
  __syncthreads();
  // ---- P3: base_net.3 half rows requested; wave r: x1 = SiLU(LN1(pre1[r])) ----
  const int j = tid >> 1, hf = tid & 1, kh = a1 >> 1;  // thread: output j, K half hf
  const bool wthr = j < a2;
  float4 w3[AT_KH4];
  {
    const float* W3 = dr_uni(a.w3);
#pragma unroll
    for (int i = 0; i < AT_KH4; ++i) {
      const bool ok = wthr && 4 * i < kh;
      w3[i] = dr_ld4(W3, ok ? (unsigned)(j * a1 + hf * kh + 4 * i) : 0u);
    }
  }
  const float b3 = dr_ld1(dr_uni(a.b3), wthr ? (unsigned)j : 0u);
  {
    const int m = m0 + wave;
    const bool ok = lane < c4n;
    const unsigned kk = ok ? 4u * lane : 0u;
    const float4 gv = dr_ld4(dr_uni(a.n1g), kk), bv = dr_ld4(dr_uni(a.n1b), kk);
    const float4 x = ok ? *reinterpret_cast<const float4*>(&s_x[wave][4 * lane]) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 y = at_ln_silu(x, ok, a1, gv, bv);
    __syncthreads();  // every wave has read its pre1 row before x1 overwrites it
    if (ok) {
      *reinterpret_cast<float4*>(&s_x[wave][4 * lane]) = y;
      if (m < M) dr_st4(a.x1, (unsigned)(m * (int)a.ld1 + 4 * lane), y);
    }
  }
  __syncthreads();
  // ---- P4: pre2 = x1 W3^T + b3 ----
  {
    float acc[AT_ROWS];
#pragma unroll
    for (int r = 0; r < AT_ROWS; ++r) acc[r] = 0.f;
#pragma unroll
    for (int i = 0; i < AT_KH4; ++i) {
      if (4 * i < kh) {
        const int k = hf * kh + 4 * i;
#pragma unroll
        for (int r = 0; r < AT_ROWS; ++r) {
          const float4 xv = *reinterpret_cast<const float4*>(&s_x[r][k]);
          acc[r] = fmaf(xv.x, w3[i].x, acc[r]);
          acc[r] = fmaf(xv.y, w3[i].y, acc[r]);
          acc[r] = fmaf(xv.z, w3[i].z, acc[r]);
          acc[r] = fmaf(xv.w, w3[i].w, acc[r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < AT_ROWS; ++r) {
      const float o = __shfl_xor(acc[r], 1, 64);
      const float v = (acc[r] + o) + b3;  // (hf 0 writes: first half + second half)
      if (wthr && hf == 0) {
        s_p2[r][j] = v;
        if (m0 + r < M) dr_g(a.pre2)[(long long)(m0 + r) * a.ld2 + j] = v;
      }
    }
  }
  __syncthreads();
  // ---- P5: wave r: x2 = SiLU(LN4(pre2[r])), then the 2A head dot products ----
  const int m = m0 + wave;
  const bool ok2 = lane < (a2 >> 2);
  const unsigned k2 = ok2 ? 4u * lane : 0u;
  float4 x2;
  {
    const float4 gv = dr_ld4(dr_uni(a.n4g), k2), bv = dr_ld4(dr_uni(a.n4b), k2);
    const float4 x = ok2 ? *reinterpret_cast<const float4*>(&s_p2[wave][4 * lane]) : make_float4(0.f, 0.f, 0.f, 0.f);
    x2 = at_ln_silu(x, ok2, a2, gv, bv);
    if (ok2 && m < M) dr_st4(a.x2, (unsigned)(m * (int)a.ld2 + 4 * lane), x2);
  }
  if (m >= M) return;  // whole waves
  float hd[AT_MAXH];
#pragma unroll
  for (int o = 0; o < AT_MAXH; ++o) {
    if (o < 2 * A) {
      float p = 0.f;
      if (ok2) {
        const float4 wv = *reinterpret_cast<const float4*>(&s_wst[o][4 * lane]);
        p = fmaf(x2.x, wv.x, p);
        p = fmaf(x2.y, wv.y, p);
        p = fmaf(x2.z, wv.z, p);
        p = fmaf(x2.w, wv.w, p);
      }
      hd[o] = wave_sum(p) + (o < A ? dr_g(a.bmu)[o] : dr_g(a.bls)[o - A]);
    }
  }
  // ---- P6: lanes i < A: the rsample epilogue (EPI_ACTOR, Agent.py:202-210) ----
  if (lane < A) {
    const int i = lane;
    float muv = 0.f, lr = 0.f;  // hd[i], hd[A + i] (compile-time register indices)
#pragma unroll
    for (int o = 0; o < AT_MAXH; ++o) {
      if (o < A && o == i) muv = hd[o];
      if (o >= A && o < 2 * A && o - A == i) lr = hd[o];
    }
    const float ls = fminf(fmaxf(lr, -5.0f), 2.0f);
    const float sg = dr_softplus(ls) + 1e-3f;
    float av;
    if (a.det) {
      av = tanhf(muv);
    } else {
      float e;
      if (a.noise.eps) {
        e = dr_g(a.noise.eps)[((long long)a.step * M + m) * A + i];
      } else {
        const unsigned long long* so = a.noise.rng;
        e = dr_normal_k(so[0], so[1], (uint32_t)(a.noise.stream + a.step), (uint32_t)(a.noise.row0 + m), (uint32_t)i);
      }
      if (a.eps_save) dr_g(a.eps_save)[(long long)m * A + i] = e;
      av = tanhf(muv + e * sg);
    }
    dr_g(a.act)[(long long)m * a.ldA + i] = av;
    dr_g(a.mu)[(long long)m * a.ldA + i] = muv;
    dr_g(a.sig)[(long long)m * a.ldA + i] = sg;
    if (a.ls_save) dr_g(a.ls_save)[(long long)m * a.ldA + i] = lr;
  }
}

bool op_actor_tail_ok(const ActorTailArgs& a) {
  const uintptr_t al = (uintptr_t)a.wzt | (uintptr_t)a.hpart | (uintptr_t)a.w3 | (uintptr_t)a.wmu | (uintptr_t)a.wls | (uintptr_t)a.n1g |
                       (uintptr_t)a.n1b | (uintptr_t)a.n4g | (uintptr_t)a.n4b | (uintptr_t)a.pre1 | (uintptr_t)a.x1 |
                       (uintptr_t)a.x2;
  return a.M > 0 && a.A >= 1 && 2 * a.A <= AT_MAXH && a.R >= 1 && a.R <= AT_MAXR && a.C >= 1 && a.a1 % 8 == 0 &&
         a.a1 / 2 <= 4 * AT_KH4 && a.a1 <= AT_MAXW && a.a2 % 4 == 0 && a.a2 <= AT_MAXW && 2 * a.a2 <= AT_NT &&
         AT_ROWS * (a.a1 / 4) <= AT_NT && (al & 15) == 0 && a.ldw % 4 == 0 && a.ldh % 4 == 0 && a.ld1 % 4 == 0 &&
         a.ld2 % 4 == 0 && (long long)a.R * a.C * a.ldw < (1LL << 31) && (long long)a.M * std::max(a.ld1, a.ld2) < (1LL << 31) &&
         (long long)a.M * a.ldh < (1LL << 31) && a.idx && a.zval && a.act && a.mu && a.sig &&
         (a.det || a.noise.eps || a.noise.rng);
}

int op_actor_tail(const ActorTailArgs& a, hipStream_t s) {
  if (!op_actor_tail_ok(a)) {
    dr_set_error("actor_tail: unsupported dims / alignment (a1 %% 8 == 0, a1 <= 200, a2 <= 256, 2A <= 16, R <= 32)");
    return DR_E_INVALID;
  }
  hipLaunchKernelGGL(k_actor_tail, dim3((unsigned)((a.M + AT_ROWS - 1) / AT_ROWS)), dim3(AT_NT), 0, s, a);
  return dr_check_launch("actor_tail");
}

// ---------------------------------------------------------------------------
// k_actor_tail_bwd: the backward of k_actor_tail's layers (chain.h).  It
// replaces the head backward (k_actor_head_bwd_x), the fused LN-backward +
// base_net.3 input-gradient product, and base_net.1's LN-SiLU backward pass:
// three launches per BPTT step.  Same row-block layout as the forward: a
// workgroup owns AT_ROWS batch rows, wave r row r for the LayerNorms, thread
// (k, half) one column of W3 over half of its rows in registers.
// LayerNorm-SiLU backward (k_ln_silu_bwd's arithmetic): x_hat, y = x_hat g + b,
// s = sigmoid(y), dy = gx s (1 + y (1 - s)), dx_hat = dy g,
// g_pre = rstd (dx_hat - mean(dx_hat) - x_hat mean(dx_hat x_hat)).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float4 at_ln_silu_bwd(float4 gx, float4 p, bool ok, int K, float4 gm, float4 bt,
                                                 float4& gy, float4& xh) {
  const float mean = wave_sum(ok ? (p.x + p.y) + (p.z + p.w) : 0.f) / (float)K;
  float sq = 0.f;
  if (ok) {
    const float dx = p.x - mean, dy = p.y - mean, dz = p.z - mean, dw = p.w - mean;
    sq = (dx * dx + dy * dy) + (dz * dz + dw * dw);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(sq) / (float)K + 1e-5f);
  const float pv[4] = {p.x, p.y, p.z, p.w}, gv[4] = {gx.x, gx.y, gx.z, gx.w};
  const float gmv[4] = {gm.x, gm.y, gm.z, gm.w}, btv[4] = {bt.x, bt.y, bt.z, bt.w};
  float xhv[4], gyv[4], gxh[4];
  float c1 = 0.f, c2 = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    xhv[c] = (pv[c] - mean) * rstd;
    const float y = xhv[c] * gmv[c] + btv[c];
    const float sg = 1.0f / (1.0f + expf(-y));
    gyv[c] = gv[c] * (sg * (1.0f + y * (1.0f - sg)));
    gxh[c] = gyv[c] * gmv[c];
    if (ok) {
      c1 += gxh[c];
      c2 += gxh[c] * xhv[c];
    }
  }
  c1 = wave_sum(c1) / (float)K;
  c2 = wave_sum(c2) / (float)K;
  gy = make_float4(gyv[0], gyv[1], gyv[2], gyv[3]);
  xh = make_float4(xhv[0], xhv[1], xhv[2], xhv[3]);
  return make_float4(rstd * (gxh[0] - c1 - xhv[0] * c2), rstd * (gxh[1] - c1 - xhv[1] * c2),
                     rstd * (gxh[2] - c1 - xhv[2] * c2), rstd * (gxh[3] - c1 - xhv[3] * c2));
}

__global__ __launch_bounds__(AT_NT) void k_actor_tail_bwd(ActorTailBwdArgs aa) {
  __shared__ ActorTailBwdArgs a;
  dr_stage_args(aa, a, threadIdx.x);
  __shared__ float s_gh[AT_ROWS][AT_MAXH];
  __shared__ __attribute__((aligned(16))) float s_w[AT_MAXH][AT_MAXW];  // head weights
  __shared__ __attribute__((aligned(16))) float s_g2[AT_ROWS][AT_MAXW];  // g_pre2
  __shared__ __attribute__((aligned(16))) float s_g1[AT_ROWS][AT_MAXW];  // gx1
  const int M = dr_uni(a.M), A = dr_uni(a.A), a1 = dr_uni(a.a1), a2 = dr_uni(a.a2);
  const int m0 = blockIdx.x * AT_ROWS;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int m = m0 + wave;  // this wave's row in the LayerNorm phases
  // ---- P1: head weights -> LDS, head backward of the rows -> LDS (+ save) ----
  for (int x = tid; x < 2 * A * (a2 >> 2); x += AT_NT) {
    const int o = x / (a2 >> 2), k4 = x - o * (a2 >> 2);
    const float* src = o < A ? dr_uni(a.wmu) : dr_uni(a.wls);
    const int oo = o < A ? o : o - A;
    *reinterpret_cast<float4*>(&s_w[o][4 * k4]) = dr_ld4(src, (unsigned)(oo * a2 + 4 * k4));
  }
  // the LN rows of the first phase and their parameters, issued with the above
  const bool ok2 = lane < (a2 >> 2);
  const unsigned k2 = ok2 ? 4u * lane : 0u;
  const bool live = m < M;
  const float4 p2 = dr_ld4(dr_uni(a.pre2), live && ok2 ? (unsigned)(m * (int)a.ld2) + k2 : 0u);
  const float4 g4 = dr_ld4(dr_uni(a.n4g), k2), b4 = dr_ld4(dr_uni(a.n4b), k2);
  if (tid < AT_ROWS * A) {
    const int ml = tid / A, k = tid - ml * A, mm = m0 + ml;
    float gmu = 0.f, gls = 0.f;
    if (mm < M) {
      gmu = a.g_mu ? dr_g(a.g_mu)[(long long)mm * a.ldgl + k] : 0.0f;
      float gsg = a.g_sig ? dr_g(a.g_sig)[(long long)mm * a.ldgl + k] : 0.0f;
      if (a.g_a) {
        const float av = dr_g(a.act)[(long long)mm * a.ldact + k];
        const float gp = dr_g(a.g_a)[(long long)mm * a.ldga + k] * (1.0f - av * av);
        gmu = gmu + gp;
        gsg = gsg + gp * dr_g(a.eps)[(long long)mm * A + k];
      }
      const float lr = dr_g(a.ls_raw)[(long long)mm * a.ldl + k];
      const float lc = fminf(fmaxf(lr, -5.0f), 2.0f);
      if (lr >= -5.0f && lr <= 2.0f) {
        const float ez = expf(lc);
        gls = (lc > 20.0f) ? gsg : gsg * ez / (ez + 1.0f);
      }
      dr_g(a.gheads)[(long long)mm * a.ldh + k] = gmu;
      dr_g(a.gheads)[(long long)mm * a.ldh + A + k] = gls;
    }
    s_gh[ml][k] = gmu;
    s_gh[ml][A + k] = gls;
  }
  __syncthreads();
  // ---- P2: wave r: gx2 = gheads [W_mu; W_ls], g_pre2 = LN4-SiLU backward; W3^T half rows requested ----
  const int j = tid >> 1, hf = tid & 1, kh = a2 >> 1;  // thread: column j of W3 (row j of W3^T), half hf
  const bool wthr = j < a1;
  float4 w3[AT_KH4];
  {
    const float* W = dr_uni(a.w3t);
#pragma unroll
    for (int i = 0; i < AT_KH4; ++i) {
      const bool ok = wthr && 4 * i < kh;
      w3[i] = dr_ld4(W, ok ? (unsigned)(j * a2 + hf * kh + 4 * i) : 0u);
    }
  }
  {
    float4 gx = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok2) {
#pragma unroll
      for (int o = 0; o < AT_MAXH; ++o) {
        if (o < 2 * A) {
          const float gh = s_gh[wave][o];
          const float4 wv = *reinterpret_cast<const float4*>(&s_w[o][4 * lane]);
          gx.x = fmaf(gh, wv.x, gx.x);
          gx.y = fmaf(gh, wv.y, gx.y);
          gx.z = fmaf(gh, wv.z, gx.z);
          gx.w = fmaf(gh, wv.w, gx.w);
        }
      }
    }
    float4 gy, xh;
    const float4 gp = at_ln_silu_bwd(gx, p2, ok2, a2, g4, b4, gy, xh);
    if (ok2) {
      *reinterpret_cast<float4*>(&s_g2[wave][4 * lane]) = gp;
      if (live) {
        const unsigned e = (unsigned)(m * (int)a.ld2) + k2;
        dr_st4(a.gpre2, e, gp);
        dr_st4(a.gy2, e, gy);
        dr_st4(a.xh2, e, xh);
      }
    }
  }
  __syncthreads();
  // ---- P3: gx1 = g_pre2 W3 (thread (j, half): 2 x AT_ROWS partial dots over its half of a2) ----
  {
    float acc[AT_ROWS];
#pragma unroll
    for (int r = 0; r < AT_ROWS; ++r) acc[r] = 0.f;
#pragma unroll
    for (int i = 0; i < AT_KH4; ++i) {
      if (4 * i < kh) {
        const int k = hf * kh + 4 * i;
#pragma unroll
        for (int r = 0; r < AT_ROWS; ++r) {
          const float4 gv = *reinterpret_cast<const float4*>(&s_g2[r][k]);
          acc[r] = fmaf(gv.x, w3[i].x, acc[r]);
          acc[r] = fmaf(gv.y, w3[i].y, acc[r]);
          acc[r] = fmaf(gv.z, w3[i].z, acc[r]);
          acc[r] = fmaf(gv.w, w3[i].w, acc[r]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < AT_ROWS; ++r) {
      const float o = __shfl_xor(acc[r], 1, 64);
      if (wthr && hf == 0) s_g1[r][j] = acc[r] + o;
    }
  }
  __syncthreads();
  // ---- P4: wave r: g_pre1 = LN1-SiLU backward of gx1 ----
  {
    const bool ok1 = lane < (a1 >> 2);
    const unsigned k1 = ok1 ? 4u * lane : 0u;
    const float4 p1 = dr_ld4(dr_uni(a.pre1), live && ok1 ? (unsigned)(m * (int)a.ld1) + k1 : 0u);
    const float4 g1 = dr_ld4(dr_uni(a.n1g), k1), b1 = dr_ld4(dr_uni(a.n1b), k1);
    const float4 gx = ok1 ? *reinterpret_cast<const float4*>(&s_g1[wave][4 * lane]) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 gy, xh;
    const float4 gp = at_ln_silu_bwd(gx, p1, ok1, a1, g1, b1, gy, xh);
    if (ok1 && live) {
      const unsigned e = (unsigned)(m * (int)a.ld1) + k1;
      dr_st4(a.gpre1, e, gp);
      dr_st4(a.gy1, e, gy);
      dr_st4(a.xh1, e, xh);
    }
  }
}

bool op_actor_tail_bwd_ok(const ActorTailBwdArgs& a) {
  const uintptr_t al = (uintptr_t)a.wmu | (uintptr_t)a.wls | (uintptr_t)a.pre2 | (uintptr_t)a.n4g | (uintptr_t)a.n4b |
                       (uintptr_t)a.gpre2 | (uintptr_t)a.gy2 | (uintptr_t)a.xh2 | (uintptr_t)a.w3t | (uintptr_t)a.pre1 |
                       (uintptr_t)a.n1g | (uintptr_t)a.n1b | (uintptr_t)a.gpre1 | (uintptr_t)a.gy1 | (uintptr_t)a.xh1;
  return a.M > 0 && a.A >= 1 && 2 * a.A <= AT_MAXH && a.a2 % 8 == 0 && a.a2 / 2 <= 4 * AT_KH4 && a.a2 <= AT_MAXW &&
         a.a1 % 4 == 0 && a.a1 <= AT_MAXW && 2 * a.a1 <= AT_NT && (al & 15) == 0 && a.ld1 % 4 == 0 && a.ld2 % 4 == 0 &&
         (long long)a.M * std::max(a.ld1, a.ld2) < (1LL << 31) && a.act && a.ls_raw && a.eps && a.gheads &&
         (!a.g_a || a.act);
}

int op_actor_tail_bwd(const ActorTailBwdArgs& a, hipStream_t s) {
  if (!op_actor_tail_bwd_ok(a)) {
    dr_set_error("actor_tail_bwd: unsupported dims / alignment (a2 %% 8 == 0, a2 <= 200, a1 <= 256, 2A <= 16)");
    return DR_E_INVALID;
  }
  hipLaunchKernelGGL(k_actor_tail_bwd, dim3((unsigned)((a.M + AT_ROWS - 1) / AT_ROWS)), dim3(AT_NT), 0, s, a);
  return dr_check_launch("actor_tail_bwd");
}
