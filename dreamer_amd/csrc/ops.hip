// Row / elementwise kernels of libdreamer_hip: GRU gates, categorical
// sampler, heads, LayerNorm-SiLU backward, losses, returns, quantile,
// optimiser.  Built with -ffp-contract=off: each expression rounds like the
// corresponding PyTorch CPU op sequence of the reference (cited per kernel).
#include <stdarg.h>

#include <algorithm>
#include <stdio.h>

#include "ops.h"

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local char g_err[512] = "";

void dr_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int dr_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    dr_set_error("%s: %s", what, hipGetErrorString(e));
    return DR_E_HIP;
  }
  return DR_OK;
}

extern "C" const char* dr_last_error(void) { return g_err; }
extern "C" int dr_version(void) { return 1; }

static inline int blocks_for(long long n, int t) { return (int)((n + t - 1) / t); }

// ---------------------------------------------------------------------------
// GRU gates (SequenceModel.py:13-23 -> torch gru_cell)
// ---------------------------------------------------------------------------
__global__ void k_gru_fwd(int B, int Hd, const float* __restrict__ gi, const float* __restrict__ gh,
                          const float* __restrict__ h, long long ldh, float* __restrict__ hout, long long ldo,
                          float* sr, float* su, float* sn, float* sghn) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * Hd) return;
  const int b = (int)(i / Hd), j = (int)(i - (long long)b * Hd);
  const float* gib = gi + (long long)b * 3 * Hd;
  const float* ghb = gh + (long long)b * 3 * Hd;
  const float r = 1.0f / (1.0f + expf(-(ghb[j] + gib[j])));
  const float u = 1.0f / (1.0f + expf(-(ghb[Hd + j] + gib[Hd + j])));
  const float hn = ghb[2 * Hd + j];
  const float n = tanhf(gib[2 * Hd + j] + hn * r);
  const float hv = h ? h[(long long)b * ldh + j] : 0.0f;
  hout[(long long)b * ldo + j] = (hv - n) * u + n;
  if (sr) {
    sr[i] = r;
    su[i] = u;
    sn[i] = n;
    sghn[i] = hn;
  }
}

int op_gru_fwd(int B, int Hd, const float* gi, const float* gh, const float* h, long long ldh, float* hout,
               long long ldo, float* sr, float* su, float* sn, float* sghn, hipStream_t s) {
  const long long n = (long long)B * Hd;
  if (n == 0) return DR_OK;
  hipLaunchKernelGGL(k_gru_fwd, dim3(blocks_for(n, 256)), dim3(256), 0, s, B, Hd, gi, gh, h, ldh, hout, ldo, sr,
                     su, sn, sghn);
  return dr_check_launch("gru_fwd");
}

__global__ void k_gru_bwd(int B, int Hd, const float* __restrict__ g_hp, long long ldg, const float* __restrict__ h,
                          long long ldh, const float* sr, const float* su, const float* sn, const float* sghn,
                          float* g_gi, float* g_gh, float* gh_out, long long ldo, int accumulate) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * Hd) return;
  const int b = (int)(i / Hd), j = (int)(i - (long long)b * Hd);
  const float g = g_hp[(long long)b * ldg + j];
  const float r = sr[i], u = su[i], n = sn[i], hn = sghn[i];
  const float hv = h ? h[(long long)b * ldh + j] : 0.0f;
  // h' = (h - n)*u + n
  const float g_hmn = g * u;
  const float g_u = g * (hv - n);
  const float g_n = g + (-g_hmn);
  // n = tanh(in + hn*r)
  const float g_pn = g_n * (1.0f - n * n);
  const float g_r = g_pn * hn;
  const float g_hn = g_pn * r;
  const float g_pr = g_r * (1.0f - r) * r;
  const float g_pu = g_u * (1.0f - u) * u;
  float* gib = g_gi + (long long)b * 3 * Hd;
  float* ghb = g_gh + (long long)b * 3 * Hd;
  gib[j] = g_pr;
  gib[Hd + j] = g_pu;
  gib[2 * Hd + j] = g_pn;
  ghb[j] = g_pr;
  ghb[Hd + j] = g_pu;
  ghb[2 * Hd + j] = g_hn;
  float* o = gh_out + (long long)b * ldo + j;
  if (accumulate) *o = *o + g_hmn;
  else *o = g_hmn;
}

int op_gru_bwd(int B, int Hd, const float* g_hp, long long ldg, const float* h, long long ldh, const float* sr,
               const float* su, const float* sn, const float* sghn, float* g_gi, float* g_gh, float* gh_out,
               long long ldo, int accumulate, hipStream_t s) {
  const long long n = (long long)B * Hd;
  if (n == 0) return DR_OK;
  hipLaunchKernelGGL(k_gru_bwd, dim3(blocks_for(n, 256)), dim3(256), 0, s, B, Hd, g_hp, ldg, h, ldh, sr, su, sn,
                     sghn, g_gi, g_gh, gh_out, ldo, accumulate);
  return dr_check_launch("gru_bwd");
}

// ---------------------------------------------------------------------------
// Categorical sample with 1% unimix and straight-through value
// (VAE.py:88-98, DynamicsPredictors.py:33-39; torch Categorical normalises
// p by its sum, multinomial(n=1) == argmax(p_hat / Exp(1))).
// One aligned group of W = pow2 >= C lanes per (row, latent group).
// ---------------------------------------------------------------------------
__global__ void k_sample(int M, int R, int C, int W, const float* __restrict__ logits, long long ldl, dr_noise nz,
                         int step, float unimix_add, float* __restrict__ z, long long ldz, int* idx, float* soft,
                         long long lds) {
  const int gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const int grp = gtid / W, c = gtid - grp * W;
  const bool valid = grp < M * R;
  const int m = valid ? grp / R : 0, r = valid ? grp - m * R : 0;
  const bool act = valid && c < C;
  const float x = act ? logits[(long long)m * ldl + r * C + c] : -INFINITY;
  const float mx = group_max(x, W);
  const float e = act ? expf(x - mx) : 0.0f;
  const float se = group_sum(e, W);
  const float p = e / se;
  const float pu = act ? (0.99f * p + unimix_add) : 0.0f;
  const float sp = group_sum(pu, W);
  const float ph = pu / sp;
  float q = 1.0f;
  if (act) {
    if (nz.q) q = nz.q[((long long)step * M * R + grp) * C + c];
    else q = dr_exp1(nz.rng, (uint32_t)(nz.stream + step), (uint32_t)(nz.row0 + m), (uint32_t)(r * C + c));
  }
  float best = act ? ph / q : -INFINITY;
  int bi = act ? c : 0x7fffffff;
  group_argmax(best, bi, W);
  if (act) {
    z[(long long)m * ldz + r * C + c] = (c == bi) ? ((1.0f + pu) - pu) : 0.0f;
    if (soft) soft[(long long)m * lds + r * C + c] = p;
    if (idx && c == 0) idx[grp] = bi;
  }
}

static int pow2_at_least(int c) {
  int w = 1;
  while (w < c) w <<= 1;
  return w;
}

int op_sample(int M, int R, int C, const float* logits, long long ldl, const dr_noise* nz, int step, float* z,
              long long ldz, int* idx, float* soft, long long lds, hipStream_t s) {
  if (C < 1 || C > 64) {
    dr_set_error("sample: latent classes must be in [1,64], got %d", C);
    return DR_E_INVALID;
  }
  const int W = pow2_at_least(C);
  const long long threads = (long long)M * R * W;
  if (threads == 0) return DR_OK;
  const float unimix = (float)(0.01 * (1.0 / C));
  hipLaunchKernelGGL(k_sample, dim3(blocks_for(threads, 256)), dim3(256), 0, s, M, R, C, W, logits, ldl, *nz, step,
                     unimix, z, ldz, idx, soft, lds);
  return dr_check_launch("sample");
}

extern "C" int dr_categorical_sample(int M, int R, int C, const float* logits, dr_noise noise, float* z_out,
                                     int* idx_out, float* soft_out, hipStream_t stream) {
  return op_sample(M, R, C, logits, (long long)R * C, &noise, 0, z_out, (long long)R * C, idx_out, soft_out,
                   (long long)R * C, stream);
}

// softmax backward through the STE value: g_logit = s*(g_s - sum(g_s*s)), g_s = 0.99*g_z
__global__ void k_softmax_ste_bwd(int M, int R, int C, int W, const float* __restrict__ gz, long long ldg,
                                  const float* __restrict__ soft, long long lds, float* __restrict__ gl) {
  const int gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const int grp = gtid / W, c = gtid - grp * W;
  const bool valid = grp < M * R;
  const int m = valid ? grp / R : 0, r = valid ? grp - m * R : 0;
  const bool act = valid && c < C;
  const float gs = act ? gz[(long long)m * ldg + r * C + c] * 0.99f : 0.0f;
  const float sv = act ? soft[(long long)m * lds + r * C + c] : 0.0f;
  const float dot = group_sum(gs * sv, W);
  if (act) gl[(long long)m * R * C + r * C + c] = sv * (gs - dot);
}

int op_softmax_ste_bwd(int M, int R, int C, const float* gz, long long ldg, const float* soft, long long lds,
                       float* g_logits, hipStream_t s) {
  const int W = pow2_at_least(C);
  const long long threads = (long long)M * R * W;
  if (threads == 0) return DR_OK;
  hipLaunchKernelGGL(k_softmax_ste_bwd, dim3(blocks_for(threads, 256)), dim3(256), 0, s, M, R, C, W, gz, ldg, soft,
                     lds, g_logits);
  return dr_check_launch("softmax_ste_bwd");
}

// ---------------------------------------------------------------------------
// LayerNorm(eps=1e-5) + SiLU backward, one wave per row
// ---------------------------------------------------------------------------
// one wave per row; the row (pre, upstream grad, gamma, beta) is loaded into
// registers once (K <= 64 * LNB_NPL), so the kernel makes one memory round
// trip; the reductions keep the k = lane, lane + 64, ... order
#define LNB_NPL 16
template <bool REG>
__global__ void k_ln_silu_bwd(int M, int K, const float* __restrict__ gx, long long ldgx,
                              const float* __restrict__ pre, long long ldp, const float* __restrict__ gamma,
                              const float* __restrict__ beta, float* __restrict__ g_pre, long long ldgp, float* gy_out,
                              float* xhat_out, unsigned short* __restrict__ g_pre16) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* p = pre + (long long)row * ldp;
  const float* g = gx + (long long)row * ldgx;
  if (REG) {
    float pv[LNB_NPL], gv[LNB_NPL], gm[LNB_NPL], bt[LNB_NPL];
#pragma unroll
    for (int i = 0; i < LNB_NPL; ++i) {
      const int k = lane + 64 * i;
      const bool ok = k < K;
      const int kk = ok ? k : 0;
      pv[i] = p[kk]; gv[i] = g[kk]; gm[i] = gamma[kk]; bt[i] = beta[kk];
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < LNB_NPL; ++i)
      if (lane + 64 * i < K) s += pv[i];
    const float mean = wave_sum(s) / (float)K;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < LNB_NPL; ++i)
      if (lane + 64 * i < K) {
        const float d = pv[i] - mean;
        v += d * d;
      }
    const float rstd = 1.0f / sqrtf(wave_sum(v) / (float)K + 1e-5f);
    float c1 = 0.f, c2 = 0.f;
#pragma unroll
    for (int i = 0; i < LNB_NPL; ++i) {
      const int k = lane + 64 * i;
      if (k >= K) continue;
      const float xh = (pv[i] - mean) * rstd;
      const float y = xh * gm[i] + bt[i];
      const float sg = 1.0f / (1.0f + expf(-y));
      const float gyv = gv[i] * (sg * (1.0f + y * (1.0f - sg)));
      const float gxh = gyv * gm[i];
      c1 += gxh;
      c2 += gxh * xh;
      if (gy_out) {
        gy_out[(long long)row * ldgp + k] = gyv;
        xhat_out[(long long)row * ldgp + k] = xh;
      }
      pv[i] = xh;   // keep x_hat and d/dx_hat for the last pass
      gv[i] = gxh;
    }
    c1 = wave_sum(c1) / (float)K;
    c2 = wave_sum(c2) / (float)K;
#pragma unroll
    for (int i = 0; i < LNB_NPL; ++i) {
      const int k = lane + 64 * i;
      if (k < K) {
        const float gp = rstd * (gv[i] - c1 - pv[i] * c2);
        g_pre[(long long)row * ldgp + k] = gp;
        if (g_pre16) g_pre16[(long long)row * ldgp + k] = __builtin_bit_cast(unsigned short, (__bf16)gp);
      }
    }
    return;
  }
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s += p[k];
  const float mean = wave_sum(s) / (float)K;
  float v = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float d = p[k] - mean;
    v += d * d;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(v) / (float)K + 1e-5f);
  float c1 = 0.f, c2 = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float xh = (p[k] - mean) * rstd;
    const float y = xh * gamma[k] + beta[k];
    const float sg = 1.0f / (1.0f + expf(-y));
    const float gyv = g[k] * (sg * (1.0f + y * (1.0f - sg)));
    const float gxh = gyv * gamma[k];
    c1 += gxh;
    c2 += gxh * xh;
    if (gy_out) {
      gy_out[(long long)row * ldgp + k] = gyv;
      xhat_out[(long long)row * ldgp + k] = xh;
    }
  }
  c1 = wave_sum(c1) / (float)K;
  c2 = wave_sum(c2) / (float)K;
  for (int k = lane; k < K; k += 64) {
    const float xh = (p[k] - mean) * rstd;
    const float y = xh * gamma[k] + beta[k];
    const float sg = 1.0f / (1.0f + expf(-y));
    const float gxh = g[k] * (sg * (1.0f + y * (1.0f - sg))) * gamma[k];
    const float gp = rstd * (gxh - c1 - xh * c2);
    g_pre[(long long)row * ldgp + k] = gp;
    if (g_pre16) g_pre16[(long long)row * ldgp + k] = __builtin_bit_cast(unsigned short, (__bf16)gp);
  }
}

int op_ln_silu_bwd(int M, int K, const float* gx, long long ldgx, const float* pre, long long ldp,
                   const float* gamma, const float* beta, float* g_pre, long long ldgp, float* gy, float* xhat,
                   hipStream_t s, unsigned short* g_pre16) {
  if (M == 0) return DR_OK;
  if (K <= 64 * LNB_NPL)
    hipLaunchKernelGGL(k_ln_silu_bwd<true>, dim3(dr_cdiv(M, 4)), dim3(256), 0, s, M, K, gx, ldgx, pre, ldp, gamma,
                       beta, g_pre, ldgp, gy, xhat, g_pre16);
  else
    hipLaunchKernelGGL(k_ln_silu_bwd<false>, dim3(dr_cdiv(M, 4)), dim3(256), 0, s, M, K, gx, ldgx, pre, ldp, gamma,
                       beta, g_pre, ldgp, gy, xhat, g_pre16);
  return dr_check_launch("ln_silu_bwd");
}

// ---------------------------------------------------------------------------
// column sums (bias / LayerNorm parameter gradients), deterministic order
// ---------------------------------------------------------------------------
// one CS_W-column slab per workgroup, CS_RG row groups; rows summed in a fixed
// order (deterministic), 8 rows of loads in flight per thread.  16-column
// slabs: the bias gradients have 200-1600 columns, so 64-column slabs gave
// 4-25 workgroups for the whole GPU, each walking 240 rows per thread
// (37 us per epoch launch, 33 us per WM-step launch, r04z)
#define CS_W 16
#define CS_RG (1024 / CS_W)
__device__ __forceinline__ void colsum_slab(int M, int N, const float* __restrict__ X, long long ldx,
                                            const float* __restrict__ Y, long long ldy, float* out, int accumulate,
                                            int slab, float (&part)[CS_RG][CS_W]) {
  const int c = threadIdx.x % CS_W, rg = threadIdx.x / CS_W;
  const int n = slab * CS_W + c;
  float acc = 0.f;
  if (n < N) {
    int m = rg;
    for (; m + CS_RG * 7 < M; m += CS_RG * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = X[(long long)(m + CS_RG * u) * ldx + n];
      if (Y) {
        float w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) w[u] = Y[(long long)(m + CS_RG * u) * ldy + n];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = v[u] * w[u];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; m < M; m += CS_RG) {
      float v = X[(long long)m * ldx + n];
      if (Y) v = v * Y[(long long)m * ldy + n];
      acc += v;
    }
  }
  part[rg][c] = acc;
  __syncthreads();
  // fixed-order tree: 8 groups of 8 row-group partials, then the 8 group sums
  constexpr int G = 8, PER = CS_RG / G;
  __shared__ float grp[G][CS_W];
  if (rg < G) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k) t += part[rg * PER + k][c];
    grp[rg][c] = t;
  }
  __syncthreads();
  if (rg == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < G; ++k) t += grp[k][c];
    out[n] = accumulate ? out[n] + t : t;
  }
}

__global__ __launch_bounds__(1024) void k_colsum(int M, int N, const float* __restrict__ X, long long ldx,
                                                 const float* __restrict__ Y, long long ldy, float* out,
                                                 int accumulate) {
  __shared__ float part[CS_RG][CS_W];
  colsum_slab(M, N, X, ldx, Y, ldy, out, accumulate, blockIdx.x, part);
}

struct ColsumBatch {
  ColsumJob j[DR_MAX_CSJOBS];
  int first_slab[DR_MAX_CSJOBS + 1];
  int n;
};
__global__ __launch_bounds__(1024) void k_colsum_multi(int M, ColsumBatch cb) {
  __shared__ float part[CS_RG][CS_W];
  int j = 0;
  while (j + 1 < cb.n && (int)blockIdx.x >= cb.first_slab[j + 1]) ++j;
  const ColsumJob& J = cb.j[j];
  colsum_slab(M, J.N, J.X, J.ldx, J.Y, J.ldy, J.out, 0, blockIdx.x - cb.first_slab[j], part);
}

int op_colsum_multi(int M, const ColsumJob* jobs, int n, hipStream_t s) {
  if (n <= 0) return DR_OK;
  if (n > DR_MAX_CSJOBS) {
    dr_set_error("colsum_multi: at most %d jobs", DR_MAX_CSJOBS);
    return DR_E_INVALID;
  }
  ColsumBatch cb;
  cb.n = n;
  int slabs = 0;
  for (int i = 0; i < n; ++i) {
    cb.j[i] = jobs[i];
    cb.first_slab[i] = slabs;
    slabs += dr_cdiv(jobs[i].N, CS_W);
  }
  cb.first_slab[n] = slabs;
  if (slabs == 0) return DR_OK;
  hipLaunchKernelGGL(k_colsum_multi, dim3(slabs), dim3(1024), 0, s, M, cb);
  return dr_check_launch("colsum_multi");
}

int op_colsum(int M, int N, const float* X, long long ldx, const float* Y, long long ldy, float* out, int accumulate,
              hipStream_t s) {
  if (N == 0) return DR_OK;
  hipLaunchKernelGGL(k_colsum, dim3(dr_cdiv(N, CS_W)), dim3(1024), 0, s, M, N, X, ldx, Y, ldy, out, accumulate);
  return dr_check_launch("colsum");
}

// ---------------------------------------------------------------------------
// heads
// ---------------------------------------------------------------------------
// RewardPredictor.predict / Critic.value: symexp(sum(softmax(l) * buckets))
// (DynamicsPredictors.py:70-74, Agent.py:237-241); one wave per row
__global__ void k_bucket_value(int M, int nb, const float* __restrict__ logits, long long ldl,
                               const float* __restrict__ buckets, float* out, long long ostride) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float* l = logits + (long long)row * ldl;
  float mx = -INFINITY;
  for (int k = lane; k < nb; k += 64) mx = fmaxf(mx, l[k]);
  mx = wave_max(mx);
  float se = 0.f;
  for (int k = lane; k < nb; k += 64) se += expf(l[k] - mx);
  se = wave_sum(se);
  float acc = 0.f;
  for (int k = lane; k < nb; k += 64) acc += (expf(l[k] - mx) / se) * buckets[k];
  acc = wave_sum(acc);
  if (lane == 0) out[(long long)row * ostride] = dr_symexp(acc);
}

int op_bucket_value(int M, int nb, const float* logits, long long ldl, const float* buckets, float* out,
                    long long ostride, hipStream_t s) {
  if (M == 0) return DR_OK;
  hipLaunchKernelGGL(k_bucket_value, dim3(dr_cdiv(M, 4)), dim3(256), 0, s, M, nb, logits, ldl, buckets, out,
                     ostride);
  return dr_check_launch("bucket_value");
}

extern "C" int dr_bucket_value(int M, int nb, const float* logits, const float* buckets, float* out,
                               hipStream_t stream) {
  return op_bucket_value(M, nb, logits, nb, buckets, out, 1, stream);
}

// ContinuePredictor.predict: sigmoid(logit) (DynamicsPredictors.py:95-105)
__global__ void k_sigmoid(int M, const float* x, long long ldx, float* out, long long ostride) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  out[(long long)i * ostride] = 1.0f / (1.0f + expf(-x[(long long)i * ldx]));
}

int op_sigmoid(int M, const float* x, long long ldx, float* out, long long ostride, hipStream_t s) {
  if (M == 0) return DR_OK;
  hipLaunchKernelGGL(k_sigmoid, dim3(dr_cdiv(M, 256)), dim3(256), 0, s, M, x, ldx, out, ostride);
  return dr_check_launch("sigmoid");
}

// Actor.forward tail + act (Agent.py:196-210)
__global__ void k_actor_head(int M, int A, const float* __restrict__ mu_raw, long long ldm,
                             const float* __restrict__ ls_raw, long long ldl, dr_noise nz, int step, int det,
                             float* a, long long lda, float* mu, long long ldmu, float* sigma, long long lds,
                             float* eps_save) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * A) return;
  const int m = i / A, k = i - m * A;
  const float muv = mu_raw[(long long)m * ldm + k];
  const float ls = fminf(fmaxf(ls_raw[(long long)m * ldl + k], -5.0f), 2.0f);
  const float sg = dr_softplus(ls) + 1e-3f;
  float av;
  if (det) {
    av = tanhf(muv);
  } else {
    float e;
    if (nz.eps) e = nz.eps[((long long)step * M + m) * A + k];
    else e = dr_normal(nz.rng, (uint32_t)(nz.stream + step), (uint32_t)(nz.row0 + m), (uint32_t)k);
    if (eps_save) eps_save[i] = e;
    av = tanhf(muv + e * sg);
  }
  if (a) a[(long long)m * lda + k] = av;
  if (mu) mu[(long long)m * ldmu + k] = muv;
  if (sigma) sigma[(long long)m * lds + k] = sg;
}

int op_actor_head(int M, int A, const float* mu_raw, long long ldm, const float* ls_raw, long long ldl,
                  const dr_noise* nz, int step, int deterministic, float* a, long long lda, float* mu,
                  long long ldmu, float* sigma, long long lds, float* eps_save, hipStream_t s) {
  if (M * A == 0) return DR_OK;
  hipLaunchKernelGGL(k_actor_head, dim3(dr_cdiv(M * A, 256)), dim3(256), 0, s, M, A, mu_raw, ldm, ls_raw, ldl, *nz,
                     step, deterministic, a, lda, mu, ldmu, sigma, lds, eps_save);
  return dr_check_launch("actor_head");
}

// backward of a = tanh(mu + eps*sigma), sigma = softplus(clamp(ls)) + 1e-3,
// plus the loss gradients on mu/sigma; g_heads [M][2A] = [g_mu | g_ls]
__global__ void k_actor_head_bwd(int M, int A, const float* g_a, long long ldga, const float* g_mu_l,
                                 const float* g_sig_l, long long ldgl, const float* a, long long lda,
                                 const float* sigma, long long lds, const float* ls_raw, long long ldl,
                                 const float* eps, float* g_heads, long long ldh) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * A) return;
  const int m = i / A, k = i - m * A;
  float gmu = g_mu_l ? g_mu_l[(long long)m * ldgl + k] : 0.0f;
  float gsg = g_sig_l ? g_sig_l[(long long)m * ldgl + k] : 0.0f;
  if (g_a) {
    const float av = a[(long long)m * lda + k];
    const float gp = g_a[(long long)m * ldga + k] * (1.0f - av * av);
    gmu = gmu + gp;
    gsg = gsg + gp * eps[i];
  }
  const float lr = ls_raw[(long long)m * ldl + k];
  const float lc = fminf(fmaxf(lr, -5.0f), 2.0f);
  float gls = 0.0f;
  if (lr >= -5.0f && lr <= 2.0f) {
    const float ez = expf(lc);
    gls = (lc > 20.0f) ? gsg : gsg * ez / (ez + 1.0f);
  }
  g_heads[(long long)m * ldh + k] = gmu;
  g_heads[(long long)m * ldh + A + k] = gls;
}

int op_actor_head_bwd(int M, int A, const float* g_a, long long ldga, const float* g_mu_l, const float* g_sig_l,
                      long long ldgl, const float* a, long long lda, const float* sigma, long long lds,
                      const float* ls_raw, long long ldl, const float* eps, float* g_heads, long long ldh,
                      hipStream_t s) {
  if (M * A == 0) return DR_OK;
  hipLaunchKernelGGL(k_actor_head_bwd, dim3(dr_cdiv(M * A, 256)), dim3(256), 0, s, M, A, g_a, ldga, g_mu_l, g_sig_l,
                     ldgl, a, lda, sigma, lds, ls_raw, ldl, eps, g_heads, ldh);
  return dr_check_launch("actor_head_bwd");
}

// The same head backward fused with the input gradient of the stacked
// mu / log-sigma heads: gx[m][n] = sum_k g_heads[m][k] * wt[n][k] (wt = the
// heads' weights transposed, [N][2A]).  A block owns 16 rows x 64 columns:
// it forms the 16 x 2A head gradients in LDS (the blockIdx.x == 0 column of
// blocks also stores them for the weight gradients), then its outputs.
__global__ __launch_bounds__(256) void k_actor_head_bwd_x(int M, int A, int N, const float* g_a, long long ldga,
                                                          const float* g_mu_l, const float* g_sig_l, long long ldgl,
                                                          const float* a, long long lda, const float* ls_raw,
                                                          long long ldl, const float* eps, float* g_heads,
                                                          long long ldh, const float* wt, float* gx, long long ldx) {
  __shared__ float gh[16][2 * 8];
  const int m0 = blockIdx.y * 16, n0 = blockIdx.x * 64, tid = threadIdx.x;
  // weights of this thread's column, issued first
  const int nl = tid & 63, mq = tid >> 6;  // column, row quarter (4 rows each)
  const int n = n0 + nl;
  float w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = (k < 2 * A && n < N) ? wt[(long long)n * 2 * A + k] : 0.f;
  if (tid < 16 * A) {
    const int ml = tid / A, k = tid - ml * A, m = m0 + ml;
    float gmu = 0.f, gls = 0.f;
    if (m < M) {
      gmu = g_mu_l ? g_mu_l[(long long)m * ldgl + k] : 0.0f;
      float gsg = g_sig_l ? g_sig_l[(long long)m * ldgl + k] : 0.0f;
      if (g_a) {
        const float av = a[(long long)m * lda + k];
        const float gp = g_a[(long long)m * ldga + k] * (1.0f - av * av);
        gmu = gmu + gp;
        gsg = gsg + gp * eps[(long long)m * A + k];
      }
      const float lr = ls_raw[(long long)m * ldl + k];
      const float lc = fminf(fmaxf(lr, -5.0f), 2.0f);
      if (lr >= -5.0f && lr <= 2.0f) {
        const float ez = expf(lc);
        gls = (lc > 20.0f) ? gsg : gsg * ez / (ez + 1.0f);
      }
      if (blockIdx.x == 0) {
        g_heads[(long long)m * ldh + k] = gmu;
        g_heads[(long long)m * ldh + A + k] = gls;
      }
    }
    gh[ml][k] = gmu;
    gh[ml][A + k] = gls;
  }
  __syncthreads();
  if (n >= N) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ml = 4 * mq + i, m = m0 + ml;
    if (m >= M) break;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < 2 * A) v = fmaf(gh[ml][k], w[k], v);
    gx[(long long)m * ldx + n] = v;
  }
}

int op_actor_head_bwd_x(int M, int A, int N, const float* g_a, long long ldga, const float* g_mu_l,
                        const float* g_sig_l, long long ldgl, const float* a, long long lda, const float* ls_raw,
                        long long ldl, const float* eps, float* g_heads, long long ldh, const float* wt, float* gx,
                        long long ldx, hipStream_t s) {
  if (M == 0) return DR_OK;
  if (A > 8) {
    dr_set_error("actor_head_bwd_x: at most 8 actions");
    return DR_E_INVALID;
  }
  hipLaunchKernelGGL(k_actor_head_bwd_x, dim3(dr_cdiv(N, 64), dr_cdiv(M, 16)), dim3(256), 0, s, M, A, N, g_a, ldga,
                     g_mu_l, g_sig_l, ldgl, a, lda, ls_raw, ldl, eps, g_heads, ldh, wt, gx, ldx);
  return dr_check_launch("actor_head_bwd_x");
}

// ---------------------------------------------------------------------------
// lambda returns (Agent.py:156-172), one thread per batch row
// ---------------------------------------------------------------------------
__global__ void k_lambda_returns(int B, int H, const float* r, const float* c, const float* V, float gamma,
                                 float lam, float lam_c, float* R) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* rb = r + (long long)b * H;
  const float* cb = c + (long long)b * H;
  const float* vb = V + (long long)b * (H + 1);
  float* Rb = R + (long long)b * H;
  float nxt = rb[H - 1] + (gamma * cb[H - 1]) * vb[H];
  Rb[H - 1] = nxt;
  for (int t = H - 2; t >= 0; --t) {
    const float v = rb[t] + (gamma * cb[t]) * ((lam_c * vb[t + 1]) + (lam * nxt));
    Rb[t] = v;
    nxt = v;
  }
}

extern "C" int dr_lambda_returns(int B, int H, const float* r, const float* c, const float* V, float gamma,
                                 float lam, float* R, hipStream_t stream) {
  if (B <= 0 || H <= 0) {
    dr_set_error("lambda_returns: bad dims B=%d H=%d", B, H);
    return DR_E_INVALID;
  }
  const float lam_c = (float)(1.0 - (double)lam);
  hipLaunchKernelGGL(k_lambda_returns, dim3(dr_cdiv(B, 64)), dim3(64), 0, stream, B, H, r, c, V, gamma, lam, lam_c,
                     R);
  return dr_check_launch("lambda_returns");
}

// ---------------------------------------------------------------------------
// update_S (Agent.py:78-88): quantiles 0.95/0.05 (torch linear interpolation)
// over all returns, EMA of the range, norm=max(S,1).  Up to DR_SORT_MAX values
// by a sort in one workgroup's registers (k_update_S_reg: 47.9 -> 12.2 us
// against the LDS bitonic sort it replaced, r04), above by radix select
// ---------------------------------------------------------------------------
#define DR_SORT_MAX 16384

__device__ float torch_lerp(float a, float b, float w) {
  return (w < 0.5f) ? a + w * (b - a) : b - (b - a) * (1.0f - w);
}

// Above DR_SORT_MAX returns (e.g. 8 ranks x 256 rows x H 15 = 30720 under
// data parallelism) the four order statistics torch.quantile interpolates
// between are found by an exact radix select instead of a full sort: the
// float bits are mapped to order-preserving u32 keys and 4 passes of 8-bit
// LDS histograms narrow each target rank to a single key.  One workgroup;
// the returns (<= a few MB) stream from L2 once per pass.
__device__ __forceinline__ unsigned f2key(float x) {
  const unsigned u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ __launch_bounds__(1024) void k_update_S_select(int n, const float* R, float* S, float* norm_out) {
  __shared__ unsigned hist[4][256];
  __shared__ unsigned prefix[4], want[4];
  __shared__ int bad;
  const float r95 = 0.95f * (float)(n - 1), r05 = 0.05f * (float)(n - 1);
  if (threadIdx.x == 0) {
    bad = 0;
    want[0] = (unsigned)(int)r95;
    want[1] = (unsigned)(int)ceilf(r95);
    want[2] = (unsigned)(int)r05;
    want[3] = (unsigned)(int)ceilf(r05);
  }
  if (threadIdx.x < 4) prefix[threadIdx.x] = 0u;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    const unsigned hi_mask = pass == 0 ? 0u : (0xffffffffu << (shift + 8));
    for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) (&hist[0][0])[i] = 0u;
    __syncthreads();
    unsigned pf[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) pf[t] = prefix[t];
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const float x = R[i];
      if (pass == 0 && !isfinite(x)) bad = 1;
      const unsigned k = f2key(x);
      const unsigned bin = (k >> shift) & 255u;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if ((k & hi_mask) == pf[t]) atomicAdd(&hist[t][bin], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 4) {
      const int t = threadIdx.x;
      unsigned below = 0u, w = want[t];
      int b = 0;
      for (; b < 255; ++b) {
        const unsigned c = hist[t][b];
        if (below + c > w) break;
        below += c;
      }
      prefix[t] = pf[t] | ((unsigned)b << shift);
      want[t] = w - below;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float s = *S;
    if (!bad) {
      const float q95 = torch_lerp(key2f(prefix[0]), key2f(prefix[1]), r95 - (float)(int)r95);
      const float q05 = torch_lerp(key2f(prefix[2]), key2f(prefix[3]), r05 - (float)(int)r05);
      const float range = fmaxf(q95 - q05, 1.0f);
      s = 0.99f * s + 0.01f * range;
      *S = s;
    }
    if (norm_out) *norm_out = fmaxf(s, 1.0f);
  }
}

// The same exact radix select with the returns held in registers (n <= 1024
// VPT): the bitonic sort of k_update_S ran 78 barrier-separated LDS stages
// (48 us at n = 3840); here one load, then per 8-bit pass one LDS histogram
// (atomics) and a wave-parallel prefix search per target rank.
template <int VPT>
__global__ __launch_bounds__(1024) void k_update_S_reg(int n, const float* R, float* S, float* norm_out) {
  __shared__ unsigned hist[4][256];
  __shared__ unsigned prefix[4], want[4];
  __shared__ int bad;
  const float r95 = 0.95f * (float)(n - 1), r05 = 0.05f * (float)(n - 1);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (tid == 0) {
    bad = 0;
    want[0] = (unsigned)(int)r95;
    want[1] = (unsigned)(int)ceilf(r95);
    want[2] = (unsigned)(int)r05;
    want[3] = (unsigned)(int)ceilf(r05);
  }
  if (tid < 4) prefix[tid] = 0u;
  unsigned key[VPT];
  bool nonfinite = false;
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const int i = tid + 1024 * v;
    const float x = R[i < n ? i : 0];
    nonfinite = nonfinite || (i < n && !isfinite(x));
    key[v] = f2key(x);
  }
  __syncthreads();
  if (nonfinite) bad = 1;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    const unsigned hi_mask = pass == 0 ? 0u : (0xffffffffu << (shift + 8));
    (&hist[0][0])[tid] = 0u;  // 1024 threads, 4 x 256 bins
    __syncthreads();
    unsigned pf[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) pf[t] = prefix[t];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      if (tid + 1024 * v < n) {
        const unsigned k = key[v], bin = (k >> shift) & 255u;
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if ((k & hi_mask) == pf[t]) atomicAdd(&hist[t][bin], 1u);
      }
    }
    __syncthreads();
    if (wave < 4) {  // wave t: the bin holding rank want[t]; lane l sums bins 4l .. 4l+3
      const int t = wave;
      const unsigned w = want[t];
      const unsigned c0 = hist[t][4 * lane], c1 = hist[t][4 * lane + 1], c2 = hist[t][4 * lane + 2],
                     c3 = hist[t][4 * lane + 3];
      const unsigned sum = c0 + c1 + c2 + c3;
      unsigned inc = sum;  // inclusive prefix over lanes
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned up = __shfl_up(inc, o, 64);
        if (lane >= o) inc += up;
      }
      const unsigned ex = inc - sum;
      if (ex <= w && w < inc) {  // exactly one lane
        unsigned below = ex, b = 4 * lane;
        if (below + c0 <= w) { below += c0; ++b;
          if (below + c1 <= w) { below += c1; ++b;
            if (below + c2 <= w) { below += c2; ++b; } } }
        prefix[t] = pf[t] | (b << shift);
        want[t] = w - below;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    float s = *S;
    if (!bad) {
      const float q95 = torch_lerp(key2f(prefix[0]), key2f(prefix[1]), r95 - (float)(int)r95);
      const float q05 = torch_lerp(key2f(prefix[2]), key2f(prefix[3]), r05 - (float)(int)r05);
      const float range = fmaxf(q95 - q05, 1.0f);
      s = 0.99f * s + 0.01f * range;
      *S = s;
    }
    if (norm_out) *norm_out = fmaxf(s, 1.0f);
  }
}


extern "C" int dr_update_S(int n, const float* R, float* S, float* norm_out, void* ws, size_t ws_bytes,
                           hipStream_t stream) {
  (void)ws;
  (void)ws_bytes;
  if (n <= 0 || !R || !S) {
    dr_set_error("update_S: n=%d or null pointer", n);
    return DR_E_INVALID;
  }
  if (n <= 4096) {
    hipLaunchKernelGGL(k_update_S_reg<4>, dim3(1), dim3(1024), 0, stream, n, R, S, norm_out);
    return dr_check_launch("update_S_reg");
  }
  if (n <= 16384) {
    hipLaunchKernelGGL(k_update_S_reg<16>, dim3(1), dim3(1024), 0, stream, n, R, S, norm_out);
    return dr_check_launch("update_S_reg");
  }
  hipLaunchKernelGGL(k_update_S_select, dim3(1), dim3(1024), 0, stream, n, R, S, norm_out);
  return dr_check_launch("update_S_select");
}

// ---------------------------------------------------------------------------
// actor loss (Agent.py:105-125) and dL/dmu, dL/dsigma
// ---------------------------------------------------------------------------
__global__ void k_actor_loss_grad(int B, int H, int A, const float* mus, const float* sigmas, const float* actions,
                                  const float* R, const float* V, const float* norm, float nu, float scale,
                                  float* row_loss, float* g_mus, float* g_sigmas) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (b,t)
  if (i >= B * H) return;
  const int b = i / H, t = i - b * H;
  const float adv = R[i] - V[(long long)b * (H + 1) + t];
  const float sadv = adv / (*norm);
  const float HALF_LOG_2PI = 0.91893853320467274178f;  // math.log(math.sqrt(2*math.pi))
  const float LOG2 = 0.69314718055994530942f;
  float logp = 0.f;
  for (int k = 0; k < A; ++k) {
    const long long o = (long long)i * A + k;
    float y = fminf(fmaxf(actions[o], -1.0f + 1e-6f), 1.0f - 1e-6f);
    const float x = atanhf(y);
    const float mu = mus[o], sg = sigmas[o];
    const float d = x - mu;
    const float var = sg * sg;
    const float lp = -(d * d) / (2.0f * var) - logf(sg) - HALF_LOG_2PI;
    const float ladj = 2.0f * (LOG2 - x - dr_softplus(-2.0f * x));
    logp += -ladj + lp;
  }
  const float gl = scale * (nu - sadv);
  for (int k = 0; k < A; ++k) {
    const long long o = (long long)i * A + k;
    float y = fminf(fmaxf(actions[o], -1.0f + 1e-6f), 1.0f - 1e-6f);
    const float x = atanhf(y);
    const float mu = mus[o], sg = sigmas[o];
    const float d = x - mu;
    g_mus[o] = gl * (d / (sg * sg));
    g_sigmas[o] = gl * ((d * d) / (sg * sg * sg) - 1.0f / sg);
  }
  row_loss[i] = -(logp * sadv) - (nu * (-logp));
}

__global__ __launch_bounds__(1024) void k_mean(int n, const float* x, float* out) {
  __shared__ float part[1024];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) acc += x[i];
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = part[0] / (float)n;
}

int op_mean(int n, const float* x, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_mean, dim3(1), dim3(1024), 0, s, n, x, out);
  return dr_check_launch("mean");
}

extern "C" int dr_actor_loss_grad(int B, int H, int A, const float* mus, const float* sigmas, const float* actions,
                                  const float* R, const float* V, const float* norm, float nu, float scale,
                                  float* loss_out, float* g_mus, float* g_sigmas, hipStream_t stream) {
  // row losses are staged in g_sigmas' tail? no: use a small scratch in loss_out[1..]
  if (B <= 0 || H <= 0 || A <= 0) {
    dr_set_error("actor_loss_grad: bad dims");
    return DR_E_INVALID;
  }
  float* row_loss = loss_out + 1;  // caller provides 1 + B*H floats
  hipLaunchKernelGGL(k_actor_loss_grad, dim3(dr_cdiv(B * H, 128)), dim3(128), 0, stream, B, H, A, mus, sigmas,
                     actions, R, V, norm, nu, scale, row_loss, g_mus, g_sigmas);
  DR_TRY(dr_check_launch("actor_loss_grad"));
  return op_mean(B * H, row_loss, loss_out, stream);
}

// ---------------------------------------------------------------------------
// critic two-hot CE (Agent.py:127-135, DreamerUtils.py:39-50): one wave per
// row (b,t<H) of logits [B][H+1][nb]; rows t==H get zero gradient.
// ---------------------------------------------------------------------------
__global__ void k_critic_ce(int B, int H, int nb, const float* __restrict__ logits, const float* __restrict__ R,
                            const float* __restrict__ buckets, float scale, float* row_loss, float* g_logits) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B * (H + 1)) return;
  const int b = row / (H + 1), t = row - b * (H + 1);
  const float* l = logits + (long long)row * nb;
  float* g = g_logits + (long long)row * nb;
  if (t == H) {
    for (int k = lane; k < nb; k += 64) g[k] = 0.0f;
    return;
  }
  // target two-hot of symlog(R)
  const float bmin = buckets[0], bmax = buckets[nb - 1];
  float v = dr_symlog(R[(long long)b * H + t]);
  v = fminf(fmaxf(v, bmin), bmax);
  int cnt = 0;
  for (int k = lane; k < nb; k += 64) cnt += (buckets[k] <= v) ? 1 : 0;
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  int lo = cnt - 1;
  if (lo > nb - 2) lo = nb - 2;
  const float blo = buckets[lo], bhi = buckets[lo + 1];
  const float w = (v - blo) / (bhi - blo + 1e-8f);
  const float wlo = 1.0f - w;
  const float sum_th = wlo + w;
  // log_softmax
  float mx = -INFINITY;
  for (int k = lane; k < nb; k += 64) mx = fmaxf(mx, l[k]);
  mx = wave_max(mx);
  float se = 0.f;
  for (int k = lane; k < nb; k += 64) se += expf(l[k] - mx);
  se = wave_sum(se);
  const float lse = logf(se);
  for (int k = lane; k < nb; k += 64) {
    const float sm = expf(l[k] - mx) / se;
    const float th = (k == lo) ? wlo : ((k == lo + 1) ? w : 0.0f);
    g[k] = scale * (sm * sum_th - th);
  }
  if (lane == 0) {
    const float ls_lo = (l[lo] - mx) - lse, ls_hi = (l[lo + 1] - mx) - lse;
    row_loss[(long long)b * H + t] = -(wlo * ls_lo + w * ls_hi);
  }
}

int op_critic_ce(int B, int H, int nb, const float* logits, const float* R, const float* buckets, float scale,
                 float* row_loss, float* g_logits, hipStream_t s) {
  const int rows = B * (H + 1);
  hipLaunchKernelGGL(k_critic_ce, dim3(dr_cdiv(rows, 4)), dim3(256), 0, s, B, H, nb, logits, R, buckets, scale,
                     row_loss, g_logits);
  return dr_check_launch("critic_ce");
}

// ---------------------------------------------------------------------------
// optimiser: clip_grad_norm_(100) + AdamW (torch single-tensor op order) + EMA
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_sqnorm(long long n, const float* g, float* acc) {
  __shared__ float part[1024];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  const long long n4 = ((uintptr_t)g & 15) == 0 ? n / 4 : 0;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long long i = threadIdx.x; i < n4; i += 1024) {
    const float4 v = g4[i];
    s0 += v.x * v.x;
    s1 += v.y * v.y;
    s2 += v.z * v.z;
    s3 += v.w * v.w;
  }
  for (long long i = 4 * n4 + threadIdx.x; i < n; i += 1024) s0 += g[i] * g[i];
  part[threadIdx.x] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  for (int k = 512; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) part[threadIdx.x] += part[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) *acc = *acc + part[0];
}

extern "C" int dr_sqnorm(long long n, const float* g, float* acc, hipStream_t stream) {
  hipLaunchKernelGGL(k_sqnorm, dim3(1), dim3(1024), 0, stream, n, g, acc);
  return dr_check_launch("sqnorm");
}

// multi-block squared norm for large buffers (world-model gradients, 7.8 M
// floats): pass 1 writes one partial per block (contiguous chunks, float4
// loads), pass 2 adds them in a fixed order -- deterministic, no atomics
#define SQ_BLOCKS 512
__global__ __launch_bounds__(256) void k_sqnorm_part(long long n4, const float4* __restrict__ g4, long long chunk,
                                                     float* __restrict__ part) {
  __shared__ float red[256];
  const long long b0 = (long long)blockIdx.x * chunk;
  const long long b1 = b0 + chunk < n4 ? b0 + chunk : n4;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (long long i = b0 + threadIdx.x; i < b1; i += 256) {
    const float4 v = g4[i];
    s0 += v.x * v.x;
    s1 += v.y * v.y;
    s2 += v.z * v.z;
    s3 += v.w * v.w;
  }
  red[threadIdx.x] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(256) void k_sqnorm_final(int nb, const float* __restrict__ part, long long n,
                                                      long long n4, const float* __restrict__ g, float* acc) {
  __shared__ float red[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) s += part[i];
  for (long long i = 4 * n4 + threadIdx.x; i < n; i += 256) s += g[i] * g[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) *acc = *acc + red[0];
}

extern "C" int dr_sqnorm_multi(long long n, const float* g, float* acc, float* scratch, hipStream_t stream) {
  if (((uintptr_t)g & 15) || !scratch) return dr_sqnorm(n, g, acc, stream);
  const long long n4 = n / 4;
  long long nb = (n4 + 4095) / 4096;
  nb = nb < 1 ? 1 : (nb > SQ_BLOCKS ? SQ_BLOCKS : nb);
  const long long chunk = (n4 + nb - 1) / nb;
  hipLaunchKernelGGL(k_sqnorm_part, dim3((unsigned)nb), dim3(256), 0, stream, n4,
                     reinterpret_cast<const float4*>(g), chunk, scratch);
  DR_TRY(dr_check_launch("sqnorm_part"));
  hipLaunchKernelGGL(k_sqnorm_final, dim3(1), dim3(256), 0, stream, (int)nb, scratch, n, n4, g, acc);
  return dr_check_launch("sqnorm_final");
}

// The agent's clip statistics in ONE launch (Agent.py:137-148): sq[0] =
// |g_a|^2, sq[1] = |g_c|^2 (written, not accumulated) and skip = any
// non-finite value in the loss slots.  Blocks [0, nba) take contiguous float4
// chunks of buffer a, the rest buffer b; each writes one partial, and the
// last block to arrive (device-scope ticket) adds the partials in a fixed
// order -- deterministic, no float atomics -- and re-arms the ticket.
// Optional AdamW preludes (dr_ac_optimiser_step): the last block also runs
// k_adamw_prelude's step / bias-correction update of both optimisers.
struct AdamPre {
  int* step[2];
  float* hyper[2];
  double lr[2], b1[2], b2[2];
};
__device__ __forceinline__ void adamw_prelude_body(int* step, float* hyper, double lr, double b1, double b2) {
  const int st = *step + 1;
  *step = st;
  const double bc1 = 1.0 - pow(b1, (double)st);
  const double bc2 = 1.0 - pow(b2, (double)st);
  hyper[0] = (float)(lr / bc1);  // step_size
  hyper[1] = (float)sqrt(bc2);   // bias_correction2_sqrt
}

__global__ __launch_bounds__(256) void k_clip_stats(long long na, const float* __restrict__ ga, long long nb,
                                                    const float* __restrict__ gb, int nba, long long cha,
                                                    long long chb, int nloss, const float* __restrict__ loss,
                                                    float* part, unsigned* ticket, float* sq, int* skip,
                                                    AdamPre pre) {
  __shared__ float red[256];
  __shared__ int last;
  const bool isa = (int)blockIdx.x < nba;
  const float4* g4 = reinterpret_cast<const float4*>(isa ? ga : gb);
  const long long n4 = (isa ? na : nb) / 4;
  const long long ch = isa ? cha : chb;
  const long long b0 = (long long)(isa ? blockIdx.x : blockIdx.x - nba) * ch;
  const long long b1 = b0 + ch < n4 ? b0 + ch : n4;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (long long i = b0 + threadIdx.x; i < b1; i += 256) {
    const float4 v = g4[i];
    s0 += v.x * v.x;
    s1 += v.y * v.y;
    s2 += v.z * v.z;
    s3 += v.w * v.w;
  }
  red[threadIdx.x] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[blockIdx.x] = red[0];
    __threadfence();
    last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  for (int w = 0; w < 2; ++w) {
    const int p0 = w ? nba : 0, p1 = w ? (int)gridDim.x : nba;
    const float* g = w ? gb : ga;
    const long long n = w ? nb : na;
    float v = 0.f;
    for (int i = p0 + (int)threadIdx.x; i < p1; i += 256) v += __builtin_nontemporal_load(&part[i]);
    for (long long i = 4 * (n / 4) + threadIdx.x; i < n; i += 256) v += g[i] * g[i];
    __syncthreads();
    red[threadIdx.x] = v;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
      if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
      __syncthreads();
    }
    if (threadIdx.x == 0) sq[w] = red[0];
  }
  if (threadIdx.x == 0) {
    int bad = 0;
    for (int i = 0; i < nloss; ++i) bad |= !isfinite(loss[i]);
    *skip = bad;
    *ticket = 0u;
    if (!bad)
      for (int w = 0; w < 2; ++w)
        if (pre.step[w]) adamw_prelude_body(pre.step[w], pre.hyper[w], pre.lr[w], pre.b1[w], pre.b2[w]);
  }
}

extern "C" int dr_clip_stats(long long na, const float* ga, long long nb, const float* gb, int nloss,
                             const float* loss, float* sq, int* skip, void* scratch, hipStream_t stream) {
  DR_REQUIRE(ga && gb && sq && skip && scratch && na > 0 && nb > 0, "dr_clip_stats: bad arguments");
  DR_REQUIRE(!(((uintptr_t)ga | (uintptr_t)gb) & 15), "dr_clip_stats: buffers must be 16-byte aligned");
  auto blocks = [](long long n4) { long long b = (n4 + 2047) / 2048; return (int)(b < 1 ? 1 : (b > 256 ? 256 : b)); };
  const int nba = blocks(na / 4), nbb = blocks(nb / 4);
  const long long cha = (na / 4 + nba - 1) / nba, chb = (nb / 4 + nbb - 1) / nbb;
  float* part = static_cast<float*>(scratch);
  unsigned* ticket = reinterpret_cast<unsigned*>(part + DR_CLIP_SCRATCH_FLOATS - 1);
  AdamPre none = {};
  hipLaunchKernelGGL(k_clip_stats, dim3(nba + nbb), dim3(256), 0, stream, na, ga, nb, gb, nba, cha, chb, nloss,
                     loss, part, ticket, sq, skip, none);
  return dr_check_launch("clip_stats");
}

// prelude: step += 1 (unless skipped), bias corrections in double like
// torch's python scalars (adam.py: bias_correction1 = 1 - beta1**step ...)
__global__ void k_adamw_prelude(int* step, float* hyper, double lr, double b1, double b2, const int* skip) {
  if (skip && *skip) return;
  adamw_prelude_body(step, hyper, lr, b1, b2);
}

// one AdamW element (clip scale applied to the gradient in place first);
// returns the new parameter
__device__ __forceinline__ float adamw_elem(long long i, float* p, float* g, float* m, float* v, float clip, float keep,
                                            float omb1, float b2, float omb2, const float* hyper, float eps) {
  float gv = g[i];
  if (clip != 1.0f) {  // clip_grad_norm_ scales p.grad in place (Agent.py:147-148)
    gv = gv * clip;
    g[i] = gv;
  }
  const float pv = p[i] * keep;
  const float mv = m[i];
  const float mn = (omb1 < 0.5f) ? mv + omb1 * (gv - mv) : gv - (gv - mv) * (1.0f - omb1);
  const float vn = v[i] * b2 + (omb2 * gv) * gv;
  const float den = sqrtf(vn) / hyper[1] + eps;
  const float pn = pv + ((-hyper[0]) * mn) / den;
  p[i] = pn;
  m[i] = mn;
  v[i] = vn;
  return pn;
}

__global__ void k_adamw(long long n, float* p, float* g, float* m, float* v, const float* sqnorm,
                        float max_norm, float keep, float omb1, float b2, float omb2, const float* hyper, float eps,
                        const int* skip) {
  if (skip && *skip) return;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float clip = 1.0f;
  if (sqnorm) clip = fminf(max_norm / (sqrtf(*sqnorm) + 1e-6f), 1.0f);
  adamw_elem(i, p, g, m, v, clip, keep, omb1, b2, omb2, hyper, eps);
}

extern "C" int dr_adamw(long long n, float* p, float* g, float* m, float* v, const float* sqnorm,
                        float max_norm, double lr, double b1, double b2, double eps, double wd, int* step,
                        float* hyper, const int* skip, hipStream_t stream) {
  if (n <= 0) return DR_OK;
  hipLaunchKernelGGL(k_adamw_prelude, dim3(1), dim3(1), 0, stream, step, hyper, lr, b1, b2, skip);
  DR_TRY(dr_check_launch("adamw_prelude"));
  // torch's python-scalar math: 1 - lr*wd, 1 - beta in double, then one
  // rounding to f32 where the tensor op consumes them (a beta passed as f32
  // first would give 1 - 0.999f = 0.00099998713: 1.3e-5 off in exp_avg_sq)
  const float keep = (float)(1.0 - lr * wd);
  const float omb1 = (float)(1.0 - b1), omb2 = (float)(1.0 - b2);
  hipLaunchKernelGGL(k_adamw, dim3(blocks_for(n, 256)), dim3(256), 0, stream, n, p, g, m, v, sqnorm, max_norm, keep,
                     omb1, (float)b2, omb2, hyper, (float)eps, skip);
  return dr_check_launch("adamw");
}

__global__ void k_ema(long long n, float* t, const float* s, float keep, float tau, const int* skip) {
  if (skip && *skip) return;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a = t[i] * keep;
  t[i] = a + tau * s[i];
}

extern "C" int dr_ema(long long n, float* target, const float* src, float keep, float tau, const int* skip,
                      hipStream_t stream) {
  if (n <= 0) return DR_OK;
  hipLaunchKernelGGL(k_ema, dim3(blocks_for(n, 256)), dim3(256), 0, stream, n, target, src, keep, tau, skip);
  return dr_check_launch("ema");
}

// The actor-critic optimiser step of one train_Agent epoch in two launches
// (Agent.py:137-153): clip statistics + both AdamW preludes (k_clip_stats),
// then both AdamW updates and the critic -> target EMA in one elementwise
// pass (blocks [0, nbc) the critic, whose new parameters feed the EMA in
// registers; the rest the actor).  Same per-element arithmetic as dr_clip_stats
// + dr_adamw x2 + dr_ema, so the same bits.
struct AdamNet {
  long long n;
  float *p, *g, *m, *v, *hyper;
  const float* sq;
  float max_norm, keep, omb1, b2, omb2, eps;
};
__global__ void k_adamw2_ema(AdamNet c, AdamNet a, int nbc, float* target, float ema_keep, float tau,
                             const int* skip) {
  if (*skip) return;
  const bool isc = (int)blockIdx.x < nbc;
  const long long i = (long long)(isc ? blockIdx.x : blockIdx.x - nbc) * blockDim.x + threadIdx.x;
  const AdamNet& q = isc ? c : a;
  if (i >= q.n) return;
  const float clip = fminf(q.max_norm / (sqrtf(*q.sq) + 1e-6f), 1.0f);
  const float pn = adamw_elem(i, q.p, q.g, q.m, q.v, clip, q.keep, q.omb1, q.b2, q.omb2, q.hyper, q.eps);
  if (isc) {
    const float t = target[i] * ema_keep;
    target[i] = t + tau * pn;
  }
}

extern "C" int dr_ac_optimiser_step(long long na, float* pa, float* ga, float* ma, float* va, int* step_a,
                                    float* hyper_a, double lr_a, double b1_a, double b2_a, double eps_a, double wd_a,
                                    long long nc, float* pc, float* gc, float* mc, float* vc, int* step_c,
                                    float* hyper_c, double lr_c, double b1_c, double b2_c, double eps_c, double wd_c,
                                    float max_norm, float* target, float ema_keep, float tau, int nloss,
                                    const float* loss, float* sq, int* skip, void* scratch, hipStream_t stream) {
  DR_REQUIRE(pa && ga && ma && va && step_a && hyper_a && pc && gc && mc && vc && step_c && hyper_c && target && sq &&
                 skip && scratch && na > 0 && nc > 0,
             "dr_ac_optimiser_step: bad arguments");
  DR_REQUIRE(!(((uintptr_t)ga | (uintptr_t)gc) & 15), "dr_ac_optimiser_step: gradients must be 16-byte aligned");
  auto blocks = [](long long n4) { long long b = (n4 + 2047) / 2048; return (int)(b < 1 ? 1 : (b > 256 ? 256 : b)); };
  const int nba = blocks(na / 4), nbb = blocks(nc / 4);
  const long long cha = (na / 4 + nba - 1) / nba, chb = (nc / 4 + nbb - 1) / nbb;
  float* part = static_cast<float*>(scratch);
  unsigned* ticket = reinterpret_cast<unsigned*>(part + DR_CLIP_SCRATCH_FLOATS - 1);
  AdamPre pre = {{step_a, step_c}, {hyper_a, hyper_c}, {lr_a, lr_c}, {b1_a, b1_c}, {b2_a, b2_c}};
  hipLaunchKernelGGL(k_clip_stats, dim3(nba + nbb), dim3(256), 0, stream, na, ga, nc, gc, nba, cha, chb, nloss,
                     loss, part, ticket, sq, skip, pre);
  DR_TRY(dr_check_launch("clip_stats"));
  // torch's python-scalar math as dr_adamw
  const AdamNet c = {nc, pc, gc, mc, vc, hyper_c, sq + 1, max_norm, (float)(1.0 - lr_c * wd_c), (float)(1.0 - b1_c),
                     (float)b2_c, (float)(1.0 - b2_c), (float)eps_c};
  const AdamNet a = {na, pa, ga, ma, va, hyper_a, sq, max_norm, (float)(1.0 - lr_a * wd_a), (float)(1.0 - b1_a),
                     (float)b2_a, (float)(1.0 - b2_a), (float)eps_a};
  const int nbc = (int)blocks_for(nc, 256);
  hipLaunchKernelGGL(k_adamw2_ema, dim3(nbc + (unsigned)blocks_for(na, 256)), dim3(256), 0, stream, c, a, nbc, target,
                     ema_keep, tau, skip);
  return dr_check_launch("adamw2_ema");
}

__global__ void k_nonfinite(long long n, const float* x, int* flag) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  bool bad = (i < n) && !isfinite(x[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

extern "C" int dr_nonfinite(long long n, const float* x, int* flag, hipStream_t stream) {
  if (n <= 0) return DR_OK;
  hipLaunchKernelGGL(k_nonfinite, dim3(blocks_for(n, 256)), dim3(256), 0, stream, n, x, flag);
  return dr_check_launch("nonfinite");
}

// ---------------------------------------------------------------------------
// misc
// ---------------------------------------------------------------------------
// Fills and strided copies are kernels, not hipMemsetAsync / hipMemcpy2DAsync:
// inside a captured phase graph the runtime's memset / 2-D copy nodes were
// seen not to re-execute on replay on this stack (the BPTT's zeroed gradient
// accumulators then carried the previous epoch's values:
// tests/test_gpu_determinism.py), while kernel nodes always do.
__global__ void k_fill(long long n, float* x, float v) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = v;
}
__global__ void k_fill4(long long n4, float4* x, float v) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x)
    x[i] = make_float4(v, v, v, v);
}

int op_fill(long long n, float* x, float v, hipStream_t s) {
  if (n <= 0) return DR_OK;
  if (((uintptr_t)x & 15) == 0 && n % 4 == 0) {
    const long long n4 = n / 4;
    hipLaunchKernelGGL(k_fill4, dim3((unsigned)std::min<long long>(blocks_for(n4, 256), 2048)), dim3(256), 0, s, n4,
                       reinterpret_cast<float4*>(x), v);
  } else {
    hipLaunchKernelGGL(k_fill, dim3(blocks_for(n, 256)), dim3(256), 0, s, n, x, v);
  }
  return dr_check_launch("fill");
}

// up to DR_COPY_MAX independent strided copies in one launch (blockIdx.y =
// copy): the boundary copies around the unroll and the weight-gradient stage
// were one launch each
struct Copy2dBatch {
  Copy2dJob j[DR_COPY_MAX];
  int n;
};
__global__ void k_copy2d_multi(Copy2dBatch b) {
  const Copy2dJob& c = b.j[blockIdx.y];
  const bool v4 = c.v4 != 0;
  const long long wv = v4 ? c.width / 4 : c.width;
  const long long total = wv * c.rows;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / wv, k = i - r * wv;
    if (v4) reinterpret_cast<float4*>(c.dst + r * c.dp)[k] = reinterpret_cast<const float4*>(c.src + r * c.sp)[k];
    else c.dst[r * c.dp + k] = c.src[r * c.sp + k];
  }
}

int op_copy2d_multi(const Copy2dJob* jobs, int n, hipStream_t s) {
  if (n < 0 || n > DR_COPY_MAX) {
    dr_set_error("copy2d_multi: %d copies (at most %d)", n, DR_COPY_MAX);
    return DR_E_INVALID;
  }
  Copy2dBatch b = {};
  long long most = 0;
  int k = 0;
  for (int i = 0; i < n; ++i) {
    Copy2dJob c = jobs[i];
    if (c.rows <= 0 || c.width <= 0) continue;
    c.v4 = ((((uintptr_t)c.dst | (uintptr_t)c.src) & 15) == 0) && c.dp % 4 == 0 && c.sp % 4 == 0 && c.width % 4 == 0;
    most = std::max(most, (c.v4 ? c.width / 4 : c.width) * c.rows);
    b.j[k++] = c;
  }
  if (k == 0) return DR_OK;
  b.n = k;
  const unsigned blocks = (unsigned)std::min<long long>(blocks_for(most, 256), 2048);
  hipLaunchKernelGGL(k_copy2d_multi, dim3(blocks, (unsigned)k), dim3(256), 0, s, b);
  return dr_check_launch("copy2d_multi");
}

// rows x width floats, row pitches dp / sp (floats); float4 when everything is
// 16-byte aligned
template <bool V4>
__global__ void k_copy2d(float* dst, long long dp, const float* src, long long sp, long long width, long long rows) {
  const long long wv = V4 ? width / 4 : width;
  const long long total = wv * rows;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / wv, c = i - r * wv;
    if (V4) reinterpret_cast<float4*>(dst + r * dp)[c] = reinterpret_cast<const float4*>(src + r * sp)[c];
    else dst[r * dp + c] = src[r * sp + c];
  }
}

int op_copy2d(float* dst, long long dp, const float* src, long long sp, long long width, long long rows,
              hipStream_t s) {
  if (rows <= 0 || width <= 0) return DR_OK;
  const bool v4 = ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) && dp % 4 == 0 && sp % 4 == 0 && width % 4 == 0;
  const long long total = (v4 ? width / 4 : width) * rows;
  const unsigned blocks = (unsigned)std::min<long long>(blocks_for(total, 256), 2048);
  if (v4) hipLaunchKernelGGL(k_copy2d<true>, dim3(blocks), dim3(256), 0, s, dst, dp, src, sp, width, rows);
  else hipLaunchKernelGGL(k_copy2d<false>, dim3(blocks), dim3(256), 0, s, dst, dp, src, sp, width, rows);
  return dr_check_launch("copy2d");
}

// Conv2d weight [co][ci][4][4] -> [co][tap][ci] for NHWC implicit GEMM
__global__ void k_conv_repack(int cout, int cin, const float* w, float* wr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cout * cin * 16) return;
  const int co = i / (cin * 16), rem = i - co * cin * 16;
  const int ci = rem / 16, tap = rem - ci * 16;
  wr[(long long)co * cin * 16 + tap * cin + ci] = w[i];
}

int op_conv_repack(int cout, int cin, const float* w, float* wr, hipStream_t s) {
  hipLaunchKernelGGL(k_conv_repack, dim3(dr_cdiv(cout * cin * 16, 256)), dim3(256), 0, s, cout, cin, w, wr);
  return dr_check_launch("conv_repack");
}

// Buffer.sample_sequences gather (Buffer.py:49-61): u8 frames -> f32 0..255
__global__ void k_replay_gather(long long cap, int B, int S, int fe, int A, const unsigned char* frames,
                                const float* actions, const float* rewards, const float* continues,
                                const long long* starts, float* obs, float* act, float* rew, float* cont) {
  const long long bs = blockIdx.y;  // (b, s)
  const int b = (int)(bs / S), s = (int)(bs - (long long)b * S);
  const long long slot = (starts[b] + s) % cap;
  if (fe > 0) {
    const unsigned char* src = frames + slot * fe;
    float* dst = obs + bs * fe;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < fe; e += gridDim.x * blockDim.x) dst[e] = (float)src[e];
  }
  if (blockIdx.x == 0) {
    if ((int)threadIdx.x < A) act[bs * A + threadIdx.x] = actions[slot * A + threadIdx.x];
    if (threadIdx.x == 0) {
      if (rew) rew[bs] = rewards[slot];
      if (cont) cont[bs] = continues[slot];
    }
  }
}

extern "C" int dr_replay_gather(long long cap, int B, int S, int frame_elems, int A, const unsigned char* frames,
                                const float* actions, const float* rewards, const float* continues,
                                const long long* starts, float* obs_out, float* act_out, float* rew_out,
                                float* cont_out, hipStream_t stream) {
  if (B <= 0 || S <= 0 || A > 256) {
    dr_set_error("replay_gather: bad dims");
    return DR_E_INVALID;
  }
  const int gx = frame_elems > 0 ? dr_cdiv(frame_elems, 1024) : 1;
  hipLaunchKernelGGL(k_replay_gather, dim3(gx, B * S), dim3(256), 0, stream, cap, B, S,
                     frame_elems, A, frames, actions, rewards, continues, starts, obs_out, act_out, rew_out,
                     cont_out);
  return dr_check_launch("replay_gather");
}

__global__ void k_rng_advance(unsigned long long* rng, unsigned long long d) { rng[1] += d; }

extern "C" int dr_rng_advance(unsigned long long* rng, unsigned long long delta, hipStream_t stream) {
  hipLaunchKernelGGL(k_rng_advance, dim3(1), dim3(1), 0, stream, rng, delta);
  return dr_check_launch("rng_advance");
}

// CU-masked streams (include/dreamer_hip.h): the warm stream of the pipelined
// epochs (engine.py run_many)
extern "C" int dr_stream_create_cumask(int n_words, const unsigned* mask, hipStream_t* out) {
  DR_REQUIRE(n_words > 0 && n_words <= 64 && mask && out, "cu mask: 1..64 words and an output slot required");
  unsigned any = 0;
  for (int i = 0; i < n_words; ++i) any |= mask[i];
  DR_REQUIRE(any != 0, "cu mask: no CU selected");
  DR_TRY_HIP(hipExtStreamCreateWithCUMask(out, (uint32_t)n_words, mask));
  return DR_OK;
}
extern "C" int dr_stream_destroy(hipStream_t s) {
  DR_REQUIRE(s != nullptr, "null stream");
  DR_TRY_HIP(hipStreamDestroy(s));
  return DR_OK;
}
extern "C" int dr_device_cus(int* out) {
  DR_REQUIRE(out, "null output");
  int dev = 0;
  DR_TRY_HIP(hipGetDevice(&dev));
  DR_TRY_HIP(hipDeviceGetAttribute(out, hipDeviceAttributeMultiprocessorCount, dev));
  return DR_OK;
}
extern "C" int dr_host_device_ptr(void* host, void** dev) {
  DR_REQUIRE(host && dev, "null pointer");
  DR_TRY_HIP(hipHostGetDevicePointer(dev, host, 0));
  return DR_OK;
}

// ---------------------------------------------------------------------------
// vector observations (BASELINE configs[4]): gather the window rows of the
// f32 ring (Buffer.sample_sequences for D-float observations) time-major
// ---------------------------------------------------------------------------
__global__ void k_vec_gather(int n, int nb, int D, dr_frames src, float* __restrict__ X) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)n * D) return;
  const long long f = i / D;
  const int c = (int)(i - f * D);
  const int b = (int)(f % nb), t = (int)(f / nb) + src.t0;
  float v;
  if (src.ring) {
    const float* ring = reinterpret_cast<const float*>(src.ring);
    v = ring[((src.starts[b] + t) % src.ring_cap) * D + c];
  } else {
    v = src.obs[(long long)b * src.stride_b + (long long)t * src.stride_t + c];
  }
  X[i] = v;
}

int op_vec_gather(int n, int nb, int D, const dr_frames* src, float* X, hipStream_t s) {
  if (n <= 0) return DR_OK;
  if (D <= 0 || nb <= 0 || (!src->ring && !src->obs) || (src->ring && (!src->starts || src->ring_cap <= 0))) {
    dr_set_error("vec_gather: bad source (D=%d)", D);
    return DR_E_INVALID;
  }
  const long long total = (long long)n * D;
  hipLaunchKernelGGL(k_vec_gather, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, n, nb, D, *src, X);
  return dr_check_launch("vec_gather");
}
