// Internal launchers for the non-GEMM kernels of libdreamer_hip.
#pragma once
#include "common.h"

// GRU gates (torch gru_cell CPU op order: r = sig(hr+ir), u = sig(hz+iz),
// n = tanh(in + hn*r), h' = (h-n)*u + n).  gi/gh already hold the biases.
int op_gru_fwd(int B, int Hd, const float* gi, const float* gh, const float* h, long long ldh, float* hout,
               long long ldo, float* sr, float* su, float* sn, float* sghn, hipStream_t s);
// backward of the gate block: g_hp = dL/dh'; writes g_gi, g_gh [B][3H] and
// dL/dh (direct path g_hp*u) into gh_out (accumulate or overwrite).
int op_gru_bwd(int B, int Hd, const float* g_hp, long long ldg, const float* h, long long ldh, const float* sr,
               const float* su, const float* sn, const float* sghn, float* g_gi, float* g_gh, float* gh_out,
               long long ldo, int accumulate, hipStream_t s);
// categorical sampler over M rows x R groups x C classes
int op_sample(int M, int R, int C, const float* logits, long long ldl, const dr_noise* nz, int step, float* z,
              long long ldz, int* idx, float* soft, long long lds, hipStream_t s);
// dL/dlogits for z = onehot + p - p.detach(), p = 0.99*softmax + 0.01/C
int op_softmax_ste_bwd(int M, int R, int C, const float* gz, long long ldg, const float* soft, long long lds,
                       float* g_logits, hipStream_t s);
// LayerNorm(eps 1e-5) + SiLU backward per row: gx = dL/d silu-out, pre = LN input
int op_ln_silu_bwd(int M, int K, const float* gx, long long ldgx, const float* pre, long long ldp,
                   const float* gamma, const float* beta, float* g_pre, long long ldgp, float* gy, float* xhat,
                   hipStream_t s, unsigned short* g_pre16 = nullptr);  // g_pre16: optional bf16 (RNE) copy of g_pre
// out[n] (+)= sum_m X[m][n] * (Y ? Y[m][n] : 1)
// several column sums in one launch (bias / LayerNorm parameter gradients)
struct ColsumJob {
  int N;
  const float* X; long long ldx;
  const float* Y; long long ldy;  // optional elementwise factor
  float* out;
};
#define DR_MAX_CSJOBS 8
int op_colsum_multi(int M, const ColsumJob* jobs, int n, hipStream_t s);
int op_colsum(int M, int N, const float* X, long long ldx, const float* Y, long long ldy, float* out, int accumulate,
              hipStream_t s);
// symexp(sum softmax(logits) * buckets) per row -> out[m*ostride]
int op_bucket_value(int M, int nb, const float* logits, long long ldl, const float* buckets, float* out,
                    long long ostride, hipStream_t s);
int op_sigmoid(int M, const float* x, long long ldx, float* out, long long ostride, hipStream_t s);
// actor head: mu, clamp(ls,-5,2), sigma = softplus+1e-3, a = tanh(mu + eps*sigma)
int op_actor_head(int M, int A, const float* mu_raw, long long ldm, const float* ls_raw, long long ldl,
                  const dr_noise* nz, int step, int deterministic, float* a, long long lda, float* mu,
                  long long ldmu, float* sigma, long long lds, float* eps_save, hipStream_t s);
int op_actor_head_bwd_x(int M, int A, int N, const float* g_a, long long ldga, const float* g_mu_l,
                        const float* g_sig_l, long long ldgl, const float* a, long long lda, const float* ls_raw,
                        long long ldl, const float* eps, float* g_heads, long long ldh, const float* wt, float* gx,
                        long long ldx, hipStream_t s);
int op_actor_head_bwd(int M, int A, const float* g_a, long long ldga, const float* g_mu_l, const float* g_sig_l,
                      long long ldgl, const float* a, long long lda, const float* sigma, long long lds,
                      const float* ls_raw, long long ldl, const float* eps, float* g_heads, long long ldh,
                      hipStream_t s);
int op_conv_repack(int cout, int cin, const float* w, float* wr, hipStream_t s);
int op_fill(long long n, float* x, float v, hipStream_t s);
int op_copy2d(float* dst, long long dp, const float* src, long long sp, long long width, long long rows,
              hipStream_t s);
// several strided copies (dst rows dp apart, src rows sp apart) in one launch
struct Copy2dJob {
  float* dst;
  long long dp;
  const float* src;
  long long sp, width, rows;
  int v4, pad_;
};
#define DR_COPY_MAX 4
int op_copy2d_multi(const Copy2dJob* jobs, int n, hipStream_t s);
int op_mean(int n, const float* x, float* out, hipStream_t s);

// Vector observations (dr_dims.obs_dim = D > 0): frame f = t*nb + b of `src`
// (f32 ring rows [cap][D] or strided f32 obs) -> X[f][D]
int op_vec_gather(int n, int nb, int D, const dr_frames* src, float* X, hipStream_t s);
