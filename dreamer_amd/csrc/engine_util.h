// Internal helpers shared by the composite entry points (engine.hip, wm.hip):
// workspace carving, GEMM argument builders, GRU step wrappers.
#pragma once
#include <limits.h>
#include <string.h>

#include "conv.h"
#include "gemm.h"
#include "gru.h"
#include "ops.h"

int op_critic_ce(int B, int H, int nb, const float* logits, const float* R, const float* buckets, float scale,
                 float* row_loss, float* g_logits, hipStream_t s);

// ---------------------------------------------------------------------------
// workspace carving (the same sequence runs in "dry" mode for size queries)
// ---------------------------------------------------------------------------
struct Carve {
  char* base;
  size_t off;
  explicit Carve(void* b) : base((char*)b), off(0) {}
  float* f(long long n) { return (float*)raw(n * sizeof(float)); }
  int* i(long long n) { return (int*)raw(n * sizeof(int)); }
  void* raw(size_t bytes) {
    const size_t o = (off + 255) & ~(size_t)255;
    off = o + bytes;
    return base ? (void*)(base + o) : nullptr;
  }
};

#define WS_CHECK(c, bytes)                                                                 \
  do {                                                                                     \
    if ((c).off > (bytes)) {                                                               \
      dr_set_error("%s: workspace too small (%zu < %zu)", __func__, (size_t)(bytes), (c).off); \
      return DR_E_WORKSPACE;                                                               \
    }                                                                                      \
  } while (0)

// kernels, not hipMemcpy2DAsync / hipMemsetAsync: see op_fill in ops.hip
static inline int copy2d(float* dst, long long dpitch, const float* src, long long spitch, long long width, long long rows,
                  hipStream_t s) {
  return op_copy2d(dst, dpitch, src, spitch, width, rows, s);
}

static inline int zero(float* p, long long n, hipStream_t s) { return op_fill(n, p, 0.f, s); }

static inline int latent(const dr_dims* d) { return d->rows * d->cols; }
// stride-2 layers of the VAE (dr_dims.enc_depth: 0 / 4 = the reference's, 5 = configs[3]'s deeper VAE)
static inline int vae_depth(const dr_dims* d) { return d->enc_depth == 5 ? 5 : 4; }
static inline bool vae_depth_ok(const dr_dims* d) { return d->enc_depth == 0 || d->enc_depth == 4 || d->enc_depth == 5; }
// encoder channels e[0..N]: 3, f1, f2, 2 f2, 4 f2 (, 4 f2)  (VAE.py:33-42 and its one-layer deepening)
static inline int enc_chans(const dr_dims* d, int* e) {
  const int N = vae_depth(d);
  e[0] = 3; e[1] = d->enc_f1; e[2] = d->enc_f2; e[3] = 2 * d->enc_f2; e[4] = 4 * d->enc_f2;
  if (N == 5) e[5] = 4 * d->enc_f2;
  return N;
}
// decoder channels c[0..N]: 4 d2 (, 4 d2), 2 d2, d2, d1, 3  (VAE.py:128-137 and its mirror of the deepening)
static inline int dec_chans(const dr_dims* d, int* c) {
  const int N = vae_depth(d);
  int k = 0;
  c[k++] = 4 * d->dec_f2;
  if (N == 5) c[k++] = 4 * d->dec_f2;
  c[k++] = 2 * d->dec_f2; c[k++] = d->dec_f2; c[k++] = d->dec_f1; c[k++] = 3;
  return N;
}
// encoder feature width F (latent_mapper.0 input minus h): the flattened conv
// stack, or the vector-observation MLP's width 4*enc_f2 (dr_dims.obs_dim > 0)
static inline int enc_feat_dim(const dr_dims* d) {
  const int N = vae_depth(d);
  return d->obs_dim > 0 ? 4 * d->enc_f2 : 4 * d->enc_f2 * (d->img_h >> N) * (d->img_w >> N);
}

// Y[M][N] = A[M][K] W^T + b  (torch Linear), A row stride lda
static inline GemmArgs lin(int M, int N, int K, const float* A, long long lda, const float* W, long long ldw,
                    const float* bias, float* Y, long long ldy) {
  GemmArgs g = gemm_args();
  g.M = M; g.N = N; g.K = K;
  g.A = A; g.lda = lda;
  g.W = W; g.ldb = ldw;
  g.bias = bias;
  g.Y = Y; g.ldy = ldy;
  return g;
}
// Linear over the concatenation [A (Ka cols) | A2 (K2 cols)]
static inline GemmArgs lin2(int M, int N, const float* A, long long lda, int Ka, const float* A2, long long lda2, int K2,
                     const float* W, const float* bias, float* Y, long long ldy) {
  GemmArgs g = lin(M, N, Ka + K2, A, lda, W, Ka + K2, bias, Y, ldy);
  g.A2 = A2; g.lda2 = lda2; g.ksplitA = Ka;
  return g;
}
// Linear applied to SiLU(LayerNorm(pre)) (the LN+SiLU of the previous layer fused on load)
static inline GemmArgs lin_ln(int M, int N, int K, const float* pre, long long ldp, const dr_linear& ln, const float* W,
                       const float* bias, float* Y, long long ldy) {
  GemmArgs g = lin(M, N, K, pre, ldp, W, K, bias, Y, ldy);
  g.ln_g = ln.w; g.ln_b = ln.b;
  return g;
}
// input gradient: Y[M][N] (+)= G[M][K] W[K][N]  (W = torch weight [out=K][in=N])
static inline GemmArgs bwd_in(int M, int N, int K, const float* G, long long ldg, const float* W, long long ldw, float* Y,
                       long long ldy, int accumulate) {
  GemmArgs g = gemm_args();
  g.M = M; g.N = N; g.K = K;
  g.A = G; g.lda = ldg;
  g.W = W; g.ldb = ldw;
  g.Y = Y; g.ldy = ldy;
  g.accumulate = accumulate;
  return g;
}
// input gradient against a transposed weight WT [N=in][K=out] (NT, float4 loads)
static inline GemmArgs bwd_nt(int M, int N, int K, const float* G, long long ldg, const float* WT, float* Y, long long ldy,
                       int accumulate) {
  GemmArgs g = gemm_args();
  g.M = M; g.N = N; g.K = K;
  g.A = G; g.lda = ldg;
  g.W = WT; g.ldb = K;
  g.Y = Y; g.ldy = ldy;
  g.accumulate = accumulate;
  return g;
}
static inline int run(GemmLayout lay, int amode, const GemmArgs& a, hipStream_t s) { return gemm_launch(lay, amode, &a, 1, s); }

// split-K scratch for the tile GEMM: hand problem g up to 4 partial planes
// from a carved region (grouped problems take disjoint slices)
#define DR_SPLITK_MAX 4
static inline void give_splitk(GemmArgs& g, float*& cur, long long& left) {
  const long long need = (long long)DR_SPLITK_MAX * g.M * g.N;
  if (!cur || left < need) return;
  g.splitk_ws = cur;
  g.splitk_floats = need;
  cur += need;
  left -= need;
}
static inline long long splitk_floats(long long M, long long N) { return DR_SPLITK_MAX * M * N; }

// input gradient through SiLU(LayerNorm(pre)) and a transposed weight, fused:
// the GEMM's staged prologue computes g_pre from (gx, pre) (gemm.h AM_LNBWD);
// g_pre and the LN-parameter saves are written when requested.  Falls back to
// k_ln_silu_bwd + NT GEMM where the fused path does not apply.
static inline int lnbwd_nt(int M, int N, int K, const float* gx, long long ldgx, const float* pre, long long ld_pre,
                    const dr_linear& ln, const float* WT, float* Y, long long ldy, int accumulate, float* gpre,
                    long long ld_gpre, float* gy, float* xh, float* Y2, long long ldy2, int nsplitY, hipStream_t s,
                    const GruBwdEpi* gru_epi = nullptr, const void* planes = nullptr, float* sk = nullptr,
                    long long sk_n = 0) {
  GemmArgs g = bwd_nt(M, N, K, gx, ldgx, WT, Y, ldy, accumulate);
  g.Y2 = Y2; g.ldy2 = ldy2; g.nsplitY = nsplitY;
  if (gru_epi) g.gb = *gru_epi;
  const bool r16 = gemm_bwd_rows16(&g, 1);
  const bool ok = K % 4 == 0 && K <= (r16 ? 1024 : 256) && M <= 4096 && ldgx % 4 == 0 && ld_pre % 4 == 0 &&
                  ((((uintptr_t)gx | (uintptr_t)pre | (uintptr_t)WT | (uintptr_t)ln.w | (uintptr_t)ln.b) & 15) == 0);
  // on 64-row tiles (tall problems) the staged prologue, recomputed by every
  // column tile, costs more than one elementwise pass + a plain GEMM (B = 256,
  // N = 1624: 26.5 us fused vs the two launches; the 200-wide layers 16.5 us
  // against 5.0 + 6.3, profiles/r03x_epoch_kernel_table.txt); on 16-row tiles
  // (per-step products up to ~2.5 dispatch rounds) the prologue is fused
  const bool split = gpre != nullptr && M >= 128 && !r16;
  if (ok && !split) {
    g.pre = pre; g.ld_pre = ld_pre; g.ln_g = ln.w; g.ln_b = ln.b;
    g.a_out = gpre; g.ld_aout = ld_gpre;
    g.sv_gy = gy; g.sv_xh = xh; g.ld_sv = ld_gpre;
    return run(G_NT, AM_LNBWD, g, s);
  }
  DR_REQUIRE(gpre != nullptr, "LN-backward fallback needs a g_pre buffer");
  DR_TRY(op_ln_silu_bwd(M, K, gx, ldgx, pre, ld_pre, ln.w, ln.b, gpre, ld_gpre, gy, xh, s));
  g.A = gpre; g.lda = ld_gpre;
  if (planes) {  // tall products with weight planes: the split3 tall GEMM (gemm.hip s3_tall_ok; wplanes' layout)
    g.wsplit = reinterpret_cast<const unsigned short*>(planes);
    g.wsplit_np = (g.N + 127) / 128 * 128;
    g.splitk_ws = sk;  // (its split-K partial sums, when given)
    g.splitk_floats = sk ? sk_n : 0;
  }
  return run(G_NT, AM_PLAIN, g, s);
}

// weight gradient: dW[M=out][N=in] = sum_r G[r][m] X[r][n]  (rows r < R)
static inline GemmArgs bwd_w(int out, int in, int R, const float* G, long long ldg, const float* X, long long ldx, float* dW) {
  GemmArgs g = gemm_args();
  g.M = out; g.N = in; g.K = R;
  g.A = G; g.lda = ldg;
  g.W = X; g.ldb = ldx;
  g.Y = dW; g.ldy = in;
  return g;
}

// weight-gradient (TN) problems built by bwd_w: on the split3 bf16 MFMA,
// up to 4 problems per grouped launch (op_gemm_tn_split3_multi) when `ws`
// holds all their planes, else one problem after another through the same
// scratch; the f32 tile GEMM when a problem does not fit the split3 path
static inline bool tn_split3_ok(const GemmArgs& g) {
  return g.alpha == 1.0f && !g.act && !g.bias && !g.addend && g.ksplitB >= g.K && g.nsplitY >= g.N && !g.out_conv &&
         g.ksplitA >= g.K && g.epi == EPI_NONE && op_gemm_tn_split3_supported(g.M, g.N, g.K);
}
static inline TnProblem tn_problem(const GemmArgs& g) {
  return {g.M, g.N, g.K, g.A, g.lda, g.W, g.ldb, g.W2, g.ldb2, g.nsplitB < g.N ? g.nsplitB : g.N, g.Y, g.ldy,
          g.accumulate};
}
// scratch for n grouped problems of at most this size each
static inline size_t tn_group_bytes(size_t one, int n) { return one * (size_t)(n < 4 ? n : 4); }
static inline int tn_launch(const GemmArgs* p, int n, void* ws, size_t ws_bytes, hipStream_t s, int terms = 3) {
  bool ok = ws != nullptr;
  for (int i = 0; i < n && ok; ++i) ok = tn_split3_ok(p[i]) && op_gemm_tn_split3_ws_bytes(p[i].M, p[i].N, p[i].K) <= ws_bytes;
  if (!ok) return gemm_launch(G_TN, AM_PLAIN, p, n, s);
  for (int i0 = 0; i0 < n;) {
    TnProblem q[4];
    int k = 0;
    while (i0 + k < n && k < 4) {
      q[k] = tn_problem(p[i0 + k]);
      if (k > 0 && op_gemm_tn_split3_multi_ws_bytes(q, k + 1) > ws_bytes) break;
      ++k;
    }
    DR_TRY(op_gemm_tn_split3_multi(q, k, ws, ws_bytes, s, terms));
    i0 += k;
  }
  return DR_OK;
}

// per-step chain products on the bf16 MFMA (gemm.hip k_gemm_wks3): the weight
// [N][K] (row stride ldw) split once per call into bf16 planes; wplanes() then
// hands them to the problem
static inline int split_planes(int N, int K, const float* W, long long ldw, void* planes, hipStream_t s) {
  if (!planes) return DR_OK;
  return op_nt_repack_split3(N, K, W, (int)ldw, planes, s);
}
static inline void wplanes(GemmArgs& g, const void* planes) {
  if (!planes) return;
  g.wsplit = reinterpret_cast<const unsigned short*>(planes);
  g.wsplit_np = (g.N + 127) / 128 * 128;  // op_nt_split3_ws_bytes' row padding
}

// one-hot index buffers hold [B][R] class indices followed by the [B][R]
// straight-through values at those indices (what the fused GRU gathers)
static inline float* onehot_vals(int* idx, long long B, int R) { return reinterpret_cast<float*>(idx + B * R); }

// fused categorical-sampler epilogue on a logits GEMM (VAE.py:88-98,
// DynamicsPredictors.py:33-39): z (STE value), idx, softmax for the backward
static inline void with_sampler(GemmArgs& g, const dr_dims* d, const dr_noise& nz, int step, float* z, long long ldz,
                         int* idx, float* soft, long long ld_soft) {
  g.epi = EPI_SAMPLE;
  g.noise = nz;
  g.step = step;
  g.R = d->rows;
  g.C = d->cols;
  g.unimix = (float)(0.01 * (1.0 / d->cols));
  g.z_out = z; g.ldz = ldz; g.idx_out = idx; g.soft_out = soft; g.ld_soft = ld_soft;
  g.zval_out = idx ? onehot_vals(idx, g.M, d->rows) : nullptr;
}

// LN-SiLU -> Linear -> LN-SiLU -> Linear tail of a 3-layer head (mlp2_launch)
// from the first Linear's output X; e = the last Linear (plus its epilogue)
static inline Mlp2Args mlp2(int M, int K1, int K2, const float* X, long long ldx, const dr_linear& ln1,
                            const dr_linear& l3, const dr_linear& ln4, const GemmArgs& e) {
  Mlp2Args a;
  memset(&a, 0, sizeof(a));
  a.M = M; a.K1 = K1; a.K2 = K2;
  a.X = X; a.ldx = ldx;
  a.ln1_g = ln1.w; a.ln1_b = ln1.b;
  a.W3 = l3.w; a.b3 = l3.b;
  a.ln4_g = ln4.w; a.ln4_b = ln4.b;
  a.e = e;
  return a;
}

// fused actor-head epilogue on the stacked [mu_head; log_sig_head] GEMM
static inline void with_actor_head(GemmArgs& g, int A, const dr_noise& nz, int step, int det, float* act, long long ld_act,
                            float* mu, long long ld_mu, float* sig, long long ld_sig, float* eps_save, float* ls_save,
                            long long ld_ls) {
  g.epi = EPI_ACTOR;
  g.noise = nz;
  g.step = step;
  g.na = A;
  g.det = det;
  g.act_out = act; g.ld_act = ld_act; g.mu_out = mu; g.ld_mu = ld_mu; g.sig_out = sig; g.ld_sig = ld_sig;
  g.eps_save = eps_save; g.ls_save = ls_save; g.ld_ls = ld_ls;
  g.Y = nullptr;
}

// [mu_head; log_sig_head] stacked into one [2A][in] weight (+ bias) so one
// workgroup sees both halves of a row
static inline int stack_heads(const dr_actor* ac, int A, int in, float* w, float* b, hipStream_t s) {
  DR_TRY(copy2d(w, in, ac->mu.w, in, in, A, s));
  DR_TRY(copy2d(w + (long long)A * in, in, ac->ls.w, in, in, A, s));
  DR_TRY(copy2d(b, A, ac->mu.b, A, A, 1, s));
  return copy2d(b + A, A, ac->ls.b, A, A, 1, s);
}

// GRU step on a sampled one-hot latent (idx) via the fused kernel
// z / ldz: the latent rows idx came from (read only for dense-marked groups; NULL
// where idx always comes from the sampler)
static inline int gru_onehot(const dr_dims* d, const dr_world_model* wm, int B, int* idx, const float* a, long long lda, const float* h, long long ldh, float* hout,
                      long long ldo, const float* wt, float* sr, float* su, float* sn, float* sghn, hipStream_t s,
                      const float* z = nullptr, long long ldz = 0, float* gh_ws = nullptr, int gh_ready = 0,
                      unsigned short* hout16 = nullptr) {
  GruArgs g;
  memset(&g, 0, sizeof(g));
  g.gh_ws = gh_ws;
  g.gh_ready = gh_ready;
  g.z = z; g.ldz = ldz;
  g.B = B; g.Hd = d->hidden; g.R = d->rows; g.C = d->cols; g.A = d->action;
  g.idx = idx; g.zval = onehot_vals(idx, B, d->rows); g.a = a; g.lda = lda; g.h = h; g.ldh = ldh;
  g.wt = wt; g.b_ih = wm->b_ih; g.w_hh = wm->w_hh; g.b_hh = wm->b_hh;
  g.hout = hout; g.hout16 = hout16; g.ldo = ldo; g.sr = sr; g.su = su; g.sn = sn; g.sghn = sghn;
  return op_gru_fused(g, s);
}

// h' = GRU(z, a, h) with gi/gh from one grouped GEMM launch
static inline int gru_step(const dr_dims* d, const dr_world_model* wm, int B, const float* z, long long ldz,
                    const float* a, long long lda, const float* h, long long ldh, float* hout, long long ldo,
                    float* gi, float* gh, float* sr, float* su, float* sn, float* sghn, hipStream_t s) {
  const int L = latent(d), Hd = d->hidden, A = d->action;
  GemmArgs p[2];
  p[0] = lin2(B, 3 * Hd, z, ldz, L, a, lda, A, wm->w_ih, wm->b_ih, gi, 3 * Hd);
  p[1] = lin(B, 3 * Hd, h ? Hd : 0, h, ldh, wm->w_hh, Hd, wm->b_hh, gh, 3 * Hd);
  DR_TRY(gemm_launch(G_NT, AM_PLAIN, p, 2, s));
  return op_gru_fwd(B, Hd, gi, gh, h, ldh, hout, ldo, sr, su, sn, sghn, s);
}

