// a19/a20: the world-model training step (WorldModel.training_step,
// WorldModel.py:148-198; unroll_model 84-146; Decoder.forward
// VariationalAutoEncoder.py:139-161) as one fixed launch sequence.
//
// Rows are time-major (m = t*B + b).  The posterior scan runs per step (B
// rows); every head that does not feed the recurrence (prior, decoder, reward,
// continue) runs once over the M1 = (T-1)*B rows t >= 1 -- the only rows the
// losses read (WorldModel.py:141-145), so row t = 0 of the decoder / prior is
// never computed.  The backward mirrors it: batched head backward into dL/dh,
// dL/dz, then the reverse scan (straight-through sampler, latent_mapper, GRU),
// then the encoder convolutions over all M frames.
#include <algorithm>

#include "engine_util.h"

// ---------------------------------------------------------------------------
// small kernels of the loss
// ---------------------------------------------------------------------------
// window actions / rewards / continues -> time-major [T][B](*A)
__global__ void k_wm_gather(int B, int T, int A, dr_wm_batch bt, float* act_tm, float* rew_tm, float* cont_tm) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * T) return;
  const int t = i / B, b = i - t * B;
  for (int a = 0; a < A; ++a) act_tm[(long long)i * A + a] = bt.actions[b * bt.act_sb + t * bt.act_st + a];
  rew_tm[i] = bt.rewards[b * bt.rc_sb + t * bt.rc_st];
  cont_tm[i] = bt.continues[b * bt.rc_sb + t * bt.rc_st];
}

// block-wide sum in a fixed order (deterministic)
__device__ float block_sum256(float v, float* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}

// mask = continues[:, :T-1] (WorldModel.py:170); row i < M1 of every head /
// decoder frame is (t = i/B + 1, b) and its mask is cont_tm[i].
// stats[0] = local mask.sum() (all-reduced by a data-parallel caller)
__global__ __launch_bounds__(256) void k_wm_masksum(int M1, const float* cont_tm, float* stats) {
  __shared__ float red[256];
  float s = 0.0f;
  for (int i = threadIdx.x; i < M1; i += 256) s += cont_tm[i];
  s = block_sum256(s, red);
  if (threadIdx.x == 0) stats[0] = s;
}

// scal[0] = mask.sum() + 1e-5 (WorldModel.py:185, global); coef_row =
// beta_pred * mask / denom (the factor of every prediction-loss gradient);
// coef_obs = 2 * coef_row
__global__ __launch_bounds__(256) void k_wm_coef(int M1, const float* cont_tm, float beta_pred, const float* stats,
                                                 float* scal, float* coef_row, float* coef_obs) {
  const float denom = stats[0] + 1e-5f;
  if (threadIdx.x == 0) scal[0] = denom;
  for (int i = threadIdx.x; i < M1; i += 256) {
    const float c = beta_pred * cont_tm[i] / denom;
    coef_row[i] = c;
    coef_obs[i] = 2.0f * c;
  }
}

// KL(post || prior) per (row, latent group) (WorldModel.py:175-183;
// torch.distributions.kl._kl_categorical_categorical on normalised logits).
// MODE 0: kl_grp[row][g].  MODE 1: gradients -- dyn: d/d prior = cd*(q - p);
// rep: d/d post = cr * p * (lp - lq - KL_g), cd/cr = scal[1]/scal[2] * mask.
template <int MODE>
__global__ void k_wm_kl(int M1, int R, int C, int W, const float* __restrict__ prior, const float* __restrict__ post,
                        const float* __restrict__ cont_tm, const float* __restrict__ scal, float* kl_grp,
                        float* g_prior, float* g_post) {
  const int gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const int grp = gtid / W, c = gtid - grp * W;
  const bool valid = grp < M1 * R;
  const int row = valid ? grp / R : 0, g = valid ? grp - row * R : 0;
  const bool act = valid && c < C;
  const long long o = (long long)row * R * C + (long long)g * C + c;
  const float xp = act ? post[o] : -INFINITY;
  const float xq = act ? prior[o] : -INFINITY;
  const float mp = group_max(xp, W), mq = group_max(xq, W);
  const float ep = act ? expf(xp - mp) : 0.0f, eq = act ? expf(xq - mq) : 0.0f;
  const float sp = group_sum(ep, W), sq = group_sum(eq, W);
  const float lp = xp - (mp + logf(sp)), lq = xq - (mq + logf(sq));
  const float p = ep / sp;
  const float term = act ? p * (lp - lq) : 0.0f;
  const float klg = group_sum(term, W);
  if (MODE == 0) {
    if (act && c == 0) kl_grp[(long long)row * R + g] = klg;
  } else if (act) {
    const float m = cont_tm[row];
    const float cd = scal[1] * m, cr = scal[2] * m;
    g_prior[o] = cd * (eq / sq - p);
    g_post[o] = cr * (p * (lp - lq - klg));
  }
}

// reward two-hot log-likelihood and continue BCE per row (WorldModel.py:125-138)
// and their gradients scaled by coef_row; one wave per row
__global__ __launch_bounds__(256) void k_wm_heads(int M1, int nb, const float* __restrict__ rlog,
                                                  const float* __restrict__ clog, const float* __restrict__ rew_tm,
                                                  const float* __restrict__ cont_tm,
                                                  const float* __restrict__ buckets,
                                                  const float* __restrict__ coef_row, float* rew_row, float* cont_row,
                                                  float* g_rew, float* g_cont) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M1) return;
  const float* x = rlog + (long long)row * nb;
  float mx = -INFINITY;
  for (int j = lane; j < nb; j += 64) mx = fmaxf(mx, x[j]);
  mx = wave_max(mx);
  float se = 0.0f;
  for (int j = lane; j < nb; j += 64) se += expf(x[j] - mx);
  se = wave_sum(se);
  const float lse = mx + logf(se);
  // to_twohot (DreamerUtils.py:39-50): clamp, searchsorted(right=True) - 1, clamp <= nb-2
  const float rv = rew_tm[row];  // torch.clamp keeps NaN (-> non-finite loss -> skipped step)
  const float v = isnan(rv) ? rv : fminf(fmaxf(rv, buckets[0]), buckets[nb - 1]);
  float cnt = 0.0f;
  for (int j = lane; j < nb; j += 64) cnt += (buckets[j] <= v) ? 1.0f : 0.0f;
  int lo = (int)wave_sum(cnt) - 1;
  lo = lo > nb - 2 ? nb - 2 : (lo < 0 ? 0 : lo);
  const float blo = buckets[lo], bhi = buckets[lo + 1];
  const float w = (v - blo) / (bhi - blo + 1e-8f);
  const float coef = coef_row[row];
  for (int j = lane; j < nb; j += 64) {
    const float th = (j == lo) ? 1.0f - w : ((j == lo + 1) ? w : 0.0f);
    g_rew[(long long)row * nb + j] = coef * (expf(x[j] - mx) / se - th);
  }
  if (lane == 0) {
    rew_row[row] = (1.0f - w) * (x[lo] - lse) + w * (x[lo + 1] - lse);
    const float xc = clog[row], y = cont_tm[row];
    // binary_cross_entropy_with_logits: (1 - y) x + max(-x, 0) + log(exp(-max) + exp(-x - max))
    const float mv = fmaxf(-xc, 0.0f);
    cont_row[row] = (1.0f - y) * xc + mv + logf(expf(-mv) + expf(-xc - mv));
    g_cont[row] = coef * (1.0f / (1.0f + expf(-xc)) - y);
  }
}

// local masked sums of the loss terms: stats[1..4] = sum mask * (squared
// error, reward log-lik, continue BCE, KL) over this rank's rows
__global__ __launch_bounds__(256) void k_wm_stats(int M1, int R, int nparts, const float* __restrict__ obs_part,
                                                  const float* __restrict__ rew_row,
                                                  const float* __restrict__ cont_row,
                                                  const float* __restrict__ kl_grp, const float* __restrict__ cont_tm,
                                                  float* stats) {
  __shared__ float red[256];
  float so = 0.f, sr = 0.f, sc = 0.f, sk = 0.f;
  for (int i = threadIdx.x; i < M1; i += 256) {
    const float m = cont_tm[i];
    float o = 0.f;
    for (int j = 0; j < nparts; ++j) o += obs_part[(long long)i * nparts + j];
    float k = 0.f;
    for (int g = 0; g < R; ++g) k += kl_grp[(long long)i * R + g];
    so += o * m;
    sr += rew_row[i] * m;
    sc += cont_row[i] * m;
    sk += k * m;
  }
  so = block_sum256(so, red);
  sr = block_sum256(sr, red);
  sc = block_sum256(sc, red);
  sk = block_sum256(sk, red);
  if (threadIdx.x == 0) {
    stats[1] = so;
    stats[2] = sr;
    stats[3] = sc;
    stats[4] = sk;
  }
}

// losses (WorldModel.py:170-189) from the (global) sums and the KL-gradient
// factors of the free-bit clamp max(1, KL): d max(1, k)/dk = 1 (k > 1),
// 1/2 (k == 1), 0 (k < 1).  rows = B_global * (T - 1) (torch.mean's count).
__global__ void k_wm_final(const float* stats, int rows, dr_wm_loss_cfg cfg, float* scal, float* losses, int* skip) {
  if (threadIdx.x != 0) return;
  const float denom = stats[0] + 1e-5f;
  const float pred = (stats[1] - stats[2] + stats[3]) / denom;
  const float kl = stats[4] / (float)rows;
  const float total = cfg.beta_pred * pred + cfg.beta_dyn * fmaxf(1.0f, kl) + cfg.beta_rep * fmaxf(1.0f, kl);
  const float wk = kl > 1.0f ? 1.0f : (kl == 1.0f ? 0.5f : 0.0f);
  scal[1] = cfg.beta_dyn * wk / (float)rows;
  scal[2] = cfg.beta_rep * wk / (float)rows;
  losses[0] = total;
  losses[1] = pred;
  losses[2] = kl;
  losses[3] = kl;
  if (skip) *skip = isfinite(total) ? 0 : 1;
}

// gl = 0.99 * softmax-backward(gz) (+ extra): the straight-through sampler's
// gradient (VAE.py:92-98) plus the KL-rep gradient of the same logits
__global__ void k_ste_bwd_add(int M, int R, int C, int W, const float* __restrict__ gz, long long ldg,
                              const float* __restrict__ soft, long long lds, const float* __restrict__ extra,
                              long long lde, float* __restrict__ gl, long long ldl) {
  const int gtid = blockIdx.x * blockDim.x + threadIdx.x;
  const int grp = gtid / W, c = gtid - grp * W;
  const bool valid = grp < M * R;
  const int m = valid ? grp / R : 0, r = valid ? grp - m * R : 0;
  const bool act = valid && c < C;
  const float gs = act ? gz[(long long)m * ldg + r * C + c] * 0.99f : 0.0f;
  const float sv = act ? soft[(long long)m * lds + r * C + c] : 0.0f;
  const float dot = group_sum(gs * sv, W);
  if (act) {
    float v = sv * (gs - dot);
    if (extra) v += extra[(long long)m * lde + r * C + c];
    gl[(long long)m * ldl + r * C + c] = v;
  }
}

__global__ void k_mul_dsilu(long long n, float* __restrict__ g, const float* __restrict__ pre) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) g[i] = g[i] * dr_dsilu(pre[i]);
}

// rows of a [C*P][K] matrix between the NCHW flatten order (c*P + p) and NHWC
// (p*C + c): to_nhwc: out[p*C + c] = in[c*P + p], else the inverse
__global__ void k_perm_rows(int C, int P, int K, const float* __restrict__ in, float* __restrict__ out, int to_nhwc) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)C * P * K) return;
  const long long row = i / K;
  const int k = (int)(i - row * K);
  const int c = (int)(row / P), p = (int)(row - (long long)c * P);  // row in NCHW order
  const long long nh = ((long long)p * C + c) * K + k;
  if (to_nhwc) out[nh] = in[i];
  else out[i] = in[nh];
}

__global__ void k_silu(long long n, const float* __restrict__ x, float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = dr_silu(x[i]);
}

// vector observations: decoder output mu (no Tanh) against the target rows,
// squared error per row into part[row] (one part per frame for k_wm_stats)
// and dL/dmu = coef[row] * (mu - x) (coef carries the 2 and the mask weights,
// as CT_EPI_TANH_MSE's does before its (1 - mu^2)); a wave per row
__global__ __launch_bounds__(256) void k_vec_mse(int M1, int D, const float* __restrict__ mu,
                                                 const float* __restrict__ x, const float* __restrict__ coef,
                                                 float* __restrict__ g, float* __restrict__ part) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M1) return;
  const float cf = coef[row];
  float sq = 0.f;
  for (int c = lane; c < D; c += 64) {
    const long long o = (long long)row * D + c;
    const float err = mu[o] - x[o];
    sq += err * err;
    g[o] = cf * err;
  }
  sq = wave_sum(sq);
  if (lane == 0) part[row] = sq;
}

static int blocks(long long n, int t) { return (int)((n + t - 1) / t); }

// split-K scratch for one launch's problems (disjoint slices of the pool)
static void splitk_all(GemmArgs* p, int n, float* pool, long long pool_n) {
  float* cur = pool;
  long long left = pool_n;
  for (int i = 0; i < n; ++i) give_splitk(p[i], cur, left);
}

static int perm_rows(int C, int P, int K, const float* in, float* out, int to_nhwc, hipStream_t s) {
  const long long n = (long long)C * P * K;
  hipLaunchKernelGGL(k_perm_rows, dim3(blocks(n, 256)), dim3(256), 0, s, C, P, K, in, out, to_nhwc);
  return dr_check_launch("perm_rows");
}

static int pow2_ge(int c) {
  int w = 1;
  while (w < c) w <<= 1;
  return w;
}

// ---------------------------------------------------------------------------
// workspace
// ---------------------------------------------------------------------------
struct MlpBwd {  // backward scratch of one 3-layer head (and its LayerNorm saves)
  float *gx2, *gp2, *gy2, *xh2, *gx1, *gp1, *gy1, *xh1;
};
struct WmWs {
  void* tn;         // split3 TN scratch (tn_launch)
  size_t tn_bytes;
  // encoder (all M frames): conv k's pre-activation (NHWC) and output (NHWC; the last NCHW = the flatten order)
  float *x0, *pre[DR_MAX_DEPTH], *a[DR_MAX_DEPTH], *feat;
  float *wr[DR_MAX_DEPTH], *wqe[DR_MAX_DEPTH];  // conv k repacked (forward) / as a convT (data gradient, k >= 1)
  // window data, scan tape
  float *act_tm, *rew_tm, *cont_tm, *zeros, *h_all, *z_all, *soft, *plog, *pre_m, *x_m, *sr, *su, *sn, *sghn, *gi, *gh,
      *wt;
  int* idx;
  // heads (M1 rows)
  float *pp1, *px1, *pp2, *px2, *prior_lg, *rp1, *rx1, *rp2, *rx2, *rew_lg, *cp1, *cx1, *cp2, *cx2, *cont_lg;
  // decoder: upscaler pre-activations (du1, du2 = .3 output NHWC), convT k's output pre-activation dq[k] (k < N-1;
  // vector mode: dq[0] = image_builder.0 pre, dq[1] = mu) and its SiLU dqp[k]; dgout = dL/d(pre-tanh output)
  float *du1, *dx1, *du2, *du2p, *dq[DR_MAX_DEPTH], *dqp[DR_MAX_DEPTH], *dgout, *w3p, *b3p;
  float *wqd[DR_MAX_DEPTH], *wrd[DR_MAX_DEPTH];
  // split3 bf16 weight planes (conv_split.hip) of encoder conv k (forward) and
  // of decoder convT k read as a Conv2d (its data gradient); NULL: f32 path
  void *s3e[DR_MAX_DEPTH], *s3d[DR_MAX_DEPTH];
  // ... and of decoder convT k (forward) / encoder conv k's data gradient as upsampling convs
  void *t3d[DR_MAX_DEPTH], *t3e[DR_MAX_DEPTH];
  void* e12w1;  // conv1's split3 weight planes for k_enc12_split3
  // the posterior scan's per-step products (latent_mapper.0's h-columns, W_hh)
  // as split3 planes for k_gemm_wks3 (B >= 128), as in dr_observe_scan
  void *s3m0, *s3whh;
  // ... and of the scan backward's input-gradient products (W_ih^T's latent
  // rows, W_hh^T; K = 3 Hd)
  void *s3wtb, *s3twhh;
  // split3 planes of the tall (B (T-1) / B T rows) NT products' weights: the
  // heads' input-gradient Linears (.3 / .0 of each, the prior's .6), the
  // decoder upscaler's .3 / .0, the encoder projection (forward, and its
  // transposed input gradient) -- k_gemm_split3 instead of the f32 tile kernel
  void *pl_h3[3], *pl_h0[3], *pl_h6, *pl_up3, *pl_up0, *pl_w0tp, *pl_map0f;
  // ... and of the forward heads / upscaler over B (T - 1) rows: the first
  // Linears (prior, reward, continue, upscaler.0), the .3 layers, the prior's
  // .6, upscaler.3 (permuted rows)
  void *pl_f0[4], *pl_f3[3], *pl_f6, *pl_fup3;
  // loss
  float *coef_row, *coef_obs, *obs_part, *obs_bpart, *kl_grp, *rew_row, *cont_row, *scal, *stats;
  float* csp;  // per-tile channel sums of the last decoder layer's input gradient (k_conv_nhwc csum)
  // backward
  float *gH, *gZ, *glog, *gpost, *g_prior, *g_rew, *g_cont;
  MlpBwd bp, br, bc;
  float *gxu, *gpu, *gyu, *xhu, *dgq[DR_MAX_DEPTH], *dgu2, *dw3p, *db3p;  // dgq[k]: dL/d dq[k]
  float *ggi, *ggh, *gpre_m, *gy_m, *xh_m, *gx_s, *gh_dummy;
  float* gp[DR_MAX_DEPTH];  // dL/d pre[k]
  // transposed / permuted weights
  float *t_pl6, *t_pl3, *t_pl0, *t_rl6, *t_rl3, *t_rl0, *t_cl6, *t_cl3, *t_cl0, *t_up3, *t_up0, *t_map3, *t_map0, *t_whh,
      *w0tp;
  float *cws;  // conv weight-gradient / channel-sum scratch
  long long cws_n;
  float* sk;  // split-K partial planes of the tile GEMMs (reused launch to launch)
  long long sk_n;
};

struct WmDims {
  int B, T, M, M1, L, Hd, A, eh, nb, IH, IW, Pf, F, d1, d2, C0, dh, Fd, ph1, ph2, rh1, rh2, ch1, ch2;
  int N;                                        // VAE depth (4 = the reference, 5 = configs[3]'s deeper VAE)
  int e[DR_MAX_DEPTH + 1], cd[DR_MAX_DEPTH + 1];  // encoder / decoder channels (engine_util.h enc_chans / dec_chans)
  long long pix[DR_MAX_DEPTH + 1];              // pixels per frame at resolution level k: (IH >> k) (IW >> k)
  int Dv;  // vector observations (dr_dims.obs_dim): MLP encoder / decoder, no conv planes
  // bf16 operand terms of the split-conv kernels: 3 = f32-accurate (parity
  // mode), 1 = bf16 perf mode (dr_dims.precision)
  int terms;
};
static WmDims wm_dims(const dr_dims* d, int B, int T) {
  WmDims w;
  memset(&w, 0, sizeof(w));
  w.B = B; w.T = T; w.M = B * T; w.M1 = B * (T - 1);
  w.L = latent(d); w.Hd = d->hidden; w.A = d->action; w.eh = d->enc_hidden; w.nb = d->buckets;
  w.IH = d->img_h; w.IW = d->img_w;
  w.N = enc_chans(d, w.e);
  dec_chans(d, w.cd);
  for (int k = 0; k <= w.N; ++k) w.pix[k] = (long long)(w.IH >> k) * (w.IW >> k);
  w.Pf = (int)w.pix[w.N];
  w.F = w.e[w.N] * w.Pf;
  w.d1 = d->dec_f1; w.d2 = d->dec_f2; w.C0 = 4 * d->dec_f2; w.dh = d->dec_hidden; w.Fd = w.C0 * w.Pf;
  w.ph1 = d->prior_h1; w.ph2 = d->prior_h2; w.rh1 = d->rew_h1; w.rh2 = d->rew_h2; w.ch1 = d->cont_h1; w.ch2 = d->cont_h2;
  w.Dv = d->obs_dim > 0 ? d->obs_dim : 0;
  w.terms = d->precision == DR_PREC_BF16 ? 1 : 3;
  if (w.Dv) {  // widths of the MLP stand-ins (include/dreamer_hip.h, dr_dims.obs_dim)
    w.IH = w.IW = 0;
    w.Pf = 1;
    w.F = 4 * d->enc_f2;
    w.Fd = w.C0;
    for (int k = 0; k <= w.N; ++k) w.pix[k] = 0;
  }
  return w;
}
// channel stride of conv k's input (the frames are padded to 4 channels) and of convT k's output (3 -> 4)
static inline int enc_cin_st(const WmDims& D, int k) { return k == 0 ? 4 : D.e[k]; }
static inline int dec_cout_st(const WmDims& D, int k) { return k == D.N - 1 ? 4 : D.cd[k + 1]; }

// the convolutions that run f32-accurate on the bf16 MFMA (3-term split):
// encoder conv k >= 1 (conv1's 4-channel input stays on the f32 MFMA) and the
// data gradient of decoder convT k (a Conv2d from cout_t to cin_t channels)
static inline bool enc_s3(const WmDims& D, int k) {
  return !D.Dv && k >= 1 && op_conv_split3_supported(D.M, D.e[k], D.IH >> k, D.IW >> k, D.e[k + 1]);
}
static inline bool dec_s3(const WmDims& D, int k) {
  const int lvl = D.N - 1 - k;  // convT k's output resolution level
  return !D.Dv && dec_cout_st(D, k) == D.cd[k + 1] &&
         op_conv_split3_supported(D.M1, D.cd[k + 1], D.IH >> lvl, D.IW >> lvl, D.cd[k]);
}

// upsampling convs on the split3 path: decoder convT k < N - 1 (forward;
// the last, 3-channel layer runs k_convT_out3) and encoder conv k >= 1's data
// gradient (an upsampling conv from e[k + 1] to e[k] channels)
static inline bool dect_s3(const WmDims& D, int k) {
  return !D.Dv && k < D.N - 1 &&
         op_convT_split3_supported(D.M1, D.cd[k], D.IH >> (D.N - k), D.IW >> (D.N - k), D.cd[k + 1], D.terms);
}
static inline bool encg_s3(const WmDims& D, int k) {
  return !D.Dv && k >= 1 &&
         op_convT_split3_supported(D.M, D.e[k + 1], D.IH >> (k + 1), D.IW >> (k + 1), D.e[k], D.terms);
}

// conv / convT weight gradient: f32-accurate split3 kernel where the shape
// allows (conv_split.hip), else the f32 MFMA kernel (wmconv.hip)
static size_t wgrad_ws_floats(int n, int h, int w, int ca, int cb) {
  size_t f = op_conv_wgrad_ws_floats(n, h, w, ca, cb);
  if (op_wgrad_split3_supported(n, h, w, ca, cb, 1)) f = std::max(f, op_wgrad_split3_ws_floats(n, h, w, ca, cb));
  return f;
}
// lo_silu: lo holds pre-activations, SiLU applied on load (the f32 kernel only)
static int wgrad(int n, int h, int w, int ca, int cb, const float* lo, int lda, const float* hi, int ldb, float* dw,
                 int cbo, float* ws, size_t ws_floats, hipStream_t s, int terms, int lo_silu = 0) {
  if (!lo_silu && op_wgrad_split3_supported(n, h, w, ca, cb, terms))
    return op_wgrad_split3(n, h, w, ca, cb, lo, lda, hi, ldb, dw, cbo, 1.0f, 0, ws, ws_floats, s, terms);
  return op_conv_wgrad(n, h, w, ca, cb, lo, lda, lo_silu, hi, ldb, dw, cbo, 1.0f, 0, ws, ws_floats, s);
}

static void mlp_bwd_carve(Carve& c, long long M1, int w1, int w2, MlpBwd& b) {
  b.gx2 = c.f(M1 * w2); b.gp2 = c.f(M1 * w2); b.gy2 = c.f(M1 * w2); b.xh2 = c.f(M1 * w2);
  b.gx1 = c.f(M1 * w1); b.gp1 = c.f(M1 * w1); b.gy1 = c.f(M1 * w1); b.xh1 = c.f(M1 * w1);
}

static long long wm_conv_scratch(const WmDims& D) {
  if (D.Dv) return 0;  // vector observations: no convolution planes
  const int n = D.M, n1 = D.M1, N = D.N;
  long long m = 0;
  auto mx = [&](long long v) { if (v > m) m = v; };
  for (int k = 0; k < N; ++k) {
    // encoder conv k: lo = output grad (res k + 1), hi = input; its bias sum
    mx(wgrad_ws_floats(n, D.IH >> (k + 1), D.IW >> (k + 1), D.e[k + 1], enc_cin_st(D, k)));
    mx(op_chan_sum_ws_floats((long long)n * D.pix[k + 1], D.e[k + 1]));
    // decoder convT k: lo = input (res N - k), hi = output grad; its bias sum
    mx(wgrad_ws_floats(n1, D.IH >> (N - k), D.IW >> (N - k), D.cd[k], dec_cout_st(D, k)));
    mx(op_chan_sum_ws_floats((long long)n1 * D.pix[N - k - 1], D.cd[k + 1]));
  }
  return m;
}

static void wm_carve(Carve& c, const dr_dims* d, const WmDims& D, WmWs& w) {
  memset(&w, 0, sizeof(w));
  const long long M = D.M, M1 = D.M1, B = D.B;
  const int L = D.L, Hd = D.Hd, A = D.A, eh = D.eh, N = D.N;
  const long long Dv = D.Dv;
  w.x0 = c.f(Dv ? M * Dv : M * D.pix[0] * 4);
  w.s3m0 = c.raw(op_nt_split3_ws_bytes(eh, Hd));
  w.s3whh = c.raw(op_nt_split3_ws_bytes(3 * Hd, Hd));
  w.s3wtb = c.raw(op_nt_split3_ws_bytes(L, 3 * Hd));
  for (int i = 0; i < 3; ++i) {
    w.pl_h3[i] = c.raw(op_nt_split3_ws_bytes(std::max(D.ph1, std::max(D.rh1, D.ch1)),
                                             std::max(D.ph2, std::max(D.rh2, D.ch2))));
    w.pl_h0[i] = c.raw(op_nt_split3_ws_bytes(Hd + L, std::max(D.ph1, std::max(D.rh1, D.ch1))));
  }
  w.pl_h6 = c.raw(op_nt_split3_ws_bytes(D.ph2, L));
  if (!Dv) {
    w.pl_up3 = c.raw(op_nt_split3_ws_bytes(D.dh, D.Fd));
    w.pl_up0 = c.raw(op_nt_split3_ws_bytes(Hd + L, D.dh));
  }
  w.pl_w0tp = c.raw(op_nt_split3_ws_bytes(D.F, eh));
  {
    const int h1 = std::max(D.ph1, std::max(D.rh1, std::max(D.ch1, D.dh)));
    const int h2 = std::max(D.ph2, std::max(D.rh2, D.ch2));
    for (int i = 0; i < 4; ++i) w.pl_f0[i] = c.raw(op_nt_split3_ws_bytes(h1, Hd + L));
    for (int i = 0; i < 3; ++i) w.pl_f3[i] = c.raw(op_nt_split3_ws_bytes(h2, h1));
    w.pl_f6 = c.raw(op_nt_split3_ws_bytes(L, D.ph2));
    if (!Dv) w.pl_fup3 = c.raw(op_nt_split3_ws_bytes(D.Fd, D.dh));
  }
  w.pl_map0f = c.raw(op_nt_split3_ws_bytes(eh, D.F));
  w.s3twhh = c.raw(op_nt_split3_ws_bytes(Hd, 3 * Hd));
  if (Dv) {  // MLP stand-in: layer 0 and the last layer of the conv slots, [M][F] each
    w.pre[0] = c.f(M * D.F); w.a[0] = c.f(M * D.F);
    w.pre[N - 1] = c.f(M * D.F); w.a[N - 1] = c.f(M * D.F);
  } else {
    for (int k = 0; k < N; ++k) {
      w.pre[k] = c.f(M * D.pix[k + 1] * D.e[k + 1]);
      w.a[k] = c.f(M * D.pix[k + 1] * D.e[k + 1]);
    }
  }
  w.feat = c.f(M * eh);
  for (int k = 0; k < N; ++k) {
    w.wr[k] = c.f((long long)D.e[k + 1] * 16 * enc_cin_st(D, k));
    if (k > 0) w.wqe[k] = c.f((long long)16 * D.e[k + 1] * D.e[k]);
  }
  w.act_tm = c.f(M * A); w.rew_tm = c.f(M); w.cont_tm = c.f(M);
  w.zeros = c.f(B * (L + A + Hd));
  w.h_all = c.f(M * Hd); w.z_all = c.f(M * L); w.soft = c.f(M * L); w.plog = c.f(M * L);
  w.pre_m = c.f(M * eh); w.x_m = c.f(M * eh);
  w.sr = c.f(M * Hd); w.su = c.f(M * Hd); w.sn = c.f(M * Hd); w.sghn = c.f(M * Hd);
  w.gi = c.f(B * 3 * Hd); w.gh = c.f(B * 3 * Hd);
  w.wt = c.f((long long)(L + A) * 3 * Hd);
  w.idx = c.i((long long)D.T * 2 * B * d->rows);
  w.pp1 = c.f(M1 * D.ph1); w.px1 = c.f(M1 * D.ph1); w.pp2 = c.f(M1 * D.ph2); w.px2 = c.f(M1 * D.ph2);
  w.prior_lg = c.f(M1 * L);
  w.rp1 = c.f(M1 * D.rh1); w.rx1 = c.f(M1 * D.rh1); w.rp2 = c.f(M1 * D.rh2); w.rx2 = c.f(M1 * D.rh2);
  w.rew_lg = c.f(M1 * D.nb);
  w.cp1 = c.f(M1 * D.ch1); w.cx1 = c.f(M1 * D.ch1); w.cp2 = c.f(M1 * D.ch2); w.cx2 = c.f(M1 * D.ch2);
  w.cont_lg = c.f(M1);
  w.du1 = c.f(M1 * D.dh); w.dx1 = c.f(M1 * D.dh); w.du2 = c.f(M1 * D.Fd); w.du2p = c.f(M1 * D.Fd);
  if (Dv) {  // dq[0] / dqp[0] = image_builder.0 pre / post SiLU [M1][Fd], dq[1] = the output mu [M1][Dv]
    w.dq[0] = c.f(M1 * D.Fd); w.dqp[0] = c.f(M1 * D.Fd); w.dq[1] = c.f(M1 * Dv);
    w.dgq[0] = c.f(M1 * D.Fd);
  } else {
    for (int k = 0; k + 1 < N; ++k) {  // convT k output at resolution level N - k - 1
      const long long sz = M1 * D.pix[N - k - 1] * D.cd[k + 1];
      // the last layer's input is never stored post-SiLU: its two readers (the
      // fused tanh-MSE layer, its weight gradient) apply SiLU on load -- the
      // 32-channel activation (B = 256: 470 MB) written once less
      w.dq[k] = c.f(sz); w.dqp[k] = k == N - 2 ? nullptr : c.f(sz); w.dgq[k] = c.f(sz);
    }
  }
  w.dgout = c.f(Dv ? M1 * Dv : M1 * D.pix[0] * 4);
  w.w3p = c.f((long long)D.Fd * D.dh); w.b3p = c.f(D.Fd);
  for (int k = 0; k < N; ++k) {
    w.wqd[k] = c.f((long long)16 * D.cd[k] * D.cd[k + 1]);
    w.wrd[k] = c.f((long long)16 * D.cd[k] * dec_cout_st(D, k));
  }
  for (int k = 0; k < N; ++k) {  // 3 bf16 planes = 1.5 floats per weight
    w.s3e[k] = enc_s3(D, k) ? c.f((3LL * 16 * D.e[k] * D.e[k + 1] + 1) / 2) : nullptr;
    w.s3d[k] = dec_s3(D, k) ? c.f((3LL * 16 * D.cd[k] * D.cd[k + 1] + 1) / 2) : nullptr;
    w.t3d[k] = dect_s3(D, k) ? c.f((3LL * 16 * D.cd[k] * D.cd[k + 1] + 1) / 2) : nullptr;
    w.t3e[k] = encg_s3(D, k) ? c.f((3LL * 16 * D.e[k] * D.e[k + 1] + 1) / 2) : nullptr;
  }
  w.coef_row = c.f(M1); w.coef_obs = c.f(M1);
  w.obs_part = c.f(Dv ? M1 : M1 * op_convT_mse_parts(D.IH / 2, D.IW / 2));
  // the last decoder layer's bias-gradient partials (k_convT_out3), 3 per tile
  w.obs_bpart = Dv ? nullptr : c.f(3LL * M1 * op_convT_mse_parts(D.IH / 2, D.IW / 2));
  w.csp = Dv ? nullptr : c.f(((long long)M1 * (D.IH / 2) * (D.IW / 2) + 127) / 128 * D.cd[N - 1]);
  w.kl_grp = c.f(M1 * d->rows); w.rew_row = c.f(M1); w.cont_row = c.f(M1); w.scal = c.f(8); w.stats = c.f(8);
  w.gH = c.f(M * Hd); w.gZ = c.f(M * L); w.glog = c.f(M * L); w.gpost = c.f(M1 * L);
  w.g_prior = c.f(M1 * L); w.g_rew = c.f(M1 * D.nb); w.g_cont = c.f(M1);
  mlp_bwd_carve(c, M1, D.ph1, D.ph2, w.bp);
  mlp_bwd_carve(c, M1, D.rh1, D.rh2, w.br);
  mlp_bwd_carve(c, M1, D.ch1, D.ch2, w.bc);
  w.gxu = c.f(M1 * D.dh); w.gpu = c.f(M1 * D.dh); w.gyu = c.f(M1 * D.dh); w.xhu = c.f(M1 * D.dh);
  w.dgu2 = c.f(M1 * D.Fd);
  w.dw3p = c.f((long long)D.Fd * D.dh); w.db3p = c.f(D.Fd);
  w.ggi = c.f(M * 3 * Hd); w.ggh = c.f(M * 3 * Hd);
  w.gpre_m = c.f(M * eh); w.gy_m = c.f(M * eh); w.xh_m = c.f(M * eh);
  w.gx_s = c.f(B * eh); w.gh_dummy = c.f(B * Hd);
  if (Dv) {
    w.gp[0] = c.f(M * D.F); w.gp[N - 1] = c.f(M * D.F);
  } else {
    for (int k = 0; k < N; ++k) w.gp[k] = c.f(M * D.pix[k + 1] * D.e[k + 1]);
  }
  w.t_pl6 = c.f((long long)L * D.ph2); w.t_pl3 = c.f((long long)D.ph2 * D.ph1); w.t_pl0 = c.f((long long)D.ph1 * Hd);
  w.t_rl6 = c.f((long long)D.nb * D.rh2); w.t_rl3 = c.f((long long)D.rh2 * D.rh1);
  w.t_rl0 = c.f((long long)D.rh1 * (Hd + L));
  w.t_cl6 = c.f(D.ch2); w.t_cl3 = c.f((long long)D.ch2 * D.ch1); w.t_cl0 = c.f((long long)D.ch1 * (Hd + L));
  w.t_up3 = c.f((long long)D.Fd * D.dh); w.t_up0 = c.f((long long)D.dh * (Hd + L));
  w.t_map3 = c.f((long long)L * eh); w.t_map0 = c.f((long long)eh * (D.F + Hd));
  w.t_whh = c.f((long long)3 * Hd * Hd); w.w0tp = c.f((long long)D.F * eh);
  w.e12w1 = D.Dv ? nullptr : c.raw((size_t)D.e[1] * 64 * 6);
  w.cws_n = wm_conv_scratch(D);
  w.cws = c.f(w.cws_n);
  {
    const long long hd = D.Hd, L = D.L, eh = D.eh;
    long long mx = splitk_floats(1, L * eh + eh * (D.F + hd) + 3 * hd * (L + D.A) + 3 * hd * hd);
    mx = std::max(mx, splitk_floats(1, (long long)D.Fd * D.dh + (long long)D.dh * (hd + L)));
    mx = std::max(mx, splitk_floats(M, std::max(eh, (long long)D.dh)));
    // the forward heads' four first Linears, each with its own slice (split-K
    // of their K = Hd + L products on the split3 tall GEMM)
    mx = std::max(mx, splitk_floats(D.M1, (long long)D.ph1 + D.rh1 + D.ch1 + D.dh));
    mx = std::max(mx, splitk_floats(1, (long long)D.nb * D.rh2 + (long long)D.rh2 * D.rh1 + D.rh1 * (hd + L)));
    w.sk_n = mx;
    w.sk = c.f(w.sk_n);
  }
  {
    // split3 TN scratch: room for four of the largest weight-gradient problem
    // over K = M rows (tn_launch groups up to four per launch)
    const int hd = D.Hd, L = D.L, eh = D.eh;
    const int mn[][2] = {{D.nb, D.rh2}, {D.rh2, D.rh1}, {D.rh1, hd + L}, {1, D.ch2}, {D.ch2, D.ch1}, {D.ch1, hd + L},
                         {L, D.ph2}, {D.ph2, D.ph1}, {D.ph1, hd + L}, {D.Fd, D.dh}, {D.dh, hd + L}, {L, eh},
                         {eh, D.F + hd}, {3 * hd, L + D.A}, {3 * hd, hd}, {D.Dv, D.Fd}, {D.Fd, D.Fd}, {D.F, D.F},
                         {D.F, D.Dv}};
    size_t mx = 0;
    for (const auto& q : mn)
      if (q[0] > 0 && q[1] > 0) mx = std::max(mx, op_gemm_tn_split3_ws_bytes(q[0], q[1], M));
    w.tn_bytes = tn_group_bytes(mx, 4);
    w.tn = c.raw(w.tn_bytes);
  }
}

extern "C" size_t dr_wm_train_workspace_bytes(const dr_dims* d, int B, int T) {
  if (!d || B <= 0 || T < 2) return 0;
  Carve c(nullptr);
  WmWs w;
  wm_carve(c, d, wm_dims(d, B, T), w);
  return c.off;
}

// input-gradient + weight-gradient pass of one head MLP (Linear-LN-SiLU x2 +
// Linear) over M1 rows whose input is [h | z] (in_z = 0: h only).  Adds the
// input gradient into gH/gZ rows t >= 1.
static int head_bwd(const WmDims& D, const dr_mlp3& m, const dr_mlp3& g, int w1, int w2, int nout, const float* glog,
                    const float* t6, const float* t3, const float* t0, const float* x1, const float* x2,
                    const float* pre1, const float* pre2, int in_z, const float* hB, const float* zB, float* gHB,
                    float* gZB, MlpBwd& b, float* sk, long long sk_n, void* tn, size_t tn_bytes, hipStream_t s,
                    void* pl6 = nullptr, void* pl3 = nullptr, void* pl0 = nullptr) {
  const int terms = D.terms;
  const int M1 = D.M1, Hd = D.Hd, L = D.L;
  const int n0 = in_z ? Hd + L : Hd;
  // tall (>= 1024 rows): the input-gradient products on split3 planes of the
  // transposed weights, split here (the weights change every step)
  const bool tall = M1 >= 1024;
  if (!tall) pl6 = pl3 = pl0 = nullptr;
  if (nout % 4) pl6 = nullptr;
  if (pl6) DR_TRY(op_nt_repack_split3(w2, nout, t6, nout, pl6, s));
  if (pl3) DR_TRY(op_nt_repack_split3(w1, w2, t3, w2, pl3, s));
  if (pl0) DR_TRY(op_nt_repack_split3(n0, w1, t0, w1, pl0, s));
  {
    GemmArgs g6 = bwd_nt(M1, w2, nout, glog, nout, t6, b.gx2, w2, 0);
    wplanes(g6, pl6);
    DR_TRY(run(G_NT, AM_PLAIN, g6, s));
  }
  DR_TRY(lnbwd_nt(M1, w1, w2, b.gx2, w2, pre2, w2, m.n4, t3, b.gx1, w1, 0, b.gp2, w2, b.gy2, b.xh2, nullptr, 0,
                  INT_MAX, s, nullptr, pl3, sk, sk_n));
  DR_TRY(lnbwd_nt(M1, n0, w1, b.gx1, w1, pre1, w1, m.n1, t0, gHB, Hd, 1, b.gp1, w1, b.gy1, b.xh1,
                  in_z ? gZB : nullptr, L, in_z ? Hd : INT_MAX, s, nullptr, pl0, sk, sk_n));
  GemmArgs p[3];
  p[0] = bwd_w(nout, w2, M1, glog, nout, x2, w2, g.l6.w);
  p[1] = bwd_w(w2, w1, M1, b.gp2, w2, x1, w1, g.l3.w);
  p[2] = bwd_w(w1, in_z ? Hd + L : Hd, M1, b.gp1, w1, hB, Hd, g.l0.w);
  if (in_z) {
    p[2].W2 = zB; p[2].ldb2 = L; p[2].nsplitB = Hd;
  }
  splitk_all(p, 3, sk, sk_n);
  DR_TRY(tn_launch(p, 3, tn, tn_bytes, s, terms));
  ColsumJob cj[7] = {
      {nout, glog, nout, nullptr, 0, g.l6.b}, {w2, b.gp2, w2, nullptr, 0, g.l3.b},
      {w2, b.gy2, w2, b.xh2, w2, g.n4.w},     {w2, b.gy2, w2, nullptr, 0, g.n4.b},
      {w1, b.gp1, w1, nullptr, 0, g.l0.b},    {w1, b.gy1, w1, b.xh1, w1, g.n1.w},
      {w1, b.gy1, w1, nullptr, 0, g.n1.b},
  };
  return op_colsum_multi(M1, cj, 7, s);
}

static int wm_run(int phases, const dr_dims* d, const dr_world_model* wm, const dr_decoder* dec, int B, int T,
                  const dr_frames* src, const dr_wm_batch* bt, dr_noise noise, dr_wm_loss_cfg cfg, float* stats,
                  int rows_global, float* losses, int* skip, const dr_world_model* gw, const dr_decoder* gd,
                  float* hiddens_out, float* latents_out, float* post_logits_out, void* ws, size_t ws_bytes,
                  hipStream_t s) {
  DR_REQUIRE(d && wm && dec && src && bt && losses && gw && gd && stats && B > 0 && T >= 2, "null argument or T < 2");
  DR_REQUIRE(bt->actions && bt->rewards && bt->continues, "window actions / rewards / continues required");
  DR_REQUIRE(vae_depth_ok(d), "enc_depth must be 0, 4 or 5");
  DR_REQUIRE(d->obs_dim > 0 || (d->img_h % (1 << vae_depth(d)) == 0 && d->img_w % (1 << vae_depth(d)) == 0),
             "image size must be a multiple of 2^depth (16, or 32 for the 5-layer VAE)");
  DR_REQUIRE(d->enc_f1 % 8 == 0 && d->enc_f2 % 8 == 0 && d->dec_f1 % 8 == 0 && d->dec_f2 % 8 == 0,
             "encoder / decoder filter counts must be multiples of 8");
  DR_REQUIRE(d->cols <= 64, "latent classes must be <= 64");
  DR_REQUIRE(d->obs_dim == 0 || d->obs_dim % 4 == 0, "vector observations: obs_dim % 4 == 0 required");
  const WmDims D = wm_dims(d, B, T);
  // the NT products that take the tile route stay f32 in both modes (on the
  // bf16 tile GEMM in bf16 mode they saved 0.1 ms but raised the posterior
  // flips 1.7e-4 -> 1.7e-3, r04p)
  GemmBf16Scope bf16_scope(false);
  const bool vec = D.Dv > 0;
  const int Dv = D.Dv;
  Carve c(ws);
  WmWs w;
  wm_carve(c, d, D, w);
  WS_CHECK(c, ws_bytes);
  const int M = D.M, M1 = D.M1, L = D.L, Hd = D.Hd, A = D.A, eh = D.eh, nb = D.nb, F = D.F, R = d->rows;
  const int IH = D.IH, IW = D.IW, N = D.N;
  const float* hB = w.h_all + (long long)B * Hd;
  const float* zB = w.z_all + (long long)B * L;
  float* gHB = w.gH + (long long)B * Hd;
  float* gZB = w.gZ + (long long)B * L;

  const int* cin_t = D.cd;       // convT k: cd[k] -> cd[k + 1] channels
  const int* cout_t = D.cd + 1;
  if (rows_global <= 0) rows_global = M1;
  if (phases & DR_WM_PREP) {
  // ---- weights: repacks, transposes, permutations (fixed for the call) ----
  if (!vec) {
  // (the f32 layouts only for the layers without split planes: each repack is
  // a ~5 us launch, 13 of them per step unused, r04zd)
  for (int k = 0; k < N; ++k) {
    if (!w.s3e[k]) DR_TRY(op_conv_repack_pad(D.e[k + 1], D.e[k], enc_cin_st(D, k), wm->conv[k].w, w.wr[k], s));
    // Conv2d data gradient = upsampling conv with the weight read as [cin=co][cout=ci]
    if (k > 0 && !w.t3e[k]) DR_TRY(op_convT_repack(D.e[k + 1], D.e[k], wm->conv[k].w, w.wqe[k], s));
  }
  for (int k = 0; k < N; ++k) {
    if (k < N - 1) {
      if (!w.t3d[k]) DR_TRY(op_convT_repack(cin_t[k], cout_t[k], dec->convt[k].w, w.wqd[k], s));
    } else {
      DR_TRY(op_convT_out3_repack(cin_t[k], dec->convt[k].w, w.wqd[k], s));
    }
    // ConvTranspose2d data gradient = strided Conv2d with the weight read as [out=ci][in=co]
    if (!w.s3d[k]) DR_TRY(op_conv_repack_pad(cin_t[k], cout_t[k], dec_cout_st(D, k), dec->convt[k].w, w.wrd[k], s));
  }
  for (int k = 0; k < N; ++k) {
    if (w.s3e[k]) DR_TRY(op_conv_repack_split3(D.e[k + 1], D.e[k], wm->conv[k].w, w.s3e[k], s));
    if (w.s3d[k]) DR_TRY(op_conv_repack_split3(cin_t[k], cout_t[k], dec->convt[k].w, w.s3d[k], s));
    if (w.t3d[k]) DR_TRY(op_convT_repack_split3(cin_t[k], cout_t[k], dec->convt[k].w, w.t3d[k], s));
    if (w.t3e[k]) DR_TRY(op_convT_repack_split3(D.e[k + 1], D.e[k], wm->conv[k].w, w.t3e[k], s));
  }
  }  // !vec
  // decoder.upscaler.3 rows to NHWC order (vector mode: Pf = 1, the identity), so its output is the first convT's NHWC input
  DR_TRY(perm_rows(D.C0, D.Pf, D.dh, dec->up3.w, w.w3p, 1, s));
  DR_TRY(perm_rows(D.C0, D.Pf, 1, dec->up3.b, w.b3p, 1, s));
  {
    TransposeJob tj[10] = {
        {L, D.ph2, L, wm->prior.l6.w, w.t_pl6},          {D.ph2, D.ph1, D.ph2, wm->prior.l3.w, w.t_pl3},
        {D.ph1, Hd, D.ph1, wm->prior.l0.w, w.t_pl0},     {nb, D.rh2, nb, wm->reward.l6.w, w.t_rl6},
        {D.rh2, D.rh1, D.rh2, wm->reward.l3.w, w.t_rl3}, {D.rh1, Hd + L, D.rh1, wm->reward.l0.w, w.t_rl0},
        {1, D.ch2, 1, wm->cont.l6.w, w.t_cl6},           {D.ch2, D.ch1, D.ch2, wm->cont.l3.w, w.t_cl3},
        {D.ch1, Hd + L, D.ch1, wm->cont.l0.w, w.t_cl0},  {3 * Hd, L + A, 3 * Hd, wm->w_ih, w.wt},
    };
    DR_TRY(op_transpose_multi(tj, 10, s));
    TransposeJob tj2[5] = {
        {D.Fd, D.dh, D.Fd, w.w3p, w.t_up3},          {D.dh, Hd + L, D.dh, dec->up0.w, w.t_up0},
        {L, eh, L, wm->map3.w, w.t_map3},            {eh, F + Hd, eh, wm->map0.w, w.t_map0},
        {3 * Hd, Hd, 3 * Hd, wm->w_hh, w.t_whh},
    };
    DR_TRY(op_transpose_multi(tj2, 5, s));
  }
  // latent_mapper.0 feature rows (of its transpose) to NHWC: dL/d conv4-out comes out NHWC
  DR_TRY(perm_rows(D.e[N], D.Pf, eh, w.t_map0, w.w0tp, 1, s));

  // ---- window data ----
  hipLaunchKernelGGL(k_wm_gather, dim3(blocks(M, 256)), dim3(256), 0, s, B, T, A, *bt, w.act_tm, w.rew_tm, w.cont_tm);
  DR_TRY(dr_check_launch("wm_gather"));
  DR_TRY(zero(w.zeros, (long long)B * (L + A + Hd), s));
  hipLaunchKernelGGL(k_wm_masksum, dim3(1), dim3(256), 0, s, M1, w.cont_tm, stats);
  DR_TRY(dr_check_launch("wm_masksum"));
  }  // DR_WM_PREP

  if (phases & DR_WM_FWD) {
  hipLaunchKernelGGL(k_wm_coef, dim3(1), dim3(256), 0, s, M1, w.cont_tm, cfg.beta_pred, stats, w.scal, w.coef_row,
                     w.coef_obs);
  DR_TRY(dr_check_launch("wm_coef"));

  // ---- encoder over all M frames (VAE.py:57-75), activations kept ----
  float* aL = w.a[N - 1];  // the flattened features (NCHW; vector mode: the MLP's last activation)
  if (vec) {  // MLP stand-in: pre[0] = X W1^T + b1, a[0] = SiLU, pre[N-1] = a[0] W2^T + b2, a[N-1] = SiLU
    DR_TRY(op_vec_gather(M, B, Dv, src, w.x0, s));
    DR_TRY(run(G_NT, AM_PLAIN, lin(M, F, Dv, w.x0, Dv, wm->conv[0].w, Dv, wm->conv[0].b, w.pre[0], F), s));
    hipLaunchKernelGGL(k_silu, dim3(blocks((long long)M * F, 256)), dim3(256), 0, s, (long long)M * F, w.pre[0], w.a[0]);
    DR_TRY(dr_check_launch("silu"));
    DR_TRY(run(G_NT, AM_PLAIN, lin(M, F, F, w.a[0], F, wm->conv[1].w, F, wm->conv[1].b, w.pre[N - 1], F), s));
    hipLaunchKernelGGL(k_silu, dim3(blocks((long long)M * F, 256)), dim3(256), 0, s, (long long)M * F, w.pre[N - 1], aL);
    DR_TRY(dr_check_launch("silu"));
  } else {
  // (conv1's weight gradient reads it; pad channel = 1: its bias gradient comes
  // out of the same product, enc_bias_fused below)
  DR_TRY(op_frames_nhwc4(M, B, IH, IW, src, w.x0, s, 1.0f));
  // conv1 + conv2 in one kernel from the u8 ring (k_enc12_split3) with the
  // backward's saves; other shapes / sources take the per-layer kernels
  int k0 = 0;
  if (N >= 2 && w.e12w1 && w.s3e[1]) {
    // DR_E_INVALID: shape / source not covered (per-layer kernels below); any
    // other failure (a launch or occupancy query) is returned
    const int rc12 = op_enc12_split3_ex(M, B, IH, IW, D.e[1], D.e[2], src, wm->conv[0].w, wm->conv[0].b,
                                        wm->conv[1].w, wm->conv[1].b, w.e12w1, w.s3e[1], w.a[1], w.pre[0], w.a[0],
                                        w.pre[1], s, D.terms);
    if (rc12 == DR_OK) k0 = 2;
    else if (rc12 != DR_E_INVALID) return rc12;
  }
  for (int k = k0; k < N; ++k) {
    if (w.s3e[k])
      DR_TRY(op_conv_split3_ex(M, D.e[k], IH >> k, IW >> k, D.e[k + 1], w.a[k - 1], w.s3e[k], wm->conv[k].b, w.a[k],
                               k == N - 1 ? 1 : 0, w.pre[k], CONV_EPI_FWD, s, D.terms));
    else
      DR_TRY(op_conv_nhwc_ex(M, enc_cin_st(D, k), IH >> k, IW >> k, D.e[k + 1], k ? w.a[k - 1] : w.x0, w.wr[k],
                             wm->conv[k].b, w.a[k], k == N - 1 ? 1 : 0, w.pre[k], CONV_EPI_FWD, s));
  }
  }
  {
    GemmArgs g = lin(M, eh, F, aL, F, wm->map0.w, F + Hd, wm->map0.b, w.feat, eh);
    splitk_all(&g, 1, w.sk, w.sk_n);
    if (M >= 1024) {  // the feature projection on split3 planes (as the epoch's warm-start encoder)
      DR_TRY(op_nt_repack_split3(eh, F, wm->map0.w, F + Hd, w.pl_map0f, s));
      wplanes(g, w.pl_map0f);
    }
    DR_TRY(run(G_NT, AM_PLAIN, g, s));
  }

  // ---- posterior scan (unroll_model, WorldModel.py:97-107) ----
  const long long idx_stride = 2LL * B * R;
  // B >= 128 (split GRU): the next step's hidden product h W_hh^T + b_hh rides
  // in the same grouped launch as latent_mapper.0 (both read only h_t)
  bool gh_pre = false;
  // B >= 128: the grouped per-step products on the split3 wave-K kernel from
  // weight planes split once per step (f32-accurate): 12.8 us per launch against
  // the f32 k_gemm_wk's 23.5 (WM step bf16 9.22 -> 9.17 ms, fp32 unchanged, r06m)
  // (bf16 mode keeps the six products here: one-term scan products measured
  // 8.46 -> 8.36 ms per bf16 WM step but took the posterior flip fraction against
  // the fp32 oracle from ~2e-4 to 1.8e-3 of its 2e-3 bound, profiles/r06z9_ab_wm_scan_one_term.txt)
  const bool planes = B >= 128 && T > 1 && Hd % 8 == 0;
  if (planes) {
    DR_TRY(split_planes(eh, Hd, wm->map0.w + F, F + Hd, w.s3m0, s));
    DR_TRY(split_planes(3 * Hd, Hd, wm->w_hh, Hd, w.s3whh, s));
  }
  for (int t = 0; t < T; ++t) {
    const long long rb = (long long)t * B;
    float* h_t = w.h_all + rb * Hd;
    float* z_t = w.z_all + rb * L;
    if (t == 0) {  // GRU from z = 0, a = 0, h = 0
      DR_TRY(gru_step(d, wm, B, w.zeros, L, w.zeros + (long long)B * L, A, w.zeros + (long long)B * (L + A), Hd, h_t,
                      Hd, w.gi, w.gh, w.sr, w.su, w.sn, w.sghn, s));
    } else {
      DR_TRY(gru_onehot(d, wm, B, w.idx + (t - 1) * idx_stride, w.act_tm + (rb - B) * A, A, h_t - (long long)B * Hd,
                        Hd, h_t, Hd, w.wt, w.sr + rb * Hd, w.su + rb * Hd, w.sn + rb * Hd, w.sghn + rb * Hd, s,
                        nullptr, 0, w.gh, gh_pre));
    }
    GemmArgs g[2];
    g[0] = lin(B, eh, Hd, h_t, Hd, wm->map0.w + F, F + Hd, nullptr, w.pre_m + rb * eh, eh);
    g[0].addend = w.feat + rb * eh;
    g[0].ld_add = eh;
    gh_pre = B >= 128 && t + 1 < T;
    if (gh_pre) g[1] = lin(B, 3 * Hd, Hd, h_t, Hd, wm->w_hh, Hd, wm->b_hh, w.gh, 3 * Hd);
    if (planes) {
      wplanes(g[0], w.s3m0);
      if (gh_pre) wplanes(g[1], w.s3whh);
    }
    DR_TRY(gemm_launch(G_NT, AM_PLAIN, g, gh_pre ? 2 : 1, s));
    GemmArgs gp = lin_ln(B, L, eh, w.pre_m + rb * eh, eh, wm->map1, wm->map3.w, wm->map3.b, w.plog + rb * L, L);
    gp.a_out = w.x_m + rb * eh;
    gp.ld_aout = eh;
    with_sampler(gp, d, noise, t, z_t, L, w.idx + t * idx_stride, w.soft + rb * L, L);
    DR_TRY(run(G_NT, AM_LNSILU, gp, s));
  }

  // ---- heads on rows t >= 1 (WorldModel.py:116-119) ----
  {
    GemmArgs p[4];
    p[0] = lin(M1, D.ph1, Hd, hB, Hd, wm->prior.l0.w, Hd, wm->prior.l0.b, w.pp1, D.ph1);
    p[1] = lin2(M1, D.rh1, hB, Hd, Hd, zB, L, L, wm->reward.l0.w, wm->reward.l0.b, w.rp1, D.rh1);
    p[2] = lin2(M1, D.ch1, hB, Hd, Hd, zB, L, L, wm->cont.l0.w, wm->cont.l0.b, w.cp1, D.ch1);
    p[3] = lin2(M1, D.dh, hB, Hd, Hd, zB, L, L, dec->up0.w, dec->up0.b, w.du1, D.dh);
    if (M1 >= 1024) {  // tall: on split3 planes of the weights (gemm.hip s3_tall_ok), split per step
      DR_TRY(op_nt_repack_split3(D.ph1, Hd, wm->prior.l0.w, Hd, w.pl_f0[0], s));
      DR_TRY(op_nt_repack_split3(D.rh1, Hd + L, wm->reward.l0.w, Hd + L, w.pl_f0[1], s));
      DR_TRY(op_nt_repack_split3(D.ch1, Hd + L, wm->cont.l0.w, Hd + L, w.pl_f0[2], s));
      DR_TRY(op_nt_repack_split3(D.dh, Hd + L, dec->up0.w, Hd + L, w.pl_f0[3], s));
      for (int i = 0; i < 4; ++i) wplanes(p[i], w.pl_f0[i]);
      splitk_all(p, 4, w.sk, w.sk_n);
    }
    DR_TRY(gemm_launch(G_NT, AM_PLAIN, p, 4, s));
  }
  {
    GemmArgs p[3];
    p[0] = lin_ln(M1, D.ph2, D.ph1, w.pp1, D.ph1, wm->prior.n1, wm->prior.l3.w, wm->prior.l3.b, w.pp2, D.ph2);
    p[0].a_out = w.px1; p[0].ld_aout = D.ph1;
    p[1] = lin_ln(M1, D.rh2, D.rh1, w.rp1, D.rh1, wm->reward.n1, wm->reward.l3.w, wm->reward.l3.b, w.rp2, D.rh2);
    p[1].a_out = w.rx1; p[1].ld_aout = D.rh1;
    p[2] = lin_ln(M1, D.ch2, D.ch1, w.cp1, D.ch1, wm->cont.n1, wm->cont.l3.w, wm->cont.l3.b, w.cp2, D.ch2);
    p[2].a_out = w.cx1; p[2].ld_aout = D.ch1;
    if (M1 >= 1024) {
      DR_TRY(op_nt_repack_split3(D.ph2, D.ph1, wm->prior.l3.w, D.ph1, w.pl_f3[0], s));
      DR_TRY(op_nt_repack_split3(D.rh2, D.rh1, wm->reward.l3.w, D.rh1, w.pl_f3[1], s));
      DR_TRY(op_nt_repack_split3(D.ch2, D.ch1, wm->cont.l3.w, D.ch1, w.pl_f3[2], s));
      for (int i = 0; i < 3; ++i) wplanes(p[i], w.pl_f3[i]);
    }
    DR_TRY(gemm_launch(G_NT, AM_LNSILU, p, 3, s));
  }
  {
    GemmArgs p[3];
    p[0] = lin_ln(M1, L, D.ph2, w.pp2, D.ph2, wm->prior.n4, wm->prior.l6.w, wm->prior.l6.b, w.prior_lg, L);
    p[0].a_out = w.px2; p[0].ld_aout = D.ph2;
    p[1] = lin_ln(M1, nb, D.rh2, w.rp2, D.rh2, wm->reward.n4, wm->reward.l6.w, wm->reward.l6.b, w.rew_lg, nb);
    p[1].a_out = w.rx2; p[1].ld_aout = D.rh2;
    p[2] = lin_ln(M1, 1, D.ch2, w.cp2, D.ch2, wm->cont.n4, wm->cont.l6.w, wm->cont.l6.b, w.cont_lg, 1);
    p[2].a_out = w.cx2; p[2].ld_aout = D.ch2;
    if (M1 >= 1024) {  // (the prior's 1024 outputs; the reward's 255 / continue's 1 stay on the tile kernel)
      DR_TRY(op_nt_repack_split3(L, D.ph2, wm->prior.l6.w, D.ph2, w.pl_f6, s));
      wplanes(p[0], w.pl_f6);
    }
    DR_TRY(gemm_launch(G_NT, AM_LNSILU, p, 3, s));
  }
  // decoder (VAE.py:139-161): upscaler.3 pre-activation in NHWC, SiLU applied by the consumers
  {
    GemmArgs g = lin_ln(M1, D.Fd, D.dh, w.du1, D.dh, dec->up1, w.w3p, w.b3p, w.du2, D.Fd);
    g.a_out = w.dx1; g.ld_aout = D.dh;
    if (M1 >= 1024 && !vec) {
      DR_TRY(op_nt_repack_split3(D.Fd, D.dh, w.w3p, D.dh, w.pl_fup3, s));
      wplanes(g, w.pl_fup3);
    }
    DR_TRY(run(G_NT, AM_LNSILU, g, s));
  }
  if (vec) {
    // image_builder stand-in: q = SiLU(du2) Wd1^T + bd1, mu = SiLU(q) Wd2^T + bd2; squared error vs rows t >= 1
    const long long MF = (long long)M1 * D.Fd;
    hipLaunchKernelGGL(k_silu, dim3(blocks(MF, 256)), dim3(256), 0, s, MF, w.du2, w.du2p);
    DR_TRY(dr_check_launch("silu"));
    DR_TRY(run(G_NT, AM_PLAIN, lin(M1, D.Fd, D.Fd, w.du2p, D.Fd, dec->convt[0].w, D.Fd, dec->convt[0].b, w.dq[0], D.Fd), s));
    hipLaunchKernelGGL(k_silu, dim3(blocks(MF, 256)), dim3(256), 0, s, MF, w.dq[0], w.dqp[0]);
    DR_TRY(dr_check_launch("silu"));
    DR_TRY(run(G_NT, AM_PLAIN, lin(M1, Dv, D.Fd, w.dqp[0], D.Fd, dec->convt[1].w, D.Fd, dec->convt[1].b, w.dq[1], Dv), s));
    hipLaunchKernelGGL(k_vec_mse, dim3(blocks(M1, 4)), dim3(256), 0, s, M1, Dv, w.dq[1], w.x0 + (long long)B * Dv,
                       w.coef_obs, w.dgout, w.obs_part);
    DR_TRY(dr_check_launch("vec_mse"));
  } else {
    hipLaunchKernelGGL(k_silu, dim3(blocks((long long)M1 * D.Fd, 256)), dim3(256), 0, s, (long long)M1 * D.Fd,
                       w.du2, w.du2p);
    DR_TRY(dr_check_launch("silu"));
    for (int k = 0; k < N; ++k) {
      ConvTArgs a = {};
      a.n = M1; a.cin = cin_t[k]; a.h = IH >> (N - k); a.w = IW >> (N - k); a.cout = cout_t[k];
      a.in = k ? w.dqp[k - 1] : w.du2p; a.silu_in = 0; a.wq = w.wqd[k]; a.bias = dec->convt[k].b;
      if (k == N - 1 && k > 0) {  // SiLU of the pre-activations on load (dqp[N - 2] is not stored)
        a.in = w.dq[k - 1];
        a.silu_in = 1;
      }
      if (k < N - 1) {
        a.out = w.dq[k]; a.out2 = w.dqp[k]; a.ldc = cout_t[k];
        if (w.t3d[k]) DR_TRY(op_convT_split3(CT_EPI_BIAS, a, w.t3d[k], s, D.terms));
        else DR_TRY(op_convT_nhwc(CT_EPI_BIAS, a, s));
      } else {
        // Tanh + squared error against frames t >= 1 (WorldModel.py:129); writes dL/d(pre-tanh)
        a.out = w.dgout; a.ldc = 4;
        a.target = w.x0 + (long long)B * D.pix[0] * 4; a.tstride = 4;
        a.coef = w.coef_obs; a.part = w.obs_part; a.bpart = w.obs_bpart;
        DR_TRY(op_convT_nhwc(CT_EPI_TANH_MSE, a, s));
      }
    }
  }

  // ---- losses ----
  {
    const int W = pow2_ge(d->cols);
    const long long th = (long long)M1 * R * W;
    const float* post1 = w.plog + (long long)B * L;
    hipLaunchKernelGGL(k_wm_kl<0>, dim3(blocks(th, 256)), dim3(256), 0, s, M1, R, d->cols, W, w.prior_lg, post1,
                       w.cont_tm, w.scal, w.kl_grp, nullptr, nullptr);
    DR_TRY(dr_check_launch("wm_kl"));
    hipLaunchKernelGGL(k_wm_heads, dim3(blocks(M1, 4)), dim3(256), 0, s, M1, nb, w.rew_lg, w.cont_lg, w.rew_tm,
                       w.cont_tm, wm->buckets_rew, w.coef_row, w.rew_row, w.cont_row, w.g_rew, w.g_cont);
    DR_TRY(dr_check_launch("wm_heads"));
    hipLaunchKernelGGL(k_wm_stats, dim3(1), dim3(256), 0, s, M1, R, vec ? 1 : op_convT_mse_parts(IH / 2, IW / 2), w.obs_part,
                       w.rew_row, w.cont_row, w.kl_grp, w.cont_tm, stats);
    DR_TRY(dr_check_launch("wm_stats"));
  }
  if (hiddens_out) DR_TRY(copy2d(hiddens_out, Hd, w.h_all, Hd, Hd, M, s));
  if (latents_out) DR_TRY(copy2d(latents_out, L, w.z_all, L, L, M, s));
  if (post_logits_out) DR_TRY(copy2d(post_logits_out, L, w.plog, L, L, M, s));
  }  // DR_WM_FWD

  const bool bwd_heads = (phases & (DR_WM_BWD | DR_WM_BWD_HEADS)) != 0;
  const bool bwd_scan = (phases & (DR_WM_BWD | DR_WM_BWD_SCAN)) != 0;
  const bool bwd_enc = (phases & (DR_WM_BWD | DR_WM_BWD_ENC)) != 0;
  if (!(bwd_heads || bwd_scan || bwd_enc)) return DR_OK;
  if (bwd_heads) {
  {
    const int W = pow2_ge(d->cols);
    const long long th = (long long)M1 * R * W;
    const float* post1 = w.plog + (long long)B * L;
    hipLaunchKernelGGL(k_wm_final, dim3(1), dim3(64), 0, s, stats, rows_global, cfg, w.scal, losses, skip);
    DR_TRY(dr_check_launch("wm_final"));
    hipLaunchKernelGGL(k_wm_kl<1>, dim3(blocks(th, 256)), dim3(256), 0, s, M1, R, d->cols, W, w.prior_lg, post1,
                       w.cont_tm, w.scal, nullptr, w.g_prior, w.gpost);
    DR_TRY(dr_check_launch("wm_kl_bwd"));
  }

  // ---- backward: heads (rows t >= 1) into dL/dh, dL/dz ----
  DR_TRY(zero(w.gH, (long long)M * Hd, s));
  DR_TRY(zero(w.gZ, (long long)M * L, s));
  DR_TRY(head_bwd(D, wm->prior, gw->prior, D.ph1, D.ph2, L, w.g_prior, w.t_pl6, w.t_pl3, w.t_pl0, w.px1, w.px2, w.pp1,
                  w.pp2, 0, hB, zB, gHB, gZB, w.bp, w.sk, w.sk_n, w.tn, w.tn_bytes, s, w.pl_h6, w.pl_h3[0],
                  w.pl_h0[0]));
  DR_TRY(head_bwd(D, wm->reward, gw->reward, D.rh1, D.rh2, nb, w.g_rew, w.t_rl6, w.t_rl3, w.t_rl0, w.rx1, w.rx2, w.rp1,
                  w.rp2, 1, hB, zB, gHB, gZB, w.br, w.sk, w.sk_n, w.tn, w.tn_bytes, s, nullptr, w.pl_h3[1],
                  w.pl_h0[1]));
  DR_TRY(head_bwd(D, wm->cont, gw->cont, D.ch1, D.ch2, 1, w.g_cont, w.t_cl6, w.t_cl3, w.t_cl0, w.cx1, w.cx2, w.cp1,
                  w.cp2, 1, hB, zB, gHB, gZB, w.bc, w.sk, w.sk_n, w.tn, w.tn_bytes, s, nullptr, w.pl_h3[2],
                  w.pl_h0[2]));
  // decoder: image_builder.6 .. .0 (data grads as strided convs, weight grads, bias sums)
  if (vec) {
    // image_builder stand-in backward: dgout = dL/dmu -> Wd2 / bd2 grads, dL/dq = (dgout Wd2) SiLU'(q)
    // -> Wd1 / bd1 grads, dL/d du2 = (dL/dq Wd1) SiLU'(du2)  (NN products with the weights as stored)
    const long long MF = (long long)M1 * D.Fd;
    auto nn = [&](int N, int K, const float* A, const float* Wkn, float* Y) {
      GemmArgs g = gemm_args();
      g.M = M1; g.N = N; g.K = K; g.A = A; g.lda = K; g.W = Wkn; g.ldb = N; g.Y = Y; g.ldy = N;
      return gemm_launch(G_NN, AM_PLAIN, &g, 1, s);
    };
    DR_TRY(nn(D.Fd, Dv, w.dgout, dec->convt[1].w, w.dgq[0]));
    hipLaunchKernelGGL(k_mul_dsilu, dim3(blocks(MF, 256)), dim3(256), 0, s, MF, w.dgq[0], w.dq[0]);
    DR_TRY(dr_check_launch("mul_dsilu"));
    DR_TRY(nn(D.Fd, D.Fd, w.dgq[0], dec->convt[0].w, w.dgu2));
    hipLaunchKernelGGL(k_mul_dsilu, dim3(blocks(MF, 256)), dim3(256), 0, s, MF, w.dgu2, w.du2);
    DR_TRY(dr_check_launch("mul_dsilu"));
    GemmArgs p[2];
    p[0] = bwd_w(Dv, D.Fd, M1, w.dgout, Dv, w.dqp[0], D.Fd, gd->convt[1].w);
    p[1] = bwd_w(D.Fd, D.Fd, M1, w.dgq[0], D.Fd, w.du2p, D.Fd, gd->convt[0].w);
    splitk_all(p, 2, w.sk, w.sk_n);
    DR_TRY(tn_launch(p, 2, w.tn, w.tn_bytes, s, D.terms));
    ColsumJob cj[2] = {{Dv, w.dgout, Dv, nullptr, 0, gd->convt[1].b}, {D.Fd, w.dgq[0], D.Fd, nullptr, 0, gd->convt[0].b}};
    DR_TRY(op_colsum_multi(M1, cj, 2, s));
  } else {
    bool csum_next = false;  // gout of this layer was summed per tile by the layer above's input-gradient conv
    for (int k = N - 1; k >= 0; --k) {
      const int ih = IH >> (N - 1 - k), iw = IW >> (N - 1 - k);  // output (high-res) size of convT k
      const int co = cout_t[k], co_st = dec_cout_st(D, k);
      float* gin = k ? w.dgq[k - 1] : w.dgu2;              // dL/d(pre-activation) of convT k's input
      const float* pre = k ? w.dq[k - 1] : w.du2;
      // input of convT k after SiLU; the last layer's is recomputed from dq (not stored)
      const bool post_silu = k == N - 1 && k > 0;
      const float* post = post_silu ? w.dq[k - 1] : k ? w.dqp[k - 1] : w.du2p;
      const float* gout = k < N - 1 ? w.dgq[k] : w.dgout;  // dL/d(convT k's output pre-activation)
      // the f32 4-channel input-gradient conv of the last layer also sums its
      // output per tile: the bias gradient of convT k - 1 without re-reading
      // that 0.5 GB gradient (csum_next below)
      const bool csum_here = !w.s3d[k] && k == N - 1 && k > 0;
      if (w.s3d[k])
        DR_TRY(op_conv_split3_ex(M1, co_st, ih, iw, cin_t[k], gout, w.s3d[k], nullptr, gin, 0, const_cast<float*>(pre),
                                 CONV_EPI_DSILU, s, D.terms));
      else
        DR_TRY(op_conv_nhwc_ex(M1, co_st, ih, iw, cin_t[k], gout, w.wrd[k], nullptr, gin, 0, const_cast<float*>(pre),
                               CONV_EPI_DSILU, s, csum_here ? w.csp : nullptr));
      DR_TRY(wgrad(M1, ih / 2, iw / 2, cin_t[k], co_st, post, cin_t[k], gout, co_st, gd->convt[k].w, co, w.cws, w.cws_n,
                   s, D.terms, post_silu ? 1 : 0));
      // (the per-tile partials -- 1.5e4 / 2.9e4 rows -- go through the same
      // two-pass channel sum: one workgroup per channel over them took 40-70 us)
      if (k == N - 1 && co == 3)  // the tanh-MSE layer summed its gradient per tile (k_convT_out3)
        DR_TRY(op_chan_sum((long long)M1 * op_convT_mse_parts(ih / 2, iw / 2), 3, w.obs_bpart, 3, gd->convt[k].b, 0,
                           w.cws, w.cws_n, s));
      else if (csum_next)
        DR_TRY(op_chan_sum(((long long)M1 * ih * iw + 127) / 128, co, w.csp, co, gd->convt[k].b, 0, w.cws, w.cws_n, s));
      else
        DR_TRY(op_chan_sum((long long)M1 * ih * iw, co, gout, co_st, gd->convt[k].b, 0, w.cws, w.cws_n, s));
      csum_next = csum_here;
    }
  }
  // decoder.upscaler: .3 (permuted rows) then LN-SiLU(.1) and .0 into dL/d[h | z]
  {
    GemmArgs g = bwd_nt(M1, D.dh, D.Fd, w.dgu2, D.Fd, w.t_up3, w.gxu, D.dh, 0);
    splitk_all(&g, 1, w.sk, w.sk_n);
    if (M1 >= 1024) {
      DR_TRY(op_nt_repack_split3(D.dh, D.Fd, w.t_up3, D.Fd, w.pl_up3, s));
      DR_TRY(op_nt_repack_split3(Hd + L, D.dh, w.t_up0, D.dh, w.pl_up0, s));
      wplanes(g, w.pl_up3);
    }
    DR_TRY(run(G_NT, AM_PLAIN, g, s));
  }
  DR_TRY(lnbwd_nt(M1, Hd + L, D.dh, w.gxu, D.dh, w.du1, D.dh, dec->up1, w.t_up0, gHB, Hd, 1, w.gpu, D.dh, w.gyu, w.xhu,
                  gZB, L, Hd, s, nullptr, M1 >= 1024 ? w.pl_up0 : nullptr, w.sk, w.sk_n));
  {
    GemmArgs p[2];
    p[0] = bwd_w(D.Fd, D.dh, M1, w.dgu2, D.Fd, w.dx1, D.dh, w.dw3p);
    p[1] = bwd_w(D.dh, Hd + L, M1, w.gpu, D.dh, hB, Hd, gd->up0.w);
    p[1].W2 = zB; p[1].ldb2 = L; p[1].nsplitB = Hd;
    splitk_all(p, 2, w.sk, w.sk_n);
    DR_TRY(tn_launch(p, 2, w.tn, w.tn_bytes, s, D.terms));
    ColsumJob cj[4] = {
        {D.Fd, w.dgu2, D.Fd, nullptr, 0, w.db3p},
        {D.dh, w.gpu, D.dh, nullptr, 0, gd->up0.b},
        {D.dh, w.gyu, D.dh, w.xhu, D.dh, gd->up1.w},
        {D.dh, w.gyu, D.dh, nullptr, 0, gd->up1.b},
    };
    DR_TRY(op_colsum_multi(M1, cj, 4, s));
    DR_TRY(perm_rows(D.C0, D.Pf, D.dh, w.dw3p, gd->up3.w, 0, s));
    DR_TRY(perm_rows(D.C0, D.Pf, 1, w.db3p, gd->up3.b, 0, s));
  }
  }  // bwd_heads

  if (bwd_scan) {
  // ---- backward through the posterior scan, t = T-1 .. 0 ----
  const int Wc = pow2_ge(d->cols);
  // B >= 128: the per-step input-gradient products (K = 3 Hd) on the split3
  // wave-K kernel from weight planes split once per step (the f32 wave-K
  // kernel took 30.7 us per grouped launch at B = 256)
  const bool bplanes = B >= 128 && T > 1 && (3 * Hd) % 8 == 0;
  if (bplanes) {
    DR_TRY(split_planes(L, 3 * Hd, w.wt, 3 * Hd, w.s3wtb, s));
    DR_TRY(split_planes(Hd, 3 * Hd, w.t_whh, 3 * Hd, w.s3twhh, s));
  }
  for (int t = T - 1; t >= 0; --t) {
    const long long rb = (long long)t * B;
    float* gH_t = w.gH + rb * Hd;
    // straight-through sampler (+ KL-rep on rows t >= 1) -> dL/d logits
    hipLaunchKernelGGL(k_ste_bwd_add, dim3(blocks((long long)B * R * Wc, 256)), dim3(256), 0, s, B, R, d->cols, Wc,
                       w.gZ + rb * L, (long long)L, w.soft + rb * L, (long long)L,
                       t > 0 ? w.gpost + (rb - B) * L : nullptr, (long long)L, w.glog + rb * L, (long long)L);
    DR_TRY(dr_check_launch("ste_bwd_add"));
    // latent_mapper.3, then LN-SiLU(.1) fused into latent_mapper.0's h-columns input gradient
    DR_TRY(run(G_NT, AM_PLAIN, bwd_nt(B, eh, L, w.glog + rb * L, L, w.t_map3, w.gx_s, eh, 0), s));
    DR_TRY(lnbwd_nt(B, Hd, eh, w.gx_s, eh, w.pre_m + rb * eh, eh, wm->map1, w.t_map0 + (long long)F * eh, gH_t, Hd, 1,
                    w.gpre_m + rb * eh, eh, w.gy_m + rb * eh, w.xh_m + rb * eh, nullptr, 0, INT_MAX, s));
    // GRU (SequenceModel.py:19-24): h_t = GRU([z_{t-1}, a_{t-1}], h_{t-1})
    const float* hprev = t > 0 ? w.h_all + (rb - B) * Hd : w.zeros + (long long)B * (L + A);
    DR_TRY(op_gru_bwd(B, Hd, gH_t, Hd, hprev, Hd, w.sr + rb * Hd, w.su + rb * Hd, w.sn + rb * Hd, w.sghn + rb * Hd,
                      w.ggi + rb * 3 * Hd, w.ggh + rb * 3 * Hd, t > 0 ? gH_t - (long long)B * Hd : w.gh_dummy, Hd,
                      t > 0 ? 1 : 0, s));
    if (t > 0) {
      GemmArgs p[2];
      p[0] = bwd_nt(B, L, 3 * Hd, w.ggi + rb * 3 * Hd, 3 * Hd, w.wt, w.gZ + (rb - B) * L, L, 1);
      p[1] = bwd_nt(B, Hd, 3 * Hd, w.ggh + rb * 3 * Hd, 3 * Hd, w.t_whh, gH_t - (long long)B * Hd, Hd, 1);
      if (bplanes) {
        wplanes(p[0], w.s3wtb);
        wplanes(p[1], w.s3twhh);
      }
      DR_TRY(gemm_launch(G_NT, AM_PLAIN, p, 2, s));
    }
  }
  // scan weight gradients over all rows
  {
    GemmArgs p[4];
    p[0] = bwd_w(L, eh, M, w.glog, L, w.x_m, eh, gw->map3.w);
    p[1] = bwd_w(eh, F + Hd, M, w.gpre_m, eh, w.a[N - 1], F, gw->map0.w);
    p[1].W2 = w.h_all; p[1].ldb2 = Hd; p[1].nsplitB = F;
    p[2] = bwd_w(3 * Hd, L + A, M1, w.ggi + (long long)B * 3 * Hd, 3 * Hd, w.z_all, L, gw->w_ih);
    p[2].W2 = w.act_tm; p[2].ldb2 = A; p[2].nsplitB = L;
    p[3] = bwd_w(3 * Hd, Hd, M1, w.ggh + (long long)B * 3 * Hd, 3 * Hd, w.h_all, Hd, gw->w_hh);
    splitk_all(p, 4, w.sk, w.sk_n);
    DR_TRY(tn_launch(p, 4, w.tn, w.tn_bytes, s, D.terms));
    ColsumJob cj[6] = {
        {L, w.glog, L, nullptr, 0, gw->map3.b},       {eh, w.gpre_m, eh, nullptr, 0, gw->map0.b},
        {eh, w.gy_m, eh, w.xh_m, eh, gw->map1.w},     {eh, w.gy_m, eh, nullptr, 0, gw->map1.b},
        {3 * Hd, w.ggi, 3 * Hd, nullptr, 0, gw->b_ih}, {3 * Hd, w.ggh, 3 * Hd, nullptr, 0, gw->b_hh},
    };
    DR_TRY(op_colsum_multi(M, cj, 6, s));
  }
  }  // bwd_scan

  if (bwd_enc) {
  // ---- backward through the encoder convolutions (all M frames) ----
  float* gL = w.gp[N - 1];  // dL/d pre[N-1], NHWC (w0tp's rows are permuted to NHWC)
  {
    GemmArgs g = bwd_nt(M, F, eh, w.gpre_m, eh, w.w0tp, gL, F, 0);
    if (M >= 1024) {
      DR_TRY(op_nt_repack_split3(F, eh, w.w0tp, eh, w.pl_w0tp, s));
      wplanes(g, w.pl_w0tp);
    }
    DR_TRY(run(G_NT, AM_PLAIN, g, s));
  }
  hipLaunchKernelGGL(k_mul_dsilu, dim3(blocks((long long)M * F, 256)), dim3(256), 0, s, (long long)M * F, gL,
                     w.pre[N - 1]);
  DR_TRY(dr_check_launch("mul_dsilu"));
  if (vec) {
    // MLP stand-in backward: W2 / b2 grads from dL/d pre[N-1], dL/d pre[0] = (gL W2) SiLU'(pre[0]), W1 / b1 grads
    GemmArgs g = gemm_args();
    g.M = M; g.N = F; g.K = F; g.A = gL; g.lda = F; g.W = wm->conv[1].w; g.ldb = F; g.Y = w.gp[0]; g.ldy = F;
    DR_TRY(gemm_launch(G_NN, AM_PLAIN, &g, 1, s));
    hipLaunchKernelGGL(k_mul_dsilu, dim3(blocks((long long)M * F, 256)), dim3(256), 0, s, (long long)M * F, w.gp[0],
                       w.pre[0]);
    DR_TRY(dr_check_launch("mul_dsilu"));
    GemmArgs p[2];
    p[0] = bwd_w(F, F, M, gL, F, w.a[0], F, gw->conv[1].w);
    p[1] = bwd_w(F, Dv, M, w.gp[0], F, w.x0, Dv, gw->conv[0].w);
    splitk_all(p, 2, w.sk, w.sk_n);
    DR_TRY(tn_launch(p, 2, w.tn, w.tn_bytes, s, D.terms));
    ColsumJob cj[2] = {{F, gL, F, nullptr, 0, gw->conv[1].b}, {F, w.gp[0], F, nullptr, 0, gw->conv[0].b}};
    DR_TRY(op_colsum_multi(M, cj, 2, s));
  } else {
    for (int k = N - 1; k >= 0; --k) {
      const int oh = IH >> (k + 1), ow = IW >> (k + 1);
      const int cin = enc_cin_st(D, k), cout = D.e[k + 1];
      const float* hi = k ? w.a[k - 1] : w.x0;  // conv k's input
      if (k == 0 && cin > D.e[0]) {
        // conv1: x0's pad channel holds 1, so the weight-gradient product's
        // pad column is the bias gradient -- the 0.5 GB gradient gp[0] is not
        // re-read by a channel-sum pass (op_conv_wgrad bias_out)
        DR_TRY(op_conv_wgrad(M, oh, ow, cout, cin, w.gp[0], cout, 0, hi, cin, gw->conv[0].w, D.e[0], 1.0f, 0, w.cws,
                             w.cws_n, s, gw->conv[0].b));
        continue;
      }
      DR_TRY(wgrad(M, oh, ow, cout, cin, w.gp[k], cout, hi, cin, gw->conv[k].w, D.e[k], w.cws, w.cws_n, s, D.terms));
      DR_TRY(op_chan_sum((long long)M * oh * ow, cout, w.gp[k], cout, gw->conv[k].b, 0, w.cws, w.cws_n, s));
      if (k > 0) {
        ConvTArgs a = {};
        a.n = M; a.cin = cout; a.h = oh; a.w = ow; a.cout = cin;
        a.in = w.gp[k]; a.wq = w.wqe[k]; a.out = w.gp[k - 1]; a.ldc = cin; a.pre = w.pre[k - 1];
        if (w.t3e[k]) DR_TRY(op_convT_split3(CT_EPI_DSILU, a, w.t3e[k], s, D.terms));
        else DR_TRY(op_convT_nhwc(CT_EPI_DSILU, a, s));
      }
    }
  }
  }  // bwd_enc

  return DR_OK;
}

extern "C" int dr_wm_train_phase(const dr_dims* d, const dr_world_model* wm, const dr_decoder* dec, int B, int T,
                                 const dr_frames* src, const dr_wm_batch* bt, dr_noise noise, dr_wm_loss_cfg cfg,
                                 int phases, float* stats, int rows_global, float* losses, int* skip,
                                 const dr_world_model* gw, const dr_decoder* gd, float* hiddens_out,
                                 float* latents_out, float* post_logits_out, void* ws, size_t ws_bytes,
                                 hipStream_t s) {
  return wm_run(phases, d, wm, dec, B, T, src, bt, noise, cfg, stats, rows_global, losses, skip, gw, gd, hiddens_out,
                latents_out, post_logits_out, ws, ws_bytes, s);
}

extern "C" int dr_wm_train_grads(const dr_dims* d, const dr_world_model* wm, const dr_decoder* dec, int B, int T,
                                 const dr_frames* src, const dr_wm_batch* bt, dr_noise noise, dr_wm_loss_cfg cfg,
                                 float* losses, int* skip, const dr_world_model* gw, const dr_decoder* gd,
                                 float* hiddens_out, float* latents_out, float* post_logits_out, void* ws,
                                 size_t ws_bytes, hipStream_t s) {
  DR_REQUIRE(d && B > 0 && T >= 2, "null argument or T < 2");
  Carve c(ws);
  WmWs w;
  wm_carve(c, d, wm_dims(d, B, T), w);
  WS_CHECK(c, ws_bytes);
  return wm_run(DR_WM_PREP | DR_WM_FWD | DR_WM_BWD, d, wm, dec, B, T, src, bt, noise, cfg, w.stats, 0, losses, skip,
                gw, gd, hiddens_out, latents_out, post_logits_out, ws, ws_bytes, s);
}

// ===========================================================================
// a20  Decoder.forward (VariationalAutoEncoder.py:139-161), inference
// ===========================================================================
struct DecWs {
  float *u1, *u2, *q[DR_MAX_DEPTH], *w3p, *b3p, *wq[DR_MAX_DEPTH];
};
static void dec_carve(Carve& c, const dr_dims* d, int M, DecWs& w) {
  memset(&w, 0, sizeof(w));
  const WmDims D = wm_dims(d, 1, 2);
  const int N = D.N;
  w.u1 = c.f((long long)M * D.dh);
  w.u2 = c.f((long long)M * D.Fd);
  if (D.Dv) {
    w.q[0] = c.f((long long)M * D.Fd);
  } else {
    for (int k = 0; k + 1 < N; ++k) w.q[k] = c.f((long long)M * D.pix[N - k - 1] * D.cd[k + 1]);
  }
  w.w3p = c.f((long long)D.Fd * D.dh);
  w.b3p = c.f(D.Fd);
  for (int k = 0; k < N; ++k) w.wq[k] = c.f((long long)16 * D.cd[k] * D.cd[k + 1]);
}

extern "C" size_t dr_decoder_workspace_bytes(const dr_dims* d, int M) {
  if (!d || M <= 0) return 0;
  Carve c(nullptr);
  DecWs w;
  dec_carve(c, d, M, w);
  return c.off;
}

extern "C" int dr_decoder_fwd(const dr_dims* d, const dr_decoder* dec, int M, const float* h, long long ldh,
                              const float* z, long long ldz, float* mu, void* ws, size_t ws_bytes, hipStream_t s) {
  DR_REQUIRE(d && dec && h && z && mu && M > 0, "null argument or empty batch");
  DR_REQUIRE(vae_depth_ok(d), "enc_depth must be 0, 4 or 5");
  DR_REQUIRE(d->obs_dim > 0 || (d->img_h % (1 << vae_depth(d)) == 0 && d->img_w % (1 << vae_depth(d)) == 0),
             "image size must be a multiple of 2^depth (16, or 32 for the 5-layer VAE)");
  DR_REQUIRE(d->dec_f1 % 8 == 0 && d->dec_f2 % 8 == 0, "decoder filter counts must be multiples of 8");
  Carve c(ws);
  DecWs w;
  dec_carve(c, d, M, w);
  WS_CHECK(c, ws_bytes);
  const WmDims D = wm_dims(d, 1, 2);
  const int* cin_t = D.cd;
  const int* cout_t = D.cd + 1;
  const int Hd = D.Hd, L = D.L, N = D.N;
  if (D.Dv) {  // vector observations: upscaler, then the image_builder MLP stand-in -> mu [M][D]
    DR_TRY(run(G_NT, AM_PLAIN, lin2(M, D.dh, h, ldh, Hd, z, ldz, L, dec->up0.w, dec->up0.b, w.u1, D.dh), s));
    GemmArgs g = lin_ln(M, D.Fd, D.dh, w.u1, D.dh, dec->up1, dec->up3.w, dec->up3.b, w.u2, D.Fd);
    g.act = 1;
    DR_TRY(run(G_NT, AM_LNSILU, g, s));
    GemmArgs g1 = lin(M, D.Fd, D.Fd, w.u2, D.Fd, dec->convt[0].w, D.Fd, dec->convt[0].b, w.q[0], D.Fd);
    g1.act = 1;
    DR_TRY(run(G_NT, AM_PLAIN, g1, s));
    return run(G_NT, AM_PLAIN, lin(M, D.Dv, D.Fd, w.q[0], D.Fd, dec->convt[1].w, D.Fd, dec->convt[1].b, mu, D.Dv), s);
  }
  DR_TRY(perm_rows(D.C0, D.Pf, D.dh, dec->up3.w, w.w3p, 1, s));
  DR_TRY(perm_rows(D.C0, D.Pf, 1, dec->up3.b, w.b3p, 1, s));
  for (int k = 0; k + 1 < N; ++k) DR_TRY(op_convT_repack(cin_t[k], cout_t[k], dec->convt[k].w, w.wq[k], s));
  DR_TRY(op_convT_out3_repack(cin_t[N - 1], dec->convt[N - 1].w, w.wq[N - 1], s));
  // upscaler: cat(h, flatten z) -> Linear -> LN -> SiLU -> Linear (rows permuted to NHWC); its SiLU runs in convT1's loader
  DR_TRY(run(G_NT, AM_PLAIN, lin2(M, D.dh, h, ldh, Hd, z, ldz, L, dec->up0.w, dec->up0.b, w.u1, D.dh), s));
  {
    GemmArgs g = lin_ln(M, D.Fd, D.dh, w.u1, D.dh, dec->up1, w.w3p, w.b3p, w.u2, D.Fd);
    g.act = 1;  // upscaler.4 SiLU
    DR_TRY(run(G_NT, AM_LNSILU, g, s));
  }
  for (int k = 0; k < N; ++k) {
    ConvTArgs a = {};
    a.n = M; a.cin = cin_t[k]; a.h = D.IH >> (N - k); a.w = D.IW >> (N - k); a.cout = cout_t[k];
    a.in = k ? w.q[k - 1] : w.u2; a.silu_in = 0; a.wq = w.wq[k]; a.bias = dec->convt[k].b;
    if (k < N - 1) {
      a.out = w.q[k]; a.silu_out = 1; a.ldc = cout_t[k];
      DR_TRY(op_convT_nhwc(CT_EPI_BIAS, a, s));
    } else {
      a.out = mu; a.ldc = 3;
      DR_TRY(op_convT_out3(a, s));
    }
  }
  return DR_OK;
}
