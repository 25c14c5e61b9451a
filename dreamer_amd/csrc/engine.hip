// Composite entry points of libdreamer_hip: encoder, posterior scan (warm
// start), imagination unroll forward/backward, critic forward/backward.
// Each is a fixed sequence of kernel launches on one stream (no host sync,
// no allocation) so a whole train_Agent epoch can be captured in a hipGraph.
#include "engine_util.h"
#include "scan.h"
#include "dream.h"
#include "bptt.h"


// fp32 mode, tall batches: the first Linear of a head over [h | z] on the
// split3 bf16 MFMA (conv_split.hip) when the workspace holds its weight planes
static bool s3_first_layer(const dr_dims* d, int M, int N, const float* h, long long ldh, const float* z,
                           long long ldz) {
  return d->precision != DR_PREC_BF16 && M >= 1024 && ldh < INT_MAX && ldz < INT_MAX &&
         op_gemm_nt_split3_supported(M, N, d->hidden + latent(d), h, (int)ldh, z, (int)ldz, d->hidden, N);
}

// ===========================================================================
// a3  encoder features
// ===========================================================================
struct EncWs {
  float *x0, *a[DR_MAX_DEPTH], *wr[DR_MAX_DEPTH], *sk;  // a[k] / wr[k]: conv k's output / repacked weight
  long long sk_n;
  void* wproj;  // bf16 mode: latent_mapper.0 feature columns as bf16 [enc_hidden][F]
  void* s3proj;  // fp32 mode: the same columns as split3 bf16 planes (op_nt_repack_split3)
  float* s3part;  // fp32 mode: split-K partial sums of the projection
  size_t s3part_n;
};

// bf16 mode stores activations / repacked weights as bf16 (2 bytes): the same
// carve with half-size regions (the last a[] holds the NCHW flatten, x0 is unused)
static void enc_carve(Carve& c, const dr_dims* d, int n, EncWs& w) {
  memset(&w, 0, sizeof(w));
  if (d->obs_dim > 0) {  // vector observations: X [n][D], two MLP activations [n][F] (a[0], a[1])
    const int F = enc_feat_dim(d);
    w.x0 = c.f((long long)n * d->obs_dim);
    w.a[0] = c.f((long long)n * F);
    w.a[1] = c.f((long long)n * F);
    w.sk_n = splitk_floats(n, d->enc_hidden);
    w.sk = c.f(w.sk_n);
    return;
  }
  const bool bf = d->precision == DR_PREC_BF16;
  int e[DR_MAX_DEPTH + 1];
  const int N = enc_chans(d, e);
  const long long p0 = (long long)d->img_h * d->img_w;
  auto act = [&](long long elems) { return bf ? (float*)c.raw(elems * 2) : c.f(elems); };
  w.sk_n = bf ? 0 : splitk_floats(n, d->enc_hidden);
  w.sk = bf ? nullptr : c.f(w.sk_n);
  w.x0 = bf ? nullptr : c.f((long long)n * p0 * 4);
  for (int k = 0; k < N; ++k) w.a[k] = act((long long)n * (p0 >> (2 * (k + 1))) * e[k + 1]);
  // conv1 weights: f32 [cout][64] (k_conv1_frames) or three bf16 planes
  // (k_enc12_split3, both modes; the bf16 repack of k_enc12_bf16 fits in it)
  w.wr[0] = (float*)c.raw((size_t)e[1] * 64 * 6);
  // conv2..N weights as three bf16 planes (op_conv_repack_split3, 6 bytes per
  // weight; the f32 / bf16 repacks of the fallbacks fit in the same slot)
  for (int k = 1; k < N; ++k) w.wr[k] = (float*)c.raw((long long)e[k + 1] * e[k] * 16 * 6);
  w.wproj = bf ? c.raw((size_t)d->enc_hidden * enc_feat_dim(d) * 2) : nullptr;
  w.s3proj = bf ? nullptr : c.raw(op_nt_split3_ws_bytes(d->enc_hidden, enc_feat_dim(d)));
  w.s3part_n = bf ? op_gemm_nt_glds_part_floats(n, d->enc_hidden, enc_feat_dim(d))
                  : op_gemm_nt_split3_part_floats(n, d->enc_hidden);
  w.s3part = w.s3part_n ? c.f((long long)w.s3part_n) : nullptr;
}

extern "C" size_t dr_encoder_workspace_bytes(const dr_dims* d, int n_frames) {
  Carve c(nullptr);
  EncWs w;
  enc_carve(c, d, n_frames, w);
  return c.off;
}

// bf16 perf mode (conv_bf16.hip): conv1 straight from the frames (fused with
// conv2 where the shape allows), conv3..N as bf16 NHWC implicit GEMMs, the
// feature projection as a bf16 NT GEMM
static int encoder_bf16(const dr_dims* d, const dr_world_model* wm, const dr_frames* src, int B, int n, float* feat,
                        const EncWs& w, hipStream_t s) {
  int e[DR_MAX_DEPTH + 1];
  const int N = enc_chans(d, e);
  const int h0 = d->img_h, w0 = d->img_w;
  const int F = enc_feat_dim(d);
  // the weight preparation of the fast path (conv1 + conv2 planes, conv3..N
  // planes, the projection's bf16 copy) as ONE launch
  const bool e12 = N >= 2 && op_enc12_split3_ok(n, h0, w0, e[1], e[2], src) && !((uintptr_t)w.a[1] & 15);
  RepackJob rj[DR_RJ_MAX];
  int nj = 0;
  if (e12) {
    rj[nj++] = rj_conv1(e[1], wm->conv[0].w, w.wr[0]);
    rj[nj++] = rj_conv(e[2], e[1], wm->conv[1].w, w.wr[1]);
  }
  bool s3[DR_MAX_DEPTH + 1] = {};
  for (int k = 2; k < N; ++k) {
    s3[k] = op_conv_split3_supported(n, e[k], h0 >> k, w0 >> k, e[k + 1]) && nj < DR_RJ_MAX - 1;
    if (s3[k]) rj[nj++] = rj_conv(e[k + 1], e[k], wm->conv[k].w, w.wr[k]);
    else DR_TRY(op_conv_repack_bf16(e[k + 1], e[k], e[k], wm->conv[k].w, w.wr[k], s));
  }
  rj[nj++] = rj_bf16(d->enc_hidden, F, wm->map0.w, F + d->hidden, w.wproj);
  DR_TRY(op_repack_multi(rj, nj, s));
  // conv1 + conv2: k_enc12_split3 with one term (64 x 64 from the u8 ring), else
  // k_enc12_bf16, else two launches
  // (DR_E_INVALID = shape / source not covered: next form; any other failure is returned)
  const int rc_s1 = e12 ? op_enc12_s1_bf16(n, B, h0, w0, e[1], e[2], src, wm->conv[0].w, wm->conv[0].b, wm->conv[1].w,
                                           wm->conv[1].b, w.wr[0], w.wr[1], w.a[1], s, 1)
                        : DR_E_INVALID;
  if (rc_s1 != DR_OK) {
    if (rc_s1 != DR_E_INVALID) return rc_s1;
    DR_TRY(op_conv_repack_bf16(e[1], 3, 4, wm->conv[0].w, w.wr[0], s));
    DR_TRY(op_conv_repack_bf16(e[2], e[1], e[1], wm->conv[1].w, w.wr[1], s));
    const int rc_b = op_enc12_bf16(n, B, h0, w0, e[1], e[2], src, w.wr[0], wm->conv[0].b, w.wr[1], wm->conv[1].b,
                                   w.a[1], s);
    if (rc_b != DR_OK) {
      if (rc_b != DR_E_INVALID) return rc_b;
      DR_TRY(op_conv1_bf16(n, B, h0, w0, e[1], src, w.wr[0], wm->conv[0].b, w.a[0], s));
      DR_TRY(op_conv_bf16(n, e[1], h0 / 2, w0 / 2, e[2], w.a[0], w.wr[1], wm->conv[1].b, w.a[1], 0, s));
    }
  }
  for (int k = 2; k < N; ++k) {
    // the split-conv tiling with one bf16 term where the shape allows, else k_conv_bf16
    if (s3[k]) {
      DR_TRY(op_conv_s1_bf16(n, e[k], h0 >> k, w0 >> k, e[k + 1], w.a[k - 1], w.wr[k], wm->conv[k].b, w.a[k],
                             k == N - 1 ? 1 : 0, s));
    } else {
      DR_TRY(op_conv_bf16(n, e[k], h0 >> k, w0 >> k, e[k + 1], w.a[k - 1], w.wr[k], wm->conv[k].b, w.a[k],
                          k == N - 1 ? 1 : 0, s));
    }
  }
  // the projection on the LDS-DMA bf16 GEMM with split-K where it tiles (conv_glds.hip), else k_conv_bf16
  const int rcp = op_gemm_nt_glds_bf16(n, d->enc_hidden, F, w.a[N - 1], F, w.wproj, F, wm->map0.b, feat, d->enc_hidden,
                                       w.s3part, w.s3part_n, s);
  if (rcp != DR_E_INVALID) return rcp;
  return op_gemm_nt_bf16(n, d->enc_hidden, F, w.a[N - 1], F, w.wproj, wm->map0.b, feat, d->enc_hidden, s);
}

extern "C" int dr_encoder_features(const dr_dims* d, const dr_world_model* wm, const dr_frames* src, int B, int T,
                                   float* feat, void* ws, size_t ws_bytes, hipStream_t s) {
  DR_REQUIRE(d && wm && src && feat && B > 0 && T > 0, "null argument or empty batch");
  DR_REQUIRE(vae_depth_ok(d), "enc_depth must be 0, 4 or 5");
  if (d->obs_dim > 0) {
    // vector observations (dr_dims.obs_dim): Linear-SiLU x2, then the feature
    // columns of latent_mapper.0 -- the MLP stand-in for VAE.py:57-75's convs
    DR_REQUIRE(d->enc_f2 > 0 && d->obs_dim % 4 == 0, "vector observations: obs_dim % 4 == 0 required");
    const int n = B * T, F = enc_feat_dim(d), D = d->obs_dim;
    Carve c(ws);
    EncWs w;
    enc_carve(c, d, n, w);
    WS_CHECK(c, ws_bytes);
    DR_TRY(op_vec_gather(n, B, D, src, w.x0, s));
    GemmArgs g1 = lin(n, F, D, w.x0, D, wm->conv[0].w, D, wm->conv[0].b, w.a[0], F);
    g1.act = 1;
    DR_TRY(run(G_NT, AM_PLAIN, g1, s));
    GemmArgs g2 = lin(n, F, F, w.a[0], F, wm->conv[1].w, F, wm->conv[1].b, w.a[1], F);
    g2.act = 1;
    DR_TRY(run(G_NT, AM_PLAIN, g2, s));
    GemmArgs gp = lin(n, d->enc_hidden, F, w.a[1], F, wm->map0.w, F + d->hidden, wm->map0.b, feat, d->enc_hidden);
    float* sk = w.sk;
    long long skn = w.sk_n;
    give_splitk(gp, sk, skn);
    return run(G_NT, AM_PLAIN, gp, s);
  }
  int e[DR_MAX_DEPTH + 1];
  const int N = enc_chans(d, e);
  DR_REQUIRE(d->img_h % (1 << N) == 0 && d->img_w % (1 << N) == 0,
             "image size must be a multiple of 2^depth (16, or 32 for the 5-layer encoder)");
  DR_REQUIRE(d->enc_f1 % 4 == 0 && d->enc_f2 % 4 == 0, "encoder filter counts must be multiples of 4");
  DR_REQUIRE(d->precision == DR_PREC_FP32 || d->precision == DR_PREC_BF16, "precision must be DR_PREC_FP32/BF16");
  const int n = B * T;
  Carve c(ws);
  EncWs w;
  enc_carve(c, d, n, w);
  WS_CHECK(c, ws_bytes);
  if (d->precision == DR_PREC_BF16) return encoder_bf16(d, wm, src, B, n, feat, w, s);
  const int h0 = d->img_h, w0 = d->img_w;
  const int F = enc_feat_dim(d);
  // the weight preparation of the fast path (conv1 + conv2 planes, conv3..N
  // planes, the projection's planes) as ONE launch
  const bool e12 = N >= 2 && op_enc12_split3_ok(n, h0, w0, e[1], e[2], src);
  const bool s3p = w.s3proj && n >= 1024 &&
                   op_gemm_nt_split3_supported(n, d->enc_hidden, F, w.a[N - 1], F, nullptr, 0, F, d->enc_hidden);
  RepackJob rj[DR_RJ_MAX];
  int nj = 0;
  if (e12) {
    rj[nj++] = rj_conv1(e[1], wm->conv[0].w, w.wr[0]);
    rj[nj++] = rj_conv(e[2], e[1], wm->conv[1].w, w.wr[1]);
  }
  bool s3[DR_MAX_DEPTH + 1] = {};
  for (int k = e12 ? 2 : 1; k < N; ++k) {
    s3[k] = op_conv_split3_supported(n, e[k], h0 >> k, w0 >> k, e[k + 1]) && nj < DR_RJ_MAX - 1;
    if (s3[k]) rj[nj++] = rj_conv(e[k + 1], e[k], wm->conv[k].w, w.wr[k]);
  }
  if (s3p) rj[nj++] = rj_nt(d->enc_hidden, F, wm->map0.w, F + d->hidden, w.s3proj);
  DR_TRY(op_repack_multi(rj, nj, s));
  // conv1 + conv2 in one launch from the u8 ring (conv_split.hip) where the
  // shape allows; else the first conv straight from the frames (u8 ring or
  // f32), and shapes that does not tile through the normalised NHWC4 copy
  int k0 = 1;
  const int rc12 = e12 ? op_enc12_split3(n, B, h0, w0, e[1], e[2], src, wm->conv[0].w, wm->conv[0].b, wm->conv[1].w,
                                         wm->conv[1].b, w.wr[0], w.wr[1], w.a[1], s, 1)
                       : DR_E_INVALID;
  if (rc12 == DR_OK) {
    k0 = 2;
  } else {
    if (rc12 != DR_E_INVALID) return rc12;
    DR_TRY(op_conv_repack_pad(e[1], 3, 4, wm->conv[0].w, w.wr[0], s));
    if (op_conv1_frames(n, B, h0, w0, e[1], src, w.wr[0], wm->conv[0].b, w.a[0], s) != DR_OK) {
      DR_TRY(op_frames_nhwc4(n, B, h0, w0, src, w.x0, s));
      DR_TRY(op_conv_nhwc(n, 4, h0, w0, e[1], w.x0, w.wr[0], wm->conv[0].b, w.a[0], 0, s));
    }
  }
  // conv2..N: NHWC implicit GEMMs, f32-accurate on the bf16 MFMA (3-term split,
  // conv_split.hip) where the shape tiles, else on the f32 MFMA; the last layer
  // in NCHW == nn.Flatten order of Encoder.forward (VAE.py:72)
  for (int k = k0; k < N; ++k) {
    const int cin = e[k], cout = e[k + 1], hin = h0 >> k, win = w0 >> k, last = k == N - 1;
    const float* cw = wm->conv[k].w;
    const float* cb = wm->conv[k].b;
    if (s3[k]) {
      DR_TRY(op_conv_split3(n, cin, hin, win, cout, w.a[k - 1], w.wr[k], cb, w.a[k], last, s));
    } else {
      DR_TRY(op_conv_repack_pad(cout, cin, cin, cw, w.wr[k], s));
      DR_TRY(op_conv_nhwc(n, cin, hin, win, cout, w.a[k - 1], w.wr[k], cb, w.a[k], last, s));
    }
  }
  if (s3p) {
    // latent_mapper.0's feature columns (VAE.py:57-75 -> WorldModel.py) on the split3 bf16 MFMA
    // K split by K alone (32 chunks of 32 per split, at most 8): the frames
    // of a window step get the same sums whether the window is encoded whole
    // or in time chunks (engine.py's overlapped warm start)
    const int ksplits = std::max(1, std::min(8, (F + 1023) / 1024));
    return op_gemm_nt_split3_sk(n, d->enc_hidden, F, w.a[N - 1], F, nullptr, 0, F, w.s3proj, wm->map0.b, 0, feat,
                                d->enc_hidden, w.s3part, w.s3part_n, s, ksplits);
  }
  GemmArgs gp = lin(n, d->enc_hidden, F, w.a[N - 1], F, wm->map0.w, F + d->hidden, wm->map0.b, feat, d->enc_hidden);
  float* sk = w.sk;
  long long skn = w.sk_n;
  give_splitk(gp, sk, skn);
  return run(G_NT, AM_PLAIN, gp, s);
}

// ===========================================================================
// a2/a5  posterior scan
// ===========================================================================
struct ObsWs {
  float *gi, *gh, *pre1, *logits, *wt, *hb[2];
  unsigned short* hb16[2];  // bf16 mode: hb[] rounded to bf16 by the gates kernel (k_gemm_wks3's A16)
  int* idx;
  void *s3m0, *s3whh;  // bf16 planes of latent_mapper.0's h-columns and W_hh (k_gemm_wks3)
  void* ring;          // persistent scan: ring buffers + counters (scan.hip)
};
static void obs_carve(Carve& c, const dr_dims* d, int B, ObsWs& w) {
  w.ring = c.raw(op_pscan_ring_bytes(B));
  w.s3m0 = c.raw(op_nt_split3_ws_bytes(d->enc_hidden, d->hidden));
  w.s3whh = c.raw(op_nt_split3_ws_bytes(3 * d->hidden, d->hidden));
  w.gi = c.f((long long)B * 3 * d->hidden);
  w.gh = c.f((long long)B * 3 * d->hidden);
  w.pre1 = c.f((long long)B * d->enc_hidden);
  w.logits = c.f((long long)B * latent(d));
  w.wt = c.f((long long)(latent(d) + d->action) * 3 * d->hidden);
  w.hb[0] = c.f((long long)B * d->hidden);
  w.hb[1] = c.f((long long)B * d->hidden);
  w.hb16[0] = (unsigned short*)c.raw(sizeof(unsigned short) * B * d->hidden);
  w.hb16[1] = (unsigned short*)c.raw(sizeof(unsigned short) * B * d->hidden);
  w.idx = c.i(2LL * B * d->rows);
}

extern "C" size_t dr_observe_workspace_bytes(const dr_dims* d, int B) {
  Carve c(nullptr);
  ObsWs w;
  obs_carve(c, d, B, w);
  return c.off;
}

extern "C" int dr_observe_scan(const dr_dims* d, const dr_world_model* wm, int B, int T, const float* feat,
                               const float* actions, long long act_sb, long long act_st, const float* h_init,
                               const float* z_init, dr_noise noise, float* z_out, float* h_out, float* logits_out,
                               void* ws, size_t ws_bytes, hipStream_t s) {
  DR_REQUIRE(d && wm && feat && z_out && h_out && B > 0 && T > 0, "null argument or empty batch");
  GemmBf16Scope bf16_scope(d->precision == DR_PREC_BF16);
  DR_REQUIRE(T == 1 || (z_init == nullptr ? T > 1 : true), "bad T");
  DR_REQUIRE(actions || (z_init == nullptr && T == 1), "actions required");
  Carve c(ws);
  ObsWs w;
  obs_carve(c, d, B, w);
  WS_CHECK(c, ws_bytes);
  const int L = latent(d), Hd = d->hidden, eh = d->enc_hidden;
  const int F = enc_feat_dim(d);
  // W_ih^T for the one-hot gather of the fused GRU (weights are fixed for the
  // call); only needed when a GRU step runs (an encode-only call passes a
  // world model without GRU weights)
  const bool any_gru = (z_init != nullptr) || T > 1;
  if (any_gru) {
    DR_REQUIRE(wm->w_ih && wm->w_hh && wm->b_ih && wm->b_hh, "GRU weights required");
    DR_TRY(op_transpose(3 * Hd, L + d->action, wm->w_ih, w.wt, s));
  }
  // the warm start (no z_init / h_init) as ONE persistent launch (scan.hip)
  if (z_init == nullptr && h_init == nullptr && op_pscan_supported(d, B, T, d->action)) {
    const int rc = op_pscan(d, wm, B, T, d->action, feat, actions, act_sb, act_st, w.wt, wm->map0.w + F, F + Hd,
                            noise, 0, z_out, h_out, logits_out, w.ring, s);
    if (rc != DR_E_UNSUPPORTED) return rc;
  }
  const bool planes = B >= 128 && T > 1 && Hd % 8 == 0;
  if (planes) {
    DR_TRY(split_planes(eh, Hd, wm->map0.w + F, F + Hd, w.s3m0, s));
    DR_TRY(split_planes(3 * Hd, Hd, wm->w_hh, Hd, w.s3whh, s));
  }
  const float* h = h_init;  // current hidden (NULL = zeros)
  const unsigned short* h16 = nullptr;  // its bf16 copy when the gates kernel wrote one
  // bf16 mode on the weight planes: the gates kernel also writes h rounded to
  // bf16, which the grouped products read instead of rounding h themselves
  const bool a16 = planes && d->precision == DR_PREC_BF16;
  int hb = 0;
  // B >= 128 (split GRU): the next step's hidden product h W_hh^T + b_hh rides
  // in the same grouped launch as latent_mapper.0 (both read only h)
  const bool split_gru = B >= 128;
  bool gh_pre = false;
  if (z_init) {
    if (z_init != z_out) DR_TRY(copy2d(z_out, L, z_init, L, L, B, s));
    DR_TRY(op_onehot_index(B, d->rows, d->cols, z_out, L, w.idx, onehot_vals(w.idx, B, d->rows), s));
    if (split_gru && planes && h_init) {
      // a continuing chunk: the first GRU's hidden product on the same kernel
      // and planes as the grouped launch that computes it inside one call, so
      // a time-chunked scan equals the whole-window scan bit for bit
      GemmArgs gh = lin(B, 3 * Hd, Hd, h_init, Hd, wm->w_hh, Hd, wm->b_hh, w.gh, 3 * Hd);
      wplanes(gh, w.s3whh);
      DR_TRY(gemm_launch(G_NT, AM_PLAIN, &gh, 1, s));
      gh_pre = true;
    }
  }
  for (int t = 0; t < T; ++t) {
    const bool do_gru = (z_init != nullptr) || t > 0;
    if (do_gru) {
      const int ai = t - (z_init == nullptr ? 1 : 0);
      float* hn = w.hb[hb];
      unsigned short* hn16 = a16 ? w.hb16[hb] : nullptr;
      hb ^= 1;
      DR_TRY(gru_onehot(d, wm, B, w.idx, actions + ai * act_st, act_sb, h, Hd, hn, Hd, w.wt, nullptr,
                        nullptr, nullptr, nullptr, s, z_out, L, w.gh, gh_pre, hn16));
      h = hn;
      h16 = hn16;
    }
    // latent_mapper.0 on cat(features, h): feature part precomputed in feat[t]
    GemmArgs g[2];
    g[0] = lin(B, eh, h ? Hd : 0, h, Hd, wm->map0.w + F, F + Hd, nullptr, w.pre1, eh);
    g[0].addend = feat + (long long)t * B * eh;
    g[0].ld_add = eh;
    gh_pre = split_gru && h && t + 1 < T;
    if (gh_pre) {
      g[1] = lin(B, 3 * Hd, Hd, h, Hd, wm->w_hh, Hd, wm->b_hh, w.gh, 3 * Hd);
      if (planes) {
        // bf16 mode: plane 0 times bf16-rounded h (k_gemm_wks3<1>); fp32 mode: the 3-term split
        wplanes(g[0], w.s3m0);
        wplanes(g[1], w.s3whh);
        g[0].A16 = g[1].A16 = h16;
      } else {
        g[0].bf16 = g[1].bf16 = 0;  // (bf16 mode: these products stay f32)
      }
    }
    DR_TRY(gemm_launch(G_NT, AM_PLAIN, g, gh_pre ? 2 : 1, s));
    float* lg = (t == T - 1 && logits_out) ? logits_out : nullptr;
    GemmArgs gp = lin_ln(B, L, eh, w.pre1, eh, wm->map1, wm->map3.w, wm->map3.b, lg, L);
    with_sampler(gp, d, noise, t, z_out, L, w.idx, nullptr, 0);
    DR_TRY(run(G_NT, AM_LNSILU, gp, s));
  }
  if (h) DR_TRY(copy2d(h_out, Hd, h, Hd, Hd, B, s));
  else DR_TRY(zero(h_out, (long long)B * Hd, s));
  return DR_OK;
}

// ===========================================================================
// a7  imagination unroll
// ===========================================================================
struct Tape {
  float *eps, *ls_raw;                // [H][B][A], [B][H][A]
  float *pre1a, *x1a, *pre2a, *x2a;   // [B][H][ah*]
  float *r, *u, *n, *ghn;             // [H][B][hidden]
  float *pre1p, *pre2p, *soft;        // [H][B][*]
};
static void tape_carve(Carve& c, const dr_dims* d, int B, int H, Tape& t) {
  const long long BH = (long long)B * H;
  t.eps = c.f(BH * d->action);
  t.ls_raw = c.f(BH * d->action);
  t.pre1a = c.f(BH * d->actor_h1);
  t.x1a = c.f(BH * d->actor_h1);
  t.pre2a = c.f(BH * d->actor_h2);
  t.x2a = c.f(BH * d->actor_h2);
  t.r = c.f(BH * d->hidden);
  t.u = c.f(BH * d->hidden);
  t.n = c.f(BH * d->hidden);
  t.ghn = c.f(BH * d->hidden);
  t.pre1p = c.f(BH * d->prior_h1);
  t.pre2p = c.f(BH * d->prior_h2);
  t.soft = c.f(BH * latent(d));
}

extern "C" size_t dr_imagine_tape_bytes(const dr_dims* d, int B, int H) {
  Carve c(nullptr);
  Tape t;
  tape_carve(c, d, B, H, t);
  return c.off;
}

struct ImWs {
  float *gi, *gh, *plog, *p1r, *p1c, *p2r, *p2c, *rlog, *clog, *rval, *wt, *wst, *bst;  // forward scratch
  unsigned short* hid16;  // bf16 mode, launch form: hiddens rounded to bf16 by the gates kernel ([B][H+1][Hd])
  float *tl0f, *hpart;  // forward: actor Linear 0 transposed ([Hd+L][a1]), its h-part + bias [B][a1]
  void *s3r, *s3c;  // split3 weight planes of the reward / continue heads' first Linear
  void *s3p0, *s3a0, *s3whh, *s3wt, *s3twhh, *s3tl0a;  // bf16 planes of the per-step chain weights (k_gemm_wks3)
  float* s3part;    // their split-K partial sums
  size_t s3part_n;
  int* idx[2];
  // backward
  float *gH, *gZ, *gA, *glog, *gx2, *gp2, *gx1, *gp1, *ggi, *ggh, *gheads, *gx2a, *gpre2a, *gy2a, *xh2a, *gx1a,
      *gpre1a, *gy1a, *xh1a, *hcat, *zcat, *sk;
  unsigned short *ggi16, *ggh16, *gpre1a16;  // bf16 mode: bf16 copies of ggi / ggh / gpre1a (GemmArgs.A16)
  long long sk_n;
  // transposed weights for the input-gradient GEMMs (NT with float4 loads)
  float *tl6p, *tl3p, *tl0p, *twhh, *thead, *tl3a, *tl0a;
  void* tn;  // split3 TN scratch of the actor weight gradients (tn_launch)
  size_t tn_bytes;
  void* pd;  // the persistent unroll's hand-off buffers and counters (dream.hip), carved last
  void* pb;  // the persistent BPTT's (bptt.hip), after it
};
static void imws_carve(Carve& c, const dr_dims* d, int B, int H, ImWs& w) {
  const long long Bl = B, BH = (long long)B * H, B1 = (long long)B * (H + 1);
  const int L = latent(d), Hd = d->hidden, A = d->action;
  w.gi = c.f(Bl * 3 * Hd);
  w.gh = c.f(Bl * 3 * Hd);
  w.plog = c.f(Bl * L);
  // reward / continue heads, batched over all B (H + 1) imagined states after the unroll
  w.p1r = c.f(B1 * d->rew_h1);
  w.p1c = c.f(B1 * d->cont_h1);
  w.p2r = c.f(B1 * d->rew_h2);
  w.p2c = c.f(B1 * d->cont_h2);
  w.rlog = c.f(B1 * d->buckets);
  w.clog = c.f(B1);
  w.rval = c.f(B1);
  w.s3p0 = c.raw(op_nt_split3_ws_bytes(d->prior_h1, Hd));
  w.s3a0 = c.raw(op_nt_split3_ws_bytes(d->actor_h1, Hd));
  w.s3whh = c.raw(op_nt_split3_ws_bytes(3 * Hd, Hd));
  w.s3wt = c.raw(op_nt_split3_ws_bytes(L + A, 3 * Hd));
  w.s3twhh = c.raw(op_nt_split3_ws_bytes(Hd, 3 * Hd));
  w.s3tl0a = c.raw(op_nt_split3_ws_bytes(Hd + L, d->actor_h1));
  w.s3r = c.raw(op_nt_split3_ws_bytes(d->rew_h1, d->hidden + L));
  w.s3c = c.raw(op_nt_split3_ws_bytes(d->cont_h1, d->hidden + L));
  w.s3part_n = op_gemm_nt_split3_part_floats((int)B1, std::max(d->rew_h1, d->cont_h1));
  w.s3part = c.f((long long)w.s3part_n);
  w.wt = c.f((long long)(L + A) * 3 * Hd);
  w.hid16 = (unsigned short*)c.raw(sizeof(unsigned short) * Bl * (H + 1) * Hd);
  w.tl0f = c.f((long long)(Hd + L) * d->actor_h1);
  w.hpart = c.f(Bl * d->actor_h1);
  w.wst = c.f((long long)2 * A * d->actor_h2);
  w.bst = c.f((long long)2 * A);
  w.idx[0] = c.i(2 * Bl * d->rows);
  w.idx[1] = c.i(2 * Bl * d->rows);
  w.tl6p = c.f((long long)L * d->prior_h2);
  w.tl3p = c.f((long long)d->prior_h2 * d->prior_h1);
  w.tl0p = c.f((long long)d->prior_h1 * Hd);
  w.twhh = c.f((long long)3 * Hd * Hd);
  w.thead = c.f((long long)2 * A * d->actor_h2);
  w.tl3a = c.f((long long)d->actor_h2 * d->actor_h1);
  w.tl0a = c.f((long long)d->actor_h1 * (Hd + L));
  w.gH = c.f(B1 * Hd);  // gH | gZ | gA back to back: zeroed by one fill
  w.gZ = c.f(B1 * L);
  w.gA = c.f(BH * A);
  w.glog = c.f(Bl * L);
  w.gx2 = c.f(Bl * d->prior_h2);
  w.gp2 = c.f(Bl * d->prior_h2);
  w.gx1 = c.f(Bl * d->prior_h1);
  w.gp1 = c.f(Bl * d->prior_h1);
  w.ggi = c.f(Bl * 3 * Hd);
  w.ggh = c.f(Bl * 3 * Hd);
  w.ggi16 = (unsigned short*)c.raw(sizeof(unsigned short) * Bl * 3 * Hd);
  w.ggh16 = (unsigned short*)c.raw(sizeof(unsigned short) * Bl * 3 * Hd);
  w.gheads = c.f(BH * 2 * A);
  w.gx2a = c.f(Bl * d->actor_h2);
  w.gpre2a = c.f(BH * d->actor_h2);
  w.gy2a = c.f(BH * d->actor_h2);
  w.xh2a = c.f(BH * d->actor_h2);
  w.gx1a = c.f(Bl * d->actor_h1);
  w.gpre1a = c.f(BH * d->actor_h1);
  w.gpre1a16 = (unsigned short*)c.raw(sizeof(unsigned short) * BH * d->actor_h1);
  w.gy1a = c.f(BH * d->actor_h1);
  w.xh1a = c.f(BH * d->actor_h1);
  w.hcat = c.f(BH * Hd);
  w.zcat = c.f(BH * L);
  w.sk_n = splitk_floats(d->actor_h1, Hd + L) + splitk_floats(d->actor_h2, d->actor_h1) +
           2 * splitk_floats(A, d->actor_h2);
  w.sk = c.f(w.sk_n);
  const int BHi = (int)BH;
  // the four weight-gradient problems side by side (one grouped launch)
  w.tn_bytes = op_gemm_tn_split3_ws_bytes(d->actor_h1, Hd + L, BHi) +
               op_gemm_tn_split3_ws_bytes(d->actor_h2, d->actor_h1, BHi) +
               2 * op_gemm_tn_split3_ws_bytes(A, d->actor_h2, BHi);
  w.tn = c.raw(w.tn_bytes);
  w.pd = c.raw(op_pdream_ws_bytes(d, B, H));
  w.pb = c.raw(op_pbptt_ws_bytes(d, B, H));
}

extern "C" size_t dr_imagine_workspace_bytes(const dr_dims* d, int B, int H) {
  Carve c(nullptr);
  ImWs w;
  imws_carve(c, d, B, H, w);
  return c.off;
}

// the unroll as seven launches per step (shapes outside dream.hip, launch_form)
static int imagine_launch_form(const dr_dims* d, const dr_world_model* wm, const dr_actor* ac, int B, int H,
                               const dr_noise& noise, const dr_noise& nq, int deterministic, float* latents,
                               float* hiddens, float* actions, float* mus, float* sigmas, const Tape& tp, ImWs& w,
                               bool split_gru, bool zg, hipStream_t s) {
  const int L = latent(d), Hd = d->hidden, A = d->action, a1 = d->actor_h1, a2 = d->actor_h2;
  const long long ldH = (long long)(H + 1) * Hd, ldL = (long long)(H + 1) * L, ldA = (long long)H * A;
  const long long lda1 = (long long)H * a1, lda2 = (long long)H * a2;
  const bool planes = split_gru && H > 1 && Hd % 8 == 0;
  const bool a16 = planes && d->precision == DR_PREC_BF16;
  if (planes) {
    DR_TRY(split_planes(d->prior_h1, Hd, wm->prior.l0.w, Hd, w.s3p0, s));
    if (zg) DR_TRY(split_planes(a1, Hd, ac->l0.w, Hd + L, w.s3a0, s));
    DR_TRY(split_planes(3 * Hd, Hd, wm->w_hh, Hd, w.s3whh, s));
  }

  // actor at step 0 (Agent.py:191-210)
  {
    DR_TRY(run(G_NT, AM_PLAIN, lin2(B, a1, hiddens, ldH, Hd, latents, ldL, L, ac->l0.w, ac->l0.b, tp.pre1a, lda1), s));
    GemmArgs g = lin_ln(B, a2, a1, tp.pre1a, lda1, ac->n1, ac->l3.w, ac->l3.b, tp.pre2a, lda2);
    g.a_out = tp.x1a; g.ld_aout = lda1;
    DR_TRY(run(G_NT, AM_LNSILU, g, s));
  }
  DR_TRY(stack_heads(ac, A, a2, w.wst, w.bst, s));
  {
    GemmArgs h = lin_ln(B, 2 * A, a2, tp.pre2a, lda2, ac->n4, w.wst, w.bst, nullptr, 0);
    h.a_out = tp.x2a; h.ld_aout = lda2;
    with_actor_head(h, A, noise, 0, deterministic, actions, ldA, mus, ldA, sigmas, ldA, tp.eps, tp.ls_raw, ldA);
    DR_TRY(run(G_NT, AM_LNSILU, h, s));
  }
  for (int t = 0; t < H; ++t) {
    const long long hb = (long long)Hd * B * t;
    float* h_t = hiddens + (long long)t * Hd;
    float* h_n = hiddens + (long long)(t + 1) * Hd;
    float* z_t = latents + (long long)t * L;
    float* z_n = latents + (long long)(t + 1) * L;
    // WorldModel.imagine_step (WorldModel.py:72-77)
    unsigned short* h_n16 = a16 ? w.hid16 + (long long)(t + 1) * Hd : nullptr;
    DR_TRY(gru_onehot(d, wm, B, w.idx[t & 1], actions + (long long)t * A, ldA, h_t, ldH, h_n, ldH, w.wt,
                      tp.r + hb, tp.u + hb, tp.n + hb, tp.ghn + hb, s, z_t, ldL, w.gh, split_gru && t > 0, h_n16));
    float* p1 = tp.pre1p + (long long)t * B * d->prior_h1;
    float* p2 = tp.pre2p + (long long)t * B * d->prior_h2;
    {
      const bool more = t + 1 < H;
      GemmArgs p[3];
      int np = 0;
      p[np] = lin(B, d->prior_h1, Hd, h_n, ldH, wm->prior.l0.w, Hd, wm->prior.l0.b, p1, d->prior_h1);
      if (planes) wplanes(p[np], w.s3p0);
      ++np;
      if (more && zg) {
        p[np] = lin(B, a1, Hd, h_n, ldH, ac->l0.w, Hd + L, ac->l0.b, w.hpart, a1);
        if (planes) wplanes(p[np], w.s3a0);
        ++np;
      }
      if (more && split_gru) {
        p[np] = lin(B, 3 * Hd, Hd, h_n, ldH, wm->w_hh, Hd, wm->b_hh, w.gh, 3 * Hd);
        if (planes) wplanes(p[np], w.s3whh);
        ++np;
      }
      // bf16 mode: on the weight planes the products run in bf16 (k_gemm_wks3<1>),
      // else they stay f32; fp32 mode: h_{t+1}'s split3 planes from the gates kernel
      for (int i = 0; i < np; ++i) {
        if (!planes) p[i].bf16 = 0;
        p[i].A16 = h_n16;  // bf16 mode: the gates kernel's bf16 copy of h_{t+1}
      }
      DR_TRY(gemm_launch(G_NT, AM_PLAIN, p, np, s));
    }
    DR_TRY(run(G_NT, AM_LNSILU, lin_ln(B, d->prior_h2, d->prior_h1, p1, d->prior_h1, wm->prior.n1, wm->prior.l3.w,
                                       wm->prior.l3.b, p2, d->prior_h2), s));
    GemmArgs g = lin_ln(B, L, d->prior_h2, p2, d->prior_h2, wm->prior.n4, wm->prior.l6.w, wm->prior.l6.b, nullptr, 0);
    with_sampler(g, d, nq, t, z_n, ldL, w.idx[(t + 1) & 1], tp.soft + (long long)t * B * L, L);
    DR_TRY(run(G_NT, AM_LNSILU, g, s));
    // the actor for step t+1 (the reward / continue heads run once after the unroll)
    if (t + 1 < H) {
      const long long o1 = (long long)(t + 1) * a1, o2 = (long long)(t + 1) * a2, o = (long long)(t + 1) * A;
      if (zg) {
        int* ix = w.idx[(t + 1) & 1];
        DR_TRY(op_zgather_add(B, a1, d->rows, d->cols, ix, onehot_vals(ix, B, d->rows), z_n, ldL,
                              w.tl0f + (long long)Hd * a1, a1, w.hpart, a1, tp.pre1a + o1, lda1, s));
      } else {
        DR_TRY(run(G_NT, AM_PLAIN, lin2(B, a1, h_n, ldH, Hd, z_n, ldL, L, ac->l0.w, ac->l0.b, tp.pre1a + o1, lda1), s));
      }
      GemmArgs g3 = lin_ln(B, a2, a1, tp.pre1a + o1, lda1, ac->n1, ac->l3.w, ac->l3.b, tp.pre2a + o2, lda2);
      g3.a_out = tp.x1a + o1;
      g3.ld_aout = lda1;
      DR_TRY(run(G_NT, AM_LNSILU, g3, s));
      GemmArgs hd = lin_ln(B, 2 * A, a2, tp.pre2a + o2, lda2, ac->n4, w.wst, w.bst, nullptr, 0);
      hd.a_out = tp.x2a + o2;
      hd.ld_aout = lda2;
      with_actor_head(hd, A, noise, t + 1, deterministic, actions + o, ldA, mus + o, ldA, sigmas + o, ldA,
                      tp.eps + (long long)(t + 1) * B * A, tp.ls_raw + o, ldA);
      DR_TRY(run(G_NT, AM_LNSILU, hd, s));
    }
  }
  return DR_OK;
}

extern "C" int dr_imagine_fwd(const dr_dims* d, const dr_world_model* wm, const dr_actor* ac, int B, int H,
                              const float* z0, const float* h0, dr_noise noise, int deterministic, float* latents,
                              float* hiddens, float* actions, float* rewards, float* continues, float* mus,
                              float* sigmas, void* tape, void* ws, size_t ws_bytes, hipStream_t s) {
  DR_REQUIRE(d && wm && ac && z0 && h0 && latents && hiddens && actions && rewards && continues && mus && sigmas &&
                 tape && B > 0 && H > 0,
             "null argument or empty batch");
  GemmBf16Scope bf16_scope(d->precision == DR_PREC_BF16);
  Carve c(ws);
  ImWs w;
  imws_carve(c, d, B, H, w);
  WS_CHECK(c, ws_bytes);
  Carve ct(tape);
  Tape tp;
  tape_carve(ct, d, B, H, tp);
  const int L = latent(d), Hd = d->hidden, A = d->action, a1 = d->actor_h1, a2 = d->actor_h2;
  const long long ldH = (long long)(H + 1) * Hd, ldL = (long long)(H + 1) * L, ldA = (long long)H * A;
  const long long lda1 = (long long)H * a1, lda2 = (long long)H * a2;
  {
    const Copy2dJob cj[2] = {{latents, ldL, z0, L, L, B}, {hiddens, ldH, h0, Hd, Hd, B}};
    DR_TRY(op_copy2d_multi(cj, 2, s));
  }
  dr_noise nq = noise;  // Categorical draws: a Philox stream apart from the actor's
  nq.stream += 65536;
  // per-step structure: the three products that read only
  // h_{t+1} -- the prior's first Linear, the h-part of the next actor's first
  // Linear and (B >= 128, split GRU) the next GRU step's hidden product --
  // run as ONE grouped launch right after the GRU; the actor's latent part is
  // then a gather of R rows of its transposed z-columns (z is one-hot)
  const bool split_gru = B >= 128;
  const bool zg = d->rows <= 32 && a1 % 4 == 0;
  {
    TransposeJob tj[2] = {{3 * Hd, L + A, 3 * Hd, wm->w_ih, w.wt}, {a1, Hd + L, a1, ac->l0.w, w.tl0f}};
    DR_TRY(op_transpose_multi(tj, zg ? 2 : 1, s));
  }
  DR_TRY(op_onehot_index(B, d->rows, d->cols, latents, ldL, w.idx[0], onehot_vals(w.idx[0], B, d->rows), s));

  // the whole unroll as one persistent launch where the shape and the stream's
  // CUs allow it (dream.hip); the reward / continue heads below either way
  bool unrolled = false;
  if (zg && op_pdream_supported(d, B, H, A)) {
    const PDreamTape pt = {tp.eps, tp.ls_raw, tp.pre1a, tp.x1a, tp.pre2a, tp.x2a, tp.r, tp.u, tp.n, tp.ghn,
                           tp.pre1p, tp.pre2p, tp.soft};
    const int rc = op_pdream(d, wm, ac, B, H, w.wt, w.tl0f + (long long)Hd * a1, w.idx[0], noise, nq, deterministic,
                             latents, hiddens, actions, mus, sigmas, pt, w.pd, s);
    if (rc != DR_E_UNSUPPORTED && rc != DR_OK) return rc;
    unrolled = rc == DR_OK;
  }
  if (!unrolled) DR_TRY(imagine_launch_form(d, wm, ac, B, H, noise, nq, deterministic, latents, hiddens, actions, mus,
                                            sigmas, tp, w, split_gru, zg, s));

  // RewardPredictor / ContinuePredictor (DynamicsPredictors.py:64-74, 95-105)
  // on every imagined state (h_{t+1}, z_{t+1}) at once: rows m = b (H+1) + t'
  // of the contiguous [B][H+1] hiddens / latents (t' = 0 rides along unused);
  // forward only -- the actor loss takes no gradient through the heads
  {
    const int M1 = B * (H + 1);
    GemmArgs p[2];
    if (s3_first_layer(d, M1, d->rew_h1, hiddens, Hd, latents, L) &&
        s3_first_layer(d, M1, d->cont_h1, hiddens, Hd, latents, L)) {
      DR_TRY(op_nt_repack_split3(d->rew_h1, Hd + L, wm->reward.l0.w, Hd + L, w.s3r, s));
      DR_TRY(op_nt_repack_split3(d->cont_h1, Hd + L, wm->cont.l0.w, Hd + L, w.s3c, s));
      DR_TRY(op_gemm_nt_split3_sk(M1, d->rew_h1, Hd + L, hiddens, Hd, latents, L, Hd, w.s3r, wm->reward.l0.b, 0,
                                  w.p1r, d->rew_h1, w.s3part, w.s3part_n, s));
      DR_TRY(op_gemm_nt_split3_sk(M1, d->cont_h1, Hd + L, hiddens, Hd, latents, L, Hd, w.s3c, wm->cont.l0.b, 0,
                                  w.p1c, d->cont_h1, w.s3part, w.s3part_n, s));
    } else {
      p[0] = lin2(M1, d->rew_h1, hiddens, Hd, Hd, latents, L, L, wm->reward.l0.w, wm->reward.l0.b, w.p1r, d->rew_h1);
      p[1] = lin2(M1, d->cont_h1, hiddens, Hd, Hd, latents, L, L, wm->cont.l0.w, wm->cont.l0.b, w.p1c, d->cont_h1);
      DR_TRY(gemm_launch(G_NT, AM_PLAIN, p, 2, s));
    }
    p[0] = lin_ln(M1, d->buckets, d->rew_h2, w.p2r, d->rew_h2, wm->reward.n4, wm->reward.l6.w, wm->reward.l6.b, w.rlog,
                  d->buckets);
    p[1] = lin_ln(M1, 1, d->cont_h2, w.p2c, d->cont_h2, wm->cont.n4, wm->cont.l6.w, wm->cont.l6.b, w.clog, 1);
    p[1].act = 2;  // sigmoid
    if (std::max(std::max(d->rew_h1, d->rew_h2), std::max(d->cont_h1, d->cont_h2)) <= 208) {
      // LN-SiLU, Linear, LN-SiLU, Linear of both heads in one launch (k_mlp2_tail:
      // 16 rows per workgroup, the 200-wide middle layer recomputed per
      // 128-column block); the two-launch form below is the general path
      Mlp2Args m2[2];
      const float* x1[2] = {w.p1r, w.p1c};
      const dr_mlp3* hm[2] = {&wm->reward, &wm->cont};
      const int k1[2] = {d->rew_h1, d->cont_h1}, k2[2] = {d->rew_h2, d->cont_h2};
      for (int i = 0; i < 2; ++i) {
        memset(&m2[i], 0, sizeof(Mlp2Args));
        m2[i].M = M1; m2[i].K1 = k1[i]; m2[i].K2 = k2[i];
        m2[i].X = x1[i]; m2[i].ldx = k1[i];
        m2[i].ln1_g = hm[i]->n1.w; m2[i].ln1_b = hm[i]->n1.b;
        m2[i].W3 = hm[i]->l3.w; m2[i].b3 = hm[i]->l3.b;
        m2[i].ln4_g = hm[i]->n4.w; m2[i].ln4_b = hm[i]->n4.b;
        m2[i].e = p[i];
        m2[i].e.A = nullptr;
      }
      DR_TRY(mlp2_launch(m2, 2, s));
    } else {
      GemmArgs q[2];
      q[0] = lin_ln(M1, d->rew_h2, d->rew_h1, w.p1r, d->rew_h1, wm->reward.n1, wm->reward.l3.w, wm->reward.l3.b, w.p2r,
                    d->rew_h2);
      q[1] = lin_ln(M1, d->cont_h2, d->cont_h1, w.p1c, d->cont_h1, wm->cont.n1, wm->cont.l3.w, wm->cont.l3.b, w.p2c,
                    d->cont_h2);
      DR_TRY(gemm_launch(G_NT, AM_LNSILU, q, 2, s));
      DR_TRY(gemm_launch(G_NT, AM_LNSILU, p, 2, s));
    }
    DR_TRY(op_bucket_value(M1, d->buckets, w.rlog, d->buckets, wm->buckets_rew, w.rval, 1, s));
    const Copy2dJob cj[2] = {{rewards, H, w.rval + 1, H + 1, H, B}, {continues, H, w.clog + 1, H + 1, H, B}};
    DR_TRY(op_copy2d_multi(cj, 2, s));
  }
  return DR_OK;
}

// part 1 of the backward: upstream state gradients into the workspace and the
// transposed weights (independent of dL/dmus, dL/dsigmas: may run early, on
// another stream).  part 2 (main) is the reverse loop + weight gradients.
static int imagine_bwd_impl(const dr_dims* d, const dr_world_model* wm, const dr_actor* ac, int B, int H,
                            const float* latents, const float* hiddens, const float* actions,
                            const float* g_mus, const float* g_sigmas,
                            const float* g_actions, const float* g_latents, const float* g_hiddens,
                            const void* tape, const dr_actor* gr, void* ws, size_t ws_bytes, hipStream_t s,
                            bool do_prep, bool do_main);

extern "C" int dr_imagine_bwd(const dr_dims* d, const dr_world_model* wm, const dr_actor* ac, int B, int H,
                              const float* latents, const float* hiddens, const float* actions,
                              const float* g_mus, const float* g_sigmas,
                              const float* g_actions, const float* g_latents, const float* g_hiddens,
                              const void* tape, const dr_actor* gr, void* ws, size_t ws_bytes, hipStream_t s) {
  return imagine_bwd_impl(d, wm, ac, B, H, latents, hiddens, actions, g_mus, g_sigmas, g_actions, g_latents,
                          g_hiddens, tape, gr, ws, ws_bytes, s, true, true);
}

extern "C" int dr_imagine_bwd_prep(const dr_dims* d, const dr_world_model* wm, const dr_actor* ac, int B, int H,
                                   const float* g_actions, const float* g_latents, const float* g_hiddens, void* ws,
                                   size_t ws_bytes, hipStream_t s) {
  DR_REQUIRE(d && wm && ac && B > 0 && H > 0, "null argument or empty batch");
  return imagine_bwd_impl(d, wm, ac, B, H, nullptr, nullptr, nullptr, nullptr, nullptr, g_actions, g_latents,
                          g_hiddens, nullptr, nullptr, ws, ws_bytes, s, true, false);
}

extern "C" int dr_imagine_bwd_main(const dr_dims* d, const dr_world_model* wm, const dr_actor* ac, int B, int H,
                                   const float* latents, const float* hiddens, const float* actions,
                                   const float* g_mus, const float* g_sigmas, int upstream_state, const void* tape,
                                   const dr_actor* gr, void* ws, size_t ws_bytes, hipStream_t s) {
  const float* flag = upstream_state ? reinterpret_cast<const float*>(ws) : nullptr;  // non-NULL marker only
  return imagine_bwd_impl(d, wm, ac, B, H, latents, hiddens, actions, g_mus, g_sigmas, nullptr, flag, nullptr, tape,
                          gr, ws, ws_bytes, s, false, true);
}

static int imagine_bwd_impl(const dr_dims* d, const dr_world_model* wm, const dr_actor* ac, int B, int H,
                            const float* latents, const float* hiddens, const float* actions,
                            const float* g_mus, const float* g_sigmas,
                            const float* g_actions, const float* g_latents, const float* g_hiddens,
                            const void* tape, const dr_actor* gr, void* ws, size_t ws_bytes, hipStream_t s,
                            bool do_prep, bool do_main) {
  DR_REQUIRE(d && wm && ac && B > 0 && H > 0, "null argument or empty batch");
  GemmBf16Scope bf16_scope(d->precision == DR_PREC_BF16);
  DR_REQUIRE(!do_main || (latents && hiddens && actions && tape && gr), "null argument");
  Carve c(ws);
  ImWs w;
  imws_carve(c, d, B, H, w);
  WS_CHECK(c, ws_bytes);
  Carve ct((void*)tape);
  Tape tp;
  if (do_main) tape_carve(ct, d, B, H, tp);
  const int L = latent(d), Hd = d->hidden, A = d->action, a1 = d->actor_h1, a2 = d->actor_h2;
  const long long ldH = (long long)(H + 1) * Hd, ldL = (long long)(H + 1) * L, ldA = (long long)H * A;
  const long long lda1 = (long long)H * a1, lda2 = (long long)H * a2;
  const int BH = B * H;
  const bool upstream_state = g_latents || g_hiddens;
  if (do_prep) {
  // upstream gradients
  if (!g_hiddens && !g_latents && !g_actions) {
    // gH | gZ | gA are carved back to back: one fill (train_Agent's case)
    DR_TRY(zero(w.gH, (long long)((w.gA + (long long)BH * A) - w.gH), s));
  } else {
    if (g_hiddens) DR_TRY(copy2d(w.gH, Hd, g_hiddens, Hd, Hd, (long long)B * (H + 1), s));
    else DR_TRY(zero(w.gH, (long long)B * (H + 1) * Hd, s));
    if (g_latents) DR_TRY(copy2d(w.gZ, L, g_latents, L, L, (long long)B * (H + 1), s));
    else DR_TRY(zero(w.gZ, (long long)B * (H + 1) * L, s));
    if (g_actions) DR_TRY(copy2d(w.gA, A, g_actions, A, A, (long long)BH, s));
    else DR_TRY(zero(w.gA, (long long)BH * A, s));
  }
  {
    // weights are constant over the backward: transpose them once (one launch)
    // so every input-gradient GEMM below runs NT with 16-byte weight loads
    const int h1 = d->prior_h1, h2 = d->prior_h2;
    TransposeJob tj[9] = {
        {L, h2, L, wm->prior.l6.w, w.tl6p},
        {h2, h1, h2, wm->prior.l3.w, w.tl3p},
        {h1, Hd, h1, wm->prior.l0.w, w.tl0p},
        {3 * Hd, L + A, 3 * Hd, wm->w_ih, w.wt},
        {3 * Hd, Hd, 3 * Hd, wm->w_hh, w.twhh},
        {A, a2, 2 * A, ac->mu.w, w.thead},
        {A, a2, 2 * A, ac->ls.w, w.thead + A},
        {a2, a1, a2, ac->l3.w, w.tl3a},
        {a1, Hd + L, a1, ac->l0.w, w.tl0a},
    };
    DR_TRY(op_transpose_multi(tj, 9, s));
    if (B >= 128 && (3 * Hd) % 8 == 0) {
      DR_TRY(split_planes(L + A, 3 * Hd, w.wt, 3 * Hd, w.s3wt, s));
      DR_TRY(split_planes(Hd, 3 * Hd, w.twhh, 3 * Hd, w.s3twhh, s));
      if (d->actor_h1 % 8 == 0) DR_TRY(split_planes(Hd + L, d->actor_h1, w.tl0a, d->actor_h1, w.s3tl0a, s));
    }
  }
  }  // do_prep
  const bool planes = B >= 128 && (3 * Hd) % 8 == 0;
  if (!do_main) return DR_OK;

  // the reverse loop as one persistent launch where the shape and the stream's
  // CUs allow it (bptt.hip); the weight gradients below either way
  bool looped = false;
  if (op_pbptt_supported(d, B, H, A)) {
    const PBpttIO io = {w.tl6p, w.tl3p, w.tl0p, w.wt, w.twhh, w.thead, w.tl3a, w.tl0a,
                        tp.soft, tp.pre2p, tp.pre1p, tp.r, tp.u, tp.n, tp.ghn, tp.pre2a, tp.pre1a, tp.ls_raw, tp.eps,
                        hiddens, actions, g_mus, g_sigmas, w.gH, w.gZ, w.gA,
                        w.gheads, w.gpre2a, w.gy2a, w.xh2a, w.gpre1a, w.gy1a, w.xh1a};
    const int rc = op_pbptt(d, wm, ac, B, H, io, w.pb, s);
    if (rc != DR_E_UNSUPPORTED && rc != DR_OK) return rc;
    looped = rc == DR_OK;
  }
  for (int t = H - 1; t >= 0 && !looped; --t) {
    const long long hb = (long long)Hd * B * t;
    float* gH_t = w.gH + (long long)t * Hd;
    float* gH_n = w.gH + (long long)(t + 1) * Hd;
    float* gZ_t = w.gZ + (long long)t * L;
    float* gZ_n = w.gZ + (long long)(t + 1) * L;
    const bool state_grad = upstream_state || t < H - 1;
    if (state_grad) {
      // z_{t+1} = STE(prior(h_{t+1}))   (DynamicsPredictors.py:31-40)
      const int h1 = d->prior_h1, h2 = d->prior_h2;
      const int gl = d->cols / 4;
      GemmArgs gs = bwd_nt(B, h2, L, gZ_n, ldL, w.tl6p, w.gx2, h2, 0);
      if (L <= 1024 && d->cols % 4 == 0 && gl <= 64 && (gl & (gl - 1)) == 0 && gemm_bwd_rows16(&gs, 1)) {
        // straight-through softmax backward fused into the prior head's
        // input-gradient GEMM (its A-operand prologue)
        GemmArgs g = bwd_nt(B, h2, L, gZ_n, ldL, w.tl6p, w.gx2, h2, 0);
        g.pre = tp.soft + (long long)t * B * L;
        g.ld_pre = L;
        g.C = d->cols;
        DR_TRY(run(G_NT, AM_STEBWD, g, s));
      } else {
        DR_TRY(op_softmax_ste_bwd(B, d->rows, d->cols, gZ_n, ldL, tp.soft + (long long)t * B * L, L, w.glog, s));
        DR_TRY(run(G_NT, AM_PLAIN, bwd_nt(B, h2, L, w.glog, L, w.tl6p, w.gx2, h2, 0), s));
      }
      // dynamic_predictor.4/.3 and .1/.0: LN-SiLU backward fused into the next input-gradient GEMM
      DR_TRY(lnbwd_nt(B, h1, h2, w.gx2, h2, tp.pre2p + (long long)t * B * h2, h2, wm->prior.n4, w.tl3p, w.gx1, h1, 0,
                      w.gp2, h2, nullptr, nullptr, nullptr, 0, INT_MAX, s));
      // ... whose epilogue (the last addend of dL/dh_{t+1}) also runs the GRU
      // backward of h_{t+1} = GRU(z_t, a_t, h_t) (SequenceModel.py:19-24)
      GruBwdEpi ge;
      memset(&ge, 0, sizeof(ge));
      ge.h = hiddens + (long long)t * Hd; ge.ldh = ldH;
      ge.r = tp.r + hb; ge.u = tp.u + hb; ge.n = tp.n + hb; ge.ghn = tp.ghn + hb;
      ge.gi = w.ggi; ge.gh = w.ggh; ge.ho = gH_t; ge.ldo = ldH; ge.Hd = Hd;
      // bf16 mode on the weight planes: bf16 copies of the gates' gradients for
      // the input-gradient products below (GemmArgs.A16; bitwise the same)
      const bool a16 = planes && d->precision == DR_PREC_BF16;
      if (a16) {
        ge.gi16 = w.ggi16;
        ge.gh16 = w.ggh16;
      }
      DR_TRY(lnbwd_nt(B, Hd, h1, w.gx1, h1, tp.pre1p + (long long)t * B * h1, h1, wm->prior.n1, w.tl0p, gH_n, ldH, 1,
                      w.gp1, h1, nullptr, nullptr, nullptr, 0, INT_MAX, s, &ge));
      if (t > 0) {
        GemmArgs p[2];
        p[0] = bwd_nt(B, L + A, 3 * Hd, w.ggi, 3 * Hd, w.wt, gZ_t, ldL, 1);
        p[0].Y2 = w.gA + (long long)t * A; p[0].ldy2 = ldA; p[0].nsplitY = L;
        p[1] = bwd_nt(B, Hd, 3 * Hd, w.ggh, 3 * Hd, w.twhh, gH_t, ldH, 1);
        if (planes) {
          wplanes(p[0], w.s3wt);
          wplanes(p[1], w.s3twhh);
        }
        if (a16) {
          p[0].A16 = w.ggi16;
          p[1].A16 = w.ggh16;
        }
        DR_TRY(gemm_launch(G_NT, AM_PLAIN, p, 2, s));
      } else {
        // only the action gradient is consumed at t = 0
        DR_TRY(run(G_NT, AM_PLAIN, bwd_nt(B, A, 3 * Hd, w.ggi, 3 * Hd, w.wt + (long long)L * 3 * Hd, w.gA, ldA, 1), s));
      }
    }
    // actor at step t: heads, then base_net (Agent.py:191-210)
    const long long ot = (long long)t * A;
    float* gh_t = w.gheads + (long long)t * 2 * A;
    const long long o2 = (long long)t * a2, o1 = (long long)t * a1;
    // head backward + its input gradient (K = 2A) in one launch
    DR_TRY(op_actor_head_bwd_x(B, A, a2, w.gA + ot, ldA, g_mus ? g_mus + ot : nullptr,
                               g_sigmas ? g_sigmas + ot : nullptr, ldA, actions + ot, ldA, tp.ls_raw + ot, ldA,
                               tp.eps + (long long)t * B * A, gh_t, (long long)H * 2 * A, w.thead, w.gx2a, a2, s));
    // base_net.4/.3: LN-SiLU backward fused into the .3 input-gradient GEMM; the
    // prologue also writes g_pre and the LN-parameter saves for the weight grads
    DR_TRY(lnbwd_nt(B, a1, a2, w.gx2a, a2, tp.pre2a + o2, lda2, ac->n4, w.tl3a, w.gx1a, a1, 0, w.gpre2a + o2, lda2,
                    w.gy2a + o2, w.xh2a + o2, nullptr, 0, INT_MAX, s));
    if (t > 0 && planes && a1 % 8 == 0) {
      // B >= 128: the LN-SiLU backward as its own pass, then the K = a1 input
      // gradient [gH_t | gZ_t] on the wave-K split3 kernel (weight planes of
      // the transposed base_net.0, split once per call)
      const bool a16 = d->precision == DR_PREC_BF16 && lda1 % 8 == 0;
      DR_TRY(op_ln_silu_bwd(B, a1, w.gx1a, a1, tp.pre1a + o1, lda1, ac->n1.w, ac->n1.b, w.gpre1a + o1, lda1,
                            w.gy1a + o1, w.xh1a + o1, s, a16 ? w.gpre1a16 + o1 : nullptr));
      GemmArgs g = bwd_nt(B, Hd + L, a1, w.gpre1a + o1, lda1, w.tl0a, gH_t, ldH, 1);
      if (a16) g.A16 = w.gpre1a16 + o1;  // (bitwise the same one-term products)
      g.Y2 = gZ_t; g.ldy2 = ldL; g.nsplitY = Hd;
      wplanes(g, w.s3tl0a);
      DR_TRY(run(G_NT, AM_PLAIN, g, s));
    } else if (t > 0) {
      DR_TRY(lnbwd_nt(B, Hd + L, a1, w.gx1a, a1, tp.pre1a + o1, lda1, ac->n1, w.tl0a, gH_t, ldH, 1, w.gpre1a + o1,
                      lda1, w.gy1a + o1, w.xh1a + o1, gZ_t, ldL, Hd, s));
    } else {
      // step 0 feeds no state gradient: only the saves for the weight grads
      DR_TRY(op_ln_silu_bwd(B, a1, w.gx1a, a1, tp.pre1a + o1, lda1, ac->n1.w, ac->n1.b, w.gpre1a + o1, lda1,
                            w.gy1a + o1, w.xh1a + o1, s));
    }
  }
  // ---- actor weight gradients over all B*H rows (rows r = b*H + t) ----
  {
    const Copy2dJob cj[2] = {{w.hcat, (long long)H * Hd, hiddens, ldH, (long long)H * Hd, B},
                             {w.zcat, (long long)H * L, latents, ldL, (long long)H * L, B}};
    DR_TRY(op_copy2d_multi(cj, 2, s));
  }
  {
    GemmArgs p[4];
    p[0] = bwd_w(a1, Hd + L, BH, w.gpre1a, a1, w.hcat, Hd, gr->l0.w);
    p[0].W2 = w.zcat; p[0].ldb2 = L; p[0].nsplitB = Hd;
    p[1] = bwd_w(a2, a1, BH, w.gpre2a, a2, tp.x1a, a1, gr->l3.w);
    p[2] = bwd_w(A, a2, BH, w.gheads, 2 * A, tp.x2a, a2, gr->mu.w);
    p[3] = bwd_w(A, a2, BH, w.gheads + A, 2 * A, tp.x2a, a2, gr->ls.w);
    float* sk = w.sk;
    long long skn = w.sk_n;
    for (int i = 0; i < 4; ++i) give_splitk(p[i], sk, skn);
    // bf16 perf mode: one-term bf16 operands, f32 accumulation (as the WM step's)
    DR_TRY(tn_launch(p, 4, w.tn, w.tn_bytes, s, d->precision == DR_PREC_BF16 ? 1 : 3));
  }
  {
    ColsumJob cj[8] = {
        {a1, w.gpre1a, a1, nullptr, 0, gr->l0.b}, {a1, w.gy1a, a1, w.xh1a, a1, gr->n1.w},
        {a1, w.gy1a, a1, nullptr, 0, gr->n1.b},   {a2, w.gpre2a, a2, nullptr, 0, gr->l3.b},
        {a2, w.gy2a, a2, w.xh2a, a2, gr->n4.w},   {a2, w.gy2a, a2, nullptr, 0, gr->n4.b},
        {A, w.gheads, 2 * A, nullptr, 0, gr->mu.b}, {A, w.gheads + A, 2 * A, nullptr, 0, gr->ls.b},
    };
    DR_TRY(op_colsum_multi(BH, cj, 8, s));
  }
  return DR_OK;
}

// ===========================================================================
// a13  critic forward / a16 critic loss + backward
// ===========================================================================
struct CTape {
  float *pre1, *x1, *pre2, *x2, *logits;
};
static void ctape_carve(Carve& c, const dr_dims* d, int M, CTape& t) {
  t.pre1 = c.f((long long)M * d->critic_h1);
  t.x1 = c.f((long long)M * d->critic_h1);
  t.pre2 = c.f((long long)M * d->critic_h2);
  t.x2 = c.f((long long)M * d->critic_h2);
  t.logits = c.f((long long)M * d->buckets);
}

extern "C" size_t dr_critic_tape_bytes(const dr_dims* d, int M) {
  Carve c(nullptr);
  CTape t;
  ctape_carve(c, d, M, t);
  return c.off;
}

static size_t critic_ws_bytes(const dr_dims* d, int M) {
  Carve c(nullptr);
  CTape t;
  ctape_carve(c, d, M, t);
  c.f(splitk_floats(M, d->critic_h1));
  c.raw(op_nt_split3_ws_bytes(d->critic_h1, d->hidden + latent(d)));
  c.f((long long)op_gemm_nt_split3_part_floats(M, d->critic_h1));
  return c.off + 256;
}


extern "C" int dr_critic_fwd(const dr_dims* d, const dr_critic* cr, int M, const float* h, long long ldh,
                             const float* z, long long ldz, float* logits, float* values, void* tape, void* ws,
                             size_t ws_bytes, hipStream_t s) {
  DR_REQUIRE(d && cr && h && z && M > 0, "null argument or empty batch");
  GemmBf16Scope bf16_scope(d->precision == DR_PREC_BF16);
  CTape t;
  float* sk = nullptr;
  long long skn = 0;
  void* s3w = nullptr;  // split3 weight planes of value_net.0 (fp32 mode)
  float* s3part = nullptr;  // and their split-K partial sums, when the workspace holds them
  size_t s3part_n = 0;
  if (tape) {
    Carve c(tape);
    ctape_carve(c, d, M, t);
  }
  if (ws) {  // scratch: the tape (when none is given), then split-K partials if they fit
    Carve c(ws);
    CTape tw;
    ctape_carve(c, d, M, tw);
    if (!tape) {
      t = tw;
      WS_CHECK(c, ws_bytes);
    }
    const long long want = splitk_floats(M, d->critic_h1);
    if (c.off + (size_t)want * sizeof(float) + 256 <= ws_bytes) {
      skn = want;
      sk = c.f(skn);
      const size_t pb = op_nt_split3_ws_bytes(d->critic_h1, d->hidden + latent(d));
      if (c.off + pb + 256 <= ws_bytes) s3w = c.raw(pb);
      const size_t pn = op_gemm_nt_split3_part_floats(M, d->critic_h1);
      if (s3w && c.off + pn * sizeof(float) + 256 <= ws_bytes) {
        s3part = c.f((long long)pn);
        s3part_n = pn;
      }
    }
  }
  DR_REQUIRE(tape || ws, "dr_critic_fwd needs a tape or a workspace");
  const int L = latent(d), Hd = d->hidden, c1 = d->critic_h1, c2 = d->critic_h2, nb = d->buckets;
  if (s3w && s3_first_layer(d, M, c1, h, ldh, z, ldz)) {
    DR_TRY(op_nt_repack_split3(c1, Hd + L, cr->net.l0.w, Hd + L, s3w, s));
    DR_TRY(op_gemm_nt_split3_sk(M, c1, Hd + L, h, (int)ldh, z, (int)ldz, Hd, s3w, cr->net.l0.b, 0, t.pre1, c1,
                                s3part, s3part_n, s));
  } else {
    GemmArgs g1 = lin2(M, c1, h, ldh, Hd, z, ldz, L, cr->net.l0.w, cr->net.l0.b, t.pre1, c1);
    give_splitk(g1, sk, skn);
    DR_TRY(run(G_NT, AM_PLAIN, g1, s));
  }
  GemmArgs g2 = lin_ln(M, c2, c1, t.pre1, c1, cr->net.n1, cr->net.l3.w, cr->net.l3.b, t.pre2, c2);
  g2.a_out = t.x1; g2.ld_aout = c1;
  DR_TRY(run(G_NT, AM_LNSILU, g2, s));
  float* lg = logits ? logits : t.logits;
  GemmArgs g3 = lin_ln(M, nb, c2, t.pre2, c2, cr->net.n4, cr->net.l6.w, cr->net.l6.b, lg, nb);
  g3.a_out = t.x2; g3.ld_aout = c2;
  DR_TRY(run(G_NT, AM_LNSILU, g3, s));
  if (tape && logits && logits != t.logits) DR_TRY(copy2d(t.logits, nb, logits, nb, nb, M, s));
  if (values) DR_TRY(op_bucket_value(M, nb, lg, nb, cr->buckets, values, 1, s));
  return DR_OK;
}

struct CBws {
  float *row_loss, *glog, *gx2, *gp2, *gy2, *xh2, *gx1, *gp1, *gy1, *xh1;
  float *tl6, *tl3;  // transposed value_net.6 / .3 weights
  float* sk;         // split-K partials of the weight-gradient GEMMs
  long long sk_n;
  void* tn;          // split3 TN scratch (tn_launch)
  size_t tn_bytes;
};
static void cbws_carve(Carve& c, const dr_dims* d, int B, int H, CBws& w) {
  const long long M = (long long)B * (H + 1);
  // the three weight-gradient problems side by side (one grouped launch)
  w.tn_bytes = op_gemm_tn_split3_ws_bytes(d->buckets, d->critic_h2, (int)M) +
               op_gemm_tn_split3_ws_bytes(d->critic_h2, d->critic_h1, (int)M) +
               op_gemm_tn_split3_ws_bytes(d->critic_h1, d->hidden + latent(d), (int)M);
  w.tn = c.raw(w.tn_bytes);
  w.row_loss = c.f((long long)B * H);
  w.sk_n = splitk_floats(d->buckets, d->critic_h2) + splitk_floats(d->critic_h2, d->critic_h1) +
           splitk_floats(d->critic_h1, d->hidden + latent(d));
  w.sk = c.f(w.sk_n);
  w.tl6 = c.f((long long)d->buckets * d->critic_h2);
  w.tl3 = c.f((long long)d->critic_h2 * d->critic_h1);
  w.glog = c.f(M * d->buckets);
  w.gx2 = c.f(M * d->critic_h2);
  w.gp2 = c.f(M * d->critic_h2);
  w.gy2 = c.f(M * d->critic_h2);
  w.xh2 = c.f(M * d->critic_h2);
  w.gx1 = c.f(M * d->critic_h1);
  w.gp1 = c.f(M * d->critic_h1);
  w.gy1 = c.f(M * d->critic_h1);
  w.xh1 = c.f(M * d->critic_h1);
}

extern "C" size_t dr_critic_workspace_bytes(const dr_dims* d, int B, int H) {
  Carve c(nullptr);
  CBws w;
  cbws_carve(c, d, B, H, w);
  const size_t a = c.off, b = critic_ws_bytes(d, B * (H + 1));
  return a > b ? a : b;
}

extern "C" int dr_critic_loss_bwd(const dr_dims* d, const dr_critic* cr, int B, int H, const float* hiddens,
                                  const float* latents, const float* R, const void* tape, float scale,
                                  float* loss_out, const dr_critic* gr, void* ws, size_t ws_bytes, hipStream_t s) {
  DR_REQUIRE(d && cr && hiddens && latents && R && tape && loss_out && gr && B > 0 && H > 0, "null argument");
  GemmBf16Scope bf16_scope(d->precision == DR_PREC_BF16);
  Carve c(ws);
  CBws w;
  cbws_carve(c, d, B, H, w);
  WS_CHECK(c, ws_bytes);
  const int M = B * (H + 1);
  Carve ct((void*)tape);
  CTape t;
  ctape_carve(ct, d, M, t);
  const int L = latent(d), Hd = d->hidden, c1 = d->critic_h1, c2 = d->critic_h2, nb = d->buckets;
  DR_TRY(op_critic_ce(B, H, nb, t.logits, R, cr->buckets, scale, w.row_loss, w.glog, s));
  DR_TRY(op_mean(B * H, w.row_loss, loss_out, s));
  // value_net.6
  {
    TransposeJob tj[2] = {{nb, c2, nb, cr->net.l6.w, w.tl6}, {c2, c1, c2, cr->net.l3.w, w.tl3}};
    DR_TRY(op_transpose_multi(tj, 2, s));
  }
  DR_TRY(run(G_NT, AM_PLAIN, bwd_nt(M, c2, nb, w.glog, nb, w.tl6, w.gx2, c2, 0), s));
  DR_TRY(lnbwd_nt(M, c1, c2, w.gx2, c2, t.pre2, c2, cr->net.n4, w.tl3, w.gx1, c1, 0, w.gp2, c2, w.gy2, w.xh2, nullptr,
                  0, INT_MAX, s));
  DR_TRY(op_ln_silu_bwd(M, c1, w.gx1, c1, t.pre1, c1, cr->net.n1.w, cr->net.n1.b, w.gp1, c1, w.gy1, w.xh1, s));
  {
    GemmArgs p[3];
    p[0] = bwd_w(nb, c2, M, w.glog, nb, t.x2, c2, gr->net.l6.w);
    p[1] = bwd_w(c2, c1, M, w.gp2, c2, t.x1, c1, gr->net.l3.w);
    p[2] = bwd_w(c1, Hd + L, M, w.gp1, c1, hiddens, Hd, gr->net.l0.w);
    p[2].W2 = latents; p[2].ldb2 = L; p[2].nsplitB = Hd;
    float* sk = w.sk;
    long long skn = w.sk_n;
    for (int i = 0; i < 3; ++i) give_splitk(p[i], sk, skn);
    DR_TRY(tn_launch(p, 3, w.tn, w.tn_bytes, s, d->precision == DR_PREC_BF16 ? 1 : 3));
  }
  {
    ColsumJob cj[7] = {
        {nb, w.glog, nb, nullptr, 0, gr->net.l6.b}, {c2, w.gp2, c2, nullptr, 0, gr->net.l3.b},
        {c2, w.gy2, c2, w.xh2, c2, gr->net.n4.w},   {c2, w.gy2, c2, nullptr, 0, gr->net.n4.b},
        {c1, w.gp1, c1, nullptr, 0, gr->net.l0.b},  {c1, w.gy1, c1, w.xh1, c1, gr->net.n1.w},
        {c1, w.gy1, c1, nullptr, 0, gr->net.n1.b},
    };
    DR_TRY(op_colsum_multi(M, cj, 7, s));
  }
  return DR_OK;
}

// ===========================================================================
// single steps
// ===========================================================================
static size_t step_ws(const dr_dims* d, int B) {
  Carve c(nullptr);
  c.f((long long)B * 3 * d->hidden);
  c.f((long long)B * 3 * d->hidden);
  c.f((long long)B * latent(d));
  const int mx = d->prior_h1 > d->rew_h1 ? d->prior_h1 : d->rew_h1;
  c.f((long long)B * (mx > d->actor_h1 ? mx : d->actor_h1) * 2);
  c.f((long long)B * (d->buckets + 8) * 2);
  return c.off;
}

extern "C" size_t dr_step_workspace_bytes(const dr_dims* d, int B) { return step_ws(d, B) + 4096; }

// generic 3-layer MLP forward on [h | z] (z may be NULL / in_z = 0)
static int mlp3(const dr_mlp3& m, int M, int in_h, const float* h, long long ldh, int in_z, const float* z,
                long long ldz, int h1, int h2, int n_out, float* out, long long ldo, float* p1, float* p2,
                hipStream_t s) {
  GemmArgs g = in_z ? lin2(M, h1, h, ldh, in_h, z, ldz, in_z, m.l0.w, m.l0.b, p1, h1)
                    : lin(M, h1, in_h, h, ldh, m.l0.w, in_h, m.l0.b, p1, h1);
  DR_TRY(run(G_NT, AM_PLAIN, g, s));
  DR_TRY(run(G_NT, AM_LNSILU, lin_ln(M, h2, h1, p1, h1, m.n1, m.l3.w, m.l3.b, p2, h2), s));
  return run(G_NT, AM_LNSILU, lin_ln(M, n_out, h2, p2, h2, m.n4, m.l6.w, m.l6.b, out, ldo), s);
}

extern "C" int dr_mlp3_fwd(const dr_mlp3* m, int M, int in_h, const float* h, long long ldh, int in_z,
                           const float* z, long long ldz, int h1, int h2, int n_out, float* out, long long ldo,
                           void* ws, size_t ws_bytes, hipStream_t s) {
  DR_REQUIRE(m && h && out && M > 0 && h1 > 0 && h2 > 0 && n_out > 0, "null argument or bad widths");
  Carve c(ws);
  float* p1 = c.f((long long)M * h1);
  float* p2 = c.f((long long)M * h2);
  WS_CHECK(c, ws_bytes);
  return mlp3(*m, M, in_h, h, ldh, in_z, z, ldz, h1, h2, n_out, out, ldo, p1, p2, s);
}

extern "C" int dr_gru_cell(const dr_dims* d, const dr_world_model* wm, int B, const float* z, const float* h,
                           const float* a, float* h_out, void* ws, size_t ws_bytes, hipStream_t s) {
  DR_REQUIRE(d && wm && z && a && h_out && B > 0, "null argument");
  Carve c(ws);
  float* gi = c.f((long long)B * 3 * d->hidden);
  float* gh = c.f((long long)B * 3 * d->hidden);
  WS_CHECK(c, ws_bytes);
  return gru_step(d, wm, B, z, latent(d), a, d->action, h, d->hidden, h_out, d->hidden, gi, gh, nullptr, nullptr,
                  nullptr, nullptr, s);
}

extern "C" int dr_imagine_step(const dr_dims* d, const dr_world_model* wm, int B, const float* h, const float* z,
                               const float* a, dr_noise noise, float* h_out, float* z_out, float* r_out,
                               float* c_out, void* ws, size_t ws_bytes, hipStream_t s) {
  DR_REQUIRE(d && wm && z && a && h_out && z_out && B > 0, "null argument");
  const int L = latent(d), Hd = d->hidden;
  Carve c(ws);
  float* gi = c.f((long long)B * 3 * Hd);
  float* gh = c.f((long long)B * 3 * Hd);
  float* lg = c.f((long long)B * L);
  const int mx = d->prior_h1 > d->rew_h1 ? d->prior_h1 : d->rew_h1;
  const int w1 = mx > d->cont_h1 ? mx : d->cont_h1;
  float* p1 = c.f((long long)B * w1 * 2);
  float* p2 = c.f((long long)B * (d->buckets + 8) * 2);
  WS_CHECK(c, ws_bytes);
  DR_TRY(gru_step(d, wm, B, z, L, a, d->action, h, Hd, h_out, Hd, gi, gh, nullptr, nullptr, nullptr, nullptr, s));
  DR_TRY(mlp3(wm->prior, B, Hd, h_out, Hd, 0, nullptr, 0, d->prior_h1, d->prior_h2, L, lg, L, p1, p2, s));
  DR_TRY(op_sample(B, d->rows, d->cols, lg, L, &noise, 0, z_out, L, nullptr, nullptr, 0, s));
  if (r_out) {
    DR_TRY(mlp3(wm->reward, B, Hd, h_out, Hd, L, z_out, L, d->rew_h1, d->rew_h2, d->buckets, lg, d->buckets, p1, p2, s));
    DR_TRY(op_bucket_value(B, d->buckets, lg, d->buckets, wm->buckets_rew, r_out, 1, s));
  }
  if (c_out) {
    DR_TRY(mlp3(wm->cont, B, Hd, h_out, Hd, L, z_out, L, d->cont_h1, d->cont_h2, 1, lg, 1, p1, p2, s));
    DR_TRY(op_sigmoid(B, lg, 1, c_out, 1, s));
  }
  return DR_OK;
}

struct ActWs {
  float *p1, *p2, *ls;
};
static void act_carve(Carve& c, const dr_dims* d, int B, ActWs& w) {
  w.p1 = c.f((long long)B * d->actor_h1);
  w.p2 = c.f((long long)B * d->actor_h2);
  w.ls = c.f((long long)B * d->action);
}

extern "C" size_t dr_actor_act_workspace_bytes(const dr_dims* d, int B) {
  Carve c(nullptr);
  ActWs w;
  act_carve(c, d, B, w);
  return c.off;
}

extern "C" int dr_actor_act(const dr_dims* d, const dr_actor* ac, int B, const float* h, const float* z,
                            dr_noise noise, int deterministic, float* a_out, float* mu_out, float* sigma_out,
                            void* ws, size_t ws_bytes, hipStream_t s) {
  DR_REQUIRE(d && ac && h && z && a_out && mu_out && sigma_out && B > 0, "null argument");
  const int L = latent(d), Hd = d->hidden, A = d->action, a1 = d->actor_h1, a2 = d->actor_h2;
  Carve c(ws);
  ActWs w;
  act_carve(c, d, B, w);
  WS_CHECK(c, ws_bytes);
  float *p1 = w.p1, *p2 = w.p2, *ls = w.ls;
  DR_TRY(run(G_NT, AM_PLAIN, lin2(B, a1, h, Hd, Hd, z, L, L, ac->l0.w, ac->l0.b, p1, a1), s));
  DR_TRY(run(G_NT, AM_LNSILU, lin_ln(B, a2, a1, p1, a1, ac->n1, ac->l3.w, ac->l3.b, p2, a2), s));
  GemmArgs p[2];
  p[0] = lin_ln(B, A, a2, p2, a2, ac->n4, ac->mu.w, ac->mu.b, mu_out, A);
  p[1] = lin_ln(B, A, a2, p2, a2, ac->n4, ac->ls.w, ac->ls.b, ls, A);
  DR_TRY(gemm_launch(G_NT, AM_LNSILU, p, 2, s));
  return op_actor_head(B, A, mu_out, A, ls, A, &noise, 0, deterministic, a_out, A, nullptr, 0, sigma_out, A, nullptr,
                       s);
}

// which entry points of one train_Agent epoch run as their ONE persistent
// launch for these dims and shapes (stream CU masks aside): bit 0 the warm
// start's posterior scan (T = S / 2 steps), bit 1 the imagination unroll, bit 2
// the BPTT.  The data-parallel schedule (dreamer_amd/engine.py) keeps
// collective kernels away from a persistent BPTT with it.
extern "C" int dr_persistent_kernels(const dr_dims* d, int B, int T, int H) {
  if (!d || B <= 0 || T <= 0 || H <= 0) return 0;
  const int A = d->action;
  int m = 0;
  if (op_pscan_supported(d, B, T, A)) m |= 1;
  if (d->rows <= 32 && d->actor_h1 % 4 == 0 && op_pdream_supported(d, B, H, A)) m |= 2;
  if (op_pbptt_supported(d, B, H, A)) m |= 4;
  return m;
}
