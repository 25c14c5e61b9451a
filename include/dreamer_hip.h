/*
 * libdreamer_hip -- C ABI of the MI355X (gfx950) Dreamer imagination engine.
 *
 * The reference (youngers2006/Dreamer) has no FFI: its hot path is a
 * composition of PyTorch ops inside Python classes.  Each entry point below
 * replaces one of those compositions and cites the reference code it
 * restates (file:line in /root/reference).  The Python package
 * ``dreamer_amd`` binds them with ctypes behind the reference's own class API
 * (Dreamer / WorldModel / Agent / Buffer ...).
 *
 * Conventions
 *  - every function returns 0 (DR_OK) or an error code; dr_last_error() gives
 *    a thread-local message.  Nothing throws across the ABI.
 *  - all pointers are device pointers owned by the caller (the PyTorch caching
 *    allocator); the library never allocates, frees, or keeps a pointer after
 *    returning.  Scratch comes from the caller's workspace (sizes from the
 *    *_bytes queries).
 *  - calls are asynchronous on the given hipStream_t; no implicit sync, so the
 *    whole train_Agent epoch can be captured into one hipGraph.
 *  - parameters are read in PyTorch's own layouts (Linear weight [out][in],
 *    GRUCell weight_ih [3H][in] gate order r,z,n, Conv2d [out][in][4][4]).
 *  - arithmetic is fp32 (parity mode) unless dr_dims.precision selects bf16:
 *    fp32 GEMMs use the exact-f32 MFMA (v_mfma_f32_16x16x4_f32), elementwise
 *    code is built -ffp-contract=off; bf16 mode runs the encoder convolutions
 *    and feature projection on v_mfma_f32_16x16x32_bf16 (f32 accumulate).
 */
#ifndef DREAMER_HIP_H
#define DREAMER_HIP_H

#include <hip/hip_runtime.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DR_OK 0
#define DR_E_INVALID 1001   /* bad dims / pointers */
#define DR_E_HIP 1002       /* a HIP launch failed */
#define DR_E_WORKSPACE 1003 /* workspace too small */
#define DR_E_UNSUPPORTED 1004 /* valid call outside what this entry point covers (dims / device):
                                 use the unfused entry points (dr_act_step) */

/* Linear (or LayerNorm) parameters: w [out][in] (LN: gamma [n]), b [out]. */
typedef struct { float* w; float* b; } dr_linear;

/* nn.Sequential(Linear, LayerNorm, SiLU, Linear, LayerNorm, SiLU, Linear)
 * indices 0,1,3,4,6 (DynamicsPredictors.py:15-23,52-60,85-93; Agent.py:219-227). */
typedef struct { dr_linear l0, n1, l3, n4, l6; } dr_mlp3;

/* Model widths (Dreamer.py:20-64 config keys). */
typedef struct {
  int hidden;          /* hidden_state_dims (600) */
  int rows, cols;      /* latent_state_dims (32, 32) */
  int action;          /* action_dims (3) */
  int img_h, img_w;    /* observation_dims (64, 64) */
  int enc_f1, enc_f2;  /* encoder_filter_num_1/2 (32, 64): conv channels f1, f2, 2*f2, 4*f2 */
  int enc_hidden;      /* encoder_hidden_layer_nodes (200) */
  int prior_h1, prior_h2, rew_h1, rew_h2, cont_h1, cont_h2;
  int actor_h1, actor_h2, critic_h1, critic_h2;
  int buckets;         /* critic_reward_buckets (255) */
  int dec_f1, dec_f2;  /* decoder_filter_num_1/2 (32, 64): convT channels 4*f2 -> 2*f2 -> f2 -> f1 -> 3 */
  int dec_hidden;      /* decoder_hidden_layer_nodes (200) */
  int precision;       /* DR_PREC_FP32 (parity mode, default) or DR_PREC_BF16 (perf mode: bf16 MFMA
                          operands, f32 accumulation; the extra `precision` config key) */
  int obs_dim;         /* 0: pixel observations img_h x img_w x 3 (the reference).  D > 0: proprioceptive
                          vector observations of D floats (BASELINE configs[4]; the reference has no such
                          encoder, VAE.py:33-42 is always convolutional).  The convolution slots then hold
                          an MLP: encoder conv[0] = Linear(D, 4*enc_f2), conv[1] =
                          Linear(4*enc_f2, 4*enc_f2), each + SiLU (F = 4*enc_f2 features, conv[2..3]
                          unused); decoder upscaler.3 -> 4*dec_f2, convt[0] = Linear(4*dec_f2, 4*dec_f2)
                          + SiLU, convt[1] = Linear(4*dec_f2, D) (no Tanh; convt[2..3] unused). */
  int enc_depth;       /* k4 s2 p1 convolutions of the encoder (and transposed convolutions of the decoder):
                          0 or 4 = the reference's VAE (VAE.py:33-42, 128-137); 5 = the "deeper VAE" of BASELINE
                          configs[3] (the extra config key encoder_depth; no reference definition -- one more
                          stride-2 layer each way, so 128x128 frames reach the same 4x4 grid 64x64 frames reach
                          in the reference): encoder channels 3, f1, f2, 2 f2, 4 f2, 4 f2 (conv[0..4]); decoder
                          4 d2 (H/32 x W/32) -> 4 d2 -> 2 d2 -> d2 -> d1 -> 3 (convt[0..4]). */
  int launch_form;     /* 0 (default): an entry point may run as ONE persistent launch where the shape and the
                          stream's CUs allow it (the warm start's posterior scan, scan.hip); 1: always the
                          launch sequence.  Set for work captured on one stream and replayed on a CU-masked
                          one (the pipelined epochs' warm start), and by DREAMER_PERSISTENT=0. */
  float* fault;        /* device float, may be NULL: the fault slot of the persistent launches (posterior
                          scan, imagination unroll, BPTT).  Their waits on other workgroups are bounded; if
                          one times out (a workgroup was not resident, e.g. held off by other work on the
                          CUs), the launch's outputs are written NaN and *fault = NaN.  Sticky: the library
                          never clears it.  The engine keeps it among the agent's loss slots, so the
                          non-finite skip (Agent.py:137-139) rejects that epoch's update on every rank.  Test
                          hook: DREAMER_PERSIST_FORCE=timeout (or scan / dream / bptt) makes every wait of
                          those launches time out, read at each call. */
  unsigned* fault_host; /* may be NULL: a word of pinned host memory (its device address,
                          dr_host_device_ptr) set to 1 on the same timeouts, so the host notices a fault
                          without a copy or a sync (dreamer_amd/engine.py check_faults raises).  Sticky. */
} dr_dims;
#define DR_MAX_DEPTH 5
#define DR_PREC_FP32 0
#define DR_PREC_BF16 1

/* WorldModel parameters (WorldModel.py:55-60). */
typedef struct {
  dr_linear conv[DR_MAX_DEPTH];   /* encoder.feature_extractor.{0,2,4,6(,8)} (dr_dims.enc_depth layers) */
  dr_linear map0, map1, map3;     /* encoder.latent_mapper.{0, 1 (LN), 3} */
  float *w_ih, *w_hh, *b_ih, *b_hh; /* sequence_model.GRU */
  dr_mlp3 prior;                  /* dynamics_predictor.logit_net */
  dr_mlp3 reward;                 /* reward_predictor.logit_net */
  dr_mlp3 cont;                   /* continue_predictor.logit_generator */
  float* buckets_rew;             /* reward_predictor.buckets_rew */
} dr_world_model;

/* Decoder parameters (VariationalAutoEncoder.py:118-137). */
typedef struct {
  dr_linear up0, up1, up3;        /* decoder.upscaler.{0, 1 (LN), 3} */
  dr_linear convt[DR_MAX_DEPTH];  /* decoder.image_builder.{0,2,4,6(,8)}: ConvTranspose2d w [in][out][4][4] */
} dr_decoder;

/* Actor (Agent.py:174-200): base_net.{0,1,3,4}, mu_head, log_sig_head. */
typedef struct { dr_linear l0, n1, l3, n4, mu, ls; } dr_actor;

/* Critic (Agent.py:212-241): value_net, buckets_crit. */
typedef struct { dr_mlp3 net; float* buckets; } dr_critic;

/* Randomness.  Explicit-noise mode reproduces the reference's draws
 * (parity); Philox mode generates them in-kernel keyed by
 * (seed, offset, stream, global row, element) so a data-parallel shard draws
 * exactly what the single-GPU run draws for the same global rows. */
typedef struct {
  const float* q;   /* Exp(1) variates [steps][rows*R][C] (Categorical sample), or NULL */
  const float* eps; /* N(0,1) variates [steps][rows][A] (actor rsample), or NULL */
  const unsigned long long* rng; /* device {seed, offset}; used where q/eps are NULL */
  int row0;         /* global index of local row 0 */
  int stream;       /* Philox stream id (distinct per call site) */
} dr_noise;

/* Source of observation frames for the encoder.  Frame f = t*B + b. */
typedef struct {
  const unsigned char* ring; /* u8 replay ring [cap][3][H][W] (Buffer.py:7), or NULL; with dr_dims.obs_dim
                                = D > 0 the ring holds f32 rows [cap][D] (pointer cast) */
  long long ring_cap;
  const long long* starts;   /* device [B] window starts (Buffer.py:36-50) */
  const float* obs;          /* f32 frames (when ring == NULL) */
  long long stride_b, stride_t; /* f32: element offset of frame (b,t) = b*stride_b + t*stride_t */
  int raw255;                /* 1: values are 0..255 -> x/255-0.5 (Dreamer.py:251); 0: already normalised */
  int t0;                    /* time offset: frame (b, t) is window step t0 + t (chunked encoding) */
} dr_frames;

const char* dr_last_error(void);
int dr_version(void);

/* A HIP stream whose kernels run only on the CUs set in mask (n_words 32-bit
 * words, bit i = CU i of the device's CU-mask order; hipExtStreamCreateWithCUMask).
 * The pipelined AC_epochs > 1 schedule (dreamer_amd/engine.py run_many) fences
 * the next epoch's warm start (conv encoder + posterior scan) off part of the
 * chip so that the latency-bound imagination / update chain keeps free CUs.
 * No Dreamer.py counterpart: a scheduling aid of this implementation. */
int dr_stream_create_cumask(int n_words, const unsigned* mask, hipStream_t* out);
int dr_stream_destroy(hipStream_t s);
/* the device's CU count (hipDeviceAttributeMultiprocessorCount) */
int dr_device_cus(int* out);
/* the device address of pinned host memory (hipHostGetDevicePointer): dr_dims.fault_host */
int dr_host_device_ptr(void* host, void** dev);

/* ---- a3  Encoder conv stack + latent_mapper.0 feature columns ---------------
 * feat[f][enc_hidden] = flatten(SiLU(conv4(...SiLU(conv1(frame f)))))
 *                       . map0.w[:, :F]^T + map0.b            (VAE.py:57-75)
 * for the n = B*T frames of `src` (time-major: f = t*B + b). */
size_t dr_encoder_workspace_bytes(const dr_dims* d, int n_frames);
int dr_encoder_features(const dr_dims* d, const dr_world_model* wm, const dr_frames* src, int B, int T,
                        float* feat, void* ws, size_t ws_bytes, hipStream_t stream);

/* ---- a2/a5  posterior scan (warm_start_generator, Dreamer.py:244-262;
 *      observe_step, WorldModel.py:79-82; Encoder.encode, VAE.py:77-99) -----
 * If z_init == NULL, frame 0 is an encode from h_init (zeros if NULL) and
 * frame t>=1 runs GRU(z, actions[t-1], h) first.  If z_init != NULL every
 * frame t runs GRU(z, actions[t], h) first.  actions element (b,t,i) is at
 * actions[b*act_sb + t*act_st + i].  Writes the last frame's z, h (and
 * logits if non-NULL). */
size_t dr_observe_workspace_bytes(const dr_dims* d, int B);
int dr_observe_scan(const dr_dims* d, const dr_world_model* wm, int B, int T, const float* feat,
                    const float* actions, long long act_sb, long long act_st, const float* h_init,
                    const float* z_init, dr_noise noise, float* z_out, float* h_out, float* logits_out,
                    void* ws, size_t ws_bytes, hipStream_t stream);

/* ---- a7  imagination unroll (dream_episodes, Dreamer.py:143-175) -----------
 * Outputs use the reference's layouts: latents [B][H+1][R*C], hiddens
 * [B][H+1][hidden], actions/mus/sigmas [B][H][A], rewards/continues [B][H].
 * `tape` (dr_imagine_tape_bytes) keeps what dr_imagine_bwd needs. */
size_t dr_imagine_tape_bytes(const dr_dims* d, int B, int H);
size_t dr_imagine_workspace_bytes(const dr_dims* d, int B, int H);
int dr_imagine_fwd(const dr_dims* d, const dr_world_model* wm, const dr_actor* actor, int B, int H,
                   const float* z0, const float* h0, dr_noise noise, int deterministic, float* latents,
                   float* hiddens, float* actions, float* rewards, float* continues, float* mus,
                   float* sigmas, void* tape, void* ws, size_t ws_bytes, hipStream_t stream);

/* Backprop through the unroll for the actor (Agent.py:141-145 backward):
 * given dL/dmus, dL/dsigmas (and optionally dL/dactions, dL/dlatents,
 * dL/dhiddens; NULL = 0), writes dL/d(actor params) into `grad` (overwrite).
 * World-model weights receive no gradient (the reference's WM grads from this
 * path are discarded by WorldModel.training_step's zero_grad, WorldModel.py:195). */
int dr_imagine_bwd(const dr_dims* d, const dr_world_model* wm, const dr_actor* actor, int B, int H,
                   const float* latents, const float* hiddens, const float* actions, const float* g_mus,
                   const float* g_sigmas,
                   const float* g_actions, const float* g_latents, const float* g_hiddens,
                   const void* tape, const dr_actor* grad, void* ws, size_t ws_bytes, hipStream_t stream);
/* dr_imagine_bwd in two parts on the same workspace: _prep writes the upstream
 * state gradients (NULL = 0) and the transposed weights -- it needs neither
 * dL/dmus nor the tape, so it can run on a second stream while the returns and
 * losses are formed; _main runs the reverse loop and the weight gradients
 * (upstream_state: 1 if _prep was given dL/dlatents or dL/dhiddens). */
int dr_imagine_bwd_prep(const dr_dims* d, const dr_world_model* wm, const dr_actor* actor, int B, int H,
                        const float* g_actions, const float* g_latents, const float* g_hiddens, void* ws,
                        size_t ws_bytes, hipStream_t stream);
int dr_imagine_bwd_main(const dr_dims* d, const dr_world_model* wm, const dr_actor* actor, int B, int H,
                        const float* latents, const float* hiddens, const float* actions, const float* g_mus,
                        const float* g_sigmas, int upstream_state, const void* tape, const dr_actor* grad, void* ws,
                        size_t ws_bytes, hipStream_t stream);

/* ---- single steps (batch-1 acting path and per-block API) ------------------ */
/* imagine_step (WorldModel.py:72-77): h' = GRU(z,h,a); z' ~ prior(h'); r; c */
int dr_imagine_step(const dr_dims* d, const dr_world_model* wm, int B, const float* h, const float* z,
                    const float* a, dr_noise noise, float* h_out, float* z_out, float* r_out, float* c_out,
                    void* ws, size_t ws_bytes, hipStream_t stream);
/* Actor.act (Agent.py:202-210); workspace from dr_actor_act_workspace_bytes */
size_t dr_actor_act_workspace_bytes(const dr_dims* d, int B);
int dr_actor_act(const dr_dims* d, const dr_actor* actor, int B, const float* h, const float* z,
                 dr_noise noise, int deterministic, float* a_out, float* mu_out, float* sigma_out, void* ws,
                 size_t ws_bytes, hipStream_t stream);
/* Batch-1 acting step in ONE launch with in-kernel grid barriers (rollout_policy
 * / evaluate_agent / Run, Dreamer.py:177-226, 295-322, 374-401): if has_prev,
 * h' = GRU(z_prev, h, a_prev) (observe_step, WorldModel.py:79-82), else h' = h
 * (episode start, h = 0: Dreamer.py:186-187); z' = Encoder.encode(h', frame)
 * (VAE.py:57-99); a = Actor.act(h', z', deterministic) (Agent.py:202-210).
 * frame: the env observation [H][W][3] u8 on the device.  Noise: the sampler
 * draws stream `noise.stream`, the actor `noise.stream + 1` (explicit q [R*C],
 * eps [A] when given).  logits_out may be NULL.  Inputs and outputs may alias
 * (h / h_out, z_prev / z_out, a_prev / a_out).
 * Co-residency of the grid is checked once per device (occupancy query); the
 * call returns DR_E_UNSUPPORTED when the device cannot hold it, or for dims
 * outside the kernel's staging (callers then use the unfused entry points).
 * status (device int, may be NULL; the caller zeroes it): set to 1 if a grid
 * barrier timed out at run time; it is the authoritative signal -- the outputs
 * then hold NaN whenever workgroup 0 saw the failure, and must not be used.
 * Test hook: the environment variable DREAMER_ACT_FORCE=timeout (every grid
 * barrier times out at once) or =nonresident (the co-residency check fails),
 * read at each call. */
size_t dr_act_step_workspace_bytes(const dr_dims* d);
int dr_act_step(const dr_dims* d, const dr_world_model* wm, const dr_actor* actor, const unsigned char* frame,
                int has_prev, const float* z_prev, const float* h, const float* a_prev, dr_noise noise,
                int deterministic, float* z_out, float* h_out, float* a_out, float* mu_out, float* sigma_out,
                float* logits_out, int* status, void* ws, size_t ws_bytes, hipStream_t stream);

/* GRU cell (SequenceModel.py:19-24) */
int dr_gru_cell(const dr_dims* d, const dr_world_model* wm, int B, const float* z, const float* h,
                const float* a, float* h_out, void* ws, size_t ws_bytes, hipStream_t stream);
/* Categorical sampler with unimix + straight-through value (VAE.py:88-98,
 * DynamicsPredictors.py:33-39): z = onehot(argmax(p_hat/q)) + p - p (value). */
int dr_categorical_sample(int M, int R, int C, const float* logits, dr_noise noise, float* z_out,
                          int* idx_out, float* soft_out, hipStream_t stream);
/* heads: prior logits, reward value (symexp E[bucket]), continue prob */
int dr_mlp3_fwd(const dr_mlp3* m, int M, int in_h, const float* h, long long ldh, int in_z, const float* z,
                long long ldz, int h1, int h2, int n_out, float* out, long long ldo, void* ws, size_t ws_bytes,
                hipStream_t stream);
size_t dr_step_workspace_bytes(const dr_dims* d, int B);
int dr_bucket_value(int M, int nb, const float* logits, const float* buckets, float* out, hipStream_t stream);

/* ---- a13-a16  actor-critic update pieces (Agent.py:78-172) ----------------- */
size_t dr_critic_tape_bytes(const dr_dims* d, int M);
size_t dr_critic_workspace_bytes(const dr_dims* d, int B, int H);
/* logits [M][nb] (optional), values [M] (optional); tape (optional) for bwd */
int dr_critic_fwd(const dr_dims* d, const dr_critic* c, int M, const float* h, long long ldh, const float* z,
                  long long ldz, float* logits, float* values, void* tape, void* ws, size_t ws_bytes,
                  hipStream_t stream);
/* lambda returns (Agent.py:156-172): V [B][H+1] target values */
int dr_lambda_returns(int B, int H, const float* r, const float* c, const float* V, float gamma, float lam,
                      float* R, hipStream_t stream);
/* update_S (Agent.py:78-88) over n returns; S is a device scalar updated in
 * place unless R holds NaN/Inf; norm_out = max(S, 1) (Agent.py:120). */
int dr_update_S(int n, const float* R, float* S, float* norm_out, void* ws, size_t ws_bytes,
                hipStream_t stream);
/* actor loss (Agent.py:105-125) and its gradient wrt mus/sigmas; loss_out
 * holds 1 + B*H floats: [0] = mean loss over the B*H local rows, the rest is
 * per-row scratch.  scale = dL/d(row loss) (1/(B*H) on one device). */
int dr_actor_loss_grad(int B, int H, int A, const float* mus, const float* sigmas, const float* actions,
                       const float* R, const float* V, const float* norm, float nu, float scale,
                       float* loss_out, float* g_mus, float* g_sigmas, hipStream_t stream);
/* critic two-hot cross-entropy (Agent.py:127-135) + backward into `grad`
 * (overwrite); rows are (b,t) with t<=H of hiddens/latents; row t=H is unused. */
int dr_critic_loss_bwd(const dr_dims* d, const dr_critic* c, int B, int H, const float* hiddens,
                       const float* latents, const float* R, const void* tape, float scale, float* loss_out,
                       const dr_critic* grad, void* ws, size_t ws_bytes, hipStream_t stream);

/* ---- optimiser (torch.optim.AdamW + clip_grad_norm_ + soft target) -------- */
int dr_sqnorm(long long n, const float* g, float* acc, hipStream_t stream);
/* as dr_sqnorm, many workgroups (large buffers); scratch >= 512 floats */
int dr_sqnorm_multi(long long n, const float* g, float* acc, float* scratch, hipStream_t stream);
/* The agent's pre-update statistics in one launch (Agent.py:137-148):
 * sq[0] = |ga|^2 (actor grads), sq[1] = |gb|^2 (critic grads), *skip = any
 * non-finite value among loss[0..nloss).  Replaces the NaN check and the two
 * clip_grad_norm_ reductions.  scratch: DR_CLIP_SCRATCH_FLOATS floats,
 * zeroed once by the caller (holds the partials and an arrival ticket the
 * kernel re-arms); buffers 16-byte aligned.  Deterministic. */
#define DR_CLIP_SCRATCH_FLOATS 1024
int dr_clip_stats(long long na, const float* ga, long long nb, const float* gb, int nloss, const float* loss,
                  float* sq, int* skip, void* scratch, hipStream_t stream);
/* p <- AdamW(p, g*clip) (torch.optim.AdamW single-tensor op order) where
 * clip = min(1, max_norm/(sqrt(*sqnorm)+1e-6)) (sqnorm NULL: no clip).  The
 * step counter lives on the device: a prelude increments *step and writes
 * hyper[0] = lr/(1-b1^step), hyper[1] = sqrt(1-b2^step) (double math, like
 * torch's python scalars; the hyperparameters are doubles, like the python
 * floats torch.optim.AdamW computes 1 - beta etc. from).  g is scaled in place
 * by clip (as clip_grad_norm_ does).  Everything is skipped when *skip != 0. */
int dr_adamw(long long n, float* p, float* g, float* m, float* v, const float* sqnorm, float max_norm,
             double lr, double b1, double b2, double eps, double wd, int* step, float* hyper, const int* skip,
             hipStream_t stream);
int dr_ema(long long n, float* target, const float* src, float keep, float tau, const int* skip,
           hipStream_t stream);
/* Agent.train_step's whole optimiser tail in two launches (Agent.py:137-153):
 * dr_clip_stats over (actor, critic) grads with both AdamW preludes run by its
 * last workgroup, then dr_adamw(actor, clip by sq[0]), dr_adamw(critic, clip by
 * sq[1]) and dr_ema(target <- ema_keep * target + tau * critic) in one
 * elementwise pass.  Same per-element arithmetic (same bits) as those five
 * calls; scratch as dr_clip_stats. */
int dr_ac_optimiser_step(long long na, float* pa, float* ga, float* ma, float* va, int* step_a, float* hyper_a,
                         double lr_a, double b1_a, double b2_a, double eps_a, double wd_a, long long nc, float* pc,
                         float* gc, float* mc, float* vc, int* step_c, float* hyper_c, double lr_c, double b1_c,
                         double b2_c, double eps_c, double wd_c, float max_norm, float* target, float ema_keep,
                         float tau, int nloss, const float* loss, float* sq, int* skip, void* scratch,
                         hipStream_t stream);
/* non-finite flag: *flag = any(!isfinite(x[0..n))) (OR-accumulate) */
int dr_nonfinite(long long n, const float* x, int* flag, hipStream_t stream);

/* ---- a19/a20  world-model training step (WorldModel.training_step,
 *      WorldModel.py:148-198; unroll_model 84-146; Decoder.forward VAE.py:139-161)
 * Loss and gradients of one step over a window of T = horizon frames per row:
 * posterior scan (observe_step with the GRU run from zeros at t = 0), batched
 * prior / decoder / reward / continue heads on steps 1..T-1, the masked
 * reconstruction / reward / continue / KL losses with the max(1, KL) free-bit
 * clamps, and backprop through everything (decoder and encoder convolutions,
 * the posterior scan's GRU and straight-through samples) into `g_wm` /
 * `g_dec` (overwrite).  Arithmetic is fp32: the reference's fp16 autocast +
 * GradScaler is, in fp32, the plain backward (the scaler only skips steps with
 * non-finite gradients -- `skip` reports a non-finite loss; callers OR in a
 * gradient check).  losses (device, 4 floats): total, loss_pred, KL_dyn,
 * KL_rep (both KL means; the free-bit clamp is applied in `total`).
 * Frames: src frame (b, t) is window step t (time-major f = t*B + b).
 * Optional outputs (time-major [T][B][...]): posterior hiddens, latents, logits. */
typedef struct {
  const float* actions; long long act_sb, act_st;                     /* (b,t,i) at b*sb + t*st + i */
  const float* rewards; const float* continues; long long rc_sb, rc_st; /* (b,t) at b*sb + t*st */
} dr_wm_batch;
typedef struct { float beta_pred, beta_dyn, beta_rep; } dr_wm_loss_cfg;
size_t dr_wm_train_workspace_bytes(const dr_dims* d, int B, int T);
/* The same step in three phases for data parallelism (one shard of B rows per
 * rank, same workspace across the phases).  `stats` (device, 8 floats) carries
 * the loss sums that must be global: after DR_WM_PREP the caller all-reduces
 * (sum) stats[0] (mask.sum(), WorldModel.py:185), after DR_WM_FWD stats[1..4]
 * (masked squared-error, reward, continue and KL sums); DR_WM_BWD then forms
 * the global losses (rows_global = global B * (T-1) for the KL means,
 * 182-183) and gradients whose all-reduce SUM is the global gradient. */
#define DR_WM_PREP 1
#define DR_WM_FWD 2
#define DR_WM_BWD 4
/* DR_WM_BWD in three stages, called in this order with the same workspace;
 * each leaves one bucket of the gradient final, so a data-parallel caller can
 * all-reduce it while the next stage runs (WorldModel.py:195-200 backward +
 * SURVEY 8e "bucketed to overlap the backward"):
 *   HEADS: the loss grads, prior / reward / continue heads and the decoder
 *          (g_wm->prior, ->reward, ->cont, every g_dec field) final;
 *   SCAN:  the posterior scan: latent_mapper and GRU (->map0/1/3, ->w_ih,
 *          ->w_hh, ->b_ih, ->b_hh) final;
 *   ENC:   the encoder convolutions (->conv[0..3]) final. */
#define DR_WM_BWD_HEADS 8
#define DR_WM_BWD_SCAN 16
#define DR_WM_BWD_ENC 32
int dr_wm_train_phase(const dr_dims* d, const dr_world_model* wm, const dr_decoder* dec, int B, int T,
                      const dr_frames* src, const dr_wm_batch* batch, dr_noise noise, dr_wm_loss_cfg cfg, int phases,
                      float* stats, int rows_global, float* losses, int* skip, const dr_world_model* g_wm,
                      const dr_decoder* g_dec, float* hiddens_out, float* latents_out, float* post_logits_out,
                      void* ws, size_t ws_bytes, hipStream_t stream);
int dr_wm_train_grads(const dr_dims* d, const dr_world_model* wm, const dr_decoder* dec, int B, int T,
                      const dr_frames* src, const dr_wm_batch* batch, dr_noise noise, dr_wm_loss_cfg cfg,
                      float* losses, int* skip, const dr_world_model* g_wm, const dr_decoder* g_dec,
                      float* hiddens_out, float* latents_out, float* post_logits_out, void* ws, size_t ws_bytes,
                      hipStream_t stream);

/* ---- a20  Decoder.forward (VAE.py:139-161), inference: mu [M][3][H][W] (NCHW)
 * from cat(h, flatten z) rows (h row stride ldh, z row stride ldz). */
size_t dr_decoder_workspace_bytes(const dr_dims* d, int M);
int dr_decoder_fwd(const dr_dims* d, const dr_decoder* dec, int M, const float* h, long long ldh, const float* z,
                   long long ldz, float* mu, void* ws, size_t ws_bytes, hipStream_t stream);

/* ---- a1  replay gather (Buffer.sample_sequences, Buffer.py:49-61) --------- */
int dr_replay_gather(long long cap, int B, int S, int frame_elems, int A, const unsigned char* frames,
                     const float* actions, const float* rewards, const float* continues,
                     const long long* starts, float* obs_out, float* act_out, float* rew_out,
                     float* cont_out, hipStream_t stream);

/* Which parts of a train_Agent epoch (Dreamer.py:264-287) run as ONE persistent
 * launch for these dims and shapes (the stream's CU mask aside): bit 0 the warm
 * start's posterior scan over T steps (Dreamer.py:255-261), bit 1 the
 * imagination unroll (Dreamer.py:158-164), bit 2 its BPTT (Agent.py:141-145
 * backward).  0 when dims->launch_form is set. */
int dr_persistent_kernels(const dr_dims* d, int B, int T, int H);

/* Philox offset bump (keeps graph replays drawing fresh noise) */
int dr_rng_advance(unsigned long long* rng, unsigned long long delta, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif
