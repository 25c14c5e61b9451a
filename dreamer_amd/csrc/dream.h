// Persistent imagination unroll (dream.hip): the H-step actor / GRU / prior /
// sampler chain of dr_imagine_fwd in one launch.
#pragma once
#include "common.h"

#define PDREAM_CNT_BYTES (7 * 16 * 32 * 4)  // [stage 0..5, status][16-row block][32 words apart]
#ifdef DR_PDREAM_TS
#define PDREAM_TS_BYTES (16 * 6 * 8 * 256 * 8)  // stage timestamps (tools/pdream_probe.py)
#else
#define PDREAM_TS_BYTES 0
#endif

// the tape regions the unroll writes (engine.hip Tape)
struct PDreamTape {
  float *eps, *ls_raw, *pre1a, *x1a, *pre2a, *x2a, *r, *u, *n, *ghn, *pre1p, *pre2p, *soft;
};

// the reference's widths (hidden 600, 32 x 32 latents, 200-wide prior / actor
// layers), 1 <= A <= 8, B <= 128 (shape only: the workspace is sized by it)
bool op_pdream_shape_ok(const dr_dims* d, int B, int H, int A);
// shape_ok and not d->launch_form
bool op_pdream_supported(const dr_dims* d, int B, int H, int A);
// workspace of one launch (0 where the shape is not covered)
size_t op_pdream_ws_bytes(const dr_dims* d, int B, int H);
// latents[:, 0] / hiddens[:, 0] hold z_0 / h_0; idx0 = op_onehot_index of z_0
// ([B][R] classes, then [B][R] values); wt = W_ih^T, wazt = the actor's
// base_net.0 z-columns transposed ([L][actor_h1]); nq = the Categorical draws'
// noise.  Writes latents / hiddens [:, 1..H], actions, mus, sigmas and the tape.
// DR_E_UNSUPPORTED when the shape or the stream's CUs do not allow every
// workgroup to be resident (the caller then runs the launch form).
int op_pdream(const dr_dims* d, const dr_world_model* wm, const dr_actor* ac, int B, int H, const float* wt,
              const float* wazt, const int* idx0, dr_noise noise, dr_noise nq, int det, float* latents, float* hiddens,
              float* actions, float* mus, float* sigmas, const PDreamTape& tp, void* ws, hipStream_t s);
