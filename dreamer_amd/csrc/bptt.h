// Persistent BPTT (bptt.hip): the reverse loop of dr_imagine_bwd -- the
// H-step backward through the prior, the GRU and the actor -- in one launch.
#pragma once
#include "common.h"

#define PBPTT_CNT_BYTES (8 * 8 * 32 * 4)  // [stage Q1..Q7, status][16-row block][32 words apart]
#ifdef DR_PBPTT_TS
#define PBPTT_TS_BYTES (16 * 7 * 8 * 256 * 8)  // stage timestamps (tools/pbptt_probe.py)
#else
#define PBPTT_TS_BYTES 0
#endif

// operands of one launch (engine.hip imagine_bwd_impl's names)
struct PBpttIO {
  // transposed weights (the backward prologue's op_transpose_multi)
  const float *tl6p, *tl3p, *tl0p, *wt, *twhh, *thead, *tl3a, *tl0a;
  // the forward tape, states and upstream gradients
  const float *soft, *pre2p, *pre1p, *r, *u, *n, *ghn, *pre2a, *pre1a, *ls_raw, *eps;
  const float *hiddens, *actions, *g_mus, *g_sigmas;
  const float *gH, *gZ, *gA;  // [B][H+1][hidden], [B][H+1][L], [B][H][A] (copied / zeroed by the prologue)
  // saves for the actor weight gradients
  float *gheads, *gpre2a, *gy2a, *xh2a, *gpre1a, *gy1a, *xh1a;
};

// the reference's widths (hidden 600, 32 x 32 latents, 200-wide prior / actor
// layers), 1 <= A <= 8, 16 <= B <= 64, B % 16 == 0 (shape only)
bool op_pbptt_shape_ok(const dr_dims* d, int B, int H, int A);
bool op_pbptt_supported(const dr_dims* d, int B, int H, int A);  // shape_ok and not d->launch_form
size_t op_pbptt_ws_bytes(const dr_dims* d, int B, int H);       // 0 where the shape is not covered
// DR_E_UNSUPPORTED when not every workgroup can be resident on the stream's CUs
int op_pbptt(const dr_dims* d, const dr_world_model* wm, const dr_actor* ac, int B, int H, const PBpttIO& io, void* ws,
             hipStream_t s);
