// Persistent posterior scan (scan.hip): the warm start's GRU / latent_mapper /
// sampler chain of all T steps in one launch.
#pragma once
#include "common.h"

#define PSCAN_CNT_BYTES 6400  // counter block (49 counters 128 B apart), a multiple of 16
#ifdef DR_PSCAN_TS
#define PSCAN_TS_BYTES (64 * 24 * 256 * 8)  // stage timestamps (tools/pscan_probe.py)
#else
#define PSCAN_TS_BYTES 0
#endif

// B rows, T >= 2 steps, the reference's widths (hidden 600, latent_mapper 200, 32 x 32 latents)
bool op_pscan_supported(const dr_dims* d, int B, int T, int A);
// caller-owned ring buffers + counters of one launch
size_t op_pscan_ring_bytes(int B);
// z_init = h_init = NULL form of dr_observe_scan.  wt = W_ih^T [L + A][3 hidden]
// (op_transpose); m0h = latent_mapper.0's h-columns (row stride ldm0).  DR_E_UNSUPPORTED when the shape or the stream's CUs do not
// allow every workgroup to be resident (the caller then runs the launch form).
int op_pscan(const dr_dims* d, const dr_world_model* wm, int B, int T, int A, const float* feat, const float* actions,
             long long act_sb, long long act_st, const float* wt, const float* m0h, long long ldm0, dr_noise noise, int step0, float* z_out, float* h_out, float* logits_out,
             void* ring, hipStream_t s);
