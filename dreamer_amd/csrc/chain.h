// Fused per-step kernels of the imagination chain (chain.hip).
#pragma once
#include "common.h"

// The actor for one imagined step after the sampler (Agent.py:191-210 on
// cat(h, z) with a one-hot z), in ONE launch:
//   pre1 = hpart + sum over the R groups of zval * wzt[u*C + idx]   (base_net.0)
//   x1 = SiLU(LN(pre1)); pre2 = x1 W3^T + b3; x2 = SiLU(LN(pre2))   (base_net.1-5)
//   [mu | log_sig] = x2 Wst^T + bst; a = tanh(mu + eps sigma)        (heads, Agent.py:202-210)
// hpart = the h-part of base_net.0 plus its bias (computed beside the prior's
// first layer); pre1 / x1 / pre2 / x2 / eps / raw log_sig are the tape the
// BPTT reads.
struct alignas(16) ActorTailArgs {
  int M, A, a1, a2, R, C, step, det;
  const int* idx;       // [M][R] sampled class per group
  const float* zval;    // [M][R] straight-through value at idx
  const float* z;       // the latent rows (row stride ldz): groups marked dense (idx < 0) sum every class
  long long ldz;
  const float* wzt;     // z-columns of base_net.0 transposed [R*C][a1] (row stride ldw)
  long long ldw;
  const float* hpart;   // [M][a1] (row stride ldh)
  long long ldh;
  const float *n1g, *n1b, *w3, *b3, *n4g, *n4b;  // base_net.1 / .3 ([a2][a1]) / .4
  const float *wmu, *bmu, *wls, *bls;            // mu_head / log_sig_head: [A][a2], [A]
  float* pre1; float* x1; long long ld1;         // tape rows (stride ld1)
  float* pre2; float* x2; long long ld2;
  dr_noise noise;
  float* act; float* mu; float* sig; long long ldA;  // outputs [M] x A (row stride ldA)
  float* eps_save;      // [M][A] (may be NULL)
  float* ls_save;       // raw log_sig, row stride ldA (may be NULL)
};
bool op_actor_tail_ok(const ActorTailArgs& a);
int op_actor_tail(const ActorTailArgs& a, hipStream_t s);

// The actor's backward for one imagined step (Agent.py:191-210, backward), in
// ONE launch up to the input gradient of base_net.0:
//   heads: g_mu = dL/dmu + g_a (1 - a^2), g_ls through clamp + softplus      (saved: gheads)
//   gx2 = [g_mu | g_ls] [W_mu; W_ls];  g_pre2 = LN-SiLU backward (pre2, n4)     (saved: gpre2, gy2, xh2)
//   gx1 = g_pre2 W3;                   g_pre1 = LN-SiLU backward (pre1, n1)     (saved: gpre1, gy1, xh1)
// The caller then runs the input-gradient GEMM of base_net.0 on g_pre1.
struct alignas(16) ActorTailBwdArgs {
  int M, A, a1, a2;
  const float* g_a; long long ldga;        // dL/da through the GRU (may be NULL)
  const float *g_mu, *g_sig; long long ldgl;  // direct dL/dmu, dL/dsigma (may be NULL)
  const float* act; long long ldact;       // the actions (tanh outputs)
  const float* ls_raw; long long ldl;      // raw log_sig head outputs
  const float* eps;                        // [M][A] rsample noise
  const float *wmu, *wls;                  // mu_head / log_sig_head weights [A][a2]
  float* gheads; long long ldh;            // [M] x 2A save
  const float* pre2; long long ld2;        // base_net.3 output rows (LN4 input)
  const float *n4g, *n4b;
  float *gpre2, *gy2, *xh2;                // saves, row stride ld2
  const float* w3t;                        // base_net.3 weight transposed [a1][a2]
  const float* pre1; long long ld1;        // base_net.0 output rows (LN1 input)
  const float *n1g, *n1b;
  float *gpre1, *gy1, *xh1;                // saves, row stride ld1
};
bool op_actor_tail_bwd_ok(const ActorTailBwdArgs& a);
int op_actor_tail_bwd(const ActorTailBwdArgs& a, hipStream_t s);
