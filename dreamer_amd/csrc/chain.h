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
