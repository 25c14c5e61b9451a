// Generic fused f32 GEMM on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32).
//   Y[m][n] (+)= act( alpha * sum_k opA(m,k) * opB(k,n) + bias[n] + addend[m][n] )
// A operand: row-major [M][K] ("MK", optional 2nd K-segment, optional
// LayerNorm+SiLU applied on load, or conv im2col) or [K][M] ("KM").
// B operand: [N][K] ("NK": Y = A W^T, forward Linear) or [K][N] ("KN":
// Y = A W, backward input-grad / weight-grad), optional 2nd segment.
#pragma once
#include "common.h"

enum { AM_PLAIN = 0, AM_LNSILU = 1, AM_CONV = 2, AM_CONV_SRC = 3, AM_LNBWD = 4, AM_STEBWD = 5 };
// AM_STEBWD (NT skinny only): A = d/d(logits) of the straight-through
// categorical sample (DynamicsPredictors.py:31-40) given dL/dz = A-argument
// rows and the unimixed softmax `pre` rows: per group of C classes,
// a = s * (0.99 g - sum_group(0.99 g * s))  (ops.hip k_softmax_ste_bwd).
// AM_LNBWD (NT skinny only): A = d/d(pre) of SiLU(LayerNorm(pre)) given the
// upstream gradient gx = A-argument rows; the LN input `pre` and gamma/beta
// (ln_g/ln_b) come from the fields below.  a_out receives g_pre, sv_gy /
// sv_xh the SiLU-input gradient and x_hat (for the LayerNorm parameter grads).

struct alignas(16) GemmArgs {
  int M, N, K;
  // A
  const float* A; long long lda;
  const float* A2; long long lda2; int ksplitA;  // MK: k >= ksplitA reads A2[m][k-ksplitA]
  const float* ln_g; const float* ln_b;          // AM_LNSILU (LN width == K)
  float* a_out; long long ld_aout;               // optional copy of the transformed A (n-tile 0 writes)
  const float* pre; long long ld_pre;            // AM_LNBWD: LayerNorm input rows
  float* splitk_ws; long long splitk_floats;     // optional scratch for split-K partials (tile GEMM)
  float* sv_gy; float* sv_xh; long long ld_sv;   // AM_LNBWD: optional saves (n-tile 0 writes)
  // conv im2col (k4 s2 p1), A = NCHW activations [frame][cin][ih][iw]
  int cin, ih, iw, oh, ow;
  dr_frames src;                                 // AM_CONV_SRC: frames, f = t*nb + b
  int nb;
  // B
  const float* W; long long ldb;
  const float* W2; long long ldb2; int ksplitB; int nsplitB;  // KN: k>=ksplitB | n>=nsplitB -> W2
  // epilogue
  const float* bias; const float* addend; long long ld_add;
  float* Y; long long ldy;
  float* Y2; long long ldy2; int nsplitY;        // n >= nsplitY -> Y2[m][n-nsplitY]
  int accumulate, act, out_conv;                 // act 1 = SiLU, 2 = sigmoid; out_conv: Y NCHW [frame][N][oh*ow]
  float alpha;
  // fused epilogues of the skinny kernel (epi != EPI_NONE; Y may be NULL)
  int epi;
  dr_noise noise; int step;
  // EPI_SAMPLE: rows of R groups x C classes -> straight-through one-hot
  int R, C; float unimix;
  float* z_out; long long ldz; int* idx_out; float* soft_out; long long ld_soft;
  float* zval_out;  // optional compact [M][R] straight-through value at idx
  // EPI_ACTOR: columns [mu (A) | log_sig (A)] -> clamp, softplus, tanh(mu + eps*sigma)
  int na, det;
  float* act_out; long long ld_act; float* mu_out; long long ld_mu; float* sig_out; long long ld_sig;
  float* eps_save; float* ls_save; long long ld_ls;
};

enum { EPI_NONE = 0, EPI_SAMPLE = 1, EPI_ACTOR = 2 };

enum GemmLayout { G_NT = 0, G_NN = 1, G_TN = 2 };

GemmArgs gemm_args();  // zero-initialised with neutral defaults
// Launch up to 4 problems sharing layout/A-mode in one dispatch.
int gemm_launch(GemmLayout lay, int amode, const GemmArgs* probs, int count, hipStream_t s);
