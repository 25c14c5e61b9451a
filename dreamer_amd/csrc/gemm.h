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

// Fused GRU backward (SequenceModel.py:19-24 -> torch gru_cell) on the FINAL
// value of an accumulated hidden-state gradient g = dL/dh' (the last GEMM that
// adds into it, engine.hip's BPTT): for output (m, j < Hd) the epilogue writes
// gi[m][{r,u,n}] / gh[m][{r,u,n}] and adds dL/dh through h' = (h - n) u + n to
// ho[m][j] -- ops.hip k_gru_bwd's arithmetic, one launch fewer per BPTT step.
struct GruBwdEpi {
  const float* h; long long ldh;        // h (NULL = zeros)
  const float *r, *u, *n, *ghn;          // forward saves [M][Hd]
  float *gi, *gh;                        // [M][3 Hd]
  float* ho; long long ldo;              // dL/dh (+=)
  int Hd, pad_;
  unsigned short *gi16, *gh16;           // optional bf16 (RNE) copies of gi / gh (bf16 mode's GemmArgs.A16)
};

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
  // bf16 perf mode (dr_dims.precision): NT products that take the tile route
  // run on v_mfma_f32_16x16x32_bf16 with operands rounded to bf16 as they are
  // staged (f32 accumulation, f32 in / out); set by the engine per call
  int bf16;
  GruBwdEpi gb;  // gb.Hd > 0: fused GRU backward on the stored values (see GruBwdEpi)
  // NT B operand also given as bf16 planes [K/32][3][wsplit_np][32] (conv.h
  // op_nt_repack_split3 of W): per-step chain products then run on the bf16
  // MFMA -- f32-accurate 3-term split (fp32 mode) or plane 0 alone (bf16 mode)
  const unsigned short* wsplit; int wsplit_np, pad2_;
  // bf16 mode: A also given rounded to bf16 (RNE, row stride lda) by its
  // producer -- k_gemm_wks3<1> then loads 8 bf16 per lane instead of 8 f32 and
  // skips the rounding (bitwise the same products)
  const unsigned short* A16;
};

enum { EPI_NONE = 0, EPI_SAMPLE = 1, EPI_ACTOR = 2 };

enum GemmLayout { G_NT = 0, G_NN = 1, G_TN = 2 };

GemmArgs gemm_args();  // zero-initialised with neutral defaults
// While alive, gemm_args() returns bf16 = on (the engine's bf16 perf mode
// around the imagination-epoch entry points); restores the previous value.
struct GemmBf16Scope {
  explicit GemmBf16Scope(bool on);
  ~GemmBf16Scope();
  int prev;
};
// Launch up to 4 problems sharing layout/A-mode in one dispatch.
int gemm_launch(GemmLayout lay, int amode, const GemmArgs* probs, int count, hipStream_t s);
// true when AM_LNBWD / AM_STEBWD problems run on 16-row skinny tiles (K <= 1024)
bool gemm_bwd_rows16(const GemmArgs* p, int count);

// The tail of the reference's 3-layer heads (Linear, LN, SiLU, Linear, LN,
// SiLU, Linear -- DynamicsPredictors.py:15-23, Agent.py:180-190) from the
// first Linear's output X on, in ONE launch:
//   y1 = SiLU(LN1(X)); h2 = y1 W3^T + b3; y2 = SiLU(LN4(h2)); out = y2 W6^T + b6
// followed by `e`'s epilogue (plain / activation store to e.Y, or EPI_SAMPLE,
// or EPI_ACTOR).  A workgroup owns 16 rows x 128 output columns and computes
// y1, h2, y2 for its rows itself (the two small layers are recomputed by
// each column block instead of a grid-wide seam).  K1, K2 <= 256.
struct alignas(16) Mlp2Args {
  int M, K1, K2, pad_;
  const float* X; long long ldx;     // [M][K1] first Linear's output (pre-LN1)
  const float* ln1_g; const float* ln1_b;
  const float* W3; const float* b3;  // [K2][K1]
  const float* ln4_g; const float* ln4_b;
  float* a1_out; long long ld_a1;    // optional y1 (column block 0 writes)
  float* pre2; long long ld_pre2;    // optional h2
  float* a2_out; long long ld_a2;    // optional y2
  GemmArgs e;                        // last Linear: e.N, e.W [N][K2] (e.ldb), e.bias, epilogue
};
int mlp2_launch(const Mlp2Args* probs, int count, hipStream_t s);
