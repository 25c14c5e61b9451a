// Fused GRU step with a one-hot latent input (gru.hip).
#pragma once
#include "common.h"

struct alignas(16) GruArgs {
  int B, Hd, R, C, A;
  const int* idx;       // [B][R] sampled class per latent group
  const float* zval;    // [B][R] straight-through latent value at idx
  const float* z;       // the latent rows idx was taken from (row stride ldz), read only for
  long long ldz;        //   groups marked dense (idx < 0: more than one non-zero class)
  const float* a;       // actions [B][A], row stride lda
  long long lda;
  const float* h;       // previous hidden (NULL = zeros), row stride ldh
  long long ldh;
  const float* wt;      // W_ih^T [R*C + A][3*Hd]
  const float* b_ih;
  const float* w_hh;    // [3*Hd][Hd]
  const float* b_hh;
  float* hout;          // row stride ldo; must NOT alias h (other workgroups still read h)
  unsigned short* hout16;  // optional: h' also rounded to bf16 (RNE), row stride ldo (bf16 mode's GemmArgs.A16)
  long long ldo;
  float *sr, *su, *sn, *sghn;  // optional saves [B][Hd] for the backward
  float* gh_ws;                // optional [B][3*Hd] scratch: enables the split path at B >= 128
  int gh_ready;                // split path: gh_ws already holds h W_hh^T + b_hh (computed by the
                               //   caller's grouped launch of the previous step), skip the GEMM
};

int op_gru_fused(const GruArgs& g, hipStream_t s);
// out[m][n] = base[m][n] + sum over the R latent groups of zval[m][u] * wt[u*C + idx[m][u]][n]
// (groups with idx < 0: every class, z[m][u*C + c] * wt[u*C + c][n]).  The latent
// part of a Linear on cat(h, z) with a one-hot z: wt = the z-columns of its weight,
// transposed ([R*C][N], row stride ldw), base = the h-part plus bias.
int op_zgather_add(int M, int N, int R, int C, const int* idx, const float* zval, const float* z, long long ldz,
                   const float* wt, long long ldw, const float* base, long long ldb, float* out, long long ldo,
                   hipStream_t s);
int op_transpose(int rows, int cols, const float* in, float* out, hipStream_t s);
// batched transposes in one launch: out[c * ldo + r] = in[r * cols + c]
struct TransposeJob {
  int rows, cols, ldo;
  const float* in;
  float* out;
};
#define DR_MAX_TJOBS 10
int op_transpose_multi(const TransposeJob* jobs, int n, hipStream_t s);
int op_onehot_index(int M, int R, int C, const float* z, long long ldz, int* idx, float* zval, hipStream_t s);
