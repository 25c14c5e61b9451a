// NHWC implicit-GEMM convolutions: the encoder's Conv2d stack (conv.hip) and
// the world-model training step's transposed convolutions, conv data
// gradients and weight gradients (wmconv.hip).
#pragma once
#include "common.h"

// k4 s2 p1 conv + bias + SiLU; in NHWC [n][ih][iw][cin], wr [cout][16][cin]
// (op_conv_repack_pad layout); out NHWC [n][ih/2][iw/2][cout] or, with
// out_nchw, [n][cout][ih/2][iw/2] (the encoder's flatten order).
int op_conv_nhwc(int n, int cin, int ih, int iw, int cout, const float* in, const float* wr, const float* bias,
                 float* out, int out_nchw, hipStream_t s);
enum { CONV_EPI_FWD = 0, CONV_EPI_DSILU = 1 };
// as op_conv_nhwc, plus: pre (optional with CONV_EPI_FWD) receives acc + bias
// in NHWC; CONV_EPI_DSILU writes acc * SiLU'(pre) (no bias, NHWC out) and, with
// csum, each 128-pixel tile's per-channel sums of that output:
// csum[tile][cout], tiles = ceil(n * oh * ow / 128) (op_chan_sum_final reduces them).
int op_conv_nhwc_ex(int n, int cin, int ih, int iw, int cout, const float* in, const float* wr, const float* bias,
                    float* out, int out_nchw, float* pre, int epi, hipStream_t s, float* csum = nullptr);
int op_frames_nhwc4(int n, int nb, int h, int w, const dr_frames* src, float* out, hipStream_t s, float pad = 0.0f);
// first conv straight from the frames (u8 ring or f32 tensor): the frame rows
// a tile reads are normalised into LDS once, no NHWC4 f32 copy in HBM.  Same
// fragments and MFMA order as op_frames_nhwc4 + k_conv1_direct: bitwise equal.
// Returns DR_E_INVALID (nothing launched) for shapes it does not tile.
int op_conv1_frames(int n, int nb, int ih, int iw, int cout, const dr_frames* src, const float* wr, const float* bias,
                    float* out, hipStream_t s);
int op_conv_repack_pad(int cout, int cin, int cin_pad, const float* w, float* wr, hipStream_t s);

// ---- conv_split.hip (fp32-accurate convs on the bf16 MFMA: 3-term split) ----
// weights: Conv2d [co][ci][4][4] f32 -> 3 bf16 planes [3][co][16][cin] (6 bytes per weight)
int op_conv_repack_split3(int cout, int cin, const float* w, void* wr, hipStream_t s);
bool op_conv_split3_supported(int n, int cin, int ih, int iw, int cout);
// bf16 perf mode's conv3..: the split-conv tiling with one bf16 term (bf16 NHWC in,
// bf16 NHWC / NCHW out, weights in op_conv_repack_split3 planes)
// bf16 perf mode's conv1 + conv2: k_enc12_split3 with one bf16 term (64 x 64,
// 32 -> 64 channels, u8 ring only; DR_E_INVALID, nothing launched, otherwise)
int op_enc12_s1_bf16(int n, int nb, int h, int w, int c1, int c2, const dr_frames* src, const float* w1,
                     const float* b1, const float* w2, const float* b2, void* wr1, void* wr2, void* out,
                     hipStream_t s, int prepacked = 0);
int op_conv_s1_bf16(int n, int cin, int ih, int iw, int cout, const void* in, const void* wr, const float* bias,
                    void* out, int out_nchw, hipStream_t s);
// the same convolution with LDS-DMA staged operands, four stages deep (conv_glds.hip; cout % 128 == 0)
bool op_conv_glds_bf16_supported(int n, int cin, int ih, int iw, int cout);
// fp32 (six split3 products) on the LDS-DMA staging: f32 NHWC in, CONV_EPI_FWD / CONV_EPI_DSILU epilogues
bool op_conv_glds_s3_supported(int n, int cin, int ih, int iw, int cout);
int op_conv_glds_s3(int n, int cin, int ih, int iw, int cout, const float* in, const void* wr, const float* bias,
                    float* out, int out_nchw, float* pre, int epi, hipStream_t s);
// bf16 NT GEMM Y = X W^T + bias (X [M][K], W [N][K] bf16; K % 32 == 0, N % 4 == 0) on the same
// LDS-DMA pipeline with split-K; part: op_gemm_nt_glds_part_floats(M, N, K) floats (may be 0)
size_t op_gemm_nt_glds_part_floats(int M, int N, int K);
int op_gemm_nt_glds_bf16(int M, int N, int K, const void* X, int ldx, const void* W, int ldw, const float* bias,
                         float* Y, int ldy, float* part, size_t part_floats, hipStream_t s);
int op_conv_glds_bf16(int n, int cin, int ih, int iw, int cout, const void* in, const void* wr, const float* bias,
                      void* out, int out_nchw, hipStream_t s);
// k4 s2 p1 conv + bias + SiLU, f32 NHWC in -> f32 NHWC (or NCHW) out, as op_conv_nhwc
int op_conv_split3(int n, int cin, int ih, int iw, int cout, const float* in, const void* wr, const float* bias,
                   float* out, int out_nchw, hipStream_t s);
// with the world-model step's epilogues (as op_conv_nhwc_ex): CONV_EPI_FWD +
// optional pre = acc + bias (NHWC), or CONV_EPI_DSILU: out = acc * SiLU'(pre).
// terms = 1: the bf16 world-model step's form (activations RNE-rounded to one
// bf16 term as they are staged, the weights' first plane = their RNE bf16, one
// MFMA per block; f32 in / out and the same epilogues)
int op_conv_split3_ex(int n, int cin, int ih, int iw, int cout, const float* in, const void* wr, const float* bias,
                      float* out, int out_nchw, float* pre, int epi, hipStream_t s, int terms = 3);

// tall NT products f32-accurate on the bf16 MFMA (conv_split.hip):
// Y = act(A W^T + bias), A [M][K] row-major with an optional second K segment
// (A2 at k >= ksA, ksA % 4 == 0), W pre-split by op_nt_repack_split3 into a
// scratch of op_nt_split3_ws_bytes(N, K); N % 4 == 0, K % 4 == 0, act 1 = SiLU
size_t op_nt_split3_ws_bytes(int N, int K);
int op_nt_repack_split3(int N, int K, const float* W, int ldw, void* wr, hipStream_t s);
bool op_gemm_nt_split3_supported(int M, int N, int K, const float* A, int lda, const float* A2, int lda2, int ksA,
                                 int ldy);
int op_gemm_nt_split3(int M, int N, int K, const float* A, int lda, const float* A2, int lda2, int ksA, const void* wr,
                      const float* bias, int act, float* Y, int ldy, hipStream_t s);
// the same with split-K partial sums in `part` (op_gemm_nt_split3_part_floats(M, N) floats,
// 16-byte aligned) when the tile grid alone leaves the chip under-filled
size_t op_gemm_nt_split3_part_floats(int M, int N);
// splits_fixed > 0: that many K splits whatever M is (the sums then do not
// depend on M: the time-chunked encoder equals the whole-window one bit for bit)
int op_gemm_nt_split3_sk(int M, int N, int K, const float* A, int lda, const float* A2, int lda2, int ksA,
                         const void* wr, const float* bias, int act, float* Y, int ldy, float* part,
                         size_t part_floats, hipStream_t s, int splits_fixed = 0);
// ... with Y += (accumulate) and columns n >= nsplitY stored to Y2 (the data-gradient products)
int op_gemm_nt_split3_ex(int M, int N, int K, const float* A, int lda, const float* A2, int lda2, int ksA,
                         const void* wr, const float* bias, int act, float* Y, int ldy, int accumulate, float* Y2,
                         int ldy2, int nsplitY, float* part, size_t part_floats, hipStream_t s, int splits_fixed = 0);

// ---- conv_bf16.hip (bf16 perf mode; activations bf16, accumulation f32) ----
// weights: Conv2d [co][ci][4][4] f32 -> bf16 [co][tap][cin_pad]; matrix slice -> bf16 [rows][cols]
int op_conv_repack_bf16(int cout, int cin, int cin_pad, const float* w, void* wr, hipStream_t s);
int op_to_bf16_2d(int rows, int cols, const float* x, long long ld, void* y, hipStream_t s);
// first conv from the frames (u8 ring or f32): out bf16 NHWC [n][h/2][w/2][cout]; wr cin_pad = 4
int op_conv1_bf16(int n, int nb, int h, int w, int cout, const dr_frames* src, const void* wr, const float* bias,
                  void* out, hipStream_t s);
// conv1 + conv2 fused (c1 = 32, c2 = 64, square 64 / 128 frames); DR_E_INVALID = shape not covered
// conv1 + conv2 (32 -> 64 channels, 64 x 64 frames from the u8 ring), f32-accurate
// (conv_split.hip); repacks both weights into wr1 (3 x cout1 x 64 bf16) and wr2
// (op_conv_repack_split3); DR_E_INVALID (nothing launched) for other shapes/sources
// prepacked = 1: wr1 / wr2 already hold the planes (op_repack_multi), no repack launched
bool op_enc12_split3_ok(int n, int h, int w, int c1, int c2, const dr_frames* src);
int op_enc12_split3(int n, int nb, int h, int w, int c1, int c2, const dr_frames* src, const float* w1,
                    const float* b1, const float* w2, const float* b2, void* wr1, void* wr2, float* out,
                    hipStream_t s, int prepacked = 0);
// the same with the world-model step's saves (NHWC f32, pre0 / a0 together or
// neither): conv1's pre-activation and output, conv2's pre-activation
int op_enc12_split3_ex(int n, int nb, int h, int w, int c1, int c2, const dr_frames* src, const float* w1,
                       const float* b1, const float* w2, const float* b2, void* wr1, void* wr2, float* out,
                       float* pre0, float* a0, float* pre1, hipStream_t s, int terms = 3, int prepacked = 0);
// several weight repacks in one launch: conv1 planes (op_enc12_split3's wr1),
// conv planes (op_conv_repack_split3), NT planes (op_nt_repack_split3), bf16
// copy (op_to_bf16_2d) -- the same element code as those ops
enum { RJ_CONV1 = 0, RJ_CONV = 1, RJ_NT = 2, RJ_BF16 = 3 };
struct RepackJob {
  int kind, a, b, c;  // conv1: cout; conv: cout, cin; nt: N, K, Np; bf16: rows, cols
  const float* w;
  void* out;
  long long ld;       // nt: ldw; bf16: row stride
  long long total;    // elements of the job
};
#define DR_RJ_MAX 6
RepackJob rj_conv1(int cout, const float* w, void* wr);
RepackJob rj_conv(int cout, int cin, const float* w, void* wr);
RepackJob rj_nt(int N, int K, const float* W, int ldw, void* wr);
RepackJob rj_bf16(int rows, int cols, const float* x, long long ld, void* y);
int op_repack_multi(const RepackJob* jobs, int n, hipStream_t s);
int op_enc12_bf16(int n, int nb, int h, int w, int c1, int c2, const dr_frames* src, const void* wr1, const float* b1,
                  const void* wr2, const float* b2, void* out, hipStream_t s);
// k4 s2 p1 conv + bias + SiLU, bf16 NHWC in -> bf16 NHWC (or NCHW) out
int op_conv_bf16(int n, int cin, int ih, int iw, int cout, const void* in, const void* wr, const float* bias,
                 void* out, int out_nchw, hipStream_t s);
// Y (f32) = X W^T + bias with X [M][K], W [N][K] bf16
int op_gemm_nt_bf16(int M, int N, int K, const void* X, int ldx, const void* W, const float* bias, float* Y, int ldy,
                    hipStream_t s);

// ---- wmconv.hip -------------------------------------------------------------
// Upsampling k4 s2 p1 (ConvTranspose2d, or the data gradient of a Conv2d):
//   out[f][Y][X][co] = sum_{ci, (y,ky): Y = 2y-1+ky, (x,kx): X = 2x-1+kx} in[f][y][x][ci] * wt[ci][co][ky][kx]
// in NHWC [n][h][w][cin]; wt in ConvTranspose2d layout [cin][cout][4][4] (a
// Conv2d weight [co][ci][4][4] read as [cin=co][cout=ci] gives the Conv2d
// input gradient).  wq = op_convT_repack(wt) scratch [4 parity classes][cout][4 taps][cin].
enum { CT_EPI_BIAS = 0, CT_EPI_DSILU = 1, CT_EPI_TANH_MSE = 2 };
struct ConvTArgs {
  int n, cin, h, w, cout;
  const float* in;
  int silu_in;          // apply SiLU to `in` on load (in holds pre-activations)
  const float* wq;
  const float* bias;    // CT_EPI_BIAS / CT_EPI_TANH_MSE
  float* out;           // NHWC [n][2h][2w][ldc]
  float* out2;          // CT_EPI_BIAS: optional SiLU(acc + bias) (same layout), for the consumers
  int silu_out;         // CT_EPI_BIAS: out receives SiLU(acc + bias) instead of acc + bias
  int ldc;              // channel stride of out (>= cout; extra channels written as 0)
  const float* pre;     // CT_EPI_DSILU: out = acc * SiLU'(pre) (pre NHWC, stride cout)
  // CT_EPI_TANH_MSE: mu = tanh(acc + bias); err = mu - target; out = coef[f] * err * (1 - mu^2)
  // (the gradient wrt the pre-tanh value); part[f * nparts + j] = sum err^2 over tile j of frame f
  const float* target;  // NHWC [n][2h][2w][tstride]
  int tstride;
  const float* coef;    // [n]
  float* part;          // [n][parts_per_frame()]
  float* bpart;         // CT_EPI_TANH_MSE, optional: [n][parts_per_frame()][3] sums of out (bias-gradient partials)
};
int op_convT_repack(int cin, int cout, const float* wt, float* wq, hipStream_t s);
int op_convT_nhwc(int epi, const ConvTArgs& a, hipStream_t s);
int op_convT_mse_parts(int h, int w);  // partial sums per frame written by CT_EPI_TANH_MSE
// CT_EPI_TANH_MSE runs a direct VALU kernel (cout = 3): wq must come from
// op_convT_out3_repack ([ci][4 classes][4 taps][3]), out has ldc = 4
int op_convT_out3_repack(int cin, const float* wt, float* wq, hipStream_t s);
// the same direct kernel; target == NULL: mu = tanh(acc + bias) written NCHW [n][3][2h][2w]
int op_convT_out3(const ConvTArgs& a, hipStream_t s);
// conv_split.hip: the same upsampling conv f32-accurate on the bf16 MFMA (3-term
// split) for CT_EPI_BIAS / CT_EPI_DSILU, NHWC out with ldc == cout, no silu_in;
// wr = op_convT_repack_split3(wt) scratch, 6 bytes per weight
int op_convT_repack_split3(int cin, int cout, const float* wt, void* wr, hipStream_t s);
// terms = 1: the bf16 world-model step's one-term form (as op_conv_split3_ex),
// which also covers cout = 32
bool op_convT_split3_supported(int n, int cin, int h, int w, int cout, int terms = 3);
// the all-parity-class form op_convT_split3 takes for 64 -> 32 channels (8 x 16 anchor tiles)
bool op_convT_cls_supported(int n, int cin, int h, int w, int cout);
int op_convT_split3(int epi, const ConvTArgs& a, const void* wr, hipStream_t s, int terms = 3);
// the six-product form on the LDS-DMA ping-pong kernel (conv_glds.hip), taken by op_convT_split3 where it applies
bool op_convT_glds_s3_supported(const ConvTArgs& a, int epi);
int op_convT_glds_s3(int epi, const ConvTArgs& a, const void* wr, hipStream_t s);

// Weight gradient of a k4 s2 p1 (transposed) convolution:
//   dW[a][b][ky][kx] (+)= scale * sum_{f,y,x} lo[f][y][x][a] * hi[f][2y-1+ky][2x-1+kx][b]
// lo NHWC [n][h][w][ca] (stride lda), hi NHWC [n][2h][2w][cb] (stride ldb).
// Conv2d: lo = output gradient, hi = input -> dW [cout][cin][4][4];
// ConvTranspose2d: lo = input, hi = output gradient -> dW [cin][cout][4][4].
// lo_silu: lo holds pre-activations, SiLU is applied on load.
size_t op_conv_wgrad_ws_floats(int n, int h, int w, int ca, int cb);
// the ordered partial-plane reduction of both weight-gradient kernels
int op_wgrad_reduce(int ca, int cb, int cbo, int nsplit, const float* part, float* dw, float scale, int accumulate,
                    hipStream_t s);
// conv_split.hip: the same weight gradient f32-accurate on the bf16 MFMA (both
// operands split3 while staged); ca in {64, 128, 256}, cb % 8 == 0, h and w
// powers of two, lo without SiLU on load
bool op_wgrad_split3_supported(int n, int h, int w, int ca, int cb, int terms = 3);  // terms 1: also ca = 32
size_t op_wgrad_split3_ws_floats(int n, int h, int w, int ca, int cb);
// terms = 1: both operands RNE-rounded to one bf16 term (bf16 world-model step)
int op_wgrad_split3(int n, int h, int w, int ca, int cb, const float* lo, int lda, const float* hi, int ldb,
                    float* dw, int cbo, float scale, int accumulate, float* ws, size_t ws_floats, hipStream_t s,
                    int terms = 3);
// dW has cbo <= cb channels per row (cbo < cb when hi carries zero padding channels).
// bias_out (optional): hi's channel cbo is a pad of ones (op_frames_nhwc4 pad = 1),
// so its tap-(1, 1) column is sum_k lo[k][a]: bias_out[a] (+)= scale * that.
int op_conv_wgrad(int n, int h, int w, int ca, int cb, const float* lo, int lda, int lo_silu, const float* hi, int ldb,
                  float* dw, int cbo, float scale, int accumulate, float* ws, size_t ws_floats, hipStream_t s,
                  float* bias_out = nullptr);
// out[c] (+)= sum_r X[r][c] for c < C (row stride ldx); two deterministic passes
size_t op_chan_sum_ws_floats(long long rows, int C);
int op_chan_sum(long long rows, int C, const float* X, int ldx, float* out, int accumulate, float* ws, size_t ws_floats,
                hipStream_t s);
// out[c] (+)= sum_b part[b][c] over nb partial rows (fixed order)
int op_chan_sum_final(int nb, int C, const float* part, float* out, int accumulate, hipStream_t s);

// TN products dW[m][n] = sum_k G[k][m] X[k][n] (Linear weight gradients over
// K rows; X columns n >= nsplitB from X2[k][n - nsplitB]) f32-accurate on the
// bf16 MFMA: both operands split3 once into planes, then a pre-split GEMM
// (conv_split.hip).  Y (+)= dW with row stride ldy.
size_t op_gemm_tn_split3_ws_bytes(int M, int N, int K);
// shape / size limits of op_gemm_tn_split3 (32-bit plane offsets): callers
// route problems it rejects to the f32 tile GEMM instead
bool op_gemm_tn_split3_supported(int M, int N, int K);
int op_gemm_tn_split3(int M, int N, int K, const float* G, long long ldg, const float* X, long long ldx,
                      const float* X2, long long ldx2, int nsplitB, float* Y, long long ldy, int accumulate, void* ws,
                      size_t ws_bytes, hipStream_t s, int terms = 3);  // terms = 1: RNE bf16 operands (bf16 WM step)
// up to 4 such problems in one launch per pass (repack / products / finish),
// each with its own scratch carved in order from `ws`; bitwise equal to
// running them one after another
struct TnProblem {
  int M, N, K;
  const float* G;
  long long ldg;
  const float* X;
  long long ldx;
  const float* X2;
  long long ldx2;
  int nsplitB;
  float* Y;
  long long ldy;
  int accumulate;
};
size_t op_gemm_tn_split3_multi_ws_bytes(const TnProblem* p, int n);
int op_gemm_tn_split3_multi(const TnProblem* p, int n, void* ws, size_t ws_bytes, hipStream_t s, int terms);
