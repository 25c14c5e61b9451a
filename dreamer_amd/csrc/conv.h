// NHWC implicit-GEMM encoder convolutions (conv.hip).
#pragma once
#include "common.h"

// k4 s2 p1 conv + bias + SiLU; in NHWC [n][ih][iw][cin], wr [cout][16][cin]
// (op_conv_repack_pad layout); out NHWC [n][ih/2][iw/2][cout] or, with
// out_nchw, [n][cout][ih/2][iw/2] (the encoder's flatten order).
int op_conv_nhwc(int n, int cin, int ih, int iw, int cout, const float* in, const float* wr, const float* bias,
                 float* out, int out_nchw, hipStream_t s);
int op_frames_nhwc4(int n, int nb, int h, int w, const dr_frames* src, float* out, hipStream_t s);
int op_conv_repack_pad(int cout, int cin, int cin_pad, const float* w, float* wr, hipStream_t s);
