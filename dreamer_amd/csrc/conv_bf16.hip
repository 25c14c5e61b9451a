// bf16 perf mode of the encoder (VariationalAutoEncoder.py:33-42 + latent_mapper.0
// feature columns, VAE.py:57-75): bf16 operands on the gfx950 bf16 MFMA
// (v_mfma_f32_16x16x32_bf16, 16x the f32 MFMA rate), f32 accumulation, bias and
// SiLU in f32, activations stored as bf16 NHWC (half the HBM bytes of the f32
// path).  The fp32 parity mode (conv.hip) is untouched.
//
//   k_conv1_bf16   frames (u8 ring or f32) -> x/255 - 0.5 -> conv1 + SiLU, read
//                  straight from the replay ring: a 4-output-row tile stages its
//                  10 input rows in LDS as bf16 [row][col][4 ch] so every MFMA
//                  B fragment (2 taps x 4 channels of one pixel) is one 16-byte
//                  LDS read; no f32 NHWC4 copy of the frames is materialised.
//   k_conv_bf16    conv2..4 as NHWC implicit GEMMs (and a dense NT mode for the
//                  feature projection): 64-k chunks staged global -> registers
//                  -> LDS (two buffers, loads PIPE chunks ahead), 16-byte units
//                  XOR-swizzled by row (unit ^ row&7) so the ds_read_b128
//                  fragment reads of every 16-lane group hit 16 distinct bank
//                  quads; each wave owns a 64 x 64 output tile (4 x 4 MFMA tiles).
//
// MFMA operand order is chosen by the output layout (as in conv.hip): weights
// as the A operand give each lane 4 consecutive channels of one pixel (one
// 8-byte NHWC store); pixels as A give 4 consecutive pixels of one channel
// (NCHW, the flatten order that feeds the projection).
#include "conv.h"

#include <algorithm>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

__device__ __forceinline__ u16 dr_bf16(float f) { return __builtin_bit_cast(u16, (__bf16)f); }  // RNE
__device__ __forceinline__ uint2 dr_pack_bf16x4(float a, float b, float c, float d) {
  const bf16x4 v = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
  return __builtin_bit_cast(uint2, v);
}
__device__ __forceinline__ f32x4 dr_mfma_bf16(uint4 a, uint4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                  0, 0);
}

// ---------------------------------------------------------------------------
// first layer: frames -> NHWC bf16 [n][h/2][w/2][cout]
// ---------------------------------------------------------------------------
#define C1_OR 8          // output rows per workgroup (2 per wave)
#define C1_IR (2 * C1_OR + 2)
#define C1_MAXW 256

template <int FN>  // cout = 16 * FN
__global__ __launch_bounds__(256) void k_conv1_bf16(int n, int nb, int h, int w, dr_frames src,
                                                    const u16* __restrict__ wr, const float* __restrict__ bias,
                                                    u16* __restrict__ out) {
  constexpr int COUT = 16 * FN;
  constexpr int LW = C1_MAXW + 2;
  __shared__ __attribute__((aligned(16))) uint2 xin[C1_IR][LW];  // [input row][x + 1][4 ch] bf16
  const int ow = w / 2, oh = h / 2;
  const int tiles_y = oh / C1_OR;
  const int f = blockIdx.x / tiles_y, ty = blockIdx.x - f * tiles_y;
  if (f >= n) return;
  const int oy0 = ty * C1_OR, iy0 = 2 * oy0 - 1;
  const int tid = threadIdx.x;
  const int W2 = w + 2;
  // weights and bias first: their latency overlaps the frame staging
  const int wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;
  uint4 wa[2][FN];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < FN; ++j)
      wa[s][j] = *reinterpret_cast<const uint4*>(wr + (16 * j + r) * 64 + 32 * s + 8 * q);
  float bv[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[j][e] = bias[16 * j + 4 * q + e];
  // zero the tile (borders, rows outside the frame, channel 3)
  for (int i = tid; i < C1_IR * W2; i += 256) {
    const int rr = i / W2;
    xin[rr][i - rr * W2] = make_uint2(0u, 0u);
  }
  const unsigned hw = (unsigned)(h * w);
  const int b = f % nb, t = f / nb + src.t0;
  const unsigned char* fr8 = nullptr;
  const float* fr32 = nullptr;
  if (src.ring) fr8 = src.ring + ((src.starts[b] + t) % src.ring_cap) * 3 * (long long)hw;
  else fr32 = src.obs + (long long)b * src.stride_b + (long long)t * src.stride_t;
  const int w4 = w >> 2, per_c = C1_IR * w4;
  // issue every load of the tile before the first LDS write
  constexpr int MAXI = (3 * C1_IR * (C1_MAXW / 4) + 255) / 256;
  float v[MAXI][4];
#pragma unroll
  for (int k = 0; k < MAXI; ++k) {
    const int i = tid + 256 * k;
    const int c = i / per_c, rem = i - c * per_c, rr = rem / w4, x4 = rem - rr * w4;
    const int y = iy0 + rr;
    const bool ok = i < 3 * per_c && y >= 0 && y < h;
    const unsigned off = ok ? (unsigned)c * hw + (unsigned)(y * w + 4 * x4) : 0u;
    if (fr8) {
      const unsigned u = ok ? *reinterpret_cast<const unsigned*>(fr8 + off) : 0u;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[k][e] = (float)((u >> (8 * e)) & 255u);
    } else {
      const float4 qv = ok ? *reinterpret_cast<const float4*>(fr32 + off) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[k][0] = qv.x; v[k][1] = qv.y; v[k][2] = qv.z; v[k][3] = qv.w;
    }
  }
  __syncthreads();  // zero fill done
  u16* xs = reinterpret_cast<u16*>(&xin[0][0]);
#pragma unroll
  for (int k = 0; k < MAXI; ++k) {
    const int i = tid + 256 * k;
    const int c = i / per_c, rem = i - c * per_c, rr = rem / w4, x4 = rem - rr * w4;
    const int y = iy0 + rr;
    if (i >= 3 * per_c || y < 0 || y >= h) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float x = src.raw255 ? v[k][e] / 255.0f - 0.5f : v[k][e];  // Dreamer.py:251
      xs[(rr * LW + 4 * x4 + e + 1) * 4 + c] = dr_bf16(x);
    }
  }
  __syncthreads();
  // wave w: output rows oy0 + 2w, 2w + 1 (ow pixels each = ow/16 fragments), all COUT channels
  const int nfr = ow / 16;
  for (int oyl = 2 * wave; oyl < 2 * wave + 2; ++oyl)
    for (int i = 0; i < nfr; ++i) {
      const int ox = 16 * i + r;
      f32x4 acc[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        // k = 32 s + 8 q .. +7: taps t0 = 8 s + 2 q, t0 + 1 (same ky, kx even / odd), 4 channels each
        const int t0 = 8 * s + 2 * q, ky = t0 >> 2, kx = t0 & 3;
        const uint4 pb = *reinterpret_cast<const uint4*>(&xin[2 * oyl + ky][2 * ox + kx]);
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[j] = dr_mfma_bf16(wa[s][j], pb, acc[j]);
      }
      // lane: pixel ox, channels 16 j + 4 q .. +3
      u16* o = out + (((long long)f * oh + oy0 + oyl) * ow + ox) * COUT;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        float y[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = dr_silu_fast(acc[j][e] + bv[j][e]);
        *reinterpret_cast<uint2*>(o + 16 * j + 4 * q) = dr_pack_bf16x4(y[0], y[1], y[2], y[3]);
      }
    }
}

#define DR_E12B_WAVES 4  // 8 waves measured slower (172 VGPRs, one workgroup per CU)
// ---------------------------------------------------------------------------
// conv1 + conv2 fused (enc_f1 = 32 -> enc_f2 = 64): a workgroup owns R2 rows of
// conv2 output (128 pixels); it stages the u8 input rows they depend on, runs
// conv1 for the R1 = 2 R2 + 2 conv1 rows into LDS (bf16, never written to
// HBM), then conv2 from LDS.  conv1 rows shared by two workgroups are
// recomputed (2 of 32 rows at 64 x 64).
// LDS image of the conv1 output: 16-byte units [c8 = channel / 8][pixel + pad]
// with a plane stride of NP + 1 units, so the 16 lanes of every ds_read_b128
// group of a conv2 B fragment (16 pixels at stride 2, two 8-channel chunks)
// land on 16 distinct bank quads.
// ---------------------------------------------------------------------------
// Persistent (round 3): each workgroup walks tiles blockIdx.x, + gridDim.x, ...
// and loads its next tile's input rows into registers under the current
// tile's conv2; NW = 8 waves, wave w owning 128 / 16 / NW pixel fragments x 64
// channels of conv2 (two workgroups per CU by LDS: four waves per SIMD).
template <int R2, int OW1, int NW>  // conv2 rows per workgroup, conv1 output width (= w / 2), waves
__global__ __launch_bounds__(64 * NW) void k_enc12_bf16(int n, int nb, int h, int w, dr_frames src,
                                                        const u16* __restrict__ wr1, const float* __restrict__ b1,
                                                        const u16* __restrict__ wr2, const float* __restrict__ b2,
                                                        u16* __restrict__ out) {
  constexpr int R1 = 2 * R2 + 2, RI = 2 * R1 + 2, OW2 = OW1 / 2, W = 2 * OW1;
  constexpr int NP = R1 * OW1, PS = NP + 1;  // conv1 pixels in the tile, unit plane stride
  constexpr int LWI = W + 2;
  constexpr int NTH = 64 * NW, FPW = 8 / NW;  // conv2 pixel fragments per wave
  static_assert(R2 * OW2 == 128 && (NW == 4 || NW == 8), "128 conv2 pixels per workgroup");
  __shared__ __attribute__((aligned(16))) uint2 xin[RI][LWI];  // input [row][x + 1][4 ch] bf16
  __shared__ __attribute__((aligned(16))) uint4 c1o[4 * PS];   // conv1 output, 8-channel units
  const int oh1 = h / 2, oh2 = h / 4;
  const int tiles_y = oh2 / R2, ntiles = n * tiles_y;
  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;
  // conv1 weights (A fragments, both k-steps, both channel tiles) and biases
  uint4 wa1[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j) wa1[s][j] = *reinterpret_cast<const uint4*>(wr1 + (16 * j + r) * 64 + 32 * s + 8 * q);
  float bb1[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bb1[j][e] = b1[16 * j + 4 * q + e];
  // ---- input rows (u8 ring or f32 frames): padding columns / channel slot 3
  // zeroed once; every tile rewrites all other entries (zeros outside the frame)
  for (int i = tid; i < RI * LWI; i += NTH) {
    const int rr = i / LWI;
    xin[rr][i - rr * LWI] = make_uint2(0u, 0u);
  }
  const unsigned hw = (unsigned)(h * w);
  constexpr int W4 = W / 4, PERC = RI * W4, MAXI = (3 * PERC + NTH - 1) / NTH;
  float v[MAXI][4];
  auto in_load = [&](int tl) __attribute__((always_inline)) {
    const int f = tl / tiles_y, ty = tl - f * tiles_y;
    const int iy0 = 2 * (2 * (ty * R2) - 1) - 1;
    const int b = f % nb, t = f / nb + src.t0;
    const unsigned char* fr8 = nullptr;
    const float* fr32 = nullptr;
    if (src.ring) fr8 = src.ring + ((src.starts[b] + t) % src.ring_cap) * 3 * (long long)hw;
    else fr32 = src.obs + (long long)b * src.stride_b + (long long)t * src.stride_t;
#pragma unroll
    for (int k = 0; k < MAXI; ++k) {
      const int i = tid + NTH * k;
      const int c = i / PERC, rem = i - c * PERC, rr = rem / W4, x4 = rem - rr * W4;
      const int y = iy0 + rr;
      const bool ok = i < 3 * PERC && y >= 0 && y < h;
      const unsigned off = ok ? (unsigned)c * hw + (unsigned)(y * w + 4 * x4) : 0u;
      if (fr8) {
        const unsigned u = ok ? *reinterpret_cast<const unsigned*>(fr8 + off) : 0u;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[k][e] = (float)((u >> (8 * e)) & 255u);
      } else {
        const float4 qv = ok ? *reinterpret_cast<const float4*>(fr32 + off) : make_float4(0.f, 0.f, 0.f, 0.f);
        v[k][0] = qv.x; v[k][1] = qv.y; v[k][2] = qv.z; v[k][3] = qv.w;
      }
    }
  };
  u16* xs = reinterpret_cast<u16*>(&xin[0][0]);
  auto in_store = [&](int tl) __attribute__((always_inline)) {
    const int ty = tl % tiles_y;
    const int iy0 = 2 * (2 * (ty * R2) - 1) - 1;
#pragma unroll
    for (int k = 0; k < MAXI; ++k) {
      const int i = tid + NTH * k;
      if (i >= 3 * PERC) continue;
      const int c = i / PERC, rem = i - c * PERC, rr = rem / W4, x4 = rem - rr * W4;
      const int y = iy0 + rr;
      const bool ok = y >= 0 && y < h;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = src.raw255 ? v[k][e] / 255.0f - 0.5f : v[k][e];  // Dreamer.py:251
        xs[(rr * LWI + 4 * x4 + e + 1) * 4 + c] = ok ? dr_bf16(x) : (u16)0;
      }
    }
  };
  in_load(tile);
  __syncthreads();  // the zero fill before other threads' stores
  in_store(tile);
  __syncthreads();
  int py[FPW], px[FPW];
#pragma unroll
  for (int i = 0; i < FPW; ++i) {
    const int pl = 16 * (FPW * wave + i) + r;  // tile pixel
    py[i] = pl / OW2;
    px[i] = pl - py[i] * OW2;
  }
  float bb2[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bb2[j][e] = b2[16 * j + 4 * q + e];
  for (;;) {
    const int f = tile / tiles_y, ty = tile - f * tiles_y;
    const int y2_0 = ty * R2, y1_0 = 2 * y2_0 - 1;
    const int next = tile + (int)gridDim.x;
    // ---- conv1 over the tile's R1 rows (rows outside the frame are conv2 padding: zeros) ----
    constexpr int F1 = NP / 16;  // conv1 pixel fragments
    for (int i = wave; i < F1; i += NW) {
      const int p0 = 16 * i, yl = p0 / OW1, x1 = p0 - yl * OW1 + r;
      const int y1 = y1_0 + yl;
      const int p = p0 + r;
      u16* dst0 = reinterpret_cast<u16*>(c1o);
      if (y1 < 0 || y1 >= oh1) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c8 = 2 * j + (q >> 1);
          *reinterpret_cast<uint2*>(dst0 + (c8 * PS + p) * 8 + (q & 1) * 4) = make_uint2(0u, 0u);
        }
        continue;
      }
      f32x4 acc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int t0 = 8 * s + 2 * q, ky = t0 >> 2, kx = t0 & 3;
        const uint4 pb = *reinterpret_cast<const uint4*>(&xin[2 * yl + ky][2 * x1 + kx]);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[j] = dr_mfma_bf16(wa1[s][j], pb, acc[j]);
      }
      // lane: pixel p, channels 16 j + 4 q .. +3 = half (q & 1) of 8-channel unit 2 j + (q >> 1)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c8 = 2 * j + (q >> 1);
        *reinterpret_cast<uint2*>(dst0 + (c8 * PS + p) * 8 + (q & 1) * 4) =
            dr_pack_bf16x4(dr_silu_fast(acc[j][0] + bb1[j][0]), dr_silu_fast(acc[j][1] + bb1[j][1]),
                           dr_silu_fast(acc[j][2] + bb1[j][2]), dr_silu_fast(acc[j][3] + bb1[j][3]));
      }
    }
    __syncthreads();
    if (next < ntiles) in_load(next);  // under conv2 (xin is free now)
    // ---- conv2: weights as the A operand (lane -> 4 channels of one pixel); K = 16 taps x 32 channels ----
    f32x4 acc[FPW][4];
#pragma unroll
    for (int i = 0; i < FPW; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // weight fragments one tap ahead in a two-slot register ring (compile-time
    // slots: two taps per loop iteration, the loop itself not unrolled)
    uint4 wa0[4], wa1r[4];
    auto wload = [&](uint4 (&wa)[4], int tap) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 4; ++j) wa[j] = *reinterpret_cast<const uint4*>(wr2 + (16 * j + r) * 512 + 32 * tap + 8 * q);
    };
    auto tap_step = [&](int tap, uint4 (&wa)[4], uint4 (&wn)[4]) __attribute__((always_inline)) {
      wload(wn, tap + 1 < 16 ? tap + 1 : 15);
      const int ky = tap >> 2, kx = tap & 3;
      uint4 pb[FPW];
#pragma unroll
      for (int i = 0; i < FPW; ++i) {
        // conv1 pixel (2 y2 - 1 + ky, 2 x2 - 1 + kx) in tile coordinates
        const int yl = 2 * py[i] + ky, x1 = 2 * px[i] - 1 + kx;
        const bool ok = x1 >= 0 && x1 < OW1;
        pb[i] = ok ? c1o[q * PS + yl * OW1 + x1] : make_uint4(0u, 0u, 0u, 0u);
      }
#pragma unroll
      for (int i = 0; i < FPW; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = dr_mfma_bf16(wa[j], pb[i], acc[i][j]);
    };
    wload(wa0, 0);
#pragma unroll 1
    for (int tap = 0; tap < 16; tap += 2) {
      tap_step(tap, wa0, wa1r);
      tap_step(tap + 1, wa1r, wa0);
    }
#pragma unroll
    for (int i = 0; i < FPW; ++i) {
      u16* o = out + (((long long)f * oh2 + y2_0 + py[i]) * OW2 + px[i]) * 64;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<uint2*>(o + 16 * j + 4 * q) =
            dr_pack_bf16x4(dr_silu_fast(acc[i][j][0] + bb2[j][0]), dr_silu_fast(acc[i][j][1] + bb2[j][1]),
                           dr_silu_fast(acc[i][j][2] + bb2[j][2]), dr_silu_fast(acc[i][j][3] + bb2[j][3]));
    }
    if (next >= ntiles) break;  // uniform over the workgroup
    in_store(next);
    __syncthreads();  // next input staged; every wave is past its conv2 reads of c1o
    tile = next;
  }
}

// ---------------------------------------------------------------------------
// conv2..4 (NHWC implicit GEMM) and the dense NT projection
// ---------------------------------------------------------------------------
enum { CB_NHWC = 0, CB_NCHW = 1, CB_DENSE = 2 };
template <int BM, int BN, int CIN, int MODE, int CB_PIPE>
__global__ __launch_bounds__(256) void k_conv_bf16(int M_dense, int n_frames, int ih, int iw, int N, int K_dense,
                                                   const u16* __restrict__ in, int lda, const u16* __restrict__ wr,
                                                   const float* __restrict__ bias, void* __restrict__ out, int ldo) {
  constexpr bool DENSE = MODE == CB_DENSE;
  constexpr int AJ = BM / 32, BJ = BN / 32;  // 16-byte units per thread per chunk (A rows, B rows)
  constexpr int WN = BN / 64, WM = 4 / WN;   // waves over (M, N); 64 x 64 per wave
  static_assert(WM * 64 == BM && WN * 64 == BN, "tile");
  __shared__ __attribute__((aligned(16))) uint4 sm[2][BM + BN][8];
  const int K = DENSE ? K_dense : 16 * CIN;
  const int oh = ih / 2, ow = iw / 2, hw = oh * ow;
  const long long M = DENSE ? (long long)M_dense : (long long)n_frames * hw;
  const int tiles_n = (N + BN - 1) / BN;
  const long long tiles = ((M + BM - 1) / BM) * tiles_n;
  const int lt = dr_xcd_tile(blockIdx.x, (int)tiles);
  if (lt < 0) return;
  const long long m0 = (long long)(lt / tiles_n) * BM;
  const int n0 = (lt % tiles_n) * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;
  const int u = tid & 7, row0 = tid >> 3;  // this thread stages unit u of rows row0 + 32 j

  // A rows of this thread (fixed over the K loop)
  long long abase[AJ];
  int piy[AJ], pix[AJ];
  bool pv[AJ];
#pragma unroll
  for (int j = 0; j < AJ; ++j) {
    const long long m = m0 + row0 + 32 * j;
    pv[j] = m < M;
    const long long mm = pv[j] ? m : 0;
    if (DENSE) {
      abase[j] = mm * lda;
      piy[j] = pix[j] = 0;
    } else {
      const long long f = mm / hw;
      const int p = (int)(mm - f * hw), oy = p / ow, ox = p - oy * ow;
      abase[j] = f * ih * iw * CIN;
      piy[j] = 2 * oy - 1;
      pix[j] = 2 * ox - 1;
    }
  }
  const int nch = (K + 63) / 64;
  uint4 ra[CB_PIPE][AJ], rb[CB_PIPE][BJ];
  auto load = [&](int c, int sl) {
    const int k = 64 * c + 8 * u;
    const bool kok = k < K;
    int tap = 0, ci = k;
    if (!DENSE) {
      tap = k / CIN;
      ci = k - tap * CIN;
    }
    const int ky = tap >> 2, kx = tap & 3;
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      const u16* src = nullptr;
      if (DENSE) {
        if (pv[j] && kok) src = in + abase[j] + k;
      } else {
        const int y = piy[j] + ky, x = pix[j] + kx;
        if (pv[j] && kok && y >= 0 && y < ih && x >= 0 && x < iw)
          src = in + abase[j] + ((long long)y * iw + x) * CIN + ci;
      }
      ra[sl][j] = src ? *reinterpret_cast<const uint4*>(src) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
      const int nn = n0 + row0 + 32 * j;
      rb[sl][j] = (nn < N && kok) ? *reinterpret_cast<const uint4*>(wr + (long long)nn * K + k)
                                  : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto store = [&](int sl, int buf) {
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      const int rr = row0 + 32 * j;
      sm[buf][rr][u ^ (rr & 7)] = ra[sl][j];
    }
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
      const int rr = BM + row0 + 32 * j;
      sm[buf][rr][u ^ (rr & 7)] = rb[sl][j];
    }
  };

  const int wm0 = (wave / WN) * 64, wn0 = (wave % WN) * 64;
  f32x4 acc[4][4];  // [pixel tile][channel tile]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < CB_PIPE; ++p)
    if (p < nch) load(p, p);
  store(0, 0);
  __syncthreads();
  // the ring slot of chunk c is c % CB_PIPE: unrolled over the slots so every
  // register-array index is a compile-time constant (a rolled loop indexing
  // the ring at run time puts it in scratch memory)
  for (int cb = 0; cb < nch; cb += CB_PIPE) {
#pragma unroll
    for (int uu = 0; uu < CB_PIPE; ++uu) {
      const int c = cb + uu;
      if (c >= nch) break;
      const int buf = c & 1;
      if (c + CB_PIPE < nch) load(c + CB_PIPE, uu);  // slot uu was stored to LDS last iteration
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        uint4 fa[4], fb[4];
        const int un = 4 * s + q;
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = sm[buf][wm0 + 16 * i + r][un ^ (r & 7)];
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[j] = sm[buf][BM + wn0 + 16 * j + r][un ^ (r & 7)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = (MODE == CB_NCHW) ? dr_mfma_bf16(fa[i], fb[j], acc[i][j]) : dr_mfma_bf16(fb[j], fa[i], acc[i][j]);
      }
      if (c + 1 < nch) store((uu + 1) % CB_PIPE, buf ^ 1);
      dr_lds_barrier();
    }
  }

#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (MODE == CB_NCHW) {
        // lane: channel 16 j + r, pixels 16 i + 4 q .. +3 (one frame: hw % 4 == 0)
        const long long m = m0 + wm0 + 16 * i + 4 * q;
        const int co = n0 + wn0 + 16 * j + r;
        if (m >= M || co >= N) continue;
        const float bv = bias[co];
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = dr_silu_fast(acc[i][j][e] + bv);
        const long long f = m / hw;
        *reinterpret_cast<uint2*>(reinterpret_cast<u16*>(out) + (f * N + co) * hw + (m - f * hw)) =
            dr_pack_bf16x4(v[0], v[1], v[2], v[3]);
      } else {
        // lane: pixel / row 16 i + r, channels 16 j + 4 q .. +3 (N % 4 == 0)
        const long long m = m0 + wm0 + 16 * i + r;
        const int co = n0 + wn0 + 16 * j + 4 * q;
        if (m >= M || co >= N) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bias[co + e];
        if (DENSE) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + m * ldo + co) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = dr_silu_fast(v[e]);
          *reinterpret_cast<uint2*>(reinterpret_cast<u16*>(out) + m * N + co) = dr_pack_bf16x4(v[0], v[1], v[2], v[3]);
        }
      }
    }
}

// ---------------------------------------------------------------------------
// weight conversion (per call: the f32 parameters stay the master copy)
// ---------------------------------------------------------------------------
// Conv2d [co][ci][4][4] f32 -> [co][tap][ci_pad] bf16 (channels past ci zero)
__global__ void k_conv_repack_bf16(int cout, int cin, int cin_pad, const float* w, u16* wr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cout * 16 * cin_pad) return;
  const int co = i / (16 * cin_pad), rem = i - co * 16 * cin_pad;
  const int tap = rem / cin_pad, ci = rem - tap * cin_pad;
  wr[i] = dr_bf16((ci < cin) ? w[((long long)co * cin + ci) * 16 + tap] : 0.0f);
}
// rows x cols slice of an f32 matrix (row stride ld) -> bf16 [rows][cols]
__global__ void k_to_bf16_2d(int rows, int cols, const float* x, long long ld, u16* y) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)rows * cols) return;
  const int rr = (int)(i / cols), cc = (int)(i - (long long)rr * cols);
  y[i] = dr_bf16(x[(long long)rr * ld + cc]);
}

int op_conv_repack_bf16(int cout, int cin, int cin_pad, const float* w, void* wr, hipStream_t s) {
  const int total = cout * 16 * cin_pad;
  hipLaunchKernelGGL(k_conv_repack_bf16, dim3((total + 255) / 256), dim3(256), 0, s, cout, cin, cin_pad, w, (u16*)wr);
  return dr_check_launch("conv_repack_bf16");
}

int op_to_bf16_2d(int rows, int cols, const float* x, long long ld, void* y, hipStream_t s) {
  const long long total = (long long)rows * cols;
  hipLaunchKernelGGL(k_to_bf16_2d, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, rows, cols, x, ld, (u16*)y);
  return dr_check_launch("to_bf16_2d");
}

int op_conv1_bf16(int n, int nb, int h, int w, int cout, const dr_frames* src, const void* wr, const float* bias,
                  void* out, hipStream_t s) {
  if (h % (2 * C1_OR) != 0 || w % 32 != 0 || w > C1_MAXW || (cout != 16 && cout != 32 && cout != 64)) {
    dr_set_error("conv1_bf16: needs h %% 8 == 0, w %% 32 == 0, w <= %d, cout in {16, 32, 64} (h=%d w=%d cout=%d)",
                 C1_MAXW, h, w, cout);
    return DR_E_INVALID;
  }
  if (!src->ring && ((uintptr_t)src->obs & 15)) {
    dr_set_error("conv1_bf16: f32 frames must be 16-byte aligned");
    return DR_E_INVALID;
  }
  const long long blocks = (long long)n * ((h / 2) / C1_OR);
  if (blocks >= (1LL << 31)) {
    dr_set_error("conv1_bf16: too many frames");
    return DR_E_INVALID;
  }
  const dim3 g((unsigned)blocks), b(256);
  const u16* W = (const u16*)wr;
  if (cout == 16) hipLaunchKernelGGL(k_conv1_bf16<1>, g, b, 0, s, n, nb, h, w, *src, W, bias, (u16*)out);
  else if (cout == 32) hipLaunchKernelGGL(k_conv1_bf16<2>, g, b, 0, s, n, nb, h, w, *src, W, bias, (u16*)out);
  else hipLaunchKernelGGL(k_conv1_bf16<4>, g, b, 0, s, n, nb, h, w, *src, W, bias, (u16*)out);
  return dr_check_launch("conv1_bf16");
}

// conv1 + conv2 in one launch (enc_f1 = 32, enc_f2 = 64, 64 x 64 or 128 x 128 frames);
// returns DR_E_INVALID (nothing launched) for other shapes
int op_enc12_bf16(int n, int nb, int h, int w, int c1, int c2, const dr_frames* src, const void* wr1, const float* b1,
                  const void* wr2, const float* b2, void* out, hipStream_t s) {
  if (c1 != 32 || c2 != 64 || h != w || (h != 64 && h != 128) || (!src->ring && ((uintptr_t)src->obs & 15)))
    return DR_E_INVALID;
  const long long blocks = (long long)n * (h == 64 ? 2 : 8);
  if (blocks >= (1LL << 31)) return DR_E_INVALID;
  // persistent: as many workgroups as are resident at once (occupancy API x CUs)
  static int slots[64][2];
  int dev = 0;
  DR_TRY_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return DR_E_INVALID;
  const int vi = h == 64 ? 0 : 1;
  if (slots[dev][vi] == 0) {
    int cus = 0, per = 0;
    DR_TRY_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (h == 64)
      DR_TRY_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_enc12_bf16<8, 32, DR_E12B_WAVES>,
                                                              64 * DR_E12B_WAVES, 0));
    else
      DR_TRY_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_enc12_bf16<4, 64, DR_E12B_WAVES>,
                                                              64 * DR_E12B_WAVES, 0));
    slots[dev][vi] = std::max(1, per) * std::max(1, cus);
  }
  const unsigned grid = (unsigned)std::min(blocks, (long long)slots[dev][vi]);
  if (h == 64)
    hipLaunchKernelGGL((k_enc12_bf16<8, 32, DR_E12B_WAVES>), dim3(grid), dim3(64 * DR_E12B_WAVES), 0, s, n, nb, h, w,
                       *src, (const u16*)wr1, b1, (const u16*)wr2, b2, (u16*)out);
  else
    hipLaunchKernelGGL((k_enc12_bf16<4, 64, DR_E12B_WAVES>), dim3(grid), dim3(64 * DR_E12B_WAVES), 0, s, n, nb, h, w,
                       *src, (const u16*)wr1, b1, (const u16*)wr2, b2, (u16*)out);
  return dr_check_launch("enc12_bf16");
}

template <int BM, int BN, int CIN, int MODE, int PIPE = (BM == 128 ? 4 : 2)>
static int launch_cb(int M_dense, int n, int ih, int iw, int N, int K, const void* in, int lda, const void* wr,
                     const float* bias, void* out, int ldo, hipStream_t s) {
  const long long M = MODE == CB_DENSE ? (long long)M_dense : (long long)n * (ih / 2) * (iw / 2);
  const long long tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (tiles >= (1LL << 30)) {
    dr_set_error("conv_bf16: too many tiles");
    return DR_E_INVALID;
  }
  hipLaunchKernelGGL((k_conv_bf16<BM, BN, CIN, MODE, PIPE>), dim3((unsigned)dr_xcd_grid((int)tiles)), dim3(256), 0, s,
                     M_dense, n, ih, iw, N, K, (const u16*)in, lda, (const u16*)wr, bias, out, ldo);
  return dr_check_launch("conv_bf16");
}

// k4 s2 p1 conv + bias + SiLU on bf16 NHWC [n][ih][iw][cin] -> bf16 NHWC
// [n][ih/2][iw/2][cout] (out_nchw: [n][cout][ih/2][iw/2]); wr from
// op_conv_repack_bf16 (cin_pad = cin)
int op_conv_bf16(int n, int cin, int ih, int iw, int cout, const void* in, const void* wr, const float* bias,
                 void* out, int out_nchw, hipStream_t s) {
  if (cout % 64 != 0 || ((ih / 2) * (iw / 2)) % 4 != 0) {
    dr_set_error("conv_bf16: needs cout %% 64 == 0 and (ih/2)(iw/2) %% 4 == 0 (cout=%d)", cout);
    return DR_E_INVALID;
  }
#define DR_CB(C)                                                                                                  \
  if (cin == C) {                                                                                                 \
    if (out_nchw) {                                                                                               \
      if (cout == 64) return launch_cb<256, 64, C, CB_NCHW>(0, n, ih, iw, cout, 16 * C, in, 0, wr, bias, out, 0, s); \
      return launch_cb<128, 128, C, CB_NCHW>(0, n, ih, iw, cout, 16 * C, in, 0, wr, bias, out, 0, s);            \
    }                                                                                                             \
    if (cout == 64) return launch_cb<256, 64, C, CB_NHWC>(0, n, ih, iw, cout, 16 * C, in, 0, wr, bias, out, 0, s); \
    return launch_cb<128, 128, C, CB_NHWC>(0, n, ih, iw, cout, 16 * C, in, 0, wr, bias, out, 0, s);              \
  }
  DR_CB(16)
  DR_CB(32)
  DR_CB(64)
  DR_CB(128)
  DR_CB(256)
#undef DR_CB
  dr_set_error("conv_bf16: unsupported input channels %d", cin);
  return DR_E_INVALID;
}

// Y[M][N] (f32, row stride ldy) = X[M][K] W[N][K]^T + bias, X and W bf16
// row-major (row strides ldx and K); K % 8 == 0, N % 4 == 0
int op_gemm_nt_bf16(int M, int N, int K, const void* X, int ldx, const void* W, const float* bias, float* Y, int ldy,
                    hipStream_t s) {
  if (K % 8 || ldx % 8 || N % 4 || ldy % 4 || ((uintptr_t)X & 15) || ((uintptr_t)W & 15) || ((uintptr_t)Y & 15)) {
    dr_set_error("gemm_nt_bf16: needs K, ldx %% 8 == 0, N, ldy %% 4 == 0, 16-byte aligned operands");
    return DR_E_INVALID;
  }
  return launch_cb<128, 128, 8, CB_DENSE>(M, 0, 0, 0, N, K, X, ldx, W, bias, Y, ldy, s);
}
