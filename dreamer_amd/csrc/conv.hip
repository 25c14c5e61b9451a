// Encoder convolutions (VariationalAutoEncoder.py:33-42: 4x Conv2d(k4, s2, p1)
// + SiLU) as NHWC implicit GEMMs on the exact-f32 MFMA.
//
//   out[pix][co] = SiLU(bias[co] + sum_{tap, ci} in[f][2oy-1+ky][2ox-1+kx][ci] * Wr[co][tap][ci])
//
// Tile BM pixels x BN output channels, K chunk = 32 (a run of channels of one
// or more taps; CIN % 4 == 0 so every float4 stays inside one tap).  Each
// thread keeps the (frame, oy, ox) of its pixels in registers for the whole K
// loop; A/B chunks are double-buffered in LDS with one barrier per chunk.  MFMA
// fragments are read with ds_read_b128: lane (r, q) takes 4 consecutive k of
// its row, and the same k permutation is used for A and B, so MFMA step c of
// a 16-k slice sums k = {c, 4+c, 8+c, 12+c} -- every product is still an
// exact f32 fma.
#include "conv.h"

#define CBK 32
#define CLDS (CBK + 8)  // 160-byte rows (= 8 mod 16 dwords): conflict-free ds_read_b128 fragments

// CONV_EPI_FWD: out = SiLU(acc + bias), optionally pre[m][co] = acc + bias
// (NHWC, kept for the backward).  CONV_EPI_DSILU (world-model backward, a
// transposed conv's input gradient): out[m][co] = acc * SiLU'(pre[m][co]).
// MFMA operand order of the conv tile: the output layout decides which of
// pixels / channels ends up 4-consecutive in a lane (see the epilogue)
#define DR_CONV_MFMA(A_, B_, C_) \
  (OUT_NCHW ? __builtin_amdgcn_mfma_f32_16x16x4f32(A_, B_, C_, 0, 0, 0) : __builtin_amdgcn_mfma_f32_16x16x4f32(B_, A_, C_, 0, 0, 0))

template <int BM, int BN, int CIN, bool OUT_NCHW, int EPI>
__global__ __launch_bounds__(256) void k_conv_nhwc(int n_frames, int ih, int iw, int cout,
                                                   const float* __restrict__ in, const float* __restrict__ wr,
                                                   const float* __restrict__ bias, float* __restrict__ out,
                                                   float* __restrict__ pre, float* __restrict__ csum) {
  constexpr int K = CIN * 16;
  constexpr int APT = BM / 32;  // pixel rows loaded per thread (8 float4 per 32-k row)
  constexpr int BPT = BN >= 32 ? BN / 32 : 1;
  constexpr int WN = BN >= 32 ? 2 : 1, WM = 4 / WN;
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  static_assert(FM >= 1 && FN >= 1, "conv tile too small");
  __shared__ __attribute__((aligned(16))) float As[2][BM][CLDS];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][CLDS];

  const int oh = ih / 2, ow = iw / 2, hw = oh * ow;
  const long long M = (long long)n_frames * hw;
  // XCD-aware 1-D tile order, channel tiles fastest: the channel tiles of one
  // pixel tile and the neighbouring pixel tiles (which share input halo rows)
  // run on one XCD and re-read activations from its L2, not from the fabric
  const int tiles_n = (cout + BN - 1) / BN;
  const long long tiles = ((M + BM - 1) / BM) * tiles_n;
  const int lt = dr_xcd_tile(blockIdx.x, (int)tiles);
  if (lt < 0) return;
  const long long m0 = (long long)(lt / tiles_n) * BM;
  const int n0 = (lt % tiles_n) * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int quad = tid & 7, prow = tid >> 3;  // 8 float4 per 32-k row

  // per-thread pixel coordinates (fixed over the K loop)
  long long pbase[APT];
  int piy[APT], pix[APT];
  bool pvalid[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const long long m = m0 + prow + 32 * i;
    pvalid[i] = m < M;
    const long long mm = pvalid[i] ? m : 0;
    const long long f = mm / hw;
    const int p = (int)(mm - f * hw);
    const int oy = p / ow, ox = p - oy * ow;
    pbase[i] = f * ih * iw * CIN;
    piy[i] = 2 * oy - 1;
    pix[i] = 2 * ox - 1;
  }

  // register ring: the global loads of chunk c+PIPE are issued while chunk c
  // computes (an L2/HBM round trip outlasts one chunk's MFMAs)
  constexpr int NCH = K / CBK;
  constexpr int PIPE = NCH >= 8 ? 3 : 1;
  float4 ra_[PIPE][APT], rb_[PIPE][BPT];
  unsigned okm_[PIPE];  // bit i: A row i's tap lies inside the frame
  auto load = [&](int k0, int sl) {
    float4* ra = ra_[sl];
    float4* rb = rb_[sl];
    const int k = k0 + 4 * quad;
    const int tap = k / CIN, ci = k - tap * CIN;
    const int ky = tap >> 2, kx = tap & 3;
    unsigned okm = 0;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      // unconditional load (padding taps read a valid address, zeroed at the
      // LDS store): a conditional load compiled to a branch that waited for
      // each load before issuing the next
      const int y = piy[i] + ky, x = pix[i] + kx;
      const bool ok = pvalid[i] && y >= 0 && y < ih && x >= 0 && x < iw;
      ra[i] = *reinterpret_cast<const float4*>(in + (ok ? pbase[i] + ((long long)y * iw + x) * CIN + ci : 0));
      okm |= ok ? (1u << i) : 0u;
    }
    okm_[sl] = okm;
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int co = n0 + prow + 32 * i;
      rb[i] = (co < cout && prow + 32 * i < BN) ? *reinterpret_cast<const float4*>(wr + (long long)co * K + k)
                                                : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&](int sl, int buf) {
    const float4* ra = ra_[sl];
    const float4* rb = rb_[sl];
#pragma unroll
    for (int i = 0; i < APT; ++i)
      *reinterpret_cast<float4*>(&As[buf][prow + 32 * i][4 * quad]) =
          (okm_[sl] >> i) & 1u ? ra[i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < BPT; ++i)
      if (prow + 32 * i < BN) *reinterpret_cast<float4*>(&Bs[buf][prow + 32 * i][4 * quad]) = rb[i];
  };

  const int wm0 = (wave / WN) * WTM, wn0 = (wave % WN) * WTN;
  const int r = lane & 15, q = lane >> 4;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int u = 0; u < PIPE; ++u)
    if (u < NCH) load(u * CBK, u);
  store(0, 0);
  __syncthreads();
  if (PIPE == 1 && NCH > 1) load(CBK, 0);
  for (int cb = 0; cb < NCH; cb += PIPE) {
#pragma unroll
    for (int u = 0; u < PIPE; ++u) {
      const int c = cb + u;  // slot of chunk c is u (cb is a multiple of PIPE)
      if (c >= NCH) break;
      const int buf = c & 1;
      // slot u was stored to LDS at the end of the previous chunk: refill it
      // (unconditional: the last chunks reload chunk NCH - 1, unused; a
      // conditional refill made every LDS store wait for all loads in flight)
      if (PIPE > 1) load(min(c + PIPE, NCH - 1) * CBK, u);
#pragma unroll
      for (int s = 0; s < CBK; s += 16) {
        float4 a[FM], b[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const float4*>(&As[buf][wm0 + 16 * i + r][s + 4 * q]);
#pragma unroll
        for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const float4*>(&Bs[buf][wn0 + 16 * j + r][s + 4 * q]);
        // k-step outer, independent accumulators inner: consecutive MFMAs never
        // wait on each other's result (40-cycle latency vs 32-cycle issue)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = DR_CONV_MFMA(a[i].x, b[j].x, acc[i][j]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = DR_CONV_MFMA(a[i].y, b[j].y, acc[i][j]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = DR_CONV_MFMA(a[i].z, b[j].z, acc[i][j]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = DR_CONV_MFMA(a[i].w, b[j].w, acc[i][j]);
      }
      if (c + 1 < NCH) {
        store((u + 1) % PIPE, buf ^ 1);
        if (PIPE == 1 && c + 2 < NCH) load((c + 2) * CBK, 0);
      }
      dr_lds_barrier();
    }
  }

  // NHWC output: weights are the MFMA A operand (DR_CONV_MFMA), so lane (r, q)
  // holds channels 4q..4q+3 of pixel r and stores float4s along c.  NCHW
  // output: pixels are the A operand, so the lane holds 4 consecutive pixels
  // of channel r, one float4 along the plane (hw % 4 == 0, checked on the host).
  float cs[FN][4];  // CONV_EPI_DSILU with csum: this lane's channel sums
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) cs[j][e] = 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if (OUT_NCHW) {
        const long long m = m0 + wm0 + 16 * i + 4 * q;
        const int co = n0 + wn0 + 16 * j + r;
        if (m >= M || co >= cout) continue;
        const float bv = bias[co];
        f32x4 v = acc[i][j] + bv;
        if (pre) {
#pragma unroll
          for (int e = 0; e < 4; ++e) pre[(m + e) * cout + co] = v[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] / (1.0f + expf(-v[e]));
        const long long f = m / hw;
        *reinterpret_cast<f32x4*>(out + (f * cout + co) * hw + (m - f * hw)) = v;
      } else {
        const long long m = m0 + wm0 + 16 * i + r;
        const int co = n0 + wn0 + 16 * j + 4 * q;
        if (m >= M || co >= cout) continue;
        f32x4 v;
        if (EPI == CONV_EPI_DSILU) {
          const f32x4 pv = *reinterpret_cast<const f32x4*>(pre + m * cout + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * dr_dsilu_fast(pv[e]);
#pragma unroll
          for (int e = 0; e < 4; ++e) cs[j][e] += v[e];
        } else {
          const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bv[e];
          if (pre) *reinterpret_cast<f32x4*>(pre + m * cout + co) = v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] / (1.0f + expf(-v[e]));
        }
        *reinterpret_cast<f32x4*>(out + m * cout + co) = v;
      }
    }
  // CONV_EPI_DSILU with csum: the tile's per-channel sums of its output (the
  // next layer's bias-gradient partials), fixed order: lanes of one channel
  // (xor over r), then the WM waves of one column block in LDS
  if (EPI == CONV_EPI_DSILU && !OUT_NCHW && csum) {
    float* s_cs = &As[0][0][0];  // the staging buffers are free after the K loop
    __syncthreads();
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = cs[j][e];
        t += __shfl_xor(t, 1, 64);
        t += __shfl_xor(t, 2, 64);
        t += __shfl_xor(t, 4, 64);
        t += __shfl_xor(t, 8, 64);
        if (r == 0) s_cs[(wave / WN) * BN + wn0 + 16 * j + 4 * q + e] = t;
      }
    __syncthreads();
    if (tid < BN && n0 + tid < cout) {
      float t = 0.f;
#pragma unroll
      for (int wm = 0; wm < WM; ++wm) t += s_cs[wm * BN + tid];
      csum[(m0 / BM) * cout + n0 + tid] = t;
    }
  }
}

// First layer (CIN = 4, K = 64): no LDS.  Every MFMA fragment piece is one
// float4 of global memory -- lane (r, q) of A slice s is pixel r's tap
// s/4 + q (4 channels), of B the 4 weights of that tap -- so each wave loads
// all 16 of its fragments up front and runs its 32 x 32 tile on its own: no
// barriers, occupancy bounded by VGPRs only (the LDS-tiled kernel spends this
// short K loop waiting on its staging round trip).  Same k permutation and MFMA
// order as k_conv_nhwc<.., 4, ..>: bitwise the same outputs.
__global__ __launch_bounds__(256) void k_conv1_direct(int n_frames, int ih, int iw, int cout,
                                                      const float* __restrict__ in, const float* __restrict__ wr,
                                                      const float* __restrict__ bias, float* __restrict__ out,
                                                      float* __restrict__ pre) {
  constexpr int K = 64, WPX = 32;  // pixels per wave; 4 waves = 128 pixels x 32 channels per workgroup
  const int oh = ih / 2, ow = iw / 2, hw = oh * ow;
  const long long M = (long long)n_frames * hw;
  const int tiles_n = cout / 32;
  const long long tiles = ((M + 127) / 128) * tiles_n;
  const int lt = dr_xcd_tile(blockIdx.x, (int)tiles);
  if (lt < 0) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const long long m0 = (long long)(lt / tiles_n) * 128 + wave * WPX;
  const int n0 = (lt % tiles_n) * 32;

  float4 a[4][2], b[4][2];  // [slice][fragment]
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long long m = m0 + 16 * i + r;
    const bool ok = m < M;
    const long long mm = ok ? m : 0;
    const long long f = mm / hw;
    const int p = (int)(mm - f * hw), oy = p / ow, ox = p - oy * ow;
    const float* base = in + f * ih * iw * 4;
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) {
      const int tap = 4 * sl + q, y = 2 * oy - 1 + (tap >> 2), x = 2 * ox - 1 + (tap & 3);
      a[sl][i] = (ok && y >= 0 && y < ih && x >= 0 && x < iw)
                     ? *reinterpret_cast<const float4*>(base + ((long long)y * iw + x) * 4)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int sl = 0; sl < 4; ++sl)
      b[sl][j] = *reinterpret_cast<const float4*>(wr + (long long)(n0 + 16 * j + r) * K + 16 * sl + 4 * q);

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int sl = 0; sl < 4; ++sl) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[sl][j].x, a[sl][i].x, acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[sl][j].y, a[sl][i].y, acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[sl][j].z, a[sl][i].z, acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[sl][j].w, a[sl][i].w, acc[i][j], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      // weights are the MFMA A operand, pixels the B operand: lane (r, q) holds
      // channels 4q..4q+3 of pixel r, stored as one float4 per tensor
      const long long m = m0 + 16 * i + r;
      if (m >= M) continue;
      const int co = n0 + 16 * j + 4 * q;
      const float4 bv = *reinterpret_cast<const float4*>(bias + co);
      float4 v = make_float4(acc[i][j][0] + bv.x, acc[i][j][1] + bv.y, acc[i][j][2] + bv.z, acc[i][j][3] + bv.w);
      if (pre) *reinterpret_cast<float4*>(pre + m * cout + co) = v;
      v.x = v.x / (1.0f + expf(-v.x));
      v.y = v.y / (1.0f + expf(-v.y));
      v.z = v.z / (1.0f + expf(-v.z));
      v.w = v.w / (1.0f + expf(-v.w));
      *reinterpret_cast<float4*>(out + m * cout + co) = v;
    }
}


// The SiLU-backward form of k_conv1_direct (CONV_EPI_DSILU, NHWC): the input
// gradient of the decoder's last transposed conv (dL/d pre-tanh, 4 channels at
// 64^2) into the 32-channel layer below, out = acc * SiLU'(pre).  The
// LDS-tiled kernel ran it as three dependent round trips per workgroup (stage,
// stage, then the epilogue's pre loads) at three workgroups per CU: 380 us for
// 1.18 GB, 3.1 TB/s (WM step fp32 12.44 -> 12.35 ms, bf16 8.52 -> 8.44 ms with
// this kernel, profiles/r06z1_ab_conv4_direct_dsilu.txt).  Here every wave issues its A / B fragments AND its pre
// float4s up front, so one round trip covers the whole tile.  Same k
// permutation and MFMA order: bitwise the same `out`.  csum (the tile's
// per-channel sums, the next layer's bias-gradient partials): lanes of one
// channel (xor over r, fragments i in order), then the 4 waves in LDS.
__global__ __launch_bounds__(256) void k_conv4_direct_dsilu(int n_frames, int ih, int iw, int cout,
                                                           const float* __restrict__ in, const float* __restrict__ wr,
                                                           const float* __restrict__ pre, float* __restrict__ out,
                                                           float* __restrict__ csum) {
  constexpr int K = 64, WPX = 32;
  __shared__ float s_cs[4][32];
  const int oh = ih / 2, ow = iw / 2, hw = oh * ow;
  const long long M = (long long)n_frames * hw;
  const int tiles_n = cout / 32;
  const long long tiles = ((M + 127) / 128) * tiles_n;
  const int lt = dr_xcd_tile(blockIdx.x, (int)tiles);
  if (lt < 0) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const long long mt = (long long)(lt / tiles_n) * 128;
  const long long m0 = mt + wave * WPX;
  const int n0 = (lt % tiles_n) * 32;

  float4 a[4][2], b[4][2];
  f32x4 pv[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const long long m = m0 + 16 * i + r;
    const bool ok = m < M;
    const long long mm = ok ? m : 0;
    const long long f = mm / hw;
    const int p = (int)(mm - f * hw), oy = p / ow, ox = p - oy * ow;
    const float* base = in + f * ih * iw * 4;
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) {
      const int tap = 4 * sl + q, y = 2 * oy - 1 + (tap >> 2), x = 2 * ox - 1 + (tap & 3);
      const bool in_ok = ok && y >= 0 && y < ih && x >= 0 && x < iw;
      const float4 t = *reinterpret_cast<const float4*>(base + (in_ok ? ((long long)y * iw + x) * 4 : 0));
      a[sl][i] = in_ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) pv[i][j] = *reinterpret_cast<const f32x4*>(pre + mm * cout + n0 + 16 * j + 4 * q);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int sl = 0; sl < 4; ++sl)
      b[sl][j] = *reinterpret_cast<const float4*>(wr + (long long)(n0 + 16 * j + r) * K + 16 * sl + 4 * q);

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int sl = 0; sl < 4; ++sl) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[sl][j].x, a[sl][i].x, acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[sl][j].y, a[sl][i].y, acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[sl][j].z, a[sl][i].z, acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[sl][j].w, a[sl][i].w, acc[i][j], 0, 0, 0);
  }
  float cs[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) cs[j][e] = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const long long m = m0 + 16 * i + r;
      if (m >= M) continue;
      const int co = n0 + 16 * j + 4 * q;
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * dr_dsilu_fast(pv[i][j][e]);
#pragma unroll
      for (int e = 0; e < 4; ++e) cs[j][e] += v[e];
      *reinterpret_cast<f32x4*>(out + m * cout + co) = v;
    }
  if (csum) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = cs[j][e];
        t += __shfl_xor(t, 1, 64);
        t += __shfl_xor(t, 2, 64);
        t += __shfl_xor(t, 4, 64);
        t += __shfl_xor(t, 8, 64);
        if (r == 0) s_cs[wave][16 * j + 4 * q + e] = t;
      }
    __syncthreads();
    if (threadIdx.x < 32)
      csum[(mt / 128) * cout + n0 + threadIdx.x] =
          ((s_cs[0][threadIdx.x] + s_cs[1][threadIdx.x]) + s_cs[2][threadIdx.x]) + s_cs[3][threadIdx.x];
  }
}

// k_conv1_direct fed from the frames themselves (with the hardware-exp2 SiLU,
// so no longer bitwise equal to it: ~2 ulp, tests/test_gpu_bf16.py checks the
// fp32 stack against torch at 1e-5).  A workgroup's 128 output
// pixels are 128 / ow whole output rows of one frame, which read 2*128/ow + 2
// input rows: the workgroup loads them once (u8 NCHW planes as 4-byte loads
// along x, or f32 float4s), applies x/255 - 0.5 (Dreamer.py:251, the same IEEE
// div-then-sub as k_frames_nhwc4) and writes NHWC4 with zero rows / columns
// for the padding into LDS; every lane then reads its A fragments (4 channels
// of one pixel-tap) from LDS exactly as k_conv1_direct reads them from HBM.
#define C1F_MAXW 130  // iw + 2 pad columns, iw <= 128
#define C1F_MAXR 10   // 2 * (128 / ow) + 2 input rows, ow >= 32
template <int IW>  // frame width (64: CarRacing, 128: configs[3]); the frame height is a runtime multiple
__global__ __launch_bounds__(256) void k_conv1_frames(int n_frames, int nb, int ih, int cout, int tpw, dr_frames src,
                                                      const float* __restrict__ wr, const float* __restrict__ bias,
                                                      float* __restrict__ out) {
  constexpr int K = 64, WPX = 32, iw = IW, ow = IW / 2, ro = 128 / ow, ri = 2 * ro + 2, xw = iw + 2;
  static_assert(ri <= C1F_MAXR && xw <= C1F_MAXW, "conv1_frames tile");
  constexpr int x4n = iw / 4, items = ri * 3 * x4n, NIT = (items + 255) / 256;
  // staged frame rows (NHWC4 + pad columns) and the output tile (128 x 36 floats)
  __shared__ __attribute__((aligned(16))) float xs[ri * xw * 4];
  __shared__ __attribute__((aligned(16))) float os[128 * 36];
  // 32-bit index math throughout (n_frames * hw < 2^31, host-checked)
  const int oh = ih / 2, hw = oh * ow;
  const int tiles_n = cout / 32;
  const int tiles = (n_frames * hw / 128) * tiles_n;
  const int groups = (tiles + tpw - 1) / tpw;
  const int lg = dr_xcd_tile(blockIdx.x, groups);
  if (lg < 0) return;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;
  const int plane = ih * iw;
  const int t_begin = lg * tpw, t_end = min(tiles, t_begin + tpw);
  // u8 -> x/255 - 0.5 by table: the same IEEE div-then-sub values, one LDS read each
  __shared__ float lut[256];
  lut[tid] = src.raw255 ? (float)tid / 255.0f - 0.5f : (float)tid;

  // this workgroup's run of tiles, software-pipelined: the frame rows of tile
  // k+1 (a window-start load, then the row loads) are in flight while tile k
  // runs its MFMAs and stores
  float vv[NIT][4];
  int cur_n0 = 0;
#define C1F_ISSUE(LT)                                                                                   \
  do {                                                                                                  \
    const int mt_ = ((LT) / tiles_n) * 128, f_ = mt_ / hw;                                             \
    const int b_ = (int)(f_ % nb), t_ = (int)(f_ / nb) + src.t0;                                       \
    const unsigned char* fr8 =                                                                          \
        src.ring ? src.ring + ((src.starts[b_] + t_) % src.ring_cap) * 3 * plane : nullptr;             \
    const float* fr32 = src.ring ? nullptr : src.obs + (long long)b_ * src.stride_b + (long long)t_ * src.stride_t; \
    const int y0_ = 2 * ((int)(mt_ - f_ * hw) / ow) - 1;                                                \
    _Pragma("unroll") for (int k = 0; k < NIT; ++k) {                                                   \
      const int it = tid + 256 * k;                                                                     \
      const int yy = it / (3 * x4n), rem = it - yy * 3 * x4n, c = rem / x4n, x4 = rem - c * x4n;      \
      const int y = y0_ + yy;                                                                           \
      const bool ok = it < items && y >= 0 && y < ih;                                                   \
      const int o = ok ? c * plane + y * iw + 4 * x4 : 0;                                               \
      if (fr8) {                                                                                        \
        const uchar4 u = *reinterpret_cast<const uchar4*>(fr8 + o);                                     \
        vv[k][0] = (float)u.x; vv[k][1] = (float)u.y; vv[k][2] = (float)u.z; vv[k][3] = (float)u.w;    \
      } else {                                                                                          \
        const float4 w4 = *reinterpret_cast<const float4*>(fr32 + o);                                   \
        vv[k][0] = w4.x; vv[k][1] = w4.y; vv[k][2] = w4.z; vv[k][3] = w4.w;                            \
      }                                                                                                 \
    }                                                                                                   \
  } while (0)
  // zero pad columns / channel 3 once: the staging pass never writes them
  for (int i = tid; i < ri * xw; i += 256) {
    const int xx = i % xw;
    xs[i * 4 + 3] = 0.f;
    if (xx == 0 || xx == xw - 1) {
      xs[i * 4 + 0] = 0.f;
      xs[i * 4 + 1] = 0.f;
      xs[i * 4 + 2] = 0.f;
    }
  }
  float4 bw[4][2];  // this channel tile's weights, reloaded only when the channel tile changes
  if (t_begin < t_end) C1F_ISSUE(t_begin);
  for (int lt = t_begin; lt < t_end; ++lt) {
    const int mt = (lt / tiles_n) * 128;
    const int n0 = (lt % tiles_n) * 32;
    const int f = mt / hw;
    const int y0 = 2 * ((int)(mt - f * hw) / ow) - 1;
    if (lt == t_begin || n0 != cur_n0) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int sl = 0; sl < 4; ++sl)
          bw[sl][j] = *reinterpret_cast<const float4*>(wr + (long long)(n0 + 16 * j + r) * K + 16 * sl + 4 * q);
      cur_n0 = n0;
    }
    __syncthreads();  // the previous tile's fragment reads of xs are done
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int it = tid + 256 * k;
      if (it >= items) break;
      const int yy = it / (3 * x4n), rem = it - yy * 3 * x4n, c = rem / x4n, x4 = rem - c * x4n;
      const int y = y0 + yy;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (y >= 0 && y < ih) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = src.ring ? lut[(int)vv[k][e]] : (src.raw255 ? vv[k][e] / 255.0f - 0.5f : vv[k][e]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) xs[(yy * xw + 4 * x4 + e + 1) * 4 + c] = v[e];
    }
    __syncthreads();
    if (lt + 1 < t_end) C1F_ISSUE(lt + 1);

    float4 a[4][2];
    const int m0 = mt + wave * WPX;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = (int)(m0 + 16 * i + r - f * hw), oy = p / ow, ox = p - oy * ow;
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) {
        const int tap = 4 * sl + q;
        const int yy = 2 * oy - 1 + (tap >> 2) - y0, xx = 2 * ox + (tap & 3);  // xx = x + 1 (pad column)
        a[sl][i] = *reinterpret_cast<const float4*>(&xs[(yy * xw + xx) * 4]);
      }
    }
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bw[sl][j].x, a[sl][i].x, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bw[sl][j].y, a[sl][i].y, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bw[sl][j].z, a[sl][i].z, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bw[sl][j].w, a[sl][i].w, acc[i][j], 0, 0, 0);
    }
    // the tile is one contiguous 16 KB NHWC run when cout == 32: stage it in
    // LDS and store whole 1 KB pieces per wave instruction
    const bool contiguous = cout == 32;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const long long m = m0 + 16 * i + r;
        const int co = n0 + 16 * j + 4 * q;
        const float4 bv = *reinterpret_cast<const float4*>(bias + co);
        float4 v = make_float4(acc[i][j][0] + bv.x, acc[i][j][1] + bv.y, acc[i][j][2] + bv.z, acc[i][j][3] + bv.w);
        // hardware exp2 / reciprocal SiLU (~2 ulp; this output-heavy layer
        // spent most of its VALU time in the IEEE expf + division)
        v.x = dr_silu_fast(v.x);
        v.y = dr_silu_fast(v.y);
        v.z = dr_silu_fast(v.z);
        v.w = dr_silu_fast(v.w);
        if (contiguous)
          *reinterpret_cast<float4*>(&os[(wave * WPX + 16 * i + r) * 36 + 16 * j + 4 * q]) = v;
        else
          *reinterpret_cast<float4*>(out + m * cout + co) = v;
      }
    if (contiguous) {
      __syncthreads();
      float* dst = out + (long long)mt * 32;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = tid + 256 * k, px = e >> 3, c4 = e & 7;
        *reinterpret_cast<float4*>(dst + 4 * e) = *reinterpret_cast<const float4*>(&os[px * 36 + 4 * c4]);
      }
    }
  }
#undef C1F_ISSUE
}

int op_conv1_frames(int n, int nb, int ih, int iw, int cout, const dr_frames* src, const float* wr, const float* bias,
                    float* out, hipStream_t s) {
  const int ow = iw / 2, hw = (ih / 2) * ow;
  const bool src_ok = src->ring ? (src->starts && src->ring_cap > 0)
                                : (src->obs && src->stride_b % 4 == 0 && src->stride_t % 4 == 0 &&
                                   ((uintptr_t)src->obs & 15) == 0);
  if (n <= 0 || nb <= 0 || cout % 32 != 0 || ih % 2 || iw % 8 || ow < 32 || ow > 128 || 128 % ow != 0 ||
      hw % 128 != 0 || 2 * (128 / ow) + 2 > C1F_MAXR || iw + 2 > C1F_MAXW || !src_ok) {
    dr_set_error("conv1_frames: unsupported shape (ih=%d iw=%d cout=%d)", ih, iw, cout);
    return DR_E_INVALID;
  }
  const long long tiles = ((long long)n * hw / 128) * (cout / 32);
  if (tiles >= (1LL << 30) || (long long)n * hw >= (1LL << 31) || (iw != 64 && iw != 128)) {
    dr_set_error("conv1_frames: too many tiles or width not 64 / 128");
    return DR_E_INVALID;
  }
  // one tile per workgroup: a 4-tile pipelined run was measured slower
  // (688 vs 620 us at 8192 frames: fewer waves resident, more barriers)
  const int tpw = 1;
  const dim3 grid((unsigned)dr_xcd_grid((int)((tiles + tpw - 1) / tpw)));
  if (iw == 64) hipLaunchKernelGGL(k_conv1_frames<64>, grid, dim3(256), 0, s, n, nb, ih, cout, tpw, *src, wr, bias, out);
  else hipLaunchKernelGGL(k_conv1_frames<128>, grid, dim3(256), 0, s, n, nb, ih, cout, tpw, *src, wr, bias, out);
  return dr_check_launch("conv1_frames");
}

template <int BM, int BN, int CIN, bool OUT_NCHW, int EPI>
static int launch_conv(int n, int ih, int iw, int cout, const float* in, const float* wr, const float* bias,
                       float* out, float* pre, hipStream_t s, float* csum = nullptr) {
  if (cout % 4 != 0 || (OUT_NCHW && ((ih / 2) * (iw / 2)) % 4 != 0)) {
    dr_set_error("conv: float4 epilogue needs cout %% 4 == 0 (and oh*ow %% 4 == 0 for NCHW output)");
    return DR_E_INVALID;
  }
  const long long M = (long long)n * (ih / 2) * (iw / 2);
  const long long tiles = ((M + BM - 1) / BM) * ((cout + BN - 1) / BN);
  if (tiles >= (1LL << 30)) {
    dr_set_error("conv: too many tiles");
    return DR_E_INVALID;
  }
  dim3 grid((unsigned)dr_xcd_grid((int)tiles));
  static bool raised = [] {
    (void)hipFuncSetAttribute((const void*)k_conv_nhwc<BM, BN, CIN, OUT_NCHW, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    return true;
  }();
  (void)raised;
  hipLaunchKernelGGL((k_conv_nhwc<BM, BN, CIN, OUT_NCHW, EPI>), grid, dim3(256), 0, s, n, ih, iw, cout,
                     in, wr, bias, out, pre, csum);
  return dr_check_launch("conv");
}

int op_conv_nhwc_ex(int n, int cin, int ih, int iw, int cout, const float* in, const float* wr, const float* bias,
                    float* out, int out_nchw, float* pre, int epi, hipStream_t s, float* csum) {
  if (csum && (epi != CONV_EPI_DSILU || out_nchw)) {
    dr_set_error("conv: channel sums only with the NHWC SiLU-backward epilogue");
    return DR_E_INVALID;
  }
  if (cin == 4 && epi == CONV_EPI_FWD && !out_nchw && cout % 32 == 0) {
    const long long tiles = (((long long)n * (ih / 2) * (iw / 2) + 127) / 128) * (cout / 32);
    if (tiles >= (1LL << 30)) {
      dr_set_error("conv: too many tiles");
      return DR_E_INVALID;
    }
    hipLaunchKernelGGL(k_conv1_direct, dim3((unsigned)dr_xcd_grid((int)tiles)), dim3(256), 0, s, n, ih, iw, cout, in, wr,
                       bias, out, pre);
    return dr_check_launch("conv1_direct");
  }
  if (epi == CONV_EPI_DSILU && (out_nchw || !pre)) {
    dr_set_error("conv: the SiLU-backward epilogue needs NHWC output and a pre-activation tensor");
    return DR_E_INVALID;
  }
  if (cin == 4 && epi == CONV_EPI_DSILU && cout % 32 == 0 &&
      ((((uintptr_t)in | (uintptr_t)wr | (uintptr_t)pre | (uintptr_t)out) & 15) == 0)) {
    const long long tiles = (((long long)n * (ih / 2) * (iw / 2) + 127) / 128) * (cout / 32);
    if (tiles >= (1LL << 30)) {
      dr_set_error("conv: too many tiles");
      return DR_E_INVALID;
    }
    hipLaunchKernelGGL(k_conv4_direct_dsilu, dim3((unsigned)dr_xcd_grid((int)tiles)), dim3(256), 0, s, n, ih, iw, cout,
                       in, wr, pre, out, csum);
    return dr_check_launch("conv4_direct_dsilu");
  }
#define DR_CONV_L(BM, BN, C, NCHW)                                                                \
  (epi == CONV_EPI_DSILU                                                                          \
       ? launch_conv<BM, BN, C, NCHW, CONV_EPI_DSILU>(n, ih, iw, cout, in, wr, bias, out, pre, s, csum) \
       : launch_conv<BM, BN, C, NCHW, CONV_EPI_FWD>(n, ih, iw, cout, in, wr, bias, out, pre, s))
#define DR_CONV_CASE(C)                                                                                     \
  if (cin == C) {                                                                                           \
    if (cout <= 16) {                                                                                       \
      if (out_nchw) return launch_conv<128, 16, C, true, CONV_EPI_FWD>(n, ih, iw, cout, in, wr, bias, out, pre, s); \
      return DR_CONV_L(128, 16, C, false);                                                                  \
    }                                                                                                       \
    if (out_nchw) return launch_conv<128, 64, C, true, CONV_EPI_FWD>(n, ih, iw, cout, in, wr, bias, out, pre, s); \
    if (cout % 64 == 0) return DR_CONV_L(128, 64, C, false);                                                \
    return DR_CONV_L(128, 32, C, false);                                                                    \
  }
  DR_CONV_CASE(4)
  DR_CONV_CASE(8)
  DR_CONV_CASE(16)
  DR_CONV_CASE(32)
  DR_CONV_CASE(64)
  DR_CONV_CASE(128)
  DR_CONV_CASE(256)
#undef DR_CONV_CASE
#undef DR_CONV_L
  dr_set_error("conv: unsupported input channels %d", cin);
  return DR_E_INVALID;
}

int op_conv_nhwc(int n, int cin, int ih, int iw, int cout, const float* in, const float* wr, const float* bias,
                 float* out, int out_nchw, hipStream_t s) {
  return op_conv_nhwc_ex(n, cin, ih, iw, cout, in, wr, bias, out, out_nchw, nullptr, CONV_EPI_FWD, s);
}

// frames (u8 replay ring or f32 tensor, NCHW 3 channels) -> normalised f32
// NHWC with 4 channels (channel 3 = pad, 0 or 1), frame f = t*nb + b.  x/255 - 0.5 is
// evaluated exactly as the reference does (IEEE div, then sub; Dreamer.py:251).
// pad = 1 (the world-model step): conv1's weight gradient then also yields its
// bias gradient in the pad column (op_conv_wgrad's bias_out); the pad channel
// meets only zero weights in the forward convs.
__global__ void k_frames_nhwc4(int n, int nb, int h, int w, dr_frames src, float* out, float pad) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // (f, y, x)
  const long long hw = (long long)h * w;
  if (i >= (long long)n * hw) return;
  const long long f = i / hw;
  const long long p = i - f * hw;
  const int b = (int)(f % nb), t = (int)(f / nb) + src.t0;
  float v[3];
  if (src.ring) {
    const unsigned char* fr = src.ring + ((src.starts[b] + t) % src.ring_cap) * 3 * hw;
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = (float)fr[c * hw + p];
  } else {
    const float* fr = src.obs + (long long)b * src.stride_b + (long long)t * src.stride_t;
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = fr[c * hw + p];
  }
  if (src.raw255) {
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = v[c] / 255.0f - 0.5f;
  }
  reinterpret_cast<float4*>(out)[i] = make_float4(v[0], v[1], v[2], pad);
}

int op_frames_nhwc4(int n, int nb, int h, int w, const dr_frames* src, float* out, hipStream_t s, float pad) {
  const long long total = (long long)n * h * w;
  hipLaunchKernelGGL(k_frames_nhwc4, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, n, nb, h, w, *src, out,
                     pad);
  return dr_check_launch("frames_nhwc4");
}

// Conv2d weight [co][ci][4][4] -> [co][tap][cin_pad] (zero-padded channels)
__global__ void k_conv_repack_pad(int cout, int cin, int cin_pad, const float* w, float* wr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cout * 16 * cin_pad) return;
  const int co = i / (16 * cin_pad), rem = i - co * 16 * cin_pad;
  const int tap = rem / cin_pad, ci = rem - tap * cin_pad;
  wr[i] = (ci < cin) ? w[((long long)co * cin + ci) * 16 + tap] : 0.0f;
}

int op_conv_repack_pad(int cout, int cin, int cin_pad, const float* w, float* wr, hipStream_t s) {
  const int total = cout * 16 * cin_pad;
  hipLaunchKernelGGL(k_conv_repack_pad, dim3((total + 255) / 256), dim3(256), 0, s, cout, cin, cin_pad, w, wr);
  return dr_check_launch("conv_repack_pad");
}
