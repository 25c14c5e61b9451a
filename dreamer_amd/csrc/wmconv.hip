// Convolutions of the world-model training step (WorldModel.training_step,
// WorldModel.py:148-202): the decoder's ConvTranspose2d stack
// (VariationalAutoEncoder.py:128-137), the encoder's Conv2d data gradients and
// the weight gradients of both.  NHWC implicit GEMMs on the exact-f32 MFMA
// (v_mfma_f32_16x16x4_f32), like the forward encoder convs in conv.hip.
//
// Upsampling (k4 s2 p1): output row Y = 2y - 1 + ky, so each output parity
// class (Y % 2, X % 2) sees exactly 2 x 2 of the 16 taps -- a dense implicit
// GEMM with K = 4 * cin per class (no zero-inserted input, no wasted MFMA).
//   py = 0: (y, ky = 1), (y - 1, ky = 3);   py = 1: (y + 1, ky = 0), (y, ky = 2)
// i.e. tap dy in {0, 1}: iy = y + py - dy, ky = 1 - py + 2 dy.
#include "conv.h"

#define TBK 32
#define O3_TY 8
#define O3_TX 32
int op_convT_mse_parts(int h, int w);
#define TLDS (TBK + 8)  // 160-byte rows: conflict-free ds_read_b128 fragments (as conv.hip)

// wq[cls][co][tap][ci] = wt[ci][co][ky][kx], cls = py*2+px, tap = dy*2+dx
__global__ void k_convT_repack(int cin, int cout, const float* __restrict__ wt, float* __restrict__ wq) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = 4 * cout * 4 * cin;
  if (i >= total) return;
  const int ci = i % cin;
  const int tap = (i / cin) & 3;
  const int co = (i / (4 * cin)) % cout;
  const int cls = i / (4 * cin * cout);
  const int py = cls >> 1, px = cls & 1, dy = tap >> 1, dx = tap & 1;
  const int ky = 1 - py + 2 * dy, kx = 1 - px + 2 * dx;
  wq[i] = wt[(((long long)ci * cout + co) * 4 + ky) * 4 + kx];
}

int op_convT_repack(int cin, int cout, const float* wt, float* wq, hipStream_t s) {
  const int total = 16 * cout * cin;
  hipLaunchKernelGGL(k_convT_repack, dim3((total + 255) / 256), dim3(256), 0, s, cin, cout, wt, wq);
  return dr_check_launch("convT_repack");
}

template <int BM, int BN, int CIN, int EPI, bool SILU_IN>
__global__ __launch_bounds__(256) void k_convT_nhwc(ConvTArgs a) {
  constexpr int K = CIN * 4;
  // TR: weights are the MFMA A operand, so a lane's 4 accumulators are 4
  // consecutive channels of one pixel (float4 epilogue); the TANH_MSE
  // epilogue keeps pixels-as-A so its err^2 partial sums keep their order
  constexpr bool TR = EPI != CT_EPI_TANH_MSE;
  constexpr int APT = BM / 32;
  constexpr int BPT = BN >= 32 ? BN / 32 : 1;
  constexpr int WN = BN >= 32 ? 2 : 1, WM = 4 / WN;
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  static_assert(FM >= 1 && FN >= 1, "convT tile too small");
  static_assert(K % TBK == 0, "cin must be a multiple of 8");
  __shared__ __attribute__((aligned(16))) float As[2][BM][TLDS];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][TLDS];
  __shared__ float red[4];

  const int h = a.h, w = a.w, hw = h * w, cout = a.cout;
  const long long M = (long long)a.n * hw;
  const int tiles_n = (cout + BN - 1) / BN;
  const long long tiles_m = (M + BM - 1) / BM;
  const int lt = dr_xcd_tile(blockIdx.x, (int)(4 * tiles_m * tiles_n));
  if (lt < 0) return;
  // parity class fastest (as k_convT_split3): the four classes of a pixel
  // tile share an XCD's L2 and read their common input from HBM about once
  const int cls = lt & 3;
  const long long rem = lt >> 2;
  const long long m0 = (rem / tiles_n) * BM;
  const int n0 = (int)(rem % tiles_n) * BN;
  const int py = cls >> 1, px = cls & 1;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int quad = tid & 7, prow = tid >> 3;
  const float* __restrict__ in = a.in;
  const float* __restrict__ wq = a.wq + (long long)cls * cout * K;

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
    const int y = p / w, x = p - y * w;
    pbase[i] = f * hw * CIN;
    piy[i] = y + py;
    pix[i] = x + px;
  }

  // loads are issued unconditionally (out-of-range taps read offset 0) and
  // masked / activated at the LDS store: a bounds-checked load compiled to a
  // branch that waited for it at once, so chunk c+1's loads did not overlap
  // chunk c's MFMAs
  float4 ra[APT], rb[BPT];
  unsigned mka = 0u, mkb = 0u;
  auto load = [&](int k0) {
    const int k = k0 + 4 * quad;
    const int tap = k / CIN, ci = k - tap * CIN;
    const int dy = tap >> 1, dx = tap & 1;
    mka = mkb = 0u;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int y = piy[i] - dy, x = pix[i] - dx;
      const bool ok = pvalid[i] && y >= 0 && y < h && x >= 0 && x < w;
      ra[i] = *reinterpret_cast<const float4*>(in + (ok ? pbase[i] + ((long long)y * w + x) * CIN + ci : 0));
      mka |= ok ? (1u << i) : 0u;
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int co = n0 + prow + 32 * i;
      const bool ok = co < cout && prow + 32 * i < BN;
      rb[i] = *reinterpret_cast<const float4*>(wq + (ok ? (long long)co * K + k : 0));
      mkb |= ok ? (1u << i) : 0u;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      float4 v = (mka >> i) & 1u ? ra[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      if (SILU_IN) v = make_float4(dr_silu_fast(v.x), dr_silu_fast(v.y), dr_silu_fast(v.z), dr_silu_fast(v.w));
      *reinterpret_cast<float4*>(&As[buf][prow + 32 * i][4 * quad]) = v;
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i)
      if (prow + 32 * i < BN)
        *reinterpret_cast<float4*>(&Bs[buf][prow + 32 * i][4 * quad]) =
            (mkb >> i) & 1u ? rb[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  };

  const int wm0 = (wave / WN) * WTM, wn0 = (wave % WN) * WTN;
  const int r = lane & 15, q = lane >> 4;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  load(0);
  store(0);
  __syncthreads();
  constexpr int NCH = K / TBK;
  for (int c = 0; c < NCH; ++c) {
    const int buf = c & 1;
    load(min(c + 1, NCH - 1) * TBK);  // (the last chunk reloads itself, unused)
#pragma unroll
    for (int s = 0; s < TBK; s += 16) {
      float4 av[FM], bv[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) av[i] = *reinterpret_cast<const float4*>(&As[buf][wm0 + 16 * i + r][s + 4 * q]);
#pragma unroll
      for (int j = 0; j < FN; ++j) bv[j] = *reinterpret_cast<const float4*>(&Bs[buf][wn0 + 16 * j + r][s + 4 * q]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = TR ? __builtin_amdgcn_mfma_f32_16x16x4f32(bv[j].x, av[i].x, acc[i][j], 0, 0, 0)
                                : __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].x, bv[j].x, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = TR ? __builtin_amdgcn_mfma_f32_16x16x4f32(bv[j].y, av[i].y, acc[i][j], 0, 0, 0)
                                : __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].y, bv[j].y, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = TR ? __builtin_amdgcn_mfma_f32_16x16x4f32(bv[j].z, av[i].z, acc[i][j], 0, 0, 0)
                                : __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].z, bv[j].z, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = TR ? __builtin_amdgcn_mfma_f32_16x16x4f32(bv[j].w, av[i].w, acc[i][j], 0, 0, 0)
                                : __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].w, bv[j].w, acc[i][j], 0, 0, 0);
    }
    if (c + 1 < NCH) store(buf ^ 1);
    dr_lds_barrier();
  }

  const int OW = 2 * w, OH = 2 * h, ldc = a.ldc;
  float sq = 0.0f;
  if (TR) {
    const bool vec = (cout % 4 == 0) && (ldc % 4 == 0);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const long long m = m0 + wm0 + 16 * i + r;
      if (m >= M) continue;
      const long long f = m / hw;
      const int p = (int)(m - f * hw);
      const int y = p / w, x = p - y * w;
      const long long opix = (f * OH + 2 * y + py) * OW + 2 * x + px;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int co0 = n0 + wn0 + 16 * j + 4 * q;
        if (co0 >= ldc) continue;
        if (vec && co0 < cout) {
          f32x4 v = acc[i][j];
          if (EPI == CT_EPI_BIAS) {
            v += *reinterpret_cast<const f32x4*>(a.bias + co0);
            f32x4 sv = v;
            if (a.out2 || a.silu_out) {
#pragma unroll
              for (int e = 0; e < 4; ++e) sv[e] = dr_silu_fast(v[e]);
            }
            *reinterpret_cast<f32x4*>(a.out + opix * ldc + co0) = a.silu_out ? sv : v;
            if (a.out2) *reinterpret_cast<f32x4*>(a.out2 + opix * ldc + co0) = sv;
          } else {
            const f32x4 pv = *reinterpret_cast<const f32x4*>(a.pre + opix * cout + co0);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = v[e] * dr_dsilu_fast(pv[e]);
            *reinterpret_cast<f32x4*>(a.out + opix * ldc + co0) = v;
          }
          continue;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = co0 + e;
          if (co >= ldc) break;
          if (co >= cout) {
            a.out[opix * ldc + co] = 0.0f;
            continue;
          }
          const float v = acc[i][j][e];
          if (EPI == CT_EPI_BIAS) {
            const float pv = v + a.bias[co];
            const float sv = (a.out2 || a.silu_out) ? dr_silu_fast(pv) : 0.0f;
            a.out[opix * ldc + co] = a.silu_out ? sv : pv;
            if (a.out2) a.out2[opix * ldc + co] = sv;
          } else {
            a.out[opix * ldc + co] = v * dr_dsilu_fast(a.pre[opix * cout + co]);
          }
        }
      }
    }
  } else
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long m = m0 + wm0 + 16 * i + 4 * q + e;
      if (m >= M) continue;
      const long long f = m / hw;
      const int p = (int)(m - f * hw);
      const int y = p / w, x = p - y * w;
      const long long opix = (f * OH + 2 * y + py) * OW + 2 * x + px;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int co = n0 + wn0 + 16 * j + r;
        if (co >= ldc) continue;
        if (co >= cout) {  // padding channels of a wider output row
          a.out[opix * ldc + co] = 0.0f;
          continue;
        }
        const float v = acc[i][j][e];
        if (EPI == CT_EPI_BIAS) {
          const float pv = v + a.bias[co];
          const float sv = (a.out2 || a.silu_out) ? dr_silu_fast(pv) : 0.0f;
          a.out[opix * ldc + co] = a.silu_out ? sv : pv;
          if (a.out2) a.out2[opix * ldc + co] = sv;
        } else if (EPI == CT_EPI_DSILU) {
          a.out[opix * ldc + co] = v * dr_dsilu_fast(a.pre[opix * cout + co]);
        } else {  // CT_EPI_TANH_MSE (VAE.py:136 Tanh; WorldModel.py:129 squared error)
          const float mu = tanhf(v + a.bias[co]);
          const float err = mu - a.target[opix * a.tstride + co];
          sq += err * err;
          a.out[opix * ldc + co] = a.coef[f] * err * (1.0f - mu * mu);
        }
      }
    }
  if (EPI == CT_EPI_TANH_MSE) {
    // per-tile partial sums of err^2; a tile never straddles two frames
    // (the launcher checks hw % BM == 0) and there is one channel tile
    sq = wave_sum(sq);
    if (lane == 0) red[wave] = sq;
    __syncthreads();
    if (tid == 0) {
      const int per_cls = hw / BM;
      const long long f = m0 / hw;
      const int j = (int)((m0 - f * hw) / BM);
      a.part[f * 4 * per_cls + cls * per_cls + j] = ((red[0] + red[1]) + red[2]) + red[3];
    }
  }
}

int op_convT_mse_parts(int h, int w) { return (h / O3_TY) * ((w + O3_TX - 1) / O3_TX); }

template <int BM, int BN, int CIN, int EPI>
static int launch_convT(const ConvTArgs& a, hipStream_t s) {
  const long long M = (long long)a.n * a.h * a.w;
  const long long tiles = 4 * ((M + BM - 1) / BM) * ((a.cout + BN - 1) / BN);
  if (tiles >= (1LL << 30)) {
    dr_set_error("convT: too many tiles");
    return DR_E_INVALID;
  }
  dim3 grid((unsigned)dr_xcd_grid((int)tiles));
  if (a.silu_in)
    hipLaunchKernelGGL((k_convT_nhwc<BM, BN, CIN, EPI, true>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((k_convT_nhwc<BM, BN, CIN, EPI, false>), grid, dim3(256), 0, s, a);
  return dr_check_launch("convT");
}

// ---------------------------------------------------------------------------
// The decoder's last layer (ConvTranspose2d(f1 -> 3) + Tanh, VAE.py:135-136)
// fused with the reconstruction loss (WorldModel.py:129).  Three output
// channels leave an MFMA tile 3/16 full and make every input pixel a 16-fold
// re-read, so this layer runs on the VALU instead: a workgroup stages an
// (8+2) x (32+2) halo patch of the input in LDS once, and each thread owns one
// input-resolution anchor (y, x) and its 2 x 2 output pixels (all 4 parity
// classes x 3 channels = 12 accumulators).  Per input channel a thread reads
// its 9 neighbours from LDS (row pitch cin + 1: conflict-free) and the 48
// weights of that channel are wave-uniform (scalar loads).
// ---------------------------------------------------------------------------
template <int CIN, bool LOSS>
__global__ __launch_bounds__(256) void k_convT_out3(ConvTArgs a) {
  // the input channels pass through LDS CH at a time: a 16-channel patch
  // (23 KB) lets ~5 workgroups share a CU where the whole 32-channel patch
  // (45 KB) held 3, too few waves to cover the staging and LDS latency
  constexpr int CH = CIN > 16 ? 16 : CIN;
  constexpr int PW = O3_TX + 2, PH = O3_TY + 2, PITCH = CH + 1;
  __shared__ float patch[PH * PW * PITCH];
  __shared__ float red[4], redb[4][3];
  const int h = a.h, w = a.w;
  const int tiles_x = (w + O3_TX - 1) / O3_TX, tiles_y = h / O3_TY;
  const int per_frame = tiles_x * tiles_y;
  const long long f = blockIdx.x / per_frame;
  const int tile = (int)(blockIdx.x - f * per_frame);
  const int y0 = (tile / tiles_x) * O3_TY, x0 = (tile % tiles_x) * O3_TX;
  const int tid = threadIdx.x;
  const float* __restrict__ in = a.in + f * h * w * CIN;
  const int ty = tid / O3_TX, tx = tid - ty * O3_TX;
  float acc[4][3];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int o = 0; o < 3; ++o) acc[c][o] = 0.0f;
  const float* pb = patch + (ty * PW + tx) * PITCH;
  for (int c0 = 0; c0 < CIN; c0 += CH) {
    if (c0) __syncthreads();  // the previous pass's reads are done
    // stage the halo patch (SiLU of the pre-activations; zero outside the image)
    for (int e = tid; e < PH * PW * (CH / 4); e += 256) {
      const int c4 = e % (CH / 4), pix = e / (CH / 4);
      const int py = pix / PW, px = pix - py * PW;
      const int y = y0 - 1 + py, x = x0 - 1 + px;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (y >= 0 && y < h && x >= 0 && x < w) {
        v = *reinterpret_cast<const float4*>(in + ((long long)y * w + x) * CIN + c0 + 4 * c4);
        if (a.silu_in) v = make_float4(dr_silu_fast(v.x), dr_silu_fast(v.y), dr_silu_fast(v.z), dr_silu_fast(v.w));
      }
      float* d = patch + pix * PITCH + 4 * c4;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
    __syncthreads();
    const float* __restrict__ wo = a.wq + c0 * 48;  // [ci][cls][tap][co]
    for (int ci = 0; ci < CH; ++ci) {
      float xv[3][3];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) xv[r][c] = pb[(r * PW + c) * PITCH + ci];
      const float* wc = wo + ci * 48;
#pragma unroll
      for (int cls = 0; cls < 4; ++cls) {
        const int py = cls >> 1, px = cls & 1;
#pragma unroll
        for (int tap = 0; tap < 4; ++tap) {
          const int dy = tap >> 1, dx = tap & 1;
          const float x = xv[1 + py - dy][1 + px - dx];
#pragma unroll
          for (int o = 0; o < 3; ++o) acc[cls][o] = fmaf(x, wc[(cls * 4 + tap) * 3 + o], acc[cls][o]);
        }
      }
    }
  }
  const int y = y0 + ty, x = x0 + tx;
  if (!LOSS) {  // Decoder.forward: mu = tanh(.) written NCHW [f][3][2h][2w] (VAE.py:153-161)
    if (y < h && x < w) {
      const long long plane = 4LL * h * w;
#pragma unroll
      for (int cls = 0; cls < 4; ++cls) {
        const int py = cls >> 1, px = cls & 1;
        const long long pix = (long long)(2 * y + py) * (2 * w) + 2 * x + px;
#pragma unroll
        for (int o = 0; o < 3; ++o) a.out[(f * 3 + o) * plane + pix] = tanhf(acc[cls][o] + a.bias[o]);
      }
    }
    return;
  }
  // epilogue: tanh, squared error vs the target frame, dL/d(pre-tanh)
  // (+ the tile's per-channel sums of dL/d(pre-tanh): the bias gradient's
  // partials, so that 250 MB gradient is not re-read by a channel-sum pass)
  float sq = 0.0f, gs0 = 0.0f, gs1 = 0.0f, gs2 = 0.0f;
  if (y < h && x < w) {
    const int OW = 2 * w;
    const float cf = a.coef[f];
#pragma unroll
    for (int cls = 0; cls < 4; ++cls) {
      const int py = cls >> 1, px = cls & 1;
      const long long opix = (f * 2 * h + 2 * y + py) * OW + 2 * x + px;
      float tg[3];
      if (a.tstride == 4) {  // NHWC4 frames: one 16-byte load
        const float4 t4 = *reinterpret_cast<const float4*>(a.target + opix * 4);
        tg[0] = t4.x; tg[1] = t4.y; tg[2] = t4.z;
      } else {
#pragma unroll
        for (int o = 0; o < 3; ++o) tg[o] = a.target[opix * a.tstride + o];
      }
      float g[3];
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        const float mu = dr_tanh_fast(acc[cls][o] + a.bias[o]);
        const float err = mu - tg[o];
        sq += err * err;
        g[o] = cf * err * (1.0f - mu * mu);
      }
      gs0 += g[0];
      gs1 += g[1];
      gs2 += g[2];
      *reinterpret_cast<float4*>(a.out + opix * 4) = make_float4(g[0], g[1], g[2], 0.0f);
    }
  }
  sq = wave_sum(sq);
  if ((tid & 63) == 0) red[tid >> 6] = sq;
  float* bpart = a.bpart;
  if (bpart) {
    gs0 = wave_sum(gs0);
    gs1 = wave_sum(gs1);
    gs2 = wave_sum(gs2);
    if ((tid & 63) == 0) {
      redb[tid >> 6][0] = gs0;
      redb[tid >> 6][1] = gs1;
      redb[tid >> 6][2] = gs2;
    }
  }
  __syncthreads();
  if (tid == 0) a.part[f * per_frame + tile] = ((red[0] + red[1]) + red[2]) + red[3];
  if (bpart && tid < 3) bpart[(f * per_frame + tile) * 3 + tid] = ((redb[0][tid] + redb[1][tid]) + redb[2][tid]) + redb[3][tid];
}

// [cin][3][4][4] -> [ci][cls][tap][co] (48 weights per input channel)
__global__ void k_convT_out3_repack(int cin, const float* __restrict__ wt, float* __restrict__ wo) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cin * 48) return;
  const int ci = i / 48, r = i - ci * 48;
  const int ct = r / 3, co = r - ct * 3;
  const int cls = ct >> 2, tap = ct & 3;
  const int py = cls >> 1, px = cls & 1, dy = tap >> 1, dx = tap & 1;
  const int ky = 1 - py + 2 * dy, kx = 1 - px + 2 * dx;
  wo[i] = wt[(((long long)ci * 3 + co) * 4 + ky) * 4 + kx];
}

int op_convT_out3_repack(int cin, const float* wt, float* wo, hipStream_t s) {
  hipLaunchKernelGGL(k_convT_out3_repack, dim3((cin * 48 + 255) / 256), dim3(256), 0, s, cin, wt, wo);
  return dr_check_launch("convT_out3_repack");
}

int op_convT_out3(const ConvTArgs& a, hipStream_t s) {
  const bool loss = a.target != nullptr;
  if (a.cout != 3 || a.h % O3_TY != 0 || !a.bias || !a.in || !a.wq || !a.out ||
      (loss && (a.ldc != 4 || a.tstride < 3 || !a.coef || !a.part))) {
    dr_set_error("convT_out3: needs cout 3, h %% 8 == 0, bias (and ldc 4, coef, part with a target)");
    return DR_E_INVALID;
  }
  const long long blocks = (long long)a.n * op_convT_mse_parts(a.h, a.w);
  if (blocks >= (1LL << 31)) {
    dr_set_error("convT_out3: too many frames");
    return DR_E_INVALID;
  }
#define DR_O3(C)                                                                       \
  do {                                                                                 \
    if (loss)                                                                          \
      hipLaunchKernelGGL((k_convT_out3<C, true>), dim3((unsigned)blocks), dim3(256), 0, s, a);  \
    else                                                                               \
      hipLaunchKernelGGL((k_convT_out3<C, false>), dim3((unsigned)blocks), dim3(256), 0, s, a); \
  } while (0)
  switch (a.cin) {
    case 8: DR_O3(8); break;
    case 16: DR_O3(16); break;
    case 32: DR_O3(32); break;
    case 64: DR_O3(64); break;
    default: dr_set_error("convT_out3: unsupported input channels %d", a.cin); return DR_E_INVALID;
  }
#undef DR_O3
  return dr_check_launch("convT_out3");
}

template <int CIN>
static int convT_cin(int epi, const ConvTArgs& a, hipStream_t s) {
  if (epi == CT_EPI_TANH_MSE) return op_convT_out3(a, s);
  if (epi == CT_EPI_DSILU) {
    if (!a.pre || a.ldc != a.cout) {
      dr_set_error("convT: the SiLU-backward epilogue needs pre and ldc == cout");
      return DR_E_INVALID;
    }
    if (a.cout <= 16) return launch_convT<128, 16, CIN, CT_EPI_DSILU>(a, s);
    if (a.cout % 64 == 0) return launch_convT<128, 64, CIN, CT_EPI_DSILU>(a, s);
    return launch_convT<128, 32, CIN, CT_EPI_DSILU>(a, s);
  }
  if (!a.bias) {
    dr_set_error("convT: bias required");
    return DR_E_INVALID;
  }
  if (a.cout <= 16) return launch_convT<128, 16, CIN, CT_EPI_BIAS>(a, s);
  if (a.cout % 64 == 0) return launch_convT<128, 64, CIN, CT_EPI_BIAS>(a, s);
  return launch_convT<128, 32, CIN, CT_EPI_BIAS>(a, s);
}

int op_convT_nhwc(int epi, const ConvTArgs& a, hipStream_t s) {
  if (a.n <= 0 || !a.in || !a.wq || !a.out || a.ldc < a.cout) {
    dr_set_error("convT: bad arguments");
    return DR_E_INVALID;
  }
  switch (a.cin) {
    case 8: return convT_cin<8>(epi, a, s);
    case 16: return convT_cin<16>(epi, a, s);
    case 32: return convT_cin<32>(epi, a, s);
    case 64: return convT_cin<64>(epi, a, s);
    case 128: return convT_cin<128>(epi, a, s);
    case 256: return convT_cin<256>(epi, a, s);
    default: break;
  }
  dr_set_error("convT: unsupported input channels %d", a.cin);
  return DR_E_INVALID;
}

// ---------------------------------------------------------------------------
// (Round 6: a row-staged form for the 4-channel layers -- contiguous loads of
// whole low-resolution rows and the 4 hi rows they need, B fragments built by
// offset from LDS, 4x finer splits -- measured the same WM step, 12.35 -> 12.36
// ms fp32, 8.44 -> 8.48 ms bf16, profiles/r06z2_ab_conv4_wgrad.txt: this loop is
// bound by its own LDS reads and barrier, not by the gathered loads.)
// weight gradient: GEMM [ca] x [16*cb] over K = n*h*w low-res pixels, split-K
// into deterministic partial planes (no atomics) and one ordered reduction.
// Column n = tap * cb + b, so a float4 of the hi operand is 4 channels of one
// tap.  LDS holds both operands pixel-major ([k][m], [k][n]); MFMA step c of a
// 16-pixel slice takes pixel s + 4q + c on lane group q for A and B alike.
// ---------------------------------------------------------------------------
#define WBK 32
template <int BM>
__global__ __launch_bounds__(256) void k_conv_wgrad(int n, int h, int w, int ca, int cb, const float* __restrict__ lo,
                                                    int lda, int lo_silu, const float* __restrict__ hi, int ldb,
                                                    int nsplit, int chunk, float* __restrict__ part) {
  constexpr int BN = 64;
  constexpr int AP = BM + 4, BP = BN + 4;  // row pitch = 4 mod 16 dwords: lane groups q hit distinct banks
  constexpr int WTM = BM / 2, WTN = BN / 2, FM = WTM / 16, FN = WTN / 16;
  constexpr int ACOL = BM / 4, AROWS = 256 / ACOL, APT = WBK / AROWS;
  constexpr int BROWS = 16, BPT = WBK / BROWS;
  __shared__ __attribute__((aligned(16))) float As[2][WBK][AP];
  __shared__ __attribute__((aligned(16))) float Bs[2][WBK][BP];

  const int N = 16 * cb;
  const int tiles_m = (ca + BM - 1) / BM, tiles_n = N / BN;
  const int tiles = tiles_m * tiles_n;
  const int split = blockIdx.x / tiles;
  const int lt = blockIdx.x - split * tiles;
  const int m0 = (lt / tiles_n) * BM, n0 = (lt % tiles_n) * BN;
  const long long K = (long long)n * h * w;
  const long long k_begin = (long long)split * chunk;
  const long long k_end = k_begin + chunk < K ? k_begin + chunk : K;
  const int hw = h * w, H2 = 2 * h, W2 = 2 * w;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int acol = tid % ACOL, arow = tid / ACOL;
  const int bcol = tid % 16, brow = tid / 16;
  // the 4 hi channels this thread loads: fixed over the K loop
  const int bn = n0 + 4 * bcol;
  const int btap = bn / cb, bch = bn - btap * cb;
  const int bky = btap >> 2, bkx = btap & 3;
  const int am = m0 + 4 * acol;

  // unconditional loads, masked (and activated) at the LDS store: see k_convT_nhwc.
  // The hi pixel (frame, y, x) of each of this thread's B rows is decomposed
  // once and then advanced by WBK pixels per chunk: a 64-bit division per
  // load per chunk made this kernel VALU-bound (311 us for the 32-channel
  // layers at 3840 frames, r04o; the host checks n*h*w < 2^31)
  float4 ra[APT], rb[BPT];
  unsigned mka = 0u, mkb = 0u;
  int bk[BPT], bf[BPT], by[BPT], bx[BPT];
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    const int k = (int)k_begin + brow + BROWS * i;
    bk[i] = k;
    bf[i] = k / hw;
    const int p = k - bf[i] * hw;
    by[i] = p / w;
    bx[i] = p - by[i] * w;
  }
  auto advance = [&]() {
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      bk[i] += WBK;
      bx[i] += WBK;
      while (bx[i] >= w) {
        bx[i] -= w;
        if (++by[i] == h) {
          by[i] = 0;
          ++bf[i];
        }
      }
    }
  };
  auto load = [&](long long k0) {
    mka = mkb = 0u;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const long long k = k0 + arow + AROWS * i;
      const bool ok = k < k_end && am < ca;
      ra[i] = *reinterpret_cast<const float4*>(lo + (ok ? k * lda + am : 0));
      mka |= ok ? (1u << i) : 0u;
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int Y = 2 * by[i] - 1 + bky, X = 2 * bx[i] - 1 + bkx;
      const bool ok = bk[i] < k_end && Y >= 0 && Y < H2 && X >= 0 && X < W2;
      rb[i] = *reinterpret_cast<const float4*>(hi + (ok ? (((long long)bf[i] * H2 + Y) * W2 + X) * ldb + bch : 0));
      mkb |= ok ? (1u << i) : 0u;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      float4 v = (mka >> i) & 1u ? ra[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      if (lo_silu) v = make_float4(dr_silu_fast(v.x), dr_silu_fast(v.y), dr_silu_fast(v.z), dr_silu_fast(v.w));
      *reinterpret_cast<float4*>(&As[buf][arow + AROWS * i][4 * acol]) = v;
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i)
      *reinterpret_cast<float4*>(&Bs[buf][brow + BROWS * i][4 * bcol]) =
          (mkb >> i) & 1u ? rb[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  };

  const int wm0 = (wave >> 1) * WTM, wn0 = (wave & 1) * WTN;
  const int r = lane & 15, q = lane >> 4;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (k_begin < k_end) {
    load(k_begin);
    store(0);
    __syncthreads();
    const int nch = (int)((k_end - k_begin + WBK - 1) / WBK);
    for (int c = 0; c < nch; ++c) {
      const int buf = c & 1;
      if (c + 1 < nch) {
        advance();
        load(k_begin + (long long)(c + 1) * WBK);
      }
#pragma unroll
      for (int s = 0; s < WBK; s += 16) {
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          float av[FM], bv[FN];
#pragma unroll
          for (int i = 0; i < FM; ++i) av[i] = As[buf][s + 4 * q + cc][wm0 + 16 * i + r];
#pragma unroll
          for (int j = 0; j < FN; ++j) bv[j] = Bs[buf][s + 4 * q + cc][wn0 + 16 * j + r];
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
        }
      }
      if (c + 1 < nch) store(buf ^ 1);
      dr_lds_barrier();
    }
  }
  float* P = part + (long long)split * ca * N;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm0 + 16 * i + 4 * q + e;
        const int nn = n0 + wn0 + 16 * j + r;
        if (m < ca) P[(long long)m * N + nn] = acc[i][j][e];
      }
}

// dW[a][b][tap] (+)= scale * sum_s part[s][a][tap*cb + b]   (b < cbo)
// 64 consecutive outputs per workgroup, 16 split-lanes per output (coalesced
// 256-byte partial rows), fixed-order combine in LDS
__global__ __launch_bounds__(1024) void k_wgrad_reduce(int ca, int cb, int cbo, int nsplit,
                                                       const float* __restrict__ part, float* __restrict__ dw,
                                                       float scale, int accumulate, float* __restrict__ bias_out) {
  __shared__ float red[16][65];
  const int N = 16 * cb;
  const long long total = (long long)ca * N;
  const int lo = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const long long i = (long long)blockIdx.x * 64 + lo;
  float s = 0.0f;
  if (i < total)
    for (int k = sl; k < nsplit; k += 16) s += part[(long long)k * total + i];
  red[sl][lo] = s;
  __syncthreads();
  if (sl == 0 && i < total) {
    float t = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][lo];
    const int a = (int)(i / N), nn = (int)(i - (long long)a * N);
    const int tap = nn / cb, b = nn - tap * cb;
    if (b < cbo) {
      float* o = dw + ((long long)a * cbo + b) * 16 + tap;
      *o = accumulate ? *o + scale * t : scale * t;
    } else if (bias_out && b == cbo && tap == 5) {
      // pad channel cbo of the hi operand holds 1 (op_frames_nhwc4 pad = 1):
      // tap (1, 1) reads pixel (2y, 2x), inside the image for every low-res
      // pixel, so this column is sum_k lo[k][a] -- the bias gradient
      bias_out[a] = accumulate ? bias_out[a] + scale * t : scale * t;
    }
  }
}

static void wgrad_plan(int n, int h, int w, int ca, int cb, int& bm, int& nsplit, int& chunk) {
  bm = ca <= 32 ? 32 : (ca <= 64 ? 64 : 128);
  const int tiles = ((ca + bm - 1) / bm) * (16 * cb / 64);
  const long long K = (long long)n * h * w;
  const long long kch = (K + WBK - 1) / WBK;
  long long ns = (1024 + tiles - 1) / tiles;  // about 4 workgroups per CU
  const long long ns_max = (kch + 1) / 2;  // at least 2 chunks per split
  if (ns > ns_max) ns = ns_max;
  if (ns < 1) ns = 1;
  const long long ch = ((kch + ns - 1) / ns) * WBK;
  chunk = (int)ch;
  nsplit = (int)((K + ch - 1) / ch);
}

int op_wgrad_reduce(int ca, int cb, int cbo, int nsplit, const float* part, float* dw, float scale, int accumulate,
                    hipStream_t s) {
  const int total = ca * 16 * cb;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((total + 63) / 64), dim3(1024), 0, s, ca, cb, cbo, nsplit, part, dw, scale,
                     accumulate, nullptr);
  return dr_check_launch("wgrad_reduce");
}

size_t op_conv_wgrad_ws_floats(int n, int h, int w, int ca, int cb) {
  int bm, ns, ch;
  wgrad_plan(n, h, w, ca, cb, bm, ns, ch);
  return (size_t)ns * ca * 16 * cb;
}

int op_conv_wgrad(int n, int h, int w, int ca, int cb, const float* lo, int lda, int lo_silu, const float* hi, int ldb,
                  float* dw, int cbo, float scale, int accumulate, float* ws, size_t ws_floats, hipStream_t s,
                  float* bias_out) {
  if (bias_out && cbo >= cb) {
    dr_set_error("conv_wgrad: bias_out needs a pad channel (cbo < cb)");
    return DR_E_INVALID;
  }
  if (n <= 0 || ca % 4 || cb % 4 || lda % 4 || ldb % 4 || lda < ca || ldb < cb || cbo < 1 || cbo > cb || !lo || !hi ||
      !dw || (long long)n * h * w + 2 * WBK >= (1LL << 31)) {
    dr_set_error("conv_wgrad: bad arguments (channels and strides must be multiples of 4, n*h*w < 2^31)");
    return DR_E_INVALID;
  }
  int bm, ns, ch;
  wgrad_plan(n, h, w, ca, cb, bm, ns, ch);
  if ((size_t)ns * ca * 16 * cb > ws_floats) {
    dr_set_error("conv_wgrad: workspace too small");
    return DR_E_WORKSPACE;
  }
  const int tiles = ((ca + bm - 1) / bm) * (16 * cb / 64);
  dim3 grid((unsigned)(tiles * ns));
  if (bm == 32)
    hipLaunchKernelGGL(k_conv_wgrad<32>, grid, dim3(256), 0, s, n, h, w, ca, cb, lo, lda, lo_silu, hi, ldb, ns, ch, ws);
  else if (bm == 128)
    hipLaunchKernelGGL(k_conv_wgrad<128>, grid, dim3(256), 0, s, n, h, w, ca, cb, lo, lda, lo_silu, hi, ldb, ns, ch, ws);
  else
    hipLaunchKernelGGL(k_conv_wgrad<64>, grid, dim3(256), 0, s, n, h, w, ca, cb, lo, lda, lo_silu, hi, ldb, ns, ch, ws);
  DR_TRY(dr_check_launch("conv_wgrad"));
  const int total = ca * 16 * cb;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((total + 63) / 64), dim3(1024), 0, s, ca, cb, cbo, ns, ws, dw, scale,
                     accumulate, bias_out);
  return dr_check_launch("wgrad_reduce");
}

// ---------------------------------------------------------------------------
// per-channel sums over many rows (bias gradients of the conv layers)
// ---------------------------------------------------------------------------
static int chan_pow2(int C) {
  int p = 1;
  while (p < C) p <<= 1;
  return p;
}
static int chan_blocks(long long rows, int C) {
  const int rpp = 256 / chan_pow2(C);
  long long b = (rows + (long long)rpp * 16 - 1) / ((long long)rpp * 16);
  return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

__global__ __launch_bounds__(256) void k_chan_sum_part(long long rows, int C, int Cp, const float* __restrict__ X,
                                                       int ldx, long long chunk, float* __restrict__ part) {
  __shared__ float red[256];
  const int tid = threadIdx.x;
  const int c = tid % Cp, rl = tid / Cp, rpp = 256 / Cp;
  const long long r0 = (long long)blockIdx.x * chunk;
  const long long r1 = r0 + chunk < rows ? r0 + chunk : rows;
  float s = 0.0f;
  if (c < C)
    for (long long rr = r0 + rl; rr < r1; rr += rpp) s += X[rr * ldx + c];
  red[tid] = s;
  __syncthreads();
  if (tid < Cp) {
    float t = 0.0f;
    for (int k = 0; k < rpp; ++k) t += red[k * Cp + tid];
    if (tid < C) part[(long long)blockIdx.x * C + tid] = t;
  }
}

// the same partial sums with 16-byte loads: thread = (row lane, 4 channels),
// eight rows in flight per thread (independent accumulators, fixed order).
// Needs ldx % 4 == 0, a 16-byte aligned X and the padded channel quads inside
// the row (rows of the world-model gradient tensors: C = 3 at stride 4, 32..256)
__global__ __launch_bounds__(256) void k_chan_sum_part4(long long rows, int C, int Cp, const float* __restrict__ X,
                                                        int ldx, long long chunk, float* __restrict__ part) {
  constexpr int U = 8;
  __shared__ float4 red[256];
  const int tid = threadIdx.x, tpr = Cp >> 2, rpi = 256 / tpr;
  const int c0 = 4 * (tid % tpr), rl = tid / tpr;
  const long long r0 = (long long)blockIdx.x * chunk;
  const long long r1 = r0 + chunk < rows ? r0 + chunk : rows;
  float4 acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c0 < C) {
    long long rr = r0 + rl;
    for (; rr + (long long)(U - 1) * rpi < r1; rr += (long long)U * rpi) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const float4*>(X + (rr + (long long)u * rpi) * ldx + c0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[u].x += v[u].x; acc[u].y += v[u].y; acc[u].z += v[u].z; acc[u].w += v[u].w;
      }
    }
    for (; rr < r1; rr += rpi) {
      const float4 v = *reinterpret_cast<const float4*>(X + rr * ldx + c0);
      acc[0].x += v.x; acc[0].y += v.y; acc[0].z += v.z; acc[0].w += v.w;
    }
  }
  float4 t = acc[0];
#pragma unroll
  for (int u = 1; u < U; ++u) {
    t.x += acc[u].x; t.y += acc[u].y; t.z += acc[u].z; t.w += acc[u].w;
  }
  red[tid] = t;
  __syncthreads();
  if (tid < tpr) {
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < rpi; ++k) {
      const float4 v = red[k * tpr + tid];
      q.x += v.x; q.y += v.y; q.z += v.z; q.w += v.w;
    }
    const float qs[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (c0 + e < C) part[(long long)blockIdx.x * C + c0 + e] = qs[e];
  }
}

// one workgroup per channel: strided partial sums, then a fixed-order tree
__global__ __launch_bounds__(256) void k_chan_sum_final(int nb, int C, const float* __restrict__ part,
                                                        float* __restrict__ out, int accumulate) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  float s = 0.0f;
  for (int b = threadIdx.x; b < nb; b += 256) s += part[(long long)b * C + c];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[c] = accumulate ? out[c] + red[0] : red[0];
}

size_t op_chan_sum_ws_floats(long long rows, int C) { return (size_t)chan_blocks(rows, C) * C; }

int op_chan_sum_final(int nb, int C, const float* part, float* out, int accumulate, hipStream_t s) {
  if (nb <= 0 || C <= 0 || !part || !out) {
    dr_set_error("chan_sum_final: bad arguments");
    return DR_E_INVALID;
  }
  hipLaunchKernelGGL(k_chan_sum_final, dim3(C), dim3(256), 0, s, nb, C, part, out, accumulate);
  return dr_check_launch("chan_sum_final");
}

int op_chan_sum(long long rows, int C, const float* X, int ldx, float* out, int accumulate, float* ws,
                size_t ws_floats, hipStream_t s) {
  if (C <= 0 || C > 256 || rows <= 0 || ldx < C) {
    dr_set_error("chan_sum: bad arguments");
    return DR_E_INVALID;
  }
  const int nb = chan_blocks(rows, C);
  if ((size_t)nb * C > ws_floats) {
    dr_set_error("chan_sum: workspace too small");
    return DR_E_WORKSPACE;
  }
  const long long chunk = (rows + nb - 1) / nb;
  const int cp4 = chan_pow2(C < 4 ? 4 : C);
  if (ldx % 4 == 0 && ((uintptr_t)X & 15) == 0 && ldx >= ((C + 3) & ~3))
    hipLaunchKernelGGL(k_chan_sum_part4, dim3(nb), dim3(256), 0, s, rows, C, cp4, X, ldx, chunk, ws);
  else
    hipLaunchKernelGGL(k_chan_sum_part, dim3(nb), dim3(256), 0, s, rows, C, chan_pow2(C), X, ldx, chunk, ws);
  DR_TRY(dr_check_launch("chan_sum_part"));
  hipLaunchKernelGGL(k_chan_sum_final, dim3(C), dim3(256), 0, s, nb, C, ws, out, accumulate);
  return dr_check_launch("chan_sum_final");
}
