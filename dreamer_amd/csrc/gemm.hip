// Generic fused f32 GEMM for libdreamer_hip (see gemm.h).
//
// Tile: BM x BN per 256-thread workgroup (4 waves, 2x2 or 1x4), BK = 32.
// Operands are staged through LDS with a row stride of BK+2 floats, which
// makes the MFMA fragment reads (16 rows x 4 k per wave-instruction)
// conflict-free for ds_read_b32.  The next K-slice is prefetched into
// registers while the current one feeds the MFMAs.  Every product is an
// exact f32 fma (v_mfma_f32_16x16x4_f32), so results differ from the CPU
// oracle only by summation order.
#include <limits.h>
#include <stdint.h>
#include <string.h>

#include "gemm.h"

#define BK 32
#define LDS_K (BK + 2)

struct GemmBatch {
  GemmArgs p[4];
};

GemmArgs gemm_args() {
  GemmArgs g;
  memset(&g, 0, sizeof(g));
  g.ksplitA = INT_MAX;
  g.ksplitB = INT_MAX;
  g.nsplitB = INT_MAX;
  g.nsplitY = INT_MAX;
  g.alpha = 1.0f;
  g.nb = 1;
  return g;
}

template <int AMODE>
__device__ __forceinline__ float load_a_mk(const GemmArgs& g, int m, int k, float mean, float rstd) {
  if (AMODE == AM_PLAIN) {
    if (k < g.ksplitA) return g.A[(long long)m * g.lda + k];
    return g.A2[(long long)m * g.lda2 + (k - g.ksplitA)];
  } else if (AMODE == AM_LNSILU) {
    float v = g.A[(long long)m * g.lda + k];
    float x = (v - mean) * rstd;
    x = x * g.ln_g[k] + g.ln_b[k];
    return x / (1.0f + expf(-x));
  } else if (AMODE == AM_CONV) {
    // NHWC activations, K ordered (ky, kx, ci) -- weights repacked to match
    const int hw = g.oh * g.ow;
    const int f = m / hw, pix = m - f * hw;
    const int oy = pix / g.ow, ox = pix - oy * g.ow;
    const int tap = k / g.cin, ci = k - tap * g.cin;
    const int iy = 2 * oy - 1 + (tap >> 2), ix = 2 * ox - 1 + (tap & 3);
    if (iy < 0 || iy >= g.ih || ix < 0 || ix >= g.iw) return 0.0f;
    return g.A[(((long long)f * g.ih + iy) * g.iw + ix) * g.cin + ci];
  } else {
    // first layer: NCHW frames from the replay ring (u8) or an f32 tensor,
    // K ordered like the PyTorch weight (ci, ky, kx)
    const int hw = g.oh * g.ow;
    const int f = m / hw, pix = m - f * hw;
    const int oy = pix / g.ow, ox = pix - oy * g.ow;
    const int ci = k >> 4, iy = 2 * oy - 1 + ((k >> 2) & 3), ix = 2 * ox - 1 + (k & 3);
    if (iy < 0 || iy >= g.ih || ix < 0 || ix >= g.iw) return 0.0f;
    const long long off = ((long long)ci * g.ih + iy) * g.iw + ix;
    const int b = f % g.nb, t = f / g.nb;
    float v;
    if (g.src.ring) {
      const long long slot = (g.src.starts[b] + t) % g.src.ring_cap;
      v = (float)g.src.ring[slot * (long long)g.cin * g.ih * g.iw + off];
    } else {
      v = g.src.obs[(long long)b * g.src.stride_b + (long long)t * g.src.stride_t + off];
    }
    if (g.src.raw255) v = v / 255.0f - 0.5f;  // Dreamer.py:251 (IEEE div, then sub)
    return v;
  }
}

__device__ __forceinline__ float load_b(const GemmArgs& g, bool kn, int n, int k) {
  if (!kn) return g.W[(long long)n * g.ldb + k];
  if (k >= g.ksplitB) return g.W2[(long long)(k - g.ksplitB) * g.ldb2 + n];
  if (n >= g.nsplitB) return g.W2[(long long)k * g.ldb2 + (n - g.nsplitB)];
  return g.W[(long long)k * g.ldb + n];
}

template <int BM, int BN, int AMODE, bool A_KM, bool B_KN>
__global__ __launch_bounds__(256) void k_gemm(GemmBatch gb) {
  const GemmArgs& g = gb.p[blockIdx.z];
  const int tiles_n = (g.N + BN - 1) / BN;
  const int tiles_m = (g.M + BM - 1) / BM;
  if ((int)blockIdx.x >= tiles_m * tiles_n) return;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int M = g.M, N = g.N, K = g.K;

  __shared__ float As[BM][LDS_K];
  __shared__ float Bs[BN][LDS_K];
  __shared__ float s_mean[BM], s_rstd[BM];

  if (AMODE == AM_LNSILU) {
    for (int r = wave; r < BM; r += 4) {
      const int m = m0 + r;
      float mean = 0.f, rstd = 0.f;
      if (m < M) {
        const float* row = g.A + (long long)m * g.lda;
        float s = 0.f;
        for (int k = lane; k < K; k += 64) s += row[k];
        mean = wave_sum(s) / (float)K;
        float v = 0.f;
        for (int k = lane; k < K; k += 64) {
          const float d = row[k] - mean;
          v += d * d;
        }
        rstd = 1.0f / sqrtf(wave_sum(v) / (float)K + 1e-5f);
      }
      if (lane == 0) {
        s_mean[r] = mean;
        s_rstd[r] = rstd;
      }
    }
    __syncthreads();
  }

  constexpr int NA = BM * BK / 256, NB = BN * BK / 256;
  float ra[NA], rb[NB];
  const bool store_a = (g.a_out != nullptr) && (tn == 0);

  auto load_tiles = [&](int k0) {
    if (!A_KM) {
      const int kk = tid & 31, mb = tid >> 5;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int ml = mb + 8 * i, m = m0 + ml, k = k0 + kk;
        float v = 0.f;
        if (m < M && k < K) {
          v = load_a_mk<AMODE>(g, m, k, (AMODE == AM_LNSILU) ? s_mean[ml] : 0.f,
                               (AMODE == AM_LNSILU) ? s_rstd[ml] : 0.f);
          if (store_a) g.a_out[(long long)m * g.ld_aout + k] = v;
        }
        ra[i] = v;
      }
    } else {
      const int ml = tid % BM, kb = tid / BM;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int k = k0 + kb + (256 / BM) * i, m = m0 + ml;
        ra[i] = (m < M && k < K) ? g.A[(long long)k * g.lda + m] : 0.f;
      }
    }
    if (!B_KN) {
      const int kk = tid & 31, nb = tid >> 5;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int n = n0 + nb + 8 * i, k = k0 + kk;
        rb[i] = (n < N && k < K) ? load_b(g, false, n, k) : 0.f;
      }
    } else {
      const int nl = tid % BN, kb = tid / BN;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int k = k0 + kb + (256 / BN) * i, n = n0 + nl;
        rb[i] = (n < N && k < K) ? load_b(g, true, n, k) : 0.f;
      }
    }
  };
  auto store_tiles = [&]() {
    if (!A_KM) {
      const int kk = tid & 31, mb = tid >> 5;
#pragma unroll
      for (int i = 0; i < NA; ++i) As[mb + 8 * i][kk] = ra[i];
    } else {
      const int ml = tid % BM, kb = tid / BM;
#pragma unroll
      for (int i = 0; i < NA; ++i) As[ml][kb + (256 / BM) * i] = ra[i];
    }
    if (!B_KN) {
      const int kk = tid & 31, nb = tid >> 5;
#pragma unroll
      for (int i = 0; i < NB; ++i) Bs[nb + 8 * i][kk] = rb[i];
    } else {
      const int nl = tid % BN, kb = tid / BN;
#pragma unroll
      for (int i = 0; i < NB; ++i) Bs[nl][kb + (256 / BN) * i] = rb[i];
    }
  };

  constexpr int WAVES_M = (BM >= 32) ? 2 : 1, WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  static_assert(FM >= 1 && FN >= 1, "tile too small for 4 waves");
  const int wm0 = (wave / WAVES_N) * WTM, wn0 = (wave % WAVES_N) * WTN;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fk = lane >> 4;
  load_tiles(0);
  for (int k0 = 0; k0 < K; k0 += BK) {
    __syncthreads();
    store_tiles();
    __syncthreads();
    if (k0 + BK < K) load_tiles(k0 + BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      float a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = As[wm0 + i * 16 + fr][kk + fk];
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = Bs[wn0 + j * 16 + fr][kk + fk];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue: lane holds D[row = 4*(lane>>4) + r][col = lane & 15]
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm0 + i * 16 + fk * 4 + r;
        const int n = n0 + wn0 + j * 16 + fr;
        if (m >= M || n >= N) continue;
        float v = (g.alpha == 1.0f) ? acc[i][j][r] : g.alpha * acc[i][j][r];
        if (g.bias) v = v + g.bias[n];
        if (g.addend) v = v + g.addend[(long long)m * g.ld_add + n];
        if (g.act == 1) v = v / (1.0f + expf(-v));
        float* dst;
        if (g.out_conv) {
          const int hw = g.oh * g.ow;
          const int f = m / hw, pix = m - f * hw;
          dst = g.Y + ((long long)f * N + n) * hw + pix;
        } else if (n < g.nsplitY) {
          dst = g.Y + (long long)m * g.ldy + n;
        } else {
          dst = g.Y2 + (long long)m * g.ldy2 + (n - g.nsplitY);
        }
        if (g.accumulate) *dst = *dst + v;
        else *dst = v;
      }
}

// ---------------------------------------------------------------------------
// Skinny GEMM for per-step activations (M <= 64..256 rows): a workgroup owns
// MT rows x 16 columns and splits K over its 8 waves.  Operands go straight
// from global memory into MFMA fragments -- each lane loads 4 consecutive k
// (one float4) of its row / weight row, and the 16-k chunk's k order is
// permuted identically for A and B, so MFMA step c of a chunk sums over
// k = k0 + c + {0,4,8,12}.  No LDS staging and no barriers in the K loop; the
// 8 partial accumulators are reduced through LDS in fixed order
// (deterministic), then the shared epilogue runs.
// ---------------------------------------------------------------------------
template <int AMODE, bool VEC>
__device__ __forceinline__ void skinny_load_a(const GemmArgs& g, int m, int kq, float mean, float rstd, float (&a)[4]) {
  const int M = g.M, K = g.K;
  if (m >= M) {
    a[0] = a[1] = a[2] = a[3] = 0.f;
    return;
  }
  if (VEC) {
    if (kq >= K) {
      a[0] = a[1] = a[2] = a[3] = 0.f;
      return;
    }
    const float* src = (kq < g.ksplitA) ? g.A + (long long)m * g.lda + kq
                                        : g.A2 + (long long)m * g.lda2 + (kq - g.ksplitA);
    const float4 v = *reinterpret_cast<const float4*>(src);
    a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int k = kq + c;
      if (k >= K) { a[c] = 0.f; continue; }
      a[c] = (k < g.ksplitA) ? g.A[(long long)m * g.lda + k] : g.A2[(long long)m * g.lda2 + (k - g.ksplitA)];
    }
  }
  if (AMODE == AM_LNSILU) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int k = kq + c;
      if (k < K) {
        float x = (a[c] - mean) * rstd;
        x = x * g.ln_g[k] + g.ln_b[k];
        a[c] = x / (1.0f + expf(-x));
      }
    }
  }
}

template <bool B_KN, bool VEC>
__device__ __forceinline__ void skinny_load_b(const GemmArgs& g, int n, int kq, float (&b)[4]) {
  const int N = g.N, K = g.K;
  if (n >= N) {
    b[0] = b[1] = b[2] = b[3] = 0.f;
    return;
  }
  if (!B_KN && VEC) {
    if (kq >= K) {
      b[0] = b[1] = b[2] = b[3] = 0.f;
      return;
    }
    const float4 v = *reinterpret_cast<const float4*>(g.W + (long long)n * g.ldb + kq);
    b[0] = v.x; b[1] = v.y; b[2] = v.z; b[3] = v.w;
    return;
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int k = kq + c;
    b[c] = (k < K) ? load_b(g, B_KN, n, k) : 0.f;
  }
}

__device__ __forceinline__ void epilogue_store(const GemmArgs& g, int m, int n, float acc) {
  float v = (g.alpha == 1.0f) ? acc : g.alpha * acc;
  if (g.bias) v = v + g.bias[n];
  if (g.addend) v = v + g.addend[(long long)m * g.ld_add + n];
  if (g.act == 1) v = v / (1.0f + expf(-v));
  float* dst;
  if (n < g.nsplitY) dst = g.Y + (long long)m * g.ldy + n;
  else dst = g.Y2 + (long long)m * g.ldy2 + (n - g.nsplitY);
  if (g.accumulate) *dst = *dst + v;
  else *dst = v;
}

template <int MT, int AMODE, bool B_KN, bool VEC>
__global__ __launch_bounds__(512) void k_gemm_skinny(GemmBatch gb) {
  constexpr int NWAVE = 8, FT = MT / 16;
  const GemmArgs& g = gb.p[blockIdx.z];
  const int M = g.M, N = g.N, K = g.K;
  const int tiles_n = (N + 15) / 16;
  const int tiles_m = (M + MT - 1) / MT;
  if ((int)blockIdx.x >= tiles_m * tiles_n) return;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x - tm * tiles_n;
  const int m0 = tm * MT, n0 = tn * 16;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;

  __shared__ float s_mean[MT], s_rstd[MT];
  __shared__ float red[NWAVE][FT][4][64];

  if (AMODE == AM_LNSILU) {
    for (int rr = wave; rr < MT; rr += NWAVE) {
      const int m = m0 + rr;
      float mean = 0.f, rstd = 0.f;
      if (m < M) {
        const float* row = g.A + (long long)m * g.lda;
        float s = 0.f;
        for (int k = lane; k < K; k += 64) s += row[k];
        mean = wave_sum(s) / (float)K;
        float v = 0.f;
        for (int k = lane; k < K; k += 64) {
          const float d = row[k] - mean;
          v += d * d;
        }
        rstd = 1.0f / sqrtf(wave_sum(v) / (float)K + 1e-5f);
      }
      if (lane == 0) {
        s_mean[rr] = mean;
        s_rstd[rr] = rstd;
      }
    }
    __syncthreads();
  }

  f32x4 acc[FT];
#pragma unroll
  for (int t = 0; t < FT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int kw = ((K + NWAVE * 16 - 1) / (NWAVE * 16)) * 16;
  const int kb = wave * kw;
  const int ke = min(K, kb + kw);
  const bool store_a = (g.a_out != nullptr) && (tn == 0);
#pragma unroll 2
  for (int k0 = kb; k0 < ke; k0 += 16) {
    const int kq = k0 + 4 * q;
    float b[4];
    float a[FT][4];
    skinny_load_b<B_KN, VEC>(g, n0 + r, kq, b);
#pragma unroll
    for (int t = 0; t < FT; ++t) {
      const int ml = t * 16 + r;
      skinny_load_a<AMODE, VEC>(g, m0 + ml, kq, (AMODE == AM_LNSILU) ? s_mean[ml] : 0.f,
                                (AMODE == AM_LNSILU) ? s_rstd[ml] : 0.f, a[t]);
      if (store_a && m0 + ml < M) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (kq + c < K) g.a_out[(long long)(m0 + ml) * g.ld_aout + kq + c] = a[t][c];
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int t = 0; t < FT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][c], b[c], acc[t], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < FT; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) red[wave][t][j][lane] = acc[t][j];
  __syncthreads();
  // output element e = (t, j, l): D[row 4*(l>>4)+j][col l&15] of m-tile t
  for (int e = tid; e < FT * 256; e += 512) {
    const int t = e >> 8, j = (e >> 6) & 3, l = e & 63;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) v += red[w][t][j][l];
    const int m = m0 + t * 16 + 4 * (l >> 4) + j, n = n0 + (l & 15);
    if (m < M && n < N) epilogue_store(g, m, n, v);
  }
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static bool skinny_vec_ok(const GemmArgs& g, bool b_kn) {
  if (g.K % 4 != 0 || !aligned16(g.A) || g.lda % 4 != 0) return false;
  if (g.ksplitA < g.K && (!aligned16(g.A2) || g.lda2 % 4 != 0 || g.ksplitA % 4 != 0)) return false;
  if (!b_kn && (!aligned16(g.W) || g.ldb % 4 != 0)) return false;
  return true;
}

template <int MT, int AMODE, bool B_KN>
static void launch_skinny(const GemmBatch& gb, int count, bool vec, hipStream_t s) {
  int maxt = 0;
  for (int i = 0; i < count; ++i) {
    const int t = dr_cdiv(gb.p[i].M, MT) * dr_cdiv(gb.p[i].N, 16);
    maxt = t > maxt ? t : maxt;
  }
  if (maxt == 0) return;
  if (vec) hipLaunchKernelGGL((k_gemm_skinny<MT, AMODE, B_KN, true>), dim3(maxt, 1, count), dim3(512), 0, s, gb);
  else hipLaunchKernelGGL((k_gemm_skinny<MT, AMODE, B_KN, false>), dim3(maxt, 1, count), dim3(512), 0, s, gb);
}

template <int AMODE, bool B_KN>
static bool try_skinny(const GemmBatch& gb, int count, hipStream_t s) {
  int maxM = 0;
  bool vec = true;
  for (int i = 0; i < count; ++i) {
    const GemmArgs& g = gb.p[i];
    if (g.out_conv) return false;
    maxM = g.M > maxM ? g.M : maxM;
    vec = vec && skinny_vec_ok(g, B_KN);
  }
  if (maxM > 256) return false;
  if (maxM > 64) launch_skinny<64, AMODE, B_KN>(gb, count, vec, s);
  else launch_skinny<16, AMODE, B_KN>(gb, count, vec, s);
  return true;
}

template <int BM, int BN, int AMODE, bool A_KM, bool B_KN>
static void launch_tile(const GemmBatch& gb, int count, hipStream_t s) {
  int maxt = 0;
  for (int i = 0; i < count; ++i) {
    const int t = dr_cdiv(gb.p[i].M, BM) * dr_cdiv(gb.p[i].N, BN);
    maxt = t > maxt ? t : maxt;
  }
  if (maxt == 0) return;
  hipLaunchKernelGGL((k_gemm<BM, BN, AMODE, A_KM, B_KN>), dim3(maxt, 1, count), dim3(256), 0, s, gb);
}

template <int AMODE, bool A_KM, bool B_KN>
static void launch_pick(const GemmBatch& gb, int count, hipStream_t s) {
  if (!A_KM && (AMODE == AM_PLAIN || AMODE == AM_LNSILU)) {
    if (try_skinny<(AMODE == AM_LNSILU ? AM_LNSILU : AM_PLAIN), B_KN>(gb, count, s)) return;
  }
  long long work = 0;
  for (int i = 0; i < count; ++i) work += (long long)gb.p[i].M * gb.p[i].N;
  // large problems: 64x64 tiles; small (per-step, M = batch rows): 32x32 tiles
  // so that the launch spreads over more CUs.
  if (work >= 256LL * 1024) launch_tile<64, 64, AMODE, A_KM, B_KN>(gb, count, s);
  else launch_tile<32, 32, AMODE, A_KM, B_KN>(gb, count, s);
}

int gemm_launch(GemmLayout lay, int amode, const GemmArgs* probs, int count, hipStream_t s) {
  if (count < 1 || count > 4) {
    dr_set_error("gemm_launch: bad problem count %d", count);
    return DR_E_INVALID;
  }
  GemmBatch gb;
  for (int i = 0; i < count; ++i) {
    gb.p[i] = probs[i];
    if (probs[i].M < 0 || probs[i].N < 0 || probs[i].K < 0) {
      dr_set_error("gemm_launch: negative dims");
      return DR_E_INVALID;
    }
  }
  switch (lay) {
    case G_NT:
      switch (amode) {
        case AM_PLAIN: launch_pick<AM_PLAIN, false, false>(gb, count, s); break;
        case AM_LNSILU: launch_pick<AM_LNSILU, false, false>(gb, count, s); break;
        case AM_CONV: launch_pick<AM_CONV, false, false>(gb, count, s); break;
        case AM_CONV_SRC: launch_pick<AM_CONV_SRC, false, false>(gb, count, s); break;
        default: dr_set_error("gemm_launch: bad amode"); return DR_E_INVALID;
      }
      break;
    case G_NN: launch_pick<AM_PLAIN, false, true>(gb, count, s); break;
    case G_TN: launch_pick<AM_PLAIN, true, true>(gb, count, s); break;
  }
  return dr_check_launch("gemm");
}
