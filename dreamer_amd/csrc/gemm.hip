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
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#include "gemm.h"

#include <algorithm>

#define BK 32
#define LDS_K (BK + 2)

struct GemmBatch {
  GemmArgs p[4];
};

// Grouped launches pack their problems' tiles into one linear grid (npack > 0):
// block b -> XCD-ordered logical tile over the concatenated tile lists, then
// (problem z, tile within z).  Without packing a blockIdx.z slice is sized for
// the largest problem and the smaller problems' surplus workgroups idle in it.
// Returns -1 for padding blocks; npack == 0 keeps blockIdx.z (lt = -2: the
// caller computes its tile from its own problem).
template <int BM, int BN>
__device__ __forceinline__ int dr_pack_tile(const GemmBatch& gb, int npack, int& z) {
  z = blockIdx.z;
  if (npack <= 0) return -2;
  int tot = 0;
  for (int i = 0; i < npack; ++i) tot += ((gb.p[i].M + BM - 1) / BM) * ((gb.p[i].N + BN - 1) / BN);
  int lt = dr_xcd_tile(blockIdx.x, tot);
  if (lt < 0) return -1;
  z = 0;
  for (int i = 0; i + 1 < npack; ++i) {
    const int ti = ((gb.p[i].M + BM - 1) / BM) * ((gb.p[i].N + BN - 1) / BN);
    if (lt < ti) break;
    lt -= ti;
    z = i + 1;
  }
  return lt;
}
static int pack_tiles(const GemmBatch& gb, int count, int bm, int bn) {
  int tot = 0;
  for (int i = 0; i < count; ++i) tot += ((gb.p[i].M + bm - 1) / bm) * ((gb.p[i].N + bn - 1) / bn);
  return tot;
}

static thread_local int g_gemm_bf16 = 0;
GemmBf16Scope::GemmBf16Scope(bool on) : prev(g_gemm_bf16) { g_gemm_bf16 = on ? 1 : 0; }
GemmBf16Scope::~GemmBf16Scope() { g_gemm_bf16 = prev; }

GemmArgs gemm_args() {
  GemmArgs g;
  memset(&g, 0, sizeof(g));
  g.bf16 = g_gemm_bf16;
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
    const int b = f % g.nb, t = f / g.nb + g.src.t0;
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
  if (!kn) return dr_g(g.W)[(long long)n * g.ldb + k];
  if (k >= g.ksplitB) return dr_g(g.W2)[(long long)(k - g.ksplitB) * g.ldb2 + n];
  if (n >= g.nsplitB) return dr_g(g.W2)[(long long)k * g.ldb2 + (n - g.nsplitB)];
  return dr_g(g.W)[(long long)k * g.ldb + n];
}

template <int BM, int BN, int AMODE, bool A_KM, bool B_KN>
__global__ __launch_bounds__(256) void k_gemm(GemmBatch gb) {
  const GemmArgs& g = gb.p[blockIdx.z];  // kernarg pointers: the compiler keeps them global
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
        else if (g.act == 2) v = 1.0f / (1.0f + expf(-v));
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
// Skinny GEMM for per-step activations (M up to a few thousand rows, N
// moderate): a workgroup owns MT rows x NT columns and splits K over its 8
// waves.  Operands go straight from global memory into MFMA fragments -- each
// lane loads 4 consecutive k (one float4) of its row / weight row, and the
// 16-k chunk's k order is permuted identically for A and B, so MFMA step c of
// a chunk sums k = k0 + c + {0,4,8,12}.  No LDS staging of the weights and no
// barriers in the K loop; the weight chunk is prefetched one step ahead.
// With LayerNorm+SiLU on load, the MT input rows are staged once in LDS (one
// global pass) and the row statistics come from there.  The 8 partial
// accumulators are reduced through LDS in fixed order (deterministic), then
// either the element epilogue or a fused row epilogue runs:
//   EPI_SAMPLE  softmax / 1% unimix / argmax(p_hat / Exp(1)) / one-hot STE per
//               latent group (VAE.py:88-98, DynamicsPredictors.py:33-39)
//   EPI_ACTOR   mu, clamp(log_sig), softplus + 1e-3, tanh(mu + eps*sigma)
//               (Agent.py:196-210)
// ---------------------------------------------------------------------------
#ifdef DR_PHASE_TIMING
__device__ long long dr_tbuf_gemm[1024 * DR_TS_SLOTS];
extern "C" int dr_debug_tbuf_gemm(long long* out, int n) {  // read, then clear
  const int rc = (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(dr_tbuf_gemm), (size_t)n * sizeof(long long));
  static long long zeros[1024 * DR_TS_SLOTS];
  return rc | (int)hipMemcpyToSymbol(HIP_SYMBOL(dr_tbuf_gemm), zeros, sizeof(zeros));
}
#endif
#define SK_LN_MAXF 33280  // floats of staged LayerNorm rows (MT * (K + 4)); 130 KB of the 160 KB LDS
#define SK_LN_MAXK 2048   // LayerNorm width staged with its gamma / beta
#define SK_STAGE 8        // float4 staging loads in flight per thread

// hot operands of a skinny problem as wave-uniform scalars (see dr_uni)
struct SkOps {
  const float *A, *A2, *W, *W2;
  int lda, lda2, ksA, ldb, ldb2, ksB, nsB, M, N, K;
};

template <bool B_KN, bool VEC>
__device__ __forceinline__ void skinny_load_b(const SkOps& o, int n, int kq, float (&b)[4]) {
  if (!B_KN && VEC) {
    const bool ok = (n < o.N) && (kq < o.K);
    float4 v = dr_ld4(o.W, ok ? (unsigned)(n * o.ldb + kq) : 0u);
    if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
    b[0] = v.x; b[1] = v.y; b[2] = v.z; b[3] = v.w;
    return;
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int k = kq + c;
    const bool ok = (n < o.N) && (k < o.K);
    float v;
    if (!B_KN) {
      v = dr_ld1(o.W, ok ? (unsigned)(n * o.ldb + k) : 0u);
    } else if (k >= o.ksB) {  // KN second segment: rows past ksplitB or columns past nsplitB
      v = dr_ld1(o.W2, ok ? (unsigned)((k - o.ksB) * o.ldb2 + n) : 0u);
    } else if (n >= o.nsB) {
      v = dr_ld1(o.W2, ok ? (unsigned)(k * o.ldb2 + n - o.nsB) : 0u);
    } else {
      v = dr_ld1(o.W, ok ? (unsigned)(k * o.ldb + n) : 0u);
    }
    b[c] = ok ? v : 0.f;
  }
}

// A rows: the 16-k chunk starting at k16 lies in one segment (A below ksA, A2
// above) unless ksA is not a multiple of 16, in which case lanes pick theirs
template <bool VEC>
__device__ __forceinline__ void skinny_load_a(const SkOps& o, int m, int k16, int kq, float (&a)[4]) {
  if (VEC) {
    const bool ok = (m < o.M) && (kq < o.K);
    float4 v;
    if (k16 + 16 <= o.ksA) {
      v = dr_ld4(o.A, ok ? (unsigned)(m * o.lda + kq) : 0u);
    } else if (k16 >= o.ksA) {
      v = dr_ld4(o.A2, ok ? (unsigned)(m * o.lda2 + kq - o.ksA) : 0u);
    } else {
      const float* src = (kq < o.ksA) ? o.A + (long long)m * o.lda + kq : o.A2 + (long long)m * o.lda2 + (kq - o.ksA);
      v = dr_ld4(ok ? src : o.A, 0u);
    }
    if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
    a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int k = kq + c;
      const bool ok = (m < o.M) && (k < o.K);
      float v;
      if (k < o.ksA) v = dr_ld1(o.A, ok ? (unsigned)(m * o.lda + k) : 0u);
      else v = dr_ld1(o.A2, ok ? (unsigned)(m * o.lda2 + k - o.ksA) : 0u);
      a[c] = ok ? v : 0.f;
    }
  }
}

__device__ __forceinline__ float epi_act(const GemmArgs& g, float v) {
  if (g.act == 1) return v / (1.0f + expf(-v));
  if (g.act == 2) return 1.0f / (1.0f + expf(-v));
  return v;
}

// GruBwdEpi: the gru_cell backward of one (row, unit) from the final dL/dh'
__device__ __noinline__ void gru_bwd_elem(const GruBwdEpi& e, int m, int j, float g) {
  const int Hd = e.Hd;
  const long long i = (long long)m * Hd + j;
  const float r = dr_g(e.r)[i], u = dr_g(e.u)[i], n = dr_g(e.n)[i], hn = dr_g(e.ghn)[i];
  const float hv = e.h ? dr_g(e.h)[(long long)m * e.ldh + j] : 0.0f;
  // h' = (h - n)*u + n
  const float g_hmn = g * u;
  const float g_u = g * (hv - n);
  const float g_n = g + (-g_hmn);
  // n = tanh(in + hn*r)
  const float g_pn = g_n * (1.0f - n * n);
  const float g_r = g_pn * hn;
  const float g_hn = g_pn * r;
  const float g_pr = g_r * (1.0f - r) * r;
  const float g_pu = g_u * (1.0f - u) * u;
  DR_GLOBAL float* gib = dr_g(e.gi) + (long long)m * 3 * Hd;
  DR_GLOBAL float* ghb = dr_g(e.gh) + (long long)m * 3 * Hd;
  gib[j] = g_pr;
  gib[Hd + j] = g_pu;
  gib[2 * Hd + j] = g_pn;
  ghb[j] = g_pr;
  ghb[Hd + j] = g_pu;
  ghb[2 * Hd + j] = g_hn;
  if (e.gi16) {
    DR_GLOBAL unsigned short* gi16 = dr_g(e.gi16) + (long long)m * 3 * Hd;
    DR_GLOBAL unsigned short* gh16 = dr_g(e.gh16) + (long long)m * 3 * Hd;
    gi16[j] = __builtin_bit_cast(unsigned short, (__bf16)g_pr);
    gi16[Hd + j] = __builtin_bit_cast(unsigned short, (__bf16)g_pu);
    gi16[2 * Hd + j] = __builtin_bit_cast(unsigned short, (__bf16)g_pn);
    gh16[j] = __builtin_bit_cast(unsigned short, (__bf16)g_pr);
    gh16[Hd + j] = __builtin_bit_cast(unsigned short, (__bf16)g_pu);
    gh16[2 * Hd + j] = __builtin_bit_cast(unsigned short, (__bf16)g_hn);
  }
  DR_GLOBAL float* o = dr_g(e.ho) + (long long)m * e.ldo + j;
  *o = *o + g_hmn;
}

__device__ __forceinline__ void epilogue_store_b(const GemmArgs& g, int m, int n, float acc, float bias) {
  float v = (g.alpha == 1.0f) ? acc : g.alpha * acc;
  if (g.bias) v = v + bias;
  if (g.addend) v = v + dr_g(g.addend)[(long long)m * g.ld_add + n];
  v = epi_act(g, v);
  DR_GLOBAL float* dst;
  if (n < g.nsplitY) dst = dr_g(g.Y) + (long long)m * g.ldy + n;
  else dst = dr_g(g.Y2) + (long long)m * g.ldy2 + (n - g.nsplitY);
  const float fin = g.accumulate ? *dst + v : v;
  *dst = fin;
  if (g.gb.Hd > 0 && n < g.gb.Hd) gru_bwd_elem(g.gb, m, n, fin);
}

#define DR_SKW 8  // waves per skinny-GEMM workgroup (K split over them; 4 measured slower, r05)
template <int MT, int NT, int AMODE, bool B_KN, bool VEC, int EPI>
__global__ __launch_bounds__(64 * DR_SKW) void k_gemm_skinny(GemmBatch gb, int npack) {
  constexpr int NWAVE = DR_SKW, NTH = 64 * DR_SKW, FT = MT / 16, FN = NT / 16;
  __shared__ GemmArgs s_args;
  int pz;
  const int plt = dr_pack_tile<MT, NT>(gb, npack, pz);
  if (plt == -1) return;
  dr_stage_args(gb.p[pz], s_args, threadIdx.x);
  const GemmArgs& g = s_args;
  SkOps o;
  o.M = dr_uni(g.M); o.N = dr_uni(g.N); o.K = dr_uni(g.K);
  o.A = dr_uni(g.A); o.A2 = dr_uni(g.A2); o.W = dr_uni(g.W);
  o.lda = dr_uni((int)g.lda); o.lda2 = dr_uni((int)g.lda2); o.ksA = dr_uni(g.ksplitA); o.ldb = dr_uni((int)g.ldb);
  o.W2 = dr_uni(g.W2); o.ldb2 = dr_uni((int)g.ldb2); o.ksB = dr_uni(g.ksplitB); o.nsB = dr_uni(g.nsplitB);
  const int M = o.M, N = o.N, K = o.K;
  const int tiles_n = (N + NT - 1) / NT;
  const int tiles_m = (M + MT - 1) / MT;
  // logical tiles column-major: the row tiles reading one weight slice are
  // adjacent and share an XCD's L2
  const int lt = plt >= 0 ? plt : dr_xcd_tile(blockIdx.x, tiles_m * tiles_n);
  if (lt < 0) return;
  const int tn = lt / tiles_m, tm = lt - tn * tiles_m;
  const int m0 = tm * MT, n0 = tn * NT;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
  DR_TS(dr_tbuf_gemm, 0);

  // dynamic LDS, sized by the host for this launch (skinny_lds_floats):
  // [ max(reduction slab, staged LN rows) | LN gamma (K) | LN beta (K) ]
  constexpr int RED = NWAVE * FT * FN * 4 * 64;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float s_mean[MT], s_rstd[MT];
  __shared__ float s_out[MT][NT + 1];
  // bias of the output columns this thread finalises, issued now and waited
  // for only in the epilogue
  constexpr int NEPI = (FT * FN * 256 + NTH - 1) / NTH;
  float ebias[NEPI];
  {
    const float* bias = dr_uni(g.bias);
#pragma unroll
    for (int i = 0; i < NEPI; ++i) {
      const int x = tid + NTH * i;
      const int n = n0 + ((x >> 8) % FN) * 16 + (x & 15);
      const bool ok = bias && x < FT * FN * 256 && n < N;
      const float v = dr_ld1(ok ? bias : o.W, ok ? (unsigned)n : 0u);
      ebias[i] = ok ? v : 0.f;
    }
  }

  // Philox state of the sampler / actor epilogues, fetched now (not after the K loop)
  unsigned long long rng_seed = 0, rng_off = 0;
  if ((EPI == EPI_SAMPLE || EPI == EPI_ACTOR) && g.epi != EPI_NONE && !g.noise.q && !g.noise.eps && g.noise.rng) {
    rng_seed = g.noise.rng[0];
    rng_off = g.noise.rng[1];
  }
  const int kw = ((K + NWAVE * 16 - 1) / (NWAVE * 16)) * 16;
  const int kb = wave * kw;
  const int ke = min(K, kb + kw);

  // ---- operand path ---------------------------------------------------
  // Staged (LayerNorm-SiLU A, NT, 16-byte aligned, K <= 1024): every row of the A tile and of
  // the weight tile is read by one wave with coalesced 1 KB row pieces
  // (lane -> float4 column), all loads issued before the first wait; the
  // LayerNorm-SiLU prologue (rows in registers: DPP statistics, one
  // normalise + activate per element) runs on the way; both tiles land in LDS
  // with a padded stride (K + 4 floats: the 16 rows an MFMA fragment reads
  // fall in distinct banks); the K loop then reads fragments from LDS.
  // Direct (otherwise): each lane loads its MFMA fragments from global memory.
  const int KP = K + ((8 - (K & 15)) & 15);  // row stride = 8 mod 16 dwords: ds_read_b128 fragments conflict-free
  const int K4 = K >> 2;
  constexpr int RPW = MT / NWAVE;                    // A rows per wave
  constexpr int BPW = (NT + NWAVE - 1) / NWAVE;      // weight rows per wave
  constexpr int SV = (MT == 16) ? 4 : 1;             // float4 per lane per staged row (K <= 256 * SV)
  float* a_out = dr_uni(g.a_out);
  const int ld_aout = dr_uni((int)g.ld_aout);
  const bool store_a = (a_out != nullptr) && (tn == 0);
  // (measured: staging pays only where the LayerNorm needs the barrier anyway;
  // a plain GEMM is faster with direct fragment loads, profiles/r01_v5_kbench.txt)
  const bool staged = (AMODE == AM_LNSILU || AMODE == AM_LNBWD || AMODE == AM_STEBWD) && VEC && !B_KN &&
                     (K4 <= 64 * SV) &&
                     ((MT + NT) * KP <= SK_LN_MAXF);
  // with few accumulator tiles, alternate 16-k chunks between two accumulator
  // sets so consecutive MFMAs are independent (40-cycle result latency)
  constexpr bool DUAL = FT * FN < 4;
  f32x4 acc[FT][FN], acc2[FT][FN];
#pragma unroll
  for (int t = 0; t < FT; ++t)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[t][j] = acc2[t][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  DR_TS(dr_tbuf_gemm, 1);
  if (staged) {
    float* sA = smem;
    float* sB = smem + MT * KP;
    constexpr int PRW = (AMODE == AM_LNBWD || AMODE == AM_STEBWD) ? RPW : 1;
    float4 xa[RPW][SV], xb[BPW][SV], gv[SV], bv[SV], xp[PRW][SV];
    const float* lg = dr_uni(g.ln_g);
    const float* lb = dr_uni(g.ln_b);
    const float* pre = dr_uni(g.pre);
    const int ld_pre = dr_uni((int)g.ld_pre);
#pragma unroll
    for (int i = 0; i < SV; ++i) {
      if (64 * i >= K4) break;  // wave-uniform: no dummy loads past the row
      const int k4 = lane + 64 * i, k = 4 * k4;
      const bool okk = k4 < K4;
#pragma unroll
      for (int rr = 0; rr < RPW; ++rr) {
        const int m = m0 + wave + NWAVE * rr;
        const bool ok = okk && m < M;
        const bool seg1 = k < o.ksA;
        const float* base = seg1 ? o.A : o.A2;
        const unsigned e = ok ? (unsigned)(seg1 ? m * o.lda + k : m * o.lda2 + k - o.ksA) : 0u;
        xa[rr][i] = dr_ld4(ok ? base : o.W, e);
        if (!ok) xa[rr][i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (AMODE == AM_LNBWD || AMODE == AM_STEBWD) {
          xp[rr][i] = dr_ld4(pre, ok ? (unsigned)(m * ld_pre + k) : 0u);
          if (!ok) xp[rr][i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int jj = 0; jj < BPW; ++jj) {
        const int nl = wave + NWAVE * jj, n = n0 + nl;
        const bool ok = okk && nl < NT && n < N;
        xb[jj][i] = dr_ld4(o.W, ok ? (unsigned)(n * o.ldb + k) : 0u);
        if (!ok) xb[jj][i] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (AMODE == AM_LNSILU || AMODE == AM_LNBWD) {
        gv[i] = dr_ld4(lg, okk ? (unsigned)k : 0u);
        bv[i] = dr_ld4(lb, okk ? (unsigned)k : 0u);
      }
    }
    DR_TS(dr_tbuf_gemm, 2);
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const int ml = wave + NWAVE * rr, m = m0 + ml;
      if (AMODE == AM_LNSILU) {
        float sm = 0.f;
#pragma unroll
        for (int i = 0; i < SV; ++i) {
          if (64 * i >= K4) break;
          sm += (xa[rr][i].x + xa[rr][i].y) + (xa[rr][i].z + xa[rr][i].w);
        }
        const float mean = wave_sum(sm) / (float)K;
        float sq = 0.f;
#pragma unroll
        for (int i = 0; i < SV; ++i) {
          if (64 * i >= K4) break;
          if (lane + 64 * i < K4) {
            const float dx = xa[rr][i].x - mean, dy = xa[rr][i].y - mean;
            const float dz = xa[rr][i].z - mean, dw = xa[rr][i].w - mean;
            sq += (dx * dx + dy * dy) + (dz * dz + dw * dw);
          }
        }
        const float rstd = 1.0f / sqrtf(wave_sum(sq) / (float)K + 1e-5f);
#pragma unroll
        for (int i = 0; i < SV; ++i) {
          if (64 * i >= K4) break;
          float4& x = xa[rr][i];
          x.x = dr_silu_fast((x.x - mean) * rstd * gv[i].x + bv[i].x);
          x.y = dr_silu_fast((x.y - mean) * rstd * gv[i].y + bv[i].y);
          x.z = dr_silu_fast((x.z - mean) * rstd * gv[i].z + bv[i].z);
          x.w = dr_silu_fast((x.w - mean) * rstd * gv[i].w + bv[i].w);
          if (m >= M) x = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
      if (AMODE == AM_STEBWD) {
        // straight-through softmax backward: a group of C classes is C/4
        // consecutive lanes of one float4 chunk (K % C == 0, host-checked)
        const int gl = dr_uni(g.C) >> 2;
#pragma unroll
        for (int i = 0; i < SV; ++i) {
          if (64 * i >= K4) break;
          float4& x = xa[rr][i];
          const float4& sv = xp[rr][i];
          const float gx = 0.99f * x.x, gy = 0.99f * x.y, gz = 0.99f * x.z, gw = 0.99f * x.w;
          float dot = (gx * sv.x + gy * sv.y) + (gz * sv.z + gw * sv.w);
          for (int o = 1; o < gl; o <<= 1) dot += __shfl_xor(dot, o, 64);
          x.x = sv.x * (gx - dot);
          x.y = sv.y * (gy - dot);
          x.z = sv.z * (gz - dot);
          x.w = sv.w * (gw - dot);
          if (m >= M) x = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
      if (AMODE == AM_LNBWD) {
        // SiLU(LayerNorm(pre)) backward (ops.hip k_ln_silu_bwd, restated on
        // registers): x_hat, y, s = sigmoid(y), dy = gx * s(1 + y(1 - s)),
        // dx_hat = dy*gamma, g_pre = rstd (dx_hat - mean(dx_hat) - x_hat mean(dx_hat x_hat))
        const int PR = (AMODE == AM_LNBWD) ? rr : 0;
        float sm = 0.f;
#pragma unroll
        for (int i = 0; i < SV; ++i) {
          if (64 * i >= K4) break;
          sm += (xp[PR][i].x + xp[PR][i].y) + (xp[PR][i].z + xp[PR][i].w);
        }
        const float mean = wave_sum(sm) / (float)K;
        float sq = 0.f;
#pragma unroll
        for (int i = 0; i < SV; ++i) {
          if (64 * i >= K4) break;
          if (lane + 64 * i < K4) {
            const float dx = xp[PR][i].x - mean, dy = xp[PR][i].y - mean;
            const float dz = xp[PR][i].z - mean, dw = xp[PR][i].w - mean;
            sq += (dx * dx + dy * dy) + (dz * dz + dw * dw);
          }
        }
        const float rstd = 1.0f / sqrtf(wave_sum(sq) / (float)K + 1e-5f);
        float c1 = 0.f, c2 = 0.f;
        float* sgy = dr_uni(g.sv_gy);
        float* sxh = dr_uni(g.sv_xh);
        const int ld_sv = dr_uni((int)g.ld_sv);
        const bool save = sgy && tn == 0 && m < M;
#pragma unroll
        for (int i = 0; i < SV; ++i) {
          if (64 * i >= K4) break;
          const int k4 = lane + 64 * i;
          const bool okk = k4 < K4;
          float4 xh, gy;
          float* xhp = &xh.x;
          float* gyp = &gy.x;
          const float* pp = &xp[PR][i].x;
          const float* gxp = &xa[rr][i].x;
          const float* gg = &gv[i].x;
          const float* bb4 = &bv[i].x;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const float x_h = (pp[c] - mean) * rstd;
            const float y = x_h * gg[c] + bb4[c];
            const float sg = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(y * -1.4426950408889634f));
            const float gyv = gxp[c] * (sg * (1.0f + y * (1.0f - sg)));
            const float gxh = gyv * gg[c];
            xhp[c] = x_h;
            gyp[c] = gxh;  // keep dx_hat for the last pass
            if (okk) {
              c1 += gxh;
              c2 += gxh * x_h;
            }
            if (save && okk) {
              dr_g(sgy)[(unsigned)(m * ld_sv + 4 * k4 + c)] = gyv;
              dr_g(sxh)[(unsigned)(m * ld_sv + 4 * k4 + c)] = x_h;
            }
          }
          xa[rr][i] = gy;   // dx_hat
          xp[PR][i] = xh;   // x_hat
        }
        c1 = wave_sum(c1) / (float)K;
        c2 = wave_sum(c2) / (float)K;
#pragma unroll
        for (int i = 0; i < SV; ++i) {
          if (64 * i >= K4) break;
          float4& x = xa[rr][i];
          const float4& h = xp[PR][i];
          x.x = rstd * (x.x - c1 - h.x * c2);
          x.y = rstd * (x.y - c1 - h.y * c2);
          x.z = rstd * (x.z - c1 - h.z * c2);
          x.w = rstd * (x.w - c1 - h.w * c2);
          if (m >= M) x = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int i = 0; i < SV; ++i) {
        if (64 * i >= K4) break;
        const int k4 = lane + 64 * i;
        if (k4 < K4) {
          *reinterpret_cast<float4*>(&sA[ml * KP + 4 * k4]) = xa[rr][i];
          if (store_a && m < M) dr_st4(a_out, (unsigned)(m * ld_aout + 4 * k4), xa[rr][i]);
        }
      }
    }
#pragma unroll
    for (int jj = 0; jj < BPW; ++jj) {
      const int nl = wave + NWAVE * jj;
      if (nl >= NT) break;
#pragma unroll
      for (int i = 0; i < SV; ++i) {
        if (64 * i >= K4) break;
        const int k4 = lane + 64 * i;
        if (k4 < K4) *reinterpret_cast<float4*>(&sB[nl * KP + 4 * k4]) = xb[jj][i];
      }
    }
    DR_TS(dr_tbuf_gemm, 6);
    __syncthreads();
    DR_TS(dr_tbuf_gemm, 3);
    for (int k16 = kb; k16 < ke; k16 += 16) {
      const int kq = k16 + 4 * q;
      const bool okq = kq < K;
      f32x4 (&ac)[FT][FN] = (DUAL && (((k16 - kb) >> 4) & 1)) ? acc2 : acc;
      float4 fa[FT], fb[FN];
#pragma unroll
      for (int t = 0; t < FT; ++t) {
        fa[t] = *reinterpret_cast<const float4*>(&sA[(t * 16 + r) * KP + (okq ? kq : 0)]);
        if (!okq) fa[t] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        fb[j] = *reinterpret_cast<const float4*>(&sB[(j * 16 + r) * KP + (okq ? kq : 0)]);
        if (!okq) fb[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int t = 0; t < FT; ++t)
#pragma unroll
        for (int j = 0; j < FN; ++j) ac[t][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[t].x, fb[j].x, ac[t][j], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < FT; ++t)
#pragma unroll
        for (int j = 0; j < FN; ++j) ac[t][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[t].y, fb[j].y, ac[t][j], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < FT; ++t)
#pragma unroll
        for (int j = 0; j < FN; ++j) ac[t][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[t].z, fb[j].z, ac[t][j], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < FT; ++t)
#pragma unroll
        for (int j = 0; j < FN; ++j) ac[t][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[t].w, fb[j].w, ac[t][j], 0, 0, 0);
    }
  } else {
    // K loop in batches of PRE 16-k chunks: every load of a batch is issued
    // before its first MFMA, so a wave pays one memory round trip per batch
    // (one in total for K <= PRE*16*8 = 1024).  The first batch of weights (and
    // of plain A rows) is issued before the LayerNorm staging.
    constexpr int PRE = (FT >= 4) ? 4 : 8;
    float bb[PRE][FN][4];
    float aa[PRE][FT][4];
    auto load_batch = [&](int kc) {
  #pragma unroll
      for (int p = 0; p < PRE; ++p) {
        const int k16 = kc + 16 * p;
        const int kq = k16 + 4 * q;
        const bool live = k16 < ke;
  #pragma unroll
        for (int j = 0; j < FN; ++j) {
          if (live) {
            skinny_load_b<B_KN, VEC>(o, n0 + j * 16 + r, kq, bb[p][j]);
          } else {
  #pragma unroll
            for (int c = 0; c < 4; ++c) bb[p][j][c] = 0.f;
          }
        }
        if (AMODE != AM_LNSILU) {
  #pragma unroll
          for (int t = 0; t < FT; ++t) {
            if (live) {
              skinny_load_a<VEC>(o, m0 + t * 16 + r, k16, kq, aa[p][t]);
            } else {
  #pragma unroll
              for (int c = 0; c < 4; ++c) aa[p][t][c] = 0.f;
            }
          }
        }
      }
    };
    if (kb < ke) load_batch(kb);

    // direct path: LayerNorm (when K > 1024) from global memory; large-K rows
    // staged (K <= 256 * LNV) like the staged path's A tile
    constexpr int LNV = (MT == 16) ? 8 : 2;
    const bool ln_lds = (AMODE == AM_LNSILU) && VEC && (MT * KP <= SK_LN_MAXF) && (K4 <= 64 * LNV);
    if (AMODE == AM_LNSILU) {
      if (ln_lds) {
        const float* lg = dr_uni(g.ln_g);
        const float* lb = dr_uni(g.ln_b);
        float4 xv[RPW][LNV], gv[LNV], bv[LNV];
  #pragma unroll
        for (int i = 0; i < LNV; ++i) {
          if (64 * i >= K4) break;  // wave-uniform: no dummy loads past the row
          const int k4 = lane + 64 * i;
          const bool okk = k4 < K4;
          gv[i] = dr_ld4(lg, okk ? (unsigned)(4 * k4) : 0u);
          bv[i] = dr_ld4(lb, okk ? (unsigned)(4 * k4) : 0u);
  #pragma unroll
          for (int rr = 0; rr < RPW; ++rr) {
            const int m = m0 + wave + NWAVE * rr;
            const bool ok = okk && m < M;
            xv[rr][i] = dr_ld4(o.A, ok ? (unsigned)(m * o.lda + 4 * k4) : 0u);
            if (!ok) xv[rr][i] = make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
  #pragma unroll
        for (int rr = 0; rr < RPW; ++rr) {
          const int ml = wave + NWAVE * rr, m = m0 + ml;
          float sm = 0.f;
  #pragma unroll
          for (int i = 0; i < LNV; ++i) {
            if (64 * i >= K4) break;
            sm += (xv[rr][i].x + xv[rr][i].y) + (xv[rr][i].z + xv[rr][i].w);
          }
          const float mean = wave_sum(sm) / (float)K;
          float sq = 0.f;
  #pragma unroll
          for (int i = 0; i < LNV; ++i) {
            if (64 * i >= K4) break;
            if (lane + 64 * i < K4) {
              const float dx = xv[rr][i].x - mean, dy = xv[rr][i].y - mean;
              const float dz = xv[rr][i].z - mean, dw = xv[rr][i].w - mean;
              sq += (dx * dx + dy * dy) + (dz * dz + dw * dw);
            }
          }
          const float rstd = 1.0f / sqrtf(wave_sum(sq) / (float)K + 1e-5f);
  #pragma unroll
          for (int i = 0; i < LNV; ++i) {
            if (64 * i >= K4) break;
            const int k4 = lane + 64 * i;
            if (k4 < K4) {
              float4 y;
              y.x = dr_silu_fast((xv[rr][i].x - mean) * rstd * gv[i].x + bv[i].x);
              y.y = dr_silu_fast((xv[rr][i].y - mean) * rstd * gv[i].y + bv[i].y);
              y.z = dr_silu_fast((xv[rr][i].z - mean) * rstd * gv[i].z + bv[i].z);
              y.w = dr_silu_fast((xv[rr][i].w - mean) * rstd * gv[i].w + bv[i].w);
              if (m >= M) y = make_float4(0.f, 0.f, 0.f, 0.f);
              *reinterpret_cast<float4*>(&smem[ml * KP + 4 * k4]) = y;
              if (store_a && m < M) dr_st4(a_out, (unsigned)(m * ld_aout + 4 * k4), y);
            }
          }
        }
      } else {
        for (int rr = wave; rr < MT; rr += NWAVE) {
          const int m = m0 + rr;
          float mean = 0.f, rstd = 0.f;
          if (m < M) {
            const DR_GLOBAL float* row = dr_g(o.A) + (long long)m * o.lda;
            float s = 0.f, v = 0.f;
            for (int k = lane; k < K; k += 64) s += row[k];
            mean = wave_sum(s) / (float)K;
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
      }
      __syncthreads();
    }

    const float* lg = dr_uni(g.ln_g);
    const float* lb = dr_uni(g.ln_b);
    for (int kc = kb; kc < ke; kc += PRE * 16) {
      if (kc != kb) load_batch(kc);
      if (AMODE == AM_LNSILU) {
  #pragma unroll
        for (int p = 0; p < PRE; ++p) {
          const int k16 = kc + 16 * p;
          const int kq = k16 + 4 * q;
          const bool live = k16 < ke;
  #pragma unroll
          for (int t = 0; t < FT; ++t) {
            const int ml = t * 16 + r, m = m0 + ml;
            if (!live) {
  #pragma unroll
              for (int c = 0; c < 4; ++c) aa[p][t][c] = 0.f;
            } else if (ln_lds) {
              if (m < M && kq < K) {
                const float4 v = *reinterpret_cast<const float4*>(&smem[ml * KP + kq]);
                aa[p][t][0] = v.x; aa[p][t][1] = v.y; aa[p][t][2] = v.z; aa[p][t][3] = v.w;
              } else {
                aa[p][t][0] = aa[p][t][1] = aa[p][t][2] = aa[p][t][3] = 0.f;
              }
            } else {
              skinny_load_a<VEC>(o, m, k16, kq, aa[p][t]);
            }
          }
        }
      }
  #pragma unroll
      for (int p = 0; p < PRE; ++p) {
        if (kc + 16 * p >= ke) break;
        const int kq = kc + 16 * p + 4 * q;
  #pragma unroll
        for (int t = 0; t < FT; ++t) {
          const int ml = t * 16 + r, m = m0 + ml;
          if (AMODE == AM_LNSILU && !ln_lds) {  // global fallback: transform on the fly
            const float mean = s_mean[ml], rstd = s_rstd[ml];
  #pragma unroll
            for (int c = 0; c < 4; ++c) {
              const int k = kq + c;
              if (m < M && k < K) {
                float x = (aa[p][t][c] - mean) * rstd;
                x = x * dr_ld1(lg, (unsigned)k) + dr_ld1(lb, (unsigned)k);
                aa[p][t][c] = dr_silu_fast(x);
              }
            }
          }
          if (store_a && m < M && !(AMODE == AM_LNSILU && ln_lds)) {
  #pragma unroll
            for (int c = 0; c < 4; ++c)
              if (kq + c < K) dr_g(a_out)[(unsigned)(m * ld_aout + kq + c)] = aa[p][t][c];
          }
        }
        f32x4 (&ac)[FT][FN] = (DUAL && (p & 1)) ? acc2 : acc;
  #pragma unroll
        for (int c = 0; c < 4; ++c)
  #pragma unroll
          for (int t = 0; t < FT; ++t)
  #pragma unroll
            for (int j = 0; j < FN; ++j)
              ac[t][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(aa[p][t][c], bb[p][j][c], ac[t][j], 0, 0, 0);
      }
    }
  }
  if (DUAL) {
#pragma unroll
    for (int t = 0; t < FT; ++t)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[t][j] += acc2[t][j];
  }
  DR_TS(dr_tbuf_gemm, 4);
  if (staged || AMODE == AM_LNSILU) __syncthreads();  // smem held the staged rows
#pragma unroll
  for (int t = 0; t < FT; ++t)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) smem[(((wave * FT + t) * FN + j) * 4 + e) * 64 + lane] = acc[t][j][e];
  __syncthreads();
  DR_TS(dr_tbuf_gemm, 5);
  // element (t, j, e, l): D[row 4*(l>>4)+e][col l&15] of tile (t, j)
#pragma unroll
  for (int i = 0; i < NEPI; ++i) {
    const int x = tid + NTH * i;
    if (x >= FT * FN * 256) break;
    const int l = x & 63, e = (x >> 6) & 3, tj = x >> 8;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) v += smem[((w * FT * FN + tj) * 4 + e) * 64 + l];
    const int t = tj / FN, j = tj - t * FN;
    const int ml = t * 16 + 4 * (l >> 4) + e, nl = j * 16 + (l & 15);
    const int m = m0 + ml, n = n0 + nl;
    if (EPI == EPI_NONE || g.epi == EPI_NONE) {
      if (m < M && n < N) epilogue_store_b(g, m, n, v, ebias[i]);
    } else {
      if (m < M && n < N) {
        float y = v + ebias[i];
        if (g.Y) dr_g(g.Y)[(long long)m * g.ldy + n] = y;
        s_out[ml][nl] = y;
      }
    }
  }
  if (EPI == EPI_SAMPLE) {
    // groups of C classes inside this NT-column tile; W lanes per group
    __syncthreads();
    const int C = g.C;
    int W = 1;
    while (W < C) W <<= 1;
    const int gpr = NT / C;                // groups per row in this tile
    const int npairs = MT * gpr;           // (row, group) pairs
    const int per_wave = 64 / W;
    for (int pbase = wave * per_wave; pbase < npairs; pbase += NWAVE * per_wave) {
      const int pidx = pbase + lane / W, c = lane % W;
      const bool valid = pidx < npairs;
      const int ml = valid ? pidx / gpr : 0, gl = valid ? pidx - ml * gpr : 0;
      const int m = m0 + ml, grp = (n0 / C) + gl;
      const bool act = valid && c < C && m < M && (n0 + gl * C + c) < N;
      const float x = act ? s_out[ml][gl * C + c] : -INFINITY;
      const float mx = group_max(x, W);
      const float ex = act ? expf(x - mx) : 0.0f;
      const float se = group_sum(ex, W);
      const float p = ex / se;
      const float pu = act ? (0.99f * p + g.unimix) : 0.0f;
      const float sp = group_sum(pu, W);
      const float ph = pu / sp;
      float qv = 1.0f;
      const int Rg = g.R;
      if (act) {
        if (g.noise.q) qv = dr_g(g.noise.q)[((long long)g.step * M * Rg + (long long)m * Rg + grp) * C + c];
        else qv = dr_exp1_k(rng_seed, rng_off, (uint32_t)(g.noise.stream + g.step), (uint32_t)(g.noise.row0 + m),
                            (uint32_t)(grp * C + c));
      }
      float best = act ? ph / qv : -INFINITY;
      int bi = act ? c : 0x7fffffff;
      group_argmax(best, bi, W);
      if (act) {
        dr_g(g.z_out)[(long long)m * g.ldz + grp * C + c] = (c == bi) ? ((1.0f + pu) - pu) : 0.0f;
        if (g.soft_out) dr_g(g.soft_out)[(long long)m * g.ld_soft + grp * C + c] = p;
        if (g.idx_out && c == 0) dr_g(g.idx_out)[m * Rg + grp] = bi;
        if (g.zval_out && c == bi) dr_g(g.zval_out)[m * Rg + grp] = (1.0f + pu) - pu;
      }
    }
    DR_TS(dr_tbuf_gemm, 7);
  } else if (EPI == EPI_ACTOR && g.epi == EPI_ACTOR) {
    __syncthreads();
    const int A = g.na;
    for (int x = tid; x < MT * A; x += NTH) {
      const int ml = x / A, i = x - ml * A, m = m0 + ml;
      if (m >= M) continue;
      const float muv = s_out[ml][i];
      const float lr = s_out[ml][A + i];
      const float ls = fminf(fmaxf(lr, -5.0f), 2.0f);
      const float sg = dr_softplus(ls) + 1e-3f;
      float av;
      if (g.det) {
        av = tanhf(muv);
      } else {
        float e;
        if (g.noise.eps) e = dr_g(g.noise.eps)[((long long)g.step * M + m) * A + i];
        else e = dr_normal_k(rng_seed, rng_off, (uint32_t)(g.noise.stream + g.step), (uint32_t)(g.noise.row0 + m),
                             (uint32_t)i);
        if (g.eps_save) dr_g(g.eps_save)[(long long)m * A + i] = e;
        av = tanhf(muv + e * sg);
      }
      if (g.act_out) dr_g(g.act_out)[(long long)m * g.ld_act + i] = av;
      if (g.mu_out) dr_g(g.mu_out)[(long long)m * g.ld_mu + i] = muv;
      if (g.sig_out) dr_g(g.sig_out)[(long long)m * g.ld_sig + i] = sg;
      if (g.ls_save) dr_g(g.ls_save)[(long long)m * g.ld_ls + i] = lr;
    }
  }
}

__device__ __forceinline__ void epilogue_store(const GemmArgs& g, int m, int n, float acc) {
  epilogue_store_b(g, m, n, acc, g.bias ? dr_g(g.bias)[n] : 0.f);
}

// ---------------------------------------------------------------------------
// The categorical-sampler head as its own kernel: logits = SiLU(LN(x)) W^T + b
// (K <= 256), then per group of C = 32 classes softmax, 1 % unimix,
// argmax(p_hat / Exp(1)) and the straight-through one-hot (VAE.py:77-99 on
// latent_mapper.3; DynamicsPredictors.py:31-40 on logit_net.6).  It runs once
// per warm-start / imagination step, 46 times per epoch, and the general
// skinny kernel spent 15.3 us on it at 256 rows (8 waves splitting a K of only
// 200, an 8-way LDS reduction, 512 workgroups in two dispatch rounds).  Here a
// workgroup of 4 waves owns 16 rows x 64 columns (two groups): the 16 rows and
// 64 weight rows are read once into LDS with every load issued before the
// first wait, the LayerNorm-SiLU runs on the way (a wave per row, DPP
// statistics), wave w then accumulates output columns 16w..16w+15 over the
// whole K (two accumulators alternating per 16-k chunk: consecutive MFMAs are
// independent), and the logits pass through LDS to the sampler, two (row,
// group) pairs per wave instruction.  256 rows = 256 workgroups, one round.
// ---------------------------------------------------------------------------
#define LS_MT 16
#define LS_NT 64
#define LS_KMAX 256
#define LS_SO (LS_NT + 4)  // logit row stride: float4 rows, the 16 x 4 fragment writes hit 64 banks
static size_t ln_sample_lds_bytes(int K) {
  const int KP = ((K + 15) & ~15) + 8;  // 8 mod 16 dwords: conflict-free ds_read_b128 fragments
  return sizeof(float) * ((size_t)(LS_MT + LS_NT) * KP + (size_t)LS_MT * LS_SO);
}

// NK = K16 / 16 k-chunks, a compile-time count: the fragment reads of the
// whole K are ds_read_b128s the compiler can issue ahead of the MFMA chain.
// Nothing after the first barrier loads from global memory: the sampler noise
// (explicit q, or the Philox draws computed while the tile loads are in
// flight) is in registers before the LayerNorm, and every load is branch-free
// (a load inside a branch is waited for at the join, one round trip each).
template <int NK>
__global__ __launch_bounds__(256) void k_ln_gemm_sample(GemmArgs ga) {
  __shared__ GemmArgs g;
  dr_stage_args(ga, g, threadIdx.x);
  const int M = dr_uni(g.M), N = dr_uni(g.N), K = dr_uni(g.K);
  const int tiles_m = (M + LS_MT - 1) / LS_MT, tiles_n = N / LS_NT;
  // row tiles reading one weight slice are adjacent (one XCD's L2)
  const int lt = dr_xcd_tile(blockIdx.x, tiles_m * tiles_n);
  if (lt < 0) return;
  const int tn = lt / tiles_m, tm = lt - tn * tiles_m;
  const int m0 = tm * LS_MT, n0 = tn * LS_NT;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;
  DR_TS(dr_tbuf_gemm, 0);
  constexpr int K16 = 16 * NK, KP = K16 + 8;
  const int K4 = K >> 2;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sA = smem;                  // [LS_MT][KP]   SiLU(LN(x)) rows
  float* sB = smem + LS_MT * KP;     // [LS_NT][KP]   weight rows
  float* sO = sB + LS_NT * KP;       // [LS_MT][LS_SO] logits
  const float* A = dr_uni(g.A);
  const float* W = dr_uni(g.W);
  const int lda = dr_uni((int)g.lda), ldb = dr_uni((int)g.ldb);
  // every global load of the tile, issued together: 4 LayerNorm rows, 16
  // weight rows, gamma / beta (one float4 per lane each: K <= 256), the bias
  // of the column this lane finalises and the sampler noise / Philox state
  // the Philox state through the scalar cache (lgkmcnt): the draws below do
  // not wait for the tile loads
  typedef const __attribute__((address_space(4))) unsigned long long* dr_cu64;
  const unsigned long long* rngp = g.noise.rng ? g.noise.rng : reinterpret_cast<const unsigned long long*>(W);
  const unsigned long long rng_seed = ((dr_cu64)rngp)[0], rng_off = ((dr_cu64)rngp)[1];
  const bool okk = lane < K4;
  const unsigned ek = okk ? (unsigned)(4 * lane) : 0u;
  float4 xa[4], xb[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wave + 4 * i;
    const bool ok = okk && m < M;
    xa[i] = dr_ld4(A, ok ? (unsigned)m * (unsigned)lda + 4u * lane : 0u);
    if (!ok) xa[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int n = n0 + 16 * wave + j;
    xb[j] = dr_ld4(W, okk ? (unsigned)n * (unsigned)ldb + 4u * lane : 0u);
    if (!okk) xb[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float4 gv = dr_ld4(dr_uni(g.ln_g), ek), bv = dr_ld4(dr_uni(g.ln_b), ek);
  const float* bias = dr_uni(g.bias);
  const int ncol = n0 + 16 * wave + r;
  const float bcol = dr_ld1(bias ? bias : W, bias ? (unsigned)ncol : 0u);
  // sampler: 16 rows x 2 groups = 32 (row, group) pairs, 8 lanes per pair
  // and 4 consecutive classes per lane: lane -> row 4 wave + lane / 16, group
  // (lane / 8) % 2, classes 4 (lane % 8) .. + 3
  constexpr int C = 32;
  const int Rg = dr_uni(g.R), sub = lane & 7, ml_s = 4 * wave + (lane >> 4), gl_s = (lane >> 3) & 1;
  const int m_s = m0 + ml_s, grp_s = (n0 >> 5) + gl_s, c_s = 4 * sub;
  const bool act_s = m_s < M;
  const float* qsrc = dr_uni(g.noise.q);
  const bool explicit_q = qsrc != nullptr;
  // explicit q: one float4 per lane, loaded branch-free (from W, unused, in
  // Philox mode) into registers of its own -- a load in a branch, or one
  // whose registers the Philox branch overwrites, is waited for right there
  const float* qb = explicit_q ? qsrc + (long long)g.step * M * Rg * C : W;
  const float4 qx = dr_ld4(qb, explicit_q ? (unsigned)(((act_s ? m_s : 0) * Rg + grp_s) * C + c_s) : 0u);
  float4 qn = make_float4(1.f, 1.f, 1.f, 1.f);
  float* a_out = dr_uni(g.a_out);
  const int ld_aout = dr_uni((int)g.ld_aout);
  const bool store_a = a_out != nullptr && tn == 0;
  DR_TS(dr_tbuf_gemm, 1);
  if (!explicit_q) {
    // Philox Exp(1) draws (VALU only) while the tile loads are in flight
    const uint32_t stream = (uint32_t)(g.noise.stream + g.step), row = (uint32_t)(g.noise.row0 + m_s);
    const uint32_t e0 = (uint32_t)(grp_s * C + c_s);
    qn.x = dr_exp1_k(rng_seed, rng_off, stream, row, e0);
    qn.y = dr_exp1_k(rng_seed, rng_off, stream, row, e0 + 1);
    qn.z = dr_exp1_k(rng_seed, rng_off, stream, row, e0 + 2);
    qn.w = dr_exp1_k(rng_seed, rng_off, stream, row, e0 + 3);
  }
  // LayerNorm (eps 1e-5) + SiLU of this wave's 4 rows, as the skinny kernel's prologue
  const bool in16 = lane < (K16 >> 2);  // lanes that write the zero-padded K16 row
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ml = wave + 4 * i, m = m0 + ml;
    float4 x = xa[i];
    const float mean = wave_sum(okk ? (x.x + x.y) + (x.z + x.w) : 0.f) / (float)K;
    float sq = 0.f;
    if (okk) {
      const float dx = x.x - mean, dy = x.y - mean, dz = x.z - mean, dw = x.w - mean;
      sq = (dx * dx + dy * dy) + (dz * dz + dw * dw);
    }
    const float rstd = 1.0f / sqrtf(wave_sum(sq) / (float)K + 1e-5f);
    float4 y;
    y.x = dr_silu_fast((x.x - mean) * rstd * gv.x + bv.x);
    y.y = dr_silu_fast((x.y - mean) * rstd * gv.y + bv.y);
    y.z = dr_silu_fast((x.z - mean) * rstd * gv.z + bv.z);
    y.w = dr_silu_fast((x.w - mean) * rstd * gv.w + bv.w);
    if (!okk || m >= M) y = make_float4(0.f, 0.f, 0.f, 0.f);
    if (in16) *reinterpret_cast<float4*>(&sA[ml * KP + 4 * lane]) = y;
    if (store_a && okk && m < M) dr_st4(a_out, (unsigned)m * (unsigned)ld_aout + 4u * lane, y);
  }
#pragma unroll
  for (int j = 0; j < 16; ++j)
    if (in16) *reinterpret_cast<float4*>(&sB[(16 * wave + j) * KP + 4 * lane]) = xb[j];
  DR_TS(dr_tbuf_gemm, 2);
  __syncthreads();
  DR_TS(dr_tbuf_gemm, 3);
  // wave w: output columns 16w..16w+15 of the 16 rows, the whole K; two
  // accumulators alternating per 16-k chunk (consecutive MFMAs independent)
  f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  const float* pa = sA + r * KP + 4 * q;
  const float* pb = sB + (16 * wave + r) * KP + 4 * q;
#pragma unroll
  for (int kc = 0; kc < NK; ++kc) {
    const float4 a = *reinterpret_cast<const float4*>(pa + 16 * kc);
    const float4 b = *reinterpret_cast<const float4*>(pb + 16 * kc);
    f32x4& t = acc[kc & 1];
    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, t, 0, 0, 0);
    t = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, t, 0, 0, 0);
  }
  DR_TS(dr_tbuf_gemm, 4);
  // logits: lane (r, q) holds rows 4q..4q+3 of column ncol
  float* Y = dr_uni(g.Y);
  const long long ldy = g.ldy;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int ml = 4 * q + e, m = m0 + ml;
    const float v = (acc[0][e] + acc[1][e]) + bcol;
    sO[ml * LS_SO + 16 * wave + r] = v;
    if (Y && m < M) dr_g(Y)[(long long)m * ldy + ncol] = v;
  }
  __syncthreads();
  DR_TS(dr_tbuf_gemm, 5);
  // the sampler (softmax, 1 % unimix, argmax(p_hat / q), straight-through
  // one-hot): 8-lane DPP reductions, no loads, no LDS permutes
  const float unimix = g.unimix;
  float x[4];
  {
    const float4 xv = *reinterpret_cast<const float4*>(&sO[ml_s * LS_SO + gl_s * C + c_s]);
    x[0] = xv.x, x[1] = xv.y, x[2] = xv.z, x[3] = xv.w;
  }
  if (explicit_q) qn = qx;
  const float qv[4] = {qn.x, qn.y, qn.z, qn.w};
  float mx = act_s ? fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])) : -INFINITY;
  mx = group_max(mx, 8);
  float ex[4], pu[4], p[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) ex[t] = act_s ? expf(x[t] - mx) : 0.0f;
  const float se = group_sum((ex[0] + ex[1]) + (ex[2] + ex[3]), 8);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    p[t] = ex[t] / se;
    pu[t] = act_s ? (0.99f * p[t] + unimix) : 0.0f;
  }
  const float sp = group_sum((pu[0] + pu[1]) + (pu[2] + pu[3]), 8);
  float best = -INFINITY;
  int bi = 0x7fffffff;
  if (act_s) {
    best = (pu[0] / sp) / qv[0];
    bi = c_s;
#pragma unroll
    for (int t = 1; t < 4; ++t) {
      const float v = (pu[t] / sp) / qv[t];
      bi = v > best ? c_s + t : bi;  // ties keep the lower class
      best = fmaxf(best, v);
    }
  }
  group_argmax(best, bi, 8);
  if (act_s) {
    float4 z;
    z.x = (c_s + 0 == bi) ? ((1.0f + pu[0]) - pu[0]) : 0.0f;
    z.y = (c_s + 1 == bi) ? ((1.0f + pu[1]) - pu[1]) : 0.0f;
    z.z = (c_s + 2 == bi) ? ((1.0f + pu[2]) - pu[2]) : 0.0f;
    z.w = (c_s + 3 == bi) ? ((1.0f + pu[3]) - pu[3]) : 0.0f;
    *(DR_GLOBAL dr_f4*)(dr_g(g.z_out) + ((long long)m_s * g.ldz + grp_s * C + c_s)) = dr_f4{z.x, z.y, z.z, z.w};
    if (g.soft_out)
      *(DR_GLOBAL dr_f4*)(dr_g(g.soft_out) + ((long long)m_s * g.ld_soft + grp_s * C + c_s)) = dr_f4{p[0], p[1], p[2], p[3]};
    if (g.idx_out && sub == 0) dr_g(g.idx_out)[m_s * Rg + grp_s] = bi;
    if (g.zval_out && (unsigned)(bi - c_s) < 4u) {
      const int t = bi - c_s;
      const float pb = t == 0 ? pu[0] : t == 1 ? pu[1] : t == 2 ? pu[2] : pu[3];
      dr_g(g.zval_out)[m_s * Rg + grp_s] = (1.0f + pb) - pb;
    }
  }
  DR_TS(dr_tbuf_gemm, 6);
}

// ---------------------------------------------------------------------------
// Tile GEMM for the mid-size problems (M >= 256 rows or TN weight gradients):
// BM x BN output tile, 4 waves (2 x 2), K in chunks of 32 double-buffered
// through LDS (rows padded to 36 floats, fragments read as float4 along k).
// Operand layouts: A [M][K] (MK) or [K][M] (KM), B [N][K] (NK) or [K][N]
// (KN); MK/NK rows load as float4 (VEC), KM/KN as coalesced scalars
// transposed into LDS.  Optional deterministic split-K: each split writes a
// partial tile to splitk_ws and k_splitk_finish sums the splits in order and
// applies the epilogue.
// ---------------------------------------------------------------------------
#define DR_TILE_SPLITS 4  // = DR_SPLITK_MAX (engine_util.h): scratch sized for it
#define TBK 32  // k-chunk granularity of the split-K ranges (kernel chunks are a multiple)

__device__ __forceinline__ float tile_b_kn(const GemmArgs& g, const float* W, int ldb, int n, int k) {
  if (k >= g.ksplitB) return dr_g(g.W2)[(long long)(k - g.ksplitB) * g.ldb2 + n];
  if (n >= g.nsplitB) return dr_g(g.W2)[(long long)k * g.ldb2 + (n - g.nsplitB)];
  return dr_ld1(W, (unsigned)(k * ldb + n));
}
// the same element as tile_b_kn as ONE branch-free load (address by select):
// a load inside a branch is waited for before the branch joins, which turned
// the tile kernel's load-ahead ring into one round trip per chunk
__device__ __forceinline__ float tile_b_kn_ld(const GemmArgs& g, const float* W, int ldb, int n, int k) {
  const bool w2k = k >= g.ksplitB, w2n = n >= g.nsplitB;
  const float* base = (w2k || w2n) ? g.W2 : W;
  const long long e = w2k ? (long long)(k - g.ksplitB) * g.ldb2 + n
                          : (w2n ? (long long)k * g.ldb2 + (n - g.nsplitB) : (long long)k * ldb + n);
  return dr_g(base)[e];
}

// NW waves: 4 as 2 x 2 (32 x 32 wave tiles at 64 x 64), 8 as 4 x 2 (16 x 16
// wave tiles at 64 x 32: two waves per SIMD hide the per-chunk barrier and
// LDS latency that one wave per SIMD exposes at these short K ranges)
template <int BM, int BN, int KC, bool A_KM, bool B_KN, bool VEC, int NW = 4>
__global__ __launch_bounds__(64 * NW) void k_gemm_tile(GemmBatch gb, int splits, int npack) {
  constexpr int NTH = 64 * NW;
  constexpr int TLDS = KC + 8;  // = 8 mod 16 dwords: conflict-free ds_read_b128 fragments
  constexpr int KQ = KC / 4;  // float4 per row piece
  __shared__ GemmArgs s_args;
  int pz;
  const int plt = dr_pack_tile<BM, BN>(gb, npack, pz);
  if (plt == -1) return;
  dr_stage_args(gb.p[pz], s_args, threadIdx.x);
  const GemmArgs& g = s_args;
  const int M = dr_uni(g.M), N = dr_uni(g.N), K = dr_uni(g.K);
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int lt = plt >= 0 ? plt : dr_xcd_tile(blockIdx.x, tiles_m * tiles_n);
  if (lt < 0) return;
  const int tn = lt / tiles_m, tm = lt - tn * tiles_m;  // m-tiles sharing a weight slice are adjacent
  const int m0 = tm * BM, n0 = tn * BN;
  const int nch = (K + KC - 1) / KC;
  const int per = (nch + splits - 1) / splits;
  const int c0 = blockIdx.y * per, c1 = min(nch, c0 + per);
  const float* A = dr_uni(g.A);
  const float* W = dr_uni(g.W);
  const int lda = dr_uni((int)g.lda), ldb = dr_uni((int)g.ldb);
  const int ksA = dr_uni(g.ksplitA);
  const float* A2 = dr_uni(g.A2);
  const int lda2 = dr_uni((int)g.lda2);

  __shared__ __attribute__((aligned(16))) float As[2][BM][TLDS];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][TLDS];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;

  // row-major loader (MK / NK): thread -> (row prow + RS i, float4 quad)
  constexpr int RS = NTH / KQ;
  constexpr int APT = BM * KQ / NTH, BPT = BN * KQ / NTH;
  // transposed loader (KM / KN): thread -> (m = tid % BM, k quad tid / BM + AQ i):
  // four scalar loads down k, each coalesced over the wave's consecutive m,
  // land as ONE float4 row piece in LDS -- the same [m][k] layout and
  // conflict-free ds_write_b128 as the row-major path (a transposing scatter
  // of float4-along-m loads hits one LDS bank 16 times)
  constexpr int AQ = NTH / BM, BQ = NTH / BN;
  constexpr int APTT = KQ / AQ, BPTT = KQ / BQ;
  static_assert(APT >= 1 && BPT >= 1 && AQ >= 1 && BQ >= 1, "tile");
  static_assert(A_KM ? APTT == APT : true, "loader");
  static_assert(B_KN ? BPTT == BPT : true, "loader");
  // register ring: chunk loads are issued PIPE chunks ahead of their use
  constexpr int PIPE = 3;
  float4 ra[PIPE][APT], rb[PIPE][BPT];
  // every load is issued unconditionally (out-of-range elements read a valid
  // address) and zeroed at the LDS store by these masks: loads under a
  // condition were each waited for before the next could issue
  unsigned mka[PIPE], mkb[PIPE];  // bit (4 i + cc) of A / B: element in range
  const int quad = tid % KQ, prow = tid / KQ;
  auto load = [&](int c, int sl) {
    const int k0 = c * KC;
    unsigned ma = 0u, mb = 0u;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      if (!A_KM) {
        const int m = m0 + prow + RS * i, k = k0 + 4 * quad;
        if (VEC) {
          const bool ok = m < M && k < K;
          const bool s1 = k < ksA;
          const float* base = s1 ? A : A2;
          const unsigned e = ok ? (unsigned)(s1 ? m * lda + k : m * lda2 + k - ksA) : 0u;
          ra[sl][i] = dr_ld4(ok ? base : W, e);
          ma |= ok ? (15u << (4 * i)) : 0u;
        } else {
          // (unaligned operands, rare: conditional scalar loads as before)
          float* v = &ra[sl][i].x;
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) {
            const int kk = k + cc;
            v[cc] = (m < M && kk < K) ? ((kk < ksA) ? dr_ld1(A, (unsigned)(m * lda + kk))
                                                    : dr_ld1(A2, (unsigned)(m * lda2 + kk - ksA)))
                                      : 0.f;
          }
          ma |= 15u << (4 * i);
        }
      } else {
        const int m = m0 + tid % BM, k = k0 + 4 * (tid / BM + AQ * i);
        float* v = &ra[sl][i].x;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          const bool ok = k + cc < K && m < M;
          v[cc] = dr_ld1(A, ok ? (unsigned)((k + cc) * lda + m) : 0u);
          ma |= ok ? (1u << (4 * i + cc)) : 0u;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      if (!B_KN) {
        const int n = n0 + prow + RS * i, k = k0 + 4 * quad;
        if (VEC) {
          const bool ok = n < N && k < K;
          rb[sl][i] = dr_ld4(W, ok ? (unsigned)(n * ldb + k) : 0u);
          mb |= ok ? (15u << (4 * i)) : 0u;
        } else {
          float* v = &rb[sl][i].x;
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) v[cc] = (n < N && k + cc < K) ? dr_ld1(W, (unsigned)(n * ldb + k + cc)) : 0.f;
          mb |= 15u << (4 * i);
        }
      } else {
        const int n = n0 + tid % BN, k = k0 + 4 * (tid / BN + BQ * i);
        float* v = &rb[sl][i].x;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          const bool ok = k + cc < K && n < N;
          v[cc] = tile_b_kn_ld(g, W, ldb, ok ? n : 0, ok ? k + cc : 0);
          mb |= ok ? (1u << (4 * i + cc)) : 0u;
        }
      }
    }
    mka[sl] = ma;
    mkb[sl] = mb;
  };
  auto masked = [](float4 v, unsigned m, int i) {
    const unsigned b = m >> (4 * i);
    return make_float4(b & 1u ? v.x : 0.f, b & 2u ? v.y : 0.f, b & 4u ? v.z : 0.f, b & 8u ? v.w : 0.f);
  };
  auto store = [&](int sl, int buf) {
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const float4 v = masked(ra[sl][i], mka[sl], i);
      if (!A_KM) {
        *reinterpret_cast<float4*>(&As[buf][prow + RS * i][4 * quad]) = v;
      } else {
        *reinterpret_cast<float4*>(&As[buf][tid % BM][4 * (tid / BM + AQ * i)]) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const float4 v = masked(rb[sl][i], mkb[sl], i);
      if (!B_KN) {
        *reinterpret_cast<float4*>(&Bs[buf][prow + RS * i][4 * quad]) = v;
      } else {
        *reinterpret_cast<float4*>(&Bs[buf][tid % BN][4 * (tid / BN + BQ * i)]) = v;
      }
    }
  };

  constexpr int WGM = NW / 2;  // waves along M (2 along N)
  constexpr int WTM = BM / WGM, WTN = BN / 2, FM = WTM / 16, FN = WTN / 16;
  static_assert(FM >= 1 && FN >= 1, "wave tile");
  const int wm0 = (wave >> 1) * WTM, wn0 = (wave & 1) * WTN;
  const int r = lane & 15, q = lane >> 4;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // (a split past the last chunk, c0 >= c1, loads chunk 0 and computes nothing)
  const int clast = max(c1 - 1, 0);
#pragma unroll
  for (int u = 0; u < PIPE; ++u) load(min(c0 + u, clast), u);
  if (c0 < c1) store(0, 0);
  __syncthreads();
  for (int cb = c0; cb < c1; cb += PIPE) {
#pragma unroll
    for (int u = 0; u < PIPE; ++u) {
      const int c = cb + u;
      if (c >= c1) break;
      const int buf = (c - c0) & 1;
      load(min(c + PIPE, clast), u);  // slot u was stored to LDS last iteration; past the end: unused
#pragma unroll
      for (int s = 0; s < KC; s += 16) {
        float4 a[FM], b[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const float4*>(&As[buf][wm0 + 16 * i + r][s + 4 * q]);
#pragma unroll
        for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const float4*>(&Bs[buf][wn0 + 16 * j + r][s + 4 * q]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
      }
      if (c + 1 < c1) store((u + 1) % PIPE, buf ^ 1);
      dr_lds_barrier();  // keeps the PIPE-ahead loads in flight
    }
  }
  float* part = g.splitk_ws;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm0 + 16 * i + 4 * q + e, n = n0 + wn0 + 16 * j + r;
        if (m >= M || n >= N) continue;
        if (splits == 1) epilogue_store(g, m, n, acc[i][j][e]);
        else dr_g(part)[((long long)blockIdx.y * M + m) * N + n] = acc[i][j][e];
      }
}

// ---------------------------------------------------------------------------
// bf16 perf-mode tile GEMM (GemmArgs.bf16): NT, f32 operands in HBM rounded to
// bf16 (RNE) as they are staged into LDS, v_mfma_f32_16x16x32_bf16 with f32
// accumulation, the f32 tile kernel's epilogue / split-K.  K chunks of 64:
// a thread stages units of 8 consecutive k (two float4 loads -> one 16-byte
// LDS row piece); rows are 40 dwords (8 mod 16): conflict-free ds_read_b128
// fragments, lane (r, q) reading k = 8q..8q+7 of its row.
// ---------------------------------------------------------------------------
typedef __bf16 dr_bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ uint32_t dr_pack_bf16x2(float a, float b) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

template <int BM, int BN, int NW>
__global__ __launch_bounds__(64 * NW) void k_gemm_tile_b16(GemmBatch gb, int splits) {
  constexpr int NTH = 64 * NW, KC = 64, UPR = KC / 8, TL = KC / 2 + 8;
  __shared__ GemmArgs s_args;
  dr_stage_args(gb.p[blockIdx.z], s_args, threadIdx.x);
  const GemmArgs& g = s_args;
  const int M = dr_uni(g.M), N = dr_uni(g.N), K = dr_uni(g.K);
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int lt = dr_xcd_tile(blockIdx.x, tiles_m * tiles_n);
  if (lt < 0) return;
  const int tn = lt / tiles_m, tm = lt - tn * tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nch = (K + KC - 1) / KC;
  const int per = (nch + splits - 1) / splits;
  const int c0 = blockIdx.y * per, c1 = min(nch, c0 + per);
  const float* A = dr_uni(g.A);
  const float* A2 = dr_uni(g.A2);
  const float* W = dr_uni(g.W);
  const int lda = dr_uni((int)g.lda), lda2 = dr_uni((int)g.lda2), ldb = dr_uni((int)g.ldb);
  const int ksA = dr_uni(g.ksplitA);
  __shared__ __attribute__((aligned(16))) uint32_t As[2][BM][TL];
  __shared__ __attribute__((aligned(16))) uint32_t Bs[2][BN][TL];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  constexpr int APT = (BM * UPR + NTH - 1) / NTH, BPT = (BN * UPR + NTH - 1) / NTH;
  // the chunk in flight stays f32 in registers, masked and rounded to bf16 at
  // the LDS store (rounding in the loader waited for the loads at once, so the
  // next chunk's loads did not overlap this chunk's MFMAs); macros, not
  // lambdas: capturing lambdas left the kernel's scalars in scratch memory
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  f32x4 ra0[APT], ra1[APT], rb0[BPT], rb1[BPT];
  unsigned mka = 0u, mkb = 0u;
#define B16_LOAD(C_)                                                                                 \
  do {                                                                                               \
    const int k0 = (C_) * KC;                                                                        \
    mka = mkb = 0u;                                                                                  \
    _Pragma("unroll") for (int i = 0; i < APT; ++i) {                                                \
      const int u = tid + NTH * i, row = u / UPR, k = k0 + 8 * (u - row * UPR), m = m0 + row;        \
      const bool ok = u < BM * UPR && m < M && k < K;                                                \
      const bool s1 = k < ksA;                                                                       \
      const float* base = ok ? (s1 ? A : A2) : W;                                                    \
      const unsigned e = ok ? (unsigned)(s1 ? m * lda + k : m * lda2 + k - ksA) : 0u;                \
      ra0[i] = *(const DR_GLOBAL f32x4*)((const DR_GLOBAL char*)base + (e << 2));                    \
      ra1[i] = *(const DR_GLOBAL f32x4*)((const DR_GLOBAL char*)base + ((e + 4u) << 2));             \
      mka |= ok ? (1u << i) : 0u;                                                                    \
    }                                                                                                \
    _Pragma("unroll") for (int i = 0; i < BPT; ++i) {                                                \
      const int u = tid + NTH * i, row = u / UPR, k = k0 + 8 * (u - row * UPR), n = n0 + row;        \
      const bool ok = u < BN * UPR && n < N && k < K;                                                \
      const unsigned e = ok ? (unsigned)(n * ldb + k) : 0u;                                          \
      rb0[i] = *(const DR_GLOBAL f32x4*)((const DR_GLOBAL char*)W + (e << 2));                       \
      rb1[i] = *(const DR_GLOBAL f32x4*)((const DR_GLOBAL char*)W + ((e + 4u) << 2));                \
      mkb |= ok ? (1u << i) : 0u;                                                                    \
    }                                                                                                \
  } while (0)
#define B16_PACK(X0_, X1_, OK_)                                                                      \
  (u32x4_t){dr_pack_bf16x2((OK_) ? (X0_)[0] : 0.f, (OK_) ? (X0_)[1] : 0.f),                          \
            dr_pack_bf16x2((OK_) ? (X0_)[2] : 0.f, (OK_) ? (X0_)[3] : 0.f),                          \
            dr_pack_bf16x2((OK_) ? (X1_)[0] : 0.f, (OK_) ? (X1_)[1] : 0.f),                          \
            dr_pack_bf16x2((OK_) ? (X1_)[2] : 0.f, (OK_) ? (X1_)[3] : 0.f)}
#define B16_STORE(BUF_)                                                                              \
  do {                                                                                               \
    _Pragma("unroll") for (int i = 0; i < APT; ++i) {                                                \
      const int u = tid + NTH * i, row = u / UPR, uc = u - row * UPR;                                \
      const bool ok = (mka >> i) & 1u;                                                               \
      if (u < BM * UPR) *reinterpret_cast<u32x4_t*>(&As[BUF_][row][4 * uc]) = B16_PACK(ra0[i], ra1[i], ok); \
    }                                                                                                \
    _Pragma("unroll") for (int i = 0; i < BPT; ++i) {                                                \
      const int u = tid + NTH * i, row = u / UPR, uc = u - row * UPR;                                \
      const bool ok = (mkb >> i) & 1u;                                                               \
      if (u < BN * UPR) *reinterpret_cast<u32x4_t*>(&Bs[BUF_][row][4 * uc]) = B16_PACK(rb0[i], rb1[i], ok); \
    }                                                                                                \
  } while (0)
  constexpr int WGM = NW / 2;
  constexpr int WTM = BM / WGM, WTN = BN / 2, FM = WTM / 16, FN = WTN / 16;
  static_assert(FM >= 1 && FN >= 1, "wave tile");
  const int wm0 = (wave >> 1) * WTM, wn0 = (wave & 1) * WTN;
  const int r = lane & 15, q = lane >> 4;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int clast = max(c1 - 1, 0);  // (a split past the last chunk loads chunk 0 and computes nothing)
  B16_LOAD(min(c0, clast));
  if (c0 < c1) B16_STORE(0);
  __syncthreads();
  for (int c = c0; c < c1; ++c) {
    const int buf = (c - c0) & 1;
    B16_LOAD(min(c + 1, clast));  // in flight while this chunk's MFMAs run (past the end: unused)
#pragma unroll
    for (int s = 0; s < KC / 32; ++s) {
      uint4 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const uint4*>(&As[buf][wm0 + 16 * i + r][16 * s + 4 * q]);
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const uint4*>(&Bs[buf][wn0 + 16 * j + r][16 * s + 4 * q]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(dr_bf16x8, a[i]),
                                                              __builtin_bit_cast(dr_bf16x8, b[j]), acc[i][j], 0, 0, 0);
    }
    if (c + 1 < c1) B16_STORE(buf ^ 1);
    __syncthreads();
  }
#undef B16_LOAD
#undef B16_PACK
#undef B16_STORE
  float* part = g.splitk_ws;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm0 + 16 * i + 4 * q + e, n = n0 + wn0 + 16 * j + r;
        if (m >= M || n >= N) continue;
        if (splits == 1) epilogue_store(g, m, n, acc[i][j][e]);
        else dr_g(part)[((long long)blockIdx.y * M + m) * N + n] = acc[i][j][e];
      }
}

// ---------------------------------------------------------------------------
// Per-step chain products at 128-512 rows (GRU hidden product, heads' first
// layers, BPTT input gradients): NT, f32 MFMA, no LDS staging.  Every wave of
// the workgroup computes the WHOLE BM x BN tile over its own run of 32-k
// blocks (K split over the waves), so no operand fragment is shared between
// waves: each lane loads its MFMA fragments straight from L2 into registers
// (lane (r, q) reads 8 consecutive k of row r: a 16-row x 128-B coalesced
// line per pair of float4 loads), D blocks ahead in a register ring, with no
// barrier in the K loop.  The 8 k of a lane feed 8 consecutive MFMAs; A and B
// use the same k order, so the sum is the product's.  The NW partial tiles
// meet once in LDS at the end.  K % 8 == 0, ksplitA % 8 == 0 (a lane's 8-run
// never straddles A / A2), 16-byte aligned rows (host-checked: wk_ok).
// ---------------------------------------------------------------------------
// npack > 0: the npack problems' tiles are packed into one linear grid (no
// workgroups of a smaller problem idle in a blockIdx.z slice sized for the
// largest: a grouped launch of the GRU hidden product (456 tiles) with a
// 56-tile Linear ran 21.7 us against 12.3 for the product alone)
template <int BM, int BN, int NW, int D, int KMAP = 0>
__global__ __launch_bounds__(64 * NW) void k_gemm_wk(GemmBatch gb, int splits, int npack) {
  constexpr int NTH = 64 * NW, FM = BM / 16, FN = BN / 16, NT4 = FM * FN * 256;
  static_assert(FM * FN >= 4, "at least 4 independent accumulators per wave (40-cycle MFMA latency)");
  __shared__ GemmArgs s_args;
  __shared__ __attribute__((aligned(16))) float red[NW][FM * FN * 4][64];
  int z = blockIdx.z, lt = -1;
  if (npack > 0) {
    int tot = 0;
    for (int i = 0; i < npack; ++i) tot += ((gb.p[i].M + BM - 1) / BM) * ((gb.p[i].N + BN - 1) / BN);
    lt = dr_xcd_tile(blockIdx.x, tot);
    if (lt < 0) return;
    z = 0;
    for (int i = 0; i + 1 < npack; ++i) {
      const int ti = ((gb.p[i].M + BM - 1) / BM) * ((gb.p[i].N + BN - 1) / BN);
      if (lt < ti) break;
      lt -= ti;
      z = i + 1;
    }
  }
  dr_stage_args(gb.p[z], s_args, threadIdx.x);
  const GemmArgs& g = s_args;
  const int M = dr_uni(g.M), N = dr_uni(g.N), K = dr_uni(g.K);
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  if (npack == 0) lt = dr_xcd_tile(blockIdx.x, tiles_m * tiles_n);
  if (lt < 0) return;
  const int tn = lt / tiles_m, tm = lt - tn * tiles_m;  // m-tiles sharing a weight slice are adjacent
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
  const float* A = dr_uni(g.A);
  const float* A2 = dr_uni(g.A2);
  const float* W = dr_uni(g.W);
  const int lda = dr_uni((int)g.lda), lda2 = dr_uni((int)g.lda2), ldb = dr_uni((int)g.ldb);
  const int ksA = dr_uni(g.ksplitA);

  // bias of the outputs this thread finalises: issued now, waited for at the end
  constexpr int NEPI = (NT4 + NTH - 1) / NTH;
  float ebias[NEPI];
  {
    const float* bias = dr_uni(g.bias);
#pragma unroll
    for (int i = 0; i < NEPI; ++i) {
      const int x = tid + NTH * i, l = x & 63, tj = x >> 8;
      const int n = n0 + (tj % FN) * 16 + (l & 15);
      const bool ok = bias && splits == 1 && x < NT4 && n < N;
      const float v = dr_ld1(ok ? bias : W, ok ? (unsigned)n : 0u);
      ebias[i] = ok ? v : 0.f;
    }
  }

  // this workgroup's 32-k blocks (split-K over blockIdx.y), then this wave's
  const int nkb = (K + 31) >> 5;
  const int per = (nkb + splits - 1) / splits;
  const int kb0 = min(nkb, (int)blockIdx.y * per), kb1 = min(nkb, kb0 + per);
  const int nbg = kb1 - kb0;
  const int b0 = kb0 + (nbg * wave) / NW, b1 = kb0 + (nbg * (wave + 1)) / NW;
  const int blast = max(min(b1, nkb) - 1, 0);  // loads past this wave's run re-read its last block (unused)

  // per-lane row offsets (rows past M / N read row M-1 / N-1: valid addresses, outputs discarded)
  unsigned oa[FM], oa2[FM], ob[FN];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = min(m0 + 16 * i + r, M - 1);
    oa[i] = (unsigned)(m * lda);
    oa2[i] = (unsigned)(m * lda2);
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) ob[j] = (unsigned)(min(n0 + 16 * j + r, N - 1) * ldb);

  f32x4 ra[D][FM][2], rb[D][FN][2];
  // KMAP 0: lane q reads k = 8q..8q+7 of the block (two float4, one 32-B run);
  // KMAP 1: k = 4q..4q+3 and 16+4q..16+4q+3 (each instruction a 64-B run per row)
  constexpr int KL = KMAP == 0 ? 8 : 4, KH = KMAP == 0 ? 4 : 16;
  auto load = [&](int b, int sl) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = 32 * b + KL * q + KH * h;
      const int kk = k < K ? k : 0;  // lanes past K re-read k = 0 (zeroed before use)
      const bool s1 = kk < ksA;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const float* base = s1 ? A : A2;
        const unsigned e = s1 ? oa[i] + (unsigned)kk : oa2[i] + (unsigned)(kk - ksA);
        ra[sl][i][h] = *(const DR_GLOBAL f32x4*)((const DR_GLOBAL char*)base + (e << 2));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const unsigned e = ob[j] + (unsigned)kk;
        rb[sl][j][h] = *(const DR_GLOBAL f32x4*)((const DR_GLOBAL char*)W + (e << 2));
      }
    }
  };
  f32x4 acc[1][FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[0][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < D; ++u) load(min(b0 + u, blast), u);
  const int nbw = b1 - b0;
  const bool ktail = (K & 31) != 0;
  for (int bb = 0; bb < nbw; bb += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      if (bb + u >= nbw) break;
      const int b = b0 + bb + u;
      if (ktail && b == nkb - 1) {  // the K tail: zero the runs past K
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (32 * b + KL * q + KH * h < K) continue;
#pragma unroll
          for (int i = 0; i < FM; ++i) ra[u][i][h] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < FN; ++j) rb[u][j][h] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[0][i][j] =
                  __builtin_amdgcn_mfma_f32_16x16x4f32(ra[u][i][h][c], rb[u][j][h][c], acc[0][i][j], 0, 0, 0);
      load(min(b + D, blast), u);  // unconditional: a load under a branch is waited for at once
    }
  }
  // the NW partial tiles meet in LDS; element (t, e, l) of tile t = (i, j):
  // D[row 4 (l >> 4) + e][col l & 15]
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const f32x4 v = acc[0][i][j];
#pragma unroll
      for (int e = 0; e < 4; ++e) red[wave][(i * FN + j) * 4 + e][lane] = v[e];
    }
  __syncthreads();
  float* part = g.splitk_ws;
#pragma unroll
  for (int ii = 0; ii < NEPI; ++ii) {
    const int x = tid + NTH * ii;
    if (x >= NT4) break;
    const int l = x & 63, e = (x >> 6) & 3, tj = x >> 8;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][tj * 4 + e][l];
    const int t = tj / FN, j = tj - t * FN;
    const int m = m0 + t * 16 + 4 * (l >> 4) + e, n = n0 + j * 16 + (l & 15);
    if (m >= M || n >= N) continue;
    if (splits == 1) epilogue_store_b(g, m, n, v, ebias[ii]);
    else dr_g(part)[((long long)blockIdx.y * M + m) * N + n] = v;
  }
}

// ---------------------------------------------------------------------------
// The wave-K chain kernel on the bf16 MFMA (v_mfma_f32_16x16x32_bf16).  Same
// work split as k_gemm_wk<32, 32, 4> -- every wave computes the whole 32 x 32
// tile over its own run of 32-k chunks, fragments straight from L2 into a
// register ring, the partial tiles met once in LDS -- but the products run on
// bf16 planes: W pre-split once per call into [K/32][3][Np][32]
// (op_nt_repack_split3, RNE), the A rows split in registers as they arrive
// (split3_pair: truncation, exact residuals).  NTP = 3: the six products of
// order >= 2^-16 (conv_split.hip's f32-accurate scheme, 2.67x the f32 MFMA
// rate); NTP = 1: A rounded to bf16 (RNE) times plane 0 (bf16 perf mode).
// Lane (r, q) loads k = 8q .. 8q + 7 of its rows -- the MFMA fragment -- and
// the accumulator holds row r, columns 4q .. 4q + 3 (B fragment first).
// ---------------------------------------------------------------------------
typedef unsigned wk_u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 wk_bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 wk_mfma(wk_u32x4 a, wk_u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(wk_bf16x8, a), __builtin_bit_cast(wk_bf16x8, b),
                                                  c, 0, 0, 0);
}
__device__ __forceinline__ unsigned wk_pack_rne(float x0, float x1) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  const b2 v = {(__bf16)x0, (__bf16)x1};
  return __builtin_bit_cast(unsigned, v);
}

template <int NTP, int D, int NW = 4, int FM = 2, bool A16 = false>
__global__ __launch_bounds__(64 * NW) void k_gemm_wks3(GemmBatch gb, int npack) {
  static_assert(!A16 || NTP == 1, "bf16 A copies feed the one-term form only");
  constexpr int FN = 2, BM = 16 * FM, NTH = 64 * NW, NT4 = FM * FN * 256;
  __shared__ GemmArgs s_args;
  __shared__ __attribute__((aligned(16))) float red[NW][FM * FN * 4][64];
  int z = 0;
  const int plt = dr_pack_tile<BM, 32>(gb, npack, z);
  if (plt == -1) return;
  dr_stage_args(gb.p[z], s_args, threadIdx.x);
  const GemmArgs& g = s_args;
  const int M = dr_uni(g.M), N = dr_uni(g.N), K = dr_uni(g.K);
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + 31) / 32;
  const int lt = plt >= 0 ? plt : dr_xcd_tile(blockIdx.x, tiles_m * tiles_n);
  if (lt < 0) return;
  const int tn = lt / tiles_m, tm = lt - tn * tiles_m;  // row tiles of one weight slice adjacent
  const int m0 = tm * BM, n0 = tn * 32;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;
  const float* A = dr_uni(g.A);
  const unsigned short* A16p = dr_uni(g.A16);
  const int lda = dr_uni((int)g.lda);
  const unsigned short* wr = dr_uni(g.wsplit);
  const int Np = dr_uni(g.wsplit_np);
  // bias of the outputs this thread finalises (waited for at the end)
  constexpr int NEPI = (NT4 + NTH - 1) / NTH;
  float ebias[NEPI];
  {
    const float* bias = dr_uni(g.bias);
#pragma unroll
    for (int i = 0; i < NEPI; ++i) {
      const int x = tid + NTH * i, l = x & 63, e = (x >> 6) & 3, tj = x >> 8;
      const int n = n0 + (tj % FN) * 16 + 4 * (l >> 4) + e;
      const bool ok = bias && x < NT4 && n < N;
      ebias[i] = ok ? dr_ld1(bias, (unsigned)n) : 0.f;
    }
  }
  const int nkc = (K + 31) >> 5;
  const int c0 = (nkc * wave) / NW, c1 = (nkc * (wave + 1)) / NW;
  const int clast = max(c1 - 1, 0);
  unsigned oa[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) oa[i] = (unsigned)(min(m0 + 16 * i + r, M - 1) * lda);
  unsigned ob[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) ob[j] = (unsigned)(n0 + 16 * j + r) * 32u + 8u * q;  // within a plane (Np >= n rows)
  f32x4 ra[A16 ? 1 : D][FM][2];
  wk_u32x4 ra16[A16 ? D : 1][FM];
  wk_u32x4 rb[D][NTP][FN];
  auto load = [&](int c, int sl) {
    const int k = 32 * c + 8 * q;
    const unsigned kk = k < K ? (unsigned)k : 0u;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if constexpr (A16) {
        ra16[sl][i] = *(const DR_GLOBAL wk_u32x4*)((const DR_GLOBAL char*)A16p + ((oa[i] + kk) << 1));
      } else {
        ra[sl][i][0] = *(const DR_GLOBAL f32x4*)((const DR_GLOBAL char*)A + ((oa[i] + kk) << 2));
        ra[sl][i][1] = *(const DR_GLOBAL f32x4*)((const DR_GLOBAL char*)A + ((oa[i] + kk + 4) << 2));
      }
    }
#pragma unroll
    for (int p = 0; p < NTP; ++p)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const unsigned e = (unsigned)((c * 3 + p) * Np) * 32u + ob[j];
        rb[sl][p][j] = *(const DR_GLOBAL wk_u32x4*)((const DR_GLOBAL char*)wr + (e << 1));
      }
  };
  constexpr int NA = 1;
  f32x4 acc[NA][FM][FN];
#pragma unroll
  for (int a3 = 0; a3 < NA; ++a3)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[a3][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < D; ++u) load(min(c0 + u, clast), u);
  const int ncw = c1 - c0;
  for (int cc = 0; cc < ncw; cc += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      if (cc + u >= ncw) break;
      const int c = c0 + cc + u;
      const bool kin = 32 * c + 8 * q < K;  // K % 8 == 0: a lane's 8-run is all in or all out
      wk_u32x4 a[NTP][FM];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if constexpr (A16) {
          a[0][i] = kin ? ra16[u][i] : (wk_u32x4){0u, 0u, 0u, 0u};
          continue;
        }
        f32x4 x0 = ra[A16 ? 0 : u][i][0], x1 = ra[A16 ? 0 : u][i][1];
        if (!kin) x0 = x1 = (f32x4){0.f, 0.f, 0.f, 0.f};
        if constexpr (NTP == 3) {
          unsigned h[4], m[4], l[4];
          split3_pair(x0[0], x0[1], h[0], m[0], l[0]);
          split3_pair(x0[2], x0[3], h[1], m[1], l[1]);
          split3_pair(x1[0], x1[1], h[2], m[2], l[2]);
          split3_pair(x1[2], x1[3], h[3], m[3], l[3]);
          a[0][i] = (wk_u32x4){h[0], h[1], h[2], h[3]};
          a[1 % NTP][i] = (wk_u32x4){m[0], m[1], m[2], m[3]};
          a[2 % NTP][i] = (wk_u32x4){l[0], l[1], l[2], l[3]};
        } else {
          a[0][i] = (wk_u32x4){wk_pack_rne(x0[0], x0[1]), wk_pack_rne(x0[2], x0[3]), wk_pack_rne(x1[0], x1[1]),
                               wk_pack_rne(x1[2], x1[3])};
        }
      }
#define DR_WK3(PA, PB, X)                        \
  _Pragma("unroll") for (int i = 0; i < FM; ++i) _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[X][i][j] = \
      wk_mfma(rb[u][PB][j], a[PA][i], acc[X][i][j]);
      if constexpr (NTP == 3) {  // the six products of order >= 2^-16, smallest first
        DR_WK3(2 % NTP, 0, 0)
        DR_WK3(1 % NTP, 1 % NTP, 0)
        DR_WK3(0, 2 % NTP, 0)
        DR_WK3(1 % NTP, 0, 0)
        DR_WK3(0, 1 % NTP, 0)
      }
      DR_WK3(0, 0, 0)
#undef DR_WK3
      // unconditional: a load under a branch is waited for at once
      load(min(c + D, clast), u);
    }
  }
  // partial tiles meet in LDS; element (t, e, l) of tile t = (i, j): row 16 i + (l & 15), column 16 j + 4 (l >> 4) + e
  {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const f32x4 v = acc[0][i][j];
#pragma unroll
        for (int e = 0; e < 4; ++e) red[wave][(i * FN + j) * 4 + e][lane] = v[e];
      }
  }
  __syncthreads();
#pragma unroll
  for (int ii = 0; ii < NEPI; ++ii) {
    const int x = tid + NTH * ii;
    if (x >= NT4) break;
    const int l = x & 63, e = (x >> 6) & 3, tj = x >> 8;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][tj * 4 + e][l];
    const int t = tj / FN, j = tj - t * FN;
    const int m = m0 + t * 16 + (l & 15), n = n0 + j * 16 + 4 * (l >> 4) + e;
    if (m >= M || n >= N) continue;
    epilogue_store_b(g, m, n, v, ebias[ii]);
  }
}

__global__ __launch_bounds__(256) void k_splitk_finish(GemmBatch gb, int splits) {
  // the problem's arguments staged in LDS: read straight from the by-value
  // batch at a run-time index, the 624-byte GemmArgs was copied to scratch
  // per thread (2.6 KB per lane, ~370 us per WM-step finish, r04g)
  __shared__ GemmArgs s_args;
  dr_stage_args(gb.p[blockIdx.z], s_args, threadIdx.x);
  const GemmArgs& g = s_args;
  const long long MN = (long long)g.M * g.N;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= MN) return;
  float v = 0.f;
  for (int sp = 0; sp < splits; ++sp) v += dr_g(g.splitk_ws)[sp * MN + i];
  const int m = (int)(i / g.N), n = (int)(i - (long long)m * g.N);
  epilogue_store(g, m, n, v);
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static bool skinny_vec_ok(const GemmArgs& g, bool b_kn) {
  if (g.K % 4 != 0 || !aligned16(g.A) || g.lda % 4 != 0) return false;
  if (g.ksplitA < g.K && (!aligned16(g.A2) || g.lda2 % 4 != 0 || g.ksplitA % 4 != 0)) return false;
  if (!b_kn && (!aligned16(g.W) || g.ldb % 4 != 0)) return false;
  return true;
}

// the skinny kernel addresses A, A2, W and a_out with 32-bit element offsets
static bool skinny_offsets_ok(const GemmArgs& g, bool b_kn) {
  const long long lim = 1LL << 30;
  if ((long long)g.M * g.lda >= lim || (long long)g.M * g.lda2 >= lim) return false;
  if ((b_kn ? (long long)g.K * g.ldb : (long long)g.N * g.ldb) >= lim) return false;
  if (g.W2 && (long long)(g.K + g.N) * g.ldb2 >= lim) return false;
  if (g.a_out && (long long)g.M * g.ld_aout >= lim) return false;
  return true;
}

// Microbenchmark A/B knobs (tools/kbench) exist only in the phase-timing
// debug build; the product library has no process-wide mutable state here.
#ifdef DR_PHASE_TIMING
static size_t g_min_lds = 0;       // minimum dynamic LDS per skinny workgroup (bytes)
static int g_skinny_variant = 0;   // 1 = 64-row tiles for M <= 64, 2 = never 32-column tiles, 5 = 64-row sampler tiles
static int g_tile_wgs = 512;       // split-K target: workgroups per launch
static int g_tile_variant = 0;     // tile-GEMM shape variant
extern "C" void dr_debug_gemm_min_lds(long long bytes) { g_min_lds = (size_t)bytes; }
extern "C" void dr_debug_skinny_variant(int v) { g_skinny_variant = v; }
extern "C" void dr_debug_tile_wgs(int v) { g_tile_wgs = v > 0 ? v : 512; }
extern "C" void dr_debug_tile_variant(int v) { g_tile_variant = v; }
#else
static constexpr size_t g_min_lds = 0;
static constexpr int g_skinny_variant = 0;
static constexpr int g_tile_wgs = 512;
static constexpr int g_tile_variant = 0;
#endif
static size_t min_lds() { return g_min_lds; }

// floats of dynamic LDS a skinny launch needs (mirrors the kernel's layout)
template <int MT, int NT, int AMODE, bool B_KN>
static size_t skinny_lds_floats(const GemmBatch& gb, int count, bool vec) {
  const size_t red = (size_t)DR_SKW * (MT / 16) * (NT / 16) * 4 * 64;  // the kernel's RED
  size_t need = red;
  if (!vec) return need;
  for (int i = 0; i < count; ++i) {
    const size_t K = gb.p[i].K, KP = K + ((8 - (K & 15)) & 15);
    const size_t staged = (size_t)(MT + NT) * KP, rows = (size_t)MT * KP;
    if ((AMODE == AM_LNSILU || AMODE == AM_LNBWD || AMODE == AM_STEBWD) && !B_KN &&
        K / 4 <= 64 * (MT == 16 ? 4 : 1) &&
        staged <= SK_LN_MAXF)
      need = std::max(need, staged);  // kernel's `staged`
    else if (AMODE == AM_LNSILU && rows <= SK_LN_MAXF && K / 4 <= 64 * (MT == 16 ? 8 : 2))
      need = std::max(need, rows);  // direct path, LN rows in LDS
  }
  return need;
}

template <int MT, int NT, int AMODE, bool B_KN, int EPI>
static void launch_skinny(const GemmBatch& gb, int count, bool vec, hipStream_t s) {
  int maxt = 0;
  for (int i = 0; i < count; ++i) {
    const int t = dr_cdiv(gb.p[i].M, MT) * dr_cdiv(gb.p[i].N, NT);
    maxt = t > maxt ? t : maxt;
  }
  if (maxt == 0) return;
  const size_t lds = std::max(skinny_lds_floats<MT, NT, AMODE, B_KN>(gb, count, vec) * sizeof(float), min_lds());
  if (lds > 64 * 1024) {  // opt in to more than the default dynamic LDS (once per instantiation)
    static const bool raised = [] {
      (void)hipFuncSetAttribute((const void*)k_gemm_skinny<MT, NT, AMODE, B_KN, true, EPI>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
      (void)hipFuncSetAttribute((const void*)k_gemm_skinny<MT, NT, AMODE, B_KN, false, EPI>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
      return true;
    }();
    (void)raised;
  }
  const int npack = count > 1 ? count : 0;
  const dim3 grid(dr_xcd_grid(npack ? pack_tiles(gb, count, MT, NT) : maxt), 1, npack ? 1 : count);
  if (vec)
    hipLaunchKernelGGL((k_gemm_skinny<MT, NT, AMODE, B_KN, true, EPI>), grid, dim3(64 * DR_SKW), lds, s, gb, npack);
  else
    hipLaunchKernelGGL((k_gemm_skinny<MT, NT, AMODE, B_KN, false, EPI>), grid, dim3(64 * DR_SKW), lds, s, gb, npack);
}



// The staged backward prologues (AM_LNBWD, AM_STEBWD) run on 16-row tiles
// (K <= 1024) when the problem has at most 64 rows or its 16 x 16 grid stays
// within ~2.5 dispatch rounds (try_skinny), else on 64-row tiles (K <= 256).
bool gemm_bwd_rows16(const GemmArgs* p, int count) {
  int maxM = 0, t16 = 0;
  for (int i = 0; i < count; ++i) {
    maxM = std::max(maxM, p[i].M);
    t16 += dr_cdiv(p[i].M, 16) * dr_cdiv(p[i].N, 16);
  }
  return maxM <= 64 || (g_skinny_variant == 0 && maxM <= 4096 && t16 <= 640);
}

template <int AMODE, bool B_KN>
static bool try_skinny(const GemmBatch& gb, int count, hipStream_t s) {
  int maxM = 0, epi = EPI_NONE;
  bool vec = true;
  for (int i = 0; i < count; ++i) {
    const GemmArgs& g = gb.p[i];
    if (g.out_conv) return false;
    if ((g.epi == EPI_SAMPLE) != (gb.p[0].epi == EPI_SAMPLE)) return false;  // 32-column tiles for all or none
    if (g.epi != EPI_NONE) epi = g.epi;
    maxM = g.M > maxM ? g.M : maxM;
    if (!skinny_offsets_ok(g, B_KN)) return false;
    vec = vec && skinny_vec_ok(g, B_KN);
  }
  // fused row epilogues are validated for M <= 4096 (gemm_launch); plain
  // epilogues take any M the 32-bit offsets allow (64-row tiles past 64 rows)
  if (maxM > (epi == EPI_NONE ? (1 << 20) : 4096)) return false;
  if (g_skinny_variant == 1 && maxM > 16) maxM = 65;
  if (g_skinny_variant == 3) maxM = std::min(maxM, 64);  // 16-row tiles at any M
  // 16-row tiles past 64 rows while the grid stays within ~2.5 dispatch
  // rounds: a B = 256 per-step product (N = 200) then spreads over 208
  // workgroups instead of 52 (K = 1624: 19.3 -> 8.4 us, profiles/r02_kbench_B256.txt)
  // (also the staged LayerNorm- and softmax-STE-backward prologues:
  // at 64-row tiles a B = 256 LN-backward product ran on 52 workgroups, 16.5 us)
  if ((g_skinny_variant == 0 || g_skinny_variant == 5) && maxM > 64 &&
      (AMODE == AM_PLAIN || AMODE == AM_LNSILU || (AMODE == AM_LNBWD || AMODE == AM_STEBWD)) &&
      !(g_skinny_variant == 5 && epi == EPI_SAMPLE)) {
    int t16 = 0;
    for (int i = 0; i < count; ++i) t16 += dr_cdiv(gb.p[i].M, 16) * dr_cdiv(gb.p[i].N, epi == EPI_SAMPLE ? 32 : 16);
    if (t16 <= 640) maxM = 64;
  }
  // 16-column tiles by default; 32-column tiles when the 16-column grid would
  // exceed one workgroup per CU (these 512-thread tiles hold 1 per CU by VGPRs,
  // so a second dispatch round costs more than the wider tile's extra MFMAs)
  int tiles16 = 0;
  for (int i = 0; i < count; ++i)
    tiles16 += dr_cdiv(gb.p[i].M, maxM > 64 ? 64 : 16) * dr_cdiv(gb.p[i].N, 16);
  bool wide = g_skinny_variant != 2 && maxM <= 64 && tiles16 > 256;
  // the backward prologues exist only on the staged path (A and weight rows of
  // the tile in LDS, k_gemm_skinny `staged`): a tile whose rows do not fit
  // would read the raw operand.  At K = 1024 (the STE backward of a 32 x 32
  // latent) the 32-column tile does not fit (48 x 1032 floats), so a B = 512
  // grid (416 16-column tiles) stays on 16 columns
  if (AMODE == AM_LNBWD || AMODE == AM_STEBWD) {
    const int mt = maxM > 64 ? 64 : 16;
    for (int i = 0; i < count; ++i) {
      const int K = gb.p[i].K, KP = K + ((8 - (K & 15)) & 15);
      const int nt = (epi == EPI_SAMPLE || wide) ? 32 : 16;
      if ((mt + nt) * KP > SK_LN_MAXF && nt == 32 && epi != EPI_SAMPLE) wide = false;
      if ((mt + (wide || epi == EPI_SAMPLE ? 32 : 16)) * KP > SK_LN_MAXF || K / 4 > 64 * (mt == 16 ? 4 : 1) || !vec)
        return false;
    }
  }
  if (epi == EPI_SAMPLE) {
    if (maxM > 64) launch_skinny<64, 32, AMODE, B_KN, EPI_SAMPLE>(gb, count, vec, s);
    else launch_skinny<16, 32, AMODE, B_KN, EPI_SAMPLE>(gb, count, vec, s);
  } else if (epi == EPI_ACTOR) {
    if (maxM > 64) launch_skinny<64, 16, AMODE, B_KN, EPI_ACTOR>(gb, count, vec, s);
    else launch_skinny<16, 16, AMODE, B_KN, EPI_ACTOR>(gb, count, vec, s);
  } else {
    if (maxM > 64) launch_skinny<64, 16, AMODE, B_KN, EPI_NONE>(gb, count, vec, s);
    else if (wide) launch_skinny<16, 32, AMODE, B_KN, EPI_NONE>(gb, count, vec, s);
    else launch_skinny<16, 16, AMODE, B_KN, EPI_NONE>(gb, count, vec, s);
  }
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

// ---------------------------------------------------------------------------
// k_mlp2_tail: LN-SiLU -> Linear -> LN-SiLU -> Linear (+ epilogue), one launch
// ---------------------------------------------------------------------------
#define MLP2_KMAX 208  // K1, K2 <= 208 (the reference heads are 200 wide)
#define MLP2_NC 128
struct Mlp2Batch {
  Mlp2Args p[3];
};

// SiLU(LayerNorm(row)) of a row held one float4 per lane (k = 4 lane)
__device__ __forceinline__ float4 mlp2_ln_silu(float4 x, bool ok, int K, const float* gam, const float* bet, int k) {
  const float mean = wave_sum(ok ? (x.x + x.y) + (x.z + x.w) : 0.f) / (float)K;
  float sq = 0.f;
  if (ok) {
    const float dx = x.x - mean, dy = x.y - mean, dz = x.z - mean, dw = x.w - mean;
    sq = (dx * dx + dy * dy) + (dz * dz + dw * dw);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(sq) / (float)K + 1e-5f);
  if (!ok) return make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 gv = dr_ld4(gam, (unsigned)k), bv = dr_ld4(bet, (unsigned)k);
  return make_float4(dr_silu_fast((x.x - mean) * rstd * gv.x + bv.x), dr_silu_fast((x.y - mean) * rstd * gv.y + bv.y),
                     dr_silu_fast((x.z - mean) * rstd * gv.z + bv.z), dr_silu_fast((x.w - mean) * rstd * gv.w + bv.w));
}

// [16 rows] x [16 cols of W] over K (padded to 16): lane (r, q) holds 4
// consecutive k of weight row n (loaded up front by mlp2_wload) and reads the
// matching 4 k of LDS row r; four accumulator chains keep consecutive MFMAs
// independent
#define MLP2_KS (MLP2_KMAX / 16)
__device__ __forceinline__ void mlp2_wload(float4 (&wv)[MLP2_KS], const float* W, int ldw, int n, bool nok, int K,
                                           int q) {
  const int ks = (K + 15) >> 4;
#pragma unroll
  for (int s = 0; s < MLP2_KS; ++s) {
    const int k = 16 * s + 4 * q;
    const bool ok = s < ks && nok && k < K;
    wv[s] = dr_ld4(W, ok ? (unsigned)(n * ldw + k) : 0u);
    if (!ok) wv[s] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
template <int LP>
__device__ __forceinline__ f32x4 mlp2_tile(const float (*ys)[LP], const float4 (&wv)[MLP2_KS], int K, int r, int q) {
  const int ks = (K + 15) >> 4;
  f32x4 c[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) c[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < MLP2_KS; ++s) {
    if (s < ks) {
      const float4 a = *reinterpret_cast<const float4*>(&ys[r][16 * s + 4 * q]);
      c[s & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, wv[s].x, c[s & 3], 0, 0, 0);
      c[s & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, wv[s].y, c[s & 3], 0, 0, 0);
      c[s & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, wv[s].z, c[s & 3], 0, 0, 0);
      c[s & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, wv[s].w, c[s & 3], 0, 0, 0);
    }
  }
  f32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = (c[0][e] + c[1][e]) + (c[2][e] + c[3][e]);
  return o;
}

__global__ __launch_bounds__(512) void k_mlp2_tail(Mlp2Batch mb) {
  __shared__ Mlp2Args s_a;
  dr_stage_args(mb.p[blockIdx.z], s_a, threadIdx.x);
  const Mlp2Args& a = s_a;
  const GemmArgs& g = a.e;
  const int M = dr_uni(a.M), K1 = dr_uni(a.K1), K2 = dr_uni(a.K2), N = dr_uni(g.N);
  const int n0 = blockIdx.x * MLP2_NC, m0 = blockIdx.y * 16;
  if (n0 >= N || m0 >= M) return;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
  constexpr int LP = MLP2_KMAX + 8;  // 8 mod 16 dwords: conflict-free ds_read_b128 fragments
  __shared__ __attribute__((aligned(16))) float ys[16][LP];
  __shared__ __attribute__((aligned(16))) float hs[16][LP];
  __shared__ float so[16][MLP2_NC + 1];
  const bool c0 = blockIdx.x == 0;
  const int k = 4 * lane;
  const int ncols = min(MLP2_NC, N - n0);
  // every global operand of this wave is issued before the first use: its two
  // input rows, its (up to) two W3 tiles, its W6 tile
  const float* X = dr_uni(a.X);
  const int ldx = dr_uni((int)a.ldx);
  float4 xr[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + wave + 8 * i;
    const bool ok = m < M && k < K1;
    xr[i] = dr_ld4(X, ok ? (unsigned)(m * ldx + k) : 0u);
  }
  const int nt3 = (K2 + 15) >> 4;
  float4 w3[2][MLP2_KS];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int n = (wave + 8 * i) * 16 + r;
    mlp2_wload(w3[i], a.W3, K1, n, wave + 8 * i < nt3 && n < K2, K1, q);
  }
  const int ntd = (ncols + 15) >> 4;
  float4 w6[MLP2_KS];
  {
    const int nl = wave * 16 + r;
    mlp2_wload(w6, dr_uni(g.W), dr_uni((int)g.ldb), n0 + nl, wave < ntd && nl < ncols, K2, q);
  }

  // A: y1 = SiLU(LN1(X)), two rows per wave
  {
    const int KP = (K1 + 15) & ~15;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rr = wave + 8 * i, m = m0 + rr;
      const bool ok = m < M && k < K1;
      const float4 y = mlp2_ln_silu(xr[i], ok, K1, a.ln1_g, a.ln1_b, k);
      if (k < KP) *reinterpret_cast<float4*>(&ys[rr][k]) = y;
      if (c0 && a.a1_out && ok) dr_st4(a.a1_out, (unsigned)(m * a.ld_a1 + k), y);
    }
  }
  __syncthreads();
  // B: h2 = y1 W3^T + b3 (16-column tiles over the 8 waves)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int tj = wave + 8 * i;
    if (tj < nt3) {
      const int n = tj * 16 + r;
      const f32x4 acc = mlp2_tile<LP>(ys, w3[i], K1, r, q);
      const float bv = (n < K2 && a.b3) ? dr_ld1(a.b3, (unsigned)n) : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ml = 4 * q + e, m = m0 + ml;
        const float v = (n < K2) ? acc[e] + bv : 0.f;
        hs[ml][n] = v;
        if (c0 && a.pre2 && m < M && n < K2) dr_g(a.pre2)[(long long)m * a.ld_pre2 + n] = v;
      }
    }
  }
  __syncthreads();
  // C: y2 = SiLU(LN4(h2)), back into ys
  {
    const int KP = (K2 + 15) & ~15;
    for (int rr = wave; rr < 16; rr += 8) {
      const int m = m0 + rr;
      const bool ok = k < K2;
      float4 x = ok ? *reinterpret_cast<const float4*>(&hs[rr][k]) : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 y = mlp2_ln_silu(x, ok, K2, a.ln4_g, a.ln4_b, k);
      if (m >= M) y = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < KP) *reinterpret_cast<float4*>(&ys[rr][k]) = y;
      if (c0 && a.a2_out && ok && m < M) dr_st4(a.a2_out, (unsigned)(m * a.ld_a2 + k), y);
    }
  }
  __syncthreads();
  // D: out = y2 W6^T + b6 for columns [n0, n0 + 128): one 16-column tile per wave
  if (wave < ntd) {
    const int nl = wave * 16 + r, n = n0 + nl;
    const f32x4 acc = mlp2_tile<LP>(ys, w6, K2, r, q);
    const float bv = (nl < ncols && g.bias) ? dr_ld1(g.bias, (unsigned)n) : 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) so[4 * q + e][nl] = acc[e] + bv;
  }
  __syncthreads();
  // E: epilogue
  if (g.epi == EPI_SAMPLE) {
    const int C = g.C;
    int W = 1;
    while (W < C) W <<= 1;
    const int gpr = ncols / C, npairs = 16 * gpr, per_wave = 64 / W;
    for (int pbase = wave * per_wave; pbase < npairs; pbase += 8 * per_wave) {
      const int pidx = pbase + lane / W, c = lane % W;
      const bool valid = pidx < npairs;
      const int ml = valid ? pidx / gpr : 0, gl = valid ? pidx - ml * gpr : 0;
      const int m = m0 + ml, grp = (n0 / C) + gl;
      const bool act = valid && c < C && m < M;
      const float x = act ? so[ml][gl * C + c] : -INFINITY;
      if (act && g.Y) dr_g(g.Y)[(long long)m * g.ldy + n0 + gl * C + c] = x;
      const float mx = group_max(x, W);
      const float ex = act ? expf(x - mx) : 0.0f;
      const float se = group_sum(ex, W);
      const float p = ex / se;
      const float pu = act ? (0.99f * p + g.unimix) : 0.0f;
      const float sp = group_sum(pu, W);
      const float ph = pu / sp;
      float qv = 1.0f;
      const int Rg = g.R;
      if (act) {
        if (g.noise.q) qv = dr_g(g.noise.q)[((long long)g.step * M * Rg + (long long)m * Rg + grp) * C + c];
        else qv = dr_exp1(g.noise.rng, (uint32_t)(g.noise.stream + g.step), (uint32_t)(g.noise.row0 + m),
                          (uint32_t)(grp * C + c));
      }
      float best = act ? ph / qv : -INFINITY;
      int bi = act ? c : 0x7fffffff;
      group_argmax(best, bi, W);
      if (act) {
        dr_g(g.z_out)[(long long)m * g.ldz + grp * C + c] = (c == bi) ? ((1.0f + pu) - pu) : 0.0f;
        if (g.soft_out) dr_g(g.soft_out)[(long long)m * g.ld_soft + grp * C + c] = p;
        if (g.idx_out && c == 0) dr_g(g.idx_out)[m * Rg + grp] = bi;
        if (g.zval_out && c == bi) dr_g(g.zval_out)[m * Rg + grp] = (1.0f + pu) - pu;
      }
    }
  } else if (g.epi == EPI_ACTOR) {
    const int A = g.na;
    for (int x = tid; x < 16 * A; x += 512) {
      const int ml = x / A, i = x - ml * A, m = m0 + ml;
      if (m >= M) continue;
      const float muv = so[ml][i];
      const float lr = so[ml][A + i];
      const float ls = fminf(fmaxf(lr, -5.0f), 2.0f);
      const float sg = dr_softplus(ls) + 1e-3f;
      float av;
      if (g.det) {
        av = tanhf(muv);
      } else {
        float e;
        if (g.noise.eps) e = dr_g(g.noise.eps)[((long long)g.step * M + m) * A + i];
        else e = dr_normal(g.noise.rng, (uint32_t)(g.noise.stream + g.step), (uint32_t)(g.noise.row0 + m),
                           (uint32_t)i);
        if (g.eps_save) dr_g(g.eps_save)[(long long)m * A + i] = e;
        av = tanhf(muv + e * sg);
      }
      if (g.act_out) dr_g(g.act_out)[(long long)m * g.ld_act + i] = av;
      if (g.mu_out) dr_g(g.mu_out)[(long long)m * g.ld_mu + i] = muv;
      if (g.sig_out) dr_g(g.sig_out)[(long long)m * g.ld_sig + i] = sg;
      if (g.ls_save) dr_g(g.ls_save)[(long long)m * g.ld_ls + i] = lr;
    }
  } else {
    for (int x = tid; x < 16 * ncols; x += 512) {
      const int ml = x / ncols, nl = x - ml * ncols, m = m0 + ml;
      if (m >= M) continue;
      dr_g(g.Y)[(long long)m * g.ldy + n0 + nl] = epi_act(g, so[ml][nl]);
    }
  }
}

int mlp2_launch(const Mlp2Args* probs, int count, hipStream_t s) {
  if (count < 1 || count > 3) {
    dr_set_error("mlp2_launch: bad problem count %d", count);
    return DR_E_INVALID;
  }
  Mlp2Batch mb;
  int gx = 1, gy = 1;
  for (int i = 0; i < count; ++i) {
    const Mlp2Args& a = probs[i];
    const GemmArgs& g = a.e;
    const bool al = !(((uintptr_t)a.X | (uintptr_t)a.W3 | (uintptr_t)g.W | (uintptr_t)a.ln1_g | (uintptr_t)a.ln1_b |
                       (uintptr_t)a.ln4_g | (uintptr_t)a.ln4_b) & 15) &&
                    !((uintptr_t)a.a1_out & 15) && !((uintptr_t)a.a2_out & 15);
    if (a.M < 1 || a.K1 < 4 || a.K2 < 4 || a.K1 > MLP2_KMAX || a.K2 > MLP2_KMAX || a.K1 % 4 || a.K2 % 4 ||
        a.ldx % 4 || g.ldb % 4 || a.ld_a1 % 4 || a.ld_a2 % 4 || g.K != a.K2 || g.N < 1 || !al ||
        (g.epi == EPI_SAMPLE && (g.C < 1 || g.C > 32 || 32 % g.C != 0 || MLP2_NC % g.C != 0)) ||
        (g.epi == EPI_ACTOR && (g.N != 2 * g.na || g.N > 16)) || (g.epi == EPI_NONE && !g.Y) ||
        g.accumulate || g.addend || g.alpha != 1.0f) {
      dr_set_error("mlp2_launch: unsupported problem (M=%d K1=%d K2=%d N=%d epi=%d)", a.M, a.K1, a.K2, g.N, g.epi);
      return DR_E_INVALID;
    }
    mb.p[i] = a;
    gx = std::max(gx, dr_cdiv(g.N, MLP2_NC));
    gy = std::max(gy, dr_cdiv(a.M, 16));
  }
  hipLaunchKernelGGL(k_mlp2_tail, dim3(gx, gy, count), dim3(512), 0, s, mb);
  return dr_check_launch("mlp2_tail");
}


// mid-size GEMMs: LDS double-buffered tile kernel, split-K when the tile grid
// is too small to fill the chip and every problem brought scratch for it
template <int BM, int BN, int KC, bool A_KM, bool B_KN, int NW = 4>
static void launch_tile2(GemmBatch& gb, int count, hipStream_t s) {
  int maxt = 0, nch = 1 << 30, tot = 0;
  long long maxMN = 0;
  bool vec = true, ws = true;
  for (int i = 0; i < count; ++i) {
    const GemmArgs& g = gb.p[i];
    const int t = dr_cdiv(g.M, BM) * dr_cdiv(g.N, BN);
    maxt = std::max(maxt, t);
    tot += t;
    nch = std::min(nch, dr_cdiv(g.K, KC));
    maxMN = std::max(maxMN, (long long)g.M * g.N);
    if (!A_KM) {
      vec = vec && g.K % 4 == 0 && g.lda % 4 == 0 && aligned16(g.A);
      if (g.ksplitA < g.K) vec = vec && g.lda2 % 4 == 0 && g.ksplitA % 4 == 0 && aligned16(g.A2);
    }
    if (!B_KN) vec = vec && g.ldb % 4 == 0 && aligned16(g.W);
    ws = ws && g.splitk_ws != nullptr;
  }
  if (maxt == 0) return;
  int splits = 1;
  if (ws) {
    // about two workgroups per CU over the problems' real tiles (the grid's
    // surplus blocks of the smaller problems exit at once)
    splits = std::max(1, std::min(DR_TILE_SPLITS, dr_cdiv(g_tile_wgs, tot)));
    splits = std::min(splits, std::max(1, nch / 2));  // at least 2 chunks per split
    for (int i = 0; i < count; ++i)
      while (splits > 1 && (long long)splits * gb.p[i].M * gb.p[i].N > gb.p[i].splitk_floats) --splits;
  }
  const int npack = count > 1 ? count : 0;
  dim3 grid(dr_xcd_grid(npack ? tot : maxt), splits, npack ? 1 : count);
  if (vec) hipLaunchKernelGGL((k_gemm_tile<BM, BN, KC, A_KM, B_KN, true, NW>), grid, dim3(64 * NW), 0, s, gb, splits, npack);
  else hipLaunchKernelGGL((k_gemm_tile<BM, BN, KC, A_KM, B_KN, false, NW>), grid, dim3(64 * NW), 0, s, gb, splits, npack);
  if (splits > 1)
    hipLaunchKernelGGL(k_splitk_finish, dim3((unsigned)((maxMN + 255) / 256), 1, count), dim3(256), 0, s, gb, splits);
}


// bf16 tile launcher: split-K as launch_tile2 (partials + k_splitk_finish)
template <int BM, int BN, int NW>
static void launch_tile_b16(GemmBatch& gb, int count, hipStream_t s) {
  int maxt = 0, nch = 1 << 30, tot = 0;
  long long maxMN = 0;
  bool ws = true;
  for (int i = 0; i < count; ++i) {
    const GemmArgs& g = gb.p[i];
    const int t = dr_cdiv(g.M, BM) * dr_cdiv(g.N, BN);
    maxt = std::max(maxt, t);
    tot += t;
    nch = std::min(nch, dr_cdiv(g.K, 64));
    maxMN = std::max(maxMN, (long long)g.M * g.N);
    ws = ws && g.splitk_ws != nullptr;
  }
  if (maxt == 0) return;
  int splits = 1;
  if (ws && tot < 256) {
    splits = std::max(1, std::min(DR_TILE_SPLITS, dr_cdiv(512, tot)));
    splits = std::min(splits, std::max(1, nch / 2));
    for (int i = 0; i < count; ++i)
      while (splits > 1 && (long long)splits * gb.p[i].M * gb.p[i].N > gb.p[i].splitk_floats) --splits;
  }
  dim3 grid(dr_xcd_grid(maxt), splits, count);
  hipLaunchKernelGGL((k_gemm_tile_b16<BM, BN, NW>), grid, dim3(64 * NW), 0, s, gb, splits);
  if (splits > 1)
    hipLaunchKernelGGL(k_splitk_finish, dim3((unsigned)((maxMN + 255) / 256), 1, count), dim3(256), 0, s, gb, splits);
}

// wave-K chain kernel: 8-wide k runs on 16-byte boundaries in every operand
static bool wk_ok(const GemmBatch& gb, int count) {
  for (int i = 0; i < count; ++i) {
    const GemmArgs& g = gb.p[i];
    if (g.K % 8 || g.K < 8 || g.lda % 4 || g.ldb % 4 || ((uintptr_t)g.A & 15) || ((uintptr_t)g.W & 15)) return false;
    if (g.ksplitA < g.K && (g.ksplitA % 8 || g.lda2 % 4 || ((uintptr_t)g.A2 & 15))) return false;
    if (g.W2 || g.epi != EPI_NONE || g.out_conv || g.M < 1 || g.N < 1) return false;
  }
  return true;
}

// every problem with pre-split weight planes and the wave-K shape (NT, no second
// A segment or B segment, K % 8 == 0, 16-byte aligned rows, 32-bit offsets)
static bool wks3_ok(const GemmBatch& gb, int count) {
  for (int i = 0; i < count; ++i) {
    const GemmArgs& g = gb.p[i];
    if (!g.wsplit || g.wsplit_np < ((g.N + 31) & ~31) || g.K % 8 || g.K < 8 || g.lda % 4 || ((uintptr_t)g.A & 15) ||
        ((uintptr_t)g.wsplit & 15) || g.ksplitA < g.K || g.W2 || g.epi != EPI_NONE || g.out_conv || g.M < 1 || g.N < 1 ||
        (long long)g.M * g.lda >= (1LL << 30) || (long long)((g.K + 31) / 32) * 3 * g.wsplit_np * 32 >= (1LL << 30))
      return false;
  }
  return true;
}
// 4 waves per 32 x 32 (bf16: 16 x 32) tile, each over its own run of
// k-chunks through a register ring (r04g: 8 waves, whole-wave prefetch and A
// planes measured slower, profiles/r04g_ab_wks3.txt, r04t_ab_aplanes.txt)
// (r06o / r06p: the K loop fully unrolled -- the rolled loop's back edge makes
// the compiler wait for every outstanding load at each chunk, so the ring never
// overlaps loads with MFMAs; unrolled, the waits are per slot -- bitwise the
// same epoch, and no faster: B = 256 fp32 596 -> 596 k, bf16 909 -> 900 k (864 k
// unrolled for short K too), B = 128 fp32 446 -> 454 k; not kept,
// profiles/r06p_ab_wks3_unroll.txt.  The per-wave latency chain is not what
// bounds these launches.)
// (r05w: 64-row tiles, each weight plane read by half as many row tiles,
// measured slower -- 548 k vs 566 k fp32, 776 k vs 803 k bf16 at B = 256)
// register-ring depth (K chunks in flight per wave).  1: the fp32 kernel at 83
// VGPRs (4 waves per SIMD) instead of 140 (3), bf16 48 instead of 86 (7 / 4):
// fp32 headline 581 -> 592 k, bf16 818 -> 828 k; depth 3 / 4 slower still
// than 2 (profiles/r05zf_ab_wks3_depth.txt)
#define DR_WKS3_D 1
// 16-row fragments per tile: 2 (32 x 32 tiles) for the fp32 products, 1 for
// bf16 mode's (16 x 32 tiles: 828 -> 838 k bf16 headline; fp32 595 -> 587 k,
// kept at 2; 8 or 2 waves per tile: +0.2 % / -6 %, profiles/r05zh_ab_wks3_shape.txt)
// (64-column tiles, half the A re-reads: fp32 32 x 64 596 -> 567 k, 16 x 64
// 567 k, bf16 16 x 64 917 -> 899 k; not kept, profiles/r06w_ab_wks3_columns.txt)
#define DR_WKS3_NW 4  // waves per tile (each a 1/NW share of K)
#define DR_WKS3_FM 2
#define DR_WKS3_FM_B16 1
static void launch_wks3(const GemmBatch& gb, int count, hipStream_t s, bool bf16) {
  const int fm = bf16 ? DR_WKS3_FM_B16 : DR_WKS3_FM;
  int tot = 0, maxt = 0;
  for (int i = 0; i < count; ++i) {
    const GemmArgs& g = gb.p[i];
    const int t = dr_cdiv(g.M, 16 * fm) * dr_cdiv(g.N, 32);
    tot += t;
    maxt = std::max(maxt, t);
  }
  const int npack = count > 1 ? count : 0;
  const dim3 grid(dr_xcd_grid(npack ? tot : maxt));
  const dim3 blk(64 * DR_WKS3_NW);
  // bf16 A copies from the producers where every problem of the batch has one
  // (bitwise the same epoch; bf16 headline B = 256 891 -> 909 k, profiles/r06n_ab_a16_convT_cls.txt)
  bool a16 = bf16;
  for (int i = 0; i < count && a16; ++i) {
    const GemmArgs& g = gb.p[i];
    a16 = g.A16 && ((uintptr_t)g.A16 & 15) == 0 && g.lda % 8 == 0;
  }
  if (a16)
    hipLaunchKernelGGL((k_gemm_wks3<1, DR_WKS3_D, DR_WKS3_NW, DR_WKS3_FM_B16, true>), grid, blk, 0, s, gb, npack);
  else if (bf16) hipLaunchKernelGGL((k_gemm_wks3<1, DR_WKS3_D, DR_WKS3_NW, DR_WKS3_FM_B16>), grid, blk, 0, s, gb, npack);
  else hipLaunchKernelGGL((k_gemm_wks3<3, DR_WKS3_D, DR_WKS3_NW, DR_WKS3_FM>), grid, blk, 0, s, gb, npack);
}

// split-K over workgroups only when the tile grid is under one workgroup per
// CU and every problem brought scratch for it
template <int BM, int BN, int NW, int D, int KMAP = 0>
static void launch_wk(GemmBatch& gb, int count, hipStream_t s, int target = 256) {
  int maxt = 0, tot = 0, nkb = 1 << 30;
  long long maxMN = 0;
  bool ws = true;
  for (int i = 0; i < count; ++i) {
    const GemmArgs& g = gb.p[i];
    const int t = dr_cdiv(g.M, BM) * dr_cdiv(g.N, BN);
    maxt = std::max(maxt, t);
    tot += t;
    nkb = std::min(nkb, dr_cdiv(g.K, 32));
    maxMN = std::max(maxMN, (long long)g.M * g.N);
    ws = ws && g.splitk_ws != nullptr;
  }
  if (maxt == 0) return;
  int splits = 1;
  if (ws && tot < target) {
    splits = std::max(1, std::min(DR_TILE_SPLITS, dr_cdiv(target, tot)));
    splits = std::min(splits, std::max(1, nkb / (2 * NW)));  // at least 2 blocks per wave
    for (int i = 0; i < count; ++i)
      while (splits > 1 && (long long)splits * gb.p[i].M * gb.p[i].N > gb.p[i].splitk_floats) --splits;
  }
  if (count > 1)
    hipLaunchKernelGGL((k_gemm_wk<BM, BN, NW, D, KMAP>), dim3(dr_xcd_grid(tot), splits, 1), dim3(64 * NW), 0, s, gb,
                       splits, count);
  else
    hipLaunchKernelGGL((k_gemm_wk<BM, BN, NW, D, KMAP>), dim3(dr_xcd_grid(maxt), splits, 1), dim3(64 * NW), 0, s, gb,
                       splits, 0);
  if (splits > 1)
    hipLaunchKernelGGL(k_splitk_finish, dim3((unsigned)((maxMN + 255) / 256), 1, count), dim3(256), 0, s, gb, splits);
}

// every problem bf16 and 16-byte-aligned 8-wide k runs (ksplitA on an 8 boundary)
static bool b16_ok(const GemmBatch& gb, int count) {
  for (int i = 0; i < count; ++i) {
    const GemmArgs& g = gb.p[i];
    if (!g.bf16 || g.K % 8 || g.lda % 4 || g.ldb % 4 || ((uintptr_t)g.A & 15) || ((uintptr_t)g.W & 15)) return false;
    if (g.ksplitA < g.K && (g.ksplitA % 8 || g.lda2 % 4 || ((uintptr_t)g.A2 & 15))) return false;
    if (g.W2 || g.epi != EPI_NONE || g.out_conv) return false;
  }
  return true;
}

static bool tile_offsets_ok(const GemmBatch& gb, int count) {
  const long long lim = 1LL << 30;
  for (int i = 0; i < count; ++i) {
    const GemmArgs& g = gb.p[i];
    const long long arows = std::max((long long)g.M, (long long)g.K), brows = std::max((long long)g.N, (long long)g.K);
    if (arows * g.lda >= lim || arows * g.lda2 >= lim || brows * g.ldb >= lim) return false;
    if (g.epi != EPI_NONE || g.out_conv) return false;
  }
  return true;
}

// tall NT products (>= 1024 rows) whose caller split the weights into planes,
// f32 mode: the split3 tall GEMM of conv_split.hip (k_gemm_split3) with the
// data-gradient epilogue (accumulate, split output).  The world-model
// backward's K = 200 input gradients ran on the f32 tile kernel at ~21 TF/s.
int op_gemm_nt_split3_ex(int M, int N, int K, const float* A, int lda, const float* A2, int lda2, int ksA,
                         const void* wr, const float* bias, int act, float* Y, int ldy, int accumulate, float* Y2,
                         int ldy2, int nsplitY, float* part, size_t part_floats, hipStream_t s, int splits_fixed);
static bool s3_tall_ok(const GemmArgs& g) {
  const bool seg = g.ksplitA < g.K;  // second A segment (A2 at k >= ksplitA)
  return g.wsplit && !g.bf16 && g.M >= 1024 && g.epi == EPI_NONE && !g.out_conv && !g.W2 && !g.addend &&
         g.alpha == 1.0f && (g.act == 0 || g.act == 1) &&
         (!seg || (g.A2 && aligned16(g.A2) && g.ksplitA % 4 == 0 && g.lda2 % 4 == 0 &&
                   (long long)g.M * g.lda2 < (1LL << 31))) &&
         g.wsplit_np == (g.N + 127) / 128 * 128 &&
         g.N % 4 == 0 && g.K % 4 == 0 && g.lda % 4 == 0 && g.ldy % 4 == 0 && aligned16(g.A) && aligned16(g.Y) &&
         (!g.bias || aligned16(g.bias)) && (g.nsplitY >= g.N || (g.Y2 && aligned16(g.Y2) && g.ldy2 % 4 == 0 &&
                                                                  g.nsplitY % 4 == 0)) &&
         (long long)g.M * g.lda < (1LL << 31) && g.lda < INT_MAX && g.ldy < INT_MAX && g.ldy2 < INT_MAX;
}

// bf16 mode's chain products without weight planes on k_gemm_tile_b16 (the
// f32 wave-K kernel measured 723.3 k against 730.5 k bf16 headline,
// profiles/r03zf_ab_bf16_chain_route.txt)
template <int AMODE, bool A_KM, bool B_KN>
static int launch_pick(const GemmBatch& gb, int count, hipStream_t s) {
  if (AMODE == AM_PLAIN && !A_KM && !B_KN) {
    // problems of the batch that qualify run one after another on the split3
    // tall GEMM, the rest as a (smaller) batch below
    GemmBatch rest;
    int nrest = 0;
    for (int i = 0; i < count; ++i) {
      const GemmArgs& g = gb.p[i];
      if (!s3_tall_ok(g)) {
        rest.p[nrest++] = g;
        continue;
      }
      // (the 200-wide, K <= 1024 problems on the wave-K split3 kernel's 32 x 32
      // tiles instead -- it fills the chip where 64 x 64 tiles leave ~450 waves
      // -- measured the same WM step, r06t: not kept)
      DR_TRY(op_gemm_nt_split3_ex(g.M, g.N, g.K, g.A, (int)g.lda, g.A2, (int)g.lda2, g.ksplitA < g.K ? g.ksplitA : g.K,
                                  g.wsplit, g.bias, g.act, g.Y, (int)g.ldy, g.accumulate, g.Y2, (int)g.ldy2,
                                  g.nsplitY < g.N ? g.nsplitY : INT_MAX, g.splitk_ws,
                                  g.splitk_ws ? (size_t)g.splitk_floats : 0, s, 0));
    }
    if (nrest == 0) return DR_OK;
    if (nrest < count) return launch_pick<AMODE, A_KM, B_KN>(rest, nrest, s);
  }
  if (AMODE == AM_PLAIN && tile_offsets_ok(gb, count)) {
    int maxM = 0, minK = 1 << 30, tiles = 0;
    bool ws = true;
    for (int i = 0; i < count; ++i) {
      maxM = std::max(maxM, gb.p[i].M);
      minK = std::min(minK, gb.p[i].K);
      tiles += dr_cdiv(gb.p[i].M, 64) * dr_cdiv(gb.p[i].N, 64);
      ws = ws && gb.p[i].splitk_ws != nullptr;
    }
    // per-step products at 128-512 rows with a deep K (BPTT input gradients,
    // K = 1800; the heads' first layers, K = 1624) or a wide N (the GRU's
    // hidden product): 32 x 32 tiles, K chunks of 64, split-K only while the
    // tile grid is under one workgroup per CU.  Against the 16/64-row skinny
    // tiles, which re-read the weights per row tile and the activations per
    // 16 columns: 44 -> 32 us (BPTT, 2 problems), 23 -> 15 us (heads, 3
    // problems, split-K 4), profiles/r02h_kbench_tile_B256.txt
    // shallow-K products the caller gave weight planes (the BPTT's actor
    // input gradient, K = 200, N = 1624): the wave-K split3 kernel
    if (!A_KM && !B_KN && maxM >= 128 && maxM <= 512 && minK < 512 && g_tile_variant == 0 &&
        wks3_ok(gb, count)) {
      launch_wks3(gb, count, s, b16_ok(gb, count));
      return DR_OK;
    }
    if (!A_KM && !B_KN && maxM >= 128 && maxM <= 512 && g_tile_variant != 26) {
      int tiles32 = 0;
      for (int i = 0; i < count; ++i) tiles32 += dr_cdiv(gb.p[i].M, 32) * dr_cdiv(gb.p[i].N, 32);
      // (f32 under ~112 tiles -- one per-step Linear of 200 outputs, K = 1624 --
      // the 16-row skinny tiles spread wider: 8.4 against 13.0 us)
      if ((g_tile_variant == 0 || g_tile_variant >= 8) && maxM <= 512 &&
          ((minK >= 1024 && (tiles32 >= 112 || g_tile_variant != 0 || b16_ok(gb, count))) ||
           (minK >= 512 && tiles32 >= 256))) {
        GemmBatch gt = gb;
        if (tiles32 >= 256)
          for (int i = 0; i < count; ++i) gt.p[i].splitk_ws = nullptr;
        // f32: the wave-K kernel (32 x 32 tiles, 4 waves, no split-K: heads
        // 15.8 -> 13.0 us, BPTT 32.2 -> 25.7, GRU hidden product 13.3 -> 12.3,
        // profiles/r03g_kbench_wk.txt); the LDS tile kernel stays for the
        // shapes the wave-K kernel does not take (and as kbench variant 25)
        if (wks3_ok(gb, count)) launch_wks3(gt, count, s, b16_ok(gb, count));
        else if (b16_ok(gb, count)) launch_tile_b16<32, 32, 4>(gt, count, s);
        else if (g_tile_variant == 0 && wk_ok(gb, count)) launch_wk<32, 32, 4, 2, 1>(gt, count, s, 0);
        else if (g_tile_variant >= 12 && g_tile_variant < 25 && wk_ok(gb, count)) {
          GemmBatch gw = gb;  // (split-K scratch kept: launch_wk splits only under 256 tiles)
          switch (g_tile_variant) {
            case 12: launch_wk<32, 32, 4, 4>(gw, count, s); break;
            case 13: launch_wk<32, 32, 8, 4>(gw, count, s); break;
            case 14: launch_wk<64, 32, 8, 3>(gw, count, s); break;
            case 15: launch_wk<32, 64, 8, 3>(gw, count, s); break;
            case 16: launch_wk<32, 32, 4, 4, 1>(gw, count, s); break;
            case 18: launch_wk<32, 32, 4, 2>(gw, count, s); break;
            case 19: launch_wk<32, 32, 4, 2, 1>(gw, count, s); break;
            case 20: launch_wk<32, 32, 8, 2, 1>(gw, count, s); break;
            case 21: launch_wk<64, 64, 4, 2, 1>(gw, count, s, g_tile_wgs); break;
            case 22: launch_wk<64, 32, 4, 2, 1>(gw, count, s, g_tile_wgs); break;
            case 23: launch_wk<32, 64, 4, 2, 1>(gw, count, s, g_tile_wgs); break;
            case 24: launch_wk<64, 64, 8, 2, 1>(gw, count, s, g_tile_wgs); break;
            default:
              if (tiles32 >= 256) launch_wk<32, 32, 4, 4>(gw, count, s);
              else launch_wk<32, 32, 8, 4>(gw, count, s);
              break;
          }
        } else if (g_tile_variant == 8) launch_tile2<32, 64, 64, false, false, 4>(gt, count, s);
        else if (g_tile_variant == 9) launch_tile2<64, 32, 64, false, false, 4>(gt, count, s);
        else if (g_tile_variant == 10) launch_tile2<64, 64, 64, false, false, 4>(gt, count, s);
        else if (g_tile_variant == 11) launch_tile2<32, 64, 32, false, false, 4>(gt, count, s);
        else launch_tile2<32, 32, 64, false, false, 4>(gt, count, s);
        return DR_OK;
      }
    }
    // weight gradients (TN) and tall, deep products go to the tile kernel --
    // when it can fill the chip: a per-step product at B = 256 (16 tiles of
    // 64 x 64, no split-K scratch) runs on 52+ skinny 64-row workgroups instead
    // tall products with a small K (M >= 1024: the world-model heads' and
    // decoder's layers over B (T - 1) rows, the critic's over B (H + 1)): the
    // 64-row skinny tiles re-read the weights per row tile and run 16 columns
    // per workgroup (480 us for the decoder's 3584 x 4096 x 200 product)
    const bool tall = !A_KM && !B_KN && maxM >= 1024 && tiles >= 256 && g_tile_variant == 0;
    if (A_KM || (maxM >= 256 && minK >= 512 && (ws || tiles >= 128) && g_tile_variant != 26) || tall ||
        (g_tile_variant >= 4 && g_tile_variant < 26 && maxM >= 128)) {
      GemmBatch gt = gb;
      // tall NT products with a deep K (the encoder feature projection, the
      // critic's first layer over B*(H+1) rows): 8 waves as 4 x 2 over 64 x 64
      // with K chunks of 64 -- 198 -> 171 us (M 8192, K 4096), 51 -> 47 us
      // (M 4096, K 1624), profiles/r02m_kbench_tall_tiles.txt
      if (g_tile_variant == 0 && !A_KM && !B_KN && minK >= 1024) {
        if (b16_ok(gb, count)) launch_tile_b16<64, 64, 8>(gt, count, s);
        else launch_tile2<64, 64, 64, false, false, 8>(gt, count, s);
        return DR_OK;
      }
      switch (g_tile_variant) {
        case 1: launch_tile2<64, 64, 64, A_KM, B_KN>(gt, count, s); break;
        case 2: launch_tile2<128, 64, 32, A_KM, B_KN>(gt, count, s); break;
        case 3: launch_tile2<128, 64, 64, A_KM, B_KN>(gt, count, s); break;
        case 4: launch_tile2<64, 32, 64, A_KM, B_KN, 8>(gt, count, s); break;
        case 5: launch_tile2<128, 32, 64, A_KM, B_KN, 8>(gt, count, s); break;
        case 6: launch_tile2<64, 64, 64, A_KM, B_KN, 8>(gt, count, s); break;
        case 7: launch_tile2<32, 32, 64, A_KM, B_KN, 4>(gt, count, s); break;
        default: launch_tile2<64, 64, 32, A_KM, B_KN>(gt, count, s); break;
      }
      return DR_OK;
    }
  }
  if (AMODE == AM_LNBWD) {
    if (!A_KM && !B_KN && try_skinny<AM_LNBWD, false>(gb, count, s)) return DR_OK;
    dr_set_error("gemm: LayerNorm-backward prologue needs the staged NT skinny path");
    return DR_E_INVALID;
  }
  if (AMODE == AM_STEBWD) {
    if (!A_KM && !B_KN && try_skinny<AM_STEBWD, false>(gb, count, s)) return DR_OK;
    dr_set_error("gemm: softmax-STE-backward prologue needs the staged NT skinny path");
    return DR_E_INVALID;
  }
  if (!A_KM && (AMODE == AM_PLAIN || AMODE == AM_LNSILU)) {
    if (try_skinny<(AMODE == AM_LNSILU ? AM_LNSILU : AM_PLAIN), B_KN>(gb, count, s)) return DR_OK;
  }
  long long work = 0;
  for (int i = 0; i < count; ++i) work += (long long)gb.p[i].M * gb.p[i].N;
  // large problems: 64x64 tiles; small (per-step, M = batch rows): 32x32 tiles
  // so that the launch spreads over more CUs.
  if (work >= 256LL * 1024) launch_tile<64, 64, AMODE, A_KM, B_KN>(gb, count, s);
  else launch_tile<32, 32, AMODE, A_KM, B_KN>(gb, count, s);
  return DR_OK;
}

// the sampler-head kernel's shape: one LN-SiLU NT problem, C = 32, K <= 256
static bool ln_sample_ok(const GemmArgs& g) {
  return g.epi == EPI_SAMPLE && g.C == 32 && g.R * g.C == g.N && g.N % LS_NT == 0 && g.K > 0 && g.K % 4 == 0 &&
         g.K <= LS_KMAX && g.M > 0 && g.M <= 65536 && g.ln_g && g.ln_b && g.ksplitA >= g.K && !g.addend &&
         g.alpha == 1.0f && g.act == 0 && !g.accumulate && !g.W2 && aligned16(g.A) && aligned16(g.W) &&
         aligned16(g.ln_g) && aligned16(g.ln_b) && g.lda % 4 == 0 && g.ldb % 4 == 0 &&
         (!g.a_out || (aligned16(g.a_out) && g.ld_aout % 4 == 0)) && skinny_offsets_ok(g, false) &&
         (long long)g.M * g.ldz < (1LL << 31) && aligned16(g.z_out) && g.ldz % 4 == 0 &&
         (!g.soft_out || (aligned16(g.soft_out) && g.ld_soft % 4 == 0)) && (!g.noise.q || aligned16(g.noise.q));
}
#ifdef DR_PHASE_TIMING
static int g_ln_sample_off = 0;  // kbench A/B: 1 = the skinny kernel's sampler epilogue instead
extern "C" void dr_debug_ln_sample_off(int v) { g_ln_sample_off = v; }
#else
static constexpr int g_ln_sample_off = 0;
#endif

template <int NK>
static int launch_ln_sample_nk(const GemmArgs& g, hipStream_t s) {
  const size_t lds = ln_sample_lds_bytes(g.K);
  if (lds > 64 * 1024) {
    static const bool raised = [] {
      (void)hipFuncSetAttribute((const void*)k_ln_gemm_sample<NK>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)ln_sample_lds_bytes(16 * NK));
      return true;
    }();
    (void)raised;
  }
  const int tiles = dr_cdiv(g.M, LS_MT) * (g.N / LS_NT);
  hipLaunchKernelGGL(k_ln_gemm_sample<NK>, dim3(dr_xcd_grid(tiles)), dim3(256), lds, s, g);
  return dr_check_launch("ln_gemm_sample");
}

static int launch_ln_sample(const GemmArgs& g, hipStream_t s) {
  switch ((g.K + 15) >> 4) {  // ln_sample_ok: 0 < K <= LS_KMAX
#define DR_LS_CASE(n) \
  case n:             \
    return launch_ln_sample_nk<n>(g, s);
    DR_LS_CASE(1) DR_LS_CASE(2) DR_LS_CASE(3) DR_LS_CASE(4) DR_LS_CASE(5) DR_LS_CASE(6) DR_LS_CASE(7)
    DR_LS_CASE(8) DR_LS_CASE(9) DR_LS_CASE(10) DR_LS_CASE(11) DR_LS_CASE(12) DR_LS_CASE(13) DR_LS_CASE(14)
    DR_LS_CASE(15) DR_LS_CASE(16)
#undef DR_LS_CASE
    default:
      dr_set_error("ln_gemm_sample: K %d out of range", g.K);
      return DR_E_INVALID;
  }
}

// SiLU(LayerNorm(x)) of whole rows, one wave per row: the staged prologue of
// k_gemm_skinny (same lane -> k mapping and summation order, so the same
// values) as its own pass for tall products, whose consumers then run a plain
// tile GEMM on the result instead of re-normalising the rows per column tile
template <int LNV>
__global__ __launch_bounds__(256) void k_ln_silu_rows(int M, int K, const float* __restrict__ X, int ldx,
                                                      const float* __restrict__ gam, const float* __restrict__ bet,
                                                      float* __restrict__ Y, int ldy) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + wave;
  if (m >= M) return;  // whole waves: wave_sum stays within a live wave
  const int K4 = K >> 2;
  float4 xv[LNV], gv[LNV], bv[LNV];
#pragma unroll
  for (int i = 0; i < LNV; ++i) {
    const int k4 = lane + 64 * i;
    const bool ok = k4 < K4;
    xv[i] = ok ? *reinterpret_cast<const float4*>(X + (long long)m * ldx + 4 * k4) : make_float4(0.f, 0.f, 0.f, 0.f);
    gv[i] = ok ? *reinterpret_cast<const float4*>(gam + 4 * k4) : make_float4(0.f, 0.f, 0.f, 0.f);
    bv[i] = ok ? *reinterpret_cast<const float4*>(bet + 4 * k4) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float sm = 0.f;
#pragma unroll
  for (int i = 0; i < LNV; ++i) sm += (xv[i].x + xv[i].y) + (xv[i].z + xv[i].w);
  const float mean = wave_sum(sm) / (float)K;
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < LNV; ++i) {
    if (lane + 64 * i < K4) {
      const float dx = xv[i].x - mean, dy = xv[i].y - mean, dz = xv[i].z - mean, dw = xv[i].w - mean;
      sq += (dx * dx + dy * dy) + (dz * dz + dw * dw);
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(sq) / (float)K + 1e-5f);
#pragma unroll
  for (int i = 0; i < LNV; ++i) {
    const int k4 = lane + 64 * i;
    if (k4 < K4) {
      float4 y;
      y.x = dr_silu_fast((xv[i].x - mean) * rstd * gv[i].x + bv[i].x);
      y.y = dr_silu_fast((xv[i].y - mean) * rstd * gv[i].y + bv[i].y);
      y.z = dr_silu_fast((xv[i].z - mean) * rstd * gv[i].z + bv[i].z);
      y.w = dr_silu_fast((xv[i].w - mean) * rstd * gv[i].w + bv[i].w);
      *reinterpret_cast<float4*>(Y + (long long)m * ldy + 4 * k4) = y;
    }
  }
}

// tall LN-SiLU products (M >= 1024 rows: the world-model heads / decoder over
// B (T - 1) rows, the critic over B (H + 1)) whose transformed rows are saved
// anyway (a_out): normalise once, then the plain GEMM on the saved rows
static bool tall_ln_ok(const GemmArgs* probs, int count) {
  for (int i = 0; i < count; ++i) {
    const GemmArgs& g = probs[i];
    if (g.M < 1024 || g.epi != EPI_NONE || !g.a_out || g.K % 4 || g.K > 1024 || g.K < 4 || g.ksplitA < g.K ||
        g.lda % 4 || g.ld_aout % 4 || ((uintptr_t)g.A | (uintptr_t)g.a_out | (uintptr_t)g.ln_g | (uintptr_t)g.ln_b) & 15 ||
        (long long)g.M * std::max(g.lda, g.ld_aout) >= (1LL << 31))
      return false;
  }
  return true;
}

int gemm_launch(GemmLayout lay, int amode, const GemmArgs* probs, int count, hipStream_t s) {
  if (count < 1 || count > 4) {
    dr_set_error("gemm_launch: bad problem count %d", count);
    return DR_E_INVALID;
  }
  if (lay == G_NT && amode == AM_LNSILU && tall_ln_ok(probs, count)) {
    GemmArgs pp[4];
    for (int i = 0; i < count; ++i) {
      const GemmArgs& g = probs[i];
      const dim3 grid((unsigned)((g.M + 3) / 4));
      if (g.K <= 256)
        hipLaunchKernelGGL(k_ln_silu_rows<1>, grid, dim3(256), 0, s, g.M, g.K, g.A, (int)g.lda, g.ln_g, g.ln_b, g.a_out,
                           (int)g.ld_aout);
      else
        hipLaunchKernelGGL(k_ln_silu_rows<4>, grid, dim3(256), 0, s, g.M, g.K, g.A, (int)g.lda, g.ln_g, g.ln_b, g.a_out,
                           (int)g.ld_aout);
      DR_TRY(dr_check_launch("ln_silu_rows"));
      pp[i] = g;
      pp[i].A = g.a_out;
      pp[i].lda = g.ld_aout;
      pp[i].ln_g = pp[i].ln_b = nullptr;
      pp[i].a_out = nullptr;
    }
    return gemm_launch(G_NT, AM_PLAIN, pp, count, s);
  }
  if (lay == G_NT && amode == AM_LNSILU && count == 1 && !g_ln_sample_off && ln_sample_ok(probs[0]))
    return launch_ln_sample(probs[0], s);
  for (int i = 0; i < count; ++i) {
    const GemmArgs& g = probs[i];
    if (g.epi == EPI_SAMPLE && (g.C < 1 || g.C > 32 || 32 % g.C != 0 || g.N != g.R * g.C)) {
      dr_set_error("gemm_launch: sampler epilogue needs C | 32 and N == R*C (C=%d R=%d N=%d)", g.C, g.R, g.N);
      return DR_E_INVALID;
    }
    if (g.epi == EPI_ACTOR && (g.N != 2 * g.na || g.na > 8)) {
      dr_set_error("gemm_launch: actor epilogue needs N == 2A <= 16");
      return DR_E_INVALID;
    }
    if (g.epi != EPI_NONE && (lay != G_NT || (amode != AM_PLAIN && amode != AM_LNSILU) || g.M > 4096 ||
                              !skinny_offsets_ok(g, false))) {
      dr_set_error("gemm_launch: fused epilogues need the NT skinny path");
      return DR_E_INVALID;
    }
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
        case AM_PLAIN: DR_TRY((launch_pick<AM_PLAIN, false, false>(gb, count, s))); break;
        case AM_LNSILU: DR_TRY((launch_pick<AM_LNSILU, false, false>(gb, count, s))); break;
        case AM_CONV: DR_TRY((launch_pick<AM_CONV, false, false>(gb, count, s))); break;
        case AM_CONV_SRC: DR_TRY((launch_pick<AM_CONV_SRC, false, false>(gb, count, s))); break;
        case AM_LNBWD: {
          const bool r16 = gemm_bwd_rows16(probs, count);
          for (int i = 0; i < count; ++i) {
            const GemmArgs& g = probs[i];
            const int lim = r16 ? 1024 : 256;  // staged rows per lane: SV = 4 (MT 16) / 1 (MT 64)
            if (g.K % 4 || g.K > lim || g.lda % 4 || g.ld_pre % 4 || g.ldb % 4 ||
                ((uintptr_t)g.A | (uintptr_t)g.pre | (uintptr_t)g.W | (uintptr_t)g.ln_g | (uintptr_t)g.ln_b) & 15) {
              dr_set_error("gemm_launch: AM_LNBWD needs K %% 4 == 0, K <= %d, 16-byte aligned rows (K=%d)", lim, g.K);
              return DR_E_INVALID;
            }
          }
          DR_TRY((launch_pick<AM_LNBWD, false, false>(gb, count, s)));
          break;
        }
        case AM_STEBWD: {
          const bool r16 = gemm_bwd_rows16(probs, count);
          for (int i = 0; i < count; ++i) {
            const GemmArgs& g = probs[i];
            const int lim = r16 ? 1024 : 256;
            const int gl = g.C / 4;
            if (g.K % 4 || g.K > lim || g.lda % 4 || g.ld_pre % 4 || g.ldb % 4 || g.C < 4 || g.C % 4 ||
                (gl & (gl - 1)) || gl > 64 || g.K % g.C || !r16 ||
                ((uintptr_t)g.A | (uintptr_t)g.pre | (uintptr_t)g.W) & 15) {
              dr_set_error("gemm_launch: AM_STEBWD needs 16-row tiles (gemm_bwd_rows16), K %% C == 0, C/4 a power "
                           "of two, K <= %d, 16-byte aligned rows (K=%d C=%d)", lim, g.K, g.C);
              return DR_E_INVALID;
            }
          }
          DR_TRY((launch_pick<AM_STEBWD, false, false>(gb, count, s)));
          break;
        }
        default: dr_set_error("gemm_launch: bad amode"); return DR_E_INVALID;
      }
      break;
    case G_NN: DR_TRY((launch_pick<AM_PLAIN, false, true>(gb, count, s))); break;
    case G_TN: DR_TRY((launch_pick<AM_PLAIN, true, true>(gb, count, s))); break;
  }
  return dr_check_launch("gemm");
}
