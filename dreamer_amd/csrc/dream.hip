// Persistent imagination unroll: Dreamer.dream_episodes (Dreamer.py:143-175)
// as ONE launch instead of seven launches per imagined step.
//
// Per step s = 0 .. H-1 (WorldModel.imagine_step WorldModel.py:72-77, the
// actor Agent.py:191-210, the prior DynamicsPredictors.py:25-40):
//
//   DA   pre1a_s = hA_s + sum_g zval W_a0z^T[g * 32 + idx_g]       actor base_net.0 (hA_s = h_s W_a0h^T + b)
//   DB   x1a_s = SiLU(LN(pre1a_s)),  pre2a_s = x1a_s W_a3^T + b     actor base_net.1-3
//   DG   x2a_s = SiLU(LN(pre2a_s)), [mu | log_sig] = x2a_s W_st^T + b, a_s = tanh(mu + eps sigma)
//        (heads, recomputed for the tile's rows in every unit slice), then
//        h_{s+1} = GRUCell(cat(z_s, a_s), h_s)                      SequenceModel.py:19-24
//   DP0  pre1p_s = h_{s+1} W_p0^T + b  and (s + 1 < H) hA_{s+1}     prior logit_net.0, actor h-columns
//   DP1  pre2p_s = SiLU(LN(pre1p_s)) W_p3^T + b                     prior logit_net.1-3
//   DSM  z_{s+1} = sample(SiLU(LN(pre2p_s)) W_p6^T + b)              prior logit_net.4-6 + Categorical
//
// hA_0 is a prologue stage.  The launch writes the outputs and the tape in the
// layouts dr_imagine_bwd reads (engine.hip tape_carve); the reward / continue
// heads run once over all B (H + 1) states after it, as in the launch form.
//
// Each workgroup (one per CU) owns a fixed tile of every stage: DG = MR rows x
// 10 hidden units (W_hh fragments in registers, the tile's 30 columns of W_ih^T
// in LDS, as scan.hip's GRU stage), the others 16 rows x 16 columns (weights
// from L2, loaded with the stage's inputs), the sampler 16 rows x one 32-class
// group.  Hand-offs: write-through (sc1) stores, a counter per 16-row block and
// stage, sc1 loads; z travels as tagged 8-byte granules (persist.h).  Every
// hand-off buffer is a distinct per-step region (the tape, hiddens, latents),
// so no slot is ever overwritten while a reader may still need it.
#include "common.h"
#include "dream.h"
#include "persist.h"
#include "ops.h"

#include <string.h>
#include <algorithm>

namespace {
constexpr int HD = 600, KSH = 19, MW = 200, KSE = 7, NR = 32, NCL = 32, LAT = NR * NCL;
constexpr int UPT = 10, NUS = HD / UPT, NC = (MW + 15) / 16, NC0 = 2 * NC, WLD = 3 * UPT;
constexpr int NTH = 256;
constexpr int KSW = 5;   // 32-k steps per wave over K = HD
constexpr int KSW3 = 2;  // 32-k steps per wave over K = MW
constexpr int KP3 = 232;
constexpr int SCR_F = 8192;
constexpr int SHW = 4352;  // scr offset of the actor heads' weights [2 A][MW] (DG tiles; other stages use < 3712)
constexpr int SLN4 = SHW + 16 * MW;  // base_net.4's gamma, beta [2][MW], then the heads' biases [16]
constexpr int CNT_LD = 32;
// counters per 16-row block: [stage][block]
enum { C_A = 0, C_B = 1, C_G = 2, C_P0 = 3, C_P1 = 4, C_PRE = 5, C_STATUS = 6 };  // exit ticket: block 1 of C_STATUS
constexpr int CNT_BLOCKS = 16;  // B <= 256
}  // namespace

struct alignas(16) PDreamArgs {
  int B, H, A, det;
  const float* wt;  // W_ih^T [LAT + A][3 HD]
  const float* b_ih;
  const float* b_hh;
  const float* whh;  // [3 HD][HD]
  const float *wp0, *bp0, *pn1g, *pn1b, *wp3, *bp3, *pn4g, *pn4b, *wp6, *bp6;  // prior
  const float *wa0, *ba0;  // actor base_net.0 [MW][HD + LAT] (h-columns first)
  const float* wazt;       // its z-columns transposed [LAT][MW]
  const float *an1g, *an1b, *wa3, *ba3, *an4g, *an4b;  // actor base_net.1/.3/.4
  const float *wmu, *bmu, *wls, *bls;                  // heads [A][MW], [A]
  const int* idx0;         // z_0: [B][NR] class per group, then [B][NR] straight-through values
  dr_noise noise;          // actor rsample
  dr_noise nq;             // categorical draws
  float unimix;
  int spin_limit;
  float *latents, *hiddens, *actions, *mus, *sigmas;  // [B][H+1][LAT], [B][H+1][HD], [B][H][A]
  float *eps, *ls_raw;                                 // [H][B][A], [B][H][A]
  float *pre1a, *x1a, *pre2a, *x2a;                    // [B][H][MW]
  float *tr, *tu, *tn, *tghn;                          // [H][B][HD]
  float *pre1p, *pre2p, *soft;                         // [H][B][MW], [H][B][MW], [H][B][LAT]
  float* hA;                                           // [H][B][MW]
  unsigned long long* zg;                              // [H + 1][B][NR]
  unsigned* cnt;
  long long* ts;  // DR_PDREAM_TS builds: [16 steps][6 stages][8 marks][grid] wall-clock stamps
  PsPoison pz;    // outputs NaN-filled on a timeout (persist.h ps_exit)
};
#ifdef DR_PDREAM_TS
#define PD_TS(st, mk) \
  do { \
    if (threadIdx.x == 0 && s < 16) g.ts[((s * 6 + (st)) * 8 + (mk)) * gridDim.x + blockIdx.x] = (long long)wall_clock64(); \
  } while (0)
#else
#define PD_TS(st, mk) do {} while (0)
#endif

// the weight fragments of one 16-column tile over K (W [N][K] rows n0..; the
// wave's K-slice of KS 32-k steps): issued before the stage's poll
template <int NT, int KS>
__device__ __forceinline__ void pd_wfrag(PsFrag<NT> (&wf)[KS], const float* W, unsigned ldw, int n0, int N, int K,
                                         int wave, int r, int q) {
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 32 * (KS * wave + s) + 8 * q, n = n0 + r;
    const bool ok = k < K && n < N;
    wf[s] = ps_frag<NT>(W, ps_opaque(ok ? (unsigned)n * ldw + (unsigned)k : 0u), ok);
  }
}

// one 16-row x 16-column tile of Y = X W^T over K (X rows from an sc1 buffer,
// row stride ldx floats; wf from pd_wfrag): the wave's K-slice, to be reduced
// across the 4 waves by the caller.  NT terms (split3 or bf16).
template <int NT, int KS>
__device__ __forceinline__ f32x4 pd_tile_global(const PsFrag<NT> (&wf)[KS], __amdgpu_buffer_rsrc_t rx, unsigned xrow0,
                                                unsigned ldx, int K, int wave, int r, int q) {
  f32x4 xa[KS][2];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 32 * (KS * wave + s) + 8 * q;
    const bool ok = k < K;
    const unsigned o = 4u * (xrow0 + (unsigned)r * ldx + (ok ? (unsigned)k : 0u));
    xa[s][0] = ps_ld4(rx, o);
    xa[s][1] = ps_ld4(rx, o + 16u);
    if (!ok) xa[s][0] = xa[s][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    ps_pin(xa[s][0]);
    ps_pin(xa[s][1]);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (32 * (KS * wave + s) < K) {
      ps_u32x4 a[NT], w[NT];
      ps_split<NT>(xa[s][0], xa[s][1], a);
      ps_wsplit<NT>(wf[s], w);
      acc = ps_prod<NT>(w, a, acc);
    }
  }
  return acc;
}

// LN-SiLU (eps 1e-5, hardware exp2 SiLU: k_ln_gemm_sample's arithmetic) of 16
// rows of MW floats from an sc1 buffer into LDS rows of stride KP3 (zero to
// 224); optionally also the normalised rows to `out` (plain stores, stride
// ldo).  Wave w takes rows 4 w .. 4 w + 3, 16 lanes per row (DPP-only sums).
struct PdLn {
  float4 g[4], b[4];
};
// the LN's gamma / beta chunks of this lane (issued before the stage's poll)
__device__ __forceinline__ PdLn pd_lnparams(const float* lng, const float* lnb, int lane) {
  PdLn p;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = (lane & 15) + 16 * j;
    p.g[j] = dr_ld4(lng, ps_opaque(c < MW / 4 ? 4u * c : 0u));
    p.b[j] = dr_ld4(lnb, ps_opaque(c < MW / 4 ? 4u * c : 0u));
  }
  return p;
}
__device__ __forceinline__ void pd_ln16(__amdgpu_buffer_rsrc_t rx, unsigned xrow0, unsigned ldx, const PdLn& ln,
                                        float* sA, float* out, unsigned ldo, int wave, int lane) {
  const int ml = wave * 4 + (lane >> 4), sub = lane & 15;
  f32x4 x[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = sub + 16 * j;
    x[j] = ps_ld4(rx, 4u * (xrow0 + (unsigned)ml * ldx + ps_opaque(c < MW / 4 ? 4u * c : 0u)));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) ps_pin(x[j]);
  float sm = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (sub + 16 * j < MW / 4) sm += (x[j][0] + x[j][1]) + (x[j][2] + x[j][3]);
  const float mean = row16_sum(sm) / (float)MW;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (sub + 16 * j < MW / 4) {
      const float dx = x[j][0] - mean, dy = x[j][1] - mean, dz = x[j][2] - mean, dw = x[j][3] - mean;
      sq += (dx * dx + dy * dy) + (dz * dz + dw * dw);
    }
  const float rstd = 1.0f / sqrtf(row16_sum(sq) / (float)MW + 1e-5f);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = sub + 16 * j;
    float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < MW / 4) {
      y.x = dr_silu_fast((x[j][0] - mean) * rstd * ln.g[j].x + ln.b[j].x);
      y.y = dr_silu_fast((x[j][1] - mean) * rstd * ln.g[j].y + ln.b[j].y);
      y.z = dr_silu_fast((x[j][2] - mean) * rstd * ln.g[j].z + ln.b[j].z);
      y.w = dr_silu_fast((x[j][3] - mean) * rstd * ln.g[j].w + ln.b[j].w);
      if (out) dr_st4(out, (unsigned)ml * ldo + 4u * c, y);
    }
    if (c < KSE * 8) *reinterpret_cast<float4*>(&sA[ml * KP3 + 4 * c]) = y;
  }
}

// the K = MW product of the 16 LN-SiLU rows in LDS with 16 x CT columns of W
// (rows n0..; fragments from pd_wfrag3, split3): acc[ct] per wave (K split
// over the waves)
template <int CT>
__device__ __forceinline__ void pd_wfrag3(PsFrag<3> (&wf)[KSW3][CT], const float* W, int n0, int N, int wave, int r,
                                          int q) {
#pragma unroll
  for (int s = 0; s < KSW3; ++s) {
    const int ks = KSW3 * wave + s, k = 32 * ks + 8 * q;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int n = n0 + 16 * ct + r;
      const bool ok = ks < KSE && k < MW && n < N;
      wf[s][ct] = ps_frag<3>(W, ps_opaque(ok ? (unsigned)(n * MW + k) : 0u), ok);
    }
  }
}
template <int CT>
__device__ __forceinline__ void pd_lds_mfma(const float* sA, const PsFrag<3> (&wf)[KSW3][CT], f32x4 (&acc)[CT],
                                            int wave, int r, int q) {
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) acc[ct] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KSW3; ++s) {
    const int ks = KSW3 * wave + s;
    if (ks < KSE) {
      const float* pa = sA + r * KP3 + 32 * ks + 8 * q;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(pa), x1 = *reinterpret_cast<const f32x4*>(pa + 4);
      ps_u32x4 a[3];
      ps_split<3>(x0, x1, a);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        ps_u32x4 w[3];
        ps_wsplit<3>(wf[s][ct], w);
        acc[ct] = ps_prod<3>(w, a, acc[ct]);
      }
    }
  }
}

// lane 0 polls counters c[0 .. n) >= target, then the workgroup barrier
__device__ __forceinline__ bool pd_wait(int* s_ok, const unsigned* c0, int n, unsigned target, int lim,
                                        unsigned* status) {
  if (threadIdx.x == 0) {
    bool ok = true;
    for (int i = 0; i < n && ok; ++i) ok = ps_poll(c0 + CNT_LD * i, target, lim, status);
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}
// every storing wave drained; one lane adds 1 to counters c[0 .. n)
__device__ __forceinline__ void pd_signal(unsigned* c0, int n) {
  ps_drain();
  __syncthreads();
  if (threadIdx.x < n) __hip_atomic_fetch_add(c0 + CNT_LD * threadIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NT, int MR>
__device__ __forceinline__ void pdream_body(const PDreamArgs& g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int s_ok;
  const int B = g.B, H = g.H, A = g.A;
  const int b = blockIdx.x, tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
  const int RB = B / 16;
  const int nG = (B / MR) * NUS, nA = RB * NC, nP0 = RB * NC0, nS = RB * NR;
  const bool doG = b < nG, doA = b < nA, doP0 = b < nP0, doS = b < nS;
  float* wih = smem;                                 // [LAT + A][WLD]
  float* scr = smem + (((LAT + A) * WLD + 3) & ~3);  // [SCR_F]
  float* sbias = scr + SCR_F;                        // [64]
  unsigned* cnt = g.cnt;
  unsigned* status = cnt + CNT_LD * CNT_BLOCKS * C_STATUS;
  auto ctr = [&](int st, int blk) { return cnt + CNT_LD * (CNT_BLOCKS * st + blk); };
  const int lim = g.spin_limit;
  const unsigned ldH = (unsigned)((H + 1) * HD), ldL = (unsigned)((H + 1) * LAT), ldM = (unsigned)(H * MW);
  const __amdgpu_buffer_rsrc_t rhid = ps_rsrc(g.hiddens, 4u * B * ldH);
  const __amdgpu_buffer_rsrc_t rp1a = ps_rsrc(g.pre1a, 4u * B * ldM);
  const __amdgpu_buffer_rsrc_t rp2a = ps_rsrc(g.pre2a, 4u * B * ldM);
  const __amdgpu_buffer_rsrc_t rp1p = ps_rsrc(g.pre1p, 4u * H * B * MW);
  const __amdgpu_buffer_rsrc_t rp2p = ps_rsrc(g.pre2p, 4u * H * B * MW);
  const __amdgpu_buffer_rsrc_t rhA = ps_rsrc(g.hA, 4u * H * B * MW);

  // ---- tiles --------------------------------------------------------------
  const int rg = b / NUS, us = b - rg * NUS, r0 = rg * MR, u0 = us * UPT;  // DG
  const int rbA = b / NC, ctA = b - rbA * NC;                              // DA, DB, DP1
  const int rb0 = b / NC0, ct0 = b - rb0 * NC0;                            // DP0 (400 columns)
  const int rbS = b / NR, gq = b - rbS * NR;                               // DSM
  PsFrag<NT> w1[KSW][2];  // DG's W_hh fragments stay in registers for the unroll
#pragma unroll
  for (int s = 0; s < KSW; ++s) {
    const int ks = KSW * wave + s, k = 32 * ks + 8 * q;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const int c = ct * 16 + r;
      const bool ok = doG && ks < KSH && k < HD && c < WLD;
      const int n = ok ? (c / UPT) * HD + u0 + (c % UPT) : 0;
      w1[s][ct] = ps_frag<NT>(g.whh, (unsigned)(n * HD + k), ok);
    }
  }
  float* shw = scr + SHW;
  float* sln4 = scr + SLN4;
  static_assert(SLN4 + 2 * MW + 16 <= SCR_F, "heads' parameters in the scratch");
  if (doG) {
    for (int x = tid; x < 2 * A * MW; x += NTH) {
      const int i = x / MW, k = x - i * MW;
      shw[x] = i < A ? dr_ld1(g.wmu, (unsigned)(i * MW + k)) : dr_ld1(g.wls, (unsigned)((i - A) * MW + k));
    }
    for (int x = tid; x < 2 * MW + 16; x += NTH)
      sln4[x] = x < MW ? dr_ld1(g.an4g, (unsigned)x)
              : x < 2 * MW ? dr_ld1(g.an4b, (unsigned)(x - MW))
              : (x - 2 * MW < A ? dr_ld1(g.bmu, (unsigned)(x - 2 * MW))
                 : x - 2 * MW < 2 * A ? dr_ld1(g.bls, (unsigned)(x - 2 * MW - A)) : 0.f);
    const int nrow = LAT + A;
    for (int x = tid; x < nrow * WLD; x += NTH) {
      const int k = x / WLD, c = x - k * WLD;
      wih[x] = dr_ld1(g.wt, (unsigned)(k * 3 * HD + (c / UPT) * HD + u0 + (c % UPT)));
    }
    if (tid < 64) {
      const int c = tid & 31;
      const unsigned col = (unsigned)((c / UPT) * HD + u0 + (c % UPT));
      sbias[tid] = c < WLD ? dr_ld1(tid < 32 ? g.b_ih : g.b_hh, col) : 0.f;
    }
  }
  const unsigned long long* rng = g.noise.rng;
  const unsigned long long a_seed = rng ? rng[0] : 0ull, a_off = rng ? rng[1] : 0ull;
  const unsigned long long* rngq = g.nq.rng;
  const unsigned long long q_seed = rngq ? rngq[0] : 0ull, q_off = rngq ? rngq[1] : 0ull;
  __syncthreads();

  // ---- prologue: hA_0 = h_0 W_a0h^T + b (actor columns of DP0's layout) ----
  if (b < RB * NC) {
    const int m0 = rbA * 16, n0 = ctA * 16;
    PsFrag<NT> wf[KSW];
    pd_wfrag<NT, KSW>(wf, g.wa0, HD + LAT, n0, MW, HD, wave, r, q);
    const f32x4 acc = pd_tile_global<NT, KSW>(wf, rhid, (unsigned)m0 * ldH, ldH, HD, wave, r, q);
#pragma unroll
    for (int e = 0; e < 4; ++e) scr[(wave * 4 + e) * 64 + lane] = acc[e];
    __syncthreads();
    const int e2 = tid >> 6, l2 = tid & 63, row2 = l2 & 15, col2 = 4 * (l2 >> 4) + e2, n = n0 + col2;
    if (n < MW) {
      const float v = ((scr[e2 * 64 + l2] + scr[(4 + e2) * 64 + l2]) + scr[(8 + e2) * 64 + l2]) + scr[(12 + e2) * 64 + l2];
      ps_st1(rhA, 4u * (unsigned)((m0 + row2) * MW + n), v + dr_ld1(g.ba0, (unsigned)n));
    }
    pd_signal(ctr(C_PRE, rbA), 1);
  }

  constexpr int NP1 = (MR * UPT + NTH - 1) / NTH;
  for (int s = 0; s < H; ++s) {
    // ===================== DA: actor base_net.0 = hA + z-gather ============
    if (doA) {
      const int m0 = rbA * 16, n0 = ctA * 16;
      PD_TS(0, 0);
      // thread = (row tid >> 4, column n0 + (tid & 15)); it fetches 2 of the
      // row's 32 (class, value) pairs of z_s into LDS
      const int row = tid >> 4, cc = tid & 15, n = n0 + cc, m = m0 + row;
      int2* sz = reinterpret_cast<int2*>(scr);  // [16][NR]
      bool okz = true;
      if (s == 0) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int u = 2 * cc + j;
          sz[row * NR + u] =
              make_int2(g.idx0[m * NR + u], __float_as_int(reinterpret_cast<const float*>(g.idx0 + B * NR)[m * NR + u]));
        }
      } else {
        const ps_u64* src = g.zg + ((size_t)s * B + m) * NR + 2 * cc;
        ps_u64 v0 = ps_gld(src), v1 = ps_gld(src + 1);
        int spins = 0;
        while (((unsigned)((v0 >> 16) & 0xFFFFu) != (unsigned)s || (unsigned)((v1 >> 16) & 0xFFFFu) != (unsigned)s) &&
               ++spins <= lim) {
          __builtin_amdgcn_s_sleep(1);
          v0 = ps_gld(src);
          v1 = ps_gld(src + 1);
        }
        okz = spins <= lim;
        if (!okz) __hip_atomic_store(status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sz[row * NR + 2 * cc] = make_int2((int)(v0 & 0xFFFFu), (int)(v0 >> 32));
        sz[row * NR + 2 * cc + 1] = make_int2((int)(v1 & 0xFFFFu), (int)(v1 >> 32));
      }
      if (!(s == 0 ? pd_wait(&s_ok, ctr(C_PRE, rbA), 1, (unsigned)NC, lim, status)
                   : pd_wait(&s_ok, ctr(C_P0, rbA), 1, (unsigned)(NC0 * s), lim, status)))
        return;
      if (!__syncthreads_and(okz)) return;
      PD_TS(0, 1);
      if (n < MW) {
        const int2* iz = sz + row * NR;
        // all 32 gathered weights in flight at once, then the sum in group order
        float wv[NR];
#pragma unroll
        for (int u = 0; u < NR; ++u) wv[u] = dr_ld1(g.wazt, (unsigned)((u * NCL + max(iz[u].x, 0)) * MW + n));
        const float base = ps_ld1(rhA, 4u * (unsigned)(((size_t)s * B + m) * MW + n));
        float v = 0.f;
#pragma unroll
        for (int u = 0; u < NR; ++u) v = fmaf(wv[u], __int_as_float(iz[u].y), v);
        if (s == 0) {
          // dense groups of a given z_0 (k_onehot_index marks them idx -1, value 0)
          for (int u = 0; u < NR; ++u)
            if (iz[u].x < 0)
              for (int c = 0; c < NCL; ++c)
                v = fmaf(dr_ld1(g.wazt, (unsigned)((u * NCL + c) * MW + n)), g.latents[(size_t)m * ldL + u * NCL + c], v);
        }
        ps_st1(rp1a, 4u * (unsigned)(m * ldM + s * MW + n), base + v);
      }
      PD_TS(0, 6);
      pd_signal(ctr(C_A, rbA), 1);
      PD_TS(0, 7);
    }
    // ===================== DB: actor base_net.1-3 ===========================
    if (doA) {
      const int m0 = rbA * 16, n0 = ctA * 16;
      PD_TS(1, 0);
      PsFrag<3> wf[KSW3][1];
      pd_wfrag3<1>(wf, g.wa3, n0, MW, wave, r, q);
      const PdLn ln = pd_lnparams(g.an1g, g.an1b, lane);
      const float bias = dr_ld1(g.ba3, ps_opaque((unsigned)min(n0 + 4 * ((tid & 63) >> 4) + (tid >> 6), MW - 1)));
      if (!pd_wait(&s_ok, ctr(C_A, rbA), 1, (unsigned)(NC * (s + 1)), lim, status)) return;
      PD_TS(1, 1);
      pd_ln16(rp1a, (unsigned)(m0 * ldM + s * MW), ldM, ln, scr, ctA == 0 ? g.x1a + (size_t)m0 * ldM + s * MW : nullptr,
              ldM, wave, lane);
      __syncthreads();
      f32x4 acc[1];
      pd_lds_mfma<1>(scr, wf, acc, wave, r, q);
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 4; ++e) scr[(wave * 4 + e) * 64 + lane] = acc[0][e];
      __syncthreads();
      const int e2 = tid >> 6, l2 = tid & 63, row2 = l2 & 15, col2 = 4 * (l2 >> 4) + e2, n = n0 + col2;
      if (n < MW) {
        const float v = ((scr[e2 * 64 + l2] + scr[(4 + e2) * 64 + l2]) + scr[(8 + e2) * 64 + l2]) + scr[(12 + e2) * 64 + l2];
        ps_st1(rp2a, 4u * (unsigned)((m0 + row2) * ldM + s * MW + n), v + bias);
      }
      PD_TS(1, 6);
      pd_signal(ctr(C_B, rbA), 1);
      PD_TS(1, 7);
    }
    // ===================== DG: actor heads + GRU ============================
    if (doG) {
      // z_s (granules / the given z_0), pre2a_s of the MR rows, h_s
      int2* siz = reinterpret_cast<int2*>(scr);  // [MR][NR]
      float* red = scr;                          // [2][PF]: K-split partials (siz consumed by then)
      float* sact = scr + 2048;                  // [MR][8]: a_s
      float* sgi = scr + 2304;                   // [MR][32]
      float* sgh = scr + 3328;                   // [MR][32]
      constexpr int PF = (MR / 16) * 2 * 256;
      static_assert(2 * MR * NR <= 2048 && 2 * PF <= 2048 && 3328 + 32 * MR <= SHW, "DG LDS layout");
      constexpr int NZ = MR * NR / NTH;
      PD_TS(2, 0);
      unsigned zpend = 0;
      if (s == 0) {
#pragma unroll
        for (int i = 0; i < NZ; ++i) {
          const int x = tid + NTH * i;
          siz[x] = make_int2(g.idx0[r0 * NR + x], __float_as_int(reinterpret_cast<const float*>(g.idx0 + B * NR)[r0 * NR + x]));
        }
      } else {
        const ps_u64* zsrc = g.zg + ((size_t)s * B + r0) * NR;
#pragma unroll
        for (int i = 0; i < NZ; ++i) {
          const ps_u64 v = ps_gld(zsrc + tid + NTH * i);
          siz[tid + NTH * i] = make_int2((int)(v & 0xFFFFu), (int)(v >> 32));
          if ((unsigned)((v >> 16) & 0xFFFFu) != (unsigned)s) zpend |= 1u << i;
        }
      }
      // h_s for the gate pairs and the product (h_0 is the given start state),
      // loaded while the actor stages run; then the heads' inputs
      if (s >= 1 && !pd_wait(&s_ok, ctr(C_G, r0 / 16), MR / 16, (unsigned)(NUS * s), lim, status)) return;
      const unsigned hs = (unsigned)(s * HD);
      float hv[NP1];
#pragma unroll
      for (int i = 0; i < NP1; ++i) {
        const int p = tid + NTH * i;
        const int row = p / UPT, j = p - row * UPT;
        const bool ok = p < MR * UPT;
        hv[i] = ps_ld1(rhid, ok ? 4u * ((unsigned)(r0 + row) * ldH + hs + (unsigned)(u0 + j)) : 0u);
      }
      f32x4 ha[KSW][MR / 16][2];
#pragma unroll
      for (int sk = 0; sk < KSW; ++sk) {
        const int ks = KSW * wave + sk, k = 32 * ks + 8 * q;
        const bool ok = ks < KSH && k < HD;
#pragma unroll
        for (int rt = 0; rt < MR / 16; ++rt) {
          const unsigned o = 4u * ((unsigned)(r0 + rt * 16 + r) * ldH + hs + (ok ? (unsigned)k : 0u));
          ha[sk][rt][0] = ps_ld4(rhid, o);
          ha[sk][rt][1] = ps_ld4(rhid, o + 16u);
          if (!ok) ha[sk][rt][0] = ha[sk][rt][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int sk = 0; sk < KSW; ++sk)
#pragma unroll
        for (int rt = 0; rt < MR / 16; ++rt) {
          ps_pin(ha[sk][rt][0]);
          ps_pin(ha[sk][rt][1]);
        }
#pragma unroll
      for (int i = 0; i < NP1; ++i) ps_pin(hv[i]);
      float epv[MR / 16];
#pragma unroll
      for (int pass = 0; pass < MR / 16; ++pass) {
        const int m = r0 + pass * 16 + wave * 4 + (lane >> 4), sub = lane & 15;
        epv[pass] = 0.f;
        if (!g.det && sub < A) {
          if (g.noise.eps) epv[pass] = g.noise.eps[((size_t)s * B + m) * A + sub];
          else epv[pass] = dr_normal_k(a_seed, a_off, (uint32_t)(g.noise.stream + s), (uint32_t)(g.noise.row0 + m),
                                       (uint32_t)sub);
        }
      }
      if (!pd_wait(&s_ok, ctr(C_B, r0 / 16), MR / 16, (unsigned)(NC * (s + 1)), lim, status)) return;
      PD_TS(2, 1);
      f32x4 xr[MR / 4];
#pragma unroll
      for (int pass = 0; pass < MR / 16; ++pass)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = (lane & 15) + 16 * j;
          const unsigned row = (unsigned)(r0 + pass * 16 + wave * 4 + (lane >> 4));
          xr[pass * 4 + j] = ps_ld4(rp2a, 4u * (row * ldM + (unsigned)(s * MW) + ps_opaque(c < MW / 4 ? 4u * c : 0u)));
        }
#pragma unroll
      for (int i = 0; i < MR / 4; ++i) ps_pin(xr[i]);
      // the heads, 4 rows per wave at a time (16 lanes per row, DPP-only row
      // sums): x2a = SiLU(LN(pre2a)), [mu | log_sig] = x2a W^T + b,
      // a = tanh(mu + eps sigma); the unit slice 0 tile writes the outputs and the tape
#pragma unroll
      for (int pass = 0; pass < MR / 16; ++pass) {
        const int ml = pass * 16 + wave * 4 + (lane >> 4), m = r0 + ml, sub = lane & 15;
        f32x4 x[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = xr[pass * 4 + j];
        float sm = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (sub + 16 * j < MW / 4) sm += (x[j][0] + x[j][1]) + (x[j][2] + x[j][3]);
        const float mean = row16_sum(sm) / (float)MW;
        float sq = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (sub + 16 * j < MW / 4) {
            const float dx = x[j][0] - mean, dy = x[j][1] - mean, dz = x[j][2] - mean, dw = x[j][3] - mean;
            sq += (dx * dx + dy * dy) + (dz * dz + dw * dw);
          }
        const float rstd = 1.0f / sqrtf(row16_sum(sq) / (float)MW + 1e-5f);
        f32x4 y[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = sub + 16 * j;
          y[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
          if (c < MW / 4) {
            const float4 gv = *reinterpret_cast<const float4*>(sln4 + 4 * c),
                         bv = *reinterpret_cast<const float4*>(sln4 + MW + 4 * c);
            y[j][0] = dr_silu_fast((x[j][0] - mean) * rstd * gv.x + bv.x);
            y[j][1] = dr_silu_fast((x[j][1] - mean) * rstd * gv.y + bv.y);
            y[j][2] = dr_silu_fast((x[j][2] - mean) * rstd * gv.z + bv.z);
            y[j][3] = dr_silu_fast((x[j][3] - mean) * rstd * gv.w + bv.w);
            if (us == 0)
              dr_st4(g.x2a, (unsigned)m * ldM + (unsigned)(s * MW + 4 * c), make_float4(y[j][0], y[j][1], y[j][2], y[j][3]));
          }
        }
        float muv = 0.f, lr = 0.f;
#pragma unroll
        for (int i2 = 0; i2 < 16; ++i2) {
          if (i2 < 2 * A) {
            float v = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int c = sub + 16 * j;
              if (c < MW / 4) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(shw + i2 * MW + 4 * c);
                v += (y[j][0] * w[0] + y[j][1] * w[1]) + (y[j][2] * w[2] + y[j][3] * w[3]);
              }
            }
            v = row16_sum(v);
            if (i2 == sub) muv = v;
            if (i2 == sub + A) lr = v;
          }
        }
        if (sub < A) {
          muv += sln4[2 * MW + sub];
          lr += sln4[2 * MW + A + sub];
          const float ls = fminf(fmaxf(lr, -5.0f), 2.0f);
          const float sg = dr_softplus(ls) + 1e-3f;
          float av;
          if (g.det) {
            av = tanhf(muv);
          } else {
            const float e = epv[pass];
            if (us == 0) g.eps[((size_t)s * B + m) * A + sub] = e;
            av = tanhf(muv + e * sg);
          }
          sact[ml * 8 + sub] = av;
          if (us == 0) {
            const size_t o = (size_t)m * H * A + (size_t)s * A + sub;
            g.actions[o] = av;
            g.mus[o] = muv;
            g.sigmas[o] = sg;
            g.ls_raw[o] = lr;
          }
        }
      }
      PD_TS(2, 2);
      // the rest of z_s
      {
        int spins = 0;
        const ps_u64* zsrc = g.zg + ((size_t)s * B + r0) * NR;
        while (zpend && ++spins <= lim) {
          __builtin_amdgcn_s_sleep(1);
#pragma unroll
          for (int i = 0; i < NZ; ++i)
            if (zpend & (1u << i)) {
              const ps_u64 v = ps_gld(zsrc + tid + NTH * i);
              siz[tid + NTH * i] = make_int2((int)(v & 0xFFFFu), (int)(v >> 32));
              if ((unsigned)((v >> 16) & 0xFFFFu) == (unsigned)s) zpend &= ~(1u << i);
            }
        }
        if (zpend) __hip_atomic_store(status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!__syncthreads_and(zpend == 0)) return;
      }
      PD_TS(2, 3);
      // gi by gather from the LDS slice (scan.hip's order: groups, actions, + b_ih);
      // thread = (row, column pair)
      for (int p = tid; p < MR * 16; p += NTH) {
        const int row = p >> 4, c0 = 2 * (p & 15);
        if (c0 < WLD) {
          float v0 = 0.f, v1 = 0.f;
          const int2* iz = siz + row * NR;
#pragma unroll 8
          for (int u = 0; u < NR; ++u) {
            const int2 pz = iz[u];
            const float zv = __int_as_float(pz.y);
            const float2 w = *reinterpret_cast<const float2*>(wih + (u * NCL + max(pz.x, 0)) * WLD + c0);
            v0 = fmaf(w.x, zv, v0);
            v1 = fmaf(w.y, zv, v1);
          }
          if (s == 0) {
            // dense groups of a given z_0 (idx -1, value 0 above)
            const float* zr = g.latents + (size_t)(r0 + row) * ldL;
            for (int u = 0; u < NR; ++u)
              if (iz[u].x < 0)
                for (int c = 0; c < NCL; ++c) {
                  const float zc = zr[u * NCL + c];
                  const float2 w = *reinterpret_cast<const float2*>(wih + (u * NCL + c) * WLD + c0);
                  v0 = fmaf(w.x, zc, v0);
                  v1 = fmaf(w.y, zc, v1);
                }
          }
          for (int ia = 0; ia < A; ++ia) {
            const float av = sact[row * 8 + ia];
            const float2 w = *reinterpret_cast<const float2*>(wih + (LAT + ia) * WLD + c0);
            v0 = fmaf(w.x, av, v0);
            v1 = fmaf(w.y, av, v1);
          }
          sgi[row * 32 + c0] = v0 + sbias[c0];
          sgi[row * 32 + c0 + 1] = v1 + sbias[c0 + 1];
        }
      }
      // gh = h_s W_hh^T over this wave's k-steps
      f32x4 acc[MR / 16][2];
#pragma unroll
      for (int rt = 0; rt < MR / 16; ++rt) acc[rt][0] = acc[rt][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sk = 0; sk < KSW; ++sk) {
        if (KSW * wave + sk < KSH) {
          ps_u32x4 w[2][NT];
          ps_wsplit<NT>(w1[sk][0], w[0]);
          ps_wsplit<NT>(w1[sk][1], w[1]);
#pragma unroll
          for (int rt = 0; rt < MR / 16; ++rt) {
            ps_u32x4 a[NT];
            ps_split<NT>(ha[sk][rt][0], ha[sk][rt][1], a);
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) acc[rt][ct] = ps_prod<NT>(w[ct], a, acc[rt][ct]);
          }
        }
      }
      PD_TS(2, 5);
      // K-split partials in two rounds, (w0 + w2) + (w1 + w3)
      __syncthreads();
      if (wave >= 2) {
#pragma unroll
        for (int rt = 0; rt < MR / 16; ++rt)
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int e = 0; e < 4; ++e) red[(wave - 2) * PF + ((rt * 2 + ct) * 4 + e) * 64 + lane] = acc[rt][ct][e];
      }
      __syncthreads();
      if (wave < 2) {
#pragma unroll
        for (int rt = 0; rt < MR / 16; ++rt)
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[rt][ct][e] += red[wave * PF + ((rt * 2 + ct) * 4 + e) * 64 + lane];
      }
      __syncthreads();
      if (wave == 1) {
#pragma unroll
        for (int rt = 0; rt < MR / 16; ++rt)
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int e = 0; e < 4; ++e) red[((rt * 2 + ct) * 4 + e) * 64 + lane] = acc[rt][ct][e];
      }
      __syncthreads();
      if (wave == 0) {
#pragma unroll
        for (int rt = 0; rt < MR / 16; ++rt)
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int c = ct * 16 + 4 * q + e;
              const float v = acc[rt][ct][e] + red[((rt * 2 + ct) * 4 + e) * 64 + lane];
              if (c < WLD) sgh[(rt * 16 + r) * 32 + c] = v + sbias[32 + c];
            }
      }
      __syncthreads();
      // gates (torch gru_cell op order); the tape saves r, u, n, gh_n
#pragma unroll
      for (int i = 0; i < NP1; ++i) {
        const int p = tid + NTH * i;
        if (p < MR * UPT) {
          const int row = p / UPT, j = p - row * UPT, m = r0 + row;
          const float* gh = sgh + row * 32 + j;
          const float* gi = sgi + row * 32 + j;
          const float rr = 1.0f / (1.0f + expf(-(gh[0] + gi[0])));
          const float uu = 1.0f / (1.0f + expf(-(gh[UPT] + gi[UPT])));
          const float nn = tanhf(gi[2 * UPT] + gh[2 * UPT] * rr);
          const float ho = (hv[i] - nn) * uu + nn;
          ps_st1(rhid, 4u * ((unsigned)m * ldH + (unsigned)((s + 1) * HD + u0 + j)), ho);
          const size_t o = ((size_t)s * B + m) * HD + u0 + j;
          g.tr[o] = rr;
          g.tu[o] = uu;
          g.tn[o] = nn;
          g.tghn[o] = gh[2 * UPT];
        }
      }
      PD_TS(2, 6);
      pd_signal(ctr(C_G, r0 / 16), MR / 16);
      PD_TS(2, 7);
    }
    // ===================== DP0: prior logit_net.0 | actor h-columns ==========
    if (doP0) {
      // tiles ct0 < NC: the prior's columns; NC .. 2 NC - 1: the next step's actor h-columns
      const int m0 = rb0 * 16;
      const bool prior = ct0 < NC, live = prior || s + 1 < H;
      PD_TS(3, 0);
      const float* W = prior ? g.wp0 : g.wa0;
      const unsigned ldw = prior ? (unsigned)HD : (unsigned)(HD + LAT);
      const int nb = 16 * (prior ? ct0 : ct0 - NC);
      PsFrag<NT> wf[KSW];
      pd_wfrag<NT, KSW>(wf, W, ldw, nb, live ? MW : 0, HD, wave, r, q);
      const float bias = dr_ld1(prior ? g.bp0 : g.ba0,
                                ps_opaque((unsigned)min(nb + 4 * ((tid & 63) >> 4) + (tid >> 6), MW - 1)));
      if (!pd_wait(&s_ok, ctr(C_G, rb0), 1, (unsigned)(NUS * (s + 1)), lim, status)) return;
      PD_TS(3, 1);
      if (live) {
        const f32x4 acc = pd_tile_global<NT, KSW>(wf, rhid, (unsigned)m0 * ldH + (unsigned)((s + 1) * HD), ldH, HD, wave, r, q);
#pragma unroll
        for (int e = 0; e < 4; ++e) scr[(wave * 4 + e) * 64 + lane] = acc[e];
        __syncthreads();
        const int e2 = tid >> 6, l2 = tid & 63, row2 = l2 & 15, col2 = 4 * (l2 >> 4) + e2, n = nb + col2;
        if (n < MW) {
          const float v =
              ((scr[e2 * 64 + l2] + scr[(4 + e2) * 64 + l2]) + scr[(8 + e2) * 64 + l2]) + scr[(12 + e2) * 64 + l2];
          if (prior)
            ps_st1(rp1p, 4u * (unsigned)(((size_t)s * B + m0 + row2) * MW + n), v + bias);
          else
            ps_st1(rhA, 4u * (unsigned)(((size_t)(s + 1) * B + m0 + row2) * MW + n), v + bias);
        }
      }
      PD_TS(3, 6);
      pd_signal(ctr(C_P0, rb0), 1);
      PD_TS(3, 7);
    }
    // ===================== DP1: prior logit_net.1-3 ==========================
    if (doA) {
      const int m0 = rbA * 16, n0 = ctA * 16;
      PD_TS(4, 0);
      PsFrag<3> wf[KSW3][1];
      pd_wfrag3<1>(wf, g.wp3, n0, MW, wave, r, q);
      const PdLn ln = pd_lnparams(g.pn1g, g.pn1b, lane);
      const float bias = dr_ld1(g.bp3, ps_opaque((unsigned)min(n0 + 4 * ((tid & 63) >> 4) + (tid >> 6), MW - 1)));
      if (!pd_wait(&s_ok, ctr(C_P0, rbA), 1, (unsigned)(NC0 * (s + 1)), lim, status)) return;
      PD_TS(4, 1);
      pd_ln16(rp1p, (unsigned)(((size_t)s * B + m0) * MW), MW, ln, scr, nullptr, 0, wave, lane);
      __syncthreads();
      f32x4 acc[1];
      pd_lds_mfma<1>(scr, wf, acc, wave, r, q);
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 4; ++e) scr[(wave * 4 + e) * 64 + lane] = acc[0][e];
      __syncthreads();
      const int e2 = tid >> 6, l2 = tid & 63, row2 = l2 & 15, col2 = 4 * (l2 >> 4) + e2, n = n0 + col2;
      if (n < MW) {
        const float v = ((scr[e2 * 64 + l2] + scr[(4 + e2) * 64 + l2]) + scr[(8 + e2) * 64 + l2]) + scr[(12 + e2) * 64 + l2];
        ps_st1(rp2p, 4u * (unsigned)(((size_t)s * B + m0 + row2) * MW + n), v + bias);
      }
      PD_TS(4, 6);
      pd_signal(ctr(C_P1, rbA), 1);
      PD_TS(4, 7);
    }
    // ===================== DSM: prior logit_net.4-6 + Categorical sample =====
    if (doS) {
      const int m0 = rbS * 16;
      const int ml3 = tid >> 3, sub = tid & 7, c3 = 4 * sub;
      const bool act3 = ml3 < 16;
      float qn[4] = {1.f, 1.f, 1.f, 1.f};
      if (act3) {
        const int m = m0 + ml3;
        if (g.nq.q) {
          const float4 qx = dr_ld4(g.nq.q, (unsigned)((((size_t)s * B + m) * NR + gq) * NCL + c3));
          qn[0] = qx.x, qn[1] = qx.y, qn[2] = qx.z, qn[3] = qx.w;
        } else {
          const uint32_t st = (uint32_t)(g.nq.stream + s), row = (uint32_t)(g.nq.row0 + m), e0 = (uint32_t)(gq * NCL + c3);
#pragma unroll
          for (int i = 0; i < 4; ++i) qn[i] = dr_exp1_k(q_seed, q_off, st, row, e0 + i);
        }
      }
      PD_TS(5, 0);
      PsFrag<3> wf[KSW3][2];
      pd_wfrag3<2>(wf, g.wp6, gq * NCL, LAT, wave, r, q);
      const PdLn ln = pd_lnparams(g.pn4g, g.pn4b, lane);
      const float4 bc = dr_ld4(g.bp6, ps_opaque((unsigned)(gq * NCL + c3)));
      if (!pd_wait(&s_ok, ctr(C_P1, rbS), 1, (unsigned)(NC * (s + 1)), lim, status)) return;
      PD_TS(5, 1);
      pd_ln16(rp2p, (unsigned)(((size_t)s * B + m0) * MW), MW, ln, scr, nullptr, 0, wave, lane);
      __syncthreads();
      f32x4 acc[2];
      pd_lds_mfma<2>(scr, wf, acc, wave, r, q);
      __syncthreads();
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int e = 0; e < 4; ++e) scr[((wave * 2 + ct) * 4 + e) * 64 + lane] = acc[ct][e];
      __syncthreads();
      if (act3) {
        float x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = c3 + i, ct = c >> 4, ql = (c & 15) >> 2, e = c & 3, l = ml3 + 16 * ql;
          float v = 0.f;
#pragma unroll
          for (int w = 0; w < 4; ++w) v += scr[((w * 2 + ct) * 4 + e) * 64 + l];
          x[i] = v + (i == 0 ? bc.x : i == 1 ? bc.y : i == 2 ? bc.z : bc.w);
        }
        const float unimix = g.unimix;
        float mx = fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3]));
        mx = group_max(mx, 8);
        float ex[4], pu[4], pp[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) ex[i] = expf(x[i] - mx);
        const float se = group_sum((ex[0] + ex[1]) + (ex[2] + ex[3]), 8);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pp[i] = ex[i] / se;
          pu[i] = 0.99f * pp[i] + unimix;
        }
        const float sp = group_sum((pu[0] + pu[1]) + (pu[2] + pu[3]), 8);
        float best = (pu[0] / sp) / qn[0];
        int bi = c3;
#pragma unroll
        for (int i = 1; i < 4; ++i) {
          const float v = (pu[i] / sp) / qn[i];
          bi = v > best ? c3 + i : bi;
          best = fmaxf(best, v);
        }
        group_argmax(best, bi, 8);
        const int m = m0 + ml3;
        float4 z;
        z.x = (c3 + 0 == bi) ? ((1.0f + pu[0]) - pu[0]) : 0.0f;
        z.y = (c3 + 1 == bi) ? ((1.0f + pu[1]) - pu[1]) : 0.0f;
        z.z = (c3 + 2 == bi) ? ((1.0f + pu[2]) - pu[2]) : 0.0f;
        z.w = (c3 + 3 == bi) ? ((1.0f + pu[3]) - pu[3]) : 0.0f;
        dr_st4(g.latents, (unsigned)m * ldL + (unsigned)((s + 1) * LAT + gq * NCL + c3), z);
        dr_st4(g.soft, (unsigned)(((size_t)s * B + m) * LAT + gq * NCL + c3), make_float4(pp[0], pp[1], pp[2], pp[3]));
        if ((unsigned)(bi - c3) < 4u) {
          const int i = bi - c3;
          const float zsv = (1.0f + pu[i]) - pu[i];
          ps_gst(g.zg + ((size_t)(s + 1) * B + m) * NR + gq,
                 ((ps_u64)__float_as_uint(zsv) << 32) | ((ps_u64)(unsigned)(s + 1) << 16) | (unsigned)bi);
        }
      }
      PD_TS(5, 6);
      __syncthreads();  // the LDS slabs are reused by the next step's stages
      PD_TS(5, 7);
    }
  }
}

// every workgroup leaves through ps_exit (also after a timed-out wait): the
// last one NaN-fills latents / hiddens / actions / mus / sigmas and the fault
// slot on a timeout
template <int NT, int MR>
__global__ __launch_bounds__(NTH, 1) void k_pdream(PDreamArgs g) {
  pdream_body<NT, MR>(g);
  ps_exit(g.cnt + CNT_LD * (CNT_BLOCKS * C_STATUS + 1), g.cnt + CNT_LD * CNT_BLOCKS * C_STATUS, g.pz);
}

// ---------------------------------------------------------------------------
static size_t pdream_lds_bytes(int A) {
  return sizeof(float) * ((((size_t)(LAT + A) * WLD + 3) & ~(size_t)3) + SCR_F + 64);
}

bool op_pdream_shape_ok(const dr_dims* d, int B, int H, int A) {
  return d->hidden == HD && d->rows == NR && d->cols == NCL && d->prior_h1 == MW && d->prior_h2 == MW &&
         d->actor_h1 == MW && d->actor_h2 == MW && A >= 1 && A <= 8 && H >= 1 && H < 65535 && B >= 16 && B <= 128 &&
         B % 16 == 0 && (B <= 64 || B % 32 == 0);
}

// B <= 128 as the persistent scan (scan.hip): the GRU tiles' per-step h reads
// bound larger batches
bool op_pdream_supported(const dr_dims* d, int B, int H, int A) {
  return !d->launch_form && op_pdream_shape_ok(d, B, H, A);
}

size_t op_pdream_ws_bytes(const dr_dims* d, int B, int H) {
  if (!op_pdream_shape_ok(d, B, H, d->action)) return 0;
  return sizeof(float) * (size_t)H * B * MW + sizeof(unsigned long long) * (size_t)(H + 1) * B * NR + PDREAM_CNT_BYTES +
         PDREAM_TS_BYTES;
}

template <int NT, int MR>
static int launch_pdream(const PDreamArgs& a, int grid, hipStream_t s) {
  auto k = k_pdream<NT, MR>;
  const size_t lds = pdream_lds_bytes(a.A);
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k, NTH, lds) != hipSuccess || per_cu < 1) {
    dr_set_error("pdream: no residency");
    return DR_E_UNSUPPORTED;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(NTH), lds, s, a);
  return dr_check_launch("pdream");
}

int op_pdream(const dr_dims* d, const dr_world_model* wm, const dr_actor* ac, int B, int H, const float* wt,
              const float* wazt, const int* idx0, dr_noise noise, dr_noise nq, int det, float* latents, float* hiddens,
              float* actions, float* mus, float* sigmas, const PDreamTape& tp, void* ws, hipStream_t s) {
  const int A = d->action;
  if (!op_pdream_supported(d, B, H, A)) {
    dr_set_error("pdream: unsupported shape (B=%d H=%d)", B, H);
    return DR_E_UNSUPPORTED;
  }
  const int MR = B <= 64 ? 16 : 32;
  const int RB = B / 16;
  const int grid = std::max(std::max((B / MR) * NUS, RB * NC0), RB * NR);
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    dr_set_error("pdream: device query");
    return DR_E_HIP;
  }
  unsigned mask[16] = {0};
  int avail = cus;
  if (hipExtStreamGetCUMask(s, 16, mask) == hipSuccess) {
    int n = 0;
    for (int i = 0; i < 16; ++i) n += __builtin_popcount(mask[i]);
    if (n > 0) avail = std::min(avail, n);
  }
  if (grid > avail) {
    dr_set_error("pdream: grid %d > %d CUs of the stream", grid, avail);
    return DR_E_UNSUPPORTED;
  }
  PDreamArgs a;
  memset(&a, 0, sizeof(a));
  a.B = B; a.H = H; a.A = A; a.det = det;
  a.wt = wt; a.b_ih = wm->b_ih; a.b_hh = wm->b_hh; a.whh = wm->w_hh;
  a.wp0 = wm->prior.l0.w; a.bp0 = wm->prior.l0.b; a.pn1g = wm->prior.n1.w; a.pn1b = wm->prior.n1.b;
  a.wp3 = wm->prior.l3.w; a.bp3 = wm->prior.l3.b; a.pn4g = wm->prior.n4.w; a.pn4b = wm->prior.n4.b;
  a.wp6 = wm->prior.l6.w; a.bp6 = wm->prior.l6.b;
  a.wa0 = ac->l0.w; a.ba0 = ac->l0.b; a.wazt = wazt;
  a.an1g = ac->n1.w; a.an1b = ac->n1.b; a.wa3 = ac->l3.w; a.ba3 = ac->l3.b; a.an4g = ac->n4.w; a.an4b = ac->n4.b;
  a.wmu = ac->mu.w; a.bmu = ac->mu.b; a.wls = ac->ls.w; a.bls = ac->ls.b;
  a.idx0 = idx0; a.noise = noise; a.nq = nq;
  a.unimix = (float)(0.01 * (1.0 / d->cols));
  a.spin_limit = ps_spin_limit("dream");
  a.latents = latents; a.hiddens = hiddens; a.actions = actions; a.mus = mus; a.sigmas = sigmas;
  {
    const unsigned long long BH = (unsigned long long)B * H;
    float* const outs[5] = {latents, hiddens, actions, mus, sigmas};
    const unsigned long long ns[5] = {(unsigned long long)B * (H + 1) * LAT, (unsigned long long)B * (H + 1) * HD,
                                      BH * A, BH * A, BH * A};
    for (int i = 0; i < 5; ++i) {
      a.pz.p[i] = outs[i];
      a.pz.n[i] = ns[i];
    }
    a.pz.fault = d->fault;
    a.pz.fault_host = d->fault_host;
  }
  a.eps = tp.eps; a.ls_raw = tp.ls_raw; a.pre1a = tp.pre1a; a.x1a = tp.x1a; a.pre2a = tp.pre2a; a.x2a = tp.x2a;
  a.tr = tp.r; a.tu = tp.u; a.tn = tp.n; a.tghn = tp.ghn; a.pre1p = tp.pre1p; a.pre2p = tp.pre2p; a.soft = tp.soft;
  char* base = reinterpret_cast<char*>(ws);
  a.hA = reinterpret_cast<float*>(base);
  a.zg = reinterpret_cast<unsigned long long*>(a.hA + (size_t)H * B * MW);
  a.cnt = reinterpret_cast<unsigned*>(a.zg + (size_t)(H + 1) * B * NR);
  a.ts = reinterpret_cast<long long*>(reinterpret_cast<char*>(a.cnt) + PDREAM_CNT_BYTES);
  // granule tags and counters (adjacent) zeroed by one kernel before every launch
  DR_TRY(op_fill((long long)2 * (H + 1) * B * NR + PDREAM_CNT_BYTES / 4, reinterpret_cast<float*>(a.zg), 0.f, s));
  const bool bf = d->precision == DR_PREC_BF16;
  if (MR == 16) return bf ? launch_pdream<1, 16>(a, grid, s) : launch_pdream<3, 16>(a, grid, s);
  return bf ? launch_pdream<1, 32>(a, grid, s) : launch_pdream<3, 32>(a, grid, s);
}
