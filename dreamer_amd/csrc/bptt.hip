// Persistent BPTT of the imagination unroll: the reverse loop of
// dr_imagine_bwd (engine.hip imagine_bwd_impl; the gradient of the actor loss,
// Agent.py:96-154, through Dreamer.dream_episodes' graph, Dreamer.py:143-175)
// as ONE launch instead of seven launches per step.
//
// Step t = H-1 .. 0 (i = H-1-t), all sums in the launch form's order:
//
//   Q1  g_logit = STE-softmax backward of dL/dz_{t+1} (0.99 g, soft_t);
//       g_x2 partial = g_logit[K-quarter] . W_p6             prior logit_net.6 (K = 1024 in 4 parts)
//   Q2  g_pre2 = LN-SiLU backward (sum of the 4 parts, pre2p_t);  g_x1 = g_pre2 . W_p3
//   Q3  g_pre1 = LN-SiLU backward (g_x1, pre1p_t);  dL/dh_{t+1} = ht + g_pre1 . W_p0;
//       GRU backward (SequenceModel.py:19-24): g_gi, g_gh, the (1 - u) path hu_t
//   Q4  [dz_t | da_t] part = g_gi . W_ih,  dh_t part = g_gh . W_hh   (K = 1800)
//   Q5  actor heads backward (tanh rsample, clamp, softplus; Agent.py:191-210) with
//       dL/da_t = upstream + Q4's part;  g_x2a = g_heads . [W_mu; W_ls]
//   Q6  g_pre2a = LN-SiLU backward (g_x2a, pre2a_t);  g_x1a = g_pre2a . W_a3
//   Q7  g_pre1a = LN-SiLU backward (g_x1a, pre1a_t);  (t > 0) the totals
//       ht_t = ((gH_t + hu_t) + Q4's h part) + g_pre1a . W_a0h,
//       zt_t = (gZ_t + Q4's z part) + g_pre1a . W_a0z
//
// The actor weight gradients (TN products over all B H rows, column sums) run
// after the launch from the saves (g_heads, g_pre*, g_y*, x_hat*), as in the
// launch form.  Hand-offs as dream.hip (persist.h): sc1 stores, a counter per
// 16-row block and stage, sc1 loads; every hand-off buffer is per step.
#include "common.h"
#include "bptt.h"
#include "persist.h"
#include "ops.h"

#include <string.h>
#include <algorithm>

namespace {
constexpr int HD = 600, G3 = 3 * HD, MW = 200, NR = 32, NCL = 32, LAT = NR * NCL;
constexpr int NTH = 256;
constexpr int NCT = (MW + 15) / 16;                 // 13 16-column tiles over 200
constexpr int NQ1 = 4;                              // Q1 K-quarters (256 classes = 8 groups)
constexpr int NT1 = NCT * NQ1;                      // 52
constexpr int NU3 = (HD + 15) / 16;                 // 38 16-unit tiles
constexpr int NZB = LAT / 32, NHB = (HD + 31) / 32;  // 32 z and 19 h blocks of 32 columns
constexpr int NQ4 = NZB + 1 + NHB;                  // 52: z blocks, the action block, h blocks
constexpr int NQ7 = NHB + NZB;                      // 51: h blocks, z blocks
constexpr int P4H = LAT + 32;                       // p4 row: z [0, 1024) | a [1024, 1024 + A) | h [1056, 1656)
constexpr int P4W = P4H + NHB * 32;                 // 1664
constexpr int KPS = 232;                            // LDS A-tile stride, K = 200 (zero to 224)
constexpr int KP1 = 264;                            // K = 256
constexpr int KPA = 1832;                           // K = 1800 (zero to 1824)
constexpr int SA_F = 16 * KPA;                      // A tile
constexpr int RED_F = 4 * 2 * 4 * 64;               // the 4 waves' partial tiles (2 column fragments)
constexpr int CNT_LD = 32, CNT_BLOCKS = 8;
enum { C_Q1 = 0, C_Q2, C_Q3, C_Q4, C_Q5, C_Q6, C_Q7, C_STATUS };
}  // namespace

struct alignas(16) PBpttArgs {
  int B, H, A, spin_limit;
  PBpttIO io;
  const float *pn4g, *pn4b, *pn1g, *pn1b, *an4g, *an4b, *an1g, *an1b;
  // per-step hand-offs
  float *pgx2;  // [H][NQ1][B][MW]
  float *gx1;   // [H][B][MW]
  float *ggi, *ggh;  // [H][B][G3]
  float *hu;    // [H][B][HD]
  float *p4;    // [H][B][P4W]
  float *gx2a, *gx1a;  // [H][B][MW]
  float *zt;    // [H][B][LAT]
  float *ht;    // [H][B][HD]
  unsigned* cnt;
  long long* ts;  // DR_PBPTT_TS builds: [16 steps][7 stages][8 marks][grid] wall-clock stamps (first tile)
  PsPoison pz;    // the actor weight gradients' saves NaN-filled on a timeout (persist.h ps_exit)
};
#ifdef DR_PBPTT_TS
#define PB_TS(st, mk) \
  do { \
    if (threadIdx.x == 0 && i < 16 && p == slot) \
      g.ts[((i * 7 + (st)) * 8 + (mk)) * gridDim.x + blockIdx.x] = (long long)wall_clock64(); \
  } while (0)
#else
#define PB_TS(st, mk) do {} while (0)
#endif

// acc[cf] = A (16 rows x K, LDS rows of stride lda, zero-padded to a multiple of
// 32) . W^T for W rows n0 + 16 cf + r (K contiguous, row stride ldw): the
// wave's k-steps ks = wave, wave + 4, ...; NT terms (split3 or bf16)
constexpr int PD = 3;  // weight fragments loaded PD iterations ahead
template <int NT, int NCF>
struct PbW {
  PsFrag<NT> f[PD][NCF];
};
template <int NT, int NCF, int K>
__device__ __forceinline__ void pb_wload(PsFrag<NT> (&f)[NCF], int it, const float* W, unsigned ldw, int n0, int N,
                                         int wave, int r, int q) {
  constexpr int NKS = (K + 31) / 32;
  const int ks = wave + 4 * it, k = 32 * ks + 8 * q;
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf) {
    const int n = n0 + 16 * cf + r;
    const bool ok = ks < NKS && n < N && k < K;
    f[cf] = ps_frag<NT>(W, ps_opaque(ok ? (unsigned)n * ldw + (unsigned)k : 0u), ok);
  }
}
// the first PD iterations' weight fragments (issued before the stage's poll)
template <int NT, int NCF, int K>
__device__ __forceinline__ PbW<NT, NCF> pb_wpre(const float* W, unsigned ldw, int n0, int N, int wave, int r, int q) {
  constexpr int NIT = ((K + 31) / 32 + 3) / 4;
  PbW<NT, NCF> w;
#pragma unroll
  for (int it = 0; it < PD; ++it)
    if (it < NIT) pb_wload<NT, NCF, K>(w.f[it], it, W, ldw, n0, N, wave, r, q);
  return w;
}

// acc[cf] = A (16 rows x K, LDS rows of stride lda, zero-padded to a multiple of
// 32) . W^T for W rows n0 + 16 cf + r (K contiguous, row stride ldw): the
// wave's k-steps ks = wave, wave + 4, ...; NT terms (split3 or bf16); wp from
// pb_wpre, the later fragments loaded PD iterations ahead
template <int NT, int NCF, int K>
__device__ __forceinline__ void pb_mfma(const float* sA, int lda, PbW<NT, NCF>& wp, const float* W, unsigned ldw, int n0,
                                        int N, f32x4 (&acc)[NCF], int wave, int r, int q) {
  constexpr int NKS = (K + 31) / 32, NIT = (NKS + 3) / 4;
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf) acc[cf] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int ks = wave + 4 * it;
    PsFrag<NT> cur[NCF];
#pragma unroll
    for (int cf = 0; cf < NCF; ++cf) cur[cf] = wp.f[it % PD][cf];
    if (it + PD < NIT) pb_wload<NT, NCF, K>(wp.f[it % PD], it + PD, W, ldw, n0, N, wave, r, q);
    if (ks < NKS) {
      const float* pa = sA + r * lda + 32 * ks + 8 * q;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(pa), x1 = *reinterpret_cast<const f32x4*>(pa + 4);
      ps_u32x4 a[NT];
      ps_split<NT>(x0, x1, a);
#pragma unroll
      for (int cf = 0; cf < NCF; ++cf) {
        ps_u32x4 w[NT];
        ps_wsplit<NT>(cur[cf], w);
        acc[cf] = ps_prod<NT>(w, a, acc[cf]);
      }
    }
  }
}

// the 4 waves' partial tiles meet in LDS in a fixed order; f(row, col, value)
// for the 16 x 16 NCF outputs (D lane (r, q), element e = row r, column 4 q + e)
template <int NCF, typename F>
__device__ __forceinline__ void pb_reduce(float* red, const f32x4 (&acc)[NCF], int wave, int lane, F&& f) {
#pragma unroll
  for (int cf = 0; cf < NCF; ++cf)
#pragma unroll
    for (int e = 0; e < 4; ++e) red[((wave * NCF + cf) * 4 + e) * 64 + lane] = acc[cf][e];
  __syncthreads();
  for (int x = threadIdx.x; x < NCF * 256; x += NTH) {
    const int l = x & 63, e = (x >> 6) & 3, cf = x >> 8;
    const float v = ((red[((0 * NCF + cf) * 4 + e) * 64 + l] + red[((1 * NCF + cf) * 4 + e) * 64 + l]) +
                     red[((2 * NCF + cf) * 4 + e) * 64 + l]) +
                    red[((3 * NCF + cf) * 4 + e) * 64 + l];
    f(l & 15, 16 * cf + 4 * (l >> 4) + e, v);
  }
}

struct PbLn {
  float4 g[4], b[4];
};
__device__ __forceinline__ PbLn pb_lnparams(const float* lng, const float* lnb, int lane) {
  PbLn p;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = (lane & 15) + 16 * j;
    p.g[j] = dr_ld4(lng, ps_opaque(c < MW / 4 ? 4u * c : 0u));
    p.b[j] = dr_ld4(lnb, ps_opaque(c < MW / 4 ? 4u * c : 0u));
  }
  return p;
}

// SiLU(LayerNorm(pre)) backward of 16 rows (k_ln_silu_bwd's arithmetic; 16
// lanes per row, wave w takes rows 4 w .. 4 w + 3): g_x = the sum of np sc1
// sources (row r of source i at float offset g0 + i * gps + r * gld), pre from
// the tape (row r at pre + r * pld).  g_pre goes to the LDS A tile (stride
// KPS, zero to 224); with sv, also g_pre, g_y and x_hat rows (stride svld).
__device__ __forceinline__ void pb_lnbwd16(__amdgpu_buffer_rsrc_t rg, unsigned g0, unsigned gps, int np, unsigned gld,
                                           const float* pre, unsigned pld, const PbLn& ln, float* sA, float* sv_gpre,
                                           float* sv_gy, float* sv_xh, unsigned svld, int wave, int lane) {
  const int ml = wave * 4 + (lane >> 4), sub = lane & 15;
  f32x4 gx[4][4], pv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = sub + 16 * j;
    const unsigned o = ps_opaque(c < MW / 4 ? 4u * c : 0u);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      gx[i][j] = i < np ? ps_ld4(rg, 4u * (g0 + (unsigned)i * gps + (unsigned)ml * gld + o)) : (f32x4){0.f, 0.f, 0.f, 0.f};
    const float4 p4v = dr_ld4(pre, (unsigned)ml * pld + o);
    pv[j] = (f32x4){p4v.x, p4v.y, p4v.z, p4v.w};
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) ps_pin(gx[i][j]);
  float sm = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (sub + 16 * j < MW / 4) sm += (pv[j][0] + pv[j][1]) + (pv[j][2] + pv[j][3]);
  const float mean = row16_sum(sm) / (float)MW;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (sub + 16 * j < MW / 4)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float dd = pv[j][e] - mean;
        sq += dd * dd;
      }
  const float rstd = 1.0f / sqrtf(row16_sum(sq) / (float)MW + 1e-5f);
  float c1 = 0.f, c2 = 0.f;
  f32x4 xh[4], gxh[4], gyv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float gg[4] = {ln.g[j].x, ln.g[j].y, ln.g[j].z, ln.g[j].w};
    const float bb[4] = {ln.b[j].x, ln.b[j].y, ln.b[j].z, ln.b[j].w};
    const bool ok = sub + 16 * j < MW / 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float g = ((gx[0][j][e] + gx[1][j][e]) + gx[2][j][e]) + gx[3][j][e];
      const float x = (pv[j][e] - mean) * rstd;
      const float y = x * gg[e] + bb[e];
      const float sg = 1.0f / (1.0f + expf(-y));
      const float gy = g * (sg * (1.0f + y * (1.0f - sg)));
      const float gh = gy * gg[e];
      xh[j][e] = x;
      gyv[j][e] = gy;
      gxh[j][e] = gh;
      if (ok) {
        c1 += gh;
        c2 += gh * x;
      }
    }
  }
  c1 = row16_sum(c1) / (float)MW;
  c2 = row16_sum(c2) / (float)MW;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = sub + 16 * j;
    float4 gp = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < MW / 4) {
      gp.x = rstd * (gxh[j][0] - c1 - xh[j][0] * c2);
      gp.y = rstd * (gxh[j][1] - c1 - xh[j][1] * c2);
      gp.z = rstd * (gxh[j][2] - c1 - xh[j][2] * c2);
      gp.w = rstd * (gxh[j][3] - c1 - xh[j][3] * c2);
      if (sv_gpre) {
        const unsigned o = (unsigned)ml * svld + 4u * c;
        dr_st4(sv_gpre, o, gp);
        dr_st4(sv_gy, o, make_float4(gyv[j][0], gyv[j][1], gyv[j][2], gyv[j][3]));
        dr_st4(sv_xh, o, make_float4(xh[j][0], xh[j][1], xh[j][2], xh[j][3]));
      }
    }
    if (c < 7 * 8) *reinterpret_cast<float4*>(&sA[ml * KPS + 4 * c]) = gp;
  }
}

// A stage's tiles are (row block rb, column tile c).  Column tile c runs on
// the XCD c % 8 (workgroup b runs on XCD b % 8 when the grid is a multiple of
// 8: for speed only -- the protocol does not depend on placement), so each
// XCD's L2 holds the weight columns of its tiles once; the XCD's 8-strided
// workgroups walk its (column, row block) pairs.
#define PB_TILES(NCOL)                                     \
  for (int p = slot;; p += SL)                             \
    if (const int jj = p / RB, rb = p - jj * RB, c = xcd + 8 * jj; c >= (NCOL)) \
      break;                                               \
    else

template <int NT>
__device__ __forceinline__ void pbptt_body(const PBpttArgs& g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int s_ok;
  __shared__ float s_gh[16][16];
  const int B = g.B, H = g.H, A = g.A, G = gridDim.x;
  const int b = blockIdx.x, tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
  const int RB = B / 16;
  const int xcd = b & 7, slot = b >> 3, SL = G >> 3;
  float* sA = smem;
  float* red = smem + SA_F;
  unsigned* cnt = g.cnt;
  unsigned* status = cnt + CNT_LD * CNT_BLOCKS * C_STATUS;
  auto ctr = [&](int st, int blk) { return cnt + CNT_LD * (CNT_BLOCKS * st + blk); };
  const int lim = g.spin_limit;
  const PBpttIO& io = g.io;
  const unsigned ldH = (unsigned)((H + 1) * HD), ldL = (unsigned)((H + 1) * LAT);
  const unsigned ldM = (unsigned)(H * MW);
  const __amdgpu_buffer_rsrc_t rpg = ps_rsrc(g.pgx2, 4u * H * NQ1 * B * MW);
  const __amdgpu_buffer_rsrc_t rgx1 = ps_rsrc(g.gx1, 4u * H * B * MW);
  const __amdgpu_buffer_rsrc_t rgi = ps_rsrc(g.ggi, 4u * H * B * G3);
  const __amdgpu_buffer_rsrc_t rgh = ps_rsrc(g.ggh, 4u * H * B * G3);
  const __amdgpu_buffer_rsrc_t rhu = ps_rsrc(g.hu, 4u * H * B * HD);
  const __amdgpu_buffer_rsrc_t rp4 = ps_rsrc(g.p4, 4u * H * B * P4W);
  const __amdgpu_buffer_rsrc_t rg2a = ps_rsrc(g.gx2a, 4u * H * B * MW);
  const __amdgpu_buffer_rsrc_t rg1a = ps_rsrc(g.gx1a, 4u * H * B * MW);
  const __amdgpu_buffer_rsrc_t rzt = ps_rsrc(g.zt, 4u * H * B * LAT);
  const __amdgpu_buffer_rsrc_t rht = ps_rsrc(g.ht, 4u * H * B * HD);
  const __amdgpu_buffer_rsrc_t rgz = ps_rsrc(io.gZ, 4u * B * ldL);
  const __amdgpu_buffer_rsrc_t rgH = ps_rsrc(io.gH, 4u * B * ldH);

  for (int i = 0; i < H; ++i) {
    const int t = H - 1 - i;
    // ======================= Q1: STE backward + W_p6 (K-quarter) ============
    PB_TILES(NT1) {
      PB_TS(0, 0);
      const int kq = c / NCT, ct = c - kq * NCT;
      const int m0 = rb * 16, n0 = ct * 16;
      auto wp = pb_wpre<NT, 1, 256>(io.tl6p + kq * 256, LAT, n0, MW, wave, r, q);
      if (i >= 1 && !ps_wait(&s_ok, ctr(C_Q7, rb), CNT_LD, 1, (unsigned)(NQ7 * i), lim, status)) return;
      PB_TS(0, 1);
      // dL/dz_{t+1}: the upstream gradient at t = H-1, else Q7's total
      const __amdgpu_buffer_rsrc_t rz = i == 0 ? rgz : rzt;
      const unsigned z0 = i == 0 ? (unsigned)m0 * ldL + (unsigned)((t + 1) * LAT) : (unsigned)((t + 1) * B + m0) * LAT;
      const unsigned zld = i == 0 ? ldL : (unsigned)LAT;
      f32x4 gz[4];
      float4 sv[4];
#pragma unroll
      for (int pass = 0; pass < 4; ++pass) {
        const int p = pass * 32 + (tid >> 3), row = p >> 3, grp = p & 7, c4 = 4 * (tid & 7);
        const unsigned cls = (unsigned)(kq * 256 + grp * 32 + c4);
        gz[pass] = ps_ld4(rz, 4u * (z0 + (unsigned)row * zld + cls));
        sv[pass] = dr_ld4(io.soft, (unsigned)((t * B + m0 + row) * LAT) + cls);
      }
#pragma unroll
      for (int pass = 0; pass < 4; ++pass) ps_pin(gz[pass]);
#pragma unroll
      for (int pass = 0; pass < 4; ++pass) {
        const int p = pass * 32 + (tid >> 3), row = p >> 3, grp = p & 7, c4 = 4 * (tid & 7);
        const float s4[4] = {sv[pass].x, sv[pass].y, sv[pass].z, sv[pass].w};
        float gs[4], dot = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          gs[e] = gz[pass][e] * 0.99f;
          dot += gs[e] * s4[e];
        }
        dot = group_sum(dot, 8);
        float4 gl;
        gl.x = s4[0] * (gs[0] - dot);
        gl.y = s4[1] * (gs[1] - dot);
        gl.z = s4[2] * (gs[2] - dot);
        gl.w = s4[3] * (gs[3] - dot);
        *reinterpret_cast<float4*>(&sA[row * KP1 + grp * 32 + c4]) = gl;
      }
      __syncthreads();
      f32x4 acc[1];
      pb_mfma<NT, 1, 256>(sA, KP1, wp, io.tl6p + kq * 256, LAT, n0, MW, acc, wave, r, q);
      pb_reduce<1>(red, acc, wave, lane, [&](int row, int col, float v) {
        const int n = n0 + col;
        if (n < MW) ps_st1(rpg, 4u * (unsigned)((((size_t)t * NQ1 + kq) * B + m0 + row) * MW + n), v);
      });
      PB_TS(0, 6);
      ps_signal_n(ctr(C_Q1, rb), 0, 1);
      PB_TS(0, 7);
    }
    // ======================= Q2: LN-SiLU backward (prior.4) + W_p3 ==========
    PB_TILES(NCT) {
      PB_TS(1, 0);
      const int ct = c, m0 = rb * 16, n0 = ct * 16;
      const PbLn ln = pb_lnparams(g.pn4g, g.pn4b, lane);
      auto wp = pb_wpre<NT, 1, MW>(io.tl3p, MW, n0, MW, wave, r, q);
      if (!ps_wait(&s_ok, ctr(C_Q1, rb), CNT_LD, 1, (unsigned)(NT1 * (i + 1)), lim, status)) return;
      PB_TS(1, 1);
      pb_lnbwd16(rpg, (unsigned)(((size_t)t * NQ1 * B + m0) * MW), (unsigned)(B * MW), NQ1, MW,
                 io.pre2p + (size_t)(t * B + m0) * MW, MW, ln, sA, nullptr, nullptr, nullptr, 0, wave, lane);
      __syncthreads();
      f32x4 acc[1];
      pb_mfma<NT, 1, MW>(sA, KPS, wp, io.tl3p, MW, n0, MW, acc, wave, r, q);
      pb_reduce<1>(red, acc, wave, lane, [&](int row, int col, float v) {
        const int n = n0 + col;
        if (n < MW) ps_st1(rgx1, 4u * (unsigned)(((size_t)t * B + m0 + row) * MW + n), v);
      });
      PB_TS(1, 6);
      ps_signal_n(ctr(C_Q2, rb), 0, 1);
      PB_TS(1, 7);
    }
    // ======================= Q3: LN-SiLU backward (prior.1) + W_p0 + GRU backward
    PB_TILES(NU3) {
      PB_TS(2, 0);
      const int ut = c, m0 = rb * 16, u0 = ut * 16;
      const PbLn ln = pb_lnparams(g.pn1g, g.pn1b, lane);
      auto wp = pb_wpre<NT, 1, MW>(io.tl0p, MW, u0, HD, wave, r, q);
      // this thread's output of the reduce (row, column): its GRU-backward
      // operands, loaded before the poll (Q7's total of step t+1 is complete
      // once Q1 of this step could start)
      const int xr_ = tid & 15, xc_ = 4 * ((tid & 63) >> 4) + ((tid >> 6) & 3);
      const int jx = min(u0 + xc_, HD - 1), mx = m0 + xr_;
      const size_t ox = ((size_t)t * B + mx) * HD + jx;
      const float rr = io.r[ox], uu = io.u[ox], nn = io.n[ox], hn = io.ghn[ox];
      const float hvx = io.hiddens[(size_t)mx * ldH + (size_t)t * HD + jx];
      if (i >= 1 && !ps_wait(&s_ok, ctr(C_Q7, rb), CNT_LD, 1, (unsigned)(NQ7 * i), lim, status)) return;
      float hs = i == 0 ? ps_ld1(rgH, 4u * ((unsigned)mx * ldH + (unsigned)((t + 1) * HD + jx)))
                        : ps_ld1(rht, 4u * (unsigned)(((size_t)(t + 1) * B + mx) * HD + jx));
      ps_pin(hs);
      if (!ps_wait(&s_ok, ctr(C_Q2, rb), CNT_LD, 1, (unsigned)(NCT * (i + 1)), lim, status)) return;
      PB_TS(2, 1);
      pb_lnbwd16(rgx1, (unsigned)(((size_t)t * B + m0) * MW), 0u, 1, MW, io.pre1p + (size_t)(t * B + m0) * MW, MW, ln,
                 sA, nullptr, nullptr, nullptr, 0, wave, lane);
      __syncthreads();
      f32x4 acc[1];
      pb_mfma<NT, 1, MW>(sA, KPS, wp, io.tl0p, MW, u0, HD, acc, wave, r, q);
      pb_reduce<1>(red, acc, wave, lane, [&](int row, int col, float v) {
        const int j = u0 + col, m = m0 + row;
        if (j >= HD) return;
        // (row, col) is this thread's (xr_, xc_): one output per thread
        // dL/dh_{t+1} = (upstream at t = H-1, else Q7's total) + the prior's part
        const float gg = hs + v;
        const size_t o = ((size_t)t * B + m) * HD + j;
        const float hv = hvx;
        // k_gru_bwd's arithmetic
        const float g_hmn = gg * uu;
        const float g_u = gg * (hv - nn);
        const float g_n = gg + (-g_hmn);
        const float g_pn = g_n * (1.0f - nn * nn);
        const float g_r = g_pn * hn;
        const float g_hn = g_pn * rr;
        const float g_pr = g_r * (1.0f - rr) * rr;
        const float g_pu = g_u * (1.0f - uu) * uu;
        const unsigned gb = (unsigned)(((size_t)t * B + m) * G3 + j);
        ps_st1(rgi, 4u * gb, g_pr);
        ps_st1(rgi, 4u * (gb + HD), g_pu);
        ps_st1(rgi, 4u * (gb + 2 * HD), g_pn);
        ps_st1(rgh, 4u * gb, g_pr);
        ps_st1(rgh, 4u * (gb + HD), g_pu);
        ps_st1(rgh, 4u * (gb + 2 * HD), g_hn);
        ps_st1(rhu, 4u * (unsigned)o, g_hmn);
      });
      PB_TS(2, 6);
      ps_signal_n(ctr(C_Q3, rb), 0, 1);
      PB_TS(2, 7);
    }
    // ======================= Q4: g_gi . W_ih, g_gh . W_hh (K = 1800) ========
    PB_TILES(NQ4) {
      PB_TS(3, 0);
      const int cb = c, m0 = rb * 16;
      const bool zb = cb < NZB, ab = cb == NZB;
      const bool live = t > 0 || ab;  // at t = 0 only the action gradient is consumed
      const float* W = (zb || ab) ? io.wt : io.twhh;
      const int n0 = zb ? 32 * cb : ab ? LAT : 32 * (cb - NZB - 1);
      const int N = !live ? 0 : zb ? LAT : ab ? LAT + A : HD;
      auto wp = pb_wpre<NT, 2, G3>(W, G3, n0, N, wave, r, q);
      if (!ps_wait(&s_ok, ctr(C_Q3, rb), CNT_LD, 1, (unsigned)(NU3 * (i + 1)), lim, status)) return;
      PB_TS(3, 1);
      if (live) {
        const __amdgpu_buffer_rsrc_t ra = (zb || ab) ? rgi : rgh;
        const unsigned a0 = (unsigned)(((size_t)t * B + m0) * G3);
        // the 16 x 1800 A tile into LDS (zero to 1824): all 28.1 float4 per
        // thread issued at once (one round trip), then stored
        constexpr int NA4 = 16 * (G3 / 4), NPT = (NA4 + NTH - 1) / NTH;
        f32x4 v[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int x = k * NTH + tid;
          const int row = x / (G3 / 4), c4 = x - row * (G3 / 4);
          v[k] = x < NA4 ? ps_ld4(ra, 4u * (a0 + (unsigned)row * G3 + 4u * c4)) : (f32x4){0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int k = 0; k < NPT; ++k) ps_pin(v[k]);
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int x = k * NTH + tid;
          const int row = x / (G3 / 4), c4 = x - row * (G3 / 4);
          if (x < NA4) *reinterpret_cast<f32x4*>(&sA[row * KPA + 4 * c4]) = v[k];
        }
        if (tid < 16 * 6)
          *reinterpret_cast<f32x4*>(&sA[(tid / 6) * KPA + G3 + 4 * (tid % 6)]) = (f32x4){0.f, 0.f, 0.f, 0.f};
        __syncthreads();
        const int c0 = zb ? 32 * cb : ab ? LAT : P4H + 32 * (cb - NZB - 1);  // column in p4
        f32x4 acc[2];
        pb_mfma<NT, 2, G3>(sA, KPA, wp, W, G3, n0, N, acc, wave, r, q);
        pb_reduce<2>(red, acc, wave, lane, [&](int row, int col, float v) {
          if (n0 + col < N) ps_st1(rp4, 4u * (unsigned)(((size_t)t * B + m0 + row) * P4W + c0 + col), v);
        });
      }
      PB_TS(3, 6);
      ps_signal_n(ctr(C_Q4, rb), 0, 1);
      PB_TS(3, 7);
    }
    // ======================= Q5: actor heads backward + [W_mu; W_ls] =========
    PB_TILES(NCT) {
      PB_TS(4, 0);
      const int ct = c, m0 = rb * 16, n0 = ct * 16;
      const int nl = tid & 15, ml4 = tid >> 4, n = n0 + nl;
      float w[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = (k < 2 * A && n < MW) ? io.thead[(size_t)n * 2 * A + k] : 0.f;
      if (!ps_wait(&s_ok, ctr(C_Q4, rb), CNT_LD, 1, (unsigned)(NQ4 * (i + 1)), lim, status)) return;
      PB_TS(4, 1);
      if (tid < 16 * A) {
        const int ml = tid / A, k = tid - ml * A, m = m0 + ml;
        const size_t o = (size_t)m * H * A + (size_t)t * A + k;
        float gmu = io.g_mus ? io.g_mus[o] : 0.0f;
        float gsg = io.g_sigmas ? io.g_sigmas[o] : 0.0f;
        const float ga = io.gA[o] + ps_ld1(rp4, 4u * (unsigned)(((size_t)t * B + m) * P4W + LAT + k));
        const float av = io.actions[o];
        const float gp = ga * (1.0f - av * av);
        gmu = gmu + gp;
        gsg = gsg + gp * io.eps[((size_t)t * B + m) * A + k];
        const float lr = io.ls_raw[o];
        const float lc = fminf(fmaxf(lr, -5.0f), 2.0f);
        float gls = 0.f;
        if (lr >= -5.0f && lr <= 2.0f) {
          const float ez = expf(lc);
          gls = (lc > 20.0f) ? gsg : gsg * ez / (ez + 1.0f);
        }
        if (ct == 0) {
          io.gheads[(size_t)m * H * 2 * A + (size_t)t * 2 * A + k] = gmu;
          io.gheads[(size_t)m * H * 2 * A + (size_t)t * 2 * A + A + k] = gls;
        }
        s_gh[ml][k] = gmu;
        s_gh[ml][A + k] = gls;
      }
      __syncthreads();
      if (n < MW) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (k < 2 * A) v = fmaf(s_gh[ml4][k], w[k], v);
        ps_st1(rg2a, 4u * (unsigned)(((size_t)t * B + m0 + ml4) * MW + n), v);
      }
      PB_TS(4, 6);
      ps_signal_n(ctr(C_Q5, rb), 0, 1);
      PB_TS(4, 7);
    }
    // ======================= Q6: LN-SiLU backward (actor.4) + W_a3 ==========
    PB_TILES(NCT) {
      PB_TS(5, 0);
      const int ct = c, m0 = rb * 16, n0 = ct * 16;
      const PbLn ln = pb_lnparams(g.an4g, g.an4b, lane);
      auto wp = pb_wpre<NT, 1, MW>(io.tl3a, MW, n0, MW, wave, r, q);
      if (!ps_wait(&s_ok, ctr(C_Q5, rb), CNT_LD, 1, (unsigned)(NCT * (i + 1)), lim, status)) return;
      PB_TS(5, 1);
      const size_t so = (size_t)m0 * ldM + (size_t)t * MW;
      pb_lnbwd16(rg2a, (unsigned)(((size_t)t * B + m0) * MW), 0u, 1, MW, io.pre2a + so, ldM, ln, sA,
                 ct == 0 ? io.gpre2a + so : nullptr, io.gy2a + so, io.xh2a + so, ldM, wave, lane);
      __syncthreads();
      f32x4 acc[1];
      pb_mfma<NT, 1, MW>(sA, KPS, wp, io.tl3a, MW, n0, MW, acc, wave, r, q);
      pb_reduce<1>(red, acc, wave, lane, [&](int row, int col, float v) {
        const int n = n0 + col;
        if (n < MW) ps_st1(rg1a, 4u * (unsigned)(((size_t)t * B + m0 + row) * MW + n), v);
      });
      PB_TS(5, 6);
      ps_signal_n(ctr(C_Q6, rb), 0, 1);
      PB_TS(5, 7);
    }
    // ======================= Q7: LN-SiLU backward (actor.1) + W_a0 + totals ==
    PB_TILES(NQ7) {
      PB_TS(6, 0);
      const int cb = c, m0 = rb * 16;
      const bool hb = cb < NHB;
      const PbLn ln = pb_lnparams(g.an1g, g.an1b, lane);
      const int j0 = hb ? 32 * cb : 32 * (cb - NHB);  // column within h / z
      const int n0 = hb ? j0 : HD + j0;                // row of W_a0^T
      const int N = t == 0 ? 0 : hb ? HD : HD + LAT;
      auto wp = pb_wpre<NT, 2, MW>(io.tl0a, MW, n0, N, wave, r, q);
      // this thread's two outputs of the reduce (columns xc_, xc_ + 16 of row
      // xr_): their addends, loaded before the poll on Q6 (Q3 / Q4 of this
      // step complete first)
      const int xr_ = tid & 15, xc_ = 4 * ((tid & 63) >> 4) + ((tid >> 6) & 3), mx = m0 + xr_;
      float ad[2] = {0.f, 0.f};
      if (t > 0) {
        if (!ps_wait(&s_ok, ctr(C_Q4, rb), CNT_LD, 1, (unsigned)(NQ4 * (i + 1)), lim, status)) return;
#pragma unroll
        for (int cf = 0; cf < 2; ++cf) {
          const int j = min(j0 + xc_ + 16 * cf, hb ? HD - 1 : LAT - 1);
          if (hb) {
            const float up = io.gH[(size_t)mx * ldH + (size_t)t * HD + j];
            const float hv = ps_ld1(rhu, 4u * (unsigned)(((size_t)t * B + mx) * HD + j));
            const float p4v = ps_ld1(rp4, 4u * (unsigned)(((size_t)t * B + mx) * P4W + P4H + j));
            ad[cf] = (up + hv) + p4v;
          } else {
            const float up = io.gZ[(size_t)mx * ldL + (size_t)t * LAT + j];
            const float p4v = ps_ld1(rp4, 4u * (unsigned)(((size_t)t * B + mx) * P4W + j));
            ad[cf] = up + p4v;
          }
        }
        ps_pin(ad[0]);
        ps_pin(ad[1]);
      }
      if (!ps_wait(&s_ok, ctr(C_Q6, rb), CNT_LD, 1, (unsigned)(NCT * (i + 1)), lim, status)) return;
      PB_TS(6, 1);
      const size_t so = (size_t)m0 * ldM + (size_t)t * MW;
      pb_lnbwd16(rg1a, (unsigned)(((size_t)t * B + m0) * MW), 0u, 1, MW, io.pre1a + so, ldM, ln, sA,
                 cb == 0 ? io.gpre1a + so : nullptr, io.gy1a + so, io.xh1a + so, ldM, wave, lane);
      if (t > 0) {
        __syncthreads();
        f32x4 acc[2];
        pb_mfma<NT, 2, MW>(sA, KPS, wp, io.tl0a, MW, n0, N, acc, wave, r, q);
        pb_reduce<2>(red, acc, wave, lane, [&](int row, int col, float v) {
          // (row, col) = (xr_, xc_ + 16 cf): the addends prefetched above
          const int j = j0 + col, m = m0 + row;
          const float a = ad[col >= 16 ? 1 : 0];
          if (hb) {
            if (j >= HD) return;
            ps_st1(rht, 4u * (unsigned)(((size_t)t * B + m) * HD + j), a + v);
          } else {
            ps_st1(rzt, 4u * (unsigned)(((size_t)t * B + m) * LAT + j), a + v);
          }
        });
      }
      PB_TS(6, 6);
      ps_signal_n(ctr(C_Q7, rb), 0, 1);
      PB_TS(6, 7);
    }
  }
}

// every workgroup leaves through ps_exit (also after a timed-out wait): the
// last one NaN-fills the saves the actor weight gradients are formed from and
// the fault slot on a timeout
template <int NT>
__global__ __launch_bounds__(NTH, 1) void k_pbptt(PBpttArgs g) {
  pbptt_body<NT>(g);
  ps_exit(g.cnt + CNT_LD * (CNT_BLOCKS * C_STATUS + 1), g.cnt + CNT_LD * CNT_BLOCKS * C_STATUS, g.pz);
}

// ---------------------------------------------------------------------------
// B <= 64: at B = 128 the K = 1800 stage has two tiles per workgroup and the
// launch form measured faster (424.9 k against 439.1 k steps/s, profiles/r05q_ab_persistent.txt)
bool op_pbptt_shape_ok(const dr_dims* d, int B, int H, int A) {
  return d->hidden == HD && d->rows == NR && d->cols == NCL && d->prior_h1 == MW && d->prior_h2 == MW &&
         d->actor_h1 == MW && d->actor_h2 == MW && A >= 1 && A <= 8 && H >= 1 && B >= 16 && B <= 64 && B % 16 == 0;
}

bool op_pbptt_supported(const dr_dims* d, int B, int H, int A) {
  return !d->launch_form && op_pbptt_shape_ok(d, B, H, A);
}

static size_t pbptt_floats(int B, int H) {
  const size_t per = (size_t)NQ1 * MW + MW + 2 * G3 + HD + P4W + 2 * MW + LAT + HD;
  return per * (size_t)B * H;
}

size_t op_pbptt_ws_bytes(const dr_dims* d, int B, int H) {
  if (!op_pbptt_shape_ok(d, B, H, d->action)) return 0;
  return sizeof(float) * pbptt_floats(B, H) + PBPTT_CNT_BYTES + PBPTT_TS_BYTES;
}

static size_t pbptt_lds_bytes() { return sizeof(float) * (SA_F + RED_F); }

template <int NT>
static int launch_pbptt(const PBpttArgs& a, int grid, hipStream_t s) {
  auto k = k_pbptt<NT>;
  const size_t lds = pbptt_lds_bytes();
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k, NTH, lds) != hipSuccess || per_cu < 1) {
    dr_set_error("pbptt: no residency");
    return DR_E_UNSUPPORTED;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(NTH), lds, s, a);
  return dr_check_launch("pbptt");
}

int op_pbptt(const dr_dims* d, const dr_world_model* wm, const dr_actor* ac, int B, int H, const PBpttIO& io, void* ws,
             hipStream_t s) {
  const int A = d->action;
  if (!op_pbptt_supported(d, B, H, A)) {
    dr_set_error("pbptt: unsupported shape (B=%d H=%d)", B, H);
    return DR_E_UNSUPPORTED;
  }
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    dr_set_error("pbptt: device query");
    return DR_E_HIP;
  }
  unsigned mask[16] = {0};
  int avail = cus;
  if (hipExtStreamGetCUMask(s, 16, mask) == hipSuccess) {
    int n = 0;
    for (int i = 0; i < 16; ++i) n += __builtin_popcount(mask[i]);
    if (n > 0) avail = std::min(avail, n);
  }
  // every stage loops over its tiles with a grid stride: any grid works, one
  // workgroup per CU keeps them all resident
  const int grid = std::min(avail, 256) & ~7;
  if (grid < 32) {
    dr_set_error("pbptt: %d CUs", avail);
    return DR_E_UNSUPPORTED;
  }
  PBpttArgs a;
  memset(&a, 0, sizeof(a));
  a.B = B; a.H = H; a.A = A; a.spin_limit = ps_spin_limit("bptt");
  a.io = io;
  {
    const unsigned long long BH = (unsigned long long)B * H;
    float* const outs[7] = {io.gheads, io.gpre2a, io.gy2a, io.xh2a, io.gpre1a, io.gy1a, io.xh1a};
    for (int i = 0; i < 7; ++i) {
      a.pz.p[i] = outs[i];
      a.pz.n[i] = i == 0 ? BH * 2 * A : BH * MW;
    }
    a.pz.fault = d->fault;
    a.pz.fault_host = d->fault_host;
  }
  a.pn4g = wm->prior.n4.w; a.pn4b = wm->prior.n4.b; a.pn1g = wm->prior.n1.w; a.pn1b = wm->prior.n1.b;
  a.an4g = ac->n4.w; a.an4b = ac->n4.b; a.an1g = ac->n1.w; a.an1b = ac->n1.b;
  float* f = reinterpret_cast<float*>(ws);
  const size_t BH = (size_t)B * H;
  a.pgx2 = f; f += BH * NQ1 * MW;
  a.gx1 = f; f += BH * MW;
  a.ggi = f; f += BH * G3;
  a.ggh = f; f += BH * G3;
  a.hu = f; f += BH * HD;
  a.p4 = f; f += BH * P4W;
  a.gx2a = f; f += BH * MW;
  a.gx1a = f; f += BH * MW;
  a.zt = f; f += BH * LAT;
  a.ht = f; f += BH * HD;
  a.cnt = reinterpret_cast<unsigned*>(f);
  a.ts = reinterpret_cast<long long*>(reinterpret_cast<char*>(a.cnt) + PBPTT_CNT_BYTES);
  DR_TRY(op_fill(PBPTT_CNT_BYTES / 4, reinterpret_cast<float*>(a.cnt), 0.f, s));
  return d->precision == DR_PREC_BF16 ? launch_pbptt<1>(a, grid, s) : launch_pbptt<3>(a, grid, s);
}
