// Persistent posterior scan: Dreamer.warm_start_generator (Dreamer.py:244-262)
// as ONE launch instead of three launches per step.
//
//   t = 0:   pre_0 = feat_0                                  (h_0 = 0: latent_mapper.0 sees only features)
//   t >= 1:  h_t   = GRUCell(cat(z_{t-1}, a_{t-1}), h_{t-1}) (SequenceModel.py:19-24)
//            pre_t = feat_t + h_t W_m0h^T                    (latent_mapper.0 on cat(features, h), VAE.py:71-72)
//   all t:   z_t   = sample(SiLU(LN(pre_t)) W_m3^T + b_m3)    (VAE.py:73-99: softmax, 1 % unimix, argmax(p/Exp(1)))
//
// feat_t (the conv encoder + latent_mapper.0's feature columns + bias of all
// S/2 frames) is one time-batched launch before this one (dr_encoder_features).
//
// Why one launch.  The launch form spends ~41 us per step at B = 256 on three
// dependent kernels that each re-read their weights from L2 / MALL (the GRU's
// hidden product alone re-streams 7.9 MB of split weight planes per step, and
// the one-hot gather of W_ih^T another ~60 MB of L2 traffic).  Here every
// workgroup (one per CU) owns a FIXED tile of each of the three stages for the
// whole scan, so its weights are loaded once per scan -- the W_hh / latent
// mapper split3 planes into registers (228 VGPRs per wave in fp32 mode), the
// tile's 30 columns of W_ih^T into LDS (123 KB) -- and per step only the
// activations move between CUs:
//
//   S1 GRU      tile = MR batch rows x 10 hidden units (3 x 10 gate columns):
//               gh = h_{t-1} W_hh^T on the bf16 MFMA (split3 6-product f32 scheme,
//               K split over the 4 waves), gi by gather from the LDS W_ih^T slice
//               (k_gru_gates' summation order: identical gi), gates.  Reads the
//               MR rows of h_{t-1} (154 KB at MR = 64).
//   S2 lm0      tile = 16 rows x 16 of the 200 latent_mapper.0 outputs, K = 600
//   S3 sampler  tile = MS rows x one 32-class group: LN-SiLU of the MS pre rows,
//               the group's 32 logits (split3, K = 200), the categorical sampler
//               (k_ln_gemm_sample's arithmetic and noise keys).
//
// Hand-offs (MI355X_MICROARCH.md "Inter-workgroup visibility", valid-form table
// row 1): every handed-off byte is stored write-through (sc1) and loaded sc1 by
// its consumers; each storing wave drains (vmcnt 0), the workgroup barriers and
// ONE lane adds to a per-row-block counter (agent-scope atomic); a consumer's
// lane 0 polls the counters its rows need (relaxed sc1 loads + s_sleep), then
// the workgroup barrier releases its loads.  Counters are monotonic within the
// launch (zeroed by a fill kernel before it), so a stage waits for
// "count >= producers x steps".  Each stage's outputs sit in a two-slot ring:
// a producer can only be one step ahead of any reader of the slot it
// overwrites (DESIGN.md section 5f walks the dependency chain).
//
// Deadlock freedom needs every workgroup resident: grid <= CUs of the stream
// (CU-masked streams fall back to the launch form), 1 workgroup per CU by LDS.
// Spins are bounded; a timeout sets the status word and the workgroup exits.
#include "common.h"
#include "scan.h"
#include "persist.h"
#include "ops.h"

#include <stdlib.h>
#include <string.h>
#include <algorithm>

namespace {
constexpr int HD = 600, KSH = 19, EH = 200, KSE = 7, NR = 32, NCL = 32, LAT = NR * NCL;
constexpr int UPT = 10, NUS = HD / UPT, NC2 = (EH + 15) / 16, WLD = 3 * UPT;
constexpr int NTH = 256;
constexpr int KSW = 5;     // 32-k steps per wave over K = HD (19 over 4 waves)
constexpr int KSW3 = 2;    // 32-k steps per wave over K = EH (7 over 4 waves)
constexpr int KP3 = 232;   // LDS row stride of the LN-SiLU rows (8 mod 16 dwords)
constexpr int SCR_F = 8192;  // scratch floats (32 KB): idx/zval staging, K-split partials, LN rows
constexpr int CNT_LD = 32;   // counters 128 B apart
constexpr int CNT_H = 0, CNT_PRE = 16, CNT_Z = 32, CNT_STATUS = 48, CNT_EXIT = 49;
}  // namespace


struct alignas(16) PScanArgs {
  int B, T, A, step0;
  const float* wt;  // W_ih^T [LAT + A][3 HD]
  const float* b_ih;
  const float* b_hh;
  const float* whh;  // W_hh [3 HD][HD]
  const float* wm0;  // latent_mapper.0 [EH][F + HD]: its h-columns start at column F
  long long ldm0;
  const float* wm3;  // latent_mapper.3 [LAT][EH]
  const float* ln_g;
  const float* ln_b;
  const float* b3;
  const float* feat;  // [T][B][EH]
  const float* act;
  long long act_sb, act_st;
  dr_noise noise;
  float unimix;
  int spin_limit;
  float* z_out;
  float* h_out;
  float* logits_out;
  float* hb;      // [2][B][HD]
  float* pre;     // [2][B][EH]
  int* iz;        // [2][2][B][NR]: slot s: idx [B][NR] then zval [B][NR]
  unsigned* cnt;  // counters, status
  unsigned long long* zg;  // [B][NR] z granules {zval bits | step + 1 | class} (S3 -> S1)
  long long* ts;  // DR_PSCAN_TS builds: [64 steps][3 stages][8 marks][grid] wall-clock stamps
  PsPoison pz;    // outputs NaN-filled on a timeout (persist.h ps_exit)
};
#ifdef DR_PSCAN_TS
#define PS_TS(st, mk) \
  do { \
    if (threadIdx.x == 0 && t < 64) g.ts[((t * 3 + (st)) * 8 + (mk)) * gridDim.x + blockIdx.x] = (long long)wall_clock64(); \
  } while (0)
#else
#define PS_TS(st, mk) do {} while (0)
#endif

template <int NT, int MR, int MS>
__device__ __forceinline__ void pscan_body(const PScanArgs& g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int s_ok;
  const int B = g.B, T = g.T, A = g.A;
  const int b = blockIdx.x, tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;
  const int n1 = (B / MR) * NUS, n2 = (B / 16) * NC2, n3 = (B / MS) * NR;
  const bool do1 = b < n1, do2 = b < n2, do3 = b < n3;
  float* wih = smem;                                  // [LAT + A][WLD]
  float* scr = smem + (((LAT + A) * WLD + 3) & ~3);   // [SCR_F]
  float* sbias = scr + SCR_F;                         // [64]: S1's b_ih, b_hh of the tile's gate columns
  unsigned* cnt = g.cnt;
  unsigned* status = cnt + CNT_LD * CNT_STATUS;
  const int lim = g.spin_limit;
  const __amdgpu_buffer_rsrc_t rh = ps_rsrc(g.hb, 2u * B * HD * 4u);
  const __amdgpu_buffer_rsrc_t rp = ps_rsrc(g.pre, 2u * B * EH * 4u);
  const __amdgpu_buffer_rsrc_t rz = ps_rsrc(g.iz, 4u * B * NR * 4u);

  // ---- tiles and their resident weights -------------------------------------
  const int rg = b / NUS, us = b - rg * NUS, r0 = rg * MR, u0 = us * UPT;  // S1
  const int rt2 = b / NC2, ct2 = b - rt2 * NC2;                            // S2
  const int rs = b / NR, gq = b - rs * NR, m3 = rs * MS;                   // S3
  PsFrag<NT> w1[KSW][2];  // S1's W_hh fragments stay in registers for the scan
#pragma unroll
  for (int s = 0; s < KSW; ++s) {
    const int ks = KSW * wave + s, k = 32 * ks + 8 * q;
    const bool kok = ks < KSH && k < HD;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const int c = ct * 16 + r;
      const bool ok = do1 && kok && c < WLD;
      const int n = ok ? (c / UPT) * HD + u0 + (c % UPT) : 0;
      w1[s][ct] = ps_frag<NT>(g.whh, (unsigned)(n * HD + k), ok);
    }
  }
  // S1's W_ih^T slice: rows k of W_ih^T (latents, then actions), the tile's 30 gate columns
  if (do1) {
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
  __syncthreads();

  // S3 sampler lanes: row ml3 = tid / 8 of the MS-row block, classes 4 sub .. 4 sub + 3
  const int ml3 = tid >> 3, sub = tid & 7, c3 = 4 * sub;
  const bool act3 = do3 && ml3 < MS;
  const int m3r = m3 + (act3 ? ml3 : 0);
  const float bc[4] = {dr_ld1(g.b3, (unsigned)(gq * NCL + c3)), dr_ld1(g.b3, (unsigned)(gq * NCL + c3 + 1)),
                       dr_ld1(g.b3, (unsigned)(gq * NCL + c3 + 2)), dr_ld1(g.b3, (unsigned)(gq * NCL + c3 + 3))};
  const unsigned long long* rngp = g.noise.rng;
  const unsigned long long rng_seed = rngp ? rngp[0] : 0ull, rng_off = rngp ? rngp[1] : 0ull;

  constexpr int NP1 = (MR * UPT + NTH - 1) / NTH;  // S1 (row, unit) pairs per thread

  for (int t = 0; t < T; ++t) {
    const int step = g.step0 + t;
    // ======================= S1: GRU (t >= 1) ===============================
    if (t >= 1 && do1) {
      PS_TS(0, 0);
      // Loads in the order they are consumed (vmcnt retires in issue order): z
      // granules, a_{t-1} and h_{t-1} for the gate pairs, then -- once the h
      // counter says h_{t-1} is complete (long before z_{t-1}: it is S1 of the
      // previous step) -- all of this wave's h fragments for the product
      int2* siz = reinterpret_cast<int2*>(scr);  // [MR][NR] (class, straight-through value bits)
      float* sact = scr + 2 * MR * NR;           // [MR][8]
      float* sgi = sact + 8 * MR;                // [MR][32]: gi (+ b_ih) of the tile's 30 gate columns
      constexpr int NZ = MR * NR / NTH;
      constexpr int NA1 = (MR * 8 + NTH - 1) / NTH;
      const ps_u64* zsrc = g.zg + (size_t)r0 * NR;
      ps_u64 zv[NZ];
#pragma unroll
      for (int i = 0; i < NZ; ++i) zv[i] = ps_gld(zsrc + tid + NTH * i);
      float av[NA1];
#pragma unroll
      for (int i = 0; i < NA1; ++i) {
        const int x = tid + NTH * i, row = x >> 3, ia = x & 7;
        const bool ok = row < MR && ia < A;
        av[i] = dr_ld1(g.act, ok ? (unsigned)((r0 + row) * g.act_sb + (t - 1) * g.act_st + ia) : 0u);
      }
      const unsigned hprev = (unsigned)(((t - 1) & 1) * B * HD);
      float hv[NP1];
#pragma unroll
      for (int i = 0; i < NP1; ++i) {
        const int p = tid + NTH * i;
        const int row = p / UPT, j = p - row * UPT;
        const bool ok = t >= 2 && p < MR * UPT;
        hv[i] = ps_ld1(rh, ok ? 4u * (hprev + (unsigned)((r0 + row) * HD + u0 + j)) : 0u);
        if (!ok) hv[i] = 0.f;
      }
      if (tid == 0) s_ok = t < 2 || ps_poll(cnt + CNT_LD * (CNT_H + rg), (unsigned)(NUS * (t - 1)), lim, status);
      __syncthreads();
      if (!s_ok) return;
      // h_{t-1} fragments of this wave's k-steps, HR steps ahead (h_0 = 0: t = 1 skips the product)
      constexpr int HR = 5;
      f32x4 ha[HR][MR / 16][2];
      auto load_h = [&](int s, int slot) {
        const int ks = KSW * wave + s;
        const int k = 32 * ks + 8 * q;
        const bool ok = ks < KSH && k < HD;
#pragma unroll
        for (int rt = 0; rt < MR / 16; ++rt) {
          const unsigned o = 4u * (hprev + (unsigned)((r0 + rt * 16 + r) * HD) + (ok ? (unsigned)k : 0u));
          ha[slot][rt][0] = ps_ld4(rh, o);
          ha[slot][rt][1] = ps_ld4(rh, o + 16u);
          if (!ok) ha[slot][rt][0] = ha[slot][rt][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
      };
      if (t >= 2) {
#pragma unroll
        for (int s = 0; s < HR; ++s) load_h(s, s);
      }
      PS_TS(0, 1);
      // z_{t-1} of the MR rows: the sampler's granules, re-read until every
      // tag is step t (no counter: the data carries its own flag)
      {
        unsigned zpend = 0;
#pragma unroll
        for (int i = 0; i < NZ; ++i)
          if ((unsigned)((zv[i] >> 16) & 0xFFFFu) != (unsigned)t) zpend |= 1u << i;
        int spins = 0;
        while (zpend && ++spins <= lim) {
          __builtin_amdgcn_s_sleep(1);
#pragma unroll
          for (int i = 0; i < NZ; ++i)
            if (zpend & (1u << i)) {
              zv[i] = ps_gld(zsrc + tid + NTH * i);
              if ((unsigned)((zv[i] >> 16) & 0xFFFFu) == (unsigned)t) zpend &= ~(1u << i);
            }
        }
        if (zpend) __hip_atomic_store(status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int i = 0; i < NZ; ++i) siz[tid + NTH * i] = make_int2((int)(zv[i] & 0xFFFFu), (int)(zv[i] >> 32));
#pragma unroll
        for (int i = 0; i < NA1; ++i) {
          const int x = tid + NTH * i;
          if (x < MR * 8) sact[x] = av[i];
        }
        if (!__syncthreads_and(zpend == 0)) return;
      }
      PS_TS(0, 2);
      // gi by gather from the LDS slice, thread = (row, column pair): the
      // sampled W_ih^T row of every group read as one 8-byte piece; groups
      // ascending (fmaf), actions, + b_ih (k_gru_gates' summation order)
      for (int p = tid; p < MR * 16; p += NTH) {
        const int row = p >> 4, c0 = 2 * (p & 15);
        if (c0 < WLD) {
          float v0 = 0.f, v1 = 0.f;
          const int2* iz = siz + row * NR;
#pragma unroll 8
          for (int u = 0; u < NR; ++u) {
            const int2 pz = iz[u];
            const float zv = __int_as_float(pz.y);
            const float2 w = *reinterpret_cast<const float2*>(wih + (u * NCL + pz.x) * WLD + c0);
            v0 = fmaf(w.x, zv, v0);
            v1 = fmaf(w.y, zv, v1);
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
      PS_TS(0, 3);
      // gh partial over this wave's k-steps
      f32x4 acc[MR / 16][2];
#pragma unroll
      for (int rt = 0; rt < MR / 16; ++rt) acc[rt][0] = acc[rt][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (t >= 2) {
#pragma unroll
        for (int s = 0; s < KSW; ++s) {
          const int slot = s % HR;
          if (KSW * wave + s < KSH) {
            ps_u32x4 w[2][NT];
            ps_wsplit<NT>(w1[s][0], w[0]);
            ps_wsplit<NT>(w1[s][1], w[1]);
#pragma unroll
            for (int rt = 0; rt < MR / 16; ++rt) {
              ps_u32x4 a[NT];
              ps_split<NT>(ha[slot][rt][0], ha[slot][rt][1], a);
#pragma unroll
              for (int ct = 0; ct < 2; ++ct) acc[rt][ct] = ps_prod<NT>(w[ct], a, acc[rt][ct]);
            }
          }
          if (s + HR < KSW) load_h(s + HR, slot);
        }
      }
      PS_TS(0, 4);
      // K-split partials meet in LDS in two rounds (waves 2, 3 -> 0, 1 -> 0):
      // (w0 + w2) + (w1 + w3); the staged indices are dead (the gather is done)
      constexpr int PF = (MR / 16) * 2 * 256;  // floats of one wave's partial tile set
      __syncthreads();
      if (wave >= 2) {
#pragma unroll
        for (int rt = 0; rt < MR / 16; ++rt)
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int e = 0; e < 4; ++e) scr[(wave - 2) * PF + ((rt * 2 + ct) * 4 + e) * 64 + lane] = acc[rt][ct][e];
      }
      __syncthreads();
      if (wave < 2) {
#pragma unroll
        for (int rt = 0; rt < MR / 16; ++rt)
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[rt][ct][e] += scr[wave * PF + ((rt * 2 + ct) * 4 + e) * 64 + lane];
      }
      __syncthreads();
      if (wave == 1) {
#pragma unroll
        for (int rt = 0; rt < MR / 16; ++rt)
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int e = 0; e < 4; ++e) scr[((rt * 2 + ct) * 4 + e) * 64 + lane] = acc[rt][ct][e];
      }
      __syncthreads();
      float* sgh = scr + PF;  // [MR][32]: gh (+ b_hh)
      if (wave == 0) {
#pragma unroll
        for (int rt = 0; rt < MR / 16; ++rt)
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int c = ct * 16 + 4 * q + e;
              const float v = acc[rt][ct][e] + scr[((rt * 2 + ct) * 4 + e) * 64 + lane];
              if (c < WLD) sgh[(rt * 16 + r) * 32 + c] = v + sbias[32 + c];
            }
      }
      __syncthreads();
      PS_TS(0, 5);
      // gates (torch gru_cell op order) for this thread's pairs
      const unsigned hcur = (unsigned)((t & 1) * B * HD);
#pragma unroll
      for (int i = 0; i < NP1; ++i) {
        const int p = tid + NTH * i;
        if (p < MR * UPT) {
          const int row = p / UPT, j = p - row * UPT;
          const float* gh = sgh + row * 32 + j;
          const float* gi = sgi + row * 32 + j;
          const float rr = 1.0f / (1.0f + expf(-(gh[0] + gi[0])));
          const float uu = 1.0f / (1.0f + expf(-(gh[UPT] + gi[UPT])));
          const float nn = tanhf(gi[2 * UPT] + gh[2 * UPT] * rr);
          const float ho = (hv[i] - nn) * uu + nn;
          const unsigned o = (unsigned)((r0 + row) * HD + u0 + j);
          ps_st1(rh, 4u * (hcur + o), ho);
          if (t == T - 1) g.h_out[o] = ho;
        }
      }
      PS_TS(0, 6);
      ps_signal(cnt + CNT_LD * (CNT_H + rg));
      PS_TS(0, 7);
    }
    // ======================= S2: latent_mapper.0 h-part (t >= 1) ===========
    if (t >= 1 && do2) {
      const int m0 = rt2 * 16, n0 = ct2 * 16;
      PS_TS(1, 0);
      // latent_mapper.0's h-columns of the tile (40 KB, L2-resident across the
      // steps), issued with the granule sweep
      PsFrag<NT> w2[KSW];
#pragma unroll
      for (int s = 0; s < KSW; ++s) {
        const int ks = KSW * wave + s, k = 32 * ks + 8 * q, c2 = ct2 * 16 + r;
        const bool ok2 = ks < KSH && k < HD && c2 < EH;
        w2[s] = ps_frag<NT>(g.wm0, ps_opaque(ok2 ? (unsigned)(c2 * g.ldm0 + k) : 0u), ok2);
      }
      // the feature part of this thread's output (plain: written before the launch)
      const int e2 = tid >> 6, l2 = tid & 63, row2 = l2 & 15, col2 = 4 * (l2 >> 4) + e2;
      const bool ok2 = n0 + col2 < EH;
      const float fv = dr_ld1(g.feat, ok2 ? (unsigned)((t * B + m0 + row2) * EH + n0 + col2) : 0u);
      if (tid == 0) s_ok = ps_poll(cnt + CNT_LD * (CNT_H + m0 / MR), (unsigned)(NUS * t), lim, status);
      __syncthreads();
      if (!s_ok) return;
      PS_TS(1, 1);
      const unsigned hcur = (unsigned)((t & 1) * B * HD);
      f32x4 ha[KSW][2];
#pragma unroll
      for (int s = 0; s < KSW; ++s) {
        const int ks = KSW * wave + s, k = 32 * ks + 8 * q;
        const bool ok = ks < KSH && k < HD;
        const unsigned o = 4u * (hcur + (unsigned)((m0 + r) * HD) + (ok ? (unsigned)k : 0u));
        ha[s][0] = ps_ld4(rh, o);
        ha[s][1] = ps_ld4(rh, o + 16u);
        if (!ok) ha[s][0] = ha[s][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
      }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KSW; ++s) {
        if (KSW * wave + s < KSH) {
          ps_u32x4 a[NT], w[NT];
          ps_split<NT>(ha[s][0], ha[s][1], a);
          ps_wsplit<NT>(w2[s], w);
          acc = ps_prod<NT>(w, a, acc);
        }
      }
      PS_TS(1, 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) scr[(wave * 4 + e) * 64 + lane] = acc[e];
      __syncthreads();
      if (ok2) {
        const float v = (((scr[(0 * 4 + e2) * 64 + l2] + scr[(1 * 4 + e2) * 64 + l2]) + scr[(2 * 4 + e2) * 64 + l2]) +
                         scr[(3 * 4 + e2) * 64 + l2]);
        ps_st1(rp, 4u * (unsigned)((t & 1) * B * EH + (m0 + row2) * EH + n0 + col2), v + fv);
      }
      ps_signal(cnt + CNT_LD * (CNT_PRE + rt2));
      PS_TS(1, 7);
    }
    // ======================= S3: LN-SiLU -> logits -> sampler ===============
    if (do3) {
      // noise of this lane's 4 classes first (VALU only, before any wait)
      float qn[4] = {1.f, 1.f, 1.f, 1.f};
      if (act3) {
        const int m = m3 + ml3;
        if (g.noise.q) {
          const float4 qx = dr_ld4(g.noise.q, (unsigned)((((long long)step * B + m) * NR + gq) * NCL + c3));
          qn[0] = qx.x, qn[1] = qx.y, qn[2] = qx.z, qn[3] = qx.w;
        } else {
          const uint32_t st = (uint32_t)(g.noise.stream + step), row = (uint32_t)(g.noise.row0 + m);
          const uint32_t e0 = (uint32_t)(gq * NCL + c3);
#pragma unroll
          for (int i = 0; i < 4; ++i) qn[i] = dr_exp1_k(rng_seed, rng_off, st, row, e0 + i);
        }
      }
      // latent_mapper.3's rows of the group (28 KB, L2-resident across the
      // steps) and this lane's LayerNorm chunks, issued before the poll
      PsFrag<3> w3[KSW3][2];
#pragma unroll
      for (int s = 0; s < KSW3; ++s) {
        const int ks = KSW3 * wave + s, k = 32 * ks + 8 * q;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const bool ok = ks < KSE && k < EH;
          w3[s][ct] = ps_frag<3>(g.wm3, ps_opaque((unsigned)((gq * NCL + ct * 16 + r) * EH + k)), ok);
        }
      }
      const int sub16 = lane & 15;
      float4 lg4[4], lb4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = sub16 + 16 * j;
        lg4[j] = dr_ld4(g.ln_g, ps_opaque(c < EH / 4 ? 4u * c : 0u));
        lb4[j] = dr_ld4(g.ln_b, ps_opaque(c < EH / 4 ? 4u * c : 0u));
      }
      PS_TS(2, 0);
      if (t >= 1) {
        if (tid == 0) {
          bool ok = true;
          for (int i = 0; i < MS / 16 && ok; ++i)
            ok = ps_poll(cnt + CNT_LD * (CNT_PRE + m3 / 16 + i), (unsigned)(NC2 * t), lim, status);
          s_ok = ok;
        }
        __syncthreads();
        if (!s_ok) return;
      }
      PS_TS(2, 1);
      // LN-SiLU of the block's rows into LDS (16 lanes per row, wave w takes
      // rows 4 w .. 4 w + 3 of each 16-row pass, DPP-only sums; k_ln_gemm_sample's
      // element arithmetic), zero-padded to 224
      float* sA = scr;
#pragma unroll
      for (int pass = 0; pass < MS / 16; ++pass) {
        const int ml = pass * 16 + wave * 4 + (lane >> 4), m = m3 + ml;
        f32x4 xr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = sub16 + 16 * j;
          const unsigned o = ps_opaque(c < EH / 4 ? 4u * c : 0u);
          if (t == 0) {
            const float4 xf = dr_ld4(g.feat, (unsigned)(m * EH) + o);
            xr[j] = (f32x4){xf.x, xf.y, xf.z, xf.w};
          } else {
            xr[j] = ps_ld4(rp, 4u * ((unsigned)((t & 1) * B * EH + m * EH) + o));
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) ps_pin(xr[j]);
        float sm = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (sub16 + 16 * j < EH / 4) sm += (xr[j][0] + xr[j][1]) + (xr[j][2] + xr[j][3]);
        const float mean = row16_sum(sm) / (float)EH;
        float sq = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (sub16 + 16 * j < EH / 4) {
            const float dx = xr[j][0] - mean, dy = xr[j][1] - mean, dz = xr[j][2] - mean, dw = xr[j][3] - mean;
            sq += (dx * dx + dy * dy) + (dz * dz + dw * dw);
          }
        const float rstd = 1.0f / sqrtf(row16_sum(sq) / (float)EH + 1e-5f);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = sub16 + 16 * j;
          float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
          if (c < EH / 4) {
            y.x = dr_silu_fast((xr[j][0] - mean) * rstd * lg4[j].x + lb4[j].x);
            y.y = dr_silu_fast((xr[j][1] - mean) * rstd * lg4[j].y + lb4[j].y);
            y.z = dr_silu_fast((xr[j][2] - mean) * rstd * lg4[j].z + lb4[j].z);
            y.w = dr_silu_fast((xr[j][3] - mean) * rstd * lg4[j].w + lb4[j].w);
          }
          if (c < KSE * 8) *reinterpret_cast<float4*>(&sA[ml * KP3 + 4 * c]) = y;
        }
      }
      __syncthreads();
      PS_TS(2, 2);
      f32x4 acc[MS / 16][2];
#pragma unroll
      for (int rt = 0; rt < MS / 16; ++rt) acc[rt][0] = acc[rt][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KSW3; ++s) {
        const int ks = KSW3 * wave + s;
        if (ks < KSE) {
#pragma unroll
          for (int rt = 0; rt < MS / 16; ++rt) {
            const float* pa = sA + (rt * 16 + r) * KP3 + 32 * ks + 8 * q;
            const f32x4 x0 = *reinterpret_cast<const f32x4*>(pa), x1 = *reinterpret_cast<const f32x4*>(pa + 4);
            ps_u32x4 a[3];
            ps_split<3>(x0, x1, a);
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
              ps_u32x4 w[3];
              ps_wsplit<3>(w3[s][ct], w);
              acc[rt][ct] = ps_prod<3>(w, a, acc[rt][ct]);
            }
          }
        }
      }
      PS_TS(2, 4);
      __syncthreads();  // sA consumed: the scratch takes the partials
#pragma unroll
      for (int rt = 0; rt < MS / 16; ++rt)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
          for (int e = 0; e < 4; ++e) scr[((wave * (MS / 16) * 2 + rt * 2 + ct) * 4 + e) * 64 + lane] = acc[rt][ct][e];
      __syncthreads();
      PS_TS(2, 5);
      if (act3) {
        // logits of classes c3 .. c3 + 3 of row ml3: tile (rt, ct), lane r + 16 q, element e
        float x[4];
        const int rt = ml3 >> 4, rr16 = ml3 & 15;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = c3 + i, ct = c >> 4, ql = (c & 15) >> 2, e = c & 3, l = rr16 + 16 * ql;
          float v = 0.f;
#pragma unroll
          for (int w = 0; w < 4; ++w) v += scr[((w * (MS / 16) * 2 + rt * 2 + ct) * 4 + e) * 64 + l];
          x[i] = v + bc[i];
        }
        // the sampler (softmax, 1 % unimix, argmax(p_hat / q), straight-through one-hot)
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
          bi = v > best ? c3 + i : bi;  // ties keep the lower class
          best = fmaxf(best, v);
        }
        group_argmax(best, bi, 8);
        const int m = m3 + ml3;
        if ((unsigned)(bi - c3) < 4u) {
          const int i = bi - c3;
          const float zsv = (1.0f + pu[i]) - pu[i];
          ps_gst(g.zg + (size_t)m * NR + gq,
                 ((ps_u64)__float_as_uint(zsv) << 32) | ((ps_u64)(unsigned)(t + 1) << 16) | (unsigned)bi);
        }
        if (t == T - 1) {
          float4 z;
          z.x = (c3 + 0 == bi) ? ((1.0f + pu[0]) - pu[0]) : 0.0f;
          z.y = (c3 + 1 == bi) ? ((1.0f + pu[1]) - pu[1]) : 0.0f;
          z.z = (c3 + 2 == bi) ? ((1.0f + pu[2]) - pu[2]) : 0.0f;
          z.w = (c3 + 3 == bi) ? ((1.0f + pu[3]) - pu[3]) : 0.0f;
          const unsigned o = (unsigned)(m * LAT + gq * NCL + c3);
          dr_st4(g.z_out, o, z);
          if (g.logits_out) dr_st4(g.logits_out, o, make_float4(x[0], x[1], x[2], x[3]));
        }
      }
      PS_TS(2, 7);
    }
  }
}

// every workgroup leaves through ps_exit (also after a timed-out wait): the
// last one NaN-fills z_out / h_out / logits_out and the fault slot on a timeout
template <int NT, int MR, int MS>
__global__ __launch_bounds__(NTH, 1) void k_pscan(PScanArgs g) {
  pscan_body<NT, MR, MS>(g);
  ps_exit(g.cnt + CNT_LD * CNT_EXIT, g.cnt + CNT_LD * CNT_STATUS, g.pz);
}

int ps_spin_limit(const char* kernel) {
  const char* f = getenv("DREAMER_PERSIST_FORCE");
  if (f && (strcmp(f, "timeout") == 0 || strcmp(f, kernel) == 0)) return -1;
  return 1 << 22;
}

static size_t pscan_lds_bytes(int A) {
  return sizeof(float) * ((((size_t)(LAT + A) * WLD + 3) & ~(size_t)3) + SCR_F + 64);
}

size_t op_pscan_ring_bytes(int B) {
  // hb [2][B][HD], pre [2][B][EH], iz [2][2][B][NR], counters
  return sizeof(float) * ((size_t)2 * B * HD + (size_t)2 * B * EH + (size_t)4 * B * NR) + PSCAN_CNT_BYTES +
         sizeof(unsigned long long) * (size_t)B * NR + PSCAN_TS_BYTES;
}

// B <= 128 by measurement (profiles/r05j_ab_pscan.txt, r05r_ab_scan_B256.txt): configs[1]'s B = 64 gains
// 7-10 % per epoch; at B = 256 the 64-row GRU tiles read 154 KB of h per step per CU, bound by the per-CU
// L2 / MALL rate, and the launch form stays 1 % faster (566.1 k vs 560.8 k fp32, 780.2 k vs 774.4 k bf16)
#ifndef PSCAN_MAX_B
#define PSCAN_MAX_B 128  // B = 256 (64-row GRU tiles, 32-row sampler tiles) builds: 560.8 k vs 566.1 k fp32 (r05r)
#endif
bool op_pscan_supported(const dr_dims* d, int B, int T, int A) {
  // T < 65535: the z granules carry step + 1 in a 16-bit tag (a tag of 0 would match the zeroed granules)
  return !d->launch_form && d->hidden == HD && d->enc_hidden == EH && d->rows == NR && d->cols == NCL && A >= 1 &&
         A <= 8 && T >= 2 && T < 65535 && B >= 16 && B <= PSCAN_MAX_B && B % 16 == 0 && (B <= 64 || B % 32 == 0) &&
         (B <= 128 || B % 64 == 0);
}

template <int NT, int MR, int MS>
static int launch_pscan(const PScanArgs& a, int grid, hipStream_t s) {
  auto k = k_pscan<NT, MR, MS>;
  const size_t lds = pscan_lds_bytes(a.A);
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k, NTH, lds) != hipSuccess || per_cu < 1) {
    dr_set_error("pscan: no residency");
    return DR_E_UNSUPPORTED;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(NTH), lds, s, a);
  return dr_check_launch("pscan");
}

int op_pscan(const dr_dims* d, const dr_world_model* wm, int B, int T, int A, const float* feat, const float* actions,
             long long act_sb, long long act_st, const float* wt, const float* m0h, long long ldm0, dr_noise noise, int step0, float* z_out, float* h_out, float* logits_out,
             void* ring, hipStream_t s) {
  if (!op_pscan_supported(d, B, T, A)) {
    dr_set_error("pscan: unsupported shape (B=%d T=%d)", B, T);
    return DR_E_UNSUPPORTED;
  }
  const int MR = B <= 64 ? 16 : B <= 128 ? 32 : 64, MS = B <= 128 ? 16 : 32;
  const int grid = std::max(std::max((B / MR) * NUS, (B / 16) * NC2), (B / MS) * NR);
  // every workgroup must be resident: all CUs of an unmasked stream
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    dr_set_error("pscan: device query");
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
    dr_set_error("pscan: grid %d > %d CUs of the stream", grid, avail);
    return DR_E_UNSUPPORTED;
  }
  char* base = reinterpret_cast<char*>(ring);
  PScanArgs a;
  memset(&a, 0, sizeof(a));
  a.B = B; a.T = T; a.A = A; a.step0 = step0;
  a.wt = wt; a.b_ih = wm->b_ih; a.b_hh = wm->b_hh;
  a.whh = wm->w_hh;
  a.wm0 = m0h;
  a.ldm0 = ldm0;
  a.wm3 = wm->map3.w;
  a.ln_g = wm->map1.w; a.ln_b = wm->map1.b; a.b3 = wm->map3.b;
  a.feat = feat; a.act = actions; a.act_sb = act_sb; a.act_st = act_st;
  a.noise = noise;
  a.unimix = (float)(0.01 * (1.0 / d->cols));
  a.spin_limit = ps_spin_limit("scan");
  a.z_out = z_out; a.h_out = h_out; a.logits_out = logits_out;
  a.pz.p[0] = z_out; a.pz.n[0] = (unsigned long long)B * LAT;
  a.pz.p[1] = h_out; a.pz.n[1] = (unsigned long long)B * HD;
  a.pz.p[2] = logits_out; a.pz.n[2] = logits_out ? (unsigned long long)B * LAT : 0ull;
  a.pz.fault = d->fault;
  a.pz.fault_host = d->fault_host;
  a.hb = reinterpret_cast<float*>(base);
  a.pre = a.hb + (size_t)2 * B * HD;
  a.iz = reinterpret_cast<int*>(a.pre + (size_t)2 * B * EH);
  a.cnt = reinterpret_cast<unsigned*>(a.iz + (size_t)4 * B * NR);
  a.zg = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(a.cnt) + PSCAN_CNT_BYTES);
  a.ts = reinterpret_cast<long long*>(a.zg + (size_t)B * NR);
  // counters zeroed by a kernel (captured graphs replay it; a memset node was seen not to)
  // counters and granule tags zeroed by a kernel (captured graphs replay it; a
  // memset node was seen not to): no granule of an earlier launch carries a
  // tag this launch waits for
  DR_TRY(op_fill(PSCAN_CNT_BYTES / 4 + (long long)2 * B * NR, reinterpret_cast<float*>(a.cnt), 0.f, s));
  const bool bf = d->precision == DR_PREC_BF16;
#define PS_L(NT, MRv, MSv) \
  if (MR == MRv && MS == MSv) return launch_pscan<NT, MRv, MSv>(a, grid, s);
  if (bf) {
    PS_L(1, 16, 16) PS_L(1, 32, 16) PS_L(1, 64, 32)
  } else {
    PS_L(3, 16, 16) PS_L(3, 32, 16) PS_L(3, 64, 32)
  }
#undef PS_L
  dr_set_error("pscan: no instance");
  return DR_E_INVALID;
}
