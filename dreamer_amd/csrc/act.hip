// Batch-1 acting step in ONE launch: the per-env-step
// device work of Dreamer.rollout_policy / evaluate_agent / Run
// (Dreamer.py:177-226, 295-322, 374-401):
//
//   h' = GRU(z, h, a)               WorldModel.observe_step -> SequenceModel   (skipped at an
//                                   episode start, where h' = h = 0, Dreamer.py:186-187, 222)
//   z' = Encoder.encode(h', frame)  conv x4 + latent_mapper + categorical sampler (VAE.py:57-99)
//   a  = Actor.act(h', z')          Agent.py:202-210
//
// At batch 1 every stage is a handful of dot products, so the unfused path
// (about 20 launches per env step) is launch- and dependency-latency bound.
// Here one cooperative grid of ACT_NB workgroups walks the stages with a grid
// barrier between dependent ones; inside a stage a wave owns one output row
// (dense) or one output channel of a 2-row pixel block (conv), holds that
// row's weights in registers (loads issued together: one round trip), reads
// the stage input from LDS and reduces with DPP.  f32 VALU arithmetic (no
// MFMA: at batch 1 no weight fragment has more than 16 rows to serve).
//
// Barrier: one monotonic arrival counter per launch (zeroed by the host before
// the launch); round k is complete when it reaches k * ACT_NB.  Polling uses
// agent-scope acquire loads; a bounded spin turns a lost workgroup into NaN
// outputs instead of a hung GPU.
#include "common.h"
#include "ops.h"

#include <string.h>

#define ACT_NB 128
#define ACT_NT 256
#define ACT_SPIN_LIMIT (1 << 22)
#define ACT_BAR_BYTES (4 * 32 * 17)  // 8 group counters, the top counter, 8 generations (128 B apart)
#define ACT_LDS 6400  // floats of dynamic LDS (25 KB): conv input slabs, GRU / projection inputs

struct alignas(16) ActArgs {
  dr_dims d;
  dr_world_model wm;
  dr_actor ac;
  const unsigned char* frame;  // [H][W][3] u8 (env observation layout)
  int has_prev, det;
  const float *z_prev, *h, *a_prev;
  dr_noise noise;
  float *z_out, *h_out, *a_out, *mu_out, *sig_out, *logits_out;
  int* status;  // caller's status word (may be NULL): set to 1 if a grid barrier timed out
  // workspace
  unsigned* bar;
  float *c1, *c2, *c3, *c4, *gi, *gh, *hn, *pre1, *prea;
  int* fail;
  int spin_limit;  // polls before a grid barrier gives up (ACT_SPIN_LIMIT; 0 under DREAMER_ACT_FORCE=timeout)
  long long* ts;  // workgroup 0's stage timestamps (100 MHz wall clock), for profiling
};

// XCD-hierarchical grid barrier (MI355X_MICROARCH.md "barrier-xcd"): the
// workgroups of group x = blockIdx % 8 (the XCD the dispatcher deals them to;
// placement only affects speed) count on their own line; the last arriver of a
// group carries the group to the top counter and, once all 8 groups arrived,
// publishes the round on the group's generation line, which the other members
// poll.  Arrivals are agent-scope releases, every exit an agent-scope acquire.
// bar: [0..8) group counters, [16] top counter, [32..40) generations (128-B apart).
#define ACT_GROUPS 8
__device__ __forceinline__ bool act_sync(unsigned* bar, unsigned& round, int* s_ok, int spin_limit) {
  __syncthreads();
  if (threadIdx.x == 0) {
    ++round;
    const int x = blockIdx.x % ACT_GROUPS;
    const unsigned per = ACT_NB / ACT_GROUPS;
    unsigned* cnt = bar + 32 * x;
    unsigned* top = bar + 32 * ACT_GROUPS;
    unsigned* gen = bar + 32 * (ACT_GROUPS + 1 + x);
    int ok = 1, spins = 0;
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == round * per) {  // group leader
      __hip_atomic_fetch_add(top, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      while (__hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < round * ACT_GROUPS) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > spin_limit) {
          ok = 0;
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(gen, round, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < round) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > spin_limit) {
          ok = 0;
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}
#define ACT_TS(a, i)                                                        \
  do {                                                                      \
    if (blockIdx.x == 0 && threadIdx.x == 0) (a).ts[i] = wall_clock64();    \
  } while (0)

// Stage helpers.  Work is split into wave tasks over the whole grid (ACT_NB x
// 4 waves); a task issues every global load it needs before its first FMA,
// so it pays one memory round trip, and reads its stage input from LDS (each
// workgroup stages the input map / vector it needs).

// k4 s2 p1 conv + bias + SiLU.  Workgroup b owns a block of 2 output rows
// (pb = b % NPB) and 4 output channels (one per wave): it stages the 6 input
// rows the block reads into LDS (NHWC, channel stride cin + 1: the pad breaks
// the stride-2 bank aliasing; rows outside the map are zero padding), each
// wave holds its channel's weight row [ci][ky][kx] in registers (k = lane +
// 64 j: coalesced, all issued before the first FMA), then every pixel is one
// LDS gather + FMA per k and a wave reduction.  cout == 4 * ACT_NB / NPB.
// FRAME: the input is the u8 HWC frame, normalised x/255 - 0.5 (Dreamer.py:251).
template <int KJ, bool FRAME, bool NCHW>
__device__ __forceinline__ void act_conv(int ih, int iw, int cin, int cout, const float* in, const unsigned char* frame,
                         const float* __restrict__ w, const float* __restrict__ b, float* out, float* xs) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int oh = ih / 2, ow = iw / 2, K = cin * 16, cs = cin + 1;
  const int npb = oh / 2, pb = blockIdx.x % npb, co = (blockIdx.x / npb) * 4 + wave;
  const int y0 = 4 * pb - 1;
  // weights first: their latency overlaps the staging
  float wv[KJ];
#pragma unroll
  for (int j = 0; j < KJ; ++j) {
    const int k = lane + 64 * j;
    wv[j] = (k < K && co < cout) ? w[(long long)co * K + k] : 0.f;
  }
  const float bias = co < cout ? b[co] : 0.f;
  const int n = 6 * iw * cin;
  if (FRAME) {
    for (int i = threadIdx.x; i < n; i += ACT_NT) {
      const int r = i / (iw * cin), rem = i - r * iw * cin, y = y0 + r;
      const int px = rem / cin, ch = rem - px * cin;
      xs[(r * iw + px) * cs + ch] = (y >= 0 && y < ih) ? (float)frame[(y * iw) * cin + rem] / 255.0f - 0.5f : 0.f;
    }
  } else {
    // 6 float4 per thread at the CarRacing widths (6 x iw x cin = 6144 floats)
    constexpr int U = 8;
    const int n4 = n / 4;
    for (int i0 = threadIdx.x; i0 < n4; i0 += U * ACT_NT) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i4 = i0 + u * ACT_NT, e = 4 * i4;
        const int r = e / (iw * cin), y = y0 + r;
        v[u] = (i4 < n4 && y >= 0 && y < ih) ? *reinterpret_cast<const float4*>(in + (long long)y0 * iw * cin + e)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i4 = i0 + u * ACT_NT, e = 4 * i4;
        if (i4 >= n4) break;
        const int r = e / (iw * cin), rem = e - r * iw * cin, px = rem / cin, ch = rem - px * cin;
        float* dst = xs + (r * iw + px) * cs + ch;
        dst[0] = v[u].x; dst[1] = v[u].y; dst[2] = v[u].z; dst[3] = v[u].w;
      }
    }
  }
  __syncthreads();
  if (co < cout) {
    for (int pl = 0; pl < 2 * ow; ++pl) {
      const int oy = 2 * pb + pl / ow, ox = pl % ow;
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < KJ; ++j) {
        const int k = lane + 64 * j, ci = k >> 4, ky = (k >> 2) & 3, kx = k & 3;
        const int yl = 2 * oy - 1 + ky - y0, x = 2 * ox - 1 + kx;
        const bool ok = k < K && x >= 0 && x < iw;
        acc = fmaf(wv[j], ok ? xs[(yl * iw + x) * cs + ci] : 0.f, acc);
      }
      acc = wave_sum(acc);
      if (lane == 0) {
        const float v = acc + bias;
        const int p = oy * ow + ox;
        out[NCHW ? co * oh * ow + p : p * cout + co] = v / (1.0f + expf(-v));
      }
    }
  }
}

// y[o] = b[o] + W[o][0:K] . x for x in LDS: one wave task per output row,
// k = lane + 64 j (coalesced row reads, KJ loads in flight per batch)
template <int KJ>
__device__ __forceinline__ void act_dense(int nout, int K, const float* __restrict__ W, long long ldw, const float* __restrict__ b,
                          const float* xs, float* y, int gw, int nw) {
  const int lane = threadIdx.x & 63;
  for (int o = gw; o < nout; o += nw) {
    const float* wr = W + (long long)o * ldw;
    float acc = 0.f;
    for (int k0 = 0; k0 < K; k0 += 64 * KJ) {
      float wv[KJ];
#pragma unroll
      for (int j = 0; j < KJ; ++j) {
        const int k = k0 + lane + 64 * j;
        wv[j] = k < K ? wr[k] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < KJ; ++j) {
        const int k = k0 + lane + 64 * j;
        acc = fmaf(wv[j], k < K ? xs[k] : 0.f, acc);
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) y[o] = acc + (b ? b[o] : 0.f);
  }
}

// dst[i] = src(i) for i < n, every load of a thread issued before its first
// LDS store (one memory round trip per U * ACT_NT elements)
template <int U, typename Src>
__device__ __forceinline__ void act_stage(float* dst, int n, Src src) {
  for (int i0 = threadIdx.x; i0 < n; i0 += U * ACT_NT) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * ACT_NT;
      v[u] = i < n ? src(i) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * ACT_NT;
      if (i < n) dst[i] = v[u];
    }
  }
}

// SiLU(LayerNorm(x)) of an n-vector (n <= 256) by one wave, x read once into
// registers (torch LayerNorm, eps 1e-5); result into dst (LDS)
__device__ __forceinline__ void act_ln_silu(const float* x, int n, const float* g, const float* bb, float* dst) {
  const int lane = threadIdx.x & 63;
  float xv[4], gv[4], bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = lane + 64 * j;
    xv[j] = i < n ? x[i] : 0.f;
    gv[j] = i < n ? g[i] : 0.f;
    bv[j] = i < n ? bb[i] : 0.f;
  }
  const float mean = wave_sum((xv[0] + xv[1]) + (xv[2] + xv[3])) / (float)n;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float dx = lane + 64 * j < n ? xv[j] - mean : 0.f;
    q += dx * dx;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)n + 1e-5f);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = lane + 64 * j;
    if (i < n) {
      const float v = (xv[j] - mean) * rstd * gv[j] + bv[j];
      dst[i] = v / (1.0f + expf(-v));
    }
  }
}

// one output per thread (n <= ACT_NT rows, K % 4 == 0): y[t] = b[t] + W[t] . x,
// the thread's weight row loaded KQ float4 at a time (one round trip per
// 4 KQ weights), x broadcast from LDS
template <int KQ>
__device__ __forceinline__ void act_rows(int n, int K, const float* __restrict__ W, const float* __restrict__ b, const float* xs,
                         float* y) {
  const int t = threadIdx.x;
  if (t >= n) return;
  const float4* wr = reinterpret_cast<const float4*>(W + (long long)t * K);
  float acc = 0.f;
  for (int j0 = 0; 4 * j0 < K; j0 += KQ) {
    float4 w4[KQ];
#pragma unroll
    for (int j = 0; j < KQ; ++j) w4[j] = 4 * (j0 + j) < K ? wr[j0 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < KQ; ++j) {
      const int k = min(4 * (j0 + j), K - 4);  // past K: w4 is zero, any in-range x
      acc = fmaf(w4[j].x, xs[k], acc);
      acc = fmaf(w4[j].y, xs[k + 1], acc);
      acc = fmaf(w4[j].z, xs[k + 2], acc);
      acc = fmaf(w4[j].w, xs[k + 3], acc);
    }
  }
  y[t] = acc + b[t];
}

__global__ __launch_bounds__(ACT_NT) void k_act_step(ActArgs ga) {
  __shared__ ActArgs a;
  __shared__ int s_ok;
  // stage inputs: the largest is conv2's input map, 32 x 32 pixels x 32 channels at a
  // channel stride of 33 (ACT_LDS floats)
  extern __shared__ __attribute__((aligned(16))) float xs[];
  if (threadIdx.x < sizeof(ActArgs) / 16)
    reinterpret_cast<int4*>(&a)[threadIdx.x] = reinterpret_cast<const int4*>(&ga)[threadIdx.x];
  __syncthreads();
  const dr_dims& d = a.d;
  const int gw = blockIdx.x * (ACT_NT / 64) + (threadIdx.x >> 6), nw = ACT_NB * (ACT_NT / 64);
  const int Hd = d.hidden, R = d.rows, C = d.cols, L = R * C, A = d.action;
  const int c1 = d.enc_f1, c2 = d.enc_f2, c3 = 2 * c2, c4 = 4 * c2;
  const int H0 = d.img_h, W0 = d.img_w, F = c4 * (H0 / 16) * (W0 / 16);
  unsigned round = 0;
  bool ok = true;
  ACT_TS(a, 0);

  // ---- stage 1: GRU pre-activations gi = W_ih [z; a] + b, gh = W_hh h + b  ||  conv1 from the frame ----
  const int off = 2048;  // conv slabs use xs[0, 6 * 64 * 4)
  if (a.has_prev) {
    act_stage<5>(xs + off, L + A, [&](int i) { return i < L ? a.z_prev[i] : a.a_prev[i - L]; });
    act_stage<3>(xs + off + 2048, Hd, [&](int i) { return a.h[i]; });
    __syncthreads();
    act_dense<17>(3 * Hd, L + A, a.wm.w_ih, L + A, a.wm.b_ih, xs + off, a.gi, gw, nw);
    act_dense<10>(3 * Hd, Hd, a.wm.w_hh, Hd, a.wm.b_hh, xs + off + 2048, a.gh, gw, nw);
  }
  act_conv<1, true, false>(H0, W0, 3, c1, nullptr, a.frame, a.wm.conv[0].w, a.wm.conv[0].b, a.c1, xs);
  ok = act_sync(a.bar, round, &s_ok, a.spin_limit);
  ACT_TS(a, 1);
  // ---- stage 2: conv2  ||  GRU gates (torch gru_cell order r, z, n) ----
  if (ok) {
    const int gt = blockIdx.x * ACT_NT + threadIdx.x;
    for (int j = gt; j < Hd; j += ACT_NB * ACT_NT) {
      const float hv = a.h[j];
      float hn = hv;
      if (a.has_prev) {
        const float rr = 1.0f / (1.0f + expf(-(a.gh[j] + a.gi[j])));
        const float uu = 1.0f / (1.0f + expf(-(a.gh[Hd + j] + a.gi[Hd + j])));
        const float nn = tanhf(a.gi[2 * Hd + j] + a.gh[2 * Hd + j] * rr);
        hn = (hv - nn) * uu + nn;
      }
      a.hn[j] = hn;
      a.h_out[j] = hn;
    }
    act_conv<8, false, false>(H0 / 2, W0 / 2, c1, c2, a.c1, nullptr, a.wm.conv[1].w, a.wm.conv[1].b, a.c2, xs);
  }
  if (ok) ok = act_sync(a.bar, round, &s_ok, a.spin_limit);
  ACT_TS(a, 2);
  if (ok) act_conv<16, false, false>(H0 / 4, W0 / 4, c2, c3, a.c2, nullptr, a.wm.conv[2].w, a.wm.conv[2].b, a.c3, xs);
  if (ok) ok = act_sync(a.bar, round, &s_ok, a.spin_limit);
  ACT_TS(a, 3);
  if (ok) act_conv<32, false, true>(H0 / 8, W0 / 8, c3, c4, a.c3, nullptr, a.wm.conv[3].w, a.wm.conv[3].b, a.c4, xs);
  if (ok) ok = act_sync(a.bar, round, &s_ok, a.spin_limit);
  ACT_TS(a, 4);
  // ---- stage 5: latent_mapper.0 on cat(features, h') (VAE.py:73) ----
  if (ok) {
    act_stage<19>(xs, F + Hd, [&](int i) { return i < F ? a.c4[i] : a.hn[i - F]; });
    __syncthreads();
    act_dense<25>(d.enc_hidden, F + Hd, a.wm.map0.w, F + Hd, a.wm.map0.b, xs, a.pre1, gw, nw);
  }
  if (ok) ok = act_sync(a.bar, round, &s_ok, a.spin_limit);
  ACT_TS(a, 5);
  // ---- stage 6: LN-SiLU, latent_mapper.3 and the categorical sampler: one wave per latent group ----
  if (ok && gw < R) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float* x1 = xs + wave * 256;
    float* lgs = xs + 1024 + wave * 64;
    act_ln_silu(a.pre1, d.enc_hidden, a.wm.map1.w, a.wm.map1.b, x1);
    const int grp = gw;
    // the group's C logits: the weights (k = lane + 64 j) of 16 rows per batch
    float xv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) xv[j] = lane + 64 * j < d.enc_hidden ? x1[lane + 64 * j] : 0.f;
    float mylg = 0.f;
    for (int u0 = 0; u0 < C; u0 += 16) {
      float wv[16][4];
#pragma unroll
      for (int u = 0; u < 16; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = lane + 64 * j;
          wv[u][j] = (u0 + u < C && k < d.enc_hidden)
                         ? a.wm.map3.w[(long long)(grp * C + u0 + u) * d.enc_hidden + k] : 0.f;
        }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = fmaf(wv[u][j], xv[j], acc);
        acc = wave_sum(acc);
        if (lane == u0 + u) mylg = acc;
      }
    }
    if (lane < C) lgs[lane] = mylg + a.wm.map3.b[grp * C + lane];
    const bool act = lane < C;
    const float lg = act ? lgs[lane] : -INFINITY;
    if (act && a.logits_out) a.logits_out[grp * C + lane] = lg;
    // softmax, 1% unimix, argmax(p_hat / Exp(1)), straight-through one-hot (VAE.py:88-98)
    const float mx = wave_max(lg);
    const float ex = act ? expf(lg - mx) : 0.f;
    const float se = wave_sum(ex);
    const float p = ex / se;
    const float pu = act ? 0.99f * p + (float)(0.01 * (1.0 / C)) : 0.f;
    const float sp = wave_sum(pu);
    const float ph = pu / sp;
    float qv = 1.0f;
    if (act) {
      if (a.noise.q) qv = a.noise.q[(long long)grp * C + lane];
      else qv = dr_exp1(a.noise.rng, (uint32_t)a.noise.stream, (uint32_t)a.noise.row0, (uint32_t)(grp * C + lane));
    }
    float best = act ? ph / qv : -INFINITY;
    int bi = act ? lane : 0x7fffffff;
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) {
        best = ob;
        bi = oi;
      }
    }
    if (act) a.z_out[grp * C + lane] = (lane == bi) ? ((1.0f + pu) - pu) : 0.0f;
  }
  if (ok) ok = act_sync(a.bar, round, &s_ok, a.spin_limit);
  ACT_TS(a, 6);
  // ---- stage 7: actor base_net.0 on cat(h', z') (Agent.py:191-200) ----
  if (ok) {
    act_stage<7>(xs, Hd + L, [&](int i) { return i < Hd ? a.hn[i] : a.z_out[i - Hd]; });
    __syncthreads();
    act_dense<26>(d.actor_h1, Hd + L, a.ac.l0.w, Hd + L, a.ac.l0.b, xs, a.prea, gw, nw);
  }
  if (ok) ok = act_sync(a.bar, round, &s_ok, a.spin_limit);
  ACT_TS(a, 7);
  // A barrier that timed out (a workgroup never arrived: the grid was not
  // co-resident) is reported, never silent: every workgroup that saw it raises
  // the status word the host checks after the step, and writes NaN to every
  // output (action, mu, sigma, z', h') so nothing downstream can mistake them
  // for a state.
  // Workgroup 0 also re-reads the shared fail flag after the last barrier: a
  // workgroup that timed out there raised it after arriving (its stage data is
  // complete), but the outputs are poisoned all the same.  `status` stays the
  // authoritative signal (a flag raised after this read is seen only there).
  if (blockIdx.x == 0) {  // (uniform over the workgroup: every wave takes both barriers)
    __shared__ int s_fail;
    if (threadIdx.x == 0) s_fail = __hip_atomic_load(a.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (s_fail) ok = false;
  }
  if (!ok) {
    if (threadIdx.x == 0) {
      __hip_atomic_store(a.fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (a.status) __hip_atomic_store(a.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // every failing workgroup poisons every output after its own writes: a
    // workgroup that got past the barrier workgroup 0 gave up on still writes
    // its h' / z' slice (a forced-timeout run caught workgroup 0's NaN being
    // overwritten that way), but it cannot pass the next barrier (workgroup 0
    // never arrives), so it fails too and poisons after its writes
    const float qnan = __int_as_float(0x7fc00000);
    for (int i = threadIdx.x; i < A; i += ACT_NT) a.a_out[i] = a.mu_out[i] = a.sig_out[i] = qnan;
    for (int i = threadIdx.x; i < L; i += ACT_NT) a.z_out[i] = qnan;
    for (int i = threadIdx.x; i < Hd; i += ACT_NT) a.h_out[i] = qnan;
    return;
  }
  // ---- stage 8 (workgroup 0): LN-SiLU, base_net.3, LN-SiLU, mu / log_sigma heads, tanh(mu + eps sigma) ----
  if (blockIdx.x != 0) return;
  const int wave = threadIdx.x >> 6;
  const int a1 = d.actor_h1, a2 = d.actor_h2;
  float* x1 = xs;          // SiLU(LN(pre1))
  float* p2 = xs + 1024;   // base_net.3 output
  float* x2 = xs + 2048;   // SiLU(LN(p2))
  if (wave == 0) act_ln_silu(a.prea, a1, a.ac.n1.w, a.ac.n1.b, x1);
  __syncthreads();
  act_rows<25>(a2, a1, a.ac.l3.w, a.ac.l3.b, x1, p2);
  __syncthreads();
  if (wave == 0) act_ln_silu(p2, a2, a.ac.n4.w, a.ac.n4.b, x2);
  __syncthreads();
  float* hd = xs + 3072;  // [mu (A) | log_sigma (A)]
  for (int o = wave; o < 2 * A; o += ACT_NT / 64) {
    const int lane = threadIdx.x & 63;
    const float* hw = o < A ? a.ac.mu.w : a.ac.ls.w;
    const float* hb = o < A ? a.ac.mu.b : a.ac.ls.b;
    const int oo = o < A ? o : o - A;
    float wv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wv[j] = lane + 64 * j < a2 ? hw[(long long)oo * a2 + lane + 64 * j] : 0.f;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = fmaf(wv[j], lane + 64 * j < a2 ? x2[lane + 64 * j] : 0.f, acc);
    acc = wave_sum(acc);
    if (lane == 0) hd[o] = acc + hb[oo];
  }
  __syncthreads();
  if (threadIdx.x < A) {
    const int i = threadIdx.x;
    const float muv = hd[i];
    const float ls = fminf(fmaxf(hd[A + i], -5.0f), 2.0f);
    const float sg = dr_softplus(ls) + 1e-3f;
    float av;
    if (a.det) {
      av = tanhf(muv);
    } else {
      float e;
      if (a.noise.eps) e = a.noise.eps[i];
      else e = dr_normal(a.noise.rng, (uint32_t)(a.noise.stream + 1), (uint32_t)a.noise.row0, (uint32_t)i);
      av = tanhf(muv + e * sg);
    }
    a.a_out[i] = av;
    a.mu_out[i] = muv;
    a.sig_out[i] = sg;
  }
  ACT_TS(a, 15);
}

static void act_carve(char* base, const dr_dims* d, ActArgs& a, size_t& off) {
  auto take = [&](size_t bytes) {
    const size_t o = (off + 255) & ~(size_t)255;
    off = o + bytes;
    return base ? base + o : nullptr;
  };
  const int c1 = d->enc_f1, c2 = d->enc_f2;
  const long long p1 = (long long)(d->img_h / 2) * (d->img_w / 2);
  a.ts = (long long*)take(16 * sizeof(long long));  // first: tools read it at offset 0
  a.bar = (unsigned*)take(ACT_BAR_BYTES);
  a.fail = (int*)take(256);
  a.c1 = (float*)take(4 * p1 * c1);
  a.c2 = (float*)take(4 * (p1 / 4) * c2);
  a.c3 = (float*)take(4 * (p1 / 16) * 2 * c2);
  a.c4 = (float*)take(4 * (p1 / 64) * 4 * c2);
  a.gi = (float*)take(4 * 3 * d->hidden);
  a.gh = (float*)take(4 * 3 * d->hidden);
  a.hn = (float*)take(4 * d->hidden);
  a.pre1 = (float*)take(4 * d->enc_hidden);
  a.prea = (float*)take(4 * d->actor_h1);
}

extern "C" size_t dr_act_step_workspace_bytes(const dr_dims* d) {
  ActArgs a;
  size_t off = 0;
  act_carve(nullptr, d, a, off);
  return off;
}

extern "C" int dr_act_step(const dr_dims* d, const dr_world_model* wm, const dr_actor* ac, const unsigned char* frame,
                           int has_prev, const float* z_prev, const float* h, const float* a_prev, dr_noise noise,
                           int deterministic, float* z_out, float* h_out, float* a_out, float* mu_out,
                           float* sigma_out, float* logits_out, int* status, void* ws, size_t ws_bytes,
                           hipStream_t s) {
  DR_REQUIRE(d && wm && ac && frame && h && z_out && h_out && a_out && mu_out && sigma_out && ws, "null argument");
  DR_REQUIRE(!has_prev || (z_prev && a_prev), "has_prev needs z_prev and a_prev");
  DR_REQUIRE(d->obs_dim == 0, "dr_act_step: pixel observations only (vector observations use the unfused path)");
  const int F = 4 * d->enc_f2 * (d->img_h / 16) * (d->img_w / 16), L = d->rows * d->cols;
  // the stage helpers' register batches (KJ) and the LDS staging are sized for the
  // CarRacing encoder (Dreamer.py:20-64 config); other shapes use the unfused calls
  if (!((d->enc_depth == 0 || d->enc_depth == 4) && d->img_h == 64 && d->img_w == 64 && d->enc_f1 == 32 &&
        d->enc_f2 == 64 && F + d->hidden <= 64 * 74 && L + d->action <= 64 * 17 && d->hidden <= 64 * 10 &&
        d->hidden + L <= 64 * 26 && d->cols <= 64 && d->rows <= ACT_NB * (ACT_NT / 64) && d->enc_hidden <= 256 &&
        d->actor_h1 <= 256 && d->actor_h2 <= 1024 && d->action <= 64)) {
    dr_set_error("dr_act_step: dims outside the batch-1 acting kernel (64x64 frames, encoder 32/64 filters, widths "
                 "<= the staging)");
    return DR_E_UNSUPPORTED;
  }
  const char* force = getenv("DREAMER_ACT_FORCE");  // test hook (include/dreamer_hip.h)
  const bool force_timeout = force && strcmp(force, "timeout") == 0;
  const bool force_nonres = force && strcmp(force, "nonresident") == 0;
  ActArgs a;
  memset(&a, 0, sizeof(a));
  a.d = *d;
  a.wm = *wm;
  a.ac = *ac;
  a.frame = frame;
  a.has_prev = has_prev;
  a.det = deterministic;
  a.z_prev = z_prev;
  a.h = h;
  a.a_prev = a_prev;
  a.noise = noise;
  a.z_out = z_out;
  a.h_out = h_out;
  a.a_out = a_out;
  a.mu_out = mu_out;
  a.sig_out = sigma_out;
  a.logits_out = logits_out;
  a.status = status;
  size_t off = 0;
  act_carve((char*)ws, d, a, off);
  DR_REQUIRE(off <= ws_bytes, "workspace too small");
  // barrier lines + fail flag (a kernel, so a captured graph re-arms them too)
  static_assert((ACT_BAR_BYTES + 512) % 4 == 0, "barrier bytes");
  DR_TRY(op_fill((ACT_BAR_BYTES + 512) / 4, reinterpret_cast<float*>(a.bar), 0.f, s));
  // A plain launch whose grid barrier needs all ACT_NB workgroups resident at
  // once.  The cooperative launch would add exactly that check at +15-19 us of
  // host time per env step (MI355X_MICROARCH.md coop-launch), so it is made
  // once per device here instead: the occupancy API's blocks per CU (one lower
  // than reported, the guide's sgpr-count margin) times the CU count must
  // cover the grid, else the call fails and the caller runs the unfused path.
  // What no launch-time check can cover -- other work holding CUs for longer
  // than the bounded spin -- comes back through `status` (and NaN outputs).
  static int resident_ok[64];  // per device: 0 unknown, 1 ok, -1 too small (idempotent, benign race)
  int dev = 0;
  DR_TRY_HIP(hipGetDevice(&dev));
  DR_REQUIRE(dev >= 0 && dev < 64, "device index");
  if (resident_ok[dev] == 0) {
    (void)hipFuncSetAttribute((const void*)k_act_step, hipFuncAttributeMaxDynamicSharedMemorySize, ACT_LDS * 4);
    int per_cu = 0, cus = 0;
    DR_TRY_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_act_step, ACT_NT, ACT_LDS * 4));
    DR_TRY_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    resident_ok[dev] = (long long)(per_cu - 1 > 0 ? per_cu - 1 : per_cu) * cus >= ACT_NB ? 1 : -1;
  }
  if (resident_ok[dev] != 1 || force_nonres) {
    dr_set_error("dr_act_step: the device cannot hold the acting grid co-resident");
    return DR_E_UNSUPPORTED;
  }
  a.spin_limit = force_timeout ? 0 : ACT_SPIN_LIMIT;
  hipLaunchKernelGGL(k_act_step, dim3(ACT_NB), dim3(ACT_NT), ACT_LDS * 4, s, a);
  return dr_check_launch("act_step");
}
