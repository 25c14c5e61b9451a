// Kernel latency microbenchmark: links the engine's objects and times single
// kernels launched back to back on one stream (HIP events around REPS
// launches).  Build: python tools/kbench/build.py ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <functional>
#include "../../dreamer_amd/csrc/gemm.h"
#include "../../dreamer_amd/csrc/gru.h"
#include "../../dreamer_amd/csrc/ops.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static const char* g_filter = nullptr;
static int g_reps = 200;
extern "C" int dr_debug_tbuf_gru(long long* out, int n);
extern "C" int dr_debug_tbuf_gemm(long long* out, int n);
extern "C" void dr_debug_tile_variant(int v);
extern "C" void dr_debug_skinny_variant(int v);
extern "C" void dr_debug_tile_wgs(int v);
extern "C" void dr_debug_gates_batch(int v);
extern "C" void dr_debug_ln_sample_off(int v);

// one more launch, then the per-phase times of wave 0 of each workgroup
// (relative to its own start) averaged over the workgroups that wrote them
static void phases(const char* name, std::function<void(hipStream_t)> f, int (*rd)(long long*, int), hipStream_t s) {
  if (g_filter && !strstr(name, g_filter)) return;
  const int n = 1024 * DR_TS_SLOTS;
  std::vector<long long> z(n, 0), t(n);
  hipStreamSynchronize(s);
  rd(t.data(), n);  // clears stale stamps
  f(s);
  hipStreamSynchronize(s);
  rd(t.data(), n);
  double sum[DR_TS_SLOTS] = {0};
  int cnt[DR_TS_SLOTS] = {0};
  long long smin = -1, smax = 0, emax = 0;
  for (int b = 0; b < 1024; ++b) {
    const long long* r = &t[b * DR_TS_SLOTS];
    if (r[0] == 0) continue;
    if (smin < 0 || r[0] < smin) smin = r[0];
    if (r[0] > smax) smax = r[0];
    for (int i = 1; i < DR_TS_SLOTS; ++i)
      if (r[i] >= r[0] && r[i] - r[0] < 1000000) {
        sum[i] += r[i] - r[0];
        cnt[i]++;
        if (r[i] > emax) emax = r[i];
      }
  }
  printf("   phases %-38s start spread %.2f us, last stamp %.2f us after first start |", name, (smax - smin) * 0.01,
         (emax - smin) * 0.01);
  for (int i = 1; i < DR_TS_SLOTS; ++i)
    if (cnt[i]) printf(" p%d %.2f", i, sum[i] / cnt[i] * 0.01);
  printf("\n");
}

// I-cache probe: the same 4096 independent FMAs as straight-line code or as a loop
__global__ __launch_bounds__(512) void k_code_unrolled(float* out, float x) {
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = x + i;
#pragma unroll
  for (int it = 0; it < 512; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = a[i] * 0.999f + 0.001f * (float)(it + i);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a[i];
  if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(512) void k_code_rolled(float* out, float x) {
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = x + i;
#pragma unroll 1
  for (int it = 0; it < 512; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = a[i] * 0.999f + 0.001f * (float)(it + i);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a[i];
  if (s == 12345.f) out[threadIdx.x] = s;
}

// dependent-load chain: per-round-trip latency with the whole grid loading
__global__ __launch_bounds__(512) void k_chase(const unsigned* __restrict__ nxt, int rounds, unsigned* out) {
  unsigned i = (blockIdx.x * 512 + threadIdx.x) * 97u & ((1u << 18) - 1);
  for (int r = 0; r < rounds; ++r) i = nxt[i];
  if (i == 0xffffffffu) out[0] = i;
}

// busy kernel: each workgroup spins for `iters` dependent FMAs
__global__ __launch_bounds__(256) void k_spin(float* out, int iters) {
  float a = threadIdx.x;
  for (int i = 0; i < iters; ++i) a = a * 0.9999f + 0.5f;
  if (a == 12345.f) out[0] = a;
}

// two independent chains captured on two streams (fork/join) vs one stream
static void concurrency_probe(float* dummy) {
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t fork, join, a, b;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto big = [&](hipStream_t st) { hipLaunchKernelGGL(k_spin, dim3(512), dim3(256), 0, st, dummy, 20000); };
  auto chain = [&](hipStream_t st) {
    for (int i = 0; i < 40; ++i) hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, st, dummy, 1000);
  };
  for (int mode = 0; mode < 4; ++mode) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
    if (mode == 0) {
      big(s1);
    } else if (mode == 1) {
      chain(s1);
    } else if (mode == 2) {
      big(s1);
      chain(s1);
    } else {
      CK(hipEventRecord(fork, s1));
      CK(hipStreamWaitEvent(s2, fork, 0));
      big(s2);
      chain(s1);
      CK(hipEventRecord(join, s2));
      CK(hipStreamWaitEvent(s1, join, 0));
    }
    CK(hipStreamEndCapture(s1, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s1));
    CK(hipStreamSynchronize(s1));
    CK(hipEventRecord(a, s1));
    for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, s1));
    CK(hipEventRecord(b, s1));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const char* nm[] = {"big alone", "chain of 40 alone", "big then chain (1 stream)", "big || chain (fork/join)"};
    printf("graph concurrency: %-28s %8.1f us\n", nm[mode], 1000.f * ms / 5);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
}

// N float4 loads per lane issued back to back, then one reduction + store.
// STRIDED: lanes r = 0..15 read 16 different rows (2400-byte stride), the
// four q-lanes of a row read consecutive 16-byte pieces (the skinny GEMM's
// weight-fragment pattern); otherwise fully coalesced 1 KB per wave load.
template <int N, bool STRIDED>
__global__ __launch_bounds__(512) void k_loads(const float* __restrict__ buf, float* out) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float4 v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    unsigned e;
    if (STRIDED) {
      const int r = lane & 15, q = lane >> 4;
      e = (unsigned)(((blockIdx.x * 16 + r) * 600 + (wave * N + i) * 16 + 4 * q) & ((1 << 22) - 1));
    } else {
      e = (unsigned)(((blockIdx.x * 512 + tid) * 4 + i * 262144) & ((1 << 22) - 1));
    }
    v[i] = dr_ld4(buf, e);
  }
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < N; ++i) acc += v[i].x + v[i].y + v[i].z + v[i].w;
  if (acc == 1234.5f) out[0] = acc;
}

// MFMA issue rate: each wave runs `iters` x 8 independent f32 16x16x4 MFMAs
// (register operands only); 256 workgroups x 256 threads = one wave per SIMD
__global__ __launch_bounds__(256) void k_mfma_rate(float* out, int iters) {
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float a = threadIdx.x * 1e-3f, b = 1.0f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ void k_clock(long long* out, int spin) {
  const long long t0 = wall_clock64(), c0 = clock64();
  float a = 1.f;
  for (int i = 0; i < spin; ++i) a = a * 0.9999f + 0.5f;
  const long long t1 = wall_clock64(), c1 = clock64();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = c1 - c0; out[2] = (long long)a; }
}

struct Big { long long f[200]; };
__global__ void k_empty_small(int* p) { if (p && threadIdx.x == 9999) *p = 1; }
__global__ void k_empty_big(Big b) { if (threadIdx.x == 9999) ((int*)b.f[3])[0] = (int)b.f[150]; }

static float* frand(size_t n, float scale = 0.1f) {
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = scale * ((rand() / (float)RAND_MAX) - 0.5f);
  float* d;
  CK(hipMalloc(&d, n * sizeof(float)));
  CK(hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return d;
}

static void timeit(const char* name, std::function<void(hipStream_t)> f, hipStream_t s, int reps = 0) {
  if (g_filter && !strstr(name, g_filter)) return;
  if (reps == 0) reps = g_reps;
  for (int i = 0; i < 10; ++i) f(s);
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // graph-captured chain (what the engine replays)
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < reps; ++i) f(s);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(a, s));
  CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("%-48s %8.2f us/launch (graph chain of %d)\n", name, 1000.f * ms / reps, reps);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
}

int main(int argc, char** argv) {
  if (argc > 1) g_filter = argv[1];
  if (getenv("KB_REPS")) g_reps = atoi(getenv("KB_REPS"));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const int B = getenv("KB_B") ? atoi(getenv("KB_B")) : 64, Hd = 600, R = 32, C = 32, A = 3, L = R * C;
  timeit("empty kernel (1 WG, small args)", [&](hipStream_t st) { hipLaunchKernelGGL(k_empty_small, dim3(1), dim3(64), 0, st, nullptr); }, s);
  timeit("empty kernel (128 WG x 512, small args)", [&](hipStream_t st) { hipLaunchKernelGGL(k_empty_small, dim3(128), dim3(512), 0, st, nullptr); }, s);
  Big big;
  memset(&big, 0, sizeof(big));
  timeit("empty kernel (128 WG x 512, 1.6 KB args)", [&](hipStream_t st) { hipLaunchKernelGGL(k_empty_big, dim3(128), dim3(512), 0, st, big); }, s);

  float* dummy;
  CK(hipMalloc(&dummy, 4096));
  timeit("4096 FMA straight-line (128 WG x 512)", [&](hipStream_t st) { hipLaunchKernelGGL(k_code_unrolled, dim3(128), dim3(512), 0, st, dummy, 1.0f); }, s);
  timeit("4096 FMA rolled loop   (128 WG x 512)", [&](hipStream_t st) { hipLaunchKernelGGL(k_code_rolled, dim3(128), dim3(512), 0, st, dummy, 1.0f); }, s);
  timeit("4096 FMA straight-line (1 WG x 64)", [&](hipStream_t st) { hipLaunchKernelGGL(k_code_unrolled, dim3(1), dim3(64), 0, st, dummy, 1.0f); }, s);
  timeit("4096 FMA rolled loop   (1 WG x 64)", [&](hipStream_t st) { hipLaunchKernelGGL(k_code_rolled, dim3(1), dim3(64), 0, st, dummy, 1.0f); }, s);

  {
    const int n = 1 << 18;  // 1 MB of indices
    std::vector<unsigned> h(n);
    for (int i = 0; i < n; ++i) h[i] = (unsigned)((i * 2654435761u + 12345u) & (n - 1));
    unsigned* d;
    CK(hipMalloc(&d, n * 4));
    CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    for (int rounds : {1, 4, 16}) {
      char nm[96];
      snprintf(nm, sizeof nm, "pointer chase %2d rounds (128 WG x 512)", rounds);
      timeit(nm, [&](hipStream_t st) { hipLaunchKernelGGL(k_chase, dim3(128), dim3(512), 0, st, d, rounds, (unsigned*)dummy); }, s);
      snprintf(nm, sizeof nm, "pointer chase %2d rounds (1 WG x 64)", rounds);
      timeit(nm, [&](hipStream_t st) { hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, st, d, rounds, (unsigned*)dummy); }, s);
    }
  }

  if (!g_filter || strstr("concurrency", g_filter)) concurrency_probe(dummy);
  if (!g_filter || strstr("mfma rate", g_filter)) {
    for (int iters : {1000, 4000}) {
      char nm[96];
      snprintf(nm, sizeof nm, "mfma rate: 8 x %d f32 16x16x4 per wave, 256 WG x 4 waves", iters);
      timeit(nm, [&](hipStream_t st) { hipLaunchKernelGGL(k_mfma_rate, dim3(256), dim3(256), 0, st, dummy, iters); }, s, 20);
    }
    long long* ck;
    CK(hipMalloc(&ck, 64));
    hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, s, ck, 2000000);
    long long h[3];
    CK(hipMemcpy(h, ck, 24, hipMemcpyDeviceToHost));
    printf("clock probe: %lld shader cycles in %lld x 10 ns -> %.0f MHz (idle chip, 1 wave)\n", h[1], h[0],
           (double)h[1] / (h[0] * 10e-9) / 1e6);
  }
  {
    float* buf = frand((size_t)1 << 22);
#define KB_LOADS(NN)                                                                                        \
    timeit("loads " #NN " float4/lane coalesced (128 WG x 512)",                                         \
           [&](hipStream_t st) { hipLaunchKernelGGL((k_loads<NN, false>), dim3(128), dim3(512), 0, st, buf, dummy); }, s); \
    timeit("loads " #NN " float4/lane strided   (128 WG x 512)",                                         \
           [&](hipStream_t st) { hipLaunchKernelGGL((k_loads<NN, true>), dim3(128), dim3(512), 0, st, buf, dummy); }, s);
    KB_LOADS(1)
    KB_LOADS(4)
    KB_LOADS(8)
    KB_LOADS(16)
    KB_LOADS(32)
  }

  // GRU
  float* wih = frand((size_t)3 * Hd * (L + A));
  float* wt = frand((size_t)3 * Hd * (L + A));
  float* whh = frand((size_t)3 * Hd * Hd);
  float* bih = frand(3 * Hd);
  float* bhh = frand(3 * Hd);
  float* h = frand((size_t)B * Hd);
  float* hout = frand((size_t)B * Hd);
  float* act = frand((size_t)B * A);
  float* save = frand((size_t)4 * B * Hd);
  std::vector<int> hidx(2 * B * R);
  for (int i = 0; i < B * R; ++i) hidx[i] = rand() % C;
  float one = 1.0f;
  for (int i = 0; i < B * R; ++i) memcpy(&hidx[B * R + i], &one, 4);
  int* idx;
  CK(hipMalloc(&idx, hidx.size() * 4));
  CK(hipMemcpy(idx, hidx.data(), hidx.size() * 4, hipMemcpyHostToDevice));
  if (op_transpose(3 * Hd, L + A, wih, wt, s)) { printf("transpose failed\n"); return 1; }
  GruArgs ga;
  memset(&ga, 0, sizeof(ga));
  ga.B = B; ga.Hd = Hd; ga.R = R; ga.C = C; ga.A = A;
  ga.idx = idx; ga.zval = reinterpret_cast<float*>(idx + B * R); ga.a = act; ga.lda = A; ga.h = h; ga.ldh = Hd;
  ga.wt = wt; ga.b_ih = bih; ga.w_hh = whh; ga.b_hh = bhh; ga.hout = hout; ga.ldo = Hd;
  timeit("gru_fused B64 H600 R32 (no saves)", [&](hipStream_t st) { op_gru_fused(ga, st); }, s);

  phases("gru_fused", [&](hipStream_t st) { op_gru_fused(ga, st); }, dr_debug_tbuf_gru, s);
  GruArgs gs = ga;
  gs.sr = save; gs.su = save + B * Hd; gs.sn = save + 2 * B * Hd; gs.sghn = save + 3 * B * Hd;
  timeit("gru_fused B64 H600 R32 (saves)", [&](hipStream_t st) { op_gru_fused(gs, st); }, s);
  {  // split path (tile-GEMM hidden product + gather/gates kernel) by gather batch
    float* ghw = frand((size_t)B * 3 * Hd);
    for (int gbv : {4, 8, 16, 32}) {
      dr_debug_gates_batch(gbv);
      GruArgs gsp = gs;
      gsp.gh_ws = ghw;
      char nm[96];
      snprintf(nm, sizeof nm, "gru split B%d (saves) gather batch %d", B, gbv);
      timeit(nm, [&](hipStream_t st) { op_gru_fused(gsp, st); }, s);
      GruArgs gz = gsp;
      gz.h = nullptr;  // gates kernel alone (no hidden product)
      snprintf(nm, sizeof nm, "gru split B%d gates only, batch %d", B, gbv);
      timeit(nm, [&](hipStream_t st) { op_gru_fused(gz, st); }, s);
    }
    dr_debug_gates_batch(8);
  }
  GruArgs gn = ga;
  gn.h = nullptr;
  timeit("gru_fused h=NULL (gather only)", [&](hipStream_t st) { op_gru_fused(gn, st); }, s);
  GruArgs g0 = ga;
  g0.R = 0;
  g0.A = 0;
  timeit("gru_fused R=0 A=0 (MFMA only)", [&](hipStream_t st) { op_gru_fused(g0, st); }, s);

  // skinny GEMMs
  float* X = frand((size_t)1024 * 2048);
  float* W = frand((size_t)2048 * 2048);
  float* bias = frand(2048);
  float* Y = frand((size_t)1024 * 2048);
  float* lng = frand(2048, 1.0f);
  float* lnb = frand(2048);
  auto nt_ = [&](int M, int N, int K) {
    GemmArgs g = gemm_args();
    g.M = M; g.N = N; g.K = K; g.A = X; g.lda = K; g.ksplitA = K; g.W = W; g.ldb = K; g.bias = bias; g.Y = Y; g.ldy = N;
    return g;
  };
  char buf[128];
  int shapes[][3] = {{B, 200, 600}, {B, 200, 200}, {B, 1024, 200}, {B, 200, 1624}, {B, 255, 200}, {960, 200, 200},
                     {B, 1027, 1800}, {B, 600, 1800}};
  for (auto& sh : shapes) {
    GemmArgs g = nt_(sh[0], sh[1], sh[2]);
    snprintf(buf, sizeof buf, "NT plain M%d N%d K%d", sh[0], sh[1], sh[2]);
    timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_PLAIN, &g, 1, st); }, s);
    phases(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_PLAIN, &g, 1, st); }, dr_debug_tbuf_gemm, s);
    GemmArgs gl = g;
    gl.ln_g = lng; gl.ln_b = lnb;
    snprintf(buf, sizeof buf, "NT lnsilu M%d N%d K%d", sh[0], sh[1], sh[2]);
    timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_LNSILU, &gl, 1, st); }, s);
    phases(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_LNSILU, &gl, 1, st); }, dr_debug_tbuf_gemm, s);
    GemmArgs gk = g;
    gk.ldb = sh[1];
    snprintf(buf, sizeof buf, "NN plain M%d N%d K%d", sh[0], sh[1], sh[2]);
    timeit(buf, [&](hipStream_t st) { gemm_launch(G_NN, AM_PLAIN, &gk, 1, st); }, s);
  }
  // fused head tail (LN-SiLU, Linear, LN-SiLU, Linear) vs its two launches
  {
    GemmArgs e = nt_(64, 1024, 200);
    e.A = nullptr;
    Mlp2Args a;
    memset(&a, 0, sizeof(a));
    a.M = 64; a.K1 = 200; a.K2 = 200; a.X = X; a.ldx = 200; a.ln1_g = lng; a.ln1_b = lnb; a.W3 = W; a.b3 = bias;
    a.ln4_g = lng; a.ln4_b = lnb; a.pre2 = Y + 300000; a.ld_pre2 = 200; a.e = e;
    timeit("mlp2 tail M64 200-200-1024", [&](hipStream_t st) { mlp2_launch(&a, 1, st); }, s);
    Mlp2Args a3[3] = {a, a, a};
    a3[0].e.N = 255; a3[1].e.N = 1; a3[2].e.N = 6;
    timeit("mlp2 tail x3 M64 200-200-{255,1,6}", [&](hipStream_t st) { mlp2_launch(a3, 3, st); }, s);
    GemmArgs g1 = nt_(64, 200, 200);
    g1.ln_g = lng; g1.ln_b = lnb; g1.Y = Y + 300000;
    GemmArgs g2 = nt_(64, 1024, 200);
    g2.A = Y + 300000; g2.ln_g = lng; g2.ln_b = lnb;
    timeit("unfused 2x lnsilu M64 200-200-1024", [&](hipStream_t st) { gemm_launch(G_NT, AM_LNSILU, &g1, 1, st);
                                                                       gemm_launch(G_NT, AM_LNSILU, &g2, 1, st); }, s);
  }
  // B = 256 chain products: current routing (variant 0) against the 8-wave
  // tile variants, without and with split-K scratch
  {
    float* skw = frand((size_t)8 * 256 * 2048);
    // correctness of the wave-K variants against variant 0 (same inputs, own outputs)
    if (!g_filter || strstr("tv check", g_filter) || strstr(g_filter, "tv")) {
      float* Yc = frand((size_t)3 * B * 2048);
      auto run_shapes = [&](int var, std::vector<float>& out) {
        dr_debug_tile_variant(var);
        CK(hipMemset(Yc, 0, (size_t)3 * B * 2048 * 4));
        GemmArgs a = nt_(B, 1027, 1800), b = nt_(B, 600, 1800);
        a.Y = Yc; a.ldy = 1027; b.Y = Yc + (size_t)B * 1027; b.ldy = 600;
        GemmArgs p2[2] = {a, b};
        gemm_launch(G_NT, AM_PLAIN, p2, 2, s);
        GemmArgs h3[3];
        for (int i = 0; i < 3; ++i) {
          h3[i] = nt_(B, 200, 1624);
          h3[i].A = X; h3[i].lda = 600; h3[i].ksplitA = 600; h3[i].A2 = X + 700000; h3[i].lda2 = 1024;
          h3[i].W = W + 100 * i; h3[i].Y = Yc + (size_t)B * 1627 + (size_t)B * 200 * i; h3[i].ldy = 200;
          h3[i].splitk_ws = skw + (size_t)i * 1024 * 1024; h3[i].splitk_floats = 1024LL * 1024;
        }
        gemm_launch(G_NT, AM_PLAIN, h3, 3, s);
        GemmArgs gg = nt_(B, 1800, 600);
        gg.Y = Yc + (size_t)B * 2227; gg.ldy = 1800;
        gemm_launch(G_NT, AM_PLAIN, &gg, 1, s);
        CK(hipStreamSynchronize(s));
        out.resize((size_t)B * 4027);
        CK(hipMemcpy(out.data(), Yc, out.size() * 4, hipMemcpyDeviceToHost));
      };
      std::vector<float> ref, got;
      run_shapes(0, ref);
      for (int var : {19, 25}) {
        run_shapes(var, got);
        const size_t cut[4] = {0, (size_t)B * 1627, (size_t)B * 2227, (size_t)B * 4027};
        for (int rg = 0; rg < 3; ++rg) {
          double md = 0, mr = 0;
          for (size_t i = cut[rg]; i < cut[rg + 1]; ++i) {
            md = std::max(md, (double)fabsf(got[i] - ref[i]));
            mr = std::max(mr, (double)fabsf(ref[i]));
          }
          printf("tv%d check vs tv0 (%s): max|d| %.3e (max|ref| %.3e)\n", var, rg == 0 ? "BPTT" : rg == 1 ? "heads" : "GRU", md, mr);
        }
      }
      dr_debug_tile_variant(0);
    }
    for (int var : {0, 13, 20, 25, 26}) {
      dr_debug_tile_variant(var);
      for (int sk = 0; sk < 2; ++sk) {
        if ((var >= 8 && var < 12) && sk) continue;
        auto prep = [&](GemmArgs g) {
          if (sk) { g.splitk_ws = skw; g.splitk_floats = 8LL * 256 * 2048; }
          return g;
        };
        GemmArgs s1[2] = {prep(nt_(B, 1027, 1800)), prep(nt_(B, 600, 1800))};
        snprintf(buf, sizeof buf, "tv%d%s BPTT gZ+gH N1027+600 K1800", var, sk ? " sk" : "");
        timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_PLAIN, s1, 2, st); }, s);
        GemmArgs s2[3] = {prep(nt_(B, 200, 1624)), prep(nt_(B, 200, 1624)), prep(nt_(B, 200, 1624))};
        snprintf(buf, sizeof buf, "tv%d%s heads L1 3x N200 K1624", var, sk ? " sk" : "");
        timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_PLAIN, s2, 3, st); }, s);
        GemmArgs s3 = prep(nt_(B, 1800, 600));
        snprintf(buf, sizeof buf, "tv%d%s GRU gh N1800 K600", var, sk ? " sk" : "");
        timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_PLAIN, &s3, 1, st); }, s);
        GemmArgs s5 = prep(nt_(B, 200, 1624));
        snprintf(buf, sizeof buf, "tv%d%s actor L1 1x N200 K1624", var, sk ? " sk" : "");
        timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_PLAIN, &s5, 1, st); }, s);
        GemmArgs s4 = prep(nt_(B, 200, 600));
        snprintf(buf, sizeof buf, "tv%d%s prior L1 N200 K600", var, sk ? " sk" : "");
        timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_PLAIN, &s4, 1, st); }, s);
      }
    }
    dr_debug_tile_variant(0);
  }
  // tall products: the encoder feature projection (M = B*S/2 frames, K = 4096)
  // and the critic's first layer over B*(H+1) rows, by tile variant
  {
    float* Xb = frand((size_t)8192 * 4096);
    float* Wb = frand((size_t)256 * 4096);
    float* Yb = frand((size_t)8192 * 256);
    float* skw = frand((size_t)4 * 8192 * 256);
    for (int var : {0, 4, 5, 6, 7}) {
      dr_debug_tile_variant(var);
      int shp[][3] = {{8192, 200, 4096}, {4096, 200, 1624}, {2048, 200, 4096}};
      for (auto& sh : shp) {
        GemmArgs g = gemm_args();
        g.M = sh[0]; g.N = sh[1]; g.K = sh[2]; g.A = Xb; g.lda = sh[2]; g.ksplitA = sh[2]; g.W = Wb; g.ldb = sh[2];
        g.bias = bias; g.Y = Yb; g.ldy = sh[1];
        g.splitk_ws = skw; g.splitk_floats = 4LL * 8192 * 256;
        snprintf(buf, sizeof buf, "tw%d NT M%d N%d K%d (split-K scratch)", var, sh[0], sh[1], sh[2]);
        timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_PLAIN, &g, 1, st); }, s);
      }
    }
    dr_debug_tile_variant(0);
  }
  // the prior head's last layer with the sampler epilogue (LN-SiLU prologue,
  // N = 1024 = 32 groups x 32 classes): default 16-row tiles vs 64-row tiles
  {
    unsigned long long* rng;
    CK(hipMalloc(&rng, 16));
    CK(hipMemset(rng, 0, 16));
    float* zo = frand((size_t)B * 1024);
    int* io;
    CK(hipMalloc(&io, (size_t)B * 32 * 8));
    for (int var : {0, 1, 5}) {
      // 0: the dedicated sampler-head kernel (k_ln_gemm_sample); 1 / 5: the skinny kernel's
      // sampler epilogue with 16-row (default) / 64-row tiles
      dr_debug_ln_sample_off(var != 0);
      dr_debug_skinny_variant(var == 5 ? 5 : 0);
      GemmArgs g = nt_(B, 1024, 200);
      g.ln_g = lng; g.ln_b = lnb;
      g.epi = EPI_SAMPLE; g.R = 32; g.C = 32; g.unimix = 0.01f / 32;
      g.noise.rng = rng; g.noise.stream = 7;
      g.z_out = zo; g.ldz = 1024; g.idx_out = io; g.zval_out = reinterpret_cast<float*>(io + B * 32);
      g.soft_out = Y; g.ld_soft = 1024; g.Y = nullptr;
      snprintf(buf, sizeof buf, "ts%d sampler lnsilu M%d N1024 K200", var, B);
      timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_LNSILU, &g, 1, st); }, s);
      phases(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_LNSILU, &g, 1, st); }, dr_debug_tbuf_gemm, s);
      GemmArgs gn = g;
      gn.epi = EPI_NONE; gn.Y = Y; gn.ldy = 1024;
      snprintf(buf, sizeof buf, "ts%d same, plain epilogue", var);
      timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_LNSILU, &gn, 1, st); }, s);
      phases(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_LNSILU, &gn, 1, st); }, dr_debug_tbuf_gemm, s);
    }
    dr_debug_skinny_variant(0);
    dr_debug_ln_sample_off(0);
  }
  // per-step shapes of the imagination / BPTT chain, both row-tile variants
  for (int var = 0; var < 5; ++var) {
    if (var == 1 || var == 2) continue;
    dr_debug_skinny_variant(var);
    int sh2[][3] = {{B, 1027, 1800}, {B, 600, 1800}, {B, 200, 1624}, {B, 1024, 200}, {B, 200, 1024}, {B, 200, 600}};
    for (auto& sh : sh2) {
      GemmArgs g = nt_(sh[0], sh[1], sh[2]);
      snprintf(buf, sizeof buf, "s%d NT plain M%d N%d K%d", var, sh[0], sh[1], sh[2]);
      timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_PLAIN, &g, 1, st); }, s);
    }
    int sh3[][3] = {{B, 200, 200}, {B, 1024, 200}, {B, 6, 200}, {B, 255, 200}};
    for (auto& sh : sh3) {
      GemmArgs gl = nt_(sh[0], sh[1], sh[2]);
      gl.ln_g = lng; gl.ln_b = lnb;
      snprintf(buf, sizeof buf, "s%d NT lnsilu M%d N%d K%d", var, sh[0], sh[1], sh[2]);
      timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_LNSILU, &gl, 1, st); }, s);
    }
    GemmArgs gp[2] = {nt_(B, 1027, 1800), nt_(B, 600, 1800)};
    snprintf(buf, sizeof buf, "s%d NT plain grouped BPTT gZ+gH", var);
    timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_PLAIN, gp, 2, st); }, s);
    GemmArgs gb2 = nt_(64, 1624, 200);
    gb2.ln_g = lng; gb2.ln_b = lnb; gb2.pre = X; gb2.ld_pre = 200;
    snprintf(buf, sizeof buf, "s%d NT lnbwd M64 N1624 K200", var);
    timeit(buf, [&](hipStream_t st) { gemm_launch(G_NT, AM_LNBWD, &gb2, 1, st); }, s);
  }
  dr_debug_skinny_variant(0);
  // mid-size shapes (tile GEMM, split-K scratch when given)
  {
    float* skw = frand((size_t)8 << 20);
    float* Xm = frand((size_t)2048 * 4096);  // largest A of the cases below
    float* Wm = frand((size_t)1624 * 1024);  // largest B
    float* Ym = frand((size_t)2048 * 1624);
    struct Mid { int M, N, K; bool tn; bool sk; } mids[] = {
        {1024, 200, 1624, false, false}, {1024, 200, 1624, false, true}, {2048, 200, 4096, false, true},
        {200, 1624, 960, true, false},   {200, 1624, 960, true, true},   {200, 200, 1024, true, true}};
    for (int var = 0; var < 6; ++var)
    for (auto& c : mids) {
      dr_debug_tile_variant(var < 4 ? var : 0);
      dr_debug_tile_wgs(var == 4 ? 256 : var == 5 ? 1024 : 512);
      GemmArgs g = gemm_args();
      g.M = c.M; g.N = c.N; g.K = c.K;
      if (!c.tn) { g.A = Xm; g.lda = c.K; g.W = Wm; g.ldb = c.K; }
      else { g.A = Xm; g.lda = c.M; g.W = Wm; g.ldb = c.N; }
      g.ksplitA = INT_MAX;
      g.Y = Ym; g.ldy = c.N;
      if (c.sk) { g.splitk_ws = skw; g.splitk_floats = (long long)8 << 20; }
      snprintf(buf, sizeof buf, "v%d %s M%d N%d K%d%s", var, c.tn ? "TN" : "NT", c.M, c.N, c.K, c.sk ? " splitK" : "");
      timeit(buf, [&](hipStream_t st) { gemm_launch(c.tn ? G_TN : G_NT, AM_PLAIN, &g, 1, st); }, s, 50);
    }
    dr_debug_tile_variant(0);
  }
  // ln_silu_bwd / colsum
  timeit("ln_silu_bwd M64 K512", [&](hipStream_t st) { op_ln_silu_bwd(64, 512, X, 512, Y, 512, lng, lnb, W, 512, nullptr, nullptr, st); }, s);
  timeit("ln_silu_bwd M64 K512 +saves", [&](hipStream_t st) { op_ln_silu_bwd(64, 512, X, 512, Y, 512, lng, lnb, W, 512, W + 65536, W + 2 * 65536, st); }, s);
  timeit("colsum M960 N512", [&](hipStream_t st) { op_colsum(960, 512, X, 512, nullptr, 0, bias, 0, st); }, s);
  timeit("colsum M64 N512", [&](hipStream_t st) { op_colsum(64, 512, X, 512, nullptr, 0, bias, 0, st); }, s);
  CK(hipDeviceSynchronize());
  printf("ok\n");
  return 0;
}
