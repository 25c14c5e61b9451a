// Shared device/host helpers for libdreamer_hip (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dreamer_hip.h"

#define DR_WAVE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// error plumbing (thread-local last error string, no exceptions across the ABI)
// ---------------------------------------------------------------------------
void dr_set_error(const char* fmt, ...);
int dr_check_launch(const char* what);

#define DR_TRY(expr)                      \
  do {                                    \
    int _rc = (expr);                     \
    if (_rc != 0) return _rc;             \
  } while (0)

#define DR_TRY_HIP(expr)                                                          \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      dr_set_error("%s: %s: %s", __func__, #expr, hipGetErrorString(_e));         \
      return DR_E_HIP;                                                            \
    }                                                                             \
  } while (0)

#define DR_REQUIRE(cond, msg)                         \
  do {                                                \
    if (!(cond)) {                                    \
      dr_set_error("%s: %s", __func__, msg);          \
      return DR_E_INVALID;                            \
    }                                                 \
  } while (0)

// ---------------------------------------------------------------------------
// device math.  Parity mode keeps IEEE f32 (the library is built with
// -ffp-contract=off so elementwise code rounds exactly like the CPU oracle's
// op sequence; MFMA chains are exact f32 fma chains).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float dr_sigmoid(float x) { return 1.0f / (1.0f + __expf(-x)); }
__device__ __forceinline__ float dr_sigmoid_precise(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float dr_silu(float x) { return x / (1.0f + expf(-x)); }
// d SiLU(x) / dx as torch's silu_backward: s * (1 + x * (1 - s))
__device__ __forceinline__ float dr_dsilu(float x) {
  const float s = 1.0f / (1.0f + expf(-x));
  return s * (1.0f + x * (1.0f - s));
}
__device__ __forceinline__ float dr_softplus(float x) {  // torch softplus(beta=1, threshold=20)
  return x > 20.0f ? x : log1pf(expf(x));
}
__device__ __forceinline__ float dr_symexp(float x) {  // DreamerUtils.py:35-37
  x = fminf(fmaxf(x, -20.0f), 20.0f);
  float s = (x > 0.0f) ? 1.0f : ((x < 0.0f) ? -1.0f : 0.0f);
  return s * (expf(fabsf(x)) - 1.0f);
}
__device__ __forceinline__ float dr_symlog(float x) {  // DreamerUtils.py:29-30
  float s = (x > 0.0f) ? 1.0f : ((x < 0.0f) ? -1.0f : 0.0f);
  return s * logf(1.0f + fabsf(x));
}

// Phase timestamps for the kernel microbenchmark (tools/kbench): compiled in
// only with -DDR_PHASE_TIMING; wave 0 of each workgroup records the 100 MHz
// constant clock at phase boundaries.
#define DR_TS_SLOTS 8
#ifdef DR_PHASE_TIMING
#define DR_TS(buf, i)                                                        \
  do {                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 1024 && blockIdx.y == 0 && blockIdx.z == 0) \
      buf[blockIdx.x * DR_TS_SLOTS + (i)] = (long long)wall_clock64();      \
  } while (0)
#else
#define DR_TS(buf, i) \
  do {                \
  } while (0)
#endif

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup
// release/acquire fence on all memory, so it waits for every outstanding
// global load (s_waitcnt vmcnt(0)) -- including loads a pipelined loop issued
// for later iterations.  The LDS-scoped fences wait only on lgkmcnt.
__device__ __forceinline__ void dr_lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Kernel-argument staging.  A kernel that reads a large argument block field by
// field issues one dependent scalar load per field, and on a graph replay the
// argument lines are cold (each miss ~0.5 us), so the fields arrive one after
// another.  Copying the block into LDS with one parallel vector load per
// 16 bytes turns that chain into a single round trip.
template <typename T>
__device__ __forceinline__ void dr_stage_args(const T& src, T& dst, int tid) {
  static_assert(sizeof(T) % 16 == 0, "argument block must be a multiple of 16 bytes");
  constexpr int N16 = sizeof(T) / 16;
  if (tid < N16) reinterpret_cast<int4*>(&dst)[tid] = reinterpret_cast<const int4*>(&src)[tid];
  __syncthreads();
}

// Wave-uniform values.  Arguments read back from LDS are VGPRs as far as the
// compiler knows; readfirstlane turns them into SGPRs, so address math runs
// on the scalar unit and loads use the saddr + 32-bit voffset form.
__device__ __forceinline__ int dr_uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ float dr_uni(float x) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
template <typename T>
__device__ __forceinline__ T* dr_uni(T* p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (T*)(((unsigned long long)hi << 32) | lo);
}
// Global-memory access through pointers the compiler cannot trace to a
// kernel argument (e.g. fields of an argument block staged in LDS): without
// the explicit address space they become flat accesses, which count on both
// vmcnt and lgkmcnt -- every LDS wait would then drain all global loads.
#define DR_GLOBAL __attribute__((address_space(1)))
typedef float dr_f4 __attribute__((ext_vector_type(4)));
template <typename T>
__device__ __forceinline__ DR_GLOBAL T* dr_g(T* p) {
  return (DR_GLOBAL T*)p;
}
// loads at a 32-bit element offset from a uniform base (callers guarantee
// offsets < 2^30 elements): global_load with saddr + voffset
__device__ __forceinline__ float4 dr_ld4(const float* base, unsigned e) {
  const dr_f4 t = *(const DR_GLOBAL dr_f4*)((const DR_GLOBAL char*)base + (e << 2));
  return make_float4(t.x, t.y, t.z, t.w);
}
__device__ __forceinline__ float dr_ld1(const float* base, unsigned e) {
  return *(const DR_GLOBAL float*)((const DR_GLOBAL char*)base + (e << 2));
}
__device__ __forceinline__ void dr_st4(float* base, unsigned e, float4 v) {
  dr_f4 t = {v.x, v.y, v.z, v.w};
  *(DR_GLOBAL dr_f4*)((DR_GLOBAL char*)base + (e << 2)) = t;
}

// SiLU on the hardware exp2 / reciprocal (~2 ulp, 6 VALU instead of ~25 for
// the IEEE expf + division); used where the input is transformed once per
// consuming tile, inside the GEMM prologue
__device__ __forceinline__ float dr_silu_fast(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
// tanh on the hardware exp2 / rcp: 1 - 2 / (e^{2x} + 1) (saturates to +-1)
__device__ __forceinline__ float dr_tanh_fast(float x) {
  return 1.0f - 2.0f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(x * 2.8853900817779268f) + 1.0f);
}
// d SiLU / dx on the hardware exp2 / rcp (the conv epilogues over 10^8
// elements: the IEEE expf + division cost ~30 VALU per element there)
__device__ __forceinline__ float dr_dsilu_fast(float x) {
  const float s = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
  return s * (1.0f + x * (1.0f - s));
}

// XCD-aware tile order.  Workgroups are dealt to the 8 XCDs round-robin
// (block b runs on XCD b % 8, each XCD has its own L2).  Mapping block b to
// logical tile (b % 8) * per + b / 8 gives every XCD a contiguous run of
// logical tiles, so tiles that share operands (ordered next to each other by
// the caller) share one L2.  Launch 8 * per blocks, per = ceil(tiles / 8);
// returns -1 for the padding blocks.
#define DR_XCDS 8
__host__ __device__ __forceinline__ int dr_xcd_grid(int tiles) { return DR_XCDS * ((tiles + DR_XCDS - 1) / DR_XCDS); }
__device__ __forceinline__ int dr_xcd_tile(int b, int tiles) {
  const int per = (tiles + DR_XCDS - 1) / DR_XCDS;
  const int k = b / DR_XCDS;
  if (k >= per) return -1;  // a grid sized for a larger problem of the batch
  const int t = (b % DR_XCDS) * per + k;
  return t < tiles ? t : -1;
}

// wave64 reductions (call with the whole wave active).  In-row butterfly on
// DPP (quad xor 1, quad xor 2, half-row mirror, row mirror: every lane of a
// 16-lane row ends with the row total, bitwise identical by commutativity),
// then the four row totals read as scalars -- no LDS crossbar round trips.
template <int CTRL>
__device__ __forceinline__ float dr_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float dr_lane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dr_dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dr_dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dr_dpp<0x141>(v);  // row_half_mirror
  v += dr_dpp<0x140>(v);  // row_mirror
  return ((dr_lane(v, 0) + dr_lane(v, 16)) + dr_lane(v, 32)) + dr_lane(v, 48);
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dr_dpp<0xB1>(v));
  v = fmaxf(v, dr_dpp<0x4E>(v));
  v = fmaxf(v, dr_dpp<0x141>(v));
  v = fmaxf(v, dr_dpp<0x140>(v));
  return fmaxf(fmaxf(dr_lane(v, 0), dr_lane(v, 16)), fmaxf(dr_lane(v, 32), dr_lane(v, 48)));
}
// reductions inside aligned sub-groups of `width` lanes (power of two <= 64,
// wave-uniform): DPP inside 16-lane rows, lane shuffles across rows
__device__ __forceinline__ float group_sum(float v, int width) {
  if (width >= 2) v += dr_dpp<0xB1>(v);
  if (width >= 4) v += dr_dpp<0x4E>(v);
  if (width >= 8) v += dr_dpp<0x141>(v);
  if (width >= 16) v += dr_dpp<0x140>(v);
  if (width >= 32) v += __shfl_xor(v, 16, 64);
  if (width >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}
__device__ __forceinline__ float group_max(float v, int width) {
  if (width >= 2) v = fmaxf(v, dr_dpp<0xB1>(v));
  if (width >= 4) v = fmaxf(v, dr_dpp<0x4E>(v));
  if (width >= 8) v = fmaxf(v, dr_dpp<0x141>(v));
  if (width >= 16) v = fmaxf(v, dr_dpp<0x140>(v));
  if (width >= 32) v = fmaxf(v, __shfl_xor(v, 16, 64));
  if (width >= 64) v = fmaxf(v, __shfl_xor(v, 32, 64));
  return v;
}

// (max, lowest index) over the same sub-groups: the pair combine is
// commutative and associative, so the DPP tree gives the shuffle loop's
// result -- with 4 DPP moves instead of a chain of LDS-crossbar permutes
template <int CTRL>
__device__ __forceinline__ int dr_dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ void arg_step(float& best, int& bi, float ob, int oi) {
  if (ob > best || (ob == best && oi < bi)) {
    best = ob;
    bi = oi;
  }
}
__device__ __forceinline__ void group_argmax(float& best, int& bi, int width) {
  if (width >= 2) arg_step(best, bi, dr_dpp<0xB1>(best), dr_dpp_i<0xB1>(bi));
  if (width >= 4) arg_step(best, bi, dr_dpp<0x4E>(best), dr_dpp_i<0x4E>(bi));
  if (width >= 8) arg_step(best, bi, dr_dpp<0x141>(best), dr_dpp_i<0x141>(bi));
  if (width >= 16) arg_step(best, bi, dr_dpp<0x140>(best), dr_dpp_i<0x140>(bi));
  if (width >= 32) arg_step(best, bi, __shfl_xor(best, 16, 64), __shfl_xor(bi, 16, 64));
  if (width >= 64) arg_step(best, bi, __shfl_xor(best, 32, 64), __shfl_xor(bi, 32, 64));
}

// ---------------------------------------------------------------------------
// Philox4x32-10 counter RNG (perf-mode noise).  Keys: (seed), counter:
// (offset_lo, offset_hi ^ stream, row, element) so a row's noise does not
// depend on how the batch is sharded across ranks.
// ---------------------------------------------------------------------------
struct dr_u4 { uint32_t x, y, z, w; };
__device__ __forceinline__ dr_u4 philox4x32(dr_u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    dr_u4 n;
    n.x = hi1 ^ c.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ c.w ^ k1;
    n.w = lo0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
// uniform on the 2^23-point grid (k + 1/2) 2^-23 in [2^-24, 1 - 2^-24]: never 0
// and never 1, so an Exp(1) variate -log(u) is > 0 (p_hat / q stays finite; a
// u of exactly 1 once gave q = 0 with probability 2^-24 per draw) and
// Box-Muller's log(u1) is finite (torch's exponential_ avoids a zero variate
// likewise)
__device__ __forceinline__ float dr_u01(uint32_t x) { return ((float)(x >> 9) + 0.5f) * (1.0f / 8388608.0f); }

__device__ __forceinline__ dr_u4 dr_rand4(const unsigned long long* so, uint32_t stream, uint32_t row,
                                          uint32_t elem) {
  unsigned long long seed = so[0], off = so[1];
  dr_u4 c = {(uint32_t)off, (uint32_t)(off >> 32) ^ (stream * 0x85EBCA6Bu), row, elem};
  return philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}
// the same with the {seed, offset} pair already in registers (prefetched at
// kernel entry: the epilogue then pays no dependent load of the RNG state)
__device__ __forceinline__ dr_u4 dr_rand4_k(unsigned long long seed, unsigned long long off, uint32_t stream,
                                            uint32_t row, uint32_t elem) {
  dr_u4 c = {(uint32_t)off, (uint32_t)(off >> 32) ^ (stream * 0x85EBCA6Bu), row, elem};
  return philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}
__device__ __forceinline__ float dr_exp1_k(unsigned long long seed, unsigned long long off, uint32_t stream,
                                           uint32_t row, uint32_t elem) {
  return -logf(dr_u01(dr_rand4_k(seed, off, stream, row, elem).x));
}
__device__ __forceinline__ float dr_normal_k(unsigned long long seed, unsigned long long off, uint32_t stream,
                                             uint32_t row, uint32_t elem) {
  dr_u4 r = dr_rand4_k(seed, off, stream, row, elem);
  float u1 = dr_u01(r.x), u2 = dr_u01(r.y);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}
// Exp(1) variate for (stream,row,elem) -- element-exact, independent of launch shape
__device__ __forceinline__ float dr_exp1(const unsigned long long* so, uint32_t stream, uint32_t row,
                                         uint32_t elem) {
  dr_u4 r = dr_rand4(so, stream, row, elem);
  return -logf(dr_u01(r.x));
}
__device__ __forceinline__ float dr_normal(const unsigned long long* so, uint32_t stream, uint32_t row,
                                           uint32_t elem) {
  dr_u4 r = dr_rand4(so, stream, row, elem);
  float u1 = dr_u01(r.x), u2 = dr_u01(r.y);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

static inline int dr_cdiv(int a, int b) { return (a + b - 1) / b; }

// fp32 operands on the bf16 MFMA (conv_split.hip, k_gemm_tile_s3): f32 values
// split by truncation: h = x with the low 16 bits cleared (the
// bf16 head), r1 = x - h and r2 = r1 - m (m = r1 truncated) are exact, l = r2
// truncated: |x - (h + m + l)| < 2^-23 |x|.  Pairs of elements are packed into
// bf16x2 words by v_perm_b32 (the high halves of two f32 words)
__device__ __forceinline__ void split3_pair(float x0, float x1, unsigned& h, unsigned& m, unsigned& l) {
  constexpr unsigned HI = 0xFFFF0000u, SEL = 0x07060302u;  // bytes 2,3 of S1 then 2,3 of S0
  const unsigned b0 = __builtin_bit_cast(unsigned, x0), b1 = __builtin_bit_cast(unsigned, x1);
  const float r10 = x0 - __builtin_bit_cast(float, b0 & HI), r11 = x1 - __builtin_bit_cast(float, b1 & HI);
  const unsigned c0 = __builtin_bit_cast(unsigned, r10), c1 = __builtin_bit_cast(unsigned, r11);
  const float r20 = r10 - __builtin_bit_cast(float, c0 & HI), r21 = r11 - __builtin_bit_cast(float, c1 & HI);
  h = __builtin_amdgcn_perm(b1, b0, SEL);
  m = __builtin_amdgcn_perm(c1, c0, SEL);
  l = __builtin_amdgcn_perm(__builtin_bit_cast(unsigned, r21), __builtin_bit_cast(unsigned, r20), SEL);
}
