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

// wave64 reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reductions inside aligned sub-groups of `width` lanes (power of two <= 64)
__device__ __forceinline__ float group_sum(float v, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float group_max(float v, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
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
// uniform in (0, 1]
__device__ __forceinline__ float dr_u01(uint32_t x) { return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f); }

__device__ __forceinline__ dr_u4 dr_rand4(const unsigned long long* so, uint32_t stream, uint32_t row,
                                          uint32_t elem) {
  unsigned long long seed = so[0], off = so[1];
  dr_u4 c = {(uint32_t)off, (uint32_t)(off >> 32) ^ (stream * 0x85EBCA6Bu), row, elem};
  return philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
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
