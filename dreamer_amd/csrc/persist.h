// Device helpers of the persistent (one launch per scan / unroll) kernels:
// split3 bf16 MFMA products, resident weight fragments, write-through (sc1)
// hand-off buffers, counters and tagged granules (scan.hip, dream.hip).
// Protocol: MI355X_MICROARCH.md "Inter-workgroup visibility", valid-form
// table row 1 (every handed-off byte stored and loaded sc1, each storing wave
// drained before ONE lane signals) and the 8-byte {data, tag} granules.
#pragma once
#include "common.h"

typedef unsigned ps_u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 ps_bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 ps_mfma(ps_u32x4 w, ps_u32x4 a, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(ps_bf16x8, w), __builtin_bit_cast(ps_bf16x8, a),
                                                  c, 0, 0, 0);
}
// NT = 3: the six products of order >= 2^-16, smallest first (k_gemm_wks3's
// order); NT = 1: bf16 perf mode (plane 0 x RNE(a))
template <int NT>
__device__ __forceinline__ f32x4 ps_prod(const ps_u32x4 (&w)[NT], const ps_u32x4 (&a)[NT], f32x4 c) {
  if constexpr (NT == 3) {
    c = ps_mfma(w[0], a[2], c);
    c = ps_mfma(w[1], a[1], c);
    c = ps_mfma(w[2], a[0], c);
    c = ps_mfma(w[0], a[1], c);
    c = ps_mfma(w[1], a[0], c);
  }
  return ps_mfma(w[0], a[0], c);
}
__device__ __forceinline__ unsigned ps_rne2(float x0, float x1) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  const b2 v = {(__bf16)x0, (__bf16)x1};
  return __builtin_bit_cast(unsigned, v);
}
// 8 consecutive k of one row -> the MFMA fragment(s)
template <int NT>
__device__ __forceinline__ void ps_split(f32x4 x0, f32x4 x1, ps_u32x4 (&a)[NT]) {
  if constexpr (NT == 3) {
    unsigned h[4], m[4], l[4];
    split3_pair(x0[0], x0[1], h[0], m[0], l[0]);
    split3_pair(x0[2], x0[3], h[1], m[1], l[1]);
    split3_pair(x1[0], x1[1], h[2], m[2], l[2]);
    split3_pair(x1[2], x1[3], h[3], m[3], l[3]);
    a[0] = (ps_u32x4){h[0], h[1], h[2], h[3]};
    a[1] = (ps_u32x4){m[0], m[1], m[2], m[3]};
    a[2] = (ps_u32x4){l[0], l[1], l[2], l[3]};
  } else {
    a[0] = (ps_u32x4){ps_rne2(x0[0], x0[1]), ps_rne2(x0[2], x0[3]), ps_rne2(x1[0], x1[1]), ps_rne2(x1[2], x1[3])};
  }
}

// A resident weight fragment: the 8 consecutive k of one weight row a lane
// feeds to the MFMA.  NT = 3 keeps them f32 (8 VGPRs) and splits them per use
// (exact truncation split, 6 products); NT = 1 keeps their RNE bf16 (4 VGPRs).
template <int NT>
struct PsFrag {
  f32x4 x0, x1;
};
template <>
struct PsFrag<1> {
  ps_u32x4 b;
};
// an offset the compiler cannot see through: keeps per-step weight loads in
// the step loop (hoisted, they would stay live in registers across the scan)
__device__ __forceinline__ unsigned ps_opaque(unsigned x) {
  asm volatile("" : "+v"(x));
  return x;
}
// "these loaded values are needed here": one wait for a batch of loads issued
// together (the scheduler would otherwise sink each load to its use and pay a
// round trip per use under register pressure)
__device__ __forceinline__ void ps_pin(f32x4& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void ps_pin(float& x) { asm volatile("" : "+v"(x)); }
template <int NT>
__device__ __forceinline__ PsFrag<NT> ps_frag(const float* W, unsigned e, bool ok) {
  const float4 a = dr_ld4(W, ok ? e : 0u), c = dr_ld4(W, ok ? e + 4u : 0u);
  f32x4 x0 = {a.x, a.y, a.z, a.w}, x1 = {c.x, c.y, c.z, c.w};
  if (!ok) x0 = x1 = (f32x4){0.f, 0.f, 0.f, 0.f};
  PsFrag<NT> f;
  if constexpr (NT == 3) {
    f.x0 = x0;
    f.x1 = x1;
  } else {
    ps_u32x4 b[1];
    ps_split<1>(x0, x1, b);
    f.b = b[0];
  }
  return f;
}
// the opaque copy keeps the compiler from hoisting the split of a resident
// fragment out of the step loop (that would re-create the 12-VGPR planes)
template <int NT>
__device__ __forceinline__ void ps_wsplit(const PsFrag<NT>& f, ps_u32x4 (&w)[NT]) {
  if constexpr (NT == 3) {
    f32x4 x0 = f.x0, x1 = f.x1;
    asm volatile("" : "+v"(x0), "+v"(x1));
    ps_split<3>(x0, x1, w);
  } else {
    w[0] = f.b;
  }
}

// write-through (sc1) buffer accesses of the handed-off rings
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ps_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 ps_ld4(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 16));
}
__device__ __forceinline__ float ps_ld1(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)byte_off, 0, 16));
}
__device__ __forceinline__ void ps_st1(__amdgpu_buffer_rsrc_t r, unsigned byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)byte_off, 0, 16);
}
__device__ __forceinline__ void ps_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// 8-byte {data, tag} granules (MI355X_MICROARCH.md: the data IS the flag): ONE
// aligned 8-byte sc1 store per granule, sc1 loads re-read until the tag matches
typedef unsigned long long ps_u64;
__device__ __forceinline__ void ps_gst(ps_u64* p, ps_u64 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ ps_u64 ps_gld(const ps_u64* p) {
  return __hip_atomic_load(const_cast<ps_u64*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// lane 0 of the workgroup: poll until *c >= target (relaxed sc1 loads + s_sleep).
// limit < 0 (DREAMER_PERSIST_FORCE, the failure-path test hook): every poll times out
__device__ __forceinline__ bool ps_poll(const unsigned* c, unsigned target, int limit, unsigned* status) {
  if (limit < 0) {
    __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  int spins = 0;
  while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    __builtin_amdgcn_s_sleep(2);
    if (++spins > limit) {
      __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}
// every storing wave drained, then one lane signals for the workgroup
__device__ __forceinline__ void ps_signal(unsigned* c) {
  ps_drain();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// the total over each 16-lane row, in every lane of the row (DPP only)
__device__ __forceinline__ float row16_sum(float v) {
  v += dr_dpp<0xB1>(v);
  v += dr_dpp<0x4E>(v);
  v += dr_dpp<0x141>(v);
  v += dr_dpp<0x140>(v);
  return v;
}

// lane 0 polls counters c0, c0 + ld, ... (n of them) >= target, then the
// workgroup barrier; false on a timeout (the status word is set)
__device__ __forceinline__ bool ps_wait(int* s_ok, const unsigned* c0, int ld, int n, unsigned target, int lim,
                                        unsigned* status) {
  if (threadIdx.x == 0) {
    bool ok = true;
    for (int i = 0; i < n && ok; ++i) ok = ps_poll(c0 + ld * i, target, lim, status);
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}
// The failure path of a persistent launch.  Every workgroup ends in ps_exit,
// also after a timed-out wait; the LAST one to arrive (an exit ticket) reads
// the status word and, if any wait timed out, writes NaN over the launch's
// outputs and the caller's fault slot (dr_dims.fault).  A partly written result
// therefore never passes for a valid one: NaN flows into the losses, the
// agent's non-finite skip (Agent.py:137-139, dr_clip_stats over the loss slots,
// which include the fault slot) rejects the update, and the host raises when it
// sees the host-mapped fault word (engine.py check_faults).  Both are sticky:
// the library never clears them.
struct PsPoison {
  float* p[8];
  unsigned long long n[8];  // floats at p[i]
  float* fault;             // dr_dims.fault (device)
  unsigned* fault_host;     // dr_dims.fault_host (pinned host memory, device-mapped)
};
__device__ __forceinline__ void ps_exit(unsigned* ticket, const unsigned* status, const PsPoison& pz) {
  __shared__ int s_last;
  ps_drain();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t + 1u == gridDim.x &&
             __hip_atomic_load(const_cast<unsigned*>(status), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  }
  __syncthreads();
  if (!s_last) return;
  const float nan = __builtin_nanf("");
#pragma unroll 1
  for (int i = 0; i < 8; ++i) {
    float* p = pz.p[i];
    if (!p) continue;
    for (unsigned long long x = threadIdx.x; x < pz.n[i]; x += blockDim.x) p[x] = nan;
  }
  if (threadIdx.x == 0) {
    if (pz.fault) *pz.fault = nan;
    if (pz.fault_host) __hip_atomic_store(pz.fault_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
// the spin limit of a persistent launch: DREAMER_PERSIST_FORCE=timeout (or
// the kernel's name: scan / dream / bptt) makes every wait of that kernel time
// out at once (test hook of the failure path, read at each call like
// DREAMER_ACT_FORCE; a captured graph keeps the value of its capture)
int ps_spin_limit(const char* kernel);

// every storing wave drained; lanes 0 .. n-1 add 1 to counters c0, c0 + ld, ...
__device__ __forceinline__ void ps_signal_n(unsigned* c0, int ld, int n) {
  ps_drain();
  __syncthreads();
  if ((int)threadIdx.x < n)
    __hip_atomic_fetch_add(c0 + ld * threadIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
