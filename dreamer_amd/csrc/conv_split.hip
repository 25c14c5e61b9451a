// fp32-accurate encoder convolutions on the bf16 MFMA (conv2..4 of
// VariationalAutoEncoder.py:33-42, k4 s2 p1 + SiLU, f32 NHWC activations).
//
// The f32-input MFMA runs at the f32 vector rate (64 FLOP/clk/SIMD), 1/16 of
// v_mfma_f32_16x16x32_bf16.  Every f32 operand x is split exactly into three
// bf16 terms, x = h + m + l (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m);
// both subtractions are exact, so |x - (h + m + l)| <= 2^-24 |x| up to the
// final rounding), and a product is accumulated from the six terms of order
// >= 2^-16 relative:
//
//   a*b ~ ah*bh + (ah*bm + am*bh) + (ah*bl + am*bm + al*bh)
//
// The dropped terms (am*bl, al*bm, al*bl) are <= 3 * 2^-24 |a b|, the size of
// one f32 rounding, so the result is an f32-accuracy convolution (checked
// against torch's f32 conv at 1e-5 in tests/test_gpu_bf16.py) at 6 bf16 MFMAs
// per 16x16x32 block instead of 8 f32 MFMAs of twice the cycles: 2.67x the
// f32 MFMA peak (416.7 TFLOP/s of f32 work).
//
// Layout: implicit GEMM, M = pixels (frame, oy, ox), N = output channels,
// K = tap * CIN + ci in chunks of 32 (one MFMA k-step).  Activations are read
// as f32 float4s, split while they are staged into LDS (once per workgroup, not
// per wave); the weights are split once per call by op_conv_repack_split3 into
// three bf16 planes [3][cout][K].  LDS holds each plane as rows of 4 16-byte
// units, unit u of row r at u ^ ((r >> 2) & 3): the 16 rows one MFMA fragment
// read touches fall on 16 distinct 16-byte bank groups.
#include "conv.h"

#include <algorithm>
#include <climits>
#include <type_traits>

namespace {
typedef unsigned short u16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
// native vector (HIP's uint4 is a struct: its copies became memcpys that kept
// the staging ring in scratch memory)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x4 mfma_b16(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                  0);
}
__device__ __forceinline__ unsigned b16bits(__bf16 v) { return (unsigned)__builtin_bit_cast(u16, v); }
// x = h + m + l (RNE at each step; the two residuals are exact in f32)
__device__ __forceinline__ void split3(float x, unsigned& h, unsigned& m, unsigned& l) {
  const __bf16 bh = (__bf16)x;
  const float r1 = x - (float)bh;
  const __bf16 bm = (__bf16)r1;
  const float r2 = r1 - (float)bm;
  h = b16bits(bh);
  m = b16bits(bm);
  l = b16bits((__bf16)r2);
}
// LDS unit swizzle of a 64-byte plane row: unit u of row r sits at
// u ^ G[(r >> 2) & 3], G = {0, 2, 3, 1}.  An MFMA fragment read (ds_read_b128,
// lane (r, q) -> row r, unit q) is serviced in the lane groups {0-3, 12-15,
// 20-27}, {4-11, 16-19, 28-31}, ... (MI355X_MICROARCH.md, LDS): with G every
// group's 16 lanes hit 16 distinct 16-byte bank quads (the plain (r >> 2) & 3
// swizzle left 2-way conflicts)
__device__ __forceinline__ int swz(int row) { return (0x1320 >> (((row >> 2) & 3) * 4)) & 3; }
// four f32 -> four bf16 (RNE), packed
__device__ __forceinline__ u32x2 pack_bf16x4(f32x4 v) {
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  const bf16x4_t b = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  return __builtin_bit_cast(u32x2, b);
}
// two f32 -> two bf16 (RNE), x0 in the low half (split3_pair's packing)
__device__ __forceinline__ unsigned pack_bf16x2(float x0, float x1) { return b16bits((__bf16)x0) | (b16bits((__bf16)x1) << 16); }
}  // namespace

// (s_setprio around each chunk's MFMA cluster, or for the younger half of the
// waves, measured neutral to slower: profiles/r04zm_conv_prio_ab.txt)
// EPI (conv.h): CONV_EPI_FWD: out = SiLU(acc + bias), optionally pre = acc + bias
// (NHWC, for the world-model backward); CONV_EPI_DSILU (NHWC only, no bias):
// out = acc * SiLU'(pre) -- the input gradient of a transposed conv followed by
// the SiLU backward of the layer below (WorldModel.training_step's decoder)
// NT3 = 1: the bf16 perf mode's form of the same tile -- bf16 NHWC activations
// staged as they are (one plane), the weights' first split plane (= their RNE
// bf16), one MFMA per block, bf16 output (RNE after bias + SiLU); `in` / `out`
// then point at u16 data.  NT3 = 1 with IO16 = false: the bf16 world-model
// step's form -- f32 activations rounded (RNE) to one bf16 plane as they are
// staged, f32 outputs and every epilogue of the three-term form
// K-loop position c -> (tap, first channel, chunk index of the natural
// tap-major order).  Channel chunks outer; within one, the 16 taps in four
// parity groups {ky, ky + 2} x {kx, kx + 2}: the four taps of a group read the
// same input pixels (output row oy + 1 at ky reads oy's ky + 2 row), so a
// workgroup's input is reused within 4 consecutive chunks.  In tap-major order
// a pixel came back 4-16 chunks later, after 128-512 KB of other traffic per
// workgroup, and the XCD's 4 MB L2 had dropped it: fp32 conv3 fetched 1.23 GB
// for a 0.54 GB input (profiles/r04zf_traffic_B256_r64_fp32.json).
template <int CIN>
__device__ __forceinline__ void conv_chunk(int c, int& tap, int& ci0, int& kc) {
  constexpr int CPT = CIN / 32;
  const int cc = c >> 4, t = c & 15;
  const int g = t >> 2, j = t & 3;
  const int ky = (g >> 1) + 2 * (j >> 1), kx = (g & 1) + 2 * (j & 1);
  tap = ky * 4 + kx;
  ci0 = 32 * cc;
  kc = tap * CPT + cc;
}

template <int BM, int BN, int CIN, bool OUT_NCHW, int PIPE, int EPI = CONV_EPI_FWD, int NT3 = 3, bool IO16 = (NT3 == 1)>
__global__ __launch_bounds__(BM * 2) void k_conv_split3(int n_frames, int ih, int iw, int cout,
                                                         const float* __restrict__ in, const u16* __restrict__ wr,
                                                         const float* __restrict__ bias, float* __restrict__ out,
                                                         float* __restrict__ pre) {
  static_assert(NT3 == 3 || (NT3 == 1 && (EPI == CONV_EPI_FWD || !IO16)), "conv_split3 terms");
  static_assert(!IO16 || NT3 == 1, "bf16 storage is the one-term form's");
  const u16* __restrict__ in16 = reinterpret_cast<const u16*>(in);
  u16* __restrict__ out16 = reinterpret_cast<u16*>(out);
  constexpr int NT = BM * 2;         // WM = BM / 64 waves over pixels x 2 waves over channels
  constexpr int K = CIN * 16;
  constexpr int NCH = K / 32;
  constexpr int WTN = BN / 2, FM = 4, FN = WTN / 16;
  constexpr int APT = BM * 8 / NT;   // float4 of A per thread per chunk (= 4)
  constexpr int BU = NT3 * BN * 4;   // 16-byte B units per chunk (NT3 planes x BN rows x 4)
  constexpr int BPT = (BU + NT - 1) / NT;
  static_assert(CIN % 32 == 0 && APT == 4 && FN >= 1, "conv_split3 tile");
  __shared__ __attribute__((aligned(16))) u32x4 As[2][NT3][BM][4];
  __shared__ __attribute__((aligned(16))) u32x4 Bs[2][NT3][BN][4];

  const int oh = ih / 2, ow = iw / 2, hw = oh * ow;
  const long long M = (long long)n_frames * hw;
  const int tiles_n = cout / BN;
  const long long tiles = ((M + BM - 1) / BM) * tiles_n;
  const int lt = dr_xcd_tile(blockIdx.x, (int)tiles);
  if (lt < 0) return;
  const long long m0 = (long long)(lt / tiles_n) * BM;
  const int n0 = (lt % tiles_n) * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;
  const int quad = tid & 7, prow = tid >> 3;  // A staging: float4 `quad` of rows prow + (NT/8) i

  // per A row: element offset of its (2 oy - 1, 2 ox - 1) input corner (32-bit:
  // n_frames * ih * iw * CIN < 2^31, host-checked) and the taps inside the
  // frame (bits 0-3: ky, bits 4-7: kx; rows past M: none)
  int pb[APT];
  unsigned vm[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const long long m = m0 + prow + (NT / 8) * i;
    const int mm = (int)(m < M ? m : 0);
    const int f = mm / hw, p = mm - f * hw, oy = p / ow, ox = p - oy * ow;
    const int y0 = 2 * oy - 1, x0 = 2 * ox - 1;
    pb[i] = ((f * ih + y0) * iw + x0) * CIN;
    unsigned v = 0u;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      v |= (y0 + t >= 0 && y0 + t < ih) ? (1u << t) : 0u;
      v |= (x0 + t >= 0 && x0 + t < iw) ? (16u << t) : 0u;
    }
    vm[i] = m < M ? v : 0u;
  }

  // two ring slots as separate arrays picked at compile time (one 2-D ring
  // array indexed by slot was left in scratch memory by the compiler)
  f32x4 ra0[APT], ra1[APT];
  u32x2 rh0[APT], rh1[APT];  // NT3 = 1: 4 bf16 channels
  u32x4 rb0[BPT], rb1[BPT];
  unsigned ok0 = 0, ok1 = 0;  // per slot: bit i = A row i's tap is inside the frame
  auto load = [&](int c, auto slot) __attribute__((always_inline)) {
    f32x4* ra = decltype(slot)::value == 0 ? ra0 : ra1;
    u32x2* rh = decltype(slot)::value == 0 ? rh0 : rh1;
    unsigned& okm = decltype(slot)::value == 0 ? ok0 : ok1;
    u32x4* rb = decltype(slot)::value == 0 ? rb0 : rb1;
    // CIN % 32 == 0: a chunk is 32 channels of one tap (uniform over the workgroup)
    int tap, ci0, kc;
    conv_chunk<CIN>(c, tap, ci0, kc);
    const int ky = tap >> 2, kx = tap & 3;
    const int toff = (ky * iw + kx) * CIN + ci0 + 4 * quad;
    unsigned om = 0u;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      // always load (padding taps read offset 0) and zero the padding at the
      // LDS store: a conditional load compiled to a branch that waited for
      // each load before issuing the next
      const bool ok = (vm[i] >> ky) & (vm[i] >> (4 + kx)) & 1u;
      if constexpr (IO16) rh[i] = *reinterpret_cast<const u32x2*>(in16 + (ok ? pb[i] + toff : 0));
      else ra[i] = *reinterpret_cast<const f32x4*>(in + (ok ? pb[i] + toff : 0));
      om |= ok ? (1u << i) : 0u;
    }
    okm = om;
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int e = tid + NT * j;  // (plane, row, unit)
      if (BU % NT == 0 || e < BU) {
        const int pl = e / (BN * 4), rem = e - pl * BN * 4, row = rem >> 2, u = rem & 3;
        rb[j] = *reinterpret_cast<const u32x4*>(wr + (((long long)kc * 3 + pl) * cout + n0 + row) * 32 + 8 * u);
      }
    }
  };
  auto store = [&](auto slot, int buf) __attribute__((always_inline)) {
    const f32x4* ra = decltype(slot)::value == 0 ? ra0 : ra1;
    const u32x2* rh = decltype(slot)::value == 0 ? rh0 : rh1;
    const u32x4* rb = decltype(slot)::value == 0 ? rb0 : rb1;
    const unsigned okm = decltype(slot)::value == 0 ? ok0 : ok1;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int row = prow + (NT / 8) * i;
      const int unit = (quad >> 1) ^ swz(row), half = quad & 1;
      if constexpr (IO16) {
        reinterpret_cast<u32x2*>(&As[buf][0][row][unit])[half] = (okm >> i) & 1u ? rh[i] : (u32x2){0u, 0u};
      } else if constexpr (NT3 == 1) {
        const f32x4 v = (okm >> i) & 1u ? ra[i] : (f32x4){0.f, 0.f, 0.f, 0.f};
        reinterpret_cast<u32x2*>(&As[buf][0][row][unit])[half] = pack_bf16x4(v);
      } else {
        const f32x4 v = (okm >> i) & 1u ? ra[i] : (f32x4){0.f, 0.f, 0.f, 0.f};
        unsigned h0, m0_, l0, h1, m1, l1;
        split3_pair(v[0], v[1], h0, m0_, l0);
        split3_pair(v[2], v[3], h1, m1, l1);
        reinterpret_cast<u32x2*>(&As[buf][0][row][unit])[half] = (u32x2){h0, h1};
        reinterpret_cast<u32x2*>(&As[buf][1][row][unit])[half] = (u32x2){m0_, m1};
        reinterpret_cast<u32x2*>(&As[buf][2][row][unit])[half] = (u32x2){l0, l1};
      }
    }
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int e = tid + NT * j;
      if (BU % NT == 0 || e < BU) {
        const int pl = e / (BN * 4), rem = e - pl * BN * 4, row = rem >> 2, u = rem & 3;
        Bs[buf][pl][row][u ^ swz(row)] = rb[j];
      }
    }
  };

  const int wm0 = (wave >> 1) * 64, wn0 = (wave & 1) * WTN;
  const int fu = q ^ swz(r);  // fragment rows are 16-aligned: swz(row) = swz(r)
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  load(0, S0{});
  load(1, S1{});
  store(S0{}, 0);
  __syncthreads();
  // the ring slot of chunk c is c % PIPE; every slot index is a compile-time
  // constant (a run-time index puts the ring in scratch memory)
  auto step = [&](int c, auto slot) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot)::value;
    using Next = std::integral_constant<int, 1 - SL>;
    const int buf = c & 1;
    // slot SL went to LDS at the end of the previous chunk: refill it.  Issued
    // unconditionally (the last two chunks reload chunk NCH - 1, unused): a
    // conditional refill made the compiler wait for every outstanding load
    // before the next LDS store, a one-deep pipeline
    load(min(c + PIPE, NCH - 1), slot);
    u32x4 a[NT3][FM], b[NT3][FN];
#pragma unroll
    for (int pl = 0; pl < NT3; ++pl) {
#pragma unroll
      for (int i = 0; i < FM; ++i) a[pl][i] = As[buf][pl][wm0 + 16 * i + r][fu];
#pragma unroll
      for (int j = 0; j < FN; ++j) b[pl][j] = Bs[buf][pl][wn0 + 16 * j + r][fu];
    }
    // smallest terms first; independent accumulators innermost
#define DR_S3(PA, PB)                                                                                   \
  _Pragma("unroll") for (int i = 0; i < FM; ++i) _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[i][j] = \
      OUT_NCHW ? mfma_b16(a[PA][i], b[PB][j], acc[i][j]) : mfma_b16(b[PB][j], a[PA][i], acc[i][j]);
    if constexpr (NT3 == 3) {
      DR_S3(2, 0)
      DR_S3(1, 1)
      DR_S3(0, 2)
      DR_S3(1, 0)
      DR_S3(0, 1)
    }
    DR_S3(0, 0)
#undef DR_S3
    if (c + 1 < NCH) store(Next{}, buf ^ 1);
    dr_lds_barrier();
  };
  static_assert(PIPE == 2 && NCH % 2 == 0, "conv_split3 ring");
  for (int c = 0; c < NCH; c += 2) {
    step(c, S0{});
    step(c + 1, S1{});
  }

  // NHWC: weights were the MFMA A operand, lane (r, q) holds channels 4q..4q+3
  // of pixel r; NCHW: pixels were A, the lane holds pixels 4q..4q+3 of channel r
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if (OUT_NCHW) {
        const long long m = m0 + wm0 + 16 * i + 4 * q;
        const int co = n0 + wn0 + 16 * j + r;
        if (m >= M) continue;
        const float bv = bias[co];
        f32x4 v = acc[i][j] + bv;
        if constexpr (IO16) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = dr_silu_fast(v[e]);
          const long long f = m / hw;
          *reinterpret_cast<u32x2*>(out16 + (f * cout + co) * hw + (m - f * hw)) = pack_bf16x4(v);
          continue;
        }
        if (pre) {
#pragma unroll
          for (int e = 0; e < 4; ++e) pre[(m + e) * cout + co] = v[e];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = dr_silu_fast(v[e]);
        const long long f = m / hw;
        *reinterpret_cast<f32x4*>(out + (f * cout + co) * hw + (m - f * hw)) = v;
      } else {
        const long long m = m0 + wm0 + 16 * i + r;
        const int co = n0 + wn0 + 16 * j + 4 * q;
        if (m >= M) continue;
        f32x4 v;
        if (EPI == CONV_EPI_DSILU) {
          const f32x4 pv = *reinterpret_cast<const f32x4*>(pre + m * cout + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * dr_dsilu_fast(pv[e]);
        } else {
          const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bv[e];
          if (pre) *reinterpret_cast<f32x4*>(pre + m * cout + co) = v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = dr_silu_fast(v[e]);
        }
        if constexpr (IO16) {
          *reinterpret_cast<u32x2*>(out16 + m * cout + co) = pack_bf16x4(v);
          continue;
        }
        *reinterpret_cast<f32x4*>(out + m * cout + co) = v;
      }
    }
}

// Conv2d weight [co][ci][4][4] f32 -> bf16 [K/32 chunks][3 planes][co][32]
// (k = tap * cin + ci) with w = plane0 + plane1 + plane2 (split3): the BN rows
// of one chunk and plane are one contiguous run of whole 128-byte lines
__device__ __forceinline__ void conv_repack_split3_elem(int i, int cout, int cin, const float* __restrict__ w,
                                                        u16* __restrict__ wr) {
  const int co = i / (16 * cin), k = i - co * 16 * cin;
  const int tap = k / cin, ci = k - tap * cin;
  unsigned h, m, l;
  split3(w[((long long)co * cin + ci) * 16 + tap], h, m, l);
  const long long base = ((long long)(k >> 5) * 3 * cout + co) * 32 + (k & 31), plane = (long long)cout * 32;
  wr[base] = (u16)h;
  wr[base + plane] = (u16)m;
  wr[base + 2 * plane] = (u16)l;
}
__global__ void k_conv_repack_split3(int cout, int cin, const float* __restrict__ w, u16* __restrict__ wr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cout * 16 * cin) return;
  conv_repack_split3_elem(i, cout, cin, w, wr);
}

int op_conv_repack_split3(int cout, int cin, const float* w, void* wr, hipStream_t s) {
  const int total = cout * 16 * cin;
  hipLaunchKernelGGL(k_conv_repack_split3, dim3((total + 255) / 256), dim3(256), 0, s, cout, cin, w, (u16*)wr);
  return dr_check_launch("conv_repack_split3");
}

// ---------------------------------------------------------------------------
// conv1 + conv2 fused, f32-accurate (enc_f1 = 32 -> enc_f2 = 64, 64 x 64
// frames from the u8 replay ring; VariationalAutoEncoder.py:33-42 first two
// layers, input x/255 - 0.5 as Dreamer.py:251).  Removes the f32 conv1
// activation round trip through HBM (8192 frames: 1.07 GB written, 1.5 GB
// re-read by conv2).
//
// conv1 needs no split of its input: the centred pixel values x - 127.5 are
// exact in bf16 (8 significant bits), so x/255 - 0.5 = (x - 127.5) / 255 enters
// the MFMA as ONE bf16 term against the three split3 planes of the weights (3
// MFMAs per block), and the 1/255 is applied to the f32 sum.  The padding of
// the normalised input is 0 = x - 127.5 at x = 127.5: zero in the centred
// space too.  conv1's output (+ bias, SiLU) is split3 once, into three bf16
// planes in LDS, and conv2 runs the usual six split products from them.
//
// A workgroup (4 waves) owns R2 = 8 rows of conv2 output (128 pixels x 64
// channels, half a frame): it stages the RI = 38 input rows (bf16 [row][x+1][4
// ch], as k_enc12_bf16), computes the R1 = 18 conv1 rows they feed (2 rows
// recomputed per frame), then conv2 tap by tap with the tap's weight planes
// (12 KB) double-buffered through LDS.  Wave w: conv2 rows 4 (w & 1) .. + 3,
// channels 32 (w >> 1) .. + 31.
// LDS: conv1 planes [3][4 c8][PS] 16-byte units, PS = 18 * 32 + 1 (odd plane
// stride: the ds_read_b128 lane groups of a stride-2 pixel fragment fall on
// distinct bank quads, as in k_enc12_bf16), 110.8 KB; input rows 20 KB;
// weight ring 2 x 12 KB.  One workgroup per CU.
// ---------------------------------------------------------------------------
#define E12_R2 8
#define E12_R1 (2 * E12_R2 + 2)
#define E12_RI (2 * E12_R1 + 2)
#define E12_PS (E12_R1 * 32 + 1)
#define E12_LWI 66
static constexpr size_t e12_lds_bytes(int terms = 3) {
  return (size_t)terms * 4 * E12_PS * 16 + (size_t)E12_RI * E12_LWI * 8;
}

// NW = 8: two waves per SIMD -- waves 0-3 run conv2's taps 0-7 and waves 4-7
// taps 8-15 over the same 64 x 32 output blocks, the two partial sums meet in
// LDS (fixed order: taps 0-7 + taps 8-15) before the epilogue
// Optional saves for the world-model backward (NHWC f32, NULL = none): pre0 /
// a0 = conv1's pre-activation / output (the tile's own 16 conv1 rows), pre1 =
// conv2's pre-activation (out receives conv2's output as always).
// NTM = 1: the bf16 perf mode's form -- the weights' first plane (their RNE
// bf16) only, conv1's output rounded (RNE) to ONE bf16 plane in LDS, one MFMA
// per block, conv2's output written as bf16 NHWC (`out` then points at u16
// data); no saves.  One third of the LDS, so two workgroups fit per CU.
// one-term form (bf16 mode), measured at B = 256 (profiles/r03za_ab_enc12_s1.txt):
// 4 waves, two workgroups per CU (57 KB of LDS each; 164 VGPRs, no spill):
// encoder 0.936 ms; 8 waves at two workgroups per CU (128 VGPRs, 104 B spilled)
// 1.01-1.02 ms; 8 waves at one (165 VGPRs) 0.962 ms
#define DR_E12S1_WAVES 4  // waves per workgroup of the one-term form
#define DR_E12S1_OCC 2    // min waves per SIMD of the one-term form
// O16 = false with NTM = 1: the bf16 world-model step's form -- one term, f32
// output and the saves
template <int NW, int NTM = 3, bool O16 = (NTM == 1)>
__global__ __launch_bounds__(64 * NW, NTM == 1 ? DR_E12S1_OCC : 1) void k_enc12_split3(int n, int nb, dr_frames src, const u16* __restrict__ wr1,
                                                          const float* __restrict__ b1, const u16* __restrict__ wr2,
                                                          const float* __restrict__ b2, float* __restrict__ out,
                                                          float* __restrict__ pre0, float* __restrict__ a0,
                                                          float* __restrict__ pre1) {
  static_assert((NW == 4 || NW == 8) && (NTM == 1 || NTM == 3) && (!O16 || NTM == 1), "enc12 waves / terms");
  constexpr int NTH = 64 * NW, TAPS = NW == 8 ? 8 : 16;
  constexpr int R2 = E12_R2, R1 = E12_R1, RI = E12_RI, PS = E12_PS, LWI = E12_LWI;
  constexpr int OW1 = 32, OW2 = 16, W = 64, H = 64, C1 = 32, C2 = 64;
  extern __shared__ __attribute__((aligned(16))) u32x4 e12_smem[];
  u32x4* c1o = e12_smem;                                                       // [3][4][PS]
  uint2* xin = reinterpret_cast<uint2*>(e12_smem + NTM * 4 * PS);             // [RI][LWI]
  u16* xs = reinterpret_cast<u16*>(xin);
  u16* c1h = reinterpret_cast<u16*>(c1o);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;
  const int ntiles = 2 * n;
  int tile = blockIdx.x;
  if (tile >= ntiles) return;

  // ---- input rows: bf16 of the centred pixel values, [row][x + 1][4 ch] ----
  // columns 0 / LWI - 1 and channel slot 3 are zero padding, written once here;
  // every tile rewrites all other entries (zeros for rows outside the frame)
  for (int i = tid; i < RI * LWI; i += NTH) xin[i] = make_uint2(0u, 0u);
  constexpr int W4 = W / 4, PERC = RI * W4, MAXI = (3 * PERC + NTH - 1) / NTH;
  const unsigned hw = (unsigned)(H * W);
  const float centre = src.raw255 ? 127.5f : 0.0f, scale = src.raw255 ? 1.0f / 255.0f : 1.0f;
  unsigned uv[MAXI];
  auto in_load = [&](int tl) __attribute__((always_inline)) {
    const int f = tl >> 1, iy0 = 2 * (2 * (tl & 1) * R2 - 1) - 1;
    const int b = f % nb, t = f / nb + src.t0;
    const unsigned char* fr8 = src.ring + ((src.starts[b] + t) % src.ring_cap) * 3 * (long long)hw;
#pragma unroll
    for (int k = 0; k < MAXI; ++k) {
      const int i = tid + NTH * k;
      const int c = i / PERC, rem = i - c * PERC, rr = rem / W4, x4 = rem - rr * W4;
      const int y = iy0 + rr;
      const bool ok = i < 3 * PERC && y >= 0 && y < H;
      uv[k] = *reinterpret_cast<const unsigned*>(fr8 + (ok ? (unsigned)c * hw + (unsigned)(y * W + 4 * x4) : 0u));
    }
  };
  auto in_store = [&](int tl) __attribute__((always_inline)) {
    const int iy0 = 2 * (2 * (tl & 1) * R2 - 1) - 1;
#pragma unroll
    for (int k = 0; k < MAXI; ++k) {
      const int i = tid + NTH * k;
      if (i >= 3 * PERC) continue;
      const int c = i / PERC, rem = i - c * PERC, rr = rem / W4, x4 = rem - rr * W4;
      const int y = iy0 + rr;
      const bool ok = y >= 0 && y < H;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        xs[(rr * LWI + 4 * x4 + e + 1) * 4 + c] =
            ok ? b16bits((__bf16)((float)((uv[k] >> (8 * e)) & 255u) - centre)) : (u16)0;
    }
  };
  in_load(tile);
  __syncthreads();  // the zero fill before the stores of other threads
  in_store(tile);
  __syncthreads();

  const int w4 = wave & 3, kh = wave >> 2, ph = w4 & 1, ch = w4 >> 1;
  // conv2 weight fragments straight from L2 (the 196 KB of split planes stay
  // resident): lane (r, q) of wf[pl][jj] = row 32 ch + 16 jj + r, k 8 q .. + 7
  const u16* wbase = wr2 + ((long long)(32 * ch + r)) * 32 + 8 * q;
  auto wld = [&](u32x4 (&wf)[NTM][2], int tap) __attribute__((always_inline)) {
#pragma unroll
    for (int pl = 0; pl < NTM; ++pl)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
        wf[pl][jj] = *reinterpret_cast<const u32x4*>(wbase + ((long long)(tap * 3 + pl) * C2 + 16 * jj) * 32);
  };

  for (;;) {
    const int f = tile >> 1, y2_0 = (tile & 1) * R2, y1_0 = 2 * y2_0 - 1;
    const int next = tile + (int)gridDim.x;
    // conv1 weights (A operand: lane -> channel 16 j + r, k = 32 s + 8 q .. + 7), three
    // planes: re-read per tile (L2) so that they hold no registers during conv2
    u32x4 wa1[NTM][2][2];
#pragma unroll
    for (int pl = 0; pl < NTM; ++pl)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          wa1[pl][s][j] = *reinterpret_cast<const u32x4*>(wr1 + ((long long)pl * C1 + 16 * j + r) * 64 + 32 * s + 8 * q);
    float bb1[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) bb1[j][e] = b1[16 * j + 4 * q + e];
    u32x4 wfa[NTM][2], wfb[NTM][2];
    wld(wfa, TAPS * kh);
    // ---- conv1 over the R1 tile rows; rows outside the frame are conv2's zero padding ----
    constexpr int F1 = R1 * OW1 / 16;
    for (int i = wave; i < F1; i += NW) {
      const int p0 = 16 * i, yl = p0 / OW1, x1 = p0 - yl * OW1 + r, p = p0 + r;
      const int y1 = y1_0 + yl;
      uint2 hv[2], mv[2], lv[2];
      if (y1 < 0 || y1 >= H / 2) {
#pragma unroll
        for (int j = 0; j < 2; ++j) hv[j] = mv[j] = lv[j] = make_uint2(0u, 0u);
      } else {
        f32x4 acc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int t0 = 8 * s + 2 * q, ky = t0 >> 2, kx = t0 & 3;
          const u32x4 pb = *reinterpret_cast<const u32x4*>(&xin[(2 * yl + ky) * LWI + 2 * x1 + kx]);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int pl = NTM - 1; pl >= 0; --pl) acc[j] = mfma_b16(wa1[pl][s][j], pb, acc[j]);
          }
        }
        // lane: pixel p, channels 16 j + 4 q .. + 3
        const bool own = !O16 && pre0 && yl >= 1 && yl <= 2 * R2;  // this tile's own conv1 rows
        const long long o1 = (((long long)f * (H / 2) + y1) * OW1 + x1) * C1;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float v[4], pv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            pv[e] = acc[j][e] * scale + bb1[j][e];
            v[e] = dr_silu_fast(pv[e]);
          }
          if (own) {
            *reinterpret_cast<f32x4*>(pre0 + o1 + 16 * j + 4 * q) = (f32x4){pv[0], pv[1], pv[2], pv[3]};
            *reinterpret_cast<f32x4*>(a0 + o1 + 16 * j + 4 * q) = (f32x4){v[0], v[1], v[2], v[3]};
          }
          if constexpr (NTM == 1) {
            const u32x2 pk = pack_bf16x4((f32x4){v[0], v[1], v[2], v[3]});
            hv[j] = make_uint2(pk[0], pk[1]);
          } else {
            split3_pair(v[0], v[1], hv[j].x, mv[j].x, lv[j].x);
            split3_pair(v[2], v[3], hv[j].y, mv[j].y, lv[j].y);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c8 = 2 * j + (q >> 1);
        const int o = (c8 * PS + p) * 8 + (q & 1) * 4;  // u16 offset inside a plane
        *reinterpret_cast<uint2*>(c1h + o) = hv[j];
        if constexpr (NTM == 3) {
          *reinterpret_cast<uint2*>(c1h + 4 * PS * 8 + o) = mv[j];
          *reinterpret_cast<uint2*>(c1h + 2 * 4 * PS * 8 + o) = lv[j];
        }
      }
    }
    __syncthreads();
    // the next tile's input rows: loads in flight under conv2 (xin is free now)
    if (next < ntiles) in_load(next);

    // ---- conv2: K = 16 taps x 32 channels, one MFMA k-step per tap; c1o is
    // read-only here and the weights come from L2, so no barrier in the loop ----
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};
    auto tap_step = [&](int tap, u32x4 (&wf)[NTM][2], u32x4 (&wn)[NTM][2]) __attribute__((always_inline)) {
      wld(wn, tap + 1 < TAPS * (kh + 1) ? tap + 1 : tap);  // one tap ahead (the last reload is unused)
      const int ky = tap >> 2, kx = tap & 3;
      const int x1 = 2 * r - 1 + kx;
      const bool xok = x1 >= 0 && x1 < OW1;
      u32x4 pf[NTM][4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int yl = 2 * (4 * ph + i) + ky;
        const int u = q * PS + yl * OW1 + (xok ? x1 : 0);
#pragma unroll
        for (int pl = 0; pl < NTM; ++pl) {
          const u32x4 v = c1o[pl * 4 * PS + u];
          pf[pl][i] = xok ? v : (u32x4){0u, 0u, 0u, 0u};
        }
      }
      // smallest terms first (weight plane x activation plane)
#define E12_S3(PW, PA)                       \
  _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int jj = 0; jj < 2; ++jj) acc[i][jj] = \
      mfma_b16(wf[PW][jj], pf[PA][i], acc[i][jj]);
      if constexpr (NTM == 3) {
        E12_S3(2, 0)
        E12_S3(1, 1)
        E12_S3(0, 2)
        E12_S3(1, 0)
        E12_S3(0, 1)
      }
      E12_S3(0, 0)
#undef E12_S3
    };
#pragma unroll 1
    for (int tap = TAPS * kh; tap < TAPS * (kh + 1); ++tap) {
      tap_step(tap, wfa, wfb);
#pragma unroll
      for (int pl = 0; pl < NTM; ++pl)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) wfa[pl][jj] = wfb[pl][jj];
    }
    if (NW == 8) {
      // taps 8-15 partials through LDS (c1o is free once every wave is past conv2)
      f32x4* red = reinterpret_cast<f32x4*>(e12_smem);  // [4 waves][8 blocks][64 lanes]
      __syncthreads();
      if (kh == 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) red[(w4 * 8 + i * 2 + jj) * 64 + lane] = acc[i][jj];
      }
      __syncthreads();
      if (kh == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) acc[i][jj] += red[(w4 * 8 + i * 2 + jj) * 64 + lane];
      }
    }
    // lane (r, q) of acc[i][jj]: channels 32 ch + 16 jj + 4 q .. + 3 of conv2 pixel (row 4 ph + i, column r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (kh) break;
      float* o = out + (((long long)f * OW2 + y2_0 + 4 * ph + i) * OW2 + r) * C2;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int co = 32 * ch + 16 * jj + 4 * q;
        const f32x4 bv = *reinterpret_cast<const f32x4*>(b2 + co);
        f32x4 v;
        const f32x4 pv = acc[i][jj] + bv;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = dr_silu_fast(pv[e]);
        if constexpr (O16) {
          *reinterpret_cast<u32x2*>(reinterpret_cast<u16*>(out) + (o - out) + co) = pack_bf16x4(v);
          continue;
        }
        *reinterpret_cast<f32x4*>(o + co) = v;
        if (pre1) *reinterpret_cast<f32x4*>(pre1 + (o - out) + co) = pv;
      }
    }
    if (next >= ntiles) break;  // uniform over the workgroup: every wave leaves here
    in_store(next);
    __syncthreads();  // next input staged; every wave is past its conv2 reads of c1o
    tile = next;
  }
}

// conv1 weight [cout][3][4][4] f32 -> three bf16 planes [3][cout][64], k = tap * 4 + c (c = 3: zero)
__device__ __forceinline__ void conv1_repack_split3_elem(int i, int cout, const float* __restrict__ w,
                                                         u16* __restrict__ wr) {
  const int co = i >> 6, k = i & 63, tap = k >> 2, c = k & 3;
  unsigned h, m, l;
  split3(c < 3 ? w[((long long)co * 3 + c) * 16 + tap] : 0.f, h, m, l);
  wr[i] = (u16)h;
  wr[cout * 64 + i] = (u16)m;
  wr[2 * cout * 64 + i] = (u16)l;
}
__global__ void k_conv1_repack_split3(int cout, const float* __restrict__ w, u16* __restrict__ wr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cout * 64) return;
  conv1_repack_split3_elem(i, cout, w, wr);
}

bool op_enc12_split3_ok(int n, int h, int w, int c1, int c2, const dr_frames* src) {
  return c1 == 32 && c2 == 64 && h == 64 && w == 64 && src->ring && src->starts && src->ring_cap > 0 && n > 0 &&
         (long long)n * 2 < (1LL << 31);
}

int op_enc12_split3(int n, int nb, int h, int w, int c1, int c2, const dr_frames* src, const float* w1,
                    const float* b1, const float* w2, const float* b2, void* wr1, void* wr2, float* out,
                    hipStream_t s, int prepacked) {
  return op_enc12_split3_ex(n, nb, h, w, c1, c2, src, w1, b1, w2, b2, wr1, wr2, out, nullptr, nullptr, nullptr, s, 3,
                            prepacked);
}

int op_enc12_split3_ex(int n, int nb, int h, int w, int c1, int c2, const dr_frames* src, const float* w1,
                       const float* b1, const float* w2, const float* b2, void* wr1, void* wr2, float* out,
                       float* pre0, float* a0, float* pre1, hipStream_t s, int terms, int prepacked) {
  if ((pre0 != nullptr) != (a0 != nullptr) || ((uintptr_t)pre0 | (uintptr_t)a0 | (uintptr_t)pre1) & 15 ||
      (terms != 1 && terms != 3))
    return DR_E_INVALID;
  if (!op_enc12_split3_ok(n, h, w, c1, c2, src)) return DR_E_INVALID;
  static const bool raised = [] {
    (void)hipFuncSetAttribute((const void*)k_enc12_split3<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)e12_lds_bytes());
    (void)hipFuncSetAttribute((const void*)k_enc12_split3<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)e12_lds_bytes());
    return true;
  }();
  (void)raised;
  if (!prepacked) {
    hipLaunchKernelGGL(k_conv1_repack_split3, dim3((c1 * 64 + 255) / 256), dim3(256), 0, s, c1, w1, (u16*)wr1);
    DR_TRY(dr_check_launch("conv1_repack_split3"));
    DR_TRY(op_conv_repack_split3(c2, c1, w2, wr2, s));
  }
  if (terms == 1) {  // one term, f32 out + saves: the one-term form's occupancy (op_enc12_s1_bf16)
    static int slots1[64];
    int dev = 0;
    DR_TRY_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return DR_E_INVALID;
    auto kf = k_enc12_split3<DR_E12S1_WAVES, 1, false>;
    if (slots1[dev] == 0) {
      (void)hipFuncSetAttribute((const void*)kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)e12_lds_bytes(1));
      int cus = 0, per = 0;
      DR_TRY_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      DR_TRY_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kf, 64 * DR_E12S1_WAVES, e12_lds_bytes(1)));
      slots1[dev] = std::max(1, per) * std::max(1, cus);
    }
    const int grid = std::min(n * 2, slots1[dev]);
    hipLaunchKernelGGL(kf, dim3((unsigned)grid), dim3(64 * DR_E12S1_WAVES), e12_lds_bytes(1), s, n, nb, *src,
                       (const u16*)wr1, b1, (const u16*)wr2, b2, out, pre0, a0, pre1);
    return dr_check_launch("enc12_split3 (one term)");
  }
  // persistent: one workgroup per CU (the LDS allows no second), each walks
  // tiles blockIdx.x, + gridDim.x, ... so that its next tile's input loads
  // run under the current tile's conv2
  static int cus[64];
  int dev = 0;
  DR_TRY_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return DR_E_INVALID;
  if (cus[dev] == 0) DR_TRY_HIP(hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = std::min(n * 2, std::max(1, cus[dev]));
  // 8 waves (two per SIMD); one wave per SIMD measured 517.0 k against 532.9 k (r03o)
  hipLaunchKernelGGL(k_enc12_split3<8>, dim3((unsigned)grid), dim3(512), e12_lds_bytes(), s, n, nb, *src,
                     (const u16*)wr1, b1, (const u16*)wr2, b2, out, pre0, a0, pre1);
  return dr_check_launch("enc12_split3");
}

// bf16 perf mode: k_enc12_split3<DR_E12S1_WAVES, 1> (one bf16 term; out = bf16 NHWC).
// wr1 / wr2 are the split3 repack slots (c1 * 64 * 6 and c2 * c1 * 16 * 6
// bytes; plane 0 is read).  DR_E_INVALID (nothing launched) for other shapes.
int op_enc12_s1_bf16(int n, int nb, int h, int w, int c1, int c2, const dr_frames* src, const float* w1,
                     const float* b1, const float* w2, const float* b2, void* wr1, void* wr2, void* out,
                     hipStream_t s, int prepacked) {
  if (!op_enc12_split3_ok(n, h, w, c1, c2, src) || ((uintptr_t)out & 15)) return DR_E_INVALID;
  // persistent: as many workgroups as are resident at once (occupancy x CUs)
  static int slots[64];
  int dev = 0;
  DR_TRY_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return DR_E_INVALID;
  if (slots[dev] == 0) {
    (void)hipFuncSetAttribute((const void*)k_enc12_split3<DR_E12S1_WAVES, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)e12_lds_bytes(1));
    int cus = 0, per = 0;
    DR_TRY_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    DR_TRY_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_enc12_split3<DR_E12S1_WAVES, 1>,
                                                            64 * DR_E12S1_WAVES, e12_lds_bytes(1)));
    slots[dev] = std::max(1, per) * std::max(1, cus);
  }
  if (!prepacked) {
    hipLaunchKernelGGL(k_conv1_repack_split3, dim3((c1 * 64 + 255) / 256), dim3(256), 0, s, c1, w1, (u16*)wr1);
    DR_TRY(dr_check_launch("conv1_repack_split3"));
    DR_TRY(op_conv_repack_split3(c2, c1, w2, wr2, s));
  }
  const int grid = std::min(n * 2, slots[dev]);
  hipLaunchKernelGGL((k_enc12_split3<DR_E12S1_WAVES, 1>), dim3((unsigned)grid), dim3(64 * DR_E12S1_WAVES),
                     e12_lds_bytes(1), s, n, nb, *src,
                     (const u16*)wr1, b1, (const u16*)wr2, b2, (float*)out, nullptr, nullptr, nullptr);
  return dr_check_launch("enc12_s1_bf16");
}

template <int BM, int BN, int CIN, bool NCHW, int PIPE, int EPI = CONV_EPI_FWD, int TERMS = 3>
static int launch_s3(int n, int ih, int iw, int cout, const float* in, const void* wr, const float* bias, float* out,
                     float* pre, hipStream_t s) {
  const long long M = (long long)n * (ih / 2) * (iw / 2);
  const long long tiles = ((M + BM - 1) / BM) * (cout / BN);
  if (tiles >= (1LL << 30)) {
    dr_set_error("conv_split3: too many tiles");
    return DR_E_INVALID;
  }
  hipLaunchKernelGGL((k_conv_split3<BM, BN, CIN, NCHW, PIPE, EPI, TERMS, false>), dim3((unsigned)dr_xcd_grid((int)tiles)),
                     dim3(BM * 2), 0, s, n, ih, iw, cout, in, (const u16*)wr, bias, out, pre);
  return dr_check_launch("conv_split3");
}

bool op_conv_split3_supported(int n, int cin, int ih, int iw, int cout) {
  const bool cin_ok = cin == 32 || cin == 64 || cin == 128 || cin == 256;
  return cin_ok && cout % 64 == 0 && ih % 2 == 0 && iw % 2 == 0 && ((ih / 2) * (iw / 2)) % 4 == 0 &&
         (long long)n * ih * iw * cin < (1LL << 31) - (1LL << 20);
}

int op_conv_split3_ex(int n, int cin, int ih, int iw, int cout, const float* in, const void* wr, const float* bias,
                      float* out, int out_nchw, float* pre, int epi, hipStream_t s, int terms) {
  if (!op_conv_split3_supported(n, cin, ih, iw, cout) || (terms != 1 && terms != 3)) {
    dr_set_error("conv_split3: unsupported shape (cin=%d ih=%d iw=%d cout=%d)", cin, ih, iw, cout);
    return DR_E_INVALID;
  }
  if (epi == CONV_EPI_DSILU && (out_nchw || !pre)) {
    dr_set_error("conv_split3: the SiLU-backward epilogue needs NHWC output and a pre-activation tensor");
    return DR_E_INVALID;
  }
  // six products: the LDS-DMA ping-pong kernel (conv_glds.hip) where it applies
  if (terms == 3 && (epi == CONV_EPI_FWD ? bias != nullptr : pre != nullptr) && op_conv_glds_s3_supported(n, cin, ih, iw, cout) &&
      !(((uintptr_t)in | (uintptr_t)wr | (uintptr_t)out | (uintptr_t)bias | (uintptr_t)pre) & 15))
    return op_conv_glds_s3(n, cin, ih, iw, cout, in, wr, bias, out, out_nchw, pre, epi, s);
  // measured at 8192 frames (tools/conv_ab.py): 256 x 64 tiles
  // for 64 output channels (980 us; 128 x 64 at two workgroups per CU: 1004),
  // 256 x 128 for 128 / 256 channels (709 / 658 us; 128 x 128: ~1.1 ms): the
  // weights are re-read once per pixel tile, so taller tiles pay
#define DR_S3E(BN, C, NCHW, T)                                                                                         \
  (epi == CONV_EPI_DSILU ? launch_s3<256, BN, C, NCHW, 2, CONV_EPI_DSILU, T>(n, ih, iw, cout, in, wr, bias, out, pre, s) \
                         : launch_s3<256, BN, C, NCHW, 2, CONV_EPI_FWD, T>(n, ih, iw, cout, in, wr, bias, out, pre, s))
#define DR_S3L(C, T)                                                                                                 \
  if (cin == C) {                                                                                                    \
    if (cout % 128 == 0)                                                                                             \
      return out_nchw ? launch_s3<256, 128, C, true, 2, CONV_EPI_FWD, T>(n, ih, iw, cout, in, wr, bias, out, pre, s) \
                      : DR_S3E(128, C, false, T);                                                                    \
    return out_nchw ? launch_s3<256, 64, C, true, 2, CONV_EPI_FWD, T>(n, ih, iw, cout, in, wr, bias, out, pre, s)    \
                    : DR_S3E(64, C, false, T);                                                                       \
  }
  if (terms == 1) {
    DR_S3L(32, 1)
    DR_S3L(64, 1)
    DR_S3L(128, 1)
    DR_S3L(256, 1)
  } else {
    DR_S3L(32, 3)
    DR_S3L(64, 3)
    DR_S3L(128, 3)
    DR_S3L(256, 3)
  }
#undef DR_S3L
#undef DR_S3E
  return DR_E_INVALID;
}

int op_conv_split3(int n, int cin, int ih, int iw, int cout, const float* in, const void* wr, const float* bias,
                   float* out, int out_nchw, hipStream_t s) {
  return op_conv_split3_ex(n, cin, ih, iw, cout, in, wr, bias, out, out_nchw, nullptr, CONV_EPI_FWD, s);
}

// bf16 perf mode: the same tiling with one term (k_conv_split3<..., NT3 = 1>):
// bf16 NHWC in, bf16 NHWC / NCHW out, weights as op_conv_repack_split3 planes
// (plane 0 read).  Replaces k_conv_bf16 for conv3.. (its 128 x 128 tiles ran
// at 0.16 of the bf16 peak).
template <int BN, int C, bool NCHW>
static int launch_s1(int n, int ih, int iw, int cout, const void* in, const void* wr, const float* bias, void* out,
                     hipStream_t s) {
  const long long M = (long long)n * (ih / 2) * (iw / 2);
  const long long tiles = ((M + 255) / 256) * (cout / BN);
  if (tiles >= (1LL << 30)) {
    dr_set_error("conv_s1_bf16: too many tiles");
    return DR_E_INVALID;
  }
  hipLaunchKernelGGL((k_conv_split3<256, BN, C, NCHW, 2, CONV_EPI_FWD, 1>), dim3((unsigned)dr_xcd_grid((int)tiles)),
                     dim3(512), 0, s, n, ih, iw, cout, (const float*)in, (const u16*)wr, bias, (float*)out, nullptr);
  return dr_check_launch("conv_s1_bf16");
}

int op_conv_s1_bf16(int n, int cin, int ih, int iw, int cout, const void* in, const void* wr, const float* bias,
                    void* out, int out_nchw, hipStream_t s) {
  if (!op_conv_split3_supported(n, cin, ih, iw, cout) || (((uintptr_t)in | (uintptr_t)out | (uintptr_t)bias) & 15)) {
    dr_set_error("conv_s1_bf16: unsupported shape (cin=%d ih=%d iw=%d cout=%d)", cin, ih, iw, cout);
    return DR_E_INVALID;
  }
  if (op_conv_glds_bf16_supported(n, cin, ih, iw, cout))
    return op_conv_glds_bf16(n, cin, ih, iw, cout, in, wr, bias, out, out_nchw, s);
#define DR_S1L(C)                                                                              \
  if (cin == C) {                                                                              \
    if (cout % 128 == 0)                                                                       \
      return out_nchw ? launch_s1<128, C, true>(n, ih, iw, cout, in, wr, bias, out, s)         \
                      : launch_s1<128, C, false>(n, ih, iw, cout, in, wr, bias, out, s);       \
    return out_nchw ? launch_s1<64, C, true>(n, ih, iw, cout, in, wr, bias, out, s)            \
                    : launch_s1<64, C, false>(n, ih, iw, cout, in, wr, bias, out, s);          \
  }
  DR_S1L(32)
  DR_S1L(64)
  DR_S1L(128)
  DR_S1L(256)
#undef DR_S1L
  return DR_E_INVALID;
}

// ---------------------------------------------------------------------------
// Upsampling k4 s2 p1 (ConvTranspose2d of the decoder, VAE.py:128-137, and the
// data gradient of an encoder Conv2d), f32-accurate on the bf16 MFMA: the
// implicit GEMM of wmconv.hip's k_convT_nhwc -- per output parity class
// (py, px) a dense K = 4 taps x CIN, tap (dy, dx): input (y + py - dy,
// x + px - dx), kernel (1 - py + 2 dy, 1 - px + 2 dx) -- with the operands of
// k_conv_split3: activations split3 as they are staged (truncation split,
// v_perm packing, swizzled 64-byte plane rows), weights split once per call
// into [class][K/32][3 planes][cout][32].  Epilogues of the world-model step
// (NHWC out, ldc == cout): CT_EPI_BIAS (out = acc + bias, out2 / silu_out =
// SiLU) and CT_EPI_DSILU (out = acc * SiLU'(pre)).  TERMS = 1: the bf16
// world-model step's form (activations RNE-rounded to one bf16 plane while
// staged, weight plane 0, one MFMA per block).
// ---------------------------------------------------------------------------
template <int BM, int BN, int CIN, int EPI, int TERMS = 3>
__global__ __launch_bounds__(BM * 2) void k_convT_split3(ConvTArgs a, const u16* __restrict__ wr) {
  constexpr int NT = BM * 2;
  constexpr int K = CIN * 4;
  constexpr int NCH = K / 32;
  constexpr int WTN = BN / 2, FM = 4, FN = WTN / 16;
  constexpr int APT = BM * 8 / NT;
  constexpr int BU = TERMS * BN * 4;
  constexpr int BPT = (BU + NT - 1) / NT;
  static_assert(CIN % 32 == 0 && APT == 4 && FN >= 1 && NCH % 2 == 0 && (TERMS == 1 || TERMS == 3),
                "convT_split3 tile");
  __shared__ __attribute__((aligned(16))) u32x4 As[2][TERMS][BM][4];
  __shared__ __attribute__((aligned(16))) u32x4 Bs[2][TERMS][BN][4];

  const int h = a.h, w = a.w, hw = h * w, cout = a.cout;
  const long long M = (long long)a.n * hw;  // input-resolution pixels of one parity class
  const int tiles_n = cout / BN;
  const long long tiles_m = (M + BM - 1) / BM;
  const int lt = dr_xcd_tile(blockIdx.x, (int)(4 * tiles_m * tiles_n));
  if (lt < 0) return;
  // parity class fastest: the four classes of one pixel tile read the same
  // input, and adjacent logical tiles share an XCD (dr_xcd_tile), so that
  // input comes from HBM about once (class-major order sent each class to
  // other XCDs: four HBM reads, one per L2)
  const int cls = lt & 3;
  const long long rem = lt >> 2;
  const long long m0 = (rem / tiles_n) * BM;
  const int n0 = (int)(rem % tiles_n) * BN;
  const int py = cls >> 1, px = cls & 1;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;
  const int quad = tid & 7, prow = tid >> 3;
  const float* __restrict__ in = a.in;
  const u16* __restrict__ wc = wr + (long long)cls * NCH * 3 * cout * 32;

  // per A row: element offset of input pixel (y, x) (32-bit: n h w CIN < 2^31,
  // host-checked) and the valid taps (bit dy * 2 + dx); rows past M: none
  int pb[APT];
  unsigned vm[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const long long m = m0 + prow + (NT / 8) * i;
    const int mm = (int)(m < M ? m : 0);
    const int f = mm / hw, p = mm - f * hw, y = p / w, x = p - y * w;
    pb[i] = ((f * h + y) * w + x) * CIN;
    unsigned v = 0u;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int iy = y + py - (t >> 1), ix = x + px - (t & 1);
      v |= (iy >= 0 && iy < h && ix >= 0 && ix < w) ? (1u << t) : 0u;
    }
    vm[i] = m < M ? v : 0u;
  }

  f32x4 ra0[APT], ra1[APT];
  u32x4 rb0[BPT], rb1[BPT];
  unsigned ok0 = 0, ok1 = 0;
  auto load = [&](int c, auto slot) __attribute__((always_inline)) {
    f32x4* ra = decltype(slot)::value == 0 ? ra0 : ra1;
    unsigned& okm = decltype(slot)::value == 0 ? ok0 : ok1;
    u32x4* rb = decltype(slot)::value == 0 ? rb0 : rb1;
    const int tap = (32 * c) / CIN, ci0 = 32 * c - tap * CIN;
    const int toff = ((py - (tap >> 1)) * w + (px - (tap & 1))) * CIN + ci0 + 4 * quad;
    unsigned om = 0u;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const bool ok = (vm[i] >> tap) & 1u;
      ra[i] = *reinterpret_cast<const f32x4*>(in + (ok ? pb[i] + toff : 0));
      om |= ok ? (1u << i) : 0u;
    }
    okm = om;
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int e = tid + NT * j;
      if (BU % NT == 0 || e < BU) {
        const int pl = e / (BN * 4), rm = e - pl * BN * 4, row = rm >> 2, u = rm & 3;
        rb[j] = *reinterpret_cast<const u32x4*>(wc + (((long long)c * 3 + pl) * cout + n0 + row) * 32 + 8 * u);
      }
    }
  };
  auto store = [&](auto slot, int buf) __attribute__((always_inline)) {
    const f32x4* ra = decltype(slot)::value == 0 ? ra0 : ra1;
    const u32x4* rb = decltype(slot)::value == 0 ? rb0 : rb1;
    const unsigned okm = decltype(slot)::value == 0 ? ok0 : ok1;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int row = prow + (NT / 8) * i;
      const f32x4 v = (okm >> i) & 1u ? ra[i] : (f32x4){0.f, 0.f, 0.f, 0.f};
      const int unit = (quad >> 1) ^ swz(row), half = quad & 1;
      if constexpr (TERMS == 1) {
        reinterpret_cast<u32x2*>(&As[buf][0][row][unit])[half] = pack_bf16x4(v);
      } else {
        unsigned h0, m0_, l0, h1, m1, l1;
        split3_pair(v[0], v[1], h0, m0_, l0);
        split3_pair(v[2], v[3], h1, m1, l1);
        reinterpret_cast<u32x2*>(&As[buf][0][row][unit])[half] = (u32x2){h0, h1};
        reinterpret_cast<u32x2*>(&As[buf][1][row][unit])[half] = (u32x2){m0_, m1};
        reinterpret_cast<u32x2*>(&As[buf][2][row][unit])[half] = (u32x2){l0, l1};
      }
    }
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int e = tid + NT * j;
      if (BU % NT == 0 || e < BU) {
        const int pl = e / (BN * 4), rm = e - pl * BN * 4, row = rm >> 2, u = rm & 3;
        Bs[buf][pl][row][u ^ swz(row)] = rb[j];
      }
    }
  };

  const int wm0 = (wave >> 1) * 64, wn0 = (wave & 1) * WTN;
  const int fu = q ^ swz(r);
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  load(0, S0{});
  load(1, S1{});
  store(S0{}, 0);
  __syncthreads();
  auto step = [&](int c, auto slot) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot)::value;
    using Next = std::integral_constant<int, 1 - SL>;
    const int buf = c & 1;
    load(min(c + 2, NCH - 1), slot);
    u32x4 av[TERMS][FM], bv[TERMS][FN];
#pragma unroll
    for (int pl = 0; pl < TERMS; ++pl) {
#pragma unroll
      for (int i = 0; i < FM; ++i) av[pl][i] = As[buf][pl][wm0 + 16 * i + r][fu];
#pragma unroll
      for (int j = 0; j < FN; ++j) bv[pl][j] = Bs[buf][pl][wn0 + 16 * j + r][fu];
    }
    // weights as the MFMA A operand (lane: 4 consecutive channels of one pixel)
#define DR_T3(PA, PB)                                                                                   \
  _Pragma("unroll") for (int i = 0; i < FM; ++i) _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[i][j] = \
      mfma_b16(bv[PB][j], av[PA][i], acc[i][j]);
    if constexpr (TERMS == 3) {
      DR_T3(2, 0)
      DR_T3(1, 1)
      DR_T3(0, 2)
      DR_T3(1, 0)
      DR_T3(0, 1)
    }
    DR_T3(0, 0)
#undef DR_T3
    if (c + 1 < NCH) store(Next{}, buf ^ 1);
    dr_lds_barrier();
  };
  for (int c = 0; c < NCH; c += 2) {
    step(c, S0{});
    step(c + 1, S1{});
  }

  const int OW = 2 * w, OH = 2 * h;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const long long m = m0 + wm0 + 16 * i + r;
    if (m >= M) continue;
    const int f = (int)(m / hw), p = (int)(m - (long long)f * hw), y = p / w, x = p - y * w;
    const long long opix = ((long long)f * OH + 2 * y + py) * OW + 2 * x + px;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int co = n0 + wn0 + 16 * j + 4 * q;
      f32x4 v = acc[i][j];
      if (EPI == CT_EPI_BIAS) {
        v += *reinterpret_cast<const f32x4*>(a.bias + co);
        f32x4 sv = v;
        if (a.out2 || a.silu_out) {
#pragma unroll
          for (int e = 0; e < 4; ++e) sv[e] = dr_silu_fast(v[e]);
        }
        *reinterpret_cast<f32x4*>(a.out + opix * cout + co) = a.silu_out ? sv : v;
        if (a.out2) *reinterpret_cast<f32x4*>(a.out2 + opix * cout + co) = sv;
      } else {
        const f32x4 pv = *reinterpret_cast<const f32x4*>(a.pre + opix * cout + co);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] * dr_dsilu_fast(pv[e]);
        *reinterpret_cast<f32x4*>(a.out + opix * cout + co) = v;
      }
    }
  }
}

// ConvTranspose2d weight [cin][cout][4][4] (or a Conv2d weight [co][ci][4][4]
// read as [cin = co][cout = ci]) -> bf16 [class][K/32][3 planes][cout][32],
// k = tap * cin + ci, tap = dy * 2 + dx
__global__ void k_convT_repack_split3(int cin, int cout, const float* __restrict__ wt, u16* __restrict__ wr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int K = 4 * cin;
  if (i >= 4 * cout * K) return;
  const int cls = i / (cout * K), rm = i - cls * cout * K, co = rm / K, k = rm - co * K;
  const int tap = k / cin, ci = k - tap * cin;
  const int py = cls >> 1, px = cls & 1, ky = 1 - py + 2 * (tap >> 1), kx = 1 - px + 2 * (tap & 1);
  unsigned hh, mm, ll;
  split3(wt[(((long long)ci * cout + co) * 4 + ky) * 4 + kx], hh, mm, ll);
  const long long plane = (long long)cout * 32;
  const long long base = (((long long)cls * (K / 32) + (k >> 5)) * 3 * cout + co) * 32 + (k & 31);
  wr[base] = (u16)hh;
  wr[base + plane] = (u16)mm;
  wr[base + 2 * plane] = (u16)ll;
}

int op_convT_repack_split3(int cin, int cout, const float* wt, void* wr, hipStream_t s) {
  const int total = 16 * cout * cin;
  hipLaunchKernelGGL(k_convT_repack_split3, dim3((total + 255) / 256), dim3(256), 0, s, cin, cout, wt, (u16*)wr);
  return dr_check_launch("convT_repack_split3");
}

// ---------------------------------------------------------------------------
// All four parity classes of a 64 -> 32-channel upsampling conv in one
// workgroup (the decoder's ConvTranspose2d(64, 32) at 16x16 -> 32x32,
// VAE.py:131-133, and the data gradient of the encoder's Conv2d(32, 64),
// VAE.py:37-38).  The per-class kernels stage an im2col row per (class, tap):
// every input element is fetched and split 16 times, and at 32 output channels
// that staging outweighs the MFMAs (k_convT_nhwc: 790 / 950 us at B = 256
// T = 15 on the f32 MFMA, 5.5 VALU per MFMA; k_convT_split3<.., 32, 64, ., 1>:
// 365 / 450 us).  Here a workgroup owns 8 x 16 input anchors of one frame: it
// stages their (8 + 2) x (16 + 2) x 64 input patch ONCE -- split3 (or RNE
// bf16) into LDS planes, pixel rows of 144 bytes (64 bf16 + 16 bytes of pad:
// the 16 pixels of a fragment read land on distinct bank quads) -- and wave w
// computes parity class w (py, px) = (w >> 1, w & 1) for all 128 anchors and
// 32 output channels: per tap (dy, dx) and 32-channel chunk, 8 anchor-row
// fragments read straight from the patch at offset (py - dy, px - dx), the
// weight fragments (op_convT_repack_split3 planes, class-major) from L2, one
// tap-chunk ahead in registers.  Products per chunk in k_convT_split3's order
// (six for TERMS = 3, f32-accurate; one for TERMS = 1).  WM step B = 256 T = 15:
// fp32 13.67 -> 12.71 ms (the two layers 790 / 952 -> ~360 / 410 us), bf16
// 9.18 -> 8.80 ms (365 / 450 -> ~240 / 267 us; the data-gradient form moves
// 1.24 GB of input / pre-activation / output: HBM-bound), profiles/r06n_*.
// ---------------------------------------------------------------------------
constexpr int CC_TY = 8, CC_TX = 16, CC_PH = CC_TY + 2, CC_PW = CC_TX + 2, CC_PIX = CC_PH * CC_PW;
constexpr int CC_ROWB = 144;  // bytes per staged pixel: 64 bf16 + 16 pad

template <int EPI, int TERMS>
__global__ __launch_bounds__(256) void k_convT_cls(ConvTArgs a, const u16* __restrict__ wr) {
  constexpr int CIN = 64, COUT = 32, K = 4 * CIN, KCH = K / 32;
  constexpr int PLANE = CC_PIX * CC_ROWB;
  __shared__ __attribute__((aligned(16))) unsigned char sp[TERMS * PLANE];
  const int h = a.h, w = a.w;
  const int tiles_y = h / CC_TY, tiles_x = w / CC_TX;
  const long long tiles = (long long)a.n * tiles_y * tiles_x;
  const int lt = dr_xcd_tile(blockIdx.x, (int)tiles);
  if (lt < 0) return;
  const int f = lt / (tiles_y * tiles_x), rem = lt - f * tiles_y * tiles_x;
  const int y0 = (rem / tiles_x) * CC_TY, x0 = (rem % tiles_x) * CC_TX;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;

  // ---- stage the input patch once: unit = (pixel, 8 channels) ----
  constexpr int UNITS = CC_PIX * 8, UPT = (UNITS + 255) / 256;
  const float* __restrict__ in = a.in + (long long)f * h * w * CIN;
  f32x4 v[UPT][2];
#pragma unroll
  for (int j = 0; j < UPT; ++j) {
    const int u = tid + 256 * j, pix = u >> 3, g = u & 7;
    const int iy = y0 - 1 + pix / CC_PW, ix = x0 - 1 + pix % CC_PW;
    const bool ok = u < UNITS && iy >= 0 && iy < h && ix >= 0 && ix < w;
    const float* src = in + (ok ? ((long long)iy * w + ix) * CIN + 8 * g : 0);
    const f32x4 t0 = *reinterpret_cast<const f32x4*>(src), t1 = *reinterpret_cast<const f32x4*>(src + 4);
    v[j][0] = ok ? t0 : (f32x4){0.f, 0.f, 0.f, 0.f};
    v[j][1] = ok ? t1 : (f32x4){0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int j = 0; j < UPT; ++j) {
    const int u = tid + 256 * j, pix = u >> 3, g = u & 7;
    if (u >= UNITS) continue;
    unsigned char* dst = sp + pix * CC_ROWB + 16 * g;
    if constexpr (TERMS == 1) {
      const u32x4 hv = {pack_bf16x2(v[j][0][0], v[j][0][1]), pack_bf16x2(v[j][0][2], v[j][0][3]),
                        pack_bf16x2(v[j][1][0], v[j][1][1]), pack_bf16x2(v[j][1][2], v[j][1][3])};
      *reinterpret_cast<u32x4*>(dst) = hv;
    } else {
      unsigned hh[4], mm[4], ll[4];
      split3_pair(v[j][0][0], v[j][0][1], hh[0], mm[0], ll[0]);
      split3_pair(v[j][0][2], v[j][0][3], hh[1], mm[1], ll[1]);
      split3_pair(v[j][1][0], v[j][1][1], hh[2], mm[2], ll[2]);
      split3_pair(v[j][1][2], v[j][1][3], hh[3], mm[3], ll[3]);
      *reinterpret_cast<u32x4*>(dst) = (u32x4){hh[0], hh[1], hh[2], hh[3]};
      *reinterpret_cast<u32x4*>(dst + PLANE) = (u32x4){mm[0], mm[1], mm[2], mm[3]};
      *reinterpret_cast<u32x4*>(dst + 2 * PLANE) = (u32x4){ll[0], ll[1], ll[2], ll[3]};
    }
  }
  __syncthreads();

  // ---- wave = parity class ----
  const int cls = wave, py = cls >> 1, px = cls & 1;
  const u16* __restrict__ wc = wr + (long long)cls * KCH * 3 * COUT * 32;
  f32x4 acc[CC_TY][2];
#pragma unroll
  for (int i = 0; i < CC_TY; ++i) acc[i][0] = acc[i][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  u32x4 bw[2][TERMS][2];
  auto loadb = [&](int kc, int sl) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < TERMS; ++p)
#pragma unroll
      for (int jn = 0; jn < 2; ++jn)
        bw[sl][p][jn] =
            *reinterpret_cast<const u32x4*>(wc + ((long long)(kc * 3 + p) * COUT + 16 * jn + r) * 32 + 8 * q);
  };
  loadb(0, 0);
#pragma unroll
  for (int kc = 0; kc < KCH; ++kc) {  // k = 32 kc: tap = kc / 2, channels 32 (kc % 2) ..
    const int sl = kc & 1;
    if (kc + 1 < KCH) loadb(kc + 1, sl ^ 1);
    const int tap = kc >> 1, dy = tap >> 1, dx = tap & 1, c0 = 32 * (kc & 1);
    // anchor (y0 + i, x0 + r) reads input (y + py - dy, x + px - dx) = patch (i + 1 + py - dy, r + 1 + px - dx)
    const unsigned char* pa = sp + ((1 + py - dy) * CC_PW + (r + 1 + px - dx)) * CC_ROWB + 2 * (c0 + 8 * q);
#pragma unroll
    for (int i = 0; i < CC_TY; ++i) {
      u32x4 av[TERMS];
#pragma unroll
      for (int p = 0; p < TERMS; ++p)
        av[p] = *reinterpret_cast<const u32x4*>(pa + p * PLANE + i * CC_PW * CC_ROWB);
#define DR_CC(PA, PB)                                                                   \
  _Pragma("unroll") for (int jn = 0; jn < 2; ++jn) acc[i][jn] = mfma_b16(bw[sl][PB][jn], av[PA], acc[i][jn]);
      if constexpr (TERMS == 3) {
        DR_CC(2, 0)
        DR_CC(1, 1)
        DR_CC(0, 2)
        DR_CC(1, 0)
        DR_CC(0, 1)
      }
      DR_CC(0, 0)
#undef DR_CC
    }
  }

  // ---- epilogue: lane (r, q) of acc[i][jn] = anchor (y0 + i, x0 + r), channels 16 jn + 4 q .. + 3 ----
  const int OH = 2 * h, OW = 2 * w;
#pragma unroll
  for (int i = 0; i < CC_TY; ++i) {
    const long long opix = ((long long)f * OH + 2 * (y0 + i) + py) * OW + 2 * (x0 + r) + px;
#pragma unroll
    for (int jn = 0; jn < 2; ++jn) {
      const int co = 16 * jn + 4 * q;
      f32x4 val = acc[i][jn];
      if (EPI == CT_EPI_BIAS) {
        val += *reinterpret_cast<const f32x4*>(a.bias + co);
        f32x4 sv = val;
        if (a.out2 || a.silu_out) {
#pragma unroll
          for (int e = 0; e < 4; ++e) sv[e] = dr_silu_fast(val[e]);
        }
        *reinterpret_cast<f32x4*>(a.out + opix * COUT + co) = a.silu_out ? sv : val;
        if (a.out2) *reinterpret_cast<f32x4*>(a.out2 + opix * COUT + co) = sv;
      } else {
        const f32x4 pv = *reinterpret_cast<const f32x4*>(a.pre + opix * COUT + co);
#pragma unroll
        for (int e = 0; e < 4; ++e) val[e] = val[e] * dr_dsilu_fast(pv[e]);
        *reinterpret_cast<f32x4*>(a.out + opix * COUT + co) = val;
      }
    }
  }
}

bool op_convT_cls_supported(int n, int cin, int h, int w, int cout) {
  return cin == 64 && cout == 32 && n > 0 && h % CC_TY == 0 && w % CC_TX == 0 &&
         (long long)n * h * w * cin < (1LL << 31) - (1LL << 20) && (long long)n * (h / CC_TY) * (w / CC_TX) < (1LL << 30);
}

static int launch_convT_cls(int epi, const ConvTArgs& a, const void* wr, hipStream_t s, int terms) {
  const long long tiles = (long long)a.n * (a.h / CC_TY) * (a.w / CC_TX);
  const dim3 grid((unsigned)dr_xcd_grid((int)tiles));
#define DR_CCL(E, T) hipLaunchKernelGGL((k_convT_cls<E, T>), grid, dim3(256), 0, s, a, (const u16*)wr)
  if (epi == CT_EPI_DSILU) {
    if (terms == 1) DR_CCL(CT_EPI_DSILU, 1);
    else DR_CCL(CT_EPI_DSILU, 3);
  } else {
    if (terms == 1) DR_CCL(CT_EPI_BIAS, 1);
    else DR_CCL(CT_EPI_BIAS, 3);
  }
#undef DR_CCL
  return dr_check_launch("convT_cls");
}

// cout >= 64: at 32 output channels the 256 x 32 tile's split of the staged
// activations outweighs its 24 MFMAs per wave and chunk (975 / 887 us against
// 991 / 900 us on the f32 MFMA, WM step B = 256 T = 15, profiles/r03i_wm_step_kernels.txt)
// (one term: the split's cost is gone, so cout = 32 takes the 256 x 32 tile)
bool op_convT_split3_supported(int n, int cin, int h, int w, int cout, int terms) {
  if ((terms == 1 || terms == 3) && op_convT_cls_supported(n, cin, h, w, cout)) return true;
  const bool cin_ok = cin == 32 || cin == 64 || cin == 128 || cin == 256;
  return cin_ok && (terms == 1 || terms == 3) && cout % (terms == 1 ? 32 : 64) == 0 && cout > 0 &&
         (long long)n * h * w * cin < (1LL << 31) - (1LL << 20) &&
         4LL * (((long long)n * h * w + 255) / 256) * (cout / 32) < (1LL << 30);
}

template <int BN, int C, int EPI, int T>
static int launch_t3(const ConvTArgs& a, const void* wr, hipStream_t s) {
  const long long tiles = 4 * (((long long)a.n * a.h * a.w + 255) / 256) * (a.cout / BN);
  hipLaunchKernelGGL((k_convT_split3<256, BN, C, EPI, T>), dim3((unsigned)dr_xcd_grid((int)tiles)), dim3(512), 0, s,
                     a, (const u16*)wr);
  return dr_check_launch("convT_split3");
}

int op_convT_split3(int epi, const ConvTArgs& a, const void* wr, hipStream_t s, int terms) {
  if (!op_convT_split3_supported(a.n, a.cin, a.h, a.w, a.cout, terms) || a.silu_in || a.ldc != a.cout ||
      (epi != CT_EPI_BIAS && epi != CT_EPI_DSILU) || (epi == CT_EPI_DSILU && !a.pre) ||
      (epi == CT_EPI_BIAS && !a.bias)) {
    dr_set_error("convT_split3: unsupported problem (cin=%d cout=%d h=%d w=%d epi=%d)", a.cin, a.cout, a.h, a.w, epi);
    return DR_E_INVALID;
  }
  if (op_convT_cls_supported(a.n, a.cin, a.h, a.w, a.cout) && ((uintptr_t)a.in & 15) == 0 &&
      ((uintptr_t)a.out & 15) == 0 && (!a.out2 || ((uintptr_t)a.out2 & 15) == 0) &&
      (epi != CT_EPI_DSILU || ((uintptr_t)a.pre & 15) == 0) && (epi != CT_EPI_BIAS || ((uintptr_t)a.bias & 15) == 0))
    return launch_convT_cls(epi, a, wr, s, terms);
  if (terms == 3 && op_convT_glds_s3_supported(a, epi) && !((uintptr_t)wr & 15)) return op_convT_glds_s3(epi, a, wr, s);
#define DR_T3E(BN, C, T) \
  (epi == CT_EPI_DSILU ? launch_t3<BN, C, CT_EPI_DSILU, T>(a, wr, s) : launch_t3<BN, C, CT_EPI_BIAS, T>(a, wr, s))
#define DR_T3L(C)                                                                          \
  if (a.cin == C) {                                                                        \
    if (terms == 1) {                                                                      \
      if (a.cout % 128 == 0) return DR_T3E(128, C, 1);                                     \
      if (a.cout % 64 == 0) return DR_T3E(64, C, 1);                                       \
      return DR_T3E(32, C, 1);                                                             \
    }                                                                                      \
    if (a.cout % 128 == 0) return DR_T3E(128, C, 3);                                       \
    return DR_T3E(64, C, 3);                                                               \
  }
  DR_T3L(32)
  DR_T3L(64)
  DR_T3L(128)
  DR_T3L(256)
#undef DR_T3L
#undef DR_T3E
  return DR_E_INVALID;
}

// ---------------------------------------------------------------------------
// Weight gradient of a k4 s2 p1 (transposed) convolution, f32-accurate on the
// bf16 MFMA (the k_conv_wgrad GEMM of wmconv.hip: [ca] x [16 cb] over K = the
// low-resolution pixels, column n = tap * cb + b).  Both operands are
// activations, so both are split3 while they are staged: a thread stages one
// unit of 8 consecutive pixels x 4 channels (8 float4 loads), splits the 4
// pixel pairs of each channel and writes one 16-byte unit per channel and
// plane -- the transpose to the [channel][pixel] rows the MFMA fragments read
// happens in registers.  Rows of 64 pixels (8 units) are padded to 9 units:
// the 16 rows of a fragment read fall on distinct bank quads.  One LDS buffer
// (the next chunk's loads are in flight in registers meanwhile), 8 waves as
// 2 (a) x 4 (n), partial planes per pixel split reduced by k_wgrad_reduce.
// Low-resolution sizes are powers of two (shift addressing).
// ---------------------------------------------------------------------------
// (Round 6: the six-product form runs on k_wgrad_split3_db below; this kernel
// keeps the one-term form, whose single buffer is 55-83 KB: on the
// double-buffered kernel the one-term WM step measured 8.50 -> 8.64 ms with
// 32-pixel chunks, 8.52 with 64 for the 128-channel layers,
// profiles/r06x_ab_wgrad_db_one_term.txt -- without the split there is little
// VALU for the second buffer to overlap.)
// TERMS = 1: both operands RNE-rounded to one bf16 plane (bf16 world-model
// step); that form also takes BN = 256 column tiles (the output-gradient rows
// re-read half as often: 255 -> 209 us for the 128-channel layers, r04r) and
// BM = 32.  (The 32 x 4-channel layers next to the frames stay on the f32
// kernel: a BN = 64 one-term form measured 314 us against 311, and with
// SiLU on load 752 us.)
template <int BM, int TERMS = 3, int BN = 128>
__global__ __launch_bounds__(512) void k_wgrad_split3(int n, int lh, int lw, int ca, int cb,
                                                      const float* __restrict__ lo, int lda,
                                                      const float* __restrict__ hi, int ldb, int chunk,
                                                      float* __restrict__ part) {
  constexpr int KC = 64, RP = KC / 8 + 1;
  constexpr int FM = BM / 32, FN = BN / 64;  // wave tile (BM / 2) x (BN / 4)
  static_assert((TERMS == 1 || TERMS == 3) && FM >= 1 &&
                    (BN == 128 || BN == 256 || (BN == 512 && TERMS == 1 && BM <= 64)),
                "wgrad_split3 tile");
  __shared__ __attribute__((aligned(16))) u32x4 S[TERMS][BM + BN][RP];
  const int N = 16 * cb;
  const int tiles_n = N / BN, tiles = (ca / BM) * tiles_n;
  // XCD-contiguous logical order (dr_xcd_tile), tiles of one pixel split
  // adjacent: the tiles that read the same pixels share an XCD's L2 instead of
  // each fetching them from HBM through its own
  const int h = 1 << lh, w = 1 << lw, H2 = 2 * h, W2 = 2 * w;
  const long long K = (long long)n * h * w;
  const int nsplit = (int)((K + chunk - 1) / chunk);
  const int lb = dr_xcd_tile(blockIdx.x, tiles * nsplit);
  if (lb < 0) return;
  const int split = lb / tiles, lt = lb - split * tiles;
  const int m0 = (lt / tiles_n) * BM, n0 = (lt % tiles_n) * BN;
  const long long k_begin = (long long)split * chunk;
  const long long k_end = k_begin + chunk < K ? k_begin + chunk : K;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;

  // staging units of this thread (UPT of them): channel quad cq, pixel octet
  // oct (A: rows of ca channels m0 + 4 cq; B: columns n0 + 4 cq, one tap, 4 channels)
  constexpr int AU = BM / 4 * 8, BUn = BN / 4 * 8, UPT = (AU + BUn + 511) / 512;
  bool isA[UPT], active[UPT];
  int oct[UPT], row0[UPT], bch[UPT], bky[UPT], bkx[UPT];
  const float* src[UPT];
#pragma unroll
  for (int j = 0; j < UPT; ++j) {
    const int id = tid + 512 * j;
    isA[j] = id < AU;
    active[j] = id < AU + BUn;
    const int u = isA[j] ? id : id - AU, cq = u >> 3;
    oct[j] = u & 7;
    row0[j] = isA[j] ? 4 * cq : BM + 4 * cq;
    const int bn = n0 + 4 * cq, btap = bn / cb;
    bch[j] = bn - btap * cb;
    bky[j] = btap >> 2;
    bkx[j] = btap & 3;
    src[j] = isA[j] ? lo + m0 + 4 * cq : hi;
  }
  f32x4 v[UPT][8];
  auto load = [&](long long p0c) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < UPT; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const long long p = p0c + 8 * oct[j] + i;
        bool ok = active[j] && p < k_end;
        long long off;
        if (isA[j]) {
          off = p * lda;
        } else {
          const long long f = p >> (lw + lh);
          const int y = (int)(p >> lw) & (h - 1), x = (int)p & (w - 1);
          const int Y = 2 * y - 1 + bky[j], X = 2 * x - 1 + bkx[j];
          ok = ok && Y >= 0 && Y < H2 && X >= 0 && X < W2;
          off = ((f * H2 + Y) * W2 + X) * ldb + bch[j];
        }
        const f32x4 t = *reinterpret_cast<const f32x4*>(src[j] + (ok ? off : 0));
        v[j][i] = ok ? t : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
  };
  auto store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      if (!active[j]) continue;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if constexpr (TERMS == 1) {
          u32x4 ph;
#pragma unroll
          for (int i = 0; i < 4; ++i) ph[i] = pack_bf16x2(v[j][2 * i][c], v[j][2 * i + 1][c]);
          S[0][row0[j] + c][oct[j]] = ph;
        } else {
          u32x4 ph, pm, pl;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            unsigned hh, mm, ll;
            split3_pair(v[j][2 * i][c], v[j][2 * i + 1][c], hh, mm, ll);
            ph[i] = hh;
            pm[i] = mm;
            pl[i] = ll;
          }
          S[0][row0[j] + c][oct[j]] = ph;
          S[1][row0[j] + c][oct[j]] = pm;
          S[2][row0[j] + c][oct[j]] = pl;
        }
      }
    }
  };

  const int wm0 = (wave >> 2) * (BM / 2), wn0 = (wave & 3) * (BN / 4);
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const long long nch = k_end > k_begin ? (k_end - k_begin + KC - 1) / KC : 0;
  if (nch > 0) {
    load(k_begin);
    store();
    __syncthreads();
    for (long long c = 0; c < nch; ++c) {
      // next chunk in flight (the last chunk reloads itself, unused)
      load(k_begin + (c + 1 < nch ? c + 1 : c) * KC);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        u32x4 av[TERMS][FM], bv[TERMS][FN];
#pragma unroll
        for (int pl = 0; pl < TERMS; ++pl) {
#pragma unroll
          for (int i = 0; i < FM; ++i) av[pl][i] = S[pl][wm0 + 16 * i + r][4 * ks + q];
#pragma unroll
          for (int j = 0; j < FN; ++j) bv[pl][j] = S[pl][BM + wn0 + 16 * j + r][4 * ks + q];
        }
#define DR_W3(PA, PB)                                                                                   \
  _Pragma("unroll") for (int i = 0; i < FM; ++i) _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[i][j] = \
      mfma_b16(av[PA][i], bv[PB][j], acc[i][j]);
        if constexpr (TERMS == 3) {
          DR_W3(2, 0)
          DR_W3(1, 1)
          DR_W3(0, 2)
          DR_W3(1, 0)
          DR_W3(0, 1)
        }
        DR_W3(0, 0)
#undef DR_W3
      }
      __syncthreads();
      if (c + 1 < nch) {
        store();
        __syncthreads();
      }
    }
  }
  // lane (r, q) of acc[i][j]: a = 4 q + e of row block i, n = r of column block j
  float* P = part + (long long)split * ca * N;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) P[(long long)(m0 + wm0 + 16 * i + 4 * q + e) * N + n0 + wn0 + 16 * j + r] = acc[i][j][e];
}

// Double-buffered form (the six-product tiles): the single LDS buffer above
// makes every chunk two phases -- all waves split and store, barrier, all
// waves run the MFMAs, barrier -- so the VALU split never overlaps the matrix
// core.  Here the pixel chunks are 32 deep (KC = 32: a 128 x 128 six-product
// tile's two buffers take 120 KB), a thread stages units of 4 pixels x 4
// channels (4 float4 loads, 2 pixel pairs per channel, 8-byte LDS pieces), and
// chunk c + 1 is loaded before and stored after chunk c's MFMAs into the other
// buffer: one barrier per chunk, the split of one wave beside the MFMAs of its
// SIMD partner.  Per split the products run over the same pixels in the same
// order as the single-buffer kernel (its 64-pixel chunk = two 32-deep steps),
// so the partial planes are bitwise the same.
template <int BM, int TERMS, int BN, int KC>
__global__ __launch_bounds__(512) void k_wgrad_split3_db(int n, int lh, int lw, int ca, int cb,
                                                         const float* __restrict__ lo, int lda,
                                                         const float* __restrict__ hi, int ldb, int chunk,
                                                         float* __restrict__ part) {
  constexpr int RP = KC / 8 + 1, NQ = KC / 4;  // 16-byte units per row (+1 pad), pixel quartets per chunk
  constexpr int FM = BM / 32, FN = BN / 64;
  static_assert((KC == 32 || KC == 64) && FM >= 1 && FN >= 1, "wgrad_split3_db tile");
  __shared__ __attribute__((aligned(16))) u32x4 S[2][TERMS][BM + BN][RP];
  const int N = 16 * cb;
  const int tiles_n = N / BN, tiles = (ca / BM) * tiles_n;
  const int h = 1 << lh, w = 1 << lw, H2 = 2 * h, W2 = 2 * w;
  const long long K = (long long)n * h * w;
  const int nsplit = (int)((K + chunk - 1) / chunk);
  const int lb = dr_xcd_tile(blockIdx.x, tiles * nsplit);
  if (lb < 0) return;
  const int split = lb / tiles, lt = lb - split * tiles;
  const int m0 = (lt / tiles_n) * BM, n0 = (lt % tiles_n) * BN;
  const long long k_begin = (long long)split * chunk;
  const long long k_end = k_begin + chunk < K ? k_begin + chunk : K;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;

  // staging units: channel quad cq, pixel quartet qt (A: channels m0 + 4 cq of
  // lo; B: columns n0 + 4 cq, one tap, 4 channels of hi)
  constexpr int AU = BM / 4 * NQ, BUn = BN / 4 * NQ, UPT = (AU + BUn + 511) / 512;
  bool isA[UPT], active[UPT];
  int qt[UPT], row0[UPT], bch[UPT], bky[UPT], bkx[UPT];
  const float* src[UPT];
#pragma unroll
  for (int j = 0; j < UPT; ++j) {
    const int id = tid + 512 * j;
    isA[j] = id < AU;
    active[j] = id < AU + BUn;
    const int u = isA[j] ? id : id - AU, cq = u / NQ;
    qt[j] = u - cq * NQ;
    row0[j] = isA[j] ? 4 * cq : BM + 4 * cq;
    const int bn = n0 + 4 * cq, btap = bn / cb;
    bch[j] = bn - btap * cb;
    bky[j] = btap >> 2;
    bkx[j] = btap & 3;
    src[j] = isA[j] ? lo + m0 + 4 * cq : hi;
  }
  f32x4 v[UPT][4];
  auto load = [&](long long p0c) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < UPT; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long long p = p0c + 4 * qt[j] + i;
        bool ok = active[j] && p < k_end;
        long long off;
        if (isA[j]) {
          off = p * lda;
        } else {
          const long long f = p >> (lw + lh);
          const int y = (int)(p >> lw) & (h - 1), x = (int)p & (w - 1);
          const int Y = 2 * y - 1 + bky[j], X = 2 * x - 1 + bkx[j];
          ok = ok && Y >= 0 && Y < H2 && X >= 0 && X < W2;
          off = ((f * H2 + Y) * W2 + X) * ldb + bch[j];
        }
        const f32x4 t = *reinterpret_cast<const f32x4*>(src[j] + (ok ? off : 0));
        v[j][i] = ok ? t : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < UPT; ++j) {
      if (!active[j]) continue;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if constexpr (TERMS == 1) {
          const u32x2 ph = {pack_bf16x2(v[j][0][c], v[j][1][c]), pack_bf16x2(v[j][2][c], v[j][3][c])};
          reinterpret_cast<u32x2*>(&S[buf][0][row0[j] + c][0])[qt[j]] = ph;
        } else {
          unsigned h0, m0w, l0, h1, m1, l1;
          split3_pair(v[j][0][c], v[j][1][c], h0, m0w, l0);
          split3_pair(v[j][2][c], v[j][3][c], h1, m1, l1);
          reinterpret_cast<u32x2*>(&S[buf][0][row0[j] + c][0])[qt[j]] = (u32x2){h0, h1};
          reinterpret_cast<u32x2*>(&S[buf][1][row0[j] + c][0])[qt[j]] = (u32x2){m0w, m1};
          reinterpret_cast<u32x2*>(&S[buf][2][row0[j] + c][0])[qt[j]] = (u32x2){l0, l1};
        }
      }
    }
  };

  const int wm0 = (wave >> 2) * (BM / 2), wn0 = (wave & 3) * (BN / 4);
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const long long nch = k_end > k_begin ? (k_end - k_begin + KC - 1) / KC : 0;
  if (nch > 0) {
    load(k_begin);
    store(0);
    __syncthreads();
    for (long long c = 0; c < nch; ++c) {
      const int buf = (int)(c & 1);
      const bool more = c + 1 < nch;
      if (more) load(k_begin + (c + 1) * KC);
#pragma unroll
      for (int ks = 0; ks < KC / 32; ++ks) {
        u32x4 av[TERMS][FM], bv[TERMS][FN];
#pragma unroll
        for (int pl = 0; pl < TERMS; ++pl) {
#pragma unroll
          for (int i = 0; i < FM; ++i) av[pl][i] = S[buf][pl][wm0 + 16 * i + r][4 * ks + q];
#pragma unroll
          for (int j = 0; j < FN; ++j) bv[pl][j] = S[buf][pl][BM + wn0 + 16 * j + r][4 * ks + q];
        }
#define DR_W3(PA, PB)                                                                                   \
  _Pragma("unroll") for (int i = 0; i < FM; ++i) _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[i][j] = \
      mfma_b16(av[PA][i], bv[PB][j], acc[i][j]);
        if constexpr (TERMS == 3) {
          DR_W3(2, 0)
          DR_W3(1, 1)
          DR_W3(0, 2)
          DR_W3(1, 0)
          DR_W3(0, 1)
        }
        DR_W3(0, 0)
#undef DR_W3
      }
      if (more) store(buf ^ 1);
      __syncthreads();
    }
  }
  float* P = part + (long long)split * ca * N;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) P[(long long)(m0 + wm0 + 16 * i + 4 * q + e) * N + n0 + wn0 + 16 * j + r] = acc[i][j][e];
}


static int ilog2_exact(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return (1 << l) == v ? l : -1;
}

bool op_wgrad_split3_supported(int n, int h, int w, int ca, int cb, int terms) {
  const bool cb_ok = cb % 8 == 0 && cb >= 8;
  return (ca == 64 || ca == 128 || ca == 256 || (terms == 1 && ca == 32)) && cb_ok && ilog2_exact(h) >= 0 &&
         ilog2_exact(w) >= 0 && n > 0 && (long long)n * 4 * h * w * cb < (1LL << 31);
}

// tile of a problem: BM by the a-channels; the one-term form takes BN = 256
// where N = 16 cb allows it.  The 64-channel layers (the encoder's conv2, the
// decoder's 64 -> 32 transposed conv) re-read their staged bytes per output
// more than the 128-channel ones at BN = 128 (64 x 128 tiles: 48 KB staged per
// 64-pixel chunk for 1 MFLOP against 64 KB for 2), so BM = 64 takes wider
// column tiles: 256 in the six-product form, 512 in the one-term form (WM step
// B = 256 T = 15: fp32 14.16 -> 13.87 ms, bf16 9.30 -> 9.20 ms;
// profiles/r06l_ab_gates_wgrad.txt)
static void wgrad3_tile(int ca, int cb, int terms, int& bm, int& bn) {
  bm = ca >= 128 ? 128 : ca >= 64 ? 64 : 32;
  const int n = 16 * cb;
  if (bm == 64) bn = terms == 1 && n % 512 == 0 ? 512 : n % 256 == 0 ? 256 : 128;
  else bn = terms == 1 && n % 256 == 0 ? 256 : 128;
}

static void wgrad3_plan(int n, int h, int w, int ca, int cb, int bm, int bn, int& nsplit, int& chunk) {
  const int tiles = (ca / bm) * (16 * cb / bn);
  const long long K = (long long)n * h * w;
  const long long kch = (K + 63) / 64;
  long long ns = (512 + tiles - 1) / tiles;  // about 2 workgroups per CU
  if (ns > (kch + 1) / 2) ns = (kch + 1) / 2;  // at least 2 chunks per split
  if (ns < 1) ns = 1;
  const long long ch = ((kch + ns - 1) / ns) * 64;
  chunk = (int)ch;
  nsplit = (int)((K + ch - 1) / ch);
}

size_t op_wgrad_split3_ws_floats(int n, int h, int w, int ca, int cb) {
  size_t f = 0;
  for (int terms : {1, 3}) {  // either form's partial planes
    int bm, bn, ns, ch;
    wgrad3_tile(ca, cb, terms, bm, bn);
    wgrad3_plan(n, h, w, ca, cb, bm, bn, ns, ch);
    f = std::max(f, (size_t)ns * ca * 16 * cb);
  }
  return f;
}

int op_wgrad_split3(int n, int h, int w, int ca, int cb, const float* lo, int lda, const float* hi, int ldb,
                    float* dw, int cbo, float scale, int accumulate, float* ws, size_t ws_floats, hipStream_t s,
                    int terms) {
  if (!op_wgrad_split3_supported(n, h, w, ca, cb, terms) || (terms != 1 && terms != 3) || lda % 4 || ldb % 4 || lda < ca || ldb < cb || cbo < 1 ||
      cbo > cb || !lo || !hi || !dw || ((uintptr_t)lo & 15) || ((uintptr_t)hi & 15)) {
    dr_set_error("wgrad_split3: unsupported problem (ca=%d cb=%d h=%d w=%d)", ca, cb, h, w);
    return DR_E_INVALID;
  }
  int bm, bn, ns, ch;
  wgrad3_tile(ca, cb, terms, bm, bn);
  wgrad3_plan(n, h, w, ca, cb, bm, bn, ns, ch);
  if ((size_t)ns * ca * 16 * cb > ws_floats) {
    dr_set_error("wgrad_split3: workspace too small");
    return DR_E_WORKSPACE;
  }
  const int tiles = (ca / bm) * (16 * cb / bn);
  const int lh = ilog2_exact(h), lw = ilog2_exact(w);
#define DR_W3L(BM, T, ...)                                                                                     \
  hipLaunchKernelGGL((k_wgrad_split3<BM, T, ##__VA_ARGS__>), dim3((unsigned)dr_xcd_grid(tiles * ns)), dim3(512), 0, s, n, lh, lw, \
                     ca, cb, lo, lda, hi, ldb, ch, ws)
  if (terms == 1) {
    if (bn == 512) {
      DR_W3L(64, 1, 512);
    } else if (bn == 256) {
      if (bm == 128) DR_W3L(128, 1, 256);
      else if (bm == 64) DR_W3L(64, 1, 256);
      else DR_W3L(32, 1, 256);
    } else {
      if (bm == 128) DR_W3L(128, 1);
      else if (bm == 64) DR_W3L(64, 1);
      else DR_W3L(32, 1);
    }
  } else {  // six products: the double-buffered kernel (WM step fp32 13.87 -> 13.82 ms, r06l)
#define DR_W3D(BM, BN)                                                                                            \
  hipLaunchKernelGGL((k_wgrad_split3_db<BM, 3, BN, 32>), dim3((unsigned)dr_xcd_grid(tiles * ns)), dim3(512), 0, s, n, \
                     lh, lw, ca, cb, lo, lda, hi, ldb, ch, ws)
    if (bm == 128) DR_W3D(128, 128);
    else if (bn == 256) DR_W3D(64, 256);
    else DR_W3D(64, 128);
#undef DR_W3D
  }
#undef DR_W3L
  DR_TRY(dr_check_launch("wgrad_split3"));
  return op_wgrad_reduce(ca, cb, cbo, ns, ws, dw, scale, accumulate, s);
}

// ---------------------------------------------------------------------------
// Tall NT products, f32-accurate on the bf16 MFMA: Y[m][n] = act(sum_k A[m][k]
// W[n][k] + bias[n]) for M in the thousands (the encoder feature projection
// over B S / 2 frames, K = 4096; the critic's and the reward / continue heads'
// first layers over B (H + 1) imagined states, K = Hd + L).  The k_conv_split3
// pipeline with a row-major A (optional second K segment at ksA, k % 4
// aligned) in place of the im2col gather; W split once per call into planes
// [K/32][3][Np][32] (Np = N rounded up to BN, zero rows past N).
// ---------------------------------------------------------------------------
#define DR_S3_SPLITS 8
struct GemmS3 {
  int M, N, K, ksA, lda, lda2, ldy, act, Np;
  const float* A;
  const float* A2;
  const u16* wr;
  const float* bias;
  float* Y;
  int splits;   // split-K over blockIdx.y (> 1: raw partial sums to part, k_s3_finish applies the epilogue)
  float* part;  // [splits][M][N]
  // the world-model backward's data-gradient products: Y += (accumulate), and
  // columns n >= nsplitY go to Y2[m][n - nsplitY] (nsplitY % 4 == 0)
  int accumulate, ldy2, nsplitY, pad_;
  float* Y2;
};
// the epilogue store of 4 consecutive columns n..n+3 (never straddling nsplitY)
__device__ __forceinline__ void s3_store(const GemmS3& g, int m, int n, f32x4 v) {
  float* dst = n < g.nsplitY ? g.Y + (long long)m * g.ldy + n : g.Y2 + (long long)m * g.ldy2 + (n - g.nsplitY);
  if (g.accumulate) v += *reinterpret_cast<const f32x4*>(dst);
  *reinterpret_cast<f32x4*>(dst) = v;
}

template <int BM, int BN>
__global__ __launch_bounds__(BM * 2) void k_gemm_split3(GemmS3 g) {
  constexpr int NT = BM * 2;
  constexpr int WTN = BN / 2, FM = 4, FN = WTN / 16;
  constexpr int APT = BM * 8 / NT;
  constexpr int BU = 3 * BN * 4;
  constexpr int BPT = (BU + NT - 1) / NT;
  static_assert(APT == 4 && FN >= 1 && BM % 64 == 0, "gemm_split3 tile");
  __shared__ __attribute__((aligned(16))) u32x4 As[2][3][BM][4];
  __shared__ __attribute__((aligned(16))) u32x4 Bs[2][3][BN][4];
  const int M = g.M, N = g.N, K = g.K, ksA = g.ksA, Np = g.Np;
  const int tiles_n = (N + BN - 1) / BN;
  const int tiles = ((M + BM - 1) / BM) * tiles_n;
  const int lt = dr_xcd_tile(blockIdx.x, tiles);
  if (lt < 0) return;
  const int m0 = (lt / tiles_n) * BM, n0 = (lt % tiles_n) * BN;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;
  const int quad = tid & 7, prow = tid >> 3;
  const int NCH_ALL = (K + 31) / 32;
  const int per = (NCH_ALL + g.splits - 1) / g.splits;
  const int cb = min(NCH_ALL, (int)blockIdx.y * per), NCH = min(NCH_ALL, cb + per);  // chunks [cb, NCH)
  // per A row: element offsets of the row in both segments (rows past M read row M - 1)
  unsigned oa[APT], oa2[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const int m = min(m0 + prow + (NT / 8) * i, M - 1);
    oa[i] = (unsigned)(m * g.lda);
    oa2[i] = (unsigned)(m * g.lda2);
  }
  f32x4 ra0[APT], ra1[APT];
  u32x4 rb0[BPT], rb1[BPT];
  bool kv0 = true, kv1 = true;  // this thread's float4 lies below K
  auto load = [&](int c, auto slot) __attribute__((always_inline)) {
    f32x4* ra = decltype(slot)::value == 0 ? ra0 : ra1;
    u32x4* rb = decltype(slot)::value == 0 ? rb0 : rb1;
    bool& kv = decltype(slot)::value == 0 ? kv0 : kv1;
    const int k = 32 * c + 4 * quad;
    kv = k < K;
    const int kk = kv ? k : 0;
    const bool s1 = kk < ksA;
    const float* base = s1 ? g.A : g.A2;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const unsigned e = s1 ? oa[i] + (unsigned)kk : oa2[i] + (unsigned)(kk - ksA);
      ra[i] = *reinterpret_cast<const f32x4*>(base + e);
    }
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int e = tid + NT * j;
      if (BU % NT == 0 || e < BU) {
        const int pl = e / (BN * 4), rm = e - pl * BN * 4, row = rm >> 2, u = rm & 3;
        rb[j] = *reinterpret_cast<const u32x4*>(g.wr + (((long long)c * 3 + pl) * Np + n0 + row) * 32 + 8 * u);
      }
    }
  };
  auto store = [&](auto slot, int buf) __attribute__((always_inline)) {
    const f32x4* ra = decltype(slot)::value == 0 ? ra0 : ra1;
    const u32x4* rb = decltype(slot)::value == 0 ? rb0 : rb1;
    const bool kv = decltype(slot)::value == 0 ? kv0 : kv1;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int row = prow + (NT / 8) * i;
      const f32x4 v = kv ? ra[i] : (f32x4){0.f, 0.f, 0.f, 0.f};
      unsigned h0, m0_, l0, h1, m1, l1;
      split3_pair(v[0], v[1], h0, m0_, l0);
      split3_pair(v[2], v[3], h1, m1, l1);
      const int unit = (quad >> 1) ^ swz(row), half = quad & 1;
      reinterpret_cast<u32x2*>(&As[buf][0][row][unit])[half] = (u32x2){h0, h1};
      reinterpret_cast<u32x2*>(&As[buf][1][row][unit])[half] = (u32x2){m0_, m1};
      reinterpret_cast<u32x2*>(&As[buf][2][row][unit])[half] = (u32x2){l0, l1};
    }
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int e = tid + NT * j;
      if (BU % NT == 0 || e < BU) {
        const int pl = e / (BN * 4), rm = e - pl * BN * 4, row = rm >> 2, u = rm & 3;
        Bs[buf][pl][row][u ^ swz(row)] = rb[j];
      }
    }
  };
  const int wm0 = (wave >> 1) * 64, wn0 = (wave & 1) * WTN;
  const int fu = q ^ swz(r);
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if (cb < NCH) {
  load(cb, S0{});
  load(min(cb + 1, NCH - 1), S1{});
  store(S0{}, 0);
  __syncthreads();
  auto step = [&](int c, auto slot) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot)::value;
    using Next = std::integral_constant<int, 1 - SL>;
    const int buf = (c - cb) & 1;
    load(min(c + 2, NCH - 1), slot);
    u32x4 av[3][FM], bv[3][FN];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int i = 0; i < FM; ++i) av[pl][i] = As[buf][pl][wm0 + 16 * i + r][fu];
#pragma unroll
      for (int j = 0; j < FN; ++j) bv[pl][j] = Bs[buf][pl][wn0 + 16 * j + r][fu];
    }
#define DR_G3(PA, PB)                                                                                   \
  _Pragma("unroll") for (int i = 0; i < FM; ++i) _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[i][j] = \
      mfma_b16(bv[PB][j], av[PA][i], acc[i][j]);
    DR_G3(2, 0)
    DR_G3(1, 1)
    DR_G3(0, 2)
    DR_G3(1, 0)
    DR_G3(0, 1)
    DR_G3(0, 0)
#undef DR_G3
    if (c + 1 < NCH) store(Next{}, buf ^ 1);
    dr_lds_barrier();
  };
  int c = cb;
  for (; c + 1 < NCH; c += 2) {
    step(c, S0{});
    step(c + 1, S1{});
  }
  if (c < NCH) step(c, S0{});
  }
  // lane (r, q) of acc[i][j]: row m0 + wm0 + 16 i + r, columns n0 + wn0 + 16 j + 4 q .. + 3
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm0 + 16 * i + r;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn0 + 16 * j + 4 * q;
      if (n >= N) continue;
      f32x4 v = acc[i][j];
      if (g.splits > 1) {
        *reinterpret_cast<f32x4*>(g.part + ((long long)blockIdx.y * M + m) * N + n) = v;
        continue;
      }
      if (g.bias) v += *reinterpret_cast<const f32x4*>(g.bias + n);
      if (g.act == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] / (1.0f + expf(-v[e]));
      }
      s3_store(g, m, n, v);
    }
  }
}

// split-K partial planes of k_gemm_split3 -> Y (fixed order over the splits), bias, activation
__global__ void k_s3_finish(GemmS3 g) {
  const long long i4 = (long long)blockIdx.x * 256 + threadIdx.x;
  const int N4 = g.N / 4;
  if (i4 >= (long long)g.M * N4) return;
  const int m = (int)(i4 / N4), n = 4 * (int)(i4 - (long long)m * N4);
  f32x4 v = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int sp = 0; sp < g.splits; ++sp) v += *reinterpret_cast<const f32x4*>(g.part + ((long long)sp * g.M + m) * g.N + n);
  if (g.bias) v += *reinterpret_cast<const f32x4*>(g.bias + n);
  if (g.act == 1) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = v[e] / (1.0f + expf(-v[e]));
  }
  s3_store(g, m, n, v);
}

// W [N][K] (row stride ldw) -> bf16 planes [K/32][3][Np][32], zero past N and K
__device__ __forceinline__ void nt_repack_split3_elem(long long i, int N, int K, int Np, const float* __restrict__ W,
                                                      long long ldw, u16* __restrict__ wr) {
  const int KC = (K + 31) / 32;
  const int n = (int)(i / (KC * 32)), k = (int)(i - (long long)n * KC * 32);
  unsigned hh = 0, mm = 0, ll = 0;
  if (n < N && k < K) split3(W[(long long)n * ldw + k], hh, mm, ll);
  const long long plane = (long long)Np * 32;
  const long long base = ((long long)(k >> 5) * 3 * Np + n) * 32 + (k & 31);
  wr[base] = (u16)hh;
  wr[base + plane] = (u16)mm;
  wr[base + 2 * plane] = (u16)ll;
}
__global__ void k_nt_repack_split3(int N, int K, int Np, const float* __restrict__ W, int ldw, u16* __restrict__ wr) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)((K + 31) / 32) * 32 * Np) return;
  nt_repack_split3_elem(i, N, K, Np, W, ldw, wr);
}

// Several weight repacks in ONE launch (the encoder's per-call weight
// preparation: conv1 / conv2..N planes, the projection's planes or bf16 copy),
// blocks over the concatenated element ranges; the same element code as the
// single-job kernels
struct RepackBatch {
  RepackJob j[DR_RJ_MAX];
  int blk0[DR_RJ_MAX + 1];  // first block of job i; [n..] = total
  int n;
};
__global__ __launch_bounds__(256) void k_repack_multi(RepackBatch b) {
  __shared__ __attribute__((aligned(16))) RepackJob J;
  int z = 0;
#pragma unroll
  for (int i = 1; i < DR_RJ_MAX; ++i)
    if ((int)blockIdx.x >= b.blk0[i]) z = i;
  dr_stage_args(b.j[z], J, threadIdx.x);
  const long long i = (long long)(blockIdx.x - b.blk0[z]) * 256 + threadIdx.x;
  if (i >= J.total) return;
  u16* out = static_cast<u16*>(J.out);
  switch (J.kind) {
    case RJ_CONV1: conv1_repack_split3_elem((int)i, J.a, J.w, out); break;
    case RJ_CONV: conv_repack_split3_elem((int)i, J.a, J.b, J.w, out); break;
    case RJ_NT: nt_repack_split3_elem(i, J.a, J.b, J.c, J.w, J.ld, out); break;
    default: {  // RJ_BF16: rows x cols (row stride ld) -> bf16 [rows][cols], RNE
      const int rr = (int)(i / J.b), cc = (int)(i - (long long)rr * J.b);
      out[i] = __builtin_bit_cast(u16, (__bf16)J.w[(long long)rr * J.ld + cc]);
    }
  }
}

RepackJob rj_conv1(int cout, const float* w, void* wr) { return {RJ_CONV1, cout, 0, 0, w, wr, 0, (long long)cout * 64}; }
RepackJob rj_conv(int cout, int cin, const float* w, void* wr) {
  return {RJ_CONV, cout, cin, 0, w, wr, 0, (long long)cout * 16 * cin};
}
RepackJob rj_nt(int N, int K, const float* W, int ldw, void* wr) {
  const int Np = (N + 127) / 128 * 128;
  return {RJ_NT, N, K, Np, W, wr, ldw, (long long)((K + 31) / 32) * 32 * Np};
}
RepackJob rj_bf16(int rows, int cols, const float* x, long long ld, void* y) {
  return {RJ_BF16, rows, cols, 0, x, y, ld, (long long)rows * cols};
}

int op_repack_multi(const RepackJob* jobs, int n, hipStream_t s) {
  if (n < 0 || n > DR_RJ_MAX) {
    dr_set_error("repack_multi: %d jobs (at most %d)", n, DR_RJ_MAX);
    return DR_E_INVALID;
  }
  if (n == 0) return DR_OK;
  RepackBatch b = {};
  int tot = 0;
  for (int i = 0; i < DR_RJ_MAX; ++i) {
    b.blk0[i] = tot;
    if (i < n) {
      b.j[i] = jobs[i];
      tot += (int)((jobs[i].total + 255) / 256);
    }
  }
  b.blk0[DR_RJ_MAX] = tot;
  b.n = n;
  hipLaunchKernelGGL(k_repack_multi, dim3((unsigned)tot), dim3(256), 0, s, b);
  return dr_check_launch("repack_multi");
}

// weight planes hold N rounded up to 128 rows (either column tile reads whole tiles)
static int s3_np(int N) { return (N + 127) / 128 * 128; }
size_t op_nt_split3_ws_bytes(int N, int K) {
  return (size_t)((K + 31) / 32) * 32 * 3 * s3_np(N) * sizeof(u16);
}
int op_nt_repack_split3(int N, int K, const float* W, int ldw, void* wr, hipStream_t s) {
  const int Np = s3_np(N);
  const long long total = (long long)((K + 31) / 32) * 32 * Np;
  hipLaunchKernelGGL(k_nt_repack_split3, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, N, K, Np, W, ldw,
                     (u16*)wr);
  return dr_check_launch("nt_repack_split3");
}
bool op_gemm_nt_split3_supported(int M, int N, int K, const float* A, int lda, const float* A2, int lda2, int ksA,
                                 int ldy) {
  const bool seg = ksA < K;
  return M > 0 && N > 0 && N % 4 == 0 && ldy % 4 == 0 && K % 4 == 0 && lda % 4 == 0 && !((uintptr_t)A & 15) &&
         (!seg || (ksA % 4 == 0 && lda2 % 4 == 0 && A2 && !((uintptr_t)A2 & 15))) &&
         (long long)M * lda < (1LL << 31) && (!seg || (long long)M * lda2 < (1LL << 31));
}
size_t op_gemm_nt_split3_part_floats(int M, int N) { return (size_t)DR_S3_SPLITS * M * N; }

int op_gemm_nt_split3(int M, int N, int K, const float* A, int lda, const float* A2, int lda2, int ksA, const void* wr,
                      const float* bias, int act, float* Y, int ldy, hipStream_t s) {
  return op_gemm_nt_split3_sk(M, N, K, A, lda, A2, lda2, ksA, wr, bias, act, Y, ldy, nullptr, 0, s);
}

int op_gemm_nt_split3_sk(int M, int N, int K, const float* A, int lda, const float* A2, int lda2, int ksA,
                         const void* wr, const float* bias, int act, float* Y, int ldy, float* part,
                         size_t part_floats, hipStream_t s, int splits_fixed) {
  return op_gemm_nt_split3_ex(M, N, K, A, lda, A2, lda2, ksA, wr, bias, act, Y, ldy, 0, nullptr, 0, INT_MAX, part,
                              part_floats, s, splits_fixed);
}

int op_gemm_nt_split3_ex(int M, int N, int K, const float* A, int lda, const float* A2, int lda2, int ksA,
                         const void* wr, const float* bias, int act, float* Y, int ldy, int accumulate, float* Y2,
                         int ldy2, int nsplitY, float* part, size_t part_floats, hipStream_t s, int splits_fixed) {
  const bool y2 = nsplitY < N;
  if (!op_gemm_nt_split3_supported(M, N, K, A, lda, A2, lda2, ksA, ldy) || ((uintptr_t)Y & 15) ||
      (bias && ((uintptr_t)bias & 15)) || ((uintptr_t)part & 15) || splits_fixed < 0 ||
      splits_fixed > DR_S3_SPLITS || (splits_fixed > 1 && (!part || (size_t)splits_fixed * M * N > part_floats)) ||
      (y2 && (!Y2 || ((uintptr_t)Y2 & 15) || ldy2 % 4 || nsplitY % 4 || nsplitY < 0))) {
    dr_set_error("gemm_nt_split3: unsupported problem (M=%d N=%d K=%d)", M, N, K);
    return DR_E_INVALID;
  }
  GemmS3 g = {M, N, K, ksA < K ? ksA : K, lda, lda2, ldy, act, s3_np(N), A, A2, (const u16*)wr, bias, Y, 1, part,
              accumulate ? 1 : 0, ldy2, y2 ? nsplitY : INT_MAX, 0, Y2};
  auto tl = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  auto waves = [&](int bm, int bn) { return (long long)tl(bm, bn) * (bm / 32); };
  // the largest tile (256 x 128, 256 x 64, 128 x 128, 128 x 64, else 64 x 64)
  // that gives ~two waves per SIMD over the chip (2048 waves), splitting K
  // (>= 8 chunks per split, when the caller brought partial-sum scratch) to
  // get there: taller / wider tiles re-read less.  The N = 200 products over
  // 4096-8192 rows (projection, critic / heads' first layers) otherwise ran
  // 64 x 64 tiles at 75 TF/s.
  const int nch = (K + 31) / 32;
  auto splits_for = [&](int bm, int bn) {
    if (splits_fixed > 0) return splits_fixed;  // the caller's K partition (summation order independent of M)
    int sp = 1;
    while (part && sp < DR_S3_SPLITS && waves(bm, bn) * sp < 2048 && nch / (2 * sp) >= 8 &&
           (size_t)(2 * sp) * M * N <= part_floats)
      sp *= 2;
    return sp;
  };
  const int shapes[5][2] = {{256, 128}, {256, 64}, {128, 128}, {128, 64}, {64, 64}};
  int pick = 4;
  for (int c = 0; c < 5; ++c) {
    if (waves(shapes[c][0], shapes[c][1]) * splits_for(shapes[c][0], shapes[c][1]) >= 2048) {
      pick = c;
      break;
    }
  }
  g.splits = splits_for(shapes[pick][0], shapes[pick][1]);
  const unsigned gy = (unsigned)g.splits;
  switch (pick) {
    case 0: hipLaunchKernelGGL((k_gemm_split3<256, 128>), dim3(dr_xcd_grid(tl(256, 128)), gy), dim3(512), 0, s, g); break;
    case 1: hipLaunchKernelGGL((k_gemm_split3<256, 64>), dim3(dr_xcd_grid(tl(256, 64)), gy), dim3(512), 0, s, g); break;
    case 2: hipLaunchKernelGGL((k_gemm_split3<128, 128>), dim3(dr_xcd_grid(tl(128, 128)), gy), dim3(256), 0, s, g); break;
    case 3: hipLaunchKernelGGL((k_gemm_split3<128, 64>), dim3(dr_xcd_grid(tl(128, 64)), gy), dim3(256), 0, s, g); break;
    default: hipLaunchKernelGGL((k_gemm_split3<64, 64>), dim3(dr_xcd_grid(tl(64, 64)), gy), dim3(128), 0, s, g); break;
  }
  DR_TRY(dr_check_launch("gemm_nt_split3"));
  if (g.splits > 1) {
    hipLaunchKernelGGL(k_s3_finish, dim3((unsigned)(((long long)M * (N / 4) + 255) / 256)), dim3(256), 0, s, g);
    DR_TRY(dr_check_launch("s3_finish"));
  }
  return DR_OK;
}

// ---------------------------------------------------------------------------
// TN products (the weight gradients of the Linears over many rows:
// dW[m][n] = sum_k G[k][m] X[k][n], k = rows, WorldModel.training_step's
// heads / decoder / posterior-scan layers, Agent.train_step's actor and
// critic), f32-accurate on the bf16 MFMA.  Both operands are activations in
// row-major [K][.] layout: each is split3 (truncation split) ONCE by a repack
// pass into chunk-major planes [K/32][3][P][32] (P = M or N rounded up to
// 128, zero past the edge and past K), so the GEMM loop stages both operands
// as whole 16-byte units (no split VALU, no transpose in the loop), with the
// k_gemm_split3 tile, swizzle and six-product order; split-K over workgroups
// while the tile grid is under two workgroups per CU, partial planes reduced
// in a fixed order.
// ---------------------------------------------------------------------------
static int s3_pad(int n) { return (n + 127) / 128 * 128; }

// thread = (column n, 32-row chunk kc): 32 rows of one column (coalesced over
// the threads of a row), split and written as three 64-byte plane runs
// (TERMS = 1: plane 0 only, RNE -- the bf16 world-model step)
struct KnRepack {
  int K, N, P, nsplit;
  const float* X;
  const float* X2;
  long long ldx, ldx2;
  u16* wr;
  long long pad_;  // 16-byte multiple (staged in LDS)
};

template <int TERMS>
__device__ __forceinline__ void kn_repack_body(int K, int N, int P, const float* __restrict__ X, long long ldx,
                                               const float* __restrict__ X2, long long ldx2, int nsplit,
                                               u16* __restrict__ wr) {
  const int n = blockIdx.x * 256 + threadIdx.x, kc = blockIdx.y;
  if (n >= P) return;
  const bool seg2 = n >= nsplit;
  const float* src = seg2 ? X2 : X;
  const long long ld = seg2 ? ldx2 : ldx;
  const int nn = seg2 ? n - nsplit : n;
  // unconditional loads (clamped address, zeroed after): a bounds-checked
  // load compiled to a branch that waited for each of the 32 loads in turn
  // (16 us per world-model weight-gradient repack, r04zc)
  float v[32];
  const bool nok = n < N;
  const float* col = src + (nok ? nn : 0);
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const int kk = 32 * kc + k;
    const bool ok = nok && kk < K;
    const float t = col[ok ? (long long)kk * ld : 0LL];
    v[k] = ok ? t : 0.f;
  }
  u32x4* o = reinterpret_cast<u32x4*>(wr + (((long long)kc * 3) * P + n) * 32);
  if constexpr (TERMS == 1) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      u32x4 h;
#pragma unroll
      for (int e = 0; e < 4; ++e) h[e] = pack_bf16x2(v[8 * u + 2 * e], v[8 * u + 2 * e + 1]);
      o[u] = h;
    }
    return;
  }
  u32x4 h[4], m[4], l[4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      unsigned hh, mm, ll;
      split3_pair(v[8 * u + 2 * e], v[8 * u + 2 * e + 1], hh, mm, ll);
      h[u][e] = hh;
      m[u][e] = mm;
      l[u][e] = ll;
    }
  const long long pl = (long long)P * 32 / 8;  // plane stride in u32x4 units
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    o[u] = h[u];
    o[pl + u] = m[u];
    o[2 * pl + u] = l[u];
  }
}

struct GemmPP {
  int M, N, K, Mp, Np, splits, accumulate, tiles;  // tiles: output tiles of the launch's BM x BN shape
  long long ldy;
  const u16* wa;  // planes of the A side (rows m), [K/32][3][Mp][32]
  const u16* wb;  // planes of the B side (rows n), [K/32][3][Np][32]
  float* Y;
  float* part;    // splits > 1: [splits][M][N] partial sums
  long long pad_;  // 16-byte multiple (staged in LDS)
};

// up to DR_TN_MAX weight-gradient problems of one backward stage in one
// launch per pass (repack, products, split-K finish): the actor's four and
// the critic's three were 12 / 9 dependent launches of a few us each.  Every
// problem keeps its own planes, splits and summation order, so the grouped
// launch is bitwise the one-at-a-time sequence.
#define DR_TN_MAX 4
struct TnBatch {
  KnRepack r[2 * DR_TN_MAX];  // repack operands (G of problem i at 2 i, X at 2 i + 1)
  GemmPP g[DR_TN_MAX];
  int blk0[DR_TN_MAX + 1];    // first flat product block of problem i (tiles * splits each); [n..] = total
  int fin0[DR_TN_MAX + 1];    // first finish block of problem i (0 blocks when splits == 1); [n..] = total
  int n, nrep, pad_[2];
};

template <int TERMS>
__global__ __launch_bounds__(256) void k_kn_repack_multi(TnBatch b) {
  __shared__ __attribute__((aligned(16))) KnRepack s;
  dr_stage_args(b.r[blockIdx.z], s, threadIdx.x);
  const int P = dr_uni(s.P), K = dr_uni(s.K);
  if ((int)blockIdx.x * 256 >= P || (int)blockIdx.y * 32 >= K) return;
  kn_repack_body<TERMS>(K, dr_uni(s.N), P, dr_uni(s.X), s.ldx, dr_uni(s.X2), s.ldx2, dr_uni(s.nsplit), dr_uni(s.wr));
}

// the flat block list: problem z (uniform), then split and tile within it
__device__ __forceinline__ int tn_find(const int* blk0, int flat) {
  int z = 0;
#pragma unroll
  for (int i = 1; i < DR_TN_MAX; ++i)
    if (flat >= blk0[i]) z = i;
  return z;
}

template <int BM, int BN, int TERMS = 3>
__global__ __launch_bounds__(BM * 2) void k_gemm_pp_multi(TnBatch b) {
  constexpr int NT = BM * 2;
  constexpr int WTN = BN / 2, FM = 4, FN = WTN / 16;
  constexpr int AU = TERMS * BM * 4, BU = TERMS * BN * 4;
  constexpr int APT = (AU + NT - 1) / NT, BPT = (BU + NT - 1) / NT;
  static_assert(FN >= 1 && BM % 64 == 0 && (TERMS == 1 || TERMS == 3), "gemm_pp tile");
  __shared__ __attribute__((aligned(16))) u32x4 As[2][TERMS][BM][4];
  __shared__ __attribute__((aligned(16))) u32x4 Bs[2][TERMS][BN][4];
  __shared__ __attribute__((aligned(16))) GemmPP s_g;
  const int flat = dr_xcd_tile(blockIdx.x, b.blk0[DR_TN_MAX]);
  if (flat < 0) return;
  const int z = tn_find(b.blk0, flat);
  dr_stage_args(b.g[z], s_g, threadIdx.x);
  const int M = dr_uni(s_g.M), N = dr_uni(s_g.N), Mp = dr_uni(s_g.Mp), Np = dr_uni(s_g.Np);
  const int tiles = dr_uni(s_g.tiles), splits = dr_uni(s_g.splits);
  const int local = flat - b.blk0[z];
  const int split = local / tiles, lt = local - split * tiles;
  const int tiles_n = (N + BN - 1) / BN;
  const int m0 = (lt / tiles_n) * BM, n0 = (lt % tiles_n) * BN;
  const DR_GLOBAL u16* wa = dr_g(dr_uni(s_g.wa));
  const DR_GLOBAL u16* wb = dr_g(dr_uni(s_g.wb));
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 15, q = lane >> 4;
  const int NCH = (dr_uni(s_g.K) + 31) / 32;
  const int per = (NCH + splits - 1) / splits;
  const int c0 = min(NCH, split * per), c1 = min(NCH, c0 + per);
  u32x4 ra0[APT], ra1[APT], rb0[BPT], rb1[BPT];
  auto load = [&](int c, auto slot) __attribute__((always_inline)) {
    u32x4* ra = decltype(slot)::value == 0 ? ra0 : ra1;
    u32x4* rb = decltype(slot)::value == 0 ? rb0 : rb1;
#pragma unroll
    for (int j = 0; j < APT; ++j) {
      const int e = tid + NT * j;
      if (AU % NT == 0 || e < AU) {
        const int pl = e / (BM * 4), rm = e - pl * BM * 4, row = rm >> 2, u = rm & 3;
        ra[j] = *reinterpret_cast<const DR_GLOBAL u32x4*>(wa + (((long long)c * 3 + pl) * Mp + m0 + row) * 32 + 8 * u);
      }
    }
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int e = tid + NT * j;
      if (BU % NT == 0 || e < BU) {
        const int pl = e / (BN * 4), rm = e - pl * BN * 4, row = rm >> 2, u = rm & 3;
        rb[j] = *reinterpret_cast<const DR_GLOBAL u32x4*>(wb + (((long long)c * 3 + pl) * Np + n0 + row) * 32 + 8 * u);
      }
    }
  };
  auto store = [&](auto slot, int buf) __attribute__((always_inline)) {
    const u32x4* ra = decltype(slot)::value == 0 ? ra0 : ra1;
    const u32x4* rb = decltype(slot)::value == 0 ? rb0 : rb1;
#pragma unroll
    for (int j = 0; j < APT; ++j) {
      const int e = tid + NT * j;
      if (AU % NT == 0 || e < AU) {
        const int pl = e / (BM * 4), rm = e - pl * BM * 4, row = rm >> 2, u = rm & 3;
        As[buf][pl][row][u ^ swz(row)] = ra[j];
      }
    }
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int e = tid + NT * j;
      if (BU % NT == 0 || e < BU) {
        const int pl = e / (BN * 4), rm = e - pl * BN * 4, row = rm >> 2, u = rm & 3;
        Bs[buf][pl][row][u ^ swz(row)] = rb[j];
      }
    }
  };
  const int wm0 = (wave >> 1) * 64, wn0 = (wave & 1) * WTN;
  const int fu = q ^ swz(r);
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if (c0 < c1) {
    load(c0, S0{});
    load(min(c0 + 1, c1 - 1), S1{});
    store(S0{}, 0);
    __syncthreads();
    auto step = [&](int c, auto slot) __attribute__((always_inline)) {
      constexpr int SL = decltype(slot)::value;
      using Next = std::integral_constant<int, 1 - SL>;
      const int buf = (c - c0) & 1;
      load(min(c + 2, c1 - 1), slot);
      u32x4 av[TERMS][FM], bv[TERMS][FN];
#pragma unroll
      for (int pl = 0; pl < TERMS; ++pl) {
#pragma unroll
        for (int i = 0; i < FM; ++i) av[pl][i] = As[buf][pl][wm0 + 16 * i + r][fu];
#pragma unroll
        for (int j = 0; j < FN; ++j) bv[pl][j] = Bs[buf][pl][wn0 + 16 * j + r][fu];
      }
#define DR_P3(PA, PB)                                                                                   \
  _Pragma("unroll") for (int i = 0; i < FM; ++i) _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[i][j] = \
      mfma_b16(bv[PB][j], av[PA][i], acc[i][j]);
      if constexpr (TERMS == 3) {
        DR_P3(2, 0)
        DR_P3(1, 1)
        DR_P3(0, 2)
        DR_P3(1, 0)
        DR_P3(0, 1)
      }
      DR_P3(0, 0)
#undef DR_P3
      if (c + 1 < c1) store(Next{}, buf ^ 1);
      dr_lds_barrier();
    };
    int c = c0;
    for (; c + 1 < c1; c += 2) {
      step(c, S0{});
      step(c + 1, S1{});
    }
    if (c < c1) step(c, S0{});
  }
  // lane (r, q) of acc[i][j]: row m0 + wm0 + 16 i + r, columns n0 + wn0 + 16 j + 4 q .. + 3
  DR_GLOBAL float* part = dr_g(dr_uni(s_g.part));
  DR_GLOBAL float* Y = dr_g(dr_uni(s_g.Y));
  const long long ldy = s_g.ldy;
  const bool accum = dr_uni(s_g.accumulate) != 0;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m0 + wm0 + 16 * i + r;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + wn0 + 16 * j + 4 * q + e;
        if (n >= N) continue;
        if (splits > 1) {
          part[((long long)split * M + m) * N + n] = acc[i][j][e];
        } else {
          DR_GLOBAL float* y = Y + (long long)m * ldy + n;
          *y = accum ? *y + acc[i][j][e] : acc[i][j][e];
        }
      }
    }
  }
}

// Y (+)= the fixed-order sum of the split-K partials; block -> problem by fin0
__global__ __launch_bounds__(256) void k_pp_finish_multi(TnBatch b) {
  __shared__ __attribute__((aligned(16))) GemmPP s_g;
  const int blk = blockIdx.x;
  if (blk >= b.fin0[DR_TN_MAX]) return;
  const int z = tn_find(b.fin0, blk);
  dr_stage_args(b.g[z], s_g, threadIdx.x);
  const int M = dr_uni(s_g.M), N = dr_uni(s_g.N), splits = dr_uni(s_g.splits);
  const long long i = (long long)(blk - b.fin0[z]) * 256 + threadIdx.x;
  if (i >= (long long)M * N) return;
  const DR_GLOBAL float* part = dr_g(dr_uni(s_g.part));
  const int m = (int)(i / N), n = (int)(i - (long long)m * N);
  float v = 0.f;
  for (int sp = 0; sp < splits; ++sp) v += part[(long long)sp * M * N + i];
  DR_GLOBAL float* y = dr_g(dr_uni(s_g.Y)) + (long long)m * s_g.ldy + n;
  *y = dr_uni(s_g.accumulate) ? *y + v : v;
}

#define DR_PP_SPLITS 8
size_t op_gemm_tn_split3_ws_bytes(int M, int N, int K) {
  const size_t kc = (size_t)((K + 31) / 32);
  const size_t planes = kc * 32 * 3 * (size_t)(s3_pad(M) + s3_pad(N)) * sizeof(u16);
  return planes + 256 + (size_t)DR_PP_SPLITS * M * N * sizeof(float);
}

bool op_gemm_tn_split3_supported(int M, int N, int K) {
  // the planes [K/32][3][P][32] are addressed with 32-bit element offsets,
  // the split-K partials with 32-bit row offsets
  return M > 0 && N > 0 && K > 0 && (long long)s3_pad(std::max(M, N)) * (((long long)K + 31) & ~31LL) * 3 < (1LL << 31) &&
         (long long)DR_PP_SPLITS * M * N < (1LL << 31);
}

// host-side probe of the predicate (tests/test_host.py; not part of include/dreamer_hip.h)
extern "C" int dr_internal_tn_split3_supported(int M, int N, int K) { return op_gemm_tn_split3_supported(M, N, K); }

size_t op_gemm_tn_split3_multi_ws_bytes(const TnProblem* p, int n) {
  size_t t = 0;
  for (int i = 0; i < n; ++i) t += op_gemm_tn_split3_ws_bytes(p[i].M, p[i].N, p[i].K);
  return t;
}

int op_gemm_tn_split3_multi(const TnProblem* p, int n, void* ws, size_t ws_bytes, hipStream_t s, int terms) {
  if (n < 1 || n > DR_TN_MAX || (terms != 1 && terms != 3) || op_gemm_tn_split3_multi_ws_bytes(p, n) > ws_bytes) {
    dr_set_error("gemm_tn_split3: %d problems, terms %d, or workspace too small", n, terms);
    return DR_E_INVALID;
  }
  for (int i = 0; i < n; ++i) {
    const TnProblem& q = p[i];
    if (!op_gemm_tn_split3_supported(q.M, q.N, q.K) || !q.G || !q.X || !q.Y || (q.nsplitB < q.N && !q.X2)) {
      dr_set_error("gemm_tn_split3: unsupported problem (M=%d N=%d K=%d)", q.M, q.N, q.K);
      return DR_E_INVALID;
    }
  }
  TnBatch b = {};
  b.n = n;
  b.nrep = 2 * n;
  bool big[DR_TN_MAX];
  int pmax = 0, kcmax = 0;
  char* cur = reinterpret_cast<char*>(ws);
  for (int i = 0; i < n; ++i) {
    const TnProblem& q = p[i];
    const int KC = (q.K + 31) / 32, Mp = s3_pad(q.M), Np = s3_pad(q.N);
    u16* wa = reinterpret_cast<u16*>(cur);
    u16* wb = wa + (size_t)KC * 32 * 3 * Mp;
    float* part = reinterpret_cast<float*>(((uintptr_t)(wb + (size_t)KC * 32 * 3 * Np) + 255) & ~(uintptr_t)255);
    cur += op_gemm_tn_split3_ws_bytes(q.M, q.N, q.K);
    const int nsB = q.nsplitB < q.N ? q.nsplitB : q.N;
    b.r[2 * i] = {q.K, q.M, Mp, q.M, q.G, q.G, q.ldg, q.ldg, wa, 0};
    b.r[2 * i + 1] = {q.K, q.N, Np, nsB, q.X, q.X2 ? q.X2 : q.X, q.ldx, q.X2 ? q.ldx2 : q.ldx, wb, 0};
    pmax = std::max(pmax, std::max(Mp, Np));
    kcmax = std::max(kcmax, KC);
    auto tl = [&](int bm, int bn) { return ((q.M + bm - 1) / bm) * ((q.N + bn - 1) / bn); };
    big[i] = tl(128, 64) >= 512;
    const int tiles = big[i] ? tl(128, 64) : tl(64, 64);
    // split K while the grid is under two workgroups per CU, >= 8 chunks per split
    int splits = 1;
    while (splits < DR_PP_SPLITS && tiles * splits < 512 && KC / (2 * splits) >= 8) splits *= 2;
    b.g[i] = {q.M, q.N, q.K, Mp, Np, splits, q.accumulate, tiles, q.ldy, wa, wb, q.Y, part, 0};
  }
  const dim3 rgrid((unsigned)((pmax + 255) / 256), (unsigned)kcmax, (unsigned)(2 * n));
  if (terms == 1)
    hipLaunchKernelGGL(k_kn_repack_multi<1>, rgrid, dim3(256), 0, s, b);
  else
    hipLaunchKernelGGL(k_kn_repack_multi<3>, rgrid, dim3(256), 0, s, b);
  DR_TRY(dr_check_launch("kn_repack_multi"));
  // products: one launch per tile shape present (problems of the other shape
  // get no blocks: their blk0 run is empty)
  for (int shape = 0; shape < 2; ++shape) {
    const bool want_big = shape == 1;
    TnBatch c = b;
    int tot = 0, any = 0;
    for (int i = 0; i < DR_TN_MAX; ++i) {
      c.blk0[i] = tot;
      if (i < n && big[i] == want_big) {
        tot += b.g[i].tiles * b.g[i].splits;
        any = 1;
      }
    }
    c.blk0[DR_TN_MAX] = tot;
    if (!any) continue;
    const dim3 grid((unsigned)dr_xcd_grid(tot));
    if (want_big) {
      if (terms == 1) hipLaunchKernelGGL((k_gemm_pp_multi<128, 64, 1>), grid, dim3(256), 0, s, c);
      else hipLaunchKernelGGL((k_gemm_pp_multi<128, 64, 3>), grid, dim3(256), 0, s, c);
    } else {
      if (terms == 1) hipLaunchKernelGGL((k_gemm_pp_multi<64, 64, 1>), grid, dim3(128), 0, s, c);
      else hipLaunchKernelGGL((k_gemm_pp_multi<64, 64, 3>), grid, dim3(128), 0, s, c);
    }
    DR_TRY(dr_check_launch("gemm_pp_multi"));
  }
  int fb = 0;
  for (int i = 0; i < DR_TN_MAX; ++i) {
    b.fin0[i] = fb;
    if (i < n && b.g[i].splits > 1) fb += (int)(((long long)b.g[i].M * b.g[i].N + 255) / 256);
  }
  b.fin0[DR_TN_MAX] = fb;
  if (fb > 0) {
    hipLaunchKernelGGL(k_pp_finish_multi, dim3((unsigned)fb), dim3(256), 0, s, b);
    DR_TRY(dr_check_launch("pp_finish_multi"));
  }
  return DR_OK;
}

int op_gemm_tn_split3(int M, int N, int K, const float* G, long long ldg, const float* X, long long ldx,
                      const float* X2, long long ldx2, int nsplitB, float* Y, long long ldy, int accumulate, void* ws,
                      size_t ws_bytes, hipStream_t s, int terms) {
  const TnProblem q = {M, N, K, G, ldg, X, ldx, X2, ldx2, nsplitB, Y, ldy, accumulate};
  return op_gemm_tn_split3_multi(&q, 1, ws, ws_bytes, s, terms);
}
