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
}  // namespace

template <int BM, int BN, int CIN, bool OUT_NCHW, int PIPE>
__global__ __launch_bounds__(BM * 2) void k_conv_split3(int n_frames, int ih, int iw, int cout,
                                                         const float* __restrict__ in, const u16* __restrict__ wr,
                                                         const float* __restrict__ bias, float* __restrict__ out) {
  constexpr int NT = BM * 2;         // WM = BM / 64 waves over pixels x 2 waves over channels
  constexpr int K = CIN * 16;
  constexpr int NCH = K / 32;
  constexpr int WTN = BN / 2, FM = 4, FN = WTN / 16;
  constexpr int APT = BM * 8 / NT;   // float4 of A per thread per chunk (= 4)
  constexpr int BU = 3 * BN * 4;     // 16-byte B units per chunk (3 planes x BN rows x 4)
  constexpr int BPT = (BU + NT - 1) / NT;
  static_assert(CIN % 32 == 0 && APT == 4 && FN >= 1, "conv_split3 tile");
  __shared__ __attribute__((aligned(16))) u32x4 As[2][3][BM][4];
  __shared__ __attribute__((aligned(16))) u32x4 Bs[2][3][BN][4];

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
  u32x4 rb0[BPT], rb1[BPT];
  unsigned ok0 = 0, ok1 = 0;  // per slot: bit i = A row i's tap is inside the frame
  auto load = [&](int c, auto slot) __attribute__((always_inline)) {
    f32x4* ra = decltype(slot)::value == 0 ? ra0 : ra1;
    unsigned& okm = decltype(slot)::value == 0 ? ok0 : ok1;
    u32x4* rb = decltype(slot)::value == 0 ? rb0 : rb1;
    // CIN % 32 == 0: a chunk is 32 channels of one tap (uniform over the workgroup)
    const int tap = (32 * c) / CIN, ci0 = 32 * c - tap * CIN;
    const int ky = tap >> 2, kx = tap & 3;
    const int toff = (ky * iw + kx) * CIN + ci0 + 4 * quad;
    unsigned om = 0u;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      // always load (padding taps read offset 0) and zero the padding at the
      // LDS store: a conditional load compiled to a branch that waited for
      // each load before issuing the next
      const bool ok = (vm[i] >> ky) & (vm[i] >> (4 + kx)) & 1u;
      ra[i] = *reinterpret_cast<const f32x4*>(in + (ok ? pb[i] + toff : 0));
      om |= ok ? (1u << i) : 0u;
    }
    okm = om;
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int e = tid + NT * j;  // (plane, row, unit)
      if (BU % NT == 0 || e < BU) {
        const int pl = e / (BN * 4), rem = e - pl * BN * 4, row = rem >> 2, u = rem & 3;
        rb[j] = *reinterpret_cast<const u32x4*>(wr + (((long long)c * 3 + pl) * cout + n0 + row) * 32 + 8 * u);
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
    u32x4 a[3][FM], b[3][FN];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int i = 0; i < FM; ++i) a[pl][i] = As[buf][pl][wm0 + 16 * i + r][fu];
#pragma unroll
      for (int j = 0; j < FN; ++j) b[pl][j] = Bs[buf][pl][wn0 + 16 * j + r][fu];
    }
    // smallest terms first; independent accumulators innermost
#define DR_S3(PA, PB)                                                                                   \
  _Pragma("unroll") for (int i = 0; i < FM; ++i) _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[i][j] = \
      OUT_NCHW ? mfma_b16(a[PA][i], b[PB][j], acc[i][j]) : mfma_b16(b[PB][j], a[PA][i], acc[i][j]);
    DR_S3(2, 0)
    DR_S3(1, 1)
    DR_S3(0, 2)
    DR_S3(1, 0)
    DR_S3(0, 1)
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
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = dr_silu_fast(v[e]);
        const long long f = m / hw;
        *reinterpret_cast<f32x4*>(out + (f * cout + co) * hw + (m - f * hw)) = v;
      } else {
        const long long m = m0 + wm0 + 16 * i + r;
        const int co = n0 + wn0 + 16 * j + 4 * q;
        if (m >= M) continue;
        const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + co);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = dr_silu_fast(acc[i][j][e] + bv[e]);
        }
        *reinterpret_cast<f32x4*>(out + m * cout + co) = v;
      }
    }
}

// Conv2d weight [co][ci][4][4] f32 -> bf16 [K/32 chunks][3 planes][co][32]
// (k = tap * cin + ci) with w = plane0 + plane1 + plane2 (split3): the BN rows
// of one chunk and plane are one contiguous run of whole 128-byte lines
__global__ void k_conv_repack_split3(int cout, int cin, const float* __restrict__ w, u16* __restrict__ wr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cout * 16 * cin) return;
  const int co = i / (16 * cin), k = i - co * 16 * cin;
  const int tap = k / cin, ci = k - tap * cin;
  unsigned h, m, l;
  split3(w[((long long)co * cin + ci) * 16 + tap], h, m, l);
  const long long base = ((long long)(k >> 5) * 3 * cout + co) * 32 + (k & 31), plane = (long long)cout * 32;
  wr[base] = (u16)h;
  wr[base + plane] = (u16)m;
  wr[base + 2 * plane] = (u16)l;
}

int op_conv_repack_split3(int cout, int cin, const float* w, void* wr, hipStream_t s) {
  const int total = cout * 16 * cin;
  hipLaunchKernelGGL(k_conv_repack_split3, dim3((total + 255) / 256), dim3(256), 0, s, cout, cin, w, (u16*)wr);
  return dr_check_launch("conv_repack_split3");
}

template <int BM, int BN, int CIN, bool NCHW, int PIPE>
static int launch_s3(int n, int ih, int iw, int cout, const float* in, const void* wr, const float* bias, float* out,
                     hipStream_t s) {
  const long long M = (long long)n * (ih / 2) * (iw / 2);
  const long long tiles = ((M + BM - 1) / BM) * (cout / BN);
  if (tiles >= (1LL << 30)) {
    dr_set_error("conv_split3: too many tiles");
    return DR_E_INVALID;
  }
  hipLaunchKernelGGL((k_conv_split3<BM, BN, CIN, NCHW, PIPE>), dim3((unsigned)dr_xcd_grid((int)tiles)), dim3(BM * 2), 0,
                     s, n, ih, iw, cout, in, (const u16*)wr, bias, out);
  return dr_check_launch("conv_split3");
}

bool op_conv_split3_supported(int n, int cin, int ih, int iw, int cout) {
  const bool cin_ok = cin == 32 || cin == 64 || cin == 128 || cin == 256;
  return cin_ok && cout % 64 == 0 && ih % 2 == 0 && iw % 2 == 0 && ((ih / 2) * (iw / 2)) % 4 == 0 &&
         (long long)n * ih * iw * cin < (1LL << 31) - (1LL << 20);
}

int op_conv_split3(int n, int cin, int ih, int iw, int cout, const float* in, const void* wr, const float* bias,
                   float* out, int out_nchw, hipStream_t s) {
  if (!op_conv_split3_supported(n, cin, ih, iw, cout)) {
    dr_set_error("conv_split3: unsupported shape (cin=%d ih=%d iw=%d cout=%d)", cin, ih, iw, cout);
    return DR_E_INVALID;
  }
  // measured at 8192 frames (tools/conv_ab.py): 256 x 64 tiles
  // for 64 output channels (980 us; 128 x 64 at two workgroups per CU: 1004),
  // 256 x 128 for 128 / 256 channels (709 / 658 us; 128 x 128: ~1.1 ms): the
  // weights are re-read once per pixel tile, so taller tiles pay
#define DR_S3L(C)                                                                                          \
  if (cin == C) {                                                                                          \
    if (cout % 128 == 0)                                                                                   \
      return out_nchw ? launch_s3<256, 128, C, true, 2>(n, ih, iw, cout, in, wr, bias, out, s)            \
                      : launch_s3<256, 128, C, false, 2>(n, ih, iw, cout, in, wr, bias, out, s);          \
    return out_nchw ? launch_s3<256, 64, C, true, 2>(n, ih, iw, cout, in, wr, bias, out, s)               \
                    : launch_s3<256, 64, C, false, 2>(n, ih, iw, cout, in, wr, bias, out, s);             \
  }
  DR_S3L(32)
  DR_S3L(64)
  DR_S3L(128)
  DR_S3L(256)
#undef DR_S3L
  return DR_E_INVALID;
}
