// bf16 perf mode's encoder convolutions conv3.. (VariationalAutoEncoder.py:33-42,
// k4 s2 p1 + SiLU) as an implicit GEMM whose operands move global -> LDS by
// LDS-DMA (global_load_lds_dwordx4), three stages deep, two workgroups per CU.
//
// Why a second kernel beside k_conv_split3<.., NT3 = 1>: that tiling was built
// for the fp32 mode's six products per block.  With ONE bf16 product per block a
// 32-deep K chunk is 16 MFMAs per wave, ~260 cycles, and its register ring
// staged one chunk ahead: every chunk waited on its L2 / HBM loads (the counter
// pass read 6.2 VALU per MFMA, 45 % of wave time waiting, 0.19 of the bf16 peak
// for conv3, profiles/r05u_pmc_sq_tcc.txt).  Here the staging costs no VGPRs
// and no VALU beyond the addresses, and two workgroups share each CU.
//
// Tile: 256 pixels x 128 output channels, K = tap x 32 channels per chunk
// (conv_chunk's tap-parity order, the same chunk sequence as k_conv_split3, so
// the sums are bitwise the old kernel's), 8 waves as 4 (pixels) x 2 (channels)
// of 64 x 64, v_mfma_f32_16x16x32_bf16 with f32 accumulation.
// LDS: one array of STAGES x (256 A rows + 128 B rows) x 64 bytes (72 KB).  An
// LDS-DMA wave instruction writes 1 KiB contiguously (lane l at base + 16 l:
// 16 rows x 4 units), so the bank-conflict swizzle of the fragment reads
// (unit u of row r at u ^ swz(r)) is applied to the SOURCE address: lane
// (row, slot) fetches unit slot ^ swz(row).  Out-of-frame taps fetch from a
// 16-byte zero block (no branch, no select at the store).
// Pipeline per chunk c (MI355X guide "Pipelining across barriers"):
// s_waitcnt vmcnt(3 x chunks still in flight) -> raw s_barrier (every wave's
// DMA of chunk c has landed; every wave has finished reading chunk c - 1) ->
// issue chunk c + STAGES - 1 into chunk c - 1's stage -> fragment reads ->
// 16 MFMAs.  No __syncthreads() in the loop (its fence would drain the DMA).
#include "conv.h"

#include <algorithm>


namespace {
typedef unsigned short u16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x4 g_mfma(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                  0);
}
__device__ __forceinline__ int g_swz(int row) { return (0x1320 >> (((row >> 2) & 3) * 4)) & 3; }
__device__ __forceinline__ u32x2 g_pack4(f32x4 v) {
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  const bf16x4_t b = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  return __builtin_bit_cast(u32x2, b);
}
// chunk c -> (tap, first channel, chunk index of the tap-major weight planes):
// channel chunks outer, the 16 taps in four parity groups (conv_split.hip conv_chunk)
template <int CIN>
__device__ __forceinline__ void g_chunk(int c, int& tap, int& ci0, int& kc) {
  constexpr int CPT = CIN / 32;
  const int cc = c >> 4, t = c & 15;
  const int g = t >> 2, j = t & 3;
  const int ky = (g >> 1) + 2 * (j >> 1), kx = (g & 1) + 2 * (j & 1);
  tap = ky * 4 + kx;
  ci0 = 32 * cc;
  kc = tap * CPT + cc;
}
// s_waitcnt vmcnt(3 n): the LDS-DMA of the n newest chunks may stay in flight
__device__ __forceinline__ void g_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
  }
}
__device__ const u16 g_zero16[64] = {0};
}  // namespace

constexpr int GB_M = 256, GB_N = 128, GB_ROWS = GB_M + GB_N;

template <int CIN, bool OUT_NCHW, int STAGES>
__global__ __launch_bounds__(512, STAGES <= 3 ? 4 : 2) void k_conv_glds_bf16(int n_frames, int ih, int iw, int cout,
                                                                               const u16* __restrict__ in,
                                                                               const u16* __restrict__ wr,
                                                                               const float* __restrict__ bias,
                                                                               u16* __restrict__ out) {
  constexpr int K = CIN * 16, NCH = K / 32;
  static_assert(CIN % 32 == 0 && NCH >= STAGES, "conv_glds tile");
  // every LDS byte in ONE array (a second __shared__ object can make hipcc
  // drain the DMA before each fragment read, MI355X guide item 4(a))
  __shared__ __attribute__((aligned(16))) u32x4 sm[STAGES * GB_ROWS * 4];
  const int oh = ih / 2, ow = iw / 2, hw = oh * ow;
  const long long M = (long long)n_frames * hw;
  const int tiles_n = cout / GB_N;
  const long long tiles = ((M + GB_M - 1) / GB_M) * tiles_n;
  const int lt = dr_xcd_tile(blockIdx.x, (int)tiles);
  if (lt < 0) return;
  const long long m0 = (long long)(lt / tiles_n) * GB_M;
  const int n0 = (lt % tiles_n) * GB_N;
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;

  // DMA roles: A rows (2 wave instructions per wave), B rows (1)
  const int lrow = lane >> 2, slot = lane & 3;
  int pb[2];
  unsigned vm[2];
  int au[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 16 + lrow;
    const long long m = m0 + row;
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
    au[i] = 8 * (slot ^ g_swz(row));
  }
  const int brow = wave * 16 + lrow;
  const long long bbase = (long long)(n0 + brow) * 32 + 8 * (slot ^ g_swz(brow));

  auto issue = [&](int c) __attribute__((always_inline)) {
    int tap, ci0, kc;
    g_chunk<CIN>(c, tap, ci0, kc);
    const int ky = tap >> 2, kx = tap & 3;
    const int toff = (ky * iw + kx) * CIN + ci0;
    u32x4* st = sm + (c % STAGES) * GB_ROWS * 4;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool ok = (vm[i] >> ky) & (vm[i] >> (4 + kx)) & 1u;
      const u16* src = ok ? in + (pb[i] + toff + au[i]) : g_zero16;
      __builtin_amdgcn_global_load_lds(src, st + (wave * 2 + i) * 16 * 4, 16, 0, 0);
    }
    __builtin_amdgcn_global_load_lds(wr + ((long long)kc * 3 * cout) * 32 + bbase, st + (GB_M + wave * 16) * 4, 16, 0,
                                     0);
  };

  const int wm0 = (wave >> 1) * 64, wn0 = (wave & 1) * 64;
  const int fu = q ^ g_swz(r);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int c = 0; c < STAGES - 1; ++c) issue(c);
#pragma unroll 1
  for (int c = 0; c < NCH; ++c) {
    // chunks c .. min(c + STAGES - 2, NCH - 1) are in flight: retire chunk c
    g_vmcnt(min(STAGES - 2, NCH - 1 - c));
    __builtin_amdgcn_s_barrier();
    if (c + STAGES - 1 < NCH) issue(c + STAGES - 1);
    const u32x4* st = sm + (c % STAGES) * GB_ROWS * 4;
    u32x4 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = st[(wm0 + 16 * i + r) * 4 + fu];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = st[(GB_M + wn0 + 16 * j + r) * 4 + fu];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = OUT_NCHW ? g_mfma(a[i], b[j], acc[i][j]) : g_mfma(b[j], a[i], acc[i][j]);
  }

  // NHWC: lane (r, q) holds channels 4q..4q+3 of pixel r; NCHW: pixels 4q..4q+3 of channel r
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (OUT_NCHW) {
        const long long m = m0 + wm0 + 16 * i + 4 * q;
        const int co = n0 + wn0 + 16 * j + r;
        if (m >= M) continue;
        const float bv = bias[co];
        f32x4 v = acc[i][j] + bv;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = dr_silu_fast(v[e]);
        const long long f = m / hw;
        *reinterpret_cast<u32x2*>(out + (f * cout + co) * hw + (m - f * hw)) = g_pack4(v);
      } else {
        const long long m = m0 + wm0 + 16 * i + r;
        const int co = n0 + wn0 + 16 * j + 4 * q;
        if (m >= M) continue;
        const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + co);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = dr_silu_fast(acc[i][j][e] + bv[e]);
        *reinterpret_cast<u32x2*>(out + m * cout + co) = g_pack4(v);
      }
    }
}

bool op_conv_glds_bf16_supported(int n, int cin, int ih, int iw, int cout) {
  return (cin == 32 || cin == 64 || cin == 128 || cin == 256) && cout % GB_N == 0 && ih % 2 == 0 && iw % 2 == 0 &&
         ((ih / 2) * (iw / 2)) % 4 == 0 && (long long)n * ih * iw * cin < (1LL << 31) - (1LL << 20);
}

template <int C, bool NCHW>
static int launch_glds(int n, int ih, int iw, int cout, const void* in, const void* wr, const float* bias, void* out,
                       hipStream_t s) {
  const long long M = (long long)n * (ih / 2) * (iw / 2);
  const long long tiles = ((M + GB_M - 1) / GB_M) * (cout / GB_N);
  if (tiles >= (1LL << 30)) {
    dr_set_error("conv_glds_bf16: too many tiles");
    return DR_E_INVALID;
  }
  // (the ping-pong form of k_conv_glds_s3 in one term -- 512 x 128 tiles, 32
  // MFMAs per phase, one workgroup per CU -- measured slower: 235 / 188 us
  // against 182 / 137, bf16 headline 921 -> 898 k; with no split there is
  // little for the read phase to hide, profiles/r06zb_ab_b16_pingpong.txt)
  // three stages, two workgroups per CU (72 KB of LDS, 100 VGPRs): B = 256 bf16
  // encoder conv3 / conv4 181 / 138 us, against 219 / 180 (four stages, one
  // workgroup per CU), 229 / 186 (six) and 288 / 173 on k_conv_split3<.., 1>
  // (profiles/r06g_ab_conv_glds.txt)
  hipLaunchKernelGGL((k_conv_glds_bf16<C, NCHW, 3>), dim3((unsigned)dr_xcd_grid((int)tiles)), dim3(512), 0, s, n, ih,
                     iw, cout, (const u16*)in, (const u16*)wr, bias, (u16*)out);
  return dr_check_launch("conv_glds_bf16");
}

// bf16 NHWC in, bf16 NHWC / NCHW out, weights as op_conv_repack_split3 planes
// (plane 0 = their RNE bf16); DR_E_INVALID (nothing launched) for other shapes
int op_conv_glds_bf16(int n, int cin, int ih, int iw, int cout, const void* in, const void* wr, const float* bias,
                      void* out, int out_nchw, hipStream_t s) {
  if (!op_conv_glds_bf16_supported(n, cin, ih, iw, cout) || (((uintptr_t)in | (uintptr_t)out | (uintptr_t)bias) & 15)) {
    dr_set_error("conv_glds_bf16: unsupported shape (cin=%d ih=%d iw=%d cout=%d)", cin, ih, iw, cout);
    return DR_E_INVALID;
  }
#define DR_GL(C)                                                                                  \
  if (cin == C)                                                                                   \
    return out_nchw ? launch_glds<C, true>(n, ih, iw, cout, in, wr, bias, out, s)                 \
                    : launch_glds<C, false>(n, ih, iw, cout, in, wr, bias, out, s);
  DR_GL(32)
  DR_GL(64)
  DR_GL(128)
  DR_GL(256)
#undef DR_GL
  return DR_E_INVALID;
}

// ---------------------------------------------------------------------------
// fp32 mode's encoder convolutions conv3.. on the same LDS-DMA staging:
// f32-accurate (the six split3 products of conv_split.hip's header) with the
// f32 NHWC activations moved global -> LDS by LDS-DMA as they are, and split
// per wave when the fragments are read.
//
// Why: k_conv_split3 (256 x 128 tiles, register-staged) splits each staged
// float4 once per workgroup, but the staging sits between two barriers of the
// chunk loop -- every wave loads, splits, stores to LDS, waits, then runs its
// 96 MFMAs -- so the split and the LDS stores never overlap the MFMA pipe:
// 0.45-0.47 of the split ceiling (conv3 718 us, conv4 692 us at 8192 frames,
// profiles/r06z_epoch_kernel_table.txt).  Here the staging is LDS-DMA (8 or 6
// instructions per wave and chunk); each wave owns 32 pixel rows x all 128
// channels (8 waves x 1), so an A fragment is split by exactly one wave (no
// duplicated split: 16 f32 per lane and chunk, ~1 VALU per MFMA), and the two
// waves of a SIMD ping-pong between reading and multiplying (below): conv3 /
// conv4 627 / 587 us, ~1.3-1.4 PFLOP/s of bf16 MFMA work under the chip's
// load clock (profiles/r06z4_ab_conv_glds_s3.txt).  The per-accumulator order of
// the six products and the chunk sequence are k_conv_split3's, so the output
// is bitwise that kernel's.
// LDS per stage: A 256 rows x 128 B (f32, 8 units a row, unit u of row r at
// u ^ f[(r >> 1) & 7], f = {0,1,0,1,6,7,6,7}: the two ds_read_b128 of a lane
// (units 2q, 2q + 1) are conflict-free in every 16-lane group of the b128
// read) + B 3 planes x 128 rows x 64 B (g_swz); 56 KB, two stages, one
// workgroup (8 waves, 2 per SIMD) per CU.
// ---------------------------------------------------------------------------
namespace {
__device__ __forceinline__ int g_swz8(int row) { return (0x76761010 >> (((row >> 1) & 7) * 4)) & 7; }
__device__ const float g_zero32[16] = {0.f};
}  // namespace


// BN = 128 or 64 output channels per tile, RW = 32 or 64 pixel rows per wave (8 RW per tile); EPI =
// CONV_EPI_FWD or (NHWC) CONV_EPI_DSILU: out = acc * SiLU'(pre)
// TR: the upsampling k4 s2 p1 form of conv_split.hip's k_convT_split3 (per output
// parity class a dense K = 4 taps x CIN over input-resolution pixels; weights
// [class][K/32][3][cout][32]; its CT_EPI_BIAS / CT_EPI_DSILU epilogues), with the
// same tile, chunk and product order: bitwise that kernel's sums.
struct GS3Args {
  int n, ih, iw, cout, silu_out;  // TR: ih, iw = the input resolution
  const float* in;
  const u16* wr;
  const float* bias;
  float* out;
  float* out2;  // TR, CT_EPI_BIAS: optional SiLU(acc + bias)
  float* pre;
};

template <int CIN, bool OUT_NCHW, int BN, int EPI, int RW = 32, bool TR = false>
__global__ __launch_bounds__(512, 2) void k_conv_glds_s3(GS3Args g) {
  const int ih = g.ih, iw = g.iw, cout = g.cout;
  const float* __restrict__ in = g.in;
  const float* __restrict__ bias = g.bias;
  float* __restrict__ out = g.out;
  float* __restrict__ pre = g.pre;
  constexpr int K = TR ? CIN * 4 : CIN * 16, NCH = K / 32;
  constexpr int GS_M = 8 * RW, GS_N = BN, GS_AU = GS_M * 8, GS_STU = GS_AU + 3 * BN * 4;  // 16-byte units per stage
  constexpr int FM = RW / 16, FN = BN / 16;
  static_assert(CIN % 32 == 0 && NCH >= 2 && (BN == 128 || BN == 64) && (RW == 32 || RW == 64) &&
                    (EPI == CONV_EPI_FWD || !OUT_NCHW) && (!TR || !OUT_NCHW),
                "conv_glds_s3 tile");
  __shared__ __attribute__((aligned(16))) u32x4 sm[2 * GS_STU];
  const int oh = TR ? ih : ih / 2, ow = TR ? iw : iw / 2, hw = oh * ow;  // pixels of the GEMM rows
  const long long M = (long long)g.n * hw;
  const int tiles_n = cout / GS_N;
  const long long tiles = ((M + GS_M - 1) / GS_M) * tiles_n * (TR ? 4 : 1);
  const int lt = dr_xcd_tile(blockIdx.x, (int)tiles);
  if (lt < 0) return;
  // TR: parity class fastest (the four classes of one pixel tile read the same input, k_convT_split3)
  const int cls = TR ? (lt & 3) : 0, py = cls >> 1, px = cls & 1;
  const int lr = TR ? (lt >> 2) : lt;
  const long long m0 = (long long)(lr / tiles_n) * GS_M;
  const int n0 = (lr % tiles_n) * GS_N;
  const u16* __restrict__ wr = g.wr + (TR ? (long long)cls * NCH * 3 * cout * 32 : 0);
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;

  // Ping-pong: waves 0-3 (X, one per SIMD) and 4-7 (Y) alternate between
  // barrier-separated phases -- while X runs its 96 MFMAs on chunk c, Y reads and
  // splits chunk c from LDS; then Y multiplies while X reads chunk c + 1 -- so each
  // SIMD's MFMA pipe is fed by one wave while the other does its LDS / VALU work.
  // DMA of chunk c + 1 (two stages: the stage it refills held chunk c - 1, read
  // by X and Y in the two phases before): X issues the A rows in its read phase
  // of chunk c, Y the B planes in its read phase of chunk c, each waiting for its
  // own before the barrier that precedes X's read of chunk c + 1.  DMA issued
  // inside an MFMA phase measured slower (conv3 631 -> 746 us), all of it by X
  // in its read phase about the same (631 / 591 us against 628 / 587 us,
  // profiles/r06z5_ab_conv_glds_dma.txt).  s_setprio 1 around the MFMA phase:
  // neutral (630 / 588 against 630 / 593 us, profiles/r06za_ab_glds_setprio.txt).
  constexpr int NA = RW / 4, NB = BN / 64;  // DMA instructions per wave: A rows / 8 (X), B rows / 16 per plane (Y)
  const bool X = wave < 4;
  const int dw = wave & 3;
  // A DMA: lane l of instruction i -> row dw * 8 NA + 8 i + l / 8, LDS unit l % 8 = source unit ^ swizzle
  int pb[NA];
  unsigned vm[NA];
  int au[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int row = dw * 8 * NA + i * 8 + (lane >> 3);
    const long long m = m0 + row;
    const int mm = (int)(m < M ? m : 0);
    const int f = mm / hw, p = mm - f * hw, oy = p / ow, ox = p - oy * ow;
    unsigned v = 0u;
    if constexpr (TR) {
      // input pixel (oy, ox) of the class grid; tap t reads (oy + py - t / 2, ox + px - t % 2)
      pb[i] = ((f * ih + oy) * iw + ox) * CIN;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int yy = oy + py - (t >> 1), xx = ox + px - (t & 1);
        v |= (yy >= 0 && yy < ih && xx >= 0 && xx < iw) ? (1u << t) : 0u;
      }
    } else {
      const int y0 = 2 * oy - 1, x0 = 2 * ox - 1;
      pb[i] = ((f * ih + y0) * iw + x0) * CIN;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        v |= (y0 + t >= 0 && y0 + t < ih) ? (1u << t) : 0u;
        v |= (x0 + t >= 0 && x0 + t < iw) ? (16u << t) : 0u;
      }
    }
    vm[i] = m < M ? v : 0u;
    au[i] = 4 * ((lane & 7) ^ g_swz8(row));
  }
  // B DMA: 16-row blocks dw * NB + h of each of the 3 planes
  long long bbase[NB];
#pragma unroll
  for (int h = 0; h < NB; ++h) {
    const int brow = (dw * NB + h) * 16 + (lane >> 2);
    bbase[h] = (long long)(n0 + brow) * 32 + 8 * ((lane & 3) ^ g_swz(brow));
  }

  // parts: bit 0 = the A rows, bit 1 = the B planes
  auto issue = [&](int c, int parts) __attribute__((always_inline)) {
    int tap, ci0, kc, toff;
    if constexpr (TR) {  // k_convT_split3's chunk order: tap-major, 32 channels per chunk
      tap = (32 * c) / CIN;
      ci0 = 32 * c - tap * CIN;
      kc = c;
      toff = ((py - (tap >> 1)) * iw + (px - (tap & 1))) * CIN + ci0;
    } else {
      g_chunk<CIN>(c, tap, ci0, kc);
      toff = ((tap >> 2) * iw + (tap & 3)) * CIN + ci0;
    }
    u32x4* st = sm + (c & 1) * GS_STU;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      if (!(parts & 1)) break;
      const bool ok = TR ? ((vm[i] >> tap) & 1u) : ((vm[i] >> (tap >> 2)) & (vm[i] >> (4 + (tap & 3))) & 1u);
      const float* src = ok ? in + (pb[i] + toff + au[i]) : g_zero32;
      __builtin_amdgcn_global_load_lds(src, st + (dw * NA + i) * 64, 16, 0, 0);
    }
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int h = 0; h < NB; ++h) {
        if (!(parts & 2)) break;
        const u16* bs = wr + ((long long)kc * 3 + pl) * cout * 32 + bbase[h];
        u32x4* bd = st + GS_AU + (pl * GS_N + (dw * NB + h) * 16) * 4;
        __builtin_amdgcn_global_load_lds(bs, bd, 16, 0, 0);
      }
  };

  const int wm0 = wave * RW;
  const int fa0 = (2 * q) ^ g_swz8(r), fa1 = (2 * q + 1) ^ g_swz8(r);  // A rows are 16-aligned
  const int fu = q ^ g_swz(r);
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  u32x4 a[3][FM], b[3][FN];
  auto fetch = [&](int c) __attribute__((always_inline)) {
    const u32x4* st = sm + (c & 1) * GS_STU;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const f32x4 v0 = __builtin_bit_cast(f32x4, st[(wm0 + 16 * i + r) * 8 + fa0]);
      const f32x4 v1 = __builtin_bit_cast(f32x4, st[(wm0 + 16 * i + r) * 8 + fa1]);
      unsigned h[4], m[4], l[4];
      split3_pair(v0[0], v0[1], h[0], m[0], l[0]);
      split3_pair(v0[2], v0[3], h[1], m[1], l[1]);
      split3_pair(v1[0], v1[1], h[2], m[2], l[2]);
      split3_pair(v1[2], v1[3], h[3], m[3], l[3]);
      a[0][i] = (u32x4){h[0], h[1], h[2], h[3]};
      a[1][i] = (u32x4){m[0], m[1], m[2], m[3]};
      a[2][i] = (u32x4){l[0], l[1], l[2], l[3]};
    }
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int j = 0; j < FN; ++j) b[pl][j] = st[GS_AU + (pl * GS_N + 16 * j + r) * 4 + fu];
  };
  // k_conv_split3's order per accumulator: smallest terms first
  auto multiply = [&]() __attribute__((always_inline)) {
#define DR_GS3(PA, PB)                                                                                   \
  _Pragma("unroll") for (int i = 0; i < FM; ++i) _Pragma("unroll") for (int j = 0; j < FN; ++j) acc[i][j] = \
      OUT_NCHW ? g_mfma(a[PA][i], b[PB][j], acc[i][j]) : g_mfma(b[PB][j], a[PA][i], acc[i][j]);
    DR_GS3(2, 0)
    DR_GS3(1, 1)
    DR_GS3(0, 2)
    DR_GS3(1, 0)
    DR_GS3(0, 1)
    DR_GS3(0, 0)
#undef DR_GS3
  };

  if (X) {
    issue(0, 3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (!X) __builtin_amdgcn_s_barrier();  // Y runs one phase behind X
#pragma unroll 1
  for (int c = 0; c < NCH; ++c) {
    // read phase: chunk c's fragments into registers, split; chunk c + 1's DMA
    if (c + 1 < NCH) issue(c + 1, X ? 1 : 2);
    fetch(c);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the stage may be refilled after the next barrier
    if (!X) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // MFMA phase
    multiply();
    if (X) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // chunk c + 1's A rows landed before X reads them
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (X) __builtin_amdgcn_s_barrier();

  if constexpr (TR) {
    // k_convT_split3's epilogues at output pixel (2 y + py, 2 x + px): CT_EPI_BIAS out = acc + bias (or its
    // SiLU, silu_out), out2 = SiLU(acc + bias); CT_EPI_DSILU out = acc * SiLU'(pre)
    const int OW = 2 * iw, OH = 2 * ih;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const long long m = m0 + wm0 + 16 * i + r;
      if (m >= M) continue;
      const int f = (int)(m / hw), p = (int)(m - (long long)f * hw), y = p / iw, x = p - y * iw;
      const long long opix = ((long long)f * OH + 2 * y + py) * OW + 2 * x + px;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int co = n0 + 16 * j + 4 * q;
        f32x4 v = acc[i][j];
        if constexpr (EPI == CT_EPI_BIAS) {
          v += *reinterpret_cast<const f32x4*>(bias + co);
          f32x4 sv = v;
          if (g.out2 || g.silu_out) {
#pragma unroll
            for (int e = 0; e < 4; ++e) sv[e] = dr_silu_fast(v[e]);
          }
          *reinterpret_cast<f32x4*>(out + opix * cout + co) = g.silu_out ? sv : v;
          if (g.out2) *reinterpret_cast<f32x4*>(g.out2 + opix * cout + co) = sv;
        } else {
          const f32x4 pv = *reinterpret_cast<const f32x4*>(pre + opix * cout + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] * dr_dsilu_fast(pv[e]);
          *reinterpret_cast<f32x4*>(out + opix * cout + co) = v;
        }
      }
    }
    return;
  }
  // k_conv_split3's epilogues: CONV_EPI_FWD out = SiLU(acc + bias), pre = acc + bias (NHWC) when given;
  // CONV_EPI_DSILU out = acc * SiLU'(pre)
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if (OUT_NCHW) {
        const long long m = m0 + wm0 + 16 * i + 4 * q;
        const int co = n0 + 16 * j + r;
        if (m >= M) continue;
        f32x4 v = acc[i][j] + bias[co];
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
        const int co = n0 + 16 * j + 4 * q;
        if (m >= M) continue;
        if constexpr (EPI == CONV_EPI_DSILU) {
          const f32x4 pv = *reinterpret_cast<const f32x4*>(pre + m * cout + co);
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * dr_dsilu_fast(pv[e]);
          *reinterpret_cast<f32x4*>(out + m * cout + co) = v;
          continue;
        }
        const f32x4 bv = *reinterpret_cast<const f32x4*>(bias + co);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] + bv[e];
        if (pre) *reinterpret_cast<f32x4*>(pre + m * cout + co) = v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = dr_silu_fast(v[e]);
        *reinterpret_cast<f32x4*>(out + m * cout + co) = v;
      }
    }
}

bool op_conv_glds_s3_supported(int n, int cin, int ih, int iw, int cout) {
  return (cin == 32 || cin == 64 || cin == 128 || cin == 256) && cout % 64 == 0 && ih % 2 == 0 && iw % 2 == 0 &&
         ((ih / 2) * (iw / 2)) % 4 == 0 && (long long)n * ih * iw * cin < (1LL << 31) - (1LL << 20);
}

template <int C, bool NCHW, int BN, int EPI>
static int launch_glds_s3(int n, int ih, int iw, int cout, const float* in, const void* wr, const float* bias,
                          float* out, float* pre, hipStream_t s) {
  // 64-channel tiles take 64 pixel rows per wave (512-row tiles): 96 MFMAs per
  // phase as on the 128-channel tiles
  constexpr int RW = BN == 64 ? 64 : 32;
  const long long M = (long long)n * (ih / 2) * (iw / 2);
  const long long tiles = ((M + 8 * RW - 1) / (8 * RW)) * (cout / BN);
  if (tiles >= (1LL << 30)) {
    dr_set_error("conv_glds_s3: too many tiles");
    return DR_E_INVALID;
  }
  GS3Args g = {n, ih, iw, cout, 0, in, (const u16*)wr, bias, out, nullptr, pre};
  hipLaunchKernelGGL((k_conv_glds_s3<C, NCHW, BN, EPI, RW>), dim3((unsigned)dr_xcd_grid((int)tiles)), dim3(512), 0, s, g);
  return dr_check_launch("conv_glds_s3");
}

// f32 NHWC in, f32 NHWC / NCHW out (+ optional NHWC pre-activation), weights as
// op_conv_repack_split3 planes; epi CONV_EPI_FWD (bias given) or, NHWC out only,
// CONV_EPI_DSILU (pre given, no bias); 128-channel tiles where cout allows, else
// 64; DR_E_INVALID (nothing launched) for other shapes
int op_conv_glds_s3(int n, int cin, int ih, int iw, int cout, const float* in, const void* wr, const float* bias,
                    float* out, int out_nchw, float* pre, int epi, hipStream_t s) {
  const bool dsilu = epi == CONV_EPI_DSILU;
  if (!op_conv_glds_s3_supported(n, cin, ih, iw, cout) || (epi != CONV_EPI_FWD && !dsilu) ||
      (dsilu && (out_nchw || !pre)) || (!dsilu && !bias) ||
      (((uintptr_t)in | (uintptr_t)wr | (uintptr_t)out | (uintptr_t)bias | (uintptr_t)pre) & 15)) {
    dr_set_error("conv_glds_s3: unsupported problem (cin=%d ih=%d iw=%d cout=%d epi=%d)", cin, ih, iw, cout, epi);
    return DR_E_INVALID;
  }
#define DR_GL(C, BN)                                                                                             \
  if (cin == C)                                                                                                  \
    return dsilu ? launch_glds_s3<C, false, BN, CONV_EPI_DSILU>(n, ih, iw, cout, in, wr, bias, out, pre, s)      \
                 : out_nchw ? launch_glds_s3<C, true, BN, CONV_EPI_FWD>(n, ih, iw, cout, in, wr, bias, out, pre, s) \
                            : launch_glds_s3<C, false, BN, CONV_EPI_FWD>(n, ih, iw, cout, in, wr, bias, out, pre, s);
  if (cout % 128 == 0) {
    DR_GL(32, 128)
    DR_GL(64, 128)
    DR_GL(128, 128)
    DR_GL(256, 128)
  } else {
    DR_GL(32, 64)
    DR_GL(64, 64)
    DR_GL(128, 64)
    DR_GL(256, 64)
  }
#undef DR_GL
  return DR_E_INVALID;
}

template <int C, int BN, int EPI>
static int launch_glds_t3(const ConvTArgs& a, const void* wr, hipStream_t s) {
  constexpr int RW = BN == 64 ? 64 : 32;
  const long long M = (long long)a.n * a.h * a.w;
  const long long tiles = 4 * ((M + 8 * RW - 1) / (8 * RW)) * (a.cout / BN);
  if (tiles >= (1LL << 30)) {
    dr_set_error("convT_glds_s3: too many tiles");
    return DR_E_INVALID;
  }
  GS3Args g = {a.n, a.h, a.w, a.cout, a.silu_out, a.in, (const u16*)wr, a.bias, a.out, a.out2, const_cast<float*>(a.pre)};
  hipLaunchKernelGGL((k_conv_glds_s3<C, false, BN, EPI, RW, true>), dim3((unsigned)dr_xcd_grid((int)tiles)), dim3(512),
                     0, s, g);
  return dr_check_launch("convT_glds_s3");
}

bool op_convT_glds_s3_supported(const ConvTArgs& a, int epi) {
  const bool cin_ok = a.cin == 32 || a.cin == 64 || a.cin == 128 || a.cin == 256;
  const bool al = !(((uintptr_t)a.in | (uintptr_t)a.out | (uintptr_t)a.out2 | (uintptr_t)a.bias | (uintptr_t)a.pre) & 15);
  return cin_ok && a.cout % 64 == 0 && a.cout > 0 && a.ldc == a.cout && !a.silu_in && al &&
         (epi == CT_EPI_BIAS ? a.bias != nullptr : epi == CT_EPI_DSILU && a.pre != nullptr) &&
         (long long)a.n * a.h * a.w * a.cin < (1LL << 31) - (1LL << 20);
}

// the six-product upsampling conv (k_convT_split3's problems, terms = 3) on the
// LDS-DMA ping-pong kernel; DR_E_INVALID (nothing launched) where unsupported
int op_convT_glds_s3(int epi, const ConvTArgs& a, const void* wr, hipStream_t s) {
  if (!op_convT_glds_s3_supported(a, epi) || ((uintptr_t)wr & 15)) {
    dr_set_error("convT_glds_s3: unsupported problem (cin=%d cout=%d h=%d w=%d epi=%d)", a.cin, a.cout, a.h, a.w, epi);
    return DR_E_INVALID;
  }
#define DR_GT(C, BN)                                                                                  \
  if (a.cin == C)                                                                                     \
    return epi == CT_EPI_DSILU ? launch_glds_t3<C, BN, CT_EPI_DSILU>(a, wr, s) : launch_glds_t3<C, BN, CT_EPI_BIAS>(a, wr, s);
  if (a.cout % 128 == 0) {
    DR_GT(32, 128)
    DR_GT(64, 128)
    DR_GT(128, 128)
    DR_GT(256, 128)
  } else {
    DR_GT(32, 64)
    DR_GT(64, 64)
    DR_GT(128, 64)
    DR_GT(256, 64)
  }
#undef DR_GT
  return DR_E_INVALID;
}

// ---------------------------------------------------------------------------
// bf16 perf mode's encoder feature projection (latent_mapper.0's feature
// columns, VAE.py:71-72): Y[m][n] = X[m][:] . W[n][:] + bias[n] over the B S / 2
// warm-start frames, X = the flattened conv4 output (bf16 [M][K], K = 4096), W
// its bf16 copy [N][K] (N = 200).  The same LDS-DMA pipeline as the convolution
// above on 128 x 64 tiles (4 waves as 2 x 2 of 64 x 32), four stages, split-K
// over blockIdx so that ~512 workgroups run (k_conv_bf16's dense 128 x 128 tiles
// gave 128 workgroups at B = 256 and 32 at B = 64: 72 / 61 us); the partial sums
// meet in a fixed order in k_glds_finish (deterministic).
// ---------------------------------------------------------------------------
constexpr int GP_M = 128, GP_N = 64, GP_ROWS = GP_M + GP_N, GP_ST = 4;

struct GemmGlds {
  int M, N, K, ldx, ldw, ldy, splits, kper;  // kper: K per split (multiple of 32)
  const u16* X;
  const u16* W;
  const float* bias;
  float* Y;     // splits == 1
  float* part;  // [splits][M][N]
};

__global__ __launch_bounds__(256) void k_gemm_glds_bf16(GemmGlds g) {
  __shared__ __attribute__((aligned(16))) u32x4 sm[GP_ST * GP_ROWS * 4];
  const int tiles_m = (g.M + GP_M - 1) / GP_M, tiles_n = (g.N + GP_N - 1) / GP_N;
  const int tiles = tiles_m * tiles_n;
  const int lb = dr_xcd_tile(blockIdx.x, tiles * g.splits);
  if (lb < 0) return;
  const int split = lb / tiles, lt = lb - split * tiles;
  const int m0 = (lt / tiles_n) * GP_M, n0 = (lt % tiles_n) * GP_N;
  const int k_begin = split * g.kper, nch = min(g.kper, g.K - k_begin) / 32;
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r = lane & 15, q = lane >> 4, lrow = lane >> 2, slot = lane & 3;
  const u16* asrc[2];
  bool aok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 16 + lrow;
    aok[i] = m0 + row < g.M;
    asrc[i] = g.X + (long long)(aok[i] ? m0 + row : 0) * g.ldx + k_begin + 8 * (slot ^ g_swz(row));
  }
  const int brow = wave * 16 + lrow;
  const bool bok = n0 + brow < g.N;
  const u16* bsrc = g.W + (long long)(bok ? n0 + brow : 0) * g.ldw + k_begin + 8 * (slot ^ g_swz(brow));
  auto issue = [&](int c) __attribute__((always_inline)) {
    u32x4* st = sm + (c % GP_ST) * GP_ROWS * 4;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds(aok[i] ? asrc[i] + 32 * c : g_zero16, st + (wave * 2 + i) * 16 * 4, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(bok ? bsrc + 32 * c : g_zero16, st + (GP_M + wave * 16) * 4, 16, 0, 0);
  };
  const int wm0 = (wave >> 1) * 64, wn0 = (wave & 1) * 32;
  const int fu = q ^ g_swz(r);
  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < GP_ST - 1 && c < nch; ++c) issue(c);
#pragma unroll 1
  for (int c = 0; c < nch; ++c) {
    g_vmcnt(min(GP_ST - 2, nch - 1 - c));
    __builtin_amdgcn_s_barrier();
    if (c + GP_ST - 1 < nch) issue(c + GP_ST - 1);
    const u32x4* st = sm + (c % GP_ST) * GP_ROWS * 4;
    u32x4 a[4], b[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = st[(wm0 + 16 * i + r) * 4 + fu];
#pragma unroll
    for (int j = 0; j < 2; ++j) b[j] = st[(GP_M + wn0 + 16 * j + r) * 4 + fu];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = g_mfma(b[j], a[i], acc[i][j]);
  }
  // lane (r, q): row m0 + wm0 + 16 i + r, columns n0 + wn0 + 16 j + 4 q .. + 3
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = m0 + wm0 + 16 * i + r, n = n0 + wn0 + 16 * j + 4 * q;
      if (m >= g.M || n >= g.N) continue;
      if (g.splits == 1) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(g.bias + n);
        *reinterpret_cast<f32x4*>(g.Y + (long long)m * g.ldy + n) = acc[i][j] + bv;
      } else {
        *reinterpret_cast<f32x4*>(g.part + ((long long)split * g.M + m) * g.N + n) = acc[i][j];
      }
    }
}

// Y = sum over the splits (ascending) + bias, 4 columns per thread
__global__ void k_glds_finish(GemmGlds g) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int n4 = g.N / 4;
  if (i >= (long long)g.M * n4) return;
  const int m = (int)(i / n4), n = 4 * (int)(i - (long long)m * n4);
  f32x4 v = *reinterpret_cast<const f32x4*>(g.part + (long long)m * g.N + n);
  for (int s = 1; s < g.splits; ++s) v += *reinterpret_cast<const f32x4*>(g.part + ((long long)s * g.M + m) * g.N + n);
  *reinterpret_cast<f32x4*>(g.Y + (long long)m * g.ldy + n) = v + *reinterpret_cast<const f32x4*>(g.bias + n);
}

static int glds_splits(int M, int N, int K) {
  const int tiles = ((M + GP_M - 1) / GP_M) * ((N + GP_N - 1) / GP_N);
  int s = std::max(1, std::min(8, 512 / std::max(1, tiles)));
  while (s > 1 && (K / 32) / s < GP_ST) --s;  // at least a full pipeline of chunks per split
  return s;
}

size_t op_gemm_nt_glds_part_floats(int M, int N, int K) {
  const int s = glds_splits(M, N, K);
  return s > 1 ? (size_t)s * M * N : 0;
}

int op_gemm_nt_glds_bf16(int M, int N, int K, const void* X, int ldx, const void* W, int ldw, const float* bias,
                         float* Y, int ldy, float* part, size_t part_floats, hipStream_t s) {
  if (M <= 0 || N <= 0 || K % 32 || N % 4 || ldx % 8 || ldw % 8 || ldy % 4 || !bias ||
      (((uintptr_t)X | (uintptr_t)W | (uintptr_t)Y | (uintptr_t)bias) & 15)) {
    dr_set_error("gemm_nt_glds_bf16: unsupported problem (M=%d N=%d K=%d)", M, N, K);
    return DR_E_INVALID;
  }
  GemmGlds g;
  g.M = M; g.N = N; g.K = K; g.ldx = ldx; g.ldw = ldw; g.ldy = ldy;
  g.splits = glds_splits(M, N, K);
  g.kper = ((K / 32 + g.splits - 1) / g.splits) * 32;
  g.splits = (K + g.kper - 1) / g.kper;
  g.X = (const u16*)X; g.W = (const u16*)W; g.bias = bias; g.Y = Y; g.part = part;
  if (g.splits > 1 && (!part || (size_t)g.splits * M * N > part_floats || ((uintptr_t)part & 15))) {
    dr_set_error("gemm_nt_glds_bf16: split-K scratch too small");
    return DR_E_WORKSPACE;
  }
  const int tiles = ((M + GP_M - 1) / GP_M) * ((N + GP_N - 1) / GP_N);
  hipLaunchKernelGGL(k_gemm_glds_bf16, dim3((unsigned)dr_xcd_grid(tiles * g.splits)), dim3(256), 0, s, g);
  DR_TRY(dr_check_launch("gemm_glds_bf16"));
  if (g.splits > 1) {
    const long long work = (long long)M * (N / 4);
    hipLaunchKernelGGL(k_glds_finish, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s, g);
    DR_TRY(dr_check_launch("glds_finish"));
  }
  return DR_OK;
}
