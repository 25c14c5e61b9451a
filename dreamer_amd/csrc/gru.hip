// Fused RSSM GRU step (SequenceModel.py:19-24 -> torch gru_cell):
//   gi = W_ih [onehot(z) ; a] + b_ih     (z is a straight-through one-hot: 1 value per group)
//   gh = W_hh h + b_hh
//   r = sig(hr + ir), u = sig(hz + iz), n = tanh(in + hn*r), h' = (h - n)*u + n
// in ONE launch.  The latent part of gi is a gather of R rows of the
// transposed input weight (W_ih^T [L+A][3H], coalesced over hidden units)
// instead of a dense 1024-wide GEMM -- the z entries off the sampled index are
// exactly 0, so the dot product is the same sum without the zero terms.
// gh runs on the exact-f32 MFMA: a workgroup owns 16 batch rows x 16 hidden
// units (3 gate column tiles of W_hh) and splits K over 8 waves.
#include "gru.h"
#include "gemm.h"

#include <algorithm>

__global__ void k_transpose(int rows, int cols, const float* __restrict__ in, float* __restrict__ out) {
  __shared__ float tile[32][33];
  const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int r = by + k, c = bx + tx;
    tile[k][tx] = (r < rows && c < cols) ? in[(long long)r * cols + c] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = bx + k, r = by + tx;
    if (c < cols && r < rows) out[(long long)c * rows + r] = tile[tx][k];
  }
}

int op_transpose(int rows, int cols, const float* in, float* out, hipStream_t s) {
  dim3 grid((cols + 31) / 32, (rows + 31) / 32);
  hipLaunchKernelGGL(k_transpose, grid, dim3(256), 0, s, rows, cols, in, out);
  return dr_check_launch("transpose");
}

struct TransposeBatch {
  TransposeJob j[DR_MAX_TJOBS];
};
__global__ void k_transpose_multi(TransposeBatch tb) {
  __shared__ float tile[32][33];
  const TransposeJob& J = tb.j[blockIdx.z];
  const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  if (bx >= J.cols || by >= J.rows) return;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int k = ty; k < 32; k += 8) {
    const int r = by + k, c = bx + tx;
    tile[k][tx] = (r < J.rows && c < J.cols) ? J.in[(long long)r * J.cols + c] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = bx + k, r = by + tx;
    if (c < J.cols && r < J.rows) J.out[(long long)c * J.ldo + r] = tile[tx][k];
  }
}

int op_transpose_multi(const TransposeJob* jobs, int n, hipStream_t s) {
  if (n <= 0) return DR_OK;
  if (n > DR_MAX_TJOBS) {
    dr_set_error("transpose_multi: at most %d jobs", DR_MAX_TJOBS);
    return DR_E_INVALID;
  }
  TransposeBatch tb;
  int gx = 1, gy = 1;
  for (int i = 0; i < n; ++i) {
    tb.j[i] = jobs[i];
    gx = std::max(gx, (jobs[i].cols + 31) / 32);
    gy = std::max(gy, (jobs[i].rows + 31) / 32);
  }
  hipLaunchKernelGGL(k_transpose_multi, dim3(gx, gy, n), dim3(256), 0, s, tb);
  return dr_check_launch("transpose_multi");
}

// index of the non-zero entry of each one-hot group (z values are exactly 0
// off the sample) and its value; groups with no non-zero entry get (0, 0).
// A group with several non-zero classes (a soft / user-supplied latent) is
// marked dense (idx -1, value 0): the fused GRU then sums all C classes of it
// (SequenceModel.py:21 is a dense product over flatten(z)).
__global__ void k_onehot_index(int M, int R, int C, const float* z, long long ldz, int* idx, float* zval) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * R) return;
  const int m = i / R, g = i - m * R;
  const float* zz = z + (long long)m * ldz + g * C;
  int k = 0, nz = 0;
  float v = 0.f;
  for (int c = 0; c < C; ++c)
    if (zz[c] != 0.0f) {
      if (nz == 0) {
        k = c;
        v = zz[c];
      }
      ++nz;
    }
  idx[i] = nz > 1 ? -1 : k;
  zval[i] = nz > 1 ? 0.f : v;
}

int op_onehot_index(int M, int R, int C, const float* z, long long ldz, int* idx, float* zval, hipStream_t s) {
  if (M * R == 0) return DR_OK;
  hipLaunchKernelGGL(k_onehot_index, dim3((M * R + 255) / 256), dim3(256), 0, s, M, R, C, z, ldz, idx, zval);
  return dr_check_launch("onehot_index");
}

// Work split inside the 512-thread workgroup (16 batch rows x 16 hidden units,
// all three gates):
//   waves 0-3  gh = h W_hh^T on the exact-f32 MFMA, K split four ways, every
//              operand of a wave issued before its first MFMA;
//   waves 4-7  gi by gather: one thread per (row, gate, 4 units) reads the
//              sampled W_ih^T row of every latent group as one float4
//              (coalesced along the hidden units) and accumulates
//              z_value * w in group order, then actions and bias.
// The two halves run concurrently (one MFMA wave and one gather wave per SIMD)
// and meet at a single barrier before the gate math.
#ifndef GRU_MW
#define GRU_MW 4       // MFMA waves
#endif
#ifndef GRU_PRE
#define GRU_PRE 10     // 16-k chunks per MFMA wave held in registers (K = 600 over 4 waves: one batch)
#endif
#define GRU_MAXR 32    // latent groups
#define GRU_MAXA 8     // actions

#ifdef DR_PHASE_TIMING
__device__ long long dr_tbuf_gru[1024 * DR_TS_SLOTS];
extern "C" int dr_debug_tbuf_gru(long long* out, int n) {  // read, then clear
  const int rc = (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(dr_tbuf_gru), (size_t)n * sizeof(long long));
  static long long zeros[1024 * DR_TS_SLOTS];
  return rc | (int)hipMemcpyToSymbol(HIP_SYMBOL(dr_tbuf_gru), zeros, sizeof(zeros));
}
#endif

__global__ __launch_bounds__(512) void k_gru_fused(GruArgs ga) {
  __shared__ GruArgs g;
  dr_stage_args(ga, g, threadIdx.x);
  const int Hd = dr_uni(g.Hd), B = dr_uni(g.B);
  const int R = dr_uni(g.R), C = dr_uni(g.C), A = dr_uni(g.A), L = R * C;
  // logical tiles unit-major: the row tiles of one unit slice (same W_hh rows,
  // same W_ih^T columns) are adjacent and land on one XCD
  const int tiles_j = (Hd + 15) / 16, tiles_m = (B + 15) / 16;
  const int lt = dr_xcd_tile(blockIdx.x, tiles_j * tiles_m);
  if (lt < 0) return;
  const int tj = lt / tiles_m, tm = lt - tj * tiles_m;
  const int m0 = tm * 16, j0 = tj * 16;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  DR_TS(dr_tbuf_gru, 0);

  __shared__ float red[GRU_MW][3][4][64];
  __shared__ float gi_s[16][3][16];
  __shared__ float gh_s[16][3][16];

  const float* h = dr_uni(g.h);
  if (wave < GRU_MW) {
    // ---- gh: 16 rows x (3 gates x 16 units), K = Hd over GRU_MW waves ----
    const float* whh = dr_uni(g.w_hh);
    const int ldh = dr_uni((int)g.ldh);
    const int r = lane & 15, q = lane >> 4;
    const int K = Hd;
    const int kw = ((K + GRU_MW * 16 - 1) / (GRU_MW * 16)) * 16;
    const int kb = wave * kw, ke = min(K, kb + kw);
    const int mrow = m0 + r, jrow = j0 + r;
    const bool mok = mrow < B, jok = jrow < Hd;
    f32x4 acc[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (h) {
      for (int kc = kb; kc < ke; kc += GRU_PRE * 16) {
        float4 ha[GRU_PRE], wb[GRU_PRE][3];
#pragma unroll
        for (int p = 0; p < GRU_PRE; ++p) {
          const int kq = kc + 16 * p + 4 * q;
          const bool live = kc + 16 * p < ke && kq < K;
          const bool oka = live && mok, okb = live && jok;
          ha[p] = dr_ld4(h, oka ? (unsigned)(mrow * ldh + kq) : 0u);
          if (!oka) ha[p] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            wb[p][t] = dr_ld4(whh, okb ? (unsigned)((t * Hd + jrow) * K + kq) : 0u);
            if (!okb) wb[p][t] = make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
#pragma unroll
        for (int p = 0; p < GRU_PRE; ++p) {
          if (kc + 16 * p >= ke) break;
#pragma unroll
          for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ha[p].x, wb[p][t].x, acc[t], 0, 0, 0);
#pragma unroll
          for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ha[p].y, wb[p][t].y, acc[t], 0, 0, 0);
#pragma unroll
          for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ha[p].z, wb[p][t].z, acc[t], 0, 0, 0);
#pragma unroll
          for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ha[p].w, wb[p][t].w, acc[t], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[wave][t][e][lane] = acc[t][e];
    DR_TS(dr_tbuf_gru, 1);
  } else {
    // ---- gi: thread (row ml, gate t, units 4*j4..4*j4+3) ----
    const int x = tid - GRU_MW * 64;  // 0..255, 192 live
    if (x < 192) {
      const int j4 = x & 3, t = (x >> 2) % 3, ml = x / 12;
      const int m = m0 + ml, jj = j0 + 4 * j4;
      const bool live = m < B && jj < Hd;
      const int* idx = dr_uni(g.idx);
      const float* zval = dr_uni(g.zval);
      const float* wt = dr_uni(g.wt);
      const float* act = dr_uni(g.a);
      const int lda = dr_uni((int)g.lda);
      const unsigned ldw = 3u * Hd;
      const unsigned col = (unsigned)(t * Hd + jj);
      // indices + straight-through values of this row (one round trip)
      int iv[GRU_MAXR];
      float zv[GRU_MAXR];
#pragma unroll
      for (int u4 = 0; u4 < GRU_MAXR / 4; ++u4) {
        const bool ok = live && 4 * u4 < R;
        const unsigned e = ok ? (unsigned)(m * R + 4 * u4) : 0u;
        const dr_f4 i4f = *(const DR_GLOBAL dr_f4*)((const DR_GLOBAL char*)idx + (e << 2));
        const int4 i4 = make_int4(__float_as_int(i4f.x), __float_as_int(i4f.y), __float_as_int(i4f.z),
                                  __float_as_int(i4f.w));
        const float4 z4 = dr_ld4(zval, e);
        iv[4 * u4] = i4.x; iv[4 * u4 + 1] = i4.y; iv[4 * u4 + 2] = i4.z; iv[4 * u4 + 3] = i4.w;
        zv[4 * u4] = z4.x; zv[4 * u4 + 1] = z4.y; zv[4 * u4 + 2] = z4.z; zv[4 * u4 + 3] = z4.w;
      }
      float av[GRU_MAXA];
#pragma unroll
      for (int i = 0; i < GRU_MAXA; ++i) {
        const bool ok = live && i < A;
        const float v = dr_ld1(act, ok ? (unsigned)(m * lda + i) : 0u);
        av[i] = ok ? v : 0.f;
      }
      // sampled rows of W_ih^T (one round trip: every gather issued first)
      float4 w[GRU_MAXR];
#pragma unroll
      for (int u = 0; u < GRU_MAXR; ++u) {
        const bool ok = live && u < R;
        w[u] = dr_ld4(wt, (ok && iv[u] >= 0) ? (unsigned)(u * C + iv[u]) * ldw + col : 0u);
      }
      float4 wa[GRU_MAXA];
#pragma unroll
      for (int i = 0; i < GRU_MAXA; ++i) {
        const bool ok = live && i < A;
        wa[i] = dr_ld4(wt, ok ? (unsigned)(L + i) * ldw + col : 0u);
      }
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < GRU_MAXR; ++u) {
        if (u < R) {
          v.x = fmaf(w[u].x, zv[u], v.x);
          v.y = fmaf(w[u].y, zv[u], v.y);
          v.z = fmaf(w[u].z, zv[u], v.z);
          v.w = fmaf(w[u].w, zv[u], v.w);
        }
      }
      // dense groups (k_onehot_index marker; zval = 0 above): every class
      bool dense = false;
#pragma unroll
      for (int u = 0; u < GRU_MAXR; ++u) dense = dense || (u < R && iv[u] < 0);
      if (dense && live) {
        const float* zr = g.z + (long long)m * g.ldz;
        for (int u = 0; u < R; ++u) {
          if (iv[u] >= 0) continue;
          for (int c = 0; c < C; ++c) {
            const float zc = zr[u * C + c];
            const float4 wc = dr_ld4(wt, (unsigned)(u * C + c) * ldw + col);
            v.x = fmaf(wc.x, zc, v.x);
            v.y = fmaf(wc.y, zc, v.y);
            v.z = fmaf(wc.z, zc, v.z);
            v.w = fmaf(wc.w, zc, v.w);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < GRU_MAXA; ++i) {
        if (i < A) {
          v.x = fmaf(wa[i].x, av[i], v.x);
          v.y = fmaf(wa[i].y, av[i], v.y);
          v.z = fmaf(wa[i].z, av[i], v.z);
          v.w = fmaf(wa[i].w, av[i], v.w);
        }
      }
      const float* bih = dr_uni(g.b_ih);
      const float4 bb = dr_ld4(bih, live ? col : 0u);
      gi_s[ml][t][4 * j4 + 0] = v.x + bb.x;
      gi_s[ml][t][4 * j4 + 1] = v.y + bb.y;
      gi_s[ml][t][4 * j4 + 2] = v.z + bb.z;
      gi_s[ml][t][4 * j4 + 3] = v.w + bb.w;
    }
    DR_TS(dr_tbuf_gru, 2);
  }
  __syncthreads();
  DR_TS(dr_tbuf_gru, 3);
  // reduce the MFMA partials: element (t, e, l) -> row 4*(l>>4)+e, unit l&15
  const float* bhh = dr_uni(g.b_hh);
  for (int x = tid; x < 3 * 256; x += 512) {
    const int t = x >> 8, e = (x >> 6) & 3, l = x & 63;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < GRU_MW; ++w) v += red[w][t][e][l];
    const int ml = 4 * (l >> 4) + e, jl = l & 15, j = j0 + jl;
    const float bv = dr_ld1(bhh, (j < Hd) ? (unsigned)(t * Hd + j) : 0u);
    gh_s[ml][t][jl] = v + ((j < Hd) ? bv : 0.f);
  }
  __syncthreads();
  DR_TS(dr_tbuf_gru, 4);
  // gates (torch gru_cell op order)
  if (tid < 256) {
    const int ml = tid >> 4, jl = tid & 15, m = m0 + ml, j = j0 + jl;
    if (m < B && j < Hd) {
      const float rr = 1.0f / (1.0f + expf(-(gh_s[ml][0][jl] + gi_s[ml][0][jl])));
      const float uu = 1.0f / (1.0f + expf(-(gh_s[ml][1][jl] + gi_s[ml][1][jl])));
      const float hn = gh_s[ml][2][jl];
      const float nn = tanhf(gi_s[ml][2][jl] + hn * rr);
      const float hv = h ? dr_g(h)[(long long)m * g.ldh + j] : 0.0f;
      const float ho = (hv - nn) * uu + nn;
      dr_g(g.hout)[(long long)m * g.ldo + j] = ho;
      if (g.hout16) dr_g(g.hout16)[(long long)m * g.ldo + j] = __builtin_bit_cast(unsigned short, (__bf16)ho);
      if (g.sr) {
        const long long o = (long long)m * Hd + j;
        dr_g(g.sr)[o] = rr;
        dr_g(g.su)[o] = uu;
        dr_g(g.sn)[o] = nn;
        dr_g(g.sghn)[o] = hn;
      }
    }
  }
  DR_TS(dr_tbuf_gru, 5);
}

// ---------------------------------------------------------------------------
// Split GRU step for larger batches (B >= 128 with caller scratch): the hidden
// product gh = h W_hh^T + b_hh runs as a tile-GEMM launch (gemm.hip: 32 x 32
// tiles, W_hh read 8x at B = 256 instead of 16x by the fused kernel's 16-row
// tiles), then k_gru_gates gathers gi and applies the gates.  Workgroup =
// 8 rows x 32 hidden units x 3 gates; thread (row, gate, 4 units): the 8
// threads of a (row, gate) read one full 128-B line of every gathered W_ih^T
// row (the fused kernel reads 64-B halves), and unit slices map to XCDs so
// each XCD's L2 holds its columns of W_ih^T.  gi keeps the fused kernel's
// summation order (groups ascending, then actions, then + b_ih): identical
// gi; gh differs from the fused kernel's in f32 summation order only.
// ---------------------------------------------------------------------------
#define GG_ROWS 8
#define GG_UNITS 32
#define GG_NT (GG_ROWS * 3 * (GG_UNITS / 4))  // 192 threads

// gathered W_ih^T rows issued per batch: 4 the same (r05zh); 16 / 32 slower
// (fp32 headline 597 -> 584 / 582 k, bf16 888 -> 859 / 857 k, profiles/r06l_ab_gates_wgrad.txt)
#define DR_GATES_GB 8
template <int GB>  // gathered rows issued per batch (VGPRs vs round trips)
__global__ __launch_bounds__(GG_NT) void k_gru_gates(GruArgs ga) {
  __shared__ GruArgs g;
  dr_stage_args(ga, g, threadIdx.x);
  const int Hd = dr_uni(g.Hd), B = dr_uni(g.B);
  const int R = dr_uni(g.R), C = dr_uni(g.C), A = dr_uni(g.A), L = R * C;
  const int tiles_j = (Hd + GG_UNITS - 1) / GG_UNITS, tiles_m = (B + GG_ROWS - 1) / GG_ROWS;
  const int lt = dr_xcd_tile(blockIdx.x, tiles_j * tiles_m);
  if (lt < 0) return;
  const int tj = lt / tiles_m, tm = lt - tj * tiles_m;
  const int m0 = tm * GG_ROWS, j0 = tj * GG_UNITS;
  const int tid = threadIdx.x;
  __shared__ int s_idx[GG_ROWS][GRU_MAXR];
  __shared__ float s_zv[GG_ROWS][GRU_MAXR];
  __shared__ float4 s_gi[GG_ROWS][3][GG_UNITS / 4];
  // round trip 1: the tile's indices / straight-through values, and (threads
  // 0-63, one float4 of 4 units each for the gate phase) gh of the 3 gates
  // and h -- independent of the gather, issued with it
  const int gm = m0 + (tid >> 3), gj = j0 + 4 * (tid & 7);
  const bool gate_thr = tid < GG_ROWS * (GG_UNITS / 4) && gm < B && gj < Hd;
  const float* hp = dr_uni(g.h);
  const float* gh = hp ? dr_uni(g.gh_ws) : nullptr;
  float4 ghv[3], hv = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int t = 0; t < 3; ++t)
    ghv[t] = gh ? dr_ld4(gh, gate_thr ? (unsigned)(gm * 3 * Hd + t * Hd + gj) : 0u)
                : dr_ld4(dr_uni(g.b_hh), gate_thr ? (unsigned)(t * Hd + gj) : 0u);
  if (hp) hv = dr_ld4(hp, gate_thr ? (unsigned)(gm * (int)g.ldh + gj) : 0u);
  for (int x = tid; x < GG_ROWS * GRU_MAXR; x += GG_NT) {
    const int ml = x / GRU_MAXR, u = x - ml * GRU_MAXR, m = m0 + ml;
    const bool ok = m < B && u < R;
    const int iv = ok ? dr_g(g.idx)[m * R + u] : 0;
    const float zv = ok ? dr_g(g.zval)[m * R + u] : 0.f;
    s_idx[ml][u] = iv;
    s_zv[ml][u] = zv;
  }
  __syncthreads();
  {
    // round trip 2: every gathered W_ih^T row piece of this thread at once
    const int j8 = tid & 7, t = (tid >> 3) % 3, ml = tid / 24;
    const int m = m0 + ml, jj = j0 + 4 * j8;
    const bool live = m < B && jj < Hd;
    const float* wt = dr_uni(g.wt);
    const unsigned ldw = 3u * Hd;
    const unsigned col = (unsigned)(t * Hd + jj);
    const float* act = dr_uni(g.a);
    const int lda = dr_uni((int)g.lda);
    float av[GRU_MAXA];
    float4 wa[GRU_MAXA];
#pragma unroll
    for (int i = 0; i < GRU_MAXA; ++i) {
      const bool ok = live && i < A;
      av[i] = dr_ld1(act, ok ? (unsigned)(m * lda + i) : 0u);
      wa[i] = dr_ld4(wt, ok ? (unsigned)(L + i) * ldw + col : 0u);
    }
    const float4 bb = dr_ld4(dr_uni(g.b_ih), live ? col : 0u);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    bool dense = false;
#pragma unroll
    for (int ub = 0; ub < GRU_MAXR; ub += GB) {
      float4 w[GB];
#pragma unroll
      for (int q = 0; q < GB; ++q) {
        const int u = ub + q;
        const int iv = s_idx[ml][u];
        const bool ok = live && u < R && iv >= 0;
        w[q] = dr_ld4(wt, ok ? (unsigned)(u * C + iv) * ldw + col : 0u);
      }
#pragma unroll
      for (int q = 0; q < GB; ++q) {
        const int u = ub + q;
        if (u < R) {
          const float zv = s_zv[ml][u];
          dense = dense || s_idx[ml][u] < 0;
          v.x = fmaf(w[q].x, zv, v.x);
          v.y = fmaf(w[q].y, zv, v.y);
          v.z = fmaf(w[q].z, zv, v.z);
          v.w = fmaf(w[q].w, zv, v.w);
        }
      }
    }
    if (dense && live) {  // groups with several non-zero classes: every class (as the fused kernel)
      const float* zr = g.z + (long long)m * g.ldz;
      for (int u = 0; u < R; ++u) {
        if (s_idx[ml][u] >= 0) continue;
        for (int c = 0; c < C; ++c) {
          const float zc = zr[u * C + c];
          const float4 wc = dr_ld4(wt, (unsigned)(u * C + c) * ldw + col);
          v.x = fmaf(wc.x, zc, v.x);
          v.y = fmaf(wc.y, zc, v.y);
          v.z = fmaf(wc.z, zc, v.z);
          v.w = fmaf(wc.w, zc, v.w);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < GRU_MAXA; ++i) {
      if (i < A) {
        v.x = fmaf(wa[i].x, av[i], v.x);
        v.y = fmaf(wa[i].y, av[i], v.y);
        v.z = fmaf(wa[i].z, av[i], v.z);
        v.w = fmaf(wa[i].w, av[i], v.w);
      }
    }
    s_gi[ml][t][j8] = make_float4(v.x + bb.x, v.y + bb.y, v.z + bb.z, v.w + bb.w);
  }
  __syncthreads();
  // gates (torch gru_cell op order) for 4 units per thread, float4 stores
  if (gate_thr) {
    const int ml = tid >> 3, j8 = tid & 7;
    const float4 gr = s_gi[ml][0][j8], gu = s_gi[ml][1][j8], gn = s_gi[ml][2][j8];
    const float gi_r[4] = {gr.x, gr.y, gr.z, gr.w}, gi_u[4] = {gu.x, gu.y, gu.z, gu.w};
    const float gi_n[4] = {gn.x, gn.y, gn.z, gn.w};
    const float gh_r[4] = {ghv[0].x, ghv[0].y, ghv[0].z, ghv[0].w};
    const float gh_u[4] = {ghv[1].x, ghv[1].y, ghv[1].z, ghv[1].w};
    const float gh_n[4] = {ghv[2].x, ghv[2].y, ghv[2].z, ghv[2].w};
    const float h4[4] = {hv.x, hv.y, hv.z, hv.w};
    float ho[4], ro[4], uo[4], no[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float rr = 1.0f / (1.0f + expf(-(gh_r[e] + gi_r[e])));
      const float uu = 1.0f / (1.0f + expf(-(gh_u[e] + gi_u[e])));
      const float nn = tanhf(gi_n[e] + gh_n[e] * rr);
      ho[e] = (h4[e] - nn) * uu + nn;
      ro[e] = rr;
      uo[e] = uu;
      no[e] = nn;
    }
    dr_st4(g.hout, (unsigned)(gm * (int)g.ldo + gj), make_float4(ho[0], ho[1], ho[2], ho[3]));
    if (g.hout16) {
      typedef __bf16 gg_b4 __attribute__((ext_vector_type(4)));
      typedef unsigned gg_u2 __attribute__((ext_vector_type(2)));
      const gg_b4 hb = {(__bf16)ho[0], (__bf16)ho[1], (__bf16)ho[2], (__bf16)ho[3]};
      *(DR_GLOBAL gg_u2*)((DR_GLOBAL char*)g.hout16 + 2 * ((long long)gm * g.ldo + gj)) = __builtin_bit_cast(gg_u2, hb);
    }
    if (g.sr) {
      const unsigned o = (unsigned)(gm * Hd + gj);
      dr_st4(g.sr, o, make_float4(ro[0], ro[1], ro[2], ro[3]));
      dr_st4(g.su, o, make_float4(uo[0], uo[1], uo[2], uo[3]));
      dr_st4(g.sn, o, make_float4(no[0], no[1], no[2], no[3]));
      dr_st4(g.sghn, o, ghv[2]);
    }
  }
}


// ---------------------------------------------------------------------------
// Latent part of a Linear on cat(h, z) with a one-hot z (the actor's first
// layer inside the imagination unroll, Agent.py:191-210 on cat(h, z)):
// out = base + sum_u zval[u] * wt[u*C + idx[u]] -- R gathered rows of the
// transposed z-columns instead of a K = R*C dense product.  Thread = (row,
// 4 outputs); every gathered float4 of a thread issued before the first FMA.
// ---------------------------------------------------------------------------
#define ZG_ROWS 4
__global__ __launch_bounds__(256) void k_zgather_add(int M, int N, int R, int C, const int* __restrict__ idx,
                                                     const float* __restrict__ zval, const float* __restrict__ z,
                                                     long long ldz, const float* __restrict__ wt, long long ldw,
                                                     const float* __restrict__ base, long long ldb,
                                                     float* __restrict__ out, long long ldo) {
  __shared__ int s_idx[ZG_ROWS][GRU_MAXR];
  __shared__ float s_zv[ZG_ROWS][GRU_MAXR];
  const int m0 = blockIdx.x * ZG_ROWS, tid = threadIdx.x;
  for (int x = tid; x < ZG_ROWS * GRU_MAXR; x += 256) {
    const int ml = x / GRU_MAXR, u = x - ml * GRU_MAXR, m = m0 + ml;
    const bool ok = m < M && u < R;
    s_idx[ml][u] = ok ? idx[m * R + u] : 0;
    s_zv[ml][u] = ok ? zval[m * R + u] : 0.f;
  }
  const int ml = tid >> 6, m = m0 + ml, n = 4 * ((tid & 63) + 64 * (int)blockIdx.y);
  const bool live = m < M && n < N;
  const float4 b = dr_ld4(base, live ? (unsigned)(m * ldb + n) : 0u);
  __syncthreads();
  float4 w[GRU_MAXR];
#pragma unroll
  for (int u = 0; u < GRU_MAXR; ++u) {
    const int iv = s_idx[ml][u];
    const bool ok = live && u < R && iv >= 0;
    w[u] = dr_ld4(wt, ok ? (unsigned)((u * C + iv) * ldw + n) : 0u);
  }
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  bool dense = false;
#pragma unroll
  for (int u = 0; u < GRU_MAXR; ++u) {
    if (u < R) {
      const float zv = s_zv[ml][u];
      dense = dense || s_idx[ml][u] < 0;
      v.x = fmaf(w[u].x, zv, v.x);
      v.y = fmaf(w[u].y, zv, v.y);
      v.z = fmaf(w[u].z, zv, v.z);
      v.w = fmaf(w[u].w, zv, v.w);
    }
  }
  if (dense && live) {
    const float* zr = z + (long long)m * ldz;
    for (int u = 0; u < R; ++u) {
      if (s_idx[ml][u] >= 0) continue;
      for (int c = 0; c < C; ++c) {
        const float zc = zr[u * C + c];
        const float4 wc = dr_ld4(wt, (unsigned)((u * C + c) * ldw + n));
        v.x = fmaf(wc.x, zc, v.x);
        v.y = fmaf(wc.y, zc, v.y);
        v.z = fmaf(wc.z, zc, v.z);
        v.w = fmaf(wc.w, zc, v.w);
      }
    }
  }
  if (live) dr_st4(out, (unsigned)(m * ldo + n), make_float4(b.x + v.x, b.y + v.y, b.z + v.z, b.w + v.w));
}

int op_zgather_add(int M, int N, int R, int C, const int* idx, const float* zval, const float* z, long long ldz,
                   const float* wt, long long ldw, const float* base, long long ldb, float* out, long long ldo,
                   hipStream_t s) {
  if (M <= 0 || N <= 0 || R < 1 || R > GRU_MAXR || C < 1 || N % 4 || ldw % 4 || ldb % 4 || ldo % 4 ||
      (((uintptr_t)wt | (uintptr_t)base | (uintptr_t)out) & 15) || (long long)R * C * ldw >= (1LL << 31) ||
      (long long)M * std::max(ldb, ldo) >= (1LL << 31)) {
    dr_set_error("zgather_add: unsupported dims/alignment M=%d N=%d R=%d C=%d", M, N, R, C);
    return DR_E_INVALID;
  }
  const dim3 grid((unsigned)((M + ZG_ROWS - 1) / ZG_ROWS), (unsigned)((N / 4 + 63) / 64));
  hipLaunchKernelGGL(k_zgather_add, grid, dim3(256), 0, s, M, N, R, C, idx, zval, z, ldz, wt, ldw, base, ldb, out, ldo);
  return dr_check_launch("zgather_add");
}

int op_gru_fused(const GruArgs& g, hipStream_t s) {
  if (g.R > GRU_MAXR || g.A > GRU_MAXA || g.B <= 0 || g.Hd <= 0 || g.Hd % 4 != 0 || g.ldh % 4 != 0 ||
      (((uintptr_t)g.h | (uintptr_t)g.w_hh | (uintptr_t)g.wt | (uintptr_t)g.b_ih | (uintptr_t)g.zval |
        (uintptr_t)g.idx) & 15) != 0 || (g.R % 4) != 0) {
    dr_set_error("gru_fused: unsupported dims/alignment B=%d Hd=%d R=%d A=%d (R %% 4 == 0, R <= %d, A <= %d, "
                 "Hd %% 4 == 0, 16-byte aligned operands)", g.B, g.Hd, g.R, g.A, GRU_MAXR, GRU_MAXA);
    return DR_E_INVALID;
  }
  const long long lim = 1LL << 30;
  if ((long long)(g.R * g.C + g.A) * 3 * g.Hd >= lim || (long long)g.B * g.ldh >= lim || (long long)g.B * g.ldo >= lim ||
      3LL * g.Hd * g.Hd >= lim) {
    dr_set_error("gru_fused: operands exceed 32-bit offsets");
    return DR_E_INVALID;
  }
  if (g.gh_ws && g.B >= 128 && ((uintptr_t)g.gh_ws | (uintptr_t)g.hout | (uintptr_t)g.sr | (uintptr_t)g.su |
                                 (uintptr_t)g.sn | (uintptr_t)g.sghn) % 16 == 0 && g.ldo % 4 == 0) {
    // split path: hidden product on the tile GEMM, then gather + gates
    if (g.h && !g.gh_ready) {
      GemmArgs p = gemm_args();
      p.M = g.B; p.N = 3 * g.Hd; p.K = g.Hd;
      p.A = g.h; p.lda = g.ldh; p.ksplitA = g.Hd;
      p.W = g.w_hh; p.ldb = g.Hd;
      p.bias = g.b_hh;
      p.Y = g.gh_ws; p.ldy = 3 * g.Hd;
      DR_TRY(gemm_launch(G_NT, AM_PLAIN, &p, 1, s));
    }
    const int tiles = ((g.Hd + GG_UNITS - 1) / GG_UNITS) * ((g.B + GG_ROWS - 1) / GG_ROWS);
    hipLaunchKernelGGL(k_gru_gates<DR_GATES_GB>, dim3(dr_xcd_grid(tiles)), dim3(GG_NT), 0, s, g);
    return dr_check_launch("gru_gates");
  }
  const int tiles = ((g.Hd + 15) / 16) * ((g.B + 15) / 16);
  hipLaunchKernelGGL(k_gru_fused, dim3(dr_xcd_grid(tiles)), dim3(512), 0, s, g);
  return dr_check_launch("gru_fused");
}
