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

// index of the non-zero entry of each one-hot group (z values are exactly 0
// off the sample); groups with no non-zero entry get index 0 and value 0
__global__ void k_onehot_index(int M, int R, int C, const float* z, long long ldz, int* idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * R) return;
  const int m = i / R, g = i - m * R;
  const float* zz = z + (long long)m * ldz + g * C;
  int k = 0;
  for (int c = 0; c < C; ++c)
    if (zz[c] != 0.0f) { k = c; break; }
  idx[i] = k;
}

int op_onehot_index(int M, int R, int C, const float* z, long long ldz, int* idx, hipStream_t s) {
  if (M * R == 0) return DR_OK;
  hipLaunchKernelGGL(k_onehot_index, dim3((M * R + 255) / 256), dim3(256), 0, s, M, R, C, z, ldz, idx);
  return dr_check_launch("onehot_index");
}

template <bool VEC>
__global__ __launch_bounds__(512) void k_gru_fused(GruArgs g) {
  constexpr int NW = 8;
  const int Hd = g.Hd, B = g.B;
  const int tiles_j = (Hd + 15) / 16;
  const int tm = blockIdx.x / tiles_j, tj = blockIdx.x - tm * tiles_j;
  const int m0 = tm * 16, j0 = tj * 16;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 15, q = lane >> 4;

  __shared__ float red[NW][3][4][64];
  __shared__ float gh_s[16][3][16];
  __shared__ float gi_s[16][3][16];
  __shared__ int idx_s[16][64];
  __shared__ float zv_s[16][64];

  // stage the one-hot indices / straight-through values of the 16 rows
  const int R = g.R, C = g.C;
  for (int e = tid; e < 16 * R; e += 512) {
    const int ml = e / R, grp = e - ml * R, m = m0 + ml;
    int k = 0;
    float v = 0.f;
    if (m < B) {
      k = g.idx[m * R + grp];
      v = g.z[(long long)m * g.ldz + grp * C + k];
    }
    idx_s[ml][grp] = k;
    zv_s[ml][grp] = v;
  }

  // gh = h W_hh^T (3 gate tiles), K = Hd split over the 8 waves
  f32x4 acc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (g.h) {
    const int K = Hd;
    const int kw = ((K + NW * 16 - 1) / (NW * 16)) * 16;
    const int kb = wave * kw, ke = min(K, kb + kw);
    const int m = m0 + r;
    for (int k0 = kb; k0 < ke; k0 += 16) {
      const int kq = k0 + 4 * q;
      float a[4], b[3][4];
      if (VEC) {
        // select a valid global address (the array base) instead of a value:
        // a ternary on the dereference makes hipcc spill a zero vector and
        // emit flat loads
        const bool oka = (m < B && kq < K);
        float4 va = *reinterpret_cast<const float4*>(oka ? g.h + (long long)m * g.ldh + kq : g.h);
        if (!oka) va = make_float4(0.f, 0.f, 0.f, 0.f);
        a[0] = va.x; a[1] = va.y; a[2] = va.z; a[3] = va.w;
        const int j = j0 + r;
        const bool okb = (j < Hd && kq < K);
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          float4 vb = *reinterpret_cast<const float4*>(okb ? g.w_hh + (long long)(t * Hd + j) * K + kq : g.w_hh);
          if (!okb) vb = make_float4(0.f, 0.f, 0.f, 0.f);
          b[t][0] = vb.x; b[t][1] = vb.y; b[t][2] = vb.z; b[t][3] = vb.w;
        }
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int k = kq + c;
          a[c] = (m < B && k < K) ? g.h[(long long)m * g.ldh + k] : 0.f;
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            const int j = j0 + r;
            b[t][c] = (j < Hd && k < K) ? g.w_hh[(long long)(t * Hd + j) * K + k] : 0.f;
          }
        }
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int t = 0; t < 3; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c], b[t][c], acc[t], 0, 0, 0);
    }
  }
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) red[wave][t][e][lane] = acc[t][e];
  __syncthreads();
  // reduce the 8 partials: element (t, e, l) -> row 4*(l>>4)+e, unit l&15
  for (int x = tid; x < 3 * 256; x += 512) {
    const int t = x >> 8, e = (x >> 6) & 3, l = x & 63;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][t][e][l];
    const int ml = 4 * (l >> 4) + e, jl = l & 15, j = j0 + jl;
    gh_s[ml][t][jl] = v + ((j < Hd) ? g.b_hh[t * Hd + j] : 0.f);
  }
  // gi by gather: one thread per (row, gate, unit); consecutive threads ->
  // consecutive hidden units -> coalesced reads of the W_ih^T rows
  const int L = R * C, A = g.A;
  for (int x = tid; x < 16 * 3 * 16; x += 512) {
    const int jl = x & 15, t = (x >> 4) % 3, ml = x / 48;
    const int m = m0 + ml, j = j0 + jl;
    float v = 0.f;
    if (m < B && j < Hd) {
      const int col = t * Hd + j;
      const long long ld = 3LL * Hd;
      // issue 16 independent gathers, then accumulate them in group order
      for (int g0 = 0; g0 < R; g0 += 16) {
        float w16[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int grp = g0 + u;
          w16[u] = (grp < R) ? g.wt[(long long)(grp * C + idx_s[ml][grp]) * ld + col] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (g0 + u < R) v += w16[u] * zv_s[ml][g0 + u];
      }
      for (int i = 0; i < A; ++i) v += g.wt[(long long)(L + i) * ld + col] * g.a[(long long)m * g.lda + i];
      v = v + g.b_ih[col];
    }
    gi_s[ml][t][jl] = v;
  }
  __syncthreads();
  // gates (torch gru_cell op order)
  if (tid < 256) {
    const int ml = tid >> 4, jl = tid & 15, m = m0 + ml, j = j0 + jl;
    if (m < B && j < Hd) {
      const float rr = 1.0f / (1.0f + expf(-(gh_s[ml][0][jl] + gi_s[ml][0][jl])));
      const float uu = 1.0f / (1.0f + expf(-(gh_s[ml][1][jl] + gi_s[ml][1][jl])));
      const float hn = gh_s[ml][2][jl];
      const float nn = tanhf(gi_s[ml][2][jl] + hn * rr);
      const float hv = g.h ? g.h[(long long)m * g.ldh + j] : 0.0f;
      g.hout[(long long)m * g.ldo + j] = (hv - nn) * uu + nn;
      if (g.sr) {
        const long long o = (long long)m * Hd + j;
        g.sr[o] = rr;
        g.su[o] = uu;
        g.sn[o] = nn;
        g.sghn[o] = hn;
      }
    }
  }
}

int op_gru_fused(const GruArgs& g, hipStream_t s) {
  if (g.R > 64 || g.C > 64 || g.B <= 0) {
    dr_set_error("gru_fused: bad dims B=%d R=%d C=%d", g.B, g.R, g.C);
    return DR_E_INVALID;
  }
  const int tiles = ((g.Hd + 15) / 16) * ((g.B + 15) / 16);
  const bool vec = (g.Hd % 4 == 0) && (g.ldh % 4 == 0) && (((uintptr_t)g.h & 15) == 0) &&
                   (((uintptr_t)g.w_hh & 15) == 0);
  if (vec) hipLaunchKernelGGL(k_gru_fused<true>, dim3(tiles), dim3(512), 0, s, g);
  else hipLaunchKernelGGL(k_gru_fused<false>, dim3(tiles), dim3(512), 0, s, g);
  return dr_check_launch("gru_fused");
}
