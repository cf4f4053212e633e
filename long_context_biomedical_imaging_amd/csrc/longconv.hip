// Direct causal long convolution for short sequences (Hyena inside Swin windows) on the f32 MFMA, gfx950.
//
// Replaces fftconv_ref (model/models/hyena.py:32-51, via Filter.forward :201-216) when the sequence is a Swin
// window (backbone_swin.py:361-362: N = 64 / 343 / 512 tokens at window 4 / 7 / 8): y = causal_conv(u, k) + D u,
// evaluated exactly as the sum it is, y[t] = sum_{s <= t} k[t - s] u[s] + D u[t], instead of an n = 2L FFT. Per
// filter channel c this is Y = U . T^T with the lower-triangular Toeplitz T[t][s] = k[t - s]: an (R x L) x (L x L)
// GEMM with K = L whose B operand is generated from k in LDS, on v_mfma_f32_32x32x2_f32 (exact f32 products, f32
// accumulation — the reference computes the FFT in f32). Tiles above the diagonal are skipped.
//
// Layout: rows are channel-major f32 (R, C, L) (row r of filter c at ((r*C + c) * L)); k (C, L); D (C).
//   dconv_kernel<false>: y = conv(u) + D u               (forward)
//   dconv_kernel<true> : du = corr(dy, k) + D dy          (adjoint: sum over t >= s of dy[t] k[t - s])
//   dconv_dk_kernel    : per row split, dk[tau] = sum_r sum_t dy[r][t] u[r][t - tau]; dk[0] is also dD.
// The filter gradient runs per diagonal BAND of 32x32 tiles: band d holds sum_i dY[32i + m] U[32(i - d) + n] in ONE
// accumulator (the contraction runs over rows and tiles), and tau = 32d + m - n. Deterministic: per-split partials
// in fixed order, summed by the caller.
#include "common.hpp"

#include <algorithm>

namespace lci {

constexpr int DC_MAXL = 512;        // longest L on the direct path (16 tiles: <= 4 band accumulators per wave)
constexpr int DC_ROWS = 32;         // rows per workgroup (conv kernels)
constexpr int DK_ROWS = 16;         // rows per staged chunk (filter-gradient kernel)

struct DcArgs {
  const float* x;    // conv: u (fwd) / dy (adjoint); dk: dy
  const float* u;    // dk: u
  const float* k;    // (C, L)
  const float* D;    // (C) or null
  float* y;          // conv: y / du; dk: part (nsplit, C, L)
  int R, C, L, rows_per_split;
};

__device__ __forceinline__ f32x16 mfma_f32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// grid (ceil(R / 32), C, ceil(npairs / 4)), block 256, dynamic LDS = (32 (LP + 1) + 32 + LP) floats,
// LP = 32 ceil(L / 32), npairs = ceil(nt / 2). Wave w of grid slice z computes the output tiles (32 rows x 32
// positions) j1 = p and j2 = nt-1-p, p = 4z + w: equal work per wave. The two tiles' contraction ranges share a
// prefix (forward: s in [0, 32(j1+1))) or a suffix (adjoint: t in [32 j2, LP)) over which each A operand (X row
// value) feeds both tiles; every range runs as two interleaved accumulator chains (even / odd k-steps), so a wave
// keeps 2-4 independent MFMA chains in flight.
template <bool ADJ>
__global__ __launch_bounds__(256, 2) void dconv_kernel(DcArgs a) {
  extern __shared__ float sm[];
  const int L = a.L, nt = (L + 31) / 32, LP = nt * 32, LD = LP + 1;
  float* xs = sm;                    // [32][LD]
  float* kz = sm + 32 * LD;          // [32 + LP]: kz[32 + i] = k[i] (i < L), 0 elsewhere
  const int c = blockIdx.y, r0 = blockIdx.x * DC_ROWS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 31, kk = lane >> 5;
  for (int i = tid; i < DC_ROWS * LP; i += 256) {
    const int rr = i / LP, t = i - rr * LP, r = r0 + rr;
    xs[rr * LD + t] = (r < a.R && t < L) ? a.x[((long long)r * a.C + c) * L + t] : 0.f;
  }
  for (int i = tid; i < 32 + LP; i += 256) kz[i] = (i >= 32 && i - 32 < L) ? a.k[(long long)c * L + i - 32] : 0.f;
  __syncthreads();
  const int p = blockIdx.z * 4 + wave;
  if (2 * p >= nt) return;
  const float Dc = a.D ? a.D[c] : 0.f;
  const float* xrow = xs + m * LD + kk;
  const int j1 = p, j2 = nt - 1 - p;
  const bool two = j2 != j1;
  // B operand of tile j at contraction index i: fwd kz[32 + 32j + m - i - kk], adjoint kz[32 + i + kk - 32j - m]
  const float* kp1 = ADJ ? kz + 32 + kk - 32 * j1 - m : kz + 32 + 32 * j1 + m - kk;
  const float* kp2 = ADJ ? kz + 32 + kk - 32 * j2 - m : kz + 32 + 32 * j2 + m - kk;
  auto bval = [&](const float* kp, int i) -> float { return ADJ ? kp[i] : kp[-i]; };
  f32x16 a1{}, b1{}, a2{}, b2{};
  // ranges: fwd  tile1 [0, 32(j1+1)), tile2 [0, 32(j2+1));  adjoint  tile1 [32 j1, LP), tile2 [32 j2, LP)
  const int c0 = ADJ ? 32 * j2 : 0, c1 = ADJ ? LP : 32 * (j1 + 1);      // common range (both tiles)
  if (two) {
#pragma unroll 4
    for (int i = c0; i < c1; i += 4) {
      const float x0 = xrow[i], x1 = xrow[i + 2];
      a1 = mfma_f32(x0, bval(kp1, i), a1);
      a2 = mfma_f32(x0, bval(kp2, i), a2);
      b1 = mfma_f32(x1, bval(kp1, i + 2), b1);
      b2 = mfma_f32(x1, bval(kp2, i + 2), b2);
    }
    // the part only one tile needs: fwd tile 2 [32(j1+1), 32(j2+1)); adjoint tile 1 [32 j1, 32 j2)
    const int s0 = ADJ ? 32 * j1 : 32 * (j1 + 1), s1 = ADJ ? 32 * j2 : 32 * (j2 + 1);
    const float* kps = ADJ ? kp1 : kp2;
    f32x16 u0{}, u1{};
#pragma unroll 4
    for (int i = s0; i < s1; i += 4) {
      u0 = mfma_f32(xrow[i], bval(kps, i), u0);
      u1 = mfma_f32(xrow[i + 2], bval(kps, i + 2), u1);
    }
    if (ADJ) { a1 += u0; b1 += u1; } else { a2 += u0; b2 += u1; }
  } else {
    const int i0 = ADJ ? 32 * j1 : 0, i1 = ADJ ? LP : 32 * (j1 + 1);
#pragma unroll 4
    for (int i = i0; i < i1; i += 4) {
      a1 = mfma_f32(xrow[i], bval(kp1, i), a1);
      b1 = mfma_f32(xrow[i + 2], bval(kp1, i + 2), b1);
    }
  }
  // D skip and store: reg q holds row (q & 3) + 8 (q >> 2) + 4 kk, column m
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h == 1 && !two) break;
    const int j = h == 0 ? j1 : j2;
    const f32x16 acc = h == 0 ? a1 + b1 : a2 + b2;
    const int o = 32 * j + m;
    if (o < L) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int rr = (q & 3) + 8 * (q >> 2) + 4 * kk, r = r0 + rr;
        if (r < a.R) a.y[((long long)r * a.C + c) * L + o] = acc[q] + Dc * xs[rr * LD + o];
      }
    }
  }
}

// grid (nsplit, C, ceil(npairs / 4)), block 256, dynamic LDS = max(2 * DK_ROWS * LP, 4 * 2 * 32 * 33) floats.
// Wave w of slice z owns the band pair p = 4z + w: bands d1 = p and d2 = nt-1-p (band d: nt - d tiles; a pair: nt + 1).
// Output: bpart (nsplit, C, nt, 64) f32, the band's diagonal sums (delta = t - s + 31 in [0, 63)); dk[32 d + delta]
// = sum over bands d (delta) and d + 1 (delta - 32), assembled by the caller.
__global__ __launch_bounds__(256, 2) void dconv_dk_kernel(DcArgs a) {
  extern __shared__ float sm[];
  const int L = a.L, nt = (L + 31) / 32, LP = nt * 32;
  float* dys = sm;                   // [DK_ROWS][LP]
  float* us = sm + DK_ROWS * LP;     // [DK_ROWS][LP]
  const int c = blockIdx.y, split = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 31, kk = lane >> 5;
  const int rbeg = split * a.rows_per_split, rend = min(a.R, rbeg + a.rows_per_split);
  const int p = blockIdx.z * 4 + wave;
  const bool active = 2 * p < nt;
  const int band[2] = {p, nt - 1 - p};
  const int nb = !active ? 0 : (band[1] != band[0] ? 2 : 1);
  f32x16 acc[2][2];
#pragma unroll
  for (int b = 0; b < 2; ++b) acc[b][0] = acc[b][1] = f32x16{};
  for (int rc = rbeg; rc < rend; rc += DK_ROWS) {
    __syncthreads();
    for (int i = tid; i < DK_ROWS * LP; i += 256) {
      const int rr = i / LP, t = i - rr * LP, r = rc + rr;
      const bool ok = r < rend && t < L;
      const long long off = ((long long)r * a.C + c) * L + t;
      dys[i] = ok ? a.x[off] : 0.f;
      us[i] = ok ? a.u[off] : 0.f;
    }
    __syncthreads();
    // A[m = t][k = row] = dY[row][32i + m]; B[k = row][n = s] = U[row][32(i - d) + n]; rows in two chains
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      if (b >= nb) break;
      const int d = band[b];
      for (int i = d; i < nt; ++i) {
        const float* ap = dys + kk * LP + 32 * i + m;
        const float* bp = us + kk * LP + 32 * (i - d) + m;
#pragma unroll
        for (int q = 0; q < DK_ROWS; q += 4) {
          acc[b][0] = mfma_f32(ap[q * LP], bp[q * LP], acc[b][0]);
          acc[b][1] = mfma_f32(ap[(q + 2) * LP], bp[(q + 2) * LP], acc[b][1]);
        }
      }
    }
  }
  __syncthreads();
  // band reduction: G_d[t][s] (reg q: t = (q & 3) + 8 (q >> 2) + 4 kk, s = m) -> diagonals delta = t - s in [-31, 31]
  float* gs = sm + wave * (2 * 32 * 33);            // per wave: 2 bands x [32][33]
  for (int b = 0; b < nb; ++b) {
    const f32x16 g = acc[b][0] + acc[b][1];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int t = (q & 3) + 8 * (q >> 2) + 4 * kk;
      gs[b * 32 * 33 + t * 33 + m] = g[q];
    }
  }
  __builtin_amdgcn_wave_barrier();
  __syncthreads();
  for (int b = 0; b < nb; ++b) {
    const int delta = lane - 31;
    float s = 0.f;
    if (lane < 63)
      for (int n = max(0, -delta); n < min(32, 32 - delta); ++n) s += gs[b * 32 * 33 + (n + delta) * 33 + n];
    a.y[(((long long)split * a.C + c) * nt + band[b]) * 64 + lane] = s;
  }
}

static int dk_splits(int R, int C, int L) {
  // ~4 workgroups per CU in total (band-pair slices x channels x row splits), at least 2 row chunks per split
  const int nt = (L + 31) / 32, nz = ((nt + 1) / 2 + 3) / 4;
  int ns = std::max(1, 1024 / std::max(1, C * nz));
  ns = std::min(ns, std::max(1, (R + 2 * DK_ROWS - 1) / (2 * DK_ROWS)));
  return ns;
}

}  // namespace lci

using namespace lci;

extern "C" int lci_direct_conv_max_len(void) { return DC_MAXL; }

extern "C" int lci_direct_conv_fwd(const float* u, const float* k, const float* D, float* y, int R, int C, int L,
                                   int adjoint, void* stream) {
  LCI_CHECK(R > 0 && C > 0 && L > 0 && L <= DC_MAXL, "direct_conv: bad shape R=%d C=%d L=%d (L <= %d)", R, C, L,
            DC_MAXL);
  DcArgs a{};
  a.x = u; a.k = k; a.D = D; a.y = y; a.R = R; a.C = C; a.L = L;
  const int nt = (L + 31) / 32, LP = 32 * nt;
  const size_t lds = (size_t)(32 * (LP + 1) + 32 + LP) * sizeof(float);
  dim3 grid((R + DC_ROWS - 1) / DC_ROWS, C, ((nt + 1) / 2 + 3) / 4);
  if (adjoint) hipLaunchKernelGGL(dconv_kernel<true>, grid, dim3(256), lds, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(dconv_kernel<false>, grid, dim3(256), lds, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_direct_conv_dk_splits(int R, int C, int L) {
  if (R <= 0 || C <= 0 || L <= 0 || L > DC_MAXL) return 0;
  return dk_splits(R, C, L);
}

// bpart (lci_direct_conv_dk_splits(R, C, L), C, ceil(L / 32), 64) f32 <- per-row-split diagonal sums of the bands of
// G = dY^T U: band d, slot delta + 31 holds sum over rows and t - s = 32 d + delta of dy[r][t] u[r][s]. The caller
// sums the splits and assembles dk[32 d + e] = band[d][e + 31] + band[d + 1][e - 1] (e in [0, 32)); dD = dk[0].
extern "C" int lci_direct_conv_dk(const float* dy, const float* u, float* part, int R, int C, int L, void* stream) {
  LCI_CHECK(R > 0 && C > 0 && L > 0 && L <= DC_MAXL, "direct_conv_dk: bad shape R=%d C=%d L=%d", R, C, L);
  const int ns = dk_splits(R, C, L);
  DcArgs a{};
  a.x = dy; a.u = u; a.y = part; a.R = R; a.C = C; a.L = L;
  a.rows_per_split = DK_ROWS * ((R + ns * DK_ROWS - 1) / (ns * DK_ROWS));
  const int nt = (L + 31) / 32, LP = 32 * nt;
  const size_t lds = std::max((size_t)2 * DK_ROWS * LP, (size_t)(4 * 2 * 32 * 33)) * sizeof(float);
  hipLaunchKernelGGL(dconv_dk_kernel, dim3(ns, C, ((nt + 1) / 2 + 3) / 4), dim3(256), lds, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}
