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

// grid (ceil(R / 32), C), block 256, dynamic LDS = (32 (LP + 1) + 32 + LP) floats, LP = 32 ceil(L / 32).
// Wave w computes output tiles (32 rows x 32 positions) p and nt-1-p for p = w, w+4, ...: equal work per wave.
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
  const float Dc = a.D ? a.D[c] : 0.f;
  const float* xrow = xs + m * LD + kk;
  for (int p = wave; 2 * p < nt; p += 4) {
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      const int j = h == 0 ? p : nt - 1 - p;
      if (h == 1 && j == p) break;
      // contraction range: fwd s in [0, 32(j+1)); adjoint t in [32j, LP)
      const int i0 = ADJ ? 32 * j : 0, i1 = ADJ ? LP : 32 * (j + 1);
      // B index: fwd kz[32 + 32j + n - i - kk], adjoint kz[32 + i + kk - 32j - n] (n = m: the lane's column)
      const float* kp = ADJ ? kz + 32 + kk - 32 * j - m : kz + 32 + 32 * j + m - kk;
      f32x16 acc{};
#pragma unroll 8
      for (int i = i0; i < i1; i += 2) {
        const float av = xrow[i];
        const float bv = ADJ ? kp[i] : kp[-i];
        acc = mfma_f32(av, bv, acc);
      }
      // D skip and store: reg q holds row (q & 3) + 8 (q >> 2) + 4 kk, column m
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
}

// grid (nsplit, C), block 256, dynamic LDS = 2 * DK_ROWS * LP floats (reused for the band reduction).
// Wave w owns bands p and nt-1-p for p = w, w+4 (band d: nt - d tiles; a pair: nt + 1).
__global__ __launch_bounds__(256, 2) void dconv_dk_kernel(DcArgs a) {
  extern __shared__ float sm[];
  const int L = a.L, nt = (L + 31) / 32, LP = nt * 32;
  float* dys = sm;                   // [DK_ROWS][LP]
  float* us = sm + DK_ROWS * LP;     // [DK_ROWS][LP]
  const int c = blockIdx.y, split = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 31, kk = lane >> 5;
  const int rbeg = split * a.rows_per_split, rend = min(a.R, rbeg + a.rows_per_split);
  int band[4];
  int nb = 0;
  for (int p = wave; 2 * p < nt; p += 4) {
    band[nb++] = p;
    if (nt - 1 - p != p) band[nb++] = nt - 1 - p;
  }
  f32x16 acc[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) acc[b] = f32x16{};
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
    // A[m = t][k = row] = dY[row][32i + m]; B[k = row][n = s] = U[row][32(i - d) + n]
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (b >= nb) break;
      const int d = band[b];
      for (int i = d; i < nt; ++i) {
        const float* ap = dys + kk * LP + 32 * i + m;
        const float* bp = us + kk * LP + 32 * (i - d) + m;
#pragma unroll
        for (int q = 0; q < DK_ROWS; q += 2) acc[b] = mfma_f32(ap[q * LP], bp[q * LP], acc[b]);
      }
    }
  }
  __syncthreads();
  // band reduction: G_d[t][s] (reg q: t = (q & 3) + 8 (q >> 2) + 4 kk, s = m) -> diagonals delta = t - s in [-31, 31]
  float* gs = sm + wave * (4 * 32 * 33);            // per wave: 4 bands x [32][33]
  float* bsum = sm + 4 * 4 * 32 * 33;               // [nt][64]: band d, delta + 31
  for (int b = 0; b < nb; ++b) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int t = (q & 3) + 8 * (q >> 2) + 4 * kk;
      gs[b * 32 * 33 + t * 33 + m] = acc[b][q];
    }
  }
  __syncthreads();
  for (int b = 0; b < nb; ++b) {
    if (lane < 63) {
      const int delta = lane - 31;
      float s = 0.f;
      for (int n = max(0, -delta); n < min(32, 32 - delta); ++n) s += gs[b * 32 * 33 + (n + delta) * 33 + n];
      bsum[band[b] * 64 + lane] = s;
    }
  }
  __syncthreads();
  // dk[tau], tau = 32 d + delta: band d (delta = tau % 32 in [0, 31]) + band d + 1 (delta - 32 in [-32, -1])
  for (int tau = tid; tau < L; tau += 256) {
    const int d = tau >> 5, dl = tau & 31;
    float s = bsum[d * 64 + dl + 31];
    if (d + 1 < nt && dl >= 1) s += bsum[(d + 1) * 64 + dl - 1];
    a.y[((long long)split * a.C + c) * L + tau] = s;
  }
}

static int dk_splits(int R, int C) {
  // ~2 workgroups per CU in total, at least 2 chunks of rows per split
  int ns = std::max(1, 512 / std::max(1, C));
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
  const int LP = 32 * ((L + 31) / 32);
  const size_t lds = (size_t)(32 * (LP + 1) + 32 + LP) * sizeof(float);
  dim3 grid((R + DC_ROWS - 1) / DC_ROWS, C);
  if (adjoint) hipLaunchKernelGGL(dconv_kernel<true>, grid, dim3(256), lds, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(dconv_kernel<false>, grid, dim3(256), lds, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_direct_conv_dk_splits(int R, int C, int L) {
  if (R <= 0 || C <= 0 || L <= 0 || L > DC_MAXL) return 0;
  return dk_splits(R, C);
}

// part (lci_direct_conv_dk_splits(R, C, L), C, L) f32 <- per-row-split sums of dy[r][t] u[r][t - tau]; the caller
// sums the first axis for dk; dD[c] = dk[c][0].
extern "C" int lci_direct_conv_dk(const float* dy, const float* u, float* part, int R, int C, int L, void* stream) {
  LCI_CHECK(R > 0 && C > 0 && L > 0 && L <= DC_MAXL, "direct_conv_dk: bad shape R=%d C=%d L=%d", R, C, L);
  const int ns = dk_splits(R, C);
  DcArgs a{};
  a.x = dy; a.u = u; a.y = part; a.R = R; a.C = C; a.L = L;
  a.rows_per_split = DK_ROWS * ((R + ns * DK_ROWS - 1) / (ns * DK_ROWS));
  const int LP = 32 * ((L + 31) / 32);
  const size_t lds = std::max((size_t)2 * DK_ROWS * LP, (size_t)(4 * 4 * 32 * 33 + 16 * 64)) * sizeof(float);
  hipLaunchKernelGGL(dconv_dk_kernel, dim3(ns, C), dim3(256), lds, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}
