// LayerNorm of the transformer blocks' residual stream, with the autocast cast folded into the output.
//
// Replaces TransformerBlock / SwinTransformerBlock norm1, norm2 (nn.LayerNorm, eps 1e-5, backbone_vit.py:250-262,
// backbone_swin.py:418,431) as
// executed under the trainer's bf16 autocast (trainer_base.py:167): torch runs layer_norm in f32 (an autocast
// f32 op), writes the f32 result, and the next Linear (qkv / in_proj / mlp.linear1) reads it back to cast it
// to bf16. Here the forward writes the bf16 operand directly (the same RNE rounding of the same f32 value), and
// the backward reads the bf16 cotangent the Linear produces, so neither cast kernel nor the f32 intermediate
// exists. With dres the backward also adds the residual path's gradient (x feeds both the LN and the residual
// add of the block), so autograd's separate accumulation pass over the residual stream disappears.
// Math (f32, per row of C):
//   forward : mean = sum(x)/C, var = sum((x-mean)^2)/C, rstd = 1/sqrt(var+eps), y = (x-mean) rstd gamma + beta
//   backward: n = (x-mean) rstd, g = dy gamma, dx = [dres +] rstd (g - mean_C(g) - n mean_C(g n));
//             dgamma = sum_rows dy n, dbeta = sum_rows dy (per-workgroup partials, summed by the caller)
// One wave per row: lane l holds the 16-B column groups 4l + 256k (k < NV), so a row is NV coalesced
// 1-KB wave loads. HBM-bound: forward 4C + 2C bytes per row (f32 in, bf16 out), backward 4C + 2C + 4C.
#include "common.hpp"

namespace lci {

constexpr int LN_MAX_C = 2048;   // NV = C / 256 column groups per lane, up to 8 (Swin-large stage 4: C = 1536)

struct LnArgs {
  const float* x;       // (rows, C) f32
  const float* gamma;   // (C)
  const float* beta;    // (C)
  void* y;              // fwd: (rows, C) bf16 or f32
  const void* dy;       // bwd: (rows, C) bf16 or f32
  float* dx;            // bwd: (rows, C) f32
  void* dxb;            // bwd: (rows, C) bf16 copy of dx, or null (the gradient of a bf16 branch output)
  const float* dres;    // bwd: (rows, C) f32 residual-path gradient added into dx, or null
  const float* dres2;   // bwd: a second one (a hidden-state tap's gradient, summed with dres first), or null
  float* mean;          // (rows)
  float* rstd;          // (rows)
  float* part;          // bwd: (gridDim.x, 2, C) partial dgamma, dbeta
  const void* add;      // fwd: (rows, C) bf16 or f32 branch output added to x first (x + add is normalised), or null
  float* xsum;          // fwd with add: (rows, C) f32 x + add, the next residual stream
  int add_bf16;
  long long rows;
  int C, bf16_io;
  float eps;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ f32x4 ld_io4(const void* p, long long i, bool bf) {
  if (bf) {
    const bf16x4 h = *(const bf16x4*)((const bf16*)p + i);
    return f32x4{to_f32(h[0]), to_f32(h[1]), to_f32(h[2]), to_f32(h[3])};
  }
  return *(const f32x4*)((const float*)p + i);
}

template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(LnArgs a) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const int C = a.C;
  const float* xr = a.x + row * C;
  f32x4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = 4 * lane + 256 * k;
    v[k] = c < C ? *(const f32x4*)(xr + c) : f32x4{};
    if (a.add && c < C) {   // residual add of the block's branch output (the f32 sum torch's add produces)
      const f32x4 t = ld_io4(a.add, row * C + c, a.add_bf16);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[k][j] += t[j];
      *(f32x4*)(a.xsum + row * C + c) = v[k];
    }
    s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[k][j] - mean;
        q = fmaf(d, d, q);
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / C + a.eps);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
      const f32x4 g = *(const f32x4*)(a.gamma + c), b = *(const f32x4*)(a.beta + c);
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = fmaf((v[k][j] - mean) * rstd, g[j], b[j]);
      if (a.bf16_io) {
        bf16x4 h;
#pragma unroll
        for (int j = 0; j < 4; ++j) h[j] = to_bf16(o[j]);
        *(bf16x4*)((bf16*)a.y + row * C + c) = h;
      } else {
        *(f32x4*)((float*)a.y + row * C + c) = o;
      }
    }
  }
  if (lane == 0) {
    a.mean[row] = mean;
    a.rstd[row] = rstd;
  }
}

template <int NV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(LnArgs a) {
  __shared__ float red[4][2][NV * 256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int C = a.C;
  const bool bf = a.bf16_io;
  f32x4 gam[NV], dg[NV], db[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = 4 * lane + 256 * k;
    gam[k] = c < C ? *(const f32x4*)(a.gamma + c) : f32x4{};
    dg[k] = f32x4{};
    db[k] = f32x4{};
  }
  const float invC = 1.f / C;
  const long long stride = (long long)gridDim.x * 4;
  for (long long row = (long long)blockIdx.x * 4 + wave; row < a.rows; row += stride) {
    const float mean = a.mean[row], rstd = a.rstd[row];
    f32x4 n[NV], g[NV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = 4 * lane + 256 * k;
      if (c < C) {
        const f32x4 x = *(const f32x4*)(a.x + row * C + c);
        const f32x4 d = ld_io4(a.dy, row * C + c, bf);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          n[k][j] = (x[j] - mean) * rstd;
          g[k][j] = d[j] * gam[k][j];
          s1 += g[k][j];
          s2 = fmaf(g[k][j], n[k][j], s2);
          dg[k][j] = fmaf(d[j], n[k][j], dg[k][j]);
          db[k][j] += d[j];
        }
      } else {
        n[k] = f32x4{};
        g[k] = f32x4{};
      }
    }
    const float m1 = wave_sum(s1) * invC, m2 = wave_sum(s2) * invC;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = 4 * lane + 256 * k;
      if (c < C) {
        f32x4 o = a.dres ? *(const f32x4*)(a.dres + row * C + c) : f32x4{};
        if (a.dres2) {   // dres + dres2: the sum autograd would form of the two consumers' gradients
          const f32x4 o2 = *(const f32x4*)(a.dres2 + row * C + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] += o2[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] += rstd * (g[k][j] - m1 - n[k][j] * m2);
        *(f32x4*)(a.dx + row * C + c) = o;
        if (a.dxb) {   // the same value rounded for a bf16 branch output (no separate cast pass over dx)
          bf16x4 hb;
#pragma unroll
          for (int j = 0; j < 4; ++j) hb[j] = to_bf16(o[j]);
          *(bf16x4*)((bf16*)a.dxb + row * C + c) = hb;
        }
      }
    }
  }
  // the workgroup's dgamma / dbeta partials: 4 waves combined through LDS, one row pair per workgroup
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
      *(f32x4*)&red[wave][0][c] = dg[k];
      *(f32x4*)&red[wave][1][c] = db[k];
    }
  }
  __syncthreads();
  float* out = a.part + (long long)blockIdx.x * 2 * C;
  for (int i = threadIdx.x; i < 2 * C; i += 256) {
    const int w = i / C, c = i % C;
    out[i] = (red[0][w][c] + red[1][w][c]) + (red[2][w][c] + red[3][w][c]);
  }
}

static int ln_check(long long rows, int C, const void* x) {
  LCI_CHECK(x != nullptr, "layernorm: null input");
  LCI_CHECK(rows >= 0 && C > 0 && C % 4 == 0 && C <= LN_MAX_C, "layernorm: need C %% 4 == 0 and C <= %d", LN_MAX_C);
  LCI_CHECK(((uintptr_t)x & 15) == 0, "layernorm: misaligned input");
  return 0;
}

#define LN_SWITCH(KERNEL, NV, GRID, S, A)                                            \
  switch (NV) {                                                                      \
    case 1: hipLaunchKernelGGL(KERNEL<1>, GRID, dim3(256), 0, S, A); break;          \
    case 2: hipLaunchKernelGGL(KERNEL<2>, GRID, dim3(256), 0, S, A); break;          \
    case 3: hipLaunchKernelGGL(KERNEL<3>, GRID, dim3(256), 0, S, A); break;          \
    case 4: hipLaunchKernelGGL(KERNEL<4>, GRID, dim3(256), 0, S, A); break;          \
    case 5: hipLaunchKernelGGL(KERNEL<5>, GRID, dim3(256), 0, S, A); break;          \
    case 6: hipLaunchKernelGGL(KERNEL<6>, GRID, dim3(256), 0, S, A); break;          \
    case 7: hipLaunchKernelGGL(KERNEL<7>, GRID, dim3(256), 0, S, A); break;          \
    default: hipLaunchKernelGGL(KERNEL<8>, GRID, dim3(256), 0, S, A); break;         \
  }

}  // namespace lci

using namespace lci;

extern "C" int lci_layernorm_bwd_blocks(long long rows) {
  const long long waves = (rows + 15) / 16;   // >= 16 rows per wave amortise the partial write
  return (int)std::max(1LL, std::min(2048LL, (waves + 3) / 4));
}

extern "C" int lci_layernorm_fwd(const float* x, const float* gamma, const float* beta, void* y, int bf16_out,
                                 float* mean, float* rstd, long long rows, int C, float eps, void* stream) {
  if (ln_check(rows, C, x)) return 1;
  LCI_CHECK(((uintptr_t)gamma & 15) == 0 && ((uintptr_t)beta & 15) == 0 &&
            ((uintptr_t)y & (bf16_out ? 7 : 15)) == 0, "layernorm: misaligned gamma/beta/output");
  if (rows == 0) return 0;
  LnArgs a = {};
  a.x = x; a.gamma = gamma; a.beta = beta; a.y = y; a.mean = mean; a.rstd = rstd;
  a.rows = rows; a.C = C; a.bf16_io = bf16_out; a.eps = eps;
  const long long nb = (rows + 3) / 4;
  LCI_CHECK(nb < (1LL << 31), "layernorm: too many rows");
  const int NV = (C + 255) / 256;
  hipStream_t s = (hipStream_t)stream;
  LN_SWITCH(ln_fwd_kernel, NV, dim3((unsigned)nb), s, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

// xsum = h + add (f32; add bf16 or f32), y = LayerNorm(xsum): the mid-block residual add fused into norm2.
extern "C" int lci_layernorm_add_fwd(const float* h, const void* add, int add_bf16, float* xsum, const float* gamma,
                                     const float* beta, void* y, int bf16_out, float* mean, float* rstd, long long rows,
                                     int C, float eps, void* stream) {
  if (ln_check(rows, C, h)) return 1;
  LCI_CHECK(add && xsum && ((uintptr_t)add & (add_bf16 ? 7 : 15)) == 0 && ((uintptr_t)xsum & 15) == 0,
            "layernorm_add: misaligned or missing branch / sum");
  LCI_CHECK(((uintptr_t)gamma & 15) == 0 && ((uintptr_t)beta & 15) == 0 &&
            ((uintptr_t)y & (bf16_out ? 7 : 15)) == 0, "layernorm: misaligned gamma/beta/output");
  if (rows == 0) return 0;
  LnArgs a = {};
  a.x = h; a.add = add; a.add_bf16 = add_bf16; a.xsum = xsum;
  a.gamma = gamma; a.beta = beta; a.y = y; a.mean = mean; a.rstd = rstd;
  a.rows = rows; a.C = C; a.bf16_io = bf16_out; a.eps = eps;
  const long long nb = (rows + 3) / 4;
  LCI_CHECK(nb < (1LL << 31), "layernorm: too many rows");
  const int NV = (C + 255) / 256;
  hipStream_t s = (hipStream_t)stream;
  LN_SWITCH(ln_fwd_kernel, NV, dim3((unsigned)nb), s, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_layernorm_bwd(const float* x, const void* dy, int bf16_dy, const float* gamma, const float* mean,
                                 const float* rstd, const float* dres, const float* dres2, float* dx, void* dxb,
                                 float* part, long long rows, int C, void* stream) {
  if (ln_check(rows, C, x)) return 1;
  LCI_CHECK(!dres || ((uintptr_t)dres & 15) == 0, "layernorm: misaligned residual gradient");
  LCI_CHECK(!dres2 || (dres && ((uintptr_t)dres2 & 15) == 0), "layernorm: dres2 needs dres, 16-byte aligned");
  LCI_CHECK(((uintptr_t)dy & (bf16_dy ? 7 : 15)) == 0 && ((uintptr_t)gamma & 15) == 0 &&
            ((uintptr_t)dx & 15) == 0 && ((uintptr_t)dxb & 7) == 0, "layernorm: misaligned dy/gamma/dx");
  LnArgs a = {};
  a.dres = dres;
  a.dres2 = dres2;
  a.x = x; a.dy = dy; a.gamma = gamma; a.mean = const_cast<float*>(mean); a.rstd = const_cast<float*>(rstd);
  a.dx = dx; a.dxb = dxb; a.part = part;
  a.rows = rows; a.C = C; a.bf16_io = bf16_dy;
  const int nb = lci_layernorm_bwd_blocks(rows);
  const int NV = (C + 255) / 256;
  hipStream_t s = (hipStream_t)stream;
  LN_SWITCH(ln_bwd_kernel, NV, dim3(nb), s, a);
  LCI_LAUNCH_CHECK();
  return 0;
}
