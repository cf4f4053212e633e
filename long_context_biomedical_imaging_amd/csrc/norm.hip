// Instance normalisation (+ LeakyReLU) over channels-last volumes, for the UNETR decoder heads.
//
// Replaces MONAI-1.3 UnetResBlock's norm1 + lrelu, norm2 and norm3 (InstanceNorm{2,3}d(C), affine=False,
// eps 1e-5, biased variance; LeakyReLU(0.01)) in ViTUNETR / SwinUNETR (model/models/enhance_heads.py:30-356),
// without the NCDHW round trips torch's instance_norm needs (it runs batch_norm on a contiguous (1, B*C, ...)
// view): x stays (B, V, C) bf16 channels-last between the HIP convolutions.
//   forward : n = (x - mean[b,c]) * rstd[b,c];  z = act ? lrelu(n) : n
//   backward: dn = dz * (act && n < 0 ? slope : 1);  dx = rstd * (dn - mean_V(dn) - n * mean_V(dn * n))
// Two passes each way: a reduction (per-(b, c) partial sums over voxel chunks, combined in f64 by
// inorm_finalize_kernel into the stats / coefficients) and an elementwise pass. All HBM-bound: a thread moves 8
// channels (16 B) per voxel.
#include "common.hpp"

namespace lci {

struct NormArgs {
  const bf16* x;       // (B, V, C)
  const bf16* dz;      // bwd: (B, V, C)
  bf16* out;           // fwd: z; bwd: dx
  const float* stats;  // (B, 2, C): mean, rstd
  const float* coef;   // bwd: (B, 2, C): mean_V(dn), mean_V(dn * n)
  float* part;         // (B, 2, C, nchunk) partial sums (chunk fastest: one contiguous row per (b, sum, c))
  long long V, chunk;
  int C, nchunk, act;
  float slope;
};

__device__ __forceinline__ void load8(const bf16* p, float* f) {
  const bf16x8 v = *(const bf16x8*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = to_f32(v[j]);
}

// mean / rstd of 8 consecutive channels (st: the (2, C) stats row of one sample; 32-byte aligned: C % 8 == 0)
__device__ __forceinline__ void load_stats(const float* st, int C, float* mu, float* rs) {
  const f32x4 m0 = *(const f32x4*)st, m1 = *(const f32x4*)(st + 4);
  const f32x4 r0 = *(const f32x4*)(st + C), r1 = *(const f32x4*)(st + C + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { mu[j] = m0[j]; mu[4 + j] = m1[j]; rs[j] = r0[j]; rs[4 + j] = r1[j]; }
}

// BWD = false: sums of x and x^2.  BWD = true: sums of dn and dn * n.
template <bool BWD>
__global__ __launch_bounds__(256) void inorm_reduce_kernel(NormArgs a) {
  __shared__ float red[2][2048];
  const int G = a.C >> 3, rows = 256 / G;
  const int tid = threadIdx.x, g = tid % G, r = tid / G;
  const int b = blockIdx.y, chunk = blockIdx.x;
  const long long v0 = chunk * a.chunk, v1 = min(a.V, v0 + a.chunk);
  float s1[8], s2[8], mu[8], rs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  if (BWD && r < rows) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mu[j] = a.stats[(long long)b * 2 * a.C + 8 * g + j];
      rs[j] = a.stats[(long long)b * 2 * a.C + a.C + 8 * g + j];
    }
  }
  if (r < rows) {
    const long long base = (long long)b * a.V * a.C + 8 * g;
    // UN voxels per iteration, their loads issued together (one 16-byte load in flight per lane held the pass near
    // 2-3 TB/s); the sums keep the single-voxel order (voxel v, then v + rows, ...)
    constexpr int UN = 4;
    for (long long v = v0 + r; v < v1; v += UN * rows) {
      float x[UN][8], d[UN][8];
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        const long long vu = v + (long long)u * rows;
        if (vu < v1) {
          load8(a.x + base + vu * a.C, x[u]);
          if (BWD) load8(a.dz + base + vu * a.C, d[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        if (v + (long long)u * rows >= v1) break;
        if (!BWD) {
#pragma unroll
          for (int j = 0; j < 8; ++j) { s1[j] += x[u][j]; s2[j] += x[u][j] * x[u][j]; }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float n = (x[u][j] - mu[j]) * rs[j];
            const float dn = (a.act && n < 0.f) ? d[u][j] * a.slope : d[u][j];
            s1[j] += dn;
            s2[j] += dn * n;
          }
        }
      }
    }
  }
  // combine the `rows` voxel lanes of each channel through LDS
  for (int c = tid; c < rows * a.C; c += 256) { red[0][c] = 0.f; red[1][c] = 0.f; }
  __syncthreads();
  if (r < rows) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[0][r * a.C + 8 * g + j] = s1[j]; red[1][r * a.C + 8 * g + j] = s2[j]; }
  }
  __syncthreads();
  for (int c = tid; c < a.C; c += 256) {
    float t1 = 0.f, t2 = 0.f;
    for (int q = 0; q < rows; ++q) { t1 += red[0][q * a.C + c]; t2 += red[1][q * a.C + c]; }
    float* p = a.part + ((long long)b * 2 * a.C + c) * a.nchunk + chunk;
    p[0] = t1;
    p[(long long)a.C * a.nchunk] = t2;
  }
}

template <bool BWD>
__global__ __launch_bounds__(256) void inorm_apply_kernel(NormArgs a) {
  const int G = a.C >> 3;
  const long long e0 = blockIdx.x * 256LL;                 // 8-channel group index over (B, V, G)
  const long long e = e0 + threadIdx.x;
  const int b = blockIdx.y;
  if (e >= a.V * G) return;
  // the block's first group modulo G is workgroup-uniform (scalar); the lane's is then a 32-bit remainder
  const int g = ((int)(e0 % G) + (int)threadIdx.x) % G;
  const long long off = (long long)b * a.V * a.C + e * 8;
  float x[8], mu[8], rs[8];
  load8(a.x + off, x);
  load_stats(a.stats + (long long)b * 2 * a.C + 8 * g, a.C, mu, rs);   // f32x4 loads, not 16 scalar ones
  bf16x8 o;
  if (!BWD) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float n = (x[j] - mu[j]) * rs[j];
      if (a.act && n < 0.f) n *= a.slope;
      o[j] = to_bf16(n);
    }
  } else {
    float d[8], c1[8], c2[8];
    load8(a.dz + off, d);
    load_stats(a.coef + (long long)b * 2 * a.C + 8 * g, a.C, c1, c2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float n = (x[j] - mu[j]) * rs[j];
      const float dn = (a.act && n < 0.f) ? d[j] * a.slope : d[j];
      o[j] = to_bf16(rs[j] * (dn - c1[j] - n * c2[j]));
    }
  }
  *(bf16x8*)(a.out + off) = o;
}

// UnetResBlock's tail in one pass: out = lrelu(bf16(bf16(norm(x)) + r)), r = bf16(norm(y; stats_y)) (the norm3 /
// conv3 residual) or y itself (a bf16 block input), with torch's bf16 roundings of the unfused
// instance_norm -> add -> leaky_relu sequence (each op rounds its output to bf16).
template <bool PRE>
__global__ __launch_bounds__(256) void inorm_res_kernel(NormArgs a, const bf16* __restrict__ y,
                                                       const float* __restrict__ stats_y) {
  const int G = a.C >> 3;
  const long long e = blockIdx.x * 256LL + threadIdx.x;
  const int b = blockIdx.y;
  if (e >= a.V * G) return;
  const int g = ((int)((e - threadIdx.x) % G) + (int)threadIdx.x) % G;   // uniform 64-bit part, 32-bit lane part
  const long long off = (long long)b * a.V * a.C + e * 8;
  float x[8], r[8], mu[8], rs[8], muy[8], rsy[8];
  load8(a.x + off, x);
  load8(y + off, r);
  load_stats(a.stats + (long long)b * 2 * a.C + 8 * g, a.C, mu, rs);   // 8 consecutive channels: f32x4 loads
  if (PRE) load_stats(stats_y + (long long)b * 2 * a.C + 8 * g, a.C, muy, rsy);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float n = to_f32(to_bf16((x[j] - mu[j]) * rs[j]));
    const float rr = PRE ? to_f32(to_bf16((r[j] - muy[j]) * rsy[j])) : r[j];
    const float sum = to_f32(to_bf16(n + rr));
    o[j] = to_bf16(sum > 0.f ? sum : sum * a.slope);
  }
  *(bf16x8*)(a.out + off) = o;
}

// part (B, 2, C, nchunk) -> out (B, 2, C): one wave per (b, c) sums both rows in f64 (lane-strided, 8 loads in
// flight per lane, then a fixed xor-shuffle tree: deterministic), divided by V; mode 0: (mean, rstd = 1 / sqrt(
// max(E[x^2] - mean^2, 0) + eps)), the f64 arithmetic of the unfused torch code; mode 1: the voxel means themselves
// (the backward's coefficients).
__global__ __launch_bounds__(256) void inorm_finalize_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                             long long V, int B, int C, int nchunk, int mode,
                                                             float eps) {
  const int lane = threadIdx.x & 63;
  const long long wv = blockIdx.x * 4LL + (threadIdx.x >> 6);   // (b, c)
  if (wv >= (long long)B * C) return;
  const int b = (int)(wv / C), c = (int)(wv % C);
  const float* p1 = part + ((long long)b * 2 * C + c) * nchunk;
  const float* p2 = p1 + (long long)C * nchunk;
  double s1 = 0.0, s2 = 0.0;
  for (int k0 = 0; k0 < nchunk; k0 += 64 * 8) {
    float v1[8], v2[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + 64 * u + lane;
      v1[u] = k < nchunk ? p1[k] : 0.f;
      v2[u] = k < nchunk ? p2[k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) { s1 += (double)v1[u]; s2 += (double)v2[u]; }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  if (lane == 0) {
    const double m1 = s1 / (double)V, m2 = s2 / (double)V;
    float* o = out + (long long)b * 2 * C;
    if (mode == 0) {
      o[c] = (float)m1;
      o[C + c] = (float)(1.0 / sqrt(fmax(m2 - m1 * m1, 0.0) + (double)eps));
    } else {
      o[c] = (float)m1;
      o[C + c] = (float)m2;
    }
  }
}

// ------------------------------------------------------------------ BatchNorm (training) + ReLU, channels-last
// UperNet's conv -> BatchNorm -> ReLU (seg_heads.py PSPModule bottleneck :23-27 / FPN conv_fusion :59-62, the 2-D
// and 3-D heads) on the conv's bf16 channels-last output: the batch statistics are the instance-norm reduction over
// all B * V voxels as one sample (lci_inorm_reduce / _finalize with B = 1); these kernels apply the affine map and the
// ReLU (f32 out, what autocast's fp32 batch_norm returns) and run the backward: g = dy * [y > 0], the channel sums of
// g and g * xhat (partials, then lci_inorm_finalize mode 1), dx = (g - mean(g) - xhat mean(g xhat)) rstd w in x's
// dtype. Per element torch's expression order: xhat = (x - mean) * rstd, y = xhat * w + b.
struct BnArgs {
  const bf16* x;          // (V, C)
  const void* dy;         // bwd: (V, C) f32 or bf16
  const float* stats;     // (2, C): mean, rstd
  const float* coef;      // bwd apply: (2, C): mean(g), mean(g xhat)
  const float* w; const float* b;
  void* out;              // fwd: y f32; bwd: dx bf16
  float* part;            // bwd reduce: (2, C, nchunk)
  long long V, chunk;
  int C, nchunk, dy_f32;
};

__device__ __forceinline__ void load8f(const void* p, long long off, bool f32, float* v) {
  if (f32) {
    const f32x4 a = *(const f32x4*)((const float*)p + off), c = *(const f32x4*)((const float*)p + off + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = c[j]; }
  } else {
    load8((const bf16*)p + off, v);
  }
}

// the affine parameters of 8 consecutive channels as f32x4 loads
__device__ __forceinline__ void load_wb(const float* w, const float* b, int g, float* wv, float* bv) {
  const f32x4 w0 = *(const f32x4*)(w + 8 * g), w1 = *(const f32x4*)(w + 8 * g + 4);
  const f32x4 b0 = *(const f32x4*)(b + 8 * g), b1 = *(const f32x4*)(b + 8 * g + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { wv[j] = w0[j]; wv[4 + j] = w1[j]; bv[j] = b0[j]; bv[4 + j] = b1[j]; }
}

__global__ __launch_bounds__(256) void bn_relu_fwd_kernel(BnArgs a) {
  const int G = a.C >> 3;
  const long long e = blockIdx.x * 256LL + threadIdx.x;
  if (e >= a.V * G) return;
  const int g = ((int)((e - threadIdx.x) % G) + (int)threadIdx.x) % G;   // uniform 64-bit part, 32-bit lane part
  float x[8], mu[8], rs[8], wv[8], bv[8];
  load8(a.x + e * 8, x);
  load_stats(a.stats + 8 * g, a.C, mu, rs);
  load_wb(a.w, a.b, g, wv, bv);
  float* y = (float*)a.out + e * 8;
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = __fadd_rn(__fmul_rn(__fmul_rn(__fsub_rn(x[j], mu[j]), rs[j]), wv[j]), bv[j]);
    o[j] = v > 0.f ? v : 0.f;
  }
  *(f32x4*)y = f32x4{o[0], o[1], o[2], o[3]};
  *(f32x4*)(y + 4) = f32x4{o[4], o[5], o[6], o[7]};
}

// partial sums of g and g * xhat per (channel, voxel chunk); part (2, C, nchunk)
__global__ __launch_bounds__(256) void bn_relu_bwd_reduce_kernel(BnArgs a) {
  __shared__ float red[2][2048];
  const int G = a.C >> 3, rows = 256 / G;
  const int tid = threadIdx.x, g = tid % G, r = tid / G;
  const int chunk = blockIdx.x;
  const long long v0 = chunk * a.chunk, v1 = min(a.V, v0 + a.chunk);
  float s1[8], s2[8], mu[8], rs[8], w[8], bb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  if (r < rows) {
    load_stats(a.stats + 8 * g, a.C, mu, rs);
#pragma unroll
    for (int j = 0; j < 8; ++j) { w[j] = a.w[8 * g + j]; bb[j] = a.b[8 * g + j]; }
    for (long long v = v0 + r; v < v1; v += rows) {
      float x[8], d[8];
      load8(a.x + v * a.C + 8 * g, x);
      load8f(a.dy, v * a.C + 8 * g, a.dy_f32 != 0, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float n = __fmul_rn(__fsub_rn(x[j], mu[j]), rs[j]);
        const float gg = __fadd_rn(__fmul_rn(n, w[j]), bb[j]) > 0.f ? d[j] : 0.f;
        s1[j] += gg;
        s2[j] += gg * n;
      }
    }
  }
  for (int c = tid; c < rows * a.C; c += 256) { red[0][c] = 0.f; red[1][c] = 0.f; }
  __syncthreads();
  if (r < rows) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[0][r * a.C + 8 * g + j] = s1[j]; red[1][r * a.C + 8 * g + j] = s2[j]; }
  }
  __syncthreads();
  for (int c = tid; c < a.C; c += 256) {
    float t1 = 0.f, t2 = 0.f;
    for (int q = 0; q < rows; ++q) { t1 += red[0][q * a.C + c]; t2 += red[1][q * a.C + c]; }
    float* p = a.part + (long long)c * a.nchunk + chunk;
    p[0] = t1;
    p[(long long)a.C * a.nchunk] = t2;
  }
}

__global__ __launch_bounds__(256) void bn_relu_bwd_apply_kernel(BnArgs a) {
  const int G = a.C >> 3;
  const long long e = blockIdx.x * 256LL + threadIdx.x;
  if (e >= a.V * G) return;
  const int g = ((int)((e - threadIdx.x) % G) + (int)threadIdx.x) % G;   // uniform 64-bit part, 32-bit lane part
  float x[8], d[8], mu[8], rs[8], m1[8], m2[8], wv[8], bv[8];
  load8(a.x + e * 8, x);
  load8f(a.dy, e * 8, a.dy_f32 != 0, d);
  load_stats(a.stats + 8 * g, a.C, mu, rs);
  load_stats(a.coef + 8 * g, a.C, m1, m2);
  load_wb(a.w, a.b, g, wv, bv);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float w = wv[j];
    const float n = __fmul_rn(__fsub_rn(x[j], mu[j]), rs[j]);
    const float gg = __fadd_rn(__fmul_rn(n, w), bv[j]) > 0.f ? d[j] : 0.f;
    o[j] = to_bf16((gg - m1[j] - n * m2[j]) * (rs[j] * w));
  }
  *(bf16x8*)((bf16*)a.out + e * 8) = o;
}

}  // namespace lci

using namespace lci;

extern "C" int lci_inorm_chunks(long long V, int B);

// Training BatchNorm + ReLU over x (V, C) bf16 channels-last (all B * V voxels), stats (2, C) from lci_inorm_reduce /
// lci_inorm_finalize (B = 1): y (V, C) f32 = relu((x - mean) rstd w + b).
extern "C" int lci_bn_relu_fwd(const void* x, const float* stats, const float* w, const float* b, float* y,
                               long long V, int C, void* stream) {
  LCI_CHECK(V > 0 && C > 0 && C % 8 == 0 && C <= 2048, "bn_relu: bad shape");
  LCI_CHECK((((uintptr_t)x | (uintptr_t)y | (uintptr_t)stats) & 15) == 0, "bn_relu: misaligned buffers");
  BnArgs a = {};
  a.x = (const bf16*)x; a.stats = stats; a.w = w; a.b = b; a.out = y; a.V = V; a.C = C;
  const long long groups = V * (C / 8);
  LCI_CHECK((groups + 255) / 256 < (1LL << 31), "bn_relu: volume too large");
  hipLaunchKernelGGL(bn_relu_fwd_kernel, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

// Backward partial sums: part (2, C, lci_inorm_chunks(V, 1)) of g = dy [y > 0] and g xhat; dy (V, C) f32 or bf16.
extern "C" int lci_bn_relu_bwd_reduce(const void* x, const void* dy, int dy_f32, const float* stats, const float* w,
                                      const float* b, float* part, long long V, int C, void* stream) {
  LCI_CHECK(V > 0 && C > 0 && C % 8 == 0 && C <= 2048, "bn_relu: bad shape");
  LCI_CHECK((((uintptr_t)x | (uintptr_t)dy | (uintptr_t)stats) & 15) == 0, "bn_relu: misaligned buffers");
  BnArgs a = {};
  a.x = (const bf16*)x; a.dy = dy; a.dy_f32 = dy_f32; a.stats = stats; a.w = w; a.b = b; a.part = part;
  a.V = V; a.C = C;
  a.nchunk = lci_inorm_chunks(V, 1);
  a.chunk = (V + a.nchunk - 1) / a.nchunk;
  hipLaunchKernelGGL(bn_relu_bwd_reduce_kernel, dim3(a.nchunk), dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

// dx (V, C) bf16 = (g - coef[0]) - xhat coef[1]) rstd w; coef (2, C) = (mean(g), mean(g xhat)) from lci_inorm_finalize
// mode 1 over the reduce partials.
extern "C" int lci_bn_relu_bwd_apply(const void* x, const void* dy, int dy_f32, const float* stats, const float* coef,
                                     const float* w, const float* b, void* dx, long long V, int C, void* stream) {
  LCI_CHECK(V > 0 && C > 0 && C % 8 == 0 && C <= 2048, "bn_relu: bad shape");
  LCI_CHECK((((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx | (uintptr_t)stats | (uintptr_t)coef) & 15) == 0,
            "bn_relu: misaligned buffers");
  BnArgs a = {};
  a.x = (const bf16*)x; a.dy = dy; a.dy_f32 = dy_f32; a.stats = stats; a.coef = coef; a.w = w; a.b = b; a.out = dx;
  a.V = V; a.C = C;
  const long long groups = V * (C / 8);
  LCI_CHECK((groups + 255) / 256 < (1LL << 31), "bn_relu: volume too large");
  hipLaunchKernelGGL(bn_relu_bwd_apply_kernel, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_inorm_finalize(const float* part, float* out, long long V, int B, int C, int mode, float eps,
                                  void* stream) {
  LCI_CHECK(V > 0 && B > 0 && C > 0 && (mode == 0 || mode == 1), "inorm_finalize: bad arguments");
  const int nchunk = lci_inorm_chunks(V, B);
  hipLaunchKernelGGL(inorm_finalize_kernel, dim3((unsigned)(((long long)B * C + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, part, out, V, B, C, nchunk, mode, eps);
  LCI_LAUNCH_CHECK();
  return 0;
}

// Voxel chunks per sample for the reduction: ~2048 workgroups in total, at least 256 voxels per chunk.
extern "C" int lci_inorm_chunks(long long V, int B) {
  long long n = (2048 + B - 1) / B;
  if (n > (V + 255) / 256) n = (V + 255) / 256;
  return (int)(n < 1 ? 1 : n);
}

static int norm_check(long long V, int B, int C, const void* x) {
  LCI_CHECK(V > 0 && B > 0 && C > 0 && C % 8 == 0 && C <= 2048, "inorm: bad shape (C %% 8 == 0, C <= 2048)");
  LCI_CHECK(((uintptr_t)x & 15) == 0, "inorm: misaligned input");
  return 0;
}

extern "C" int lci_inorm_reduce(const void* x, const void* dz, const float* stats, float* part, long long V, int B,
                                int C, int act, float slope, void* stream) {
  if (norm_check(V, B, C, x)) return 1;
  NormArgs a = {};
  a.x = (const bf16*)x; a.dz = (const bf16*)dz; a.stats = stats; a.part = part;
  a.V = V; a.C = C; a.act = act; a.slope = slope;
  a.nchunk = lci_inorm_chunks(V, B);
  a.chunk = (V + a.nchunk - 1) / a.nchunk;
  dim3 grid(a.nchunk, B);
  if (dz)
    hipLaunchKernelGGL(inorm_reduce_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(inorm_reduce_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_inorm_apply(const void* x, const void* dz, const float* stats, const float* coef, void* out,
                               long long V, int B, int C, int act, float slope, void* stream) {
  if (norm_check(V, B, C, x)) return 1;
  LCI_CHECK(((uintptr_t)out & 15) == 0 && (!dz || ((uintptr_t)dz & 15) == 0), "inorm: misaligned buffers");
  NormArgs a = {};
  a.x = (const bf16*)x; a.dz = (const bf16*)dz; a.stats = stats; a.coef = coef; a.out = (bf16*)out;
  a.V = V; a.C = C; a.act = act; a.slope = slope;
  const long long groups = V * (C / 8);
  LCI_CHECK((groups + 255) / 256 < (1LL << 31), "inorm: volume too large");
  dim3 grid((unsigned)((groups + 255) / 256), B);
  if (dz)
    hipLaunchKernelGGL(inorm_apply_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(inorm_apply_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_inorm_apply_res(const void* x, const float* stats, const void* y, const float* stats_y, void* out,
                                   long long V, int B, int C, float slope, void* stream) {
  if (norm_check(V, B, C, x)) return 1;
  LCI_CHECK(((uintptr_t)out & 15) == 0 && ((uintptr_t)y & 15) == 0, "inorm: misaligned buffers");
  NormArgs a = {};
  a.x = (const bf16*)x; a.stats = stats; a.out = (bf16*)out;
  a.V = V; a.C = C; a.slope = slope;
  const long long groups = V * (C / 8);
  LCI_CHECK((groups + 255) / 256 < (1LL << 31), "inorm: volume too large");
  LCI_CHECK(((uintptr_t)stats & 15) == 0 && ((uintptr_t)stats_y & 15) == 0, "inorm: misaligned stats");
  const dim3 grid((unsigned)((groups + 255) / 256), B);
  if (stats_y)
    hipLaunchKernelGGL(inorm_res_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, a, (const bf16*)y, stats_y);
  else
    hipLaunchKernelGGL(inorm_res_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, a, (const bf16*)y, stats_y);
  LCI_LAUNCH_CHECK();
  return 0;
}
