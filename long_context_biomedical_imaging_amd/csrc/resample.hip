// Bilinear x2 up-sampling (align_corners=False) for gfx950: the last re-sampling of UperNet2D.forward
// (reference model/models/seg_heads.py:138, F.interpolate(x, size=self.input_size, mode="bilinear")) fused with the layout
// change into the next 3x3 conv's channels-last bf16 operand, and its adjoint.
//
// Forward:  x (B, C, H, W) f32 NCHW -> y (B, 2H, 2W, C) bf16 channels-last, with torch's arithmetic
//           (upsample_bilinear2d: src = max(0.5 (o + 0.5) - 0.5, 0), i0 = (int)src, i1 = i0 + (i0 < n - 1),
//           l1 = src - i0, y = l0y (l0x x00 + l1x x01) + l1y (l0x x10 + l1x x11) in f32, then the bf16 rounding the
//           conv's autocast cast would apply).
// Backward: dy (B, 2H, 2W, C) bf16 channels-last -> dx (B, C, H, W) f32 as a deterministic gather (each input pixel
//           sums its <= 4 x 4 contributing outputs) instead of torch's atomic scatter.
// Both stage 64-channel tiles through LDS so that the NCHW rows and the channels-last pixels are each accessed
// with contiguous 16-byte (channels-last) or row-coalesced (NCHW) vectors.
#include "common.hpp"

#include <algorithm>

namespace lci {

struct UpArgs {
  const float* x; bf16* y;          // forward
  const bf16* dy; float* dx;        // backward
  int B, C, H, W;                   // input size (output 2H x 2W)
};

constexpr int UP_CB = 64;           // channels per workgroup
constexpr int UP_JB = 32;           // input columns per workgroup

// Source taps of output index o along an axis of n input samples (scale 1/2, align_corners=False).
__device__ __forceinline__ void up_taps(int o, int n, int& i0, int& i1, float& l0, float& l1) {
  float src = 0.5f * ((float)o + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  i0 = (int)src;
  i1 = i0 + (i0 < n - 1 ? 1 : 0);
  l1 = src - (float)i0;
  l0 = 1.f - l1;
}

// Weight of input i in output o (sum of both taps: they coincide at the borders).
__device__ __forceinline__ float up_weight(int o, int n, int i) {
  int i0, i1;
  float l0, l1;
  up_taps(o, n, i0, i1, l0, l1);
  return (i0 == i ? l0 : 0.f) + (i1 == i ? l1 : 0.f);
}

// grid (ceil(W / UP_JB), H, B * ceil(C / UP_CB)); block 256. Output rows 2iy, 2iy + 1; input rows iy - 1 .. iy + 1.
__global__ __launch_bounds__(256) void upsample2x_fwd_kernel(UpArgs a) {
  constexpr int XC = UP_JB + 2;                      // input columns j0 - 1 .. j0 + UP_JB
  __shared__ float xs[UP_CB][3][XC];
  const int j0 = blockIdx.x * UP_JB, iy = blockIdx.y;
  const int ncb = (a.C + UP_CB - 1) / UP_CB, b = blockIdx.z / ncb, c0 = (blockIdx.z % ncb) * UP_CB;
  for (int i = threadIdx.x; i < UP_CB * 3 * XC; i += 256) {
    const int col = i % XC, r = (i / XC) % 3, c = i / (3 * XC);
    const int row = min(max(iy - 1 + r, 0), a.H - 1), gc = min(max(j0 - 1 + col, 0), a.W - 1);
    xs[c][r][col] = (c0 + c < a.C) ? a.x[(((long long)b * a.C + c0 + c) * a.H + row) * a.W + gc] : 0.f;
  }
  __syncthreads();
  const int W2 = 2 * a.W;
  for (int i = threadIdx.x; i < 2 * (2 * UP_JB) * (UP_CB / 8); i += 256) {
    const int q = i & 7, oxl = (i >> 3) % (2 * UP_JB), oyl = i / (8 * 2 * UP_JB);
    const int oy = 2 * iy + oyl, ox = 2 * j0 + oxl, c = c0 + 8 * q;
    if (ox >= W2 || c >= a.C) continue;
    int h0, h1, w0, w1;
    float hl0, hl1, wl0, wl1;
    up_taps(oy, a.H, h0, h1, hl0, hl1);
    up_taps(ox, a.W, w0, w1, wl0, wl1);
    const int r0 = h0 - (iy - 1), r1 = h1 - (iy - 1), q0 = w0 - (j0 - 1), q1 = w1 - (j0 - 1);
    bf16x8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float(*p)[XC] = xs[8 * q + k];
      v[k] = (bf16)(hl0 * (wl0 * p[r0][q0] + wl1 * p[r0][q1]) + hl1 * (wl0 * p[r1][q0] + wl1 * p[r1][q1]));
    }
    *(bf16x8*)(a.y + (((long long)b * 2 * a.H + oy) * W2 + ox) * a.C + c) = v;
  }
}

// grid (ceil(W / UP_JB), H, B * ceil(C / UP_CB)); block 256. Input row iy gathers output rows 2iy - 1 .. 2iy + 2.
__global__ __launch_bounds__(256) void upsample2x_bwd_kernel(UpArgs a) {
  constexpr int OC = 2 * UP_JB + 2;                  // output columns 2 j0 - 1 .. 2 j0 + 2 UP_JB
  __shared__ __attribute__((aligned(16))) bf16 gs[4][OC][UP_CB];
  __shared__ float out[UP_CB][UP_JB + 1];
  const int j0 = blockIdx.x * UP_JB, iy = blockIdx.y;
  const int ncb = (a.C + UP_CB - 1) / UP_CB, b = blockIdx.z / ncb, c0 = (blockIdx.z % ncb) * UP_CB;
  const int H2 = 2 * a.H, W2 = 2 * a.W;
  for (int i = threadIdx.x; i < 4 * OC * (UP_CB / 8); i += 256) {
    const int q = i & 7, col = (i >> 3) % OC, r = i / (8 * OC);
    const int oy = 2 * iy - 1 + r, ox = 2 * j0 - 1 + col, c = c0 + 8 * q;
    bf16x8 v = {};
    if (oy >= 0 && oy < H2 && ox >= 0 && ox < W2 && c < a.C)
      v = *(const bf16x8*)(a.dy + (((long long)b * H2 + oy) * W2 + ox) * a.C + c);
    *(bf16x8*)(&gs[r][col][8 * q]) = v;
  }
  __syncthreads();
  const int c = threadIdx.x & 63;
  float wy[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int oy = 2 * iy - 1 + r;
    wy[r] = (oy >= 0 && oy < H2) ? up_weight(oy, a.H, iy) : 0.f;
  }
  for (int jl = threadIdx.x >> 6; jl < UP_JB; jl += 4) {
    const int jx = j0 + jl;
    float acc = 0.f;
    if (jx < a.W) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int ox = 2 * jx - 1 + t;
        const float wx = (ox >= 0 && ox < W2) ? up_weight(ox, a.W, jx) : 0.f;
        const int col = ox - (2 * j0 - 1);
        float s = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) s += wy[r] * (float)gs[r][col][c];
        acc += wx * s;
      }
    }
    out[c][jl] = acc;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < UP_CB * UP_JB; i += 256) {
    const int jl = i % UP_JB, cl = i / UP_JB, jx = j0 + jl;
    if (jx < a.W && c0 + cl < a.C) a.dx[(((long long)b * a.C + c0 + cl) * a.H + iy) * a.W + jx] = out[cl][jl];
  }
}


// Channels-last (NHWC) variants, for a channels-last input map: x (B, H, W, C) f32 -> y (B, 2H, 2W, C) bf16, and
// dy (B, 2H, 2W, C) bf16 -> dx (B, H, W, C) f32. One thread per (pixel, 8-channel chunk): the chunks of a pixel
// are consecutive threads, so every tap is a contiguous 32-byte (f32) or 16-byte (bf16) access.
// grid (ceil(2W * C/8 / 256), B * 2H): one output row per block row, 32-bit index math (the grid-stride form's 64-bit
// divisions per 16-byte chunk held it near 2.3 TB/s at C4's 1024^2 x 384 output)
__global__ __launch_bounds__(256) void upsample2x_nhwc_fwd_kernel(UpArgs a) {
  const int C8 = a.C / 8, W2 = 2 * a.W, H2 = 2 * a.H;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < W2 * C8) {
    const int ox = i / C8, q = i - ox * C8;
    const int oy = (int)(blockIdx.y % H2), b = (int)(blockIdx.y / H2);
    int h0, h1, w0, w1;
    float hl0, hl1, wl0, wl1;
    up_taps(oy, a.H, h0, h1, hl0, hl1);
    up_taps(ox, a.W, w0, w1, wl0, wl1);
    const float* base = a.x + (long long)b * a.H * a.W * a.C + 8 * q;
    const float* p00 = base + ((long long)h0 * a.W + w0) * a.C;
    const float* p01 = base + ((long long)h0 * a.W + w1) * a.C;
    const float* p10 = base + ((long long)h1 * a.W + w0) * a.C;
    const float* p11 = base + ((long long)h1 * a.W + w1) * a.C;
    bf16x8 v;
#pragma unroll
    for (int hv = 0; hv < 2; ++hv) {
      const f32x4 x00 = *(const f32x4*)(p00 + 4 * hv), x01 = *(const f32x4*)(p01 + 4 * hv);
      const f32x4 x10 = *(const f32x4*)(p10 + 4 * hv), x11 = *(const f32x4*)(p11 + 4 * hv);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        v[4 * hv + k] = (bf16)(hl0 * (wl0 * x00[k] + wl1 * x01[k]) + hl1 * (wl0 * x10[k] + wl1 * x11[k]));
    }
    *(bf16x8*)(a.y + (((long long)b * H2 + oy) * W2 + ox) * a.C + 8 * q) = v;
  }
}

// grid (ceil(W * C/8 / 256), B * H): one input row per block row
__global__ __launch_bounds__(256) void upsample2x_nhwc_bwd_kernel(UpArgs a) {
  const int C8 = a.C / 8, W2 = 2 * a.W, H2 = 2 * a.H;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < a.W * C8) {
    const int ix = i / C8, q = i - ix * C8;
    const int iy = (int)(blockIdx.y % a.H), b = (int)(blockIdx.y / a.H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ty = 0; ty < 4; ++ty) {
      const int oy = 2 * iy - 1 + ty;
      if (oy < 0 || oy >= H2) continue;
      const float wy = up_weight(oy, a.H, iy);
      if (wy == 0.f) continue;
#pragma unroll
      for (int tx = 0; tx < 4; ++tx) {
        const int ox = 2 * ix - 1 + tx;
        if (ox < 0 || ox >= W2) continue;
        const float w = wy * up_weight(ox, a.W, ix);
        if (w == 0.f) continue;
        const bf16x8 g = *(const bf16x8*)(a.dy + (((long long)b * H2 + oy) * W2 + ox) * a.C + 8 * q);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = fmaf(w, (float)g[k], acc[k]);
      }
    }
    float* o = a.dx + (((long long)b * a.H + iy) * a.W + ix) * a.C + 8 * q;
    *(f32x4*)o = f32x4{acc[0], acc[1], acc[2], acc[3]};
    *(f32x4*)(o + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
  }
}

// ------------------------------------------------------------- trilinear up-sampling (align_corners=False)
// UperNet3D.forward's last re-sampling (seg_heads.py:273, F.interpolate(x, size=input_size, mode="trilinear")) into
// the head conv's channels-last bf16 operand, for any output size (scale = in / out per axis, as torch's
// area_pixel_compute_scale with no scale factor). Forward: one thread per (output voxel, 8-channel chunk), torch's
// upsample_trilinear3d expression in f32, rounded to bf16 (the conv's autocast cast). Backward: the adjoint applied
// one axis at a time (resample1d_adj_kernel), each a deterministic gather over the <= 2 ceil(out / in) + 2 outputs
// that touch an input sample — the fused 3-D gather would re-read every output 8 times.
struct Up3Args {
  const float* x; bf16* y;
  int B, C, D, H, W, OD, OH, OW;
  float sd, sh, sw;                 // in / out per axis
};

// torch: src = scale * (o + 0.5) - 0.5, clamped at 0 (area_pixel_compute_source_index, linear modes), products
// kept unfused so that the taps match torch's for any scale
__device__ __forceinline__ void lin_taps(int o, int n, float scale, int& i0, int& i1, float& l0, float& l1) {
  float src = __fsub_rn(__fmul_rn(scale, __fadd_rn((float)o, 0.5f)), 0.5f);
  src = src < 0.f ? 0.f : src;
  i0 = (int)src;
  i1 = i0 + (i0 < n - 1 ? 1 : 0);
  l1 = __fsub_rn(src, (float)i0);
  l0 = __fsub_rn(1.f, l1);
}

// grid (ceil(OW * C/8 / 256), OH, B * OD): one output row (b, oz, oy) per block row, so the depth / height taps are
// block-uniform and the per-thread index math is 32-bit (ox, 8-channel chunk q).
__global__ __launch_bounds__(256) void upsample3d_cl_fwd_kernel(Up3Args a) {
  const int C8 = a.C / 8;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.OW * C8) return;
  const int ox = i / C8, q = i - ox * C8;
  const int oy = blockIdx.y, oz = blockIdx.z % a.OD, b = blockIdx.z / a.OD;
  int d0, d1, h0, h1, w0, w1;
  float dl0, dl1, hl0, hl1, wl0, wl1;
  lin_taps(oz, a.D, a.sd, d0, d1, dl0, dl1);
  lin_taps(oy, a.H, a.sh, h0, h1, hl0, hl1);
  lin_taps(ox, a.W, a.sw, w0, w1, wl0, wl1);
  const float* base = a.x + (long long)b * a.D * a.H * a.W * a.C + 8 * q;
  auto at = [&](int d, int h, int w) { return base + (((long long)d * a.H + h) * a.W + w) * a.C; };
  const float* p000 = at(d0, h0, w0); const float* p001 = at(d0, h0, w1);
  const float* p010 = at(d0, h1, w0); const float* p011 = at(d0, h1, w1);
  const float* p100 = at(d1, h0, w0); const float* p101 = at(d1, h0, w1);
  const float* p110 = at(d1, h1, w0); const float* p111 = at(d1, h1, w1);
  bf16x8 v;
#pragma unroll
  for (int hv = 0; hv < 2; ++hv) {
    const f32x4 x000 = *(const f32x4*)(p000 + 4 * hv), x001 = *(const f32x4*)(p001 + 4 * hv);
    const f32x4 x010 = *(const f32x4*)(p010 + 4 * hv), x011 = *(const f32x4*)(p011 + 4 * hv);
    const f32x4 x100 = *(const f32x4*)(p100 + 4 * hv), x101 = *(const f32x4*)(p101 + 4 * hv);
    const f32x4 x110 = *(const f32x4*)(p110 + 4 * hv), x111 = *(const f32x4*)(p111 + 4 * hv);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      v[4 * hv + k] = (bf16)(dl0 * (hl0 * (wl0 * x000[k] + wl1 * x001[k]) + hl1 * (wl0 * x010[k] + wl1 * x011[k])) +
                             dl1 * (hl0 * (wl0 * x100[k] + wl1 * x101[k]) + hl1 * (wl0 * x110[k] + wl1 * x111[k])));
  }
  *(bf16x8*)(a.y + ((((long long)b * a.OD + oz) * a.OH + oy) * a.OW + ox) * a.C + 8 * q) = v;
}

// Adjoint of 1-D linear interpolation (align_corners=False, scale = n_in / n_out) along the middle axis of
// dy (outer, n_out, inner) -> dx (outer, n_in, inner) f32 (written): dx[., i, .] = sum_o w(o, i) dy[., o, .] over
// the outputs o whose taps include i, in increasing o. inner % 8 == 0; one thread per (outer, i, 8-element chunk).
struct Adj1Args {
  const void* dy; float* dx;
  long long outer, inner;
  int n_out, n_in, dy_bf16, ac;
  float scale;
};

// align_corners=True taps (torch: scale = (in - 1) / (out - 1), 0 for one output; src = scale * o)
__device__ __forceinline__ void lin_taps_ac(int o, int n, float scale, int& i0, int& i1, float& l0, float& l1) {
  const float src = __fmul_rn(scale, (float)o);
  i0 = (int)src;
  i1 = i0 + (i0 < n - 1 ? 1 : 0);
  l1 = __fsub_rn(src, (float)i0);
  l0 = __fsub_rn(1.f, l1);
}

// Outputs [lo, hi] whose source coordinate lies in (i - 1, i + 1] (one extra on each side covers the f32 rounding),
// and the weight of input i in output o (the sum of both taps: they coincide at the borders).
__device__ __forceinline__ void adj_range(const Adj1Args& a, int i, int& lo, int& hi) {
  const float r = 1.f / a.scale;    // outputs per input sample
  if (a.ac) {
    lo = a.scale > 0.f ? max(0, (int)floorf(((float)i - 1.f) * r) - 1) : 0;
    hi = a.scale > 0.f ? min(a.n_out - 1, (int)ceilf(((float)i + 1.f) * r) + 1) : a.n_out - 1;
  } else {
    lo = max(0, (int)floorf(((float)i - 1.f + 0.5f) * r - 0.5f) - 1);
    hi = min(a.n_out - 1, (int)ceilf(((float)i + 1.f + 0.5f) * r - 0.5f) + 1);
  }
}

__device__ __forceinline__ float adj_weight(const Adj1Args& a, int o, int i) {
  int i0, i1;
  float l0, l1;
  if (a.ac) lin_taps_ac(o, a.n_in, a.scale, i0, i1, l0, l1);
  else lin_taps(o, a.n_in, a.scale, i0, i1, l0, l1);
  return (i0 == i ? l0 : 0.f) + (i1 == i ? l1 : 0.f);
}

__device__ __forceinline__ void adj_acc(const Adj1Args& a, long long off, float w, float (&acc)[8]) {
  if (a.dy_bf16) {
    const bf16x8 g = *(const bf16x8*)((const bf16*)a.dy + off);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = fmaf(w, (float)g[k], acc[k]);
  } else {
    const f32x4 g0 = *(const f32x4*)((const float*)a.dy + off), g1 = *(const f32x4*)((const float*)a.dy + off + 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[k] = fmaf(w, g0[k], acc[k]);
      acc[4 + k] = fmaf(w, g1[k], acc[4 + k]);
    }
  }
}

// grid (ceil(n_in inner/8 / 256), min(outer, 65535)): 32-bit (input sample, chunk) index math, outer rows by block row
__global__ __launch_bounds__(256) void resample1d_adj_kernel(Adj1Args a) {
  const int I8 = (int)(a.inner / 8);
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= a.n_in * I8) return;
  const int i = e / I8, q = e - i * I8;
  int lo, hi;
  adj_range(a, i, lo, hi);
  for (long long ou = blockIdx.y; ou < a.outer; ou += gridDim.y) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int o = lo; o <= hi; ++o) {
      const float w = adj_weight(a, o, i);
      if (w == 0.f) continue;
      adj_acc(a, (ou * a.n_out + o) * a.inner + 8 * q, w, acc);
    }
    float* o = a.dx + (ou * a.n_in + i) * a.inner + 8 * q;
    *(f32x4*)o = f32x4{acc[0], acc[1], acc[2], acc[3]};
    *(f32x4*)(o + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
  }
}

// The same adjoint where each input sample gathers many outputs (the PSP's 1-6 pooled bins up-sampled to the
// feature grid: up to n_out per input): one thread per output there was ~1 wave per CU, each looping over hundreds of
// dependent-address loads. Here a workgroup takes (outer, i, 8 consecutive 8-element chunks of inner): 32 lanes
// per chunk split the output range (o = lo + s, lo + s + 32, ...), and the 32 partials are summed in LDS in a fixed
// order (deterministic).
constexpr int ADJ_WIDE_S = 32;
__global__ __launch_bounds__(256) void resample1d_adj_wide_kernel(Adj1Args a) {
  __shared__ float red[ADJ_WIDE_S][8][9];
  const long long I8 = a.inner / 8, QB = (I8 + 7) / 8;
  const int c = threadIdx.x & 7, s = threadIdx.x >> 3;
  const long long blk = blockIdx.x;
  const long long qb = blk % QB;
  const long long p = blk / QB;
  const int i = (int)(p % a.n_in);
  const long long ou = p / a.n_in;
  const long long q = qb * 8 + c;
  int lo, hi;
  adj_range(a, i, lo, hi);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (q < I8) {
    for (int o = lo + s; o <= hi; o += ADJ_WIDE_S) {
      const float w = adj_weight(a, o, i);
      if (w == 0.f) continue;
      adj_acc(a, (ou * a.n_out + o) * a.inner + 8 * q, w, acc);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[s][c][k] = acc[k];
  __syncthreads();
  if (threadIdx.x < 64) {   // (chunk c2, element k2): the 32 partials in order s = 0 .. 31
    const int c2 = threadIdx.x >> 3, k2 = threadIdx.x & 7;
    float v = 0.f;
#pragma unroll 8
    for (int ss = 0; ss < ADJ_WIDE_S; ++ss) v += red[ss][c2][k2];
    const long long q2 = qb * 8 + c2;
    if (q2 < I8) a.dx[(ou * a.n_in + i) * a.inner + 8 * q2 + k2] = v;
  }
}

// ------------------------------------------------ linear re-sampling to any size, f32 out (align_corners either way)
// FPN_fuse's resize (seg_heads.py:49-50, :74 / :181-182, :206: F.interpolate(x, size, mode=(bi|tri)linear, align_corners=True),
// f32 under autocast) and PSPModule's up-sampling of the pooled bins (seg_heads.py:44 / :176), on channels-last maps
// (2-D as D = OD = 1): one thread per (output voxel, 8-channel chunk), torch's upsample_{bilinear2d,trilinear3d}
// expression in f32 (products unfused), plus an optional addend of the output's shape summed in the same pass (the
// FPN's `resize(f) + lateral`, an f32 add as torch's). Input and addend f32 or bf16 (read as f32: the cast autocast
// would apply is exact). The adjoint is resample1d_adj per axis (deterministic gathers, no atomic scatter).
struct RsArgs {
  const void* x; const void* add; float* y;
  int B, C, D, H, W, OD, OH, OW;
  float sd, sh, sw;
  int x_bf16, add_bf16, ac;
};

__device__ __forceinline__ void rs_taps(int ac, int o, int n, float scale, int& i0, int& i1, float& l0, float& l1) {
  if (ac) lin_taps_ac(o, n, scale, i0, i1, l0, l1);
  else lin_taps(o, n, scale, i0, i1, l0, l1);
}

__device__ __forceinline__ void ld8f(const void* p, long long off, bool bf, float (&v)[8]) {
  if (bf) {
    const bf16x8 g = *(const bf16x8*)((const bf16*)p + off);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (float)g[k];
  } else {
    const f32x4 g0 = *(const f32x4*)((const float*)p + off), g1 = *(const f32x4*)((const float*)p + off + 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[k] = g0[k]; v[4 + k] = g1[k]; }
  }
}

// grid (ceil(OW * C/8 / 256), OH, B * OD)
__global__ __launch_bounds__(256) void resample_cl_fwd_kernel(RsArgs a) {
  const int C8 = a.C / 8;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.OW * C8) return;
  const int ox = i / C8, q = i - ox * C8;
  const int oy = blockIdx.y, oz = blockIdx.z % a.OD, b = blockIdx.z / a.OD;
  int d0, d1, h0, h1, w0, w1;
  float dl0, dl1, hl0, hl1, wl0, wl1;
  rs_taps(a.ac, oz, a.D, a.sd, d0, d1, dl0, dl1);
  rs_taps(a.ac, oy, a.H, a.sh, h0, h1, hl0, hl1);
  rs_taps(a.ac, ox, a.W, a.sw, w0, w1, wl0, wl1);
  const bool bf = a.x_bf16 != 0;
  const long long base = (long long)b * a.D * a.H * a.W * a.C + 8 * q;
  auto at = [&](int d, int h, int w) { return base + (((long long)d * a.H + h) * a.W + w) * a.C; };
  float x000[8], x001[8], x010[8], x011[8];
  ld8f(a.x, at(d0, h0, w0), bf, x000); ld8f(a.x, at(d0, h0, w1), bf, x001);
  ld8f(a.x, at(d0, h1, w0), bf, x010); ld8f(a.x, at(d0, h1, w1), bf, x011);
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k)
    v[k] = __fadd_rn(__fmul_rn(hl0, __fadd_rn(__fmul_rn(wl0, x000[k]), __fmul_rn(wl1, x001[k]))),
                     __fmul_rn(hl1, __fadd_rn(__fmul_rn(wl0, x010[k]), __fmul_rn(wl1, x011[k]))));
  if (a.D > 1 || a.OD > 1) {   // trilinear: t0 * (plane d0) + t1 * (plane d1)
    float x100[8], x101[8], x110[8], x111[8];
    ld8f(a.x, at(d1, h0, w0), bf, x100); ld8f(a.x, at(d1, h0, w1), bf, x101);
    ld8f(a.x, at(d1, h1, w0), bf, x110); ld8f(a.x, at(d1, h1, w1), bf, x111);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float p1 = __fadd_rn(__fmul_rn(hl0, __fadd_rn(__fmul_rn(wl0, x100[k]), __fmul_rn(wl1, x101[k]))),
                                 __fmul_rn(hl1, __fadd_rn(__fmul_rn(wl0, x110[k]), __fmul_rn(wl1, x111[k]))));
      v[k] = __fadd_rn(__fmul_rn(dl0, v[k]), __fmul_rn(dl1, p1));
    }
  }
  const long long oo = ((((long long)b * a.OD + oz) * a.OH + oy) * a.OW + ox) * a.C + 8 * q;
  if (a.add != nullptr) {
    float r[8];
    ld8f(a.add, oo, a.add_bf16 != 0, r);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = __fadd_rn(v[k], r[k]);
  }
  *(f32x4*)(a.y + oo) = f32x4{v[0], v[1], v[2], v[3]};
  *(f32x4*)(a.y + oo + 4) = f32x4{v[4], v[5], v[6], v[7]};
}

static unsigned up_grid(long long items) {
  const long long want = (items + 255) / 256;
  return (unsigned)std::max(1LL, std::min(want, 256LL * 64));
}

}  // namespace lci

using namespace lci;

extern "C" int lci_upsample2x_fwd(const float* x, void* y, int B, int C, int H, int W, void* stream) {
  LCI_CHECK(B > 0 && C > 0 && H > 0 && W > 0 && C % 8 == 0, "upsample2x: bad shape B=%d C=%d H=%d W=%d", B, C, H, W);
  LCI_CHECK(((uintptr_t)y & 15) == 0, "upsample2x: output must be 16-byte aligned");
  UpArgs a{};
  a.x = x; a.y = (bf16*)y; a.B = B; a.C = C; a.H = H; a.W = W;
  dim3 grid((W + UP_JB - 1) / UP_JB, H, B * ((C + UP_CB - 1) / UP_CB));
  hipLaunchKernelGGL(upsample2x_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_upsample2x_bwd(const void* dy, float* dx, int B, int C, int H, int W, void* stream) {
  LCI_CHECK(B > 0 && C > 0 && H > 0 && W > 0 && C % 8 == 0, "upsample2x: bad shape B=%d C=%d H=%d W=%d", B, C, H, W);
  LCI_CHECK(((uintptr_t)dy & 15) == 0, "upsample2x: gradient must be 16-byte aligned");
  UpArgs a{};
  a.dy = (const bf16*)dy; a.dx = dx; a.B = B; a.C = C; a.H = H; a.W = W;
  dim3 grid((W + UP_JB - 1) / UP_JB, H, B * ((C + UP_CB - 1) / UP_CB));
  hipLaunchKernelGGL(upsample2x_bwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

// Channels-last variants: x (B, H, W, C) f32 -> y (B, 2H, 2W, C) bf16; dy (B, 2H, 2W, C) bf16 -> dx (B, H, W, C) f32.
extern "C" int lci_upsample2x_nhwc_fwd(const float* x, void* y, int B, int C, int H, int W, void* stream) {
  LCI_CHECK(B > 0 && C > 0 && H > 0 && W > 0 && C % 8 == 0, "upsample2x: bad shape B=%d C=%d H=%d W=%d", B, C, H, W);
  LCI_CHECK(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0, "upsample2x: pointers must be 16-byte aligned");
  LCI_CHECK((long long)B * 2 * H <= 65535 && (long long)2 * W * (C / 8) < (1LL << 31),
            "upsample2x: output too large for the grid");
  UpArgs a{};
  a.x = x; a.y = (bf16*)y; a.B = B; a.C = C; a.H = H; a.W = W;
  hipLaunchKernelGGL(upsample2x_nhwc_fwd_kernel, dim3((unsigned)((2LL * W * (C / 8) + 255) / 256), (unsigned)(B * 2 * H)),
                     dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_upsample2x_nhwc_bwd(const void* dy, float* dx, int B, int C, int H, int W, void* stream) {
  LCI_CHECK(B > 0 && C > 0 && H > 0 && W > 0 && C % 8 == 0, "upsample2x: bad shape B=%d C=%d H=%d W=%d", B, C, H, W);
  LCI_CHECK(((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0, "upsample2x: pointers must be 16-byte aligned");
  LCI_CHECK((long long)B * H <= 65535 && (long long)W * (C / 8) < (1LL << 31), "upsample2x: input too large for the grid");
  UpArgs a{};
  a.dy = (const bf16*)dy; a.dx = dx; a.B = B; a.C = C; a.H = H; a.W = W;
  hipLaunchKernelGGL(upsample2x_nhwc_bwd_kernel, dim3((unsigned)(((long long)W * (C / 8) + 255) / 256), (unsigned)(B * H)),
                     dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

// Trilinear (align_corners=False) to any size: x (B, D, H, W, C) f32 channels-last -> y (B, OD, OH, OW, C) bf16.
extern "C" int lci_upsample3d_cl_fwd(const float* x, void* y, int B, int C, int D, int H, int W, int OD, int OH, int OW,
                                     void* stream) {
  LCI_CHECK(B > 0 && C > 0 && D > 0 && H > 0 && W > 0 && OD > 0 && OH > 0 && OW > 0 && C % 8 == 0,
            "upsample3d: bad shape B=%d C=%d in %dx%dx%d out %dx%dx%d", B, C, D, H, W, OD, OH, OW);
  LCI_CHECK(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0, "upsample3d: pointers must be 16-byte aligned");
  Up3Args a{};
  a.x = x; a.y = (bf16*)y; a.B = B; a.C = C; a.D = D; a.H = H; a.W = W; a.OD = OD; a.OH = OH; a.OW = OW;
  a.sd = (float)D / (float)OD; a.sh = (float)H / (float)OH; a.sw = (float)W / (float)OW;
  LCI_CHECK((long long)B * OD <= 65535 && OH <= 65535, "upsample3d: output too large for the grid");
  hipLaunchKernelGGL(upsample3d_cl_fwd_kernel, dim3((OW * (C / 8) + 255) / 256, OH, B * OD), dim3(256), 0,
                     (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

// torch's area_pixel_compute_scale for linear modes without a scale factor
static float rs_scale(int n_in, int n_out, int ac) {
  if (ac) return n_out > 1 ? (float)(n_in - 1) / (float)(n_out - 1) : 0.f;
  return (float)n_in / (float)n_out;
}

// Adjoint of linear interpolation along one axis: dy (outer, n_out, inner) (bf16 if dy_bf16 else f32) ->
// dx (outer, n_in, inner) f32, align_corners as given. inner % 8 == 0, 16-byte aligned.
extern "C" int lci_resample1d_adj_ac(const void* dy, int dy_bf16, float* dx, long long outer, int n_out, int n_in,
                                     long long inner, int align_corners, void* stream) {
  LCI_CHECK(outer > 0 && n_out > 0 && n_in > 0 && inner > 0 && inner % 8 == 0,
            "resample1d_adj: bad shape outer=%lld n_out=%d n_in=%d inner=%lld", outer, n_out, n_in, inner);
  LCI_CHECK(((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0, "resample1d_adj: pointers must be 16-byte aligned");
  Adj1Args a{};
  a.dy = dy; a.dx = dx; a.outer = outer; a.inner = inner; a.n_out = n_out; a.n_in = n_in; a.dy_bf16 = dy_bf16;
  a.ac = align_corners ? 1 : 0;
  a.scale = rs_scale(n_in, n_out, a.ac);
  if (n_out >= 16 * n_in) {   // >= ~32 outputs per input: the split-range kernel
    const long long nblk = outer * n_in * ((inner / 8 + 7) / 8);
    LCI_CHECK(nblk < (1LL << 31), "resample1d_adj: grid too large");
    hipLaunchKernelGGL(resample1d_adj_wide_kernel, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, a);
  } else {
    LCI_CHECK((long long)n_in * (inner / 8) < (1LL << 31), "resample1d_adj: row too wide");
    hipLaunchKernelGGL(resample1d_adj_kernel, dim3((unsigned)(((long long)n_in * (inner / 8) + 255) / 256),
                                                   (unsigned)std::min<long long>(outer, 65535)),
                       dim3(256), 0, (hipStream_t)stream, a);
  }
  LCI_LAUNCH_CHECK();
  return 0;
}

// The align_corners=False adjoint (UperNet3D's final re-sampling).
extern "C" int lci_resample1d_adj(const void* dy, int dy_bf16, float* dx, long long outer, int n_out, int n_in,
                                  long long inner, void* stream) {
  return lci_resample1d_adj_ac(dy, dy_bf16, dx, outer, n_out, n_in, inner, 0, stream);
}

// Linear re-sampling (bilinear for D = OD = 1, else trilinear) of x (B, D, H, W, C) channels-last (f32, or bf16 when
// x_bf16) to y (B, OD, OH, OW, C) f32 [+ add (B, OD, OH, OW, C), f32 or bf16 when add_bf16], align_corners as given.
// C % 8 == 0; pointers 16-byte aligned.
extern "C" int lci_resample_cl_fwd(const void* x, int x_bf16, const void* add, int add_bf16, float* y, int B, int C,
                                   int D, int H, int W, int OD, int OH, int OW, int align_corners, void* stream) {
  LCI_CHECK(B > 0 && C > 0 && D > 0 && H > 0 && W > 0 && OD > 0 && OH > 0 && OW > 0 && C % 8 == 0,
            "resample: bad shape B=%d C=%d in %dx%dx%d out %dx%dx%d", B, C, D, H, W, OD, OH, OW);
  LCI_CHECK((((uintptr_t)x | (uintptr_t)add | (uintptr_t)y) & 15) == 0, "resample: pointers must be 16-byte aligned");
  LCI_CHECK((long long)B * OD <= 65535 && OH <= 65535, "resample: output too large for the grid");
  RsArgs a{};
  a.x = x; a.add = add; a.y = y; a.B = B; a.C = C; a.D = D; a.H = H; a.W = W; a.OD = OD; a.OH = OH; a.OW = OW;
  a.ac = align_corners ? 1 : 0;
  a.sd = rs_scale(D, OD, a.ac); a.sh = rs_scale(H, OH, a.ac); a.sw = rs_scale(W, OW, a.ac);
  a.x_bf16 = x_bf16; a.add_bf16 = add_bf16;
  hipLaunchKernelGGL(resample_cl_fwd_kernel, dim3((OW * (C / 8) + 255) / 256, OH, B * OD), dim3(256), 0,
                     (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}
