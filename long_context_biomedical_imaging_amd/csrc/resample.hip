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
__global__ __launch_bounds__(256) void upsample2x_nhwc_fwd_kernel(UpArgs a) {
  const int C8 = a.C / 8, W2 = 2 * a.W, H2 = 2 * a.H;
  const long long total = (long long)a.B * H2 * W2 * C8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int q = (int)(i % C8);
    long long p = i / C8;
    const int ox = (int)(p % W2);
    p /= W2;
    const int oy = (int)(p % H2), b = (int)(p / H2);
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

__global__ __launch_bounds__(256) void upsample2x_nhwc_bwd_kernel(UpArgs a) {
  const int C8 = a.C / 8, W2 = 2 * a.W, H2 = 2 * a.H;
  const long long total = (long long)a.B * a.H * a.W * C8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int q = (int)(i % C8);
    long long p = i / C8;
    const int ix = (int)(p % a.W);
    p /= a.W;
    const int iy = (int)(p % a.H), b = (int)(p / a.H);
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
  UpArgs a{};
  a.x = x; a.y = (bf16*)y; a.B = B; a.C = C; a.H = H; a.W = W;
  hipLaunchKernelGGL(upsample2x_nhwc_fwd_kernel, dim3(up_grid((long long)B * 4 * H * W * (C / 8))), dim3(256), 0,
                     (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_upsample2x_nhwc_bwd(const void* dy, float* dx, int B, int C, int H, int W, void* stream) {
  LCI_CHECK(B > 0 && C > 0 && H > 0 && W > 0 && C % 8 == 0, "upsample2x: bad shape B=%d C=%d H=%d W=%d", B, C, H, W);
  LCI_CHECK(((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0, "upsample2x: pointers must be 16-byte aligned");
  UpArgs a{};
  a.dy = (const bf16*)dy; a.dx = dx; a.B = B; a.C = C; a.H = H; a.W = W;
  hipLaunchKernelGGL(upsample2x_nhwc_bwd_kernel, dim3(up_grid((long long)B * H * W * (C / 8))), dim3(256), 0,
                     (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}
