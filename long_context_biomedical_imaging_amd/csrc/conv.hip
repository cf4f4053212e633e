// 3x3(x3) stride-1 "same" convolution for the UNETR decoder heads, channels-last, bf16 MFMA, f32 accumulate.
//
// Replaces the MONAI-1.3 get_conv_layer(kernel_size=3, stride=1, conv_only=True, bias=False) convolutions of
// UnetResBlock (conv1 / conv2) used by ViTUNETR (enhance_heads.py:187-356) and SwinUNETR (:30-184):
//     y[b, p, n] = sum_{tap, c} x[b, p + off(tap), c] * w[n, c, tap]      (zero outside the volume)
// with off(tap) = (kd - 1, kh - 1, kw - 1) over KD x 3 x 3 taps (KD = 3 for 3-D, 1 for 2-D volumes, D = 1).
// The same kernel computes the data gradient: dx = conv(dy, w') with w'[c, tap, n] = w[n, c, 26 - tap]
// (the tap set is symmetric), packed by the caller.
//
// Implicit GEMM, no im2col: Y^T (Cout x voxels) = W (Cout x K) . X_im2col^T (K x voxels), K = taps * Cin.
// A wave owns 64 voxels x 32*NT output channels: per 16-wide k-step it loads two 16-byte X fragments
// (8 consecutive channels of one voxel's neighbour per lane; masked to zero outside the volume) and NT weight
// fragments, and issues 2*NT v_mfma_f32_32x32x16_bf16. With W as the A operand, a lane's accumulators hold 4
// consecutive output channels per register quad, so the bf16 results go out as 8-byte stores.
// Neighbour reuse (27 taps read the same voxels) is served by L1/L2: the volume is swept in voxel order.
#include <stdlib.h>

#include "common.hpp"

#ifndef LCI_CONV_MV_WIDE
#define LCI_CONV_MV_WIDE 4   // 32-voxel blocks per wave for NT >= 3 (A/B: tools/conv_variants.sh)
#endif

// scheduling-strategy hooks for A/B runs (tools/conv_variants.sh): iglp_opt(N) on the fwd / wgrad main loops
#ifdef LCI_CONV_IGLP
#define LCI_CONV_SCHED() __builtin_amdgcn_iglp_opt(LCI_CONV_IGLP)
#else
#define LCI_CONV_SCHED()
#endif
#ifdef LCI_WGRAD_IGLP
#define LCI_WGRAD_SCHED() __builtin_amdgcn_iglp_opt(LCI_WGRAD_IGLP)
#else
#define LCI_WGRAD_SCHED()
#endif

namespace lci {

struct ConvArgs {
  const bf16* x;    // (B, D, H, W, Cin)
  const bf16* w;    // (Cout, T, Cin), T = KD * 9
  bf16* y;          // (B, D, H, W, Cout)
  long long V;      // B * D * H * W
  int D, H, W, Cin, Cout, KD;
};

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
  return z;
}

// Vector path: Cin % 16 == 0. NT = 32-channel output blocks per wave, MV = 32-voxel blocks per wave.
template <int NT, int MV>
__global__ __launch_bounds__(256) void conv3_fwd_kernel(ConvArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const long long v0 = ((long long)blockIdx.x * 4 + wave) * 32 * MV;
  const int n0 = blockIdx.y * 32 * NT;
  const int T = a.KD * 9;
  const int HW = a.H * a.W;
  // voxel coordinates of this lane's B-operand columns (voxels v0 + 32m + r)
  int zc[MV], yc[MV], xc[MV];
  long long vb[MV];
  bool inb[MV];
#pragma unroll
  for (int m = 0; m < MV; ++m) {
    const long long v = v0 + 32 * m + r;
    inb[m] = v < a.V;
    const long long vv = inb[m] ? v : 0;
    const long long s = vv / ((long long)a.D * HW);
    int rem = (int)(vv - s * (long long)a.D * HW);
    zc[m] = rem / HW; rem -= zc[m] * HW;
    yc[m] = rem / a.W; xc[m] = rem - yc[m] * a.W;
    vb[m] = vv;
  }
  f32x16 acc[MV][NT];
#pragma unroll
  for (int m = 0; m < MV; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][t][i] = 0.f;

  const bf16* wrow[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wrow[t] = a.w + (long long)(n0 + 32 * t + r) * T * a.Cin + 8 * h;

  for (int tap = 0; tap < T; ++tap) {
    const int dz = (a.KD == 3 ? tap / 9 : 1) - 1, dy = (tap / 3) % 3 - 1, dx = tap % 3 - 1;
    const bf16* px[MV];
    bool ok[MV];
#pragma unroll
    for (int m = 0; m < MV; ++m) {
      const int z = zc[m] + dz, y = yc[m] + dy, xx = xc[m] + dx;
      ok[m] = inb[m] && (unsigned)z < (unsigned)a.D && (unsigned)y < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
      const long long nb = vb[m] + (long long)dz * HW + dy * a.W + dx;
      px[m] = a.x + (ok[m] ? nb : 0) * a.Cin + 8 * h;
    }
    const long long wt = (long long)tap * a.Cin;
#pragma unroll 2
    for (int c = 0; c < a.Cin; c += 16) {
      bf16x8 xb[MV], wa[NT];
#pragma unroll
      for (int m = 0; m < MV; ++m) {
        xb[m] = *(const bf16x8*)(px[m] + c);
        if (!ok[m]) xb[m] = zero8();
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) wa[t] = *(const bf16x8*)(wrow[t] + wt + c);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int m = 0; m < MV; ++m) acc[m][t] = mfma32(wa[t], xb[m], acc[m][t]);
    }
  }
  // acc[m][t] reg i: output channel n0 + 32t + (i&3) + 8(i>>2) + 4h, voxel v0 + 32m + r
#pragma unroll
  for (int m = 0; m < MV; ++m) {
    if (!inb[m]) continue;
    bf16* yp = a.y + vb[m] * a.Cout + n0 + 4 * h;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = to_bf16(acc[m][t][4 * q + j]);
        *(bf16x4*)(yp + 32 * t + 8 * q) = o;
      }
  }
}

// LDS-staged variant (Cin % 32 == 0): a workgroup owns 4*32*MV consecutive voxels. For each (dz, dy) tap
// group and 32-channel chunk it stages the contiguous source rows [v0 + off(dz,dy) - 1, ... + 4*32*MV + 1) of x
// (so the three dx taps read the same LDS rows at offsets 0, 1, 2) and the three taps' weight slabs, with
// coalesced 16-B loads; fragments then come from LDS (80-B rows). Replaces 3 global fragment loads per voxel
// block and tap by one staged row set, and shares the weight fragments across the 4 waves.
constexpr int CLD = 40;   // LDS row stride (elements): 32 channels + 8 pad = 80 B

template <int NT, int MV>
__global__ __launch_bounds__(256) void conv3_fwd_lds_kernel(ConvArgs a) {
  constexpr int WV = 4 * 32 * MV;                 // voxels per workgroup
  constexpr int XR = WV + 2;                      // staged rows (dx halo)
  __shared__ __attribute__((aligned(16))) bf16 sX[XR * CLD];
  __shared__ __attribute__((aligned(16))) bf16 sW[3 * 32 * NT * CLD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  const long long vg0 = (long long)blockIdx.x * WV;
  const int n0 = blockIdx.y * 32 * NT;
  const int T = a.KD * 9;
  const int HW = a.H * a.W;
  int zc[MV], yc[MV], xc[MV];
  bool inb[MV];
#pragma unroll
  for (int m = 0; m < MV; ++m) {
    const long long v = vg0 + wave * 32 * MV + 32 * m + r;
    inb[m] = v < a.V;
    const long long vv = inb[m] ? v : 0;
    const long long s = vv / ((long long)a.D * HW);
    int rem = (int)(vv - s * (long long)a.D * HW);
    zc[m] = rem / HW; rem -= zc[m] * HW;
    yc[m] = rem / a.W; xc[m] = rem - yc[m] * a.W;
  }
  f32x16 acc[MV][NT];
#pragma unroll
  for (int m = 0; m < MV; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][t][i] = 0.f;

  const int ngroups = a.KD * 3;
  for (int grp = 0; grp < ngroups; ++grp) {
    const int dz = (a.KD == 3 ? grp / 3 : 1) - 1, dy = grp % 3 - 1;
    const long long src0 = vg0 + (long long)dz * HW + (long long)dy * a.W - 1;   // source row of LDS row 0
    bool okzy[MV];
#pragma unroll
    for (int m = 0; m < MV; ++m)
      okzy[m] = inb[m] && (unsigned)(zc[m] + dz) < (unsigned)a.D && (unsigned)(yc[m] + dy) < (unsigned)a.H;
    for (int c0 = 0; c0 < a.Cin; c0 += 32) {
      __syncthreads();
      for (int q = tid; q < XR * 4; q += 256) {
        const int row = q >> 2, ch = q & 3;
        const long long u = src0 + row;
        u32x4 val = {0u, 0u, 0u, 0u};
        if (u >= 0 && u < a.V) val = *(const u32x4*)(a.x + u * a.Cin + c0 + 8 * ch);
        *(u32x4*)(sX + row * CLD + 8 * ch) = val;
      }
      for (int q = tid; q < 3 * 32 * NT * 4; q += 256) {
        const int row = q >> 2, ch = q & 3;                 // row = dx * 32NT + n
        const int dxi = row / (32 * NT), n = row - dxi * 32 * NT;
        const int tap = grp * 3 + dxi;
        *(u32x4*)(sW + row * CLD + 8 * ch) =
            *(const u32x4*)(a.w + ((long long)(n0 + n) * T + tap) * a.Cin + c0 + 8 * ch);
      }
      __syncthreads();
      LCI_CONV_SCHED();
#pragma unroll
      for (int dxi = 0; dxi < 3; ++dxi) {
        bool ok[MV];
#pragma unroll
        for (int m = 0; m < MV; ++m) ok[m] = okzy[m] && (unsigned)(xc[m] + dxi - 1) < (unsigned)a.W;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          bf16x8 wa[NT], xb[MV];
#pragma unroll
          for (int t = 0; t < NT; ++t)
            wa[t] = *(const bf16x8*)(sW + (dxi * 32 * NT + 32 * t + r) * CLD + 16 * ks + 8 * h);
#pragma unroll
          for (int m = 0; m < MV; ++m) {
            xb[m] = *(const bf16x8*)(sX + (wave * 32 * MV + 32 * m + r + dxi) * CLD + 16 * ks + 8 * h);
            if (!ok[m]) xb[m] = zero8();
          }
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int m = 0; m < MV; ++m) acc[m][t] = mfma32(wa[t], xb[m], acc[m][t]);
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MV; ++m) {
    if (!inb[m]) continue;
    const long long v = vg0 + wave * 32 * MV + 32 * m + r;
    bf16* yp = a.y + v * a.Cout + n0 + 4 * h;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = to_bf16(acc[m][t][4 * q + j]);
        *(bf16x4*)(yp + 32 * t + 8 * q) = o;
      }
  }
}

// Generic path (any Cin, e.g. the 1-channel image into encoder1): K = T * Cin flattened and zero-padded to
// 16; each lane gathers its 8 k-values element by element. Only used for tiny Cin, where K is small.
template <int NT>
__global__ __launch_bounds__(256) void conv3_fwd_generic_kernel(ConvArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const long long v0 = ((long long)blockIdx.x * 4 + wave) * 64;
  const int n0 = blockIdx.y * 32 * NT;
  const int T = a.KD * 9;
  const int K = T * a.Cin;
  const int HW = a.H * a.W;
  int zc[2], yc[2], xc[2];
  long long vb[2];
  bool inb[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const long long v = v0 + 32 * m + r;
    inb[m] = v < a.V;
    const long long vv = inb[m] ? v : 0;
    const long long s = vv / ((long long)a.D * HW);
    int rem = (int)(vv - s * (long long)a.D * HW);
    zc[m] = rem / HW; rem -= zc[m] * HW;
    yc[m] = rem / a.W; xc[m] = rem - yc[m] * a.W;
    vb[m] = vv;
  }
  f32x16 acc[2][NT];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][t][i] = 0.f;
  for (int k0 = 0; k0 < K; k0 += 16) {
    bf16x8 xb[2], wa[NT];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + 8 * h + j;
      const int tap = k / a.Cin, c = k - tap * a.Cin;
      const int dz = (a.KD == 3 ? tap / 9 : 1) - 1, dy = (tap / 3) % 3 - 1, dx = tap % 3 - 1;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int z = zc[m] + dz, y = yc[m] + dy, xx = xc[m] + dx;
        const bool ok = k < K && inb[m] && (unsigned)z < (unsigned)a.D && (unsigned)y < (unsigned)a.H &&
                        (unsigned)xx < (unsigned)a.W;
        const long long nb = vb[m] + (long long)dz * HW + dy * a.W + dx;
        xb[m][j] = ok ? a.x[nb * a.Cin + c] : (bf16)0.f;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t)
        wa[t][j] = k < K ? a.w[(long long)(n0 + 32 * t + r) * K + k] : (bf16)0.f;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int m = 0; m < 2; ++m) acc[m][t] = mfma32(wa[t], xb[m], acc[m][t]);
  }
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    if (!inb[m]) continue;
    bf16* yp = a.y + vb[m] * a.Cout + n0 + 4 * h;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = to_bf16(acc[m][t][4 * q + j]);
        *(bf16x4*)(yp + 32 * t + 8 * q) = o;
      }
  }
}

// Weight gradient, split over voxels: part[s, w, tap, n, c] = sum over this workgroup's voxels p (rows of
// wave w) of dy[p, n] * x[p + off(tap), c]. Both operands have the voxel as the reduction index, which is the
// slow axis of a channels-last tensor, so 128-voxel tiles of dy and of the tap-shifted x are staged row-major
// in LDS (192-B rows: conflict-free for the transposed reads) and read back as MFMA fragments with
// ds_read_b64_tr_b16. Grid x = tap (fastest: the 27 workgroups of one voxel range share it in L2),
// y = voxel split, z = (n tile, c tile). Plain stores of per-wave partials (no atomics, deterministic); the
// caller sums them.
constexpr int WG_ROWS = 128;
// LDS row stride (elements) of a 32*M-channel tile: 64 / 160 / 192-B rows keep the four rows of a transposed
// read in disjoint bank windows (a 128-B stride would pair them up)
__host__ __device__ constexpr int wg_ld(int M) { return M == 1 ? 32 : (M == 2 ? 80 : 96); }

struct WgradArgs {
  const bf16* x;    // (B, D, H, W, Cin)
  const bf16* dy;   // (B, D, H, W, Cout)
  float* part;      // (nsplit * 4, T, Cout, Cin)
  long long V, Lv;
  int D, H, W, Cin, Cout, KD;
};

template <int MT, int NT>
__global__ __launch_bounds__(256) void conv3_wgrad_kernel(WgradArgs a) {
  // two LDS buffers: tile j+1 is loaded into registers during tile j's MFMAs and stored to the other buffer
  constexpr int LDY = wg_ld(MT), LDX = wg_ld(NT);
  __shared__ __attribute__((aligned(16))) bf16 sdy[2][WG_ROWS * LDY];
  __shared__ __attribute__((aligned(16))) bf16 sx[2][WG_ROWS * LDX];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int tap = blockIdx.x, split = blockIdx.y;
  const int nct = a.Cin / (32 * NT);
  const int n0 = (blockIdx.z / nct) * 32 * MT, c0 = (blockIdx.z % nct) * 32 * NT;
  const int T = a.KD * 9;
  const int dz = (a.KD == 3 ? tap / 9 : 1) - 1, dyy = (tap / 3) % 3 - 1, dx = tap % 3 - 1;
  const int HW = a.H * a.W;
  const long long DHW = (long long)a.D * HW;
  const long long off = (long long)dz * HW + dyy * a.W + dx;
  const long long vs = (long long)split * a.Lv, ve = min(a.V, vs + a.Lv);

  f32x16 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][n][i] = 0.f;

  u32x4 rdy[2 * MT], rx[2 * NT];
  auto load = [&](long long v0) {
#pragma unroll
    for (int i = 0; i < 2 * MT; ++i) {   // dy tile: 128 rows x 4*MT 16-B chunks
      const int c = tid + 256 * i, row = c / (4 * MT), ch = c % (4 * MT);
      const long long v = v0 + row;
      rdy[i] = u32x4{0u, 0u, 0u, 0u};
      if (v < ve) rdy[i] = *(const u32x4*)(a.dy + v * a.Cout + n0 + 8 * ch);
    }
#pragma unroll
    for (int i = 0; i < 2 * NT; ++i) {   // shifted x tile: row p holds x[p + off] (zero outside the volume)
      const int c = tid + 256 * i, row = c / (4 * NT), ch = c % (4 * NT);
      const long long v = v0 + row;
      rx[i] = u32x4{0u, 0u, 0u, 0u};
      if (v < ve) {
        int rem = (int)(v % DHW);
        const int z = rem / HW;
        rem -= z * HW;
        const int y = rem / a.W, xx = rem - y * a.W;
        if ((unsigned)(z + dz) < (unsigned)a.D && (unsigned)(y + dyy) < (unsigned)a.H &&
            (unsigned)(xx + dx) < (unsigned)a.W)
          rx[i] = *(const u32x4*)(a.x + (v + off) * a.Cin + c0 + 8 * ch);
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2 * MT; ++i) {
      const int c = tid + 256 * i, row = c / (4 * MT), ch = c % (4 * MT);
      *(u32x4*)(&sdy[buf][row * LDY + 8 * ch]) = rdy[i];
    }
#pragma unroll
    for (int i = 0; i < 2 * NT; ++i) {
      const int c = tid + 256 * i, row = c / (4 * NT), ch = c % (4 * NT);
      *(u32x4*)(&sx[buf][row * LDX + 8 * ch]) = rx[i];
    }
  };

  load(vs);
  store(0);
  __syncthreads();
  int buf = 0;
  for (long long v0 = vs; v0 < ve; v0 += WG_ROWS) {
    const bool more = v0 + WG_ROWS < ve;
    if (more) load(v0 + WG_ROWS);
    const bf16* tdy = sdy[buf];
    const bf16* tx = sx[buf];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fa[MT], fb[NT];
#pragma unroll
      for (int m = 0; m < MT; ++m)
        fa[m] = s ? frag_tr<1>(tdy, LDY, 32 * wave, 32 * m, lane) : frag_tr<0>(tdy, LDY, 32 * wave, 32 * m, lane);
#pragma unroll
      for (int n = 0; n < NT; ++n)
        fb[n] = s ? frag_tr<1>(tx, LDX, 32 * wave, 32 * n, lane) : frag_tr<0>(tx, LDX, 32 * wave, 32 * n, lane);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[m][n] = mfma32(fa[m], fb[n], acc[m][n]);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // acc[m][n] reg i: n-index n0 + 32m + (i&3) + 8(i>>2) + 4h, c-index c0 + 32n + (lane&31)
  const int h = lane >> 5;
  float* out = a.part + ((long long)(split * 4 + wave) * T + tap) * a.Cout * a.Cin;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = n0 + 32 * m + (i & 3) + 8 * (i >> 2) + 4 * h;
        out[(long long)row * a.Cin + c0 + 32 * n + (lane & 31)] = acc[m][n][i];
      }
}

// Three-tap weight gradient: one workgroup computes the three dx taps of a (dz, dy) tap group for a 32*MT x 32
// (n, c) tile. Voxels are enumerated in a "gapped" row space, one zero row after every W-voxel line, so that the
// x neighbour of dy row g for tap dx is simply staged row g + dx: it falls on a zero gap row exactly when x + dx
// leaves [0, W). The dy tile is staged once per step and its fragments feed all three taps; the x tile is 130
// rows (1-row halo each side). Staging per tap drops 3x versus conv3_wgrad_kernel.
template <int MT>
__global__ __launch_bounds__(256) void conv3_wgrad3_kernel(WgradArgs a) {
  constexpr int LDY = wg_ld(MT), LDX = wg_ld(1), XR = WG_ROWS + 2;
  __shared__ __attribute__((aligned(16))) bf16 sdy[2][WG_ROWS * LDY];
  __shared__ __attribute__((aligned(16))) bf16 sx[2][(XR + 6) * LDX];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int grp = blockIdx.x, split = blockIdx.y;
  const int nct = a.Cin / 32;
  const int n0 = (blockIdx.z / nct) * 32 * MT, c0 = (blockIdx.z % nct) * 32;
  const int T = a.KD * 9;
  const int dz = (a.KD == 3 ? grp / 3 : 1) - 1, dyy = grp % 3 - 1;
  const int HW = a.H * a.W, W1 = a.W + 1;
  const long long lines = a.V / a.W, R = lines * W1;
  const long long shift = (long long)dz * HW + (long long)dyy * a.W;
  const long long gs = (long long)split * a.Lv, ge = min(R, gs + a.Lv);

  f32x16 acc[3][MT];
#pragma unroll
  for (int d = 0; d < 3; ++d)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[d][m][i] = 0.f;

  u32x4 rdy[2 * MT], rx[3];
  // Row -> (line, x) without per-element 64-bit division: one (uniform) division per step for the tile's first
  // gapped row, then a 32-bit quotient by W + 1 and a carry of (y, z) per element.
  auto load = [&](long long g0) {
    const long long gb = g0 - 1;                        // x tile row 0
    long long lb = (gb >= 0 ? gb : gb - W1 + 1) / W1;   // floor division (gb may be -1)
    const int xb = (int)(gb - lb * W1);
    const int yb = (int)(((lb % a.H) + a.H) % a.H);
    const int zb = (int)((((lb >= 0 ? lb : lb - a.H + 1) / a.H) % a.D + a.D) % a.D);
#pragma unroll
    for (int i = 0; i < 2 * MT; ++i) {   // dy rows g0 .. g0 + 127 (zero on gaps / past the split)
      const int c = tid + 256 * i, row = c / (4 * MT), ch = c % (4 * MT);
      rdy[i] = u32x4{0u, 0u, 0u, 0u};
      if (g0 + row < ge) {
        const int t = xb + 1 + row, q = t / W1, xx = t - q * W1;
        if (xx < a.W) rdy[i] = *(const u32x4*)(a.dy + ((lb + q) * a.W + xx) * a.Cout + n0 + 8 * ch);
      }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {        // x rows g0 - 1 .. g0 + 128, shifted by (dz, dy); zero on gaps / outside
      const int c = tid + 256 * i, row = c >> 2, ch = c & 3;
      rx[i] = u32x4{0u, 0u, 0u, 0u};
      if (row < XR && gb + row >= 0 && gb + row < R) {
        const int t = xb + row, q = t / W1, xx = t - q * W1;
        int yl = yb + q, zl = zb;
        while (yl >= a.H) { yl -= a.H; if (++zl == a.D) zl = 0; }
        if (xx < a.W && (unsigned)(zl + dz) < (unsigned)a.D && (unsigned)(yl + dyy) < (unsigned)a.H)
          rx[i] = *(const u32x4*)(a.x + ((lb + q) * a.W + xx + shift) * a.Cin + c0 + 8 * ch);
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2 * MT; ++i) {
      const int c = tid + 256 * i, row = c / (4 * MT), ch = c % (4 * MT);
      *(u32x4*)(&sdy[buf][row * LDY + 8 * ch]) = rdy[i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int c = tid + 256 * i, row = c >> 2, ch = c & 3;
      if (row < XR) *(u32x4*)(&sx[buf][row * LDX + 8 * ch]) = rx[i];
    }
  };

  load(gs);
  store(0);
  __syncthreads();
  int buf = 0;
  for (long long g0 = gs; g0 < ge; g0 += WG_ROWS) {
    const bool more = g0 + WG_ROWS < ge;
    if (more) load(g0 + WG_ROWS);
    LCI_WGRAD_SCHED();
    const bf16* tdy = sdy[buf];
    const bf16* tx = sx[buf];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fa[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m)
        fa[m] = s ? frag_tr<1>(tdy, LDY, 32 * wave, 32 * m, lane) : frag_tr<0>(tdy, LDY, 32 * wave, 32 * m, lane);
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const bf16x8 fb = s ? frag_tr<1>(tx, LDX, 32 * wave + d, 0, lane) : frag_tr<0>(tx, LDX, 32 * wave + d, 0, lane);
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[d][m] = mfma32(fa[m], fb, acc[d][m]);
      }
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  const int h = lane >> 5;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float* out = a.part + ((long long)(split * 4 + wave) * T + grp * 3 + d) * a.Cout * a.Cin;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = n0 + 32 * m + (i & 3) + 8 * (i >> 2) + 4 * h;
        out[(long long)row * a.Cin + c0 + (lane & 31)] = acc[d][m][i];
      }
  }
}

template <int MT, int NT>
static int launch_wgrad(const WgradArgs& a, int nsplit, hipStream_t st) {
  dim3 grid(a.KD * 9, nsplit, (a.Cout / (32 * MT)) * (a.Cin / (32 * NT)));
  hipLaunchKernelGGL((conv3_wgrad_kernel<MT, NT>), grid, dim3(256), 0, st, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

static int tile3(int c) { return (c / 32) % 3 == 0 ? 3 : ((c / 32) % 2 == 0 ? 2 : 1); }

static bool lci_conv_lds() {   // LCI_CONV_LDS=0: the direct-load kernel (A/B)
  static const bool on = !getenv("LCI_CONV_LDS") || atoi(getenv("LCI_CONV_LDS")) != 0;
  return on;
}

template <int NT>
static int launch(const ConvArgs& a, hipStream_t st) {
  constexpr int MV = NT <= 2 ? 4 : LCI_CONV_MV_WIDE;   // narrow outputs: more voxels per wave
  if (a.Cin % 32 == 0 && lci_conv_lds()) {
    constexpr int ML = NT == 4 ? 2 : 4;
    dim3 grid((unsigned)((a.V + 128 * ML - 1) / (128 * ML)), a.Cout / (32 * NT));
    hipLaunchKernelGGL((conv3_fwd_lds_kernel<NT, ML>), grid, dim3(256), 0, st, a);
  } else if (a.Cin % 16 == 0) {
    dim3 grid((unsigned)((a.V + 128 * MV - 1) / (128 * MV)), a.Cout / (32 * NT));
    hipLaunchKernelGGL((conv3_fwd_kernel<NT, MV>), grid, dim3(256), 0, st, a);
  } else {
    dim3 grid((unsigned)((a.V + 255) / 256), a.Cout / (32 * NT));
    hipLaunchKernelGGL(conv3_fwd_generic_kernel<NT>, grid, dim3(256), 0, st, a);
  }
  LCI_LAUNCH_CHECK();
  return 0;
}

}  // namespace lci

using namespace lci;

extern "C" int lci_conv3_fwd(const void* x, const void* w, void* y, int B, int D, int H, int W, int Cin, int Cout,
                             int KD, void* stream) {
  LCI_CHECK(B > 0 && D > 0 && H > 0 && W > 0 && Cin > 0, "conv3: bad shape");
  LCI_CHECK(KD == 3 || (KD == 1 && D == 1), "conv3: KD must be 3, or 1 with D == 1 (2-D)");
  LCI_CHECK(Cout % 32 == 0, "conv3: Cout (%d) must be a multiple of 32", Cout);
  LCI_CHECK(((uintptr_t)x & 15) == 0 && ((uintptr_t)w & 15) == 0 && ((uintptr_t)y & 7) == 0,
            "conv3: misaligned pointers");
  ConvArgs a;
  a.x = (const bf16*)x; a.w = (const bf16*)w; a.y = (bf16*)y;
  a.V = (long long)B * D * H * W;
  a.D = D; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.KD = KD;
  LCI_CHECK((a.V + 255) / 256 < (1LL << 31), "conv3: volume too large");
  hipStream_t st = (hipStream_t)stream;
  const int nb = Cout / 32;
  if (nb % 3 == 0) return launch<3>(a, st);
  if (nb % 4 == 0) return launch<4>(a, st);
  if (nb % 2 == 0) return launch<2>(a, st);
  return launch<1>(a, st);
}

// Voxel splits: up to 32768 voxels per workgroup, fewer (>= 1024) when that leaves under ~2048 workgroups
// (small 2-D volumes, few channel tiles), so the grid still fills the 256 CUs.
extern "C" long long lci_conv3_wgrad_splits(long long V, int Cin, int Cout, int KD) {
  const long long tiles = (long long)KD * 9 * (Cout / (32 * tile3(Cout))) * (Cin / (32 * tile3(Cin)));
  long long lv = 32768;
  while (lv > 1024 && ((V + lv - 1) / lv) * tiles < 2048) lv >>= 1;
  return (V + lv - 1) / lv;
}

extern "C" int lci_conv3_wgrad(const void* x, const void* dy, float* part, int B, int D, int H, int W, int Cin,
                               int Cout, int KD, void* stream) {
  LCI_CHECK(B > 0 && D > 0 && H > 0 && W > 0, "conv3_wgrad: bad shape");
  LCI_CHECK(KD == 3 || (KD == 1 && D == 1), "conv3_wgrad: KD must be 3, or 1 with D == 1 (2-D)");
  LCI_CHECK(Cout % 32 == 0 && Cin % 32 == 0, "conv3_wgrad: Cin (%d) and Cout (%d) must be multiples of 32", Cin,
            Cout);
  LCI_CHECK(((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)part & 3) == 0,
            "conv3_wgrad: misaligned pointers");
  WgradArgs a;
  a.x = (const bf16*)x; a.dy = (const bf16*)dy; a.part = part;
  a.V = (long long)B * D * H * W;
  a.D = D; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.KD = KD;
  const long long ns = lci_conv3_wgrad_splits(a.V, Cin, Cout, KD);
  a.Lv = (a.V + ns - 1) / ns;
  LCI_CHECK(ns < 65536, "conv3_wgrad: volume too large");
  hipStream_t st = (hipStream_t)stream;
  static const bool wg3 = !getenv("LCI_WGRAD3") || atoi(getenv("LCI_WGRAD3")) != 0;   // A/B switch
  if (wg3) {
    const long long R = (a.V / W) * (W + 1);
    a.Lv = (R + ns - 1) / ns;
    static const int mt_env = getenv("LCI_WGRAD3_MT") ? atoi(getenv("LCI_WGRAD3_MT")) : 0;   // A/B override
    const int mt = (mt_env > 0 && (Cout / 32) % mt_env == 0) ? mt_env : tile3(Cout);
    dim3 grid(KD * 3, (unsigned)ns, (Cout / (32 * mt)) * (Cin / 32));
    if (mt == 3) hipLaunchKernelGGL(conv3_wgrad3_kernel<3>, grid, dim3(256), 0, st, a);
    else if (mt == 2) hipLaunchKernelGGL(conv3_wgrad3_kernel<2>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(conv3_wgrad3_kernel<1>, grid, dim3(256), 0, st, a);
    LCI_LAUNCH_CHECK();
    return 0;
  }
  const int mt = tile3(Cout), nt = tile3(Cin);
#define LCI_WG(M, N) if (mt == M && nt == N) return launch_wgrad<M, N>(a, (int)ns, st);
  LCI_WG(3, 3) LCI_WG(3, 2) LCI_WG(3, 1) LCI_WG(2, 3) LCI_WG(2, 2) LCI_WG(2, 1) LCI_WG(1, 3) LCI_WG(1, 2)
  LCI_WG(1, 1)
#undef LCI_WG
  LCI_CHECK(false, "conv3_wgrad: no tile for Cin %d Cout %d", Cin, Cout);
}
