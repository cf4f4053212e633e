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
#include <algorithm>
#include <cstdlib>

#include "common.hpp"

namespace lci {

struct ConvArgs {
  const bf16* x;    // (B, D, H, W, Cin)
  const bf16* w;    // (Cout, T, Cin), T = KD * 9
  bf16* y;          // (B, D, H, W, Cout)
  long long V;      // B * D * H * W
  int D, H, W, Cin, Cout, KD;
  int nvb, ntile, order;   // LDS kernel: voxel blocks, Cout tiles, work order of the 1-D grid (conv_work)
  int nsplit;              // v2 kernel: reduction (slab) splits; > 1: f32 partials to part, summed by conv3_sum_kernel
  float* part;             // (nsplit, V, Cout) f32 when nsplit > 1
};

// (voxel block, Cout tile) of workgroup b for the LDS-staged forward. order 0: voxel block fastest over the plain
// launch order (consecutive voxel blocks land on different XCDs); order 1: every XCD (workgroup b -> XCD b % 8,
// observed round-robin, not relied on for correctness) takes a contiguous range of voxel blocks with the Cout
// tiles fastest, so the workgroups staging the same x rows (and the +-W row shifts of the dy = +-1 taps) share
// that XCD's L2; order 2: contiguous voxel-block ranges per XCD, Cout tile slowest.
__device__ __forceinline__ bool conv_work(const ConvArgs& a, long long& vb, int& nt, int* split = nullptr) {
  long long w = blockIdx.x;
  const long long nb = (long long)a.nvb * a.ntile;
  if (split) {   // split-K launch: the split is the slowest index, plain order inside a split
    *split = (int)(w / nb);
    if (*split >= a.nsplit) return false;
    w -= (long long)*split * nb;
    vb = w % a.nvb;
    nt = (int)(w / a.nvb);
    return true;
  }
  if (a.order != 0) {
    const long long per = (nb + 7) / 8;
    w = (long long)(blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  if (w >= nb) return false;
  if (a.order == 1) { nt = (int)(w % a.ntile); vb = w / a.ntile; }
  else { vb = w % a.nvb; nt = (int)(w / a.nvb); }
  return true;
}

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

// v2 kernel rows: 64 B (no pad) with the 16-byte chunk XORed by (row >> 2) & 3 -- conflict-free for the MFMA fragment
// reads (b128, lane = row, chunk = 2 ks + h) AND for the 16-byte staging writes, which the 80-B rows left at 8 extra
// LDS cycles per write (exhaustive bank check, tools/lds_swizzle_check.py patterns)
constexpr int CLD2 = 32;
__device__ __forceinline__ int cpos2(int row, int chunk) { return row * CLD2 + ((chunk ^ ((row >> 2) & 3)) << 3); }

// LDS-staged forward v2 (Cin % 32 == 0; run at Cout = 32, the DMA kernel below elsewhere): 8 waves x 64 voxels = 512
// voxels x 32*NT output channels per workgroup, and the staging is double-buffered: the next (tap group, 32-channel
// chunk) slab is loaded into registers while this one's MFMAs run, then written to the other LDS buffer -- one
// barrier per slab.
template <int NT>
__global__ __launch_bounds__(512) void conv3_fwd_lds2_kernel(ConvArgs a) {
  constexpr int ML = 2, NWV = 8;
  constexpr int WV = NWV * 32 * ML;            // 512 voxels
  constexpr int XR = WV + 2;                   // staged rows (dx halo)
  constexpr int XBUF = XR * CLD2, WBUF = 3 * 32 * NT * CLD2;
  constexpr int NXS = (XR * 4 + 511) / 512, NWS = (3 * 32 * NT * 4 + 511) / 512;
  extern __shared__ __attribute__((aligned(16))) bf16 smem2[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int r = lane & 31, h = lane >> 5;
  long long vblk;
  int ntl;
  if (!conv_work(a, vblk, ntl)) return;   // grid padding (uniform, before any barrier)
  const long long vg0 = vblk * WV;
  const int n0 = ntl * 32 * NT;
  const int T = a.KD * 9;
  const int HW = a.H * a.W;
  // a wave whose 64 voxels all lie past V (small volumes: V < 512) stages but skips its MFMAs
  const bool live = vg0 + wave * 32 * ML < a.V;
  int zc[ML], yc[ML], xc[ML];
  bool inb[ML];
#pragma unroll
  for (int m = 0; m < ML; ++m) {
    const long long v = vg0 + wave * 32 * ML + 32 * m + r;
    inb[m] = v < a.V;
    const long long vv = inb[m] ? v : 0;
    const long long s = vv / ((long long)a.D * HW);
    int rem = (int)(vv - s * (long long)a.D * HW);
    zc[m] = rem / HW; rem -= zc[m] * HW;
    yc[m] = rem / a.W; xc[m] = rem - yc[m] * a.W;
  }
  f32x16 acc[ML][NT];
#pragma unroll
  for (int m = 0; m < ML; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][t][i] = 0.f;

  const int nchunk = a.Cin / 32, sl0 = 0, sl1 = a.KD * 3 * nchunk;
  u32x4 vxA[NXS], vwA[NWS];
  // x rows through a buffer resource based at the slab's first in-range row (wave-uniform 64-bit arithmetic on the
  // scalar unit): per-lane offsets are 32-bit, rows before the volume give a negative offset and rows past it one
  // beyond num_records, both of which the range check reads as zero (no 64-bit address VALU, no branch per load)
  const int rowb = a.Cin * 2;
  int xoff[NXS], woff[NWS];
#pragma unroll
  for (int i = 0; i < NXS; ++i) {
    const int q = tid + 512 * i, row = q >> 2, ch = q & 3;
    xoff[i] = q < XR * 4 ? row * rowb + 16 * ch : 0x7fffffff;   // past XR: out of range, reads 0 (not stored)
  }
#pragma unroll
  for (int i = 0; i < NWS; ++i) {
    const int q = tid + 512 * i, row = q >> 2, ch = q & 3;   // row = dx * 32NT + n
    const int dxi = row / (32 * NT), n = row - dxi * 32 * NT;
    woff[i] = q < 3 * 32 * NT * 4 ? ((n0 + n) * T + dxi) * rowb + 16 * ch : 0x7fffffff;
  }
  const rsrc_t rw = make_rsrc(a.w, (uint32_t)((long long)a.Cout * T * rowb));
  auto load = [&](int sl, u32x4 (&vx)[NXS], u32x4 (&vw)[NWS]) __attribute__((always_inline)) {
    const int grp = sl / nchunk, c0 = (sl - grp * nchunk) * 32;
    const int dz = (a.KD == 3 ? grp / 3 : 1) - 1, dy = grp % 3 - 1;
    const long long src0 = vg0 + (long long)dz * HW + (long long)dy * a.W - 1;
    const long long b0 = src0 < 0 ? 0 : src0;
    const long long left = (a.V - b0) * rowb;
    const rsrc_t rx = make_rsrc(a.x + b0 * a.Cin + c0, left <= 0 ? 0u : (left > 0x7fffffffLL ? 0x7fffffffu : (uint32_t)left));
    const int sh = (int)(src0 - b0) * rowb;   // <= 0: rows before the volume
#pragma unroll
    for (int i = 0; i < NXS; ++i) vx[i] = bload16(rx, xoff[i] == 0x7fffffff ? xoff[i] : xoff[i] + sh, 0);
    const int wg = (grp * 3 * a.Cin + c0) * 2;
#pragma unroll
    for (int i = 0; i < NWS; ++i) vw[i] = bload16(rw, woff[i] == 0x7fffffff ? woff[i] : woff[i] + wg, 0);
  };
  auto store = [&](int buf, const u32x4 (&vx)[NXS], const u32x4 (&vw)[NWS]) __attribute__((always_inline)) {
    bf16* sX = smem2 + buf * (XBUF + WBUF);
    bf16* sW = sX + XBUF;
#pragma unroll
    for (int i = 0; i < NXS; ++i) {
      const int q = tid + 512 * i, row = q >> 2, ch = q & 3;
      if (q < XR * 4) *(u32x4*)(sX + cpos2(row, ch)) = vx[i];
    }
#pragma unroll
    for (int i = 0; i < NWS; ++i) {
      const int q = tid + 512 * i, row = q >> 2, ch = q & 3;
      if (q < 3 * 32 * NT * 4) *(u32x4*)(sW + cpos2(row, ch)) = vw[i];
    }
  };
  auto compute = [&](int sl, int buf) __attribute__((always_inline)) {
    const int grp = sl / nchunk;
    const int dz = (a.KD == 3 ? grp / 3 : 1) - 1, dy = grp % 3 - 1;
    bool okzy[ML];
#pragma unroll
    for (int m = 0; m < ML; ++m)
      okzy[m] = inb[m] && (unsigned)(zc[m] + dz) < (unsigned)a.D && (unsigned)(yc[m] + dy) < (unsigned)a.H;
    const bf16* sX = smem2 + buf * (XBUF + WBUF);
    const bf16* sW = sX + XBUF;
#pragma unroll
    for (int dxi = 0; dxi < 3 && live; ++dxi) {
      bool ok[ML];
#pragma unroll
      for (int m = 0; m < ML; ++m) ok[m] = okzy[m] && (unsigned)(xc[m] + dxi - 1) < (unsigned)a.W;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 wa[NT], xb[ML];
#pragma unroll
        for (int t = 0; t < NT; ++t)
          wa[t] = *(const bf16x8*)(sW + cpos2(dxi * 32 * NT + 32 * t + r, 2 * ks + h));
#pragma unroll
        for (int m = 0; m < ML; ++m)   // outside the volume: the zero chunk past the buffers (address select)
          xb[m] = *(const bf16x8*)(ok[m] ? sX + cpos2(wave * 32 * ML + 32 * m + r + dxi, 2 * ks + h)
                                         : smem2 + 2 * (XBUF + WBUF));
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int m = 0; m < ML; ++m) acc[m][t] = mfma32(wa[t], xb[m], acc[m][t]);
      }
    }
  };
  load(sl0, vxA, vwA);
  store(0, vxA, vwA);
  if (threadIdx.x == 0) *(u32x4*)(smem2 + 2 * (XBUF + WBUF)) = u32x4{0u, 0u, 0u, 0u};
  int buf = 0;
  __syncthreads();
  for (int sl = sl0; sl < sl1; ++sl) {
    const bool more = sl + 1 < sl1;
    if (more) load(sl + 1, vxA, vwA);
    compute(sl, buf);
    if (more) store(buf ^ 1, vxA, vwA);
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int m = 0; m < ML; ++m) {
    if (!inb[m]) continue;
    const long long v = vg0 + wave * 32 * ML + 32 * m + r;
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

// LDS-DMA staged forward v3 (Cin % 32 == 0; 512 voxels x 32 NT output channels per workgroup, as v2): the (tap
// group, 32-channel chunk) slabs arrive by LDS-DMA (1-KB units of 16 rows x 64 B, the rows' 16-B chunks swizzled by
// (row >> 2) & 3 through the per-lane source offset) into two LDS slots, slab s + 1 issued right after the barrier
// that frees its slot and landing during slab s's MFMAs -- no staging registers (v2 held one or two slabs in VGPRs
// and stored them itself). The freed registers hold a second fragment set: the six (dx tap, k-substep) groups of a
// slab read group g + 1's fragments while group g's MFMAs run.
template <int NT, bool SPLIT>
__global__ __launch_bounds__(512) void conv3_fwd_dma_kernel(ConvArgs a) {
  constexpr int ML = 2, NWV = 8;
  constexpr int WV = NWV * 32 * ML;            // 512 voxels
  constexpr int XU = (WV + 2 + 15) / 16;       // X units (dx halo rows included): 33
  constexpr int WU = 3 * 32 * NT / 16;         // weight units: 3 taps x 32 NT rows
  constexpr int U = XU + WU, UPW = (U + NWV - 1) / NWV;
  constexpr bool SPREAD = NT >= 4;   // next slab's DMA spread over this slab's MFMA groups (see Dma below)
  constexpr int XB = XU * 16 * 64, SLOT = XB + WU * 16 * 64;   // bytes
  extern __shared__ __attribute__((aligned(16))) char smem3[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __builtin_assume(wave >= 0 && wave < NWV);   // readfirstlane drops the range: lets each DMA piece's kind fold
  const int r = lane & 31, h = lane >> 5;
  long long vblk;
  int ntl, split = 0;
  if (!conv_work(a, vblk, ntl, SPLIT ? &split : nullptr)) return;   // grid padding (uniform, before any barrier)
  const long long vg0 = vblk * WV;
  const int n0 = ntl * 32 * NT;
  const int T = a.KD * 9;
  const int HW = a.H * a.W;
  const bool live = vg0 + wave * 32 * ML < a.V;
  int zc[ML], yc[ML], xc[ML];
  bool inb[ML];
#pragma unroll
  for (int m = 0; m < ML; ++m) {
    const long long v = vg0 + wave * 32 * ML + 32 * m + r;
    inb[m] = v < a.V;
    const long long vv = inb[m] ? v : 0;
    const long long s = vv / ((long long)a.D * HW);
    int rem = (int)(vv - s * (long long)a.D * HW);
    zc[m] = rem / HW; rem -= zc[m] * HW;
    yc[m] = rem / a.W; xc[m] = rem - yc[m] * a.W;
  }
  f32x16 acc[ML][NT];
#pragma unroll
  for (int m = 0; m < ML; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[m][t][i] = 0.f;

  const int nchunk = a.Cin / 32, nslab_all = a.KD * 3 * nchunk;
  const int sl0 = SPLIT ? (int)((long long)nslab_all * split / a.nsplit) : 0;
  const int sl1 = SPLIT ? (int)((long long)nslab_all * (split + 1) / a.nsplit) : nslab_all;
  const int rowb = a.Cin * 2;
  const unsigned lds0 = (unsigned)(uintptr_t)(LCI_LDS char*)smem3;
  const rsrc_t rw = make_rsrc(a.w, (uint32_t)((long long)a.Cout * T * rowb));
  // DMA lane mapping inside a unit: row (lane >> 2) of 16, physical chunk lane & 3 <- logical (lane & 3) ^ row bits 2-3
  int lx, lw;
  {
    int l = lane;
    asm volatile("" : "+v"(l));   // opaque: the two lane offsets stay two registers
    const int drow = l >> 2, dch = (l & 3) ^ ((l >> 4) & 3);
    lx = drow * rowb + 16 * dch;
    lw = drow * T * rowb + 16 * dch;
  }
  // slab sl into slot p: X rows [src0, src0 + 16 XU) of channels [c0, c0 + 32) (a resource based at the first
  // in-volume row: rows before it give negative offsets, rows past V offsets beyond num_records -- both read zeros),
  // then the three dx taps' weight rows (n0 + n, tap 3 grp + dx) of the same channels
  // slab sl into slot p: issue_begin() sets up the slab (resources, offsets), piece(d, i) issues this wave's unit i
  // (i < UPW). At NT = 4 the pieces are spread over the six MFMA groups of the slab being computed (an LDS-DMA
  // instruction holds its wave's issue for tens of cycles); the narrower tiles' slabs are too short for that (the
  // late pieces land after the slab ends) and issue them all before their MFMAs.
  struct Dma { rsrc_t rx; int sh, wg; unsigned sb; };
  auto issue_begin = [&](int sl, int p) __attribute__((always_inline)) {
    const int grp = sl / nchunk, c0 = (sl - grp * nchunk) * 32;
    const int dz = (a.KD == 3 ? grp / 3 : 1) - 1, dy = grp % 3 - 1;
    const long long src0 = vg0 + (long long)dz * HW + (long long)dy * a.W - 1;
    const long long b0 = src0 < 0 ? 0 : src0;
    const long long left = (a.V - b0) * rowb;
    Dma d{make_rsrc(a.x + b0 * a.Cin + c0, left <= 0 ? 0u : (left > 0x7fffffffLL ? 0x7fffffffu : (uint32_t)left)),
          (int)(src0 - b0) * rowb,   // <= 0
          (grp * 3 * a.Cin + c0) * 2, lds0 + (unsigned)(p * SLOT)};
    return d;
  };
  auto piece = [&](const Dma& d, int i) __attribute__((always_inline)) {
    const int q = wave + NWV * i;            // wave-uniform
    if (q < XU) {
      dma16_lds(d.rx, lx + 16 * q * rowb + d.sh, 0, d.sb + 1024 * q);
    } else if (q < U) {
      const int q2 = q - XU, dxi = q2 / (2 * NT), nb = 16 * (q2 - dxi * 2 * NT);
      dma16_lds(rw, lw + ((n0 + nb) * T + dxi) * rowb + d.wg, 0, d.sb + XB + 1024 * q2);
    }
  };
  auto issue = [&](int sl, int p) __attribute__((always_inline)) {
    const Dma d = issue_begin(sl, p);
#pragma unroll
    for (int i = 0; i < UPW; ++i) piece(d, i);
  };
  auto compute = [&](int sl, int p, bool iss, const Dma& nd) __attribute__((always_inline)) {
    const int grp = sl / nchunk;
    const int dz = (a.KD == 3 ? grp / 3 : 1) - 1, dy = grp % 3 - 1;
    bool okzy[ML];
#pragma unroll
    for (int m = 0; m < ML; ++m)
      okzy[m] = inb[m] && (unsigned)(zc[m] + dz) < (unsigned)a.D && (unsigned)(yc[m] + dy) < (unsigned)a.H;
    const bf16* sX = (const bf16*)(smem3 + p * SLOT);
    const bf16* sW = (const bf16*)(smem3 + p * SLOT + XB);
    const bf16* szero = (const bf16*)(smem3 + 2 * SLOT);
    bf16x8 wa[2][NT], xb[2][ML];
    auto rd = [&](int g, int s) __attribute__((always_inline)) {
      const int dxi = g >> 1, ks = g & 1;
#pragma unroll
      for (int t = 0; t < NT; ++t) wa[s][t] = *(const bf16x8*)(sW + cpos2(dxi * 32 * NT + 32 * t + r, 2 * ks + h));
#pragma unroll
      for (int m = 0; m < ML; ++m) {
        // a voxel whose tap falls outside the volume reads the 16 zero bytes past the slots (an address select, not
        // a read then a conditional overwrite, which made the compiler drain every pending LDS read first)
        const bool ok = okzy[m] && (unsigned)(xc[m] + dxi - 1) < (unsigned)a.W;
        xb[s][m] = *(const bf16x8*)(ok ? sX + cpos2(wave * 32 * ML + 32 * m + r + dxi, 2 * ks + h) : szero);
      }
    };
    rd(0, 0);
#pragma unroll
    for (int g = 0; g < 6; ++g) {
      if (g + 1 < 6) rd(g + 1, (g + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int m = 0; m < ML; ++m) acc[m][t] = mfma32(wa[g & 1][t], xb[g & 1][m], acc[m][t]);
      __builtin_amdgcn_sched_barrier(0);
      if (SPREAD && iss) {   // the next slab's units i = g, g + 6, ... of this wave
#pragma unroll
        for (int i = g; i < UPW; i += 6) piece(nd, i);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  if (threadIdx.x == 0) *(u32x4*)(smem3 + 2 * SLOT) = u32x4{0u, 0u, 0u, 0u};   // published by the loop's barrier
  issue(sl0, 0);
  int p = 0;
  for (int sl = sl0; sl < sl1; ++sl) {
    wait_vmcnt<0>();                          // this wave's units of slab sl landed
    __builtin_amdgcn_s_waitcnt(0xC07F);       // lgkmcnt(0): this wave's reads of the other slot are done
    __builtin_amdgcn_s_barrier();             // every wave's units landed; the other slot is free
    const bool iss = sl + 1 < sl1;
    const Dma nd = issue_begin(iss ? sl + 1 : sl, p ^ 1);
    if ((!SPREAD || !live) && iss) {   // the next slab's units all at once, before this slab's MFMAs
#pragma unroll
      for (int i = 0; i < UPW; ++i) piece(nd, i);
    }
    if (live) compute(sl, p, iss, nd);
    p ^= 1;
  }
  if (SPLIT) {   // f32 partial of this slab range: 16-B stores of 4 consecutive output channels
#pragma unroll
    for (int m = 0; m < ML; ++m) {
      if (!inb[m]) continue;
      const long long v = vg0 + wave * 32 * ML + 32 * m + r;
      float* pp = a.part + ((long long)split * a.V + v) * a.Cout + n0 + 4 * h;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f32x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = acc[m][t][4 * q + j];
          *(f32x4*)(pp + 32 * t + 8 * q) = o;
        }
    }
    return;
  }
#pragma unroll
  for (int m = 0; m < ML; ++m) {
    if (!inb[m]) continue;
    const long long v = vg0 + wave * 32 * ML + 32 * m + r;
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

// Split-K reduction: y = bf16(sum over splits of part), the splits added in order (deterministic). n8 = V Cout / 8.
__global__ __launch_bounds__(256) void conv3_sum_kernel(const float* __restrict__ part, bf16* __restrict__ y,
                                                        long long n8, int nsplit) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n8; e += stride) {
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < nsplit; ++sp) {
      const float* p = part + (long long)sp * n8 * 8 + e * 8;
      a0 += *(const f32x4*)p;
      a1 += *(const f32x4*)(p + 4);
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) { o[j] = to_bf16(a0[j]); o[4 + j] = to_bf16(a1[j]); }
    *(bf16x8*)(y + e * 8) = o;
  }
}

// Weight packing, one pass from the f32 parameter w (Cout, Cin, T) (T = KD * 9 taps, PyTorch's layout):
//   mode 0 (forward):       out (Cout, T, Cin) bf16 = w[n][c][t]
//   mode 1 (data gradient): out (Cin_pad, T, Cout) bf16 = w[n][c][T - 1 - t], rows c >= Cin zero
// A workgroup transposes one 64-wide block of the contiguous (c, t) or (n, t) rows through LDS, so both the f32
// reads and the bf16 writes are whole rows (autocast cast + permute [+ flip] were 2-3 separate torch copies:
// 1.4 ms per C3 step at the 1536-channel convs of the 4^3 / 8^3 stages).
__global__ __launch_bounds__(256) void conv3_pack_kernel(const float* __restrict__ w, bf16* __restrict__ out,
                                                         int Cout, int Cin, int Cin_pad, int T, int mode) {
  __shared__ float s[64 * 28];
  const int tid = threadIdx.x;
  const int row = blockIdx.x;              // mode 0: n; mode 1: c (< Cin_pad)
  const int j0 = blockIdx.y * 64;          // mode 0: c block; mode 1: n block
  const int J = mode == 0 ? Cin : Cout;    // extent of the blocked index
  for (int e = tid; e < 64 * T; e += 256) {
    const int jj = e / T, t = e - jj * T, j = j0 + jj;
    float v = 0.f;
    if (j < J) {
      if (mode == 0) v = w[((long long)row * Cin + j) * T + t];
      else if (row < Cin) v = w[((long long)j * Cin + row) * T + (T - 1 - t)];
    }
    s[jj * 28 + t] = v;
  }
  __syncthreads();
  const int Jo = mode == 0 ? Cin : Cout;   // contiguous output extent
  for (int e = tid; e < 64 * T; e += 256) {
    const int t = e / 64, jj = e - t * 64, j = j0 + jj;
    if (j < Jo) out[((long long)row * T + t) * Jo + j] = to_bf16(s[jj * 28 + t]);
  }
}

// Transposed-conv (kernel == stride) interleave: the up-sampling GEMM's rows Y (B*D*H*W, taps*C) (tap-major columns)
// moved to the channels-last output grid (B, D*kd, H*kh, W*kw) whose rows have `ld` channels (ld = C, or 2C when the
// result is written straight into the first half of UnetrUpBlock's torch.cat buffer); adjoint: the output-grid rows
// gathered back to Y's layout. One thread per (input voxel, tap, 16-byte chunk): both sides are whole 2C-byte rows.
// grid (ceil(W taps C/8 / 256), min(B D H, 65535)): one input row (b, z, y) per block row (a loop over rows beyond the
// grid), so the per-chunk index math is 32-bit (the grid-stride form's 64-bit divisions cost as much as the copy).
__global__ __launch_bounds__(256) void convup_interleave_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                                long long nrows, int D, int H, int W, int kd, int kh,
                                                                int kw, int C, int ld, int adjoint) {
  const int CC = C >> 3;                       // 16-byte chunks per row
  const int taps = kd * kh * kw;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= W * taps * CC) return;
  const int ch = e % CC, q = e / CC;
  const int t = q % taps, x = q / taps;
  const int a = t / (kh * kw), bb = (t / kw) % kh, c = t % kw;
  for (long long row = blockIdx.y; row < nrows; row += gridDim.y) {
    const int y = (int)(row % H);
    const long long r = row / H;
    const int z = (int)(r % D);
    const long long b = r / D;
    const long long v = row * W + x;           // input voxel (b, z, y, x)
    const long long o = (((b * D + z) * kd + a) * ((long long)H * kh) + (long long)y * kh + bb) * ((long long)W * kw) +
                        (long long)x * kw + c;    // output voxel
    const long long yoff = (v * taps + t) * C + 8 * ch, ooff = o * ld + 8 * ch;
    if (adjoint) *(u32x4*)(dst + yoff) = *(const u32x4*)(src + ooff);
    else *(u32x4*)(dst + ooff) = *(const u32x4*)(src + yoff);
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

// Weight gradient: dW[n, c, tap] = sum_p dy[p, n] x[p + off(tap), c]. Both operands have the voxel as the reduction
// index, which is the slow axis of a channels-last tensor, so 128-voxel tiles of dy and of the shifted x are staged
// row-major in LDS and read back as MFMA fragments with ds_read_b64_tr_b16 (64 / 160 / 192-B rows keep the four
// rows of a transposed read in disjoint bank windows). One workgroup computes the three dx taps of a (dz, dy) tap
// group for a 32*MT x 32 (n, c) tile over one voxel split. Voxels are enumerated in a "gapped" row space, one zero
// row after every W-voxel line, so that the x neighbour of dy row g for tap dx is simply staged row g + dx: it
// falls on a zero gap row exactly when x + dx leaves [0, W), with no per-element masks; the dy fragments feed all
// three taps.
//  * Row indexing is incremental: every thread stages the same rows of each 128-row step, so their (line, x, y, z)
//    advance by one add and one carry per step (the previous version spent about half of its VALU issue on a
//    32-bit division and a carry loop per element and step).
//  * The 4 waves' partial sums are reduced in LDS at the end: one (T, Cout, Cin) partial per voxel split (the
//    caller sums the splits), with splits of up to 2^17 rows -- ~16x less partial-sum traffic than one partial per
//    wave of 2^15-row splits.
// Double-buffered: the next step's rows are loaded into registers during this step's MFMAs. Deterministic.
constexpr int WG_ROWS = 128;
__host__ __device__ constexpr int wg_ld(int M) { return M == 1 ? 32 : (M == 2 ? 80 : 96); }

struct WgradArgs {
  const bf16* x;    // (B, D, H, W, Cin)
  const bf16* dy;   // (B, D, H, W, Cout)
  float* part;      // (nsplit, T, Cout, Cin)
  long long V, Lv;
  int D, H, W, Cin, Cout, KD;
  int ns, nb, order;   // work decode of the 1-D grid (see wgrad_work)
};

// Work item of workgroup b. The dispatcher places workgroup b on XCD b % 8 (observed round-robin; nothing here
// depends on it for correctness), and each XCD has its own 4 MB L2, so `order` 1/2 give every XCD a contiguous
// range of work items: the workgroups resident on one XCD at a time then share rows -- order 1: same (split,
// n tile), all tap groups / c tiles (the dy rows are common); order 2: same (split, tap group, c tile), all n
// tiles (the shifted x rows are common). order 0: tap group fastest over the plain launch order.
struct WgradWork { int grp, split, n0, c0; bool valid; };
__device__ __forceinline__ WgradWork wgrad_work(const WgradArgs& a, int MT) {
  const int b = blockIdx.x;
  const int G = a.KD * 3, NT = a.Cout / (32 * MT), NC = a.Cin / 32;
  long long w = b;
  if (a.order != 0) {
    const long long per = ((long long)a.nb + 7) / 8;
    w = (long long)(b % 8) * per + b / 8;
  }
  WgradWork r{};
  r.valid = w < a.nb;
  if (!r.valid) return r;
  int g, sp, nt, ct;
  if (a.order == 0) {
    g = (int)(w % G); long long q = w / G; sp = (int)(q % a.ns); q /= a.ns; nt = (int)(q / NC); ct = (int)(q % NC);
  } else if (a.order == 1) {
    ct = (int)(w % NC); long long q = w / NC; g = (int)(q % G); q /= G; nt = (int)(q % NT); sp = (int)(q / NT);
  } else {
    nt = (int)(w % NT); long long q = w / NT; ct = (int)(q % NC); q /= NC; g = (int)(q % G); sp = (int)(q / G);
  }
  r.grp = g; r.split = sp; r.n0 = nt * 32 * MT; r.c0 = ct * 32;
  return r;
}

// gapped row G -> line L = floor(G / (W + 1)), position X in the line, and (y, z) of the line
struct GRow {
  int L, X, y, z;
  __device__ __forceinline__ void init(long long G, int W1, int H, int D) {
    long long l = G >= 0 ? G / W1 : -((-G + W1 - 1) / W1);
    L = (int)l;
    X = (int)(G - l * W1);
    long long yy = l % H;
    if (yy < 0) yy += H;
    y = (int)yy;
    long long zq = l >= 0 ? l / H : -((-l + H - 1) / H);
    long long zz = zq % D;
    if (zz < 0) zz += D;
    z = (int)zz;
  }
  // G += 128: q128 = 128 / W1, r128 = 128 % W1
  __device__ __forceinline__ void advance(int q128, int r128, int W1, int H, int D) {
    X += r128;
    int dl = q128;
    if (X >= W1) { X -= W1; ++dl; }
    L += dl;
    y += dl;
    while (y >= H) { y -= H; if (++z == D) z = 0; }
  }
};

template <int MT>
__global__ __launch_bounds__(256) void conv3_wgrad4_kernel(WgradArgs a) {
  constexpr int LDY = wg_ld(MT), LDX = wg_ld(1), XR = WG_ROWS + 2;
  constexpr int NDY = 2 * MT, NXS = 3;
  __shared__ __attribute__((aligned(16))) bf16 sdy[2][WG_ROWS * LDY];
  __shared__ __attribute__((aligned(16))) bf16 sx[2][(XR + 6) * LDX];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const WgradWork wk = wgrad_work(a, MT);
  if (!wk.valid) return;   // padding of the 1-D grid to a multiple of 8 (uniform per workgroup, before any barrier)
  const int grp = wk.grp, split = wk.split, n0 = wk.n0, c0 = wk.c0;
  const int T = a.KD * 9;
  const int dz = (a.KD == 3 ? grp / 3 : 1) - 1, dyy = grp % 3 - 1;
  const int HW = a.H * a.W, W1 = a.W + 1;
  const long long lines = a.V / a.W, R = lines * W1;
  const long long shift = (long long)dz * HW + (long long)dyy * a.W;
  const long long gs = (long long)split * a.Lv, ge = min(R, gs + a.Lv);
  const int q128 = WG_ROWS / W1, r128 = WG_ROWS % W1;

  f32x16 acc[3][MT];
#pragma unroll
  for (int d = 0; d < 3; ++d)
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[d][m][i] = 0.f;

  // this thread's staging slots: fixed rows of every step
  int rdy[NDY], cdy[NDY], rxs[NXS], cxs[NXS];
  GRow gdy[NDY], gx[NXS];
#pragma unroll
  for (int i = 0; i < NDY; ++i) {
    const int c = tid + 256 * i;
    rdy[i] = c / (4 * MT); cdy[i] = c % (4 * MT);
    gdy[i].init(gs + rdy[i], W1, a.H, a.D);
  }
#pragma unroll
  for (int i = 0; i < NXS; ++i) {
    const int c = tid + 256 * i;
    rxs[i] = c >> 2; cxs[i] = c & 3;
    gx[i].init(gs - 1 + rxs[i], W1, a.H, a.D);
  }
  u32x4 vdy[NDY], vx[NXS];
  auto load = [&](long long g0) {
#pragma unroll
    for (int i = 0; i < NDY; ++i) {
      vdy[i] = u32x4{0u, 0u, 0u, 0u};
      if (g0 + rdy[i] < ge && gdy[i].X < a.W)
        vdy[i] = *(const u32x4*)(a.dy + ((long long)gdy[i].L * a.W + gdy[i].X) * a.Cout + n0 + 8 * cdy[i]);
    }
#pragma unroll
    for (int i = 0; i < NXS; ++i) {
      vx[i] = u32x4{0u, 0u, 0u, 0u};
      const long long G = g0 - 1 + rxs[i];
      if (rxs[i] < XR && G >= 0 && G < R && gx[i].X < a.W && (unsigned)(gx[i].z + dz) < (unsigned)a.D &&
          (unsigned)(gx[i].y + dyy) < (unsigned)a.H)
        vx[i] = *(const u32x4*)(a.x + ((long long)gx[i].L * a.W + gx[i].X + shift) * a.Cin + c0 + 8 * cxs[i]);
    }
#pragma unroll
    for (int i = 0; i < NDY; ++i) gdy[i].advance(q128, r128, W1, a.H, a.D);
#pragma unroll
    for (int i = 0; i < NXS; ++i) gx[i].advance(q128, r128, W1, a.H, a.D);
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NDY; ++i) *(u32x4*)(&sdy[buf][rdy[i] * LDY + 8 * cdy[i]]) = vdy[i];
#pragma unroll
    for (int i = 0; i < NXS; ++i)
      if (rxs[i] < XR) *(u32x4*)(&sx[buf][rxs[i] * LDX + 8 * cxs[i]]) = vx[i];
  };

  load(gs);
  store(0);
  __syncthreads();
  int buf = 0;
  for (long long g0 = gs; g0 < ge; g0 += WG_ROWS) {
    const bool more = g0 + WG_ROWS < ge;
    if (more) load(g0 + WG_ROWS);
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
  // reduce the 4 waves' partials through LDS (the staging buffers are free now), one tap at a time
  float* red = (float*)&sdy[0][0];   // [wave][m][i][lane]: 4 * 16 MT * 64 floats <= sizeof(sdy)
  const int h = lane >> 5;
  (void)h;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) red[((wave * MT + m) * 16 + i) * 64 + lane] = acc[d][m][i];
    __syncthreads();
    float* out = a.part + ((long long)split * T + grp * 3 + d) * a.Cout * a.Cin;
    for (int idx = tid; idx < MT * 16 * 64; idx += 256) {
      const int l = idx & 63, i = (idx >> 6) & 15, m = idx >> 10;
      const float v = (red[((0 * MT + m) * 16 + i) * 64 + l] + red[((1 * MT + m) * 16 + i) * 64 + l]) +
                      (red[((2 * MT + m) * 16 + i) * 64 + l] + red[((3 * MT + m) * 16 + i) * 64 + l]);
      const int row = n0 + 32 * m + (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
      out[(long long)row * a.Cin + c0 + (l & 31)] = v;
    }
    __syncthreads();
  }
}


// Weight gradient v5: the workgroup output tile grows to 32*MB*WN output x 32*WC input channels (x 3 dx taps),
// split among WN*WC waves (wave (wn, wc) owns n blocks MB wn .. MB wn + MB - 1 and c block wc over ALL 128 rows of
// a step), so every staged dy / x byte feeds many more MFMAs than in v4 (at (MB, WN, WC) = (2, 2, 4): 193 FLOP
// per staged byte vs 64) and no cross-wave reduction is needed. The staged tiles are kept as separate 32-channel LDS blocks with 64-B
// rows (conflict-free transposed reads), double-buffered with the same incremental gapped-row indexing as v4.
template <int MB, int WN, int WC>
__global__ __launch_bounds__(64 * WN * WC) void conv3_wgrad5_kernel(WgradArgs a) {
  constexpr int NTH = 64 * WN * WC;
  constexpr int XR = WG_ROWS + 2;
  constexpr int NB_DY = MB * WN, NB_X = WC;                     // 32-channel blocks staged per step
  // elements per LDS block, each padded by 64 B: the 16-B staging stores of one 8-lane group hit two adjacent blocks,
  // which would otherwise start on the same bank (4 KB / 8.5 KB multiples)
  constexpr int DYBLK = WG_ROWS * 32 + 32, XBLK = (XR + 6) * 32 + 32;
  constexpr int BUF = NB_DY * DYBLK + NB_X * XBLK;
  constexpr int NDY = (WG_ROWS * NB_DY * 4 + NTH - 1) / NTH;    // 16-B chunks per thread per step
  constexpr int NXS = (XR * NB_X * 4 + NTH - 1) / NTH;
  extern __shared__ __attribute__((aligned(16))) bf16 wsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int wn = wave / WC, wc = wave % WC;
  // work decode (XCD-contiguous, as wgrad_work order 1, for a 64WN x 32WC tile)
  const int G = a.KD * 3, NT = a.Cout / (32 * MB * WN), NC = a.Cin / (32 * WC);
  long long w = blockIdx.x;
  {
    const long long per = ((long long)a.nb + 7) / 8;
    w = (long long)(blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  if (w >= a.nb) return;
  const int ct = (int)(w % NC);
  long long q = w / NC;
  const int grp = (int)(q % G);
  q /= G;
  const int nt = (int)(q % NT), split = (int)(q / NT);
  const int n0 = nt * 32 * MB * WN, c0 = ct * 32 * WC;
  const int T = a.KD * 9;
  const int dz = (a.KD == 3 ? grp / 3 : 1) - 1, dyy = grp % 3 - 1;
  const int HW = a.H * a.W, W1 = a.W + 1;
  const long long lines = a.V / a.W, R = lines * W1;
  const long long shift = (long long)dz * HW + (long long)dyy * a.W;
  const long long gs = (long long)split * a.Lv, ge = min(R, gs + a.Lv);
  const int q128 = WG_ROWS / W1, r128 = WG_ROWS % W1;

  f32x16 acc[3][MB];
#pragma unroll
  for (int d = 0; d < 3; ++d)
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[d][m][i] = 0.f;

  int rdy[NDY], cdy[NDY], rxs[NXS], cxs[NXS];
  GRow gdy[NDY], gx[NXS];
#pragma unroll
  for (int i = 0; i < NDY; ++i) {
    const int c = tid + NTH * i;
    rdy[i] = c / (NB_DY * 4); cdy[i] = c % (NB_DY * 4);   // row, 16-B chunk of the 64WN-channel dy row
    gdy[i].init(gs + min(rdy[i], WG_ROWS - 1), W1, a.H, a.D);
  }
#pragma unroll
  for (int i = 0; i < NXS; ++i) {
    const int c = tid + NTH * i;
    rxs[i] = c / (NB_X * 4); cxs[i] = c % (NB_X * 4);
    gx[i].init(gs - 1 + min(rxs[i], XR - 1), W1, a.H, a.D);
  }
  u32x4 vdy[NDY], vx[NXS];
  auto load = [&](long long g0) {
#pragma unroll
    for (int i = 0; i < NDY; ++i) {
      vdy[i] = u32x4{0u, 0u, 0u, 0u};
      if (rdy[i] < WG_ROWS && g0 + rdy[i] < ge && gdy[i].X < a.W)
        vdy[i] = *(const u32x4*)(a.dy + ((long long)gdy[i].L * a.W + gdy[i].X) * a.Cout + n0 + 8 * cdy[i]);
    }
#pragma unroll
    for (int i = 0; i < NXS; ++i) {
      vx[i] = u32x4{0u, 0u, 0u, 0u};
      const long long Gr = g0 - 1 + rxs[i];
      if (rxs[i] < XR && Gr >= 0 && Gr < R && gx[i].X < a.W && (unsigned)(gx[i].z + dz) < (unsigned)a.D &&
          (unsigned)(gx[i].y + dyy) < (unsigned)a.H)
        vx[i] = *(const u32x4*)(a.x + ((long long)gx[i].L * a.W + gx[i].X + shift) * a.Cin + c0 + 8 * cxs[i]);
    }
#pragma unroll
    for (int i = 0; i < NDY; ++i) gdy[i].advance(q128, r128, W1, a.H, a.D);
#pragma unroll
    for (int i = 0; i < NXS; ++i) gx[i].advance(q128, r128, W1, a.H, a.D);
  };
  auto store = [&](int buf) {
    bf16* base = wsm + buf * BUF;
#pragma unroll
    for (int i = 0; i < NDY; ++i)
      if (rdy[i] < WG_ROWS)
        *(u32x4*)(base + (cdy[i] >> 2) * DYBLK + rdy[i] * 32 + 8 * (cdy[i] & 3)) = vdy[i];
#pragma unroll
    for (int i = 0; i < NXS; ++i)
      if (rxs[i] < XR)
        *(u32x4*)(base + NB_DY * DYBLK + (cxs[i] >> 2) * XBLK + rxs[i] * 32 + 8 * (cxs[i] & 3)) = vx[i];
  };

  load(gs);
  store(0);
  __syncthreads();
  int buf = 0;
  for (long long g0 = gs; g0 < ge; g0 += WG_ROWS) {
    const bool more = g0 + WG_ROWS < ge;
    if (more) load(g0 + WG_ROWS);
    const bf16* tdy0 = wsm + buf * BUF + (MB * wn) * DYBLK;
    const bf16* tx = wsm + buf * BUF + NB_DY * DYBLK + wc * XBLK;
#pragma unroll
    for (int r0 = 0; r0 < WG_ROWS; r0 += 32) {
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        if constexpr (MB == 2) {
          const bf16* tdy1 = tdy0 + DYBLK;
          const bf16x8 fa0 = sub ? frag_tr<1>(tdy0, 32, r0, 0, lane) : frag_tr<0>(tdy0, 32, r0, 0, lane);
          const bf16x8 fa1 = sub ? frag_tr<1>(tdy1, 32, r0, 0, lane) : frag_tr<0>(tdy1, 32, r0, 0, lane);
#pragma unroll
          for (int d = 0; d < 3; ++d) {
            const bf16x8 fb = sub ? frag_tr<1>(tx, 32, r0 + d, 0, lane) : frag_tr<0>(tx, 32, r0 + d, 0, lane);
            acc[d][0] = mfma32(fa0, fb, acc[d][0]);
            acc[d][MB - 1] = mfma32(fa1, fb, acc[d][MB - 1]);
          }
        } else {
          const bf16x8 fa0 = sub ? frag_tr<1>(tdy0, 32, r0, 0, lane) : frag_tr<0>(tdy0, 32, r0, 0, lane);
#pragma unroll
          for (int d = 0; d < 3; ++d) {
            const bf16x8 fb = sub ? frag_tr<1>(tx, 32, r0 + d, 0, lane) : frag_tr<0>(tx, 32, r0 + d, 0, lane);
            acc[d][0] = mfma32(fa0, fb, acc[d][0]);
          }
        }
      }
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // acc[d][m] reg i: n = n0 + 32 (MB wn + m) + (i&3) + 8(i>>2) + 4h, c = c0 + 32 wc + (lane & 31)
  const int h = lane >> 5;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float* out = a.part + ((long long)split * T + grp * 3 + d) * a.Cout * a.Cin;
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = n0 + 32 * (MB * wn + m) + (i & 3) + 8 * (i >> 2) + 4 * h;
        out[(long long)row * a.Cin + c0 + 32 * wc + (lane & 31)] = acc[d][m][i];
      }
  }
}

template <int MB, int WN, int WC>
constexpr size_t wgrad5_lds() {   // two buffers of the kernel's padded dy / x blocks
  return (size_t)2 * (MB * WN * (WG_ROWS * 32 + 32) + WC * ((WG_ROWS + 8) * 32 + 32)) * sizeof(bf16);
}

template <int MB, int WN, int WC>
static int launch_wgrad5(WgradArgs a, hipStream_t st) {
  const size_t sh = wgrad5_lds<MB, WN, WC>();
  const long long nb = (long long)a.KD * 3 * a.ns * (a.Cout / (32 * MB * WN)) * (a.Cin / (32 * WC));
  LCI_CHECK(nb < (1LL << 30), "conv3_wgrad: too many workgroups");
  a.nb = (int)nb;
  (void)hipFuncSetAttribute((const void*)conv3_wgrad5_kernel<MB, WN, WC>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL((conv3_wgrad5_kernel<MB, WN, WC>), dim3((unsigned)((nb + 7) / 8 * 8)), dim3(64 * WN * WC), sh,
                     st, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

// Weight gradient v6 (round 6): v5's (1, 3, WC) tiles (the Swin channel counts: C3) with the staging done by LDS-DMA
// into three LDS buffers. Step k+2's rows land while step k computes, so two steps of rows are in flight per
// workgroup where v5 had one (v5 stalls on each step's register-staged loads: MFMA busy 0.31 at C3,
// profiles/r06_pmc.txt), and no VGPRs hold staged rows. A 1-KB DMA unit is 16 rows x 64 B of one 32-channel block
// (lane l: row l >> 2, 16-B chunk l & 3); a step is 24 dy units (3 blocks x 128 rows) then 9 WC x units (WC blocks x
// 144 rows: the 130 a step reads, rounded up to whole units), unit u at LDS byte 1024 u of its buffer. Rows that do not
// exist (gap rows, taps outside the volume, rows past the split) are lanes with an out-of-range offset: the DMA writes
// them as zeros. Every wave issues S operations per step (spare slots repeat the last unit: the same bytes to the same
// place), so one vmcnt immediate waits for exactly the step before the newest.
// Measured (profiles/r06_wgrad_dma_ab.txt): 1.75 -> 1.655 ms at C3 128^3 96 -> 96, 3.03 -> 2.91 ms at 192 -> 96 (4-6 %).
constexpr int W6_XR = 144;
template <int WC>
constexpr int w6_buf() { return 3 * WG_ROWS * 64 + WC * W6_XR * 64; }
template <int WC>
constexpr size_t wgrad6_lds() { return (size_t)3 * w6_buf<WC>(); }

template <int WC>
__global__ __launch_bounds__(64 * 3 * WC) void conv3_wgrad6_kernel(WgradArgs a) {
  constexpr int NW = 3 * WC, U = 24 + 9 * WC, S = (U + NW - 1) / NW, BUFB = w6_buf<WC>();
  extern __shared__ __attribute__((aligned(16))) bf16 wsm[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int wn = wave / WC, wc = wave % WC;
  // work decode (XCD-contiguous, as v5)
  const int G = a.KD * 3, NT = a.Cout / 96, NC = a.Cin / (32 * WC);
  long long w;
  {
    const long long per = ((long long)a.nb + 7) / 8;
    w = (long long)(blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  if (w >= a.nb) return;
  const int ct = (int)(w % NC);
  long long q = w / NC;
  const int grp = (int)(q % G);
  q /= G;
  const int nt = (int)(q % NT), split = (int)(q / NT);
  const int n0 = nt * 96, c0 = ct * 32 * WC;
  const int T = a.KD * 9;
  const int dz = (a.KD == 3 ? grp / 3 : 1) - 1, dyy = grp % 3 - 1;
  const int HW = a.H * a.W, W1 = a.W + 1;
  const long long lines = a.V / a.W, R = lines * W1;
  const int shift = dz * HW + dyy * a.W;
  const long long gs = (long long)split * a.Lv, ge = min(R, gs + a.Lv);
  const int q128 = WG_ROWS / W1, r128 = WG_ROWS % W1;
  const rsrc_t rdy = make_rsrc(a.dy, (uint32_t)(a.V * a.Cout * 2));
  const rsrc_t rx = make_rsrc(a.x, (uint32_t)(a.V * a.Cin * 2));
  const unsigned lds0 = (unsigned)(uintptr_t)(LCI_LDS bf16*)wsm;
  const int lrow = lane >> 2, lch = lane & 3;

  f32x16 acc[3];
#pragma unroll
  for (int d = 0; d < 3; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[d][i] = 0.f;

  // slot i: unit u (wave-uniform), its row base in the step and the lane's channel byte offset; the lane's row walker
  GRow gr[S];
  int urow[S], ucb[S], uu[S];
#pragma unroll
  for (int i = 0; i < S; ++i) {
    const int u = min(wave + NW * i, U - 1);
    uu[i] = u;
    const bool isx = u >= 24;
    const int b = isx ? (u - 24) / 9 : u / 8;
    urow[i] = isx ? 16 * ((u - 24) % 9) : 16 * (u % 8);
    ucb[i] = 2 * ((isx ? c0 : n0) + 32 * b + 8 * lch);
    gr[i].init(gs + urow[i] + lrow - (isx ? 1 : 0), W1, a.H, a.D);
  }
  // this wave's S units of the step whose first gapped row is g0, into buffer p
  auto issue = [&](long long g0, int p) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < S; ++i) {
      const bool isx = uu[i] >= 24;
      const GRow& g = gr[i];
      bool ok;
      int vox;
      if (isx) {
        const long long Gr = g0 - 1 + urow[i] + lrow;
        ok = Gr >= 0 && Gr < R && g.X < a.W && (unsigned)(g.z + dz) < (unsigned)a.D &&
             (unsigned)(g.y + dyy) < (unsigned)a.H;
        vox = g.L * a.W + g.X + shift;
      } else {
        ok = g0 + urow[i] + lrow < ge && g.X < a.W;
        vox = g.L * a.W + g.X;
      }
      const int voff = ok ? vox * (isx ? a.Cin : a.Cout) * 2 + ucb[i] : 0x7FFFFFF0;
      dma16_lds(isx ? rx : rdy, voff, 0, lds0 + (unsigned)(p * BUFB + 1024 * uu[i]));
      gr[i].advance(q128, r128, W1, a.H, a.D);
    }
  };
  const int nsteps = (int)((ge - gs + WG_ROWS - 1) / WG_ROWS);
  issue(gs, 0);
  if (nsteps > 1) issue(gs + WG_ROWS, 1);
  int p = 0;
  for (int k = 0; k < nsteps; ++k) {
    if (k + 1 < nsteps) wait_vmcnt<S>();   // this wave's units of step k landed (step k+1's may be in flight)
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_waitcnt(0xC07F);     // lgkmcnt(0): this wave's reads of step k-1's buffer are done
    __builtin_amdgcn_s_barrier();           // every wave's units of step k landed; step k-1's buffer is free
    if (k + 2 < nsteps) issue(gs + (long long)(k + 2) * WG_ROWS, p == 0 ? 2 : p - 1);
    const bf16* tdy0 = (const bf16*)((const char*)wsm + p * BUFB) + wn * WG_ROWS * 32;
    const bf16* tx = (const bf16*)((const char*)wsm + p * BUFB) + 3 * WG_ROWS * 32 + wc * W6_XR * 32;
#pragma unroll
    for (int r0 = 0; r0 < WG_ROWS; r0 += 32) {
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const bf16x8 fa0 = sub ? frag_tr<1>(tdy0, 32, r0, 0, lane) : frag_tr<0>(tdy0, 32, r0, 0, lane);
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          const bf16x8 fb = sub ? frag_tr<1>(tx, 32, r0 + d, 0, lane) : frag_tr<0>(tx, 32, r0 + d, 0, lane);
          acc[d] = mfma32(fa0, fb, acc[d]);
        }
      }
    }
    p = p == 2 ? 0 : p + 1;
  }
  // acc[d] reg i: n = n0 + 32 wn + (i&3) + 8(i>>2) + 4h, c = c0 + 32 wc + (lane & 31)
  const int h = lane >> 5;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    float* out = a.part + ((long long)split * T + grp * 3 + d) * a.Cout * a.Cin;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = n0 + 32 * wn + (i & 3) + 8 * (i >> 2) + 4 * h;
      out[(long long)row * a.Cin + c0 + 32 * wc + (lane & 31)] = acc[d][i];
    }
  }
}

template <int WC>
static int launch_wgrad6(WgradArgs a, hipStream_t st) {
  const size_t sh = wgrad6_lds<WC>();
  const long long nb = (long long)a.KD * 3 * a.ns * (a.Cout / 96) * (a.Cin / (32 * WC));
  LCI_CHECK(nb < (1LL << 30), "conv3_wgrad: too many workgroups");
  a.nb = (int)nb;
  (void)hipFuncSetAttribute((const void*)conv3_wgrad6_kernel<WC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  hipLaunchKernelGGL((conv3_wgrad6_kernel<WC>), dim3((unsigned)((nb + 7) / 8 * 8)), dim3(64 * 3 * WC), sh, st, a);
  LCI_LAUNCH_CHECK();
  return 0;
}
// v6 takes v5's (1, 3, WC) shapes whose operands a 32-bit DMA offset reaches; LCI_WGRAD_DMA=0 keeps them on v5 (A/B)
static bool wgrad6_ok(const WgradArgs& a) {
  const char* e = getenv("LCI_WGRAD_DMA");   // (read per call: the tests compare v6 with v5 in one process)
  const bool on = !(e && e[0] == '0');
  return on && a.V * a.Cin * 2 <= 0x7FFFFF00LL && a.V * a.Cout * 2 <= 0x7FFFFF00LL;
}

// (MB, WN, WC) of the v5 weight gradient, or MB = 0 when the v4 kernel handles the shape. Measured
// (tools/conv_bench.py): the 8-wave (2, 2, 4) tile 1.6-1.8x over v4 (C5 512->256: 228 -> 128 ms); a 4-wave
// (1, 1, 4) tile was 5-10 % slower than v4, so v5 needs >= 6 waves: Cout % 128 -> (2, 2, 4 or 2); the Swin
// channel counts (Cout % 96) -> (1, 3, 3 or 2) (9-wave workgroups cannot hold MB = 2 without spilling).
static void wgrad5_tile(int Cin, int Cout, int& mb, int& wn, int& wc) {
  mb = wn = wc = 0;
  if (Cout % 128 == 0) { mb = 2; wn = 2; wc = Cin % 128 == 0 ? 4 : (Cin % 64 == 0 ? 2 : 0); }
  else if (Cout % 96 == 0) { mb = 1; wn = 3; wc = Cin % 96 == 0 ? 3 : (Cin % 64 == 0 ? 2 : 0); }
  if (wc == 0) mb = wn = 0;
}

template <int NT>
static int launch(const ConvArgs& a, hipStream_t st) {
  if (a.Cin % 32 == 0) {
    ConvArgs b = a;
    b.nvb = (int)((a.V + 511) / 512);
    b.ntile = a.Cout / (32 * NT);
    // measured (tools/conv_bench.py, C3/C5 shapes): order 1 gains up to 12 % from Cout >= 96 (512->256 at 256^3:
    // 164 -> 146 ms) and loses up to 15 % on the 1-2 tile Cout = 32 / 64 convs, which keep order 0
    b.order = a.Cout >= 96 ? 1 : 0;
    const long long nb = (long long)b.nvb * b.ntile;
    constexpr int XU = (512 + 2 + 15) / 16, WU = 3 * 32 * NT / 16;
    const size_t shd = (size_t)2 * (XU + WU) * 1024 + 16;   // two slots + the zero chunk
    if (a.nsplit > 1) {
      LCI_CHECK(a.part != nullptr, "conv3: split-K needs the partial workspace");
      LCI_CHECK(nb * a.nsplit < (1LL << 31), "conv3: too many workgroups");
      (void)hipFuncSetAttribute((const void*)conv3_fwd_dma_kernel<NT, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
      hipLaunchKernelGGL((conv3_fwd_dma_kernel<NT, true>), dim3((unsigned)(nb * a.nsplit)), dim3(512), shd, st, b);
      LCI_LAUNCH_CHECK();
      const long long n8 = a.V * a.Cout / 8;
      hipLaunchKernelGGL(conv3_sum_kernel, dim3((unsigned)std::min<long long>((n8 + 255) / 256, 8192)), dim3(256), 0,
                         st, (const float*)a.part, a.y, n8, a.nsplit);
    } else {
      const dim3 grid((unsigned)(b.order ? (nb + 7) / 8 * 8 : nb));
      if constexpr (NT >= 2) {
        // LDS-DMA staging: equal to v2 at the 256- / 512-channel C5 shapes, 2-8 % faster at 64 / 96 channels
        // (profiles/r05_conv_dma_ab.txt)
        (void)hipFuncSetAttribute((const void*)conv3_fwd_dma_kernel<NT, false>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipLaunchKernelGGL((conv3_fwd_dma_kernel<NT, false>), grid, dim3(512), shd, st, b);
      } else {   // Cout = 32: the register-staged v2 kernel (2-5 % ahead of the DMA one there)
        const size_t sh = (size_t)2 * (514 * CLD2 + 3 * 32 * NT * CLD2) * sizeof(bf16) + 16;   // + the zero chunk
        (void)hipFuncSetAttribute((const void*)conv3_fwd_lds2_kernel<NT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        hipLaunchKernelGGL((conv3_fwd_lds2_kernel<NT>), grid, dim3(512), sh, st, b);
      }
    }
  } else if (a.Cin % 16 == 0) {
    constexpr int MV = 4;
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

// Output-channel tile of the forward kernels (32 NT channels), shared by the launch and the split heuristic.
static int conv3_nt(int Cout) {
  const int nb = Cout / 32;
  return nb % 3 == 0 ? 3 : (nb % 4 == 0 ? 4 : (nb % 2 == 0 ? 2 : 1));
}

static int conv3_fwd_impl(const void* x, const void* w, void* y, float* part, int nsplit, int B, int D, int H, int W,
                          int Cin, int Cout, int KD, void* stream) {
  LCI_CHECK(B > 0 && D > 0 && H > 0 && W > 0 && Cin > 0, "conv3: bad shape");
  LCI_CHECK(KD == 3 || (KD == 1 && D == 1), "conv3: KD must be 3, or 1 with D == 1 (2-D)");
  LCI_CHECK(Cout % 32 == 0, "conv3: Cout (%d) must be a multiple of 32", Cout);
  LCI_CHECK(((uintptr_t)x & 15) == 0 && ((uintptr_t)w & 15) == 0 && ((uintptr_t)y & (nsplit > 1 ? 15 : 7)) == 0 &&
                ((uintptr_t)part & 15) == 0, "conv3: misaligned pointers");
  LCI_CHECK(nsplit >= 1 && (nsplit == 1 || Cin % 32 == 0), "conv3: split-K needs Cin %% 32 == 0");
  ConvArgs a{};
  a.x = (const bf16*)x; a.w = (const bf16*)w; a.y = (bf16*)y;
  a.V = (long long)B * D * H * W;
  a.D = D; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.KD = KD;
  a.nsplit = nsplit; a.part = part;
  LCI_CHECK((a.V + 255) / 256 < (1LL << 31), "conv3: volume too large");
  hipStream_t st = (hipStream_t)stream;
  switch (conv3_nt(Cout)) {
    case 3: return launch<3>(a, st);
    case 4: return launch<4>(a, st);
    case 2: return launch<2>(a, st);
    default: return launch<1>(a, st);
  }
}

extern "C" int lci_conv3_fwd(const void* x, const void* w, void* y, int B, int D, int H, int W, int Cin, int Cout,
                             int KD, void* stream) {
  return conv3_fwd_impl(x, w, y, nullptr, 1, B, D, H, W, Cin, Cout, KD, stream);
}

// Split-K for small volumes: under 256 workgroups of 512 voxels x 32 NT channels (the 4^3 - 32^3 stages of the
// SwinUNETR head: 16-128 workgroups on 256 CUs) the (tap group, channel chunk) slabs are split into ranges whose f32
// partials a second pass sums: ~512 workgroups, at most 100 MB of partials, at least 2 slabs per range.
extern "C" int lci_conv3_fwd_splits(long long V, int Cin, int Cout, int KD) {
  if (V <= 0 || Cin % 32 || Cout % 32 || (KD != 1 && KD != 3)) return 1;
  const long long nb = (V + 511) / 512 * (Cout / (32 * conv3_nt(Cout)));
  if (nb >= 256) return 1;
  const long long nslab = (long long)KD * 3 * (Cin / 32);
  long long s = (512 + nb - 1) / nb;
  s = std::min(s, nslab / 2);
  s = std::min(s, 64LL);
  while (s > 1 && s * V * Cout * 4 > (100LL << 20)) --s;
  return (int)std::max(s, 1LL);
}

extern "C" int lci_conv3_fwd_split(const void* x, const void* w, void* y, float* part, int nsplit, int B, int D, int H,
                                   int W, int Cin, int Cout, int KD, void* stream) {
  return conv3_fwd_impl(x, w, y, part, nsplit, B, D, H, W, Cin, Cout, KD, stream);
}

extern "C" int lci_conv3_pack_weight(const float* w, void* out, int Cout, int Cin, int KD, int mode, int Cin_pad,
                                     void* stream) {
  LCI_CHECK(Cout > 0 && Cin > 0 && (KD == 1 || KD == 3) && (mode == 0 || mode == 1), "conv3_pack: bad arguments");
  LCI_CHECK(mode == 0 || Cin_pad >= Cin, "conv3_pack: Cin_pad (%d) < Cin (%d)", Cin_pad, Cin);
  const int T = KD * 9;
  const int rows = mode == 0 ? Cout : Cin_pad, J = mode == 0 ? Cin : Cout;
  hipLaunchKernelGGL(conv3_pack_kernel, dim3((unsigned)rows, (unsigned)((J + 63) / 64)), dim3(256), 0,
                     (hipStream_t)stream, w, (bf16*)out, Cout, Cin, mode == 0 ? Cin : Cin_pad, T, mode);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_convup_interleave(const void* src, void* dst, int B, int D, int H, int W, int kd, int kh, int kw,
                                     int C, int ld, int adjoint, void* stream) {
  LCI_CHECK(B > 0 && D > 0 && H > 0 && W > 0 && kd > 0 && kh > 0 && kw > 0 && C > 0 && C % 8 == 0 && ld >= C &&
                ld % 8 == 0, "convup_interleave: bad shape (C, ld multiples of 8)");
  LCI_CHECK(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, "convup_interleave: pointers must be 16-byte aligned");
  const long long per_row = (long long)W * kd * kh * kw * (C / 8), nrows = (long long)B * D * H;
  LCI_CHECK(per_row < (1LL << 31), "convup_interleave: row too wide");
  hipLaunchKernelGGL(convup_interleave_kernel, dim3((unsigned)((per_row + 255) / 256),
                     (unsigned)std::min<long long>(nrows, 65535)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)src, (bf16*)dst, nrows, D, H, W, kd, kh, kw, C, ld, adjoint);
  LCI_LAUNCH_CHECK();
  return 0;
}

template <int MB, int WN, int WC>
static int wgrad5_slots_of() {   // co-resident workgroups of this tile on the whole device
  const size_t sh = wgrad5_lds<MB, WN, WC>();
  int dev = 0, ncu = 0, per = 0;
  LCI_HIP(hipGetDevice(&dev));
  LCI_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  (void)hipFuncSetAttribute((const void*)conv3_wgrad5_kernel<MB, WN, WC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  LCI_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)conv3_wgrad5_kernel<MB, WN, WC>,
                                                       64 * WN * WC, sh));
  return std::max(1, ncu * std::max(1, per));
}

static int wgrad5_slots(int mb, int wn, int wc) {
  static int cache[4] = {};
  const int i = mb == 2 ? (wc == 4 ? 0 : 1) : (wc == 3 ? 2 : 3);
  if (!cache[i]) {
#define LCI_W5(M, N, C) if (mb == M && wn == N && wc == C) cache[i] = wgrad5_slots_of<M, N, C>();
    LCI_W5(2, 2, 4) LCI_W5(2, 2, 2) LCI_W5(1, 3, 3) LCI_W5(1, 3, 2)
#undef LCI_W5
  }
  return cache[i];
}

// Voxel (gapped-row) splits. v5 tiles: at most 2^17 rows per workgroup, then as many splits as fill the last round of
// co-resident workgroups (a grid of r full rounds, not r rounds and a sliver: the C3 96-channel gradient went from
// 2304 workgroups of 8192 rows to 1 round), at least 1024 rows each. v4: up to 2^17 rows, fewer (>= 1024) when that
// leaves under ~2048 workgroups (small 2-D volumes, few channel tiles).
extern "C" long long lci_conv3_wgrad_splits(long long V, int Cin, int Cout, int KD) {
  int mb, wn, wc;
  wgrad5_tile(Cin, Cout, mb, wn, wc);
  if (mb) {
    const long long tiles = (long long)KD * 3 * (Cout / (32 * mb * wn)) * (Cin / (32 * wc));
    const long long slots = wgrad5_slots(mb, wn, wc);
    const long long ns_min = (V + (1 << 17) - 1) >> 17;
    const long long rounds = std::max(1LL, (tiles * ns_min + slots - 1) / slots);
    const long long ns = std::max(ns_min, rounds * slots / tiles);
    return std::max(1LL, std::min(ns, (V + 1023) / 1024));
  }
  const long long tiles = (long long)KD * 3 * (Cout / (32 * ((Cout / 32) % 2 == 0 ? 2 : 1))) * (Cin / 32);
  long long lv = 1 << 17;
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
  LCI_CHECK(a.V / W < (1LL << 31), "conv3_wgrad: volume too large");
  const long long ns = lci_conv3_wgrad_splits(a.V, Cin, Cout, KD);
  LCI_CHECK(ns < 65536, "conv3_wgrad: volume too large");
  const long long R = (a.V / W) * (W + 1);
  a.Lv = (R + ns - 1) / ns;
  a.Lv = (a.Lv + WG_ROWS - 1) / WG_ROWS * WG_ROWS;   // splits start on a step boundary
  hipStream_t st = (hipStream_t)stream;
  a.ns = (int)ns;
  int mb, wn, wc;
  wgrad5_tile(Cin, Cout, mb, wn, wc);
  if (mb) {
#define LCI_W5(M, N, C) if (mb == M && wn == N && wc == C) return launch_wgrad5<M, N, C>(a, st);
    if (mb == 1 && wgrad6_ok(a)) return wc == 3 ? launch_wgrad6<3>(a, st) : launch_wgrad6<2>(a, st);
    LCI_W5(2, 2, 4) LCI_W5(2, 2, 2) LCI_W5(1, 3, 3) LCI_W5(1, 3, 2)
#undef LCI_W5
  }
  // 32*MT output channels per workgroup: 2 where Cout allows (2 waves per SIMD), else 1. MT = 3 (256 registers, one
  // wave per SIMD) measured 1.2-1.4x slower than MT = 1 on the Cout = 96 / 192 C3 shapes
  const int mt = (Cout / 32) % 2 == 0 ? 2 : 1;
  a.ns = (int)ns;
  const long long nb = (long long)KD * 3 * ns * (Cout / (32 * mt)) * (Cin / 32);
  LCI_CHECK(nb < (1LL << 30), "conv3_wgrad: too many workgroups");
  a.nb = (int)nb;
  a.order = 1;
  dim3 grid((unsigned)(a.order ? (nb + 7) / 8 * 8 : nb));
  if (mt == 2) hipLaunchKernelGGL(conv3_wgrad4_kernel<2>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(conv3_wgrad4_kernel<1>, grid, dim3(256), 0, st, a);
  LCI_LAUNCH_CHECK();
  return 0;
}
