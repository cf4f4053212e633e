// Weight (and bias) gradient of the token-wise Linear layers: dW = dY^T . X, db = sum_m dY[m, :].
//
// Replaces the backward GEMM of nn.Linear for TransformerBlock qkv / out_proj / MLP (backbone_vit.py:166-167, 249),
// MambaVisionMixer in_proj / x_proj / dt_proj / out_proj (mamba.py:60-64, 90) and the Hyena projections: under the
// trainer's bf16 autocast (trainer_base.py:157-170) torch runs it as one hipBLASLt GEMM whose reduction dimension
// is the token count M (up to 2^21) against an output of only N x K (384 x 384 ... 1536 x 384); hipBLASLt picks
// small-output tiles for that and runs at 100-330 TFLOP/s (x_proj / dt_proj: 5 TFLOP/s, profiles/r02_*gemm*).
//
// Both operands have the token as the reduction index, which is the slow (row) axis of the row-major activations,
// so R-row slabs of dY (M x N, row stride ldy) and X (M x K, row stride ldx) are staged row-major in LDS, as
// 32-column blocks with 64-B rows, and read back as MFMA fragments with ds_read_b64_tr_b16 (frag_tr, common.hpp).
// The slabs arrive by LDS-DMA into a ring of LDS buffers several slabs ahead (see the kernel).
// A workgroup owns a (32 MB WN) x (32 CB WC) tile of dW for one split of the tokens; wave (wn, wc) accumulates MB x CB
// 32x32 blocks over every row of the split (no cross-wave reduction). Splits write f32 partials (ns, N, K) that the
// caller sums (deterministic, no atomics). The bias gradient rides along in the workgroups of the first K tile:
// each thread sums the same 8 columns of every staged dY slab (from LDS) in registers and the workgroup reduces the
// per-thread sums in LDS once at the end. Rows past M and columns past N / K are staged as zeros and never stored.
#include <stdlib.h>

#include <algorithm>

#include "common.hpp"

namespace lci {

constexpr int LW_R = 32;     // token rows per staged slab
constexpr int LW_NBUF = 4;   // LDS ring depth (slabs in flight: NBUF - 1)

struct LinWgradArgs {
  const bf16* dy;     // (M, ldy) row-major, columns [0, N)
  const bf16* x;      // (M, ldx) row-major, columns [0, K)
  float* part;        // (ns, N, K)
  float* dbpart;      // (ns, N) or null
  long long M, ldy, ldx, rows;   // rows per split (multiple of LW_R)
  int N, K, ns, ntn, ntk, nb;
};

// 16 zero bytes x 4 for the staging lanes whose row is past M or whose columns are past N / K (tile padding)
__device__ __attribute__((aligned(16))) bf16 kLwZero[32];

// One LDS-DMA unit: every lane's 16 bytes at gsrc land at LDS byte address lds_dst + 16 * lane. Issued from inline
// asm so that the compiler does not treat the pending DMA as an LDS write every later ds_read must wait for (it
// would drain the whole ring with vmcnt(0) before each slab); completion is counted by wait_vmcnt below. M0 is
// saved and restored inside the statement.
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

// Slabs of R token rows arrive by LDS-DMA (global_load_lds_dwordx4: lane l of a wave-instruction writes bytes
// 16 l .. 16 l + 15 of a 1-KB unit = 16 rows x 64 B of one 32-column block) into a ring of NBUF LDS buffers,
// NBUF - 1 slabs ahead: no staging registers, no ds_write pass; each wave waits (counted vmcnt) only for its own
// DMA units of the slab it is about to read, then one raw s_barrier publishes the slab and retires the buffer the
// next DMA overwrites.
template <int MB, int CB, int WN, int WC, int R, int NBUF>
__global__ __launch_bounds__(64 * WN * WC, 1) void linear_wgrad_kernel(LinWgradArgs a) {
  constexpr int NW = WN * WC, NTH = 64 * NW;
  constexpr int NBY = MB * WN, NBX = CB * WC;                 // 32-column blocks of dY / X per slab
  constexpr int BLK = R * 32, BUF = (NBY + NBX) * BLK;        // elements
  constexpr int RG = R / 16, U = (NBY + NBX) * RG;            // DMA units per slab
  constexpr int UPW = (U + NW - 1) / NW, ULO = U / NW;        // units per wave (waves < U % NW take UPW)
  static_assert(R % 32 == 0 && NBUF >= 2, "slab shape");
  constexpr int RSY = NTH / (NBY * 4);                        // bias: rows per pass of the column-chunk threads
  static_assert(NTH % (NBY * 4) == 0, "tile / thread count mismatch");
  extern __shared__ __attribute__((aligned(16))) bf16 lsm[];
  const int lane = threadIdx.x & 63, tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: DMA offsets stay scalar
  const int wn = wave / WC, wc = wave % WC;
  // XCD-contiguous work order (block b -> XCD b % 8): the K tiles, then the N tiles of one split are adjacent, so
  // the workgroups sharing a split's dY / X rows run on the same XCD (same L2)
  long long w = blockIdx.x;
  {
    const long long per = ((long long)a.nb + 7) / 8;
    w = (long long)(blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  if (w >= a.nb) return;   // grid padding, uniform per workgroup, before any barrier
  const int kt = (int)(w % a.ntk);
  long long q = w / a.ntk;
  const int nt = (int)(q % a.ntn), split = (int)(q / a.ntn);
  const int n0 = nt * 32 * NBY, k0 = kt * 32 * NBX;
  const long long ms = (long long)split * a.rows, me = min(a.M, ms + a.rows);
  const int nslab = (int)((me - ms + R - 1) / R);
  const bool do_bias = a.dbpart != nullptr && kt == 0;
  const int nunits = wave < U % NW ? UPW : ULO;

  f32x16 acc[MB][CB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // this lane's part of each of the wave's DMA units: (row in the 16-row group, 16-B chunk of the 64-B row)
  const int lr = lane >> 2, lc = lane & 3;
  const unsigned lds_base = (unsigned)(uintptr_t)(LCI_LDS bf16*)lsm;
  // per DMA unit of this wave: the lane's source address for the next slab to issue (or the zero block for columns
  // past N / K), the bytes it advances per slab, and the unit's LDS byte offset in a ring slot. Slabs are issued in
  // order, so the addresses advance by one add per unit and slab; only a split's ragged last slab checks rows.
  const char* uptr[UPW];
  unsigned ustep[UPW], urow[UPW];
  int ulds[UPW];
#pragma unroll
  for (int t = 0; t < UPW; ++t) {
    const int u = min(wave + NW * t, U - 1);
    const int blk = u / RG, rg = u - blk * RG;
    urow[t] = 16 * rg + lr;
    ulds[t] = 2 * (blk * BLK + rg * 512);
    const bool isy = blk < NBY;
    const int col = isy ? n0 + 32 * blk + 8 * lc : k0 + 32 * (blk - NBY) + 8 * lc;
    const bool ok = col < (isy ? a.N : a.K);
    const long long ld = isy ? a.ldy : a.ldx;
    uptr[t] = ok ? (const char*)((isy ? a.dy : a.x) + (ms + urow[t]) * ld + col) : (const char*)(kLwZero + 8 * lc);
    ustep[t] = ok ? (unsigned)(2 * R * ld) : 0u;
  }
  auto issue = [&](int slab) {
    const unsigned lds0 = lds_base + (unsigned)(2 * (slab % NBUF) * BUF);   // byte address of the ring slot
    const long long m0 = ms + (long long)slab * R;
    if (m0 + R <= me) {
#pragma unroll
      for (int t = 0; t < UPW; ++t) {
        if (t < nunits) glds16(uptr[t], lds0 + ulds[t]);
        uptr[t] += ustep[t];
      }
    } else {   // the split's ragged last slab: rows past its end read the zero block
#pragma unroll
      for (int t = 0; t < UPW; ++t) {
        if (t < nunits) glds16(m0 + urow[t] < me ? (const void*)uptr[t] : (const void*)(kLwZero + 8 * lc), lds0 + ulds[t]);
        uptr[t] += ustep[t];
      }
    }
  };
  // wait until at most `later` slabs' DMA units of this wave are outstanding
  auto wait_for = [&](int later) {
    if (later >= NBUF - 2) {
      if (nunits == UPW) wait_vmcnt<UPW * (NBUF - 2)>(); else wait_vmcnt<ULO * (NBUF - 2)>();
    } else if (NBUF > 3 && later == 1) {
      if (nunits == UPW) wait_vmcnt<UPW>(); else wait_vmcnt<ULO>();
    } else {
      wait_vmcnt<0>();
    }
  };

  const int ccy = tid % (NBY * 4), ry0 = tid / (NBY * 4);
  float bsum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum[j] = 0.f;

#pragma unroll
  for (int p = 0; p < NBUF - 1; ++p)
    if (p < nslab) issue(p);
  for (int sl = 0; sl < nslab; ++sl) {
    wait_for(min(NBUF - 2, nslab - 1 - sl));
    __builtin_amdgcn_s_waitcnt(15 | (3 << 14) | (7 << 4));   // lgkmcnt(0): this wave's LDS reads are done
    __builtin_amdgcn_s_barrier();
    if (sl + NBUF - 1 < nslab) issue(sl + NBUF - 1);
    const bf16* base = lsm + (sl % NBUF) * BUF;
    const bf16* ty = base + (MB * wn) * BLK;
    const bf16* tx = base + NBY * BLK + (CB * wc) * BLK;
#pragma unroll
    for (int r0 = 0; r0 < R; r0 += 32) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 fa[MB], fb[CB];
#pragma unroll
        for (int i = 0; i < MB; ++i)
          fa[i] = s ? frag_tr<1>(ty + i * BLK, 32, r0, 0, lane) : frag_tr<0>(ty + i * BLK, 32, r0, 0, lane);
#pragma unroll
        for (int j = 0; j < CB; ++j)
          fb[j] = s ? frag_tr<1>(tx + j * BLK, 32, r0, 0, lane) : frag_tr<0>(tx + j * BLK, 32, r0, 0, lane);
#pragma unroll
        for (int i = 0; i < MB; ++i)
#pragma unroll
          for (int j = 0; j < CB; ++j) acc[i][j] = mfma32(fa[i], fb[j], acc[i][j]);
      }
    }
    if (do_bias) {   // column sums of the staged dY block rows (zero rows past M contribute nothing)
#pragma unroll
      for (int r = ry0; r < R; r += RSY) {
        const bf16x8 v = *(const bf16x8*)(base + (ccy >> 2) * BLK + r * 32 + 8 * (ccy & 3));
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[j] += to_f32(v[j]);
      }
    }
  }
  // acc[i][j] reg e: n = n0 + 32 (MB wn + i) + (e&3) + 8(e>>2) + 4h, k = k0 + 32 (CB wc + j) + (lane & 31)
  const int h = lane >> 5;
  float* out = a.part + (long long)split * a.N * a.K;
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const int k = k0 + 32 * (CB * wc + j) + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int n = n0 + 32 * (MB * wn + i) + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (n < a.N && k < a.K) out[(long long)n * a.K + k] = acc[i][j][e];
      }
    }
  if (do_bias) {   // uniform per workgroup
    __syncthreads();            // every wave is done reading the ring
    float* red = (float*)lsm;   // [NTH / (4 NBY)][32 NBY]
    constexpr int G = NTH / (NBY * 4);
    const int g = tid / (NBY * 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) red[g * 32 * NBY + 8 * ccy + j] = bsum[j];
    __syncthreads();
    for (int col = tid; col < 32 * NBY; col += NTH) {
      float sum = 0.f;
      for (int gg = 0; gg < G; ++gg) sum += red[gg * 32 * NBY + col];
      if (n0 + col < a.N) a.dbpart[(long long)split * a.N + n0 + col] = sum;
    }
  }
}

struct LwTile { int mb, cb, wn, wc; };
// instantiated tiles (dW rows x cols per workgroup), in order of preference at equal padding:
// 128 x 384 as 4 waves of 128 x 96 (one wave per SIMD, 12 accumulators: 7 LDS fragments per 12 MFMAs),
// 128 x 384 as 6 waves of 64 x 128 (6 fragments per 8 MFMAs), 128 x 192 (6 waves), 128 x 128 (4),
// 64 x 192 (3: x_proj 40 x 192), 192 x 32 (3: dt_proj 192 x 24), 96 x 96 (3: Swin C = 96 projections)
// The last tile (64 x 64, the Hyena filter's layers) is only taken when no other tile fits within 2x padding.
static const LwTile kLwTiles[] = {{4, 3, 1, 4}, {2, 4, 2, 3}, {2, 2, 2, 3}, {2, 2, 2, 2},
                                  {2, 2, 1, 3}, {2, 1, 3, 1}, {1, 3, 3, 1}, {1, 1, 2, 2}};
constexpr int kLwNTiles = (int)(sizeof(kLwTiles) / sizeof(kLwTiles[0]));

// The first tile with the least padded work; -1 if every tile more than doubles the work. Narrow outputs (N x K <=
// 8192: the Mamba x_proj / dt_proj gradients of the Swin recipes, 24 x 48, 48 x 8, 32 x 96, 96 x 16) take the tile
// with the least padding whatever it is: their cost is streaming the M token rows, not the padded MFMAs (hipBLASLt
// ran 24 x 48 over 2^19 tokens in 0.27 ms, 15x the rows' read time).
static int lw_pick(int N, int K) {
  int best = -1;
  double bw = 0.0;
  for (int t = 0; t < kLwNTiles; ++t) {
    const LwTile& c = kLwTiles[t];
    const int tn = 32 * c.mb * c.wn, tk = 32 * c.cb * c.wc;
    const double padded = (double)((N + tn - 1) / tn * tn) * ((K + tk - 1) / tk * tk);
    const double waste = padded / ((double)N * K);
    if (t == kLwNTiles - 1 && best >= 0) break;
    if (waste <= 2.0 && (best < 0 || waste < bw - 1e-9)) { best = t; bw = waste; }
  }
  if (best < 0 && (long long)N * K <= 8192) {
    for (int t = 0; t < kLwNTiles; ++t) {
      const LwTile& c = kLwTiles[t];
      const int tn = 32 * c.mb * c.wn, tk = 32 * c.cb * c.wc;
      const double padded = (double)((N + tn - 1) / tn * tn) * ((K + tk - 1) / tk * tk);
      if (best < 0 || padded < bw - 1e-9) { best = t; bw = padded; }
    }
  }
  return best;
}

template <int MB, int CB, int WN, int WC>
static int launch_lw(LinWgradArgs a, hipStream_t st) {
  constexpr int NBY = MB * WN, NBX = CB * WC;
  const size_t sh = (size_t)LW_NBUF * (NBY + NBX) * LW_R * 32 * sizeof(bf16);
  LCI_CHECK(sh <= 160 * 1024, "linear_wgrad: LDS ring of %zu bytes", sh);
  a.ntn = (a.N + 32 * NBY - 1) / (32 * NBY);
  a.ntk = (a.K + 32 * NBX - 1) / (32 * NBX);
  const long long nb = (long long)a.ns * a.ntn * a.ntk;
  LCI_CHECK(nb < (1LL << 30), "linear_wgrad: too many workgroups");
  a.nb = (int)nb;
  const dim3 grid((unsigned)((nb + 7) / 8 * 8)), block(64 * WN * WC);
  (void)hipFuncSetAttribute((const void*)linear_wgrad_kernel<MB, CB, WN, WC, LW_R, LW_NBUF>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL((linear_wgrad_kernel<MB, CB, WN, WC, LW_R, LW_NBUF>), grid, block, sh, st, a);
  LCI_LAUNCH_CHECK();
  return 0;
}


// ------------------------------------------------------------------------- narrow outputs (the heads' 1x1 convs)
// y (M, N) = x (M, K) . w^T + b for N <= 8: UnetOutBlock's 1x1 conv to the class / output channels (MONAI-1.3
// get_conv_layer(kernel_size=1, bias=True), enhance_heads.py:30-356) over every voxel, as channels-last rows.
// hipBLASLt runs these 2-column GEMMs with 16-32-wide tiles at ~1% of the HBM rate (C3: 3 ms forward, 3 ms backward
// per step); they are pure streams: one thread per row, the weights in LDS as f32.
constexpr int LS_MAXN = 8, LS_MAXK = 256, LS_THREADS = 65536;   // backward: fixed grid-stride thread count

__global__ __launch_bounds__(256) void linear_small_fwd_kernel(const bf16* __restrict__ x, long long ldx,
                                                                const bf16* __restrict__ w,
                                                                const bf16* __restrict__ b, bf16* __restrict__ y,
                                                                long long M, int N, int K) {
  __shared__ float sw[LS_MAXN * LS_MAXK];
  for (int i = threadIdx.x; i < N * K; i += 256) sw[i] = to_f32(w[i]);
  __syncthreads();
  for (long long m = (long long)blockIdx.x * 256 + threadIdx.x; m < M; m += (long long)gridDim.x * 256) {
    float acc[LS_MAXN];
#pragma unroll
    for (int o = 0; o < LS_MAXN; ++o) acc[o] = 0.f;
    const bf16* xr = x + m * ldx;
    for (int c = 0; c < K; c += 8) {
      const bf16x8 v = *(const bf16x8*)(xr + c);
#pragma unroll
      for (int o = 0; o < LS_MAXN; ++o) {
        if (o >= N) break;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[o] += to_f32(v[j]) * sw[o * K + c + j];
      }
    }
    for (int o = 0; o < N; ++o) y[m * N + o] = to_bf16(acc[o] + (b ? to_f32(b[o]) : 0.f));
  }
}

// dx (M, K) = dy . w (optional); part ((N K + N), LS_THREADS) f32 = per-thread partial sums of dy^T x and of dy
template <int N>
__global__ __launch_bounds__(256) void linear_small_bwd_kernel(const bf16* __restrict__ x, long long ldx,
                                                                const bf16* __restrict__ w,
                                                                const bf16* __restrict__ dy, bf16* __restrict__ dx,
                                                                float* __restrict__ part, long long M, int K) {
  __shared__ float sw[N * LS_MAXK];
  for (int i = threadIdx.x; i < N * K; i += 256) sw[i] = to_f32(w[i]);
  __syncthreads();
  const int t = blockIdx.x * 256 + threadIdx.x;   // < LS_THREADS
  constexpr int KC = N <= 2 ? 64 : 32;             // K handled in register chunks (N KC partials per thread)
  for (int c0 = 0; c0 < K; c0 += KC) {
    const int kc = min(KC, K - c0);
    float gw[N][KC], gb[N];
#pragma unroll
    for (int o = 0; o < N; ++o) {
      gb[o] = 0.f;
#pragma unroll
      for (int j = 0; j < KC; ++j) gw[o][j] = 0.f;
    }
    for (long long m = t; m < M; m += LS_THREADS) {
      float d[N];
#pragma unroll
      for (int o = 0; o < N; ++o) { d[o] = to_f32(dy[m * N + o]); gb[o] += d[o]; }
      const bf16* xr = x + m * ldx + c0;
#pragma unroll
      for (int c = 0; c < KC; c += 8) {
        if (c >= kc) break;
        const bf16x8 v = *(const bf16x8*)(xr + c);
        bf16x8 o8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float s = 0.f;
#pragma unroll
          for (int o = 0; o < N; ++o) {
            gw[o][c + j] += d[o] * to_f32(v[j]);
            s += d[o] * sw[o * K + c0 + c + j];
          }
          o8[j] = to_bf16(s);
        }
        if (dx) *(bf16x8*)(dx + m * K + c0 + c) = o8;
      }
    }
#pragma unroll
    for (int o = 0; o < N; ++o)
#pragma unroll
      for (int j = 0; j < KC; ++j)
        if (j < kc) part[(long long)(o * K + c0 + j) * LS_THREADS + t] = gw[o][j];
    if (c0 == 0) {
#pragma unroll
      for (int o = 0; o < N; ++o) part[(long long)(N * K + o) * LS_THREADS + t] = gb[o];
    }
  }
}


// erff for the GELU kernels: the two polynomials of the device library's erff (ocml __ocml_erf_f32: |x| < 1 ->
// x + x P(x^2), else 1 - exp(-(x + x Q(x)))) with the same coefficients and operation order, both evaluated and
// selected (no divergent branches; the library's version branches per element), and the exp as one v_exp_f32 of
// the log2e-scaled argument instead of the library's extended-precision range reduction. The |x| < 1 result is
// bitwise the library's; the other side differs by <= 3e-7 absolute (exhaustive bf16 check in
// tests/test_linear_gpu.py; after the bf16 rounding the GELU results are bitwise torch's).
__device__ __forceinline__ float erf_epi(float x) {
  const float ax = fabsf(x), s = x * x;
  float p = fmaf(s, -0x1.268bc2p-11f, 0x1.420828p-8f);
  p = fmaf(s, p, -0x1.b59370p-6f);
  p = fmaf(s, p, 0x1.ce077cp-4f);
  p = fmaf(s, p, -0x1.81266p-2f);
  p = fmaf(s, p, 0x1.06eba0p-3f);
  const float lo = fmaf(ax, p, ax);
  float q = fmaf(ax, 0x1.1d3156p-16f, -0x1.8d129p-12f);
  q = fmaf(ax, q, 0x1.f9a6d2p-9f);
  q = fmaf(ax, q, -0x1.8c3164p-6f);
  q = fmaf(ax, q, 0x1.b4e9c8p-4f);
  q = fmaf(ax, q, 0x1.4515fap-1f);
  q = fmaf(ax, q, 0x1.078e5p-3f);
  const float hi = 1.f - __builtin_amdgcn_exp2f(-fmaf(ax, q, ax) * 1.44269504088896341f);
  return copysignf(ax < 1.f ? lo : hi, x);
}
__device__ __forceinline__ float gelu_erf(float v) { return 0.5f * v * (1.f + erf_epi(v * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float v) {   // torch GeluBackward (approximate = 'none')
  const float cdf = 0.5f * (1.f + erf_epi(v * 0.70710678118654752f));
  const float pdf = __builtin_amdgcn_exp2f(-0.5f * v * v * 1.44269504088896341f) * 0.39894228040143268f;
  return cdf + v * pdf;
}


// ----------------------------------------------------------------------------------- GELU (erf), bf16 stream
// MLPBlock's activation (nn.GELU(), approximate='none') between linear1 and linear2 under bf16 autocast, with
// torch's arithmetic (f32 opmath, x * 0.5 * (1 + erf(x / sqrt 2)); backward dy * (cdf + x * exp(-x^2 / 2) / sqrt(2 pi)))
// on 16-byte vectors, 8 bf16 per thread: 6-14 % faster than torch's elementwise kernels at the metric / C5 MLP
// shapes (tools/gelu_bench.py), bitwise the same results.
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, long long n8) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    const bf16x8 v = ((const bf16x8*)x)[i];
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = to_bf16(gelu_erf(to_f32(v[q])));
    ((bf16x8*)y)[i] = o;
  }
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                       bf16* __restrict__ dx, long long n8) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    const bf16x8 v = ((const bf16x8*)x)[i], g = ((const bf16x8*)dy)[i];
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = to_bf16(to_f32(g[q]) * gelu_erf_grad(to_f32(v[q])));
    ((bf16x8*)dx)[i] = o;
  }
}

// One 16-byte vector per thread, one pass (a grid capped at 16 workgroups per CU with a grid-stride loop measured
// 15-25 % slower, tools/gelu_bench.py).
static unsigned gelu_grid(long long n8) { return (unsigned)std::max(1LL, (n8 + 255) / 256); }

}  // namespace lci

using namespace lci;

template <int MB, int CB, int WN, int WC>
static int lw_slots_of() {   // co-resident workgroups of this tile on the whole device
  constexpr int NBY = MB * WN, NBX = CB * WC;
  const size_t sh = (size_t)LW_NBUF * (NBY + NBX) * LW_R * 32 * sizeof(bf16);
  int dev = 0, ncu = 0, per = 0;
  LCI_HIP(hipGetDevice(&dev));
  LCI_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  (void)hipFuncSetAttribute((const void*)linear_wgrad_kernel<MB, CB, WN, WC, LW_R, LW_NBUF>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  LCI_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per, (const void*)linear_wgrad_kernel<MB, CB, WN, WC, LW_R, LW_NBUF>, 64 * WN * WC, sh));
  return std::max(1, ncu * std::max(1, per));
}

static int lw_slots(int t) {
  static int cache[kLwNTiles] = {};
  if (!cache[t]) {
    const LwTile& c = kLwTiles[t];
#define LCI_LW(A, B, C, D) \
    if (c.mb == A && c.cb == B && c.wn == C && c.wc == D) cache[t] = lw_slots_of<A, B, C, D>();
    LCI_LW(4, 3, 1, 4) LCI_LW(2, 4, 2, 3) LCI_LW(2, 2, 2, 3) LCI_LW(2, 2, 2, 2) LCI_LW(2, 2, 1, 3) LCI_LW(2, 1, 3, 1)
    LCI_LW(1, 3, 3, 1) LCI_LW(1, 1, 2, 2)
#undef LCI_LW
  }
  return cache[t];
}

// Token splits for the weight gradient of an (N x K) Linear over M tokens (at least 256 rows each).
extern "C" long long lci_linear_wgrad_splits(long long M, int N, int K) {
  const int t = lw_pick(N, K);
  if (t < 0 || M <= 0) return 0;
  const LwTile& c = kLwTiles[t];
  const long long tiles = (long long)((N + 32 * c.mb * c.wn - 1) / (32 * c.mb * c.wn)) *
                          ((K + 32 * c.cb * c.wc - 1) / (32 * c.cb * c.wc));
  // one round of co-resident workgroups: every split's rows in one workgroup, the grid = the device's slots (a grid
  // of r rounds and a sliver ran the sliver as a whole extra round; fewer splits also cut the f32 partials the
  // caller sums: C4 fc1 256 -> 21 splits, 0.98 -> 0.81 ms with the sum, profiles/r05_split_ab.txt)
  const long long ns = std::max(1LL, lw_slots(t) / tiles);
  return std::max(1LL, std::min(ns, (M + 255) / 256));
}

extern "C" int lci_linear_wgrad(const void* dy, long long ldy, const void* x, long long ldx, long long M, int N,
                                int K, float* part, float* dbpart, void* stream) {
  LCI_CHECK(M > 0 && N > 0 && K > 0, "linear_wgrad: bad shape");
  LCI_CHECK(N % 8 == 0 && K % 8 == 0 && ldy % 8 == 0 && ldx % 8 == 0 && ldy >= N && ldx >= K,
            "linear_wgrad: N (%d), K (%d) and the row strides must be multiples of 8", N, K);
  LCI_CHECK(((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)part & 3) == 0 &&
            ((uintptr_t)dbpart & 3) == 0, "linear_wgrad: misaligned pointers");
  const int t = lw_pick(N, K);
  LCI_CHECK(t >= 0, "linear_wgrad: no tile fits N = %d, K = %d", N, K);
  const long long ns = lci_linear_wgrad_splits(M, N, K);
  LCI_CHECK(ns > 0 && ns < (1 << 24), "linear_wgrad: bad split count");
  LinWgradArgs a{};
  a.dy = (const bf16*)dy; a.x = (const bf16*)x; a.part = part; a.dbpart = dbpart;
  a.M = M; a.ldy = ldy; a.ldx = ldx; a.N = N; a.K = K; a.ns = (int)ns;
  a.rows = (M + ns - 1) / ns;
  a.rows = (a.rows + LW_R - 1) / LW_R * LW_R;
  hipStream_t st = (hipStream_t)stream;
  const LwTile& c = kLwTiles[t];
#define LCI_LW(A, B, C, D) \
  if (c.mb == A && c.cb == B && c.wn == C && c.wc == D) return launch_lw<A, B, C, D>(a, st);
  LCI_LW(4, 3, 1, 4) LCI_LW(2, 4, 2, 3) LCI_LW(2, 2, 2, 3) LCI_LW(2, 2, 2, 2) LCI_LW(2, 2, 1, 3) LCI_LW(2, 1, 3, 1) LCI_LW(1, 3, 3, 1)
  LCI_LW(1, 1, 2, 2)
#undef LCI_LW
  LCI_CHECK(false, "linear_wgrad: tile not instantiated");
  return 1;
}

extern "C" int lci_linear_small_threads(void) { return LS_THREADS; }

extern "C" int lci_linear_small_fwd(const void* x, long long ldx, const void* w, const void* bias, void* y,
                                    long long M, int N, int K, void* stream) {
  LCI_CHECK(M > 0 && N >= 1 && N <= LS_MAXN && K > 0 && K <= LS_MAXK && K % 8 == 0 && ldx % 8 == 0 && ldx >= K,
            "linear_small_fwd: unsupported shape M = %lld, N = %d, K = %d", M, N, K);
  LCI_CHECK(((uintptr_t)x & 15) == 0, "linear_small_fwd: misaligned x");
  const long long blocks = std::min((M + 255) / 256, 8192LL);
  hipLaunchKernelGGL(linear_small_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)x, ldx, (const bf16*)w, (const bf16*)bias, (bf16*)y, M, N, K);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_linear_small_bwd(const void* x, long long ldx, const void* w, const void* dy, void* dx,
                                    float* part, long long M, int N, int K, void* stream) {
  LCI_CHECK(M > 0 && N >= 1 && N <= 4 && K > 0 && K <= LS_MAXK && K % 8 == 0 && ldx % 8 == 0 && ldx >= K,
            "linear_small_bwd: unsupported shape M = %lld, N = %d, K = %d", M, N, K);
  LCI_CHECK(((uintptr_t)x & 15) == 0 && ((uintptr_t)dx & 15) == 0, "linear_small_bwd: misaligned x / dx");
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(LS_THREADS / 256), blk(256);
  const bf16 *xp = (const bf16*)x, *wp = (const bf16*)w, *dyp = (const bf16*)dy;
  bf16* dxp = (bf16*)dx;
  if (N == 1) hipLaunchKernelGGL(linear_small_bwd_kernel<1>, g, blk, 0, st, xp, ldx, wp, dyp, dxp, part, M, K);
  else if (N == 2) hipLaunchKernelGGL(linear_small_bwd_kernel<2>, g, blk, 0, st, xp, ldx, wp, dyp, dxp, part, M, K);
  else if (N == 3) hipLaunchKernelGGL(linear_small_bwd_kernel<3>, g, blk, 0, st, xp, ldx, wp, dyp, dxp, part, M, K);
  else hipLaunchKernelGGL(linear_small_bwd_kernel<4>, g, blk, 0, st, xp, ldx, wp, dyp, dxp, part, M, K);
  LCI_LAUNCH_CHECK();
  return 0;
}

// n bf16 elements, n % 8 == 0, 16-byte aligned pointers.
extern "C" int lci_gelu_fwd(const void* x, void* y, long long n, void* stream) {
  LCI_CHECK(n > 0 && n % 8 == 0, "gelu: n (%lld) must be a positive multiple of 8", n);
  LCI_CHECK(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0, "gelu: pointers must be 16-byte aligned");
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(gelu_grid(n / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x,
                     (bf16*)y, n / 8);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_gelu_bwd(const void* x, const void* dy, void* dx, long long n, void* stream) {
  LCI_CHECK(n > 0 && n % 8 == 0, "gelu: n (%lld) must be a positive multiple of 8", n);
  LCI_CHECK(((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0,
            "gelu: pointers must be 16-byte aligned");
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(gelu_grid(n / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x,
                     (const bf16*)dy, (bf16*)dx, n / 8);
  LCI_LAUNCH_CHECK();
  return 0;
}
