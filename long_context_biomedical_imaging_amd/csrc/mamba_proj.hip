// MambaVisionMixer x_proj -> (dt, B, C) split -> dt_proj, fused, for gfx950 (bf16 autocast path).
//
// Replaces (mamba.py:120-124, under the trainer's bf16 autocast):
//   x_dbl = x_proj(x)                                   (Dx -> R + 2N, no bias; bf16 output)
//   dt, B, C = split(x_dbl, [R, N, N])
//   dt = dt_proj(dt)                                    (R -> Dx, + bias; bf16 output)
// with ONE pass over the token rows: x_dbl never goes to HBM in full; dt (the scan's delta), B|C (the scan's 16-byte
// aligned rows) and dt_low (kept for dt_proj's weight gradient) are written once. The backward pass does the two data
// gradients the same way (d dt_low = bf16(ddt Wdt); dxs = bf16(d x_dbl Wx) + du, the scan's input gradient added in
// the same pass) and writes d x_dbl for x_proj's weight gradient (lci_linear_wgrad).
//
// Tiling: one wave = 32 tokens (the MFMA column), v_mfma_f32_32x32x16_bf16 with the projection rows on the MFMA row:
//   fwd  GEMM1 x_dbl^T (rows x tokens) = Wx . xs^T     B operand = 8 consecutive channels of the lane's token row
//        GEMM2 dt^T (Dx x tokens)     = Wdt' . x_dbl^T + bias   B operand = GEMM1's accumulator packed to bf16
//              (the packing permutes the k order; the host builds Wdt' with its columns in that order)
//   bwd  GEMM3 d dt_low^T = Wdt^T . ddt^T;  d x_dbl^T = [bf16(GEMM3); dB; dC] staged in LDS per token
//        GEMM4 dxs^T = Wx^T . d x_dbl^T (+ du)
#include "common.hpp"

#include <algorithm>

namespace lci {

constexpr int MP_TOK = 32;                   // tokens per wave
constexpr int MP_WAVES = 4;

struct MpArgs {
  // forward
  const bf16* xs; long long ts_x;            // (M, Dx) token stride
  const bf16* w1;                            // (nb1 * 32, Dx) Wx rows, zero-padded
  const bf16* w2p;                           // (Dxp, ks2 * 16) Wdt with columns in the accumulator-pack order
  const float* bias;                         // (Dx) dt_proj bias (bf16-rounded values)
  bf16* dt; long long ts_dt;                 // (M, Dx)
  bf16* bc;                                  // (M, 2N) contiguous
  bf16* dtl; int ld_dtl;                     // (M, ld_dtl) dt_low (columns [0, R))
  // backward
  const bf16* ddt; long long ts_ddt;         // (M, Dx)
  const bf16* dbc;                           // (M, 2N) [dB | dC] (the scan's f32 sums in autocast's bf16)
  const bf16* w2t;                           // (nb3 * 32, Dx) Wdt^T rows, zero-padded
  const bf16* w1t;                           // (Dxp, ks4 * 16) Wx^T, columns beyond R + 2N zero
  const bf16* du; long long ts_du;           // optional (M, Dx) added to dxs
  bf16* dxs; long long ts_dxs;               // (M, Dx)
  bf16* dxdbl; int ld_dxdbl;                 // (M, ld_dxdbl) d x_dbl (columns [0, R + 2N))
  long long M;
  int Dx, Dxp, R, N2, nb1, ks2, nb3, ks4, rows_lds;
};

// accumulator reg i of lane (n, h) holds row (i & 3) + 8 (i >> 2) + 4 h of its 32-row block
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ bf16x8 ld16(const bf16* p) { return *(const bf16x8*)p; }

// row of this lane's token (or zeros past M)
__device__ __forceinline__ bf16x8 tok_frag(const bf16* base, long long ts, long long tok, long long M, int col) {
  return tok < M ? ld16(base + tok * ts + col) : bf16x8{};
}

// A wave's 32 token rows of a (M, Dx) tensor with token stride == Dx are one contiguous block: stage it into the
// wave's LDS tile [token][Dx + 8] with 16-byte loads in memory order (coalesced), rows past M as zeros.
__device__ __forceinline__ void tile_in(const bf16* g, long long t0, long long M, int Dx, bf16* t, int lane) {
  const int cpr = Dx / 8, total = MP_TOK * cpr;
  for (int c = lane; c < total; c += 64) {
    const int tk = c / cpr, col = 8 * (c - tk * cpr);
    const long long tok = t0 + tk;
    *(bf16x8*)(t + tk * (Dx + 8) + col) = tok < M ? ld16(g + tok * Dx + col) : bf16x8{};
  }
}
// ... and back: 16-byte stores in memory order, optionally adding a second (M, Dx) tensor (bf16 + bf16 in f32)
__device__ __forceinline__ void tile_out(bf16* g, long long t0, long long M, int Dx, const bf16* t, int lane,
                                         const bf16* add) {
  const int cpr = Dx / 8, total = MP_TOK * cpr;
  for (int c = lane; c < total; c += 64) {
    const int tk = c / cpr, col = 8 * (c - tk * cpr);
    const long long tok = t0 + tk;
    if (tok >= M) break;
    bf16x8 v = *(const bf16x8*)(t + tk * (Dx + 8) + col);
    if (add) {
      const bf16x8 u = ld16(add + tok * Dx + col);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = to_bf16(to_f32(v[j]) + to_f32(u[j]));
    }
    *(bf16x8*)(g + tok * Dx + col) = v;
  }
}

__global__ __launch_bounds__(256) void mamba_proj_fwd_kernel(MpArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16 xdl[];   // [wave][token][rows_lds]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, n = lane & 31, h = lane >> 5;
  const long long t0 = ((long long)blockIdx.x * MP_WAVES + wave) * MP_TOK, tok = t0 + n;
  bf16* xw = xdl + wave * MP_TOK * a.rows_lds;
  bf16* tw = xdl + MP_WAVES * MP_TOK * a.rows_lds + wave * MP_TOK * (a.Dxp + 8);   // xs tile, then the dt tile
  tile_in(a.xs, t0, a.M, a.Dx, tw, lane);
  __builtin_amdgcn_wave_barrier();
  // GEMM1: x_dbl^T block b (rows 32 b ..) over K = Dx
  f32x16 acc1[2] = {f32x16{}, f32x16{}};
#pragma unroll
  for (int b = 0; b < 2; ++b) {      // compile-time block index: the accumulators stay in registers
    if (b >= a.nb1) break;
    f32x16 acc{};
    for (int k0 = 0; k0 < a.Dx; k0 += 16) {
      const bf16x8 bx = *(const bf16x8*)(tw + n * (a.Dx + 8) + k0 + 8 * h);
      const bf16x8 aw = ld16(a.w1 + (long long)(32 * b + n) * a.Dx + k0 + 8 * h);
      acc = mfma32(aw, bx, acc);
    }
    acc1[b] = acc;
    // x_dbl rounded to bf16 (the autocast Linear output) into this lane's token row of the LDS tile
#pragma unroll
    for (int i = 0; i < 16; ++i) xw[n * a.rows_lds + 32 * b + acc_row(i, h)] = to_bf16(acc[i]);
  }
  __builtin_amdgcn_wave_barrier();
  __syncthreads();
  // B | C rows (16-byte stores) and dt_low (kept for dt_proj's weight gradient), one token per lane (half 0)
  if (h == 0 && tok < a.M) {
    const bf16* row = xw + n * a.rows_lds;
    for (int c = 0; c < a.N2; c += 8) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = row[a.R + c + j];
      *(bf16x8*)(a.bc + tok * a.N2 + c) = v;
    }
    for (int c = 0; c < a.ld_dtl; c += 8) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = c + j < a.R ? row[c + j] : to_bf16(0.f);
      *(bf16x8*)(a.dtl + tok * a.ld_dtl + c) = v;
    }
  }
  // GEMM2: dt^T block db = Wdt' . x_dbl^T + bias; B operand = GEMM1 accumulators packed (pack order = Wdt' columns)
  for (int db = 0; db < a.Dxp / 32; ++db) {
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int d = 32 * db + acc_row(i, h);
      acc[i] = d < a.Dx ? a.bias[d] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (s >= a.ks2) break;
      const f32x16& src = acc1[s >> 1];
      const bf16x8 bx = (s & 1) ? pack8<1>(src) : pack8<0>(src);
      const bf16x8 aw = ld16(a.w2p + (long long)(32 * db + n) * (a.ks2 * 16) + 16 * s + 8 * h);
      acc = mfma32(aw, bx, acc);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * db + 8 * g + 4 * h;
      if (d < a.Dx) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = to_bf16(acc[4 * g + j]);
        *(bf16x4*)(tw + n * (a.Dx + 8) + d) = v;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  tile_out(a.dt, t0, a.M, a.Dx, tw, lane, nullptr);
}

__global__ __launch_bounds__(256) void mamba_proj_bwd_kernel(MpArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16 xdl[];   // [wave][token][rows_lds]: d x_dbl rows
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, n = lane & 31, h = lane >> 5;
  const long long t0 = ((long long)blockIdx.x * MP_WAVES + wave) * MP_TOK, tok = t0 + n;
  bf16* xw = xdl + wave * MP_TOK * a.rows_lds;
  bf16* tw = xdl + MP_WAVES * MP_TOK * a.rows_lds + wave * MP_TOK * (a.Dxp + 8);   // ddt tile, then the dxs tile
  const int RN = a.R + a.N2;
  tile_in(a.ddt, t0, a.M, a.Dx, tw, lane);
  __builtin_amdgcn_wave_barrier();
  // GEMM3: d dt_low^T block b = Wdt^T . ddt^T over K = Dx
  for (int b = 0; b < a.nb3; ++b) {
    f32x16 acc{};
    for (int k0 = 0; k0 < a.Dx; k0 += 16) {
      const bf16x8 bx = *(const bf16x8*)(tw + n * (a.Dx + 8) + k0 + 8 * h);
      const bf16x8 aw = ld16(a.w2t + (long long)(32 * b + n) * a.Dx + k0 + 8 * h);
      acc = mfma32(aw, bx, acc);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = 32 * b + acc_row(i, h);
      if (r < a.R) xw[n * a.rows_lds + r] = to_bf16(acc[i]);
    }
  }
  // dB | dC rows and zero padding rows
  if (h == 0) {
    bf16* row = xw + n * a.rows_lds;
    for (int c = 0; c < a.N2; ++c) row[a.R + c] = tok < a.M ? a.dbc[tok * a.N2 + c] : to_bf16(0.f);
    for (int r = RN; r < a.rows_lds; ++r) row[r] = to_bf16(0.f);
  }
  __builtin_amdgcn_wave_barrier();
  __syncthreads();
  if (h == 0 && tok < a.M) {   // d x_dbl rows for x_proj's weight gradient
    const bf16* row = xw + n * a.rows_lds;
    for (int c = 0; c < a.ld_dxdbl; c += 8) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = row[c + j];
      *(bf16x8*)(a.dxdbl + tok * a.ld_dxdbl + c) = v;
    }
  }
  // GEMM4: dxs^T block db = Wx^T . d x_dbl^T (+ du)
  for (int db = 0; db < a.Dxp / 32; ++db) {
    f32x16 acc{};
    for (int s = 0; s < a.ks4; ++s) {
      const bf16x8 bx = *(const bf16x8*)(xw + n * a.rows_lds + 16 * s + 8 * h);
      const bf16x8 aw = ld16(a.w1t + (long long)(32 * db + n) * (a.ks4 * 16) + 16 * s + 8 * h);
      acc = mfma32(aw, bx, acc);
    }
    // the data-gradient GEMM's output is bf16 (autocast); the scan's du is added to it in tile_out
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * db + 8 * g + 4 * h;
      if (d < a.Dx) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = to_bf16(acc[4 * g + j]);
        *(bf16x4*)(tw + n * (a.Dx + 8) + d) = v;
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  tile_out(a.dxs, t0, a.M, a.Dx, tw, lane, a.du);
}

static int mp_fill(MpArgs& a, long long M, int Dx, int R, int N2) {
  LCI_CHECK(M > 0 && Dx > 0 && Dx % 16 == 0 && Dx <= 1024 && R > 0 && N2 > 0 && N2 % 8 == 0 && R + N2 <= 64,
            "mamba_proj: unsupported shape M=%lld Dx=%d R=%d 2N=%d (Dx %% 16, 2N %% 8, R + 2N <= 64)", M, Dx, R, N2);
  a.M = M; a.Dx = Dx; a.R = R; a.N2 = N2;
  a.Dxp = (Dx + 31) / 32 * 32;
  a.nb1 = (R + N2 + 31) / 32;
  a.ks2 = (R + 15) / 16;
  a.nb3 = (R + 31) / 32;
  a.ks4 = (R + N2 + 15) / 16;
  a.rows_lds = 32 * a.nb1 + 8;   // rows per token in LDS (+8: the row stride is not a multiple of 64 B)
  return 0;
}

}  // namespace lci

using namespace lci;

// Weight images (built by the caller, bf16): w1 (nb1*32, Dx) = Wx rows zero-padded; w2p (Dxp, ks2*16): w2p[d][16 s +
// 8 h + j] = Wdt[d][32 (s >> 1) + 16 (s & 1) + (j & 3) + 8 (j >> 2) + 4 h] (0 past R or Dx); w2t (nb3*32, Dx) = Wdt^T
// zero-padded; w1t (Dxp, ks4*16): w1t[d][r] = Wx[r][d] (0 past R + 2N or Dx). lci_mamba_proj_dims returns
// {Dxp, nb1, ks2, nb3, ks4} for those shapes.
extern "C" int lci_mamba_proj_dims(int Dx, int R, int N2, int* dims) {
  MpArgs a{};
  if (mp_fill(a, 1, Dx, R, N2)) return 1;
  dims[0] = a.Dxp; dims[1] = a.nb1; dims[2] = a.ks2; dims[3] = a.nb3; dims[4] = a.ks4;
  return 0;
}

extern "C" int lci_mamba_proj_fwd(const void* xs, long long ts_x, const void* w1, const void* w2p, const float* bias,
                                  void* dt, long long ts_dt, void* bc, void* dtl, int ld_dtl, long long M, int Dx,
                                  int R, int N2, void* stream) {
  MpArgs a{};
  if (mp_fill(a, M, Dx, R, N2)) return 1;
  LCI_CHECK(ld_dtl % 8 == 0 && ld_dtl >= R && ts_x == Dx && ts_dt == Dx, "mamba_proj_fwd: xs / dt must be (M, Dx) rows");
  LCI_CHECK(((uintptr_t)xs | (uintptr_t)w1 | (uintptr_t)w2p | (uintptr_t)bc | (uintptr_t)dtl) % 16 == 0 &&
            (uintptr_t)dt % 16 == 0, "mamba_proj_fwd: pointers must be 16-byte aligned");
  a.xs = (const bf16*)xs; a.ts_x = ts_x; a.w1 = (const bf16*)w1; a.w2p = (const bf16*)w2p; a.bias = bias;
  a.dt = (bf16*)dt; a.ts_dt = ts_dt; a.bc = (bf16*)bc; a.dtl = (bf16*)dtl; a.ld_dtl = ld_dtl;
  const long long blocks = (M + MP_WAVES * MP_TOK - 1) / (MP_WAVES * MP_TOK);
  const size_t lds = (size_t)MP_WAVES * MP_TOK * (a.rows_lds + a.Dxp + 8) * sizeof(bf16);
  hipLaunchKernelGGL(mamba_proj_fwd_kernel, dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_mamba_proj_bwd(const void* ddt, long long ts_ddt, const void* dbc, const void* w2t,
                                  const void* w1t, const void* du, long long ts_du, void* dxs, long long ts_dxs,
                                  void* dxdbl, int ld_dxdbl, long long M, int Dx, int R, int N2, void* stream) {
  MpArgs a{};
  if (mp_fill(a, M, Dx, R, N2)) return 1;
  LCI_CHECK(ld_dxdbl % 8 == 0 && ld_dxdbl >= R + N2 && ld_dxdbl <= a.rows_lds && ts_ddt == Dx && ts_dxs == Dx &&
            (!du || ts_du == Dx), "mamba_proj_bwd: ddt / dxs / du must be (M, Dx) rows");
  LCI_CHECK(((uintptr_t)ddt | (uintptr_t)w2t | (uintptr_t)w1t | (uintptr_t)dxdbl) % 16 == 0 &&
            ((uintptr_t)dxs | (uintptr_t)du) % 16 == 0 && (uintptr_t)dbc % 2 == 0,
            "mamba_proj_bwd: pointers must be 16-byte aligned");
  a.ddt = (const bf16*)ddt; a.ts_ddt = ts_ddt; a.dbc = (const bf16*)dbc; a.w2t = (const bf16*)w2t; a.w1t = (const bf16*)w1t;
  a.du = (const bf16*)du; a.ts_du = ts_du; a.dxs = (bf16*)dxs; a.ts_dxs = ts_dxs; a.dxdbl = (bf16*)dxdbl;
  a.ld_dxdbl = ld_dxdbl;
  const long long blocks = (M + MP_WAVES * MP_TOK - 1) / (MP_WAVES * MP_TOK);
  const size_t lds = (size_t)MP_WAVES * MP_TOK * (a.rows_lds + a.Dxp + 8) * sizeof(bf16);
  hipLaunchKernelGGL(mamba_proj_bwd_kernel, dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}
