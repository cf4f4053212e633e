// Swin shifted-window attention for gfx950 (head_dim 32).
//
// Replaces WindowAttention.forward (backbone_swin.py:339-359):
//   attn = (q*scale) k^T + rpb_table[rp_index] (+ mask (-100 across regions)); softmax; (attn v)
// and, in GRID mode, the index ops around it in SwinTransformerBlock.forward_part1 (:435-487):
//   F.pad -> torch.roll(-shift) -> window_partition ... window_reverse -> torch.roll(+shift) -> crop,
// evaluated as address arithmetic on the channels-last qkv grid (B, S0, S1[, S2], 3C): window token n of
// window w reads source voxel (p + shift) mod Sp (p = padded coordinate); voxels beyond S are the zero padding,
// whose qkv row is the Linear bias. The -100 mask is recomputed from per-axis region ids exactly as
// compute_mask builds it (:591-628). WINDOWS mode takes pre-partitioned (Bw, N, 3C) and an optional mask.
//
// Additive logit term: every window of one "type" shares rpb + mask, so lci_window_bias builds, once per call,
// a log2-domain bf16 table bias[type][head][q][k] = (rpb[h][q][k] + mask) * log2(e), -1e30 for padded keys/queries
// (grid mode: type = which axes the window is the last one on, when shifted -> <= 8 types; windows mode:
// type = w % nW when a mask is given). The table tile is the INITIAL ACCUMULATOR of the score MFMAs, Q is
// prescaled by scale*log2(e): the chain yields the full log2-domain logit, no per-element bias/mask VALU.
// One workgroup = one (window, head); the whole window's K and V live in LDS; 4 waves x 32-query blocks;
// S^T = K.Q^T with the query on the MFMA lane, online softmax (lazy exact rescale) over 32-key tiles,
// O^T += V^T.P^T.
// Backward: phase 1 (query on lane): dP^T (initial accumulator -delta), dS^T, dQ^T += K^T dS^T, dS tiles for
//           d(rpb); phase 2 (key on lane, Q/dO in LDS, transposed table): dV^T += dO^T P, dK^T += Q^T dS.
//           Pad-token dK/dV go to the qkv bias gradient. d(rpb) = sum over windows of dS (reduction kernel).
#include "common.hpp"

#include <algorithm>
#include <stdlib.h>

// scheduling-strategy hooks for A/B runs (tools/attn_variants.sh): iglp_opt(N) on the fwd / bwd tile loops
#ifdef LCI_WIN_IGLP_FWD
#define LCI_WIN_FWD_SCHED() __builtin_amdgcn_iglp_opt(LCI_WIN_IGLP_FWD)
#else
#define LCI_WIN_FWD_SCHED()
#endif
#ifdef LCI_WIN_IGLP_BWD
#define LCI_WIN_BWD_SCHED() __builtin_amdgcn_iglp_opt(LCI_WIN_IGLP_BWD)
#else
#define LCI_WIN_BWD_SCHED()
#endif

namespace lci {

constexpr int WHD = 32;          // head dim (Swin: C / heads = 32 at every stage)
constexpr int WLD = 40;          // LDS row stride (elements, 80 B): b128 row reads conflict-free
constexpr int WMAXN = 768;       // max tokens per window (LDS: two Npad x 80 B tiles)
constexpr float WLOG2E = 1.4426950408889634f;
constexpr float WNEG = -1.0e30f;

struct WinArgs {
  const bf16* qkv; const float* qkv_bias;  // bias (3C) f32 or null: value of padded tokens
  const float* rpb;                        // (H, N, N) f32 rpb_table[index] (table builder only)
  const float* mask;                       // WINDOWS mode: (nW, N, N) f32 or null (table builder only)
  const bf16* bias;                        // (T, H, Npad, Npad) log2-domain logit term [q][k], bf16
  const bf16* biasT;                       // the same, transposed [k][q] (backward phase 2)
  bf16* out; const bf16* o; const bf16* dout;
  float* lse2;                             // (Bw, H, N)
  bf16* dqkv; float* dbias_pad;            // bwd
  bf16* dS;                                // (Bw, H, nqb, nkt, 64, 16) bf16 tiles or null
  float* drpb;                             // (H, N, N) f32 (reduction kernel)
  int mode, nd, S[3], ws[3], sh[3], Sp[3], nwin[3];
  int Bw, nW, N, Npad, nqb, nkt, C, H, masked, T;
  float scale, c;
};

// token row of window token n (>= 0), -1 for a padded voxel, and its region id (grid mode)
__device__ __forceinline__ int win_row(const WinArgs& a, int w, int n, int& rid) {
  rid = 0;
  if (a.mode == 0) return w * a.N + n;
  const int b = w / a.nW;
  int wi = w % a.nW;
  int widx[3], nidx[3];
  for (int s = a.nd - 1; s >= 0; --s) { widx[s] = wi % a.nwin[s]; wi /= a.nwin[s]; }
  int nn = n;
  for (int s = a.nd - 1; s >= 0; --s) { nidx[s] = nn % a.ws[s]; nn /= a.ws[s]; }
  long long row = b;
  bool pad = false;
  for (int s = 0; s < a.nd; ++s) {
    const int p = widx[s] * a.ws[s] + nidx[s];
    int r = 0;
    if (a.sh[s] > 0) r = p < a.Sp[s] - a.ws[s] ? 0 : (p < a.Sp[s] - a.sh[s] ? 1 : 2);
    rid = rid * 3 + r;
    int src = p + a.sh[s];
    if (src >= a.Sp[s]) src -= a.Sp[s];
    if (src >= a.S[s]) pad = true;
    row = row * a.S[s] + src;
  }
  return pad ? -1 : (int)row;
}

// load 8 bf16 (16 B) of token row `row` at channel offset col, or of the bias for padded tokens
__device__ __forceinline__ bf16x8 win_load8(const WinArgs& a, int row, int col, bool exists) {
  if (!exists) return bf16x8{};
  if (row >= 0) return *(const bf16x8*)(a.qkv + (long long)row * 3 * a.C + col);
  bf16x8 r;
  if (a.qkv_bias) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = to_bf16(a.qkv_bias[col + j]);
  } else {
    r = bf16x8{};
  }
  return r;
}

__device__ __forceinline__ const bf16* out_row_ptr(const WinArgs& a, const bf16* base, int w, int n, int row) {
  return base + (long long)(a.mode == 0 ? w * a.N + n : row) * a.C;
}

struct WinLds {
  bf16* t0; bf16* t1; int* row; int* rid;
};

__device__ __forceinline__ void win_setup(const WinArgs& a, char* smem, WinLds& L, int w) {
  L.t0 = (bf16*)smem;
  L.t1 = L.t0 + a.Npad * WLD;
  L.row = (int*)(L.t1 + a.Npad * WLD);
  L.rid = L.row + a.Npad;
  for (int n = threadIdx.x; n < a.Npad; n += blockDim.x) {
    int rid = 0;
    L.row[n] = n < a.N ? win_row(a, w, n, rid) : -2;
    L.rid[n] = rid;
  }
  __syncthreads();
}

// stage two (Npad x 32) tiles of the window: channel offsets c0, c1 of the token rows (or the bias)
__device__ __forceinline__ bf16x8 win_stage_src1(const WinArgs& a, const WinLds& L, int n, int ch, int c1,
                                                 bool second_is_out, const bf16* obase, int w) {
  const int row = L.row[n];
  const bool ex = n < a.N;
  if (second_is_out)
    return (ex && row != -1) ? *(const bf16x8*)(out_row_ptr(a, obase, w, n, row) + c1 + ch * 8) : bf16x8{};
  return win_load8(a, row, c1 + ch * 8, ex);
}

template <int NT>
__device__ __forceinline__ void win_stage(const WinArgs& a, const WinLds& L, int c0, int c1, bool second_is_out,
                                          const bf16* obase, int w) {
  constexpr int IT = 1536 / NT;   // Npad <= 384 (every Swin window up to 7x7x7): all row loads in flight at once
  const int items = a.Npad * 4;
  if (items <= IT * NT) {
    bf16x8 r0[IT], r1[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = it * NT + threadIdx.x;
      if (idx < items) {
        const int n = idx >> 2, ch = idx & 3;
        r0[it] = win_load8(a, L.row[n], c0 + ch * 8, n < a.N);
        r1[it] = win_stage_src1(a, L, n, ch, c1, second_is_out, obase, w);
      }
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = it * NT + threadIdx.x;
      if (idx < items) {
        const int n = idx >> 2, ch = idx & 3;
        *(bf16x8*)(L.t0 + n * WLD + ch * 8) = r0[it];
        *(bf16x8*)(L.t1 + n * WLD + ch * 8) = r1[it];
      }
    }
  } else {
    for (int idx = threadIdx.x; idx < items; idx += blockDim.x) {
      const int n = idx >> 2, ch = idx & 3;
      *(bf16x8*)(L.t0 + n * WLD + ch * 8) = win_load8(a, L.row[n], c0 + ch * 8, n < a.N);
      *(bf16x8*)(L.t1 + n * WLD + ch * 8) = win_stage_src1(a, L, n, ch, c1, second_is_out, obase, w);
    }
  }
  __syncthreads();
}

// window type (index into the bias table)
__device__ __forceinline__ int win_type(const WinArgs& a, int w) {
  if (a.mode == 0) return a.T > 1 ? w % a.nW : 0;
  if (!a.masked) return 0;
  int wi = w % a.nW, t = 0;
  for (int s = a.nd - 1; s >= 0; --s) {
    const int widx = wi % a.nwin[s];
    wi /= a.nwin[s];
    if (a.sh[s] > 0 && widx == a.nwin[s] - 1) t |= 1 << s;
  }
  return t;
}

// compute_mask's region id (backbone_swin.py:591-628) of window token n in a window of type t
__device__ __forceinline__ int win_region(const WinArgs& a, int t, int n) {
  int nidx[3] = {0, 0, 0};
  for (int s = a.nd - 1; s >= 0; --s) { nidx[s] = n % a.ws[s]; n /= a.ws[s]; }
  int rid = 0;
  for (int s = 0; s < a.nd; ++s) rid = rid * 3 + (((t >> s) & 1) ? (nidx[s] < a.ws[s] - a.sh[s] ? 1 : 2) : 0);
  return rid;
}

// One workgroup = a 32 (q) x 32 (k) tile of one (type, head). The region ids of the tile's 32 queries and 32 keys
// are computed once into LDS; a thread evaluates 4 consecutive keys of one query and writes them as one 8-byte
// chunk of a bias row; the transposed tile goes through LDS so biasT rows are written the same way. (The first
// version, one thread per element with two region evaluations each and 2-byte strided biasT stores, took 26-188 us
// per shifted call at the C3 stages.)
constexpr int WBT_LD = 36;   // LDS row stride of the transposed tile (elements): 8-byte aligned rows
__global__ __launch_bounds__(256) void win_bias_kernel(WinArgs a, bf16* bias, bf16* biasT) {
  __shared__ int rq[32], rk[32];
  __shared__ __attribute__((aligned(8))) bf16 sT[32 * WBT_LD];
  const int nt = a.Npad / 32;
  int b = blockIdx.x;
  const int kt = b % nt;
  b /= nt;
  const int qt = b % nt, th = b / nt;   // th = t * H + h
  const int h = th % a.H, t = th / a.H;
  const int tid = threadIdx.x;
  const bool regions = a.mode == 1 && a.masked;
  if (tid < 64) {
    const int n = (tid < 32 ? qt : kt) * 32 + (tid & 31);
    const int r = (regions && n < a.N) ? win_region(a, t, n) : 0;
    if (tid < 32) rq[tid] = r; else rk[tid - 32] = r;
  }
  __syncthreads();
  const int ql = tid >> 3, kl = (tid & 7) * 4;
  const int q = qt * 32 + ql;
  const long long np = a.Npad;
  bf16x4 v4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = kt * 32 + kl + j;
    float v = WNEG;
    if (q < a.N && k < a.N) {
      v = a.rpb[((long long)h * a.N + q) * a.N + k];
      if (a.mode == 0 && a.mask) v += a.mask[((long long)t * a.N + q) * a.N + k];
      if (regions && rq[ql] != rk[kl + j]) v += -100.f;
      v *= WLOG2E;
    }
    v4[j] = to_bf16(v);
    sT[(kl + j) * WBT_LD + ql] = v4[j];
  }
  if (bias) *(bf16x4*)(bias + ((long long)th * np + q) * np + kt * 32 + kl) = v4;
  if (biasT) {   // uniform per launch
    __syncthreads();
    const int kr = tid >> 3, qc = (tid & 7) * 4;
    *(bf16x4*)(biasT + ((long long)th * np + kt * 32 + kr) * np + qt * 32 + qc) = *(const bf16x4*)(sT + kr * WBT_LD + qc);
  }
}

// 16 table values of one 32x32 score tile for this lane: row r (q or key, the lane's), columns
// c0 + 8g + 4h + j  ->  register 4g + j (the 32x32x16 accumulator layout). The table is bf16 (|rpb| ~ 0.02 and
// the -100 mask lose nothing that matters at bf16 score precision): half the bytes of an f32 table, and the
// tables of one head (all window types) stay L2-resident while that head's windows run.
__device__ __forceinline__ f32x16 win_bias_tile(const bf16* row, int c0) {
  f32x16 r;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const u32x2 v = *(const u32x2*)(row + c0 + 8 * g);
    r[4 * g + 0] = __uint_as_float(v[0] << 16);
    r[4 * g + 1] = __uint_as_float(v[0] & 0xffff0000u);
    r[4 * g + 2] = __uint_as_float(v[1] << 16);
    r[4 * g + 3] = __uint_as_float(v[1] & 0xffff0000u);
  }
  return r;
}

__device__ __forceinline__ bf16x8 scaled8(bf16x8 v, float c) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = to_bf16(to_f32(v[j]) * c);
  return v;
}

// --------------------------------------------------------------------------------------------- forward
template <int NW>
__global__ __launch_bounds__(NW * 64) void win_attn_fwd_kernel(WinArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = blockIdx.x, hh = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  WinLds L;
  win_setup(a, smem, L, w);
  win_stage<NW * 64>(a, L, a.C + hh * WHD, 2 * a.C + hh * WHD, false, nullptr, w);   // K -> t0, V -> t1
  const float c = a.c;
  const bf16* bh = a.bias + ((long long)win_type(a, w) * a.H + hh) * a.Npad * a.Npad;
  bf16x8 qn[2];   // next query block's Q, loaded one block ahead
  auto load_q = [&](int qb) {
    const int q = qb * 32 + (lane & 31);
    const bool qv = q < a.N;
    const int qrow = qv ? L.row[q] : -2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qn[ks] = win_load8(a, qrow, hh * WHD + ks * 16 + 8 * half, qv);
  };
  if (wave < a.nqb) load_q(wave);
  for (int qb = wave; qb < a.nqb; qb += NW) {
    const int q = qb * 32 + (lane & 31);
    const bool qv = q < a.N;
    const int qrow = qv ? L.row[q] : -2;
    const bf16x8 qf[2] = {scaled8(qn[0], c), scaled8(qn[1], c)};
    if (qb + NW < a.nqb) load_q(qb + NW);
    const bf16* brow = bh + (long long)q * a.Npad + 4 * half;
    f32x16 o = {};
    float m = 0.f, l = 0.f;
    f32x16 b0 = win_bias_tile(brow, 0), b1;   // table tiles two ahead
    if (a.nkt > 1) b1 = win_bias_tile(brow, 32);
    for (int kt = 0; kt < a.nkt; ++kt) {
      LCI_WIN_FWD_SCHED();
      f32x16 s = b0;
      b0 = b1;
      if (kt + 2 < a.nkt) b1 = win_bias_tile(brow, (kt + 2) * 32);
      s = mfma32(frag_row(L.t0, WLD, kt * 32, 0, lane), qf[0], s);
      s = mfma32(frag_row(L.t0, WLD, kt * 32, 16, lane), qf[1], s);
      float m4[4] = {fmaxf(s[0], s[1]), fmaxf(s[2], s[3]), fmaxf(s[4], s[5]), fmaxf(s[6], s[7])};
#pragma unroll
      for (int i = 8; i < 16; i += 4) {
        m4[0] = fmaxf(m4[0], s[i]);
        m4[1] = fmaxf(m4[1], s[i + 1]);
        m4[2] = fmaxf(m4[2], s[i + 2]);
        m4[3] = fmaxf(m4[3], s[i + 3]);
      }
      const float mx = wave_max_xor32(fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3])));
      if (kt == 0 || __any(mx > m)) {   // lazy exact rescale (alpha == 1 otherwise)
        const float mn = kt == 0 ? mx : fmaxf(m, mx);
        if (kt != 0) {
          const float al = exp2_fast(m - mn);
          l *= al;
#pragma unroll
          for (int i = 0; i < 16; ++i) o[i] *= al;
        }
        m = mn;
      }
      float l4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s[i] = exp2_fast(s[i] - m);
        l4[i & 3] += s[i];
      }
      l += (l4[0] + l4[1]) + (l4[2] + l4[3]);
      o = mfma32(frag_tr<0>(L.t1, WLD, kt * 32, 0, lane), pack8<0>(s), o);
      o = mfma32(frag_tr<1>(L.t1, WLD, kt * 32, 0, lane), pack8<1>(s), o);
    }
    const float lt = wave_sum_xor32(l);
    const float inv = 1.f / lt;
    if (qv && qrow != -1) {
      bf16* op = (bf16*)out_row_ptr(a, a.out, w, q, qrow) + hh * WHD;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = to_bf16(o[4 * g + j] * inv);
        *(bf16x4*)(op + 8 * g + 4 * half) = v;
      }
    }
    if (qv && half == 0) a.lse2[((long long)w * a.H + hh) * a.N + q] = m + __log2f(lt);
  }
}

// -------------------------------------------------------------------------------------------- backward
template <int NW>
__global__ __launch_bounds__(NW * 64) void win_attn_bwd_kernel(WinArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = blockIdx.x, hh = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  WinLds L;
  win_setup(a, smem, L, w);
  float* lse_l = (float*)(L.rid + a.Npad);
  float* ndl_l = lse_l + a.Npad;   // -delta
  const float c = a.c;
  const long long tho = ((long long)win_type(a, w) * a.H + hh) * a.Npad * a.Npad;
  const float* lseg = a.lse2 + ((long long)w * a.H + hh) * a.N;

  // ---------------- phase 1: K, V in LDS; query on the lane -> dQ, dS tiles, delta
  win_stage<NW * 64>(a, L, a.C + hh * WHD, 2 * a.C + hh * WHD, false, nullptr, w);
  for (int qb = wave; qb < a.nqb; qb += NW) {
    const int q = qb * 32 + (lane & 31);
    const bool qv = q < a.N;
    const int qrow = qv ? L.row[q] : -2;
    bf16x8 qf[2], df[2];
    float dsum = 0.f;
    const bool has_out = qv && qrow != -1;   // padded queries are cropped: dO = 0
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[ks] = scaled8(win_load8(a, qrow, hh * WHD + ks * 16 + 8 * half, qv), c);
      if (has_out) {
        df[ks] = *(const bf16x8*)(out_row_ptr(a, a.dout, w, q, qrow) + hh * WHD + ks * 16 + 8 * half);
        const bf16x8 ov = *(const bf16x8*)(out_row_ptr(a, a.o, w, q, qrow) + hh * WHD + ks * 16 + 8 * half);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum = fmaf(to_f32(df[ks][j]), to_f32(ov[j]), dsum);
      } else {
        df[ks] = bf16x8{};
      }
    }
    const float delta = wave_sum_xor32(dsum);
    const float lse = qv ? lseg[q] : 0.f;   // invalid lanes: every table entry is -1e30 -> P = 0
    if (half == 0) {
      lse_l[q] = qv ? lse : 1.0e30f;
      ndl_l[q] = -delta;
    }
    f32x16 ndl;
#pragma unroll
    for (int i = 0; i < 16; ++i) ndl[i] = -delta;
    const bf16* brow = a.bias + tho + (long long)q * a.Npad + 4 * half;
    f32x16 dq = {};
    f32x16 b0 = win_bias_tile(brow, 0), b1;
    if (a.nkt > 1) b1 = win_bias_tile(brow, 32);
    for (int kt = 0; kt < a.nkt; ++kt) {
      LCI_WIN_BWD_SCHED();
      f32x16 s = b0;
      b0 = b1;
      if (kt + 2 < a.nkt) b1 = win_bias_tile(brow, (kt + 2) * 32);
      s = mfma32(frag_row(L.t0, WLD, kt * 32, 0, lane), qf[0], s);
      s = mfma32(frag_row(L.t0, WLD, kt * 32, 16, lane), qf[1], s);
      f32x16 dp = mfma32(frag_row(L.t1, WLD, kt * 32, 0, lane), df[0], ndl);
      dp = mfma32(frag_row(L.t1, WLD, kt * 32, 16, lane), df[1], dp);
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = exp2_fast(s[i] - lse) * dp[i];   // dS^T (natural-log units)
      const bf16x8 lo = pack8<0>(s), hi = pack8<1>(s);
      if (a.dS) {
        bf16* dst = a.dS + ((((long long)w * a.H + hh) * a.nqb + qb) * a.nkt + kt) * 1024 + lane * 16;
        *(bf16x8*)dst = lo;
        *(bf16x8*)(dst + 8) = hi;
      }
      dq = mfma32(frag_tr<0>(L.t0, WLD, kt * 32, 0, lane), lo, dq);
      dq = mfma32(frag_tr<1>(L.t0, WLD, kt * 32, 0, lane), hi, dq);
    }
    if (qv && qrow >= 0) {
      bf16* dqp = a.dqkv + (long long)(a.mode == 0 ? w * a.N + q : qrow) * 3 * a.C + hh * WHD;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = to_bf16(dq[4 * g + j] * a.scale);
        *(bf16x4*)(dqp + 8 * g + 4 * half) = v;
      }
    }
  }
  for (int n = a.N + threadIdx.x; n < a.Npad; n += blockDim.x) { lse_l[n] = 1.0e30f; ndl_l[n] = 0.f; }
  __syncthreads();

  // ---------------- phase 2: Q, dO in LDS; key on the lane -> dK, dV
  win_stage<NW * 64>(a, L, hh * WHD, hh * WHD, true, a.dout, w);   // Q -> t0, dO -> t1
  for (int kb = wave; kb < a.nqb; kb += NW) {
    const int key = kb * 32 + (lane & 31);
    const bool kv = key < a.N;
    const int krow = kv ? L.row[key] : -2;
    bf16x8 kf[2], vf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kf[ks] = scaled8(win_load8(a, krow, a.C + hh * WHD + ks * 16 + 8 * half, kv), c);
      vf[ks] = win_load8(a, krow, 2 * a.C + hh * WHD + ks * 16 + 8 * half, kv);
    }
    const bf16* brow = a.biasT + tho + (long long)key * a.Npad + 4 * half;
    f32x16 dk = {}, dv = {};
    f32x16 b0 = win_bias_tile(brow, 0), b1;
    if (a.nkt > 1) b1 = win_bias_tile(brow, 32);
    for (int qt = 0; qt < a.nkt; ++qt) {
      LCI_WIN_BWD_SCHED();
      f32x16 s = b0;
      b0 = b1;
      if (qt + 2 < a.nkt) b1 = win_bias_tile(brow, (qt + 2) * 32);
      f32x16 dp, lz;
#pragma unroll
      for (int g = 0; g < 4; ++g) {   // row constants of queries qt*32 + 8g + 4h + j
        const f32x4 l4 = *(const f32x4*)(lse_l + qt * 32 + 8 * g + 4 * half);
        const f32x4 d4 = *(const f32x4*)(ndl_l + qt * 32 + 8 * g + 4 * half);
#pragma unroll
        for (int j = 0; j < 4; ++j) { lz[4 * g + j] = l4[j]; dp[4 * g + j] = d4[j]; }
      }
      s = mfma32(frag_row(L.t0, WLD, qt * 32, 0, lane), kf[0], s);
      s = mfma32(frag_row(L.t0, WLD, qt * 32, 16, lane), kf[1], s);
      dp = mfma32(frag_row(L.t1, WLD, qt * 32, 0, lane), vf[0], dp);
      dp = mfma32(frag_row(L.t1, WLD, qt * 32, 16, lane), vf[1], dp);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s[i] = exp2_fast(s[i] - lz[i]);   // P (query rows, key on lane)
        dp[i] = s[i] * dp[i];             // dS
      }
      dv = mfma32(frag_tr<0>(L.t1, WLD, qt * 32, 0, lane), pack8<0>(s), dv);
      dv = mfma32(frag_tr<1>(L.t1, WLD, qt * 32, 0, lane), pack8<1>(s), dv);
      dk = mfma32(frag_tr<0>(L.t0, WLD, qt * 32, 0, lane), pack8<0>(dp), dk);
      dk = mfma32(frag_tr<1>(L.t0, WLD, qt * 32, 0, lane), pack8<1>(dp), dk);
    }
    if (kv) {
      if (krow >= 0) {
        bf16* base = a.dqkv + (long long)(a.mode == 0 ? w * a.N + key : krow) * 3 * a.C + hh * WHD;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 v0, v1;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v0[j] = to_bf16(dk[4 * g + j] * a.scale);
            v1[j] = to_bf16(dv[4 * g + j]);
          }
          *(bf16x4*)(base + a.C + 8 * g + 4 * half) = v0;
          *(bf16x4*)(base + 2 * a.C + 8 * g + 4 * half) = v1;
        }
      }
    }
    // padded voxels: their k, v are the qkv bias. All padded keys of the wave target the same 2 x 32 words,
    // so sum over the 32 key lanes of each half first (one atomic per word per wave instead of one per key:
    // per-key atomics serialised on 192 addresses cost ~37 ms at Swin-tiny stage 1, 128^3)
    const bool padk = kv && krow < 0 && a.dbias_pad != nullptr;
    if (__any(padk)) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float sk = padk ? dk[i] * a.scale : 0.f, sv = padk ? dv[i] : 0.f;
#pragma unroll
        for (int o = 16; o >= 1; o >>= 1) {
          sk += __shfl_xor(sk, o);
          sv += __shfl_xor(sv, o);
        }
        if ((lane & 31) == 0) {
          const int d = 8 * (i >> 2) + 4 * half + (i & 3);
          atomicAdd(a.dbias_pad + a.C + hh * WHD + d, sk);
          atomicAdd(a.dbias_pad + 2 * a.C + hh * WHD + d, sv);
        }
      }
    }
  }
}

// d(rpb)[h][q][k] = sum_w dS[w][h][q][k]  from the (Bw, H, nqb, nkt, 64, 16) tile layout. A thread owns 8
// consecutive tile elements (one 16-byte load per window) and sums the windows in a fixed order, 8 loads in flight
// (the v1 kernel read 2 bytes per lane per window with one load in flight). Deterministic.
__global__ __launch_bounds__(128) void win_rpb_grad_kernel(WinArgs a) {
  const long long per_w = (long long)a.H * a.nqb * a.nkt * 1024;
  const long long e8 = (blockIdx.x * 128LL + threadIdx.x) * 8;
  if (e8 >= per_w) return;
  const bf16* p = a.dS + e8;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  int w = 0;
  for (; w + 8 <= a.Bw; w += 8) {
    bf16x8 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *(const bf16x8*)(p + (w + u) * per_w);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc[j] += ((to_f32(v[0][j]) + to_f32(v[1][j])) + (to_f32(v[2][j]) + to_f32(v[3][j]))) +
                ((to_f32(v[4][j]) + to_f32(v[5][j])) + (to_f32(v[6][j]) + to_f32(v[7][j])));
  }
  for (; w < a.Bw; ++w) {
    const bf16x8 v = *(const bf16x8*)(p + w * per_w);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += to_f32(v[j]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const long long e = e8 + j;
    const int i = e & 15, lane = (e >> 4) & 63;
    long long t = e >> 10;
    const int kt = t % a.nkt; t /= a.nkt;
    const int qb = t % a.nqb;
    const int hh = t / a.nqb;
    const int q = qb * 32 + (lane & 31);
    const int k = kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
    if (q < a.N && k < a.N) a.drpb[((long long)hh * a.N + q) * a.N + k] = acc[j];
  }
}

// Index-map export (tests): for every window w and window token n, the source token row win_row() reads and the
// output scatters to (-1 = padded voxel), the region id win_row() derives on the padded grid, and the window type
// win_type() selects the bias table with, plus win_region() of the token under that type -- the same __device__
// functions the attention kernels and the table builder call.
__global__ __launch_bounds__(256) void win_index_map_kernel(WinArgs a, int* src_row, int* region, int* rid_out,
                                                            int* wtype) {
  const long long e = blockIdx.x * 256LL + threadIdx.x;
  if (e >= (long long)a.Bw * a.N) return;
  const int w = (int)(e / a.N), n = (int)(e % a.N);
  int rid = 0;
  src_row[e] = win_row(a, w, n, rid);
  const int t = win_type(a, w);
  region[e] = win_region(a, t, n);
  rid_out[e] = rid;
  if (n == 0) wtype[w] = t;
}

// Window gather / scatter for the Hyena / Mamba mixers inside Swin windows (backbone_swin.py:445-487 with
// WindowAttention :361-365): F.pad -> roll(-shift) -> window_partition as one gather of 16-byte row chunks
// (padded voxels read as zeros: the reference pads the LayerNorm output with zeros), window_reverse -> roll(+shift)
// -> crop as the inverse scatter. Both use win_row(), so the maps are the ones the attention kernels use (and
// lci_window_index_map exports). One thread per (window token, 16-byte chunk); rows of C * elem_bytes bytes.
__global__ __launch_bounds__(256) void win_gather_kernel(WinArgs a, const char* src, char* dst, int row_bytes,
                                                         int scatter) {
  const int nch = row_bytes / 16;
  const long long total = (long long)a.Bw * a.N * nch;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int ch = (int)(e % nch);
    const long long wn = e / nch;
    const int w = (int)(wn / a.N), n = (int)(wn % a.N);
    int rid;
    const int row = win_row(a, w, n, rid);
    char* wp = (scatter ? (char*)src : dst) + wn * row_bytes + 16 * ch;   // window-token row
    if (scatter) {
      if (row >= 0) *(u32x4*)(dst + (long long)row * row_bytes + 16 * ch) = *(const u32x4*)wp;
    } else {
      *(u32x4*)wp = row >= 0 ? *(const u32x4*)(src + (long long)row * row_bytes + 16 * ch) : u32x4{0u, 0u, 0u, 0u};
    }
  }
}

static int win_fill(WinArgs& a, const int* geo, float scale) {
  // geo: [mode, nd, S0, S1, S2, ws0, ws1, ws2, sh0, sh1, sh2, Bw_or_B, nW, N, C, H]
  a.mode = geo[0]; a.nd = geo[1];
  for (int s = 0; s < 3; ++s) { a.S[s] = geo[2 + s]; a.ws[s] = geo[5 + s]; a.sh[s] = geo[8 + s]; }
  a.N = geo[13]; a.C = geo[14]; a.H = geo[15];
  LCI_CHECK(a.C == a.H * WHD, "window_attn: C %d != heads %d * 32", a.C, a.H);
  LCI_CHECK(a.N > 0 && a.N <= WMAXN, "window_attn: N %d unsupported (<= %d)", a.N, WMAXN);
  a.masked = 0;
  if (a.mode == 1) {
    int nW = 1, N = 1;
    for (int s = 0; s < a.nd; ++s) {
      LCI_CHECK(a.ws[s] > 0 && a.S[s] > 0 && a.sh[s] >= 0 && a.sh[s] < a.ws[s], "window_attn: bad geometry");
      a.Sp[s] = (a.S[s] + a.ws[s] - 1) / a.ws[s] * a.ws[s];
      a.nwin[s] = a.Sp[s] / a.ws[s];
      nW *= a.nwin[s]; N *= a.ws[s];
      if (a.sh[s] > 0) a.masked = 1;
    }
    LCI_CHECK(N == a.N, "window_attn: N %d != prod(window) %d", a.N, N);
    a.nW = nW; a.Bw = geo[11] * nW;
    a.T = a.masked ? (1 << a.nd) : 1;
  } else {
    a.Bw = geo[11]; a.nW = geo[12] > 0 ? geo[12] : 1;
    a.T = 1;   // lci_window_bias / _elems set T = nW when a mask is given
  }
  a.Npad = (a.N + 31) / 32 * 32;
  a.nqb = a.nkt = a.Npad / 32;
  a.scale = scale; a.c = scale * WLOG2E;
  return 0;
}

static size_t win_lds(const WinArgs& a, bool bwd) {
  return (size_t)a.Npad * WLD * 2 * 2 + (size_t)a.Npad * 4 * 2 + (bwd ? (size_t)a.Npad * 4 * 2 : 0);
}

}  // namespace lci

using namespace lci;

extern "C" long long lci_window_bias_elems(const int* geo, int has_mask) {
  WinArgs a{};
  if (win_fill(a, geo, 1.f)) return -1;
  if (a.mode == 0 && has_mask) a.T = a.nW;
  return (long long)a.T * a.H * a.Npad * a.Npad;
}

extern "C" int lci_window_bias(const float* rpb, const float* mask, void* bias, void* biasT, const int* geo,
                               void* stream) {
  WinArgs a{};
  if (win_fill(a, geo, 1.f)) return 1;
  a.rpb = rpb; a.mask = mask;
  if (a.mode == 0 && mask) a.T = a.nW;
  LCI_CHECK(bias || biasT, "window_bias: no output");
  LCI_CHECK(((uintptr_t)bias & 7) == 0 && ((uintptr_t)biasT & 7) == 0, "window_bias: tables must be 8-byte aligned");
  const long long nt = a.Npad / 32, n = (long long)a.T * a.H * nt * nt;
  LCI_CHECK(n < (1LL << 31), "window_bias: table too large");
  hipLaunchKernelGGL(win_bias_kernel, dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream, a, (bf16*)bias,
                     (bf16*)biasT);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_window_attn_fwd(const void* qkv, const float* qkv_bias, const void* bias, int has_mask,
                                   void* out, float* lse2, const int* geo, float scale, void* stream) {
  WinArgs a{};
  if (win_fill(a, geo, scale)) return 1;
  if (a.mode == 0 && has_mask) a.T = a.nW;
  a.qkv = (const bf16*)qkv; a.qkv_bias = qkv_bias; a.bias = (const bf16*)bias; a.out = (bf16*)out; a.lse2 = lse2;
  constexpr int NW = 8;   // 8 waves share the window's K/V: 4 waves per SIMD at 2 workgroups per CU (LDS-bound)
  (void)hipFuncSetAttribute((const void*)win_attn_fwd_kernel<NW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  hipLaunchKernelGGL(win_attn_fwd_kernel<NW>, dim3(a.Bw, a.H), dim3(NW * 64), win_lds(a, false), (hipStream_t)stream,
                     a);
  LCI_LAUNCH_CHECK();
  return 0;
}

// dbias_pad (3C) accumulated (caller zeroes); dS tiles (Bw*H*nqb*nkt*1024 bf16) optional workspace;
// drpb (H, N, N) f32 written when dS and drpb are given.
extern "C" int lci_window_attn_bwd(const void* qkv, const float* qkv_bias, const void* bias, const void* biasT,
                                   int has_mask, const void* out, const void* dout, const float* lse2, void* dqkv,
                                   float* dbias_pad, void* dS, float* drpb, const int* geo, float scale,
                                   void* stream) {
  WinArgs a{};
  if (win_fill(a, geo, scale)) return 1;
  if (a.mode == 0 && has_mask) a.T = a.nW;
  a.qkv = (const bf16*)qkv; a.qkv_bias = qkv_bias; a.bias = (const bf16*)bias; a.biasT = (const bf16*)biasT; a.o = (const bf16*)out;
  a.dout = (const bf16*)dout; a.lse2 = (float*)lse2; a.dqkv = (bf16*)dqkv; a.dbias_pad = dbias_pad;
  a.dS = (bf16*)dS; a.drpb = drpb;
  hipStream_t s = (hipStream_t)stream;
  // waves per (window, head) workgroup (LCI_WIN_BWD_WAVES: A/B override)
  static const int nw_env = getenv("LCI_WIN_BWD_WAVES") ? atoi(getenv("LCI_WIN_BWD_WAVES")) : 4;
  if (nw_env == 8) {
    (void)hipFuncSetAttribute((const void*)win_attn_bwd_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    hipLaunchKernelGGL(win_attn_bwd_kernel<8>, dim3(a.Bw, a.H), dim3(512), win_lds(a, true), s, a);
  } else {
    (void)hipFuncSetAttribute((const void*)win_attn_bwd_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    hipLaunchKernelGGL(win_attn_bwd_kernel<4>, dim3(a.Bw, a.H), dim3(256), win_lds(a, true), s, a);
  }
  LCI_LAUNCH_CHECK();
  if (dS && drpb) {
    const long long per_w = (long long)a.H * a.nqb * a.nkt * 1024;
    hipLaunchKernelGGL(win_rpb_grad_kernel, dim3((unsigned)((per_w / 8 + 127) / 128)), dim3(128), 0, s, a);
    LCI_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" long long lci_window_dS_elems(const int* geo) {
  WinArgs a{};
  if (win_fill(a, geo, 1.f)) return -1;
  return (long long)a.Bw * a.H * a.nqb * a.nkt * 1024;
}

extern "C" int lci_window_index_map(const int* geo, int* src_row, int* region, int* rid, int* wtype, void* stream) {
  WinArgs a{};
  if (win_fill(a, geo, 1.f)) return 1;
  LCI_CHECK(src_row && region && rid && wtype, "window_index_map: null output");
  const long long n = (long long)a.Bw * a.N;
  hipLaunchKernelGGL(win_index_map_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a,
                     src_row, region, rid, wtype);
  LCI_LAUNCH_CHECK();
  return 0;
}

// Grid-mode window gather (scatter = 0): win (Bw, N, C) <- grid (B, S0, S1[, S2], C) with zero rows for padded
// voxels; scatter (= 1): grid <- win for every non-padded window token (each grid row written exactly once).
// elem_bytes 2 or 4; C * elem_bytes % 16 == 0; geo as lci_window_attn_fwd (mode 1; its C / H fields unused).
extern "C" int lci_window_gather(const void* src, void* dst, int elem_bytes, const int* geo, int scatter,
                                 void* stream) {
  LCI_CHECK(geo[0] == 1, "window_gather: grid mode only");
  int g[16];
  for (int i = 0; i < 16; ++i) g[i] = geo[i];
  const int C = geo[14];
  LCI_CHECK(C > 0 && (elem_bytes == 2 || elem_bytes == 4) && (C * elem_bytes) % 16 == 0,
            "window_gather: C %d x %d bytes must be a multiple of 16", C, elem_bytes);
  LCI_CHECK(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, "window_gather: pointers must be 16-byte aligned");
  g[14] = WHD; g[15] = 1;   // win_fill's head-dim check does not apply to a plain gather
  WinArgs a{};
  if (win_fill(a, g, 1.f)) return 1;
  const long long n = (long long)a.Bw * a.N * (C * elem_bytes / 16);
  const unsigned blocks = (unsigned)std::min<long long>((n + 255) / 256, 65536LL);
  hipLaunchKernelGGL(win_gather_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a, (const char*)src,
                     (char*)dst, C * elem_bytes, scatter);
  LCI_LAUNCH_CHECK();
  return 0;
}
