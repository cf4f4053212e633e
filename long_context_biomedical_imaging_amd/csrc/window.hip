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
// Backward (windows of <= 12 key blocks, win_attn_bwd1_kernel): single phase, one wave per key block, query tiles
//           in a rotation with dQ accumulated in LDS (see the kernel). Larger windows, two phases: phase 1 (query on
//           lane): dP^T (initial accumulator -delta), dS^T, dQ^T += K^T dS^T, dS tiles for d(rpb); phase 2 (key on
//           lane, Q/dO in LDS, transposed table): dV^T += dO^T P, dK^T += Q^T dS.
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
  float* pad_ws;                           // bwd1: (Bw, H, 64) per-workgroup pad-key dK | dV sums, or null
  bf16* dS;                                // (Bw, H, nqb, nkt, 64, 16) bf16 tiles or null
  float* drpb;                             // (H, N, N) f32 (reduction kernel)
  int mode, nd, S[3], ws[3], sh[3], Sp[3], nwin[3];
  int Bw, nW, N, Npad, nqb, nkt, C, H, masked, T;
  int dS_kl;                               // dS tiles in the key-on-lane layout (win_attn_bwd1_kernel)
  int bwd1_cnt;                            // win_attn_bwd1_kernel: per-tile dQ order counters instead of a barrier
  int order;                               // workgroup -> (window, head) order of the attention kernels (win_item)
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

__device__ __forceinline__ const bf16* out_row_ptr(const WinArgs& a, const bf16* base, int w, int n, int row) {
  return base + (long long)(a.mode == 0 ? w * a.N + n : row) * a.C;
}

// (window, head) of attention workgroup blockIdx.x (1-D grid of Bw * H). order 1 (default, round 6): in super-blocks of
// 8 windows x H heads, workgroup b = 8 H g + 8 hh + i is window 8 g + i, head hh -- the dispatcher deals workgroup b
// to XCD b % 8 (observed round-robin; nothing depends on it for correctness), so the H heads of a window run back to
// back on one XCD and their 64-byte pieces of the same token rows (q | k | v of 3C-channel qkv rows, the C-channel
// out / dout rows) meet in that XCD's L2 instead of being fetched from HBM H times, 1000 windows apart. The last,
// partial super-block (Bw % 8 windows) is head-major. order 0: the round-5 (window, head) grid order.
__device__ __forceinline__ void win_item(const WinArgs& a, int& w, int& hh) {
  const int b = blockIdx.x;
  if (a.order == 0) { w = b % a.Bw; hh = b / a.Bw; return; }
  const int G = a.Bw / 8, full = G * 8 * a.H;
  if (b < full) {
    const int g = b / (8 * a.H), r = b - g * 8 * a.H;
    w = 8 * g + (r & 7);
    hh = r >> 3;
  } else {
    const int rem = a.Bw - 8 * G, r = b - full;
    w = 8 * G + r % rem;
    hh = r / rem;
  }
}

struct WinLds {
  bf16* t0; bf16* t1; int* row; int* rid;
  const bf16* bias;   // the head's q | k | v bias, bf16 (3 x 32): the value of padded voxels' qkv rows
  int hoff;           // hh * WHD
};

constexpr int WBIAS_B = 256;   // LDS bytes ahead of t0: the head's bf16 qkv bias (192 B)

// 16 zero bytes: the source of the staging loads of rows that do not exist (loads are branch-free pointer selects)
__device__ __attribute__((aligned(16))) bf16 kWinZero[8];

// load 8 bf16 (16 B) of token row `row` at channel offset col (q | k | v block of the 3C-channel row), or of the bias
// for padded tokens -- from the LDS copy win_setup made. Branch-free: the global load reads the row or 16 zero bytes,
// the LDS read the bias, and a select picks. (With the f32 bias loaded and converted inside a padded-voxel branch, and
// the row loads in exec-masked branches, the compiler placed vmcnt(0) waits inside those branches: every staging load
// of the prologue waited for the previous ones; round 6.)
__device__ __forceinline__ bf16x8 win_load8(const WinArgs& a, const WinLds& L, int row, int col, bool exists) {
  const bf16* src = exists && row >= 0 ? a.qkv + (long long)row * 3 * a.C + col : kWinZero;
  const bf16x8 g = *(const bf16x8*)src;
  const int which = col >= 2 * a.C ? 2 : (col >= a.C ? 1 : 0);
  const bf16x8 b = *(const bf16x8*)(L.bias + which * WHD + (col - which * a.C - L.hoff));
  return exists && row < 0 ? b : g;
}

__device__ __forceinline__ void win_setup(const WinArgs& a, char* smem, WinLds& L, int w, int hh) {
  bf16* bl = (bf16*)smem;
  L.bias = bl;
  L.hoff = hh * WHD;
  L.t0 = (bf16*)(smem + WBIAS_B);
  L.t1 = L.t0 + a.Npad * WLD;
  L.row = (int*)(L.t1 + a.Npad * WLD);
  L.rid = L.row + a.Npad;
  // the bias values are loaded first (their latency under the row map's integer math), stored after it
  const int bi = threadIdx.x < 3 * WHD ? threadIdx.x : 0;
  const float bv = *(a.qkv_bias ? a.qkv_bias + (bi / WHD) * a.C + hh * WHD + bi % WHD : (const float*)kWinZero);
  for (int n = threadIdx.x; n < a.Npad; n += blockDim.x) {
    int rid = 0;
    L.row[n] = n < a.N ? win_row(a, w, n, rid) : -2;
    L.rid[n] = rid;
  }
  if (threadIdx.x < 3 * WHD) bl[threadIdx.x] = to_bf16(bv);
  for (int i = threadIdx.x + blockDim.x; i < 3 * WHD; i += blockDim.x)   // (workgroups of fewer than 96 threads)
    bl[i] = a.qkv_bias ? to_bf16(a.qkv_bias[(i / WHD) * a.C + hh * WHD + i % WHD]) : to_bf16(0.f);
  __syncthreads();
}

// stage two (Npad x 32) tiles of the window: channel offsets c0, c1 of the token rows (or the bias)
__device__ __forceinline__ bf16x8 win_stage_src1(const WinArgs& a, const WinLds& L, int n, int ch, int c1,
                                                 bool second_is_out, const bf16* obase, int w) {
  const int row = L.row[n];
  const bool ex = n < a.N;
  if (second_is_out)
    return *(const bf16x8*)(ex && row != -1 ? out_row_ptr(a, obase, w, n, row) + c1 + ch * 8 : kWinZero);
  return win_load8(a, L, row, c1 + ch * 8, ex);
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
        r0[it] = win_load8(a, L, L.row[n], c0 + ch * 8, n < a.N);
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
      *(bf16x8*)(L.t0 + n * WLD + ch * 8) = win_load8(a, L, L.row[n], c0 + ch * 8, n < a.N);
      *(bf16x8*)(L.t1 + n * WLD + ch * 8) = win_stage_src1(a, L, n, ch, c1, second_is_out, obase, w);
    }
  }
  __syncthreads();
}

// Runtime-width variant (blockDim.x threads, e.g. one wave per 32-token block): up to 4 row chunks per thread in
// flight before the LDS writes.
__device__ __forceinline__ void win_stage_rt(const WinArgs& a, const WinLds& L, int c0, int c1, bool second_is_out,
                                             const bf16* obase, int w) {
  const int items = a.Npad * 4, NT = blockDim.x;
  for (int base = 0; base < items; base += 4 * NT) {
    bf16x8 r0[4], r1[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = base + it * NT + threadIdx.x;
      if (idx < items) {
        const int n = idx >> 2, ch = idx & 3;
        r0[it] = win_load8(a, L, L.row[n], c0 + ch * 8, n < a.N);
        r1[it] = win_stage_src1(a, L, n, ch, c1, second_is_out, obase, w);
      }
    }
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = base + it * NT + threadIdx.x;
      if (idx < items) {
        const int n = idx >> 2, ch = idx & 3;
        *(bf16x8*)(L.t0 + n * WLD + ch * 8) = r0[it];
        *(bf16x8*)(L.t1 + n * WLD + ch * 8) = r1[it];
      }
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
// NW = 0: one wave per 32-query block (blockDim.x = nqb * 64 <= 1024), no block left over for a second pass
template <int NW>
__global__ __launch_bounds__(NW ? NW * 64 : 1024) void win_attn_fwd_kernel(WinArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int w, hh;
  win_item(a, w, hh);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  const int nw = NW ? NW : (int)(blockDim.x >> 6);
  WinLds L;
  win_setup(a, smem, L, w, hh);
  if constexpr (NW != 0) win_stage<NW * 64>(a, L, a.C + hh * WHD, 2 * a.C + hh * WHD, false, nullptr, w);   // K, V
  else win_stage_rt(a, L, a.C + hh * WHD, 2 * a.C + hh * WHD, false, nullptr, w);
  const float c = a.c;
  // bias (rpb + mask, log2 domain) from the key-major table biasT, added by two MFMAs with an identity B operand:
  // k index 8h + j of k-step u <-> query 16u + 8h + j, A[key][k] = biasT[key][query(k)] (16-byte row loads, no
  // unpacking), B[k][q] = (query(k) == q). The backward reads the same table.
  const bf16* bT = a.biasT + ((long long)win_type(a, w) * a.H + hh) * a.Npad * a.Npad;
  bf16x8 ident[2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) ident[u][j] = to_bf16(16 * u + 8 * half + j == (lane & 31) ? 1.f : 0.f);
  bf16x8 qn[2];   // next query block's Q, loaded one block ahead
  auto load_q = [&](int qb) {
    const int q = qb * 32 + (lane & 31);
    const bool qv = q < a.N;
    const int qrow = qv ? L.row[q] : -2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qn[ks] = win_load8(a, L, qrow, hh * WHD + ks * 16 + 8 * half, qv);
  };
  if (wave < a.nqb) load_q(wave);
  for (int qb = wave; qb < a.nqb; qb += nw) {
    const int q = qb * 32 + (lane & 31);
    const bool qv = q < a.N;
    const int qrow = qv ? L.row[q] : -2;
    const bf16x8 qf[2] = {scaled8(qn[0], c), scaled8(qn[1], c)};
    if (qb + nw < a.nqb) load_q(qb + nw);
    const bf16* brow = bT + (long long)(lane & 31) * a.Npad + qb * 32 + 8 * half;   // + key tile * 32 rows
    const long long kstride = 32LL * a.Npad;
    auto ld_bias = [&](int kt, bf16x8 (&bt)[2]) __attribute__((always_inline)) {
      bt[0] = *(const bf16x8*)(brow + kt * kstride);
      bt[1] = *(const bf16x8*)(brow + kt * kstride + 16);
    };
    f32x16 o = {};
    float m = 0.f, l = 0.f;
    bf16x8 b0[2], b1[2];   // table tiles two ahead
    ld_bias(0, b0);
    if (a.nkt > 1) ld_bias(1, b1);
    for (int kt = 0; kt < a.nkt; ++kt) {
      LCI_WIN_FWD_SCHED();
      f32x16 s = mfma32(b0[0], ident[0], f32x16{});
      s = mfma32(b0[1], ident[1], s);
      b0[0] = b1[0];
      b0[1] = b1[1];
      if (kt + 2 < a.nkt) ld_bias(kt + 2, b1);
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
  int w, hh;
  win_item(a, w, hh);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  WinLds L;
  win_setup(a, smem, L, w, hh);
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
      qf[ks] = scaled8(win_load8(a, L, qrow, hh * WHD + ks * 16 + 8 * half, qv), c);
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
      kf[ks] = scaled8(win_load8(a, L, krow, a.C + hh * WHD + ks * 16 + 8 * half, kv), c);
      vf[ks] = win_load8(a, L, krow, 2 * a.C + hh * WHD + ks * 16 + 8 * half, kv);
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

// ---------------------------------------------------------------------------- backward, single phase
// The two-phase kernel above computes S, dP and the exponentials twice per (query, key) tile (14 MFMAs and 32 exp2
// per 32 x 32 tile pair) and loads K, V, Q, dO, O rows from global memory inside its loops. Here one wave per key
// block (NW = nkb <= 12 waves: every 7^3 window) keeps its K / V fragments in registers and takes the query tiles in
// a rotation, qt = (kb + t) mod nkb at step t, so at every step the waves work on distinct query tiles: per tile
// S, dP (bias^T table tile and -delta as initial accumulators), P, dS, dV^T += dO^T P, dK^T += Q^T dS (10 MFMAs with
// dQ, 16 exp2), and dQ^T += K^T dS^T with dS transposed through a per-wave LDS scratch tile, added into an f32 dQ
// accumulator in LDS that this wave owns for the step (one barrier per step; the summation order is fixed by the
// rotation: deterministic). Q / dO are staged once; delta = rowsum(dO * O) is computed at staging.
// The per-wave scratch tile (K^T once, then dS^T every step; 8-byte stores, transposed reads): 64-byte rows, the
// 8-byte chunk c of row r at c ^ ((r >> 1) & 7) -- conflict-free for both (with 80-byte rows the stores took 4 extra
// LDS cycles and the reads 2, profiles/r06_pmc.txt). Its rows always start at 0, so the swizzled lane offsets are
// loop-invariant registers.
constexpr int SLD = 32;
__device__ __forceinline__ int ssw(int row, int col) {
  return row * SLD + ((((col >> 2) ^ (row >> 1)) & 7) << 2) + (col & 3);
}
template <int S>
__device__ __forceinline__ bf16x8 sfrag_tr(const bf16* t, int lane) {   // frag_tr<S>(t, ld, 0, 0, lane) on it
  const int row = 16 * S + 4 * (lane >> 5) + ((lane & 15) >> 2);
  const int col = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  return cat44(lds_tr4(t + ssw(row, col)), lds_tr4(t + ssw(row + 8, col)));
}
constexpr int DQLD = 36;   // f32 row stride of the LDS dQ accumulator: the b128 RMW of 16 query rows is conflict-free
constexpr int WBWD1_MAXW = 12;
// Phase timestamps of the single-phase backward (variant builds only, -DLCI_WIN_STAMPS: tools/r6_win_stamps.py):
// lane 0 of every wave of the first 2048 workgroups (dispatch order) writes s_memrealtime (100 MHz) at slot k of
// its 20-slot record, slot 19 the CU (__smid)
#ifdef LCI_WIN_STAMPS
constexpr int WST_WG = 2048, WST_SLOTS = 20;
__device__ long long g_win_stamps[WST_WG * WBWD1_MAXW * WST_SLOTS];
#define WSTAMP(k)                                                                                              \
  do {                                                                                                         \
    const int wg_ = blockIdx.x;                                                                                \
    if ((threadIdx.x & 63) == 0 && wg_ < WST_WG)                                                               \
      g_win_stamps[((long long)wg_ * WBWD1_MAXW + (threadIdx.x >> 6)) * WST_SLOTS + (k)] =                     \
          (k) == 19 ? (long long)__smid() : (long long)wall_clock64();                                         \
  } while (0)
#else
#define WSTAMP(k)
#endif
__global__ __launch_bounds__(WBWD1_MAXW * 64) void win_attn_bwd1_kernel(WinArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int w, hh;
  win_item(a, w, hh);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  const int nkb = a.nkt, NT = blockDim.x;
  WSTAMP(0);
  WSTAMP(19);
  WinLds L;
  win_setup(a, smem, L, w, hh);                                  // t0, t1, row, rid
  WSTAMP(1);
  float* lse_l = (float*)(L.rid + a.Npad);                   // -lse2
  float* ndl_l = lse_l + a.Npad;                             // -delta
  float* dq_l = ndl_l + a.Npad;                              // (Npad, DQLD) f32
  bf16* scr = (bf16*)(dq_l + a.Npad * DQLD) + wave * 32 * SLD;   // this wave's 32 x 32 transpose tile
  const float c = a.c;

  // Prologue: every global read of the window issued at once, then consumed -- Q and dO rows (-> t0, t1), the O rows
  // and lse2 of the row constants, this wave's K / V rows -- so the workgroup pays one memory round trip before its
  // loop instead of three in sequence. Npad * 4 16-byte chunks = exactly 2 per thread; the row-constant items are the
  // same (n, ch) chunks, so delta = rowsum(dO * O) uses the dO values in registers.
  const int kb = wave;
  const int key = kb * 32 + (lane & 31);
  const bool kv = key < a.N;
  const int krow = kv ? L.row[key] : -2;
  const float* lseg = a.lse2 + ((long long)w * a.H + hh) * a.N;
  bf16x8 r0[2], r1[2], ov[2], kr[2], vr[2];
  float lsv[2];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = it * NT + threadIdx.x, n = idx >> 2, ch = idx & 3;
    r0[it] = win_load8(a, L, L.row[n], hh * WHD + ch * 8, n < a.N);
    r1[it] = win_stage_src1(a, L, n, ch, hh * WHD, true, a.dout, w);
    const int row = L.row[n];
    ov[it] = *(const bf16x8*)(n < a.N && row != -1 ? out_row_ptr(a, a.o, w, n, row) + hh * WHD + ch * 8 : kWinZero);
    lsv[it] = *(ch == 0 && n < a.N ? lseg + n : (const float*)kWinZero);
  }
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    kr[ks] = win_load8(a, L, krow, a.C + hh * WHD + ks * 16 + 8 * half, kv);
    vr[ks] = win_load8(a, L, krow, 2 * a.C + hh * WHD + ks * 16 + 8 * half, kv);
  }
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = it * NT + threadIdx.x, n = idx >> 2, ch = idx & 3;
    *(bf16x8*)(L.t0 + n * WLD + ch * 8) = r0[it];
    *(bf16x8*)(L.t1 + n * WLD + ch * 8) = r1[it];
    // row constants: lse2 and -delta = -rowsum(dO * O), 4 threads per query row (8 channels each)
    float dsum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) dsum = fmaf(to_f32(r1[it][j]), to_f32(ov[it][j]), dsum);
    dsum += __shfl_xor(dsum, 1);
    dsum += __shfl_xor(dsum, 2);
    if (ch == 0) {
      lse_l[n] = n < a.N ? -lsv[it] : -1.0e30f;   // -lse2 (the S chain's initial accumulator); padded rows: P = 0
      ndl_l[n] = -dsum;
    }
  }
  for (int i = threadIdx.x; i < a.Npad * DQLD / 4; i += NT) ((f32x4*)dq_l)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  int* cnt = (int*)((bf16*)(dq_l + a.Npad * DQLD) + nkb * 32 * SLD);   // dQ contributions added per query tile
  if (threadIdx.x < nkb) cnt[threadIdx.x] = 0;

  // this wave's key block: K (prescaled into the exp2 domain) / V as B operands, raw K^T as the dQ A operand
  bf16x8 kf[2], vf[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const bf16x8 kk = kr[ks];
    *(bf16x4*)(scr + ssw(lane & 31, ks * 16 + 8 * half)) = bf16x4{kk[0], kk[1], kk[2], kk[3]};
    *(bf16x4*)(scr + ssw(lane & 31, ks * 16 + 8 * half + 4)) = bf16x4{kk[4], kk[5], kk[6], kk[7]};
    kf[ks] = scaled8(kr[ks], c);
    vf[ks] = vr[ks];
  }
  __syncthreads();   // staging, row constants, dQ zero, K scratch
  WSTAMP(2);
  const bf16x8 kt0 = sfrag_tr<0>(scr, lane), kt1 = sfrag_tr<1>(scr, lane);
  __builtin_amdgcn_wave_barrier();   // K^T read before the scratch takes dS tiles

  const long long tho = ((long long)win_type(a, w) * a.H + hh) * a.Npad * a.Npad;
  // bias^T (the log2-domain rpb + mask table) enters the S chain through two MFMAs with an identity A operand:
  // k index 8h + j of k-step u <-> query 16u + 8h + j, A[q][k] = (query(k) == q), B[k][key] = biasT[key][query(k)]
  // (16-byte loads, no unpacking); -lse2 and -delta are the S / dP chains' initial accumulators (LDS reads), so
  // P = exp2(S) with no per-element bias, subtract or unpack VALU.
  const bf16* brow = a.biasT + tho + (long long)key * a.Npad + 8 * half;
  bf16x8 ident[2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) ident[u][j] = to_bf16(16 * u + 8 * half + j == (lane & 31) ? 1.f : 0.f);
  auto load_bias = [&](int tile, bf16x8 (&bt)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) bt[u] = *(const bf16x8*)(brow + tile * 32 + 16 * u);
  };
  // S and dP - delta of query tile `tile` (16 x f32 each, query rows, key on the lane)
  auto chains = [&](int tile, const bf16x8 (&bt)[2], f32x16& sx, f32x16& px) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {   // queries tile*32 + 8g + 4h + j
      const f32x4 l4 = *(const f32x4*)(lse_l + tile * 32 + 8 * g + 4 * half);
      const f32x4 d4 = *(const f32x4*)(ndl_l + tile * 32 + 8 * g + 4 * half);
#pragma unroll
      for (int j = 0; j < 4; ++j) { sx[4 * g + j] = l4[j]; px[4 * g + j] = d4[j]; }
    }
    sx = mfma32(ident[0], bt[0], sx);
    sx = mfma32(ident[1], bt[1], sx);
    sx = mfma32(frag_row(L.t0, WLD, tile * 32, 0, lane), kf[0], sx);
    sx = mfma32(frag_row(L.t0, WLD, tile * 32, 16, lane), kf[1], sx);
    px = mfma32(frag_row(L.t1, WLD, tile * 32, 0, lane), vf[0], px);
    px = mfma32(frag_row(L.t1, WLD, tile * 32, 16, lane), vf[1], px);
  };
  f32x16 dk = {}, dv = {};
  // The dQ partial of step t is added into the LDS accumulator in step t + 1's interval (every wave delays by one
  // step, so the tiles touched in one interval are still distinct), and step t + 1's S / dP chains are issued before
  // step t's barrier: their MFMA latency and the RMW's LDS latency overlap the barrier wait. Steps are separated by a
  // raw s_barrier behind lgkmcnt(0) only: the bias prefetch and the dS stores stay in flight across it (a
  // __syncthreads would drain them every step).
  auto dq_rmw = [&](int tile, const f32x16& part) __attribute__((always_inline)) {
    float* dqrow = dq_l + (tile * 32 + (lane & 31)) * DQLD + 4 * half;
#pragma unroll
    for (int g = 0; g < 4; ++g) {   // d = 8g + 4h + j
      f32x4 v = *(f32x4*)(dqrow + 8 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] += part[4 * g + j];
      *(f32x4*)(dqrow + 8 * g) = v;
    }
  };
  auto step_barrier = [&]() __attribute__((always_inline)) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(15 | (3 << 14) | (7 << 4));   // lgkmcnt(0): this wave's LDS accesses are done
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // Counter mode (default): tile q receives its contributions in step order -- at step t from wave (q - t) mod nkb
  // -- so the wave holding step t's partial waits until cnt[q] == t, adds, and publishes t + 1. (wave, step) waits
  // only on (wave + 1, step - 1): no cycle, and the waves drift apart instead of meeting at a barrier every step.
  auto dq_rmw_ordered = [&](int tile, int order, const f32x16& part) __attribute__((always_inline)) {
    int spins = 0;
    while (__hip_atomic_load(cnt + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != order) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 24)) break;   // bound: a logic error must not hang the GPU
    }
    asm volatile("" ::: "memory");
    dq_rmw(tile, part);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(15 | (3 << 14) | (7 << 4));   // lgkmcnt(0): the RMW's LDS writes are done
    if (lane == 0) __hip_atomic_store(cnt + tile, order + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  int qt = kb;
  bf16x8 bt[2];
  load_bias(qt, bt);
  f32x16 s, dp;
  chains(qt, bt, s, dp);
  if (nkb > 1) load_bias(qt + 1 == nkb ? 0 : qt + 1, bt);
  f32x16 dq_prev = {};
  int qt_prev = -1;
  for (int t = 0; t < nkb; ++t) {
    LCI_WIN_BWD_SCHED();
    WSTAMP(3 + t);
    const int qn = qt + 1 == nkb ? 0 : qt + 1;
    if (t > 0) {   // the previous step's tile
      if (a.bwd1_cnt) dq_rmw_ordered(qt_prev, t - 1, dq_prev);
      else dq_rmw(qt_prev, dq_prev);   // this wave's in this interval
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      s[i] = exp2_fast(s[i]);   // P (query rows, key on lane)
      dp[i] = s[i] * dp[i];     // dS
    }
    const bf16x8 p0 = pack8<0>(s), p1 = pack8<1>(s), d0 = pack8<0>(dp), d1 = pack8<1>(dp);
    dv = mfma32(frag_tr<0>(L.t1, WLD, qt * 32, 0, lane), p0, dv);
    dv = mfma32(frag_tr<1>(L.t1, WLD, qt * 32, 0, lane), p1, dv);
    dk = mfma32(frag_tr<0>(L.t0, WLD, qt * 32, 0, lane), d0, dk);
    dk = mfma32(frag_tr<1>(L.t0, WLD, qt * 32, 0, lane), d1, dk);
    if (a.dS) {   // tile (qt, kb) in the key-on-lane layout (win_rpb_grad_kernel, dS_kl)
      bf16* dst = a.dS + ((((long long)w * a.H + hh) * a.nqb + qt) * a.nkt + kb) * 1024 + lane * 16;
      *(bf16x8*)dst = d0;
      *(bf16x8*)(dst + 8) = d1;
    }
    // dS^T through the scratch tile [key][query]: register r of this lane is query (r&3) + 8(r>>2) + 4h
    const int sr = lane & 31;
    *(bf16x4*)(scr + ssw(sr, 4 * half)) = bf16x4{d0[0], d0[1], d0[2], d0[3]};
    *(bf16x4*)(scr + ssw(sr, 4 * half + 8)) = bf16x4{d0[4], d0[5], d0[6], d0[7]};
    *(bf16x4*)(scr + ssw(sr, 4 * half + 16)) = bf16x4{d1[0], d1[1], d1[2], d1[3]};
    *(bf16x4*)(scr + ssw(sr, 4 * half + 24)) = bf16x4{d1[4], d1[5], d1[6], d1[7]};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    dq_prev = mfma32(kt0, sfrag_tr<0>(scr, lane), f32x16{});
    dq_prev = mfma32(kt1, sfrag_tr<1>(scr, lane), dq_prev);   // dQ^T[d][query], query on the lane
    qt_prev = qt;
    qt = qn;
    if (t + 1 < nkb) {
      chains(qt, bt, s, dp);                                 // next step's chains, ahead of the barrier
      if (t + 2 < nkb) load_bias(qt + 1 == nkb ? 0 : qt + 1, bt);
    }
    if (!a.bwd1_cnt) step_barrier();   // next interval: the RMW of this step's tile
  }
  WSTAMP(15);
  if (a.bwd1_cnt) dq_rmw_ordered(qt_prev, nkb - 1, dq_prev);
  else dq_rmw(qt_prev, dq_prev);
  __syncthreads();
  WSTAMP(16);
  if (kv && krow >= 0) {
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
  // padded voxels: their k, v are the qkv bias (one atomic per word per wave, as in the two-phase kernel)
  // padded voxels: their k, v are the qkv bias. Sum each wave's padded keys over its 32 key lanes, then the waves in
  // wave order through LDS (the scratch tiles are dead): one (k | v) x 32 partial per workgroup into pad_ws, summed
  // over windows by win_pad_reduce_kernel -- deterministic, and no float atomics onto the same 192 addresses from
  // every boundary window (in the model those serialised at the memory side: 3x the kernel time at C3 stage 1)
  const bool padk = kv && krow < 0 && a.dbias_pad != nullptr;
  if (a.pad_ws != nullptr) {
    float* pw = (float*)(scr);   // this wave's 64 floats
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
        pw[d] = sk;
        pw[32 + d] = sv;
      }
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      float acc = 0.f;
      for (int v = 0; v < nkb; ++v) acc += ((const float*)(scr - wave * 32 * SLD + v * 32 * SLD))[threadIdx.x];
      a.pad_ws[((long long)w * a.H + hh) * 64 + threadIdx.x] = acc;
    }
  } else if (__any(padk)) {
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
  WSTAMP(17);
  // dQ rows (the loop's last barrier ordered every RMW): 16-byte chunks of 8 channels, scaled, bf16
  for (int it = threadIdx.x; it < a.N * 4; it += NT) {
    const int n = it >> 2, ch = it & 3;
    const int row = L.row[n];
    if (row < 0) continue;   // padded voxel: cropped (its dO, hence dS and dQ, are zero)
    const f32x4 lo = *(const f32x4*)(dq_l + n * DQLD + ch * 8), hi = *(const f32x4*)(dq_l + n * DQLD + ch * 8 + 4);
    bf16x8 o8;
#pragma unroll
    for (int j = 0; j < 4; ++j) { o8[j] = to_bf16(lo[j] * a.scale); o8[j + 4] = to_bf16(hi[j] * a.scale); }
    *(bf16x8*)(a.dqkv + (long long)(a.mode == 0 ? w * a.N + n : row) * 3 * a.C + hh * WHD + ch * 8) = o8;
  }
  WSTAMP(18);
}

// dbias_pad[C | 2C + h*32 + d] += sum_w pad_ws[w][h][k|v, d]: one workgroup per (head, value), windows split over
// 256 threads and summed in a fixed tree order (deterministic).
__global__ __launch_bounds__(256) void win_pad_reduce_kernel(WinArgs a) {
  __shared__ float red[256];
  const int hh = blockIdx.x >> 6, t = blockIdx.x & 63;
  float acc = 0.f;
  for (int w = threadIdx.x; w < a.Bw; w += 256) acc += a.pad_ws[((long long)w * a.H + hh) * 64 + t];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o >= 1; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) a.dbias_pad[(t < 32 ? a.C : 2 * a.C) + hh * WHD + (t & 31)] += red[0];
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
    const int r_in = (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);   // accumulator row of element i
    const int q = qb * 32 + (a.dS_kl ? r_in : (lane & 31));
    const int k = kt * 32 + (a.dS_kl ? (lane & 31) : r_in);
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
  static const int order_env = getenv("LCI_WIN_ORDER") ? atoi(getenv("LCI_WIN_ORDER")) : 1;   // A/B hook
  a.order = order_env;
  LCI_CHECK((long long)a.Bw * a.H < (1LL << 31), "window_attn: too many (window, head) workgroups");
  return 0;
}

static size_t win_lds(const WinArgs& a, bool bwd) {
  return WBIAS_B + (size_t)a.Npad * WLD * 2 * 2 + (size_t)a.Npad * 4 * 2 + (bwd ? (size_t)a.Npad * 4 * 2 : 0);
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

extern "C" int lci_window_attn_fwd(const void* qkv, const float* qkv_bias, const void* biasT, int has_mask,
                                   void* out, float* lse2, const int* geo, float scale, void* stream) {
  WinArgs a{};
  if (win_fill(a, geo, scale)) return 1;
  if (a.mode == 0 && has_mask) a.T = a.nW;
  LCI_CHECK(biasT && ((uintptr_t)biasT & 15) == 0, "window_attn_fwd: biasT must be a 16-byte aligned table");
  a.qkv = (const bf16*)qkv; a.qkv_bias = qkv_bias; a.biasT = (const bf16*)biasT; a.out = (bf16*)out; a.lse2 = lse2;
  // 8 waves sharing the window's K/V (LCI_WIN_FWD_NW=0: one wave per query block when the window has <= 16 of
  // them -- no wave idle in a second pass, but at 114 VGPRs one 11-wave workgroup per CU instead of two 8-wave ones:
  // stage 1 of C3 0.21-0.23 vs 0.18-0.19 ms, not the default)
  static const int fwd_nw = getenv("LCI_WIN_FWD_NW") ? atoi(getenv("LCI_WIN_FWD_NW")) : 8;
  if (fwd_nw == 0 && a.nqb <= 16) {
    (void)hipFuncSetAttribute((const void*)win_attn_fwd_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    hipLaunchKernelGGL(win_attn_fwd_kernel<0>, dim3(a.Bw * a.H), dim3(a.nqb * 64), win_lds(a, false),
                       (hipStream_t)stream, a);
  } else {
    constexpr int NW = 8;
    (void)hipFuncSetAttribute((const void*)win_attn_fwd_kernel<NW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    hipLaunchKernelGGL(win_attn_fwd_kernel<NW>, dim3(a.Bw * a.H), dim3(NW * 64), win_lds(a, false),
                       (hipStream_t)stream, a);
  }
  LCI_LAUNCH_CHECK();
  return 0;
}

// LCI_WIN_BWD1 (A/B hook, default 1: the single-phase backward) read once per process, in one place: the launch and
// lci_window_bwd_needs_plain must agree even if the environment changes later
static int win_bwd1_enabled() {
  static const int v = getenv("LCI_WIN_BWD1") ? atoi(getenv("LCI_WIN_BWD1")) : 1;
  return v;
}

// dbias_pad (3C) accumulated (caller zeroes); pad_ws (lci_window_pad_ws_elems f32) required with dbias_pad;
// dS tiles (Bw*H*nqb*nkt*1024 bf16) optional workspace;
// drpb (H, N, N) f32 written when dS and drpb are given.
extern "C" int lci_window_attn_bwd(const void* qkv, const float* qkv_bias, const void* bias, const void* biasT,
                                   int has_mask, const void* out, const void* dout, const float* lse2, void* dqkv,
                                   float* dbias_pad, float* pad_ws, void* dS, float* drpb, const int* geo,
                                   float scale,
                                   void* stream) {
  WinArgs a{};
  if (win_fill(a, geo, scale)) return 1;
  if (a.mode == 0 && has_mask) a.T = a.nW;
  a.qkv = (const bf16*)qkv; a.qkv_bias = qkv_bias; a.bias = (const bf16*)bias; a.biasT = (const bf16*)biasT; a.o = (const bf16*)out;
  a.dout = (const bf16*)dout; a.lse2 = (float*)lse2; a.dqkv = (bf16*)dqkv; a.dbias_pad = dbias_pad;
  LCI_CHECK(!dbias_pad || pad_ws, "window_attn_bwd: dbias_pad needs the pad_ws workspace");
  a.dS = (bf16*)dS; a.drpb = drpb;
  hipStream_t s = (hipStream_t)stream;
  // single-phase kernel for windows of <= 12 key blocks (every 7^3 / 7^2 / 4^3 window; LCI_WIN_BWD1=0: the
  // two-phase kernel, A/B hook); waves per (window, head) workgroup of the two-phase kernel: LCI_WIN_BWD_WAVES
  const int bwd1_env = win_bwd1_enabled();
  static const int nw_env = getenv("LCI_WIN_BWD_WAVES") ? atoi(getenv("LCI_WIN_BWD_WAVES")) : 4;
  LCI_CHECK(biasT && ((uintptr_t)biasT & 15) == 0, "window_attn_bwd: biasT must be a 16-byte aligned table");
  if (bwd1_env && a.nkt <= WBWD1_MAXW) {
    a.dS_kl = 1;
    static const int cnt_env = getenv("LCI_WIN_BWD1_CNT") ? atoi(getenv("LCI_WIN_BWD1_CNT")) : 1;
    a.bwd1_cnt = cnt_env;
    const size_t lds = WBIAS_B + (size_t)a.Npad * WLD * 2 * 2 + (size_t)a.Npad * 4 * 4 + (size_t)a.Npad * DQLD * 4 +
                       (size_t)a.nkt * 32 * SLD * 2 + 64;
    LCI_CHECK(lds <= 160 * 1024, "window_attn_bwd: %zu B of LDS", lds);
    (void)hipFuncSetAttribute((const void*)win_attn_bwd1_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    a.pad_ws = dbias_pad ? pad_ws : nullptr;
    hipLaunchKernelGGL(win_attn_bwd1_kernel, dim3(a.Bw * a.H), dim3(a.nkt * 64), lds, s, a);
    LCI_LAUNCH_CHECK();
    if (dbias_pad) hipLaunchKernelGGL(win_pad_reduce_kernel, dim3(a.H * 64), dim3(256), 0, s, a);
  } else if (!bias) {
    LCI_CHECK(false, "window_attn_bwd: the two-phase kernel (N > %d or LCI_WIN_BWD1=0) needs the plain table too",
              WBWD1_MAXW * 32);
  } else if (nw_env == 8) {
    (void)hipFuncSetAttribute((const void*)win_attn_bwd_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    hipLaunchKernelGGL(win_attn_bwd_kernel<8>, dim3(a.Bw * a.H), dim3(512), win_lds(a, true), s, a);
  } else {
    (void)hipFuncSetAttribute((const void*)win_attn_bwd_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    hipLaunchKernelGGL(win_attn_bwd_kernel<4>, dim3(a.Bw * a.H), dim3(256), win_lds(a, true), s, a);
  }
  LCI_LAUNCH_CHECK();
  if (dS && drpb) {
    const long long per_w = (long long)a.H * a.nqb * a.nkt * 1024;
    hipLaunchKernelGGL(win_rpb_grad_kernel, dim3((unsigned)((per_w / 8 + 127) / 128)), dim3(128), 0, s, a);
    LCI_LAUNCH_CHECK();
  }
  return 0;
}

// 1 when lci_window_attn_bwd runs the two-phase kernel for this geometry (windows of more than WBWD1_MAXW key blocks,
// or LCI_WIN_BWD1=0), which needs the plain query-major table beside biasT; 0 for the single-phase kernel; -1 bad geo
extern "C" int lci_window_bwd_needs_plain(const int* geo) {
  WinArgs a{};
  if (win_fill(a, geo, 1.f)) return -1;
  return (win_bwd1_enabled() && a.nkt <= WBWD1_MAXW) ? 0 : 1;
}

#ifdef LCI_WIN_STAMPS
extern "C" int lci_debug_win_stamps(void* dst, long long n) {   // variant builds only (not in lci.h)
  n = std::min<long long>(n, (long long)WST_WG * WBWD1_MAXW * WST_SLOTS);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_win_stamps), n * 8, 0, hipMemcpyDeviceToHost) != hipSuccess;
}
#endif

extern "C" long long lci_window_pad_ws_elems(const int* geo) {
  WinArgs a{};
  if (win_fill(a, geo, 1.f)) return -1;
  return (long long)a.Bw * a.H * 64;
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
