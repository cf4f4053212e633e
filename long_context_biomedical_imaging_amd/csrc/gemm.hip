// Token-wise projection GEMM for gfx950: Y (M x N) = X (M x K) . W^T (+ bias), X and W both K-contiguous, bf16 in,
// f32 accumulate, bf16 out -- the forward and data-gradient GEMMs of every token-wise nn.Linear under the trainer's
// bf16 autocast (SABlock qkv / out_proj backbone_vit.py:166-167, MONAI MLPBlock :249, Hyena in/out_proj
// hyena.py:278-279, Mamba in/out_proj mamba.py:60-64,90). The data gradient dX = dY . W is the same GEMM with the
// transposed weight (the caller transposes W once per call: N x K is small).
//
// The shapes are skinny in K (384 .. 1536) and long in M (2^17 .. 2^21 tokens), so the kernel is persistent: one
// 512-thread workgroup per CU walks its output tiles (256 tokens x 384 features) and the K-slab pipeline runs across
// tile boundaries -- tile j+1's first slabs are in flight while tile j finishes and writes its epilogue, so there is
// no per-tile prologue. Tiles are dealt out XCD-contiguously (blocks b and b + 8 share an XCD): the feature tiles of
// one token tile run on one XCD at the same time and read its X rows from that XCD's L2.
//
// Per workgroup: 8 waves = 2 (tokens, 128 each) x 4 (features, 96 each); a wave holds 4 x 3 accumulator blocks of
// v_mfma_f32_32x32x16_bf16 (W the A operand: features on the accumulator registers, tokens on the lanes). K slabs of
// 32 arrive by LDS-DMA (buffer_load_dwordx4 ... lds, 1-KB units = 16 rows x 64 B) into a 3-slot ring two slabs ahead,
// 16-B chunks XOR-swizzled by (row >> 2) & 3 through the per-lane source offset so the ds_read_b128 fragment reads
// are conflict-free; one raw s_barrier per slab after a counted vmcnt (vmcnt counts the epilogue's stores too, in
// issue order). The epilogue stores each lane's 4 consecutive features as 8-B pieces straight from the registers
// (buffer stores range-checked at the token tile's end: M need not be a multiple of 256), bias from LDS.
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "common.hpp"

namespace lci {

constexpr int GM_TM = 256;        // tokens per tile
constexpr int GM_WAVES = 8;
constexpr int GM_BK = 32;         // K per slab
constexpr int GM_NSLOT = 3;
constexpr int GM_MAXN = 4096;     // bias staged in LDS

struct GemmArgs {
  const bf16* x; long long ldx;   // (M, ldx), columns [0, K)
  const bf16* w;                  // (N, K) contiguous
  const bf16* bias;               // (N) or null
  bf16* y; long long ldy;         // (M, ldy)
  long long M;
  int N, K;
  int ntn;                        // feature tiles
  long long ntiles;
  int G8, dmt, dnt;               // workgroups per XCD; G8 tiles = dmt token tiles + dnt feature tiles
  int probe;                      // timing probe (LCI_GEMM_PROBE, wrong results): 1 = no epilogue stores
};

// LDS-DMA of one 1-KB unit: lane l's 16 bytes at (voff + soff) of resource r land at LDS byte lds + 16 l
__device__ __forceinline__ void gm_dma16(rsrc_t r, int voff, int soff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds), "s"(soff) : "memory");
}
template <int N>
__device__ __forceinline__ void gm_vmcnt() {   // s_waitcnt vmcnt(N), lgkmcnt / expcnt untouched (gfx9 encoding)
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  __builtin_amdgcn_sched_barrier(0);
}

template <int TN>
__global__ __launch_bounds__(GM_WAVES * 64, 1) void gemm_bt_kernel(GemmArgs a) {
  constexpr int WN = 4, WM = 2;
  constexpr int NB = TN / WN / 32, MB = GM_TM / WM / 32;           // 32x32 blocks per wave (features, tokens)
  constexpr int ROWS = GM_TM + TN;                                 // LDS rows per slab (64 B each)
  constexpr int SLOT_B = ROWS * 64;
  constexpr int UNITS = ROWS / 16, UX = GM_TM / 16;                // 1-KB DMA units per slab; X units first
  constexpr int UPW = UNITS / GM_WAVES;
  static_assert(UNITS % GM_WAVES == 0 && UX % GM_WAVES == 0, "units per wave");
  static_assert(GM_NSLOT * SLOT_B + GM_MAXN * 2 <= 160 * 1024, "LDS");
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  bf16* sbias = (bf16*)(gsm + GM_NSLOT * SLOT_B);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int r = lane & 31, h = lane >> 5;

  // this workgroup's tiles: XCD x = blockIdx.x % 8 takes the contiguous range [x per, (x + 1) per) of tile ids (token
  // tile major, feature tile minor), its G8 = gridDim.x / 8 workgroups interleaved over it
  const int G8 = a.G8, xcd = blockIdx.x % 8, li = blockIdx.x / 8;
  const long long per = (a.ntiles + 7) / 8;
  const long long t_begin = xcd * per + li, t_end = min(a.ntiles, (xcd + 1) * per);
  const int my_tiles = t_begin < t_end ? (int)((t_end - t_begin + G8 - 1) / G8) : 0;
  const int nslab = a.K / GM_BK;
  const int S = my_tiles * nslab;

  if (a.bias) {
    for (int i = tid; i < a.N; i += GM_WAVES * 64) sbias[i] = a.bias[i];
  }
  __syncthreads();
  if (S == 0) return;

  const unsigned lds0 = (unsigned)(uintptr_t)(LCI_LDS char*)gsm;
  // DMA lane mapping inside a unit: row (lane >> 2) of 16, physical chunk lane & 3 <- logical chunk lc ^ ((row >> 2) & 3)
  const int ldx2 = (int)a.ldx * 2, K2 = a.K * 2;
  const rsrc_t rw = make_rsrc(a.w, (uint32_t)((long long)a.N * a.K * 2));
  // tile cursor: tile id t -> token tile t / ntn, feature tile t % ntn; one division here, then advanced by G8 tiles
  // (= dmt token tiles + dnt feature tiles) without dividing
  struct Cursor {
    long long mt; int nt;
    __device__ long long m0() const { return mt * GM_TM; }
    __device__ int n0() const { return nt * TN; }
  };
  Cursor c0;
  c0.mt = t_begin / a.ntn;
  c0.nt = (int)(t_begin - c0.mt * a.ntn);
  auto advance = [&](Cursor& c) {
    c.nt += a.dnt;
    c.mt += a.dmt;
    if (c.nt >= a.ntn) { c.nt -= a.ntn; ++c.mt; }
  };
  auto x_rsrc = [&](const Cursor& c) {
    const long long rows = min((long long)GM_TM, a.M - c.m0());
    return make_rsrc(a.x + c.m0() * a.ldx, (uint32_t)(rows * a.ldx * 2));
  };
  // the issue stream: slab k of tile cursor ic
  Cursor ic = c0;
  rsrc_t irx = x_rsrc(ic);
  int ik = 0, ij = 0, islot = 0;   // issue stream: slab ik of tile ij, into ring slot islot
  auto issue = [&]() {
    const unsigned sb = lds0 + (unsigned)(islot * SLOT_B);
    islot = islot == GM_NSLOT - 1 ? 0 : islot + 1;
    const int ko = ik * GM_BK * 2;
    // lane source offsets, recomputed per issue (a few VALU) rather than held across the loop in registers: the
    // lane index made opaque so the compiler does not hoist them
    int l = lane;
    asm volatile("" : "+v"(l));
    const int drow = l >> 2, dchunk = (l & 3) ^ ((l >> 4) & 3);
    const int xo = (16 * wave + drow) * ldx2 + 16 * dchunk;
    const int wo = (16 * (wave + GM_WAVES * (UX / GM_WAVES) - UX) + drow + ic.n0()) * K2 + 16 * dchunk;
#pragma unroll
    for (int q = 0; q < UX / GM_WAVES; ++q) gm_dma16(irx, xo + 16 * GM_WAVES * q * ldx2, ko, sb + 1024 * (wave + GM_WAVES * q));
#pragma unroll
    for (int q = 0; q < UPW - UX / GM_WAVES; ++q)
      gm_dma16(rw, wo + 16 * GM_WAVES * q * K2, ko, sb + 1024 * (wave + GM_WAVES * (q + UX / GM_WAVES)));
    if (++ik == nslab) {   // next tile
      ik = 0;
      ++ij;
      if (ij < my_tiles) {
        advance(ic);
        irx = x_rsrc(ic);
      }
    }
  };

  f32x16 acc[NB][MB];
  // fragment offsets within a slot: the swizzle depends on the lane's row bits 2-3 only (block rows are multiples
  // of 32), so the two k-substeps' chunk offsets are lane constants
  const int sw = (r >> 2) & 3;
  const int coff0 = 16 * ((0 + h) ^ sw), coff1 = 16 * ((2 + h) ^ sw);
  const int xrow0 = (128 * wm + r) * 64, wrow0 = (GM_TM + 96 * wn + r) * 64;

  // one slab's MFMAs (FIRST: the tile's first slab starts its accumulators from zero, no zeroing pass)
  auto compute = [&](const char* slot, auto FIRST) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int co = ks ? coff1 : coff0;
      bf16x8 fw[NB], fx[MB];
#pragma unroll
      for (int i = 0; i < NB; ++i) fw[i] = *(const bf16x8*)(slot + wrow0 + 32 * 64 * i + co);
#pragma unroll
      for (int j = 0; j < MB; ++j) fx[j] = *(const bf16x8*)(slot + xrow0 + 32 * 64 * j + co);
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < MB; ++j)
          acc[i][j] = mfma32(fw[i], fx[j], (decltype(FIRST)::value && ks == 0) ? f32x16{} : acc[i][j]);
    }
  };

  issue();
  if (S > 1) issue();
  Cursor cc = c0;             // the tile being computed
  int ck = 0, cj = 0, cslot = 0;
  int since_epi = 8;          // slabs since the last epilogue
  for (int s = 0; s < S; ++s) {
    ++since_epi;
    // slab s landed: the next slab's UPW units may still be in flight, and, in the two slabs after an epilogue, its
    // 4 NB MB stores too (they were issued between two slabs' units; vmcnt retires in issue order)
    if (s + 1 >= S) gm_vmcnt<0>();
    else if (since_epi <= 2) gm_vmcnt<UPW + 4 * NB * MB>();
    else gm_vmcnt<UPW>();
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's reads of the slot being refilled are done
    __builtin_amdgcn_s_barrier();
    if (s + 2 < S) issue();               // into slot (s + 2) % 3 = (s - 1) % 3, free after this barrier
    const char* slot = gsm + cslot * SLOT_B;
    cslot = cslot == GM_NSLOT - 1 ? 0 : cslot + 1;
    if (ck == 0) compute(slot, std::integral_constant<bool, true>{});
    else compute(slot, std::integral_constant<bool, false>{});
    if (++ck == nslab) {   // the tile's last slab: epilogue straight from the registers
      const long long rows = min((long long)GM_TM, a.M - cc.m0());
      const rsrc_t ry = make_rsrc(a.y + cc.m0() * a.ldy, (uint32_t)(rows * a.ldy * 2));
      const int ldy2 = (int)a.ldy * 2;
      const int vbase = r * ldy2 + 8 * h;   // the lane's part of every store offset; the rest is wave-uniform
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int fs = cc.n0() + 96 * wn + 32 * i + 8 * g;   // acc reg 4g + q <-> feature fs + 4h + q
          float b4[4] = {0.f, 0.f, 0.f, 0.f};
          if (a.bias) {
            const bf16x4 bb = *(const bf16x4*)(sbias + fs + 4 * h);
#pragma unroll
            for (int q = 0; q < 4; ++q) b4[q] = to_f32(bb[q]);
          }
#pragma unroll
          for (int j = 0; j < MB; ++j) {
            bf16x4 o;
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = to_bf16(acc[i][j][4 * g + q] + b4[q]);
            if (!a.probe) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), ry, vbase,
                                                  (128 * wm + 32 * j) * ldy2 + fs * 2, 0);
          }
        }
      since_epi = 0;
      ck = 0;
      if (++cj < my_tiles) advance(cc);
    }
  }
}

}  // namespace lci

using namespace lci;

// 1 when lci_gemm_bt takes (N, K): N a multiple of the 384-feature tile, K of the 32-deep slab
extern "C" int lci_gemm_bt_supported(int N, int K) { return N > 0 && N % 384 == 0 && N <= GM_MAXN && K > 0 && K % GM_BK == 0; }

// Y (M x N, row stride ldy) = X (M x K, row stride ldx) . W^T (W: N x K contiguous) + bias (N, bf16, or null); bf16.
// x, w, y 16-byte aligned; ldx, ldy multiples of 8; M * ldx and M * ldy any size (per-tile 32-bit offsets).
extern "C" int lci_gemm_bt(const void* x, long long ldx, const void* w, const void* bias, void* y, long long ldy,
                           long long M, int N, int K, void* stream) {
  LCI_CHECK(lci_gemm_bt_supported(N, K), "gemm_bt: N=%d K=%d unsupported (N %% 384, K %% 32)", N, K);
  LCI_CHECK(M > 0 && ldx >= K && ldy >= N && ldx % 8 == 0 && ldy % 8 == 0, "gemm_bt: bad M / strides");
  LCI_CHECK(((uintptr_t)x | (uintptr_t)w | (uintptr_t)y) % 16 == 0, "gemm_bt: pointers must be 16-byte aligned");
  LCI_CHECK((long long)GM_TM * ldx * 2 < (1ll << 31) && (long long)GM_TM * ldy * 2 < (1ll << 31) &&
                (long long)N * K * 2 < (1ll << 31), "gemm_bt: strides too large for 32-bit tile offsets");
  GemmArgs a{};
  a.x = (const bf16*)x; a.ldx = ldx; a.w = (const bf16*)w; a.bias = (const bf16*)bias; a.y = (bf16*)y; a.ldy = ldy;
  a.M = M; a.N = N; a.K = K;
  a.ntn = N / 384;
  a.ntiles = (M + GM_TM - 1) / GM_TM * a.ntn;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    LCI_HIP(hipGetDevice(&dev));
    LCI_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const long long grid = std::min<long long>((a.ntiles + 7) / 8 * 8, (long long)ncu / 8 * 8);
  a.G8 = (int)(grid / 8);
  a.dmt = a.G8 / a.ntn;
  a.dnt = a.G8 % a.ntn;
  static const int probe = getenv("LCI_GEMM_PROBE") ? atoi(getenv("LCI_GEMM_PROBE")) : 0;
  a.probe = probe;
  constexpr int TN = 384;
  const size_t sh = (size_t)GM_NSLOT * (GM_TM + TN) * 64 + GM_MAXN * 2;
  (void)hipFuncSetAttribute((const void*)gemm_bt_kernel<TN>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
  hipLaunchKernelGGL(gemm_bt_kernel<TN>, dim3((unsigned)grid), dim3(GM_WAVES * 64), sh, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}
