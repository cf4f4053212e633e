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
// Per workgroup: 8 waves = 4 (tokens, 64 each) x 2 (features, 192 each); a wave holds 6 x 2 accumulator blocks of
// v_mfma_f32_32x32x16_bf16 (W the A operand: features on the accumulator registers, tokens on the lanes). K slabs of
// 32 arrive by LDS-DMA (buffer_load_dwordx4 ... lds, 1-KB units = 16 rows x 64 B) into a 3-slot ring two slabs ahead,
// 16-B chunks XOR-swizzled by (row >> 2) & 3 through the per-lane source offset so the ds_read_b128 fragment reads
// are conflict-free; one raw s_barrier per slab after a counted vmcnt (vmcnt counts the epilogue's stores too, in
// issue order). A slab's 5 DMA units per wave are issued one per MFMA group of its first k-substep (an LDS-DMA
// instruction holds its wave's issue for tens of cycles), and the second k-substep's W fragments are read as the
// first substep's MFMAs release their registers.
//
// Epilogue: each wave turns 32 tokens x 64 features at a time into bf16 (+ bias) rows of 128 B in its own 4-KB LDS
// buffer (v_permlane32_swap pairs the two half-waves' 8-B pieces into 16-B chunks; chunks XOR-swizzled by row & 7,
// conflict-free both ways) and stores them back as whole 128-B lines, 8 rows per buffer_store_dwordx4. Stored
// straight from the MFMA layout instead (each instruction touching 32 rows x 16 B), the tile's stores cost as much
// as its MFMAs (profiles/r05_gemm_ab.txt). Buffer stores are range-checked at the token tile's end (M need not be a
// multiple of 256).
#include <algorithm>
#include <type_traits>

#include "common.hpp"

namespace lci {

constexpr int GM_TM = 256;        // tokens per tile
constexpr int GM_WAVES = 8;
constexpr int GM_BK = 32;         // K per slab
constexpr int GM_NSLOT = 3;
constexpr int GM_MAXN = 4096;     // bias staged in LDS
constexpr int GM_EPI = 4096;      // per-wave epilogue buffer (32 tokens x 64 features bf16)

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
};

template <int TN, bool HAS_BIAS, bool ACC = false>
__global__ __launch_bounds__(GM_WAVES * 64, 1) void gemm_bt_kernel(GemmArgs a) {
  constexpr int WN = 2, WM = 4;
  constexpr int NB = TN / WN / 32, MB = GM_TM / WM / 32;           // 32x32 blocks per wave (features, tokens)
  constexpr int ROWS = GM_TM + TN;                                 // LDS rows per slab (64 B each)
  constexpr int SLOT_B = ROWS * 64;
  constexpr int UNITS = ROWS / 16, UX = GM_TM / 16;                // 1-KB DMA units per slab; X units first
  constexpr int UPW = UNITS / GM_WAVES;
  static_assert(UNITS % GM_WAVES == 0 && UX % GM_WAVES == 0, "units per wave");
  static_assert(GM_NSLOT * SLOT_B + GM_WAVES * GM_EPI + GM_MAXN * 2 <= 160 * 1024, "LDS");
  static_assert(NB % 2 == 0, "epilogue chunks are 64 features");
  extern __shared__ __attribute__((aligned(16))) char gsm[];
  char* sepi = gsm + GM_NSLOT * SLOT_B;
  bf16* sbias = (bf16*)(sepi + GM_WAVES * GM_EPI);
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

  if (HAS_BIAS) {
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
  // One slab's DMA: issue_begin() takes the next slab of the stream (its LDS slot, K offset, lane source offsets)
  // and advances the stream; piece(d, q) issues its unit q (X units first). The pieces are spread between the first
  // k-substep's MFMA groups (an LDS-DMA instruction holds its wave's issue for tens of cycles).
  struct Dma { unsigned sb; int ko, xo, wo; rsrc_t rx; };
  auto issue_begin = [&]() {
    Dma d{lds0 + (unsigned)(islot * SLOT_B), ik * GM_BK * 2, 0, 0, irx};
    islot = islot == GM_NSLOT - 1 ? 0 : islot + 1;
    // lane source offsets, recomputed per issue (a few VALU) rather than held across the loop in registers: the
    // lane index made opaque so the compiler does not hoist them
    int l = lane;
    asm volatile("" : "+v"(l));
    const int drow = l >> 2, dchunk = (l & 3) ^ ((l >> 4) & 3);
    d.xo = (16 * wave + drow) * ldx2 + 16 * dchunk;
    d.wo = (16 * (wave + GM_WAVES * (UX / GM_WAVES) - UX) + drow + ic.n0()) * K2 + 16 * dchunk;
    if (++ik == nslab) {   // next tile
      ik = 0;
      ++ij;
      if (ij < my_tiles) {
        advance(ic);
        irx = x_rsrc(ic);
      }
    }
    return d;
  };
  auto piece = [&](const Dma& d, int q) __attribute__((always_inline)) {
    constexpr int QX = UX / GM_WAVES;
    if (q < QX) dma16_lds(d.rx, d.xo + 16 * GM_WAVES * q * ldx2, d.ko, d.sb + 1024 * (wave + GM_WAVES * q));
    else dma16_lds(rw, d.wo + 16 * GM_WAVES * (q - QX) * K2, d.ko, d.sb + 1024 * (wave + GM_WAVES * q));
  };


  f32x16 acc[NB][MB];
  constexpr int WT = GM_TM / WM, WF = TN / WN;                     // tokens, features per wave

  // one slab's MFMAs (FIRST: the tile's first slab starts its accumulators from zero, no zeroing pass). Fragment
  // offsets within a slot: the swizzle depends on the lane's row bits 2-3 only (block rows are multiples of 32), so
  // the two k-substeps' chunk offsets are lane constants -- recomputed per slab from an opaque lane index (a few VALU)
  // rather than held across the loop for every slot
  auto compute = [&](const char* slot, auto FIRST, bool iss, const Dma& d) __attribute__((always_inline)) {
    int l = lane;
    asm volatile("" : "+v"(l));
    const int fr = l & 31, fh = l >> 5, sw = (fr >> 2) & 3;
    const char* xb = slot + (WT * wm + fr) * 64;
    const char* wb = slot + (GM_TM + WF * wn + fr) * 64;
    // reads and MFMAs of the two k-substeps interleaved: substep 1's W fragment i is read into fragment i's
    // registers as soon as substep 0's two MFMAs on it have issued (LDS returns in order; the waitcnt pass counts)
    const int co0 = 16 * (fh ^ sw), co1 = 16 * ((2 + fh) ^ sw);
    bf16x8 fw[NB], fx0[MB], fx1[MB];
#pragma unroll
    for (int j = 0; j < MB; ++j) fx0[j] = *(const bf16x8*)(xb + 32 * 64 * j + co0);
#pragma unroll
    for (int i = 0; i < NB; ++i) fw[i] = *(const bf16x8*)(wb + 32 * 64 * i + co0);
#pragma unroll
    for (int j = 0; j < MB; ++j) fx1[j] = *(const bf16x8*)(xb + 32 * 64 * j + co1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < NB; ++i) {
#pragma unroll
      for (int j = 0; j < MB; ++j) acc[i][j] = mfma32(fw[i], fx0[j], decltype(FIRST)::value ? f32x16{} : acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
      fw[i] = *(const bf16x8*)(wb + 32 * 64 * i + co1);
      if (iss && i < UPW) piece(d, i);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < MB; ++j) acc[i][j] = mfma32(fw[i], fx1[j], acc[i][j]);
  };

  static_assert(UPW <= NB, "one DMA piece per MFMA group");
  for (int t = 0; t < 2 && t < S; ++t) {
    const Dma d = issue_begin();
#pragma unroll
    for (int q = 0; q < UPW; ++q) piece(d, q);
  }
  Cursor cc = c0;             // the tile being computed
  int ck = 0, cj = 0, cslot = 0;
  int since_epi = 8;          // slabs since the last epilogue
  for (int s = 0; s < S; ++s) {
    ++since_epi;
    // slab s landed: the next slab's UPW units may still be in flight, and, in the two slabs after an epilogue, its
    // 2 NB MB stores too (they were issued between two slabs' units; vmcnt retires in issue order)
    if (s + 1 >= S) wait_vmcnt<0>();
    else if (since_epi <= 2) wait_vmcnt<UPW + 2 * NB * MB>();
    else wait_vmcnt<UPW>();
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's reads of the slot being refilled are done
    __builtin_amdgcn_s_barrier();
    const bool iss = s + 2 < S;           // slab s + 2 into slot (s + 2) % 3 = (s - 1) % 3, free after this barrier
    Dma d{0u, 0, 0, 0, irx};
    if (iss) d = issue_begin();
    const char* slot = gsm + cslot * SLOT_B;
    cslot = cslot == GM_NSLOT - 1 ? 0 : cslot + 1;
    if (ck == 0) compute(slot, std::integral_constant<bool, true>{}, iss, d);
    else compute(slot, std::integral_constant<bool, false>{}, iss, d);
    if (++ck == nslab) {   // the tile's last slab: epilogue through the wave's LDS buffer
      const long long rows = min((long long)GM_TM, a.M - cc.m0());
      const rsrc_t ry = make_rsrc(a.y + cc.m0() * a.ldy, (uint32_t)(rows * a.ldy * 2));
      const int ldy2 = (int)a.ldy * 2;
      char* eb = sepi + wave * GM_EPI;
      // lane-derived offsets recomputed here from an opaque lane index (not hoisted into registers held across the
      // main loop)
      int l = lane;
      asm volatile("" : "+v"(l));
      const int er = l & 31, eh = l >> 5;
      const int erow = l >> 3, echk = l & 7;   // read-back: row erow + 8k, 16-B chunk echk of the 128-B row
#pragma unroll
      for (int j = 0; j < MB; ++j)
#pragma unroll
        for (int ip = 0; ip < NB / 2; ++ip) {
          // blocks 2ip, 2ip + 1 = the wave's features 64 ip .. + 63 of tokens 32 j .. + 31, as bf16 rows of 128 B
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int p = 0; p < 2; ++p) {
              const int i = 2 * ip + b;
              const int fs = cc.n0() + WF * wn + 32 * i + 16 * p + 4 * eh;   // regs 8p + q / 8p + 4 + q: fs + q / fs + 8 + q
              bf16x4 lo, hi;   // (+ bias: the autocast Linear's f32 sum, rounded once)
              if constexpr (HAS_BIAS) {
                const bf16x4 bb0 = *(const bf16x4*)(sbias + fs), bb1 = *(const bf16x4*)(sbias + fs + 8);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  lo[q] = to_bf16(acc[i][j][8 * p + q] + to_f32(bb0[q]));
                  hi[q] = to_bf16(acc[i][j][8 * p + 4 + q] + to_f32(bb1[q]));
                }
              } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  lo[q] = to_bf16(acc[i][j][8 * p + q]);
                  hi[q] = to_bf16(acc[i][j][8 * p + 4 + q]);
                }
              }
              // lane h gets features 16p + 8h .. + 7 of block i: 16-B chunk 4b + 2p + h of the row
              const u32x2 ul = __builtin_bit_cast(u32x2, lo), uh = __builtin_bit_cast(u32x2, hi);
              const auto s0 = __builtin_amdgcn_permlane32_swap(ul[0], uh[0], false, false);
              const auto s1 = __builtin_amdgcn_permlane32_swap(ul[1], uh[1], false, false);
              *(u32x4*)(eb + er * 128 + 16 * ((4 * b + 2 * p + eh) ^ (er & 7))) = u32x4{s0[0], s1[0], s0[1], s1[1]};
            }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int row = 8 * k + erow;
            u32x4 v = *(const u32x4*)(eb + row * 128 + 16 * (echk ^ (row & 7)));
            const int vo = erow * ldy2 + 16 * echk;
            const int so = (WT * wm + 32 * j + 8 * k) * ldy2 + (cc.n0() + WF * wn + 64 * ip) * 2;
            if constexpr (ACC) {   // y += the bf16 product: the autograd sum of two bf16 gradients, rounded once more
              bf16x8 pv = __builtin_bit_cast(bf16x8, v);
              const bf16x8 ov = __builtin_bit_cast(bf16x8, bload16(ry, vo, so));
#pragma unroll
              for (int q = 0; q < 8; ++q) pv[q] = to_bf16(to_f32(ov[q]) + to_f32(pv[q]));
              v = __builtin_bit_cast(u32x4, pv);
            }
            __builtin_amdgcn_raw_buffer_store_b128(v, ry, vo, so, 0);
          }
        }
      since_epi = 0;
      ck = 0;
      if (++cj < my_tiles) advance(cc);
    }
  }
}


// ------------------------------------------------------------------------------ small / narrow GEMM (round 6)
// The persistent kernel above wants a 256 x 384 (or 256) tile per CU. Two families of projections miss it and ran on
// hipBLASLt: the Swin stage-3 / 4 projections and their data gradients (4096 / 512 tokens, K and
// N 384 .. 3072: 16-48 tiles) and the decoder heads' 1x1 convolutions (N = 96 / 192 / 288 at up to 2^21 voxels,
// UnetResBlock conv3 / UnetOutBlock, enhance_heads.py). Here one wave owns 32 tokens x 32 NBW features and reads its
// MFMA fragments straight from global memory (no LDS, no barriers). K runs in chunks of CH 16-deep k-steps, two chunks
// of fragments in registers: chunk c + 1's loads are in flight while chunk c's MFMAs run (a first version with one
// k-step ahead was latency-bound: 30 us for a 4096 x 384 x 384 product, 1 ms for 2^21 x 192 x 96). Within a chunk
// the reduction index is permuted so that a lane's loads are contiguous: lane (row r, half h) holds columns
// c0 + 8 CH h + 8 j + t of its X row and of its W row for k-step j (t < 8) -- 16 CH bytes per row and lane, a whole
// 32 CH-byte row segment per lane pair -- and the MFMAs of a chunk sum each of its 16 CH columns once. W is the A
// operand (features on the accumulator registers, tokens on the lanes): a lane stores 4 consecutive features (8 B)
// of its token row per register group. Workgroups are numbered feature block fastest, so the waves that read the
// same X rows for other features run at the same time (L2 hits).
template <int NBW, int CH, bool HAS_BIAS, bool ACC = false>
__global__ __launch_bounds__(256) void gemm_bt_small_kernel(GemmArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nfb = a.N / (32 * NBW);
  const long long tb = blockIdx.x / nfb;
  const int fb = (int)(blockIdx.x - tb * nfb);
  const long long m0 = (tb * 4 + wave) * 32;
  if (m0 >= a.M) return;   // (no barriers in this kernel)
  const int n0 = fb * 32 * NBW;
  const int r = lane & 31, h = lane >> 5;
  const int rows = (int)min(32LL, a.M - m0);
  // rows past M read as zeros (buffer range check); their outputs are not stored
  const rsrc_t rx = make_rsrc(a.x + m0 * a.ldx, (uint32_t)((long long)rows * a.ldx * 2));
  const int xo = r * (int)a.ldx * 2 + 16 * CH * h;
  const bf16* wp = a.w + (long long)(n0 + r) * a.K + 8 * CH * h;
  const int nch = a.K / (16 * CH);
  f32x16 acc[NBW];
#pragma unroll
  for (int i = 0; i < NBW; ++i) acc[i] = f32x16{};
  bf16x8 xa[CH], wa[NBW][CH], xb[CH], wb[NBW][CH];
  auto load = [&](int c, bf16x8 (&xs)[CH], bf16x8 (&ws)[NBW][CH]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < CH; ++j) xs[j] = __builtin_bit_cast(bf16x8, bload16(rx, xo + 16 * j, 32 * CH * c));
#pragma unroll
    for (int i = 0; i < NBW; ++i)
#pragma unroll
      for (int j = 0; j < CH; ++j) ws[i][j] = *(const bf16x8*)(wp + (long long)32 * i * a.K + 16 * CH * c + 8 * j);
  };
  auto mma = [&](const bf16x8 (&xs)[CH], const bf16x8 (&ws)[NBW][CH]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int i = 0; i < NBW; ++i) acc[i] = mfma32(ws[i][j], xs[j], acc[i]);
  };
  load(0, xa, wa);
  for (int c = 0; c < nch; c += 2) {
    if (c + 1 < nch) load(c + 1, xb, wb);
    mma(xa, wa);
    if (c + 1 < nch) {
      if (c + 2 < nch) load(c + 2, xa, wa);
      mma(xb, wb);
    }
  }
  if (r >= rows) return;
  bf16* yrow = a.y + (m0 + r) * a.ldy + n0 + 4 * h;
#pragma unroll
  for (int i = 0; i < NBW; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) {   // register 4g + q <-> feature 32 i + 8 g + 4 h + q
      bf16x4 v;
      if constexpr (HAS_BIAS) {
        const bf16x4 bb = *(const bf16x4*)(a.bias + n0 + 32 * i + 8 * g + 4 * h);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = to_bf16(acc[i][4 * g + q] + to_f32(bb[q]));
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = to_bf16(acc[i][4 * g + q]);
      }
      if constexpr (ACC) {   // y += the bf16 product (lci_gemm_bt_acc's roundings)
        const bf16x4 o = *(const bf16x4*)(yrow + 32 * i + 8 * g);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = to_bf16(to_f32(o[q]) + to_f32(v[q]));
      }
      *(bf16x4*)(yrow + 32 * i + 8 * g) = v;
    }
}

}  // namespace lci

using namespace lci;

// feature tile of an output width: 384 where it divides N, else 256 (the ConvTranspose-as-GEMM widths 8 Cout:
// 512 .. 4096), 0 if neither does
static int gm_tn(int N) { return N % 384 == 0 ? 384 : (N % 256 == 0 ? 256 : 0); }

// 1 when lci_gemm_bt takes (N, K): N a multiple of a 384- or 256-feature tile, K of the 32-deep slab
extern "C" int lci_gemm_bt_supported(int N, int K) {
  return N > 0 && gm_tn(N) && N <= GM_MAXN && K > 0 && K % GM_BK == 0;
}

template <int TN>
static void gm_launch(const GemmArgs& a, long long grid, bool bias, hipStream_t st, bool acc = false) {
  const size_t sh = (size_t)GM_NSLOT * (GM_TM + TN) * 64 + GM_WAVES * GM_EPI + GM_MAXN * 2;
  if (acc) {
    (void)hipFuncSetAttribute((const void*)gemm_bt_kernel<TN, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    hipLaunchKernelGGL((gemm_bt_kernel<TN, false, true>), dim3((unsigned)grid), dim3(GM_WAVES * 64), sh, st, a);
  } else if (bias) {
    (void)hipFuncSetAttribute((const void*)gemm_bt_kernel<TN, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    hipLaunchKernelGGL((gemm_bt_kernel<TN, true>), dim3((unsigned)grid), dim3(GM_WAVES * 64), sh, st, a);
  } else {
    (void)hipFuncSetAttribute((const void*)gemm_bt_kernel<TN, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh);
    hipLaunchKernelGGL((gemm_bt_kernel<TN, false>), dim3((unsigned)grid), dim3(GM_WAVES * 64), sh, st, a);
  }
}

// Y (M x N, row stride ldy) = X (M x K, row stride ldx) . W^T (W: N x K contiguous) + bias (N, bf16, or null); bf16.
// x, w, y 16-byte aligned; ldx, ldy multiples of 8; M * ldx and M * ldy any size (per-tile 32-bit offsets).
static int gemm_bt_run(const void* x, long long ldx, const void* w, const void* bias, void* y, long long ldy,
                       long long M, int N, int K, void* stream, bool acc) {
  LCI_CHECK(lci_gemm_bt_supported(N, K), "gemm_bt: N=%d K=%d unsupported (N %% 384 or %% 256, K %% 32)", N, K);
  LCI_CHECK(M > 0 && ldx >= K && ldy >= N && ldx % 8 == 0 && ldy % 8 == 0, "gemm_bt: bad M / strides");
  LCI_CHECK(((uintptr_t)x | (uintptr_t)w | (uintptr_t)y) % 16 == 0, "gemm_bt: pointers must be 16-byte aligned");
  LCI_CHECK((long long)GM_TM * ldx * 2 < (1ll << 31) && (long long)GM_TM * ldy * 2 < (1ll << 31) &&
                (long long)N * K * 2 < (1ll << 31), "gemm_bt: strides too large for 32-bit tile offsets");
  GemmArgs a{};
  a.x = (const bf16*)x; a.ldx = ldx; a.w = (const bf16*)w; a.bias = (const bf16*)bias; a.y = (bf16*)y; a.ldy = ldy;
  a.M = M; a.N = N; a.K = K;
  const int tn = gm_tn(N);
  a.ntn = N / tn;
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
  if (tn == 384) gm_launch<384>(a, grid, bias != nullptr, (hipStream_t)stream, acc);
  else gm_launch<256>(a, grid, bias != nullptr, (hipStream_t)stream, acc);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_gemm_bt(const void* x, long long ldx, const void* w, const void* bias, void* y, long long ldy,
                           long long M, int N, int K, void* stream) {
  return gemm_bt_run(x, ldx, w, bias, y, ldy, M, N, K, stream, false);
}

// y (M x N, bf16) = bf16(y + bf16(X . W^T)): the product added into an existing bf16 gradient in the epilogue
// (UnetResBlock's 1x1 residual data gradient into conv1's, the sum autograd would form; no bias). Same support.
extern "C" int lci_gemm_bt_acc(const void* x, long long ldx, const void* w, void* y, long long ldy, long long M, int N,
                               int K, void* stream) {
  return gemm_bt_run(x, ldx, w, nullptr, y, ldy, M, N, K, stream, true);
}

// Features per wave of the small kernel (32 NBW, NBW <= 3): the widest that divides N / 32 while the grid still has
// >= 4096 waves (4 waves per workgroup, 32 tokens each: the 2^17 - 2^21-row 1x1 convolutions, where each wave then
// reads its X rows once), else 1 (the 512 / 4096-token Swin projections: as many waves as the shape has).
static int gm_small_nbw(long long M, int N) {
  if (N % 32) return 0;
  const long long mb = (M + 31) / 32;
  for (int nbw : {3, 2}) {
    if ((N / 32) % nbw == 0 && mb * (N / (32 * nbw)) >= 4096) return nbw;
  }
  return 1;
}

// k-steps per chunk: the largest of 4, 3, 2, 1 dividing K / 16
static int gm_small_ch(int K) {
  const int nk = K / 16;
  return nk % 4 == 0 ? 4 : (nk % 3 == 0 ? 3 : (nk % 2 == 0 ? 2 : 1));
}

// 1 when lci_gemm_bt_small takes (N, K): N % 32 == 0, K % 16 == 0
extern "C" int lci_gemm_bt_small_supported(int N, int K) { return N > 0 && N % 32 == 0 && K > 0 && K % 16 == 0; }

static int gemm_bt_small_run(const void* x, long long ldx, const void* w, const void* bias, void* y, long long ldy,
                             long long M, int N, int K, void* stream, bool acc) {
  LCI_CHECK(lci_gemm_bt_small_supported(N, K), "gemm_bt_small: N=%d K=%d unsupported (N %% 32, K %% 16)", N, K);
  LCI_CHECK(M > 0 && ldx >= K && ldy >= N && ldx % 8 == 0 && ldy % 8 == 0, "gemm_bt_small: bad M / strides");
  LCI_CHECK(((uintptr_t)x | (uintptr_t)w | (uintptr_t)y) % 16 == 0 && ((uintptr_t)bias % 8) == 0,
            "gemm_bt_small: x, w, y must be 16-byte aligned, bias 8-byte");
  LCI_CHECK(32LL * ldx * 2 < (1ll << 31) && (long long)N * K < (1ll << 31), "gemm_bt_small: strides too large");
  GemmArgs a{};
  a.x = (const bf16*)x; a.ldx = ldx; a.w = (const bf16*)w; a.bias = (const bf16*)bias; a.y = (bf16*)y; a.ldy = ldy;
  a.M = M; a.N = N; a.K = K;
  const int nbw = gm_small_nbw(M, N), ch = gm_small_ch(K);
  const long long nwg = (M + 127) / 128 * (N / (32 * nbw));
  LCI_CHECK(nwg < (1ll << 31), "gemm_bt_small: M too large");
  const dim3 grid((unsigned)nwg);
  hipStream_t st = (hipStream_t)stream;
#define LCI_GS(NB, C)                                                                                     \
  if (nbw == NB && ch == C) {                                                                             \
    if (acc) hipLaunchKernelGGL((gemm_bt_small_kernel<NB, C, false, true>), grid, dim3(256), 0, st, a);   \
    else if (bias) hipLaunchKernelGGL((gemm_bt_small_kernel<NB, C, true>), grid, dim3(256), 0, st, a);    \
    else hipLaunchKernelGGL((gemm_bt_small_kernel<NB, C, false>), grid, dim3(256), 0, st, a);             \
  }
  LCI_GS(1, 1) LCI_GS(1, 2) LCI_GS(1, 3) LCI_GS(1, 4) LCI_GS(2, 1) LCI_GS(2, 2) LCI_GS(2, 3) LCI_GS(2, 4)
  LCI_GS(3, 1) LCI_GS(3, 2) LCI_GS(3, 3) LCI_GS(3, 4)
#undef LCI_GS
  LCI_LAUNCH_CHECK();
  return 0;
}

// Y (M x N, row stride ldy) = X (M x K, row stride ldx) . W^T (+ bias), as lci_gemm_bt, for any M and N % 32 == 0,
// K % 16 == 0 (the small-token / narrow-output projections; see gemm_bt_small_kernel).
extern "C" int lci_gemm_bt_small(const void* x, long long ldx, const void* w, const void* bias, void* y, long long ldy,
                                 long long M, int N, int K, void* stream) {
  return gemm_bt_small_run(x, ldx, w, bias, y, ldy, M, N, K, stream, false);
}

// y = bf16(y + bf16(X . W^T)), as lci_gemm_bt_acc, with lci_gemm_bt_small's support.
extern "C" int lci_gemm_bt_small_acc(const void* x, long long ldx, const void* w, void* y, long long ldy, long long M,
                                     int N, int K, void* stream) {
  return gemm_bt_small_run(x, ldx, w, nullptr, y, ldy, M, N, K, stream, true);
}
