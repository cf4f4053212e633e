// Hyena implicit filter for gfx950: the Filter MLP + exponential modulation of hyena.py (:67-199), fused.
//
// Replaces Filter.filter(L) (reference hyena.py:178-187) for the reference's default filter MLP
//     z (L, E) -> Linear(E, 64) -> Sin -> Linear(64, 64) -> Sin -> Linear(64, 64) -> Sin -> Linear(64, D=64, no bias)
//     k = h * (exp(-t |deltas|) + shift)                                   (ExponentialModulation, :102-117)
// with one Sin module (one `freq` (1, 64) parameter) shared by the three activations, evaluated under
// bf16 autocast exactly as autograd would round it: every Linear takes bf16 inputs / weights / bias and
// rounds its f32-accumulated output to bf16, sin and the modulation run in f32 on those bf16 values.
//
// Layout: a wave owns 32 positions and keeps every activation in the MFMA accumulator layout with the
// FEATURE as the row (C^T[feature][position], v_mfma_f32_32x32x16_bf16), so one layer's output feeds the next
// layer's B operand from registers (pack8; the k-order that implies is folded into the weight fragments).
// The weight fragments (A operands, forward W_i and backward W_i^T in that permuted k-order) are built once
// per call by hf_prep_kernel into a 54 KB image that each workgroup stages in LDS.
//
// Backward (hf_bwd_kernel) recomputes the forward per tile and runs the data-gradient chain in registers:
//     dh = bf16(dk * m);  ds_i = bf16(W_{i+1}^T da_{i+1});  dp = ds * cos(freq a_i);  da_i = bf16(dp * freq)
//     dfreq += sum_pos dp * a_i;  dz = bf16(W1^T da1)
// writing dh, da3, da2 and the bf16 activations s1..s3 (columns in the permuted feature order) for the three
// 64x64 weight gradients (lci_linear_wgrad, by the caller), and reducing dfreq, db1 and dW1 (E columns)
// per wave through LDS into per-wave partials (summed by the caller; deterministic).
#include "common.hpp"

namespace lci {

constexpr int HF_NFRAG = 54;        // F1[2] F2[8] F3[8] F4[8] | B4[8] B3[8] B2[8] B1[4]
constexpr int HF_F2 = 2, HF_F3 = 10, HF_F4 = 18, HF_B4 = 26, HF_B3 = 34, HF_B2 = 42, HF_B1 = 50;
constexpr int HF_NVEC = 5 * 64;     // b1, b2, b3 (bf16-rounded), freq, |deltas|
constexpr int HF_THREADS = 512;     // forward: 8 waves x 32 positions = 256 positions per tile
constexpr int HF_TILE = HF_THREADS / 2;
constexpr int HF_BWD_THREADS = 256; // backward: 4 waves (one per SIMD: ~340 registers of live state per lane)
constexpr int HF_BWD_TILE = HF_BWD_THREADS / 2;
constexpr int HF_CS_LD = 68;        // column-sum scratch row stride (f32): 16-B aligned, rows 4 banks apart
constexpr int HF_MAX_E = 8;

struct FilterArgs {
  const float *W1, *b1, *freq, *W2, *b2, *W3, *b3, *W4, *deltas;   // prep inputs (f32 parameters / buffers)
  bf16* img; float* vec;                                           // prep outputs
  const bf16* cimg; const float* cvec;
  const float* z;   // (L, E) positional embedding rows
  const float* t;   // (L) positions in [0, 1]
  int E, L;
  float shift;
  float* k;                                        // forward out (D, L)
  const float* dk;                                 // backward in (D, L)
  bf16 *dh, *s3, *da3, *s2, *da2, *s1;             // backward out (L, 64), permuted feature columns
  float* dz;                                       // (L, E)
  float* part;                                     // (waves, 2 + E, 64): db1, dfreq, dW1[:, e]
};

// Feature held by pack element (t, jj) of lane half h: accumulator block t>>1, register 8(t&1)+jj.
__host__ __device__ constexpr int hf_feat(int t, int h, int jj) {
  return 32 * (t >> 1) + 16 * (t & 1) + 8 * (jj >> 2) + 4 * h + (jj & 3);
}
// Feature of permuted column c (the order the backward writes its (L, 64) tensors in).
__host__ __device__ constexpr int hf_col_feat(int c) { return hf_feat(c >> 4, (c >> 3) & 1, c & 7); }

__global__ void __launch_bounds__(64) hf_prep_kernel(FilterArgs a) {
  const int id = blockIdx.x, lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  if (id == HF_NFRAG) {
    a.vec[lane] = (float)(bf16)a.b1[lane];
    a.vec[64 + lane] = (float)(bf16)a.b2[lane];
    a.vec[128 + lane] = (float)(bf16)a.b3[lane];
    a.vec[192 + lane] = a.freq[lane];
    a.vec[256 + lane] = fabsf(a.deltas[lane]);
    return;
  }
  bf16x8 v;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    float x = 0.f;
    if (id < HF_F2) {                          // W1 rows, natural k = embedding column
      const int k = 8 * h + jj;
      if (k < a.E) x = a.W1[(32 * id + r) * a.E + k];
    } else if (id < HF_B4) {                   // W2, W3, W4 rows, k in accumulator order
      const int m = (id - HF_F2) / 8, b = ((id - HF_F2) % 8) / 4, s = (id - HF_F2) % 4;
      const float* W = m == 0 ? a.W2 : (m == 1 ? a.W3 : a.W4);
      x = W[(32 * b + r) * 64 + hf_feat(s, h, jj)];
    } else if (id < HF_B1) {                   // W4^T, W3^T, W2^T: rows = input feature, k = output feature
      const int m = (id - HF_B4) / 8, b = ((id - HF_B4) % 8) / 4, s = (id - HF_B4) % 4;
      const float* W = m == 0 ? a.W4 : (m == 1 ? a.W3 : a.W2);
      x = W[hf_feat(s, h, jj) * 64 + 32 * b + r];
    } else {                                   // W1^T: rows = embedding column (< E)
      const int s = id - HF_B1;
      if (r < a.E) x = a.W1[hf_feat(s, h, jj) * a.E + r];
    }
    v[jj] = (bf16)x;
  }
  *(bf16x8*)(a.img + ((size_t)id * 64 + lane) * 8) = v;
}

// 0 the compiler cannot see through: LDS reads indexed by it are not hoisted out of the tile loop (hoisting the
// loop-invariant fragment / vector reads would keep ~230 VGPRs live and spill).
__device__ __forceinline__ int hf_opaque_zero() {
  int z = 0;
  asm volatile("" : "+s"(z));
  return z;
}

__device__ __forceinline__ bf16x8 hf_frag(const bf16* limg, int id, int lane) {
  return *(const bf16x8*)(limg + (id * 64 + lane) * 8);
}

// acc[b] reg 4g+i <- per-feature vector value of row 32b + 8g + 4h + i.
__device__ __forceinline__ void hf_rows(f32x16 (&acc)[2], const float* v, int h) {
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 x = *(const f32x4*)(v + 32 * b + 8 * g + 4 * h);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[b][4 * g + i] = x[i];
    }
}

// The 8 per-feature values of pack t (features hf_feat(t, h, 0..7)).
// (Re-read per use, not CSE'd across the layers: the values are cheaper to reload than to keep live.)
__device__ __forceinline__ void hf_pack_vec(const float* v, int t, int h, float (&o)[8]) {
  v += hf_opaque_zero();
  const f32x4 lo = *(const f32x4*)(v + 32 * (t >> 1) + 16 * (t & 1) + 4 * h);
  const f32x4 hi = *(const f32x4*)(v + 32 * (t >> 1) + 16 * (t & 1) + 8 + 4 * h);
#pragma unroll
  for (int i = 0; i < 4; ++i) { o[i] = lo[i]; o[4 + i] = hi[i]; }
}

// Linear output (f32 accumulators incl. bias) -> a = bf16(acc), s = bf16(sin(freq * a)) as B-operand packs.
__device__ __forceinline__ void hf_act(const f32x16 (&acc)[2], const float* vfreq, int h, bf16x8 (&ap)[4],
                                       bf16x8 (&sp)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    float fr[8];
    hf_pack_vec(vfreq, t, h, fr);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const bf16 ab = (bf16)acc[t >> 1][8 * (t & 1) + jj];
      ap[t][jj] = ab;
      sp[t][jj] = (bf16)__sinf(fr[jj] * (float)ab);
    }
  }
}

// acc[b] (+)= sum_s A(id0 + 4b + s) x B(p[s]) over the 64-feature k dimension.
__device__ __forceinline__ void hf_gemm(f32x16 (&acc)[2], const bf16* limg, int id0, const bf16x8 (&p)[4], int lane) {
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s = 0; s < 4; ++s) acc[b] = mfma32(hf_frag(limg, id0 + 4 * b + s, lane), p[s], acc[b]);
}

// Forward through the three Sin layers for 32 positions (pos = this lane's position; zeros past L).
__device__ __forceinline__ void hf_forward(const FilterArgs& a, const bf16* limg, const float* lvec, int pos,
                                           int lane, bf16x8 (&ap)[3][4], bf16x8 (&sp)[3][4]) {
  const int h = lane >> 5;
  bf16x8 zv;
#pragma unroll
  for (int jj = 0; jj < 8; ++jj) {
    float x = 0.f;
    if (h == 0 && jj < a.E && pos < a.L) x = a.z[(long long)pos * a.E + jj];
    zv[jj] = (bf16)x;
  }
  f32x16 acc[2];
  hf_rows(acc, lvec, h);
#pragma unroll
  for (int b = 0; b < 2; ++b) acc[b] = mfma32(hf_frag(limg, b, lane), zv, acc[b]);
  hf_act(acc, lvec + 192, h, ap[0], sp[0]);
  hf_rows(acc, lvec + 64, h);
  hf_gemm(acc, limg, HF_F2, sp[0], lane);
  hf_act(acc, lvec + 192, h, ap[1], sp[1]);
  hf_rows(acc, lvec + 128, h);
  hf_gemm(acc, limg, HF_F3, sp[1], lane);
  hf_act(acc, lvec + 192, h, ap[2], sp[2]);
}

__device__ __forceinline__ void hf_stage(const FilterArgs& a, bf16* limg, float* lvec, int nfrag) {
  for (int i = threadIdx.x; i < nfrag * 64; i += blockDim.x)
    *(bf16x8*)(limg + i * 8) = *(const bf16x8*)(a.cimg + (size_t)i * 8);
  for (int i = threadIdx.x; i < HF_NVEC; i += blockDim.x) lvec[i] = a.cvec[i];
  __syncthreads();
}

__global__ void __launch_bounds__(HF_THREADS) hf_fwd_kernel(FilterArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 limg[HF_B4 * 64 * 8];
  __shared__ __attribute__((aligned(16))) float lvec[HF_NVEC];
  hf_stage(a, limg, lvec, HF_B4);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  for (int tile = blockIdx.x; tile * HF_TILE < a.L; tile += gridDim.x) {
    const int pos = tile * HF_TILE + wave * 32 + (lane & 31);
    const bf16* li = limg + hf_opaque_zero();   // keep the fragment / vector reads inside the loop
    const float* lv = lvec + hf_opaque_zero();
    bf16x8 ap[3][4], sp[3][4];
    hf_forward(a, li, lv, pos, lane, ap, sp);
    f32x16 acc[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[b] = f32x16{};
    hf_gemm(acc, li, HF_F4, sp[2], lane);
    if (pos < a.L) {
      const float tp = a.t[pos];
      float* kl = a.k + (long long)(4 * h) * a.L + pos;   // + uniform row offsets below
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int c0 = 32 * b + (e & 3) + 8 * (e >> 2);
          const float m = expf(-tp * lv[256 + c0 + 4 * h]) + a.shift;
          kl[(long long)c0 * a.L] = (float)(bf16)acc[b][e] * m;
        }
    }
  }
}

// Per-wave column sum of a 32 x 64 value tile (lane = position row, packs = permuted columns): lane l
// receives the sum of column l. Uniform across the workgroup (two barriers).
__device__ __forceinline__ float hf_colsum(float* cs, const float (&v)[4][8], int lane) {
  const int r = lane & 31, h = lane >> 5;
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    *(f32x4*)(cs + r * HF_CS_LD + 16 * t + 8 * h) = f32x4{v[t][0], v[t][1], v[t][2], v[t][3]};
    *(f32x4*)(cs + r * HF_CS_LD + 16 * t + 8 * h + 4) = f32x4{v[t][4], v[t][5], v[t][6], v[t][7]};
  }
  __syncthreads();
  float s = 0.f;
#pragma unroll 8
  for (int rr = 0; rr < 32; ++rr) s += cs[rr * HF_CS_LD + lane];
  __syncthreads();
  __builtin_amdgcn_sched_barrier(0);
  return s;
}

// Sin-layer backward: ds (f32 accumulators) -> da = bf16(bf16(ds) cos(freq a) freq) packs; q += dp * a.
__device__ __forceinline__ void hf_dact(const f32x16 (&acc)[2], const bf16x8 (&ap)[4], const float* vfreq, int h,
                                        float (&q)[4][8], bf16x8 (&dap)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    float fr[8];
    hf_pack_vec(vfreq, t, h, fr);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const float ds = (float)(bf16)acc[t >> 1][8 * (t & 1) + jj];
      const float av = (float)ap[t][jj];
      const float dp = ds * __cosf(fr[jj] * av);
      q[t][jj] += dp * av;
      dap[t][jj] = (bf16)(dp * fr[jj]);
    }
  }
}

__device__ __forceinline__ void hf_store(bf16* dst, int pos, int h, const bf16x8 (&p)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) *(bf16x8*)(dst + (long long)pos * 64 + 16 * t + 8 * h) = p[t];
}

__global__ void __launch_bounds__(HF_BWD_THREADS) hf_bwd_kernel(FilterArgs a) {
  // F1..F3 and B4..B1 (F4 is not needed: the forward output h enters the backward only through dk)
  __shared__ __attribute__((aligned(16))) bf16 limg[HF_NFRAG * 64 * 8];
  __shared__ __attribute__((aligned(16))) float lvec[HF_NVEC];
  __shared__ __attribute__((aligned(16))) float lcs[HF_BWD_THREADS / 64][32 * HF_CS_LD];
  hf_stage(a, limg, lvec, HF_NFRAG);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  float* cs = lcs[wave];
  const int nslot = 2 + a.E;
  float run[2 + HF_MAX_E];
#pragma unroll
  for (int i = 0; i < 2 + HF_MAX_E; ++i) run[i] = 0.f;
  for (int tile = blockIdx.x; tile * HF_BWD_TILE < a.L; tile += gridDim.x) {
    const int pos = tile * HF_BWD_TILE + wave * 32 + (lane & 31);
    const bool valid = pos < a.L;
    const bf16* li = limg + hf_opaque_zero();
    const float* lv = lvec + hf_opaque_zero();
    bf16x8 ap[3][4], sp[3][4];
    hf_forward(a, li, lv, pos, lane, ap, sp);
    if (valid) {
      hf_store(a.s1, pos, h, sp[0]);
      hf_store(a.s2, pos, h, sp[1]);
      hf_store(a.s3, pos, h, sp[2]);
    }
    __builtin_amdgcn_sched_barrier(0);   // phase fences: keep the scheduler from stretching live ranges
    // dh = bf16(dk * (exp(-t |delta|) + shift))
    bf16x8 gp[4];
    {
      const float tp = valid ? a.t[pos] : 0.f;
      const float* dkl = a.dk + (long long)(4 * h) * a.L + (valid ? pos : 0);   // + uniform row offsets below
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float ad[8];
        hf_pack_vec(lv + 256, t, h, ad);
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const float g = valid ? dkl[(long long)hf_feat(t, 0, jj) * a.L] : 0.f;
          gp[t][jj] = (bf16)(g * (expf(-tp * ad[jj]) + a.shift));
        }
      }
    }
    if (valid) hf_store(a.dh, pos, h, gp);
    __builtin_amdgcn_sched_barrier(0);
    float q[4][8];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) q[t][jj] = 0.f;
    f32x16 acc[2];
    bf16x8 dap[4];
    acc[0] = f32x16{}; acc[1] = f32x16{};
    hf_gemm(acc, li, HF_B4, gp, lane);                 // ds3 = W4^T dh
    hf_dact(acc, ap[2], lv + 192, h, q, dap);           // da3
    if (valid) hf_store(a.da3, pos, h, dap);
    __builtin_amdgcn_sched_barrier(0);
    acc[0] = f32x16{}; acc[1] = f32x16{};
    hf_gemm(acc, li, HF_B3, dap, lane);                 // ds2 = W3^T da3
    hf_dact(acc, ap[1], lv + 192, h, q, dap);           // da2
    if (valid) hf_store(a.da2, pos, h, dap);
    __builtin_amdgcn_sched_barrier(0);
    acc[0] = f32x16{}; acc[1] = f32x16{};
    hf_gemm(acc, li, HF_B2, dap, lane);                 // ds1 = W2^T da2
    hf_dact(acc, ap[0], lv + 192, h, q, dap);           // da1
    // dz = bf16(W1^T da1): one 32-row block, rows = embedding column
    f32x16 dzacc = f32x16{};
#pragma unroll
    for (int s = 0; s < 4; ++s) dzacc = mfma32(hf_frag(li, HF_B1 + s, lane), dap[s], dzacc);
    if (valid) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = (e & 3) + 8 * (e >> 2) + 4 * h;
        if (row < a.E) a.dz[(long long)pos * a.E + row] = (float)(bf16)dzacc[e];
      }
    }
    // per-feature sums over the 32 positions: db1, dfreq, dW1[:, e]
    run[1] += hf_colsum(cs, q, lane);
    float v[4][8];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) v[t][jj] = (float)dap[t][jj];
    run[0] += hf_colsum(cs, v, lane);
    // dW1[:, e] terms: da1 * bf16(z_e) of this lane's position (both lane halves share the position)
#pragma unroll
    for (int e = 0; e < HF_MAX_E; ++e) {
      if (e >= a.E) break;
      const float ze = (float)(bf16)(valid ? a.z[(long long)pos * a.E + e] : 0.f);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) v[t][jj] = (float)dap[t][jj] * ze;
      run[2 + e] += hf_colsum(cs, v, lane);
    }
  }
  float* out = a.part + (size_t)(blockIdx.x * (HF_BWD_THREADS / 64) + wave) * nslot * 64 + hf_col_feat(lane);
#pragma unroll
  for (int i = 0; i < 2 + HF_MAX_E; ++i)
    if (i < nslot) out[i * 64] = run[i];
}

static int hf_grid(int L, int tile) {
  const int nt = (L + tile - 1) / tile;
  return nt < 256 ? nt : 256;
}

}  // namespace lci

using namespace lci;

extern "C" int lci_hyena_filter_prep(const float* W1, const float* b1, const float* freq, const float* W2,
                                     const float* b2, const float* W3, const float* b3, const float* W4,
                                     const float* deltas, int E, void* img, float* vec, void* stream) {
  LCI_CHECK(E >= 1 && E <= HF_MAX_E, "hyena_filter: emb_dim %d unsupported (1..%d)", E, HF_MAX_E);
  LCI_CHECK(((uintptr_t)img & 15) == 0, "hyena_filter: fragment image must be 16-byte aligned");
  FilterArgs a{};
  a.W1 = W1; a.b1 = b1; a.freq = freq; a.W2 = W2; a.b2 = b2; a.W3 = W3; a.b3 = b3; a.W4 = W4; a.deltas = deltas;
  a.img = (bf16*)img; a.vec = vec; a.E = E;
  hipLaunchKernelGGL(hf_prep_kernel, dim3(HF_NFRAG + 1), dim3(64), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" long long lci_hyena_filter_img_elems() { return (long long)HF_NFRAG * 64 * 8; }

extern "C" long long lci_hyena_filter_partials(int L, int E) {
  if (L < 1 || E < 1 || E > HF_MAX_E) return -1;
  return (long long)hf_grid(L, HF_BWD_TILE) * (HF_BWD_THREADS / 64) * (2 + E) * 64;
}

extern "C" int lci_hyena_filter_fwd(const float* z, const float* t, const void* img, const float* vec, int E, int L,
                                    float shift, float* k, void* stream) {
  LCI_CHECK(E >= 1 && E <= HF_MAX_E && L >= 1, "hyena_filter: bad shape E=%d L=%d", E, L);
  FilterArgs a{};
  a.z = z; a.t = t; a.cimg = (const bf16*)img; a.cvec = vec; a.E = E; a.L = L; a.shift = shift; a.k = k;
  hipLaunchKernelGGL(hf_fwd_kernel, dim3(hf_grid(L, HF_TILE)), dim3(HF_THREADS), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_hyena_filter_bwd(const float* z, const float* t, const void* img, const float* vec, int E, int L,
                                    float shift, const float* dk, void* dh, void* s3, void* da3, void* s2, void* da2,
                                    void* s1, float* dz, float* part, void* stream) {
  LCI_CHECK(E >= 1 && E <= HF_MAX_E && L >= 1, "hyena_filter: bad shape E=%d L=%d", E, L);
  void* outs[6] = {dh, s3, da3, s2, da2, s1};
  for (void* p : outs) LCI_CHECK(((uintptr_t)p & 15) == 0, "hyena_filter: (L, 64) outputs must be 16-byte aligned");
  FilterArgs a{};
  a.z = z; a.t = t; a.cimg = (const bf16*)img; a.cvec = vec; a.E = E; a.L = L; a.shift = shift; a.dk = dk;
  a.dh = (bf16*)dh; a.s3 = (bf16*)s3; a.da3 = (bf16*)da3; a.s2 = (bf16*)s2; a.da2 = (bf16*)da2; a.s1 = (bf16*)s1;
  a.dz = dz; a.part = part;
  hipLaunchKernelGGL(hf_bwd_kernel, dim3(hf_grid(L, HF_BWD_TILE)), dim3(HF_BWD_THREADS), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}
