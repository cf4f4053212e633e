// ViT full self-attention (SABlock, backbone_vit.py:191-203) for the cases the placed bf16 kernels of attention.hip
// do not take: the reference's fp32 (non-AMP) path, whose einsums run in fp32 (backbone_vit.py:193,200), and head
// dims above 64 (the `custom` hidden / heads splits, backbone_vit.py:78-86), up to 256.
//
// Numerics: every product on v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate: bit-for-bit a k-ordered fmaf chain),
// softmax in f32 -- so with f32 I/O the result is the reference's fp32 attention up to summation order. bf16 I/O
// (autocast, head dim > 64) is converted to f32 on the way into LDS and the outputs are rounded to bf16 once.
//
// Layout: qkv (B, L, 3*H*D) in the I/O type, channel order (qkv, head, d) (backbone_vit.py:168), read in place;
// out (B, L, H*D); lse (B, H, L) f32 natural-log row logsumexp; dqkv like qkv. D <= DP (64 / 128 / 256): columns
// past D and rows past L are staged as zeros, so any D and L work. Deterministic: no atomics.
//
// Lane maps of v_mfma_f32_16x16x4_f32 (cdna_hip_programming.md §3): lane l, g = l >> 4, c = l & 15 holds
// A[i = c][k = g] and B[k = g][j = c]; accumulator register r of lane l is C[row 4g + r][col c].
// Contractions over d use k-step s <-> d = 4s + g; contractions over keys / queries take an accumulator tile
// (rows in registers) as the B operand directly: k-step s <-> row 4g + s, i.e. register s of every lane.
// LDS tiles are f32 [row][SD] with SD = DP + 20 (SD = 20 mod 64): both read patterns, [c][4s + g] (operand rows)
// and [4g + s][16 db + c] (operand columns), hit 64 distinct banks.
#include "common.hpp"

namespace lci {


__device__ __forceinline__ f32x4 mfma16f(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <typename T> __device__ __forceinline__ float ldf(const T* p);
template <> __device__ __forceinline__ float ldf<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ldf<bf16>(const bf16* p) { return to_f32(*p); }
template <typename T> __device__ __forceinline__ T stf(float x);
template <> __device__ __forceinline__ float stf<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 stf<bf16>(float x) { return to_bf16(x); }

constexpr int GT = 32;          // rows (keys or queries) per staged tile
constexpr int GNW = 4;          // waves per workgroup, 16 rows each
constexpr float G_NEG = -1.0e30f;
constexpr float LOG2E = 1.4426950408889634f;

struct GenArgs {
  const void* q; const void* k; const void* v;   // head 0 of batch 0 (element pointers of the I/O type)
  const void* o; const void* dout;
  void* out;                                     // fwd: O; bwd: dQ base (dK, dV follow)
  void* dk; void* dv;
  float* lse;                                    // (B, H, L)
  float* delta;                                  // bwd: (B, H, L)
  long long bs_qkv, bs_o;                        // batch strides (elements)
  int rs_qkv, rs_o;                              // row strides (elements)
  int H, L, D;
  float scale;
};

// Stage rows r0 .. r0 + GT - 1 (columns 0 .. DP - 1) of a (L, D) slice with row stride rs into LDS as f32 [GT][SD]
template <typename T, int DP>
__device__ __forceinline__ void g_stage(float* lds, const T* base, int rs, int r0, int L, int D, int tid) {
  constexpr int SD = DP + 20;
#pragma unroll 4
  for (int i = tid; i < GT * DP; i += GNW * 64) {
    const int r = i / DP, c = i % DP;
    float x = 0.f;
    if (r0 + r < L && c < D) x = ldf<T>(base + (long long)(r0 + r) * rs + c);
    lds[r * SD + c] = x;
  }
}

// ------------------------------------------------------------------------------------------------ forward
// Workgroup = 4 waves x 16 queries; key tiles of 32 staged (K, V) in LDS. Per wave and 16-key block:
// S^T = K Q^T (DP/4 MFMAs, the key on the accumulator row, the query on the lane), online softmax per query
// column (rows of a column live in the 4 lane groups: shuffles xor 16 / 32), O^T += V^T P^T (P^T straight from the
// accumulator as B operand).
template <typename T, int DP>
__global__ __launch_bounds__(GNW * 64) void attn_gen_fwd_kernel(GenArgs a) {
  constexpr int SD = DP + 20, NS = DP / 4, NDB = DP / 16;
  __shared__ float kt[GT * SD], vt[GT * SD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, c = lane & 15;
  const int hh = blockIdx.y, b = blockIdx.z, L = a.L, D = a.D;
  const int q = blockIdx.x * (GNW * 16) + wave * 16 + c;
  const T* qp = (const T*)a.q + b * a.bs_qkv + hh * D;
  const T* kp = (const T*)a.k + b * a.bs_qkv + hh * D;
  const T* vp = (const T*)a.v + b * a.bs_qkv + hh * D;
  float qf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int d = 4 * s + g;
    qf[s] = (q < L && d < D) ? ldf<T>(qp + (long long)q * a.rs_qkv + d) : 0.f;
  }
  f32x4 o[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = G_NEG, l = 0.f;
  const float c2 = a.scale * LOG2E;
  for (int t0 = 0; t0 < L; t0 += GT) {
    __syncthreads();
    g_stage<T, DP>(kt, kp, a.rs_qkv, t0, L, D, tid);
    g_stage<T, DP>(vt, vp, a.rs_qkv, t0, L, D, tid);
    __syncthreads();
    f32x4 sc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) sc[kb] = mfma16f(kt[(16 * kb + c) * SD + 4 * s + g], qf[s], sc[kb]);
    float mx = G_NEG;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float z = sc[kb][r] * c2;   // log2 domain
        if (t0 + 16 * kb + 4 * g + r >= L) z = G_NEG;
        sc[kb][r] = z;
        mx = fmaxf(mx, z);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mn = fmaxf(m, mx);
    const float alpha = exp2_fast(m - mn);
    m = mn;
    l *= alpha;
#pragma unroll
    for (int i = 0; i < NDB; ++i) o[i] *= alpha;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = exp2_fast(sc[kb][r] - mn);
        sc[kb][r] = p;
        l += p;
      }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int db = 0; db < NDB; ++db)
          o[db] = mfma16f(vt[(16 * kb + 4 * g + s) * SD + 16 * db + c], sc[kb][s], o[db]);
  }
  l += __shfl_xor(l, 16);
  l += __shfl_xor(l, 32);
  if (q < L) {
    const float inv = 1.f / l;
    T* op = (T*)a.out + b * a.bs_o + (long long)q * a.rs_o + hh * D;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = 16 * db + 4 * g + r;
        if (d < D) op[d] = stf<T>(o[db][r] * inv);
      }
    if (g == 0) a.lse[((long long)b * a.H + hh) * L + q] = (m + __log2f(l)) * (1.f / LOG2E);
  }
}

// ------------------------------------------------------------------------------------------ backward: delta
// delta[b, h, q] = sum_d dO * O (f32 of the I/O values); one wave per query row group of 64.
template <typename T>
__global__ __launch_bounds__(256) void attn_gen_delta_kernel(GenArgs a) {
  const int q = blockIdx.x * 256 + threadIdx.x, hh = blockIdx.y, b = blockIdx.z;
  if (q >= a.L) return;
  const T* op = (const T*)a.o + b * a.bs_o + (long long)q * a.rs_o + hh * a.D;
  const T* dp = (const T*)a.dout + b * a.bs_o + (long long)q * a.rs_o + hh * a.D;
  float acc = 0.f;
  for (int d = 0; d < a.D; ++d) acc = fmaf(ldf<T>(op + d), ldf<T>(dp + d), acc);
  a.delta[((long long)b * a.H + hh) * a.L + q] = acc;
}

// ------------------------------------------------------------------------------------------ backward: dK, dV
// Workgroup = 4 waves x 16 keys (K, V operand fragments in registers); query tiles of 32 (Q, dO, lse, delta) staged
// in LDS. Per 16-query block: S = Q K^T and dP = dO V^T (query on the accumulator row, key on the lane),
// P = exp(scale S - lse), dS = P (dP - delta), dV^T += dO^T P, dK^T += Q^T dS.
template <typename T, int DP>
__global__ __launch_bounds__(GNW * 64) void attn_gen_bwd_dkdv_kernel(GenArgs a) {
  constexpr int SD = DP + 20, NS = DP / 4, NDB = DP / 16;
  __shared__ float qt[GT * SD], dt[GT * SD], rl[GT], rd[GT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, c = lane & 15;
  const int hh = blockIdx.y, b = blockIdx.z, L = a.L, D = a.D;
  const int key = blockIdx.x * (GNW * 16) + wave * 16 + c;
  const T* qp = (const T*)a.q + b * a.bs_qkv + hh * D;
  const T* kp = (const T*)a.k + b * a.bs_qkv + hh * D;
  const T* vp = (const T*)a.v + b * a.bs_qkv + hh * D;
  const T* dop = (const T*)a.dout + b * a.bs_o + hh * D;
  const float* lse = a.lse + ((long long)b * a.H + hh) * L;
  const float* del = a.delta + ((long long)b * a.H + hh) * L;
  float kf[NS], vf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int d = 4 * s + g;
    const bool ok = key < L && d < D;
    kf[s] = ok ? ldf<T>(kp + (long long)key * a.rs_qkv + d) : 0.f;
    vf[s] = ok ? ldf<T>(vp + (long long)key * a.rs_qkv + d) : 0.f;
  }
  f32x4 dv[NDB], dk[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) dv[i] = dk[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float c2 = a.scale * LOG2E;
  for (int t0 = 0; t0 < L; t0 += GT) {
    __syncthreads();
    g_stage<T, DP>(qt, qp, a.rs_qkv, t0, L, D, tid);
    g_stage<T, DP>(dt, dop, a.rs_o, t0, L, D, tid);
    if (tid < GT) {   // rows past L: P = 0 (lse = +big), delta = 0
      rl[tid] = t0 + tid < L ? lse[t0 + tid] * LOG2E : -G_NEG;
      rd[tid] = t0 + tid < L ? del[t0 + tid] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      f32x4 sc = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sc = mfma16f(qt[(16 * qb + c) * SD + 4 * s + g], kf[s], sc);
        dp = mfma16f(dt[(16 * qb + c) * SD + 4 * s + g], vf[s], dp);
      }
      const f32x4 lv = *(const f32x4*)&rl[16 * qb + 4 * g];
      const f32x4 dv4 = *(const f32x4*)&rd[16 * qb + 4 * g];
      f32x4 p, ds;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        p[r] = exp2_fast(sc[r] * c2 - lv[r]);
        ds[r] = p[r] * (dp[r] - dv4[r]);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          dv[db] = mfma16f(dt[(16 * qb + 4 * g + s) * SD + 16 * db + c], p[s], dv[db]);
          dk[db] = mfma16f(qt[(16 * qb + 4 * g + s) * SD + 16 * db + c], ds[s], dk[db]);
        }
    }
  }
  if (key < L) {
    T* dkp = (T*)a.dk + b * a.bs_qkv + (long long)key * a.rs_qkv + hh * D;
    T* dvp = (T*)a.dv + b * a.bs_qkv + (long long)key * a.rs_qkv + hh * D;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = 16 * db + 4 * g + r;
        if (d < D) {
          dkp[d] = stf<T>(dk[db][r] * a.scale);
          dvp[d] = stf<T>(dv[db][r]);
        }
      }
  }
}

// ------------------------------------------------------------------------------------------------ backward: dQ
// Workgroup = 4 waves x 16 queries (Q, dO operand fragments in registers, lse / delta per lane); key tiles of 32
// (K, V) in LDS. Per 16-key block: S^T = K Q^T, dP^T = V dO^T (key on the accumulator row, query on the lane),
// dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T.
template <typename T, int DP>
__global__ __launch_bounds__(GNW * 64) void attn_gen_bwd_dq_kernel(GenArgs a) {
  constexpr int SD = DP + 20, NS = DP / 4, NDB = DP / 16;
  __shared__ float kt[GT * SD], vt[GT * SD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, c = lane & 15;
  const int hh = blockIdx.y, b = blockIdx.z, L = a.L, D = a.D;
  const int q = blockIdx.x * (GNW * 16) + wave * 16 + c;
  const T* qp = (const T*)a.q + b * a.bs_qkv + hh * D;
  const T* kp = (const T*)a.k + b * a.bs_qkv + hh * D;
  const T* vp = (const T*)a.v + b * a.bs_qkv + hh * D;
  const T* dop = (const T*)a.dout + b * a.bs_o + hh * D;
  float qf[NS], df[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int d = 4 * s + g;
    const bool ok = q < L && d < D;
    qf[s] = ok ? ldf<T>(qp + (long long)q * a.rs_qkv + d) : 0.f;
    df[s] = ok ? ldf<T>(dop + (long long)q * a.rs_o + d) : 0.f;
  }
  const long long ri = ((long long)b * a.H + hh) * L + (q < L ? q : 0);
  const float lq = q < L ? a.lse[ri] * LOG2E : -G_NEG;
  const float dq_ = q < L ? a.delta[ri] : 0.f;
  f32x4 dq[NDB];
#pragma unroll
  for (int i = 0; i < NDB; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float c2 = a.scale * LOG2E;
  for (int t0 = 0; t0 < L; t0 += GT) {
    __syncthreads();
    g_stage<T, DP>(kt, kp, a.rs_qkv, t0, L, D, tid);
    g_stage<T, DP>(vt, vp, a.rs_qkv, t0, L, D, tid);
    __syncthreads();
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      f32x4 sc = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sc = mfma16f(kt[(16 * kb + c) * SD + 4 * s + g], qf[s], sc);
        dp = mfma16f(vt[(16 * kb + c) * SD + 4 * s + g], df[s], dp);
      }
      f32x4 ds;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = t0 + 16 * kb + 4 * g + r < L ? exp2_fast(sc[r] * c2 - lq) : 0.f;
        ds[r] = p * (dp[r] - dq_);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int db = 0; db < NDB; ++db)
          dq[db] = mfma16f(kt[(16 * kb + 4 * g + s) * SD + 16 * db + c], ds[s], dq[db]);
    }
  }
  if (q < L) {
    T* dqp = (T*)a.out + b * a.bs_qkv + (long long)q * a.rs_qkv + hh * D;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = 16 * db + 4 * g + r;
        if (d < D) dqp[d] = stf<T>(dq[db][r] * a.scale);
      }
  }
}

}  // namespace lci

// =============================================================================== C-ABI entry points
using namespace lci;

static int gen_args(GenArgs& a, int dtype, const void* qkv, int B, int L, int H, int D, float scale) {
  LCI_CHECK(dtype == 0 || dtype == 1, "lci_attn_gen: dtype %d (0 = f32, 1 = bf16)", dtype);
  LCI_CHECK(B > 0 && L > 0 && H > 0 && D > 0 && D <= 256, "lci_attn_gen: bad shape B=%d L=%d H=%d D=%d (D <= 256)",
            B, L, H, D);
  const size_t es = dtype == 0 ? 4 : 2;
  const char* base = (const char*)qkv;
  a.q = base; a.k = base + (size_t)H * D * es; a.v = base + (size_t)2 * H * D * es;
  a.bs_qkv = (long long)L * 3 * H * D; a.rs_qkv = 3 * H * D;
  a.bs_o = (long long)L * H * D; a.rs_o = H * D;
  a.H = H; a.L = L; a.D = D; a.scale = scale;
  return 0;
}

template <typename T, int DP>
static void gen_fwd_launch(const GenArgs& a, int B, hipStream_t s) {
  hipLaunchKernelGGL((attn_gen_fwd_kernel<T, DP>), dim3((a.L + GNW * 16 - 1) / (GNW * 16), a.H, B), dim3(GNW * 64), 0,
                     s, a);
}
template <typename T, int DP>
static void gen_bwd_launch(const GenArgs& a, int B, hipStream_t s) {
  const dim3 grid((a.L + GNW * 16 - 1) / (GNW * 16), a.H, B);
  hipLaunchKernelGGL((attn_gen_bwd_dkdv_kernel<T, DP>), grid, dim3(GNW * 64), 0, s, a);
  hipLaunchKernelGGL((attn_gen_bwd_dq_kernel<T, DP>), grid, dim3(GNW * 64), 0, s, a);
}

#define GEN_DISPATCH(FN, dtype, D, ...)                                     \
  do {                                                                      \
    if (dtype == 0) {                                                       \
      if (D <= 64) FN<float, 64>(__VA_ARGS__);                              \
      else if (D <= 128) FN<float, 128>(__VA_ARGS__);                       \
      else FN<float, 256>(__VA_ARGS__);                                     \
    } else {                                                                \
      if (D <= 64) FN<bf16, 64>(__VA_ARGS__);                               \
      else if (D <= 128) FN<bf16, 128>(__VA_ARGS__);                        \
      else FN<bf16, 256>(__VA_ARGS__);                                      \
    }                                                                       \
  } while (0)

extern "C" int lci_attn_gen_fwd(int dtype, const void* qkv, void* out, float* lse, int B, int L, int H, int head_dim,
                                float scale, void* stream) {
  GenArgs a{};
  if (gen_args(a, dtype, qkv, B, L, H, head_dim, scale)) return 1;
  LCI_CHECK(out && lse, "lci_attn_gen_fwd: null output");
  a.out = out; a.lse = lse;
  GEN_DISPATCH(gen_fwd_launch, dtype, head_dim, a, B, (hipStream_t)stream);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_attn_gen_bwd(int dtype, const void* qkv, const void* out, const void* dout, const float* lse,
                                void* dqkv, float* delta_ws, int B, int L, int H, int head_dim, float scale,
                                void* stream) {
  GenArgs a{};
  if (gen_args(a, dtype, qkv, B, L, H, head_dim, scale)) return 1;
  LCI_CHECK(out && dout && lse && dqkv && delta_ws, "lci_attn_gen_bwd: null argument");
  const size_t es = dtype == 0 ? 4 : 2;
  a.o = out; a.dout = dout; a.lse = (float*)lse; a.delta = delta_ws;
  a.out = dqkv; a.dk = (char*)dqkv + (size_t)H * head_dim * es; a.dv = (char*)dqkv + (size_t)2 * H * head_dim * es;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 0)
    hipLaunchKernelGGL(attn_gen_delta_kernel<float>, dim3((L + 255) / 256, H, B), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(attn_gen_delta_kernel<bf16>, dim3((L + 255) / 256, H, B), dim3(256), 0, s, a);
  LCI_LAUNCH_CHECK();
  GEN_DISPATCH(gen_bwd_launch, dtype, head_dim, a, B, s);
  LCI_LAUNCH_CHECK();
  return 0;
}
