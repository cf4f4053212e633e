// Patch embedding (conv with kernel = stride = patch) for gfx950.
//
// Replaces MONAI-1.3 PatchEmbeddingBlock (ViT, backbone_vit.py:351-361, forward :383):
//     y[b, t, d] = bias[d] + sum_k W[d, k] * patch(b, t)[k] + pos[t, d]            (tokens channels-last)
// and MONAI-1.3 PatchEmbed (Swin, backbone_swin.py:800-806, forward :885): right zero-pad to a patch multiple,
//     y[b, d, t] = bias[d] + sum_k W[d, k] * patch(b, t)[k]                         (channels-first grid)
// k enumerates (c, i0, i1[, i2]) in the conv weight's memory order. HBM-bound: the output dominates traffic.
//
// Forward: a workgroup owns T tokens of one sample (T*K <= 4096 patch values staged in LDS), every thread
// produces 4 consecutive channels (channels-last: float4 store) or one (channel, token) (channels-first).
// Backward: dpos[t, d] = sum_b dy[b, t, d] (direct), dbias/dW block-partial sums -> f32 atomics (D*K words).
#include "common.hpp"

namespace lci {

struct PatchArgs {
  const void* x;        // (B, C, S0, S1[, S2]) f32 or bf16
  const float* w;       // (D, K) f32
  const float* bias;    // (D) or null
  const float* pos;     // (L, D) or null
  void* y;              // output, f32 or bf16
  const void* dy;       // bwd: same layout/dtype as y
  float* dw; float* db; float* dpos;
  int B, C, D, K, L, T;
  int nd;               // spatial dims (2 or 3)
  int S[3], P[3], G[3]; // image size, patch size, patch grid (ceil)
  int channels_last;    // 1: y (B, L, D); 0: y (B, D, L)
};

template <typename Tin>
__device__ __forceinline__ float ld_in(const Tin* p, long long i) { return (float)p[i]; }

// value of patch element k of token t (zero beyond the image: right padding)
template <typename Tin>
__device__ __forceinline__ float patch_val(const PatchArgs& a, const Tin* x, int b, int t, int k) {
  int g[3], i[3];
  int rem = t;
  for (int s = a.nd - 1; s >= 0; --s) { g[s] = rem % a.G[s]; rem /= a.G[s]; }
  int kr = k;
  for (int s = a.nd - 1; s >= 0; --s) { i[s] = kr % a.P[s]; kr /= a.P[s]; }
  const int c = kr;
  long long off = ((long long)b * a.C + c);
  for (int s = 0; s < a.nd; ++s) {
    const int p = g[s] * a.P[s] + i[s];
    if (p >= a.S[s]) return 0.f;
    off = off * a.S[s] + p;
  }
  return ld_in(x, off);
}

template <typename Tin, typename Tout>
__global__ __launch_bounds__(256) void patch_embed_fwd_kernel(PatchArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sp[];  // [T][K]
  const int b = blockIdx.y, t0 = blockIdx.x * a.T;
  const int T = min(a.T, a.L - t0);
  const Tin* x = (const Tin*)a.x;
  for (int idx = threadIdx.x; idx < T * a.K; idx += blockDim.x) {
    const int t = idx / a.K, k = idx % a.K;
    sp[idx] = patch_val(a, x, b, t0 + t, k);
  }
  __syncthreads();
  Tout* y = (Tout*)a.y;
  if (a.channels_last) {
    const int DQ = a.D >> 2;
    for (int idx = threadIdx.x; idx < T * DQ; idx += blockDim.x) {
      const int t = idx / DQ, d = (idx % DQ) * 4;
      float acc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = a.bias ? a.bias[d + j] : 0.f;
      const float* pv = sp + t * a.K;
      for (int k = 0; k < a.K; ++k) {
        const float v = pv[k];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = fmaf(a.w[(d + j) * a.K + k], v, acc[j]);
      }
      if (a.pos) {
        const f32x4 pp = *(const f32x4*)(a.pos + (long long)(t0 + t) * a.D + d);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += pp[j];
      }
      Tout* o = y + ((long long)b * a.L + t0 + t) * a.D + d;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (Tout)acc[j];
    }
  } else {
    for (int idx = threadIdx.x; idx < T * a.D; idx += blockDim.x) {
      const int d = idx / T, t = idx % T;
      float acc = a.bias ? a.bias[d] : 0.f;
      const float* pv = sp + t * a.K;
      const float* wr = a.w + (long long)d * a.K;
      for (int k = 0; k < a.K; ++k) acc = fmaf(wr[k], pv[k], acc);
      y[((long long)b * a.D + d) * a.L + t0 + t] = (Tout)acc;
    }
  }
}

// dW[d, k] += sum_t dy[b, t, d] patch(b, t)[k];  db[d] += sum_t dy[b, t, d]   (block-partial -> atomics)
template <typename Tin, typename Tg>
__global__ __launch_bounds__(256) void patch_embed_bwd_w_kernel(PatchArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sp[];  // [T][K]
  const int b = blockIdx.y, t0 = blockIdx.x * a.T;
  const int T = min(a.T, a.L - t0);
  const Tin* x = (const Tin*)a.x;
  for (int idx = threadIdx.x; idx < T * a.K; idx += blockDim.x) {
    const int t = idx / a.K, k = idx % a.K;
    sp[idx] = patch_val(a, x, b, t0 + t, k);
  }
  __syncthreads();
  const Tg* dy = (const Tg*)a.dy;
  const int npairs = a.D * (a.K + 1);  // k == K column is the bias
  for (int pr = threadIdx.x; pr < npairs; pr += blockDim.x) {
    const int d = pr / (a.K + 1), k = pr % (a.K + 1);
    float acc = 0.f;
    for (int t = 0; t < T; ++t) {
      const long long yi = a.channels_last ? ((long long)b * a.L + t0 + t) * a.D + d
                                           : ((long long)b * a.D + d) * a.L + t0 + t;
      const float g = (float)dy[yi];
      acc = fmaf(g, k < a.K ? sp[t * a.K + k] : 1.f, acc);
    }
    if (k < a.K) atomicAdd(a.dw + d * a.K + k, acc);
    else if (a.db) atomicAdd(a.db + d, acc);
  }
}

// dpos[t, d] = sum_b dy[b, t, d]   (channels-last only)
template <typename Tg>
__global__ __launch_bounds__(256) void patch_embed_bwd_pos_kernel(PatchArgs a) {
  const long long n = (long long)a.L * a.D;
  const Tg* dy = (const Tg*)a.dy;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float acc = 0.f;
    for (int b = 0; b < a.B; ++b) acc += (float)dy[(long long)b * n + i];
    a.dpos[i] = acc;
  }
}

static int fill_args(PatchArgs& a, int B, int C, int D, int nd, const int* S, const int* P, int channels_last) {
  LCI_CHECK(nd == 2 || nd == 3, "patch_embed: spatial dims %d", nd);
  a.B = B; a.C = C; a.D = D; a.nd = nd; a.channels_last = channels_last;
  a.K = C; a.L = 1;
  for (int s = 0; s < 3; ++s) { a.S[s] = 1; a.P[s] = 1; a.G[s] = 1; }
  for (int s = 0; s < nd; ++s) {
    LCI_CHECK(S[s] > 0 && P[s] > 0, "patch_embed: bad size/patch");
    a.S[s] = S[s]; a.P[s] = P[s]; a.G[s] = (S[s] + P[s] - 1) / P[s];
    a.K *= P[s]; a.L *= a.G[s];
  }
  LCI_CHECK(a.K <= 4096, "patch_embed: patch volume %d too large", a.K);
  a.T = 4096 / a.K; if (a.T > 64) a.T = 64;
  LCI_CHECK(!channels_last || D % 4 == 0, "patch_embed: D %% 4 != 0");
  return 0;
}

}  // namespace lci

using namespace lci;

// dtype codes: 0 = f32, 1 = bf16
extern "C" int lci_patch_embed_fwd(const void* x, int x_dtype, const float* w, const float* bias, const float* pos,
                                   void* y, int y_dtype, int B, int C, int D, int nd, const int* img_size,
                                   const int* patch, int channels_last, void* stream) {
  PatchArgs a{};
  if (fill_args(a, B, C, D, nd, img_size, patch, channels_last)) return 1;
  LCI_CHECK(!(pos && !channels_last), "patch_embed: pos only with channels-last tokens");
  a.x = x; a.w = w; a.bias = bias; a.pos = pos; a.y = y;
  dim3 grid((a.L + a.T - 1) / a.T, B);
  const size_t sh = (size_t)a.T * a.K * 4;
  hipStream_t s = (hipStream_t)stream;
  if (x_dtype == 0 && y_dtype == 0) hipLaunchKernelGGL((patch_embed_fwd_kernel<float, float>), grid, dim3(256), sh, s, a);
  else if (x_dtype == 0 && y_dtype == 1) hipLaunchKernelGGL((patch_embed_fwd_kernel<float, bf16>), grid, dim3(256), sh, s, a);
  else if (x_dtype == 1 && y_dtype == 0) hipLaunchKernelGGL((patch_embed_fwd_kernel<bf16, float>), grid, dim3(256), sh, s, a);
  else if (x_dtype == 1 && y_dtype == 1) hipLaunchKernelGGL((patch_embed_fwd_kernel<bf16, bf16>), grid, dim3(256), sh, s, a);
  else LCI_CHECK(false, "patch_embed_fwd: dtype codes %d/%d", x_dtype, y_dtype);
  LCI_LAUNCH_CHECK();
  return 0;
}

// dw (D*K) and db (D) must be zeroed by the caller (accumulated with atomics); dpos (L, D) is overwritten.
extern "C" int lci_patch_embed_bwd(const void* x, int x_dtype, const void* dy, int dy_dtype, float* dw, float* db,
                                   float* dpos, int B, int C, int D, int nd, const int* img_size, const int* patch,
                                   int channels_last, void* stream) {
  PatchArgs a{};
  if (fill_args(a, B, C, D, nd, img_size, patch, channels_last)) return 1;
  LCI_CHECK(!(dpos && !channels_last), "patch_embed: dpos only with channels-last tokens");
  a.x = x; a.dy = dy; a.dw = dw; a.db = db; a.dpos = dpos;
  hipStream_t s = (hipStream_t)stream;
  // more tokens per block for the reduction (fewer atomics), bounded by LDS
  a.T = 16384 / a.K; if (a.T > 256) a.T = 256; if (a.T < 1) a.T = 1;
  dim3 grid((a.L + a.T - 1) / a.T, B);
  const size_t sh = (size_t)a.T * a.K * 4;
  if (x_dtype == 0 && dy_dtype == 0) hipLaunchKernelGGL((patch_embed_bwd_w_kernel<float, float>), grid, dim3(256), sh, s, a);
  else if (x_dtype == 0 && dy_dtype == 1) hipLaunchKernelGGL((patch_embed_bwd_w_kernel<float, bf16>), grid, dim3(256), sh, s, a);
  else if (x_dtype == 1 && dy_dtype == 0) hipLaunchKernelGGL((patch_embed_bwd_w_kernel<bf16, float>), grid, dim3(256), sh, s, a);
  else if (x_dtype == 1 && dy_dtype == 1) hipLaunchKernelGGL((patch_embed_bwd_w_kernel<bf16, bf16>), grid, dim3(256), sh, s, a);
  else LCI_CHECK(false, "patch_embed_bwd: dtype codes %d/%d", x_dtype, dy_dtype);
  LCI_LAUNCH_CHECK();
  if (dpos) {
    const long long n = (long long)a.L * D;
    int blocks = (int)((n + 255) / 256); if (blocks > 4096) blocks = 4096;
    if (dy_dtype == 0) hipLaunchKernelGGL((patch_embed_bwd_pos_kernel<float>), dim3(blocks), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((patch_embed_bwd_pos_kernel<bf16>), dim3(blocks), dim3(256), 0, s, a);
    LCI_LAUNCH_CHECK();
  }
  return 0;
}
