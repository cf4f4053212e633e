// Adam / AdamW parameter update over a list of f32 tensors, one launch per up to ADAM_MAXT tensors.
//
// The trainer's optimizer step (trainer_base.py:171-177 -> torch.optim.Adam / AdamW, optim_base.py:87-89): torch's fused
// kernel deals each launch's tensors out in 64-K-element chunks, one workgroup each, so a 62-M-parameter model
// (SwinUNETR) runs ~1000 workgroups over 16 launches at ~1 TB/s (1.8 ms of the C3 step). Here every workgroup takes
// ADAM_CHUNK elements, so the grid covers the chip and the update streams near the HBM rate (28 bytes per parameter:
// read p, g, m, v, write p, m, v). Round 6: 4096 elements per workgroup as four 1-KB-per-wave groups, all 16 loads of a
// thread issued before the arithmetic, and the bias corrections (f64 pow) evaluated once per workgroup. The arithmetic follows torch's FusedAdamMathFunctor (ATen fused_adam_utils.cuh): the
// moment updates in f64 from f32 operands, bias corrections from the device step count (f64 pow, kept in f32),
// step size and denominator rounded to f32, the final update in f32 -- so results match torch's fused Adam.
#include "common.hpp"

namespace lci {

constexpr int ADAM_MAXT = 40;       // tensors per launch (kernel-argument space)
constexpr int ADAM_CHUNK = 4096;    // elements per workgroup (256 threads x 4 groups of 4)

struct AdamTensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  const float* step;   // this tensor's step count (already incremented for this update)
  long long n;
};

struct AdamArgs {
  AdamTensor t[ADAM_MAXT];
  int blk0[ADAM_MAXT + 1];   // first workgroup of each tensor (prefix sums), blk0[nt] = grid size
  int nt;
  double lr, beta1, beta2, wd, eps;
  int adamw, maximize;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamArgs& a, float step_size,
                                          float bc2s) {
  float grad = a.maximize ? -g : g;
  if (a.wd != 0.0) {
    if (a.adamw) p = (float)((double)p - a.lr * a.wd * (double)p);
    else grad = (float)((double)grad + (double)p * a.wd);
  }
  m = (float)(a.beta1 * (double)m + (1.0 - a.beta1) * (double)grad);
  v = (float)(a.beta2 * (double)v + (1.0 - a.beta2) * (double)grad * (double)grad);
  const float denom = (float)((double)(sqrtf(v) / bc2s) + a.eps);
  p -= step_size * m / denom;
}

__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < a.nt && a.blk0[k + 1] <= b) ++k;   // this workgroup's tensor (uniform)
  const AdamTensor& t = a.t[k];
  const long long e0 = (long long)(b - a.blk0[k]) * ADAM_CHUNK;
  __shared__ float coef[2];
  if (threadIdx.x == 0) {
    const float stp = *t.step;
    const float bc1 = (float)(1.0 - pow(a.beta1, (double)stp));
    coef[0] = (float)(a.lr / (double)bc1);                          // step size
    coef[1] = (float)sqrt(1.0 - pow(a.beta2, (double)stp));         // sqrt(bias correction 2)
  }
  __syncthreads();
  const float step_size = coef[0], bc2s = coef[1];
  const bool vec = (((uintptr_t)t.p | (uintptr_t)t.g | (uintptr_t)t.m | (uintptr_t)t.v) & 15) == 0;
  const long long i0 = e0 + 4LL * threadIdx.x;   // group h: elements i0 + 1024 h .. + 3
  if (vec && e0 + ADAM_CHUNK <= t.n) {
    f32x4 p[4], g[4], m[4], v[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const long long i = i0 + 1024 * h;
      p[h] = *(const f32x4*)(t.p + i); g[h] = *(const f32x4*)(t.g + i);
      m[h] = *(const f32x4*)(t.m + i); v[h] = *(const f32x4*)(t.v + i);
    }
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const long long i = i0 + 1024 * h;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pj = p[h][j], mj = m[h][j], vj = v[h][j];
        adam_elem(pj, g[h][j], mj, vj, a, step_size, bc2s);
        p[h][j] = pj; m[h][j] = mj; v[h][j] = vj;
      }
      *(f32x4*)(t.p + i) = p[h];
      *(f32x4*)(t.m + i) = m[h];
      *(f32x4*)(t.v + i) = v[h];
    }
  } else {
    for (int h = 0; h < 4; ++h)
      for (long long i = i0 + 1024 * h; i < i0 + 1024 * h + 4 && i < t.n; ++i) {
        float p = t.p[i], m = t.m[i], v = t.v[i];
        adam_elem(p, t.g[i], m, v, a, step_size, bc2s);
        t.p[i] = p; t.m[i] = m; t.v[i] = v;
      }
  }
}

}  // namespace lci

using namespace lci;

extern "C" int lci_adam_max_tensors(void) { return ADAM_MAXT; }

extern "C" int lci_adam_step(float* const* p, const float* const* g, float* const* m, float* const* v,
                             const float* const* step, const long long* n, int nt, double lr, double beta1,
                             double beta2, double weight_decay, double eps, int adamw, int maximize, void* stream) {
  LCI_CHECK(nt >= 1 && nt <= ADAM_MAXT, "adam_step: %d tensors (1 .. %d per call)", nt, ADAM_MAXT);
  AdamArgs a{};
  long long blocks = 0;
  for (int i = 0; i < nt; ++i) {
    LCI_CHECK(n[i] >= 0 && p[i] && g[i] && m[i] && v[i] && step[i], "adam_step: tensor %d: null pointer or bad size", i);
    a.t[i] = AdamTensor{p[i], g[i], m[i], v[i], step[i], n[i]};
    a.blk0[i] = (int)blocks;
    blocks += (n[i] + ADAM_CHUNK - 1) / ADAM_CHUNK;
    LCI_CHECK(blocks < (1LL << 31), "adam_step: too many elements in one call");
  }
  a.blk0[nt] = (int)blocks;
  a.nt = nt;
  a.lr = lr; a.beta1 = beta1; a.beta2 = beta2; a.wd = weight_decay; a.eps = eps;
  a.adamw = adamw; a.maximize = maximize;
  if (blocks == 0) return 0;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}
