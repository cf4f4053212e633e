// Hyena long convolution for gfx950.
//
// Replaces fftconv_ref (hyena.py:32-51, gelu=False, no dropout):
//     y = irfft(rfft(u, n=2L) * rfft(k, n=2L) / 2L, n=2L, norm="forward")[..., :L] + u * D
// i.e. the causal linear convolution y[t] = sum_{s<=t} k[t-s] u[s] + D u[t], evaluated exactly (fp32) with
// an FFT of size n = pow2 >= 2L. Two rows that share a filter are packed as one complex sequence
// z = u_a + i u_b (k is real, so conv(z, k) = conv(u_a, k) + i conv(u_b, k)).
//
// Four-step FFT, n = n1 * n2, index m = a*n2 + c, frequency f = k1 + n1*k2:
//   col pass   (per pair, G columns c):  T[k1][c] = FFT_n1 over a of z[a*n2+c], times W_n^(c k1)
//   row pass   (per filter j, row k1, looping over that filter's pairs): X[k1][k2] = FFT_n2 over c;
//              times K_j[k1][k2] (or conj(K_j) for the adjoint); inverse FFT_n2; conj twiddle applied in
//              the inverse column pass. The backward also accumulates sum_pairs conj(X_vg) X_dy for dk.
//   inverse col pass: IFFT_n1 over k1 -> z[m]; Re -> row a, Im -> row b, + D * u.
// Sub-FFTs are radix-2 Stockham in LDS (ping-pong); twiddles come from one W_n table built in f64.
// hyena_pre / hyena_post: the causal depthwise short conv (k = short_filter_order) and gating around the
// long conv, reading/writing the channels-last (B, L, C) tensors of in_proj / out_proj directly and
// transposing through LDS to the channel-major rows the FFT wants.
#include "common.hpp"

#include <algorithm>
#include <initializer_list>

namespace lci {

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 cmul(f32x2 a, f32x2 b) { return f32x2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ f32x2 cmulc(f32x2 a, f32x2 b) {  // a * conj(b)
  return f32x2{a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y};
}
__device__ __forceinline__ f32x2 conj2(f32x2 a) { return f32x2{a.x, -a.y}; }

struct FftArgs {
  const float* src; const float* src2;  // rows (R_outer, C, L) f32 channel-major; src2: second input (vg) for dk
  float* dst;                           // output rows
  const f32x2* tw;                      // W_n^t, t < n
  f32x2* S; f32x2* S2;                  // scratch (npairs_total, n) complex
  f32x2* So;                            // row pass output when not in place (forward with a kept input spectrum)
  f32x2* K;                             // filter spectra (C, n) in [k1][k2] layout (already / n)
  f32x2* SK;                            // dk scratch (C, n)
  const float* Dv;                      // (C) or null
  float* dk; float* dD;                 // (C, L) and (C) outputs (bwd)
  int L, C, R, P;                       // row length, filters, outer rows per filter, pairs per filter
  int n, n1, n2, ln1, ln2, G;
  int mode;                             // row pass: 0 = spectrum of filters, 1 = fwd conv, 2 = bwd (conj + dk)
  int single;                           // col passes: 1 = the source is the filter (C rows, no pairing)
  int pid0;                             // first pair (col passes) / filter (row pass) of this launch's chunk
  int pb;                               // row pass: sequences per LDS batch (ROW_PB)
};

// ------------------------------------------------------------------- sub-FFTs: radix-8/4/2 Stockham in LDS
// Each pass: a thread takes one radix-R butterfly (R points strided N/R apart) into registers, applies the
// twiddles W_{Ns R}^{m r} (from the LDS table twl[t] = W_N^t), does the R-point DFT in registers and writes the
// R outputs Ns apart (Stockham auto-sort). N = 512 is three radix-8 passes (3 LDS round trips, 3 barriers).
template <bool INV> __device__ __forceinline__ f32x2 mul_mi(f32x2 v) {   // v * (-i) forward, v * (+i) inverse
  return INV ? f32x2{-v.y, v.x} : f32x2{v.y, -v.x};
}

template <int R, bool INV> __device__ __forceinline__ void dft(f32x2 (&v)[R]) {
  if constexpr (R == 2) {
    const f32x2 a = v[0], b = v[1];
    v[0] = a + b; v[1] = a - b;
  } else if constexpr (R == 4) {
    const f32x2 t0 = v[0] + v[2], t1 = v[0] - v[2], t2 = v[1] + v[3], t3 = mul_mi<INV>(v[1] - v[3]);
    v[0] = t0 + t2; v[2] = t0 - t2; v[1] = t1 + t3; v[3] = t1 - t3;
  } else {
    constexpr float H = 0.70710678118654752f;
    const f32x2 t0 = v[0] + v[4], t1 = v[0] - v[4], t2 = v[2] + v[6], t3 = mul_mi<INV>(v[2] - v[6]);
    const f32x2 t4 = v[1] + v[5], t5 = v[1] - v[5], t6 = v[3] + v[7], t7 = mul_mi<INV>(v[3] - v[7]);
    const f32x2 e0 = t0 + t2, e2 = t0 - t2, e1 = t1 + t3, e3 = t1 - t3;   // DFT4 of the even points
    f32x2 o0 = t4 + t6, o2 = t4 - t6, o1 = t5 + t7, o3 = t5 - t7;         // DFT4 of the odd points
    // o_k *= W8^k (forward W8 = (1 - i)/sqrt2; inverse conjugate)
    o1 = INV ? f32x2{(o1.x - o1.y) * H, (o1.x + o1.y) * H} : f32x2{(o1.x + o1.y) * H, (o1.y - o1.x) * H};
    o2 = mul_mi<INV>(o2);
    o3 = INV ? f32x2{-(o3.x + o3.y) * H, (o3.x - o3.y) * H} : f32x2{(o3.y - o3.x) * H, -(o3.x + o3.y) * H};
    v[0] = e0 + o0; v[4] = e0 - o0;
    v[1] = e1 + o1; v[5] = e1 - o1;
    v[2] = e2 + o2; v[6] = e2 - o2;
    v[3] = e3 + o3; v[7] = e3 - o3;
  }
}

template <int R, bool INV>
__device__ __forceinline__ void stockham_pass(const f32x2* x, f32x2* y, int N, int Ns, int cnt, const f32x2* twl,
                                              int ld) {
  const int nb = N / R;
  const int tstep = N / (Ns * R);
  for (int idx = threadIdx.x; idx < cnt * nb; idx += blockDim.x) {
    const int sq = idx / nb, j = idx - sq * nb;
    const int m = j & (Ns - 1);
    const f32x2* xs = x + sq * ld;
    f32x2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = xs[j + r * nb];
    if (Ns > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r) {
        f32x2 w = twl[(m * r * tstep) & (N - 1)];
        if (INV) w.y = -w.y;
        v[r] = cmul(v[r], w);
      }
    }
    dft<R, INV>(v);
    f32x2* ys = y + sq * ld + (j - m) * R + m;
#pragma unroll
    for (int r = 0; r < R; ++r) ys[r * Ns] = v[r];
  }
}

// FFT of `cnt` sequences of length N = 2^lN stored ld apart in x (ping-pong through y); returns the buffer
// holding the result. twl: W_N^t for t < N (LDS). Unnormalised inverse when INV.
template <bool INV>
__device__ f32x2* lds_fft(f32x2* x, f32x2* y, int N, int lN, int cnt, const f32x2* twl, int ld) {
  int Ns = 1, left = lN;
  while (left > 0) {
    if (left >= 3 && left != 4) { stockham_pass<8, INV>(x, y, N, Ns, cnt, twl, ld); Ns *= 8; left -= 3; }
    else if (left >= 2) { stockham_pass<4, INV>(x, y, N, Ns, cnt, twl, ld); Ns *= 4; left -= 2; }
    else { stockham_pass<2, INV>(x, y, N, Ns, cnt, twl, ld); Ns *= 2; left -= 1; }
    __syncthreads();
    f32x2* t = x; x = y; y = t;
  }
  return x;
}

// twl[t] = W_N^t = W_n^(t n / N), t < N, from the f64-built table
__device__ __forceinline__ void load_twl(f32x2* twl, const f32x2* tw, int N, int n) {
  for (int t = threadIdx.x; t < N; t += blockDim.x) twl[t] = tw[(long long)t * (n / N)];
}

constexpr int UB = 8;   // global loads in flight per thread in the staging loops

__device__ __forceinline__ int pair_row(const FftArgs& a, int j, int p, int which) {
  const int ro = 2 * p + which;
  return ro < a.R ? ro * a.C + j : -1;
}

// ------------------------------------------------------------------------------------- forward columns
// grid: (n2 / G, npairs_total or C); block 256. LDS: 2 * G * n1 complex.
__global__ __launch_bounds__(256) void fft_col_fwd_kernel(FftArgs a) {
  extern __shared__ __attribute__((aligned(16))) f32x2 lds[];
  const int ld = a.n1 + 1;   // padded column stride: the G columns' transposing accesses hit distinct banks
  f32x2* x = lds;
  f32x2* y = lds + a.G * ld;
  f32x2* twl = y + a.G * ld;
  load_twl(twl, a.tw, a.n1, a.n);
  const int c0 = blockIdx.x * a.G;
  const int pid = a.pid0 + blockIdx.y;  // pair id (j * P + p) or filter id when single
  int r0, r1;
  if (a.single) { r0 = pid; r1 = -1; }
  else {
    const int j = pid / a.P, p = pid % a.P;
    r0 = pair_row(a, j, p, 0);
    r1 = pair_row(a, j, p, 1);
  }
  const float* s = a.src;
  const int total = a.G * a.n1;
  // UB items per thread in flight: all of a batch's global loads issue before any LDS store
  for (int base = 0; base < total; base += UB * blockDim.x) {
    f32x2 v[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = base + u * blockDim.x + threadIdx.x;
      const int g = idx % a.G, ai = idx / a.G;
      const int m = ai * a.n2 + c0 + g;
      v[u] = f32x2{0.f, 0.f};
      if (idx < total && m < a.L) {
        v[u].x = s[(long long)r0 * a.L + m];
        if (r1 >= 0) v[u].y = s[(long long)r1 * a.L + m];
      }
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = base + u * blockDim.x + threadIdx.x;
      if (idx < total) x[(idx % a.G) * ld + idx / a.G] = v[u];
    }
  }
  __syncthreads();
  x = lds_fft<false>(x, y, a.n1, a.ln1, a.G, twl, ld);
  f32x2* S = (a.single ? a.SK : a.S) + (long long)pid * a.n;
  for (int base = 0; base < total; base += UB * blockDim.x) {
    f32x2 w[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = base + u * blockDim.x + threadIdx.x;
      const int g = idx % a.G, k1 = idx / a.G;
      w[u] = idx < total ? a.tw[((long long)(c0 + g) * k1) & (a.n - 1)] : f32x2{0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = base + u * blockDim.x + threadIdx.x;
      const int g = idx % a.G, k1 = idx / a.G;
      if (idx < total) S[(long long)k1 * a.n2 + c0 + g] = cmul(x[g * ld + k1], w[u]);
    }
  }
}

// ------------------------------------------------------------------------------------------ row pass
// grid: (n1, C); block 512. One (filter j, row k1); the filter's pairs go through in batches of PB sequences
// (one radix-8 butterfly per thread per pass). LDS: 2 PB n2 (+ 2 PB n2 for the bwd's second operand)
// + kr + acc + twl (n2 complex each).
constexpr int ROW_PB = 4;

__global__ __launch_bounds__(512) void fft_row_kernel(FftArgs a) {
  extern __shared__ __attribute__((aligned(16))) f32x2 lds[];
  const int N = a.n2;
  const bool two = a.mode == 2 && a.SK;           // bwd with filter gradient: also FFT the vg rows
  const int PB = two ? a.pb / 2 : a.pb;
  f32x2* x = lds;                                 // PB * N
  f32x2* y = x + PB * N;                          // PB * N
  f32x2* x2 = y + PB * N;                         // PB * N (two)
  f32x2* y2 = x2 + (two ? PB * N : 0);            // PB * N (two)
  f32x2* kr = y2 + (two ? PB * N : 0);
  f32x2* acc = kr + N;
  f32x2* twl = acc + N;
  const int k1 = blockIdx.x, j = a.pid0 + blockIdx.y;
  const float invn = 1.f / (float)a.n;
  load_twl(twl, a.tw, N, a.n);
  if (a.mode == 0) {  // filter spectrum: K_j[k1][:] = FFT_n2(T[k1][:]) / n
    f32x2* S = a.SK + (long long)j * a.n + (long long)k1 * N;
    for (int i = threadIdx.x; i < N; i += blockDim.x) x[i] = S[i];
    __syncthreads();
    f32x2* r = lds_fft<false>(x, y, N, a.ln2, 1, twl, N);
    f32x2* K = a.K + (long long)j * a.n + (long long)k1 * N;
    const float dn = a.Dv ? a.Dv[j] * invn : 0.f;   // + D / n: the spectrum of D delta (the D u term)
    for (int i = threadIdx.x; i < N; i += blockDim.x) K[i] = r[i] * invn + f32x2{dn, 0.f};
    return;
  }
  const f32x2* K = a.K + (long long)j * a.n + (long long)k1 * N;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    kr[i] = K[i];
    acc[i] = f32x2{0.f, 0.f};
  }
  for (int p0 = 0; p0 < a.P; p0 += PB) {
    const int cnt = min(PB, a.P - p0);
    for (int base = 0; base < cnt * N; base += UB * blockDim.x) {
      f32x2 v[UB], v2[UB];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int i = base + u * blockDim.x + threadIdx.x;
        const int q = i / N, e = i - q * N;
        const long long off = ((long long)j * a.P + p0 + q) * a.n + (long long)k1 * N + e;
        if (i < cnt * N) {
          v[u] = a.S[off];
          if (two) v2[u] = a.S2[off];
        }
      }
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int i = base + u * blockDim.x + threadIdx.x;
        if (i < cnt * N) {
          x[i] = v[u];
          if (two) x2[i] = v2[u];
        }
      }
    }
    __syncthreads();
    f32x2* fx = lds_fft<false>(x, y, N, a.ln2, cnt, twl, N);
    f32x2* gx = fx == x ? y : x;
    if (two) {
      f32x2* fx2 = lds_fft<false>(x2, y2, N, a.ln2, cnt, twl, N);
      for (int i = threadIdx.x; i < N; i += blockDim.x) {
        f32x2 s = acc[i];
        for (int q = 0; q < cnt; ++q) s += cmulc(fx[q * N + i], fx2[q * N + i]);   // X_dy conj(X_vg)
        acc[i] = s;
      }
      __syncthreads();   // fx is overwritten in place below
    }
    for (int i = threadIdx.x; i < cnt * N; i += blockDim.x) {
      const int e = i % N;
      fx[i] = (a.mode == 1) ? cmul(fx[i], kr[e]) : cmulc(fx[i], kr[e]);
    }
    __syncthreads();
    f32x2* rx = lds_fft<true>(fx, gx, N, a.ln2, cnt, twl, N);
    for (int i = threadIdx.x; i < cnt * N; i += blockDim.x) {
      const int q = i / N, e = i - q * N;
      (a.So ? a.So : a.S)[((long long)j * a.P + p0 + q) * a.n + (long long)k1 * N + e] = rx[i];
    }
    __syncthreads();
  }
  if (two) {  // dk spectrum row (unnormalised correlation): inverse row FFT, store
    for (int i = threadIdx.x; i < N; i += blockDim.x) x[i] = acc[i];
    __syncthreads();
    f32x2* r = lds_fft<true>(x, y, N, a.ln2, 1, twl, N);
    f32x2* SK = a.SK + (long long)j * a.n + (long long)k1 * N;
    for (int i = threadIdx.x; i < N; i += blockDim.x) SK[i] = r[i] * invn;   // correlation needs 1/n
  }
}

// --------------------------------------------------------------------- row pass, n2 = 512, one wave per row
// The 512-point row FFTs run in registers, one sequence per wave (8 points per lane) as 8 x 8 x 8: lane L holds
// x[L + 64 r]; a radix-8 DFT over r, twiddle W_512^(L k), an LDS transpose, a radix-8 DFT, twiddle W_64, a second
// transpose and a third radix-8 DFT leave X[L + 64 m] in the same lane layout, so the spectrum product and the
// inverse transform follow without a reordering, and the only synchronisation is within the wave (the LDS pass
// kernel above runs 3 workgroup-barrier passes per transform). Waves of a workgroup take different pairs of the
// same (filter, row k1); the backward's filter-gradient sum over pairs is reduced across the waves at the end.
constexpr int R5_S1 = 72;    // transpose-1 row stride (complex): the column reads of a half-wave hit distinct banks
constexpr int R5_S2 = 9;     // transpose-2 row stride

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool INV>
__device__ __forceinline__ f32x2 tw_at(const f32x2* twl, int t) {
  f32x2 w = twl[t & 511];
  if (INV) w.y = -w.y;
  return w;
}

// v[r] = x[L + 64 r] in, X[L + 64 r] out (unnormalised inverse when INV). buf: this wave's 8 * R5_S1 complex.
template <bool INV>
__device__ __forceinline__ void fft512_wave(f32x2 (&v)[8], f32x2* buf, const f32x2* twl, int L) {
  dft<8, INV>(v);                                        // over r -> k (frequency mod 8)
#pragma unroll
  for (int k = 1; k < 8; ++k) v[k] = cmul(v[k], tw_at<INV>(twl, L * k));
#pragma unroll
  for (int k = 0; k < 8; ++k) buf[k * R5_S1 + L] = v[k];
  wave_lds_sync();
  const int la = L & 7, kk = L >> 3;                    // lane = (la, k): the 8 values l = la + 8 lb
#pragma unroll
  for (int lb = 0; lb < 8; ++lb) v[lb] = buf[kk * R5_S1 + la + 8 * lb];
  wave_lds_sync();
  dft<8, INV>(v);                                        // over lb -> m1
#pragma unroll
  for (int m = 1; m < 8; ++m) v[m] = cmul(v[m], tw_at<INV>(twl, 8 * la * m));
#pragma unroll
  for (int m = 0; m < 8; ++m) buf[(kk + 8 * m) * R5_S2 + la] = v[m];
  wave_lds_sync();
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = buf[L * R5_S2 + q];   // lane L = k + 8 m1: the 8 values over la
  wave_lds_sync();
  dft<8, INV>(v);                                        // over la -> m2: X[k + 8 m1 + 64 m2] = X[L + 64 m2]
}

// grid (n1, filters); block 64 * nw (waves split the filter's pairs). Same math as fft_row_kernel. (A next-pair
// prefetch measured neutral, profiles/r04_fft_ab.txt r4row.)
__global__ __launch_bounds__(256) void fft_row512_kernel(FftArgs a) {
  __shared__ f32x2 twl[512];
  __shared__ f32x2 wbuf[4][8 * R5_S1];
  const int L = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // filter spectra (mode 0): the workgroup's waves take nw consecutive rows k1; else one row k1, waves split pairs
  const int k1 = a.mode == 0 ? blockIdx.x * nw + w : blockIdx.x, j = a.pid0 + blockIdx.y;
  const float invn = 1.f / (float)a.n;
  load_twl(twl, a.tw, 512, a.n);
  __syncthreads();
  f32x2* buf = wbuf[w];
  const long long row = (long long)k1 * 512 + L;
  if (a.mode == 0) {   // filter spectrum: K_j[k1][:] = FFT_512(T[k1][:]) / n  (one wave per row)
    f32x2 v[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = a.SK[(long long)j * a.n + row + 64 * r];
    fft512_wave<false>(v, buf, twl, L);
    const float dn = a.Dv ? a.Dv[j] * invn : 0.f;   // + D / n: the spectrum of D delta (the D u term)
#pragma unroll
    for (int r = 0; r < 8; ++r) a.K[(long long)j * a.n + row + 64 * r] = v[r] * invn + f32x2{dn, 0.f};
    return;
  }
  f32x2 kr[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) kr[r] = a.K[(long long)j * a.n + row + 64 * r];
  const bool two = a.mode == 2 && a.SK;
  f32x2* so = a.So ? a.So : a.S;
  f32x2 acc[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) acc[r] = f32x2{0.f, 0.f};
  for (int p = w; p < a.P; p += nw) {
    const long long off = ((long long)j * a.P + p) * a.n + row;
    f32x2 v[8], v2[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      v[r] = a.S[off + 64 * r];
      if (two) v2[r] = a.S2[off + 64 * r];
    }
    fft512_wave<false>(v, buf, twl, L);
    if (two) {
      fft512_wave<false>(v2, buf, twl, L);
#pragma unroll
      for (int r = 0; r < 8; ++r) acc[r] += cmulc(v[r], v2[r]);   // X_dy conj(X_vg)
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = a.mode == 1 ? cmul(v[r], kr[r]) : cmulc(v[r], kr[r]);
    fft512_wave<true>(v, buf, twl, L);
#pragma unroll
    for (int r = 0; r < 8; ++r) so[off + 64 * r] = v[r];
  }
  if (!two) return;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 8; ++r) wbuf[w][L + 64 * r] = acc[r];
  __syncthreads();
  if (w != 0) return;
  f32x2 v[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    f32x2 t = wbuf[0][L + 64 * r];
    for (int q = 1; q < nw; ++q) t += wbuf[q][L + 64 * r];
    v[r] = t;
  }
  wave_lds_sync();
  fft512_wave<true>(v, buf, twl, L);                     // dk spectrum row (unnormalised correlation)
#pragma unroll
  for (int r = 0; r < 8; ++r) a.SK[(long long)j * a.n + row + 64 * r] = v[r] * invn;
}

// ---------------------------------------------------------------------------------- inverse columns
// grid: (n2 / G, npairs_total or C); out rows (+ D * src); single: dk[j][m] = Re(...) for the filter.
__global__ __launch_bounds__(256) void fft_col_inv_kernel(FftArgs a) {
  extern __shared__ __attribute__((aligned(16))) f32x2 lds[];
  const int ld = a.n1 + 1;   // padded column stride: the G columns' transposing accesses hit distinct banks
  f32x2* x = lds;
  f32x2* y = lds + a.G * ld;
  f32x2* twl = y + a.G * ld;
  load_twl(twl, a.tw, a.n1, a.n);
  const int c0 = blockIdx.x * a.G;
  const int pid = a.pid0 + blockIdx.y;
  const f32x2* S = (a.single ? a.SK : a.S) + (long long)pid * a.n;
  const int total = a.G * a.n1;
  for (int base = 0; base < total; base += UB * blockDim.x) {
    f32x2 v[UB], w[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = base + u * blockDim.x + threadIdx.x;
      const int g = idx % a.G, k1 = idx / a.G;
      if (idx < total) {
        w[u] = a.tw[((long long)(c0 + g) * k1) & (a.n - 1)];
        v[u] = S[(long long)k1 * a.n2 + c0 + g];
      }
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = base + u * blockDim.x + threadIdx.x;
      if (idx < total) x[(idx % a.G) * ld + idx / a.G] = cmulc(v[u], w[u]);
    }
  }
  __syncthreads();
  x = lds_fft<true>(x, y, a.n1, a.ln1, a.G, twl, ld);
  if (a.single) {
    for (int idx = threadIdx.x; idx < a.G * a.n1; idx += blockDim.x) {
      const int g = idx % a.G, ai = idx / a.G;
      const int m = ai * a.n2 + c0 + g;
      if (m < a.L) a.dk[(long long)pid * a.L + m] = x[g * ld + ai].x;
    }
    return;
  }
  const int j = pid / a.P, p = pid % a.P;
  const int r0 = pair_row(a, j, p, 0), r1 = pair_row(a, j, p, 1);
  const float Dj = a.Dv ? a.Dv[j] : 0.f;
  for (int base = 0; base < total; base += UB * blockDim.x) {
    float s0[UB], s1[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = base + u * blockDim.x + threadIdx.x;
      const int m = (idx / a.G) * a.n2 + c0 + idx % a.G;
      s0[u] = s1[u] = 0.f;
      if (idx < total && m < a.L) {
        s0[u] = a.src[(long long)r0 * a.L + m];
        if (r1 >= 0) s1[u] = a.src[(long long)r1 * a.L + m];
      }
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = base + u * blockDim.x + threadIdx.x;
      const int g = idx % a.G, ai = idx / a.G;
      const int m = ai * a.n2 + c0 + g;
      if (idx < total && m < a.L) {
        const f32x2 v = x[g * ld + ai];
        a.dst[(long long)r0 * a.L + m] = fmaf(Dj, s0[u], v.x);
        if (r1 >= 0) a.dst[(long long)r1 * a.L + m] = fmaf(Dj, s1[u], v.y);
      }
    }
  }
}

// --------------------------------------------------------------- column passes, wide column groups (v2)
// GW = 8192 / n1 adjacent columns per workgroup (32 at n1 = 256, 16 at n1 = 512): every global row segment is
// GW contiguous f32 (128 B / 64 B) and every spectrum segment GW complex (256 B / 128 B), where the v1 kernels'
// 8 columns gave 32-B / 64-B segments. The column FFTs run in place in ONE LDS buffer: each radix pass reads all
// of its butterflies into registers, barriers, then writes (Stockham order), so the buffer is half the v1 ping-pong.
constexpr int CW_ELEMS = 8192;   // GW * n1 complex per workgroup

template <int R, bool INV, int CW>
__device__ __forceinline__ void stockham_inplace(f32x2* x, int N, int Ns, const f32x2* twl, int ld) {
  constexpr int PER = CW / R / 256;   // butterflies per thread
  const int nb = N / R;
  const int tstep = N / (Ns * R);
  f32x2 v[PER][R];
  int pos[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int idx = k * 256 + threadIdx.x;
    const int sq = idx / nb, j = idx - sq * nb;
    const int m = j & (Ns - 1);
    const f32x2* xs = x + sq * ld;
#pragma unroll
    for (int r = 0; r < R; ++r) v[k][r] = xs[j + r * nb];
    if (Ns > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r) {
        f32x2 w = twl[(m * r * tstep) & (N - 1)];
        if (INV) w.y = -w.y;
        v[k][r] = cmul(v[k][r], w);
      }
    }
    dft<R, INV>(v[k]);
    pos[k] = sq * ld + (j - m) * R + m;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k)
#pragma unroll
    for (int r = 0; r < R; ++r) x[pos[k] + r * Ns] = v[k][r];
  __syncthreads();
}

template <bool INV, int CW>
__device__ __forceinline__ void lds_fft_inplace(f32x2* x, int N, int lN, const f32x2* twl, int ld) {
  int Ns = 1, left = lN;
  while (left > 0) {
    if (left >= 3 && left != 4) { stockham_inplace<8, INV, CW>(x, N, Ns, twl, ld); Ns *= 8; left -= 3; }
    else if (left >= 2) { stockham_inplace<4, INV, CW>(x, N, Ns, twl, ld); Ns *= 4; left -= 2; }
    else { stockham_inplace<2, INV, CW>(x, N, Ns, twl, ld); Ns *= 2; left -= 1; }
  }
}

// Inter-pass twiddles W_n^e, e < n = 2^ln, as the product of three LDS tables (W_n^e0, W_n^(e1 2^l0),
// W_n^(e2 2^(l0+l1)), copied from the f64-built table): two complex multiplies and three LDS reads instead of one
// random 8-byte gather from the n-entry global table per element (a cache line per lane).
struct Tw3 {
  const f32x2* t;   // [2^l0 | 2^l1 | 2^l2]
  int l0, l1;
};
__host__ __device__ constexpr int tw3_entries(int ln) {
  return (1 << ((ln + 2) / 3)) + (1 << ((ln + 1) / 3)) + (1 << (ln / 3));
}
__device__ __forceinline__ Tw3 load_tw3(f32x2* t, const f32x2* tw, int ln) {
  const int l0 = (ln + 2) / 3, l1 = (ln + 1) / 3, l2 = ln / 3;
  const int n0 = 1 << l0, n1 = 1 << l1, n2 = 1 << l2;
  for (int i = threadIdx.x; i < n0 + n1 + n2; i += blockDim.x) {
    long long e;
    if (i < n0) e = i;
    else if (i < n0 + n1) e = (long long)(i - n0) << l0;
    else e = (long long)(i - n0 - n1) << (l0 + l1);
    t[i] = tw[e];
  }
  return Tw3{t, l0, l1};
}
__device__ __forceinline__ f32x2 tw3(const Tw3& w, long long e) {
  const int e0 = (int)(e & ((1 << w.l0) - 1)), e1 = (int)((e >> w.l0) & ((1 << w.l1) - 1));
  const int e2 = (int)(e >> (w.l0 + w.l1));
  return cmul(cmul(w.t[e0], w.t[(1 << w.l0) + e1]), w.t[(1 << w.l0) + (1 << w.l1) + e2]);
}

// ------------------------------------------------ column FFTs of n1 = 1024 in registers, one column per wave at a time:
// lane L holds x[L + 64 r], r < 16; a 16-point DFT over r (4 x 4 in registers), twiddle
// W_1024^(L k), then for each half k = 8h + k' of the 16 frequencies the 64-point DFT over the lanes as 8 x 8 with two
// wave-local LDS transposes (the second and third stages of fft512_wave) -- X[k + 16 m], m = m1 + 8 m2, lands in
// lane k' + 8 m1. The column's own LDS region (its values are in registers by then) is the transpose buffer, so the
// only workgroup barriers are the ones around the load and store loops (the in-place Stockham passes take two per
// radix pass, 8 at n1 = 1024).
template <bool INV>
__device__ __forceinline__ f32x2 w16(int t) {   // W_16^t (forward e^{-2 pi i t / 16}), t < 16
  constexpr float C1 = 0.92387953251128674f, S1 = 0.38268343236508977f, H = 0.70710678118654752f;
  const float c[16] = {1.f, C1, H, S1, 0.f, -S1, -H, -C1, -1.f, -C1, -H, -S1, 0.f, S1, H, C1};
  const float sn[16] = {0.f, S1, H, C1, 1.f, C1, H, S1, 0.f, -S1, -H, -C1, -1.f, -C1, -H, -S1};
  return f32x2{c[t], INV ? sn[t] : -sn[t]};
}
template <bool INV>
__device__ __forceinline__ void dft16(f32x2 (&v)[16]) {   // v[c + 4 d] = sum_r v[r] W_16^(r (c + 4 d)), r = 4 a + b
  f32x2 t[4][4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    f32x2 q[4] = {v[b], v[4 + b], v[8 + b], v[12 + b]};
    dft<4, INV>(q);
#pragma unroll
    for (int c = 0; c < 4; ++c) t[b][c] = (b * c == 0) ? q[c] : cmul(q[c], w16<INV>(b * c));
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    f32x2 q[4] = {t[0][c], t[1][c], t[2][c], t[3][c]};
    dft<4, INV>(q);
#pragma unroll
    for (int d = 0; d < 4; ++d) v[c + 4 * d] = q[d];
  }
}
// 64-point DFTs over the lanes of 8 sequences: in, lane L holds v[k] = Y[k][L]; out, lane k + 8 m1 holds
// v[m2] = sum_l Y[k][l] W_64^(l (m1 + 8 m2)). twl: W_N^t (N = 64 TS entries). buf: 8 * R5_S1 complex.
template <bool INV, int TS>
__device__ __forceinline__ void dft64_lanes(f32x2 (&v)[8], f32x2* buf, const f32x2* twl, int L) {
#pragma unroll
  for (int k = 0; k < 8; ++k) buf[k * R5_S1 + L] = v[k];
  wave_lds_sync();
  const int la = L & 7, kk = L >> 3;
#pragma unroll
  for (int lb = 0; lb < 8; ++lb) v[lb] = buf[kk * R5_S1 + la + 8 * lb];
  wave_lds_sync();
  dft<8, INV>(v);
#pragma unroll
  for (int m = 1; m < 8; ++m) {
    f32x2 w = twl[(TS * la * m) & (64 * TS - 1)];
    if (INV) w.y = -w.y;
    v[m] = cmul(v[m], w);
  }
#pragma unroll
  for (int m = 0; m < 8; ++m) buf[(kk + 8 * m) * R5_S2 + la] = v[m];
  wave_lds_sync();
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = buf[L * R5_S2 + q];
  wave_lds_sync();
  dft<8, INV>(v);
}
// the columns g = wave, wave + 4, ... of x (ld apart), in place; twl: W_1024^t
template <bool INV, int GW, int NW>
__device__ __forceinline__ void col_fft1024_waves(f32x2* x, int ld, const f32x2* twl) {
  const int L = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int g = wave; g < GW; g += NW) {
    f32x2* col = x + g * ld;
    f32x2 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = col[L + 64 * r];
    wave_lds_sync();   // every lane's reads of the column are done before it becomes the transpose buffer
    dft16<INV>(v);
#pragma unroll
    for (int k = 1; k < 16; ++k) {
      f32x2 w = twl[(L * k) & 1023];
      if (INV) w.y = -w.y;
      v[k] = cmul(v[k], w);
    }
    f32x2 lo[8], hi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { lo[k] = v[k]; hi[k] = v[8 + k]; }
    dft64_lanes<INV, 16>(lo, col, twl, L);
    dft64_lanes<INV, 16>(hi, col, twl, L);
    const int base = (L & 7) + 16 * (L >> 3);   // X[8h + k' + 16 m1 + 128 m2]
#pragma unroll
    for (int m2 = 0; m2 < 8; ++m2) {
      col[base + 128 * m2] = lo[m2];
      col[base + 8 + 128 * m2] = hi[m2];
    }
    wave_lds_sync();
  }
}

// n1 = 512: fft512_wave per column; n1 = 256: two columns per call (4 points each: a 4-point DFT over r, twiddle
// W_256^(L k), and the 8 sequences (column, k) through one dft64_lanes). Both use a per-wave scratch of
// 8 R5_S1 complex after the twiddle tables (the column regions are too short for the transpose strides).
template <bool INV, int GW, int N1, int NW>
__device__ __forceinline__ void col_fft_small_waves(f32x2* x, int ld, const f32x2* twl, f32x2* scr) {
  const int L = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x2* buf = scr + wave * 8 * R5_S1;
  if constexpr (N1 == 512) {
    for (int g = wave; g < GW; g += NW) {
      f32x2* col = x + g * ld;
      f32x2 v[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = col[L + 64 * r];
      fft512_wave<INV>(v, buf, twl, L);
#pragma unroll
      for (int m = 0; m < 8; ++m) col[L + 64 * m] = v[m];
    }
  } else {
    static_assert(N1 == 256 && GW % (2 * NW) == 0, "two columns per wave and call");
    for (int g = wave; g < GW; g += 2 * NW) {   // columns g and g + NW
      f32x2* c0 = x + g * ld;
      f32x2* c1 = x + (g + NW) * ld;
      f32x2 p[4], q[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) { p[r] = c0[L + 64 * r]; q[r] = c1[L + 64 * r]; }
      dft<4, INV>(p);
      dft<4, INV>(q);
      f32x2 w[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f32x2 t = twl[(L * k) & 255];
        if (INV) t.y = -t.y;
        w[k] = k ? cmul(p[k], t) : p[k];
        w[4 + k] = k ? cmul(q[k], t) : q[k];
      }
      dft64_lanes<INV, 4>(w, buf, twl, L);
      // lane k'' + 8 m1 holds X[k + 4 (m1 + 8 m2)] of column k'' < 4 ? g : g + NW, k = k'' & 3
      f32x2* col = (L & 7) < 4 ? c0 : c1;
      const int base = (L & 3) + 4 * (L >> 3);
#pragma unroll
      for (int m2 = 0; m2 < 8; ++m2) col[base + 32 * m2] = w[m2];
    }
  }
}
__host__ __device__ constexpr bool col_wave_scratch(int n1, int gw) {
  return n1 == 512 || (n1 == 256 && gw % 8 == 0);
}
__host__ __device__ constexpr bool col_wave_path(int n1, int gw) { return n1 == 1024 || col_wave_scratch(n1, gw); }
template <bool INV, int GW, int CW, int NT>
__device__ __forceinline__ void col_fft_waves(f32x2* x, int ld, const f32x2* twl, f32x2* scr) {
  constexpr int N1 = CW / GW;
  if constexpr (N1 == 1024) {
    col_fft1024_waves<INV, GW, NT / 64>(x, ld, twl);
  } else {
    col_fft_small_waves<INV, GW, N1, NT / 64>(x, ld, twl, scr);
  }
}

// grid (n2 / GW / GP, npairs_total or C); block NT. Same math as fft_col_fwd_kernel. GP > 1 (wave FFT path, 16-B
// rows): the workgroup takes GP consecutive column groups and loads group i+1's rows into registers while group i's
// FFT and stores run (the load, FFT and store phases otherwise serialise: one 141-KB workgroup per CU at n1 = 1024).
template <int GW, int CW, int NT, int GP = 1>
__global__ __launch_bounds__(NT) void fft_colw_fwd_kernel(FftArgs a) {
  extern __shared__ __attribute__((aligned(16))) f32x2 lds[];
  const int ld = a.n1 + 1;
  f32x2* x = lds;
  f32x2* twl = x + GW * ld;
  load_twl(twl, a.tw, a.n1, a.n);
  const Tw3 tw3t = load_tw3(twl + a.n1, a.tw, a.ln1 + a.ln2);
  const int c0 = blockIdx.x * GW;
  const int pid = a.pid0 + blockIdx.y;
  int r0, r1;
  if (a.single) { r0 = pid; r1 = -1; }
  else {
    const int j = pid / a.P, p = pid % a.P;
    r0 = pair_row(a, j, p, 0);
    r1 = pair_row(a, j, p, 1);
  }
  const float* s0 = a.src + (long long)r0 * a.L;
  const float* s1 = r1 >= 0 ? a.src + (long long)r1 * a.L : nullptr;
  if constexpr (GP > 1) {
    static_assert(col_wave_path(CW / GW, GW) && (CW / 4) % NT == 0, "prefetching column groups: wave FFT path");
    constexpr int PERT = CW / 4 / NT;   // 16-B chunks per thread and group
    f32x4 v0[PERT], v1[PERT];
    auto gload = [&](int cg) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < PERT; ++u) {
        const int idx = u * NT + threadIdx.x;
        const int m = (idx / (GW / 4)) * a.n2 + cg + (idx % (GW / 4)) * 4;
        v0[u] = v1[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (m < a.L) {
          v0[u] = *(const f32x4*)(s0 + m);
          if (s1) v1[u] = *(const f32x4*)(s1 + m);
        }
      }
    };
    f32x2* S = (a.single ? a.SK : a.S) + (long long)pid * a.n;
    gload(blockIdx.x * GP * GW);
    for (int it = 0; it < GP; ++it) {
      const int cg = (blockIdx.x * GP + it) * GW;
#pragma unroll
      for (int u = 0; u < PERT; ++u) {
        const int idx = u * NT + threadIdx.x;
        const int g = (idx % (GW / 4)) * 4, ai = idx / (GW / 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) x[(g + q) * ld + ai] = f32x2{v0[u][q], v1[u][q]};
      }
      if (it + 1 < GP) gload(cg + GW);   // in flight during this group's FFT and stores
      __syncthreads();
      col_fft_waves<false, GW, CW, NT>(x, ld, twl, twl + a.n1 + tw3_entries(a.ln1 + a.ln2));
      __syncthreads();
      for (int idx = threadIdx.x; idx < CW / 2; idx += NT) {
        const int g = (idx % (GW / 2)) * 2, k1 = idx / (GW / 2);
        const long long e = (long long)(cg + g) * k1;
        const f32x2 p0 = cmul(x[g * ld + k1], tw3(tw3t, e & (a.n - 1)));
        const f32x2 p1 = cmul(x[(g + 1) * ld + k1], tw3(tw3t, (e + k1) & (a.n - 1)));
        *(f32x4*)(S + (long long)k1 * a.n2 + cg + g) = f32x4{p0.x, p0.y, p1.x, p1.y};
      }
      if (it + 1 < GP) __syncthreads();   // the store loop's LDS reads precede the next group's writes
    }
    return;
  }
  if ((a.L & 3) == 0) {   // 16-byte loads of 4 adjacent columns (rows are 16-B aligned, chunks all in or out)
    constexpr int NQ = CW / 4;
    for (int base = 0; base < NQ; base += UB * NT) {
      f32x4 v0[UB], v1[UB];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int idx = base + u * NT + threadIdx.x;
        const int g = (idx % (GW / 4)) * 4, ai = idx / (GW / 4);
        const int m = ai * a.n2 + c0 + g;
        v0[u] = v1[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (idx < NQ && m < a.L) {
          v0[u] = *(const f32x4*)(s0 + m);
          if (s1) v1[u] = *(const f32x4*)(s1 + m);
        }
      }
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int idx = base + u * NT + threadIdx.x;
        const int g = (idx % (GW / 4)) * 4, ai = idx / (GW / 4);
        if (idx < NQ) {
#pragma unroll
          for (int q = 0; q < 4; ++q) x[(g + q) * ld + ai] = f32x2{v0[u][q], v1[u][q]};
        }
      }
    }
  } else {
    for (int base = 0; base < CW; base += UB * NT) {
      f32x2 v[UB];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int idx = base + u * NT + threadIdx.x;
        const int g = idx % GW, ai = idx / GW;
        const int m = ai * a.n2 + c0 + g;
        v[u] = f32x2{0.f, 0.f};
        if (m < a.L) {
          v[u].x = s0[m];
          if (s1) v[u].y = s1[m];
        }
      }
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int idx = base + u * NT + threadIdx.x;
        x[(idx % GW) * ld + idx / GW] = v[u];
      }
    }
  }
  __syncthreads();
  if constexpr (col_wave_path(CW / GW, GW)) {
    col_fft_waves<false, GW, CW, NT>(x, ld, twl, twl + a.n1 + tw3_entries(a.ln1 + a.ln2));
    __syncthreads();
  } else {
    static_assert(NT == 256, "the LDS Stockham passes assume 256 threads");
    lds_fft_inplace<false, CW>(x, a.n1, a.ln1, twl, ld);
  }
  f32x2* S = (a.single ? a.SK : a.S) + (long long)pid * a.n;
  for (int idx = threadIdx.x; idx < CW / 2; idx += NT) {   // 16-byte stores of 2 adjacent columns
    const int g = (idx % (GW / 2)) * 2, k1 = idx / (GW / 2);
    const long long e = (long long)(c0 + g) * k1;
    const f32x2 p0 = cmul(x[g * ld + k1], tw3(tw3t, e & (a.n - 1)));
    const f32x2 p1 = cmul(x[(g + 1) * ld + k1], tw3(tw3t, (e + k1) & (a.n - 1)));
    *(f32x4*)(S + (long long)k1 * a.n2 + c0 + g) = f32x4{p0.x, p0.y, p1.x, p1.y};
  }
}

// grid (n2 / GW / GP, npairs_total or C); same math as fft_col_inv_kernel. GP > 1: as fft_colw_fwd_kernel, the next
// column group's spectrum rows are loaded into registers during this group's FFT and output pass.
template <int GW, int CW, int NT, int GP = 1>
__global__ __launch_bounds__(NT) void fft_colw_inv_kernel(FftArgs a) {
  extern __shared__ __attribute__((aligned(16))) f32x2 lds[];
  const int ld = a.n1 + 1;
  f32x2* x = lds;
  f32x2* twl = x + GW * ld;
  load_twl(twl, a.tw, a.n1, a.n);
  const Tw3 tw3t = load_tw3(twl + a.n1, a.tw, a.ln1 + a.ln2);
  const int pid = a.pid0 + blockIdx.y;
  const f32x2* S = (a.single ? a.SK : a.S) + (long long)pid * a.n;
  __syncthreads();   // the twiddle tables are read below
  constexpr int NH = CW / 2;   // 16-byte loads of 2 adjacent columns
  // output of column group c0 (after its inverse column FFTs): rows (+ D * src) or the filter gradient
  // (with a prefetched group in registers, the output pass keeps fewer of its own loads in flight: no spills)
  constexpr int UBE = GP > 1 ? 2 : UB;
  auto emit = [&](int c0) __attribute__((always_inline)) {
    // only a < ceil(L / n2) rows of the column carry outputs (m < L); the rest is the discarded wrap half
    const int na = (a.L - c0 + a.n2 - 1) / a.n2;
    if (a.single) {
      for (int idx = threadIdx.x; idx < GW * na; idx += NT) {
        const int g = idx % GW, ai = idx / GW;
        const int m = ai * a.n2 + c0 + g;
        if (m < a.L) a.dk[(long long)pid * a.L + m] = x[g * ld + ai].x;
      }
      return;
    }
    const int j = pid / a.P, p = pid % a.P;
    const int r0 = pair_row(a, j, p, 0), r1 = pair_row(a, j, p, 1);
    const float Dj = a.Dv ? a.Dv[j] : 0.f;
    const float* s0 = a.src + (long long)r0 * a.L;
    const float* s1 = r1 >= 0 ? a.src + (long long)r1 * a.L : nullptr;
    float* d0 = a.dst + (long long)r0 * a.L;
    float* d1 = r1 >= 0 ? a.dst + (long long)r1 * a.L : nullptr;
    if ((a.L & 3) == 0) {   // 16-byte loads / stores of 4 adjacent columns
      const int totq = (GW / 4) * na;
      for (int base = 0; base < totq; base += UBE * NT) {
        f32x4 u0[UBE], u1[UBE];
  #pragma unroll
        for (int u = 0; u < UBE; ++u) {
          const int idx = base + u * NT + threadIdx.x;
          const int m = (idx / (GW / 4)) * a.n2 + c0 + (idx % (GW / 4)) * 4;
          u0[u] = u1[u] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (idx < totq && m < a.L && a.Dv) {
            u0[u] = *(const f32x4*)(s0 + m);
            if (s1) u1[u] = *(const f32x4*)(s1 + m);
          }
        }
  #pragma unroll
        for (int u = 0; u < UBE; ++u) {
          const int idx = base + u * NT + threadIdx.x;
          const int g = (idx % (GW / 4)) * 4, ai = idx / (GW / 4);
          const int m = ai * a.n2 + c0 + g;
          if (idx < totq && m < a.L) {
            f32x4 o0, o1;
  #pragma unroll
            for (int q = 0; q < 4; ++q) {
              const f32x2 v = x[(g + q) * ld + ai];
              o0[q] = fmaf(Dj, u0[u][q], v.x);
              o1[q] = fmaf(Dj, u1[u][q], v.y);
            }
            *(f32x4*)(d0 + m) = o0;
            if (d1) *(f32x4*)(d1 + m) = o1;
          }
        }
      }
      return;
    }
    const int total = GW * na;
    for (int base = 0; base < total; base += UBE * NT) {
      float u0[UBE], u1[UBE];
  #pragma unroll
      for (int u = 0; u < UBE; ++u) {
        const int idx = base + u * NT + threadIdx.x;
        const int m = (idx / GW) * a.n2 + c0 + idx % GW;
        u0[u] = u1[u] = 0.f;
        if (idx < total && m < a.L) {
          u0[u] = s0[m];
          if (s1) u1[u] = s1[m];
        }
      }
  #pragma unroll
      for (int u = 0; u < UBE; ++u) {
        const int idx = base + u * NT + threadIdx.x;
        const int g = idx % GW, ai = idx / GW;
        const int m = ai * a.n2 + c0 + g;
        if (idx < total && m < a.L) {
          const f32x2 v = x[g * ld + ai];
          d0[m] = fmaf(Dj, u0[u], v.x);
          if (d1) d1[m] = fmaf(Dj, u1[u], v.y);
        }
      }
    }
  };
  if constexpr (GP > 1) {
    static_assert(col_wave_path(CW / GW, GW) && NH % NT == 0, "prefetching column groups: wave FFT path");
    constexpr int PERT = NH / NT;
    f32x4 v[PERT];
    auto sload = [&](int cg) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < PERT; ++u) {
        const int idx = u * NT + threadIdx.x;
        v[u] = *(const f32x4*)(S + (long long)(idx / (GW / 2)) * a.n2 + cg + (idx % (GW / 2)) * 2);
      }
    };
    sload(blockIdx.x * GP * GW);
    for (int it = 0; it < GP; ++it) {
      const int cg = (blockIdx.x * GP + it) * GW;
#pragma unroll
      for (int u = 0; u < PERT; ++u) {
        const int idx = u * NT + threadIdx.x;
        const int g = (idx % (GW / 2)) * 2, k1 = idx / (GW / 2);
        const long long e = (long long)(cg + g) * k1;
        x[g * ld + k1] = cmulc(f32x2{v[u][0], v[u][1]}, tw3(tw3t, e & (a.n - 1)));
        x[(g + 1) * ld + k1] = cmulc(f32x2{v[u][2], v[u][3]}, tw3(tw3t, (e + k1) & (a.n - 1)));
      }
      if (it + 1 < GP) sload(cg + GW);   // in flight during this group's FFT and output pass
      __syncthreads();
      col_fft_waves<true, GW, CW, NT>(x, ld, twl, twl + a.n1 + tw3_entries(a.ln1 + a.ln2));
      __syncthreads();
      emit(cg);
      if (it + 1 < GP) __syncthreads();
    }
    return;
  }
  const int c0 = blockIdx.x * GW;
  for (int base = 0; base < NH; base += UB * NT) {
    f32x4 v[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = base + u * NT + threadIdx.x;
      const int g = (idx % (GW / 2)) * 2, k1 = idx / (GW / 2);
      if (idx < NH) v[u] = *(const f32x4*)(S + (long long)k1 * a.n2 + c0 + g);
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int idx = base + u * NT + threadIdx.x;
      const int g = (idx % (GW / 2)) * 2, k1 = idx / (GW / 2);
      if (idx < NH) {
        const long long e = (long long)(c0 + g) * k1;
        x[g * ld + k1] = cmulc(f32x2{v[u][0], v[u][1]}, tw3(tw3t, e & (a.n - 1)));
        x[(g + 1) * ld + k1] = cmulc(f32x2{v[u][2], v[u][3]}, tw3(tw3t, (e + k1) & (a.n - 1)));
      }
    }
  }
  __syncthreads();
  if constexpr (col_wave_path(CW / GW, GW)) {
    col_fft_waves<true, GW, CW, NT>(x, ld, twl, twl + a.n1 + tw3_entries(a.ln1 + a.ln2));
    __syncthreads();
  } else {
    static_assert(NT == 256, "the LDS Stockham passes assume 256 threads");
    lds_fft_inplace<true, CW>(x, a.n1, a.ln1, twl, ld);
  }
  emit(c0);
}

// dD[j] += dk[j][0]: sum_rows sum_t dy u is the lag-0 entry of the filter gradient sum_rows corr(dy, u)
__global__ __launch_bounds__(256) void dd_from_dk_kernel(const float* dk, float* dD, int C, int L) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < C) dD[j] += dk[(long long)j * L];
}

// dD[j] += sum_rows sum_t a[row][t] * b[row][t] over rows of filter j (block partial + one atomic per block).
// grid (rows, splits): a block takes a contiguous span of its row; 16-byte loads when the rows allow them.
constexpr int RD_SPAN = 16384;   // elements per block
__global__ __launch_bounds__(256) void row_dot_kernel(const float* x, const float* y, float* out, int L, int C,
                                                      int vec) {
  __shared__ float red[4];
  const int row = blockIdx.x;   // r_outer * C + j
  const int j = row % C;
  const long long base = (long long)row * L;
  const int t0 = blockIdx.y * RD_SPAN, t1 = min(L, t0 + RD_SPAN);
  float acc = 0.f;
  if (vec) {   // L % 4 == 0 and 16-byte aligned rows
    const f32x4* xv = (const f32x4*)(x + base);
    const f32x4* yv = (const f32x4*)(y + base);
    int i = t0 / 4 + threadIdx.x;
    for (; i + 768 < t1 / 4; i += 1024) {
      const f32x4 a0 = xv[i], a1 = xv[i + 256], a2 = xv[i + 512], a3 = xv[i + 768];
      const f32x4 b0 = yv[i], b1 = yv[i + 256], b2 = yv[i + 512], b3 = yv[i + 768];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc += (a0[q] * b0[q] + a1[q] * b1[q]) + (a2[q] * b2[q] + a3[q] * b3[q]);
    }
    for (; i < t1 / 4; i += 256) {
      const f32x4 a0 = xv[i], b0 = yv[i];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = fmaf(a0[q], b0[q], acc);
    }
  } else {
    for (int t = t0 + threadIdx.x; t < t1; t += 256) acc = fmaf(x[base + t], y[base + t], acc);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out + j, (red[0] + red[1]) + (red[2] + red[3]));
}

__global__ void twiddle_kernel(f32x2* tw, int n) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  double s, c;
  sincospi(-2.0 * (double)t / (double)n, &s, &c);
  tw[t] = f32x2{(float)c, (float)s};
}

// ------------------------------------------------------------------------------- short conv + gating
// z (BB, L, 3D) channels-last; weight (3D, K) f32; bias (3D). For output channel ch = h*hd + jj of D:
// x1 = conv[h*3hd + jj], x2 = conv[h*3hd + hd + jj], v = conv[h*3hd + 2hd + jj] (hyena.py:321-330).
// Causal: conv_c(t) = bias[c] + sum_i w[c][i] z[t + i - (K-1)][c].
struct GateArgs {
  const void* z; const float* w; const float* bias;
  float* vg;            // (BB, D, L) f32 channel-major: v * x1
  void* x2;             // (BB, L, D) channels-last (z dtype)
  const float* y;       // (BB, D, L) f32 long-conv output (post)
  void* out;            // (BB, L, D) channels-last (z dtype) = y * x2 (post)
  const void* dout;     // post bwd: (BB, L, D)
  float* dy;            // post bwd: (BB, D, L) f32 = dout * x2
  void* dx2;            // post bwd: (BB, L, D) z dtype = dout * y (the dtype of x2, so no cast follows)
  const float* dvg;     // pre bwd: (BB, D, L)
  const void* gx2;      // pre bwd: dL/dx2 (BB, L, D) (z dtype)
  void* dz;             // pre bwd: (BB, L, 3D)
  float* dw; float* db; // pre bwd: (3D, K), (3D) accumulated
  int BB, L, D, H, hd, K;
};

// out[bb, t, ch] = y[bb, ch, t] * x2[bb, t, ch]
template <typename T>
__global__ __launch_bounds__(256) void hyena_post_fwd_kernel(GateArgs a) {
  __shared__ float tile[64][65];
  const int t0 = blockIdx.x * 64, ch0 = blockIdx.y * 64, bb = blockIdx.z;
  for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
    const int tl = idx & 63, cl = idx >> 6;
    const int t = t0 + tl, ch = ch0 + cl;
    tile[cl][tl] = (t < a.L && ch < a.D) ? a.y[((long long)bb * a.D + ch) * a.L + t] : 0.f;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
    const int cl = idx & 63, tl = idx >> 6;
    const int t = t0 + tl, ch = ch0 + cl;
    if (t < a.L && ch < a.D) {
      const long long o = ((long long)bb * a.L + t) * a.D + ch;
      ((T*)a.out)[o] = (T)(tile[cl][tl] * (float)((const T*)a.x2)[o]);
    }
  }
}

// dy[bb, ch, t] = dout * x2 ; dx2[bb, t, ch] = dout * y
template <typename T>
__global__ __launch_bounds__(256) void hyena_post_bwd_kernel(GateArgs a) {
  __shared__ float ty[64][65];
  __shared__ float tg[64][65];
  const int t0 = blockIdx.x * 64, ch0 = blockIdx.y * 64, bb = blockIdx.z;
  for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
    const int tl = idx & 63, cl = idx >> 6;
    const int t = t0 + tl, ch = ch0 + cl;
    ty[cl][tl] = (t < a.L && ch < a.D) ? a.y[((long long)bb * a.D + ch) * a.L + t] : 0.f;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
    const int cl = idx & 63, tl = idx >> 6;
    const int t = t0 + tl, ch = ch0 + cl;
    float g = 0.f;
    if (t < a.L && ch < a.D) {
      const long long o = ((long long)bb * a.L + t) * a.D + ch;
      const float go = (float)((const T*)a.dout)[o];
      g = go * (float)((const T*)a.x2)[o];
      ((T*)a.dx2)[o] = (T)(go * ty[cl][tl]);
    }
    tg[cl][tl] = g;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
    const int tl = idx & 63, cl = idx >> 6;
    const int t = t0 + tl, ch = ch0 + cl;
    if (t < a.L && ch < a.D) a.dy[((long long)bb * a.D + ch) * a.L + t] = tg[cl][tl];
  }
}

// ------------------------------------------------------------- short conv + gating, register-ring kernels
// One lane = one output channel ch of D (64 per workgroup), waves split the tokens: each wave runs HY_TW
// consecutive tokens with the causal short-conv taps of its three gate channels (x1, x2, v = conv channels base,
// base + hd, base + 2 hd, hyena.py:321-330) in register rings, so every z element is loaded once per wave
// (+ K - 1 halo tokens), 8 tokens' loads in flight; the channel-major f32 rows (vg / dvg, what the FFT passes
// read) go through an LDS tile so both sides of the transpose are coalesced.
constexpr int HY_TT = 128;   // tokens per workgroup tile
constexpr int HY_TW = 32;    // tokens per wave
constexpr int HY_PF = 8;     // tokens whose loads are issued together

template <typename T>
__device__ __forceinline__ float zld(const T* zb, long long t, int L, int D3, int c) {
  return (t >= 0 && t < L) ? (float)zb[t * D3 + c] : 0.f;
}

template <typename T, int KC>
__global__ __launch_bounds__(256) void hyena_pre_fwd2_kernel(GateArgs a) {
  __shared__ float vgt[64][HY_TT + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t0 = blockIdx.x * HY_TT, ch0 = blockIdx.y * 64, bb = blockIdx.z;
  const int ch = ch0 + lane, L = a.L, D3 = 3 * a.D;
  const bool valid = ch < a.D;
  const int chc = valid ? ch : a.D - 1;
  const int h = chc / a.hd, jj = chc - h * a.hd;
  const int c1 = h * 3 * a.hd + jj, c2 = c1 + a.hd, c3 = c1 + 2 * a.hd;
  const T* zb = (const T*)a.z + (long long)bb * L * D3;
  float w1[KC], w2[KC], w3[KC];
#pragma unroll
  for (int i = 0; i < KC; ++i) { w1[i] = a.w[c1 * KC + i]; w2[i] = a.w[c2 * KC + i]; w3[i] = a.w[c3 * KC + i]; }
  const float b1 = a.bias ? a.bias[c1] : 0.f, b2 = a.bias ? a.bias[c2] : 0.f, b3 = a.bias ? a.bias[c3] : 0.f;
  const int ts = t0 + wave * HY_TW, te = min(L, ts + HY_TW);
  float r1[KC], r2[KC], r3[KC];   // z[t - KC + 1 .. t] of the three channels
#pragma unroll
  for (int i = 1; i < KC; ++i) {
    r1[i] = zld(zb, ts - KC + i, L, D3, c1);
    r2[i] = zld(zb, ts - KC + i, L, D3, c2);
    r3[i] = zld(zb, ts - KC + i, L, D3, c3);
  }
  T* x2p = (T*)a.x2 + (long long)bb * L * a.D + ch;
#pragma unroll
  for (int g = 0; g < HY_TW; g += HY_PF) {
    float n1[HY_PF], n2[HY_PF], n3[HY_PF];
#pragma unroll
    for (int u = 0; u < HY_PF; ++u) {
      const long long t = ts + g + u;
      n1[u] = zld(zb, t, L, D3, c1);
      n2[u] = zld(zb, t, L, D3, c2);
      n3[u] = zld(zb, t, L, D3, c3);
    }
#pragma unroll
    for (int u = 0; u < HY_PF; ++u) {
      const int t = ts + g + u;
#pragma unroll
      for (int i = 0; i < KC - 1; ++i) { r1[i] = r1[i + 1]; r2[i] = r2[i + 1]; r3[i] = r3[i + 1]; }
      r1[KC - 1] = n1[u]; r2[KC - 1] = n2[u]; r3[KC - 1] = n3[u];
      float x1 = b1, x2 = b2, v = b3;
#pragma unroll
      for (int i = 0; i < KC; ++i) { x1 = fmaf(w1[i], r1[i], x1); x2 = fmaf(w2[i], r2[i], x2); v = fmaf(w3[i], r3[i], v); }
      if (t < te) {
        if (valid) x2p[(long long)t * a.D] = (T)x2;
        vgt[lane][t - t0] = v * x1;
      }
    }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 64 * HY_TT; idx += 256) {
    const int row = idx / HY_TT, col = idx - row * HY_TT;
    const int t = t0 + col, c = ch0 + row;
    if (c < a.D && t < L) a.vg[((long long)bb * a.D + c) * L + t] = vgt[row][col];
  }
}

// dconv_x1 = dvg * v, dconv_v = dvg * x1, dconv_x2 = gx2; dz[s][c] = sum_i w[c][i] dconv_c[s + K - 1 - i];
// dw[c][i] += sum_s dconv_c[s] z[s + i - (K - 1)][c]; db[c] += sum_s dconv_c[s]. Workgroups stride over token
// tiles (so the dw/db partials are reduced over the waves and tiles in registers / LDS first and each workgroup
// adds them once: a few hundred float atomics per address instead of one per 64-token run).
template <typename T, int KC>
__global__ __launch_bounds__(256) void hyena_pre_bwd2_kernel(GateArgs a) {
  constexpr int W = HY_TT + KC - 1;            // dvg tile width: the tile's tokens + the K - 1 lookahead
  constexpr int NR = 2 * KC - 1;               // z ring: taps of the conv at tn and of dw at s = tn - K + 1
  constexpr int NIT = HY_TW + KC - 1;          // iterations per wave run (tn = s0 .. s1 + K - 2)
  constexpr int NA = 3 * (KC + 1);             // dw (3 x K) + db (3) per channel
  __shared__ float dvt[64][W | 1];
  __shared__ float red[4][NA][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ch0 = blockIdx.y * 64, bb = blockIdx.z;
  const int ch = ch0 + lane, L = a.L, D3 = 3 * a.D;
  const bool valid = ch < a.D;
  const int chc = valid ? ch : a.D - 1;
  const int h = chc / a.hd, jj = chc - h * a.hd;
  const int c1 = h * 3 * a.hd + jj, c2 = c1 + a.hd, c3 = c1 + 2 * a.hd;
  const T* zb = (const T*)a.z + (long long)bb * L * D3;
  const T* gx2 = (const T*)a.gx2 + (long long)bb * L * a.D + chc;
  T* dzb = (T*)a.dz + (long long)bb * L * D3;
  float w1[KC], w2[KC], w3[KC];
#pragma unroll
  for (int i = 0; i < KC; ++i) { w1[i] = a.w[c1 * KC + i]; w2[i] = a.w[c2 * KC + i]; w3[i] = a.w[c3 * KC + i]; }
  const float b1 = a.bias ? a.bias[c1] : 0.f, b3 = a.bias ? a.bias[c3] : 0.f;
  float acc[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) acc[i] = 0.f;
  const int ntiles = (L + HY_TT - 1) / HY_TT;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int t0 = tile * HY_TT;
    for (int idx = threadIdx.x; idx < 64 * W; idx += 256) {
      const int row = idx / W, col = idx - row * W;
      const int t = t0 + col, c = ch0 + row;
      dvt[row][col] = (c < a.D && t < L) ? a.dvg[((long long)bb * a.D + c) * L + t] : 0.f;
    }
    __syncthreads();
    const int s0 = t0 + wave * HY_TW, s1 = min(L, s0 + HY_TW);
    float z1[NR], z2[NR], z3[NR], d1[KC], d2[KC], d3[KC];
#pragma unroll
    for (int j = 1; j < NR; ++j) {
      z1[j] = zld(zb, s0 - NR + j, L, D3, c1);
      z2[j] = zld(zb, s0 - NR + j, L, D3, c2);
      z3[j] = zld(zb, s0 - NR + j, L, D3, c3);
    }
#pragma unroll
    for (int i = 0; i < KC; ++i) d1[i] = d2[i] = d3[i] = 0.f;
#pragma unroll
    for (int g = 0; g < NIT; g += HY_PF) {
      float n1[HY_PF], n2[HY_PF], n3[HY_PF], ng[HY_PF];
#pragma unroll
      for (int u = 0; u < HY_PF; ++u) {
        const int tn = s0 + g + u;
        n1[u] = zld(zb, tn, L, D3, c1);
        n2[u] = zld(zb, tn, L, D3, c2);
        n3[u] = zld(zb, tn, L, D3, c3);
        ng[u] = (tn < L && g + u < NIT) ? (float)gx2[(long long)tn * a.D] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < HY_PF; ++u) {
        if (g + u < NIT) {
          const int tn = s0 + g + u;
#pragma unroll
          for (int j = 0; j < NR - 1; ++j) { z1[j] = z1[j + 1]; z2[j] = z2[j + 1]; z3[j] = z3[j + 1]; }
          z1[NR - 1] = n1[u]; z2[NR - 1] = n2[u]; z3[NR - 1] = n3[u];
          float x1 = b1, v = b3;
#pragma unroll
          for (int i = 0; i < KC; ++i) { x1 = fmaf(w1[i], z1[KC - 1 + i], x1); v = fmaf(w3[i], z3[KC - 1 + i], v); }
          const float dv = tn < L ? dvt[lane][tn - t0] : 0.f;
#pragma unroll
          for (int i = 0; i < KC - 1; ++i) { d1[i] = d1[i + 1]; d2[i] = d2[i + 1]; d3[i] = d3[i + 1]; }
          d1[KC - 1] = dv * v; d2[KC - 1] = ng[u]; d3[KC - 1] = dv * x1;
          const int s = tn - (KC - 1);
          if (s >= s0 && s < s1) {
            float o1 = 0.f, o2 = 0.f, o3 = 0.f;
#pragma unroll
            for (int i = 0; i < KC; ++i) {
              o1 = fmaf(w1[i], d1[KC - 1 - i], o1);
              o2 = fmaf(w2[i], d2[KC - 1 - i], o2);
              o3 = fmaf(w3[i], d3[KC - 1 - i], o3);
            }
            if (valid) {
              T* dzr = dzb + (long long)s * D3;
              dzr[c1] = (T)o1; dzr[c2] = (T)o2; dzr[c3] = (T)o3;
            }
#pragma unroll
            for (int i = 0; i < KC; ++i) {
              acc[i] = fmaf(d1[0], z1[i], acc[i]);
              acc[KC + 1 + i] = fmaf(d2[0], z2[i], acc[KC + 1 + i]);
              acc[2 * KC + 2 + i] = fmaf(d3[0], z3[i], acc[2 * KC + 2 + i]);
            }
            acc[KC] += d1[0]; acc[2 * KC + 1] += d2[0]; acc[3 * KC + 2] += d3[0];
          }
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < NA; ++i) red[wave][i][lane] = acc[i];
  __syncthreads();
  for (int idx = threadIdx.x; idx < NA * 64; idx += 256) {
    const int i = idx / 64, l = idx - i * 64, c = ch0 + l;
    if (c >= a.D) continue;
    const float sum = (red[0][i][l] + red[1][i][l]) + (red[2][i][l] + red[3][i][l]);
    const int hh = c / a.hd, jc = c - hh * a.hd;
    const int grp = i / (KC + 1), k = i - grp * (KC + 1);
    const int cc = hh * 3 * a.hd + grp * a.hd + jc;
    if (k < KC) atomicAdd(a.dw + cc * KC + k, sum);
    else if (a.db) atomicAdd(a.db + cc, sum);
  }
}

static int fft_plan(FftArgs& a, int L) {
  LCI_CHECK(L > 0 && L <= (1 << 18), "fftconv: L %d unsupported (<= 262144)", L);
  int e = 1;
  while ((1 << e) < 2 * L) ++e;
  a.n = 1 << e;
  // n1 = 256-point column FFTs over G = 8 adjacent columns, n2 = n / 256 row FFTs (512 at L = 65536): the best
  // of the (n1, G) sweep in tools/fft_sweep.sh (wider column groups cost more in LDS occupancy than they save)
  a.ln1 = e < 8 ? e : 8;
  // the row pass keeps ~11 n2-point complex rows in LDS: n2 <= 1024 (n = 2^19 at L = 262144: n1 = 512, n2 = 1024)
  if (e - a.ln1 > 10) a.ln1 = e - 10;
  a.ln2 = e - a.ln1;
  if (a.ln2 == 0) { a.ln1 = e - 1; a.ln2 = 1; }
  // n = 2^17 .. 2^19: 512-point rows on fft_row512_kernel, n1 = 256 .. 1024 columns on the wide column kernel
  if (e >= 17 && e <= 19) { a.ln2 = 9; a.ln1 = e - 9; }
  a.n1 = 1 << a.ln1; a.n2 = 1 << a.ln2;
  a.G = a.n2 < 8 ? a.n2 : 8;
  a.L = L;
  return 0;
}


// ------------------------------------------- short conv + gating, LDS-staged 16-byte global accesses (v3)
// Same math as the register-ring kernels above; every global access is a 16-byte vector (8 bf16 / 4 f32) of
// one row: the channels-last rows (z, x2, dz, out, dout, dx2, gx2) and the channel-major f32 rows (vg, dvg, y, dy)
// are staged through LDS tiles of 64 tokens x 64 output channels, and the per-channel arithmetic reads LDS with
// lane = channel. The narrow (2-byte-per-lane) global accesses of the v2 kernels held them to 1-3 TB/s.
// Preconditions (checked by the launcher, else v2 runs): bf16 activations, hd % 8 == 0, D % 8 == 0, L % 4 == 0.
constexpr int HG_TT = 64;            // tokens per tile
constexpr int HG_S = HG_TT + 1;      // odd row stride (f32) of the channel-major LDS tiles

__device__ __forceinline__ int hg_zcol(int ch, int g, int hd) {   // z channel of gate g (x1, x2, v) of channel ch
  const int h = ch / hd;
  return h * 3 * hd + g * hd + (ch - h * hd);
}

// ty[r][tl] <- rows (channels ch0 + r) x tokens [t0, t0 + 64) of a channel-major f32 tensor
__device__ __forceinline__ void hg_stage_cm(float* ty, const float* src, int bb, int ch0, int t0, int D, int L) {
  for (int i = threadIdx.x; i < 64 * (HG_TT / 4); i += 256) {
    const int r = i / (HG_TT / 4), c4 = (i - r * (HG_TT / 4)) * 4, ch = ch0 + r, t = t0 + c4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (ch < D && t < L) v = *(const f32x4*)(src + ((long long)bb * D + ch) * L + t);
#pragma unroll
    for (int j = 0; j < 4; ++j) ty[r * HG_S + c4 + j] = v[j];
  }
}

// dst rows (channel-major) <- ty
__device__ __forceinline__ void hg_store_cm(float* dst, const float* ty, int bb, int ch0, int t0, int D, int L) {
  for (int i = threadIdx.x; i < 64 * (HG_TT / 4); i += 256) {
    const int r = i / (HG_TT / 4), c4 = (i - r * (HG_TT / 4)) * 4, ch = ch0 + r, t = t0 + c4;
    if (ch >= D || t >= L) continue;
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = ty[r * HG_S + c4 + j];
    *(f32x4*)(dst + ((long long)bb * D + ch) * L + t) = v;
  }
}

__global__ __launch_bounds__(256) void hyena_post_fwd3_kernel(GateArgs a) {
  __shared__ float ty[64 * HG_S];
  const int t0 = blockIdx.x * HG_TT, ch0 = blockIdx.y * 64, bb = blockIdx.z, L = a.L, D = a.D;
  hg_stage_cm(ty, a.y, bb, ch0, t0, D, L);
  __syncthreads();
  for (int i = threadIdx.x; i < HG_TT * 8; i += 256) {
    const int q = i & 7, tl = i >> 3, t = t0 + tl, ch = ch0 + 8 * q;
    if (t >= L || ch >= D) continue;
    const long long o = ((long long)bb * L + t) * D + ch;
    const bf16x8 xv = *(const bf16x8*)((const bf16*)a.x2 + o);
    bf16x8 ov;
#pragma unroll
    for (int j = 0; j < 8; ++j) ov[j] = (bf16)(ty[(8 * q + j) * HG_S + tl] * (float)xv[j]);
    *(bf16x8*)((bf16*)a.out + o) = ov;
  }
}

__global__ __launch_bounds__(256) void hyena_post_bwd3_kernel(GateArgs a) {
  __shared__ float ty[64 * HG_S];
  __shared__ float tg[64 * HG_S];
  const int t0 = blockIdx.x * HG_TT, ch0 = blockIdx.y * 64, bb = blockIdx.z, L = a.L, D = a.D;
  hg_stage_cm(ty, a.y, bb, ch0, t0, D, L);
  __syncthreads();
  for (int i = threadIdx.x; i < HG_TT * 8; i += 256) {
    const int q = i & 7, tl = i >> 3, t = t0 + tl, ch = ch0 + 8 * q;
    if (t >= L || ch >= D) continue;
    const long long o = ((long long)bb * L + t) * D + ch;
    const bf16x8 gv = *(const bf16x8*)((const bf16*)a.dout + o);
    const bf16x8 xv = *(const bf16x8*)((const bf16*)a.x2 + o);
    bf16x8 dv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float go = (float)gv[j];
      tg[(8 * q + j) * HG_S + tl] = go * (float)xv[j];
      dv[j] = (bf16)(go * ty[(8 * q + j) * HG_S + tl]);
    }
    *(bf16x8*)((bf16*)a.dx2 + o) = dv;
  }
  __syncthreads();
  hg_store_cm(a.dy, tg, bb, ch0, t0, D, L);
}

// z tile rows r <- tokens t0 - HALO + r (zero outside [0, L)), the three gate channel runs of ch0 .. ch0 + 63.
__device__ __forceinline__ void hg_stage_z(bf16* zt, const bf16* zb, int rows, int t0, int halo, int ch0, int D,
                                           int L, int hd) {
  for (int i = threadIdx.x; i < rows * 24; i += 256) {
    const int r = i / 24, k = i - r * 24, g = k >> 3, q = k & 7;
    const int t = t0 - halo + r, ch = ch0 + 8 * q;
    bf16x8 v = {};
    if (t >= 0 && t < L && ch < D) v = *(const bf16x8*)(zb + (long long)t * 3 * D + hg_zcol(ch, g, hd));
    *(bf16x8*)(zt + r * 192 + g * 64 + 8 * q) = v;
  }
}

template <int KC>
__global__ __launch_bounds__(256) void hyena_pre_fwd3_kernel(GateArgs a) {
  constexpr int ZR = HG_TT + KC - 1;
  __shared__ __attribute__((aligned(16))) bf16 zt[ZR * 192];
  __shared__ __attribute__((aligned(16))) bf16 x2t[HG_TT * 64];
  __shared__ float vgt[64 * HG_S];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t0 = blockIdx.x * HG_TT, ch0 = blockIdx.y * 64, bb = blockIdx.z, L = a.L, D = a.D;
  hg_stage_z(zt, (const bf16*)a.z + (long long)bb * L * 3 * D, ZR, t0, KC - 1, ch0, D, L, a.hd);
  const int chc = min(ch0 + lane, D - 1);
  const int c1 = hg_zcol(chc, 0, a.hd), c2 = c1 + a.hd, c3 = c1 + 2 * a.hd;
  float w1[KC], w2[KC], w3[KC];
#pragma unroll
  for (int i = 0; i < KC; ++i) { w1[i] = a.w[c1 * KC + i]; w2[i] = a.w[c2 * KC + i]; w3[i] = a.w[c3 * KC + i]; }
  const float b1 = a.bias ? a.bias[c1] : 0.f, b2 = a.bias ? a.bias[c2] : 0.f, b3 = a.bias ? a.bias[c3] : 0.f;
  __syncthreads();
  const int sl0 = wave * (HG_TT / 4);
  auto zr = [&](int row, int g) -> float { return (float)zt[row * 192 + g * 64 + lane]; };
  float r1[KC], r2[KC], r3[KC];   // rows sl .. sl + KC - 1 = tokens s - KC + 1 .. s
#pragma unroll
  for (int i = 1; i < KC; ++i) { r1[i] = zr(sl0 + i - 1, 0); r2[i] = zr(sl0 + i - 1, 1); r3[i] = zr(sl0 + i - 1, 2); }
#pragma unroll
  for (int u = 0; u < HG_TT / 4; ++u) {
    const int sl = sl0 + u;
#pragma unroll
    for (int i = 0; i < KC - 1; ++i) { r1[i] = r1[i + 1]; r2[i] = r2[i + 1]; r3[i] = r3[i + 1]; }
    r1[KC - 1] = zr(sl + KC - 1, 0); r2[KC - 1] = zr(sl + KC - 1, 1); r3[KC - 1] = zr(sl + KC - 1, 2);
    float x1 = b1, x2 = b2, v = b3;
#pragma unroll
    for (int i = 0; i < KC; ++i) { x1 = fmaf(w1[i], r1[i], x1); x2 = fmaf(w2[i], r2[i], x2); v = fmaf(w3[i], r3[i], v); }
    x2t[sl * 64 + lane] = (bf16)x2;
    vgt[lane * HG_S + sl] = v * x1;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < HG_TT * 8; i += 256) {
    const int q = i & 7, tl = i >> 3, t = t0 + tl, ch = ch0 + 8 * q;
    if (t < L && ch < D)
      *(bf16x8*)((bf16*)a.x2 + ((long long)bb * L + t) * D + ch) = *(const bf16x8*)(x2t + tl * 64 + 8 * q);
  }
  hg_store_cm(a.vg, vgt, bb, ch0, t0, D, L);
}

// dz / dw / db of the short conv + gates (see hyena_pre_bwd2_kernel), token tiles strided over a persistent grid.
template <int KC>
__global__ __launch_bounds__(256) void hyena_pre_bwd3_kernel(GateArgs a) {
  constexpr int ZR = HG_TT + 2 * KC - 2;        // z rows: tokens t0 - KC + 1 .. t0 + TT + KC - 2
  constexpr int W = HG_TT + KC - 1;             // dconv tokens t0 .. t0 + TT + KC - 2
  constexpr int WS = W | 1;                     // odd stride of the dvg tile
  constexpr int W4 = (W + 3) / 4;
  constexpr int NR = 2 * KC - 1;
  constexpr int TW = HG_TT / 4;                 // output tokens per wave
  constexpr int NIT = TW + KC - 1;
  constexpr int NA = 3 * (KC + 1);
  static_assert(4 * NA * 64 * 4 <= ZR * 192 * 2, "reduction scratch must fit the z tile");
  __shared__ __attribute__((aligned(16))) bf16 zt[ZR * 192];    // z rows, then dz rows, then the dw/db reduction
  __shared__ float dvt[64 * WS];
  __shared__ __attribute__((aligned(16))) float gxt[W4 * 4 * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ch0 = blockIdx.y * 64, bb = blockIdx.z, L = a.L, D = a.D, D3 = 3 * D;
  const int ch = ch0 + lane, chc = min(ch, D - 1);
  const int c1 = hg_zcol(chc, 0, a.hd), c2 = c1 + a.hd, c3 = c1 + 2 * a.hd;
  const bf16* zb = (const bf16*)a.z + (long long)bb * L * D3;
  const bf16* gx2 = (const bf16*)a.gx2 + (long long)bb * L * D;
  bf16* dzb = (bf16*)a.dz + (long long)bb * L * D3;
  float w1[KC], w2[KC], w3[KC];
#pragma unroll
  for (int i = 0; i < KC; ++i) { w1[i] = a.w[c1 * KC + i]; w2[i] = a.w[c2 * KC + i]; w3[i] = a.w[c3 * KC + i]; }
  const float b1 = a.bias ? a.bias[c1] : 0.f, b3 = a.bias ? a.bias[c3] : 0.f;
  float acc[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) acc[i] = 0.f;
  const int ntiles = (L + HG_TT - 1) / HG_TT;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int t0 = tile * HG_TT;
    hg_stage_z(zt, zb, ZR, t0, KC - 1, ch0, D, L, a.hd);
    for (int i = threadIdx.x; i < 64 * W4; i += 256) {          // dvg rows, tokens t0 .. t0 + W - 1
      const int r = i / W4, c4 = (i - r * W4) * 4, c = ch0 + r, t = t0 + c4;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (c < D && t < L) v = *(const f32x4*)(a.dvg + ((long long)bb * D + c) * L + t);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (c4 + j < W) dvt[r * WS + c4 + j] = v[j];
    }
    for (int i = threadIdx.x; i < W4 * 4 * 8; i += 256) {       // gx2 rows (tokens), 64 channels, bf16 -> f32
      const int r = i >> 3, c8 = (i & 7) * 8, t = t0 + r, c = ch0 + c8;
      bf16x8 v = {};
      if (t < L && c < D) v = *(const bf16x8*)(gx2 + (long long)t * D + c);
      f32x4 lo, hi;
#pragma unroll
      for (int j = 0; j < 4; ++j) { lo[j] = (float)v[j]; hi[j] = (float)v[4 + j]; }
      *(f32x4*)(gxt + r * 64 + c8) = lo;
      *(f32x4*)(gxt + r * 64 + c8 + 4) = hi;
    }
    __syncthreads();
    const int sl0 = wave * TW, s0 = t0 + sl0;
    auto zr = [&](int row, int g) -> float { return row >= 0 ? (float)zt[row * 192 + g * 64 + lane] : 0.f; };
    float z1[NR], z2[NR], z3[NR], d1[KC], d2[KC], d3[KC], o1[TW], o2[TW], o3[TW];
#pragma unroll
    for (int j = 1; j < NR; ++j) {   // ring entry j <-> token s0 - NR + j (row sl0 - NR + j + KC - 1)
      z1[j] = zr(sl0 - NR + j + KC - 1, 0); z2[j] = zr(sl0 - NR + j + KC - 1, 1); z3[j] = zr(sl0 - NR + j + KC - 1, 2);
    }
#pragma unroll
    for (int i = 0; i < KC; ++i) d1[i] = d2[i] = d3[i] = 0.f;
#pragma unroll
    for (int k = 0; k < NIT; ++k) {
      const int tn = s0 + k, tl = sl0 + k;    // tl < W
#pragma unroll
      for (int j = 0; j < NR - 1; ++j) { z1[j] = z1[j + 1]; z2[j] = z2[j + 1]; z3[j] = z3[j + 1]; }
      z1[NR - 1] = zr(tl + KC - 1, 0); z2[NR - 1] = zr(tl + KC - 1, 1); z3[NR - 1] = zr(tl + KC - 1, 2);
      float x1 = b1, v = b3;
#pragma unroll
      for (int i = 0; i < KC; ++i) { x1 = fmaf(w1[i], z1[KC - 1 + i], x1); v = fmaf(w3[i], z3[KC - 1 + i], v); }
      const bool in = tn < L;
      const float dv = in ? dvt[lane * WS + tl] : 0.f;
#pragma unroll
      for (int i = 0; i < KC - 1; ++i) { d1[i] = d1[i + 1]; d2[i] = d2[i + 1]; d3[i] = d3[i + 1]; }
      d1[KC - 1] = dv * v; d2[KC - 1] = in ? gxt[tl * 64 + lane] : 0.f; d3[KC - 1] = dv * x1;
      if (k >= KC - 1) {
        const int u = k - (KC - 1), s = s0 + u;
        float p1 = 0.f, p2 = 0.f, p3 = 0.f;
#pragma unroll
        for (int i = 0; i < KC; ++i) {
          p1 = fmaf(w1[i], d1[KC - 1 - i], p1);
          p2 = fmaf(w2[i], d2[KC - 1 - i], p2);
          p3 = fmaf(w3[i], d3[KC - 1 - i], p3);
        }
        o1[u] = p1; o2[u] = p2; o3[u] = p3;
        if (s < L) {
#pragma unroll
          for (int i = 0; i < KC; ++i) {
            acc[i] = fmaf(d1[0], z1[i], acc[i]);
            acc[KC + 1 + i] = fmaf(d2[0], z2[i], acc[KC + 1 + i]);
            acc[2 * KC + 2 + i] = fmaf(d3[0], z3[i], acc[2 * KC + 2 + i]);
          }
          acc[KC] += d1[0]; acc[2 * KC + 1] += d2[0]; acc[3 * KC + 2] += d3[0];
        }
      }
    }
    __syncthreads();                                   // every wave is done with the z / dvg / gx2 tiles
#pragma unroll
    for (int u = 0; u < TW; ++u) {
      bf16* row = zt + (sl0 + u) * 192 + lane;
      row[0] = (bf16)o1[u]; row[64] = (bf16)o2[u]; row[128] = (bf16)o3[u];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < HG_TT * 24; i += 256) {
      const int r = i / 24, k = i - r * 24, g = k >> 3, q = k & 7, t = t0 + r, c = ch0 + 8 * q;
      if (t < L && c < D)
        *(bf16x8*)(dzb + (long long)t * D3 + hg_zcol(c, g, a.hd)) = *(const bf16x8*)(zt + r * 192 + g * 64 + 8 * q);
    }
    __syncthreads();
  }
  float* red = (float*)zt;                           // [4 waves][NA][64]
#pragma unroll
  for (int i = 0; i < NA; ++i) red[(wave * NA + i) * 64 + lane] = acc[i];
  __syncthreads();
  for (int idx = threadIdx.x; idx < NA * 64; idx += 256) {
    const int i = idx / 64, l = idx - i * 64, c = ch0 + l;
    if (c >= D) continue;
    const float sum = (red[i * 64 + l] + red[(NA + i) * 64 + l]) + (red[(2 * NA + i) * 64 + l] + red[(3 * NA + i) * 64 + l]);
    const int grp = i / (KC + 1), k = i - grp * (KC + 1);
    const int cc = hg_zcol(c, grp, a.hd);
    if (k < KC) atomicAdd(a.dw + cc * KC + k, sum);
    else if (a.db) atomicAdd(a.db + cc, sum);
  }
}

// Whether the v3 kernels take this call (else the v2 register-ring kernels run).
static bool hg_v3_ok(const GateArgs& a, int dtype, std::initializer_list<const void*> ptrs) {
  if (dtype != 1 || a.hd % 8 || a.D % 8 || a.L % 4) return false;
  for (const void* p : ptrs)
    if (p && ((uintptr_t)p & 15)) return false;
  return true;
}
}  // namespace lci

using namespace lci;

extern "C" long long lci_fft_size(int L) {
  FftArgs a{};
  if (fft_plan(a, L)) return -1;
  return a.n;
}

// tw: n complex (f32x2) workspace filled here.
extern "C" int lci_fft_twiddles(void* tw, int n, void* stream) {
  hipLaunchKernelGGL(twiddle_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (f32x2*)tw, n);
  LCI_LAUNCH_CHECK();
  return 0;
}

static int launch_col(FftArgs& a, bool inv, int nblk_y, hipStream_t s) {
  // wide column kernels: complex elements per workgroup 4096 at n1 <= 512 (~130 instead of ~245 VGPRs, 4 workgroups
  // per CU; >= 8 columns = 32-B row segments), 16384 at n1 = 1024 (16 columns, 64-B row segments, 512 threads, the
  // register column FFTs); the LDS kernels below for short columns / few columns (n2 < GW)
  const int cw = a.n1 == 1024 ? 2 * CW_ELEMS : CW_ELEMS / 2;
  const int gw = cw / a.n1;
  if ((a.n1 == 1024 || a.n1 <= 512) && (gw == 8 || gw == 16) && a.n2 % gw == 0) {
    const size_t sh = ((size_t)gw * (a.n1 + 1) + a.n1 + tw3_entries(a.ln1 + a.ln2) +
                       (col_wave_scratch(a.n1, gw) ? 4 * 8 * R5_S1 : 0)) * sizeof(f32x2);
    // GP = 4 column groups per workgroup, the next group's rows loaded during this group's FFT (wave FFT path;
    // the forward's 16-B loads need L % 4 == 0)
    const bool gp = gw == 16 && (a.n2 / gw) % 4 == 0 && (inv || (a.L & 3) == 0);
    const dim3 grid(gp ? a.n2 / gw / 4 : a.n2 / gw, nblk_y);
#define LCI_COLW(GW, CW, NT, GP)                                                                                   \
    (void)hipFuncSetAttribute((const void*)(inv ? fft_colw_inv_kernel<GW, CW, NT, GP> : fft_colw_fwd_kernel<GW, CW, NT, GP>), \
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);                           \
    if (inv) hipLaunchKernelGGL((fft_colw_inv_kernel<GW, CW, NT, GP>), grid, dim3(NT), sh, s, a);                \
    else hipLaunchKernelGGL((fft_colw_fwd_kernel<GW, CW, NT, GP>), grid, dim3(NT), sh, s, a);
    if (a.n1 == 1024) {
      if (gp) { LCI_COLW(16, 16384, 512, 4) } else { LCI_COLW(16, 16384, 512, 1) }
    } else if (gw == 16) {
      if (gp && a.n1 == 256) { LCI_COLW(16, 4096, 256, 4) } else { LCI_COLW(16, 4096, 256, 1) }
    } else {
      LCI_COLW(8, 4096, 256, 1)
    }
#undef LCI_COLW
    LCI_LAUNCH_CHECK();
    return 0;
  }
  const size_t sh = ((size_t)2 * a.G * (a.n1 + 1) + a.n1) * sizeof(f32x2);
  (void)hipFuncSetAttribute((const void*)(inv ? fft_col_inv_kernel : fft_col_fwd_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  dim3 grid(a.n2 / a.G, nblk_y);
  if (inv) hipLaunchKernelGGL(fft_col_inv_kernel, grid, dim3(256), sh, s, a);
  else hipLaunchKernelGGL(fft_col_fwd_kernel, grid, dim3(256), sh, s, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

static int launch_row(FftArgs& a, int nfilt, hipStream_t s) {
  if (a.n2 == 512) {
    int nw = 1;   // waves per workgroup: the largest divisor of the pair count up to 4 (balanced waves)
    for (int q = 4; q >= 1; --q)
      if (a.P % q == 0) { nw = q; break; }
    if (a.mode == 0) {   // filter spectra: 4 rows k1 per workgroup (one-wave workgroups were latency-bound)
      hipLaunchKernelGGL(fft_row512_kernel, dim3(a.n1 / 4, nfilt), dim3(256), 0, s, a);
      LCI_LAUNCH_CHECK();
      return 0;
    }
    hipLaunchKernelGGL(fft_row512_kernel, dim3(a.n1, nfilt), dim3(64 * nw), 0, s, a);
    LCI_LAUNCH_CHECK();
    return 0;
  }
  a.pb = ROW_PB;
  const size_t sh = ((size_t)2 * a.pb + 3) * a.n2 * sizeof(f32x2);   // x, y (+ x2, y2 at PB/2) + kr, acc, twl
  LCI_CHECK(sh <= 160 * 1024, "fft row pass: %zu bytes of LDS", sh);
  (void)hipFuncSetAttribute((const void*)fft_row_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const int thr = a.n2 >= 1024 ? 512 : 256;
  hipLaunchKernelGGL(fft_row_kernel, dim3(a.n1, nfilt), dim3(thr), sh, s, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

// Filter spectra: k (C, L) f32 -> K (C, n) complex in [k1][k2] layout, scaled by 1/n, + D / n when Dv is given
// (the conv with K then carries + D u, forward and adjoint: D is real). SK: (C, n) scratch.
extern "C" int lci_fftconv_spectrum(const float* k, const float* Dv, void* K, void* SK, const void* tw, int C, int L,
                                    void* stream) {
  FftArgs a{};
  if (fft_plan(a, L)) return 1;
  a.src = k; a.Dv = Dv; a.K = (f32x2*)K; a.SK = (f32x2*)SK; a.tw = (const f32x2*)tw; a.C = C; a.single = 1; a.mode = 0;
  hipStream_t s = (hipStream_t)stream;
  a.pid0 = 0;
  if (launch_col(a, false, C, s)) return 3;
  if (launch_row(a, C, s)) return 3;
  return 0;
}

// y = causal_conv(u, k) + D u for rows (R, C, L) f32; filter j = row % C. S: (C * ceil(R/2), n) scratch.
// Su (optional, same shape as S): receives the column spectra of u and is left intact (the row pass writes its
// products to S), so the backward's filter gradient reuses it instead of recomputing the column FFT of u.
extern "C" int lci_fftconv_fwd(const float* u, const void* K, const float* Dv, float* y, void* S, void* Su,
                               const void* tw, int R, int C, int L, void* stream) {
  FftArgs a{};
  if (fft_plan(a, L)) return 1;
  a.src = u; a.dst = y; a.K = (f32x2*)K; a.tw = (const f32x2*)tw; a.Dv = Dv;
  a.R = R; a.C = C; a.P = (R + 1) / 2; a.single = 0; a.mode = 1;
  hipStream_t s = (hipStream_t)stream;
  a.pid0 = 0;
  a.S = (f32x2*)(Su ? Su : S);
  if (launch_col(a, false, C * a.P, s)) return 3;
  a.So = Su ? (f32x2*)S : nullptr;
  if (launch_row(a, C, s)) return 3;
  a.So = nullptr;
  a.S = (f32x2*)S;
  if (launch_col(a, true, C * a.P, s)) return 3;
  return 0;
}

// Adjoint: du = corr(dy, k) + D dy; dk (C, L) = sum_rows corr(dy, u) (overwritten); dD (C) accumulated.
// S, S2: (C * ceil(R/2), n) scratch; SK: (C, n) scratch. Su: the forward's kept column spectra of u, or null (then
// S2 receives them here).
extern "C" int lci_fftconv_bwd(const float* dy, const float* u, const void* K, const float* Dv, float* du, float* dk,
                               float* dD, void* S, void* S2, const void* Su, void* SK, const void* tw, int R, int C,
                               int L, void* stream) {
  FftArgs a{};
  if (fft_plan(a, L)) return 1;
  a.tw = (const f32x2*)tw; a.K = (f32x2*)K; a.S = (f32x2*)S; a.S2 = (f32x2*)(Su ? Su : S2);
  a.SK = dk ? (f32x2*)SK : nullptr;
  a.R = R; a.C = C; a.P = (R + 1) / 2; a.Dv = Dv; a.dk = dk;
  hipStream_t s = (hipStream_t)stream;
  FftArgs c = a;
  c.single = 0;
  c.src = dy;
  c.pid0 = 0;
  if (launch_col(c, false, C * a.P, s)) return 3;            // S <- col FFT of dy pairs
  if (dk && !Su) {
    FftArgs b = c;
    b.S = (f32x2*)S2; b.src = u;
    if (launch_col(b, false, C * a.P, s)) return 3;          // S2 <- col FFT of u pairs
  }
  c.mode = 2;
  if (launch_row(c, C, s)) return 3;                         // S <- conj(K) products, SK <- dk rows
  c.src = dy; c.dst = du;
  if (launch_col(c, true, C * a.P, s)) return 3;             // du = IFFT (+ D dy)
  if (dk) {
    FftArgs b = c;
    b.single = 1;
    if (launch_col(b, true, C, s)) return 3;                 // dk[j] = Re IFFT(SK_j)
  }
  if (dD && dk) {   // the lag-0 filter-gradient entry is the dD sum
    hipLaunchKernelGGL(dd_from_dk_kernel, dim3((C + 255) / 256), dim3(256), 0, s, dk, dD, C, L);
    LCI_LAUNCH_CHECK();
  } else if (dD) {
    const int vec = (L % 4 == 0) && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)u & 15) == 0;
    hipLaunchKernelGGL(row_dot_kernel, dim3(R * C, (L + RD_SPAN - 1) / RD_SPAN), dim3(256), 0, s, dy, u, dD, L, C,
                       vec);
    LCI_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" int lci_hyena_pre_fwd(int dtype, const void* z, const float* w, const float* bias, float* vg, void* x2,
                                 int BB, int L, int H, int hd, int K, void* stream) {
  LCI_CHECK(K >= 1 && K <= 8, "hyena_pre: short filter order %d unsupported (<= 8)", K);
  GateArgs a{};
  a.z = z; a.w = w; a.bias = bias; a.vg = vg; a.x2 = x2; a.BB = BB; a.L = L; a.H = H; a.hd = hd; a.D = H * hd; a.K = K;
  if (hg_v3_ok(a, dtype, {z, vg, x2})) {
    dim3 grid3((L + HG_TT - 1) / HG_TT, (a.D + 63) / 64, BB);
#define LCI_PRE_FWD3(KK) \
  case KK: hipLaunchKernelGGL(hyena_pre_fwd3_kernel<KK>, grid3, dim3(256), 0, (hipStream_t)stream, a); LCI_LAUNCH_CHECK(); return 0;
    switch (K) {
      LCI_PRE_FWD3(1) LCI_PRE_FWD3(2) LCI_PRE_FWD3(3) LCI_PRE_FWD3(4) LCI_PRE_FWD3(5) LCI_PRE_FWD3(6) LCI_PRE_FWD3(7)
      LCI_PRE_FWD3(8)
      default: break;
    }
#undef LCI_PRE_FWD3
  }
  // register-ring kernels (every order the C-ABI accepts)
  dim3 grid2((L + HY_TT - 1) / HY_TT, (a.D + 63) / 64, BB);
#define LCI_PRE_FWD(KK)                                                                                         \
  case KK:                                                                                                    \
    if (dtype == 1)                                                                                           \
      hipLaunchKernelGGL((hyena_pre_fwd2_kernel<bf16, KK>), grid2, dim3(256), 0, (hipStream_t)stream, a);     \
    else                                                                                                      \
      hipLaunchKernelGGL((hyena_pre_fwd2_kernel<float, KK>), grid2, dim3(256), 0, (hipStream_t)stream, a);    \
    break;
  switch (K) {
    LCI_PRE_FWD(1) LCI_PRE_FWD(2) LCI_PRE_FWD(3) LCI_PRE_FWD(4) LCI_PRE_FWD(5) LCI_PRE_FWD(6) LCI_PRE_FWD(7)
    LCI_PRE_FWD(8)
    default: break;
  }
#undef LCI_PRE_FWD
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_hyena_post_fwd(int dtype, const float* y, const void* x2, void* out, int BB, int L, int D,
                                  void* stream) {
  GateArgs a{};
  a.y = y; a.x2 = (void*)x2; a.out = out; a.BB = BB; a.L = L; a.D = D; a.hd = 8;
  dim3 grid((L + 63) / 64, (D + 63) / 64, BB);
  if (hg_v3_ok(a, dtype, {y, x2, out})) {
    hipLaunchKernelGGL(hyena_post_fwd3_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
    LCI_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == 1) hipLaunchKernelGGL(hyena_post_fwd_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(hyena_post_fwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" int lci_hyena_post_bwd(int dtype, const float* y, const void* x2, const void* dout, float* dy, void* dx2,
                                  int BB, int L, int D, void* stream) {
  GateArgs a{};
  a.y = y; a.x2 = (void*)x2; a.dout = dout; a.dy = dy; a.dx2 = dx2; a.BB = BB; a.L = L; a.D = D; a.hd = 8;
  dim3 grid((L + 63) / 64, (D + 63) / 64, BB);
  if (hg_v3_ok(a, dtype, {y, x2, dout, dy, dx2})) {
    hipLaunchKernelGGL(hyena_post_bwd3_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
    LCI_LAUNCH_CHECK();
    return 0;
  }
  if (dtype == 1) hipLaunchKernelGGL(hyena_post_bwd_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(hyena_post_bwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

// dw (3D, K), db (3D) accumulated (caller zeroes). gx2 (BB, L, D) in z's dtype.
extern "C" int lci_hyena_pre_bwd(int dtype, const void* z, const float* w, const float* bias, const float* dvg,
                                 const void* gx2, void* dz, float* dw, float* db, int BB, int L, int H, int hd, int K,
                                 void* stream) {
  LCI_CHECK(K >= 1 && K <= 8, "hyena_pre: short filter order %d unsupported (<= 8)", K);
  GateArgs a{};
  a.z = z; a.w = w; a.bias = bias; a.dvg = dvg; a.gx2 = gx2; a.dz = dz; a.dw = dw; a.db = db;
  a.BB = BB; a.L = L; a.H = H; a.hd = hd; a.D = H * hd; a.K = K;
  if (hg_v3_ok(a, dtype, {z, dvg, gx2, dz})) {   // persistent: ~2 workgroups per CU stride over the token tiles
    const int ntiles = (L + HG_TT - 1) / HG_TT, ncy = (a.D + 63) / 64;
    const int gx = std::max(1, std::min(ntiles, 512 / std::max(1, ncy * BB)));
    dim3 grid3(gx, ncy, BB);
#define LCI_PRE_BWD3(KK) \
  case KK: hipLaunchKernelGGL(hyena_pre_bwd3_kernel<KK>, grid3, dim3(256), 0, (hipStream_t)stream, a); LCI_LAUNCH_CHECK(); return 0;
    switch (K) {
      LCI_PRE_BWD3(1) LCI_PRE_BWD3(2) LCI_PRE_BWD3(3) LCI_PRE_BWD3(4) LCI_PRE_BWD3(5) LCI_PRE_BWD3(6) LCI_PRE_BWD3(7)
      LCI_PRE_BWD3(8)
      default: break;
    }
#undef LCI_PRE_BWD3
  }
  // one lane per output channel, token tiles strided over ~8 workgroups/CU (every order the C-ABI accepts)
  const int ntiles = (L + HY_TT - 1) / HY_TT, ncy = (a.D + 63) / 64;
  const int gx = std::max(1, std::min(ntiles, 2048 / std::max(1, ncy * BB)));
  dim3 grid2(gx, ncy, BB);
#define LCI_PRE_BWD2(KK)                                                                                        \
  case KK:                                                                                                    \
    if (dtype == 1)                                                                                           \
      hipLaunchKernelGGL((hyena_pre_bwd2_kernel<bf16, KK>), grid2, dim3(256), 0, (hipStream_t)stream, a);     \
    else                                                                                                      \
      hipLaunchKernelGGL((hyena_pre_bwd2_kernel<float, KK>), grid2, dim3(256), 0, (hipStream_t)stream, a);    \
    break;
  switch (K) {
    LCI_PRE_BWD2(1) LCI_PRE_BWD2(2) LCI_PRE_BWD2(3) LCI_PRE_BWD2(4) LCI_PRE_BWD2(5) LCI_PRE_BWD2(6)
    LCI_PRE_BWD2(7) LCI_PRE_BWD2(8)
    default: break;
  }
#undef LCI_PRE_BWD2
  LCI_LAUNCH_CHECK();
  return 0;
}
