// Mamba mixer kernels for gfx950: selective scan (fwd / bwd) and depthwise conv + SiLU, channels-last.
//
// Replaces (MambaVisionMixer.forward, mamba.py:108-139):
//   x, z = SiLU(conv1d(x|z, k=3, padding='same', groups=C))                             (:118-119)
//   y = selective_scan_fn(x, dt, A, B, C, D, delta_bias=b, delta_softplus=True)         (:125-134)
// selective_scan_fn is mamba-ssm 1.2.0.post1's CUDA op; semantics = selective_scan_ref:
//   dt' = softplus(dt + b);  x_t[n] = exp(dt' A[n]) x_{t-1}[n] + dt' B_t[n] u_t;  y_t = sum_n C_t[n] x_t[n] + D u_t
//
// Layout: every activation is channels-last (B, L, C) with a token stride, so the Linear outputs are read in
// place (B and C are strided column slices of the x_proj output). One wave = 64 channels (lane = channel,
// 8 fp32 states in registers); B_t / C_t are wave-uniform loads. L is split into chunks of Tc steps:
//   fwd pass 1 (per chunk, zero init): end state + sum(dt')      fwd pass 2 (per channel/state): carry over chunks
//   fwd pass 3 (per chunk from the true initial state): y, and x checkpoints every 16 steps for the backward
//   bwd pass A (per chunk): local adjoint aggregate              bwd pass B: reverse carry over chunks
//   bwd pass C (per chunk, reverse 16-step sub-blocks recomputed from the checkpoints in registers):
//       du, d(dt), dA, dD, d(delta_bias), and per-token dB/dC reduced over channels (butterfly + LDS).
#include "common.hpp"

namespace lci {

#ifndef LCI_SCAN_PROBE
#define LCI_SCAN_PROBE 0   // 1: the transcendental-floor timing probe of the forward passes (build_variant only)
#endif
constexpr int SCAN_N = 8;     // d_state (the reference always uses 8: backbone_vit.py:184, backbone_swin.py:329)
constexpr int CKPT = 8;       // backward checkpoint spacing (steps); sub-block states live in registers
constexpr float LOG2E = 1.4426950408889634f;

struct ScanArgs {
  const void* u; const void* delta; const void* Bm; const void* Cm; const void* dy;
  const float* A; const float* D; const float* dbias;
  void* y; void* du; void* ddelta;
  float* xend; float* sdt; float* xinit;                // (B,nch,Dx,N) (B,nch,Dx) (B,nch,Dx,N)
  void* ckpt;                                           // (B,nck,Dx,N) states every CKPT steps, in the I/O dtype
  float* gl; float* gin;                                // (B,nch,Dx,N) x2
  float* dBC;                                           // (B, L, 2N) f32
  float* dA; float* dD; float* ddbias;                  // (Dx,N) (Dx) (Dx), accumulated
  long long bu, bd, bB, bC, by, bdy, bdu, bdd;          // batch strides (elements)
  int tu, td, tB, tC, ty, tdy, tdu, tdd;                // token strides (elements)
  int B, L, Dx, Tc, nch, nck;
  int write_ckpt;
  int softplus;                                         // delta_softplus
  int zero_carry;                                       // one chunk: no carry-in (xinit / gin not read)
  int dbc_plain;                                        // one workgroup per (b, chunk) covers every channel:
                                                        // dBC entries stored, not accumulated (no zero fill)
};

template <typename T> __device__ __forceinline__ float ldf(const T* p) { return (float)(*p); }

// One channel column of a channels-last (B, L, ·) tensor addressed through a buffer resource: the lane's channel
// byte offset is the VGPR offset, the token offset t * stride is a wave-uniform SGPR offset, so per-step loads and
// stores need no 64-bit address VALU. Lanes past Dx get an out-of-range offset: their loads read 0 and their
// stores are dropped by the range check (no exec-mask branches).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
template <typename T>
struct Col {
  rsrc_t r;
  int voff, ts;   // bytes
  // the host checks L * tstride * sizeof(T) < 2^31 (scan_fill)
  __device__ __forceinline__ Col(const void* base, int L, int tstride, int Dx, int d, bool valid) {
    const int bytes = ((L - 1) * tstride + Dx) * (int)sizeof(T);
    r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
    voff = valid ? d * (int)sizeof(T) : 0x7fffffff;
    ts = tstride * (int)sizeof(T);
  }
  __device__ __forceinline__ float ld(int t) const {
    if constexpr (sizeof(T) == 2) {
      const uint32_t v = __builtin_amdgcn_raw_buffer_load_b16(r, voff, t * ts, 0);
      return __uint_as_float(v << 16);
    } else {
      return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, t * ts, 0));
    }
  }
  __device__ __forceinline__ void st(int t, float v) const {
    if constexpr (sizeof(T) == 2) {
      const bf16 h = to_bf16(v);
      __builtin_amdgcn_raw_buffer_store_b16(*(const uint16_t*)&h, r, voff, t * ts, 0);
    } else {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, t * ts, 0);
    }
  }
};

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&v)[SCAN_N]) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 r = *(const bf16x8*)p;
#pragma unroll
    for (int n = 0; n < SCAN_N; ++n) v[n] = (float)r[n];
  } else {
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
    for (int n = 0; n < 4; ++n) { v[n] = a[n]; v[n + 4] = b[n]; }
  }
}

// B/C rows are 16-byte aligned only when the token stride keeps them so; fall back to scalar loads.
template <typename T>
__device__ __forceinline__ void ld8u(const T* p, float (&v)[SCAN_N], bool aligned) {
  if (aligned) { ld8(p, v); return; }
#pragma unroll
  for (int n = 0; n < SCAN_N; ++n) v[n] = (float)p[n];
}

// raw B_t / C_t row (8 values): one 16-B load for bf16, two for f32; converted at use
template <typename T> struct Row8;
template <> struct Row8<bf16> {
  bf16x8 v;
  __device__ __forceinline__ void load(const bf16* p) { v = *(const bf16x8*)p; }
  __device__ __forceinline__ float operator[](int n) const { return (float)v[n]; }
};
template <> struct Row8<float> {
  f32x4 lo, hi;
  __device__ __forceinline__ void load(const float* p) { lo = *(const f32x4*)p; hi = *(const f32x4*)(p + 4); }
  __device__ __forceinline__ float operator[](int n) const { return n < 4 ? lo[n] : hi[n - 4]; }
};

constexpr int PF = 8;         // timesteps whose loads are issued ahead of the dependent recurrence

constexpr float LN2 = 0.6931471805599453f;
// softplus as F.softplus / mamba-ssm's log1pf(expf(v)) with threshold 20, from one v_exp and one v_log;
// below e^-9, log(1 + e) = e to f32 precision (and 1 + e would drop e's low bits)
__device__ __forceinline__ float softplus_fast(float v) {
  const float e = exp2_fast(v * LOG2E);
  const float r = e < 1.2e-4f ? e : __builtin_amdgcn_logf(1.f + e) * LN2;
  return v > 20.f ? v : r;
}
#define softplus(v) (a.softplus ? softplus_fast(v) : (v))

// decay factors exp2(dt * A2[n]) of one step: the 8 exponent arguments as 4 packed f32 multiplies
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void decay8(float dt, const float (&A2)[SCAN_N], float (&e)[SCAN_N]) {
  const f32x2 d2 = {dt, dt};
#pragma unroll
  for (int n = 0; n < SCAN_N; n += 2) {
    const f32x2 t = d2 * f32x2{A2[n], A2[n + 1]};
    e[n] = exp2_fast(t.x);
    e[n + 1] = exp2_fast(t.y);
  }
}

constexpr int SB = 64;        // steps per LDS-staged block of B_t / C_t rows (one row per lane)
constexpr int BCS = 20;       // LDS floats per staged row (B 0..7, C 8..15, pad: 80-B rows)

// Stage the f32 B_t (and C_t) rows of steps tb .. tb+SB-1 into this wave's LDS block, lane i <- step tb+i:
// B/C are wave-uniform per step, so they are converted once here instead of in every lane at every step.
template <typename T, bool WITH_C>
__device__ __forceinline__ void stage_bc(const ScanArgs& a, float* bc, const T* Bp, const T* Cp, int tb, int t1,
                                         int lane) {
  const long long t = min(tb + lane, t1 - 1);
  Row8<T> rb;
  rb.load(Bp + t * a.tB);
  float* dst = bc + lane * BCS;
  *(f32x4*)dst = f32x4{rb[0], rb[1], rb[2], rb[3]};
  *(f32x4*)(dst + 4) = f32x4{rb[4], rb[5], rb[6], rb[7]};
  if constexpr (WITH_C) {
    Row8<T> rc;
    rc.load(Cp + t * a.tC);
    *(f32x4*)(dst + 8) = f32x4{rc[0], rc[1], rc[2], rc[3]};
    *(f32x4*)(dst + 12) = f32x4{rc[4], rc[5], rc[6], rc[7]};
  }
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void lds_row8(const float* p, float (&v)[SCAN_N]) {
  const f32x4 lo = *(const f32x4*)p, hi = *(const f32x4*)(p + 4);
#pragma unroll
  for (int n = 0; n < 4; ++n) { v[n] = lo[n]; v[n + 4] = hi[n]; }
}

// ---------------------------------------------------------------------------------- forward chunk pass
// MODE 0: zero initial state -> xend, sdt. MODE 1: xinit -> y (+ checkpoints).
// PFN: software-pipelined loads. Each group's u / dt loads are issued one group ahead and the next staging
// block's B / C rows one block ahead (held in registers, written to LDS after the block). On gfx950 vmcnt counts
// stores too, so without this the wait for a group's loads also waits for the previous group's y / checkpoint
// stores, and the B / C staging load latency is exposed once per SB steps.
template <typename T, int MODE>
__device__ __forceinline__ void scan_fwd_step(const ScanArgs& a, float (&x)[SCAN_N], const float (&A2)[SCAN_N],
                                              float bias, float Dd, float uv, float drv, const float* row, int t,
                                              bool valid, int d, T* ckb, const Col<T>& ycol, float& sumdt) {
  if (MODE == 1 && a.write_ckpt && ((t & (CKPT - 1)) == 0) && valid) {
    T* cp = (ckb + (long long)(t / CKPT) * a.Dx * SCAN_N) + d * SCAN_N;
    if constexpr (sizeof(T) == 2) {   // bf16 I/O: bf16 checkpoints (one 16-B store; the backward recomputes from them)
      bf16x8 v;
#pragma unroll
      for (int n = 0; n < SCAN_N; ++n) v[n] = to_bf16(x[n]);
      *(bf16x8*)cp = v;
    } else {
      *(f32x4*)cp = f32x4{x[0], x[1], x[2], x[3]};
      *(f32x4*)(cp + 4) = f32x4{x[4], x[5], x[6], x[7]};
    }
  }
#if LCI_SCAN_PROBE
  // transcendental-floor probe (timing only, wrong results): the same loads, softplus and 8 decay exps per
  // channel-step; the state update is one add, the B / C rows, the dtu B product and the C x dot are dropped
  {
    const float dt = softplus(drv + bias);
    float e[SCAN_N];
    decay8(dt, A2, e);
#pragma unroll
    for (int n = 0; n < SCAN_N; ++n) x[n] += e[n];
    (void)row; (void)uv; (void)Dd;
    if (MODE == 1) ycol.st(t, x[0]);
    else sumdt += dt;
    return;
  }
#endif
  float Bv[SCAN_N];
  lds_row8(row, Bv);
  const float dt = softplus(drv + bias);
  const float dtu = dt * uv;
  float e[SCAN_N];
  decay8(dt, A2, e);
#pragma unroll
  for (int n = 0; n < SCAN_N; ++n) x[n] = fmaf(e[n], x[n], dtu * Bv[n]);
  if (MODE == 1) {
    float Cv[SCAN_N];
    lds_row8(row + 8, Cv);
    float y0 = Dd * uv, y1 = 0.f;
#pragma unroll
    for (int n = 0; n < SCAN_N; n += 2) {
      y0 = fmaf(Cv[n], x[n], y0);
      y1 = fmaf(Cv[n + 1], x[n + 1], y1);
    }
    ycol.st(t, y0 + y1);
  } else {
    sumdt += dt;
  }
}

template <typename T, int MODE, bool PFN>
__global__ __launch_bounds__(256) void scan_fwd_kernel(ScanArgs a) {
  __shared__ __attribute__((aligned(16))) float bcl[4][SB * BCS];
  // wave index made provably uniform: chunk / step indices then live in SGPRs (scalar address arithmetic)
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int chunk = blockIdx.x * 4 + wv;
  const int b = blockIdx.z;
  const int d = blockIdx.y * 64 + lane;
  if (chunk >= a.nch) return;
  const bool valid = d < a.Dx;
  const int dd = valid ? d : a.Dx - 1;
  float A2[SCAN_N], x[SCAN_N];
#pragma unroll
  for (int n = 0; n < SCAN_N; ++n) A2[n] = a.A[dd * SCAN_N + n] * LOG2E;
  const float bias = a.dbias ? a.dbias[dd] : 0.f;
  const float Dd = a.D ? a.D[dd] : 0.f;
  const long long sidx = (((long long)b * a.nch + chunk) * a.Dx + dd) * SCAN_N;
#pragma unroll
  for (int n = 0; n < SCAN_N; ++n) x[n] = MODE && !a.zero_carry ? a.xinit[sidx + n] : 0.f;
  // per-step addresses = wave-uniform row base (scalar arithmetic) + this lane's channel offset
  const Col<T> ucol((const T*)a.u + b * a.bu, a.L, a.tu, a.Dx, d, valid);
  const Col<T> dcol((const T*)a.delta + b * a.bd, a.L, a.td, a.Dx, d, valid);
  const Col<T> ycol((T*)a.y + b * a.by, a.L, a.ty, a.Dx, d, valid);
  const T* Bp = (const T*)a.Bm + b * a.bB;
  const T* Cp = (const T*)a.Cm + b * a.bC;
  T* ckb = (T*)a.ckpt + (long long)b * a.nck * a.Dx * SCAN_N;
  float* bc = bcl[wv];
  const int t0 = chunk * a.Tc, t1 = min(a.L, t0 + a.Tc);
  float sumdt = 0.f;
  if constexpr (!PFN) {
    for (int tsb = t0; tsb < t1; tsb += SB) {
      stage_bc<T, MODE == 1>(a, bc, Bp, Cp, tsb, t1, lane);
      const int tse = min(t1, tsb + SB);
      for (int tb = tsb; tb < tse; tb += PF) {
        float uf[PF], dr[PF];
#pragma unroll
        for (int i = 0; i < PF; ++i) {        // the group's u / dt loads first (clamped, branch-free)
          const int t = min(tb + i, tse - 1);
          uf[i] = ucol.ld(t);
          dr[i] = dcol.ld(t);
        }
        const int nvalid = tse - tb;   // >= PF except in a chunk's ragged tail
#pragma unroll
        for (int i = 0; i < PF; ++i)
          if (i < nvalid)
            scan_fwd_step<T, MODE>(a, x, A2, bias, Dd, uf[i], dr[i], bc + (tb + i - tsb) * BCS, tb + i, valid, d,
                                   ckb, ycol, sumdt);
      }
    }
  } else {
    // two register sets for the u / dt groups (even / odd group of the chunk) and one for the next B / C rows
    float ua[PF], da[PF], ub[PF], db[PF];
    auto load_group = [&](int tb, float (&uf)[PF], float (&dr)[PF]) {
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const int t = min(tb + i, t1 - 1);   // clamped, branch-free; past the chunk end the values are unused
        uf[i] = ucol.ld(t);
        dr[i] = dcol.ld(t);
      }
    };
    auto run_group = [&](int tb, int tsb, const float (&uf)[PF], const float (&dr)[PF]) {
      const int nvalid = t1 - tb;
#pragma unroll
      for (int i = 0; i < PF; ++i)
        if (i < nvalid)
          scan_fwd_step<T, MODE>(a, x, A2, bias, Dd, uf[i], dr[i], bc + (tb + i - tsb) * BCS, tb + i, valid, d,
                                 ckb, ycol, sumdt);
    };
    Row8<T> rb, rc;
    auto load_rows = [&](int tsb) {
      const long long t = min(tsb + lane, t1 - 1);
      rb.load(Bp + t * a.tB);
      if constexpr (MODE == 1) rc.load(Cp + t * a.tC);
    };
    auto store_rows = [&]() {
      float* dst = bc + lane * BCS;
      *(f32x4*)dst = f32x4{rb[0], rb[1], rb[2], rb[3]};
      *(f32x4*)(dst + 4) = f32x4{rb[4], rb[5], rb[6], rb[7]};
      if constexpr (MODE == 1) {
        *(f32x4*)(dst + 8) = f32x4{rc[0], rc[1], rc[2], rc[3]};
        *(f32x4*)(dst + 12) = f32x4{rc[4], rc[5], rc[6], rc[7]};
      }
      __builtin_amdgcn_wave_barrier();
    };
    load_rows(t0);
    load_group(t0, ua, da);
    store_rows();
    for (int tsb = t0; tsb < t1; tsb += SB) {
      const int tse = min(t1, tsb + SB);
      if (tse < t1) load_rows(tse);           // next block's rows, written to LDS after this block's steps
      // SB / PF = 8 groups per block (even count): the two register sets alternate without copies
      for (int tb = tsb; tb < tse; tb += 2 * PF) {
        load_group(tb + PF, ub, db);
        run_group(tb, tsb, ua, da);
        if (tb + PF < tse) {
          load_group(tb + 2 * PF, ua, da);
          run_group(tb + PF, tsb, ub, db);
        }
      }
      __builtin_amdgcn_wave_barrier();        // this block's LDS row reads precede the overwrite (wave-local)
      if (tse < t1) store_rows();
    }
  }
  if (MODE == 0 && valid) {
    float* xe = a.xend + sidx;
    *(f32x4*)xe = f32x4{x[0], x[1], x[2], x[3]};
    *(f32x4*)(xe + 4) = f32x4{x[4], x[5], x[6], x[7]};
    a.sdt[((long long)b * a.nch + chunk) * a.Dx + d] = sumdt;
  }
}

// carry over chunks: xinit[c] = carry; carry = exp(A sdt[c]) carry + xend[c]
// REVERSE: gin[c] = carry; carry = gl[c] + exp(A sdt[c]) carry, chunks from last to first.
// One wave per (b, d): lane = (group g, state n), 8 groups of consecutive chunks. Each lane folds its group
// with zero carry-in (the group's decay is exp(A * sum sdt)), the 8 group maps are combined across lanes,
// then each lane replays its group from the true carry-in: 2 * nch/8 sequential steps instead of nch.
template <bool REVERSE>
__global__ __launch_bounds__(64) void scan_carry_kernel(ScanArgs a) {
  const int lane = threadIdx.x, n = lane & 7, g = lane >> 3;
  const int d = blockIdx.x, b = blockIdx.y;
  const float A2 = a.A[d * SCAN_N + n] * LOG2E;
  const float* src = REVERSE ? a.gl : a.xend;
  float* dst = REVERSE ? a.gin : a.xinit;
  const int G = (a.nch + 7) / 8;
  const int k0 = min(a.nch, g * G), k1 = min(a.nch, k0 + G);
  auto cidx = [&](int k) -> long long {
    const int c = REVERSE ? a.nch - 1 - k : k;
    return ((long long)b * a.nch + c) * a.Dx + d;
  };
  float E = 0.f, S = 0.f;
  for (int kb = k0; kb < k1; kb += PF) {
    float sv[PF], ev[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const long long ci = cidx(min(kb + i, k1 - 1));
      sv[i] = a.sdt[ci];
      ev[i] = src[ci * SCAN_N + n];
    }
#pragma unroll
    for (int i = 0; i < PF; ++i)
      if (kb + i < k1) {
        E = fmaf(exp2_fast(A2 * sv[i]), E, ev[i]);
        S += sv[i];
      }
  }
  float carry = 0.f;
#pragma unroll
  for (int gg = 0; gg < 8; ++gg) {
    const float Sg = __shfl(S, gg * 8 + n), Eg = __shfl(E, gg * 8 + n);
    if (gg < g) carry = fmaf(exp2_fast(A2 * Sg), carry, Eg);
  }
  for (int kb = k0; kb < k1; kb += PF) {
    float sv[PF], ev[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const long long ci = cidx(min(kb + i, k1 - 1));
      sv[i] = a.sdt[ci];
      ev[i] = src[ci * SCAN_N + n];
    }
#pragma unroll
    for (int i = 0; i < PF; ++i)
      if (kb + i < k1) {
        dst[cidx(kb + i) * SCAN_N + n] = carry;
        carry = fmaf(exp2_fast(A2 * sv[i]), carry, ev[i]);
      }
  }
}

// ------------------------------------------------------------------------------------- backward pass A
// local adjoint with zero carry-in from later chunks: Gl = a_{t0} g_{t0}
template <typename T>
__global__ __launch_bounds__(256) void scan_bwd_agg_kernel(ScanArgs a) {
  __shared__ __attribute__((aligned(16))) float bcl[4][SB * BCS];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int chunk = blockIdx.x * 4 + wv;
  const int b = blockIdx.z;
  const int d = blockIdx.y * 64 + lane;
  if (chunk >= a.nch) return;
  const bool valid = d < a.Dx;
  const int dd = valid ? d : a.Dx - 1;
  float A2[SCAN_N], g[SCAN_N];
#pragma unroll
  for (int n = 0; n < SCAN_N; ++n) { A2[n] = a.A[dd * SCAN_N + n] * LOG2E; g[n] = 0.f; }
  const float bias = a.dbias ? a.dbias[dd] : 0.f;
  const Col<T> dcol((const T*)a.delta + b * a.bd, a.L, a.td, a.Dx, d, valid);
  const Col<T> gcol((const T*)a.dy + b * a.bdy, a.L, a.tdy, a.Dx, d, valid);
  const T* Cp = (const T*)a.Cm + b * a.bC;
  float* bc = bcl[wv];
  const int t0 = chunk * a.Tc, t1 = min(a.L, t0 + a.Tc);
  // staging blocks of SB steps from the chunk's end; C_t rows go to LDS slots 8..15 (stage_bc's C slot)
  for (int tsb = t0 + ((t1 - 1 - t0) / SB) * SB; tsb >= t0; tsb -= SB) {
    {
      const long long t = min(tsb + lane, t1 - 1);
      Row8<T> rc;
      rc.load(Cp + t * a.tC);
      float* dst = bc + lane * BCS;
      *(f32x4*)(dst + 8) = f32x4{rc[0], rc[1], rc[2], rc[3]};
      *(f32x4*)(dst + 12) = f32x4{rc[4], rc[5], rc[6], rc[7]};
      __builtin_amdgcn_wave_barrier();
    }
    const int tse = min(t1, tsb + SB);
    for (int te = tse - 1; te >= tsb; te -= PF) {
      float dr[PF], gyv[PF];
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        const int t = max(te - i, tsb);
        dr[i] = dcol.ld(t);
        gyv[i] = gcol.ld(t);
      }
#pragma unroll
      for (int i = 0; i < PF; ++i) {
        if (te - i >= tsb) {
          float Cv[SCAN_N];
          lds_row8(bc + (te - i - tsb) * BCS + 8, Cv);
          const float dt = softplus(dr[i] + bias);
          const float gy = valid ? gyv[i] : 0.f;
          float e[SCAN_N];
          decay8(dt, A2, e);
#pragma unroll
          for (int n = 0; n < SCAN_N; ++n) g[n] = e[n] * fmaf(Cv[n], gy, g[n]);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (valid) {
    float* o = a.gl + (((long long)b * a.nch + chunk) * a.Dx + d) * SCAN_N;
    *(f32x4*)o = f32x4{g[0], g[1], g[2], g[3]};
    *(f32x4*)(o + 4) = f32x4{g[4], g[5], g[6], g[7]};
  }
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}

__device__ __forceinline__ float sel_bits(unsigned m, float x, float y) {   // m ? x : y, m all-ones or zero
  return __uint_as_float((__float_as_uint(x) & m) | (__float_as_uint(y) & ~m));
}

// Reduce 16 values over the 64 lanes of a wave (reduce-scatter butterfly); afterwards lane l holds the total of
// value index (l >> 2) & 15 (vb: the 8 dB values, vc: the 8 dC values, as 4 pairs each: dB 0-7, then dC 8-15).
// Levels: lanes l / l^32 by v_permlane32_swap and l / l^16 by v_permlane16_swap (the swap routes each half its kept
// index: one v_pk_add_f32 per value pair, no select), then l / l^8 (DPP row_ror:8) and the half-row mirror (DPP),
// then the quad (DPP quad_perm) -- no LDS round trips.
__device__ __forceinline__ float wave_reduce16p(const f32x2 (&vb)[4], const f32x2 (&vc)[4], int lane) {
  f32x2 w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {   // lanes l / l^32: keep dB (lower half) or dC (upper half) of pair k
    const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(vb[k].x), __float_as_uint(vc[k].x), false, false);
    const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(vb[k].y), __float_as_uint(vc[k].y), false, false);
    w[k] = f32x2{__uint_as_float(rx[0]), __uint_as_float(ry[0])} + f32x2{__uint_as_float(rx[1]), __uint_as_float(ry[1])};
  }
  f32x2 q[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {   // lanes l / l^16: pairs k and k + 2
    const auto rx = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[k].x), __float_as_uint(w[k + 2].x), false, false);
    const auto ry = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[k].y), __float_as_uint(w[k + 2].y), false, false);
    q[k] = f32x2{__uint_as_float(rx[0]), __uint_as_float(ry[0])} + f32x2{__uint_as_float(rx[1]), __uint_as_float(ry[1])};
  }
  // q[0] = values 0, 1 (of this lane's quarter), q[1] = values 2, 3: the rest as wave_reduce16's last levels
  const unsigned up8 = (lane & 8) ? 0xffffffffu : 0u, up4 = (lane & 4) ? 0xffffffffu : 0u;
  const float lo0 = q[0].x + dpp<0x128>(q[0].x), hi0 = q[1].x + dpp<0x128>(q[1].x);
  const float lo1 = q[0].y + dpp<0x128>(q[0].y), hi1 = q[1].y + dpp<0x128>(q[1].y);
  const float v0 = sel_bits(up8, hi0, lo0), v1 = sel_bits(up8, hi1, lo1);
  const float lo = v0 + dpp<0x141>(v0), hi = v1 + dpp<0x141>(v1);
  float r = sel_bits(up4, hi, lo);
  r += dpp<0xB1>(r);
  r += dpp<0x4E>(r);
  return r;
}

// ------------------------------------------------------------------------------------- backward pass C
// Workgroup = one (b, chunk), up to 4 waves cover 256 channels. Sub-blocks of CKPT steps in reverse: the
// sub-block's states x and decays exp(dt A) are recomputed from its checkpoint into registers, then swept back.
// B_t / C_t rows and the per-token dB/dC partial sums go through LDS in blocks of SB steps (two workgroup
// barriers per SB steps); each lane's u / dt / dy / checkpoint loads are issued one sub-block ahead.
// The per-state arithmetic runs on packed pairs of states (f32x2: v_pk_fma_f32 / v_pk_mul_f32, four instructions
// per 8 states and operation; the B_t / C_t rows read from LDS as b128 pairs), the per-step column loads and du /
// d(delta) stores go through buffer resources (wave-uniform token offsets in SGPRs: no 64-bit address VALU), and the
// kernel is held to 256 registers so two waves share each SIMD (round 5: L = 2^21 backward 8.9 -> 6.5 ms,
// profiles/r05_scan_ab.txt).
// PARTIALS: per-(b, chunk) dA / dD / d(delta_bias) partials into the lane's own gin entry (read at the start) and
// its dead gl entry, summed by scan_param_reduce_kernel, instead of B * nch float atomics per address.
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 splat2(float v) { return f32x2{v, v}; }

template <typename T, bool PARTIALS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void scan_bwd_kernel(ScanArgs a) {
  constexpr int NP = SCAN_N / 2;   // state pairs
  __shared__ float red[SB][2 * SCAN_N];
  __shared__ __attribute__((aligned(16))) float bcs[SB][BCS];
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int chunk = blockIdx.x, b = blockIdx.z;
  const int d = blockIdx.y * blockDim.x + wv * 64 + lane;
  const bool valid = d < a.Dx;
  const int dd = valid ? d : a.Dx - 1;
  const bool single = blockDim.x == 64;
  for (int i = tid; i < SB * 2 * SCAN_N; i += blockDim.x) (&red[0][0])[i] = 0.f;
  f32x2 A2[NP], h[NP], dA[NP];
  {
    const float* gi = a.gin + (((long long)b * a.nch + chunk) * a.Dx + dd) * SCAN_N;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      A2[k] = f32x2{a.A[dd * SCAN_N + 2 * k], a.A[dd * SCAN_N + 2 * k + 1]} * LOG2E;
      h[k] = valid && !a.zero_carry ? f32x2{gi[2 * k], gi[2 * k + 1]} : f32x2{0.f, 0.f};
      dA[k] = f32x2{0.f, 0.f};
    }
  }
  const float bias = a.dbias ? a.dbias[dd] : 0.f;
  const float Dd = a.D ? a.D[dd] : 0.f;
  float dDacc = 0.f, dbacc = 0.f;
  const Col<T> ucol((const T*)a.u + b * a.bu, a.L, a.tu, a.Dx, d, valid);
  const Col<T> dcol((const T*)a.delta + b * a.bd, a.L, a.td, a.Dx, d, valid);
  const Col<T> gcol((const T*)a.dy + b * a.bdy, a.L, a.tdy, a.Dx, d, valid);
  const Col<T> ducol((T*)a.du + b * a.bdu, a.L, a.tdu, a.Dx, d, valid);
  const Col<T> ddcol((T*)a.ddelta + b * a.bdd, a.L, a.tdd, a.Dx, d, valid);
  const T* Bp = (const T*)a.Bm + b * a.bB;
  const T* Cp = (const T*)a.Cm + b * a.bC;
  const T* ckb = (const T*)a.ckpt + (long long)b * a.nck * a.Dx * SCAN_N;
  const int t0 = chunk * a.Tc, t1 = min(a.L, t0 + a.Tc);
  const int nsb = (t1 - t0 + CKPT - 1) / CKPT;
  // per-lane operands of one sub-block, loaded a sub-block ahead (invalid lanes read zeros)
  float nck[SCAN_N], nu[CKPT], nd[CKPT], ng[CKPT];
  auto load_lane = [&](int s0) {
    ld8((ckb + (long long)(s0 / CKPT) * a.Dx * SCAN_N) + dd * SCAN_N, nck);
#pragma unroll
    for (int i = 0; i < CKPT; ++i) {
      const int t = min(s0 + i, t1 - 1);
      nu[i] = ucol.ld(t);
      nd[i] = dcol.ld(t);
      ng[i] = gcol.ld(t);
    }
  };
  load_lane(t0 + (nsb - 1) * CKPT);
  int blk0 = -1;   // first step of the staged block
  for (int sb = nsb - 1; sb >= 0; --sb) {
    const int s0 = t0 + sb * CKPT;
    if (blk0 < 0 || s0 < blk0) {   // new staging block [blk0, blk0 + SB) holding s0 (uniform branch)
      if (blk0 >= 0) {             // flush the finished block's dB/dC sums
        __syncthreads();
        for (int k = tid; k < SB * 2 * SCAN_N; k += blockDim.x) {
          const int i = k / (2 * SCAN_N), j = k % (2 * SCAN_N);
          const int t = blk0 + i;
          float* dst = a.dBC + ((long long)b * a.L + t) * (2 * SCAN_N) + j;
          if (t < t1) {
            if (a.dbc_plain) *dst = red[i][j];
            else atomicAdd(dst, red[i][j]);
          }
          red[i][j] = 0.f;
        }
      }
      blk0 = t0 + ((s0 - t0) / SB) * SB;
      if (tid < SB) {
        const long long t = min(blk0 + tid, t1 - 1);
        Row8<T> rb, rc;
        rb.load(Bp + t * a.tB);
        rc.load(Cp + t * a.tC);
        *(f32x4*)&bcs[tid][0] = f32x4{rb[0], rb[1], rb[2], rb[3]};
        *(f32x4*)&bcs[tid][4] = f32x4{rb[4], rb[5], rb[6], rb[7]};
        *(f32x4*)&bcs[tid][8] = f32x4{rc[0], rc[1], rc[2], rc[3]};
        *(f32x4*)&bcs[tid][12] = f32x4{rc[4], rc[5], rc[6], rc[7]};
      }
      __syncthreads();
    }
    f32x2 xck[NP];
    float uf[CKPT], gyv[CKPT], dts[CKPT];
#pragma unroll
    for (int k = 0; k < NP; ++k) xck[k] = f32x2{nck[2 * k], nck[2 * k + 1]};
#pragma unroll
    for (int i = 0; i < CKPT; ++i) {
      uf[i] = nu[i];
      gyv[i] = ng[i];   // 0 on padding lanes (range-checked loads): their dC partials vanish
      dts[i] = softplus(nd[i] + bias);
    }
    if (sb > 0) load_lane(s0 - CKPT);
    const float* rows = &bcs[s0 - blk0][0];
    auto brow = [&](int i, int k) { return *(const f32x2*)(rows + i * BCS + 2 * k); };
    auto crow = [&](int i, int k) { return *(const f32x2*)(rows + i * BCS + SCAN_N + 2 * k); };
    // forward recompute from the checkpoint: xs[i] = x after step s0 + i, at[i] = exp(dt A)
    f32x2 xs[CKPT][NP], at[CKPT][NP];
#pragma unroll
    for (int i = 0; i < CKPT; ++i) {
      const f32x2 dt2 = splat2(dts[i]), dtu2 = splat2(dts[i] * uf[i]);
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const f32x2 arg = dt2 * A2[k];
        at[i][k] = f32x2{exp2_fast(arg.x), exp2_fast(arg.y)};
        xs[i][k] = fma2(at[i][k], i == 0 ? xck[k] : xs[i - 1][k], dtu2 * brow(i, k));
      }
    }
    // reverse sweep
#pragma unroll
    for (int i = CKPT - 1; i >= 0; --i) {
      const int t = s0 + i;
      if (t < t1) {
        const float dt = dts[i], gy = gyv[i], u = uf[i];
        const f32x2 dt2 = splat2(dt), gy2 = splat2(gy), dtu2 = splat2(dt * u);   // u = 0 on padding lanes
        f32x2 sgB2 = {0.f, 0.f}, sA2 = {0.f, 0.f};   // sum_n g_n B_n, sum_n g_n (a_n x_{t-1,n}) A2_n (pairs)
        f32x2 vb[NP], vc[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          const f32x2 gt = fma2(crow(i, k), gy2, h[k]);
          vc[k] = gy2 * xs[i][k];                   // dC_t partial
          vb[k] = gt * dtu2;                        // dB_t partial
          sgB2 = fma2(gt, brow(i, k), sgB2);
          h[k] = at[i][k] * gt;                     // the adjoint carried to step t-1 (= g a)
          // g a x_{t-1}: (g a) x_{t-1} from the recomputed states; at the sub-block's first step x_{t-1} is the
          // checkpoint, no longer live: g (x_t - dt u B)
          const f32x2 gxa = i > 0 ? h[k] * xs[i - 1][k] : gt * fma2(-dtu2, brow(i, k), xs[i][k]);
          sA2 = fma2(gxa, A2[k], sA2);
          dA[k] = fma2(gxa, dt2, dA[k]);
        }
        const float sgB = sgB2.x + sgB2.y, sA = sA2.x + sA2.y;
        const float du = fmaf(dt, sgB, Dd * gy);
        const float ddt = fmaf(u, sgB, sA * LN2);
        // d softplus / dx = sigmoid(x) = 1 - exp(-softplus(x))  (1 above the threshold 20)
        const float sg = a.softplus ? 1.f - exp2_fast(-dt * LOG2E) : 1.f;
        const float ddl = ddt * sg;
        dDacc = fmaf(gy, u, dDacc);
        dbacc += ddl;
        ducol.st(t, du);
        ddcol.st(t, ddl);
        const float r = wave_reduce16p(vb, vc, lane);
        if ((lane & 3) == 0) {   // one wave per workgroup: the only writer of its (t, j) entry
          if (single) red[t - blk0][lane >> 2] = r;
          else atomicAdd(&red[t - blk0][lane >> 2], r);
        }
      }
    }
  }
  __syncthreads();
  for (int k = tid; k < SB * 2 * SCAN_N; k += blockDim.x) {
    const int i = k / (2 * SCAN_N), j = k % (2 * SCAN_N);
    const int t = blk0 + i;
    float* dst = a.dBC + ((long long)b * a.L + t) * (2 * SCAN_N) + j;
    if (t < t1) {
      if (a.dbc_plain) *dst = red[i][j];
      else atomicAdd(dst, red[i][j]);
    }
  }
  if constexpr (PARTIALS) {
    if (!valid) return;
    const long long o = (((long long)b * a.nch + chunk) * a.Dx + d) * SCAN_N;
    *(f32x4*)(a.gin + o) = f32x4{dA[0].x, dA[0].y, dA[1].x, dA[1].y};
    *(f32x4*)(a.gin + o + 4) = f32x4{dA[2].x, dA[2].y, dA[3].x, dA[3].y};
    a.gl[o] = dDacc;
    a.gl[o + 1] = dbacc;
  } else if (valid) {
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      atomicAdd(a.dA + d * SCAN_N + 2 * k, dA[k].x);
      atomicAdd(a.dA + d * SCAN_N + 2 * k + 1, dA[k].y);
    }
    atomicAdd(a.dD + d, dDacc);
    atomicAdd(a.ddbias + d, dbacc);
  }
}

// Sum of the per-(b, chunk) parameter-gradient partials: thread = (channel d, value q) with q < 8 the dA states and
// q = 8 / 9 dD / d(delta_bias); blockIdx.y takes a stride-gridDim.y subset of the (b, chunk) rows, one atomic per
// thread at the end (gridDim.y atomics per address instead of B * nch from the scan kernel's waves).
constexpr int SCAN_NP = SCAN_N + 2;
__global__ __launch_bounds__(256) void scan_param_reduce_kernel(ScanArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= a.Dx * SCAN_NP) return;
  const int d = i / SCAN_NP, q = i % SCAN_NP;
  const float* src = q < SCAN_N ? a.gin + q : a.gl + (q - SCAN_N);
  const int rows = a.B * a.nch;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int r = blockIdx.y;
  const int st = gridDim.y;
  for (; r + 3 * st < rows; r += 4 * st) {
    s0 += src[((long long)r * a.Dx + d) * SCAN_N];
    s1 += src[((long long)(r + st) * a.Dx + d) * SCAN_N];
    s2 += src[((long long)(r + 2 * st) * a.Dx + d) * SCAN_N];
    s3 += src[((long long)(r + 3 * st) * a.Dx + d) * SCAN_N];
  }
  for (; r < rows; r += st) s0 += src[((long long)r * a.Dx + d) * SCAN_N];
  float* dst = q < SCAN_N ? a.dA + d * SCAN_N + q : (q == SCAN_N ? a.dD + d : a.ddbias + d);
  atomicAdd(dst, (s0 + s1) + (s2 + s3));
}

// ------------------------------------------------------------------------------ depthwise conv + SiLU
// in (B, L, 2C) (x | z halves, channels-last), w (C, 3) x2, 'same' padding (1 left, 1 right).
// out_x (B, L, C) and out_z written at column offset zoff of a (B, L, oz_ts) buffer.
// A thread owns one channel of the 2C and a run of CONV_T tokens (lanes = consecutive channels: coalesced
// rows); the 3-tap window slides in registers, weight-gradient partials stay in registers until one atomic.
constexpr int CONV_K = 3;
constexpr int CONV_T = 256;

struct ConvArgs {
  const void* in; const float* wx; const float* bx; const float* wz; const float* bz;
  void* ox; void* oz;
  const void* gx; const void* gz;   // bwd: grads of the SiLU outputs
  void* din;                        // bwd: (B, L, 2C)
  float* part;                      // bwd: (B * ceil(L / CONV_T), 2C, 4) f32 per-run sums of (dw0, dw1, dw2, db)
  int B, L, C, in_ts, ox_ts, oz_ts, zoff;
};

template <typename T>
__global__ __launch_bounds__(256) void dwconv_silu_fwd_kernel(ConvArgs a) {
  const int cc = blockIdx.x * 256 + threadIdx.x;
  if (cc >= 2 * a.C) return;
  const int b = blockIdx.z, t0 = blockIdx.y * CONV_T, t1 = min(a.L, t0 + CONV_T);
  const int half = cc / a.C, c = cc % a.C;
  const float* w = (half ? a.wz : a.wx) + c * CONV_K;
  const float* bp = half ? a.bz : a.bx;
  const float w0 = w[0], w1 = w[1], w2 = w[2], bias = bp ? bp[c] : 0.f;
  const T* in = (const T*)a.in + (long long)b * a.L * a.in_ts + cc;
  auto X = [&](int s) -> float { return (s >= 0 && s < a.L) ? (float)in[(long long)s * a.in_ts] : 0.f; };
  float xm = X(t0 - 1), x0 = X(t0);
  for (int t = t0; t < t1; ++t) {
    const float xp = X(t + 1);
    const float pre = fmaf(w0, xm, fmaf(w1, x0, fmaf(w2, xp, bias)));
    const float sv = pre / (1.f + __expf(-pre));
    if (half == 0) ((T*)a.ox)[((long long)b * a.L + t) * a.ox_ts + c] = (T)sv;
    else ((T*)a.oz)[((long long)b * a.L + t) * a.oz_ts + a.zoff + c] = (T)sv;
    xm = x0; x0 = xp;
  }
}

// g(s) = dout(s) * silu'(pre(s)); din(t) = w0 g(t+1) + w1 g(t) + w2 g(t-1); dw[j] += g(t) x(t+j-1)
template <typename T>
__global__ __launch_bounds__(256) void dwconv_silu_bwd_kernel(ConvArgs a) {
  const int cc = blockIdx.x * 256 + threadIdx.x;
  if (cc >= 2 * a.C) return;
  const int b = blockIdx.z, t0 = blockIdx.y * CONV_T, t1 = min(a.L, t0 + CONV_T);
  const int half = cc / a.C, c = cc % a.C;
  const float* w = (half ? a.wz : a.wx) + c * CONV_K;
  const float* bp = half ? a.bz : a.bx;
  const float w0 = w[0], w1 = w[1], w2 = w[2], bias = bp ? bp[c] : 0.f;
  const T* in = (const T*)a.in + (long long)b * a.L * a.in_ts + cc;
  const T* go = half ? (const T*)a.gz + (long long)b * a.L * a.oz_ts + a.zoff + c
                     : (const T*)a.gx + (long long)b * a.L * a.ox_ts + c;
  const int gts = half ? a.oz_ts : a.ox_ts;
  auto X = [&](int s) -> float { return (s >= 0 && s < a.L) ? (float)in[(long long)s * a.in_ts] : 0.f; };
  auto G = [&](int s, float xm, float x0, float xp) -> float {
    if (s < 0 || s >= a.L) return 0.f;
    const float pre = fmaf(w0, xm, fmaf(w1, x0, fmaf(w2, xp, bias)));
    const float sg = 1.f / (1.f + __expf(-pre));
    return (float)go[(long long)s * gts] * sg * fmaf(pre, 1.f - sg, 1.f);
  };
  // window over x: x(t-2) .. x(t+2); g(t-1), g(t), g(t+1)
  float xa = X(t0 - 2), xb = X(t0 - 1), xc = X(t0), xd = X(t0 + 1);
  float gm = G(t0 - 1, xa, xb, xc), g0 = G(t0, xb, xc, xd);
  float dw0 = 0.f, dw1 = 0.f, dw2 = 0.f, db = 0.f;
  T* din = (T*)a.din + (long long)b * a.L * a.in_ts + cc;
  for (int t = t0; t < t1; ++t) {
    const float xe = X(t + 2);
    const float gp = G(t + 1, xc, xd, xe);
    din[(long long)t * a.in_ts] = (T)fmaf(w0, gp, fmaf(w1, g0, w2 * gm));
    dw0 = fmaf(g0, xb, dw0);
    dw1 = fmaf(g0, xc, dw1);
    dw2 = fmaf(g0, xd, dw2);
    db += g0;
    xa = xb; xb = xc; xc = xd; xd = xe;
    gm = g0; g0 = gp;
  }
  const int nrun = (a.L + CONV_T - 1) / CONV_T;
  float* pp = a.part + (((long long)b * nrun + blockIdx.y) * 2 * a.C + cc) * 4;
  *(f32x4*)pp = f32x4{dw0, dw1, dw2, db};
}

// ---------------------------------------------------------------- depthwise conv + SiLU, 16-byte vector path
// A thread owns V = 16 / sizeof(T) adjacent channels (one 16-byte vector of a token row; never straddling the x / z
// halves since C % V == 0) and a run of CONV_T tokens; adjacent threads take adjacent vectors, so a wave's row
// accesses are 16 bytes per lane instead of 2. Rows are loaded CONV_U tokens ahead of their use.
constexpr int CONV_U = 4;

// V channels of one token row as a T vector of V lanes (16 B: 8 bf16 / 4 f32; 8 B: 4 bf16)
template <typename T, int V>
struct VecN {
  typedef T raw __attribute__((ext_vector_type(V)));
  static __device__ __forceinline__ void unpack(const raw& r, float (&f)[V]) {
#pragma unroll
    for (int i = 0; i < V; ++i) f[i] = (float)r[i];
  }
  static __device__ __forceinline__ raw pack(const float (&f)[V]) {
    raw r;
#pragma unroll
    for (int i = 0; i < V; ++i) r[i] = (T)f[i];
    return r;
  }
};

template <typename T, int V, int TR = CONV_T>
struct ConvVecCtx {
  typedef typename VecN<T, V>::raw raw;
  int b, t0, t1, c, cc0;
  bool zhalf, ok;
  __device__ __forceinline__ ConvVecCtx(const ConvArgs& a) {
    const int G = 2 * a.C / V;                      // vectors per token row
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int run = (int)(idx / G), g = (int)(idx % G);
    const int nrun = (a.L + TR - 1) / TR;
    b = blockIdx.z;
    ok = run < nrun;
    t0 = run * TR;
    t1 = min(a.L, t0 + TR);
    cc0 = g * V;
    zhalf = cc0 >= a.C;
    c = zhalf ? cc0 - a.C : cc0;
  }
  // row s of the conv input (zero outside [0, L)), clamped address + select: no divergent loads
  __device__ __forceinline__ raw in_row(const ConvArgs& a, int s) const {
    const int sc = min(max(s, 0), a.L - 1);
    const raw r = *(const raw*)((const T*)a.in + ((long long)b * a.L + sc) * a.in_ts + cc0);
    return (s >= 0 && s < a.L) ? r : raw{};
  }
};

template <typename T, int V>
__global__ __launch_bounds__(256) void dwconv_silu_fwd_vec_kernel(ConvArgs a) {
  const ConvVecCtx<T, V> ctx(a);
  typedef VecN<T, V> Vec;
  typedef typename Vec::raw raw;
  if (!ctx.ok) return;
  const float* w = (ctx.zhalf ? a.wz : a.wx) + ctx.c * CONV_K;
  const float* bp = ctx.zhalf ? a.bz : a.bx;
  float w0[V], w1[V], w2[V], bias[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    w0[v] = w[v * CONV_K]; w1[v] = w[v * CONV_K + 1]; w2[v] = w[v * CONV_K + 2];
    bias[v] = bp ? bp[ctx.c + v] : 0.f;
  }
  T* op = ctx.zhalf ? (T*)a.oz + (long long)ctx.b * a.L * a.oz_ts + a.zoff + ctx.c
                    : (T*)a.ox + (long long)ctx.b * a.L * a.ox_ts + ctx.c;
  const int ots = ctx.zhalf ? a.oz_ts : a.ox_ts;
  float xm[V], x0[V];
  Vec::unpack(ctx.in_row(a, ctx.t0 - 1), xm);
  Vec::unpack(ctx.in_row(a, ctx.t0), x0);
  for (int tb = ctx.t0; tb < ctx.t1; tb += CONV_U) {
    raw nx[CONV_U];
#pragma unroll
    for (int u = 0; u < CONV_U; ++u) nx[u] = ctx.in_row(a, tb + 1 + u);
#pragma unroll
    for (int u = 0; u < CONV_U; ++u) {
      float xp[V], y[V];
      Vec::unpack(nx[u], xp);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float pre = fmaf(w0[v], xm[v], fmaf(w1[v], x0[v], fmaf(w2[v], xp[v], bias[v])));
        y[v] = pre / (1.f + __expf(-pre));
        xm[v] = x0[v]; x0[v] = xp[v];
      }
      if (tb + u < ctx.t1) *(raw*)(op + (long long)(tb + u) * ots) = Vec::pack(y);
    }
  }
}

// Weight / bias gradients: every (sequence, run of CONV_T tokens, channel) writes its (dw0, dw1, dw2, db) partial
// sums to a workspace the caller reduces (deterministic). The float atomics this replaced were serialised by the L2
// per address: at the Swin-window shapes (8192 sequences of 64 tokens) 2 * 10^5 threads x 16 atomics onto 384
// addresses took 0.5 ms per call, and they had forced 1024-token runs (a short grid) at long L.
constexpr int CONV_TB = CONV_T;

template <typename T, int V>
__global__ __launch_bounds__(256) void dwconv_silu_bwd_vec_kernel(ConvArgs a) {
  const ConvVecCtx<T, V, CONV_TB> ctx(a);
  typedef VecN<T, V> Vec;
  typedef typename Vec::raw raw;
  if (!ctx.ok) return;
  const float* w = (ctx.zhalf ? a.wz : a.wx) + ctx.c * CONV_K;
  const float* bp = ctx.zhalf ? a.bz : a.bx;
  float w0[V], w1[V], w2[V], bias[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    w0[v] = w[v * CONV_K]; w1[v] = w[v * CONV_K + 1]; w2[v] = w[v * CONV_K + 2];
    bias[v] = bp ? bp[ctx.c + v] : 0.f;
  }
  const T* go = ctx.zhalf ? (const T*)a.gz + (long long)ctx.b * a.L * a.oz_ts + a.zoff + ctx.c
                          : (const T*)a.gx + (long long)ctx.b * a.L * a.ox_ts + ctx.c;
  const int gts = ctx.zhalf ? a.oz_ts : a.ox_ts;
  auto go_row = [&](int s) -> raw {
    const int sc = min(max(s, 0), a.L - 1);
    const raw r = *(const raw*)(go + (long long)sc * gts);
    return (s >= 0 && s < a.L) ? r : raw{};
  };
  // g(s) = dout(s) silu'(pre(s)) from x(s-1..s+1); zero outside [0, L) (dout row is zero there)
  auto G = [&](const float (&xm)[V], const float (&x0)[V], const float (&xp)[V], const raw& gr, float (&g)[V]) {
    float gf[V];
    Vec::unpack(gr, gf);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float pre = fmaf(w0[v], xm[v], fmaf(w1[v], x0[v], fmaf(w2[v], xp[v], bias[v])));
      const float sg = 1.f / (1.f + __expf(-pre));
      g[v] = gf[v] * sg * fmaf(pre, 1.f - sg, 1.f);
    }
  };
  const int t0 = ctx.t0;
  float xa[V], xb[V], xc[V], xd[V], gm[V], g0[V];
  Vec::unpack(ctx.in_row(a, t0 - 2), xa);
  Vec::unpack(ctx.in_row(a, t0 - 1), xb);
  Vec::unpack(ctx.in_row(a, t0), xc);
  Vec::unpack(ctx.in_row(a, t0 + 1), xd);
  G(xa, xb, xc, go_row(t0 - 1), gm);
  G(xb, xc, xd, go_row(t0), g0);
  float dw0[V], dw1[V], dw2[V], db[V];
#pragma unroll
  for (int v = 0; v < V; ++v) { dw0[v] = 0.f; dw1[v] = 0.f; dw2[v] = 0.f; db[v] = 0.f; }
  T* din = (T*)a.din + (long long)ctx.b * a.L * a.in_ts + ctx.cc0;
  for (int tb = t0; tb < ctx.t1; tb += CONV_U) {
    raw nx[CONV_U], ng[CONV_U];
#pragma unroll
    for (int u = 0; u < CONV_U; ++u) {
      nx[u] = ctx.in_row(a, tb + 2 + u);
      ng[u] = go_row(tb + 1 + u);
    }
#pragma unroll
    for (int u = 0; u < CONV_U; ++u) {
      const int t = tb + u;
      if (t < ctx.t1) {
        float xe[V], gp[V], o[V];
        Vec::unpack(nx[u], xe);
        G(xc, xd, xe, ng[u], gp);
#pragma unroll
        for (int v = 0; v < V; ++v) {
          o[v] = fmaf(w0[v], gp[v], fmaf(w1[v], g0[v], w2[v] * gm[v]));
          dw0[v] = fmaf(g0[v], xb[v], dw0[v]);
          dw1[v] = fmaf(g0[v], xc[v], dw1[v]);
          dw2[v] = fmaf(g0[v], xd[v], dw2[v]);
          db[v] += g0[v];
          xa[v] = xb[v]; xb[v] = xc[v]; xc[v] = xd[v]; xd[v] = xe[v];
          gm[v] = g0[v]; g0[v] = gp[v];
        }
        *(raw*)(din + (long long)t * a.in_ts) = Vec::pack(o);
      }
    }
  }
  const int nrun = (a.L + CONV_TB - 1) / CONV_TB;
  float* pp = a.part + (((long long)ctx.b * nrun + ctx.t0 / CONV_TB) * 2 * a.C + ctx.cc0) * 4;
#pragma unroll
  for (int v = 0; v < V; ++v) *(f32x4*)(pp + 4 * v) = f32x4{dw0[v], dw1[v], dw2[v], db[v]};
}

}  // namespace lci

using namespace lci;

static int scan_fill(ScanArgs& a, int B, int L, int Dx, int N, int Tc) {
  LCI_CHECK(N == SCAN_N, "selective_scan: d_state %d unsupported (8)", N);
  LCI_CHECK(B > 0 && L > 0 && Dx > 0 && Dx <= 1024, "selective_scan: bad shape B=%d L=%d Dx=%d", B, L, Dx);
  LCI_CHECK(Tc % CKPT == 0 && Tc > 0, "selective_scan: chunk %d must be a multiple of %d", Tc, CKPT);
  a.B = B; a.L = L; a.Dx = Dx; a.Tc = Tc;
  a.nch = (L + Tc - 1) / Tc; a.nck = (L + CKPT - 1) / CKPT;
  return 0;
}

// strides: array of 16 long long: [bu,tu, bd,td, bB,tB, bC,tC, by,ty, bdy,tdy, bdu,tdu, bdd,tdd] (elements)
static int scan_check_bc(const void* Bm, const void* Cm, long long tB, long long tC, int dtype) {
  const long long es = dtype == 1 ? 2 : 4;
  LCI_CHECK(((uintptr_t)Bm) % 16 == 0 && ((uintptr_t)Cm) % 16 == 0 && (tB * es) % 16 == 0 && (tC * es) % 16 == 0,
            "selective_scan: B/C rows must be 16-byte aligned");
  return 0;
}

static int scan_strides(ScanArgs& a, const long long* s, int dtype) {
  a.bu = s[0]; a.tu = (int)s[1]; a.bd = s[2]; a.td = (int)s[3]; a.bB = s[4]; a.tB = (int)s[5];
  a.bC = s[6]; a.tC = (int)s[7]; a.by = s[8]; a.ty = (int)s[9]; a.bdy = s[10]; a.tdy = (int)s[11];
  a.bdu = s[12]; a.tdu = (int)s[13]; a.bdd = s[14]; a.tdd = (int)s[15];
  // per-sample column tensors are addressed with 32-bit buffer offsets (Col): (L + 1) rows of token stride
  for (int i = 1; i < 16; i += 2)
    LCI_CHECK((long long)(a.L + 1) * s[i] * (dtype == 1 ? 2 : 4) < (1ll << 31),
              "selective_scan: L=%d x token stride %lld too large for 32-bit buffer offsets", a.L, s[i]);
  return 0;
}

// Workspace (f32): xend, xinit (B*nch*Dx*N each), sdt (B*nch*Dx); ckpt (B*nck*Dx*N, the I/O dtype) if not null.
// With one chunk (L <= chunk: the Swin recipes' window sequences) xend / xinit / sdt may be null: the zero-init
// end-state pass and the carry are then skipped (nothing is carried into the only chunk) and only the output
// pass runs; the final state is not produced.
extern "C" int lci_selective_scan_fwd(int dtype, const void* u, const void* delta, const float* A, const void* Bm,
                                      const void* Cm, const float* D, const float* delta_bias, void* y,
                                      const long long* strides, int B, int L, int Dx, int N, int chunk,
                                      int delta_softplus, float* xend, float* xinit, float* sdt, void* ckpt,
                                      void* stream) {
  ScanArgs a{};
  if (scan_fill(a, B, L, Dx, N, chunk)) return 1;
  a.softplus = delta_softplus;
  if (scan_strides(a, strides, dtype)) return 1;
  if (scan_check_bc(Bm, Cm, strides[5], strides[7], dtype)) return 1;
  a.u = u; a.delta = delta; a.A = A; a.Bm = Bm; a.Cm = Cm; a.D = D; a.dbias = delta_bias; a.y = y;
  a.xend = xend; a.xinit = xinit; a.sdt = sdt; a.ckpt = ckpt; a.write_ckpt = ckpt != nullptr;
  const bool one = !xend || !xinit || !sdt;
  LCI_CHECK(!one || (!xend && !xinit && !sdt && a.nch == 1),
            "selective_scan_fwd: null end-state workspaces only with one chunk (L=%d, chunk %d)", L, chunk);
  a.zero_carry = one;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((a.nch + 3) / 4, (Dx + 63) / 64, B);
  // LCI_SCAN_PF=0: the forward passes without the software-pipelined loads (A/B hook)
  static const bool pf = !getenv("LCI_SCAN_PF") || atoi(getenv("LCI_SCAN_PF")) != 0;
  auto chunk_pass = [&](auto mode) {
    constexpr int M = decltype(mode)::value;
    if (dtype == 1) {
      if (pf) hipLaunchKernelGGL((scan_fwd_kernel<bf16, M, true>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((scan_fwd_kernel<bf16, M, false>), grid, dim3(256), 0, s, a);
    } else {
      if (pf) hipLaunchKernelGGL((scan_fwd_kernel<float, M, true>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((scan_fwd_kernel<float, M, false>), grid, dim3(256), 0, s, a);
    }
  };
  if (!one) {
    chunk_pass(std::integral_constant<int, 0>{});
    LCI_LAUNCH_CHECK();
    hipLaunchKernelGGL(scan_carry_kernel<false>, dim3(Dx, B), dim3(64), 0, s, a);
    LCI_LAUNCH_CHECK();
  }
  chunk_pass(std::integral_constant<int, 1>{});
  LCI_LAUNCH_CHECK();
  return 0;
}

static int scan_bwd_waves(int Tc, int Dx) {
  static const int wenv = getenv("LCI_SCAN_BWD_WAVES") ? atoi(getenv("LCI_SCAN_BWD_WAVES")) : 0;
  const int wmax = wenv > 0 ? wenv : (Tc >= 512 ? 1 : 4);
  return std::max(1, std::min(std::min(wmax, 4), (Dx + 63) / 64));
}

// 1: lci_selective_scan_bwd stores every dBC entry exactly once at this shape (one workgroup per (b, chunk) holds
// all Dx channels), so dBC needs no zero fill; 0: it accumulates into dBC with atomics.
extern "C" int lci_selective_scan_bwd_plain_dbc(int L, int Dx, int chunk) {
  (void)L;
  static const bool off = getenv("LCI_SCAN_PLAIN_DBC") && atoi(getenv("LCI_SCAN_PLAIN_DBC")) == 0;   // A/B hook
  const int nwv = scan_bwd_waves(chunk, Dx);
  return !off && (Dx + nwv * 64 - 1) / (nwv * 64) == 1;
}

// dA (Dx*N), dD (Dx), ddelta_bias (Dx) are accumulated (caller zeroes them); dBC (B, L, 2N) too, except where
// lci_selective_scan_bwd_plain_dbc says every entry is stored once (no zero fill needed).
// Workspace: gl, gin (B*nch*Dx*N each); sdt and ckpt from the forward (same chunk). sdt null (one chunk, the
// forward ran without end states): the adjoint aggregate and the reverse carry are skipped.
extern "C" int lci_selective_scan_bwd(int dtype, const void* u, const void* delta, const float* A, const void* Bm,
                                      const void* Cm, const float* D, const float* delta_bias, const void* dy,
                                      void* du, void* ddelta, float* dBC, float* dA, float* dD, float* ddelta_bias,
                                      const long long* strides, int B, int L, int Dx, int N, int chunk,
                                      int delta_softplus, const float* sdt, const void* ckpt, float* gl, float* gin,
                                      void* stream) {
  ScanArgs a{};
  if (scan_fill(a, B, L, Dx, N, chunk)) return 1;
  a.softplus = delta_softplus;
  if (scan_strides(a, strides, dtype)) return 1;
  if (scan_check_bc(Bm, Cm, strides[5], strides[7], dtype)) return 1;
  a.u = u; a.delta = delta; a.A = A; a.Bm = Bm; a.Cm = Cm; a.D = D; a.dbias = delta_bias; a.dy = dy;
  a.du = du; a.ddelta = ddelta; a.dBC = dBC; a.dA = dA; a.dD = dD; a.ddbias = ddelta_bias;
  a.sdt = (float*)sdt; a.ckpt = const_cast<void*>(ckpt); a.gl = gl; a.gin = gin;
  LCI_CHECK(sdt || a.nch == 1, "selective_scan_bwd: sdt is null with %d chunks", a.nch);
  a.zero_carry = sdt == nullptr;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((a.nch + 3) / 4, (Dx + 63) / 64, B);
  if (!a.zero_carry) {
    if (dtype == 1) hipLaunchKernelGGL((scan_bwd_agg_kernel<bf16>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((scan_bwd_agg_kernel<float>), grid, dim3(256), 0, s, a);
    LCI_LAUNCH_CHECK();
    hipLaunchKernelGGL(scan_carry_kernel<true>, dim3(Dx, B), dim3(64), 0, s, a);
    LCI_LAUNCH_CHECK();
  }
  // waves per workgroup (channel blocks of 64 sharing one chunk's B/C staging and dB/dC sums): at 254 VGPRs
  // (2 waves per SIMD) 3-wave groups leave 2 of a CU's 8 wave slots empty and two SIMDs with one wave each, so
  // long chunks run one wave per workgroup (L=2^21: 7.8 -> 6.6 ms); short chunks keep the shared staging, whose
  // per-token dB/dC flush (one set of global atomics per workgroup and token) dominates there (L=65536, Tc=64:
  // 0.60 ms at 4 waves vs 0.80 at 1). LCI_SCAN_BWD_WAVES overrides.
  const int nwv = scan_bwd_waves(a.Tc, Dx);
  dim3 gridc(a.nch, (Dx + nwv * 64 - 1) / (nwv * 64), B);
  a.dbc_plain = lci_selective_scan_bwd_plain_dbc(L, Dx, a.Tc);
  // parameter gradients: the B * nch float atomics per address from the waves' ends serialise in L2 (the dwconv
  // backward's lesson): short chunks write partials and sum them in one more launch (L=65536: 0.60 -> 0.42 ms).
  // Long chunks keep the atomics: there the partials build of the kernel measured slower (8.6 vs 6.9 ms at L=2^21,
  // a main-loop schedule change at 256 VGPRs). LCI_SCAN_PARAM_PARTIALS = 0 / 1 overrides.
  static const int penv = getenv("LCI_SCAN_PARAM_PARTIALS") ? atoi(getenv("LCI_SCAN_PARAM_PARTIALS")) : -1;
  const bool partials = penv >= 0 ? penv != 0 : a.Tc < 512;
  if (partials) {
    if (dtype == 1) hipLaunchKernelGGL((scan_bwd_kernel<bf16, true>), gridc, dim3(nwv * 64), 0, s, a);
    else hipLaunchKernelGGL((scan_bwd_kernel<float, true>), gridc, dim3(nwv * 64), 0, s, a);
  } else {
    if (dtype == 1) hipLaunchKernelGGL((scan_bwd_kernel<bf16, false>), gridc, dim3(nwv * 64), 0, s, a);
    else hipLaunchKernelGGL((scan_bwd_kernel<float, false>), gridc, dim3(nwv * 64), 0, s, a);
  }
  LCI_LAUNCH_CHECK();
  if (partials) {
    const int ny = std::max(1, std::min(64, (B * a.nch) / 16));
    hipLaunchKernelGGL(scan_param_reduce_kernel, dim3((Dx * SCAN_NP + 255) / 256, ny), dim3(256), 0, s, a);
    LCI_LAUNCH_CHECK();
  }
  return 0;
}

// The 16-byte vector kernels need C a multiple of the vector width and 16-byte aligned rows of every operand;
// LCI_DWCONV_VEC=0 forces the scalar kernels (A/B hook).
static bool dwconv_vec_ok(int dtype, int V, int C, const void* const* ptrs, int np, const int* tss, int nts,
                          int zoff) {
  static const bool on = !getenv("LCI_DWCONV_VEC") || atoi(getenv("LCI_DWCONV_VEC")) != 0;
  const int vb = V * (dtype == 1 ? 2 : 4);   // vector bytes
  if (!on || C % V || zoff % V) return false;
  for (int i = 0; i < np; ++i)
    if (ptrs[i] && ((uintptr_t)ptrs[i] % vb)) return false;
  for (int i = 0; i < nts; ++i)
    if (tss[i] % V) return false;
  return true;
}

static dim3 dwconv_vec_grid(int V, int B, int L, int C, int TR = CONV_T) {
  const long long threads = (long long)((L + TR - 1) / TR) * (2 * C / V);
  return dim3((unsigned)((threads + 255) / 256), 1, B);
}

extern "C" int lci_dwconv_silu_fwd(int dtype, const void* in, const float* wx, const float* bx, const float* wz,
                                   const float* bz, void* ox, void* oz, int B, int L, int C, int K, int in_ts,
                                   int ox_ts, int oz_ts, int zoff, void* stream) {
  LCI_CHECK(K == CONV_K, "dwconv_silu: kernel size %d unsupported (3, as mamba.py d_conv=3)", K);
  ConvArgs a{};
  a.in = in; a.wx = wx; a.bx = bx; a.wz = wz; a.bz = bz; a.ox = ox; a.oz = oz;
  a.B = B; a.L = L; a.C = C; a.in_ts = in_ts; a.ox_ts = ox_ts; a.oz_ts = oz_ts; a.zoff = zoff;
  const void* vp[] = {in, ox, oz};
  const int vt[] = {in_ts, ox_ts, oz_ts};
  if (dwconv_vec_ok(dtype, dtype == 1 ? 8 : 4, C, vp, 3, vt, 3, zoff)) {
    const dim3 gv = dwconv_vec_grid(dtype == 1 ? 8 : 4, B, L, C);
    if (dtype == 1) hipLaunchKernelGGL((dwconv_silu_fwd_vec_kernel<bf16, 8>), gv, dim3(256), 0, (hipStream_t)stream, a);
    else hipLaunchKernelGGL((dwconv_silu_fwd_vec_kernel<float, 4>), gv, dim3(256), 0, (hipStream_t)stream, a);
    LCI_LAUNCH_CHECK();
    return 0;
  }
  dim3 grid((2 * C + 255) / 256, (L + CONV_T - 1) / CONV_T, B);
  if (dtype == 1) hipLaunchKernelGGL(dwconv_silu_fwd_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(dwconv_silu_fwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}

extern "C" long long lci_dwconv_silu_bwd_part_rows(int B, int L) {
  return (long long)B * ((L + CONV_T - 1) / CONV_T);
}

// din (B, L, 2C) written with token stride in_ts; part (lci_dwconv_silu_bwd_part_rows(B, L), 2C, 4) f32 written:
// per-run sums of (dw0, dw1, dw2, db) of channel cc (x half: cc < C), summed over the first axis by the caller.
extern "C" int lci_dwconv_silu_bwd(int dtype, const void* in, const float* wx, const float* bx, const float* wz,
                                   const float* bz, const void* gx, const void* gz, void* din, float* part, int B,
                                   int L, int C, int K, int in_ts, int ox_ts, int oz_ts, int zoff, void* stream) {
  LCI_CHECK(K == CONV_K, "dwconv_silu: kernel size %d unsupported (3, as mamba.py d_conv=3)", K);
  LCI_CHECK(part && ((uintptr_t)part & 15) == 0, "dwconv_silu: part workspace must be 16-byte aligned");
  ConvArgs a{};
  a.in = in; a.wx = wx; a.bx = bx; a.wz = wz; a.bz = bz; a.gx = gx; a.gz = gz; a.din = din;
  a.part = part;
  a.B = B; a.L = L; a.C = C; a.in_ts = in_ts; a.ox_ts = ox_ts; a.oz_ts = oz_ts; a.zoff = zoff;
  // backward: 4 channels per thread (8-byte bf16 / 16-byte f32 vectors). The 8-channel bf16 version holds 16
  // windows' state in 182 VGPRs (2 waves per SIMD) and measured slower than the scalar kernels (3.5 vs 2.6 ms at
  // B=1, L=2^21, 2C=384). LCI_DWCONV_BWD_V = 0 (scalar) / 4 / 8 overrides.
  static const int bwd_v = getenv("LCI_DWCONV_BWD_V") ? atoi(getenv("LCI_DWCONV_BWD_V")) : 4;
  const void* vp[] = {in, gx, gz, din};
  const int vt[] = {in_ts, ox_ts, oz_ts};
  const int V = dtype == 1 ? bwd_v : std::min(bwd_v, 4);
  if (V > 0 && dwconv_vec_ok(dtype, V, C, vp, 4, vt, 3, zoff)) {
    const dim3 gv = dwconv_vec_grid(V, B, L, C, CONV_TB);
    if (dtype != 1) hipLaunchKernelGGL((dwconv_silu_bwd_vec_kernel<float, 4>), gv, dim3(256), 0, (hipStream_t)stream, a);
    else if (V == 8) hipLaunchKernelGGL((dwconv_silu_bwd_vec_kernel<bf16, 8>), gv, dim3(256), 0, (hipStream_t)stream, a);
    else hipLaunchKernelGGL((dwconv_silu_bwd_vec_kernel<bf16, 4>), gv, dim3(256), 0, (hipStream_t)stream, a);
    LCI_LAUNCH_CHECK();
    return 0;
  }
  dim3 grid((2 * C + 255) / 256, (L + CONV_T - 1) / CONV_T, B);
  if (dtype == 1) hipLaunchKernelGGL(dwconv_silu_bwd_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(dwconv_silu_bwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, a);
  LCI_LAUNCH_CHECK();
  return 0;
}
