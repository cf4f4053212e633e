/* ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into liblci or called by the product path.
 *
 * fp64 selective scan, forward and backward, for long sequences (L up to 2^21 and beyond), restating the
 * published semantics of mamba-ssm 1.2.0.post1 `selective_scan_ref` (mamba_ssm/ops/selective_scan_interface.py)
 * as called by the reference at model/models/mamba.py:125-134 (variable B/C of shape (B, N, L), z = None,
 * delta_softplus = True, return_last_state = False); the Python restatement of the same function is
 * oracle/selective_scan.py, pinned by tests/golden/selective_scan.npz. The per-step loop here is the same
 * recurrence evaluated in plain C so that the L = 2^21 (C5) sequence length can be checked in seconds:
 *
 *   dt_t   = softplus(delta_t + delta_bias)            (torch softplus: threshold 20 -> identity)
 *   x_t[n] = exp(dt_t A[n]) x_{t-1}[n] + dt_t B_t[n] u_t,   x_{-1} = 0
 *   y_t    = sum_n C_t[n] x_t[n] + D u_t
 *
 * and its adjoint for a cotangent dy (reverse sweep, g_t[n] = dy_t C_t[n] + exp(dt_{t+1} A[n]) g_{t+1}[n]):
 *   du_t = D dy_t + sum_n g_t[n] dt_t B_t[n]
 *   ddt_t = sum_n g_t[n] (B_t[n] u_t + A[n] exp(dt_t A[n]) x_{t-1}[n]);  ddelta_t = ddt_t softplus'(.)
 *   dA[n] += g_t[n] exp(dt_t A[n]) x_{t-1}[n] dt_t;   dB_t[n] += g_t[n] dt_t u_t;   dC_t[n] += dy_t x_t[n]
 *   dD += dy_t u_t;   ddelta_bias += ddelta_t
 *
 * Layout: channels-last f32 (token stride `ts` elements, channel stride 1), one batch element per call; B and C
 * (L, N) with token stride `bts`. Channels are independent, so they run in parallel (OpenMP); dB / dC are
 * reduced over channels in per-thread f64 buffers.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

static double softplus(double x) { return x > 20.0 ? x : log1p(exp(x)); }
static double softplus_grad(double x) { return x > 20.0 ? 1.0 : 1.0 / (1.0 + exp(-x)); }

/* y (L, Dx) f64 out. */
int scan_ref_fwd(const float* u, const float* delta, const float* Bm, const float* Cm, const double* A,
                 const double* D, const double* dbias, long long L, int Dx, int N, long long ts, long long bts,
                 double* y) {
  if (N > 64) return 1;
#pragma omp parallel for schedule(dynamic, 1)
  for (int d = 0; d < Dx; ++d) {
    double x[64] = {0};
    for (long long t = 0; t < L; ++t) {
      const double dt = softplus((double)delta[t * ts + d] + dbias[d]);
      const double uu = u[t * ts + d];
      double acc = 0.0;
      for (int n = 0; n < N; ++n) {
        x[n] = exp(dt * A[d * N + n]) * x[n] + dt * (double)Bm[t * bts + n] * uu;
        acc += (double)Cm[t * bts + n] * x[n];
      }
      y[t * Dx + d] = acc + D[d] * uu;
    }
  }
  return 0;
}

/* du, ddelta (L, Dx) f64 written; dA (Dx, N), dD (Dx), ddbias (Dx) written; dB, dC (L, N) f64 written.
 * nthreads: the number of OpenMP threads the caller allows (per-thread dB/dC buffers of 2 L N doubles). */
int scan_ref_bwd(const float* u, const float* delta, const float* Bm, const float* Cm, const double* A,
                 const double* D, const double* dbias, const float* dy, long long L, int Dx, int N, long long ts,
                 long long bts, double* du, double* ddelta, double* dA, double* dD, double* ddbias, double* dB,
                 double* dC, int nthreads) {
  if (N > 64 || nthreads < 1) return 1;
  const long long LN = L * N;
  double* part = (double*)calloc((size_t)nthreads * 2 * LN, sizeof(double));
  double* xs = (double*)malloc((size_t)nthreads * (LN + N) * sizeof(double));
  if (!part || !xs) {
    free(part);
    free(xs);
    return 2;
  }
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
  for (int d = 0; d < Dx; ++d) {
#ifdef _OPENMP
    extern int omp_get_thread_num(void);
    const int tid = omp_get_thread_num();
#else
    const int tid = 0;
#endif
    double* pB = part + (size_t)tid * 2 * LN;
    double* pC = pB + LN;
    double* xh = xs + (size_t)tid * (LN + N);   /* xh[(t + 1) N + n] = x_t[n], xh[0..N) = x_{-1} = 0 */
    for (int n = 0; n < N; ++n) xh[n] = 0.0;
    for (long long t = 0; t < L; ++t) {
      const double dt = softplus((double)delta[t * ts + d] + dbias[d]);
      const double uu = u[t * ts + d];
      for (int n = 0; n < N; ++n)
        xh[(t + 1) * N + n] = exp(dt * A[d * N + n]) * xh[t * N + n] + dt * (double)Bm[t * bts + n] * uu;
    }
    double g[64] = {0}, an[64], dAl[64] = {0};
    double dDl = 0.0, dbl = 0.0;
    for (int n = 0; n < N; ++n) an[n] = 0.0;   /* exp(dt_{t+1} A): zero past the end */
    for (long long t = L - 1; t >= 0; --t) {
      const double z = (double)delta[t * ts + d] + dbias[d];
      const double dt = softplus(z);
      const double uu = u[t * ts + d];
      const double gy = dy[t * ts + d];
      double s_du = 0.0, s_dt = 0.0;
      for (int n = 0; n < N; ++n) {
        const double a = exp(dt * A[d * N + n]);
        const double bn = Bm[t * bts + n];
        g[n] = gy * (double)Cm[t * bts + n] + an[n] * g[n];
        an[n] = a;
        const double xp = xh[t * N + n];
        s_du += g[n] * dt * bn;
        s_dt += g[n] * (bn * uu + A[d * N + n] * a * xp);
        dAl[n] += g[n] * a * xp * dt;
        pB[t * N + n] += g[n] * dt * uu;
        pC[t * N + n] += gy * xh[(t + 1) * N + n];
      }
      du[t * Dx + d] = D[d] * gy + s_du;
      const double dd = s_dt * softplus_grad(z);
      ddelta[t * Dx + d] = dd;
      dDl += gy * uu;
      dbl += dd;
    }
    for (int n = 0; n < N; ++n) dA[d * N + n] = dAl[n];
    dD[d] = dDl;
    ddbias[d] = dbl;
  }
  memset(dB, 0, (size_t)LN * sizeof(double));
  memset(dC, 0, (size_t)LN * sizeof(double));
  for (int th = 0; th < nthreads; ++th) {
    const double* pB = part + (size_t)th * 2 * LN;
    const double* pC = pB + LN;
    for (long long i = 0; i < LN; ++i) {
      dB[i] += pB[i];
      dC[i] += pC[i];
    }
  }
  free(part);
  free(xs);
  return 0;
}
