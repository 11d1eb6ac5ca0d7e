// mpcx_ipm.hip — batched primal-dual interior point solver for stage-structured NLPs.
//
// Included at the end of every generated model source (runtime/codegen.py), which
// defines MPCX_N/NX/NV/NG/NPS/NPG/TS and the four gen_stage_* device functions.
//
// What it replaces: the IPOPT solve behind ca.nlpsol (reference
// agentlib_mpc/data_structures/casadi_utils.py:191-217; called at
// optimization_backends/casadi_/core/discretization.py:203).  The algorithm is
// IPOPT's (barrier + slacks, monotone mu, inertia-corrected Newton steps,
// fraction-to-boundary, filter line search, gradient scaling, bound relaxation,
// least-squares multiplier init) and follows the oracle restatement
// oracle/ipm.py step for step.  What differs is the linear algebra: the KKT
// system of a stage-structured NLP is a block-tridiagonal chain; each block
// (stage-local primals, the state at the stage end, the stage constraint
// multipliers) is factored in LDS by a Bunch-Kaufman LDL^T and the chain is
// eliminated Riccati-style (Schur complement through the nx state columns).
// Inertia = sum of the block inertias (Haynsworth), exactly what IPOPT reads
// from MUMPS.
//
// Mapping: one agent per workgroup of one wavefront (64 lanes).  Lanes run
// over stages for function/derivative evaluation (generated straight-line
// code), over matrix entries for factorisation, and over variables for the
// vector work (wave shuffles for the reductions).  Per-agent state lives in a
// workspace slab in HBM (L2/MALL resident while the agent is active); the
// active KKT block lives in LDS.
#include <hip/hip_runtime.h>
#include <math.h>
#include "mpcx.h"
#include "mpcx_internal.h"

namespace mpcx_kernel {

constexpr int N = MPCX_N;
constexpr int NX = MPCX_NX;
constexpr int NV = MPCX_NV;
constexpr int NG = MPCX_NG;
constexpr int NPS = MPCX_NPS;
constexpr int NPG = MPCX_NPG;
constexpr int NL = 2 * NX + NV;    // stage-local vector [X0, V, X1]
constexpr int NP = NV + NX;        // primal unknowns per KKT block [V, X1]
constexpr int NB = NP + NG;        // KKT block size
constexpr int NW = NX + N * NP;    // NLP variables (reference order)
constexpr int M = N * NG;          // NLP constraints
constexpr int NPAR = NPG + N * NPS;
constexpr int LDB = (NB % 2 == 0) ? NB + 1 : NB;
constexpr int WAVE = 64;
constexpr int MAXF = 32;           // filter entries kept in LDS
constexpr double INF_BOUND = 1e19;
constexpr double TS = MPCX_TS;
#ifndef MPCX_MIN_WAVES
#define MPCX_MIN_WAVES 4
#endif

// workspace layout (doubles per agent)
constexpr long O_X = 0, O_S = O_X + NW, O_LAM = O_S + M, O_ZL = O_LAM + M, O_ZU = O_ZL + NW;
constexpr long O_VL = O_ZU + NW, O_VU = O_VL + M, O_XL = O_VU + M, O_XU = O_XL + NW;
constexpr long O_SL = O_XU + NW, O_SU = O_SL + M, O_GS = O_SU + M, O_GV = O_GS + M;
constexpr long O_DX = O_GV + M, O_DS = O_DX + NW, O_DL = O_DS + M, O_XT = O_DL + M;
constexpr long O_ST = O_XT + NW, O_GT = O_ST + M, O_LB = O_GT + M, O_UB = O_LB + M;
constexpr long O_SDG = O_UB + M;                 // [NL][N]      stage cost gradient
constexpr long O_SDJ = O_SDG + (long)NL * N;     // [NG*NL][N]   stage jacobian
constexpr long O_SDH = O_SDJ + (long)NG * NL * N;// [NL*NL][N]   stage hessian
constexpr long O_FAC = O_SDH + (long)NL * NL * N;// [N][NB*LDB]  block factors
constexpr long O_RHS = O_FAC + (long)N * NB * LDB;
constexpr long O_SOL = O_RHS + (long)N * NB;
constexpr long O_PIV = O_SOL + (long)N * NB;     // ints: perm[N][NB], piv[N][NB]
constexpr long WS_DOUBLES = O_PIV + (long)N * NB;  // 2 ints per double slot

using Args = mpcx_kernel_args;

// ---------------------------------------------------------------------------
// wave helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}
__device__ __forceinline__ double wmax(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, WAVE));
  return v;
}
__device__ __forceinline__ double wmin(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, WAVE));
  return v;
}
__device__ __forceinline__ int wsumi(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}
// argmax with smallest index on ties
__device__ __forceinline__ void wargmax(double& v, int& idx) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double ov = __shfl_xor(v, o, WAVE);
    int oi = __shfl_xor(idx, o, WAVE);
    if (ov > v || (ov == v && oi >= 0 && (idx < 0 || oi < idx))) { v = ov; idx = oi; }
  }
}
__device__ __forceinline__ void sync() { __syncthreads(); }

__device__ __forceinline__ bool isfin(double v) { return fabs(v) < INFINITY; }

// ---------------------------------------------------------------------------
// per-agent views
// ---------------------------------------------------------------------------
struct Agent {
  double* ws;
  const double* p;
  int lane;
  __device__ double* x() const { return ws + O_X; }
  __device__ double* s() const { return ws + O_S; }
  __device__ double* lam() const { return ws + O_LAM; }
  __device__ double* zL() const { return ws + O_ZL; }
  __device__ double* zU() const { return ws + O_ZU; }
  __device__ double* vL() const { return ws + O_VL; }
  __device__ double* vU() const { return ws + O_VU; }
  __device__ double* xL() const { return ws + O_XL; }
  __device__ double* xU() const { return ws + O_XU; }
  __device__ double* sL() const { return ws + O_SL; }
  __device__ double* sU() const { return ws + O_SU; }
  __device__ double* gs() const { return ws + O_GS; }
  __device__ double* gv() const { return ws + O_GV; }
  __device__ double* dx() const { return ws + O_DX; }
  __device__ double* ds() const { return ws + O_DS; }
  __device__ double* dl() const { return ws + O_DL; }
  __device__ double* xt() const { return ws + O_XT; }
  __device__ double* st() const { return ws + O_ST; }
  __device__ double* gt() const { return ws + O_GT; }
  __device__ double* lb() const { return ws + O_LB; }
  __device__ double* ub() const { return ws + O_UB; }
  __device__ double* sdg() const { return ws + O_SDG; }
  __device__ double* sdj() const { return ws + O_SDJ; }
  __device__ double* sdh() const { return ws + O_SDH; }
  __device__ double* fac(int k) const { return ws + O_FAC + (long)k * NB * LDB; }
  __device__ double* rhs(int k) const { return ws + O_RHS + (long)k * NB; }
  __device__ double* sol(int k) const { return ws + O_SOL + (long)k * NB; }
  __device__ int* perm(int k) const { return reinterpret_cast<int*>(ws + O_PIV) + k * NB; }
  __device__ int* piv(int k) const { return reinterpret_cast<int*>(ws + O_PIV) + N * NB + k * NB; }
};

__device__ __forceinline__ bool is_fixed(const Agent& a, int i) { return a.xL()[i] == a.xU()[i]; }

// ---------------------------------------------------------------------------
// evaluation (lane k evaluates stage k)
// ---------------------------------------------------------------------------
// f and unscaled g at point xv; returns wave-summed f
__device__ __noinline__ double eval_fg(const Agent& a, const double* xv, double* gout) {
  double f = 0.0;
  for (int k = a.lane; k < N; k += WAVE) {
    double fk = 0.0;
    gen_stage_fg(xv + k * NP, a.p + NPG + k * NPS, a.p, k * TS, &fk, gout + k * NG, 1);
    f += fk;
  }
  return wsum(f);
}

__device__ __noinline__ void eval_gj(const Agent& a, const double* xv) {
  for (int k = a.lane; k < N; k += WAVE)
    gen_stage_gj(xv + k * NP, a.p + NPG + k * NPS, a.p, k * TS, a.sdg() + k, a.sdj() + k, N);
}

// Hessian of sigma*f + sum lam_i * gs_i * g_i (scaled Lagrangian)
__device__ __noinline__ void eval_hess(const Agent& a, const double* xv, double sigma) {
  for (int k = a.lane; k < N; k += WAVE) {
    double lk[NG > 0 ? NG : 1];
#pragma unroll
    for (int r = 0; r < NG; ++r) lk[r] = a.lam()[k * NG + r] * a.gs()[k * NG + r];
    gen_stage_hess(xv + k * NP, a.p + NPG + k * NPS, a.p, k * TS, sigma, lk, a.sdh() + k, N);
  }
}

// gradient of the (unscaled) objective w.r.t. w[i], i >= NX
__device__ __forceinline__ double acc_grad(const Agent& a, int i) {
  const int b = (i - NX) / NP, off = (i - NX) % NP;
  double v = a.sdg()[(NX + off) * N + b];
  if (NX > 0 && off >= NV && b + 1 < N) v += a.sdg()[(off - NV) * N + b + 1];
  return v;
}
// (J~^T lam~)[i] with J~ = gs*J
__device__ __forceinline__ double acc_jtl(const Agent& a, int i, const double* lamv) {
  const int b = (i - NX) / NP, off = (i - NX) % NP;
  double v = 0.0;
  for (int r = 0; r < NG; ++r)
    v += a.sdj()[(r * NL + NX + off) * N + b] * a.gs()[b * NG + r] * lamv[b * NG + r];
  if (NX > 0 && off >= NV && b + 1 < N)
    for (int r = 0; r < NG; ++r)
      v += a.sdj()[(r * NL + off - NV) * N + b + 1] * a.gs()[(b + 1) * NG + r] * lamv[(b + 1) * NG + r];
  return v;
}

// ---------------------------------------------------------------------------
// dense Bunch-Kaufman LDL^T of the LDS block (full symmetric storage)
// ---------------------------------------------------------------------------
struct Inertia {
  int pos, neg, zero;
};

__device__ __noinline__ void bk_factor(double* A, int* perm, int* piv, int lane, Inertia& in) {
  const double alpha = 0.6403882032022076;  // (1 + sqrt(17)) / 8
  for (int i = lane; i < NB; i += WAVE) perm[i] = i;
  // zero pivots: absolute threshold (same constant as oracle/ipm.py ZERO_PIVOT);
  // the barrier terms make the block norm unbounded near active bounds, so a
  // norm-relative test would misclassify legitimate -delta_c pivots
  const double ztol = 1e-20;
  sync();
  int k = 0;
#pragma unroll 1
  while (k < NB) {
    const double akk = fabs(A[k * LDB + k]);
    double lam = -1.0;
    int r = -1;
    for (int i = k + 1 + lane; i < NB; i += WAVE) {
      const double t = fabs(A[i * LDB + k]);
      if (t > lam) { lam = t; r = i; }
    }
    wargmax(lam, r);
    if (r < 0) lam = 0.0;
    int size = 1, kp = k;
    if (fmax(akk, lam) == 0.0) {
      size = 1; kp = k;
    } else if (akk >= alpha * lam) {
      size = 1; kp = k;
    } else {
      double sg = 0.0;
      for (int j = k + lane; j < NB; j += WAVE)
        if (j != r) sg = fmax(sg, fabs(A[r * LDB + j]));
      const double sigma = wmax(sg);
      if (akk * sigma >= alpha * lam * lam) {
        size = 1; kp = k;
      } else if (fabs(A[r * LDB + r]) >= alpha * sigma) {
        size = 1; kp = r;
      } else {
        size = 2; kp = r;
      }
    }
    const int kk = k + size - 1;
    if (kp != kk) {
      for (int j = lane; j < NB; j += WAVE) {
        const double t = A[kp * LDB + j]; A[kp * LDB + j] = A[kk * LDB + j]; A[kk * LDB + j] = t;
      }
      sync();
      for (int i = lane; i < NB; i += WAVE) {
        const double t = A[i * LDB + kp]; A[i * LDB + kp] = A[i * LDB + kk]; A[i * LDB + kk] = t;
      }
      if (lane == 0) { const int t = perm[kp]; perm[kp] = perm[kk]; perm[kk] = t; }
      sync();
    }
    const int nt = NB - k - size;
    if (size == 1) {
      const double d = A[k * LDB + k];
      if (fabs(d) <= ztol) {
        in.zero++;
        for (int i = k + 1 + lane; i < NB; i += WAVE) A[i * LDB + k] = 0.0;
      } else {
        if (d > 0) in.pos++; else in.neg++;
        const double rd = 1.0 / d;
        for (int t = lane; t < nt * nt; t += WAVE) {
          const int i = k + 1 + t / nt, j = k + 1 + t % nt;
          A[i * LDB + j] -= A[i * LDB + k] * A[j * LDB + k] * rd;
        }
        sync();
        for (int i = k + 1 + lane; i < NB; i += WAVE) A[i * LDB + k] *= rd;
      }
      if (lane == 0) piv[k] = 1;
    } else {
      const double a11 = A[k * LDB + k], a21 = A[(k + 1) * LDB + k], a22 = A[(k + 1) * LDB + k + 1];
      const double det = a11 * a22 - a21 * a21;
      if (fabs(det) <= 1e-40) {
        in.zero += 2;  // treated as singular
      } else {
        if (det < 0) { in.pos++; in.neg++; }
        else if (a11 + a22 > 0) in.pos += 2;
        else in.neg += 2;
      }
      const double rdet = 1.0 / det;
      for (int t = lane; t < nt * nt; t += WAVE) {
        const int i = k + 2 + t / nt, j = k + 2 + t % nt;
        const double ai1 = A[i * LDB + k], ai2 = A[i * LDB + k + 1];
        const double l1 = (ai1 * a22 - ai2 * a21) * rdet, l2 = (ai2 * a11 - ai1 * a21) * rdet;
        A[i * LDB + j] -= l1 * A[j * LDB + k] + l2 * A[j * LDB + k + 1];
      }
      sync();
      for (int i = k + 2 + lane; i < NB; i += WAVE) {
        const double ai1 = A[i * LDB + k], ai2 = A[i * LDB + k + 1];
        A[i * LDB + k] = (ai1 * a22 - ai2 * a21) * rdet;
        A[i * LDB + k + 1] = (ai2 * a11 - ai1 * a21) * rdet;
      }
      if (lane == 0) { piv[k] = 2; piv[k + 1] = 0; }
    }
    sync();
    k += size;
  }
}

// v <- A^{-1} v using factor F (L, D in F; perm, piv); v and y in LDS
__device__ __noinline__ void bk_solve(const double* F, const int* perm, const int* piv, double* v, double* y,
                         int lane) {
  for (int i = lane; i < NB; i += WAVE) y[i] = v[perm[i]];
  sync();
  // forward: L z = y
  int k = 0;
  while (k < NB) {
    const int sz = piv[k];
    const double y0 = y[k];
    if (sz == 1) {
      for (int i = k + 1 + lane; i < NB; i += WAVE) y[i] -= F[i * LDB + k] * y0;
    } else {
      const double y1 = y[k + 1];
      for (int i = k + 2 + lane; i < NB; i += WAVE) y[i] -= F[i * LDB + k] * y0 + F[i * LDB + k + 1] * y1;
    }
    sync();
    k += sz;
  }
  // diagonal
  for (int i = lane; i < NB; i += WAVE) {
    const int sz = piv[i];
    if (sz == 1) {
      const double d = F[i * LDB + i];
      y[i] = (d != 0.0) ? y[i] / d : 0.0;
    } else if (sz == 2) {
      const double a11 = F[i * LDB + i], a21 = F[(i + 1) * LDB + i], a22 = F[(i + 1) * LDB + i + 1];
      const double det = a11 * a22 - a21 * a21;
      const double y0 = y[i], y1 = y[i + 1];
      y[i] = (a22 * y0 - a21 * y1) / det;
      y[i + 1] = (a11 * y1 - a21 * y0) / det;
    }
  }
  sync();
  // backward: L^T u = y (column sweep from the end)
  k = NB - 1;
  while (k >= 0) {
    const int start = (piv[k] == 0) ? k - 1 : k;
    const int sz = k - start + 1;
    const double u0 = y[start];
    const double u1 = (sz == 2) ? y[start + 1] : 0.0;
    for (int j = lane; j < start; j += WAVE) {
      double t = F[start * LDB + j] * u0;
      if (sz == 2) t += F[(start + 1) * LDB + j] * u1;
      y[j] -= t;
    }
    sync();
    k = start - 1;
  }
  for (int i = lane; i < NB; i += WAVE) v[perm[i]] = y[i];
  sync();
}

// ---------------------------------------------------------------------------
// KKT assembly
// ---------------------------------------------------------------------------
enum Mode { NEWTON = 0, LSQ = 1 };

struct KKTDiag {
  double dw, dc;
  Mode mode;
};

__device__ __forceinline__ double sigma_x(const Agent& a, int i) {
  const double xv = a.x()[i], lo = a.xL()[i], hi = a.xU()[i];
  double s = 0.0;
  if (lo == hi) return 0.0;
  if (isfin(lo)) s += a.zL()[i] / (xv - lo);
  if (isfin(hi)) s += a.zU()[i] / (hi - xv);
  return s;
}
__device__ __forceinline__ double sigma_s(const Agent& a, int c) {
  const double sv = a.s()[c], lo = a.sL()[c], hi = a.sU()[c];
  double s = 0.0;
  if (isfin(lo)) s += a.vL()[c] / (sv - lo);
  if (isfin(hi)) s += a.vU()[c] / (hi - sv);
  return s;
}
// constraint classes: 0 equality, 1 inequality with a finite bound, 2 free
__device__ __forceinline__ int ccls(const Agent& a, int c) {
  const double lo = a.lb()[c], hi = a.ub()[c];
  if (lo == hi) return 0;
  if (!isfin(a.sL()[c]) && !isfin(a.sU()[c])) return 2;
  return 1;
}
__device__ __forceinline__ double dual_diag(const Agent& a, int c, const KKTDiag& kd) {
  const int cl = ccls(a, c);
  if (kd.mode == LSQ) return cl == 0 ? 0.0 : 1.0;
  if (cl == 0) return kd.dc;
  if (cl == 2) return 1.0;
  return 1.0 / (sigma_s(a, c) + kd.dw) + kd.dc;
}

// coupling of block k to x_k (columns c < NX of stage k's local vector)
__device__ __forceinline__ double coupling(const Agent& a, int k, int row, int c, Mode mode) {
  if (is_fixed(a, k * NP + c)) return 0.0;
  if (row < NP) {
    if (mode == LSQ) return 0.0;
    if (is_fixed(a, NX + k * NP + row)) return 0.0;
    return a.sdh()[((NX + row) * NL + c) * N + k];
  }
  const int r = row - NP;
  return a.gs()[k * NG + r] * a.sdj()[(r * NL + c) * N + k];
}

__device__ __noinline__ void assemble(const Agent& a, int k, const KKTDiag& kd, double* A) {
  const int lane = a.lane;
  const int w0 = NX + k * NP;
  for (int t = lane; t < NP * NP; t += WAVE) {
    const int p = t / NP, q = t % NP;
    double v;
    if (is_fixed(a, w0 + p) || is_fixed(a, w0 + q)) {
      v = (p == q) ? 1.0 : 0.0;
    } else if (kd.mode == LSQ) {
      v = (p == q) ? 1.0 : 0.0;
    } else {
      v = a.sdh()[((NX + p) * NL + NX + q) * N + k];
      if (NX > 0 && p >= NV && q >= NV && k + 1 < N) v += a.sdh()[((p - NV) * NL + (q - NV)) * N + k + 1];
      if (p == q) v += sigma_x(a, w0 + p) + kd.dw;
    }
    A[p * LDB + q] = v;
  }
  for (int t = lane; t < NG * NP; t += WAVE) {
    const int r = t / NP, q = t % NP;
    const double v = is_fixed(a, w0 + q) ? 0.0 : a.gs()[k * NG + r] * a.sdj()[(r * NL + NX + q) * N + k];
    A[(NP + r) * LDB + q] = v;
    A[q * LDB + NP + r] = v;
  }
  for (int t = lane; t < NG * NG; t += WAVE) {
    const int r = t / NG, c = t % NG;
    A[(NP + r) * LDB + NP + c] = (r == c) ? -dual_diag(a, k * NG + r, kd) : 0.0;
  }
}

// Factor the whole chain; returns inertia.  Shared scratch in LDS.
struct Lds {
  double A[NB * LDB];
  double B[NB * (NX > 0 ? NX : 1)];
  double BP[NB * (NX > 0 ? NX : 1)];
  double P[(NX > 0 ? NX : 1) * (NX > 0 ? NX : 1)];
  double v[NB];
  double y[NB];
  double t[NB];
  int perm[NB];
  int piv[NB];
  double fth[MAXF];
  double fph[MAXF];
};

__device__ __noinline__ Inertia factor_chain(const Agent& a, const KKTDiag& kd, Lds& L) {
  const int lane = a.lane;
  Inertia in{0, 0, 0};
#pragma unroll 1
  for (int k = 0; k < N; ++k) {
    assemble(a, k, kd, L.A);
    if (NX > 0 && k > 0) {
      for (int t = lane; t < NB * NX; t += WAVE) L.B[t] = coupling(a, k, t / NX, t % NX, kd.mode);
      sync();
      for (int t = lane; t < NB * NX; t += WAVE) {
        const int i = t / NX, d = t % NX;
        double s = 0.0;
        for (int c = 0; c < NX; ++c) s += L.B[i * NX + c] * L.P[c * NX + d];
        L.BP[t] = s;
      }
      sync();
      for (int t = lane; t < NB * NB; t += WAVE) {
        const int i = t / NB, j = t % NB;
        double s = 0.0;
        for (int d = 0; d < NX; ++d) s += L.BP[i * NX + d] * L.B[j * NX + d];
        L.A[i * LDB + j] -= s;
      }
    }
    sync();
    bk_factor(L.A, L.perm, L.piv, lane, in);
    // store factor
    double* F = a.fac(k);
    for (int t = lane; t < NB * LDB; t += WAVE) F[t] = L.A[t];
    for (int i = lane; i < NB; i += WAVE) { a.perm(k)[i] = L.perm[i]; a.piv(k)[i] = L.piv[i]; }
    // P_k = [A_k^{-1}]_{X1,X1}
    if (NX > 0 && k + 1 < N) {
#pragma unroll 1
      for (int c = 0; c < NX; ++c) {
        for (int i = lane; i < NB; i += WAVE) L.v[i] = (i == NV + c) ? 1.0 : 0.0;
        sync();
        bk_solve(L.A, L.perm, L.piv, L.v, L.y, lane);
        for (int d = lane; d < NX; d += WAVE) L.t[d * NX + c] = L.v[NV + d];
        sync();
      }
      for (int t = lane; t < NX * NX; t += WAVE) L.P[t] = L.t[t];
    }
    sync();
  }
  return in;
}

// Solve the chain with rhs blocks a.rhs(k) -> a.sol(k)
__device__ __noinline__ void solve_chain(const Agent& a, Mode mode, Lds& L) {
  const int lane = a.lane;
  // forward
#pragma unroll 1
  for (int k = 0; k < N; ++k) {
    for (int i = lane; i < NB; i += WAVE) L.v[i] = a.rhs(k)[i];
    sync();
    if (NX > 0 && k > 0) {
      for (int t = lane; t < NB * NX; t += WAVE) L.B[t] = coupling(a, k, t / NX, t % NX, mode);
      sync();
      const double* wp = a.sol(k - 1);
      for (int i = lane; i < NB; i += WAVE) {
        double s = 0.0;
        for (int c = 0; c < NX; ++c) s += L.B[i * NX + c] * wp[NV + c];
        L.v[i] -= s;
      }
      sync();
    }
    bk_solve(a.fac(k), a.perm(k), a.piv(k), L.v, L.y, lane);
    for (int i = lane; i < NB; i += WAVE) a.sol(k)[i] = L.v[i];
    sync();
  }
  // backward
  if (NX > 0) {
#pragma unroll 1
    for (int k = N - 2; k >= 0; --k) {
      const double* un = a.sol(k + 1);
      for (int t = lane; t < NB * NX; t += WAVE) L.B[t] = coupling(a, k + 1, t / NX, t % NX, mode);
      for (int i = lane; i < NB; i += WAVE) L.v[i] = 0.0;
      sync();
      for (int c = lane; c < NX; c += WAVE) {
        double s = 0.0;
#pragma unroll 4
        for (int i = 0; i < NB; ++i) s += L.B[i * NX + c] * un[i];
        L.v[NV + c] = s;
      }
      sync();
      bk_solve(a.fac(k), a.perm(k), a.piv(k), L.v, L.y, lane);
      for (int i = lane; i < NB; i += WAVE) a.sol(k)[i] -= L.v[i];
      sync();
    }
  }
}

// ---------------------------------------------------------------------------
// scalar helpers on vectors (all lanes return the same value)
// ---------------------------------------------------------------------------
__device__ __noinline__ double theta_of(const Agent& a, const double* gval, const double* sv) {
  double t = 0.0;
  for (int c = a.lane; c < M; c += WAVE) {
    const double cv = (ccls(a, c) == 0) ? gval[c] - a.gs()[c] * a.lb()[c] : gval[c] - sv[c];
    t += fabs(cv);
  }
  return wsum(t);
}
__device__ __noinline__ double barrier_of(const Agent& a, const double* xv, const double* sv) {
  double t = 0.0;
  for (int i = NX + a.lane; i < NW; i += WAVE) {
    const double lo = a.xL()[i], hi = a.xU()[i];
    if (lo == hi) continue;
    if (isfin(lo)) t += log(xv[i] - lo);
    if (isfin(hi)) t += log(hi - xv[i]);
  }
  for (int c = a.lane; c < M; c += WAVE) {
    if (ccls(a, c) != 1) continue;
    if (isfin(a.sL()[c])) t += log(sv[c] - a.sL()[c]);
    if (isfin(a.sU()[c])) t += log(a.sU()[c] - sv[c]);
  }
  return wsum(t);
}

struct OptErr {
  double err, dual, primal, compl_, dual_u, primal_u;
};

// scaled optimality error E_mu (IPOPT eq. 5) + unscaled parts
__device__ __noinline__ OptErr opt_error(const Agent& a, double mu, double obj_scale) {
  double dmax = 0.0, dmax_u = 0.0, pmax = 0.0, pmax_u = 0.0, cmax = 0.0;
  double lsum = 0.0, zsum = 0.0;
  int nz = 0;
  for (int i = NX + a.lane; i < NW; i += WAVE) {
    if (is_fixed(a, i)) continue;
    const double rd = obj_scale * acc_grad(a, i) + acc_jtl(a, i, a.lam()) - a.zL()[i] + a.zU()[i];
    dmax = fmax(dmax, fabs(rd));
    dmax_u = fmax(dmax_u, fabs(rd) / obj_scale);
    const double lo = a.xL()[i], hi = a.xU()[i];
    if (isfin(lo)) { cmax = fmax(cmax, fabs((a.x()[i] - lo) * a.zL()[i] - mu)); zsum += fabs(a.zL()[i]); nz++; }
    if (isfin(hi)) { cmax = fmax(cmax, fabs((hi - a.x()[i]) * a.zU()[i] - mu)); zsum += fabs(a.zU()[i]); nz++; }
  }
  for (int c = a.lane; c < M; c += WAVE) {
    const int cl = ccls(a, c);
    const double gsc = a.gs()[c];
    double cv;
    if (cl == 0) {
      cv = a.gv()[c] - gsc * a.lb()[c];
    } else {
      cv = a.gv()[c] - a.s()[c];
      if (cl == 1) {
        const double rs = -a.lam()[c] - a.vL()[c] + a.vU()[c];
        dmax = fmax(dmax, fabs(rs));
        if (isfin(a.sL()[c])) { cmax = fmax(cmax, fabs((a.s()[c] - a.sL()[c]) * a.vL()[c] - mu)); zsum += fabs(a.vL()[c]); nz++; }
        if (isfin(a.sU()[c])) { cmax = fmax(cmax, fabs((a.sU()[c] - a.s()[c]) * a.vU()[c] - mu)); zsum += fabs(a.vU()[c]); nz++; }
      }
    }
    pmax = fmax(pmax, fabs(cv));
    pmax_u = fmax(pmax_u, fabs(cv) / gsc);
    lsum += fabs(a.lam()[c]);
  }
  dmax = wmax(dmax); dmax_u = wmax(dmax_u); pmax = wmax(pmax); pmax_u = wmax(pmax_u);
  cmax = wmax(cmax); lsum = wsum(lsum); zsum = wsum(zsum); nz = wsumi(nz);
  const double smax = 100.0;
  // IPOPT: s_d over all multipliers (y_c, y_d, z_L, z_U, v_L, v_U)
  const double s_d = fmax(smax, (lsum + zsum) / fmax(1.0, (double)(M + nz))) / smax;
  const double s_c = nz > 0 ? fmax(smax, zsum / (double)nz) / smax : 1.0;
  OptErr e;
  e.err = fmax(fmax(dmax / s_d, pmax), cmax / s_c);
  e.dual = dmax; e.primal = pmax; e.compl_ = cmax; e.dual_u = dmax_u; e.primal_u = pmax_u;
  return e;
}

// push v into [lo + pl, hi - pu] (IPOPT bound_push / bound_frac)
__device__ __forceinline__ double push_into(double v, double lo, double hi, double kp, double kf) {
  const bool hl = isfin(lo), hu = isfin(hi);
  double pl = hl ? kp * fmax(1.0, fabs(lo)) : 0.0;
  double pu = hu ? kp * fmax(1.0, fabs(hi)) : 0.0;
  if (hl && hu) { pl = fmin(pl, kf * (hi - lo)); pu = fmin(pu, kf * (hi - lo)); }
  const double lop = hl ? lo + pl : -INFINITY;
  const double hip = hu ? hi - pu : INFINITY;
  if (hl && hu && lop > hip) return 0.5 * (lo + hi);
  return fmin(fmax(v, lop), hip);
}
__device__ __forceinline__ double relax_lo(double b, double f) { return b - f * fmax(1.0, fabs(b)); }
__device__ __forceinline__ double relax_hi(double b, double f) { return b + f * fmax(1.0, fabs(b)); }

// ---------------------------------------------------------------------------
// IPM phases (noinline: keeps the register budget of each phase separate)
// ---------------------------------------------------------------------------
struct Scal {
  double obj_scale, fx;
};

__device__ __noinline__ Scal init_agent(const Agent& a, const Args& args, int agent) {
  const mpcx_options& o = args.opt;
  const int lane = a.lane;
  const double* lbw = args.lbw + (long)agent * NW;
  const double* ubw = args.ubw + (long)agent * NW;
  const double* wio = args.w + (long)agent * NW;
  for (long t = lane; t < (long)(NL + NG * NL + NL * NL) * N; t += WAVE) a.ws[O_SDG + t] = 0.0;
  for (int i = lane; i < NW; i += WAVE) {
    double lo = lbw[i], hi = ubw[i];
    if (lo <= -INF_BOUND) lo = -INFINITY;
    if (hi >= INF_BOUND) hi = INFINITY;
    if (i < NX) hi = lo;  // x_0 is fixed to the initial state (full.py:51-52)
    a.xL()[i] = lo;
    a.xU()[i] = hi;
    a.x()[i] = (lo == hi) ? lo : wio[i];
  }
  if (args.lbg != nullptr) {
    for (int c = lane; c < M; c += WAVE) {
      a.lb()[c] = args.lbg[(long)agent * M + c];
      a.ub()[c] = args.ubg[(long)agent * M + c];
    }
  } else {
    for (int k = lane; k < N; k += WAVE)
      gen_stage_bounds(a.p + NPG + k * NPS, a.p, k * TS, a.lb() + k * NG, a.ub() + k * NG, 1);
  }
  sync();
  for (int c = lane; c < M; c += WAVE) {
    if (a.lb()[c] <= -INF_BOUND) a.lb()[c] = -INFINITY;
    if (a.ub()[c] >= INF_BOUND) a.ub()[c] = INFINITY;
  }
  sync();
  // gradient based scaling at the user starting point
  eval_gj(a, a.x());
  sync();
  double gmax = 0.0;
  for (int i = NX + lane; i < NW; i += WAVE)
    if (!is_fixed(a, i)) gmax = fmax(gmax, fabs(acc_grad(a, i)));
  gmax = wmax(gmax);
  Scal sc;
  sc.obj_scale = 1.0;
  if (gmax > o.nlp_scaling_max_gradient)
    sc.obj_scale = fmax(o.nlp_scaling_min_value, o.nlp_scaling_max_gradient / gmax);
  for (int c = lane; c < M; c += WAVE) {
    const int k = c / NG, r = c % NG;
    double rm = 0.0;
    for (int j = 0; j < NL; ++j)
      if (!is_fixed(a, k * NP + j)) rm = fmax(rm, fabs(a.sdj()[(r * NL + j) * N + k]));
    a.gs()[c] = (rm > o.nlp_scaling_max_gradient) ? fmax(o.nlp_scaling_min_value, o.nlp_scaling_max_gradient / rm) : 1.0;
  }
  // bound relaxation + initial point
  for (int i = lane; i < NW; i += WAVE) {
    double lo = a.xL()[i], hi = a.xU()[i];
    if (i >= NX && lo != hi) {
      if (isfin(lo)) lo = relax_lo(lo, o.bound_relax_factor);
      if (isfin(hi)) hi = relax_hi(hi, o.bound_relax_factor);
      a.xL()[i] = lo;
      a.xU()[i] = hi;
      a.x()[i] = push_into(a.x()[i], lo, hi, o.bound_push, o.bound_frac);
      a.zL()[i] = isfin(lo) ? o.bound_mult_init_val : 0.0;
      a.zU()[i] = isfin(hi) ? o.bound_mult_init_val : 0.0;
    } else {
      a.zL()[i] = 0.0;
      a.zU()[i] = 0.0;
    }
  }
  sync();
  sc.fx = sc.obj_scale * eval_fg(a, a.x(), a.gv());
  sync();
  for (int c = lane; c < M; c += WAVE) {
    const double gsc = a.gs()[c];
    a.gv()[c] *= gsc;
    const double lo = a.lb()[c], hi = a.ub()[c];
    if (lo == hi) {
      a.sL()[c] = gsc * lo; a.sU()[c] = gsc * hi; a.s()[c] = gsc * lo;
      a.vL()[c] = 0.0; a.vU()[c] = 0.0;
    } else {
      const double sl = isfin(lo) ? relax_lo(gsc * lo, o.bound_relax_factor) : -INFINITY;
      const double su = isfin(hi) ? relax_hi(gsc * hi, o.bound_relax_factor) : INFINITY;
      a.sL()[c] = sl; a.sU()[c] = su;
      a.s()[c] = push_into(a.gv()[c], sl, su, o.bound_push, o.bound_frac);
      a.vL()[c] = isfin(sl) ? o.bound_mult_init_val : 0.0;
      a.vU()[c] = isfin(su) ? o.bound_mult_init_val : 0.0;
    }
    a.lam()[c] = 0.0;
  }
  sync();
  eval_gj(a, a.x());
  sync();
  return sc;
}

// least-squares estimate of the constraint multipliers (IPOPT constr_mult_init_max)
__device__ __noinline__ void ls_multipliers(const Agent& a, const mpcx_options& o, double obj_scale, Lds& L) {
  const int lane = a.lane;
  KKTDiag kd{0.0, 0.0, LSQ};
  const Inertia in = factor_chain(a, kd, L);
#pragma unroll 1
  for (int k = 0; k < N; ++k) {
    for (int q = lane; q < NP; q += WAVE) {
      const int i = NX + k * NP + q;
      a.rhs(k)[q] = is_fixed(a, i) ? 0.0 : -(obj_scale * acc_grad(a, i) - a.zL()[i] + a.zU()[i]);
    }
    for (int r = lane; r < NG; r += WAVE) {
      const int c = k * NG + r;
      a.rhs(k)[NP + r] = (ccls(a, c) == 1) ? a.vL()[c] - a.vU()[c] : 0.0;
    }
  }
  sync();
  if (in.zero != 0) return;
  solve_chain(a, LSQ, L);
  double lmax = 0.0;
  for (int c = lane; c < M; c += WAVE) lmax = fmax(lmax, fabs(a.sol(c / NG)[NP + c % NG]));
  lmax = wmax(lmax);
  if (lmax <= o.constr_mult_init_max)
    for (int c = lane; c < M; c += WAVE) a.lam()[c] = a.sol(c / NG)[NP + c % NG];
  sync();
}

__device__ __noinline__ void rhs_primal(const Agent& a, double mu, double obj_scale) {
  const int lane = a.lane;
  for (int i = NX + lane; i < NW; i += WAVE) {
    double r = 0.0;
    if (!is_fixed(a, i)) {
      const double lo = a.xL()[i], hi = a.xU()[i], xv = a.x()[i];
      double gphi = obj_scale * acc_grad(a, i);
      if (isfin(lo)) gphi -= mu / (xv - lo);
      if (isfin(hi)) gphi += mu / (hi - xv);
      r = -(gphi + acc_jtl(a, i, a.lam()));
    }
    a.rhs((i - NX) / NP)[(i - NX) % NP] = r;
  }
  sync();
}

__device__ __forceinline__ double slack_rs(const Agent& a, int c, double mu) {
  const double sv = a.s()[c];
  double gphis = 0.0;
  if (isfin(a.sL()[c])) gphis -= mu / (sv - a.sL()[c]);
  if (isfin(a.sU()[c])) gphis += mu / (a.sU()[c] - sv);
  return gphis - a.lam()[c];
}

__device__ __noinline__ void rhs_dual(const Agent& a, double mu, double dw) {
  const int lane = a.lane;
  for (int c = lane; c < M; c += WAVE) {
    const int cl = ccls(a, c);
    double rr;
    if (cl == 0) {
      rr = -(a.gv()[c] - a.gs()[c] * a.lb()[c]);
    } else {
      rr = -(a.gv()[c] - a.s()[c]);
      if (cl == 1) rr -= slack_rs(a, c, mu) / (sigma_s(a, c) + dw);
    }
    a.rhs(c / NG)[NP + c % NG] = rr;
  }
  sync();
}

struct StepInfo {
  double amax, az, gphid;
};

// full step from the chain solution + fraction-to-the-boundary step sizes
__device__ __noinline__ StepInfo recover_step(const Agent& a, double mu, double tau, double dw,
                                              double obj_scale) {
  const int lane = a.lane;
  double amax = 1.0, az = 1.0, gphid = 0.0;
  for (int i = lane; i < NW; i += WAVE) {
    double d = 0.0;
    if (i >= NX && !is_fixed(a, i)) d = a.sol((i - NX) / NP)[(i - NX) % NP];
    a.dx()[i] = d;
    if (i < NX || is_fixed(a, i)) continue;
    const double lo = a.xL()[i], hi = a.xU()[i], xv = a.x()[i];
    double gphi = obj_scale * acc_grad(a, i);
    if (isfin(lo)) {
      const double sl = xv - lo;
      gphi -= mu / sl;
      if (d < 0) amax = fmin(amax, -tau * sl / d);
      const double dz = mu / sl - a.zL()[i] - (a.zL()[i] / sl) * d;
      if (dz < 0) az = fmin(az, -tau * a.zL()[i] / dz);
    }
    if (isfin(hi)) {
      const double su = hi - xv;
      gphi += mu / su;
      if (d > 0) amax = fmin(amax, tau * su / d);
      const double dz = mu / su - a.zU()[i] + (a.zU()[i] / su) * d;
      if (dz < 0) az = fmin(az, -tau * a.zU()[i] / dz);
    }
    gphid += gphi * d;
  }
  for (int c = lane; c < M; c += WAVE) {
    const double dlam = a.sol(c / NG)[NP + c % NG];
    a.dl()[c] = dlam;
    double dsv = 0.0;
    if (ccls(a, c) == 1) {
      const double sv = a.s()[c];
      const double rs = slack_rs(a, c, mu);
      dsv = (dlam - rs) / (sigma_s(a, c) + dw);
      gphid += (rs + a.lam()[c]) * dsv;
      if (isfin(a.sL()[c])) {
        const double sl = sv - a.sL()[c];
        if (dsv < 0) amax = fmin(amax, -tau * sl / dsv);
        const double dv = mu / sl - a.vL()[c] - (a.vL()[c] / sl) * dsv;
        if (dv < 0) az = fmin(az, -tau * a.vL()[c] / dv);
      }
      if (isfin(a.sU()[c])) {
        const double su = a.sU()[c] - sv;
        if (dsv > 0) amax = fmin(amax, tau * su / dsv);
        const double dv = mu / su - a.vU()[c] + (a.vU()[c] / su) * dsv;
        if (dv < 0) az = fmin(az, -tau * a.vU()[c] / dv);
      }
    }
    a.ds()[c] = dsv;
  }
  StepInfo st;
  st.amax = wmin(amax);
  st.az = wmin(az);
  st.gphid = wsum(gphid);
  sync();
  return st;
}

struct Trial {
  double f, theta, phi;
};

__device__ __noinline__ Trial trial_point(const Agent& a, double alpha, double mu, double obj_scale) {
  const int lane = a.lane;
  for (int i = lane; i < NW; i += WAVE) a.xt()[i] = a.x()[i] + alpha * a.dx()[i];
  for (int c = lane; c < M; c += WAVE) a.st()[c] = a.s()[c] + alpha * a.ds()[c];
  sync();
  Trial t;
  t.f = obj_scale * eval_fg(a, a.xt(), a.gt());
  sync();
  for (int c = lane; c < M; c += WAVE) a.gt()[c] *= a.gs()[c];
  sync();
  t.theta = theta_of(a, a.gt(), a.st());
  t.phi = t.f - mu * barrier_of(a, a.xt(), a.st());
  return t;
}

__device__ __noinline__ void accept_step(const Agent& a, const mpcx_options& o, double mu,
                                         double alpha, double az) {
  const int lane = a.lane;
  for (int i = NX + lane; i < NW; i += WAVE) {
    if (is_fixed(a, i)) continue;
    const double d = a.dx()[i];
    const double lo = a.xL()[i], hi = a.xU()[i], xold = a.x()[i];
    const double xn = a.xt()[i];
    a.x()[i] = xn;
    if (isfin(lo)) {
      const double sl0 = xold - lo;
      const double dz = mu / sl0 - a.zL()[i] - (a.zL()[i] / sl0) * d;
      const double zn = a.zL()[i] + az * dz, sl = xn - lo;
      a.zL()[i] = fmax(fmin(zn, o.kappa_sigma * mu / sl), mu / (o.kappa_sigma * sl));
    }
    if (isfin(hi)) {
      const double su0 = hi - xold;
      const double dz = mu / su0 - a.zU()[i] + (a.zU()[i] / su0) * d;
      const double zn = a.zU()[i] + az * dz, su = hi - xn;
      a.zU()[i] = fmax(fmin(zn, o.kappa_sigma * mu / su), mu / (o.kappa_sigma * su));
    }
  }
  for (int c = lane; c < M; c += WAVE) {
    a.lam()[c] += alpha * a.dl()[c];
    a.gv()[c] = a.gt()[c];
    if (ccls(a, c) != 1) { a.s()[c] = a.st()[c]; continue; }
    const double sold = a.s()[c], sn = a.st()[c], dsv = a.ds()[c];
    a.s()[c] = sn;
    if (isfin(a.sL()[c])) {
      const double sl0 = sold - a.sL()[c];
      const double dv = mu / sl0 - a.vL()[c] - (a.vL()[c] / sl0) * dsv;
      const double vn = a.vL()[c] + az * dv, sl = sn - a.sL()[c];
      a.vL()[c] = fmax(fmin(vn, o.kappa_sigma * mu / sl), mu / (o.kappa_sigma * sl));
    }
    if (isfin(a.sU()[c])) {
      const double su0 = a.sU()[c] - sold;
      const double dv = mu / su0 - a.vU()[c] + (a.vU()[c] / su0) * dsv;
      const double vn = a.vU()[c] + az * dv, su = a.sU()[c] - sn;
      a.vU()[c] = fmax(fmin(vn, o.kappa_sigma * mu / su), mu / (o.kappa_sigma * su));
    }
  }
  sync();
}

}  // namespace mpcx_kernel

using namespace mpcx_kernel;

// ---------------------------------------------------------------------------
// the kernel: one agent NLP per workgroup (one wavefront)
// ---------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(64, MPCX_MIN_WAVES) mpcx_ipm_solve(Args args) {
  const int agent = blockIdx.x;
  if (agent >= args.n_agents) return;
  __shared__ Lds L;
  const mpcx_options& o = args.opt;
  Agent a;
  a.ws = args.ws + (long)agent * args.ws_stride;
  a.p = args.p + (long)agent * NPAR;
  a.lane = threadIdx.x;
  const int lane = a.lane;

  const Scal sc = init_agent(a, args, agent);
  const double obj_scale = sc.obj_scale;
  double fx = sc.fx;
  int n_fact = 0, n_ic = 0, n_fallback = 0, n_trials = 0;
  if (M > 0 && o.constr_mult_init_max > 0.0) {
    ls_multipliers(a, o, obj_scale, L);
    n_fact++;
  }

  double mu = o.mu_init;
  double tau = fmax(o.tau_min, 1.0 - mu);
  double dw_last = 0.0;
  const double theta0 = theta_of(a, a.gv(), a.s());
  const double theta_max = o.theta_max_fact * fmax(1.0, theta0);
  const double theta_min = o.theta_min_fact * fmax(1.0, theta0);
  int nfilt = 0;
  int status = MPCX_MAX_ITER_EXCEEDED;
  int it = 0;
  OptErr e0;
#pragma unroll 1
  for (;;) {
    e0 = opt_error(a, 0.0, obj_scale);
    if (!(e0.err == e0.err) || !(fx == fx)) { status = MPCX_INVALID_NUMBER; break; }
    if (e0.err <= o.tol && e0.dual_u <= o.dual_inf_tol && e0.primal_u <= o.constr_viol_tol &&
        e0.compl_ <= o.compl_inf_tol) {
      status = MPCX_SOLVE_SUCCEEDED;
      break;
    }
    if (it >= o.max_iter) break;
    // barrier parameter update (monotone Fiacco-McCormick)
#pragma unroll 1
    for (int mu_up = 0; mu_up < 64; ++mu_up) {
      const OptErr em = opt_error(a, mu, obj_scale);
      if (em.err > o.kappa_eps * mu || mu <= o.mu_min) break;
      mu = fmax(o.tol / 10.0, fmin(o.kappa_mu * mu, pow(mu, o.theta_mu)));
      mu = fmax(mu, o.mu_min);
      tau = fmax(o.tau_min, 1.0 - mu);
      nfilt = 0;
    }
    eval_hess(a, a.x(), obj_scale);
    sync();
    rhs_primal(a, mu, obj_scale);
    // factorisation with inertia correction (IPOPT Algorithm IC)
    double dw = 0.0, dc = 0.0;
    bool ok = false;
#pragma unroll 1
    for (int attempt = 0; attempt < 60; ++attempt) {
      KKTDiag kd{dw, dc, NEWTON};
      const Inertia in = factor_chain(a, kd, L);
      n_fact++;
      if (in.pos == N * NP && in.neg == M && in.zero == 0) {
        if (attempt > 0) dw_last = dw;
        ok = true;
        break;
      }
      n_ic++;
      if (attempt == 0) {
        if (in.zero > 0) dc = o.delta_c_bar * pow(mu, o.kappa_c);
        dw = (dw_last == 0.0) ? o.delta_w_first : fmax(o.delta_w_min, o.kappa_w_minus * dw_last);
      } else {
        dw = (dw_last == 0.0) ? o.kappa_w_plus_bar * dw : o.kappa_w_plus * dw;
        if (dw > o.delta_w_max) break;
      }
    }
    if (!ok) { status = MPCX_ERROR_IN_STEP; break; }
    rhs_dual(a, mu, dw);
    solve_chain(a, NEWTON, L);
    const StepInfo st = recover_step(a, mu, tau, dw, obj_scale);
    // filter line search
    const double theta = theta_of(a, a.gv(), a.s());
    const double phi = fx - mu * barrier_of(a, a.x(), a.s());
    const double gphid = st.gphid;
    double amin;
    if (gphid < 0 && theta <= theta_min)
      amin = o.alpha_min_frac * fmin(fmin(o.gamma_theta, o.gamma_phi * theta / (-gphid)),
                                     o.delta * pow(theta, o.s_theta) / pow(-gphid, o.s_phi));
    else if (gphid < 0)
      amin = o.alpha_min_frac * fmin(o.gamma_theta, o.gamma_phi * theta / (-gphid));
    else
      amin = o.alpha_min_frac * o.gamma_theta;
    double alpha = st.amax;
    Trial tr{0.0, 0.0, 0.0};
    bool accepted = false, ftype = false;
    if (!(amin > 0.0)) amin = o.alpha_min_frac * o.gamma_theta;  // NaN guard
#pragma unroll 1
    for (int ls = 0; ls < 64; ++ls) {
      tr = trial_point(a, alpha, mu, obj_scale);
      n_trials++;
      bool okt = (tr.theta <= theta_max) && (tr.phi == tr.phi);
      for (int j = 0; j < nfilt && okt; ++j)
        if (tr.theta >= L.fth[j] && tr.phi >= L.fph[j]) okt = false;
      if (okt) {
        const bool switching = gphid < 0 && alpha * pow(-gphid, o.s_phi) > o.delta * pow(theta, o.s_theta);
        if (theta <= theta_min && switching) {
          okt = tr.phi <= phi + o.eta_phi * alpha * gphid;
          ftype = true;
        } else {
          okt = tr.theta <= (1.0 - o.gamma_theta) * theta || tr.phi <= phi - o.gamma_phi * theta;
          ftype = false;
        }
      }
      if (okt) { accepted = true; break; }
      alpha *= 0.5;
      if (alpha < amin) break;
    }
    if (!accepted) { nfilt = 0; ftype = true; n_fallback++; }
    if (!ftype) {
      if (nfilt == MAXF) {
        if (lane == 0)
          for (int j = 1; j < MAXF; ++j) { L.fth[j - 1] = L.fth[j]; L.fph[j - 1] = L.fph[j]; }
        nfilt--;
      }
      if (lane == 0) { L.fth[nfilt] = (1.0 - o.gamma_theta) * theta; L.fph[nfilt] = phi - o.gamma_phi * theta; }
      nfilt++;
      sync();
    }
    accept_step(a, o, mu, alpha, st.az);
    fx = tr.f;
    eval_gj(a, a.x());
    sync();
    it++;
  }

  // ---- outputs ----------------------------------------------------------------
  double* wio = args.w + (long)agent * NW;
  for (int i = lane; i < NW; i += WAVE) {
    wio[i] = a.x()[i];
    if (args.lam_w != nullptr)
      args.lam_w[(long)agent * NW + i] = (i < NX) ? 0.0 : (a.zU()[i] - a.zL()[i]) / obj_scale;
  }
  if (args.lam_g != nullptr)
    for (int c = lane; c < M; c += WAVE) args.lam_g[(long)agent * M + c] = a.lam()[c] * a.gs()[c] / obj_scale;
  if (args.stats != nullptr && lane == 0) {
    mpcx_stats st;
    st.obj = fx / obj_scale;
    st.primal_inf = e0.primal_u;
    st.dual_inf = e0.dual_u;
    st.compl_inf = e0.compl_;
    st.mu = mu;
    st.obj_scale = obj_scale;
    st.iter_count = it;
    st.status = status;
    st.n_inertia_corrections = n_ic;
    st.n_linesearch_fallbacks = n_fallback;
    st.n_factorizations = n_fact;
    st.n_trials = n_trials;
    args.stats[agent] = st;
  }
}

extern "C" __global__ void mpcx_query(long* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = WS_DOUBLES;
    out[1] = N; out[2] = NX; out[3] = NV; out[4] = NG; out[5] = NPS; out[6] = NPG;
    out[7] = MPCX_ABI;
    out[8] = sizeof(Lds);
  }
}
