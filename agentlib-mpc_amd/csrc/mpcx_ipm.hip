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
constexpr long O_FAC = O_SDH + (long)NL * NL * N;// [N][NB*LDB]  blocks, then block inverses
constexpr long O_RHS = O_FAC + (long)N * NB * LDB;
constexpr long O_SOL = O_RHS + (long)N * NB;
constexpr long O_CPL = O_SOL + (long)N * NB;     // [N][NB*NX] couplings to x_k (block chain)
constexpr long O_KX = O_CPL + (long)N * NB * (NX > 0 ? NX : 1);  // [N*NP] primal KKT diagonal
constexpr long O_KD = O_KX + (long)N * NP;       // [M] dual KKT diagonal
constexpr int LPK = (NV + NG + 2 * NX) * (NV + NG + 2 * NX + 1) / 2;
constexpr long O_LF = O_KD + M;                  // [N][LPK] stage-local factors
constexpr long O_LPV = O_LF + (long)N * LPK;     // [N][2*NI] ints (perm, piv)
constexpr long O_LZ = O_LPV + (long)N * (NV + NG);
constexpr long WS_DOUBLES = O_LZ + (long)N * (NV + NG);

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
// Wavefront-scope sync for LDS-only hand-offs between lanes: a workgroup is one
// wavefront and the LDS executes one wave's DS instructions in issue order, so
// only compiler ordering is needed (no s_barrier, no vmcnt drain).
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ bool isfin(double v) { return fabs(v) < INFINITY; }

// LDS-qualified pointers: keeps ds_* addressing inside the noinline phases
// (a generic pointer would compile to flat_* accesses)
typedef __attribute__((address_space(3))) double ldsd;
typedef __attribute__((address_space(3))) int ldsi;

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
  __device__ double* cpl(int k) const { return ws + O_CPL + (long)k * NB * (NX > 0 ? NX : 1); }
  __device__ double* kx() const { return ws + O_KX; }
  __device__ double* kd() const { return ws + O_KD; }
  __device__ double* lf(int k) const { return ws + O_LF + (long)k * LPK; }
  __device__ int* lpv(int k) const { return reinterpret_cast<int*>(ws + O_LPV) + (long)k * 2 * (NV + NG); }
  __device__ double* lz(int k) const { return ws + O_LZ + (long)k * (NV + NG); }
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
// dense Bunch-Kaufman LDL^T in LDS (full symmetric storage, wave-wide)
// ---------------------------------------------------------------------------
struct Inertia {
  int pos, neg, zero;
};

// zero pivots: absolute threshold (same constant as oracle/ipm.py ZERO_PIVOT);
// the barrier terms make the block norm unbounded near active bounds, so a
// norm-relative test would misclassify legitimate -delta_c pivots
constexpr double ZERO_PIVOT = 1e-20;
constexpr double BK_ALPHA = 0.6403882032022076;  // (1 + sqrt(17)) / 8

template <int NN, int LD>
__device__ __noinline__ void bk_factor(ldsd* A, ldsi* perm, ldsi* piv, int lane, Inertia& in) {
  constexpr int NN2 = NN * NN;
  for (int i = lane; i < NN; i += WAVE) perm[i] = i;
  wsync();
  int k = 0;
#pragma unroll 1
  while (k < NN) {
    const double akk = fabs(A[k * LD + k]);
    double lam = -1.0;
    int r = -1;
    for (int i = k + 1 + lane; i < NN; i += WAVE) {
      const double t = fabs(A[i * LD + k]);
      if (t > lam) { lam = t; r = i; }
    }
    wargmax(lam, r);
    if (r < 0) lam = 0.0;
    int size = 1, kp = k;
    if (fmax(akk, lam) == 0.0 || akk >= BK_ALPHA * lam) {
      size = 1; kp = k;
    } else {
      double sg = 0.0;
      for (int j = k + lane; j < NN; j += WAVE)
        if (j != r) sg = fmax(sg, fabs(A[r * LD + j]));
      const double sigma = wmax(sg);
      if (akk * sigma >= BK_ALPHA * lam * lam) {
        size = 1; kp = k;
      } else if (fabs(A[r * LD + r]) >= BK_ALPHA * sigma) {
        size = 1; kp = r;
      } else {
        size = 2; kp = r;
      }
    }
    const int kk = k + size - 1;
    if (kp != kk) {
      for (int j = lane; j < NN; j += WAVE) {
        const double t = A[kp * LD + j]; A[kp * LD + j] = A[kk * LD + j]; A[kk * LD + j] = t;
      }
      wsync();
      for (int i = lane; i < NN; i += WAVE) {
        const double t = A[i * LD + kp]; A[i * LD + kp] = A[i * LD + kk]; A[i * LD + kk] = t;
      }
      if (lane == 0) { const int t = perm[kp]; perm[kp] = perm[kk]; perm[kk] = t; }
      wsync();
    }
    if (size == 1) {
      const double d = A[k * LD + k];
      if (fabs(d) <= ZERO_PIVOT) {
        in.zero++;
        for (int i = k + 1 + lane; i < NN; i += WAVE) A[i * LD + k] = 0.0;
      } else {
        if (d > 0) in.pos++; else in.neg++;
        const double rd = 1.0 / d;
        for (int t = lane; t < NN2; t += WAVE) {
          const int i = t / NN, j = t % NN;
          if (i > k && j > k) A[i * LD + j] -= A[i * LD + k] * A[j * LD + k] * rd;
        }
        wsync();
        for (int i = k + 1 + lane; i < NN; i += WAVE) A[i * LD + k] *= rd;
      }
      if (lane == 0) piv[k] = 1;
    } else {
      const double a11 = A[k * LD + k], a21 = A[(k + 1) * LD + k], a22 = A[(k + 1) * LD + k + 1];
      const double det = a11 * a22 - a21 * a21;
      if (fabs(det) <= ZERO_PIVOT * ZERO_PIVOT) {
        in.zero += 2;
      } else {
        if (det < 0) { in.pos++; in.neg++; }
        else if (a11 + a22 > 0) in.pos += 2;
        else in.neg += 2;
      }
      const double rdet = 1.0 / det;
      for (int t = lane; t < NN2; t += WAVE) {
        const int i = t / NN, j = t % NN;
        if (i > k + 1 && j > k + 1) {
          const double ai1 = A[i * LD + k], ai2 = A[i * LD + k + 1];
          const double l1 = (ai1 * a22 - ai2 * a21) * rdet, l2 = (ai2 * a11 - ai1 * a21) * rdet;
          A[i * LD + j] -= l1 * A[j * LD + k] + l2 * A[j * LD + k + 1];
        }
      }
      wsync();
      for (int i = k + 2 + lane; i < NN; i += WAVE) {
        const double ai1 = A[i * LD + k], ai2 = A[i * LD + k + 1];
        A[i * LD + k] = (ai1 * a22 - ai2 * a21) * rdet;
        A[i * LD + k + 1] = (ai2 * a11 - ai1 * a21) * rdet;
      }
      if (lane == 0) { piv[k] = 2; piv[k + 1] = 0; }
    }
    wsync();
    k += size;
  }
}

// Explicit inverse of a factored block, A^{-1} = P^T L^{-T} D^{-1} L^{-1} P,
// written in the ORIGINAL index order to `out` (ld LD).  W, Y: LDS scratch.
template <int NN, int LD>
__device__ __noinline__ void bk_inverse(const ldsd* A, const ldsi* perm, const ldsi* piv, ldsd* W,
                                        ldsd* Y, double* out, int lane) {
  constexpr int NN2 = NN * NN;
  for (int t = lane; t < NN2; t += WAVE) {
    const int i = t / NN, j = t % NN;
    W[i * LD + j] = (i == j) ? 1.0 : 0.0;
  }
  wsync();
  int k = 0;
#pragma unroll 1
  while (k < NN) {
    const int sz = piv[k];
    for (int t = lane; t < NN2; t += WAVE) {
      const int i = t / NN, j = t % NN;
      if (i >= k + sz && j <= k + sz - 1) {
        double v = A[i * LD + k] * W[k * LD + j];
        if (sz == 2) v += A[i * LD + k + 1] * W[(k + 1) * LD + j];
        W[i * LD + j] -= v;
      }
    }
    wsync();
    k += sz;
  }
  for (int t = lane; t < NN2; t += WAVE) {
    const int i = t / NN, j = t % NN;
    const int sz = piv[i];
    if (sz == 1) {
      const double d = A[i * LD + i];
      Y[i * LD + j] = (d != 0.0) ? W[i * LD + j] / d : 0.0;
    } else if (sz == 2) {
      const double a11 = A[i * LD + i], a21 = A[(i + 1) * LD + i], a22 = A[(i + 1) * LD + i + 1];
      const double det = a11 * a22 - a21 * a21;
      const double w0 = W[i * LD + j], w1 = W[(i + 1) * LD + j];
      Y[i * LD + j] = (a22 * w0 - a21 * w1) / det;
      Y[(i + 1) * LD + j] = (a11 * w1 - a21 * w0) / det;
    }
  }
  wsync();
  for (int t = lane; t < NN2; t += WAVE) {
    const int i = t / NN, j = t % NN;
    double acc = 0.0;
    const int mx = i > j ? i : j;
    for (int m = (mx > 0 ? mx - 1 : 0); m < NN; ++m) acc += W[m * LD + i] * Y[m * LD + j];
    out[perm[i] * LD + perm[j]] = acc;
  }
  wsync();
}

// ---------------------------------------------------------------------------
// KKT entries
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

// ---------------------------------------------------------------------------
// LDS layout
// ---------------------------------------------------------------------------
// Stage-parallel path: stage k's local system, ordered [V_k, lambda_k | x_k, x_{k+1}],
// is held packed-lower in LDS; SR stages are resident per round, G lanes per stage.
constexpr int NI = NV + NG;               // stage interior (eliminated in parallel)
constexpr int NXP = NX > 0 ? NX : 1;
constexpr int NXX = NXP * NXP;
constexpr int NLOC = NI + 2 * NX;         // local system size
constexpr int PK = NLOC * (NLOC + 1) / 2; // packed lower triangle
constexpr int PKS = PK | 1;               // odd stride between stage slots
static_assert(NI > 0, "stage interior must be non-empty");

__host__ __device__ constexpr int pow2floor(int v) { int p = 1; while (p * 2 <= v) p *= 2; return p; }
__host__ __device__ constexpr int cmin(int a, int b) { return a < b ? a : b; }
__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }

constexpr int SLOT_BYTES = 8 * (PKS + NLOC) + 8 * NI;  // F + z + perm/piv
constexpr int OTHER_BYTES = 8 * (N * 3 * NXX + N * NXX + 3 * N * NXP + 3 * NXX + 2 * MAXF) + 8 * NXP + 64;
#ifndef MPCX_LDS_TARGET
#define MPCX_LDS_TARGET 9600  // keeps 16 one-wave workgroups per CU (160 KB LDS)
#endif
constexpr int SR0 = cmax(1, cmin(cmin(N, WAVE), (MPCX_LDS_TARGET - OTHER_BYTES) / SLOT_BYTES));
constexpr int ROUNDS = (N + SR0 - 1) / SR0;
constexpr int SR = (N + ROUNDS - 1) / ROUNDS;   // stages per round (balanced)
constexpr int G = pow2floor(WAVE / SR);         // lanes per stage

constexpr int SQ = NX > 0 ? NB : 1;   // the fallback exists only when stages are coupled
constexpr int SQL = NX > 0 ? LDB : 1;
struct SeqLds {               // sequential block chain (fallback)
  double A[SQ * SQL];
  double W[SQ * SQL];
  double Y[SQ * SQL];
  double B[SQ * NXP];
  double BP[SQ * NXP];
  double P[NXX];
  double v[SQ];
  double y[SQ];
  double t[SQ];
  int perm[SQ];
  int piv[SQ];
};
struct ParLds {
  double F[SR * PKS];
  double z[SR * NLOC];
  int perm[SR * NI];
  int piv[SR * NI];
};
union LinLds {
  SeqLds s;
  ParLds p;
};

struct Lds {
  LinLds u;
  double S[N * 3 * NXX];   // local Schur blocks per stage: S00 (x_k), S11 (x_{k+1}), S10
  double Dinv[N * NXX];    // inverses of the state-chain pivots
  double zx0[N * NXP];     // forward-eliminated local rhs, x_k part
  double zx1[N * NXP];     // ... x_{k+1} part
  double xs[N * NXP];      // state-chain rhs, then solution (x_1 .. x_N)
  double C[NXX];
  double CW[NXX];
  double CY[NXX];
  int cperm[NXP];
  int cpiv[NXP];
  int seq;                 // 1: last factorisation used the sequential chain
  double fth[MAXF];
  double fph[MAXF];
#ifdef MPCX_PROFILE
  double sprof[6];
#endif
};

__shared__ Lds gL;
#ifdef MPCX_PROFILE
#define SPROF_DECL unsigned long long _st = __builtin_amdgcn_s_memtime();
#define SPROF(i) do { const unsigned long long _n = __builtin_amdgcn_s_memtime(); if (a.lane == 0) gL.sprof[i] += (double)(_n - _st); _st = _n; } while (0)
#else
#define SPROF_DECL
#define SPROF(i) do { } while (0)
#endif  // one agent per workgroup: the agent's LDS scratch
#define LDSP(x) ((ldsd*)(x))
#define LDSI(x) ((ldsi*)(x))

// per-variable / per-constraint diagonal terms of the KKT matrix, once per factorisation
// (workspace: NaN in kx marks a fixed variable)
__device__ __noinline__ void kkt_diagonals(const Agent& a, const KKTDiag& kd) {
  for (int q = a.lane; q < N * NP; q += WAVE) {
    const int i = NX + q;
    a.kx()[q] = is_fixed(a, i) ? NAN : (kd.mode == LSQ ? 1.0 : sigma_x(a, i) + kd.dw);
  }
  for (int c = a.lane; c < M; c += WAVE) a.kd()[c] = dual_diag(a, c, kd);
  sync();
}

__device__ __forceinline__ bool kfixed(const Agent& a, int k, int q) {
  const double v = a.kx()[k * NP + q];
  return v != v;
}

// ---------------------------------------------------------------------------
// sequential block chain (fallback when a stage interior is singular)
// ---------------------------------------------------------------------------
// entry (i, j) of KKT block k = [V_k, X_{k+1}, lambda_k] (before the Schur update)
__device__ __forceinline__ double kkt_entry(const Agent& a, int k, int i, int j, Mode mode) {
  if (i < NP && j < NP) {
    if (kfixed(a, k, i) || kfixed(a, k, j)) return (i == j) ? 1.0 : 0.0;
    if (mode == LSQ) return (i == j) ? 1.0 : 0.0;
    double v = a.sdh()[((NX + i) * NL + NX + j) * N + k];
    if (NX > 0 && i >= NV && j >= NV && k + 1 < N) v += a.sdh()[((i - NV) * NL + (j - NV)) * N + k + 1];
    if (i == j) v += a.kx()[k * NP + i];
    return v;
  }
  if (i >= NP && j >= NP) return (i == j) ? -a.kd()[k * NG + i - NP] : 0.0;
  const int r = (i >= NP) ? i - NP : j - NP;
  const int q = (i >= NP) ? j : i;
  if (kfixed(a, k, q)) return 0.0;
  return a.gs()[k * NG + r] * a.sdj()[(r * NL + NX + q) * N + k];
}

// coupling of block k (row) to x_k = X0 of stage k (column c < NX)
__device__ __forceinline__ double coupling(const Agent& a, int k, int row, int c, Mode mode) {
  if (k == 0 || kfixed(a, k - 1, NV + c)) return 0.0;
  if (row < NP) {
    if (mode == LSQ || kfixed(a, k, row)) return 0.0;
    return a.sdh()[((NX + row) * NL + c) * N + k];
  }
  const int r = row - NP;
  return a.gs()[k * NG + r] * a.sdj()[(r * NL + c) * N + k];
}

constexpr int NB2 = NB * NB;
constexpr int EPL = (NB2 + WAVE - 1) / WAVE;  // block elements per lane

__device__ __noinline__ void seq_assemble(const Agent& a, Mode mode) {
#pragma unroll 4
  for (int t = a.lane; t < N * NB2; t += WAVE) {
    const int k = t / NB2, e = t % NB2, i = e / NB, j = e % NB;
    a.fac(k)[i * LDB + j] = kkt_entry(a, k, i, j, mode);
  }
  if (NX > 0) {
#pragma unroll 4
    for (int t = a.lane; t < N * NB * NX; t += WAVE) {
      const int k = t / (NB * NX), e = t % (NB * NX);
      a.cpl(k)[e] = coupling(a, k, e / NX, e % NX, mode);
    }
  }
  sync();
}

// Block LDL^T through the state columns: D_k = A_k - B_k [D_{k-1}^{-1}]_{xx} B_k^T;
// each block's explicit inverse is stored (solves become mat-vecs).
__device__ __noinline__ Inertia seq_factor(const Agent& a, Mode mode) {
  SeqLds& L = gL.u.s;
  if constexpr (NX == 0) return Inertia{0, 0, 1};
  const int lane = a.lane;
  Inertia in{0, 0, 0};
  seq_assemble(a, mode);
  double pre[EPL];
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int t = lane + e * WAVE;
    pre[e] = (t < NB2) ? a.fac(0)[(t / NB) * LDB + t % NB] : 0.0;
  }
#pragma unroll 1
  for (int k = 0; k < N; ++k) {
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int t = lane + e * WAVE;
      if (t < NB2) L.A[(t / NB) * LDB + t % NB] = pre[e];
    }
    if (NX > 0 && k > 0)
      for (int t = lane; t < NB * NX; t += WAVE) L.B[t] = a.cpl(k)[t];
    sync();
    if (k + 1 < N) {  // prefetch block k+1 (consumed at the top of the next step)
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const int t = lane + e * WAVE;
        pre[e] = (t < NB2) ? a.fac(k + 1)[(t / NB) * LDB + t % NB] : 0.0;
      }
    }
    if (NX > 0 && k > 0) {
      for (int t = lane; t < NB * NX; t += WAVE) {
        const int i = t / NX, d = t % NX;
        double s = 0.0;
        for (int c = 0; c < NX; ++c) s += L.B[i * NX + c] * L.P[c * NX + d];
        L.BP[t] = s;
      }
      wsync();
      for (int t = lane; t < NB2; t += WAVE) {
        const int i = t / NB, j = t % NB;
        double s = 0.0;
        for (int d = 0; d < NX; ++d) s += L.BP[i * NX + d] * L.B[j * NX + d];
        L.A[i * LDB + j] -= s;
      }
      wsync();
    }
    bk_factor<NB, LDB>(LDSP(L.A), LDSI(L.perm), LDSI(L.piv), lane, in);
    bk_inverse<NB, LDB>(LDSP(L.A), LDSI(L.perm), LDSI(L.piv), LDSP(L.W), LDSP(L.Y), a.fac(k), lane);
    sync();
    if (NX > 0 && k + 1 < N)
      for (int t = lane; t < NX * NX; t += WAVE)
        L.P[t] = a.fac(k)[(NV + t / NX) * LDB + NV + t % NX];
    sync();
  }
  return in;
}

__device__ __noinline__ void seq_solve(const Agent& a) {
  SeqLds& L = gL.u.s;
  if constexpr (NX == 0) return;
  const int lane = a.lane;
#pragma unroll 1
  for (int k = 0; k < N; ++k) {
    for (int i = lane; i < NB; i += WAVE) {
      double v = a.rhs(k)[i];
      if (NX > 0 && k > 0)
        for (int c = 0; c < NX; ++c) v -= a.cpl(k)[i * NX + c] * L.y[NV + c];
      L.v[i] = v;
    }
    wsync();
    const double* Ai = a.fac(k);
    for (int i = lane; i < NB; i += WAVE) {
      double acc = 0.0;
#pragma unroll 8
      for (int j = 0; j < NB; ++j) acc += Ai[i * LDB + j] * L.v[j];
      a.sol(k)[i] = acc;
      L.t[i] = acc;
    }
    wsync();
    for (int i = lane; i < NB; i += WAVE) L.y[i] = L.t[i];
    wsync();
  }
  if (NX > 0) {
#pragma unroll 1
    for (int k = N - 2; k >= 0; --k) {
      for (int c = lane; c < NX; c += WAVE) {
        double s = 0.0;
        for (int i = 0; i < NB; ++i) s += a.cpl(k + 1)[i * NX + c] * L.y[i];
        L.t[c] = s;
      }
      wsync();
      const double* Ai = a.fac(k);
      for (int i = lane; i < NB; i += WAVE) {
        double u = a.sol(k)[i];
        for (int c = 0; c < NX; ++c) u -= Ai[i * LDB + NV + c] * L.t[c];
        a.sol(k)[i] = u;
        L.v[i] = u;
      }
      wsync();
      for (int i = lane; i < NB; i += WAVE) L.y[i] = L.v[i];
      wsync();
    }
  }
  sync();
}

// ---------------------------------------------------------------------------
// stage-parallel elimination (default path)
// ---------------------------------------------------------------------------
// The KKT matrix, permuted to [all stage interiors | all states], has a block-
// diagonal interior part.  Every stage's interior is Bunch-Kaufman factored in
// parallel (G lanes per stage) with the two state blocks it touches appended as
// trailing rows, which leaves the stage's local Schur complement on (x_k, x_{k+1})
// in those rows.  The states then form a block-tridiagonal chain of nx x nx
// pivots: the only sequential part.  Inertia = sum of interior and chain
// inertias (Haynsworth).  A singular interior falls back to the block chain.

__device__ __forceinline__ int pko(int i) { return (i * (i + 1)) >> 1; }

__device__ __forceinline__ double gmax(double v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, WAVE));
  return v;
}
__device__ __forceinline__ void gargmax(double& v, int& idx) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) {
    const double ov = __shfl_xor(v, o, WAVE);
    const int oi = __shfl_xor(idx, o, WAVE);
    if (ov > v || (ov == v && oi >= 0 && (idx < 0 || oi < idx))) { v = ov; idx = oi; }
  }
}

// local index -> (kind, index in the stage vector [X0, V, X1] of length NL)
// kinds: 0 primal V, 1 dual, 2 x_k, 3 x_{k+1}
__device__ __forceinline__ int lkind(int i) {
  return i < NV ? 0 : (i < NI ? 1 : (i < NI + NX ? 2 : 3));
}

// entry (i >= j) of stage k's local system
__device__ __forceinline__ double local_entry(const Agent& a, int k, int i, int j, Mode mode) {
  const int ki = lkind(i), kj = lkind(j);
  if (ki == 1 && kj == 1) return (i == j) ? -a.kd()[k * NG + i - NV] : 0.0;
  if (ki == 1 || kj == 1) {
    const int r = (ki == 1 ? i : j) - NV;
    const int q = (ki == 1 ? j : i);
    const int kq = (ki == 1 ? kj : ki);
    int nl;
    if (kq == 0) { if (kfixed(a, k, q)) return 0.0; nl = NX + q; }
    else if (kq == 2) { if (k == 0 || kfixed(a, k - 1, NV + q - NI)) return 0.0; nl = q - NI; }
    else { if (kfixed(a, k, NV + q - NI - NX)) return 0.0; nl = NX + NV + (q - NI - NX); }
    return a.gs()[k * NG + r] * a.sdj()[(r * NL + nl) * N + k];
  }
  // primal-primal
  int nli, nlj;
  bool fi, fj;
  if (ki == 0) { fi = kfixed(a, k, i); nli = NX + i; }
  else if (ki == 2) { fi = (k == 0) || kfixed(a, k - 1, NV + i - NI); nli = i - NI; }
  else { fi = kfixed(a, k, NV + i - NI - NX); nli = NX + NV + (i - NI - NX); }
  if (kj == 0) { fj = kfixed(a, k, j); nlj = NX + j; }
  else if (kj == 2) { fj = (k == 0) || kfixed(a, k - 1, NV + j - NI); nlj = j - NI; }
  else { fj = kfixed(a, k, NV + j - NI - NX); nlj = NX + NV + (j - NI - NX); }
  if (fi || fj) return (i == j && ki == 0) ? 1.0 : 0.0;   // fixed states: chain pivot 1
  if (mode == LSQ) return (i == j && ki != 2) ? 1.0 : 0.0;
  double v = a.sdh()[(nli * NL + nlj) * N + k];
  if (i == j && ki == 0) v += a.kx()[k * NP + i];
  if (i == j && ki == 3) v += a.kx()[k * NP + NV + (i - NI - NX)];
  return v;
}

// Bunch-Kaufman over the NI interior pivots of one stage (G lanes, packed lower
// storage); the trailing 2*NX rows receive the updates but never pivot.
// Sets bad on a zero pivot (singular interior).
__device__ __noinline__ void interior_bk(ldsd* F, ldsi* perm, ldsi* piv, int g, Inertia& in, int& bad) {
  int k = 0;
#pragma unroll 1
  while (k < NI) {
    const double akk = fabs(F[pko(k) + k]);
    double lam = -1.0;
    int r = -1;
    for (int i = k + 1 + g; i < NI; i += G) {
      const double t = fabs(F[pko(i) + k]);
      if (t > lam) { lam = t; r = i; }
    }
    gargmax(lam, r);
    if (r < 0) lam = 0.0;
    if (fmax(akk, lam) == 0.0) {
      if constexpr (NX > 0) { bad = 1; break; }
      in.zero++;  // independent stages: the zero column is a zero eigenvalue
      if (g == 0) piv[k] = 1;
      wsync();
      k += 1;
      continue;
    }
    int size = 1, kp = k;
    if (akk < BK_ALPHA * lam) {
      double sg = 0.0;
      for (int j = k + g; j < NI; j += G)
        if (j != r) sg = fmax(sg, fabs(F[j < r ? pko(r) + j : pko(j) + r]));
      const double sigma = gmax(sg);
      if (akk * sigma >= BK_ALPHA * lam * lam) {
        kp = k;
      } else if (fabs(F[pko(r) + r]) >= BK_ALPHA * sigma) {
        kp = r;
      } else {
        size = 2; kp = r;
      }
    }
    const int p = k + size - 1, q = kp;
    if (q != p) {  // symmetric interchange p <-> q (p < q < NI) in packed storage
      const int op = pko(p), oq = pko(q);
      for (int j = g; j < NLOC; j += G) {
        if (j == p) {
          const double t = F[op + p]; F[op + p] = F[oq + q]; F[oq + q] = t;
        } else if (j < p) {
          const double t = F[op + j]; F[op + j] = F[oq + j]; F[oq + j] = t;
        } else if (j < q) {
          const int oj = pko(j);
          const double t = F[oj + p]; F[oj + p] = F[oq + j]; F[oq + j] = t;
        } else if (j > q) {
          const int oj = pko(j);
          const double t = F[oj + p]; F[oj + p] = F[oj + q]; F[oj + q] = t;
        }
      }
      if (g == 0) { const int t = perm[p]; perm[p] = perm[q]; perm[q] = t; }
      wsync();
    }
    if (size == 1) {
      const double d = F[pko(k) + k];
      if (fabs(d) <= ZERO_PIVOT) {
        if constexpr (NX > 0) { bad = 1; break; }
        in.zero++;
      } else if (d > 0) {
        in.pos++;
      } else {
        in.neg++;
      }
      const double rd = 1.0 / d;
      const int m = NLOC - 1 - k;  // rows k+1 .. NLOC-1, paired for balance
      for (int base = 0; base < m; base += 2 * G) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int o = base + (h == 0 ? g : 2 * G - 1 - g);
          if (o < m) {
            const int i = k + 1 + o, ri = pko(i);
            const double lik = F[ri + k] * rd;
            int pj = pko(k + 1);
            for (int j = k + 1; j <= i; ++j) { F[ri + j] -= lik * F[pj + k]; pj += j + 1; }
          }
        }
      }
      wsync();
      for (int i = k + 1 + g; i < NLOC; i += G) F[pko(i) + k] *= rd;
      if (g == 0) piv[k] = 1;
    } else {
      const int ok = pko(k), ok1 = pko(k + 1);
      const double a11 = F[ok + k], a21 = F[ok1 + k], a22 = F[ok1 + k + 1];
      const double det = a11 * a22 - a21 * a21;
      if (fabs(det) <= ZERO_PIVOT * ZERO_PIVOT) {
        if constexpr (NX > 0) { bad = 1; break; }
        in.zero += 2;
      } else if (det < 0) {
        in.pos++; in.neg++;
      } else if (a11 + a22 > 0) {
        in.pos += 2;
      } else {
        in.neg += 2;
      }
      const double rdet = 1.0 / det;
      const int m = NLOC - 2 - k;  // rows k+2 .. NLOC-1
      for (int base = 0; base < m; base += 2 * G) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int o = base + (h == 0 ? g : 2 * G - 1 - g);
          if (o < m) {
            const int i = k + 2 + o, ri = pko(i);
            const double ai1 = F[ri + k], ai2 = F[ri + k + 1];
            const double l1 = (ai1 * a22 - ai2 * a21) * rdet, l2 = (ai2 * a11 - ai1 * a21) * rdet;
            int pj = pko(k + 2);
            for (int j = k + 2; j <= i; ++j) { F[ri + j] -= l1 * F[pj + k] + l2 * F[pj + k + 1]; pj += j + 1; }
          }
        }
      }
      wsync();
      for (int i = k + 2 + g; i < NLOC; i += G) {
        const int ri = pko(i);
        const double ai1 = F[ri + k], ai2 = F[ri + k + 1];
        F[ri + k] = (ai1 * a22 - ai2 * a21) * rdet;
        F[ri + k + 1] = (ai2 * a11 - ai1 * a21) * rdet;
      }
      if (g == 0) { piv[k] = 2; piv[k + 1] = 0; }
    }
    wsync();
    k += size;
  }
}

// State chain over x_1..x_N: D_j = S11^(j-1) + S00^(j) - S10^(j-1) D_{j-1}^{-1} S10^(j-1)^T
// (chain index j-1 <-> x_j; S10^(k) couples x_{k+1} (row) and x_k (col)).
__device__ __noinline__ void chain_factor(const Agent& a, Inertia& in) {
  Lds& L = gL;
  const int lane = a.lane;
  if constexpr (NX == 1) {
    double dprev = 0.0;
#pragma unroll 1
    for (int j = 0; j < N; ++j) {
      double d;
      if (kfixed(a, j, NV)) {
        d = 1.0;
      } else {
        d = L.S[j * 3 + 1] + (j + 1 < N ? L.S[(j + 1) * 3] : 0.0);
        if (j > 0) { const double t = L.S[j * 3 + 2]; d -= t * t * dprev; }
      }
      if (fabs(d) <= ZERO_PIVOT) { in.zero++; dprev = 0.0; }
      else { if (d > 0) in.pos++; else in.neg++; dprev = 1.0 / d; }
      if (lane == 0) L.Dinv[j] = dprev;
    }
  } else if constexpr (NX > 1) {
#pragma unroll 1
    for (int j = 0; j < N; ++j) {
      // CW = T_j Dinv_{j-1}   (T_j = S10 of stage j)
      if (j > 0)
        for (int e = lane; e < NXX; e += WAVE) {
          const int r = e / NX, c = e % NX;
          double s = 0.0;
          for (int m = 0; m < NX; ++m) s += L.S[(j * 3 + 2) * NXX + r * NX + m] * L.Dinv[(j - 1) * NXX + m * NX + c];
          L.CW[e] = s;
        }
      wsync();
      for (int e = lane; e < NXX; e += WAVE) {
        const int r = e / NX, c = e % NX;
        double v = L.S[(j * 3 + 1) * NXX + e] + (j + 1 < N ? L.S[((j + 1) * 3) * NXX + e] : 0.0);
        if (j > 0)
          for (int m = 0; m < NX; ++m) v -= L.CW[r * NX + m] * L.S[(j * 3 + 2) * NXX + c * NX + m];
        const bool fr = kfixed(a, j, NV + r), fc = kfixed(a, j, NV + c);
        if (fr || fc) v = (r == c) ? 1.0 : 0.0;
        L.C[e] = v;
      }
      wsync();
      bk_factor<NX, NX>(LDSP(L.C), LDSI(L.cperm), LDSI(L.cpiv), lane, in);
      bk_inverse<NX, NX>(LDSP(L.C), LDSI(L.cperm), LDSI(L.cpiv), LDSP(L.CW), LDSP(L.CY), L.Dinv + j * NXX, lane);
    }
  }
  sync();
}

__device__ __noinline__ void chain_solve(const Agent& a) {
  Lds& L = gL;
  const int lane = a.lane;
  // rhs: rho_j = z1^(j) + z0^(j+1); forward y_j = rho_j - T_j Dinv_{j-1} y_{j-1}
  if constexpr (NX == 1) {
    if (lane == 0) {
      double y = 0.0;
#pragma unroll 1
      for (int j = 0; j < N; ++j) {
        double r = L.zx1[j] + (j + 1 < N ? L.zx0[j + 1] : 0.0);
        if (j > 0) r -= L.S[j * 3 + 2] * L.Dinv[j - 1] * y;
        y = r;
        L.xs[j] = y;
      }
      double x = 0.0;
#pragma unroll 1
      for (int j = N - 1; j >= 0; --j) {
        double r = L.xs[j];
        if (j + 1 < N) r -= L.S[(j + 1) * 3 + 2] * x;
        x = L.Dinv[j] * r;
        L.xs[j] = x;
      }
    }
  } else if constexpr (NX > 1) {
    for (int c = lane; c < NX; c += WAVE) L.xs[c] = L.zx1[c] + (N > 1 ? L.zx0[NX + c] : 0.0);
    wsync();
#pragma unroll 1
    for (int j = 1; j < N; ++j) {
      for (int r = lane; r < NX; r += WAVE) {  // CY = Dinv_{j-1} y_{j-1}
        double s = 0.0;
        for (int m = 0; m < NX; ++m) s += L.Dinv[(j - 1) * NXX + r * NX + m] * L.xs[(j - 1) * NX + m];
        L.CY[r] = s;
      }
      wsync();
      for (int r = lane; r < NX; r += WAVE) {
        double v = L.zx1[j * NX + r] + (j + 1 < N ? L.zx0[(j + 1) * NX + r] : 0.0);
        for (int m = 0; m < NX; ++m) v -= L.S[(j * 3 + 2) * NXX + r * NX + m] * L.CY[m];
        L.xs[j * NX + r] = v;
      }
      wsync();
    }
#pragma unroll 1
    for (int j = N - 1; j >= 0; --j) {
      for (int r = lane; r < NX; r += WAVE) {  // CY = y_j - T_{j+1}^T x_{j+1}
        double v = L.xs[j * NX + r];
        if (j + 1 < N)
          for (int m = 0; m < NX; ++m) v -= L.S[((j + 1) * 3 + 2) * NXX + m * NX + r] * L.xs[(j + 1) * NX + m];
        L.CY[r] = v;
      }
      wsync();
      for (int r = lane; r < NX; r += WAVE) {
        double s = 0.0;
        for (int m = 0; m < NX; ++m) s += L.Dinv[j * NXX + r * NX + m] * L.CY[m];
        L.xs[j * NX + r] = s;
      }
      wsync();
    }
  }
  sync();
}

// Factor the KKT matrix; returns the inertia.
__device__ __noinline__ Inertia factor_chain(const Agent& a, const KKTDiag& kd) {
  Lds& L = gL;
  const int lane = a.lane, g = lane % G, slot = lane / G;
  SPROF_DECL
  kkt_diagonals(a, kd);
  ParLds& P = L.u.p;
  double* F = P.F + slot * PKS;
  int* perm = P.perm + slot * NI;
  int* piv = P.piv + slot * NI;
  Inertia gi{0, 0, 0};
  int bad = 0;
#pragma unroll 1
  for (int r = 0; r < ROUNDS; ++r) {
    const int k = r * SR + slot;
    const bool act = slot < SR && k < N;
    if (act) {
#pragma unroll 2
      for (int t = g; t < PK; t += G) {
        int i = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
        if (pko(i + 1) <= t) ++i;
        if (pko(i) > t) --i;
        F[t] = local_entry(a, k, i, t - pko(i), kd.mode);
      }
      for (int i = g; i < NI; i += G) perm[i] = i;
    }
    wsync();
    SPROF(0);
    if (act) interior_bk(LDSP(F), LDSI(perm), LDSI(piv), g, gi, bad);
    wsync();
    SPROF(1);
    if constexpr (NX > 0) {
      if (wsumi(g == 0 ? bad : 0) > 0) {  // singular stage interior: block chain instead
        if (lane == 0) L.seq = 1;
        sync();
        return seq_factor(a, kd.mode);
      }
    }
    if (act) {
      if (NX > 0) {  // local Schur complement of the two state blocks
        for (int e = g; e < 3 * NXX; e += G) {
          const int blk = e / NXX, rr = (e % NXX) / NX, cc = e % NX;
          int ri, ci;
          if (blk == 0) { ri = NI + rr; ci = NI + cc; }
          else if (blk == 1) { ri = NI + NX + rr; ci = NI + NX + cc; }
          else { ri = NI + NX + rr; ci = NI + cc; }
          L.S[(k * 3 + blk) * NXX + rr * NX + cc] = (ri >= ci) ? F[pko(ri) + ci] : F[pko(ci) + ri];
        }
      }
      if (ROUNDS > 1) {
        for (int t = g; t < PK; t += G) a.lf(k)[t] = F[t];
        for (int i = g; i < NI; i += G) { a.lpv(k)[i] = perm[i]; a.lpv(k)[NI + i] = piv[i]; }
      }
    }
    sync();
    SPROF(2);
  }
  Inertia in{wsumi(g == 0 ? gi.pos : 0), wsumi(g == 0 ? gi.neg : 0), wsumi(g == 0 ? gi.zero : 0)};
  if (lane == 0) L.seq = 0;
  if (NX > 0) chain_factor(a, in);
  sync();
  SPROF(3);
  return in;
}

// Solve with rhs blocks a.rhs(k) ([V, X1, lambda] per stage) -> a.sol(k).
__device__ __noinline__ void solve_chain(const Agent& a, Mode mode) {
  Lds& L = gL;
  (void)mode;
  if (L.seq) { seq_solve(a); return; }
  const int lane = a.lane, g = lane % G, slot = lane / G;
  ParLds& P = L.u.p;
  double* F = P.F + slot * PKS;
  double* z = P.z + slot * NLOC;
  int* perm = P.perm + slot * NI;
  int* piv = P.piv + slot * NI;
  SPROF_DECL
  // forward elimination of every stage interior
#pragma unroll 1
  for (int r = 0; r < ROUNDS; ++r) {
    const int k = r * SR + slot;
    const bool act = slot < SR && k < N;
    if (act) {
      if (ROUNDS > 1) {
        for (int t = g; t < PK; t += G) F[t] = a.lf(k)[t];
        for (int i = g; i < NI; i += G) { perm[i] = a.lpv(k)[i]; piv[i] = a.lpv(k)[NI + i]; }
      }
      wsync();
      const double* rk = a.rhs(k);
      for (int p = g; p < NLOC; p += G) {
        double v;
        if (p < NI) { const int o = perm[p]; v = (o < NV) ? rk[o] : rk[NP + o - NV]; }
        else if (p < NI + NX) v = 0.0;
        else v = rk[NV + p - NI - NX];
        z[p] = v;
      }
      wsync();
#pragma unroll 1
      for (int p = 0; p < NI; ++p) {
        const int pv = piv[p];
        if (pv == 1) {
          const double zp = z[p];
          for (int i = p + 1 + g; i < NLOC; i += G) z[i] -= F[pko(i) + p] * zp;
        } else if (pv == 2) {
          const double z0 = z[p], z1 = z[p + 1];
          for (int i = p + 2 + g; i < NLOC; i += G) { const int ri = pko(i); z[i] -= F[ri + p] * z0 + F[ri + p + 1] * z1; }
        }
        wsync();
      }
      for (int c = g; c < NX; c += G) { L.zx0[k * NX + c] = z[NI + c]; L.zx1[k * NX + c] = z[NI + NX + c]; }
      if (ROUNDS > 1)
        for (int i = g; i < NI; i += G) a.lz(k)[i] = z[i];
    }
    sync();
  }
  SPROF(4);
  if (NX > 0) chain_solve(a);
  // back substitution of every stage interior
#pragma unroll 1
  for (int r = 0; r < ROUNDS; ++r) {
    const int k = r * SR + slot;
    const bool act = slot < SR && k < N;
    if (act) {
      if (ROUNDS > 1) {
        for (int t = g; t < PK; t += G) F[t] = a.lf(k)[t];
        for (int i = g; i < NI; i += G) { perm[i] = a.lpv(k)[i]; piv[i] = a.lpv(k)[NI + i]; z[i] = a.lz(k)[i]; }
        wsync();
      }
      for (int p = g; p < NI; p += G) {
        const int pv = piv[p];
        if (pv == 1) {
          z[p] = z[p] / F[pko(p) + p];
        } else if (pv == 2) {
          const double a11 = F[pko(p) + p], a21 = F[pko(p + 1) + p], a22 = F[pko(p + 1) + p + 1];
          const double det = a11 * a22 - a21 * a21;
          const double z0 = z[p], z1 = z[p + 1];
          z[p] = (a22 * z0 - a21 * z1) / det;
          z[p + 1] = (a11 * z1 - a21 * z0) / det;
        }
      }
      for (int c = g; c < NX; c += G) {
        z[NI + c] = (k > 0) ? L.xs[(k - 1) * NX + c] : 0.0;
        z[NI + NX + c] = L.xs[k * NX + c];
      }
      wsync();
      if (NX > 0)
        for (int i = g; i < NI; i += G) {
          double s = 0.0;
          for (int c = 0; c < 2 * NX; ++c) s += F[pko(NI + c) + i] * z[NI + c];
          z[i] -= s;
        }
      wsync();
#pragma unroll 1
      for (int m = NI - 1; m > 0; --m) {
        const double um = z[m];
        const int skip = (piv[m - 1] == 2) ? m - 1 : -1;
        const int om = pko(m);
        for (int i = g; i < m; i += G)
          if (i != skip) z[i] -= F[om + i] * um;
        wsync();
      }
      double* sk = a.sol(k);
      for (int p = g; p < NI; p += G) {
        const int o = perm[p];
        sk[o < NV ? o : NP + o - NV] = z[p];
      }
      for (int c = g; c < NX; c += G) sk[NV + c] = L.xs[k * NX + c];
    }
  }
  sync();
  SPROF(5);
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
__device__ __noinline__ void ls_multipliers(const Agent& a, const mpcx_options& o, double obj_scale) {
  const int lane = a.lane;
  KKTDiag kd{0.0, 0.0, LSQ};
  const Inertia in = factor_chain(a, kd);
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
  solve_chain(a, LSQ);
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

// Diagnostic build only (-DMPCX_PROFILE): per-phase shader-clock cycles of each
// agent are written to lam_w[agent][0..15] instead of the bound multipliers.
#ifdef MPCX_PROFILE
#define PROF_DECL unsigned long long _pt = __builtin_amdgcn_s_memtime(); double _prof[16] = {0};
#define PROF(i) do { const unsigned long long _n = __builtin_amdgcn_s_memtime(); _prof[i] += (double)(_n - _pt); _pt = _n; } while (0)
#else
#define PROF_DECL
#define PROF(i) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// the kernel: one agent NLP per workgroup (one wavefront)
// ---------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(64, MPCX_MIN_WAVES) mpcx_ipm_solve(Args args) {
  const int agent = blockIdx.x;
  if (agent >= args.n_agents) return;
  Lds& L = gL;
  const mpcx_options& o = args.opt;
  Agent a;
  a.ws = args.ws + (long)agent * args.ws_stride;
  a.p = args.p + (long)agent * NPAR;
  a.lane = threadIdx.x;
  const int lane = a.lane;

  PROF_DECL
#ifdef MPCX_PROFILE
  if (lane < 6) gL.sprof[lane] = 0.0;
  sync();
#endif
  const Scal sc = init_agent(a, args, agent);
  PROF(0);
  const double obj_scale = sc.obj_scale;
  double fx = sc.fx;
  int n_fact = 0, n_ic = 0, n_fallback = 0, n_trials = 0;
  if (M > 0 && o.constr_mult_init_max > 0.0) {
    ls_multipliers(a, o, obj_scale);
    n_fact++;
  }
  PROF(1);

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
    PROF(2);
    eval_hess(a, a.x(), obj_scale);
    sync();
    PROF(3);
    rhs_primal(a, mu, obj_scale);
    PROF(4);
    // factorisation with inertia correction (IPOPT Algorithm IC)
    double dw = 0.0, dc = 0.0;
    bool ok = false;
#pragma unroll 1
    for (int attempt = 0; attempt < 60; ++attempt) {
      KKTDiag kd{dw, dc, NEWTON};
      const Inertia in = factor_chain(a, kd);
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
    PROF(5);
    if (!ok) { status = MPCX_ERROR_IN_STEP; break; }
    rhs_dual(a, mu, dw);
    solve_chain(a, NEWTON);
    PROF(6);
    const StepInfo st = recover_step(a, mu, tau, dw, obj_scale);
    PROF(7);
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
    PROF(8);
    accept_step(a, o, mu, alpha, st.az);
    fx = tr.f;
    eval_gj(a, a.x());
    sync();
    it++;
    PROF(9);
  }

  // ---- outputs ----------------------------------------------------------------
  double* wio = args.w + (long)agent * NW;
  for (int i = lane; i < NW; i += WAVE) {
    wio[i] = a.x()[i];
    if (args.lam_w != nullptr)
      args.lam_w[(long)agent * NW + i] = (i < NX) ? 0.0 : (a.zU()[i] - a.zL()[i]) / obj_scale;
  }
#ifdef MPCX_PROFILE
  PROF(2);
  for (int i = 0; i < 6; ++i) _prof[10 + i] = gL.sprof[i];
  if (args.lam_w != nullptr && lane == 0)
    for (int i = 0; i < 16 && i < NW; ++i) args.lam_w[(long)agent * NW + i] = _prof[i];
#endif
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
