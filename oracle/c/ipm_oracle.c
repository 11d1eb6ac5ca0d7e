/* ORACLE (test infrastructure only) — C restatement of the IPOPT algorithm for
 * stage-structured MPC NLPs, used as the all-cores CPU baseline
 * and cross-checked against oracle/ipm.py.
 *
 * The IPM is generic over a stage-model interface (model_t: dimensions + stage
 * functions).  Two models plug into it: the hand-derived one_room model below (the
 * independent checker of the C3 fleet), and, for the CPU baselines of the other
 * configurations, a generated model compiled for the host (oracle/c/gen_model.cpp,
 * oracle/cbuild.py: build_generated) — the CasADi-codegen + IPOPT analogue.
 *
 * Algorithm: IPOPT (Waechter & Biegler 2006) exactly as oracle/ipm.py restates it
 * (reference solver call: agentlib_mpc/data_structures/casadi_utils.py:191-217,
 * optimization_backends/casadi_/core/discretization.py:203).  The KKT system is
 * solved with a structure-exploiting block-tridiagonal LDL^T (Bunch-Kaufman on
 * each stage block, Riccati-style Schur complement through the state), which is
 * what an efficient CPU implementation (fatrop-like) does; one agent per OpenMP
 * thread.
 *
 * The model functions are hand-derived for the one_room model
 * (examples/one_room_mpc/physical/simple_mpc.py:98-138) transcribed by
 * direct collocation (optimization_backends/casadi_/full.py:36-98,
 * basic.py:251-392): no dependency on the product's code generator.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "ipm_oracle.h"

#define MAXD 9
#define MAXNB 160
#define MAXNX 8

/* --------------------------------------------------------------------------
 * one_room collocation stage (d collocation points)
 * local L = [X0, u, (T_j, Z_j, Y_j)_{j=1..d}, X1]; PS = (T_in, load, T_upper)_j
 * PG = [T0, u_prev, cp, C, s_T, r_mDot]
 * g = [cont, (col_j, path_j, out_j)_j]
 * -------------------------------------------------------------------------- */
typedef struct {
  int N, d, nx, nv, ng, nps, npg;
  double ts;
  double B[MAXD + 1], C[MAXD + 1][MAXD + 1], D[MAXD + 1];
} room_t;

static void room_fg(const room_t* m, const double* L, const double* PS, const double* PG,
                    double* f, double* g) {
  const int d = m->d;
  const double ts = m->ts, cp = PG[2], Cz = PG[3], sT = PG[4], r = PG[5];
  const double X0 = L[0], u = L[1], X1 = L[2 + 3 * d];
  double fk = 0.0, xe = m->D[0] * X0;
  for (int j = 0; j < d; ++j) {
    const double Z = L[2 + 3 * j + 1];
    fk += m->B[j + 1] * (r * u + sT * Z * Z) * ts;
    xe += m->D[j + 1] * L[2 + 3 * j];
  }
  *f = fk;
  g[0] = X1 - xe;
  for (int j = 0; j < d; ++j) {
    const double T = L[2 + 3 * j], Z = L[2 + 3 * j + 1], Y = L[2 + 3 * j + 2];
    double xp = m->C[0][j + 1] * X0;
    for (int q = 0; q < d; ++q) xp += m->C[q + 1][j + 1] * L[2 + 3 * q];
    const double ode = cp * u / Cz * (PS[3 * j] - T) + PS[3 * j + 1] / Cz;
    g[1 + 3 * j] = ts * ode - xp;
    g[2 + 3 * j] = T + Z;
    g[3 + 3 * j] = Y - T;
  }
}

static void room_bounds(const room_t* m, const double* PS, double* lb, double* ub) {
  for (int i = 0; i < m->ng; ++i) lb[i] = ub[i] = 0.0;
  for (int j = 0; j < m->d; ++j) ub[2 + 3 * j] = PS[3 * j + 2];
}

/* gradient (nl) and dense jacobian (ng x nl) */
static void room_gj(const room_t* m, const double* L, const double* PS, const double* PG,
                    double* grad, double* jac) {
  const int d = m->d, nl = 2 * m->nx + m->nv;
  const double ts = m->ts, cp = PG[2], Cz = PG[3], sT = PG[4], r = PG[5];
  const double u = L[1];
  memset(grad, 0, sizeof(double) * nl);
  memset(jac, 0, sizeof(double) * m->ng * nl);
  for (int j = 0; j < d; ++j) {
    grad[1] += m->B[j + 1] * r * ts;
    grad[2 + 3 * j + 1] = m->B[j + 1] * 2.0 * sT * L[2 + 3 * j + 1] * ts;
  }
  jac[0 * nl + nl - 1] = 1.0;
  jac[0 * nl + 0] = -m->D[0];
  for (int j = 0; j < d; ++j) jac[0 * nl + 2 + 3 * j] = -m->D[j + 1];
  for (int j = 0; j < d; ++j) {
    double* row = jac + (1 + 3 * j) * nl;
    const double T = L[2 + 3 * j];
    row[1] = ts * cp / Cz * (PS[3 * j] - T);
    row[0] = -m->C[0][j + 1];
    for (int q = 0; q < d; ++q) row[2 + 3 * q] = -m->C[q + 1][j + 1];
    row[2 + 3 * j] += -ts * cp * u / Cz;
    row = jac + (2 + 3 * j) * nl;
    row[2 + 3 * j] = 1.0;
    row[2 + 3 * j + 1] = 1.0;
    row = jac + (3 + 3 * j) * nl;
    row[2 + 3 * j + 2] = 1.0;
    row[2 + 3 * j] = -1.0;
  }
}

static void room_hess(const room_t* m, const double* L, const double* PS, const double* PG,
                      double sigma, const double* lam, double* H) {
  const int d = m->d, nl = 2 * m->nx + m->nv;
  const double ts = m->ts, cp = PG[2], Cz = PG[3], sT = PG[4];
  (void)L; (void)PS;
  memset(H, 0, sizeof(double) * nl * nl);
  for (int j = 0; j < d; ++j) {
    const int z = 2 + 3 * j + 1, t = 2 + 3 * j;
    H[z * nl + z] = sigma * m->B[j + 1] * 2.0 * sT * ts;
    const double c = lam[1 + 3 * j] * (-ts * cp / Cz);
    H[1 * nl + t] += c;
    H[t * nl + 1] += c;
  }
}

static void room_fg_m(const model_t* mm, const double* L, const double* PS, const double* PG, double TK, double* f,
                      double* g) {
  (void)TK;
  room_fg((const room_t*)mm->data, L, PS, PG, f, g);
}
static void room_gj_m(const model_t* mm, const double* L, const double* PS, const double* PG, double TK, double* grad,
                      double* jac) {
  (void)TK;
  room_gj((const room_t*)mm->data, L, PS, PG, grad, jac);
}
static void room_hess_m(const model_t* mm, const double* L, const double* PS, const double* PG, double TK,
                        double sigma, const double* lam, double* H) {
  (void)TK;
  room_hess((const room_t*)mm->data, L, PS, PG, sigma, lam, H);
}
static void room_bounds_m(const model_t* mm, const double* PS, const double* PG, double TK, double* lb, double* ub) {
  (void)PG; (void)TK;
  room_bounds((const room_t*)mm->data, PS, lb, ub);
}

void oracle_room_init(room_t* m, int N, int d, double ts, const double* B, const double* Cm,
                      const double* D) {
  m->N = N; m->d = d; m->nx = 1; m->nv = 1 + 3 * d; m->ng = 1 + 3 * d;
  m->nps = 3 * d; m->npg = 6; m->ts = ts;
  for (int i = 0; i <= d; ++i) {
    m->B[i] = B[i];
    m->D[i] = D[i];
    for (int j = 0; j <= d; ++j) m->C[i][j] = Cm[i * (d + 1) + j];
  }
}

/* --------------------------------------------------------------------------
 * IPM
 * -------------------------------------------------------------------------- */
typedef struct {
  int pos, neg, zero;
} inertia_t;

#define ZERO_PIVOT 1e-20

/* Bunch-Kaufman LDL^T in place (full symmetric n x n, row-major ld) */
static void bk_factor(double* A, int n, int ld, int* perm, int* piv, inertia_t* in) {
  const double alpha = 0.6403882032022076;
  for (int i = 0; i < n; ++i) perm[i] = i;
  int k = 0;
  while (k < n) {
    const double akk = fabs(A[k * ld + k]);
    double lam = 0.0;
    int r = -1;
    for (int i = k + 1; i < n; ++i) {
      const double t = fabs(A[i * ld + k]);
      if (t > lam) { lam = t; r = i; }
    }
    int size = 1, kp = k;
    if (fmax(akk, lam) == 0.0 || akk >= alpha * lam) {
      size = 1; kp = k;
    } else {
      double sigma = 0.0;
      for (int j = k; j < n; ++j)
        if (j != r) sigma = fmax(sigma, fabs(A[r * ld + j]));
      if (akk * sigma >= alpha * lam * lam) { size = 1; kp = k; }
      else if (fabs(A[r * ld + r]) >= alpha * sigma) { size = 1; kp = r; }
      else { size = 2; kp = r; }
    }
    const int kk = k + size - 1;
    if (kp != kk) {
      for (int j = 0; j < n; ++j) { double t = A[kp * ld + j]; A[kp * ld + j] = A[kk * ld + j]; A[kk * ld + j] = t; }
      for (int i = 0; i < n; ++i) { double t = A[i * ld + kp]; A[i * ld + kp] = A[i * ld + kk]; A[i * ld + kk] = t; }
      int t = perm[kp]; perm[kp] = perm[kk]; perm[kk] = t;
    }
    if (size == 1) {
      const double dv = A[k * ld + k];
      if (fabs(dv) <= ZERO_PIVOT) {
        in->zero++;
        for (int i = k + 1; i < n; ++i) A[i * ld + k] = 0.0;
      } else {
        if (dv > 0) in->pos++; else in->neg++;
        const double rd = 1.0 / dv;
        for (int i = k + 1; i < n; ++i) {
          const double aik = A[i * ld + k] * rd;
          for (int j = k + 1; j < n; ++j) A[i * ld + j] -= aik * A[j * ld + k];
        }
        for (int i = k + 1; i < n; ++i) A[i * ld + k] *= rd;
      }
      piv[k] = 1;
    } else {
      const double a11 = A[k * ld + k], a21 = A[(k + 1) * ld + k], a22 = A[(k + 1) * ld + k + 1];
      const double det = a11 * a22 - a21 * a21;
      if (fabs(det) <= 1e-40) in->zero += 2;
      else if (det < 0) { in->pos++; in->neg++; }
      else if (a11 + a22 > 0) in->pos += 2;
      else in->neg += 2;
      const double rdet = 1.0 / det;
      for (int i = k + 2; i < n; ++i) {
        const double ai1 = A[i * ld + k], ai2 = A[i * ld + k + 1];
        const double l1 = (ai1 * a22 - ai2 * a21) * rdet, l2 = (ai2 * a11 - ai1 * a21) * rdet;
        for (int j = k + 2; j < n; ++j) A[i * ld + j] -= l1 * A[j * ld + k] + l2 * A[j * ld + k + 1];
      }
      for (int i = k + 2; i < n; ++i) {
        const double ai1 = A[i * ld + k], ai2 = A[i * ld + k + 1];
        A[i * ld + k] = (ai1 * a22 - ai2 * a21) * rdet;
        A[i * ld + k + 1] = (ai2 * a11 - ai1 * a21) * rdet;
      }
      piv[k] = 2; piv[k + 1] = 0;
    }
    k += size;
  }
}

static void bk_solve(const double* F, int n, int ld, const int* perm, const int* piv, double* v) {
  double y[MAXNB];
  for (int i = 0; i < n; ++i) y[i] = v[perm[i]];
  for (int k = 0; k < n;) {
    if (piv[k] == 1) {
      for (int i = k + 1; i < n; ++i) y[i] -= F[i * ld + k] * y[k];
      k += 1;
    } else {
      for (int i = k + 2; i < n; ++i) y[i] -= F[i * ld + k] * y[k] + F[i * ld + k + 1] * y[k + 1];
      k += 2;
    }
  }
  for (int i = 0; i < n; ++i) {
    if (piv[i] == 1) {
      y[i] = F[i * ld + i] != 0.0 ? y[i] / F[i * ld + i] : 0.0;
    } else if (piv[i] == 2) {
      const double a11 = F[i * ld + i], a21 = F[(i + 1) * ld + i], a22 = F[(i + 1) * ld + i + 1];
      const double det = a11 * a22 - a21 * a21, y0 = y[i], y1 = y[i + 1];
      y[i] = (a22 * y0 - a21 * y1) / det;
      y[i + 1] = (a11 * y1 - a21 * y0) / det;
    }
  }
  for (int k = n - 1; k >= 0;) {
    const int start = piv[k] == 0 ? k - 1 : k;
    for (int j = 0; j < start; ++j) {
      y[j] -= F[start * ld + j] * y[start];
      if (start < k) y[j] -= F[(start + 1) * ld + j] * y[start + 1];
    }
    k = start - 1;
  }
  for (int i = 0; i < n; ++i) v[perm[i]] = y[i];
}

/* per-agent solver state */
typedef struct {
  const model_t* m;
  int N, NX, NV, NG, NL, NP, NB, NW, M;
  const double *p;
  double *x, *s, *lam, *zL, *zU, *vL, *vU, *xL, *xU, *sL, *sU, *gs, *gv, *lb, *ub;
  double *dx, *ds, *dl, *xt, *st, *gt, *sdg, *sdj, *sdh, *fac, *rhs, *sol;
  double *lt, *zLt, *zUt, *vLt, *vUt, *rhs0, *sol0, *res, *kb;  /* soft step trial, refinement */
  int *perm, *piv;
  double obj_scale;
} ws_t;

static int fixedv(const ws_t* w, int i) { return w->xL[i] == w->xU[i]; }
static int isfin(double v) { return fabs(v) < INFINITY; }

static double eval_fg(ws_t* w, const double* xv, double* gout) {
  double f = 0.0;
  for (int k = 0; k < w->N; ++k) {
    double fk = 0.0;
    w->m->fg(w->m, xv + k * w->NP, w->p + w->m->npg + k * w->m->nps, w->p, k * w->m->ts, &fk, gout + k * w->NG);
    f += fk;
  }
  return f;
}
static void eval_gj(ws_t* w, const double* xv) {
  memset(w->sdg, 0, sizeof(double) * w->N * w->NL);
  memset(w->sdj, 0, sizeof(double) * w->N * w->NG * w->NL);
  for (int k = 0; k < w->N; ++k)
    w->m->gj(w->m, xv + k * w->NP, w->p + w->m->npg + k * w->m->nps, w->p, k * w->m->ts, w->sdg + k * w->NL,
             w->sdj + k * w->NG * w->NL);
}
static void eval_hess(ws_t* w, const double* xv, double sigma) {
  double lk[MAXNB];
  memset(w->sdh, 0, sizeof(double) * w->N * w->NL * w->NL);
  for (int k = 0; k < w->N; ++k) {
    for (int r = 0; r < w->NG; ++r) lk[r] = w->lam[k * w->NG + r] * w->gs[k * w->NG + r];
    w->m->hess(w->m, xv + k * w->NP, w->p + w->m->npg + k * w->m->nps, w->p, k * w->m->ts, sigma, lk,
               w->sdh + k * w->NL * w->NL);
  }
}
static double acc_grad(const ws_t* w, int i) {
  const int b = (i - w->NX) / w->NP, off = (i - w->NX) % w->NP;
  double v = w->sdg[b * w->NL + w->NX + off];
  if (w->NX > 0 && off >= w->NV && b + 1 < w->N) v += w->sdg[(b + 1) * w->NL + off - w->NV];
  return v;
}
static double acc_jtl(const ws_t* w, int i, const double* lamv) {
  const int b = (i - w->NX) / w->NP, off = (i - w->NX) % w->NP;
  double v = 0.0;
  for (int r = 0; r < w->NG; ++r)
    v += w->sdj[(b * w->NG + r) * w->NL + w->NX + off] * w->gs[b * w->NG + r] * lamv[b * w->NG + r];
  if (w->NX > 0 && off >= w->NV && b + 1 < w->N)
    for (int r = 0; r < w->NG; ++r)
      v += w->sdj[((b + 1) * w->NG + r) * w->NL + off - w->NV] * w->gs[(b + 1) * w->NG + r] *
           lamv[(b + 1) * w->NG + r];
  return v;
}
static int ccls(const ws_t* w, int c) {
  if (w->lb[c] == w->ub[c]) return 0;
  if (!isfin(w->sL[c]) && !isfin(w->sU[c])) return 2;
  return 1;
}
static double sigma_x(const ws_t* w, int i) {
  double s = 0.0;
  if (fixedv(w, i)) return 0.0;
  if (isfin(w->xL[i])) s += w->zL[i] / (w->x[i] - w->xL[i]);
  if (isfin(w->xU[i])) s += w->zU[i] / (w->xU[i] - w->x[i]);
  return s;
}
static double sigma_s(const ws_t* w, int c) {
  double s = 0.0;
  if (isfin(w->sL[c])) s += w->vL[c] / (w->s[c] - w->sL[c]);
  if (isfin(w->sU[c])) s += w->vU[c] / (w->sU[c] - w->s[c]);
  return s;
}

/* coupling of block k to x_k */
static double coupling(const ws_t* w, int k, int row, int c, int lsq) {
  if (fixedv(w, k * w->NP + c)) return 0.0;
  if (row < w->NP) {
    if (lsq || fixedv(w, w->NX + k * w->NP + row)) return 0.0;
    return w->sdh[k * w->NL * w->NL + (w->NX + row) * w->NL + c];
  }
  const int r = row - w->NP;
  return w->gs[k * w->NG + r] * w->sdj[(k * w->NG + r) * w->NL + c];
}

/* KKT block k = [V_k, X_{k+1}, lambda_k] before the Schur update (row-major, ld NB) */
static void kkt_block(const ws_t* w, int k, double dw, double dc, int lsq, double* A) {
  const int NB = w->NB, NP = w->NP, NV = w->NV, NX = w->NX, NG = w->NG, NL = w->NL, N = w->N;
  const int w0 = NX + k * NP;
  for (int p = 0; p < NP; ++p)
    for (int q = 0; q < NP; ++q) {
      double val;
      if (fixedv(w, w0 + p) || fixedv(w, w0 + q)) val = p == q ? 1.0 : 0.0;
      else if (lsq) val = p == q ? 1.0 : 0.0;
      else {
        val = w->sdh[k * NL * NL + (NX + p) * NL + NX + q];
        if (NX > 0 && p >= NV && q >= NV && k + 1 < N) val += w->sdh[(k + 1) * NL * NL + (p - NV) * NL + q - NV];
        if (p == q) val += sigma_x(w, w0 + p) + dw;
      }
      A[p * NB + q] = val;
    }
  for (int r = 0; r < NG; ++r)
    for (int q = 0; q < NP; ++q) {
      const double val = fixedv(w, w0 + q) ? 0.0 : w->gs[k * NG + r] * w->sdj[(k * NG + r) * NL + NX + q];
      A[(NP + r) * NB + q] = val;
      A[q * NB + NP + r] = val;
    }
  for (int r = 0; r < NG; ++r)
    for (int c = 0; c < NG; ++c) {
      double dd = 0.0;
      if (r == c) {
        const int cc = k * NG + r, cl = ccls(w, cc);
        if (lsq) dd = cl == 0 ? 0.0 : 1.0;
        else if (cl == 0) dd = dc;
        else if (cl == 2) dd = 1.0;
        else dd = 1.0 / (sigma_s(w, cc) + dw) + dc;
      }
      A[(NP + r) * NB + NP + c] = -dd;
    }
}

static inertia_t factor_chain(ws_t* w, double dw, double dc, int lsq) {
  const int NB = w->NB, NV = w->NV, NX = w->NX, N = w->N;
  inertia_t in = {0, 0, 0};
  double P[MAXNX * MAXNX], Bm[MAXNB * MAXNX], v[MAXNB];
  for (int k = 0; k < N; ++k) {
    double* A = w->fac + k * NB * NB;
    kkt_block(w, k, dw, dc, lsq, A);
    if (NX > 0 && k > 0) {
      for (int i = 0; i < NB; ++i)
        for (int c = 0; c < NX; ++c) Bm[i * NX + c] = coupling(w, k, i, c, lsq);
      for (int i = 0; i < NB; ++i)
        for (int j = 0; j < NB; ++j) {
          double s = 0.0;
          for (int c = 0; c < NX; ++c)
            for (int e = 0; e < NX; ++e) s += Bm[i * NX + c] * P[c * NX + e] * Bm[j * NX + e];
          A[i * NB + j] -= s;
        }
    }
    bk_factor(A, NB, NB, w->perm + k * NB, w->piv + k * NB, &in);
    if (NX > 0 && k + 1 < N) {
      for (int c = 0; c < NX; ++c) {
        for (int i = 0; i < NB; ++i) v[i] = i == NV + c ? 1.0 : 0.0;
        bk_solve(A, NB, NB, w->perm + k * NB, w->piv + k * NB, v);
        for (int e = 0; e < NX; ++e) P[e * NX + c] = v[NV + e];
      }
    }
  }
  return in;
}

static void solve_chain(ws_t* w, int lsq) {
  const int NB = w->NB, NV = w->NV, NX = w->NX, N = w->N;
  double v[MAXNB];
  for (int k = 0; k < N; ++k) {
    for (int i = 0; i < NB; ++i) v[i] = w->rhs[k * NB + i];
    if (NX > 0 && k > 0)
      for (int i = 0; i < NB; ++i)
        for (int c = 0; c < NX; ++c) v[i] -= coupling(w, k, i, c, lsq) * w->sol[(k - 1) * NB + NV + c];
    bk_solve(w->fac + k * NB * NB, NB, NB, w->perm + k * NB, w->piv + k * NB, v);
    memcpy(w->sol + k * NB, v, sizeof(double) * NB);
  }
  if (NX > 0)
    for (int k = N - 2; k >= 0; --k) {
      for (int i = 0; i < NB; ++i) v[i] = 0.0;
      for (int c = 0; c < NX; ++c) {
        double s = 0.0;
        for (int i = 0; i < NB; ++i) s += coupling(w, k + 1, i, c, lsq) * w->sol[(k + 1) * NB + i];
        v[NV + c] = s;
      }
      bk_solve(w->fac + k * NB * NB, NB, NB, w->perm + k * NB, w->piv + k * NB, v);
      for (int i = 0; i < NB; ++i) w->sol[k * NB + i] -= v[i];
    }
}

/* out = K sol (the unfactored KKT matrix, block order; Newton mode) */
static void kkt_matvec(const ws_t* w, double dw, double dc, const double* sol, double* out) {
  const int NB = w->NB, NV = w->NV, NX = w->NX, N = w->N;
  double* A = w->kb;
  memset(out, 0, sizeof(double) * N * NB);
  for (int k = 0; k < N; ++k) {
    kkt_block(w, k, dw, dc, 0, A);
    for (int i = 0; i < NB; ++i) {
      double s = 0.0;
      for (int j = 0; j < NB; ++j) s += A[i * NB + j] * sol[k * NB + j];
      out[k * NB + i] += s;
    }
    if (NX > 0 && k > 0)
      for (int i = 0; i < NB; ++i)
        for (int c = 0; c < NX; ++c) {
          const double b = coupling(w, k, i, c, 0);
          out[k * NB + i] += b * sol[(k - 1) * NB + NV + c];
          out[(k - 1) * NB + NV + c] += b * sol[k * NB + i];
        }
  }
}

static double amax_abs(const double* v, int n) {
  double m = 0.0;
  for (int i = 0; i < n; ++i) m = fmax(m, fabs(v[i]));
  return m;
}

/* IPOPT PDFullSpaceSolver::Solve's iterative refinement of w->sol (rhs w->rhs): at least one
   correction, more while the residual ratio exceeds 1e-10, at most 10, stopping when a step
   does not improve the ratio (oracle/ipm.py _refine).  Returns the corrections made. */
static int refine(ws_t* w, double dw, double dc) {
  const int n = w->N * w->NB;
  memcpy(w->rhs0, w->rhs, sizeof(double) * n);
  const double nr = amax_abs(w->rhs0, n);
#define RATIO(res_, x_) ((nr + amax_abs(x_, n) > 0) ? amax_abs(res_, n) / (fmin(amax_abs(x_, n), 1e6 * nr) + nr) : 0.0)
  kkt_matvec(w, dw, dc, w->sol, w->res);
  for (int i = 0; i < n; ++i) w->res[i] = w->rhs0[i] - w->res[i];
  double rr = RATIO(w->res, w->sol), old;
  int steps = 0;
  while (steps < 1 || rr > 1e-10) {
    memcpy(w->sol0, w->sol, sizeof(double) * n);
    memcpy(w->rhs, w->res, sizeof(double) * n);
    solve_chain(w, 0);
    for (int i = 0; i < n; ++i) w->sol[i] += w->sol0[i];
    kkt_matvec(w, dw, dc, w->sol, w->res);
    for (int i = 0; i < n; ++i) w->res[i] = w->rhs0[i] - w->res[i];
    old = rr;
    rr = RATIO(w->res, w->sol);
    steps++;
    if (rr > 1e-10 && steps > 1 && (steps > 10 || rr > old)) break;
  }
#undef RATIO
  memcpy(w->rhs, w->rhs0, sizeof(double) * n);
  return steps;
}

static double theta_of(const ws_t* w, const double* gval, const double* sv) {
  double t = 0.0;
  for (int c = 0; c < w->M; ++c)
    t += fabs(ccls(w, c) == 0 ? gval[c] - w->gs[c] * w->lb[c] : gval[c] - sv[c]);
  return t;
}
static double barrier_of(const ws_t* w, const double* xv, const double* sv) {
  double t = 0.0;
  for (int i = w->NX; i < w->NW; ++i) {
    if (fixedv(w, i)) continue;
    if (isfin(w->xL[i])) t += log(xv[i] - w->xL[i]);
    if (isfin(w->xU[i])) t += log(w->xU[i] - xv[i]);
  }
  for (int c = 0; c < w->M; ++c) {
    if (ccls(w, c) != 1) continue;
    if (isfin(w->sL[c])) t += log(sv[c] - w->sL[c]);
    if (isfin(w->sU[c])) t += log(w->sU[c] - sv[c]);
  }
  return t;
}
/* scaled optimality error; unscaled dual infeasibility (x and slack parts), constraint
   violation (|c| and the violation of the relaxed bounds of d) and complementarity as IPOPT's
   unscaled_curr_* quantities */
static double opt_error(const ws_t* w, double mu, double* dual_u, double* viol_u, double* compl_) {
  double dmax = 0, du = 0, pmax = 0, pu = 0, cmax = 0, lsum = 0, zsum = 0;
  int nz = 0;
  for (int i = w->NX; i < w->NW; ++i) {
    if (fixedv(w, i)) continue;
    const double rd = w->obj_scale * acc_grad(w, i) + acc_jtl(w, i, w->lam) - w->zL[i] + w->zU[i];
    dmax = fmax(dmax, fabs(rd));
    du = fmax(du, fabs(rd) / w->obj_scale);
    if (isfin(w->xL[i])) { cmax = fmax(cmax, fabs((w->x[i] - w->xL[i]) * w->zL[i] - mu)); zsum += fabs(w->zL[i]); nz++; }
    if (isfin(w->xU[i])) { cmax = fmax(cmax, fabs((w->xU[i] - w->x[i]) * w->zU[i] - mu)); zsum += fabs(w->zU[i]); nz++; }
  }
  for (int c = 0; c < w->M; ++c) {
    const int cl = ccls(w, c);
    double cv, vv = 0.0;
    if (cl == 0) { cv = w->gv[c] - w->gs[c] * w->lb[c]; vv = fabs(cv); }
    else {
      cv = w->gv[c] - w->s[c];
      if (cl == 1) {
        const double rs = -w->lam[c] - w->vL[c] + w->vU[c];
        dmax = fmax(dmax, fabs(rs));
        du = fmax(du, fabs(rs) * w->gs[c] / w->obj_scale);
        vv = fmax(0.0, fmax(w->sL[c] - w->gv[c], w->gv[c] - w->sU[c]));
        if (isfin(w->sL[c])) { cmax = fmax(cmax, fabs((w->s[c] - w->sL[c]) * w->vL[c] - mu)); zsum += fabs(w->vL[c]); nz++; }
        if (isfin(w->sU[c])) { cmax = fmax(cmax, fabs((w->sU[c] - w->s[c]) * w->vU[c] - mu)); zsum += fabs(w->vU[c]); nz++; }
      }
    }
    pmax = fmax(pmax, fabs(cv));
    pu = fmax(pu, vv / w->gs[c]);
    lsum += fabs(w->lam[c]);
  }
  const double s_d = fmax(100.0, (lsum + zsum) / fmax(1.0, (double)(w->M + nz))) / 100.0;
  const double s_c = nz > 0 ? fmax(100.0, zsum / nz) / 100.0 : 1.0;
  if (dual_u) *dual_u = du;
  if (viol_u) *viol_u = pu;
  if (compl_) *compl_ = cmax / w->obj_scale;
  return fmax(fmax(dmax / s_d, pmax), cmax / s_c);
}
/* IPOPT primal_dual_system_error at (x, s, lam, z, v) with the derivatives in sdg / sdj and the
   scaled constraint values gval: 1-norms of the dual infeasibility, the constraint violation
   and the mu-complementarity (the normalisation cancels in the soft-restoration ratio) */
static double pd_error(const ws_t* w, const double* xv, const double* sv, const double* lamv, const double* zl,
                       const double* zu, const double* vl, const double* vu, const double* gval, double mu) {
  double e = 0.0;
  for (int i = w->NX; i < w->NW; ++i) {
    if (fixedv(w, i)) continue;
    e += fabs(w->obj_scale * acc_grad(w, i) + acc_jtl(w, i, lamv) - zl[i] + zu[i]);
    if (isfin(w->xL[i])) e += fabs((xv[i] - w->xL[i]) * zl[i] - mu);
    if (isfin(w->xU[i])) e += fabs((w->xU[i] - xv[i]) * zu[i] - mu);
  }
  for (int c = 0; c < w->M; ++c) {
    const int cl = ccls(w, c);
    e += fabs(cl == 0 ? gval[c] - w->gs[c] * w->lb[c] : gval[c] - sv[c]);
    if (cl == 1) {
      e += fabs(-lamv[c] - vl[c] + vu[c]);
      if (isfin(w->sL[c])) e += fabs((sv[c] - w->sL[c]) * vl[c] - mu);
      if (isfin(w->sU[c])) e += fabs((w->sU[c] - sv[c]) * vu[c] - mu);
    }
  }
  return e;
}
/* IPOPT OptimalityErrorConvergenceCheck::CurrentIsAcceptable (objective change between the
   last two iterations it was called at; initially -1e50) */
typedef struct { double curr_f, last_f; int last_it, count; } acc_t;
static int current_is_acceptable(acc_t* ac, const opts_t* o, int square, double err, double du,
                                 double viol, double cmpl, double fx, int it) {
  if (it != ac->last_it) { ac->last_f = ac->curr_f; ac->curr_f = fx; ac->last_it = it; }
  if (square) return err <= o->acceptable_tol && viol <= o->acceptable_constr_viol_tol;
  return err <= o->acceptable_tol && du <= o->acceptable_dual_inf_tol && viol <= o->acceptable_constr_viol_tol &&
         cmpl <= o->acceptable_compl_inf_tol &&
         fabs(ac->curr_f - ac->last_f) / fmax(1.0, fabs(ac->curr_f)) <= o->acceptable_obj_change_tol;
}

static double push_into(double v, double lo, double hi) {
  const int hl = isfin(lo), hu = isfin(hi);
  double pl = hl ? 1e-2 * fmax(1.0, fabs(lo)) : 0.0, pu = hu ? 1e-2 * fmax(1.0, fabs(hi)) : 0.0;
  if (hl && hu) { pl = fmin(pl, 1e-2 * (hi - lo)); pu = fmin(pu, 1e-2 * (hi - lo)); }
  const double lop = hl ? lo + pl : -INFINITY, hip = hu ? hi - pu : INFINITY;
  if (hl && hu && lop > hip) return 0.5 * (lo + hi);
  return fmin(fmax(v, lop), hip);
}

/* ---- filter (IPOPT Filter): one cap shared with the kernel (MAXF + FSPILL) and oracle/ipm.py ---- */
#define MAXF 1024
typedef struct { double th[MAXF], ph[MAXF]; int n, over, maxn; } filter_t;
static int filter_accepts(const filter_t* f, double th, double ph) {
  for (int j = 0; j < f->n; ++j)
    if (th >= f->th[j] && ph >= f->ph[j]) return 0;
  return 1;
}
/* Filter::AddEntry of (theta, phi) with IPOPT's margins: the entries it dominates go, a full
   filter drops its oldest entry (counted) */
static void filter_add(filter_t* f, double theta, double phi) {
  const double th = (1 - 1e-5) * theta, ph = phi - 1e-8 * theta;
  int k = 0;
  for (int j = 0; j < f->n; ++j)
    if (!(th <= f->th[j] && ph <= f->ph[j])) { f->th[k] = f->th[j]; f->ph[k] = f->ph[j]; k++; }
  f->n = k;
  if (f->n >= MAXF) {
    for (int j = 1; j < f->n; ++j) { f->th[j - 1] = f->th[j]; f->ph[j - 1] = f->ph[j]; }
    f->n--;
    f->over++;
  }
  f->th[f->n] = th; f->ph[f->n] = ph; f->n++;
  if (f->n > f->maxn) f->maxn = f->n;
}

/* ---- the restoration NLP (IPOPT RestoIpoptNLP, oracle/ipm.py _RestoNLP) as a stage model:
   per stage L' = [X0, V, p (ng), n (ng), X1] over the SCALED original constraints:
     min rho sum(p + n) + zeta/2 ||D_R (x - x_R)||^2   s.t.  c~(x) - p + n in [bounds],  p, n >= 0 */
typedef struct {
  const model_t* m;           /* the original stage model */
  const double *gs, *xR, *dr2;  /* outer constraint scaling [M], x at the start [NW], weights */
  double rho, zeta;
  double *Lo, *go, *jo, *Ho, *lo;  /* scratch of the original model's stage calls */
  int* map;
} resto_t;

static int resto_stage(const model_t* mm, double TK) { return mm->ts > 0 ? (int)lround(TK / mm->ts) : 0; }
static void resto_split(const model_t* m, const double* L, double* Lo) {
  const int nx = m->nx, nv = m->nv, ng = m->ng;
  for (int i = 0; i < nx + nv; ++i) Lo[i] = L[i];
  for (int c = 0; c < nx; ++c) Lo[nx + nv + c] = L[nx + nv + 2 * ng + c];
}
/* index of stage-local primal j (V then X1) in the outer NLP vector */
static double resto_prox(const resto_t* d, int k, const double* L, double* grad) {
  const model_t* m = d->m;
  const int nx = m->nx, nv = m->nv, ng = m->ng, np = nv + nx;
  double f = 0.0;
  for (int j = 0; j < np; ++j) {
    const int li = j < nv ? nx + j : nx + nv + 2 * ng + (j - nv), gi = nx + k * np + j;
    const double dv = L[li] - d->xR[gi];
    f += 0.5 * d->zeta * d->dr2[gi] * dv * dv;
    if (grad) grad[li] = d->zeta * d->dr2[gi] * dv;
  }
  return f;
}
static void resto_fg(const model_t* mm, const double* L, const double* PS, const double* PG, double TK, double* f,
                     double* g) {
  const resto_t* d = (const resto_t*)mm->data;
  const model_t* m = d->m;
  const int k = resto_stage(mm, TK), nx = m->nx, nv = m->nv, ng = m->ng;
  double* Lo = d->Lo;
  double fo;
  resto_split(m, L, Lo);
  m->fg(m, Lo, PS, PG, TK, &fo, g);
  double fk = 0.0;
  for (int r = 0; r < ng; ++r) {
    const double pv = L[nx + nv + r], nvv = L[nx + nv + ng + r];
    g[r] = d->gs[k * ng + r] * g[r] - pv + nvv;
    fk += d->rho * (pv + nvv);
  }
  *f = fk + resto_prox(d, k, L, 0);
}
static void resto_gj(const model_t* mm, const double* L, const double* PS, const double* PG, double TK, double* grad,
                     double* jac) {
  const resto_t* d = (const resto_t*)mm->data;
  const model_t* m = d->m;
  const int k = resto_stage(mm, TK), nx = m->nx, nv = m->nv, ng = m->ng;
  const int nl = 2 * nx + nv, nlr = nl + 2 * ng;
  double *Lo = d->Lo, *go = d->go, *jo = d->jo;
  resto_split(m, L, Lo);
  memset(go, 0, sizeof(double) * nl);
  memset(jo, 0, sizeof(double) * ng * nl);
  m->gj(m, Lo, PS, PG, TK, go, jo);
  resto_prox(d, k, L, grad);
  for (int r = 0; r < ng; ++r) {
    grad[nx + nv + r] = d->rho;
    grad[nx + nv + ng + r] = d->rho;
    const double s = d->gs[k * ng + r];
    for (int j = 0; j < nx + nv; ++j) jac[r * nlr + j] = s * jo[r * nl + j];
    for (int c = 0; c < nx; ++c) jac[r * nlr + nx + nv + 2 * ng + c] = s * jo[r * nl + nx + nv + c];
    jac[r * nlr + nx + nv + r] = -1.0;
    jac[r * nlr + nx + nv + ng + r] = 1.0;
  }
}
static void resto_hess(const model_t* mm, const double* L, const double* PS, const double* PG, double TK, double sigma,
                       const double* lam, double* H) {
  const resto_t* d = (const resto_t*)mm->data;
  const model_t* m = d->m;
  const int k = resto_stage(mm, TK), nx = m->nx, nv = m->nv, ng = m->ng;
  const int nl = 2 * nx + nv, nlr = nl + 2 * ng, np = nv + nx;
  double *Lo = d->Lo, *lo = d->lo, *Ho = d->Ho;
  int* map = d->map;
  resto_split(m, L, Lo);
  for (int r = 0; r < ng; ++r) lo[r] = lam[r] * d->gs[k * ng + r];
  memset(Ho, 0, sizeof(double) * nl * nl);
  m->hess(m, Lo, PS, PG, TK, 0.0, lo, Ho);  /* the constraints' curvature only */
  for (int i = 0; i < nl; ++i) map[i] = i < nx + nv ? i : i + 2 * ng;
  for (int i = 0; i < nl; ++i)
    for (int j = 0; j < nl; ++j) H[map[i] * nlr + map[j]] = Ho[i * nl + j];
  for (int j = 0; j < np; ++j) {
    const int li = j < nv ? nx + j : nx + nv + 2 * ng + (j - nv), gi = nx + k * np + j;
    H[li * nlr + li] += sigma * d->zeta * d->dr2[gi];
  }
}

/* ---- the interior-point run ----------------------------------------------------------
   inner == NULL: the original NLP (gradient scaling, bound relaxation and push, least-squares
   multipliers).  inner != NULL: the restoration NLP (already scaled and relaxed; the start
   point, its multipliers and mu given; the return test `check` at the head of every
   iteration; every accepted Newton step refined on the full system). */
typedef struct inner_s inner_t;
struct inner_s {
  const double *xL, *xU, *lb, *ub, *zL, *zU, *vL, *vU;
  double mu;
  resto_t* rd;                 /* zeta follows mu */
  int (*check)(void* ctx, const double* x, const double* s);
  void* ctx;
  double* s_out;               /* the slacks at the end */
};
#define ST_RESTO_RETURN 100

typedef struct { int soft, resto, resto_iters, refine, filt_over; } counts_t;

/* outer state the return test reads */
typedef struct {
  ws_t* w;               /* the original problem (its bounds, scaling, model) */
  const filter_t* f;
  double theta_max, th0, mu;
  const double* s_start;  /* original slacks at the start of restoration */
  double *xo, *so, *go;   /* scratch */
} check_ctx_t;

static void resto_to_outer(const ws_t* w, const double* xr, double* xo) {
  /* inner layout [x0, (V, p, n, X1)_k] -> outer [x0, (V, X1)_k] */
  const int NX = w->NX, NV = w->NV, NP = w->NP, NG = w->NG, NPR = NP + 2 * NG;
  for (int i = 0; i < NX; ++i) xo[i] = xr[i];
  for (int k = 0; k < w->N; ++k)
    for (int j = 0; j < NP; ++j) xo[NX + k * NP + j] = xr[NX + k * NPR + (j < NV ? j : j + 2 * NG)];
}
static int resto_check(void* vctx, const double* xr, const double* sr) {
  check_ctx_t* c = (check_ctx_t*)vctx;
  ws_t* w = c->w;
  resto_to_outer(w, xr, c->xo);
  for (int r = 0; r < w->M; ++r) c->so[r] = ccls(w, r) != 0 ? sr[r] : c->s_start[r];
  const double fo = w->obj_scale * eval_fg(w, c->xo, c->go);
  for (int r = 0; r < w->M; ++r) c->go[r] *= w->gs[r];
  const double th = theta_of(w, c->go, c->so);
  if (!(th <= 0.9 * c->th0)) return 0;
  const double ph = fo - c->mu * barrier_of(w, c->xo, c->so);
  return th <= c->theta_max && filter_accepts(c->f, th, ph);
}

static int ipm_run(const model_t* m, const double* p, const double* lbw, const double* ubw, double* wio,
                   const opts_t* o, ostats_t* st, const inner_t* inner, double* mem, int* imem, counts_t* cnt);

static long ipm_doubles(const model_t* m) {
  const int NW = m->nx + m->N * (m->nv + m->nx), M = m->N * m->ng;
  const int NB = m->nv + m->nx + m->ng, NL = 2 * m->nx + m->nv;
  return 12L * NW + 19L * M + (long)m->N * (NL + m->ng * NL + NL * NL + NB * NB + 5 * NB) + (long)NB * NB + 64;
}

/* the restoration phase from the iterate whose line search (and soft step) failed; returns the
   inner status (ST_RESTO_RETURN: back in the original problem, x / s / multipliers updated) */
static int restoration(ws_t* w, const opts_t* o, filter_t* f, double theta_max, double mu, double tau,
                       double theta, int* it, double* fx, counts_t* cnt) {
  const model_t* m = w->m;
  const int N = w->N, NX = w->NX, NV = w->NV, NP = w->NP, NG = w->NG, NW = w->NW, M = w->M;
  const int NPR = NP + 2 * NG, NWR = NX + N * NPR;
  const double rho = 1000.0;
  double mu_r = mu;
  for (int c = 0; c < M; ++c)
    mu_r = fmax(mu_r, fabs(ccls(w, c) == 0 ? w->gv[c] - w->gs[c] * w->lb[c] : w->gv[c] - w->s[c]));
  model_t rm = *m;
  rm.nv = m->nv + 2 * m->ng;
  const int nl = w->NL;
  resto_t rd = {m, w->gs, 0, 0, rho, 0.0, 0, 0, 0, 0, 0, 0};
  double* scr = (double*)malloc(sizeof(double) * (3L * nl + (long)NG * nl + (long)nl * nl + NG + 1));
  rd.Lo = scr; rd.go = scr + nl; rd.jo = rd.go + nl; rd.Ho = rd.jo + (long)NG * nl; rd.lo = rd.Ho + (long)nl * nl;
  rd.map = (int*)malloc(sizeof(int) * (nl + 1));
  rm.fg = resto_fg; rm.gj = resto_gj; rm.hess = resto_hess; rm.data = &rd;
  const long nd = ipm_doubles(&rm);
  double* buf = (double*)malloc(sizeof(double) * (nd + 12L * NWR + 8L * M + 4L * NW + 3L * M));
  int* ibuf = (int*)malloc(sizeof(int) * 2 * N * (NPR + NG));
  double* q = buf + nd;
  double *xR = q; q += NW;
  double *dr2 = q; q += NW;
  double *x0 = q; q += NWR;
  double *xl = q; q += NWR;
  double *xu = q; q += NWR;
  double *zl = q; q += NWR;
  double *zu = q; q += NWR;
  double *lb = q; q += M;
  double *ub = q; q += M;
  double *sr = q; q += M;
  double *ss = q; q += M;
  double *xo = q; q += NW;
  double *so = q; q += M;
  double *go = q; q += M;
  memcpy(xR, w->x, sizeof(double) * NW);
  for (int i = 0; i < NW; ++i) dr2[i] = fixedv(w, i) ? 0.0 : 1.0 / (fmax(1.0, fabs(xR[i])) * fmax(1.0, fabs(xR[i])));
  rd.xR = xR; rd.dr2 = dr2;
  for (int i = 0; i < NX; ++i) { x0[i] = w->x[i]; xl[i] = w->x[i]; xu[i] = w->x[i]; zl[i] = zu[i] = 0.0; }
  for (int k = 0; k < N; ++k) {
    for (int j = 0; j < NP; ++j) {
      const int gi = NX + k * NP + j, ri = NX + k * NPR + (j < NV ? j : j + 2 * NG);
      x0[ri] = w->x[gi];
      xl[ri] = fixedv(w, gi) ? w->x[gi] : w->xL[gi];
      xu[ri] = fixedv(w, gi) ? w->x[gi] : w->xU[gi];
      zl[ri] = fmin(w->zL[gi], rho);
      zu[ri] = fmin(w->zU[gi], rho);
    }
    for (int r = 0; r < NG; ++r) {
      const int c = k * NG + r;
      const double cv = ccls(w, c) == 0 ? w->gv[c] - w->gs[c] * w->lb[c] : w->gv[c] - w->s[c];
      /* p, n solving the restoration complementarity at its start (Waechter & Biegler 2006, eq. 33) */
      const double a = (mu_r - rho * cv) / (2.0 * rho);
      const double nv = a + sqrt(a * a + mu_r * cv / (2.0 * rho)), pv = cv + nv;
      const int ip = NX + k * NPR + NV + r, in_ = ip + NG;
      x0[ip] = pv; x0[in_] = nv;
      xl[ip] = xl[in_] = 0.0; xu[ip] = xu[in_] = INFINITY;
      zl[ip] = mu_r / pv; zl[in_] = mu_r / nv; zu[ip] = zu[in_] = 0.0;
    }
  }
  double* vL = (double*)malloc(sizeof(double) * 2 * M);
  double* vU = vL + M;
  for (int c = 0; c < M; ++c) {
    const int eq = ccls(w, c) == 0;
    lb[c] = eq ? w->gs[c] * w->lb[c] : w->sL[c];
    ub[c] = eq ? w->gs[c] * w->lb[c] : w->sU[c];
    vL[c] = fmin(w->vL[c], rho);
    vU[c] = fmin(w->vU[c], rho);
  }
  check_ctx_t cc = {w, f, theta_max, theta, mu, w->s, xo, so, go};
  inner_t in = {xl, xu, lb, ub, zl, zu, vL, vU, mu_r, &rd, resto_check, &cc, sr};
  opts_t orr = *o;
  orr.max_iter = o->max_iter - *it;
  ostats_t ist;
  counts_t icnt = {0, 0, 0, 0, 0};
  const int status = ipm_run(&rm, w->p, xl, xu, x0, &orr, &ist, &in, buf, ibuf, &icnt);
  cnt->resto_iters += ist.iter;
  cnt->refine += icnt.refine;
  cnt->filt_over += icnt.filt_over;
  *it += ist.iter;
  resto_to_outer(w, x0, xo);
  for (int c = 0; c < M; ++c) ss[c] = ccls(w, c) != 0 ? sr[c] : w->s[c];
  if (status == ST_RESTO_RETURN) {
    /* back to the original problem: bound multipliers by one Newton step for the
       complementarity over the whole primal change, fraction to the boundary, reset to 1 when
       too large; constraint multipliers restart at zero */
    double ad = 1.0, zmax = 0.0;
    for (int pass = 0; pass < 2; ++pass) {
      for (int i = NX; i < NW; ++i) {
        if (fixedv(w, i)) continue;
        if (isfin(w->xL[i])) {
          const double dz = (mu - w->zL[i] * (xo[i] - w->xL[i])) / (w->x[i] - w->xL[i]);
          if (pass == 0) { if (dz < 0) ad = fmin(ad, -tau * w->zL[i] / dz); }
          else { w->zL[i] += ad * dz; zmax = fmax(zmax, fabs(w->zL[i])); }
        }
        if (isfin(w->xU[i])) {
          const double dz = (mu - w->zU[i] * (w->xU[i] - xo[i])) / (w->xU[i] - w->x[i]);
          if (pass == 0) { if (dz < 0) ad = fmin(ad, -tau * w->zU[i] / dz); }
          else { w->zU[i] += ad * dz; zmax = fmax(zmax, fabs(w->zU[i])); }
        }
      }
      for (int c = 0; c < M; ++c) {
        if (ccls(w, c) != 1) continue;
        if (isfin(w->sL[c])) {
          const double dv = (mu - w->vL[c] * (ss[c] - w->sL[c])) / (w->s[c] - w->sL[c]);
          if (pass == 0) { if (dv < 0) ad = fmin(ad, -tau * w->vL[c] / dv); }
          else { w->vL[c] += ad * dv; zmax = fmax(zmax, fabs(w->vL[c])); }
        }
        if (isfin(w->sU[c])) {
          const double dv = (mu - w->vU[c] * (w->sU[c] - ss[c])) / (w->sU[c] - w->s[c]);
          if (pass == 0) { if (dv < 0) ad = fmin(ad, -tau * w->vU[c] / dv); }
          else { w->vU[c] += ad * dv; zmax = fmax(zmax, fabs(w->vU[c])); }
        }
      }
    }
    if (zmax > 1000.0) {
      for (int i = NX; i < NW; ++i) {
        if (fixedv(w, i)) continue;
        w->zL[i] = isfin(w->xL[i]) ? 1.0 : 0.0;
        w->zU[i] = isfin(w->xU[i]) ? 1.0 : 0.0;
      }
      for (int c = 0; c < M; ++c) {
        if (ccls(w, c) != 1) continue;
        w->vL[c] = isfin(w->sL[c]) ? 1.0 : 0.0;
        w->vU[c] = isfin(w->sU[c]) ? 1.0 : 0.0;
      }
    }
  }
  memcpy(w->x, xo, sizeof(double) * NW);
  memcpy(w->s, ss, sizeof(double) * M);
  for (int c = 0; c < M; ++c) w->lam[c] = 0.0;
  *fx = w->obj_scale * eval_fg(w, w->x, w->gv);
  for (int c = 0; c < M; ++c) w->gv[c] *= w->gs[c];
  eval_gj(w, w->x);
  free(vL);
  free(buf);
  free(ibuf);
  free(scr);
  free(rd.map);
  return status;
}

static int ipm_run(const model_t* m, const double* p, const double* lbw, const double* ubw, double* wio,
                   const opts_t* o, ostats_t* st, const inner_t* inner, double* mem, int* imem, counts_t* cnt) {
  ws_t W;
  ws_t* w = &W;
  w->m = m; w->N = m->N; w->NX = m->nx; w->NV = m->nv; w->NG = m->ng;
  w->NL = 2 * m->nx + m->nv; w->NP = m->nv + m->nx; w->NB = w->NP + w->NG;
  w->NW = w->NX + w->N * w->NP; w->M = w->N * w->NG; w->p = p;
  const int NW = w->NW, M = w->M, NX = w->NX, NP = w->NP, NG = w->NG, NB = w->NB, N = w->N;
  if (NB > MAXNB || NX > MAXNX) { st->status = -3; st->iter = 0; st->obj = NAN; return -3; }
  double* q = mem;
#define TAKE(ptr, n) do { ptr = q; q += (n); } while (0)
  TAKE(w->x, NW); TAKE(w->s, M); TAKE(w->lam, M); TAKE(w->zL, NW); TAKE(w->zU, NW);
  TAKE(w->vL, M); TAKE(w->vU, M); TAKE(w->xL, NW); TAKE(w->xU, NW); TAKE(w->sL, M); TAKE(w->sU, M);
  TAKE(w->gs, M); TAKE(w->gv, M); TAKE(w->lb, M); TAKE(w->ub, M); TAKE(w->dx, NW); TAKE(w->ds, M);
  TAKE(w->dl, M); TAKE(w->xt, NW); TAKE(w->st, M); TAKE(w->gt, M);
  TAKE(w->lt, M); TAKE(w->zLt, NW); TAKE(w->zUt, NW); TAKE(w->vLt, M); TAKE(w->vUt, M);
  TAKE(w->sdg, N * w->NL); TAKE(w->sdj, N * NG * w->NL); TAKE(w->sdh, N * w->NL * w->NL);
  TAKE(w->fac, N * NB * NB); TAKE(w->rhs, N * NB); TAKE(w->sol, N * NB);
  TAKE(w->rhs0, N * NB); TAKE(w->sol0, N * NB); TAKE(w->res, N * NB); TAKE(w->kb, NB * NB);
#undef TAKE
  w->perm = imem; w->piv = imem + N * NB;
  const double INF_B = 1e19;
  double fx, mu;
  if (!inner) {
    for (int i = 0; i < NW; ++i) {
      double lo = lbw[i] <= -INF_B ? -INFINITY : lbw[i], hi = ubw[i] >= INF_B ? INFINITY : ubw[i];
      if (i < NX) hi = lo;
      w->xL[i] = lo; w->xU[i] = hi; w->x[i] = lo == hi ? lo : wio[i];
    }
    for (int k = 0; k < N; ++k) m->bounds(m, p + m->npg + k * m->nps, p, k * m->ts, w->lb + k * NG, w->ub + k * NG);
    eval_gj(w, w->x);
    double gmax = 0.0;
    for (int i = NX; i < NW; ++i) if (!fixedv(w, i)) gmax = fmax(gmax, fabs(acc_grad(w, i)));
    w->obj_scale = gmax > 100.0 ? fmax(1e-8, 100.0 / gmax) : 1.0;
    for (int c = 0; c < M; ++c) {
      const int k = c / NG, r = c % NG;
      double rm = 0.0;
      for (int j = 0; j < w->NL; ++j) if (!fixedv(w, k * NP + j)) rm = fmax(rm, fabs(w->sdj[(k * NG + r) * w->NL + j]));
      w->gs[c] = rm > 100.0 ? fmax(1e-8, 100.0 / rm) : 1.0;
    }
    for (int i = 0; i < NW; ++i) {
      double lo = w->xL[i], hi = w->xU[i];
      w->zL[i] = w->zU[i] = 0.0;
      if (i >= NX && lo != hi) {
        if (isfin(lo)) lo -= 1e-8 * fmax(1.0, fabs(lo));
        if (isfin(hi)) hi += 1e-8 * fmax(1.0, fabs(hi));
        w->xL[i] = lo; w->xU[i] = hi;
        w->x[i] = push_into(w->x[i], lo, hi);
        w->zL[i] = isfin(lo) ? 1.0 : 0.0;
        w->zU[i] = isfin(hi) ? 1.0 : 0.0;
      }
    }
    fx = w->obj_scale * eval_fg(w, w->x, w->gv);
    for (int c = 0; c < M; ++c) {
      const double gsc = w->gs[c];
      w->gv[c] *= gsc;
      const double lo = w->lb[c], hi = w->ub[c];
      if (lo == hi) {
        w->sL[c] = w->sU[c] = w->s[c] = gsc * lo; w->vL[c] = w->vU[c] = 0.0;
      } else {
        const double sl = isfin(lo) ? gsc * lo - 1e-8 * fmax(1.0, fabs(gsc * lo)) : -INFINITY;
        const double su = isfin(hi) ? gsc * hi + 1e-8 * fmax(1.0, fabs(gsc * hi)) : INFINITY;
        w->sL[c] = sl; w->sU[c] = su; w->s[c] = push_into(w->gv[c], sl, su);
        w->vL[c] = isfin(sl) ? 1.0 : 0.0; w->vU[c] = isfin(su) ? 1.0 : 0.0;
      }
      w->lam[c] = 0.0;
    }
    mu = 0.1;
  } else {  /* restoration NLP: scaled and relaxed already, start point and multipliers given */
    w->obj_scale = 1.0;
    for (int i = 0; i < NW; ++i) {
      w->xL[i] = inner->xL[i]; w->xU[i] = inner->xU[i];
      w->x[i] = fixedv(w, i) ? w->xL[i] : wio[i];
      w->zL[i] = (i >= NX && !fixedv(w, i) && isfin(w->xL[i])) ? inner->zL[i] : 0.0;
      w->zU[i] = (i >= NX && !fixedv(w, i) && isfin(w->xU[i])) ? inner->zU[i] : 0.0;
    }
    mu = inner->mu;
    inner->rd->zeta = sqrt(mu);
    for (int c = 0; c < M; ++c) { w->gs[c] = 1.0; w->lb[c] = inner->lb[c]; w->ub[c] = inner->ub[c]; }
    fx = eval_fg(w, w->x, w->gv);
    for (int c = 0; c < M; ++c) {
      const double lo = w->lb[c], hi = w->ub[c];
      w->lam[c] = 0.0;
      if (lo == hi) {
        w->sL[c] = w->sU[c] = w->s[c] = lo; w->vL[c] = w->vU[c] = 0.0;
      } else {
        w->sL[c] = lo; w->sU[c] = hi; w->s[c] = w->gv[c];
        w->vL[c] = isfin(lo) ? inner->vL[c] : 0.0; w->vU[c] = isfin(hi) ? inner->vU[c] : 0.0;
      }
    }
  }
  eval_gj(w, w->x);
  int n_fact = 0, n_trials = 0;
  if (!inner) {
    inertia_t in = factor_chain(w, 0.0, 0.0, 1);
    n_fact++;
    for (int k = 0; k < N; ++k) {
      for (int qq = 0; qq < NP; ++qq) {
        const int i = NX + k * NP + qq;
        w->rhs[k * NB + qq] = fixedv(w, i) ? 0.0 : -(w->obj_scale * acc_grad(w, i) - w->zL[i] + w->zU[i]);
      }
      for (int r = 0; r < NG; ++r) {
        const int c = k * NG + r;
        w->rhs[k * NB + NP + r] = ccls(w, c) == 1 ? w->vL[c] - w->vU[c] : 0.0;
      }
    }
    if (in.zero == 0) {
      solve_chain(w, 1);
      double lmax = 0.0;
      for (int c = 0; c < M; ++c) lmax = fmax(lmax, fabs(w->sol[(c / NG) * NB + NP + c % NG]));
      if (lmax <= 1e3) for (int c = 0; c < M; ++c) w->lam[c] = w->sol[(c / NG) * NB + NP + c % NG];
    }
  }
  double tau = fmax(0.99, 1.0 - mu), dw_last = 0.0;
  const double theta0 = theta_of(w, w->gv, w->s);
  const double theta_max = 1e4 * fmax(1.0, theta0), theta_min = 1e-4 * fmax(1.0, theta0);
  filter_t F;
  F.n = 0; F.over = 0; F.maxn = 0;
  int status = -1, it = 0, in_soft = 0, soft_count = 0;
  int nfree = 0, neq = 0;
  for (int i = NX; i < NW; ++i) nfree += !fixedv(w, i);
  for (int c = 0; c < M; ++c) neq += w->lb[c] == w->ub[c];
  const int square = nfree == neq;
  acc_t acc = {-1e50, -1e50, -1, 0};
  for (;;) {
    if (inner && inner->check(inner->ctx, w->x, w->s)) { status = ST_RESTO_RETURN; break; }
    double du, pu, cmpl;
    const double err = opt_error(w, 0.0, &du, &pu, &cmpl);
    if (err != err || fx != fx) { status = -4; break; }
    if (err <= o->tol && pu <= o->constr_viol_tol && (square || (du <= o->dual_inf_tol && cmpl <= o->compl_inf_tol))) {
      status = 0;
      break;
    }
    if (o->acceptable_iter > 0 && current_is_acceptable(&acc, o, square, err, du, pu, cmpl, fx, it)) {
      if (++acc.count >= o->acceptable_iter) { status = 1; break; }
    } else {
      acc.count = 0;
    }
    if (it >= o->max_iter) break;
    for (int g = 0; g < 64; ++g) {
      if (opt_error(w, mu, 0, 0, 0) > 10.0 * mu || mu <= 1e-11) break;
      /* IPOPT MonotoneMuUpdate: floor min(tol, compl_inf_tol) / (barrier_tol_factor + 1) */
      const double new_mu = fmax(fmax(fmin(o->tol, o->compl_inf_tol) / 11.0, 1e-11), fmin(0.2 * mu, pow(mu, 1.5)));
      if (new_mu == mu) break;  /* IPOPT: done when mu no longer changes */
      mu = new_mu;
      tau = fmax(0.99, 1.0 - mu);
      F.n = 0;
      if (inner) {  /* the restoration objective depends on mu (zeta) */
        inner->rd->zeta = sqrt(mu);
        fx = eval_fg(w, w->x, w->gt);
        eval_gj(w, w->x);
      }
    }
    eval_hess(w, w->x, w->obj_scale);
    for (int i = NX; i < NW; ++i) {
      double r = 0.0;
      if (!fixedv(w, i)) {
        double gphi = w->obj_scale * acc_grad(w, i);
        if (isfin(w->xL[i])) gphi -= mu / (w->x[i] - w->xL[i]);
        if (isfin(w->xU[i])) gphi += mu / (w->xU[i] - w->x[i]);
        r = -(gphi + acc_jtl(w, i, w->lam));
      }
      w->rhs[((i - NX) / NP) * NB + (i - NX) % NP] = r;
    }
    double dw = 0.0, dc = 0.0;
    int ok = 0;
    for (int attempt = 0; attempt < 140; ++attempt) {
      inertia_t in = factor_chain(w, dw, dc, 0);
      n_fact++;
      if (in.pos == N * NP && in.neg == M && in.zero == 0) { if (attempt > 0) dw_last = dw; ok = 1; break; }
      if (attempt == 0) {
        if (in.zero > 0) dc = 1e-8 * pow(mu, 0.25);
        dw = dw_last == 0.0 ? 1e-4 : fmax(1e-20, dw_last / 3.0);
      } else {
        dw = dw_last == 0.0 ? 100.0 * dw : 8.0 * dw;
        if (dw > 1e40) {
          /* IPOPT PerturbForWrongInertia: regularise the constraint block, shift again */
          if (dc != 0.0) break;
          dc = 1e-8 * pow(mu, 0.25);
          dw = dw_last == 0.0 ? 1e-4 : fmax(1e-20, dw_last / 3.0);
        }
      }
    }
    if (!ok) { status = -3; break; }
    for (int c = 0; c < M; ++c) {
      const int cl = ccls(w, c);
      double rr;
      if (cl == 0) rr = -(w->gv[c] - w->gs[c] * w->lb[c]);
      else {
        rr = -(w->gv[c] - w->s[c]);
        if (cl == 1) {
          double gps = 0.0;
          if (isfin(w->sL[c])) gps -= mu / (w->s[c] - w->sL[c]);
          if (isfin(w->sU[c])) gps += mu / (w->sU[c] - w->s[c]);
          rr -= (gps - w->lam[c]) / (sigma_s(w, c) + dw);
        }
      }
      w->rhs[(c / NG) * NB + NP + c % NG] = rr;
    }
    solve_chain(w, 0);
    if (inner) cnt->refine += refine(w, dw, dc);  /* IPOPT PDFullSpaceSolver on the full system */
    double amax = 1.0, az = 1.0, gphid = 0.0;
    for (int i = 0; i < NW; ++i) {
      double d = 0.0;
      if (i >= NX && !fixedv(w, i)) d = w->sol[((i - NX) / NP) * NB + (i - NX) % NP];
      w->dx[i] = d;
      if (i < NX || fixedv(w, i)) continue;
      double gphi = w->obj_scale * acc_grad(w, i);
      if (isfin(w->xL[i])) {
        const double sl = w->x[i] - w->xL[i];
        gphi -= mu / sl;
        if (d < 0) amax = fmin(amax, -tau * sl / d);
        const double dz = mu / sl - w->zL[i] - (w->zL[i] / sl) * d;
        if (dz < 0) az = fmin(az, -tau * w->zL[i] / dz);
      }
      if (isfin(w->xU[i])) {
        const double su = w->xU[i] - w->x[i];
        gphi += mu / su;
        if (d > 0) amax = fmin(amax, tau * su / d);
        const double dz = mu / su - w->zU[i] + (w->zU[i] / su) * d;
        if (dz < 0) az = fmin(az, -tau * w->zU[i] / dz);
      }
      gphid += gphi * d;
    }
    for (int c = 0; c < M; ++c) {
      const double dlam = w->sol[(c / NG) * NB + NP + c % NG];
      w->dl[c] = dlam;
      double dsv = 0.0;
      if (ccls(w, c) == 1) {
        double gps = 0.0;
        if (isfin(w->sL[c])) gps -= mu / (w->s[c] - w->sL[c]);
        if (isfin(w->sU[c])) gps += mu / (w->sU[c] - w->s[c]);
        const double rs = gps - w->lam[c];
        dsv = (dlam - rs) / (sigma_s(w, c) + dw);
        gphid += gps * dsv;
        if (isfin(w->sL[c])) {
          const double sl = w->s[c] - w->sL[c];
          if (dsv < 0) amax = fmin(amax, -tau * sl / dsv);
          const double dv = mu / sl - w->vL[c] - (w->vL[c] / sl) * dsv;
          if (dv < 0) az = fmin(az, -tau * w->vL[c] / dv);
        }
        if (isfin(w->sU[c])) {
          const double su = w->sU[c] - w->s[c];
          if (dsv > 0) amax = fmin(amax, tau * su / dsv);
          const double dv = mu / su - w->vU[c] + (w->vU[c] / su) * dsv;
          if (dv < 0) az = fmin(az, -tau * w->vU[c] / dv);
        }
      }
      w->ds[c] = dsv;
    }
    const double theta = theta_of(w, w->gv, w->s);
    const double phi = fx - mu * barrier_of(w, w->x, w->s);
    double amin;
    if (gphid < 0 && theta <= theta_min)
      amin = 0.05 * fmin(fmin(1e-5, 1e-8 * theta / -gphid), pow(theta, 1.1) / pow(-gphid, 2.3));
    else if (gphid < 0) amin = 0.05 * fmin(1e-5, 1e-8 * theta / -gphid);
    else amin = 0.05 * 1e-5;
    if (!(amin > 0)) amin = 0.05 * 1e-5;
    /* the trial point of a step (x, s, lam, z, v at step sizes alpha / alpha_z): xt, st, gt, lt, *t */
#define TRIAL(alpha_, az_)                                                                      \
    do {                                                                                        \
      for (int i = 0; i < NW; ++i) w->xt[i] = w->x[i] + (alpha_) * w->dx[i];                    \
      for (int c = 0; c < M; ++c) w->st[c] = w->s[c] + (alpha_) * w->ds[c];                     \
      ft = w->obj_scale * eval_fg(w, w->xt, w->gt);                                             \
      n_trials++;                                                                               \
      for (int c = 0; c < M; ++c) w->gt[c] *= w->gs[c];                                         \
    } while (0)
    double alpha = amax, ft = 0.0, a_used = az;
    int accepted = 0, ftype = 0, soft = 0, soft_orig = 0, goto_resto = 0;
    /* IPOPT BacktrackingLineSearch::TrySoftRestoStep: the full fraction-to-the-boundary step,
       one step size for primal and dual variables; accepted by the original filter criterion
       (orig) or by a 0.9999 reduction of the primal-dual system error */
#define SOFT_STEP(ok_)                                                                            \
    do {                                                                                          \
      const double al = fmin(amax, az);                                                           \
      TRIAL(al, al);                                                                              \
      for (int c = 0; c < M; ++c) w->lt[c] = w->lam[c] + al * w->dl[c];                          \
      for (int i = NX; i < NW; ++i) {                                                             \
        w->zLt[i] = w->zL[i]; w->zUt[i] = w->zU[i];                                               \
        if (fixedv(w, i)) continue;                                                               \
        if (isfin(w->xL[i])) { const double sl = w->x[i] - w->xL[i];                              \
          w->zLt[i] = w->zL[i] + al * (mu / sl - w->zL[i] - (w->zL[i] / sl) * w->dx[i]); }        \
        if (isfin(w->xU[i])) { const double su = w->xU[i] - w->x[i];                              \
          w->zUt[i] = w->zU[i] + al * (mu / su - w->zU[i] + (w->zU[i] / su) * w->dx[i]); }        \
      }                                                                                           \
      for (int c = 0; c < M; ++c) {                                                               \
        w->vLt[c] = w->vL[c]; w->vUt[c] = w->vU[c];                                               \
        if (ccls(w, c) != 1) continue;                                                            \
        if (isfin(w->sL[c])) { const double sl = w->s[c] - w->sL[c];                              \
          w->vLt[c] = w->vL[c] + al * (mu / sl - w->vL[c] - (w->vL[c] / sl) * w->ds[c]); }        \
        if (isfin(w->sU[c])) { const double su = w->sU[c] - w->s[c];                              \
          w->vUt[c] = w->vU[c] + al * (mu / su - w->vU[c] + (w->vU[c] / su) * w->ds[c]); }        \
      }                                                                                           \
      alpha = al; a_used = al; ok_ = 0; soft_orig = 0;                                            \
      const double tht = theta_of(w, w->gt, w->st), pht = ft - mu * barrier_of(w, w->xt, w->st);  \
      if (isfin(tht) && isfin(pht)) {                                                             \
        if (tht <= theta_max && filter_accepts(&F, tht, pht) &&                                   \
            (tht <= (1 - 1e-5) * theta || pht <= phi - 1e-8 * theta)) {                           \
          ok_ = 1; soft_orig = 1;                                                                 \
        } else {                                                                                  \
          const double cur = pd_error(w, w->x, w->s, w->lam, w->zL, w->zU, w->vL, w->vU, w->gv, mu); \
          eval_gj(w, w->xt);                                                                      \
          const double nw = pd_error(w, w->xt, w->st, w->lt, w->zLt, w->zUt, w->vLt, w->vUt, w->gt, mu); \
          ok_ = nw <= 0.9999 * cur;                                                               \
          if (!ok_) eval_gj(w, w->x);                                                             \
        }                                                                                         \
      }                                                                                           \
    } while (0)
    if (in_soft) {
      soft_count++;
      int okk = 0;
      if (soft_count <= 10) SOFT_STEP(okk);
      if (okk) { soft = 1; if (soft_orig) { in_soft = 0; soft_count = 0; } }
      else goto_resto = 1;
    } else {
      for (int ls = 0; ls < 64; ++ls) {
        TRIAL(alpha, az);
        const double tht = theta_of(w, w->gt, w->st), pht = ft - mu * barrier_of(w, w->xt, w->st);
        int okt = tht <= theta_max && isfin(pht) && filter_accepts(&F, tht, pht);  /* ipm.py: finite phi */
        if (okt) {
          const int sw = gphid < 0 && alpha * pow(-gphid, 2.3) > pow(theta, 1.1);
          if (theta <= theta_min && sw) { okt = pht <= phi + 1e-8 * alpha * gphid; ftype = 1; }
          else { okt = tht <= (1 - 1e-5) * theta || pht <= phi - 1e-8 * theta; ftype = 0; }
        }
        if (okt) { accepted = 1; break; }
        alpha *= 0.5;
        if (alpha < amin) break;
      }
      if (!accepted && inner) { status = -2; break; }  /* no restoration inside the restoration phase */
      if (!accepted) {
        int okk = 0;
        SOFT_STEP(okk);
        if (okk) { soft = 1; cnt->soft++; if (!soft_orig) { in_soft = 1; soft_count = 0; } }
        else goto_resto = 1;
      }
    }
    if (goto_resto) {
      /* IPOPT: restoration phase called at an acceptable point -> Solved_To_Acceptable_Level */
      if (current_is_acceptable(&acc, o, square, err, du, pu, cmpl, fx, it)) { status = 1; break; }
      if (inner) { status = -2; break; }
      /* ---- feasibility restoration phase (MinC_1NrmRestorationPhase) ---- */
      cnt->resto++;
      filter_add(&F, theta, phi);  /* FilterLSAcceptor::PrepareRestoPhaseStart */
      in_soft = 0; soft_count = 0;
      const int rs = restoration(w, o, &F, theta_max, mu, tau, theta, &it, &fx, cnt);
      if (rs != ST_RESTO_RETURN) {
        status = (rs == 0 || rs == 1) ? -5 : rs;   /* converged restoration: local infeasibility */
        break;
      }
      continue;
    }
    if (soft) {
      if (soft_orig) filter_add(&F, theta, phi);  /* accepted by the original (h-type) criterion */
      for (int c = 0; c < M; ++c) w->lam[c] = w->lt[c];
    } else {
      if (!ftype) filter_add(&F, theta, phi);
      for (int c = 0; c < M; ++c) w->lam[c] += alpha * w->dl[c];
    }
    /* take the trial point; bound multipliers by their steps (soft: already in *t), then the
       kappa_sigma safeguard */
    for (int i = NX; i < NW; ++i) {
      if (fixedv(w, i)) continue;
      const double d = w->dx[i], xo = w->x[i], xn = w->xt[i];
      w->x[i] = xn;
      if (isfin(w->xL[i])) {
        const double sl0 = xo - w->xL[i], sl = xn - w->xL[i];
        const double zn = soft ? w->zLt[i] : w->zL[i] + a_used * (mu / sl0 - w->zL[i] - (w->zL[i] / sl0) * d);
        w->zL[i] = fmax(fmin(zn, 1e10 * mu / sl), mu / (1e10 * sl));
      }
      if (isfin(w->xU[i])) {
        const double su0 = w->xU[i] - xo, su = w->xU[i] - xn;
        const double zn = soft ? w->zUt[i] : w->zU[i] + a_used * (mu / su0 - w->zU[i] + (w->zU[i] / su0) * d);
        w->zU[i] = fmax(fmin(zn, 1e10 * mu / su), mu / (1e10 * su));
      }
    }
    for (int c = 0; c < M; ++c) {
      w->gv[c] = w->gt[c];
      if (ccls(w, c) != 1) { w->s[c] = w->st[c]; continue; }
      const double so = w->s[c], sn = w->st[c], dsv = w->ds[c];
      w->s[c] = sn;
      if (isfin(w->sL[c])) {
        const double sl0 = so - w->sL[c], sl = sn - w->sL[c];
        const double vn = soft ? w->vLt[c] : w->vL[c] + a_used * (mu / sl0 - w->vL[c] - (w->vL[c] / sl0) * dsv);
        w->vL[c] = fmax(fmin(vn, 1e10 * mu / sl), mu / (1e10 * sl));
      }
      if (isfin(w->sU[c])) {
        const double su0 = w->sU[c] - so, su = w->sU[c] - sn;
        const double vn = soft ? w->vUt[c] : w->vU[c] + a_used * (mu / su0 - w->vU[c] + (w->vU[c] / su0) * dsv);
        w->vU[c] = fmax(fmin(vn, 1e10 * mu / su), mu / (1e10 * su));
      }
    }
    fx = ft;
    eval_gj(w, w->x);
    it++;
#undef SOFT_STEP
#undef TRIAL
  }
  for (int i = 0; i < NW; ++i) wio[i] = w->x[i];
  if (inner) memcpy(inner->s_out, w->s, sizeof(double) * M);
  st->obj = fx / w->obj_scale;
  st->iter = it;
  st->status = status;
  st->n_fact = n_fact;
  st->n_trials = n_trials;
  st->n_soft = cnt->soft;
  st->n_resto = cnt->resto;
  st->n_resto_iters = cnt->resto_iters;
  cnt->filt_over += F.over;
  st->n_filter_over = cnt->filt_over;
  st->n_refine = cnt->refine;
  return status;
}

static void solve_one(const model_t* m, const double* p, const double* lbw, const double* ubw,
                      double* wio, const opts_t* o, ostats_t* st, double* mem, int* imem) {
  counts_t cnt = {0, 0, 0, 0, 0};
  ipm_run(m, p, lbw, ubw, wio, o, st, 0, mem, imem, &cnt);
}

/* Solve n_agents NLPs of one stage model (agent-major arrays); returns #converged
   (success flag: Solve_Succeeded or Solved_To_Acceptable_Level). */
int oracle_solve_fleet(const model_t* m, int n_agents, const double* p, const double* lbw, const double* ubw,
                       double* w_io, ostats_t* stats, const opts_t* opts, int threads) {
  const opts_t o = *opts;
  const int NW = m->nx + m->N * (m->nv + m->nx), NPAR = m->npg + m->N * m->nps;
  const int NB = m->nv + m->nx + m->ng;
  const long dbl = ipm_doubles(m);
  int ok = 0;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel reduction(+ : ok)
  {
    double* mem = (double*)malloc(sizeof(double) * dbl);
    int* imem = (int*)malloc(sizeof(int) * 2 * m->N * NB);
#pragma omp for schedule(dynamic, 4)
    for (int a = 0; a < n_agents; ++a) {
      solve_one(m, p + (long)a * NPAR, lbw + (long)a * NW, ubw + (long)a * NW, w_io + (long)a * NW,
                &o, &stats[a], mem, imem);
      ok += stats[a].status == 0 || stats[a].status == 1;
    }
    free(mem);
    free(imem);
  }
  return ok;
}

/* the hand-derived one_room model (the C3 checker) */
int oracle_room_solve_fleet(const room_t* rm, int n_agents, const double* p, const double* lbw,
                            const double* ubw, double* w_io, ostats_t* stats, const opts_t* opts,
                            int threads) {
  model_t m = {rm->N, rm->nx, rm->nv, rm->ng, rm->nps, rm->npg, rm->ts,
               room_fg_m, room_gj_m, room_hess_m, room_bounds_m, rm};
  return oracle_solve_fleet(&m, n_agents, p, lbw, ubw, w_io, stats, opts, threads);
}

int oracle_room_sizeof(void) { return (int)sizeof(room_t); }
int oracle_opts_sizeof(void) { return (int)sizeof(opts_t); }
