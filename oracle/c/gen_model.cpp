// ORACLE (test infrastructure only) — host build of one GENERATED stage model
// (agentlib_mpc_amd.runtime.codegen output, compiled with g++ instead of hipcc) plugged
// into the C IPM restatement (ipm_oracle.c) through its stage-model interface.
//
// Used only as the CPU baseline of the configurations without a hand-derived oracle
// model (C2, C4, C5 agents): IPOPT's algorithm on host cores over generated
// straight-line model code — what the reference does with CasADi code generation and
// IPOPT.  Parity is never judged against this build (the checkers are oracle/ipm.py with
// oracle/nlps.py, and the hand-derived one_room model of ipm_oracle.c).
//
// Build: oracle/cbuild.py build_generated(gen) -DMPCX_GEN_SOURCE="<filtered generated source>"
#include <cmath>
#include <cstring>

#define __device__
#define __forceinline__ inline
#define __constant__ static const
#include MPCX_GEN_SOURCE

extern "C" {
#include "ipm_oracle.h"
}

namespace {
constexpr int NL = 2 * MPCX_NX + MPCX_NV;
constexpr int NLOC_MAX = MPCX_NV + MPCX_NG + 2 * MPCX_NX;
constexpr int LP_SIZE = (NLOC_MAX + 2) * (NLOC_MAX + 3) / 2 + 1;
double g_ones[MPCX_NG > 0 ? MPCX_NG : 1];
const double g_zeros[MPCX_NG > 0 ? MPCX_NG : 1] = {};

void m_fg(const model_t*, const double* L, const double* PS, const double* PG, double TK, double* f, double* g) {
  double fv = 0.0;
  gen_stage_fg(L, PS, PG, TK, &fv, g, 1);
  *f = fv;
}
void m_gj(const model_t*, const double* L, const double* PS, const double* PG, double TK, double* grad,
          double* jac) {
  thread_local double lp[LP_SIZE], jtl[NL];
  gen_stage_gj(L, PS, PG, TK, grad, jac, 1, g_ones, lp, g_zeros, jtl, 1);
}
void m_hess(const model_t*, const double* L, const double* PS, const double* PG, double TK, double sigma,
            const double* lam, double* H) {
  thread_local double lp[LP_SIZE];
  gen_stage_hess(L, PS, PG, TK, sigma, lam, H, 1, lp, 1);
}
void m_bounds(const model_t*, const double* PS, const double* PG, double TK, double* lb, double* ub) {
  gen_stage_bounds(PS, PG, TK, lb, ub, 1);
}
}  // namespace

extern "C" int oracle_gen_solve_fleet(int n_agents, const double* p, const double* lbw, const double* ubw,
                                      double* w_io, ostats_t* stats, const opts_t* opts, int threads) {
  for (int r = 0; r < MPCX_NG; ++r) g_ones[r] = 1.0;
  static_assert(NL > 0, "empty stage");
  model_t m = {MPCX_N, MPCX_NX, MPCX_NV, MPCX_NG, MPCX_NPS, MPCX_NPG, MPCX_TS, m_fg, m_gj, m_hess, m_bounds, nullptr};
  return oracle_solve_fleet(&m, n_agents, p, lbw, ubw, w_io, stats, opts, threads);
}

extern "C" int oracle_gen_dims(int* out) {
  out[0] = MPCX_N; out[1] = MPCX_NX; out[2] = MPCX_NV; out[3] = MPCX_NG; out[4] = MPCX_NPS; out[5] = MPCX_NPG;
  return 6;
}
