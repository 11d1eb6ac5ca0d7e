/* ORACLE (test infrastructure only) — interface of the C IPM restatement (ipm_oracle.c):
 * the stage-model interface, IPOPT termination options, per-agent stats, fleet solve. */
#ifndef IPM_ORACLE_H
#define IPM_ORACLE_H

/* --------------------------------------------------------------------------
 * stage-model interface: local L = [X0 (nx), V (nv), X1 (nx)], per-stage
 * parameters PS, global parameters PG, stage start time TK
 * -------------------------------------------------------------------------- */
typedef struct model_s model_t;
struct model_s {
  int N, nx, nv, ng, nps, npg;
  double ts;
  void (*fg)(const model_t*, const double* L, const double* PS, const double* PG, double TK, double* f, double* g);
  /* grad [nl], jac [ng][nl] (dense, zero-initialised by the caller) */
  void (*gj)(const model_t*, const double* L, const double* PS, const double* PG, double TK, double* grad, double* jac);
  /* Hessian of sigma*f + lam^T g, dense symmetric [nl][nl] (zero-initialised by the caller) */
  void (*hess)(const model_t*, const double* L, const double* PS, const double* PG, double TK, double sigma,
               const double* lam, double* H);
  void (*bounds)(const model_t*, const double* PS, const double* PG, double TK, double* lb, double* ub);
  const void* data;
};

/* IPOPT termination options (OptimalityErrorConvergenceCheck); the reference sets
   tol 1e-4, max_iter 100, acceptable_tol 0.1, acceptable_iter 5,
   acceptable_constr_viol_tol 1, acceptable_compl_inf_tol 1 (casadi_utils.py:197-206) */
typedef struct {
  double tol, dual_inf_tol, constr_viol_tol, compl_inf_tol;
  double acceptable_tol, acceptable_dual_inf_tol, acceptable_constr_viol_tol;
  double acceptable_compl_inf_tol, acceptable_obj_change_tol;
  int max_iter, acceptable_iter;
} opts_t;

/* status: 0 Solve_Succeeded, 1 Solved_To_Acceptable_Level, -1 Maximum_Iterations_Exceeded,
   -2 Restoration_Failed, -3 Error_In_Step_Computation, -4 Invalid_Number_Detected,
   -5 Infeasible_Problem_Detected (the mpcx_status codes) */
typedef struct {
  double obj;
  int iter, status, n_fact, n_trials;
  int n_soft, n_resto, n_resto_iters, n_filter_over, n_refine;
} ostats_t;

/* Solve n_agents NLPs of one stage model (agent-major p/lbw/ubw/w_io, kernel layout);
   returns the number that succeeded (Solve_Succeeded or Solved_To_Acceptable_Level). */
int oracle_solve_fleet(const model_t* m, int n_agents, const double* p, const double* lbw, const double* ubw,
                       double* w_io, ostats_t* stats, const opts_t* opts, int threads);

#endif
