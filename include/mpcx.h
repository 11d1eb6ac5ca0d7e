/* mpcx.h — C ABI of the MI355X batched MPC / ADMM solver (libmpcx.so).
 *
 * Drop-in boundary for AgentLib-MPC's optimization backend hot path.  The
 * reference has no C ABI: its backends call CasADi/IPOPT from Python.  Each
 * entry point below replaces one reference interface (file:line relative to
 * the reference repository):
 *
 *   mpcx_problem_create   <- Discretization.initialize / SolverFactory.create_solver
 *                            (optimization_backends/casadi_/core/discretization.py:156-162,
 *                             data_structures/casadi_utils.py:282-300): load the generated
 *                             code object of one transcribed NLP structure.
 *   mpcx_problem_small_fleet <- the same call (a small-fleet specialisation, workspace in LDS)
 *   mpcx_batch_solve      <- self._optimizer(**nlp_inputs)
 *                            (optimization_backends/casadi_/core/discretization.py:203), i.e.
 *                            ca.nlpsol("mpc", "ipopt", ...)(p, x0, lbx, ubx, lbg, ubg),
 *                            batched over agents; outputs x, lam_g, lam_x and the
 *                            IPOPT-style stats (success, return_status, iter_count, obj).
 *   mpcx_admm_moments + mpcx_admm_finalize
 *                         <- ConsensusVariable.update_mean_trajectory / ExchangeVariable.
 *                            update_diff_trajectories (data_structures/admm_datatypes.py:221-236,
 *                            292-309), ADMM._set_mean_coupling_values
 *                            (modules/dmpc/admm/admm.py:528-570) and the residual norms of
 *                            ADMMCoordinator._check_convergence
 *                            (modules/dmpc/admm/admm_coordinator.py:354-435)
 *   mpcx_admm_consensus_multipliers
 *                         <- ConsensusVariable.update_multipliers (admm_datatypes.py:238-267),
 *                            ADMM.update_lambda (admm.py:612-633)
 *   mpcx_admm_exchange_update
 *                         <- ExchangeVariable.update_diff_trajectories / update_multiplier
 *                            (admm_datatypes.py:292-324), admm.py:550-570, 635-655
 *   mpcx_admm_shift       <- shift_values_by_one (admm_datatypes.py:275-282, 326-331)
 *   mpcx_admm_allreduce (+ mpcx_allreduce_register)
 *                         <- the coordinator's gather of the locals and broadcast of the means
 *                            (modules/dmpc/admm/admm_coordinator.py:284-314) across GPUs: ONE
 *                            RCCL all-reduce per ADMM iteration, issued by the library (v14)
 *   mpcx_gather_rows / mpcx_scatter_rows / mpcx_fill_column
 *                         <- moving coupling trajectories between Results and the
 *                            coordinator messages (modules/dmpc/admm/admm_coordinated.py:133-193)
 *
 * Conventions: all array arguments are DEVICE pointers (HBM-resident, fp64),
 * agent-major ([n_agents][len]).  Functions return 0 on success and a
 * negative mpcx_err code otherwise; nothing throws across the ABI.  Calls are
 * stream-ordered on the hipStream_t passed as `stream` (NULL = default
 * stream) and do not synchronise.  One host thread per handle.
 */
#ifndef MPCX_H
#define MPCX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPCX_API_VERSION 15

typedef enum mpcx_err {
  MPCX_OK = 0,
  MPCX_ERR_ARG = -1,
  MPCX_ERR_HIP = -2,
  MPCX_ERR_MODULE = -3,
  MPCX_ERR_DIMS = -4,
  MPCX_ERR_OOM = -5,
} mpcx_err;

/* per-agent solver status (IPOPT return_status equivalents) */
typedef enum mpcx_status {
  MPCX_SOLVE_SUCCEEDED = 0,          /* "Solve_Succeeded" */
  MPCX_SOLVED_TO_ACCEPTABLE = 1,     /* "Solved_To_Acceptable_Level" */
  MPCX_MAX_ITER_EXCEEDED = -1,       /* "Maximum_Iterations_Exceeded" */
  MPCX_RESTORATION_FAILED = -2,      /* "Restoration_Failed" (line search gave up) */
  MPCX_ERROR_IN_STEP = -3,           /* "Error_In_Step_Computation" */
  MPCX_INVALID_NUMBER = -4,          /* "Invalid_Number_Detected" */
  MPCX_INFEASIBLE = -5,              /* "Infeasible_Problem_Detected" (restoration converged to a
                                        point of local infeasibility) */
} mpcx_status;

/* Dimensions of one stage-structured NLP (must match the code object). */
typedef struct mpcx_problem_desc {
  int32_t n_stages;      /* N: prediction horizon */
  int32_t nx;            /* differential states per stage boundary */
  int32_t nv;            /* stage-local variables */
  int32_t ng;            /* constraints per stage */
  int32_t nps;           /* parameters per stage */
  int32_t npg;           /* global parameters */
  int32_t abi;           /* code object ABI version (MPCX_KERNEL_ABI) */
  int32_t reserved;
} mpcx_problem_desc;

/* IPOPT-named options (defaults: mpcx_default_options = IPOPT's own defaults).
 * Termination follows IPOPT's OptimalityErrorConvergenceCheck: "Solve_Succeeded" when the
 * scaled optimality error <= tol and the unscaled dual infeasibility, constraint violation
 * and complementarity are below dual_inf_tol / constr_viol_tol / compl_inf_tol;
 * "Solved_To_Acceptable_Level" after acceptable_iter consecutive iterates that meet the
 * acceptable_* tolerances (acceptable_iter = 0 disables the counter), or when the line search
 * fails at such an iterate.  The reference sets acceptable_tol 0.1, acceptable_iter 5,
 * acceptable_constr_viol_tol 1, acceptable_compl_inf_tol 1
 * (agentlib_mpc/data_structures/casadi_utils.py:197-206). */
typedef struct mpcx_options {
  double tol, dual_inf_tol, constr_viol_tol, compl_inf_tol;
  double acceptable_tol, acceptable_dual_inf_tol, acceptable_constr_viol_tol;
  double acceptable_compl_inf_tol, acceptable_obj_change_tol;
  double mu_init, mu_min, kappa_eps, kappa_mu, theta_mu, tau_min;
  double bound_push, bound_frac, bound_relax_factor, bound_mult_init_val;
  double constr_mult_init_max, kappa_sigma;
  double nlp_scaling_max_gradient, nlp_scaling_min_value;
  double delta_w_first, delta_w_min, delta_w_max;
  double kappa_w_plus_bar, kappa_w_plus, kappa_w_minus, delta_c_bar, kappa_c;
  double theta_max_fact, theta_min_fact, eta_phi, delta, s_phi, s_theta;
  double gamma_phi, gamma_theta, alpha_min_frac;
  int32_t max_iter, acceptable_iter;
  int32_t warm_start_mult; /* 1: use lam_g/lam_w inputs as initial multipliers */
  int32_t reserved;
} mpcx_options;

/* Per-agent result statistics (IPOPT stats() subset). */
typedef struct mpcx_stats {
  double obj;          /* objective at the solution (unscaled) */
  double primal_inf;   /* unscaled max constraint violation */
  double dual_inf;     /* unscaled max dual infeasibility */
  double compl_inf;    /* max complementarity */
  double mu;           /* final barrier parameter */
  double obj_scale;    /* gradient-based objective scaling factor */
  int32_t iter_count;
  int32_t status;      /* mpcx_status */
  int32_t n_inertia_corrections;
  int32_t n_restorations; /* calls of the feasibility restoration phase (IPOPT MinC_1Nrm) */
  int32_t n_factorizations;
  int32_t n_trials;    /* line-search trial points evaluated */
  int32_t n_block_chain; /* factorisations that fell back to the sequential block chain */
  int32_t n_dense_stages; /* stage factorisations redone densely (static sparse pivot rejected) */
  int32_t n_soft_restorations; /* line-search failures resolved by a soft restoration step */
  int32_t n_restoration_iters; /* iterations spent in the restoration phase (in iter_count) */
  int32_t n_filter_overflows;  /* filter insertions that dropped the oldest entry (cap 1024: 64 in
                                  LDS, the older ones in HBM; IPOPT's filter is unbounded, so 0
                                  means the run is IPOPT's) */
  int32_t n_refinement_steps;  /* iterative-refinement corrections of restoration-phase steps */
} mpcx_stats;

typedef struct mpcx_handle mpcx_handle;

int mpcx_version(void);
void mpcx_default_options(mpcx_options* opts);

/* Load a generated code object (hsaco) for one problem structure. */
int mpcx_problem_create(const mpcx_problem_desc* desc, const char* code_object_path,
                        mpcx_handle** out);
int mpcx_problem_destroy(mpcx_handle* h);
int mpcx_set_options(mpcx_handle* h, const mpcx_options* opts);
/* Pre-allocate workspace for up to n_agents (keeps the solve path allocation-free). */
int mpcx_reserve(mpcx_handle* h, int32_t n_agents);
/* Workspace bytes per agent (for capacity planning on 288 GB HBM). */
int64_t mpcx_workspace_bytes_per_agent(const mpcx_handle* h);
/* LDS bytes of one agent's workgroup on the main build (C ABI v15; -1 without a handle) */
int64_t mpcx_lds_bytes_per_agent(const mpcx_handle* h);
/* Small-fleet specialisation of the same structure (replaces the same reference call as
 * mpcx_problem_create, for a handful of agents -- the reference's usual one MPC agent per
 * process, core/discretization.py:203): a second code object built with the agent's
 * workspace in LDS (MPCX_WS_LDS, one agent per CU), so that every operand round trip of the
 * IPM is an LDS access instead of an L2 / HBM one.  code_object_path NULL keeps the loaded
 * one.  mpcx_batch_solve launches it for batches of at most max_agents agents
 * (max_agents < 0: one generation -- the CU count times the agents a CU's LDS holds of this
 * build, at most four; 0: never).  Returns
 * MPCX_ERR_MODULE if the code object is not such a variant of this structure. */
int mpcx_problem_small_fleet(mpcx_handle* h, const char* code_object_path, int32_t max_agents);

/* Optional (C ABI v9): the same structure compiled for one wave per SIMD (MPCX_MIN_WAVES=1: up
 * to 512 registers per lane, where the main build's budget follows its LDS-limited occupancy,
 * e.g. 128 at 16 agents per CU, and spills).  mpcx_batch_solve launches it for batches of at
 * most max_agents agents that the small-fleet build does not take (max_agents < 0: four per CU,
 * one generation at one wave per SIMD; 0: never).  Ignored (max 0) when the main build already
 * runs one wave per SIMD.  Returns MPCX_ERR_MODULE if the code object is not such a variant. */
int mpcx_problem_mid_fleet(mpcx_handle* h, const char* code_object_path, int32_t max_agents);

/* Optional (C ABI v13): the same structure compiled for more agents per CU than the main build
 * holds (MPCX_APC=20 where the main build holds 16: a smaller LDS share and register budget per
 * agent).  mpcx_batch_solve launches it for batches of at least min_agents agents that neither
 * the small-fleet nor the one-wave-per-SIMD build takes (min_agents < 0: more than one
 * generation of the main build, its agents per CU x the CU count; 0: never).  Returns
 * MPCX_ERR_MODULE if the code object is not such a variant (HBM workspace, same workspace, more
 * agents per CU than the main build). */
int mpcx_problem_wide_fleet(mpcx_handle* h, const char* code_object_path, int32_t min_agents);

/* Batched solve.  Shapes (agent-major, fp64, device):
 *   active [n_agents] int32 or NULL  agents with active[a] == 0 are skipped (their outputs
 *                                     are left untouched): converged ADMM blocks
 *   p      [n_agents][np]            np = npg + n_stages*nps   (reference p order)
 *   lbw/ubw[n_agents][nw]            nw = nx + n_stages*(nv+nx) (reference x order)
 *   lbg/ubg[n_agents][ng_total] or NULL (then computed from the generated bound
 *                                     expressions in p)        ng_total = n_stages*ng
 *   w_io   [n_agents][nw]            initial guess in, solution out
 *   lam_g  [n_agents][ng_total] or NULL   constraint multipliers out (in if warm_start_mult)
 *   lam_w  [n_agents][nw] or NULL         bound multipliers out (z_U - z_L)
 *   stats  [n_agents]  or NULL
 */
int mpcx_batch_solve(mpcx_handle* h, int32_t n_agents, const double* p, const double* lbw,
                     const double* ubw, const double* lbg, const double* ubg, double* w_io,
                     double* lam_g, double* lam_w, mpcx_stats* stats, const int32_t* active,
                     void* stream);

/* Mapped launch (C ABI v11): n_launch workgroups, workgroup i solving agent agent_map[i] of the
 * n_agents-agent arrays above (agent_map[i] < 0: no agent; device int32 [n_launch]).  The code
 * object is chosen by n_launch, not n_agents: a coordinated fleet whose blocks have mostly met
 * their stopping rule launches only the agents still active (mpcx_active_map compacts them) and
 * runs them on the small-fleet build however large the class is -- the straggling blocks of
 * ADMMCoordinator (admm_coordinator.py:284-309), each waiting on its agents' solves
 * (modules/dmpc/admm/admm_coordinated.py:133-193).  agent_map NULL: n_launch must equal
 * n_agents (= mpcx_batch_solve). */
int mpcx_batch_solve_mapped(mpcx_handle* h, int32_t n_agents, int32_t n_launch, const int32_t* agent_map,
                            const double* p, const double* lbw, const double* ubw, const double* lbg,
                            const double* ubg, double* w_io, double* lam_g, double* lam_w, mpcx_stats* stats,
                            const int32_t* active, void* stream);

/* Host round trip of a small batch in ONE call (C ABI v8): the reference's usual deployment
 * is one MPC agent per process whose do_step blocks on its solve (modules/mpc/mpc.py:322-340 ->
 * core/discretization.py:203).  Copies in_bytes from host_in to dev_in (pinned host memory
 * makes it asynchronous), runs mpcx_batch_solve on the device buffers (p, lbw, ubw, w_io,
 * lam_g, stats: typically views into dev_in / dev_out), copies out_bytes from dev_out back to
 * host_out and waits for the stream: on return the solution and stats are on the host.  One
 * call instead of an upload, a launch, a read-back and a wait (each a host API call).  in_bytes
 * or out_bytes 0 skips that copy. */
int mpcx_batch_solve_staged(mpcx_handle* h, int32_t n_agents, const void* host_in, void* dev_in,
                            int64_t in_bytes, void* host_out, const void* dev_out, int64_t out_bytes,
                            const double* p, const double* lbw, const double* ubw, double* w_io,
                            double* lam_g, mpcx_stats* stats, void* stream);

/* ---- ADMM kernels (agent-batched) --------------------------------------------------
 * Local trajectories are rows of `locals` [n_rows][T] (fp64, device).  The participants
 * of one coupling alias ("group") are the contiguous rows gstart[g] .. gstart[g+1]-1
 * (device int32 array); max_group_rows = max over g of the group size (host value, sizes
 * the launch grid).  Groups [0, n_global) may have participants on other GPUs: their
 * moments are all-reduced (RCCL, sum) between mpcx_admm_moments and mpcx_admm_finalize;
 * groups [n_global, n_groups) are GPU-local.
 *
 * Blocks: the groups form n_blocks independent consensus problems, each the counterpart of
 * one reference ADMMCoordinator (block_g[g] = block of group g; NULL when n_blocks == 1).
 * Residual totals are kept per block, each group may carry its own penalty rho_g[g]
 * (NULL: the scalar rho for all) and groups with active_g[g] == 0 (NULL: all active) are
 * frozen — the blocks that already met their stopping rule.  One ADMM iteration of the
 * reference coordinator (admm_coordinator.py:288-304) is
 *   moments -> [all-reduce (sum) of the first mpcx_admm_reduce_count(...) doubles] -> finalize
 *   -> consensus_multipliers / exchange_update -> scatter into the NLP parameters.
 *
 * Block numbering with several ranks: the blocks that contain a global group (participants on
 * more than one rank) are numbered FIRST, 0 .. n_global_blocks-1, identically on every rank;
 * each rank numbers its rank-local blocks after them (n_global_blocks .. n_blocks-1, so the
 * same number means different blocks on different ranks).  Only the first n_global_blocks
 * blocks' totals are summed over the ranks; summing a rank-local block's totals would add
 * unrelated blocks' residuals.
 */
#define MPCX_ADMM_TOTALS 8
/* doubles in a moments buffer (zero it before mpcx_admm_moments):
 *   [n_global x (5T+1) global-group moments][n_blocks x MPCX_ADMM_TOTALS totals][local groups]
 *   <- the per-alias sums of ADMMCoordinator._check_convergence (admm_coordinator.py:354-435) */
int64_t mpcx_admm_moments_size(int32_t n_groups, int32_t n_blocks, int32_t T);
/* The ONE collective per ADMM iteration (C ABI v10).  The caller keeps MPCX_ADMM_CONTROL control
 * doubles immediately BEFORE the moments buffer ([control][moments buffer], one allocation; the
 * kernels get the moments buffer, zero only it before mpcx_admm_moments) and all-reduces (sum)
 *   mpcx_admm_reduce_count(...) = MPCX_ADMM_CONTROL + n_global*(5T+1) + n_global_blocks*MPCX_ADMM_TOTALS
 * doubles starting at the control: the coordinated loop's number of blocks still active
 * (written by mpcx_admm_block_stop's `control` output), the global-group moments, then the
 * totals of the rank-spanning blocks, which are numbered first.  After the reduce the control
 * holds the count over all ranks after the PREVIOUS iteration: every rank reads the same value
 * and leaves the loop at the same iteration, with no second collective.  Single rank: nothing
 * to reduce.  <- the one exchange per ADMM iteration of admm_coordinator.py:288-304 when the
 * agents sit on several GPUs. */
#define MPCX_ADMM_CONTROL 1
int64_t mpcx_admm_reduce_count(int32_t n_global, int32_t n_global_blocks, int32_t T);

/* Per (group, t) moments of the locals about center = the current mean [n_groups][T]:
 * sum(x-c), sum(x-c)^2 and, if multipliers != NULL (consensus rows), sum lam, sum lam^2,
 * sum lam*(x-c); plus the participant count.  ADDED into `out`.
 *   <- ConsensusVariable.update_mean_trajectory (admm_datatypes.py:221-236),
 *      ExchangeVariable.update_diff_trajectories (:292-309), ADMM._set_mean_coupling_values
 *      (modules/dmpc/admm/admm.py:528-570) — the participant sums of np.mean(axis=0). */
int mpcx_admm_moments(int32_t n_groups, int32_t n_global, int32_t n_blocks, int32_t T,
                      const int32_t* gstart, int32_t max_group_rows, const double* locals,
                      const double* multipliers, const double* center, double* out, void* stream);

/* Active groups [g_begin, g_end): mean <- c + S1/n, delta_mean <- c - mean (groups without
 * participants keep both); ADDS to totals[block_g[g]][0..7]:
 *   {||r||^2, ||rho*delta_mean||^2, ||X||_F^2, ||mean||^2, ||Lambda_new||^2,
 *    #trajectories, #flat_multipliers, #groups}
 * with the reference's conventions: consensus r = mean - x_i and Lambda_new the updated
 * per-participant multipliers; exchange (exchange[g] != 0) r = mean and Lambda_new =
 * group_multipliers + rho*mean  <- ADMMCoordinator._check_convergence
 * (admm_coordinator.py:354-435), CouplingVariable.get_residual (admm_datatypes.py:202-214). */
int mpcx_admm_finalize(int32_t g_begin, int32_t g_end, int32_t n_global, int32_t n_blocks, int32_t T,
                       const double* moments, const int32_t* exchange,
                       const double* group_multipliers, double rho, const double* rho_g,
                       const int32_t* active_g, const int32_t* block_g, double* mean,
                       double* delta_mean, double* totals, void* stream);

/* consensus: r = mean[g] - x_i ; lambda_i <- lambda_i - rho_g * r  (res may be NULL)
 *   <- ConsensusVariable.update_multipliers (admm_datatypes.py:238-267),
 *      ADMM.update_lambda (admm.py:612-633) */
int mpcx_admm_consensus_multipliers(int32_t n_groups, int32_t T, const int32_t* gstart,
                                    int32_t max_group_rows, const double* locals,
                                    const double* mean, double rho, const double* rho_g,
                                    const int32_t* active_g, double* multipliers,
                                    double* primal_residual, void* stream);
/* exchange: diff_i <- x_i - mean[g]; if update_multiplier: lambda[g] <- lambda[g] + rho_g*mean[g]
 *   <- ExchangeVariable.update_diff_trajectories / update_multiplier
 *      (admm_datatypes.py:292-324), admm.py:550-570, 635-655 */
int mpcx_admm_exchange_update(int32_t n_groups, int32_t T, const int32_t* gstart,
                              int32_t max_group_rows, const double* locals, const double* mean,
                              double* diff, double* multiplier, int32_t update_multiplier,
                              double rho, const double* rho_g, const int32_t* active_g,
                              void* stream);
/* Participation (the reference coordinator's active agents, admm_coordinator.py:323-353:
 * only the sources with status `ready` enter means, multiplier updates and residuals,
 * ConsensusVariable/ExchangeVariable(..., sources=active_agents), admm_datatypes.py:171-331).
 * The *_masked variants take row_on[n_rows] (device int32; NULL = all rows): rows with
 * row_on == 0 are left out of the moments (sums and participant count), keep their
 * multiplier (consensus) and their diff (exchange).  The unmasked entry points above are
 * these with row_on = NULL. */
int mpcx_admm_moments_masked(int32_t n_groups, int32_t n_global, int32_t n_blocks, int32_t T,
                             const int32_t* gstart, int32_t max_group_rows, const double* locals,
                             const double* multipliers, const double* center, const int32_t* row_on,
                             double* out, void* stream);
int mpcx_admm_consensus_multipliers_masked(int32_t n_groups, int32_t T, const int32_t* gstart,
                                           int32_t max_group_rows, const double* locals,
                                           const double* mean, double rho, const double* rho_g,
                                           const int32_t* active_g, const int32_t* row_on,
                                           double* multipliers, double* primal_residual, void* stream);
int mpcx_admm_exchange_update_masked(int32_t n_groups, int32_t T, const int32_t* gstart,
                                     int32_t max_group_rows, const double* locals, const double* mean,
                                     double* diff, double* multiplier, int32_t update_multiplier,
                                     double rho, const double* rho_g, const int32_t* active_g,
                                     const int32_t* row_on, void* stream);
/* Shift rows by one control interval: x[i][:] <- x[i][shift:] ++ x[i][T-shift:]
 *   <- ConsensusVariable/ExchangeVariable.shift_values_by_one (admm_datatypes.py:275-282,
 *      326-331), ADMM._shift (admm.py:329-342) */
int mpcx_admm_shift(int32_t n_rows, int32_t T, int32_t shift, double* x, void* stream);

/* ---- the coordinators' stopping test on the device -------------------------------------
 * After mpcx_admm_finalize of ADMM iteration `it` (1-based), one thread per block applies
 * ADMMCoordinator._check_convergence (admm_coordinator.py:354-435) to the block's totals:
 * prim = sqrt(t0), dual = sqrt(t1); use_relative: prim < sqrt(t6)*abs_tol + rel_tol*max(sqrt(t2),
 * sqrt(t3)) and dual < sqrt(t5)*abs_tol + rel_tol*sqrt(t4), else prim < primal_tol and
 * dual < dual_tol.  Active blocks vary their penalty (change_threshold > 1: rho*factor if
 * prim > threshold*dual, rho/factor if dual > threshold*prim; admm_coordinator.py:467-479) and
 * record[it-1][b] = {prim, dual, rho after variation, active} (:396-402); a block meeting its
 * rule is frozen (active_b[b] = 0, iters_b[b] = it, the loop of :288-304).  n_active[it] (zero
 * it first) receives the number of blocks still active, clock[it] the device wall clock
 * (mpcx_device_clock_khz ticks; it = 0 stamps the clock and counts the blocks with
 * active_b != 0 into n_active[0]).  n_active / clock may be NULL.  control (C ABI v10, may be
 * NULL; needs n_active): receives n_active[it] as a double -- the control slot of the next
 * iteration's all-reduce (mpcx_admm_reduce_count). */
int mpcx_admm_block_stop(int32_t n_blocks, int32_t it, const double* totals, int32_t use_relative,
                         double abs_tol, double rel_tol, double primal_tol, double dual_tol,
                         double change_threshold, double change_factor, double* rho_b, int32_t* active_b,
                         int32_t* iters_b, double* record, int32_t* n_active, int64_t* clock, double* control,
                         void* stream);
/* Block state to groups / agents: out_active[i] = active_b[idx[i]] (and part[i] != 0 when
 * part != NULL: the participation mask), out_rho[i] = rho_b[idx[i]]; either output may be NULL. */
int mpcx_admm_block_expand(int32_t n, const int32_t* idx, const int32_t* active_b, const double* rho_b,
                           const int32_t* part, int32_t* out_active, double* out_rho, void* stream);
/* Compaction of an active mask (C ABI v11): map[0 .. count-1] <- the indices i with active[i] != 0
 * in increasing order, map[count .. n-1] <- -1, count[0] <- count (device int32).  The agent map
 * of mpcx_batch_solve_mapped; the host reads count with the stopping test's n_active, so the
 * launch size of the next iterations is known without an extra synchronisation. */
int mpcx_active_map(int32_t n, const int32_t* active, int32_t* map, int32_t* count, void* stream);
/* Rate of the device wall clock the stopping test stamps (kHz). */
int64_t mpcx_device_clock_khz(void);

/* Fleet bookkeeping of one batched solve (C ABI v9): counts[0] += agents whose status is
 * MPCX_SOLVE_SUCCEEDED or MPCX_SOLVED_TO_ACCEPTABLE, counts[1] += their restoration-phase calls
 * (mpcx_stats.n_restorations); agents with active[i] == 0 are skipped (active NULL: all).
 * counts: device int64[2], accumulated across calls (the converged-solve count the reference's
 * modules log per solve, `mpc.py:397-400`, summed over a round). */
int mpcx_stats_count(int32_t n, const mpcx_stats* stats, const int32_t* active, int64_t* counts, void* stream);
/* The per-iteration bookkeeping of several agent classes in ONE launch each (C ABI v15): desc holds
 * n_desc descriptors in DEVICE memory (built once per round / class set).
 * block_expand_multi: desc k = (n, idx, part or 0, out_active or 0, out_rho or 0), MPCX_EXPAND_DESC
 *   int64 words: mpcx_admm_block_expand of each (active_b, rho_b common), n <= max_n;
 * stats_count_multi: desc k = (n, stats, active or 0), MPCX_STATS_DESC words: mpcx_stats_count of
 *   each into the one counts pair. */
#define MPCX_EXPAND_DESC 5
#define MPCX_STATS_DESC 3
int mpcx_admm_block_expand_multi(int32_t n_desc, const int64_t* desc, int32_t max_n, const int32_t* active_b,
                                 const double* rho_b, void* stream);
int mpcx_stats_count_multi(int32_t n_desc, const int64_t* desc, int32_t max_n, int64_t* counts, void* stream);

/* ---- NLP vector <-> trajectory moves (no host round trip) ----------------------------
 * dst[dst_rows[a]][t] <- src[a*src_ld + cols[t]]: the coupling trajectories out of the
 * solutions w  <- Results[coupling.name] in CoordinatedADMM.optimize
 * (modules/dmpc/admm/admm_coordinated.py:170-184) / ADMM.send_coupling_values. */
int mpcx_gather_rows(int32_t n_agents, int32_t T, const double* src, int64_t src_ld,
                     const int32_t* cols, double* dst, const int32_t* dst_rows, void* stream);
/* dst[a*dst_ld + cols[t]] <- src[src_rows[a]][t] (src_rows NULL: row a): means,
 * diffs and multipliers into the NLP parameters p  <- the MPCVariable updates of
 * CoordinatedADMM.optimize (admm_coordinated.py:147-163) sampled by
 * CasADiBackend._get_current_mpc_inputs (core/casadi_backend.py:141-253). */
int mpcx_scatter_rows(int32_t n_agents, int32_t T, const double* src, const int32_t* src_rows,
                      double* dst, int64_t dst_ld, const int32_t* cols, void* stream);
/* dst[a*dst_ld + col] <- value (the penalty factor rho into p). */
int mpcx_fill_column(int32_t n_agents, double* dst, int64_t dst_ld, int32_t col, double value,
                     void* stream);
/* Several row moves in ONE launch (C ABI v12): the per-iteration marshalling of an ADMM class --
 * every coupling slot's mean / multiplier columns and the block penalty into p, every slot's
 * local trajectory out of w -- was one launch per move.  desc: n_desc descriptors of
 * MPCX_MOVE_DESC int64 words in DEVICE memory (built once per class).
 * scatter: desc k = (src, src_rows or 0, cols, T): dst[i * dst_ld + cols[t]] = src[src_rows[i] * T + t]
 * gather:  desc k = (dst, dst_rows, cols, T):     dst[dst_rows[i] * T + t] = src[i * src_ld + cols[t]]
 * for i < n_agents, t < T (<= max_T).  The moves of one call must not write the same element
 * (rows mapped to a shared scratch row excepted: what lands there is never read). */
#define MPCX_MOVE_DESC 4
int mpcx_scatter_rows_multi(int32_t n_agents, int32_t n_desc, const int64_t* desc, int32_t max_T, double* dst,
                            int64_t dst_ld, void* stream);
int mpcx_gather_rows_multi(int32_t n_agents, int32_t n_desc, const int64_t* desc, int32_t max_T,
                           const double* src, int64_t src_ld, void* stream);

/* ---- the collective of an ADMM iteration, issued by the library (C ABI v14) -----------------
 * SURVEY §8b `mpcx_allreduce_register(comm)`: the one all-reduce per ADMM iteration (sum, fp64, in
 * place, mpcx_admm_reduce_count doubles from the control on; see MPCX_ADMM_CONTROL) goes through
 * mpcx_admm_allreduce, which issues it on the registered transport.  It replaces the exchange of
 * the reference coordinator's round (modules/dmpc/admm/admm_coordinator.py:284-314: every agent's
 * locals gathered, the means sent back) when the fleet's agents sit on several GPUs.  One transport
 * per process (one process per GPU), registered before the loop:
 *   mpcx_allreduce_register(comm, rccl_library): an RCCL communicator (ncclComm_t).  RCCL is loaded
 *     with dlopen (an already loaded copy first: a communicator must be used with the library that
 *     created it; NULL = "librccl.so.1") and ncclAllReduce runs on the `stream` of each call.
 *   mpcx_allreduce_register_fn(fn, ctx): any other transport; fn(ctx, buf, count, stream) sums
 *     `count` doubles at `buf` over the ranks in place and returns 0.
 * mpcx_rccl_comm_init (unique id from mpcx_rccl_unique_id on rank 0, passed to every rank by the
 * caller) or mpcx_rccl_comm_init_file (rank 0 writes the id to `id_path` -- a path no earlier run
 * left behind --, the other ranks read it, waiting up to timeout_ms) make the communicator, so a C
 * caller needs no collective library of its own. */
#define MPCX_ERR_COMM (-6)
#define MPCX_RCCL_ID_BYTES 128
#define MPCX_COLLECTIVE_NONE 0
#define MPCX_COLLECTIVE_RCCL 1
#define MPCX_COLLECTIVE_FN 2
typedef int (*mpcx_allreduce_fn)(void* ctx, double* buf, int64_t count, void* stream);
int mpcx_allreduce_register(void* comm, const char* rccl_library);
int mpcx_allreduce_register_fn(mpcx_allreduce_fn fn, void* ctx);
int mpcx_allreduce_unregister(void);
/* the registered transport: MPCX_COLLECTIVE_NONE / _RCCL / _FN */
int mpcx_allreduce_kind(void);
/* sum `count` doubles at `buf` over the ranks, in place, stream-ordered (MPCX_ERR_COMM when no
 * transport is registered or it failed) */
int mpcx_admm_allreduce(double* buf, int64_t count, void* stream);
/* collectives issued through mpcx_admm_allreduce since the library was loaded */
int64_t mpcx_allreduce_calls(void);
int mpcx_rccl_unique_id(const char* rccl_library, void* id /* MPCX_RCCL_ID_BYTES */);
int mpcx_rccl_comm_init(const char* rccl_library, int32_t nranks, int32_t rank, const void* id, void** comm);
int mpcx_rccl_comm_init_file(const char* rccl_library, const char* id_path, int32_t nranks, int32_t rank,
                             int32_t timeout_ms, void** comm);
int mpcx_rccl_comm_destroy(const char* rccl_library, void* comm);

/* ---- streams (C ABI v15) --------------------------------------------------------------------
 * A HIP stream with a hardware queue of its own (hipExtStreamCreateWithCUMask over every CU of
 * the current device).  Ordinary streams of a process share the runtime's few hardware queues
 * (GPU_MAX_HW_QUEUES, 4 by default): two agent classes' solves on two such streams can land on
 * one queue and run one after the other (r06: the C2 rooms and air handlers);
 * an ADMM fleet gives each class a dedicated stream so that their launches overlap. */
int mpcx_stream_create_dedicated(void** stream);
int mpcx_stream_destroy(void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MPCX_H */
