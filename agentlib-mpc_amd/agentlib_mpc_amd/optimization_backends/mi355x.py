"""The MI355X optimization backends (drop-in for the CasADi/IPOPT backends).

``MI355XBackend``      <- ``CasADiFullBackend`` (type ``"casadi"``, `casadi_/full.py:169-179`)
``MI355XBaseBackend``  <- ``CasADiBaseBackend`` (type ``"casadi_basic"``, `casadi_/basic.py:555-564`)
``MI355XADMMBackend``  <- ``CasADiADMMBackend`` (type ``"casadi_admm"``, `casadi_/admm.py:341-424`)

Same config schema (``CasadiBackendConfig``, `core/casadi_backend.py:40-92`),
same ``setup_optimization(var_ref)`` / ``solve(now, current_vars) -> Results``
contract (`core/casadi_backend.py:108-139`), same variable/parameter layout and
``Results`` format.  The NLP is solved by the generated HIP interior-point
kernel.  IPOPT options given in ``solver.options`` (``{"ipopt": {...}}`` or
``"ipopt.<key>"``) are mapped onto the kernel options; the reference's
defaults (`data_structures/casadi_utils.py:197-206`: ``max_iter=100``,
``tol=1e-4``, ``acceptable_tol=0.1``, ``acceptable_iter=5``,
``acceptable_constr_viol_tol=1``, ``acceptable_compl_inf_tol=1``) are applied
unless overridden, and the kernel terminates with IPOPT's semantics
(``Solve_Succeeded`` / ``Solved_To_Acceptable_Level``, both ``success``).

Besides the per-agent ``solve``, ``solve_batch`` solves many agents of the
same structure in one launch (the fleet path used by the ADMM drivers).
"""

from __future__ import annotations

import time
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import numpy as np
import pydantic

from agentlib_mpc_amd.data_structures import admm_datatypes as adt
from agentlib_mpc_amd.data_structures.mpc_datamodels import (
    CasadiDiscretizationOptions, DiscretizationMethod, SolverOptions, stats_path,
)
from agentlib_mpc_amd.models.casadi_model import CasadiModel
from agentlib_mpc_amd.optimization_backends import discretization as disc
from agentlib_mpc_amd.optimization_backends import narx
from agentlib_mpc_amd.optimization_backends.backend import (
    ADMMBackend, BackendConfig, OptimizationBackend,
)
from agentlib_mpc_amd.optimization_backends.problem import CompiledProblem
from agentlib_mpc_amd.optimization_backends.results import Results
from agentlib_mpc_amd.optimization_backends.system import ADMMSystem, BaseSystem, FullSystem

#: reference IPOPT defaults (`casadi_utils.py:197-206`); options not named here keep
#: IPOPT's own defaults (``mpcx_default_options``)
REFERENCE_IPOPT_DEFAULTS = {"max_iter": 100, "tol": 1e-4, "acceptable_tol": 0.1,
                            "acceptable_constr_viol_tol": 1.0, "acceptable_iter": 5,
                            "acceptable_compl_inf_tol": 1.0}
#: reference fatrop defaults (`casadi_utils.py:173-178`): the acceptable tolerances stay at
#: the solver library's own defaults
REFERENCE_FATROP_DEFAULTS = {"max_iter": 100, "tol": 1e-4}


class MI355XBackendConfig(BackendConfig):
    discretization_options: CasadiDiscretizationOptions = pydantic.Field(
        default_factory=CasadiDiscretizationOptions)
    solver: SolverOptions = pydantic.Field(default_factory=SolverOptions)
    build_batch_bat: Optional[Path] = None
    do_jit: Optional[bool] = None
    save_only_stats: bool = False


#: solvers the kernel stands in for: both are primal-dual interior-point methods on
#: the same NLP (fatrop exploits the stage structure like the kernel does;
#: `casadi_utils.py:163-217`); the others (SQP, QP, MINLP) are not on this path
KERNEL_SOLVERS = ("ipopt", "fatrop")


def ipopt_options_to_kernel(options: dict, solver: str = "ipopt") -> dict:
    """Map IPOPT-style options (nested or dotted) onto kernel option names.

    ``solver="fatrop"`` reads the nested ``"fatrop"`` dict instead (the reference
    merges it into fatrop's own options, `casadi_utils.py:163-189`; its defaults
    max_iter=100, tol=1e-4 equal the IPOPT ones); fatrop's ``structure_detection``
    and ``equality`` flags describe what the kernel derives itself."""
    opts = dict(REFERENCE_IPOPT_DEFAULTS if solver == "ipopt" else REFERENCE_FATROP_DEFAULTS)
    nested = dict(options.get(solver, {}))
    for k, v in options.items():
        if k.startswith(f"{solver}."):
            nested[k[len(solver) + 1:]] = v
    aliases = {"mu_linear_decrease_factor": "kappa_mu", "mu_superlinear_decrease_power": "theta_mu",
               "barrier_tol_factor": "kappa_eps", "bound_mult_init_val": "bound_mult_init_val",
               "constr_mult_init_max": "constr_mult_init_max",
               "alpha_min_frac": "alpha_min_frac"}
    ignored = {"print_level", "sb", "print_time", "linear_solver", "hessian_approximation",
               "structure_detection", "equality", "verbose", "record_time", "expand"}
    for k, v in nested.items():
        if k in ignored:
            continue
        opts[aliases.get(k, k)] = v
    return opts


class MI355XBackend(OptimizationBackend):
    """Backend ``"casadi"`` replacement (full system with ``u_prev``)."""

    system_type = FullSystem
    discretization_types = {
        DiscretizationMethod.collocation: disc.FullCollocation,
        DiscretizationMethod.multiple_shooting: disc.FullMultipleShooting,
    }
    _supported_models = {"CasadiModel": CasadiModel}
    config_type = MI355XBackendConfig
    #: `core/discretization.py:126`: ``Results[name]`` keeps only t >= 0
    only_positive_times_in_results = True

    def __init__(self, config: dict):
        super().__init__(config)
        self.problem: Optional[CompiledProblem] = None
        self.system = None
        self._remembered: Optional[np.ndarray] = None  # [n, nw] last optimum per batch slot (host path)
        self._resident = None  # device-resident inputs + warm start of the plugin batch (plugin_batch.py)
        self._slot_ids: Optional[list] = None  # agent key of each batch slot (solve_batch agent_ids)
        name = getattr(self.config.solver.name, "value", self.config.solver.name)
        if name not in KERNEL_SOLVERS:
            raise ValueError(f"solver {name!r} is not available on the MI355X backend "
                             f"(interior-point solvers {KERNEL_SOLVERS} run on the batched kernel)")
        self.solver_options = ipopt_options_to_kernel(self.config.solver.options, name)

    # -- setup (`core/casadi_backend.py:108-131`) --------------------------------
    def setup_optimization(self, var_ref):
        self._resident = None  # a new structure: new resident inputs
        self.var_ref = var_ref
        self.system = self.system_type()
        self.system.initialize(model=self.model, var_ref=var_ref)
        opts = self.config.discretization_options
        discretization = self.discretization_types[opts.method](options=opts)
        nlp = discretization.transcribe(self.system)
        self.problem = CompiledProblem(nlp, self.system,
                                       only_positive_times=self.only_positive_times_in_results)
        self.reset_warm_start()

    def reset_warm_start(self):
        """Forget the remembered optima: the next solve starts cold (a new backend's first
        solve, `core/discretization.py:212-245`)."""
        self._remembered = None
        self._slot_ids = None
        if getattr(self, "_resident", None) is not None:
            self._resident.restart_cold()  # keep the device buffers, forget the optima

    def _native(self):
        """The structure's native handle with this backend's solver options (uploaded to the
        handle only when they differ from what it holds: a handle may serve several backends
        of one structure, and re-setting every option costs ~30 us of ctypes calls)."""
        prob = self.problem.native
        key = tuple(sorted(self.solver_options.items()))
        if getattr(prob, "options_key", None) != key:
            prob.set_options(**dict(self.solver_options))
            prob.options_key = key
        return prob

    # -- solve (`core/casadi_backend.py:133-139`) --------------------------------
    def solve(self, now: float, current_vars: dict) -> Results:
        return self.solve_batch(now, [current_vars])[0]

    def solve_batch(self, now, batch_vars: Sequence[dict], agent_ids: Optional[Sequence] = None):
        """Solve one NLP per entry of ``batch_vars`` (same structure) in one launch.

        Entry ``i`` is one agent: its warm start is ITS previous optimum (the reference
        keeps one remembered solution per backend instance, `core/discretization.py:
        221-223`, `247-251`).  ``agent_ids`` (one hashable key per entry, unique) names the
        agents: each one is warm-started from the optimum of the entry with the same key at
        the previous call, wherever it sat in that batch and whatever that batch's size was;
        a key not seen at the previous call starts cold.  Without keys the optima are kept
        per batch slot while the batch size is unchanged (entry i <- entry i).
        Marshalling is vectorised over the agents (:class:`BatchMarshal`); the returned
        :class:`FleetResults` builds each agent's ``Results`` on access."""
        if self.problem is None:
            raise RuntimeError("setup_optimization() must be called before solve()")
        prob = self.problem
        n = len(batch_vars)
        src = None  # per entry: the previous call's slot of its agent (-1: cold), or None (by slot)
        if agent_ids is not None:
            ids = list(agent_ids)
            if len(ids) != n or len(set(ids)) != n:
                raise ValueError("agent_ids: one unique key per batch entry")
            old = {k: i for i, k in enumerate(self._slot_ids or [])}
            src = np.array([old.get(k, -1) for k in ids], np.int64)
            self._slot_ids = ids
        else:
            self._slot_ids = None
        if prob.nlp.lift is None:
            res = self._solve_resident(now, batch_vars, src)
            if self.config.save_results:
                for i in range(n):
                    self.save_result_df(res[i], now)
            return res
        if src is not None:
            w_prev = None
            if self._remembered is not None:
                w_prev = np.full((n, self._remembered.shape[1]), np.nan)
                hit = src >= 0
                w_prev[hit] = self._remembered[src[hit]]
        else:
            w_prev = self._remembered if self._remembered is not None and self._remembered.shape[0] == n else None
        p, lbw, ubw, w0, sampled = prob.marshal.inputs(batch_vars, now, w_prev, return_sampled_bounds=True)
        res = self.solve_arrays(p, lbw, ubw, w0, result_bounds=sampled)
        self._remembered = res.w.copy()
        if self.config.save_results:
            for i in range(n):
                self.save_result_df(res[i], now)
        return res

    def _solve_resident(self, now, batch_vars, src=None):
        """Plugin batch on device-resident inputs (:mod:`.plugin_batch`): only the inputs
        that changed since the last call cross PCIe, the warm start stays in HBM.  ``src``:
        the previous slot of each entry's agent (-1 cold), None to keep the optima by slot."""
        import torch

        from agentlib_mpc_amd.optimization_backends.plugin_batch import ResidentBatch
        from agentlib_mpc_amd.optimization_backends.problem import FleetResults
        from agentlib_mpc_amd.runtime.native import StatsView, stats_array

        prob = self.problem
        t0 = time.perf_counter()
        rb = self._resident
        if rb is None or rb.n != len(batch_vars):
            self._remembered = None
            old = rb
            rb = self._resident = ResidentBatch(prob, self._native(), batch_vars, now, torch.device("cuda"))
            if old is not None and src is not None:
                rb.adopt_warm_starts(old, src)  # known agents keep their optima across sizes
            snap = rb.last
        else:
            self._native()  # options of this backend (set_options is per handle)
            if src is not None:
                rb.permute_warm_starts(src)
            snap = rb.update(batch_vars, now)
        w, raw = rb.solve()
        stats = StatsView(stats_array(raw), {"t_wall_total": time.perf_counter() - t0})
        return FleetResults(prob, prob.marshal, None, None, None, w, stats, rows=rb.row_source(snap))

    def solve_arrays(self, p, lbw, ubw, w0, lbg=None, ubg=None, result_bounds=None):
        """Batched solve of reference-layout NLP inputs [n, .] (host arrays): device
        copies, one kernel launch, solutions and stats back.  Returns :class:`FleetResults`
        (``result_bounds``: the bounds its lower/upper columns show, default lbw/ubw)."""
        import torch

        from agentlib_mpc_amd.runtime.native import STATS_BYTES, StatsView, stats_array

        prob = self.problem
        native = self._native()
        dev = torch.device("cuda")
        t0 = time.perf_counter()
        n = p.shape[0]
        kp, kl, ku, kw = prob.to_kernel(p, lbw, ubw, w0)
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev, non_blocking=True)  # noqa
        tp, tl, tu, tw = T(kp), T(kl), T(ku), T(kw)
        tg = tug = None
        if lbg is not None:
            tg, tug = T(lbg), T(ubg)
        lam_g = torch.empty((n, prob.nlp.kernel_ng), dtype=torch.float64, device=dev)
        st = torch.zeros(n * STATS_BYTES, dtype=torch.uint8, device=dev)
        native.solve(tp, tl, tu, tw, lbg=tg, ubg=tug, lam_g=lam_g, stats=st)
        w = prob.from_kernel(tw.cpu().numpy(), lbw)
        raw = st.cpu().numpy()
        wall = time.perf_counter() - t0
        stats = StatsView(stats_array(raw), {"t_wall_total": wall})
        from agentlib_mpc_amd.optimization_backends.problem import FleetResults

        rlb, rub = result_bounds if result_bounds is not None else (lbw, ubw)
        return FleetResults(prob, prob.marshal, p, rlb, rub, w, stats)

    # -- results file (`core/casadi_backend.py:263-323`) ---------------------------
    def save_result_df(self, results: Results, now: float = 0):
        """Results rows plus the combined stats line (``obj_<term>`` values of the
        objective on the multiple-shooting grid, then ``stats_<key>`` solver stats), as
        ``CasADiBackend.save_result_df`` writes them."""
        if not self.config.save_results:
            return
        res_file = self.config.results_file
        df = results.df
        objective_names, objective_values = self.approximate_objective(df)
        if not self.results_folder_exists():
            if not self.config.save_only_stats:
                results.write_columns(res_file)
            results.write_combined_stats_columns(stats_path(res_file), objective_names)
        with open(stats_path(res_file), "a") as f:
            f.write(results.combined_stats_line(str(now), objective_values, objective_names))
        if self.config.save_only_stats:
            return
        df.index = [str((now, x)) for x in df.index]
        df.to_csv(res_file, mode="a", header=False)

    def approximate_objective(self, results_df):
        """`core/casadi_backend.py:309-323`: objective terms on the multiple-shooting grid."""
        opts = self.config.discretization_options
        grid = np.arange(0, opts.prediction_horizon * (opts.time_step + 1), opts.time_step)
        objective = self.system.objective
        values = objective.calculate_values(results_df, grid)
        names = [o.name for o in objective.objectives] + ["total"]
        return names, values


class MI355XBaseBackend(MI355XBackend):
    """Backend ``"casadi_basic"`` replacement."""

    system_type = BaseSystem
    discretization_types = {
        DiscretizationMethod.collocation: disc.BasicCollocation,
        DiscretizationMethod.multiple_shooting: disc.BasicMultipleShooting,
    }


class MI355XADMMBackend(MI355XBackend, ADMMBackend):
    """Backend ``"casadi_admm"`` replacement (consensus and exchange terms)."""

    system_type = ADMMSystem
    discretization_types = {
        DiscretizationMethod.collocation: disc.ADMMCollocation,
        DiscretizationMethod.multiple_shooting: disc.ADMMMultipleShooting,
    }

    @property
    def coupling_grid(self) -> list:
        """`casadi_/admm.py:360-362`: grid of the multipliers parameter group."""
        return list(self.problem.nlp.par_groups[self.system.multipliers.name].grid)

    def save_result_df(self, results: Results, now: float = 0):
        """`casadi_/admm.py:364-424`: results of every ADMM iteration, indexed
        ``(now, iteration, t)``, buffered and flushed at the start of a new time
        step or every 1000 iterations."""
        if not self.config.save_results:
            return
        res_file = self.config.results_file
        if not hasattr(self, "_admm_buffer"):
            self._admm_buffer, self._admm_stats, self.it, self.now = [], [], 0, now
        if self.results_folder_exists():
            self.it += 1
            if now != self.now:
                self.it = 0
                self.now = now
        else:
            self.it = 0
            self.now = now
            results.write_columns(res_file)
            results.write_stats_columns(stats_path(res_file))
        df = results.df
        df.index = [str((now, self.it, x)) for x in df.index]
        self._admm_buffer.append(df)
        self._admm_stats.append(results.stats_line(str((now, self.it))))
        if not (self.it == 0 or self.it % 1000 == 0):
            return
        with open(res_file, "a", newline="") as f:
            for it_result in self._admm_buffer:
                it_result.to_csv(f, mode="a", header=False)
        with open(stats_path(res_file), "a") as f:
            f.writelines(self._admm_stats)
        self._admm_buffer, self._admm_stats = [], []


class MI355XMLBackend(MI355XBackend):
    """Backend ``"casadi_ml"`` / ``"casadi_nn"`` replacement (``CasADiBBBackend``,
    `casadi_/casadi_ml.py:347-397`): NARX models, multiple shooting, solved by the
    kernel on the lifted stage NLP (:mod:`.narx`)."""

    system_type = narx.MLSystem
    discretization_types = {DiscretizationMethod.multiple_shooting: narx.NarxMultipleShooting}

    def setup_optimization(self, var_ref):
        method = self.config.discretization_options.method
        if method not in self.discretization_types:
            raise ValueError(f"discretization method {method!r} is not available for ML models "
                             "(the reference supports multiple_shooting only)")
        super().setup_optimization(var_ref)

    def get_lags_per_variable(self) -> Dict[str, float]:
        """`casadi_ml.py:387-397`: history length the MPC module has to keep per variable."""
        ts = self.config.discretization_options.time_step
        names = set(self.var_ref.all_variables()) if self.var_ref is not None else set()
        return {name: (lag - 1) * ts for name, lag in self.system.lags_dict.items() if name in names}


class MI355XADMMNNBackend(MI355XMLBackend, ADMMBackend):
    """Backend ``"casadi_admm_ml"`` / ``"casadi_admm_nn"`` replacement
    (``CasADiADMMBackend_NN``, `casadi_/casadi_admm_ml.py:508-518`)."""

    system_type = narx.ADMMNNSystem
    discretization_types = {DiscretizationMethod.multiple_shooting: narx.NarxADMMMultipleShooting}

    @property
    def coupling_grid(self) -> list:
        return list(self.problem.nlp.par_groups[self.system.multipliers.name].grid)


# the NN-ADMM backend saves like the ADMM backend (`casadi_admm_ml.py:508` inherits it)
MI355XADMMNNBackend.save_result_df = MI355XADMMBackend.save_result_df
