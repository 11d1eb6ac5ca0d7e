"""A transcribed problem: layout maps, host marshalling and the native solver.

Host-side marshalling restates the reference input path:
``CasADiBackend._get_current_mpc_inputs`` (`core/casadi_backend.py:141-253`),
``Discretization._determine_initial_guess`` (`core/discretization.py:212-245`),
the NLP input map ``_mpc_inputs_to_nlp_inputs`` (:277-348), the output map
(:350-358), warm start ``_remember_solution`` (:247-251) and the result
matrix ``_result_map`` / ``_create_result_format`` (:360-484).

Everything here is O(#variables x grid) numpy bookkeeping; the solve itself
is the native batched kernel (:class:`agentlib_mpc_amd.runtime.native.NativeProblem`).
"""

from __future__ import annotations

import math
import operator
from collections.abc import Sequence
from typing import Dict, List, Optional, Tuple

import numpy as np
import pandas as pd

from agentlib_mpc_amd.optimization_backends.discretization import StageNLP
from agentlib_mpc_amd.optimization_backends.results import ResultLayout, Results
from agentlib_mpc_amd.optimization_backends.system import (
    OptimizationParameter, OptimizationVariable, System,
)
from agentlib_mpc_amd.runtime import codegen
from agentlib_mpc_amd.utils import sampling

GUESS_PREFIX = "guess_"


class CompiledProblem:
    def __init__(self, nlp: StageNLP, system: System, only_positive_times: bool = True):
        self.nlp = nlp
        self.only_positive_times = only_positive_times
        self.system = system
        self.gen = codegen.generate(nlp)
        self._native = None
        self.layout = self._result_layout()
        self._marshal = None
        self.system_group_names = {v.name: list(v.full_names) for v in system.variables}

    @property
    def marshal(self) -> "BatchMarshal":
        if self._marshal is None:
            self._marshal = BatchMarshal(self)
        return self._marshal

    # -- native ------------------------------------------------------------------
    @property
    def native(self):
        if self._native is None:
            from agentlib_mpc_amd.runtime.native import NativeProblem

            self._native = NativeProblem(self.gen)
        return self._native

    def compile(self, small_fleet: bool = True):
        """Compile the structure's code object and, when its workspace fits a CU's LDS, the
        small-fleet build (``native.SMALL_FLEET``); returns the main code object's path."""
        from agentlib_mpc_amd.runtime.native import SMALL_FLEET, compile_model

        if small_fleet:
            compile_model(self.gen, variant=SMALL_FLEET)
        return compile_model(self.gen)

    # -- inputs ------------------------------------------------------------------
    def mpc_inputs(self, current_vars: dict, now: float) -> Dict[str, np.ndarray]:
        """Sample runtime values/bounds onto the group grids (`casadi_backend.py:141-253`)."""
        out: Dict[str, np.ndarray] = {}
        for par in self.system.parameters:
            grid = self.nlp.par_groups[par.name].grid if par.name in self.nlp.par_groups else []
            mat = np.empty((par.dim, len(grid)))
            for i, name in enumerate(par.full_names):
                if name in par.ref_names:
                    var = current_vars[name]
                    if var.value is None:
                        raise ValueError(f"Input for variable {name} is empty. Cannot solve optimization problem.")
                    try:
                        method = var.interpolation_method
                    except AttributeError as e:
                        raise TypeError(
                            f"The variable {name} does not have an interpolationmethod. All Variables "
                            "used in MPC need to be of type MPCVariable (subclass of AgentVariable).") from e
                    mat[i, :] = sampling.sample(trajectory=var.value, grid=grid, current=now, method=method)
                else:
                    mat[i, :] = par.defaults[i]
            out[par.name] = mat
        for var in self.system.variables:
            grid = self.nlp.var_groups[var.name].grid if var.name in self.nlp.var_groups else []
            lb = np.empty((var.dim, len(grid)))
            ub = np.empty((var.dim, len(grid)))
            for i, name in enumerate(var.full_names):
                if name in var.ref_names:
                    av = current_vars[name]
                    method = getattr(av, "interpolation_method", "linear")
                    ub[i, :] = sampling.sample(trajectory=av.ub, grid=grid, current=now, method=method)
                    lb[i, :] = sampling.sample(trajectory=av.lb, grid=grid, current=now, method=method)
                else:
                    lb[i, :] = var.default_lb[i]
                    ub[i, :] = var.default_ub[i]
            out[f"lb_{var.name}"] = lb
            out[f"ub_{var.name}"] = ub
        return out

    def initial_guess(self, mpc_inputs: Dict[str, np.ndarray],
                      remembered: Optional[Dict[str, np.ndarray]] = None) -> Dict[str, np.ndarray]:
        """`core/discretization.py:212-245` (no time shift of the previous optimum)."""
        guesses = {}
        for name, lay in self.nlp.var_groups.items():
            g = None if remembered is None else remembered.get(name)
            if g is None:
                key = f"initial_{name}"
                if key in mpc_inputs:
                    meas = mpc_inputs[key]
                    meas = meas[:, -1:] if meas.shape[1] > 1 else meas
                    g = np.tile(meas, len(lay.grid))
                else:
                    with np.errstate(invalid="ignore"):
                        g = 0.5 * (mpc_inputs[f"lb_{name}"] + mpc_inputs[f"ub_{name}"])
                    g = np.nan_to_num(g, posinf=0, neginf=-0)
            guesses[GUESS_PREFIX + name] = np.asarray(g, dtype=float)
        return guesses

    def nlp_inputs(self, mpc_inputs: Dict[str, np.ndarray]) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        """Permutation of the MPC input matrices into (p, lbw, ubw, w0)."""
        nlp = self.nlp
        p = np.full(nlp.npar, np.nan)
        for name, lay in nlp.par_groups.items():
            if lay.dim:
                p[lay.index] = mpc_inputs[name]
        lbw = np.full(nlp.nw, np.nan)
        ubw = np.full(nlp.nw, np.nan)
        w0 = np.full(nlp.nw, np.nan)
        for name, lay in nlp.var_groups.items():
            if not lay.dim:
                continue
            idx = lay.index
            lbw[idx] = mpc_inputs[f"lb_{name}"]
            ubw[idx] = mpc_inputs[f"ub_{name}"]
            w0[idx] = mpc_inputs[GUESS_PREFIX + name]
            for t, cols in enumerate(lay.columns):
                for i, c in enumerate(cols):
                    if lay.lb_par[t][i] >= 0:
                        lbw[c] = p[lay.lb_par[t][i]]
                    if lay.ub_par[t][i] >= 0:
                        ubw[c] = p[lay.ub_par[t][i]]
                    if lay.guess_par[t][i] >= 0:
                        w0[c] = p[lay.guess_par[t][i]]
        if np.isnan(p).any() or np.isnan(lbw).any() or np.isnan(ubw).any():
            raise ValueError("incomplete NLP inputs (NaN in parameters or bounds)")
        return p, lbw, ubw, np.nan_to_num(w0)

    # -- reference layout <-> kernel layout (identity unless the NLP is lifted) ----
    def to_kernel(self, p, lbw, ubw, w0):
        """Map reference-layout NLP inputs ([n, .] or [.]) to the kernel's stage NLP.

        Lag-window copies of a lifted (NARX) NLP are unbounded and start at the
        guess of the variable they copy (see :mod:`.narx`)."""
        lift = self.nlp.lift
        if lift is None:
            return p, lbw, ubw, w0
        kp = np.array(p[..., lift.p_src], order="C")
        klb = np.array(lbw[..., lift.w_src], order="C")
        kub = np.array(ubw[..., lift.w_src], order="C")
        klb[..., lift.w_dup] = -np.inf
        kub[..., lift.w_dup] = np.inf
        kw = np.array(w0[..., lift.w_src], order="C")
        if lift.w_fix_par is not None:  # kernel-only variables fixed to a parameter
            fx = np.flatnonzero(lift.w_fix_par >= 0)
            val = p[..., lift.w_fix_par[fx]]
            klb[..., fx] = val
            kub[..., fx] = val
            kw[..., fx] = val
        if lift.w_zero is not None:  # kernel-only dummies (MHE: the fixed X_0)
            klb[..., lift.w_zero] = 0.0
            kub[..., lift.w_zero] = 0.0
            kw[..., lift.w_zero] = 0.0
        return kp, klb, kub, kw

    def from_kernel(self, w_k: np.ndarray, lbw: np.ndarray) -> np.ndarray:
        """Reference-layout solution from the kernel solution; reference variables
        the lifted NLP does not use are fixed past values (= their bound)."""
        lift = self.nlp.lift
        if lift is None:
            return w_k
        w = np.array(lbw, dtype=float, copy=True)
        used = lift.w_primary >= 0
        w[..., used] = w_k[..., lift.w_primary[used]]
        return w

    def lam_g_from_kernel(self, lam_k: np.ndarray) -> np.ndarray:
        lift = self.nlp.lift
        return lam_k if lift is None else lam_k[..., lift.g_of_ref]

    def outputs(self, w: np.ndarray) -> Dict[str, np.ndarray]:
        """``_nlp_outputs_to_mpc_outputs``: group matrices of the optimum."""
        return {name: np.asarray(w)[lay.index] for name, lay in self.nlp.var_groups.items()}

    # -- results -------------------------------------------------------------------
    def _result_layout(self) -> ResultLayout:
        nlp = self.nlp
        full = set()
        for lay in list(nlp.var_groups.values()) + list(nlp.par_groups.values()):
            full.update(lay.grid)
        full_grid = sorted(full)
        pos = {t: i for i, t in enumerate(full_grid)}
        columns, blocks, var_rows = [], [], {}
        for par in self.system.parameters:
            if not par.full_names or par.name not in nlp.par_groups:
                continue
            lay = nlp.par_groups[par.name]
            columns += [("parameter", n) for n in par.full_names]
            blocks.append(("parameter", par.name, par.dim, self._rows_cols(lay.grid, full_grid, pos)))
        for var in self.system.variables:
            if not var.full_names or var.name not in nlp.var_groups:
                continue
            lay = nlp.var_groups[var.name]
            rc = self._rows_cols(lay.grid, full_grid, pos)
            for key, header in (("var", "variable"), ("ub", "upper"), ("lb", "lower")):
                columns += [(header, n) for n in var.full_names]
                blocks.append((key, var.name, var.dim, rc))
            rows = [r for r, _ in rc if full_grid[r] >= 0 or not self.only_positive_times]
            for n in var.full_names:
                var_rows[n] = rows
        return ResultLayout(full_grid=full_grid, columns=pd.MultiIndex.from_tuples(columns),
                            variable_grid_indices=var_rows, blocks=blocks)

    @staticmethod
    def _rows_cols(grid, full_grid, pos):
        """(row in full grid, first column of the group grid at that time)."""
        first = {}
        for j, t in enumerate(grid):
            first.setdefault(t, j)
        return [(pos[t], j) for t, j in sorted(first.items(), key=lambda kv: pos[kv[0]])]

    def result_matrix(self, mpc_inputs: Dict[str, np.ndarray], w: np.ndarray) -> np.ndarray:
        lay = self.layout
        outs = self.outputs(w)
        ncol = len(lay.columns)
        mat = np.full((len(lay.full_grid), ncol), np.nan)
        col = 0
        for kind, name, dim, rc in lay.blocks:
            if kind == "parameter":
                src = mpc_inputs[name]
            elif kind == "var":
                src = outs[name]
            else:
                src = mpc_inputs[f"{kind}_{name}"]
            for r, j in rc:
                mat[r, col:col + dim] = src[:, j]
            col += dim
        return mat

    def make_results(self, mpc_inputs, w, stats) -> Results:
        lay = self.layout
        return Results(matrix=self.result_matrix(mpc_inputs, w), grid=list(lay.full_grid),
                       columns=lay.columns, stats=stats, variable_grid_indices=lay.variable_grid_indices)


def fleet_nlp_inputs(prob: CompiledProblem, template_vars: dict, overrides: Dict[str, np.ndarray],
                     now: float = 0.0):
    """NLP inputs of a fleet of agents sharing one structure.

    ``overrides`` maps a scalar MPC variable name to per-agent values (shape
    [n_agents]) for its ``value`` (parameters/states/controls) — vectorised
    equivalent of building ``current_vars`` per agent and calling
    ``mpc_inputs`` + ``initial_guess`` + ``nlp_inputs`` (cold start).
    Returns (p, lbw, ubw, w0) as [n_agents, .] float64 arrays.
    """
    n = len(next(iter(overrides.values())))
    mi = prob.mpc_inputs(template_vars, now)
    m = prob.marshal
    pars = {}
    for par in prob.system.parameters:
        mat = np.broadcast_to(mi[par.name][None], (n,) + mi[par.name].shape)
        hit = [(i, name) for i, name in enumerate(par.full_names) if name in overrides and name in par.ref_names]
        if hit:
            mat = mat.copy()
            for i, name in hit:
                mat[:, i, :] = np.asarray(overrides[name], float)[:, None]
        pars[par.name] = mat
    lbs = {v.name: np.broadcast_to(mi[f"lb_{v.name}"][None], (n,) + mi[f"lb_{v.name}"].shape)
           for v in prob.system.variables}
    ubs = {v.name: np.broadcast_to(mi[f"ub_{v.name}"][None], (n,) + mi[f"ub_{v.name}"].shape)
           for v in prob.system.variables}
    return m.assemble(n, pars, lbs, ubs)


# ---------------------------------------------------------------------------
# batched marshalling (structure of arrays over the agents of one structure)
# ---------------------------------------------------------------------------
_FAST_TYPES = (float, int, np.float64, np.int64, list)
_VLU = operator.attrgetter("value", "lb", "ub")


def _first_of_each_type(objs):
    seen = {}
    for o in objs:
        seen.setdefault(type(o), o)
    return seen.values()

class BatchMarshal:
    """Array maps of one problem structure, built once: ``mpc_inputs`` +
    ``initial_guess`` + ``nlp_inputs`` for many agents at once (reference semantics,
    `core/casadi_backend.py:141-253`, `core/discretization.py:212-348`), and the result
    matrices (`core/discretization.py:360-484`) straight from the NLP vectors.

    Values are gathered per variable across the agents; scalar values and grid-length
    lists (the common case) are written as whole columns, anything else (series, dicts,
    JSON strings) is sampled per agent exactly as :meth:`CompiledProblem.mpc_inputs`
    does."""

    def __init__(self, prob: "CompiledProblem"):
        self.prob = prob
        nlp = prob.nlp
        self.pars = []   # (group name, grid length, [(row, name | None, default)], p index [dim, G])
        for par in prob.system.parameters:
            lay = nlp.par_groups.get(par.name)
            grid = lay.grid if lay is not None else []
            rows = [(i, n if n in par.ref_names else None, par.defaults[i]) for i, n in enumerate(par.full_names)]
            self.pars.append((par.name, list(grid), rows, None if lay is None or not lay.dim else lay.index))
        self.vars = []   # (group name, grid, [(row, name | None, default lb, default ub)], w index)
        for var in prob.system.variables:
            lay = nlp.var_groups.get(var.name)
            grid = lay.grid if lay is not None else []
            rows = [(i, n if n in var.ref_names else None, var.default_lb[i], var.default_ub[i])
                    for i, n in enumerate(var.full_names)]
            self.vars.append((var.name, list(grid), rows, None if lay is None or not lay.dim else lay.index))
        # bound / guess entries taken from parameters (`lb_par`, `ub_par`, `guess_par`)
        over = {"lb": ([], []), "ub": ([], []), "guess": ([], [])}
        for lay in nlp.var_groups.values():
            for t, cols in enumerate(lay.columns):
                for i, c in enumerate(cols):
                    for key, src in (("lb", lay.lb_par), ("ub", lay.ub_par), ("guess", lay.guess_par)):
                        if src[t][i] >= 0:
                            over[key][0].append(c)
                            over[key][1].append(src[t][i])
        self.over = {k: (np.asarray(c, np.int64), np.asarray(p, np.int64)) for k, (c, p) in over.items()}
        self.initial = {}
        for name, lay in nlp.var_groups.items():
            key = f"initial_{name}"
            if lay.dim and key in nlp.par_groups and nlp.par_groups[key].dim:
                self.initial[name] = nlp.par_groups[key].index
        self._work = {}
        # result matrix scatter plan
        lay = prob.layout
        self.n_rows, self.n_cols = len(lay.full_grid), len(lay.columns)
        self.blocks = []
        col = 0
        for kind, name, dim, rc in lay.blocks:
            rows = np.array([r for r, _ in rc], np.int64)
            cols = np.array([j for _, j in rc], np.int64)
            if kind == "parameter":
                src = ("p", nlp.par_groups[name].index)
            else:
                src = ({"var": "w", "lb": "lbw", "ub": "ubw"}[kind], nlp.var_groups[name].index)
            self.blocks.append((col, dim, rows, cols) + src)
            col += dim

    @staticmethod
    def _column(values, grid, now, method_of):
        """[n, G] samples of one variable for every agent (``sampling.sample`` semantics):
        numbers are constant rows and grid-length lists are taken as they are, both in
        one numpy conversion; anything else is sampled agent by agent."""
        n, G = len(values), len(grid)
        if all(type(v) in _FAST_TYPES for v in values):
            try:
                arr = np.array(values, dtype=float)
            except (TypeError, ValueError):
                arr = None
            if arr is not None and arr.ndim == 1:
                return np.repeat(arr[:, None], G, axis=1)
            if arr is not None and arr.ndim == 2 and arr.shape[1] == G and all(type(v) is list for v in values):
                return arr
        out = np.empty((n, G))
        for a, v in enumerate(values):
            out[a] = sampling.sample(trajectory=v, grid=grid, current=now, method=method_of(a))
        return out

    def inputs(self, batch_vars: Sequence[dict], now: float, w_prev: Optional[np.ndarray] = None,
               return_sampled_bounds: bool = False):
        """(p, lbw, ubw, w0) [n, .] in the reference layout; ``w_prev`` [n, nw] (rows of
        NaN = no previous optimum) is the warm start (`core/discretization.py:212-251`).
        ``return_sampled_bounds``: also the sampled bounds before the parameter overrides
        (what the result matrix's lower/upper columns show)."""
        n = len(batch_vars)
        cache = {}

        def gather(ref):
            """(variables, values, lbs, ubs) of one name over the agents, two passes."""
            if ref not in cache:
                vs = list(map(operator.itemgetter(ref), batch_vars))
                try:
                    vals, lbs, ubs = zip(*map(_VLU, vs))
                except AttributeError:
                    vals, lbs, ubs = [getattr(v, "value", None) for v in vs], None, None
                cache[ref] = (vs, vals, lbs, ubs)
            return cache[ref]

        pars = {}
        for name, grid, rows, index in self.pars:
            mat = np.empty((n, len(rows), len(grid)))
            for i, ref, default in rows:
                if ref is None:
                    mat[:, i, :] = default
                    continue
                vs, vals, _, _ = gather(ref)
                if any(v is None for v in vals):
                    raise ValueError(f"Input for variable {ref} is empty. Cannot solve optimization problem.")
                if not all(hasattr(v, "interpolation_method") for v in _first_of_each_type(vs)):
                    raise TypeError(
                        f"The variable {ref} does not have an interpolationmethod. All Variables "
                        "used in MPC need to be of type MPCVariable (subclass of AgentVariable).")
                mat[:, i, :] = self._column(vals, grid, now, lambda a: vs[a].interpolation_method)
            pars[name] = mat
        lbs, ubs = {}, {}
        for name, grid, rows, index in self.vars:
            lb = np.empty((n, len(rows), len(grid)))
            ub = np.empty((n, len(rows), len(grid)))
            for i, ref, dlb, dub in rows:
                if ref is None:
                    lb[:, i, :], ub[:, i, :] = dlb, dub
                    continue
                vs, _, lbv, ubv = gather(ref)
                meth = lambda a: getattr(vs[a], "interpolation_method", "linear")  # noqa: E731
                ub[:, i, :] = self._column(ubv, grid, now, meth)
                lb[:, i, :] = self._column(lbv, grid, now, meth)
            lbs[name], ubs[name] = lb, ub
        return self.assemble(n, pars, lbs, ubs, w_prev, return_sampled_bounds)

    def assemble(self, n, pars, lbs, ubs, w_prev=None, return_sampled_bounds=False):
        """NLP input arrays from the group matrices ([n, dim, len(grid)] per group), built
        in transposed form (every group row is a contiguous copy of n values)."""
        nlp = self.prob.nlp
        work = self._work.get(n)
        if work is None:  # transposed work buffers, reused (no page faults per call)
            work = self._work[n] = tuple(np.empty((m, n)) for m in (nlp.npar, nlp.nw, nlp.nw, nlp.nw))
        pT, lT, uT, gT = work
        pT.fill(np.nan)
        lT.fill(np.nan)
        uT.fill(np.nan)
        gT.fill(0.0)
        for name, grid, rows, index in self.pars:
            if index is not None:
                pT[index.ravel()] = pars[name].reshape(n, -1).T
        for name, grid, rows, index in self.vars:
            if index is None:
                continue
            flat = index.ravel()
            lb, ub = lbs[name], ubs[name]
            lT[flat] = lb.reshape(n, -1).T
            uT[flat] = ub.reshape(n, -1).T
            if name in self.initial:
                ii = self.initial[name]                          # [dim, G_init] in p
                meas = pT[ii[:, -1]]                             # [dim, n]
                gT[flat] = np.repeat(meas[:, None, :], len(grid), axis=1).reshape(-1, n)
            else:
                with np.errstate(invalid="ignore"):
                    mid = np.nan_to_num(0.5 * (lb + ub), posinf=0, neginf=-0)
                gT[flat] = mid.reshape(n, -1).T
        if w_prev is not None:
            have = ~np.isnan(w_prev).any(axis=1)
            gT[:, have] = w_prev[have].T
        sampled = (np.ascontiguousarray(lT.T), np.ascontiguousarray(uT.T)) if return_sampled_bounds else None
        for key, arr in (("lb", lT), ("ub", uT), ("guess", gT)):
            cols, prs = self.over[key]
            if cols.size:
                arr[cols] = pT[prs]
        if np.isnan(pT).any() or np.isnan(lT).any() or np.isnan(uT).any():
            raise ValueError("incomplete NLP inputs (NaN in parameters or bounds)")
        p, lbw, ubw = (np.ascontiguousarray(a.T) for a in (pT, lT, uT))
        w0 = np.ascontiguousarray(np.nan_to_num(gT).T)
        if return_sampled_bounds:
            return p, lbw, ubw, w0, sampled
        return p, lbw, ubw, w0

    def result_matrices(self, p, lbw, ubw, w) -> np.ndarray:
        """[n, len(full grid), n_columns] result matrices from the NLP vectors (``lbw`` /
        ``ubw``: the sampled bounds, see :meth:`inputs`).  One gather from [p | w | lbw | ubw]
        (the cell -> vector-entry map is built once; empty cells read a NaN entry)."""
        n = p.shape[0]
        if getattr(self, "_gather", None) is None or self._gather[0] != (p.shape[1], w.shape[1]):
            npar, nw = p.shape[1], w.shape[1]
            base = {"p": 0, "w": npar, "lbw": npar + nw, "ubw": npar + 2 * nw}
            nan_at = npar + 3 * nw
            idx = np.full((self.n_rows, self.n_cols), nan_at, np.int64)
            for col, dim, rows, cols, key, index in self.blocks:
                idx[rows, col:col + dim] = (base[key] + np.asarray(index)[:, cols]).T
            self._gather = ((npar, nw), idx.ravel())
        src = np.concatenate([p, w, lbw, ubw, np.full((n, 1), np.nan)], axis=1)
        return src[:, self._gather[1]].reshape(n, self.n_rows, self.n_cols)


class FleetResults(Sequence):
    """Results of one batched solve: per-agent :class:`Results` built on access; whole-fleet
    arrays (solutions, stats) without per-agent objects.  The inputs are either the
    reference-layout arrays (``p``, sampled ``lbw`` / ``ubw``) or ``rows``, a source of
    single-agent rows (:class:`~.plugin_batch.RowSource`, the resident plugin path)."""

    def __init__(self, prob: "CompiledProblem", marshal: BatchMarshal, p, lbw, ubw, w, stats: list, rows=None):
        self.prob, self.marshal = prob, marshal
        self._p, self._lbw, self._ubw, self.w, self.stats = p, lbw, ubw, w, stats
        self._rows = rows

    def _all_rows(self):
        if self._p is None:
            rows = [self._rows.rows(i) for i in range(len(self))]
            self._p, self._lbw, self._ubw = (np.stack(a) for a in zip(*rows))

    @property
    def p(self):
        self._all_rows()
        return self._p

    @property
    def lbw(self):
        self._all_rows()
        return self._lbw

    @property
    def ubw(self):
        self._all_rows()
        return self._ubw

    def __len__(self):
        return self.w.shape[0]

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        if self._p is None:
            p, lb, ub = (a[None] for a in self._rows.rows(i))
        else:
            p, lb, ub = self._p[i:i + 1], self._lbw[i:i + 1], self._ubw[i:i + 1]
        m = self.marshal.result_matrices(p, lb, ub, self.w[i:i + 1])[0]
        lay = self.prob.layout
        return Results(matrix=m, grid=list(lay.full_grid), columns=lay.columns, stats=self.stats[i],
                       variable_grid_indices=lay.variable_grid_indices)

    def first_values(self, name: str) -> np.ndarray:
        """Value of variable ``name`` at the first grid time >= 0, every agent (the
        actuation `modules/mpc/mpc.py:342-357` reads)."""
        for gname, lay in self.prob.nlp.var_groups.items():
            full = self.prob.system_group_names.get(gname, [])
            if name in full:
                comp = full.index(name)
                j = next(j for j, t in enumerate(lay.grid) if t >= 0)
                return self.w[:, lay.index[comp, j]]
        raise KeyError(name)
