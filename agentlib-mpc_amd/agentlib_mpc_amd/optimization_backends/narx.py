"""NARX (data-driven model) transcription: backends ``casadi_ml`` / ``casadi_admm_ml``.

Reference: ``CasadiMLSystem`` + ``MultipleShooting_ML``
(`optimization_backends/casadi_/casadi_ml.py:30-344`) and
``CasadiADMMNNSystem`` + ``MultipleShootingADMMNN``
(`casadi_/casadi_admm_ml.py:35-505`).  The reference loops are followed
step for step, so the NLP vectors ``w``, ``p`` and ``g`` keep exactly the
reference layout:

* past states ``x(t)`` for ``t = -(L-1)ts .. 0`` (fixed to ``initial_state``),
* past controls (and, for ADMM, past couplings/exchange) for
  ``t = -(max(2, L)-1)ts .. -ts`` (fixed to ``initial_control`` / ``past_*``),
* per prediction step ``u, z, y`` (ADMM: ``local_exchange, local_couplings``),
* the states ``x(ts) .. x(N ts)``;
* ``g`` per step: model constraints, then ``next_states - x(t+ts)``.

``L`` is the model's maximum lag.  The stage function evaluates the ML
models on current and lagged values (`casadi_ml.py:178-227`).

**Lifting to the kernel's stage form.**  With lags, step ``k`` reads
variables of steps ``k-1 .. k-L+1``, which breaks the ``[x_k, v_k, x_{k+1}]``
stage structure the batched interior-point kernel factorises.  The kernel
therefore solves an equivalent *lifted* NLP whose stage state is
``X_k = [x_k, lag window]`` — the lag window holds a copy of every lagged
variable value ``v(t_k - j ts)`` (``1 <= j < lag(v)``) — with shift
constraints ``X_{k+1}[v, j] = X_k[v, j-1]`` (``= v_k`` for ``j = 1``).  The
copies are free variables (no bounds); every reference variable keeps one
primary position, so the lifted NLP has the same optimum and the same
multipliers on the reference constraints.  :class:`LiftMaps` records the
index maps reference ↔ kernel; the host maps inputs and outputs, so callers
see the reference layout only.
"""

from __future__ import annotations

import dataclasses
from typing import Dict, List, Tuple

import numpy as np

from agentlib_mpc_amd import symbolic as sx
from agentlib_mpc_amd.data_structures import admm_datatypes as adt
from agentlib_mpc_amd.data_structures.ml_model_datatypes import name_with_lag
from agentlib_mpc_amd.data_structures.mpc_datamodels import VariableReference
from agentlib_mpc_amd.data_structures.objective import CombinedObjective, SubObjective
from agentlib_mpc_amd.models.casadi_ml_model import CasadiMLModel
from agentlib_mpc_amd.models.casadi_model import CasadiInput, CasadiParameter
from agentlib_mpc_amd.optimization_backends.discretization import (
    Discretization, StageFunction, StageNLP, TranscriptionError, _Transcriber,
)
from agentlib_mpc_amd.optimization_backends.system import (
    FullSystem, OptimizationParameter, OptimizationVariable, System,
)


# ---------------------------------------------------------------------------
# systems
# ---------------------------------------------------------------------------

class MLSystem(System):
    """`casadi_ml.py:30-103` (``CasadiMLSystem``)."""

    def initialize(self, model: CasadiMLModel, var_ref: VariableReference):
        if not isinstance(model, CasadiMLModel):
            raise TypeError("the ML backends need a CasadiMLModel")
        self.states = OptimizationVariable.declare("state", model.get_states(var_ref.states),
                                                   var_ref.states, assert_complete=True)
        self.controls = OptimizationVariable.declare("control", model.get_inputs(var_ref.controls),
                                                     var_ref.controls, assert_complete=True)
        self.algebraics = OptimizationVariable.declare("z", model.auxiliaries, [])
        self.outputs = OptimizationVariable.declare("y", model.outputs, var_ref.outputs)
        self.non_controlled_inputs = OptimizationParameter.declare(
            "d", model.get_inputs(var_ref.inputs), var_ref.inputs, assert_complete=True)
        self.model_parameters = OptimizationParameter.declare(
            "parameter", model.parameters, var_ref.parameters)
        self.initial_state = OptimizationParameter.declare(
            "initial_state", model.get_states(var_ref.states), var_ref.states,
            use_in_stage_function=False, assert_complete=True)
        self.last_control = OptimizationParameter.declare(
            "initial_control", model.get_inputs(var_ref.controls), var_ref.controls,
            use_in_stage_function=False, assert_complete=True)
        self.model_constraints = model.get_constraints()
        self.model = model
        self.next_states = model.predict_step()
        missing = [s for s in self.states.full_names if s not in self.next_states]
        if missing:
            raise ValueError(f"States {missing} are neither predicted by an ML model nor have an ode.")
        self.lags_dict: Dict[str, int] = model.lags_dict
        self.objective: CombinedObjective = model.objective
        self.time = model.time

    @property
    def max_lag(self) -> int:
        return max(self.lags_dict.values()) if self.lags_dict else 1

    def stage_quantities(self) -> List:
        """Quantities passed to the ML step function (`casadi_ml.py:253-259`)."""
        return [q for q in self.quantities if q.use_in_stage_function]


class ADMMNNSystem(MLSystem):
    """`casadi_admm_ml.py:35-244` (``CasadiADMMNNSystem``)."""

    _omit_in_blackbox = {"global_couplings", "multipliers", "average_diff", "exchange_multipliers", "rho"}

    def initialize(self, model: CasadiMLModel, var_ref: adt.VariableReference):
        super().initialize(model, var_ref)
        coup = [c.name for c in var_ref.couplings]
        exch = [c.name for c in var_ref.exchange]
        pure = [o for o in model.outputs if o.name not in coup + exch]
        self.outputs = OptimizationVariable.declare("y", pure, var_ref.outputs)
        self.local_couplings = OptimizationVariable.declare(
            "local_couplings", [model.get(n) for n in coup], coup)
        means = [c.mean for c in var_ref.couplings]
        self.global_couplings = OptimizationParameter.declare(
            "global_couplings", [CasadiInput(name=n) for n in means], means)
        mults = [c.multiplier for c in var_ref.couplings]
        self.multipliers = OptimizationParameter.declare(
            "multipliers", [CasadiInput(name=n) for n in mults], mults)
        self.local_exchange = OptimizationVariable.declare(
            "local_exchange", [model.get(n) for n in exch], exch)
        diffs = [c.mean_diff for c in var_ref.exchange]
        self.exchange_diff = OptimizationParameter.declare(
            "average_diff", [CasadiInput(name=n) for n in diffs], diffs)
        emults = [c.multiplier for c in var_ref.exchange]
        self.exchange_multipliers = OptimizationParameter.declare(
            "exchange_multipliers", [CasadiInput(name=n) for n in emults], emults)
        self.penalty_factor = OptimizationParameter.declare(
            "rho", [CasadiParameter(name="penalty_factor")], ["penalty_factor"])
        lagged = [c.lagged for c in var_ref.couplings]
        self.past_couplings = OptimizationParameter.declare(
            "past_couplings", [CasadiInput(name=n) for n in lagged], lagged, use_in_stage_function=False)
        # reference quirk (`casadi_admm_ml.py:166-172`): the past-exchange group is
        # declared over the exchange *names* with the lagged names as ref list, which
        # only validates when there is no exchange variable.
        lagged_ex = [c.lagged for c in var_ref.exchange]
        self.past_exchange = OptimizationParameter.declare(
            "past_exchange", [CasadiInput(name=n) for n in exch], lagged_ex, use_in_stage_function=False)
        rho = self.penalty_factor.full_symbolic[0]
        terms = []
        for i in range(len(var_ref.couplings)):
            terms.append(self.multipliers.full_symbolic[i] * self.local_couplings.full_symbolic[i])
            terms.append(rho / 2 * (self.global_couplings.full_symbolic[i] - self.local_couplings.full_symbolic[i]) ** 2)
        for i in range(len(var_ref.exchange)):
            terms.append(self.exchange_multipliers.full_symbolic[i] * self.local_exchange.full_symbolic[i])
            terms.append(rho / 2 * (self.exchange_diff.full_symbolic[i] - self.local_exchange.full_symbolic[i]) ** 2)
        self.objective = CombinedObjective(
            *self.objective.objectives,
            *[SubObjective(t, name="admm_augmentation_term") for t in terms],
            normalization=self.objective.normalization)

    def stage_quantities(self) -> List:
        """`casadi_admm_ml.py:228-244` (``sim_step_quantities``) for the lags."""
        return [q for q in self.quantities if q.use_in_stage_function and q.name not in self._omit_in_blackbox]


# ---------------------------------------------------------------------------
# lifted stage form
# ---------------------------------------------------------------------------

@dataclasses.dataclass
class LiftMaps:
    """Index maps between the reference NLP and the kernel's lifted stage NLP."""

    w_src: np.ndarray        # [nw_kernel] reference variable index of each kernel variable
    w_dup: np.ndarray        # [nw_kernel] True for lag-window copies (free, unbounded)
    p_src: np.ndarray        # [np_kernel] reference parameter index of each kernel parameter
    g_of_ref: np.ndarray     # [ng_ref] kernel constraint index of each reference constraint
    w_primary: np.ndarray    # [nw_ref] kernel index of each reference variable (-1: fixed, unused)
    steps_per_stage: int = 1  # reference steps per kernel stage
    w_fix_par: "np.ndarray | None" = None  # [nw_kernel] parameter fixing the variable (-1: none)
    w_zero: "np.ndarray | None" = None     # [nw_kernel] kernel-only dummies fixed to 0 (MHE X_0)

    @property
    def nw(self) -> int:
        return len(self.w_src)

    @property
    def npar(self) -> int:
        return len(self.p_src)


class NarxMultipleShooting(Discretization):
    """`casadi_ml.py:106-227` (``MultipleShooting_ML``), lifted for the kernel."""

    system_type = MLSystem
    admm = False

    def transcribe(self, system: MLSystem) -> StageNLP:
        t = _Transcriber(self.options)
        ref = self._discretize(t, system)
        S = self._super_stage_length(system, ref["n"], ref["lagged"])
        if S is not None:
            return self._lift_super(t, system, ref, S)
        return self._lift(t, system, ref)

    @staticmethod
    def _super_stage_length(s: MLSystem, N: int, lagged) -> "int | None":
        """Steps per kernel stage: the smallest S >= (largest lag of a variable) - 1
        dividing N, so every lagged value a stage reads lies in the stage itself or
        in the previous one (no copies).  None: no such S (copy-lifting instead)."""
        var_groups = {q.name for q in s.variables}
        need = 1
        for j, per_den in lagged.items():
            if any(den in var_groups for den in per_den):
                need = max(need, j)
        for S in range(need, N + 1):
            if N % S == 0:
                return S if S < N or N == need else None
        return None

    def _lift_super(self, t: _Transcriber, s: MLSystem, ref, S: int) -> StageNLP:
        """Kernel stages of S steps.  The stage state X_b (boundary b, step bS) holds
        x(bS) and the window v(bS - j), 1 <= j < lag(v), of every lagged variable, all
        as primary reference variables (they are the last steps' variables of stage
        b-1); V holds the remaining variables of the S steps (incl. the internal
        states).  Same NLP as the reference, only permuted."""
        mx, lagged, pred, ts, N = ref["mx"], ref["lagged"], ref["pred"], ref["ts"], ref["n"]
        uid_w = {sym_.uid: i for i, sym_ in enumerate(t.w)}
        uid_p = {sym_.uid: i for i, sym_ in enumerate(t.p)}
        nx = s.states.dim
        NB = N // S
        var_groups = {q.name for q in s.variables}
        window: List[Tuple[str, int, int]] = []
        for j in sorted(lagged):
            for den, names in lagged[j].items():
                if den not in var_groups:
                    continue
                q = next(q for q in s.quantities if q.name == den)
                for v_name in names:
                    window.append((den, q.full_names.index(v_name), j))

        def xbound(b):
            tm = b * S * ts
            xs = list(mx[tm][s.states.name])
            for den, i, j in window:
                xs.append(mx[tm - j * ts][den][i])
            return xs

        def vstage(b):
            xin = {sym_.uid for sym_ in xbound(b) + xbound(b + 1)}
            out = []
            for r in range(S):
                tm = (b * S + r) * ts
                for den, syms in mx[tm].items():
                    if den not in var_groups:
                        continue
                    out += [sym_ for sym_ in syms if sym_.uid not in xin]
            out.sort(key=lambda e: uid_w[e.uid])
            return out

        NXK = nx + len(window)
        NVK = len(vstage(0))
        X0 = [sx.sym(f"X0[{i}]") for i in range(NXK)]
        V = [sx.sym(f"V[{i}]") for i in range(NVK)]
        X1 = [sx.sym(f"X1[{i}]") for i in range(NXK)]
        TK = sx.sym("TK")
        rank = {q.name: r for r, q in enumerate(s.quantities)}
        glob_idx = list(range(ref["n_global_par"]))
        PG = [sx.sym(f"PG[{i}]") for i in range(len(glob_idx))]
        step_g = [[i for i, c in enumerate(t.g) if c[3] == k] for k in range(N)]
        roles_ref, stage_exprs, PS = None, None, []
        p_src_stage: List[List[int]] = []
        g_of_ref = np.empty(len(t.g), dtype=np.int64)
        ng_stage = None
        for b in range(NB):
            vb = vstage(b)
            if len(vb) != NVK:
                raise TranscriptionError("NARX stages differ in size")
            mapping = dict(zip(xbound(b), X0))
            mapping.update(zip(vb, V))
            mapping.update(zip(xbound(b + 1), X1))
            for i, gi in enumerate(glob_idx):
                mapping[t.p[gi]] = PG[i]
            for r in range(S):
                k = b * S + r
                if k in t.tk_syms:
                    mapping[t.tk_syms[k]] = sx.add(TK, sx.const(r * ts)) if r else TK
            gidx = [i for r in range(S) for i in step_g[b * S + r]]
            ng_stage = len(gidx) if ng_stage is None else ng_stage
            if len(gidx) != ng_stage:
                raise TranscriptionError("NARX stages differ in constraint count")
            gs = [t.g[i] for i in gidx]
            cost = sx.ZERO
            for r in range(S):
                cost = sx.add(cost, t.cost.get(b * S + r, sx.ZERO))
            exprs = [cost] + [c[0] for c in gs] + [c[1] for c in gs] + [c[2] for c in gs]
            used_p = sorted({uid_p[fs.uid] for fs in sx.free_symbols(exprs) if fs.uid in uid_p} - set(glob_idx))
            t0 = b * S * ts
            roles = [(t.p_labels[pi][0], t.p_labels[pi][1], round((t0 - t.p_labels[pi][2]) / ts)) for pi in used_p]
            order = sorted(range(len(roles)), key=lambda i: (roles[i][2], rank[roles[i][0]], roles[i][1]))
            roles = [roles[i] for i in order]
            used_p = [used_p[i] for i in order]
            if roles_ref is None:
                roles_ref = roles
                PS = [sx.sym(f"PS[{i}]") for i in range(len(roles))]
            elif roles != roles_ref:
                raise TranscriptionError(f"stage {b} uses different parameters than stage 0")
            mapping.update(zip([t.p[pi] for pi in used_p], PS))
            p_src_stage.append(used_p)
            sub = sx.substitute(exprs, mapping)
            allowed = {x.uid for x in X0 + V + X1 + PS + PG + [TK]}
            for fs in sx.free_symbols(sub):
                if fs.uid not in allowed:
                    raise TranscriptionError(f"NARX stage {b} depends on {fs.name}, which is not stage-local")
            if stage_exprs is None:
                stage_exprs = sub
            elif any(a is not c for a, c in zip(stage_exprs, sub)):
                raise TranscriptionError(f"NARX stage {b} differs structurally from stage 0")
            for pos, gi in enumerate(gidx):
                g_of_ref[gi] = b * ng_stage + pos
        ngs = ng_stage
        stage = StageFunction(X0=X0, V=V, X1=X1, PS=PS, PG=PG, TK=TK, cost=stage_exprs[0],
                              g=list(stage_exprs[1:1 + ngs]), g_lb=list(stage_exprs[1 + ngs:1 + 2 * ngs]),
                              g_ub=list(stage_exprs[1 + 2 * ngs:]))
        w_src = [uid_w[x.uid] for x in xbound(0)]
        for b in range(NB):
            w_src += [uid_w[x.uid] for x in vstage(b)] + [uid_w[x.uid] for x in xbound(b + 1)]
        w_src = np.asarray(w_src, dtype=np.int64)
        w_dup = np.zeros(len(w_src), dtype=bool)
        w_primary = np.full(len(t.w), -1, dtype=np.int64)
        for ki, ri in enumerate(w_src):
            if w_primary[ri] != -1:
                raise TranscriptionError("reference variable mapped twice in the lifted NLP")
            w_primary[ri] = ki
        self._check_unused_fixed(t, w_primary)
        p_src = np.asarray(glob_idx + [pi for st in p_src_stage for pi in st], dtype=np.int64)
        lift = LiftMaps(w_src=w_src, w_dup=w_dup, p_src=p_src, g_of_ref=g_of_ref, w_primary=w_primary,
                        steps_per_stage=S)
        f_total = sx.ZERO
        for k in range(N):
            f_total = sx.add(f_total, t.cost.get(k, sx.ZERO))
        return StageNLP(
            N=NB, nx=NXK, nv=NVK, ng=ngs, nps=len(PS), npg=len(PG), ts=S * ts,
            w_syms=list(t.w), p_syms=list(t.p), w_labels=list(t.w_labels), p_labels=list(t.p_labels),
            g_exprs=[c[0] for c in t.g], g_lb=[c[1] for c in t.g], g_ub=[c[2] for c in t.g],
            f_expr=f_total, var_groups=t.var_groups, par_groups=t.par_groups, stage=stage,
            tk_values=np.arange(NB, dtype=float) * S * ts, gap_closing=[c[4] for c in t.g], lift=lift,
        )

    @staticmethod
    def _check_unused_fixed(t: _Transcriber, w_primary: np.ndarray):
        """Reference variables the kernel NLP does not contain must be fixed past values."""
        for ri in np.nonzero(w_primary < 0)[0]:
            lay = t.var_groups[t.w_labels[ri][0]]
            col = [c for c in lay.columns if ri in c][0]
            if lay.lb_par[lay.columns.index(col)][col.index(ri)] < 0:
                raise TranscriptionError(f"reference variable {t.w_labels[ri]} is not used by any stage")

    # -- reference loops -----------------------------------------------------------
    def _discretize(self, t: _Transcriber, s: MLSystem):
        if s.objective.get_delta_u_objectives():
            raise TranscriptionError("change penalties (delta-u) are not supported yet")
        n, ts = int(self.options.prediction_horizon), float(self.options.time_step)
        L = s.max_lag
        t.pred_time = 0.0
        glob = {s.model_parameters.name: t.add_opt_par(s.model_parameters)}
        if self.admm:
            glob[s.penalty_factor.name] = t.add_opt_par(s.penalty_factor)
        n_global_par = len(t.p)
        pre_states = [ts * i for i in range(-L + 1, 1)]
        inputs_lag = min(-2, -L)
        pre_inputs = [ts * i for i in range(inputs_lag + 1, 0)]
        pred = [ts * i for i in range(0, n)]
        mx: Dict[float, Dict[str, list]] = {tm: {} for tm in sorted(set(pred + pre_inputs + pre_states))}
        for tm in pre_states:
            t.pred_time = tm
            x_past = t.add_opt_par(s.initial_state)
            mx[tm][s.states.name] = t.add_opt_var(s.states, lb=x_past, ub=x_past, guess=x_past)
        for tm in pre_inputs:
            t.pred_time = tm
            mx[tm][s.non_controlled_inputs.name] = t.add_opt_par(s.non_controlled_inputs)
            u_past = t.add_opt_par(s.last_control)
            mx[tm][s.controls.name] = t.add_opt_var(s.controls, lb=u_past, ub=u_past, guess=u_past)
            if self.admm:
                pc = t.add_opt_par(s.past_couplings)
                pe = t.add_opt_par(s.past_exchange)
                mx[tm][s.local_couplings.name] = t.add_opt_var(s.local_couplings, lb=pc, ub=pc, guess=pc)
                mx[tm][s.local_exchange.name] = t.add_opt_var(s.local_exchange, lb=pe, ub=pe, guess=pe)
        for tm in pred:
            t.pred_time = tm
            mx[tm][s.controls.name] = t.add_opt_var(s.controls)
            mx[tm][s.non_controlled_inputs.name] = t.add_opt_par(s.non_controlled_inputs)
            mx[tm][s.algebraics.name] = t.add_opt_var(s.algebraics)
            mx[tm][s.outputs.name] = t.add_opt_var(s.outputs)
            if self.admm:
                mx[tm][s.multipliers.name] = t.add_opt_par(s.multipliers)
                mx[tm][s.exchange_multipliers.name] = t.add_opt_par(s.exchange_multipliers)
                mx[tm][s.exchange_diff.name] = t.add_opt_par(s.exchange_diff)
                mx[tm][s.global_couplings.name] = t.add_opt_par(s.global_couplings)
                mx[tm][s.local_exchange.name] = t.add_opt_var(s.local_exchange)
                mx[tm][s.local_couplings.name] = t.add_opt_var(s.local_couplings)
        t.pred_time = 0.0
        for tm in pred[1:]:
            t.pred_time = tm
            mx[tm][s.states.name] = t.add_opt_var(s.states)
        t.pred_time += ts
        mx[t.pred_time] = {s.states.name: t.add_opt_var(s.states)}

        # lag structure (`casadi_ml.py:261-286`): dict[lag, dict[denotation, names]]
        lagged: Dict[int, Dict[str, List[str]]] = {}
        for q in s.stage_quantities():
            for v_name in q.full_names:
                for j in range(1, s.lags_dict.get(v_name, 1)):
                    lagged.setdefault(j, {}).setdefault(q.name, []).append(v_name)
        all_q = {q.name: q for q in s.quantities}

        stages = []
        for k, tm in enumerate(pred):
            vals: Dict[sx.Expr, sx.Expr] = {}
            for q in s.quantities:
                if not q.use_in_stage_function:
                    continue
                if q.name in glob:
                    v = glob[q.name]
                else:
                    v = mx[tm].get(q.name)
                if v is None:
                    v = [sx.ZERO] * q.dim
                for sym_, val in zip(q.full_symbolic, v):
                    vals[sym_] = val
            for j, per_den in lagged.items():
                for den, names in per_den.items():
                    src = mx.get(tm - j * ts, {}).get(den)
                    if src is None:
                        raise TranscriptionError(
                            f"lag {j} of group '{den}' has no value before the horizon (the reference "
                            "transcription has no past values for this group either)")
                    for v_name in names:
                        idx = all_q[den].full_names.index(v_name)
                        vals[s.model.lags_mx_store[name_with_lag(v_name, j)]] = src[idx]
            # time: a per-stage symbol (TK in the stage function); the ADMM-NN stage
            # function has no time input (`casadi_admm_ml.py:339-357`)
            vals[s.time] = sx.ZERO if self.admm else t.tk_syms.setdefault(k, sx.sym(f"__tk_{k}"))
            cons = s.model_constraints
            nxt = [s.next_states[name] for name in s.states.full_names]
            outs = nxt + [s.objective.get_casadi_expression()] + [c[1] for c in cons] + \
                [c[0] for c in cons] + [c[2] for c in cons]
            res = sx.substitute(outs, vals)
            nx, nc = len(nxt), len(cons)
            x_next = mx[tm + ts][s.states.name]
            g_path, lb, ub = res[nx + 1:nx + 1 + nc], res[nx + 1 + nc:nx + 1 + 2 * nc], res[nx + 1 + 2 * nc:]
            t.block = k
            t.add_constraint(g_path, lb, ub)
            t.add_constraint([sx.sub(a, b) for a, b in zip(res[:nx], x_next)], gap_closing=True)
            t.add_cost(sx.mul(res[nx], ts))
            stages.append(tm)
        t.block = -1
        return {"mx": mx, "lagged": lagged, "n_global_par": n_global_par, "pred": pred, "ts": ts, "n": n}

    # -- lifting -------------------------------------------------------------------
    def _lift(self, t: _Transcriber, s: MLSystem, ref) -> StageNLP:
        mx, lagged, pred, ts, N = ref["mx"], ref["lagged"], ref["pred"], ref["ts"], ref["n"]
        uid_w = {sym_.uid: i for i, sym_ in enumerate(t.w)}
        uid_p = {sym_.uid: i for i, sym_ in enumerate(t.p)}
        nx = s.states.dim
        # lag window: (den, component, j), lag-major as in the reference's stage arguments
        var_groups = {q.name for q in s.variables}
        window: List[Tuple[str, int, int]] = []
        for j in sorted(lagged):
            for den, names in lagged[j].items():
                if den not in var_groups:
                    continue
                q = next(q for q in s.quantities if q.name == den)
                for v_name in names:
                    window.append((den, q.full_names.index(v_name), j))
        wpos = {key: nx + i for i, key in enumerate(window)}
        NXK = nx + len(window)

        def local_vars(tm):
            """Stage-local (non-state) variables at time tm in reference order."""
            out = []
            for den, syms in mx[tm].items():
                if den == s.states.name or den not in var_groups:
                    continue
                out += [(den, i, sym_) for i, sym_ in enumerate(syms)]
            out.sort(key=lambda e: uid_w[e[2].uid])
            return out

        v0 = local_vars(pred[0])
        NVK = len(v0)
        X0 = [sx.sym(f"X0[{i}]") for i in range(NXK)]
        V = [sx.sym(f"V[{i}]") for i in range(NVK)]
        X1 = [sx.sym(f"X1[{i}]") for i in range(NXK)]
        TK = sx.sym("TK")

        def xwin(tm):
            """Reference symbols of X at time tm: [x(tm), window values]."""
            xs = list(mx[tm][s.states.name])
            for den, i, j in window:
                xs.append(mx[tm - j * ts][den][i])
            return xs

        rank = {q.name: r for r, q in enumerate(s.quantities)}
        glob_idx = list(range(ref["n_global_par"]))
        PG = [sx.sym(f"PG[{i}]") for i in range(len(glob_idx))]
        stage_g = [[i for i, c in enumerate(t.g) if c[3] == k] for k in range(N)]
        roles_ref = None
        stage_exprs = None
        p_src_stage: List[List[int]] = []
        PS: List[sx.Expr] = []
        g_of_ref = np.empty(len(t.g), dtype=np.int64)
        ng_ref_stage = len(stage_g[0])
        for k, tm in enumerate(pred):
            xk, xk1 = xwin(tm), xwin(tm + ts)
            vk = [e[2] for e in local_vars(tm)]
            if len(vk) != NVK or len(stage_g[k]) != ng_ref_stage:
                raise TranscriptionError("NARX stages differ in size")
            mapping = {sym_: ph for sym_, ph in zip(xk, X0)}
            mapping.update({sym_: ph for sym_, ph in zip(vk, V)})
            for sym_, ph in zip(xk1[:nx], X1[:nx]):
                mapping[sym_] = ph
            for i, gi in enumerate(glob_idx):
                mapping[t.p[gi]] = PG[i]
            if k in t.tk_syms:
                mapping[t.tk_syms[k]] = TK
            gs = [t.g[i] for i in stage_g[k]]
            exprs = [t.cost.get(k, sx.ZERO)] + [c[0] for c in gs] + [c[1] for c in gs] + [c[2] for c in gs]
            # stage parameters by role (group, component, time offset)
            used_p = sorted({uid_p[fs.uid] for fs in sx.free_symbols(exprs) if fs.uid in uid_p} - set(glob_idx))
            roles = []
            for pi in used_p:
                name, comp, ptime = t.p_labels[pi]
                roles.append((name, comp, round((tm - ptime) / ts)))
            order = sorted(range(len(roles)), key=lambda i: (roles[i][2], rank[roles[i][0]], roles[i][1]))
            roles = [roles[i] for i in order]
            used_p = [used_p[i] for i in order]
            if roles_ref is None:
                roles_ref = roles
                PS = [sx.sym(f"PS[{i}]") for i in range(len(roles))]
            elif roles != roles_ref:
                raise TranscriptionError(f"stage {k} uses different parameters than stage 0")
            for pi, ph in zip(used_p, PS):
                mapping[t.p[pi]] = ph
            p_src_stage.append(used_p)
            sub = sx.substitute(exprs, mapping)
            allowed = {x.uid for x in X0 + V + X1 + PS + PG + [TK]}
            for e in sub:
                for fs in sx.free_symbols([e]):
                    if fs.uid not in allowed:
                        raise TranscriptionError(f"NARX stage {k} depends on {fs.name}, which is not stage-local")
            if stage_exprs is None:
                stage_exprs = sub
            elif any(a is not b for a, b in zip(stage_exprs, sub)):
                raise TranscriptionError(f"NARX stage {k} differs structurally from stage 0")
        ngr = ng_ref_stage
        cost = stage_exprs[0]
        g = list(stage_exprs[1:1 + ngr])
        g_lb = list(stage_exprs[1 + ngr:1 + 2 * ngr])
        g_ub = list(stage_exprs[1 + 2 * ngr:])
        # shift constraints of the lag window
        vpos = {(e[0], e[1]): i for i, e in enumerate(v0)}
        for (den, i, j), pos in zip(window, range(nx, NXK)):
            if j > 1:
                src = X0[wpos[(den, i, j - 1)]]
            elif den == s.states.name:
                src = X0[i]
            else:
                src = V[vpos[(den, i)]]
            g.append(sx.sub(X1[pos], src))
            g_lb.append(sx.ZERO)
            g_ub.append(sx.ZERO)
        NGK = len(g)
        for k in range(N):
            for r, gi in enumerate(stage_g[k]):
                g_of_ref[gi] = k * NGK + r
        stage = StageFunction(X0=X0, V=V, X1=X1, PS=PS, PG=PG, TK=TK, cost=cost, g=g, g_lb=g_lb, g_ub=g_ub)

        # kernel variable maps: [X_0, {V_k, X_{k+1}}]
        w_src, w_dup = [], []
        for sym_ in xwin(pred[0]):
            w_src.append(uid_w[sym_.uid]); w_dup.append(False)
        for tm in pred:
            for e in local_vars(tm):
                w_src.append(uid_w[e[2].uid]); w_dup.append(False)
            for c, sym_ in enumerate(xwin(tm + ts)):
                w_src.append(uid_w[sym_.uid]); w_dup.append(c >= nx)
        w_src = np.asarray(w_src, dtype=np.int64)
        w_dup = np.asarray(w_dup, dtype=bool)
        w_primary = np.full(len(t.w), -1, dtype=np.int64)
        for ki in np.nonzero(~w_dup)[0]:
            if w_primary[w_src[ki]] != -1:
                raise TranscriptionError("reference variable mapped twice in the lifted NLP")
            w_primary[w_src[ki]] = ki
        for ri in np.nonzero(w_primary < 0)[0]:
            lay = t.var_groups[t.w_labels[ri][0]]
            # unused reference variables must be fixed past values (lb = ub = parameter)
            col = [c for c in lay.columns if ri in c][0]
            tix = lay.columns.index(col)
            if lay.lb_par[tix][col.index(ri)] < 0:
                raise TranscriptionError(f"reference variable {t.w_labels[ri]} is not used by any stage")
        p_src = np.asarray(glob_idx + [pi for st in p_src_stage for pi in st], dtype=np.int64)
        lift = LiftMaps(w_src=w_src, w_dup=w_dup, p_src=p_src, g_of_ref=g_of_ref, w_primary=w_primary)
        f_total = sx.ZERO
        for k in range(N):
            f_total = sx.add(f_total, t.cost.get(k, sx.ZERO))
        return StageNLP(
            N=N, nx=NXK, nv=NVK, ng=NGK, nps=len(PS), npg=len(PG), ts=ts,
            w_syms=list(t.w), p_syms=list(t.p), w_labels=list(t.w_labels), p_labels=list(t.p_labels),
            g_exprs=[c[0] for c in t.g], g_lb=[c[1] for c in t.g], g_ub=[c[2] for c in t.g],
            f_expr=f_total, var_groups=t.var_groups, par_groups=t.par_groups, stage=stage,
            tk_values=np.arange(N, dtype=float) * ts, gap_closing=[c[4] for c in t.g], lift=lift,
        )


class NarxADMMMultipleShooting(NarxMultipleShooting):
    """`casadi_admm_ml.py:247-397` (``MultipleShootingADMMNN``); the stage function
    gets no time argument (`casadi_admm_ml.py:339-357`)."""

    system_type = ADMMNNSystem
    admm = True
