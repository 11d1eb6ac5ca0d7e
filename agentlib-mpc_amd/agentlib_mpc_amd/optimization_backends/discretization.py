"""Transcription of the optimal control problem into a stage-structured NLP.

The reference transcribes with CasADi symbols in
`casadi_/basic.py:113-392` (direct collocation, multiple shooting),
`casadi_/full.py:36-166` (with ``u_prev``), `casadi_/admm.py:119-338` (ADMM)
and bookkeeps through `core/discretization.py:486-595` (``add_opt_var``,
``add_opt_par``, ``add_constraint``, ``grid``).  This module follows the same
loops, in the same order, so the NLP vector ``w``, the parameter vector ``p``
and the constraint vector ``g`` have exactly the reference layout (SURVEY
§8a A6/A7):

* ``w = [x_0, (v_0, x_1), (v_1, x_2), ..., (v_{N-1}, x_N)]``
* ``p = [global params, stage params of stage 0, ..., of stage N-1]``
* ``g = [g_0, ..., g_{N-1}]`` (all constraints of a stage are contiguous).

Because every stage has the same structure, the transcription also produces
ONE generic *stage function* in placeholder symbols ``X0`` (state at the
stage start), ``V`` (stage-local variables), ``X1`` (state at the stage end),
``PS`` (stage parameters), ``PG`` (global parameters) and ``TK`` (stage start
time).  That stage function is what the code generator turns into
straight-line HIP (cost, constraints, bounds, gradient, Jacobian and
Lagrangian Hessian) for the batched interior-point kernel.
"""

from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from agentlib_mpc_amd import symbolic as sx
from agentlib_mpc_amd.data_structures.mpc_datamodels import (
    CasadiDiscretizationOptions, CollocationMethod, Integrators,
)
from agentlib_mpc_amd.optimization_backends.system import (
    ADMMSystem, BaseSystem, FullSystem, OptimizationParameter, OptimizationVariable,
)


# ---------------------------------------------------------------------------
# collocation polynomial (`casadi_/basic.py:344-392`)
# ---------------------------------------------------------------------------

def collocation_points(d: int, method: str) -> np.ndarray:
    """Roots of the collocation polynomial on [0, 1] (``ca.collocation_points``)."""
    method = CollocationMethod(method)
    if method == CollocationMethod.legendre:
        x, _ = np.polynomial.legendre.leggauss(d)
        return np.sort((x + 1.0) / 2.0)
    # Radau IIA: roots of P_d - P_{d-1} on [-1, 1] (includes x = 1)
    c = np.zeros(d + 1)
    c[d] = 1.0
    c[d - 1] = -1.0
    x = np.polynomial.legendre.legroots(c)
    x = np.sort(np.real(x))
    x[-1] = 1.0
    return (x + 1.0) / 2.0


@dataclasses.dataclass
class CollocationMatrices:
    order: int
    root: np.ndarray
    B: np.ndarray
    C: np.ndarray
    D: np.ndarray


def collocation_polynomial(d: int, method: str) -> CollocationMatrices:
    """Lagrange basis on tau = [0, roots]: derivative (C), continuity (D) and
    quadrature (B) coefficients."""
    tau = np.append(0.0, collocation_points(d, method))
    C = np.zeros((d + 1, d + 1))
    D = np.zeros(d + 1)
    B = np.zeros(d + 1)
    for j in range(d + 1):
        p = np.poly1d([1.0])
        for r in range(d + 1):
            if r != j:
                p *= np.poly1d([1.0, -tau[r]]) / (tau[j] - tau[r])
        D[j] = p(1.0)
        dp = np.polyder(p)
        for r in range(d + 1):
            C[j, r] = dp(tau[r])
        B[j] = np.polyint(p)(1.0)
    return CollocationMatrices(order=d, root=tau, B=B, C=C, D=D)


# ---------------------------------------------------------------------------
# bookkeeping containers
# ---------------------------------------------------------------------------

@dataclasses.dataclass
class GroupLayout:
    """Where one variable/parameter group lives in ``w`` / ``p``.

    ``index[i, t]`` is the position of component ``i`` at grid point ``t``.
    For variables, ``lb_par`` / ``ub_par`` / ``guess_par`` hold ``p``-indices
    that override runtime bounds (-1 = no override), used for ``x_0``.
    """

    name: str
    is_variable: bool
    dim: int
    grid: List[float] = dataclasses.field(default_factory=list)
    columns: List[List[int]] = dataclasses.field(default_factory=list)
    lb_par: List[List[int]] = dataclasses.field(default_factory=list)
    ub_par: List[List[int]] = dataclasses.field(default_factory=list)
    guess_par: List[List[int]] = dataclasses.field(default_factory=list)

    @property
    def index(self) -> np.ndarray:
        if not self.columns:
            return np.zeros((self.dim, 0), dtype=np.int64)
        return np.asarray(self.columns, dtype=np.int64).T.reshape(self.dim, len(self.grid))


@dataclasses.dataclass
class StageFunction:
    """Generic stage of the NLP in placeholder symbols."""

    X0: List[sx.Expr]
    V: List[sx.Expr]
    X1: List[sx.Expr]
    PS: List[sx.Expr]
    PG: List[sx.Expr]
    TK: sx.Expr
    cost: sx.Expr
    g: List[sx.Expr]
    g_lb: List[sx.Expr]
    g_ub: List[sx.Expr]

    @property
    def local(self) -> List[sx.Expr]:
        return list(self.X0) + list(self.V) + list(self.X1)


@dataclasses.dataclass
class StageNLP:
    """The transcribed NLP: reference layout + generic stage function."""

    N: int
    nx: int
    nv: int
    ng: int
    nps: int
    npg: int
    ts: float
    w_syms: List[sx.Expr]
    p_syms: List[sx.Expr]
    w_labels: List[Tuple[str, int, float]]
    p_labels: List[Tuple[str, int, float]]
    g_exprs: List[sx.Expr]
    g_lb: List[sx.Expr]
    g_ub: List[sx.Expr]
    f_expr: sx.Expr
    var_groups: Dict[str, GroupLayout]
    par_groups: Dict[str, GroupLayout]
    stage: StageFunction
    tk_values: np.ndarray
    gap_closing: List[bool]
    #: index maps to the kernel's lifted stage NLP (NARX transcriptions), else None
    lift: Optional[object] = None
    #: symbols of the stage start times in the reference expressions (value tk_values[k])
    tk_syms: Optional[Dict[int, sx.Expr]] = None
    #: factor every KKT system with the sequential block chain (MHE lifts, see mhe.py)
    force_block_chain: bool = False

    @property
    def nw(self) -> int:
        return len(self.w_syms)

    # sizes of the NLP the kernel solves (== reference sizes unless lifted)
    @property
    def kernel_nw(self) -> int:
        return self.nx + self.N * (self.nv + self.nx)

    @property
    def kernel_ng(self) -> int:
        return self.N * self.ng

    @property
    def kernel_np(self) -> int:
        return self.npg + self.N * self.nps

    @property
    def npar(self) -> int:
        return len(self.p_syms)

    @property
    def ng_total(self) -> int:
        return len(self.g_exprs)

    def nlp_dims(self) -> Dict[str, int]:
        return {"nw": self.nw, "ng": self.ng_total, "np": self.npar}


class TranscriptionError(NotImplementedError):
    pass


class _Transcriber:
    """Reference-ordered bookkeeping (`core/discretization.py:486-595`)."""

    def __init__(self, options: CasadiDiscretizationOptions):
        self.options = options
        self.pred_time = 0.0
        #: time of stage 0's start (0 for MPC; -N*ts for the MHE's past horizon)
        self.t_start = 0.0
        self.k = 0
        self.block = -1
        self.w: List[sx.Expr] = []
        self.w_block: List[int] = []
        self.w_labels: List[Tuple[str, int, float]] = []
        self.p: List[sx.Expr] = []
        self.p_block: List[int] = []
        self.p_labels: List[Tuple[str, int, float]] = []
        self.g: List[Tuple[sx.Expr, sx.Expr, sx.Expr, int, bool]] = []
        self.cost: Dict[int, sx.Expr] = {}
        self.var_groups: Dict[str, GroupLayout] = {}
        self.par_groups: Dict[str, GroupLayout] = {}
        self.tk_syms: Dict[int, sx.Expr] = {}
        #: change penalties: the previous controls carried in the kernel's stage state
        #: ({"v_pos": positions of u in V, "init": u_prev parameter symbols})
        self.carry: Optional[dict] = None

    # time as "stage start symbol + offset" keeps all stages structurally equal
    def time_expr(self) -> sx.Expr:
        if self.block < 0:
            return sx.const(self.pred_time)
        tk = self.tk_syms.setdefault(self.block, sx.sym(f"__tk_{self.block}"))
        return sx.add(tk, sx.const(self.pred_time - self.t_start - self.block * self.options.time_step))

    def add_opt_var(self, q: OptimizationVariable, lb=None, ub=None, guess=None) -> List[sx.Expr]:
        lay = self.var_groups.setdefault(q.name, GroupLayout(q.name, True, q.dim))
        syms, cols = [], []
        for i in range(q.dim):
            s = sx.sym(f"{q.name}_{self.pred_time}_{i}")
            cols.append(len(self.w))
            self.w.append(s)
            self.w_block.append(self.block)
            self.w_labels.append((q.name, i, self.pred_time))
            syms.append(s)
        lay.grid.append(self.pred_time)
        lay.columns.append(cols)
        lay.lb_par.append(self._par_refs(lb, q.dim))
        lay.ub_par.append(self._par_refs(ub, q.dim))
        lay.guess_par.append(self._par_refs(guess, q.dim))
        return syms

    def _par_refs(self, syms, dim) -> List[int]:
        if syms is None:
            return [-1] * dim
        pos = {s.uid: i for i, s in enumerate(self.p)}
        return [pos[s.uid] for s in syms]

    def add_opt_par(self, q: OptimizationParameter) -> List[sx.Expr]:
        lay = self.par_groups.setdefault(q.name, GroupLayout(q.name, False, q.dim))
        syms, cols = [], []
        for i in range(q.dim):
            s = sx.sym(f"{q.name}_{self.pred_time}_{i}")
            cols.append(len(self.p))
            self.p.append(s)
            self.p_block.append(self.block)
            self.p_labels.append((q.name, i, self.pred_time))
            syms.append(s)
        lay.grid.append(self.pred_time)
        lay.columns.append(cols)
        return syms

    def add_constraint(self, funcs: Sequence, lb: Sequence = None, ub: Sequence = None,
                       gap_closing: bool = False):
        funcs = [sx.as_expr(f) for f in funcs]
        lb = [sx.ZERO] * len(funcs) if lb is None else [sx.as_expr(v) for v in lb]
        ub = [sx.ZERO] * len(funcs) if ub is None else [sx.as_expr(v) for v in ub]
        for f, l, u in zip(funcs, lb, ub):
            self.g.append((f, l, u, self.block, gap_closing))

    def add_cost(self, expr):
        self.cost[self.block] = sx.add(self.cost.get(self.block, sx.ZERO), expr)

    @staticmethod
    def stage_call(system: BaseSystem, values: Dict[str, List[sx.Expr]], time: sx.Expr):
        """Evaluate ode / cost / constraints of the model at given group values
        (the reference's ``_stage_function`` call)."""
        mapping: Dict[sx.Expr, sx.Expr] = {}
        for q in system.quantities:
            if not q.use_in_stage_function:
                continue
            vals = values.get(q.name)
            if vals is None:
                vals = [sx.ZERO] * q.dim  # missing named inputs default to 0 in CasADi
            for s, v in zip(q.full_symbolic, vals):
                mapping[s] = v
        mapping[system.time] = time
        cons = system.model_constraints
        outs = list(system.ode) + [system.objective.get_casadi_expression()]
        outs += [c[1] for c in cons] + [c[0] for c in cons] + [c[2] for c in cons]
        res = sx.substitute(outs, mapping)
        nx, nc = len(system.ode), len(cons)
        ode = res[:nx]
        cost = res[nx]
        g = res[nx + 1: nx + 1 + nc]
        lb = res[nx + 1 + nc: nx + 1 + 2 * nc]
        ub = res[nx + 1 + 2 * nc:]
        return ode, cost, g, lb, ub

    # -----------------------------------------------------------------------
    def finalize(self, system: BaseSystem) -> StageNLP:
        opts = self.options
        N = int(opts.prediction_horizon)
        nx = system.states.dim
        blocks = {}
        for i, b in enumerate(self.w_block):
            blocks.setdefault(b, []).append(i)
        init = blocks.get(-1, [])
        if len(init) != nx:
            raise TranscriptionError("initial block must hold exactly the initial state")
        npg = sum(1 for b in self.p_block if b == -1)
        if any(b == -1 for b in self.p_block[npg:]):
            raise TranscriptionError("global parameters must precede stage parameters")
        if any(gb == -1 for *_, gb, _ in self.g):
            raise TranscriptionError("constraints outside the stage loop are not supported")
        if -1 in self.cost:
            raise TranscriptionError("cost terms outside the stage loop are not supported")

        stage_w = [blocks.get(k, []) for k in range(N)]
        nloc = {len(s) for s in stage_w}
        if len(nloc) != 1:
            raise TranscriptionError("stages have different numbers of variables")
        nv = nloc.pop() - nx
        stage_p = [[i for i, b in enumerate(self.p_block) if b == k] for k in range(N)]
        nps_set = {len(s) for s in stage_p}
        if len(nps_set) != 1:
            raise TranscriptionError("stages have different numbers of parameters")
        nps = nps_set.pop()
        stage_g = [[i for i, c in enumerate(self.g) if c[3] == k] for k in range(N)]
        ng_set = {len(s) for s in stage_g}
        if len(ng_set) != 1:
            raise TranscriptionError("stages have different numbers of constraints")
        ng = ng_set.pop()
        # contiguity checks (reference layout == stage layout)
        expect = list(range(nx, nx + N * (nv + nx)))
        if [i for s in stage_w for i in s] != expect:
            raise TranscriptionError("stage variables are not contiguous")
        if [i for s in stage_g for i in s] != list(range(len(self.g))):
            raise TranscriptionError("stage constraints are not contiguous")
        if [i for s in stage_p for i in s] != list(range(npg, len(self.p))):
            raise TranscriptionError("stage parameters are not contiguous")

        # change penalties read u_{k-1}: the kernel stage state carries a copy of it
        # (X_k = [x_k, u_{k-1}], shift constraint X_{k+1}[u] = u_k; X_0[u] is fixed
        # to u_prev), every reference variable keeps its primary position
        carry = self.carry
        nc = len(carry["v_pos"]) if carry else 0
        X0 = [sx.sym(f"X0[{i}]") for i in range(nx + nc)]
        V = [sx.sym(f"V[{i}]") for i in range(nv)]
        X1 = [sx.sym(f"X1[{i}]") for i in range(nx + nc)]
        PS = [sx.sym(f"PS[{i}]") for i in range(nps)]
        PG = [sx.sym(f"PG[{i}]") for i in range(npg)]
        TK = sx.sym("TK")
        ref = None
        for k in range(N):
            prev = init if k == 0 else stage_w[k - 1][-nx:] if nx else []
            mapping = {}
            for s, ph in zip([self.w[i] for i in prev], X0):
                mapping[s] = ph
            loc = stage_w[k]
            for s, ph in zip([self.w[i] for i in loc[:nv]], V):
                mapping[s] = ph
            for s, ph in zip([self.w[i] for i in loc[nv:]], X1):
                mapping[s] = ph
            for s, ph in zip([self.p[i] for i in stage_p[k]], PS):
                mapping[s] = ph
            for s, ph in zip(self.p[:npg], PG):
                mapping[s] = ph
            if carry:
                src = carry["init"] if k == 0 else [self.w[stage_w[k - 1][q]] for q in carry["v_pos"]]
                for s, ph in zip(src, X0[nx:]):
                    mapping[s] = ph
            if k in self.tk_syms:
                mapping[self.tk_syms[k]] = TK
            gs = [self.g[i] for i in stage_g[k]]
            exprs = [self.cost.get(k, sx.ZERO)] + [c[0] for c in gs] + [c[1] for c in gs] + [c[2] for c in gs]
            sub = sx.substitute(exprs, mapping)
            allowed = {s.uid for s in X0 + V + X1 + PS + PG + [TK]}
            for e in sub:
                for fs in sx.free_symbols([e]):
                    if fs.uid not in allowed:
                        raise TranscriptionError(
                            f"stage {k} depends on {fs.name}, which is not stage-local "
                            "(e.g. change penalties between controls of neighbouring stages)")
            if ref is None:
                ref = sub
            elif any(a is not b for a, b in zip(ref, sub)):
                raise TranscriptionError(f"stage {k} differs structurally from stage 0")
        g, g_lb, g_ub = list(ref[1:1 + ng]), list(ref[1 + ng:1 + 2 * ng]), list(ref[1 + 2 * ng:])
        lift = None
        if carry:
            for i, q in enumerate(carry["v_pos"]):
                g.append(sx.sub(X1[nx + i], V[q]))
                g_lb.append(sx.ZERO)
                g_ub.append(sx.ZERO)
            lift = self._carry_maps(N, nx, nv, ng, nc, stage_w, carry)
        stage = StageFunction(X0=X0, V=V, X1=X1, PS=PS, PG=PG, TK=TK, cost=ref[0], g=g, g_lb=g_lb, g_ub=g_ub)
        f_total = sx.ZERO
        for k in range(N):
            f_total = sx.add(f_total, self.cost.get(k, sx.ZERO))
        return StageNLP(
            lift=lift, tk_syms=dict(self.tk_syms),
            N=N, nx=nx + nc, nv=nv, ng=ng + nc, nps=nps, npg=npg, ts=float(opts.time_step),
            w_syms=list(self.w), p_syms=list(self.p), w_labels=list(self.w_labels),
            p_labels=list(self.p_labels), g_exprs=[c[0] for c in self.g],
            g_lb=[c[1] for c in self.g], g_ub=[c[2] for c in self.g], f_expr=f_total,
            var_groups=self.var_groups, par_groups=self.par_groups, stage=stage,
            tk_values=np.arange(N, dtype=float) * float(opts.time_step),
            gap_closing=[c[4] for c in self.g],
        )


    def _carry_maps(self, N, nx, nv, ng, nc, stage_w, carry):
        from agentlib_mpc_amd.optimization_backends.narx import LiftMaps

        pos = {s.uid: i for i, s in enumerate(self.p)}
        w_src, w_dup, w_fix = list(range(nx)), [False] * nx, [-1] * nx
        w_src += [0] * nc
        w_dup += [False] * nc
        w_fix += [pos[s.uid] for s in carry["init"]]           # X_0[u] = u_prev (fixed)
        for k in range(N):
            loc = stage_w[k]
            w_src += loc[:nv] + loc[nv:] + [loc[q] for q in carry["v_pos"]]
            w_dup += [False] * (nv + nx) + [True] * nc         # X_{k+1}[u]: copy of u_k
            w_fix += [-1] * (nv + nx + nc)
        w_src = np.asarray(w_src, dtype=np.int64)
        w_dup = np.asarray(w_dup, dtype=bool)
        w_fix = np.asarray(w_fix, dtype=np.int64)
        w_primary = np.full(len(self.w), -1, dtype=np.int64)
        for ki in np.nonzero(~w_dup & (w_fix < 0))[0]:
            w_primary[w_src[ki]] = ki
        ngk = ng + nc
        g_of_ref = np.asarray([k * ngk + r for k in range(N) for r in range(ng)], dtype=np.int64)
        return LiftMaps(w_src=w_src, w_dup=w_dup, p_src=np.arange(len(self.p), dtype=np.int64),
                        g_of_ref=g_of_ref, w_primary=w_primary, w_fix_par=w_fix)


# ---------------------------------------------------------------------------
# discretisations
# ---------------------------------------------------------------------------

def _tk_values_fix(nlp: StageNLP, tk_used: bool):
    return nlp


class Discretization:
    system_type = BaseSystem

    def __init__(self, options: CasadiDiscretizationOptions):
        self.options = options

    def transcribe(self, system: BaseSystem) -> StageNLP:
        t = _Transcriber(self.options)
        self._discretize(t, system)
        return t.finalize(system)

    def _discretize(self, t: _Transcriber, sys_: BaseSystem):
        raise NotImplementedError

    @staticmethod
    def _delta_u(t: _Transcriber, s, u_prev, uk, const_par, u_prev_par):
        """Change penalties ``w**2 * (u_k - u_{k-1})**2`` (`core/delta_u.py:13-26`;
        not multiplied by ts) added to the cost of the current stage; registers the
        carried previous control for the kernel's stage form."""
        dus = s.objective.get_delta_u_objectives()
        if not dus:
            return
        from agentlib_mpc_amd.data_structures.objective import _weight_sym

        if t.carry is None:
            t.carry = {"v_pos": list(range(s.controls.dim)), "init": list(u_prev_par)}
        sub = dict(zip(s.model_parameters.full_symbolic, const_par))
        total = sx.ZERO
        for obj in dus:
            names = list(s.controls.ref_names)
            if obj.control.name not in names:
                continue  # the reference logs an error and adds 0 (`delta_u.py:24-26`)
            idx = names.index(obj.control.name)
            w = sx.substitute([sx.as_expr(_weight_sym(obj.weight))], sub)[0]
            total = sx.add(total, sx.mul(sx.power(w, 2), sx.power(sx.sub(uk[idx], u_prev[idx]), 2)))
        t.add_cost(total)

    # shared collocation inner loop (`casadi_/basic.py:251-342`)
    def _collocation_inner_loop(self, t: _Transcriber, sys_: BaseSystem, cm: CollocationMatrices,
                                x_start: List[sx.Expr], inner_vars: List[OptimizationVariable],
                                inner_pars: List[OptimizationParameter],
                                const: Dict[str, List[sx.Expr]]):
        ts = self.options.time_step
        start = t.pred_time
        xs, var_vals, par_vals, times = [], [], [], []
        for j in range(cm.order):
            t.pred_time = start + cm.root[j + 1] * ts
            xs.append(t.add_opt_var(sys_.states))
            var_vals.append({q.name: t.add_opt_var(q) for q in inner_vars})
            par_vals.append({q.name: t.add_opt_par(q) for q in inner_pars})
            times.append(t.time_expr())
        cons = []
        x_end = [sx.mul(cm.D[0], x) for x in x_start]
        for j in range(1, cm.order + 1):
            xp = [sx.mul(cm.C[0, j], x) for x in x_start]
            for r in range(cm.order):
                xp = [sx.add(a, sx.mul(cm.C[r + 1, j], b)) for a, b in zip(xp, xs[r])]
            values = {sys_.states.name: xs[j - 1], **par_vals[j - 1], **var_vals[j - 1], **const}
            ode, cost, g, lb, ub = t.stage_call(sys_, values, times[j - 1])
            cons.append(([sx.sub(sx.mul(ts, o), x) for o, x in zip(ode, xp)], None, None))
            cons.append((g, lb, ub))
            x_end = [sx.add(a, sx.mul(cm.D[j], b)) for a, b in zip(x_end, xs[j - 1])]
            t.add_cost(sx.mul(sx.mul(cm.B[j], cost), ts))
        return x_end, cons


class BasicCollocation(Discretization):
    """`casadi_/basic.py:113-173` (backend ``casadi_basic``)."""

    def _discretize(self, t, s):
        cm = collocation_polynomial(self.options.collocation_order, self.options.collocation_method)
        n, ts = self.options.prediction_horizon, self.options.time_step
        x0 = t.add_opt_par(s.initial_state)
        xk = t.add_opt_var(s.states, lb=x0, ub=x0, guess=x0)
        const_par = t.add_opt_par(s.model_parameters)
        for k in range(n):
            t.block = k
            uk = t.add_opt_var(s.controls)
            dk = t.add_opt_par(s.non_controlled_inputs)
            const = {s.controls.name: uk, s.non_controlled_inputs.name: dk,
                     s.model_parameters.name: const_par}
            x_end, cons = self._collocation_inner_loop(t, s, cm, xk, [s.algebraics, s.outputs], [], const)
            t.pred_time = ts * (k + 1)
            xk = t.add_opt_var(s.states)
            t.add_constraint([sx.sub(a, b) for a, b in zip(xk, x_end)], gap_closing=True)
            for c in cons:
                t.add_constraint(*c)


class FullCollocation(Discretization):
    """`casadi_/full.py:36-98` (backend ``casadi``)."""

    system_type = FullSystem

    def _discretize(self, t, s):
        cm = collocation_polynomial(self.options.collocation_order, self.options.collocation_method)
        n, ts = self.options.prediction_horizon, self.options.time_step
        x0 = t.add_opt_par(s.initial_state)
        xk = t.add_opt_var(s.states, lb=x0, ub=x0, guess=x0)
        u_prev_par = uk = t.add_opt_par(s.last_control)
        const_par = t.add_opt_par(s.model_parameters)
        for k in range(n):
            t.block = k
            u_prev, uk = uk, t.add_opt_var(s.controls)
            self._delta_u(t, s, u_prev, uk, const_par, u_prev_par)
            const = {s.controls.name: uk, s.model_parameters.name: const_par}
            x_end, cons = self._collocation_inner_loop(
                t, s, cm, xk, [s.algebraics, s.outputs], [s.non_controlled_inputs], const)
            t.pred_time = ts * (k + 1)
            xk = t.add_opt_var(s.states)
            t.add_constraint([sx.sub(a, b) for a, b in zip(xk, x_end)], gap_closing=True)
            for c in cons:
                t.add_constraint(*c)


class ADMMCollocation(Discretization):
    """`casadi_/admm.py:119-195` (backend ``casadi_admm``, collocation)."""

    system_type = ADMMSystem

    def _discretize(self, t, s):
        cm = collocation_polynomial(self.options.collocation_order, self.options.collocation_method)
        n, ts = self.options.prediction_horizon, self.options.time_step
        x0 = t.add_opt_par(s.initial_state)
        xk = t.add_opt_var(s.states, lb=x0, ub=x0, guess=x0)
        u_prev_par = uk = t.add_opt_par(s.last_control)
        const_par = t.add_opt_par(s.model_parameters)
        rho = t.add_opt_par(s.penalty_factor)
        for k in range(n):
            t.block = k
            u_prev, uk = uk, t.add_opt_var(s.controls)
            self._delta_u(t, s, u_prev, uk, const_par, u_prev_par)
            inner_vars = [s.algebraics, s.outputs, s.local_couplings, s.local_exchange]
            inner_pars = [s.global_couplings, s.multipliers, s.exchange_multipliers,
                          s.exchange_diff, s.non_controlled_inputs]
            const = {s.controls.name: uk, s.model_parameters.name: const_par,
                     s.penalty_factor.name: rho}
            x_end, cons = self._collocation_inner_loop(t, s, cm, xk, inner_vars, inner_pars, const)
            t.pred_time = ts * (k + 1)
            xk = t.add_opt_var(s.states)
            t.add_constraint([sx.sub(a, b) for a, b in zip(xk, x_end)], gap_closing=True)
            for c in cons:
                t.add_constraint(*c)


def _euler(ode: List[sx.Expr], x: List[sx.Expr], ts: float) -> List[sx.Expr]:
    return [sx.add(xi, sx.mul(oi, ts)) for xi, oi in zip(x, ode)]


#: CasADi's "rk" integrator plugin: fixed-step classical RK4 over
#: ``number_of_finite_elements`` (default 20) steps of the interval
RK_FINITE_ELEMENTS = 20


def _rk4(f, x: List[sx.Expr], ts: float, steps: int = RK_FINITE_ELEMENTS) -> List[sx.Expr]:
    """``ca.integrator("system", "rk", ...)`` (`casadi_/basic.py:450-476`): the model
    inputs, parameters, algebraics and outputs are constant over the interval."""
    h = ts / steps
    for _ in range(steps):
        k1 = f(x)
        k2 = f([sx.add(a, sx.mul(h / 2, b)) for a, b in zip(x, k1)])
        k3 = f([sx.add(a, sx.mul(h / 2, b)) for a, b in zip(x, k2)])
        k4 = f([sx.add(a, sx.mul(h, b)) for a, b in zip(x, k3)])
        x = [sx.add(a, sx.mul(h / 6, sx.add(sx.add(b1, sx.mul(2.0, b2)), sx.add(sx.mul(2.0, b3), b4))))
             for a, b1, b2, b3, b4 in zip(x, k1, k2, k3, k4)]
    return x


class BasicMultipleShooting(Discretization):
    """`casadi_/basic.py:395-448` (backend ``casadi_basic``, multiple shooting)."""

    def _check_integrator(self, system=None):
        """Euler and the fixed-step "rk" plugin are restated; cvodes (adaptive) is
        not.  Without differential states (e.g. the three-zone AHU/CCA controllers,
        which keep the cvodes default) the integrator is never used."""
        if system is not None and system.states.dim == 0:
            return
        if self.options.integrator not in (Integrators.euler, Integrators.rk):
            raise TranscriptionError(
                f"integrator '{self.options.integrator.value}' is not supported on MI355X yet; "
                "use 'euler' or 'rk'")

    def _integrate(self, t, s, vals, xk, ode, time):
        """End state of the interval (`casadi_/basic.py:450-476` ``_create_ode``)."""
        ts = self.options.time_step
        if s.states.dim == 0 or self.options.integrator == Integrators.euler:
            return _euler(ode, xk, ts)
        name = s.states.name

        def f(x):
            return t.stage_call(s, {**vals, name: x}, time)[0]

        return _rk4(f, xk, ts)

    def _discretize(self, t, s):
        self._check_integrator(s)
        n, ts = self.options.prediction_horizon, self.options.time_step
        x0 = t.add_opt_par(s.initial_state)
        xk = t.add_opt_var(s.states, lb=x0, ub=x0, guess=x0)
        const_par = t.add_opt_par(s.model_parameters)
        for k in range(n):
            t.block = k
            uk = t.add_opt_var(s.controls)
            dk = t.add_opt_par(s.non_controlled_inputs)
            zk = t.add_opt_var(s.algebraics)
            yk = t.add_opt_var(s.outputs)
            vals = {s.states.name: xk, s.algebraics.name: zk, s.outputs.name: yk,
                    s.controls.name: uk, s.non_controlled_inputs.name: dk,
                    s.model_parameters.name: const_par}
            tk = t.time_expr()
            ode, cost, g, lb, ub = t.stage_call(s, vals, tk)
            t.add_constraint(g, lb, ub)
            x_end = self._integrate(t, s, vals, xk, ode, tk)
            t.pred_time = ts * (k + 1)
            xk = t.add_opt_var(s.states)
            t.add_constraint([sx.sub(a, b) for a, b in zip(x_end, xk)], gap_closing=True)
            t.add_cost(sx.mul(cost, ts))


class FullMultipleShooting(BasicMultipleShooting):
    """`casadi_/full.py:101-166` (backend ``casadi``, multiple shooting)."""

    system_type = FullSystem

    def _discretize(self, t, s):
        self._check_integrator(s)
        n, ts = self.options.prediction_horizon, self.options.time_step
        x0 = t.add_opt_par(s.initial_state)
        xk = t.add_opt_var(s.states, lb=x0, ub=x0, guess=x0)
        u_prev_par = uk = t.add_opt_par(s.last_control)
        const_par = t.add_opt_par(s.model_parameters)
        for k in range(n):
            t.block = k
            u_prev, uk = uk, t.add_opt_var(s.controls)
            self._delta_u(t, s, u_prev, uk, const_par, u_prev_par)
            dk = t.add_opt_par(s.non_controlled_inputs)
            zk = t.add_opt_var(s.algebraics)
            yk = t.add_opt_var(s.outputs)
            vals = {s.states.name: xk, s.algebraics.name: zk, s.outputs.name: yk,
                    s.controls.name: uk, s.non_controlled_inputs.name: dk,
                    s.model_parameters.name: const_par}
            tk = t.time_expr()
            ode, cost, g, lb, ub = t.stage_call(s, vals, tk)
            x_end = self._integrate(t, s, vals, xk, ode, tk)
            t.pred_time = ts * (k + 1)
            xk = t.add_opt_var(s.states)
            t.add_constraint([sx.sub(a, b) for a, b in zip(xk, x_end)], gap_closing=True)
            t.add_constraint(g, lb, ub)
            t.add_cost(sx.mul(cost, ts))


class ADMMMultipleShooting(BasicMultipleShooting):
    """`casadi_/admm.py:198-310` (backend ``casadi_admm``, multiple shooting).

    Reference quirks reproduced: ``model_parameters`` is added twice as a
    parameter (`admm.py:226-229`) and the stage function is called without a
    time argument, i.e. ``time = 0`` (`admm.py:262-276`).
    """

    system_type = ADMMSystem

    def _discretize(self, t, s):
        self._check_integrator(s)
        n, ts = self.options.prediction_horizon, self.options.time_step
        x0 = t.add_opt_par(s.initial_state)
        xk = t.add_opt_var(s.states, lb=x0, ub=x0, guess=x0)
        u_prev_par = uk = t.add_opt_par(s.last_control)
        const_par = t.add_opt_par(s.model_parameters)   # first copy weights the change penalties
        model_pars = t.add_opt_par(s.model_parameters)
        rho = t.add_opt_par(s.penalty_factor)
        for k in range(n):
            t.block = k
            u_prev, uk = uk, t.add_opt_var(s.controls)
            self._delta_u(t, s, u_prev, uk, const_par, u_prev_par)
            dk = t.add_opt_par(s.non_controlled_inputs)
            zk = t.add_opt_var(s.algebraics)
            yk = t.add_opt_var(s.outputs)
            lc = t.add_opt_var(s.local_couplings)
            gc = t.add_opt_par(s.global_couplings)
            mu = t.add_opt_par(s.multipliers)
            ed = t.add_opt_par(s.exchange_diff)
            em = t.add_opt_par(s.exchange_multipliers)
            le = t.add_opt_var(s.local_exchange)
            vals = {s.states.name: xk, s.algebraics.name: zk, s.local_couplings.name: lc,
                    s.outputs.name: yk, s.local_exchange.name: le, s.global_couplings.name: gc,
                    s.multipliers.name: mu, s.controls.name: uk,
                    s.non_controlled_inputs.name: dk, s.model_parameters.name: model_pars,
                    s.penalty_factor.name: rho, s.exchange_diff.name: ed,
                    s.exchange_multipliers.name: em}
            ode, cost, g, lb, ub = t.stage_call(s, vals, sx.ZERO)
            x_end = self._integrate(t, s, vals, xk, ode, sx.ZERO)
            t.pred_time = ts * (k + 1)
            xk = t.add_opt_var(s.states)
            t.add_constraint([sx.sub(a, b) for a, b in zip(xk, x_end)], gap_closing=True)
            t.add_constraint(g, lb, ub)
            t.add_cost(sx.mul(cost, ts))
