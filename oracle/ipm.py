"""ORACLE (test infrastructure only) — IPOPT-style primal-dual interior point method.

This is the CPU restatement of the solver the reference calls through
``ca.nlpsol("mpc", "ipopt", nlp, opts)`` (`agentlib_mpc/data_structures/casadi_utils.py:191-217`,
`282-300`; solve at `optimization_backends/casadi_/core/discretization.py:203`).
IPOPT itself is a third-party dependency absent from `/root/reference`
(bundled in the ``casadi>=3.6.6`` wheel, `pyproject.toml:30`, unpinned); this
module restates its published algorithm (Wächter & Biegler, Math. Prog. 106,
2006): barrier problem with slacks for inequalities, monotone Fiacco-McCormick
barrier update, primal-dual Newton step on the KKT system with inertia
correction (Algorithm IC), fraction-to-the-boundary rule and the filter line
search, gradient-based NLP scaling, bound relaxation and least-squares
constraint-multiplier initialisation, with IPOPT's default constants.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may use this package, and only as the checker.  The
dense KKT here is factored with ``scipy.linalg.ldl`` (Bunch-Kaufman), whose
D blocks give the inertia exactly as MUMPS does inside IPOPT.
"""

from __future__ import annotations

import dataclasses
import math
from typing import Callable, Dict, Optional

import numpy as np
import scipy.linalg

INF = 1e19  # IPOPT nlp_lower/upper_bound_inf
DEBUG = False
ZERO_PIVOT = 1e-20  # same constant as csrc/mpcx_ipm.hip


#: diagnostics only: a list receives the trials of the last line search (scripts/resto_diag.py)
LS_TRACE = None
KKT_HOOK = None  # diagnostics: called with (iteration, in restoration, dw, dc, K, npos, nneg, nzero)
IT_TRACE = None  # diagnostics: a list to collect (iteration, in restoration, mu, objective, refinement steps)


@dataclasses.dataclass
class IPMOptions:
    tol: float = 1e-8
    max_iter: int = 3000
    dual_inf_tol: float = 1.0
    constr_viol_tol: float = 1e-4
    compl_inf_tol: float = 1e-4
    # acceptable-level termination (IPOPT defaults; the reference overrides acceptable_tol,
    # acceptable_iter, acceptable_constr_viol_tol, acceptable_compl_inf_tol:
    # agentlib_mpc/data_structures/casadi_utils.py:197-206)
    acceptable_tol: float = 1e-6
    acceptable_iter: int = 15
    acceptable_dual_inf_tol: float = 1e10
    acceptable_constr_viol_tol: float = 1e-2
    acceptable_compl_inf_tol: float = 1e-2
    acceptable_obj_change_tol: float = 1e20
    mu_init: float = 0.1
    mu_min: float = 1e-11
    kappa_eps: float = 10.0
    kappa_mu: float = 0.2
    theta_mu: float = 1.5
    tau_min: float = 0.99
    bound_push: float = 1e-2
    bound_frac: float = 1e-2
    bound_relax_factor: float = 1e-8
    bound_mult_init_val: float = 1.0
    constr_mult_init_max: float = 1e3
    kappa_sigma: float = 1e10
    s_max: float = 100.0
    nlp_scaling_max_gradient: float = 100.0
    nlp_scaling_min_value: float = 1e-8
    # inertia correction
    delta_w_first: float = 1e-4
    delta_w_min: float = 1e-20
    delta_w_max: float = 1e40
    kappa_w_plus_bar: float = 100.0
    kappa_w_plus: float = 8.0
    kappa_w_minus: float = 1.0 / 3.0
    delta_c_bar: float = 1e-8
    kappa_c: float = 0.25
    # filter line search
    theta_max_fact: float = 1e4
    theta_min_fact: float = 1e-4
    eta_phi: float = 1e-8
    delta: float = 1.0
    s_phi: float = 2.3
    s_theta: float = 1.1
    gamma_phi: float = 1e-8
    gamma_theta: float = 1e-5
    alpha_min_frac: float = 0.05
    #: filter entries kept (IPOPT's list is unbounded; the kernel keeps its newest 48 in LDS and
    #: the older ones in a spill list in HBM, MAXF + FSPILL = 1024 in all, csrc/mpcx_ipm.hip): one
    #: cap for the kernel, oracle/c/ipm_oracle.c and this file; an insertion into a full filter
    #: drops the oldest entry and is counted
    max_filter: int = 1024
    # iterative refinement of the restoration-phase Newton steps on the full system (IPOPT
    # PDFullSpaceSolver: min_refinement_steps, max_refinement_steps, residual_ratio_max,
    # residual_improvement_factor)
    min_refinement_steps: int = 1
    max_refinement_steps: int = 10
    residual_ratio_max: float = 1e-10
    residual_improvement_factor: float = 1.0
    # soft restoration and the feasibility restoration phase (IPOPT defaults)
    soft_resto_pderror_reduction_factor: float = 0.9999
    max_soft_resto_iters: int = 10
    resto_penalty_parameter: float = 1000.0
    resto_proximity_weight: float = 1.0
    required_infeasibility_reduction: float = 0.9
    bound_mult_reset_threshold: float = 1000.0


@dataclasses.dataclass
class NLPFunctions:
    """Callables of one NLP instance (parameters already bound)."""

    n: int
    m: int
    f: Callable[[np.ndarray], float]
    grad_f: Callable[[np.ndarray], np.ndarray]
    g: Callable[[np.ndarray], np.ndarray]
    jac_g: Callable[[np.ndarray], np.ndarray]            # dense (m, n)
    hess_l: Callable[[np.ndarray, float, np.ndarray], np.ndarray]  # (x, sigma, lam) -> (n, n)


@dataclasses.dataclass
class IPMResult:
    x: np.ndarray
    lam_g: np.ndarray
    lam_x: np.ndarray
    f: float
    iterations: int
    status: str
    success: bool
    history: list
    s: Optional[np.ndarray] = None      # slacks of the inequality rows (scaled)
    n_soft_resto: int = 0               # line-search failures resolved by a soft restoration step
    n_resto: int = 0                    # calls of the feasibility restoration phase
    resto_iterations: int = 0           # iterations spent in it (counted in ``iterations``)
    filter_overflows: int = 0           # insertions into a full filter (oldest entry dropped)
    max_filter_size: int = 0            # largest filter held
    refine_steps: int = 0               # iterative-refinement corrections (restoration phase)


def _relax(b, lower: bool, factor: float):
    out = b.copy()
    fin = np.abs(b) < INF
    d = factor * np.maximum(1.0, np.abs(b[fin]))
    out[fin] = b[fin] - d if lower else b[fin] + d
    return out


def solve(nlp: NLPFunctions, x0, lbx, ubx, lbg, ubg, opts: IPMOptions = None,
          record: bool = False) -> IPMResult:
    o = opts or IPMOptions()
    with np.errstate(divide='ignore', invalid='ignore', over='ignore'):
        return _solve(nlp, x0, lbx, ubx, lbg, ubg, o, record)


@dataclasses.dataclass
class _Inner:
    """Restoration mode of :func:`_solve` (IPOPT runs a second IpoptAlgorithm on the
    RestoIpoptNLP, `MinC_1NrmRestorationPhase::PerformRestoration`): the NLP is already in
    the scaled space of the original one (no gradient scaling, no bound relaxation, no
    bound push), the multipliers and mu come from the original iterate, the constraint
    multipliers start at zero, and ``check(x, s)`` is the return test
    (`RestoConvergenceCheck`) evaluated at the head of every restoration iteration."""

    zL: np.ndarray
    zU: np.ndarray
    vL: np.ndarray
    vU: np.ndarray
    mu: float
    check: Callable
    set_mu: Callable


class _RestoNLP:
    """IPOPT's restoration NLP (`RestoIpoptNLP`, Wächter & Biegler 2006, eq. (30)) over the
    SCALED original constraints c~(x) (equalities) / d~(x) (with their slacks):

        min  rho * sum(p + n) + zeta(mu)/2 * || D_R (x - x_R) ||^2
        s.t. c~(x) - p + n = c~_L (equality rows),  d~(x) - p + n in [d~_L, d~_U],  p, n >= 0

    with rho = resto_penalty_parameter, zeta(mu) = resto_proximity_weight * sqrt(mu) (mu of
    the restoration problem itself), D_R = diag(1 / max(1, |x_R|)) and x_R the iterate at
    which restoration started.  Variables [x (n), p (m), n (m)]."""

    def __init__(self, F, JG, G, HC, n, m, xR, fixed, rho, weight):
        self.F, self.JG, self.G, self.HC = F, JG, G, HC
        self.n, self.m = n, m
        self.xR = xR
        self.dr2 = np.where(fixed, 0.0, 1.0 / np.maximum(1.0, np.abs(xR)) ** 2)
        self.rho, self.weight = rho, weight
        self.zeta = 0.0

    def set_mu(self, mu):
        self.zeta = self.weight * math.sqrt(mu)

    def functions(self) -> NLPFunctions:
        n, m = self.n, self.m

        def f(w):
            x = w[:n]
            return float(self.rho * np.sum(w[n:]) + 0.5 * self.zeta * np.sum(self.dr2 * (x - self.xR) ** 2))

        def grad(w):
            g = np.full(n + 2 * m, self.rho)
            g[:n] = self.zeta * self.dr2 * (w[:n] - self.xR)
            return g

        def g(w):
            return self.G(w[:n]) - w[n:n + m] + w[n + m:]

        def jac(w):
            J = np.zeros((m, n + 2 * m))
            J[:, :n] = self.JG(w[:n])
            J[:, n:n + m] = -np.eye(m)
            J[:, n + m:] = np.eye(m)
            return J

        def hess(w, sigma, lam):
            H = np.zeros((n + 2 * m, n + 2 * m))
            H[:n, :n] = self.HC(w[:n], lam) + np.diag(sigma * self.zeta * self.dr2)
            return H

        return NLPFunctions(n=n + 2 * m, m=m, f=f, grad_f=grad, g=g, jac_g=jac, hess_l=hess)


def _solve(nlp, x0, lbx, ubx, lbg, ubg, o, record, inner: Optional[_Inner] = None):
    n, m = nlp.n, nlp.m
    x = np.array(x0, dtype=float).copy()
    lbx = np.maximum(np.asarray(lbx, float), -INF)
    ubx = np.minimum(np.asarray(ubx, float), INF)
    lbg = np.maximum(np.asarray(lbg, float), -INF)
    ubg = np.minimum(np.asarray(ubg, float), INF)

    fixed = lbx == ubx
    x[fixed] = lbx[fixed]
    free = ~fixed
    # constraint classification
    eq = lbg == ubg
    ineq = ~eq

    # --- NLP scaling (gradient based, at the user starting point) ----------
    obj_scale = 1.0
    g_scale = np.ones(m)
    if inner is None:
        gf0 = nlp.grad_f(x)
        gmax = np.max(np.abs(gf0[free])) if free.any() else 0.0
        if gmax > o.nlp_scaling_max_gradient:
            obj_scale = max(o.nlp_scaling_min_value, o.nlp_scaling_max_gradient / gmax)
        J0 = nlp.jac_g(x)
        rowmax = np.max(np.abs(J0[:, free]), axis=1) if m else np.zeros(0)
        big = rowmax > o.nlp_scaling_max_gradient
        g_scale[big] = np.maximum(o.nlp_scaling_min_value, o.nlp_scaling_max_gradient / rowmax[big])

    def F(xx):
        return obj_scale * nlp.f(xx)

    def GF(xx):
        v = obj_scale * nlp.grad_f(xx)
        v[fixed] = 0.0
        return v

    def G(xx):
        return g_scale * nlp.g(xx)

    def JG(xx):
        J = g_scale[:, None] * nlp.jac_g(xx)
        J[:, fixed] = 0.0
        return J

    def H(xx, lam, sigma=None):
        Hm = nlp.hess_l(xx, obj_scale if sigma is None else sigma, lam * g_scale)
        Hm[fixed, :] = 0.0
        Hm[:, fixed] = 0.0
        return Hm

    # scaled, relaxed bounds (the restoration NLP is already relaxed and scaled)
    relax = 0.0 if inner is not None else o.bound_relax_factor
    xL = np.where(free & (lbx > -INF), _relax(lbx, True, relax), -np.inf)
    xU = np.where(free & (ubx < INF), _relax(ubx, False, relax), np.inf)
    sLb = np.where(lbg > -INF, lbg * g_scale, -np.inf)
    sUb = np.where(ubg < INF, ubg * g_scale, np.inf)
    sL = np.where(ineq, np.where(np.isfinite(sLb), _relax(np.where(np.isfinite(sLb), sLb, 0), True, relax), -np.inf), sLb)
    sU = np.where(ineq, np.where(np.isfinite(sUb), _relax(np.where(np.isfinite(sUb), sUb, 0), False, relax), np.inf), sUb)
    hasL, hasU = np.isfinite(xL), np.isfinite(xU)
    shasL, shasU = ineq & np.isfinite(sL), ineq & np.isfinite(sU)
    free_slack = ineq & ~shasL & ~shasU

    def push(v, lo, hi, hl, hu):
        v = v.copy()
        pl = np.where(hl, o.bound_push * np.maximum(1.0, np.abs(np.where(hl, lo, 0))), 0.0)
        pu = np.where(hu, o.bound_push * np.maximum(1.0, np.abs(np.where(hu, hi, 0))), 0.0)
        both = hl & hu
        width = np.where(both, np.where(both, hi, 0) - np.where(both, lo, 0), np.inf)
        pl = np.where(both, np.minimum(pl, o.bound_frac * width), pl)
        pu = np.where(both, np.minimum(pu, o.bound_frac * width), pu)
        lo_p = np.where(hl, lo + pl, -np.inf)
        hi_p = np.where(hu, hi - pu, np.inf)
        v = np.maximum(v, lo_p)
        v = np.minimum(v, hi_p)
        # degenerate interval: middle
        bad = both & (lo_p > hi_p)
        v[bad] = 0.5 * (lo[bad] + hi[bad])
        return v

    if inner is None:
        x = np.where(free, push(x, xL, xU, hasL, hasU), x)
        gx = G(x)
        s = np.where(ineq, push(gx, sL, sU, shasL, shasU), np.where(eq, lbg * g_scale, 0.0))
        zL = np.where(hasL, o.bound_mult_init_val, 0.0)
        zU = np.where(hasU, o.bound_mult_init_val, 0.0)
        vL = np.where(shasL, o.bound_mult_init_val, 0.0)
        vU = np.where(shasU, o.bound_mult_init_val, 0.0)
    else:  # the restoration starting point is interior by construction
        gx = G(x)
        s = np.where(ineq, gx, np.where(eq, lbg * g_scale, 0.0))
        zL, zU = np.where(hasL, inner.zL, 0.0), np.where(hasU, inner.zU, 0.0)
        vL, vU = np.where(shasL, inner.vL, 0.0), np.where(shasU, inner.vU, 0.0)

    mu = o.mu_init if inner is None else inner.mu
    if inner is not None:
        inner.set_mu(mu)
    fx = F(x)
    gfx = GF(x)
    Jx = JG(x)

    # --- least-squares multiplier estimate ---------------------------------
    lam = np.zeros(m)
    if inner is None and m and o.constr_mult_init_max > 0:
        K = np.zeros((n + m, n + m))
        K[:n, :n] = np.eye(n)
        K[:n, n:] = Jx.T
        K[n:, :n] = Jx
        dd = np.where(ineq, -1.0, 0.0)
        dd[free_slack] = -1.0
        K[n:, n:] = np.diag(dd)
        rhs = np.concatenate([-(gfx - zL + zU), np.where(ineq, vL - vU, 0.0)])
        try:
            sol = np.linalg.solve(K, rhs)
            lam_ls = sol[n:]
            if np.max(np.abs(lam_ls), initial=0.0) <= o.constr_mult_init_max:
                lam = lam_ls
        except np.linalg.LinAlgError:
            pass

    tau = max(o.tau_min, 1.0 - mu)
    delta_w_last = 0.0

    def residuals(x, s, lam, zL, zU, vL, vU, gfx, Jx, gx, mu_):
        rd = gfx + Jx.T @ lam - zL + zU
        rd[fixed] = 0.0
        rs = np.where(ineq & ~free_slack, -lam - vL + vU, 0.0)
        c = np.where(ineq, gx - s, gx - np.where(eq, lbg * g_scale, 0.0))
        cl = np.where(hasL, (x - np.where(hasL, xL, 0)) * zL - mu_, 0.0)
        cu = np.where(hasU, (np.where(hasU, xU, 0) - x) * zU - mu_, 0.0)
        csl = np.where(shasL, (s - np.where(shasL, sL, 0)) * vL - mu_, 0.0)
        csu = np.where(shasU, (np.where(shasU, sU, 0) - s) * vU - mu_, 0.0)
        return rd, rs, c, np.concatenate([cl, cu, csl, csu])

    def opt_error(x, s, lam, zL, zU, vL, vU, gfx, Jx, gx, mu_):
        rd, rs, c, comp = residuals(x, s, lam, zL, zU, vL, vU, gfx, Jx, gx, mu_)
        nz = np.sum(hasL) + np.sum(hasU) + np.sum(shasL) + np.sum(shasU)
        zsum = np.sum(np.abs(zL)) + np.sum(np.abs(zU)) + np.sum(np.abs(vL)) + np.sum(np.abs(vU))
        s_d = max(o.s_max, (np.sum(np.abs(lam)) + zsum) / max(1, m + nz)) / o.s_max
        s_c = max(o.s_max, zsum / max(1, nz)) / o.s_max if nz else 1.0
        dual = max(np.max(np.abs(rd), initial=0.0), np.max(np.abs(rs), initial=0.0))
        primal = np.max(np.abs(c), initial=0.0)
        compl = np.max(np.abs(comp), initial=0.0)
        return max(dual / s_d, primal, compl / s_c), dual, primal, compl

    def pd_error(x, s, lam, zL, zU, vL, vU, gfx, Jx, gx, mu_):
        """IPOPT primal_dual_system_error: 1-norms of the dual infeasibility, the
        constraint violation and the mu-complementarity (the common normalisation
        by the number of entries cancels in the soft-restoration ratio)."""
        rd, rs, c, comp = residuals(x, s, lam, zL, zU, vL, vU, gfx, Jx, gx, mu_)
        return float(np.sum(np.abs(rd)) + np.sum(np.abs(rs)) + np.sum(np.abs(c)) + np.sum(np.abs(comp)))

    def theta_of(gx, s):
        c = np.where(ineq, gx - s, gx - np.where(eq, lbg * g_scale, 0.0))
        return float(np.sum(np.abs(c)))

    def phi_of(fx, x, s, mu_):
        val = fx
        val -= mu_ * np.sum(np.log(x[hasL] - xL[hasL]))
        val -= mu_ * np.sum(np.log(xU[hasU] - x[hasU]))
        val -= mu_ * np.sum(np.log(s[shasL] - sL[shasL]))
        val -= mu_ * np.sum(np.log(sU[shasU] - s[shasU]))
        return float(val)

    def unscaled(x, s, lam, zL, zU, vL, vU, gfx, Jx, gx, compl):
        """IPOPT's unscaled_curr_dual_infeasibility (grad_lag_x and grad_lag_s * d_scale,
        divided by obj_scale), unscaled_curr_nlp_constraint_violation (|c| and the violation
        of the relaxed bounds of d - not d - s) and unscaled_curr_complementarity."""
        rd_u = (gfx + Jx.T @ lam - zL + zU) / obj_scale
        rs_u = np.where(ineq & ~free_slack, (-lam - vL + vU) * g_scale, 0.0) / obj_scale
        dual_u = max(np.max(np.abs(rd_u[free]), initial=0.0), np.max(np.abs(rs_u), initial=0.0))
        c_eq = np.where(eq, np.abs(gx - lbg * g_scale), 0.0)
        d_viol = np.where(ineq, np.maximum(0.0, np.maximum(np.where(np.isfinite(sL), sL - gx, 0.0),
                                                           np.where(np.isfinite(sU), gx - sU, 0.0))), 0.0)
        viol_u = np.max((c_eq + d_viol) / g_scale, initial=0.0) if m else 0.0
        return dual_u, viol_u, compl / obj_scale

    n_eq = int(np.sum(eq))
    square = int(np.sum(free)) == n_eq  # IPOPT IsSquareProblem
    acc = dict(curr_f=-1e50, last_f=-1e50, last_it=-1, count=0)

    def current_is_acceptable(err0, dual_u, viol_u, compl_u, fx_, it_):
        """IPOPT OptimalityErrorConvergenceCheck::CurrentIsAcceptable."""
        if it_ != acc["last_it"]:
            acc["last_f"], acc["curr_f"], acc["last_it"] = acc["curr_f"], fx_, it_
        if square:
            return err0 <= o.acceptable_tol and viol_u <= o.acceptable_constr_viol_tol
        return (err0 <= o.acceptable_tol and dual_u <= o.acceptable_dual_inf_tol
                and viol_u <= o.acceptable_constr_viol_tol and compl_u <= o.acceptable_compl_inf_tol
                and abs(acc["curr_f"] - acc["last_f"]) / max(1.0, abs(acc["curr_f"]))
                <= o.acceptable_obj_change_tol)

    theta0 = theta_of(gx, s)
    theta_max = o.theta_max_fact * max(1.0, theta0)
    theta_min = o.theta_min_fact * max(1.0, theta0)
    filt = []
    history = []
    status = "Maximum_Iterations_Exceeded"
    it = 0
    counts = dict(soft=0, resto=0, resto_iters=0, filter_overflows=0, max_filter=0)
    in_soft, soft_count = False, 0
    # IPOPT MonotoneMuUpdate::CalcNewMuAndTau: mu >= min(tol, compl_inf_tol) / (barrier_tol_factor + 1)
    mu_floor = max(min(o.tol, o.compl_inf_tol) / (o.kappa_eps + 1.0), o.mu_min)

    def filter_ok(th, ph):
        return th <= theta_max and not any(th >= a and ph >= b for a, b in filt)

    def augment(theta, phi):
        """IPOPT Filter::AddEntry: the entries the new one dominates are removed (in order),
        then it is appended; a full filter (max_filter) drops its oldest entry."""
        nt, nph = (1 - o.gamma_theta) * theta, phi - o.gamma_phi * theta
        filt[:] = [(a, b) for a, b in filt if not (nt <= a and nph <= b)]
        if len(filt) >= o.max_filter:
            filt.pop(0)
            counts["filter_overflows"] += 1
        filt.append((nt, nph))
        counts["max_filter"] = max(counts["max_filter"], len(filt))

    while True:
        if IT_TRACE is not None:  # diagnostics (scripts/resto_ab.py trace): one row per iteration
            IT_TRACE.append((it, int(inner is not None), mu, fx, counts.get("refine", 0)))
        if inner is not None and inner.check(x, s):
            status = "Resto_Return"
            break
        err0, dual, primal, compl = opt_error(x, s, lam, zL, zU, vL, vU, gfx, Jx, gx, 0.0)
        dual_u, viol_u, compl_u = unscaled(x, s, lam, zL, zU, vL, vU, gfx, Jx, gx, compl)
        if record:
            history.append(dict(iter=it, mu=mu, err=err0, f=fx / obj_scale, x=x.copy()))
        # IPOPT OptimalityErrorConvergenceCheck::CheckConvergence
        if (err0 <= o.tol and viol_u <= o.constr_viol_tol
                and (square or (dual_u <= o.dual_inf_tol and compl_u <= o.compl_inf_tol))):
            status = "Solve_Succeeded"
            break
        if o.acceptable_iter > 0 and current_is_acceptable(err0, dual_u, viol_u, compl_u, fx, it):
            acc["count"] += 1
            if acc["count"] >= o.acceptable_iter:
                status = "Solved_To_Acceptable_Level"
                break
        else:
            acc["count"] = 0
        if it >= o.max_iter:
            break
        # barrier update
        while True:
            err_mu = opt_error(x, s, lam, zL, zU, vL, vU, gfx, Jx, gx, mu)[0]
            if err_mu > o.kappa_eps * mu or mu <= o.mu_min:
                break
            new_mu = max(mu_floor, min(o.kappa_mu * mu, mu ** o.theta_mu))
            if new_mu == mu:  # IPOPT MonotoneMuUpdate: done when mu no longer changes
                break
            mu = new_mu
            tau = max(o.tau_min, 1.0 - mu)
            filt = []
            if inner is not None:  # the restoration objective depends on mu (zeta(mu))
                inner.set_mu(mu)
                fx = F(x)
                gfx = GF(x)
        Hx = H(x, lam)
        # primal-dual matrices
        dxL = np.where(hasL, x - np.where(hasL, xL, 0), 1.0)
        dxU = np.where(hasU, np.where(hasU, xU, 0) - x, 1.0)
        dsL = np.where(shasL, s - np.where(shasL, sL, 0), 1.0)
        dsU = np.where(shasU, np.where(shasU, sU, 0) - s, 1.0)
        Sx = np.where(hasL, zL / dxL, 0) + np.where(hasU, zU / dxU, 0)
        Ss = np.where(shasL, vL / dsL, 0) + np.where(shasU, vU / dsU, 0)
        gphi_x = gfx - np.where(hasL, mu / dxL, 0) + np.where(hasU, mu / dxU, 0)
        gphi_s = -np.where(shasL, mu / dsL, 0) + np.where(shasU, mu / dsU, 0)
        rhs_x = -(gphi_x + Jx.T @ lam)
        rhs_x[fixed] = 0.0
        r_s = np.where(ineq, gphi_s - lam, 0.0)
        c = np.where(ineq, gx - s, gx - np.where(eq, lbg * g_scale, 0.0))

        def factor_solve(dw, dc):
            K = np.zeros((n + m, n + m))
            W = Hx + np.diag(Sx + dw)
            W[fixed, :] = 0.0
            W[:, fixed] = 0.0
            W[fixed, fixed] = 1.0
            K[:n, :n] = W
            K[:n, n:] = Jx.T
            K[n:, :n] = Jx
            Dd = np.where(ineq, 1.0 / (Ss + dw) + dc, dc)
            Dd[free_slack] = 1.0
            K[n:, n:] = -np.diag(Dd)
            rhs_l = -c - np.where(ineq & ~free_slack, r_s / (Ss + dw), 0.0)
            _, Dm, _ = scipy.linalg.ldl(K, lower=True)
            ev = _block_eigs(Dm)
            if DEBUG:
                print("factor dw=%g dc=%g: ev min/max" % (dw, dc), np.sort(np.abs(ev))[:4], np.max(np.abs(ev)), "npos", int(np.sum(ev>0)), "nneg", int(np.sum(ev<0)), "n", n, "m", m)
            npos = int(np.sum(ev > 0))
            nneg = int(np.sum(ev < 0))
            nzero = len(ev) - npos - nneg
            if KKT_HOOK is not None:  # diagnostics: the KKT matrices of an iteration's inertia tests
                KKT_HOOK(it, inner is not None, dw, dc, K, npos, nneg, nzero)
            sol = None
            if nzero == 0:
                rhs = np.concatenate([rhs_x, rhs_l])
                if inner is None:
                    sol = np.linalg.solve(K, rhs)
                else:  # restoration phase: refined on the full system once the inertia is right
                    lu = scipy.linalg.lu_factor(K)
                    sol = scipy.linalg.lu_solve(lu, rhs)
                    last_sys[:] = [K, lu, rhs]
            return npos, nneg, nzero, sol

        last_sys = []

        dw, dc = 0.0, 0.0
        npos, nneg, nzero, sol = factor_solve(dw, dc)
        if not (npos == n and nneg == m and nzero == 0):
            if nzero > 0:
                dc = o.delta_c_bar * mu ** o.kappa_c
            dw = o.delta_w_first if delta_w_last == 0 else max(o.delta_w_min, o.kappa_w_minus * delta_w_last)
            while True:
                npos, nneg, nzero, sol = factor_solve(dw, dc)
                if npos == n and nneg == m and nzero == 0:
                    delta_w_last = dw
                    break
                dw = o.kappa_w_plus_bar * dw if delta_w_last == 0 else o.kappa_w_plus * dw
                if dw > o.delta_w_max:
                    # IPOPT PDPerturbationHandler::PerturbForWrongInertia: with the Hessian shift
                    # alone failing, the constraint block is regularised (as for a singular
                    # matrix) and the shifts run again from the start; failing that too, give up
                    if dc != 0.0:
                        raise RuntimeError("inertia correction failed")
                    dc = o.delta_c_bar * mu ** o.kappa_c
                    dw = o.delta_w_first if delta_w_last == 0 else max(o.delta_w_min, o.kappa_w_minus * delta_w_last)
        if IT_TRACE is not None:
            IT_TRACE.append(("dw", it, int(inner is not None), dw, dc))
        if inner is not None:
            # IPOPT PDFullSpaceSolver: iterative refinement of the step on the full system (here
            # the restoration NLP's, p and n explicit)
            sol = _refine(*last_sys, sol, o, counts)
        dx = sol[:n]
        dlam = sol[n:]
        dx[fixed] = 0.0
        ds = np.where(ineq & ~free_slack, (dlam - r_s) / (Ss + dw), 0.0)
        dzL = np.where(hasL, mu / dxL - zL - (zL / dxL) * dx, 0.0)
        dzU = np.where(hasU, mu / dxU - zU + (zU / dxU) * dx, 0.0)
        dvL = np.where(shasL, mu / dsL - vL - (vL / dsL) * ds, 0.0)
        dvU = np.where(shasU, mu / dsU - vU + (vU / dsU) * ds, 0.0)

        def ftb(v, dv, mask):
            a = 1.0
            sel = mask & (dv < 0)
            if np.any(sel):
                a = min(a, float(np.min(-tau * v[sel] / dv[sel])))
            return a

        a_max = min(ftb(dxL, dx, hasL), ftb(dxU, -dx, hasU), ftb(dsL, ds, shasL), ftb(dsU, -ds, shasU))
        a_z = min(ftb(zL, dzL, hasL), ftb(zU, dzU, hasU), ftb(vL, dvL, shasL), ftb(vU, dvU, shasU))

        theta = theta_of(gx, s)
        phi = phi_of(fx, x, s, mu)
        gphi_d = float(gphi_x @ dx + gphi_s @ ds)
        if gphi_d < 0 and theta <= theta_min:
            a_min = o.alpha_min_frac * min(o.gamma_theta, o.gamma_phi * theta / (-gphi_d),
                                           o.delta * theta ** o.s_theta / (-gphi_d) ** o.s_phi)
        elif gphi_d < 0:
            a_min = o.alpha_min_frac * min(o.gamma_theta, o.gamma_phi * theta / (-gphi_d))
        else:
            a_min = o.alpha_min_frac * o.gamma_theta

        def soft_step():
            """IPOPT BacktrackingLineSearch::TrySoftRestoStep: the full fraction-to-the-boundary
            step, the same step size for primal and dual variables; accepted if the original
            filter criterion holds at alpha = 0 (h-type) or the primal-dual system error drops
            by soft_resto_pderror_reduction_factor.  Returns (accepted, original, trial)."""
            al = min(a_max, a_z)
            xt, st_, lt = x + al * dx, s + al * ds, lam + al * dlam
            zt = (zL + al * dzL, zU + al * dzU, vL + al * dvL, vU + al * dvU)
            gxt, fxt = G(xt), F(xt)
            th_t, ph_t = theta_of(gxt, st_), phi_of(fxt, xt, st_, mu)
            trial = (xt, st_, lt, zt, gxt, fxt, al)
            if not (np.isfinite(th_t) and np.isfinite(ph_t)):
                return False, False, trial
            if filter_ok(th_t, ph_t) and (th_t <= (1 - o.gamma_theta) * theta or ph_t <= phi - o.gamma_phi * theta):
                return True, True, trial
            gft, Jt = GF(xt), JG(xt)
            cur = pd_error(x, s, lam, zL, zU, vL, vU, gfx, Jx, gx, mu)
            new = pd_error(xt, st_, lt, *zt, gft, Jt, gxt, mu)
            return bool(new <= o.soft_resto_pderror_reduction_factor * cur), False, trial

        accepted, ftype, goto_resto, soft = False, False, False, None
        if in_soft:
            soft_count += 1
            ok, orig, trial = soft_step() if soft_count <= o.max_soft_resto_iters else (False, False, None)
            if ok:
                soft = (orig, trial)
                if orig:
                    in_soft, soft_count = False, 0
            else:
                goto_resto = True
        else:
            alpha = a_max
            if LS_TRACE is not None:  # diagnostics (scripts/resto_diag.py): the last line search
                LS_TRACE.clear()
                LS_TRACE.append(("head", theta, phi, gphi_d, a_min, theta_min, theta_max, mu, list(filt), dw, dc))
            while True:
                xt = x + alpha * dx
                st = s + alpha * ds
                gxt = G(xt)
                fxt = F(xt)
                th_t = theta_of(gxt, st)
                ph_t = phi_of(fxt, xt, st, mu)
                ok = np.isfinite(th_t) and np.isfinite(ph_t) and filter_ok(th_t, ph_t)
                okf = ok
                if ok:
                    switching = gphi_d < 0 and alpha * (-gphi_d) ** o.s_phi > o.delta * theta ** o.s_theta
                    if theta <= theta_min and switching:
                        ok = ph_t <= phi + o.eta_phi * alpha * gphi_d
                        ftype = True
                    else:
                        ok = th_t <= (1 - o.gamma_theta) * theta or ph_t <= phi - o.gamma_phi * theta
                        ftype = False
                if LS_TRACE is not None:
                    LS_TRACE.append((alpha, th_t, ph_t, okf, ok, ftype))
                if ok:
                    accepted = True
                    break
                alpha *= 0.5
                if alpha < a_min:
                    break
            if IT_TRACE is not None and inner is not None:
                IT_TRACE.append(("ls", it, int(accepted), mu, theta, phi, gphi_d, a_min, a_max, alpha, theta_min,
                                 theta_max))
            if not accepted and inner is not None:
                # no restoration inside the restoration phase (IPOPT: "Restoration phase in
                # the restoration phase failed")
                status = "Restoration_Failed"
                break
            if not accepted:
                ok, orig, trial = soft_step()
                if ok:
                    soft = (orig, trial)
                    counts["soft"] += 1
                    if not orig:
                        in_soft, soft_count = True, 0
                else:
                    goto_resto = True
        if goto_resto:
            if current_is_acceptable(err0, dual_u, viol_u, compl_u, fx, it):
                # IPOPT BacktrackingLineSearch: "Restoration phase called at acceptable point"
                status = "Solved_To_Acceptable_Level"
                break
            if inner is not None:
                status = "Restoration_Failed"
                break
            # ---- feasibility restoration phase (MinC_1NrmRestorationPhase) ----
            counts["resto"] += 1
            augment(theta, phi)                     # FilterLSAcceptor::PrepareRestoPhaseStart
            in_soft, soft_count = False, 0
            c_now = np.where(ineq, gx - s, gx - np.where(eq, lbg * g_scale, 0.0))
            mu_r = max(mu, float(np.max(np.abs(c_now), initial=0.0)))
            rho = o.resto_penalty_parameter
            # p, n solving the complementarity of the resto problem at its start
            # (Wächter & Biegler 2006, eq. (33))
            a_ = (mu_r - rho * c_now) / (2.0 * rho)
            n_r = a_ + np.sqrt(a_ ** 2 + mu_r * c_now / (2.0 * rho))
            p_r = c_now + n_r
            theta_start, mu_orig = theta, mu
            rn = _RestoNLP(F, JG, G, lambda xx, ll: H(xx, ll, 0.0), n, m, x.copy(), fixed, rho,
                           o.resto_proximity_weight)
            sub = rn.functions()
            lbx_r = np.concatenate([np.where(fixed, x, xL), np.zeros(2 * m)])
            ubx_r = np.concatenate([np.where(fixed, x, xU), np.full(2 * m, np.inf)])
            lbg_r = np.where(eq, lbg * g_scale, sL)
            ubg_r = np.where(eq, lbg * g_scale, sU)
            x_r0 = np.concatenate([x, p_r, n_r])

            def check(xr, sr, _th0=theta_start, _mu=mu_orig):
                """RestoConvergenceCheck: back to the original problem when the original
                constraint violation dropped by required_infeasibility_reduction and the
                point is acceptable to the original filter."""
                xo = xr[:n]
                so = np.where(ineq, sr, s)
                gxo = G(xo)
                th_o = theta_of(gxo, so)
                if not th_o <= o.required_infeasibility_reduction * _th0:
                    return False
                return filter_ok(th_o, phi_of(F(xo), xo, so, _mu))

            rho_cap = lambda z_: np.minimum(z_, rho)  # noqa: E731
            inner_r = _Inner(zL=np.concatenate([rho_cap(zL), mu_r / p_r, mu_r / n_r]),
                             zU=np.concatenate([rho_cap(zU), np.zeros(2 * m)]),
                             vL=rho_cap(vL), vU=rho_cap(vU), mu=mu_r, check=check, set_mu=rn.set_mu)
            o_r = dataclasses.replace(o, max_iter=o.max_iter - it)
            r = _solve(sub, x_r0, lbx_r, ubx_r, lbg_r, ubg_r, o_r, False, inner=inner_r)
            counts["resto_iters"] += r.iterations
            counts["filter_overflows"] += r.filter_overflows
            counts["max_filter"] = max(counts["max_filter"], r.max_filter_size)
            counts["refine"] = counts.get("refine", 0) + r.refine_steps
            it += r.iterations
            if r.status != "Resto_Return":
                status = {"Solve_Succeeded": "Infeasible_Problem_Detected",
                          "Solved_To_Acceptable_Level": "Infeasible_Problem_Detected"}.get(r.status, r.status)
                x = r.x[:n]
                s = np.where(ineq, r.s, s)
                gx, fx = G(x), F(x)
                lam = np.zeros(m)
                break
            # return to the original problem: bound multipliers by one Newton step for
            # the complementarity over the whole primal change, fraction to the boundary,
            # reset to 1 when too large; constraint multipliers reset to zero
            # (bound_mult_reset_threshold, constr_mult_reset_threshold = 0)
            xn = r.x[:n]
            sn = np.where(ineq, r.s, s)
            slack_new = (np.where(hasL, xn - np.where(hasL, xL, 0), 1.0), np.where(hasU, np.where(hasU, xU, 0) - xn, 1.0),
                         np.where(shasL, sn - np.where(shasL, sL, 0), 1.0), np.where(shasU, np.where(shasU, sU, 0) - sn, 1.0))
            slack_old = (dxL, dxU, dsL, dsU)
            zs = (zL, zU, vL, vU)
            masks = (hasL, hasU, shasL, shasU)
            dz = [np.where(mk, (mu - z_ * sn_) / so_, 0.0) for z_, sn_, so_, mk in zip(zs, slack_new, slack_old, masks)]
            a_d = min(ftb(z_, d_, mk) for z_, d_, mk in zip(zs, dz, masks))
            zL, zU, vL, vU = (z_ + a_d * d_ for z_, d_ in zip(zs, dz))
            if max(np.max(np.abs(v_), initial=0.0) for v_ in (zL, zU, vL, vU)) > o.bound_mult_reset_threshold:
                zL, zU = np.where(hasL, 1.0, 0.0), np.where(hasU, 1.0, 0.0)
                vL, vU = np.where(shasL, 1.0, 0.0), np.where(shasU, 1.0, 0.0)
            x, s = xn, sn
            lam = np.zeros(m)
            fx, gx = F(x), G(x)
            gfx, Jx = GF(x), JG(x)
            continue
        if soft is not None:
            orig, (xt, st, lt, (zLt, zUt, vLt, vUt), gxt, fxt, alpha) = soft
            if orig:
                augment(theta, phi)   # accepted by the original (h-type) criterion
            x, s, lam = xt, st, lt
            zL, zU, vL, vU = zLt, zUt, vLt, vUt
        else:
            if not ftype:
                augment(theta, phi)
            x, s = xt, st
            lam = lam + alpha * dlam
            zL = zL + a_z * dzL
            zU = zU + a_z * dzU
            vL = vL + a_z * dvL
            vU = vU + a_z * dvU
        # safeguard (kappa_sigma)
        dxL = np.where(hasL, x - np.where(hasL, xL, 0), 1.0)
        dxU = np.where(hasU, np.where(hasU, xU, 0) - x, 1.0)
        dsL = np.where(shasL, s - np.where(shasL, sL, 0), 1.0)
        dsU = np.where(shasU, np.where(shasU, sU, 0) - s, 1.0)
        zL = np.where(hasL, np.maximum(np.minimum(zL, o.kappa_sigma * mu / dxL), mu / (o.kappa_sigma * dxL)), 0)
        zU = np.where(hasU, np.maximum(np.minimum(zU, o.kappa_sigma * mu / dxU), mu / (o.kappa_sigma * dxU)), 0)
        vL = np.where(shasL, np.maximum(np.minimum(vL, o.kappa_sigma * mu / dsL), mu / (o.kappa_sigma * dsL)), 0)
        vU = np.where(shasU, np.maximum(np.minimum(vU, o.kappa_sigma * mu / dsU), mu / (o.kappa_sigma * dsU)), 0)
        fx, gx = fxt, gxt
        gfx = GF(x)
        Jx = JG(x)
        it += 1

    lam_g = lam * g_scale / obj_scale
    lam_x = (zU - zL) / obj_scale
    return IPMResult(x=x, lam_g=lam_g, lam_x=lam_x, f=fx / obj_scale, iterations=it,
                     status=status, success=status in ("Solve_Succeeded", "Solved_To_Acceptable_Level"),
                     history=history, s=s, n_soft_resto=counts["soft"], n_resto=counts["resto"],
                     resto_iterations=counts["resto_iters"], filter_overflows=counts["filter_overflows"],
                     max_filter_size=counts["max_filter"], refine_steps=counts.get("refine", 0))


def _refine(K, lu, rhs, sol, o: IPMOptions, counts: dict):
    """IPOPT PDFullSpaceSolver::Solve's iterative refinement on the full system K sol = rhs:
    at least ``min_refinement_steps`` corrections, more while the residual ratio
    ||r||_inf / (min(||sol||_inf, 1e6 ||rhs||_inf) + ||rhs||_inf) exceeds
    ``residual_ratio_max``, at most ``max_refinement_steps``, stopping early when a step does
    not improve the ratio (``residual_improvement_factor``)."""

    def ratio(res, x):
        nr, nx = np.max(np.abs(rhs), initial=0.0), np.max(np.abs(x), initial=0.0)
        return np.max(np.abs(res), initial=0.0) / (min(nx, 1e6 * nr) + nr) if nr + nx > 0 else 0.0

    res = rhs - K @ sol
    rr = ratio(res, sol)
    steps = 0
    while steps < o.min_refinement_steps or rr > o.residual_ratio_max:
        sol = sol + scipy.linalg.lu_solve(lu, res)
        res = rhs - K @ sol
        old, rr = rr, ratio(res, sol)
        steps += 1
        if rr > o.residual_ratio_max and steps > o.min_refinement_steps and (
                steps > o.max_refinement_steps or rr > o.residual_improvement_factor * old):
            break
    counts["refine"] = counts.get("refine", 0) + steps
    return sol


def _block_eigs(D: np.ndarray) -> np.ndarray:
    """Eigenvalues of the 1x1/2x2 block-diagonal D of scipy's ldl."""
    n = D.shape[0]
    ev = []
    i = 0
    while i < n:
        if i + 1 < n and D[i + 1, i] != 0.0:
            ev.extend(np.linalg.eigvalsh(D[i:i + 2, i:i + 2]))
            i += 2
        else:
            ev.append(D[i, i])
            i += 1
    ev = np.asarray(ev)
    # a pivot is "zero" only when it is numerically null in absolute terms: the
    # barrier terms make the matrix norm grow without bound near active bounds,
    # so a threshold relative to it would misclassify legitimate -delta_c pivots
    ev[np.abs(ev) <= ZERO_PIVOT] = 0.0
    return ev
