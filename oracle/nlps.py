"""ORACLE (test infrastructure only) — hand restatement of the reference NLPs.

Each builder writes out the reference transcription for one benchmark
configuration with explicit variable / parameter / constraint ordering,
independent of the product's tracer and transcriber:

* ``one_room``   — backend ``casadi`` direct collocation
  (`optimization_backends/casadi_/full.py:36-98`, `basic.py:251-392`) on the
  model of `examples/one_room_mpc/physical/simple_mpc.py:95-138` (C1, C3).
* ``admm_room`` / ``admm_ahu`` — backend ``casadi_admm`` collocation
  (`casadi_/admm.py:119-195`, ADMM terms :90-116) on
  `examples/4_Room_ADMM_Coordinator/models/{room,rlt}_model.py` (C2).
* ``exchange_room`` / ``exchange_supply`` — backend ``casadi_admm`` multiple
  shooting with Euler (`casadi_/admm.py:198-310`) on
  `examples/exchange_admm/models/{room,rlt}_model.py` (C4).
* ``fixture_mpc`` — backend ``casadi`` collocation (defaults: Legendre d=3) on the
  reference test-suite model `tests/fixtures/casadi_test_model.py:13-47` with the MPC
  module config of `tests/test_mpc.py:121-146`.
* ``cubic_room`` — backend ``casadi`` collocation (Legendre d=2) on a zone with an algebraic
  quantity on a cubic characteristic (the restoration-phase case, ``models/examples.CubicRoom``).
* ``room_nn`` — backend ``casadi_admm_nn`` NARX multiple shooting
  (`casadi_/casadi_admm_ml.py:247-397`) on
  `examples/three_zone_datadriven_admm/models/Room_model.py` with two ANNs (C5).

Derivatives come from torch fp64 autograd.  Initial guesses follow
`core/discretization.py:212-245` (cold start).
"""

from __future__ import annotations

import dataclasses
from typing import Callable, Dict, List

import numpy as np
import torch

from oracle.ipm import NLPFunctions

torch.set_default_dtype(torch.float64)


def collocation(d: int, method: str = "legendre"):
    if method == "legendre":
        r, _ = np.polynomial.legendre.leggauss(d)
        roots = np.sort((r + 1) / 2)
    else:
        c = np.zeros(d + 1)
        c[d], c[d - 1] = 1.0, -1.0
        r = np.sort(np.real(np.polynomial.legendre.legroots(c)))
        r[-1] = 1.0
        roots = (r + 1) / 2
    tau = np.concatenate([[0.0], roots])
    C = np.zeros((d + 1, d + 1))
    D = np.zeros(d + 1)
    B = np.zeros(d + 1)
    for j in range(d + 1):
        # Lagrange basis polynomial l_j on tau
        coeffs = np.array([1.0])
        for r_ in range(d + 1):
            if r_ != j:
                coeffs = np.convolve(coeffs, np.array([1.0, -tau[r_]]) / (tau[j] - tau[r_]))
        D[j] = np.polyval(coeffs, 1.0)
        der = np.polyder(coeffs)
        C[j] = [np.polyval(der, t) for t in tau]
        B[j] = np.polyval(np.polyint(coeffs), 1.0)
    return tau, B, C, D


@dataclasses.dataclass
class OracleProblem:
    name: str
    n: int
    m: int
    np_: int
    f: Callable  # torch (w, p) -> scalar
    g: Callable  # torch (w, p) -> (m,)
    lbg: Callable  # numpy p -> (m,)
    ubg: Callable
    w_names: List[str]

    def functions(self, p: np.ndarray) -> NLPFunctions:
        pt = torch.as_tensor(p)

        def f(w):
            return float(self.f(torch.as_tensor(w), pt))

        def grad(w):
            wt = torch.as_tensor(w).clone().requires_grad_(True)
            return torch.autograd.grad(self.f(wt, pt), wt)[0].numpy()

        def g(w):
            return self.g(torch.as_tensor(w), pt).numpy()

        def jac(w):
            return torch.func.jacrev(lambda ww: self.g(ww, pt))(torch.as_tensor(w)).numpy().reshape(self.m, self.n)

        def hess(w, sigma, lam):
            lt = torch.as_tensor(lam)
            L = lambda ww: sigma * self.f(ww, pt) + (lt * self.g(ww, pt)).sum()  # noqa: E731
            return torch.func.hessian(L)(torch.as_tensor(w)).numpy()

        return NLPFunctions(n=self.n, m=self.m, f=f, grad_f=grad, g=g, jac_g=jac, hess_l=hess)


# ---------------------------------------------------------------------------
# C1 / C3: one room, backend "casadi", collocation
# ---------------------------------------------------------------------------

def one_room(N=15, ts=300.0, d=2, method="legendre", delta_u=False) -> OracleProblem:
    """``delta_u``: the change-penalty variant of
    `examples/one_room_mpc/physical/with_change_control_penalty.py` (extra model
    parameter r_delta_mDot; cost += r_delta_mDot**2 (u_k - u_{k-1})**2 with
    u_{-1} = u_prev, `casadi_/full.py:58-70`, `core/delta_u.py:13-26`)."""
    tau, B, C, D = collocation(d, method)
    nb = 1 + 3 * d + 1          # u, (T, T_slack, T_out) per point, T_end
    n = 1 + N * nb
    m = N * (1 + 3 * d)         # cont, (col, path, out) per point
    npg = 1 + 1 + 4 + int(delta_u)  # T0, u_prev, (cp, C, s_T, r_mDot[, r_delta_mDot])
    nps = 3 * d                 # (T_in, load, T_upper) per point
    names = ["T@0"]
    for k in range(N):
        names.append(f"mDot@{k}")
        for j in range(d):
            names += [f"T@{k},{j}", f"T_slack@{k},{j}", f"T_out@{k},{j}"]
        names.append(f"T@{k + 1}")

    def unpack(w, p):
        cp, Cz, s_T, r = p[2], p[3], p[4], p[5]
        return cp, Cz, s_T, r

    def f(w, p):
        cp, Cz, s_T, r = unpack(w, p)
        tot = w.new_zeros(())
        for k in range(N):
            o = 1 + k * nb
            u = w[o]
            if delta_u:
                u_prev = p[1] if k == 0 else w[o - nb]
                tot = tot + p[6] ** 2 * (u - u_prev) ** 2
            for j in range(d):
                zs = w[o + 1 + 3 * j + 1]
                tot = tot + B[j + 1] * (r * u + s_T * zs ** 2) * ts
        return tot

    def g(w, p):
        cp, Cz, s_T, r = unpack(w, p)
        out = []
        xk = w[0]
        for k in range(N):
            o = 1 + k * nb
            u = w[o]
            Tj = [w[o + 1 + 3 * j] for j in range(d)]
            x_end = w[o + nb - 1]
            out.append(x_end - (D[0] * xk + sum(D[j + 1] * Tj[j] for j in range(d))))
            for j in range(d):
                ps = npg + k * nps + 3 * j
                T_in, load = p[ps], p[ps + 1]
                ode = cp * u / Cz * (T_in - Tj[j]) + load / Cz
                xp = C[0, j + 1] * xk + sum(C[r_ + 1, j + 1] * Tj[r_] for r_ in range(d))
                out.append(ts * ode - xp)
                out.append(Tj[j] + w[o + 1 + 3 * j + 1])
                out.append(w[o + 1 + 3 * j + 2] - Tj[j])
            xk = x_end
        return torch.stack(out)

    def lbg(p):
        return np.zeros(m)

    def ubg(p):
        u = np.zeros(m)
        for k in range(N):
            for j in range(d):
                u[k * (1 + 3 * d) + 1 + 3 * j + 1] = p[npg + k * nps + 3 * j + 2]
        return u

    return OracleProblem("one_room", n, m, npg + N * nps, f, g, lbg, ubg, names)


def one_room_inputs(prob: OracleProblem, N=15, d=2, T0=298.16, load=150.0, T_in=290.15,
                    T_upper=295.15, s_T=0.001, r_mDot=0.01, u_prev=0.02, cp=1000.0, C=100000.0,
                    T_lb=288.15, T_ub=303.15, u_lb=0.0, u_ub=0.05, r_delta_mDot=None):
    p = [T0, u_prev, cp, C, s_T, r_mDot] + ([] if r_delta_mDot is None else [r_delta_mDot])
    for k in range(N):
        for j in range(d):
            p += [T_in, load, T_upper]
    p = np.array(p, float)
    n = prob.n
    lbw = np.full(n, -np.inf)
    ubw = np.full(n, np.inf)
    w0 = np.zeros(n)
    for i, name in enumerate(prob.w_names):
        base = name.split("@")[0]
        if base == "T":
            lbw[i], ubw[i], w0[i] = T_lb, T_ub, T0
        elif base == "mDot":
            lbw[i], ubw[i], w0[i] = u_lb, u_ub, 0.5 * (u_lb + u_ub)
    lbw[0] = ubw[0] = w0[0] = T0
    return p, lbw, ubw, w0


# ---------------------------------------------------------------------------
# C2: 4 rooms + air handler, backend "casadi_admm", collocation (d=3)
# ---------------------------------------------------------------------------

def admm_room(N=10, ts=60.0, d=3) -> OracleProblem:
    tau, B, C, D = collocation(d)
    nb = 2 * d + 1               # (T, mDot) per point, T_end
    n = 1 + N * nb
    m = N * (1 + 2 * d)          # cont, (col, path) per point
    npg = 1 + 4 + 1              # T0, (cp, cZ, q_T, q_mDot), rho  [u_prev is empty]
    nps = 6 * d                  # (zbar, lam, d, T_set, T_upper, T_in) per point
    names = ["T@0"]
    for k in range(N):
        for j in range(d):
            names += [f"T@{k},{j}", f"mDot@{k},{j}"]
        names.append(f"T@{k + 1}")

    def f(w, p):
        cp, cZ, qT, qm, rho = p[1], p[2], p[3], p[4], p[5]
        tot = w.new_zeros(())
        for k in range(N):
            o = 1 + k * nb
            for j in range(d):
                T, u = w[o + 2 * j], w[o + 2 * j + 1]
                ps = npg + k * nps + 6 * j
                zbar, lam, Tset = p[ps], p[ps + 1], p[ps + 3]
                cost = (0.0001 * qT * (T - Tset) ** 2 + 0.0001 * qm * (1 / 0.167) ** 2 * u ** 2
                        + lam * u + rho / 2 * (zbar - u) ** 2)
                tot = tot + B[j + 1] * cost * ts
        return tot

    def g(w, p):
        cp, cZ = p[1], p[2]
        out = []
        xk = w[0]
        for k in range(N):
            o = 1 + k * nb
            Tj = [w[o + 2 * j] for j in range(d)]
            x_end = w[o + nb - 1]
            out.append(x_end - (D[0] * xk + sum(D[j + 1] * Tj[j] for j in range(d))))
            for j in range(d):
                ps = npg + k * nps + 6 * j
                dist, T_in = p[ps + 2], p[ps + 5]
                u = w[o + 2 * j + 1]
                ode = cp * u / cZ * (T_in - Tj[j]) + dist / cZ
                xp = C[0, j + 1] * xk + sum(C[r + 1, j + 1] * Tj[r] for r in range(d))
                out.append(ts * ode - xp)
                out.append(Tj[j])
            xk = x_end
        return torch.stack(out)

    def ubg(p):
        u = np.zeros(m)
        for k in range(N):
            for j in range(d):
                u[k * (1 + 2 * d) + 1 + 2 * j + 1] = p[npg + k * nps + 6 * j + 4]
        return u

    return OracleProblem("admm_room", n, m, npg + N * nps, f, g, lambda p: np.zeros(m), ubg, names)


def admm_room_inputs(prob, N=10, d=3, T0=296.0, dist=150.0, T_set=296.0, T_upper=303.15, T_in=290.15,
                     rho=0.4, zbar=None, lam=None, cp=1000.0, cZ=60000.0, qT=1.0, qm=1.0,
                     T_lb=288.15, T_ub=303.15, u_lb=0.0, u_ub=0.05, guess=None):
    npts = N * d
    zbar = np.full(npts, 0.02) if zbar is None else np.asarray(zbar, float)
    lam = np.zeros(npts) if lam is None else np.asarray(lam, float)
    p = [T0, cp, cZ, qT, qm, rho]
    for k in range(N):
        for j in range(d):
            i = k * d + j
            p += [zbar[i], lam[i], dist, T_set, T_upper, T_in]
    p = np.array(p, float)
    lbw = np.zeros(prob.n)
    ubw = np.zeros(prob.n)
    w0 = np.zeros(prob.n)
    for i, name in enumerate(prob.w_names):
        if name.startswith("T@"):
            lbw[i], ubw[i], w0[i] = T_lb, T_ub, T0
        else:
            lbw[i], ubw[i], w0[i] = u_lb, u_ub, 0.5 * (u_lb + u_ub)
    lbw[0] = ubw[0] = w0[0] = T0
    if guess is not None:
        w0 = np.array(guess, float)
    return p, lbw, ubw, w0


def admm_ahu(N=10, ts=60.0, d=3, rooms=4) -> OracleProblem:
    tau, B, C, D = collocation(d)
    nb = rooms + rooms * d       # controls, couplings per point
    n = N * nb
    m = N * d * (1 + rooms)      # (sum constraint, output eqs) per point
    npg = rooms + 1 + 1          # u_prev (4 controls), mDot_max, rho  [no states]
    nps = 2 * rooms * d          # (zbar_i..., lam_i...) per point
    names = []
    for k in range(N):
        names += [f"mDot_{i + 1}@{k}" for i in range(rooms)]
        for j in range(d):
            names += [f"mDot_out_{i + 1}@{k},{j}" for i in range(rooms)]

    def f(w, p):
        rho = p[rooms + 1]
        tot = w.new_zeros(())
        for k in range(N):
            o = k * nb
            for j in range(d):
                ps = npg + k * nps + 2 * rooms * j
                cost = w.new_zeros(())
                for i in range(rooms):
                    y = w[o + rooms + rooms * j + i]
                    cost = cost + p[ps + rooms + i] * y + rho / 2 * (p[ps + i] - y) ** 2
                tot = tot + B[j + 1] * cost * ts
        return tot

    def g(w, p):
        out = []
        for k in range(N):
            o = k * nb
            u = [w[o + i] for i in range(rooms)]
            for j in range(d):
                out.append(sum(u))
                for i in range(rooms):
                    out.append(w[o + rooms + rooms * j + i] - 1 * u[i])
        return torch.stack(out)

    def ubg(p):
        u = np.zeros(m)
        u[0::1 + rooms] = p[rooms]
        return u

    return OracleProblem("admm_ahu", n, m, npg + N * nps, f, g, lambda p: np.zeros(m), ubg, names)


def admm_ahu_inputs(prob, N=10, d=3, rooms=4, mDot_max=0.1, rho=0.4, zbar=None, lam=None,
                    u_lb=0.0, u_ub=0.075):
    npts = N * d
    zbar = np.full((rooms, npts), 0.01) if zbar is None else np.asarray(zbar, float)
    lam = np.zeros((rooms, npts)) if lam is None else np.asarray(lam, float)
    p = [0.01] * rooms + [mDot_max, rho]   # u_prev = control values (rlt_admm.json)
    for k in range(N):
        for j in range(d):
            i = k * d + j
            p += list(zbar[:, i]) + list(lam[:, i])
    p = np.array(p, float)
    lbw = np.full(prob.n, -np.inf)
    ubw = np.full(prob.n, np.inf)
    w0 = np.zeros(prob.n)
    for i, name in enumerate(prob.w_names):
        if "_out_" not in name:
            lbw[i], ubw[i], w0[i] = u_lb, u_ub, 0.5 * (u_lb + u_ub)
    return p, lbw, ubw, w0


# ---------------------------------------------------------------------------
# C4: exchange ADMM, backend "casadi_admm", multiple shooting + Euler
# ---------------------------------------------------------------------------

def _rk4_step(fun, x, ts, steps=20):
    """Fixed-step RK4 over ``steps`` sub-intervals (CasADi "rk" integrator plugin,
    default ``number_of_finite_elements`` = 20; `casadi_/basic.py:450-476`)."""
    h = ts / steps
    for _ in range(steps):
        k1 = fun(x)
        k2 = fun(x + h / 2 * k1)
        k3 = fun(x + h / 2 * k2)
        k4 = fun(x + h * k3)
        x = x + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
    return x


def exchange_room(N=10, ts=120.0, integrator="euler") -> OracleProblem:
    nb = 3                       # mDot, mDot_out, T_end
    n = 1 + N * nb
    m = N * 2                    # cont, output eq
    npg = 1 + 1 + 4 + 4 + 1      # T0, u_prev, params, params (again), rho
    nps = 6                      # d, T_set, T_upper, T_in, exchange diff, exchange lambda
    names = ["T@0"]
    for k in range(N):
        names += [f"mDot@{k}", f"mDot_out@{k}", f"T@{k + 1}"]

    def pars(p):
        return p[6], p[7], p[8], p[9], p[10]  # second parameter copy + rho

    def f(w, p):
        cp, cZ, qT, qm, rho = pars(p)
        tot = w.new_zeros(())
        for k in range(N):
            o = 1 + k * nb
            T = w[o - 1] if k == 0 else w[o - 1]
            u, y = w[o], w[o + 1]
            ps = npg + k * nps
            Tset, diff, lam = p[ps + 1], p[ps + 4], p[ps + 5]
            cost = qT * (T - Tset) ** 2 + qm * (1 / 0.167) ** 2 * u ** 2 + lam * y + rho / 2 * (diff - y) ** 2
            tot = tot + cost * ts
        return tot

    def g(w, p):
        cp, cZ, qT, qm, rho = pars(p)
        out = []
        for k in range(N):
            o = 1 + k * nb
            T = w[o - 1]
            u, y, T1 = w[o], w[o + 1], w[o + 2]
            ps = npg + k * nps
            dist, T_in = p[ps], p[ps + 3]
            fun = lambda x: cp * u / cZ * (T_in - x) + dist / cZ  # noqa: E731
            x_end = T + fun(T) * ts if integrator == "euler" else _rk4_step(fun, T, ts)
            out.append(T1 - x_end)
            out.append(y - u)
        return torch.stack(out)

    return OracleProblem("exchange_room", n, m, npg + N * nps, f, g,
                         lambda p: np.zeros(m), lambda p: np.zeros(m), names)


def exchange_room_inputs(prob, N=10, T0=296.0, dist=150.0, T_set=296.0, T_upper=296.15, T_in=290.15,
                         rho=1e4, diff=None, lam=None, u_prev=0.02, cp=1000.0, cZ=60000.0,
                         qT=1.0, qm=0.0, T_lb=288.15, T_ub=303.15, u_lb=0.0, u_ub=0.05,
                         y_lb=0.0, y_ub=0.05):
    diff = np.zeros(N) if diff is None else np.asarray(diff, float)
    lam = np.zeros(N) if lam is None else np.asarray(lam, float)
    p = [T0, u_prev, cp, cZ, qT, qm, cp, cZ, qT, qm, rho]
    for k in range(N):
        p += [dist, T_set, T_upper, T_in, diff[k], lam[k]]
    p = np.array(p, float)
    lbw = np.zeros(prob.n)
    ubw = np.zeros(prob.n)
    w0 = np.zeros(prob.n)
    for i, name in enumerate(prob.w_names):
        base = name.split("@")[0]
        if base == "T":
            lbw[i], ubw[i], w0[i] = T_lb, T_ub, T0
        elif base == "mDot":
            lbw[i], ubw[i], w0[i] = u_lb, u_ub, 0.5 * (u_lb + u_ub)
        else:
            lbw[i], ubw[i], w0[i] = y_lb, y_ub, 0.5 * (y_lb + y_ub)
    lbw[0] = ubw[0] = w0[0] = T0
    return p, lbw, ubw, w0


def exchange_supply(N=10, ts=120.0) -> OracleProblem:
    n = 2 * N
    m = N
    npg = 1 + 1 + 1 + 1          # u_prev, penalty, penalty (again), rho   [no states]
    nps = 2                      # exchange diff, exchange lambda
    names = []
    for k in range(N):
        names += [f"mDot@{k}", f"mDot_out@{k}"]

    def f(w, p):
        pen, rho = p[2], p[3]
        tot = w.new_zeros(())
        for k in range(N):
            u, y = w[2 * k], w[2 * k + 1]
            diff, lam = p[npg + k * nps], p[npg + k * nps + 1]
            tot = tot + (pen * u + lam * y + rho / 2 * (diff - y) ** 2) * ts
        return tot

    def g(w, p):
        return torch.stack([w[2 * k + 1] - (-w[2 * k]) for k in range(N)])

    return OracleProblem("exchange_supply", n, m, npg + N * nps, f, g,
                         lambda p: np.zeros(m), lambda p: np.zeros(m), names)


def exchange_supply_inputs(prob, N=10, penalty=0.1, rho=1e4, diff=None, lam=None, u_prev=0.01,
                           u_lb=0.0, u_ub=0.1, y_lb=-0.1, y_ub=0.0):
    diff = np.zeros(N) if diff is None else np.asarray(diff, float)
    lam = np.zeros(N) if lam is None else np.asarray(lam, float)
    p = [u_prev, penalty, penalty, rho]
    for k in range(N):
        p += [diff[k], lam[k]]
    p = np.array(p, float)
    lbw = np.zeros(prob.n)
    ubw = np.zeros(prob.n)
    w0 = np.zeros(prob.n)
    for k in range(N):
        lbw[2 * k], ubw[2 * k], w0[2 * k] = u_lb, u_ub, 0.5 * (u_lb + u_ub)
        lbw[2 * k + 1], ubw[2 * k + 1], w0[2 * k + 1] = y_lb, y_ub, 0.5 * (y_lb + y_ub)
    return p, lbw, ubw, w0


# ---------------------------------------------------------------------------
# C5: three-zone NARX room, backend "casadi_admm_nn", multiple shooting
# ---------------------------------------------------------------------------

def _ann_torch(layers):
    """Sequential forward of a BatchNormalization -> Dense(sigmoid) -> Dense(linear)
    network given as [(kind, arrays)] (`models/casadi_predictor.py:306-376`)."""
    def fwd(x):
        for kind, arrs in layers:
            if kind == "bn":
                gamma, beta, mean, var, eps = arrs
                x = (x - torch.as_tensor(mean)) / torch.sqrt(torch.as_tensor(var) + eps) * torch.as_tensor(gamma) \
                    + torch.as_tensor(beta)
            elif kind == "sigmoid":
                W, b = arrs
                x = torch.sigmoid(x @ torch.as_tensor(W) + torch.as_tensor(b))
            else:
                W, b = arrs
                x = x @ torch.as_tensor(W) + torch.as_tensor(b)
        return x
    return fwd


def room_nn(ann_air, ann_cca, N=24, ts=1800.0) -> OracleProblem:
    """`casadi_admm_ml.py:247-397` on `three_zone_datadriven_admm/models/Room_model.py`.

    Lags (`training_direct.py:575-620`): max lag L = 3 (T_v), so past states at
    {-2ts, -ts, 0} and past couplings at {-2ts, -ts} are fixed variables.
    ``ann_air`` / ``ann_cca``: [(kind, arrays)] layer lists (see ``_ann_torch``)
    with input columns [T_CCA_0, T_ahu, mDot_ahu, d, d_1, T_amb, Q_rad, Q_rad_1,
    T_air] and [T_air, T_v, T_v_1, T_v_2, d, mDot, mDot_1, T_CCA_0].
    w = [x(-2ts), x(-ts), x(0), c(-2ts), c(-ts), {T_slack_k, c_k}_{k<N}, x(ts)..x(N ts)]
    with x = (T_air, T_CCA_0), c = (T_v, T_ahu, T_CCA_out, T_air_out);
    p = [q_T, s_T, rho, x0 x3, {d(8), past_c(4)} x2, {d(8), lam(4), zbar(4)} x N],
    d = (mDot, mDot_ahu, d, T_amb, Q_rad, T_set, T_upper, T_lower).
    """
    f_air, f_cca = _ann_torch(ann_air), _ann_torch(ann_cca)
    n = 6 + 8 + 5 * N + 2 * N
    m = 5 * N
    npar = 3 + 6 + 24 + 16 * N
    names = [f"{v}@{t}" for t in (-2, -1, 0) for v in ("T_air", "T_CCA_0")]
    names += [f"{v}@{t}" for t in (-2, -1) for v in ("T_v", "T_ahu", "T_CCA_out", "T_air_out")]
    for k in range(N):
        names += [f"T_slack@{k}"] + [f"{v}@{k}" for v in ("T_v", "T_ahu", "T_CCA_out", "T_air_out")]
    for k in range(1, N + 1):
        names += [f"T_air@{k}", f"T_CCA_0@{k}"]

    def x_at(w, k):  # state at step k (k >= -2)
        if k <= 0:
            return w[2 * (k + 2)], w[2 * (k + 2) + 1]
        i = 14 + 5 * N + 2 * (k - 1)
        return w[i], w[i + 1]

    def c_at(w, k):  # couplings at step k (k >= -2)
        if k < 0:
            i = 6 + 4 * (k + 2)
        else:
            i = 14 + 5 * k + 1
        return w[i:i + 4]

    def d_at(p, k):  # disturbances/settings at step k (k >= -2)
        i = 9 + 12 * (k + 2) if k < 0 else 33 + 16 * k
        return p[i:i + 8]

    def stage(w, p, k):
        q_T, s_T, rho = p[0], p[1], p[2]
        Ta, Tc = x_at(w, k)
        Ta1, Tc1 = x_at(w, k + 1)
        sl = w[14 + 5 * k]
        c = c_at(w, k)
        T_v, T_ahu, T_co, T_ao = c[0], c[1], c[2], c[3]
        dk, dm = d_at(p, k), d_at(p, k - 1)
        mDot, mDot_ahu, load, T_amb, Q_rad, T_set = dk[0], dk[1], dk[2], dk[3], dk[4], dk[5]
        T_v1, T_v2 = c_at(w, k - 1)[0], c_at(w, k - 2)[0]
        base = 33 + 16 * k
        lam, zbar = p[base + 8:base + 12], p[base + 12:base + 16]
        xa = torch.stack([Tc, T_ahu, mDot_ahu, load, dm[2], T_amb, Q_rad, dm[4], Ta])
        xc = torch.stack([Ta, T_v, T_v1, T_v2, load, mDot, dm[0], Tc])
        na = Ta + f_air(xa[None])[0, 0]
        ncc = Tc + f_cca(xc[None])[0, 0]
        cost = 10 * q_T * (Ta - T_set) ** 2 + 10 * s_T * sl ** 2
        for i in range(4):
            cost = cost + lam[i] * c[i] + rho / 2 * (zbar[i] - c[i]) ** 2
        g = torch.stack([Ta + sl, T_co - Tc, T_ao - Ta, na - Ta1, ncc - Tc1])
        return ts * cost, g

    def f(w, p):
        return sum(stage(w, p, k)[0] for k in range(N))

    def g(w, p):
        return torch.cat([stage(w, p, k)[1] for k in range(N)])

    def lbg(p):
        out = []
        for k in range(N):
            out += [p[33 + 16 * k + 7], 0.0, 0.0, 0.0, 0.0]
        return np.array(out, float)

    def ubg(p):
        out = []
        for k in range(N):
            out += [p[33 + 16 * k + 6], 0.0, 0.0, 0.0, 0.0]
        return np.array(out, float)

    return OracleProblem("room_nn", n, m, npar, f, g, lbg, ubg, names)


def room_nn_inputs(prob, N=24, T_air=294.0, T_CCA=294.15, load=100.0, T_amb=299.0, Q_rad=50.0,
                   T_set=295.0, T_upper=301.15, T_lower=290.15, q_T=0.0, s_T=1.0, rho=1.0,
                   mDot=0.1, mDot_ahu=0.025, zbar=None, lam=None, past_couplings=None):
    """Cold-start inputs (`core/discretization.py:212-245`) for ``room_nn``."""
    init = np.array([294.15, 295.0, 294.15, 294.0])
    bounds = [(285.0, 308.0), (285.0, 308.0), (285.0, 310.0), (285.0, 310.0)]
    zbar = np.tile(init[:, None], N) if zbar is None else np.broadcast_to(np.asarray(zbar, float).reshape(4, -1), (4, N))
    lam = np.zeros((4, N)) if lam is None else np.broadcast_to(np.asarray(lam, float).reshape(4, -1), (4, N))
    past = init if past_couplings is None else np.asarray(past_couplings, float)
    d = [mDot, mDot_ahu, load, T_amb, Q_rad, T_set, T_upper, T_lower]
    p = [q_T, s_T, rho] + [T_air, T_CCA] * 3
    for _ in range(2):
        p += d + list(past)
    for k in range(N):
        p += d + list(lam[:, k]) + list(zbar[:, k])
    p = np.array(p, float)
    lbw, ubw, w0 = np.zeros(prob.n), np.zeros(prob.n), np.zeros(prob.n)
    for i, name in enumerate(prob.w_names):
        v, t = name.split("@")
        t = int(t)
        if v in ("T_air", "T_CCA_0"):
            x = T_air if v == "T_air" else T_CCA
            if t <= 0:
                lbw[i] = ubw[i] = w0[i] = x
            else:
                lbw[i], ubw[i], w0[i] = 280.15, 303.15, x
        elif v == "T_slack":
            lbw[i], ubw[i], w0[i] = -np.inf, np.inf, 0.0
        else:
            j = ("T_v", "T_ahu", "T_CCA_out", "T_air_out").index(v)
            if t < 0:
                lbw[i] = ubw[i] = w0[i] = past[j]
            else:
                lbw[i], ubw[i] = bounds[j]
                w0[i] = 0.5 * (bounds[j][0] + bounds[j][1])
    return p, lbw, ubw, w0


def ann_layers_from_serialized(layer_specs):
    """[(kind, arrays)] from ``[{"class_name", "config", "weights"}]`` (data only)."""
    out = []
    for spec in layer_specs:
        w = [np.asarray(a, float) for a in spec["weights"]]
        if spec["class_name"] == "BatchNormalization":
            out.append(("bn", (w[0], w[1], w[2], w[3], float(spec["config"].get("epsilon", 1e-3)))))
        elif spec["class_name"] == "Dense":
            act = spec["config"].get("activation", "linear")
            out.append(("sigmoid" if act == "sigmoid" else "linear", (w[0], w[1])))
    return out


# ---------------------------------------------------------------------------
# C5: three-zone AHU and CCA supply controllers, backend "casadi_admm",
# multiple shooting without states (`casadi_/admm.py:198-310`)
# ---------------------------------------------------------------------------

def _tz_supply(kind: str, N=24, ts=1800.0) -> OracleProblem:
    """``kind`` "ahu" (`models/AHU.py`): u = T_ahu1..3, couplings (T_ahu_out_i, T_room_i);
    "cca" (`models/CCA.py`): u = T_v, couplings (T_v_out(i), T_r_i).
    Per step w = [u, W1..3, c1..c6]; g = [outputs' equations (3 supply temperatures, W1..3)];
    p = [u_prev, (r_T_v, c) x 2, rho, {d, zbar(6), lam(6)} x N] with c = cl (AHU) / cp (CCA),
    d = (mDot_0, T_amb) (AHU) / (mDot_0) (CCA)."""
    nu = 3 if kind == "ahu" else 1
    nd = 2 if kind == "ahu" else 1
    nb = nu + 3 + 6
    n, m = N * nb, N * 6
    npg = nu + 4 + 1
    nps = nd + 12
    npar = npg + N * nps
    cn = ("T_ahu_out1", "T_room1", "T_ahu_out2", "T_room2", "T_ahu_out3", "T_room3") if kind == "ahu" else \
        ("T_v_out", "T_r1", "T_v_out2", "T_r2", "T_v_out3", "T_r3")
    un = ["T_ahu1", "T_ahu2", "T_ahu3"] if kind == "ahu" else ["T_v"]
    names = []
    for k in range(N):
        names += [f"{u}@{k}" for u in un] + [f"W{i}@{k}" for i in (1, 2, 3)] + [f"{c}@{k}" for c in cn]

    def stage(w, p, k):
        r_T_v, c, rho = p[nu + 2], p[nu + 3], p[nu + 4]
        o = k * nb
        u, W, cp_ = w[o:o + nu], w[o + nu:o + nu + 3], w[o + nu + 3:o + nb]
        b = npg + k * nps
        d = p[b:b + nd]
        zbar, lam = p[b + nd:b + nd + 6], p[b + nd + 6:b + nd + 12]
        mDot = d[0]
        cost = 0.0
        sup, alg = [], []
        for i in range(3):
            if kind == "ahu":
                t_sup, t_room = u[i], cp_[2 * i + 1]
                pw = c * mDot * (t_sup - (t_room + d[1]) / 2)
            else:
                t_sup, t_r = u[0], cp_[2 * i + 1]
                pw = c * mDot * (t_sup - t_r)
            cost = cost + 0.1 * 0.001 * r_T_v * (pw ** 2 + 0.02) ** 0.5
            sup.append(cp_[2 * i] - 1 * t_sup)
            alg.append(W[i] - pw)
        for i in range(6):
            cost = cost + lam[i] * cp_[i] + rho / 2 * (zbar[i] - cp_[i]) ** 2
        return ts * cost, torch.stack(sup + alg)

    def f(w, p):
        return sum(stage(w, p, k)[0] for k in range(N))

    def g(w, p):
        return torch.cat([stage(w, p, k)[1] for k in range(N)])

    return OracleProblem(f"tz_{kind}", n, m, npar, f, g, lambda p: np.zeros(m), lambda p: np.zeros(m), names)


def tz_ahu(N=24) -> OracleProblem:
    return _tz_supply("ahu", N)


def tz_cca(N=24) -> OracleProblem:
    return _tz_supply("cca", N)


def tz_supply_inputs(prob, N=24, rho=1.0, zbar=None, lam=None, mDot_0=None, T_amb=299.0, r_T_v=1.0):
    """Cold-start inputs (`core/discretization.py:212-245`) of ``tz_ahu`` / ``tz_cca``."""
    ahu = prob.name == "tz_ahu"
    nu = 3 if ahu else 1
    mDot_0 = (0.025 if ahu else 0.1) if mDot_0 is None else mDot_0
    c = 1000.0 if ahu else 4200.0
    init = 295.0 if ahu else 294.15
    zbar = np.full((6, N), init) if zbar is None else np.broadcast_to(np.asarray(zbar, float).reshape(6, -1), (6, N))
    lam = np.zeros((6, N)) if lam is None else np.broadcast_to(np.asarray(lam, float).reshape(6, -1), (6, N))
    u0 = 295.0 if ahu else 294.15
    p = [u0] * nu + [r_T_v, c, r_T_v, c, rho]
    d = [mDot_0, T_amb] if ahu else [mDot_0]
    for k in range(N):
        p += d + list(zbar[:, k]) + list(lam[:, k])
    p = np.array(p, float)
    wlim = 500.0 if ahu else 1e5
    lbw, ubw, w0 = np.zeros(prob.n), np.zeros(prob.n), np.zeros(prob.n)
    for i, name in enumerate(prob.w_names):
        v = name.split("@")[0]
        if v.startswith("T_ahu") and not v.startswith("T_ahu_out") or v == "T_v":
            lbw[i], ubw[i], w0[i] = 285.0, 308.0, 296.5
        elif v.startswith("W"):
            lbw[i], ubw[i], w0[i] = -wlim, wlim, 0.0
        else:
            lbw[i], ubw[i], w0[i] = -np.inf, np.inf, 0.0
    return p, lbw, ubw, w0


# ---------------------------------------------------------------------------
# one room with a time-dependent (conditional) objective, backend "casadi",
# multiple shooting with Euler (`simple_mpc_time_dependent_obj.py:108-165`,
# `casadi_/full.py:101-166`, `objective.py:456-492`)
# ---------------------------------------------------------------------------

def one_room_switch(N=15, ts=300.0) -> OracleProblem:
    """w = [T0, {mDot_k, T_slack_k, T_out_k, switch_test_k, T_{k+1}}];
    g_k = [continuity, T + T_slack (<= T_upper), T_out - T, switch_test - (t_k < switch ? 1 : 2)];
    p = [T0, u_prev, cp, C, s_T, r_mDot, r_mDot2, switch, {T_in, load, T_upper}_k];
    stage cost (x ts): t_k < switch ? (r_mDot u + s_T slack^2) / 10 : r_mDot2 u + s_T slack^2."""
    nb = 5
    n = 1 + N * nb
    m = 4 * N
    npg, nps = 8, 3
    names = ["T@0"]
    for k in range(N):
        names += [f"mDot@{k}", f"T_slack@{k}", f"T_out@{k}", f"switch_test@{k}", f"T@{k + 1}"]

    def f(w, p):
        s_T, r1, r2, sw = p[4], p[5], p[6], p[7]
        tot = w.new_zeros(())
        for k in range(N):
            o = 1 + k * nb
            u, sl = w[o], w[o + 1]
            c = (r1 * u + s_T * sl ** 2) / 10 if k * ts < float(sw) else r2 * u + s_T * sl ** 2
            tot = tot + c * ts
        return tot

    def g(w, p):
        cp, Cz, sw = p[2], p[3], p[7]
        out = []
        for k in range(N):
            o = 1 + k * nb
            T = w[o - 1]
            u, sl, To, st, T1 = w[o], w[o + 1], w[o + 2], w[o + 3], w[o + 4]
            ps = npg + k * nps
            T_in, load = p[ps], p[ps + 1]
            ode = cp * u / Cz * (T_in - T) + load / Cz
            out += [T1 - (T + ode * ts), T + sl, To - T, st - (1.0 if k * ts < float(sw) else 2.0)]
        return torch.stack([torch.as_tensor(v) for v in out])

    def ubg(p):
        u = np.zeros(m)
        for k in range(N):
            u[4 * k + 1] = p[npg + k * nps + 2]
        return u

    return OracleProblem("one_room_switch", n, m, npg + N * nps, f, g, lambda p: np.zeros(m), ubg, names)


def one_room_switch_inputs(prob, N=15, T0=298.16, load=150.0, T_in=290.15, T_upper=295.15, u_prev=0.02,
                           s_T=3.0, r_mDot=1.0, r_mDot2=5.0, switch=600.0):
    p = [T0, u_prev, 1000.0, 100000.0, s_T, r_mDot, r_mDot2, switch] + [T_in, load, T_upper] * N
    p = np.array(p, float)
    lbw, ubw, w0 = np.full(prob.n, -np.inf), np.full(prob.n, np.inf), np.zeros(prob.n)
    for i, name in enumerate(prob.w_names):
        v = name.split("@")[0]
        if v == "T":
            lbw[i], ubw[i], w0[i] = 288.15, 303.15, T0
        elif v == "mDot":
            lbw[i], ubw[i], w0[i] = 0.0, 0.05, 0.025
    lbw[0] = ubw[0] = w0[0] = T0
    return p, lbw, ubw, w0


# ---------------------------------------------------------------------------
# moving horizon estimation, backend "casadi_mhe", collocation over the past
# ---------------------------------------------------------------------------

def mhe_room(N=15, ts=200.0, d=2, estimate="theta") -> OracleProblem:
    """`casadi_/mhe.py:34-196` on `examples/Estimators/mhe_example.py:142-170` (RNGRoom).

    estimate="theta": estimated parameter theta = full_capacity_from_volume_factor,
      w = [T_0, Tw_0, theta, {for j: (T, Tw, T_out, cooling, pw2z, T_slack)_kj; T_{k+1}, Tw_{k+1}}],
      p = [cp, rho, C_Wall, RZone_Wall, R_hull_amb, V, s_T, r_mDot, weight_T, weight_Tw,
           {mDot, load, T_in, T_ambient, T_upper, {meas_T, meas_Tw}_j}_k];
    estimate="mDot": estimated input mDot (one per interval, `mhe.py:163`), theta known,
      w = [T_0, Tw_0, {mDot_k, for j: (...)_kj; T_{k+1}, Tw_{k+1}}],
      p = [cp, rho, theta, C_Wall, RZone_Wall, R_hull_amb, V, s_T, r_mDot, weight_T, weight_Tw,
           {load, T_in, T_ambient, T_upper, {meas_T, meas_Tw}_j}_k].
    g_k = [{ts*ode_j - xp_j (T, Tw), T + T_slack, T_out - T, cooling - cp mDot (T_in - T),
            pw2z - (Tw - T)/RZ}_j, x_end - x_{k+1} (T, Tw)];
    f = sum_kj B_j ts (w_T (T - mT)^2 + w_Tw (Tw - mTw)^2)."""
    tau, B, C, D = collocation(d, "legendre")
    est_u = estimate == "mDot"
    nu = int(est_u)
    nb = nu + 6 * d + 2
    head = 2 if est_u else 3
    n = head + N * nb
    m = N * (6 * d + 2)
    npg = 11 if est_u else 10
    nin = 4 if est_u else 5
    nps = nin + 2 * d
    iw = npg - 2  # weight_T, weight_Tw
    names = ["T@0", "T_wall@0"] + ([] if est_u else ["theta"])
    for k in range(N):
        names += [f"mDot@{k}"] * nu
        for j in range(d):
            names += [f"{v}@{k},{j}" for v in ("T", "T_wall", "T_out", "cooling", "pw2z", "T_slack")]
        names += [f"T@{k + 1}", f"T_wall@{k + 1}"]

    def f(w, p):
        tot = w.new_zeros(())
        for k in range(N):
            o = head + k * nb + nu
            for j in range(d):
                q = o + 6 * j
                ps = npg + k * nps + nin + 2 * j
                tot = tot + B[j + 1] * ts * (p[iw] * (w[q] - p[ps]) ** 2 + p[iw + 1] * (w[q + 1] - p[ps + 1]) ** 2)
        return tot

    def g(w, p):
        if est_u:
            cp, rho, th, Cw, Rzw, Rha, Vz = p[0], p[1], p[2], p[3], p[4], p[5], p[6]
        else:
            cp, rho, Cw, Rzw, Rha, Vz = p[0], p[1], p[2], p[3], p[4], p[5]
            th = w[2]
        out = []
        xk = [w[0], w[1]]
        for k in range(N):
            o = head + k * nb + nu
            ps = npg + k * nps
            if est_u:
                mDot = w[o - 1]
                load, T_in, T_amb = p[ps], p[ps + 1], p[ps + 2]
            else:
                mDot, load, T_in, T_amb = p[ps], p[ps + 1], p[ps + 2], p[ps + 3]
            X = [[w[o + 6 * j], w[o + 6 * j + 1]] for j in range(d)]
            for j in range(d):
                q = o + 6 * j
                T, Tw = X[j]
                pw = (Tw - T) / Rzw
                cool = cp * mDot * (T_in - T)
                ode = [(load + cool + pw) / (rho * cp * Vz * th), -((Tw - T_amb) / Rha + pw) / Cw]
                for s_ in range(2):
                    xp = C[0, j + 1] * xk[s_] + sum(C[r + 1, j + 1] * X[r][s_] for r in range(d))
                    out.append(ts * ode[s_] - xp)
                out += [T + w[q + 5], w[q + 2] - T, w[q + 3] - cool, w[q + 4] - pw]
            x1 = [w[o + 6 * d], w[o + 6 * d + 1]]
            for s_ in range(2):
                x_end = D[0] * xk[s_] + sum(D[j + 1] * X[j][s_] for j in range(d))
                out.append(x_end - x1[s_])
            xk = x1
        return torch.stack(out)

    def ubg(p):
        u = np.zeros(m)
        for k in range(N):
            for j in range(d):
                u[k * (6 * d + 2) + 6 * j + 2] = p[npg + k * nps + nin - 1]
        return u

    def lbg(p):
        return np.zeros(m)

    return OracleProblem("mhe_room", n, m, npg + N * nps, f, g, lbg, ubg, names)


def mhe_room_inputs(prob, meas_T, meas_Tw, N=15, d=2, w_T=1.0, w_Tw=0.0, theta_lb=5.0, theta_ub=6.0,
                    mDot=0.22, load=0.0, T_in=17.0, T_amb=28.0, T_upper=22.0, slack_lb=-50.0,
                    estimate="theta", theta=5.5, mDot_lb=0.0, mDot_ub=1.0):
    """Cold start (`core/discretization.py:212-245`): unbounded states/outputs guess 0,
    the estimated parameter / inputs guess the middle of their bounds."""
    est_u = estimate == "mDot"
    p = [1005.0, 1.2] + ([theta] if est_u else []) + [4_569_348.0, 0.0129, 0.1128, 59.0, 1.0, 1.0, w_T, w_Tw]
    for k in range(N):
        p += ([] if est_u else [mDot]) + [load, T_in, T_amb, T_upper]
        for j in range(d):
            p += [meas_T[k * d + j], meas_Tw[k * d + j]]
    p = np.array(p, float)
    lbw, ubw, w0 = np.full(prob.n, -np.inf), np.full(prob.n, np.inf), np.zeros(prob.n)
    for i, name in enumerate(prob.w_names):
        if name == "theta":
            lbw[i], ubw[i], w0[i] = theta_lb, theta_ub, 0.5 * (theta_lb + theta_ub)
        elif name.startswith("mDot@"):
            lbw[i], ubw[i], w0[i] = mDot_lb, mDot_ub, 0.5 * (mDot_lb + mDot_ub)
        elif name.startswith("T_slack@"):  # RNGRoomMHE: slack bounded below
            lbw[i] = slack_lb  # guess 0.5 (lb + inf) = inf -> 0 (nan_to_num, posinf=0)
    return p, lbw, ubw, w0


# ---------------------------------------------------------------------------
# two-state zone + wall MPC (nx = 2 > nu = 1): backend "casadi", collocation
# ---------------------------------------------------------------------------

def rng_room_mpc(N=15, ts=200.0, d=2) -> OracleProblem:
    """`casadi_/full.py:36-98` on the MPC module of `examples/Estimators/mhe_example.py:230-268`
    (RNGRoom: states T, T_wall; control mDot; T_slack auxiliary; 3 outputs).
    w = [T_0, Tw_0, {mDot_k, for j: (T, Tw, T_slack, T_out, cooling, pw2z)_kj, T_{k+1}, Tw_{k+1}}];
    g_k = [x_{k+1} - x_end (T, Tw), {ts*ode_j - xp_j (T, Tw), T + T_slack, T_out - T,
           cooling - cp mDot (T_in - T), pw2z - (Tw - T)/RZ}_j];
    p = [T0, Tw0, u_prev, cp, rho, theta, C_Wall, RZone_Wall, R_hull_amb, V, s_T, r_mDot,
         {load, T_in, T_ambient, T_upper}_kj];
    f = sum_kj B_j ts (r_mDot mDot + s_T T_slack^2)."""
    tau, B, C, D = collocation(d, "legendre")
    nb = 1 + 6 * d + 2
    n = 2 + N * nb
    m = N * (2 + 6 * d)
    npg, nps = 12, 4 * d
    names = ["T@0", "T_wall@0"]
    for k in range(N):
        names.append(f"mDot@{k}")
        for j in range(d):
            names += [f"{v}@{k},{j}" for v in ("T", "T_wall", "T_slack", "T_out", "cooling", "pw2z")]
        names += [f"T@{k + 1}", f"T_wall@{k + 1}"]

    def f(w, p):
        s_T, r = p[10], p[11]
        tot = w.new_zeros(())
        for k in range(N):
            o = 2 + k * nb
            u = w[o]
            for j in range(d):
                tot = tot + B[j + 1] * ts * (r * u + s_T * w[o + 1 + 6 * j + 2] ** 2)
        return tot

    def g(w, p):
        cp, rho, th, Cw, Rzw, Rha, Vz = p[3], p[4], p[5], p[6], p[7], p[8], p[9]
        out = []
        xk = [w[0], w[1]]
        for k in range(N):
            o = 2 + k * nb
            u = w[o]
            X = [[w[o + 1 + 6 * j], w[o + 2 + 6 * j]] for j in range(d)]
            x1 = [w[o + nb - 2], w[o + nb - 1]]
            for s_ in range(2):
                out.append(x1[s_] - (D[0] * xk[s_] + sum(D[j + 1] * X[j][s_] for j in range(d))))
            for j in range(d):
                q = o + 1 + 6 * j
                ps = npg + k * nps + 4 * j
                load, T_in, T_amb = p[ps], p[ps + 1], p[ps + 2]
                T, Tw = X[j]
                pw = (Tw - T) / Rzw
                cool = cp * u * (T_in - T)
                ode = [(load + cool + pw) / (rho * cp * Vz * th), -((Tw - T_amb) / Rha + pw) / Cw]
                for s_ in range(2):
                    xp = C[0, j + 1] * xk[s_] + sum(C[r_ + 1, j + 1] * X[r_][s_] for r_ in range(d))
                    out.append(ts * ode[s_] - xp)
                out += [T + w[q + 2], w[q + 3] - T, w[q + 4] - cool, w[q + 5] - pw]
            xk = x1
        return torch.stack(out)

    def ubg(p):
        u = np.zeros(m)
        for k in range(N):
            for j in range(d):
                u[k * (2 + 6 * d) + 2 + 6 * j + 2] = p[npg + k * nps + 4 * j + 3]
        return u

    return OracleProblem("rng_room_mpc", n, m, npg + N * nps, f, g, lambda p: np.zeros(m), ubg, names)


def rng_room_mpc_inputs(prob, N=15, d=2, T0=25.0, Tw0=27.0, u_prev=0.02, theta=5.5, load=0.0, T_in=17.0,
                        T_amb=28.0, T_upper=23.0, T_lb=15.0, T_ub=30.0, u_lb=0.0, u_ub=0.1):
    p = [T0, Tw0, u_prev, 1005.0, 1.2, theta, 4_569_348.0, 0.0129, 0.1128, 59.0, 1.0, 1.0]
    p += [load, T_in, T_amb, T_upper] * (N * d)
    p = np.array(p, float)
    lbw, ubw, w0 = np.full(prob.n, -np.inf), np.full(prob.n, np.inf), np.zeros(prob.n)
    for i, name in enumerate(prob.w_names):
        v = name.split("@")[0]
        if v == "T":
            lbw[i], ubw[i], w0[i] = T_lb, T_ub, T0
        elif v == "T_wall":
            w0[i] = Tw0
        elif v == "mDot":
            lbw[i], ubw[i], w0[i] = u_lb, u_ub, 0.5 * (u_lb + u_ub)
    lbw[0] = ubw[0] = w0[0] = T0
    lbw[1] = ubw[1] = w0[1] = Tw0
    return p, lbw, ubw, w0


# ---------------------------------------------------------------------------
# reference test-suite model (tests/fixtures/casadi_test_model.py), backend "casadi"
# ---------------------------------------------------------------------------

def fixture_mpc(N=5, ts=900.0, d=3) -> OracleProblem:
    """w = [x_0, {u_k, {x_kj, y_kj}_j, x_{k+1}}_k] (`casadi_/full.py:36-98`), y = myout;
    g per interval: continuity, then per point collocation and the output equation
    y - x = 0 (`casadi_model.py:458-467`); p = [x0, u_prev, par, par2, {disturbance_kj}].
    ode = u + par (x - dist) - par2, cost (x - 290)^2 at the points (`casadi_test_model.py:37-47`)."""
    tau, B, C, D = collocation(d)
    nb = 1 + 2 * d + 1
    n = 1 + N * nb
    m = N * (1 + 2 * d)
    npg = 4
    names = ["state@0"]
    for k in range(N):
        names.append(f"myctrl@{k}")
        for j in range(d):
            names += [f"state@{k},{j}", f"myout@{k},{j}"]
        names.append(f"state@{k + 1}")

    def f(w, p):
        tot = w.new_zeros(())
        for k in range(N):
            o = 1 + k * nb
            for j in range(d):
                tot = tot + B[j + 1] * (w[o + 1 + 2 * j] - 290.0) ** 2 * ts
        return tot

    def g(w, p):
        par, par2 = p[2], p[3]
        out = []
        xk = w[0]
        for k in range(N):
            o = 1 + k * nb
            u = w[o]
            xj = [w[o + 1 + 2 * j] for j in range(d)]
            out.append(w[o + nb - 1] - (D[0] * xk + sum(D[j + 1] * xj[j] for j in range(d))))
            for j in range(d):
                dist = p[npg + k * d + j]
                ode = u + par * (xj[j] - dist) - par2
                xp = C[0, j + 1] * xk + sum(C[r + 1, j + 1] * xj[r] for r in range(d))
                out.append(ts * ode - xp)
                out.append(w[o + 2 + 2 * j] - xj[j])
            xk = w[o + nb - 1]
        return torch.stack(out)

    return OracleProblem("fixture_mpc", n, m, npg + N * d, f, g, lambda p: np.zeros(m), lambda p: np.zeros(m),
                         names)


def fixture_mpc_inputs(prob: OracleProblem, N=5, d=3, T0=298.16, dist=270.0, u_prev=0.02, par=12.0, par2=10.0,
                       u_lb=0.0, u_ub=1.0, T_lb=-np.inf, T_ub=np.inf):
    """Cold start (`core/discretization.py:212-245`): states at their current value, the
    control at the middle of its bounds, the unbounded output at 0."""
    p = np.array([T0, u_prev, par, par2] + [dist] * (N * d), float)
    lbw = np.full(prob.n, -np.inf)
    ubw = np.full(prob.n, np.inf)
    w0 = np.zeros(prob.n)
    for i, name in enumerate(prob.w_names):
        base = name.split("@")[0]
        if base == "state":
            lbw[i], ubw[i], w0[i] = T_lb, T_ub, T0
        elif base == "myctrl":
            lbw[i], ubw[i], w0[i] = u_lb, u_ub, 0.5 * (u_lb + u_ub)
    lbw[0] = ubw[0] = T0
    return p, lbw, ubw, w0


def cubic_room(N=4, ts=10.0, d=2, wz=0.0) -> OracleProblem:
    """w = [T_0, {u_k, {T_kj, z_kj}_j, T_{k+1}}]; g per interval: continuity, then per point
    the collocation row and z^3 - 3 z - 5 = 0; cost B_j ts (T - 290)^2 (``wz``: an optional z^2
    weight, 0 in the model).  No parameters
    beyond the initial state (and u_prev of backend "casadi")."""
    tau, B, C, D = collocation(d)
    nb = 1 + 2 * d + 1
    n = 1 + N * nb
    m = N * (1 + 2 * d)
    names = ["T@0"]
    for k in range(N):
        names.append(f"u@{k}")
        for j in range(d):
            names += [f"T@{k},{j}", f"z@{k},{j}"]
        names.append(f"T@{k + 1}")

    def f(w, p):
        tot = w.new_zeros(())
        for k in range(N):
            o = 1 + k * nb
            for j in range(d):
                tot = tot + B[j + 1] * ((w[o + 1 + 2 * j] - 290.0) ** 2 + wz * w[o + 2 + 2 * j] ** 2) * ts
        return tot

    def g(w, p):
        out = []
        xk = w[0]
        for k in range(N):
            o = 1 + k * nb
            u = w[o]
            Tj = [w[o + 1 + 2 * j] for j in range(d)]
            out.append(w[o + nb - 1] - (D[0] * xk + sum(D[j + 1] * Tj[j] for j in range(d))))
            for j in range(d):
                xp = C[0, j + 1] * xk + sum(C[r + 1, j + 1] * Tj[r] for r in range(d))
                out.append(ts * (u - 0.01 * (Tj[j] - 290.0)) - xp)
                z = w[o + 2 + 2 * j]
                out.append(z ** 3 - 3.0 * z - 5.0)
            xk = w[o + nb - 1]
        return torch.stack(out)

    return OracleProblem("cubic_room", n, m, 2, f, g, lambda p: np.zeros(m), lambda p: np.zeros(m), names)


def cubic_room_inputs(prob: OracleProblem, T0=295.0, u_prev=0.0, z_lb=-5.0, z_ub=2.6):
    p = np.array([T0, u_prev], float)
    lbw = np.full(prob.n, -np.inf)
    ubw = np.full(prob.n, np.inf)
    w0 = np.zeros(prob.n)
    for i, name in enumerate(prob.w_names):
        base = name.split("@")[0]
        if base == "T":
            w0[i] = T0
        elif base == "u":
            lbw[i], ubw[i], w0[i] = 0.0, 1.0, 0.5
        elif base == "z":
            lbw[i], ubw[i], w0[i] = z_lb, z_ub, 0.5 * (z_lb + z_ub)
    lbw[0] = ubw[0] = w0[0] = T0
    return p, lbw, ubw, w0
