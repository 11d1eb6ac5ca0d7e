"""Benchmark configurations built twice: through the product backend (MPC
variables -> host marshalling -> NLP vectors, `agentlib_mpc_amd/benchmarks.py`)
and through the oracle's hand restatement (`oracle/nlps.py`) with identical
input values.
"""

from __future__ import annotations

import dataclasses
from typing import Callable, Dict

import numpy as np

from agentlib_mpc_amd import benchmarks as bm
from oracle import nlps


@dataclasses.dataclass
class Case:
    backend: object
    current_vars: dict
    oracle: nlps.OracleProblem
    oracle_inputs: tuple  # (p, lbw, ubw, w0)


def one_room(**kw) -> Case:
    be, cv = bm.one_room(**kw)
    N, d = kw.get("N", 15), kw.get("d", 2)
    prob = nlps.one_room(N=N, d=d, method=kw.get("method", "legendre"), delta_u="r_delta_mDot" in kw)
    keys = ("T0", "load", "T_in", "T_upper", "s_T", "r_mDot", "u_prev", "r_delta_mDot")
    return Case(be, cv, prob, nlps.one_room_inputs(prob, N=N, d=d, **{k: kw[k] for k in keys if k in kw}))


def admm_room(**kw) -> Case:
    be, cv = bm.admm_room(**kw)
    N = kw.get("N", 10)
    n = len(be.coupling_grid)
    prob = nlps.admm_room(N=N)
    o = {k: kw[k] for k in ("T0", "dist", "T_set", "rho") if k in kw}
    o["zbar"] = np.asarray(bm._vals(kw.get("zbar", 0.02), n))
    o["lam"] = np.asarray(bm._vals(kw.get("lam", 0.0), n))
    return Case(be, cv, prob, nlps.admm_room_inputs(prob, N=N, **o))


def admm_ahu(**kw) -> Case:
    be, cv = bm.admm_ahu(**kw)
    N = kw.get("N", 10)
    n = len(be.coupling_grid)
    prob = nlps.admm_ahu(N=N)
    zb = np.broadcast_to(np.asarray(kw.get("zbar", 0.01), float), (4, n))
    lm = np.broadcast_to(np.asarray(kw.get("lam", 0.0), float), (4, n))
    return Case(be, cv, prob, nlps.admm_ahu_inputs(prob, N=N, rho=kw.get("rho", 0.4), zbar=zb, lam=lm))


def exchange_room(**kw) -> Case:
    be, cv = bm.exchange_room(**kw)
    N = kw.get("N", 10)
    n = len(be.coupling_grid)
    prob = nlps.exchange_room(N=N, integrator=kw.get("integrator", "euler"))
    o = {k: kw[k] for k in ("T0", "dist", "rho", "T_set") if k in kw}
    o["diff"] = np.asarray(bm._vals(kw.get("diff", 0.0), n))
    o["lam"] = np.asarray(bm._vals(kw.get("lam", 0.0), n))
    return Case(be, cv, prob, nlps.exchange_room_inputs(prob, N=N, **o))


def exchange_supply(**kw) -> Case:
    be, cv = bm.exchange_supply(**kw)
    N = kw.get("N", 10)
    n = len(be.coupling_grid)
    prob = nlps.exchange_supply(N=N)
    o = {k: kw[k] for k in ("rho", "penalty") if k in kw}
    o["diff"] = np.asarray(bm._vals(kw.get("diff", 0.0), n))
    o["lam"] = np.asarray(bm._vals(kw.get("lam", 0.0), n))
    return Case(be, cv, prob, nlps.exchange_supply_inputs(prob, N=N, **o))


def room_nn(**kw) -> Case:
    from agentlib_mpc_amd.models import examples as ex

    anns = ex.room_cca_anns()
    be, cv = bm.room_nn(anns=anns, **kw)
    N = kw.get("N", 24)
    air, cca = (nlps.ann_layers_from_serialized(a.layer_specs()) for a in anns)
    prob = nlps.room_nn(air, cca, N=N)
    keys = ("T_air", "T_CCA", "load", "T_amb", "Q_rad", "T_set", "T_upper", "T_lower", "q_T", "s_T",
            "rho", "zbar", "lam", "past_couplings")
    o = {k: kw[k] for k in keys if k in kw}
    if "zbar" in o:
        o["zbar"] = np.broadcast_to(np.asarray(o["zbar"], float).reshape(4, -1), (4, N))
    if "lam" in o:
        o["lam"] = np.broadcast_to(np.asarray(o["lam"], float).reshape(4, -1), (4, N))
    return Case(be, cv, prob, nlps.room_nn_inputs(prob, N=N, **o))


def _tz(kind, **kw) -> Case:
    be, cv = (bm.tz_ahu if kind == "ahu" else bm.tz_cca)(**kw)
    N = kw.get("N", 24)
    prob = nlps.tz_ahu(N=N) if kind == "ahu" else nlps.tz_cca(N=N)
    o = {k: kw[k] for k in ("rho", "zbar", "lam", "mDot_0", "r_T_v") if k in kw}
    for k in ("zbar", "lam"):
        if k in o and np.ndim(o[k]) == 0:
            o[k] = np.full((6, N), float(o[k]))
    if kind == "ahu" and "T_amb" in kw:
        o["T_amb"] = kw["T_amb"]
    return Case(be, cv, prob, nlps.tz_supply_inputs(prob, N=N, **o))


def tz_ahu(**kw) -> Case:
    return _tz("ahu", **kw)


def tz_cca(**kw) -> Case:
    return _tz("cca", **kw)


def one_room_radau(**kw) -> Case:
    return one_room(d=3, method="radau", **kw)


def one_room_du(**kw) -> Case:
    kw.setdefault("r_delta_mDot", 0.1)
    return one_room(**kw)


def exchange_room_rk(**kw) -> Case:
    return exchange_room(integrator="rk", **kw)


def one_room_switch(**kw) -> Case:
    be, cv = bm.one_room_switch(**kw)
    N = kw.get("N", 15)
    prob = nlps.one_room_switch(N=N)
    keys = ("T0", "load", "T_in", "T_upper", "u_prev", "s_T", "r_mDot", "r_mDot2", "switch")
    return Case(be, cv, prob, nlps.one_room_switch_inputs(prob, N=N, **{k: kw[k] for k in keys if k in kw}))


def mhe_room(**kw) -> Case:
    N, d = kw.get("N", 15), kw.get("d", 2)
    meas = kw.pop("measured", None)
    if meas is None:
        meas = bm.mhe_measurements(N=N, d=d, **{k: kw.pop(k) for k in ("theta", "noise", "seed") if k in kw})
    be, cv = bm.mhe_room(measured=meas, **kw)
    est = kw.get("estimate", "theta")
    prob = nlps.mhe_room(N=N, d=d, estimate=est)
    o = {"w_T": kw.get("w_T", 1.0), "w_Tw": kw.get("w_T_wall", 0.0), "estimate": est}
    if "theta_lb" in kw:
        o["theta_lb"] = kw["theta_lb"]
    if "theta_ub" in kw:
        o["theta_ub"] = kw["theta_ub"]
    return Case(be, cv, prob, nlps.mhe_room_inputs(prob, meas[0], meas[1], N=N, d=d, **o))


def rng_room_mpc(**kw) -> Case:
    be, cv = bm.rng_room_mpc(**kw)
    prob = nlps.rng_room_mpc(N=kw.get("N", 15))
    o = {k: kw[k] for k in ("T0", "u_prev", "T_upper", "load") if k in kw}
    if "T_wall0" in kw:
        o["Tw0"] = kw["T_wall0"]
    return Case(be, cv, prob, nlps.rng_room_mpc_inputs(prob, N=kw.get("N", 15), **o))


def fixture_mpc(**kw) -> Case:
    """The reference test-suite model under the MPC module test's config (`tests/test_mpc.py`)."""
    be, cv = bm.fixture_mpc(**kw)
    N = kw.get("N", 5)
    prob = nlps.fixture_mpc(N=N)
    o = {k: kw[k] for k in ("T0", "u_prev", "T_lb", "T_ub") if k in kw}
    if "disturbance" in kw:
        o["dist"] = kw["disturbance"]
    return Case(be, cv, prob, nlps.fixture_mpc_inputs(prob, N=N, **o))


def cubic_room(**kw) -> Case:
    """Restoration-phase case: the line search fails from the cold guess."""
    be, cv = bm.cubic_room(**kw)
    prob = nlps.cubic_room(N=kw.get("N", 4))
    return Case(be, cv, prob, nlps.cubic_room_inputs(prob, **{k: kw[k] for k in ("T0",) if k in kw}))


CASES: Dict[str, Callable[..., Case]] = {
    "one_room": one_room,
    "admm_room": admm_room,
    "admm_ahu": admm_ahu,
    "exchange_room": exchange_room,
    "exchange_supply": exchange_supply,
    "room_nn": room_nn,
    "tz_ahu": tz_ahu,
    "tz_cca": tz_cca,
    "exchange_room_rk": exchange_room_rk,
    "one_room_radau": one_room_radau,
    "one_room_du": one_room_du,
    "one_room_switch": one_room_switch,
    "mhe_room": mhe_room,
    "rng_room_mpc": rng_room_mpc,
    "fixture_mpc": fixture_mpc,
    "cubic_room": cubic_room,
    # estimating mDot per interval needs the wall temperature measured too (else mDot
    # and the unmeasured wall state trade off and the minimiser is not unique)
    "mhe_room_u": lambda **kw: mhe_room(estimate="mDot", **{"w_T_wall": 1.0, **kw}),
}


def product_nlp_inputs(case: Case, now: float = 0.0):
    prob = case.backend.problem
    mi = prob.mpc_inputs(case.current_vars, now)
    mi.update(prob.initial_guess(mi))
    return prob.nlp_inputs(mi), mi
