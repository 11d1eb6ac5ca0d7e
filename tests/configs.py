"""Benchmark configurations built twice: through the product backend (MPC
variables -> host marshalling -> NLP vectors) and through the oracle's hand
restatement, with identical input values.

Values follow the reference examples:
C1 `examples/one_room_mpc/physical/simple_mpc.py:141-187`,
C2 `examples/4_Room_ADMM_Coordinator/configs/{room_*,rlt}_admm.json`, `coordinator.json:7-18`,
C4 `examples/exchange_admm/configs/{room_1,rlt}_admm.json`.
"""

from __future__ import annotations

import dataclasses
from typing import Callable, Dict

import numpy as np

from agentlib_mpc_amd.data_structures import admm_datatypes as adt
from agentlib_mpc_amd.data_structures.mpc_datamodels import MPCVariable, VariableReference
from agentlib_mpc_amd.optimization_backends import create_optimization_backend
from oracle import nlps


def V(name, value=None, lb=-np.inf, ub=np.inf):
    return MPCVariable(name=name, value=value, lb=lb, ub=ub)


@dataclasses.dataclass
class Case:
    backend: object
    current_vars: Dict[str, MPCVariable]
    oracle: nlps.OracleProblem
    oracle_inputs: tuple  # (p, lbw, ubw, w0)


def one_room(N=15, T0=298.16, load=150.0, T_in=290.15, T_upper=295.15, u_prev=0.02,
             s_T=0.001, r_mDot=0.01, d=2) -> Case:
    be = create_optimization_backend({
        "type": "mi355x",
        "model": {"type": "agentlib_mpc_amd.models.examples.OneRoom"},
        "discretization_options": {"collocation_order": d, "collocation_method": "legendre",
                                   "prediction_horizon": N, "time_step": 300},
        "solver": {"name": "ipopt", "options": {"ipopt": {"tol": 1e-10, "max_iter": 500}}},
    })
    vr = VariableReference(states=["T"], controls=["mDot"], inputs=["T_in", "load", "T_upper"],
                           parameters=["s_T", "r_mDot"], outputs=["T_out"])
    be.setup_optimization(vr)
    cv = {
        "T": V("T", T0, 288.15, 303.15),
        "mDot": V("mDot", u_prev, 0.0, 0.05),
        "T_in": V("T_in", T_in), "load": V("load", load), "T_upper": V("T_upper", T_upper),
        "s_T": V("s_T", s_T), "r_mDot": V("r_mDot", r_mDot),
        "T_out": V("T_out"),
    }
    prob = nlps.one_room(N=N, d=d)
    oi = nlps.one_room_inputs(prob, N=N, d=d, T0=T0, load=load, T_in=T_in, T_upper=T_upper,
                              s_T=s_T, r_mDot=r_mDot, u_prev=u_prev)
    return Case(be, cv, prob, oi)


def admm_room(N=10, T0=296.0, dist=150.0, T_set=296.0, rho=0.4, zbar=0.02, lam=0.0) -> Case:
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": {"type": "agentlib_mpc_amd.models.examples.CooledRoom"},
        "discretization_options": {"prediction_horizon": N, "time_step": 60},
        "solver": {"name": "ipopt", "options": {"ipopt": {"tol": 1e-10, "max_iter": 500}}},
    })
    c = adt.CouplingEntry("mDot")
    vr = adt.VariableReference(states=["T"], controls=[], inputs=["d", "T_set", "T_upper", "T_in"],
                               parameters=["q_T", "q_mDot"], outputs=[], couplings=[c])
    be.setup_optimization(vr)
    npts = len(be.coupling_grid)
    zb = [zbar] * npts if np.isscalar(zbar) else list(zbar)
    lm = [lam] * npts if np.isscalar(lam) else list(lam)
    cv = {
        "T": V("T", T0, 288.15, 303.15),
        "d": V("d", dist), "T_set": V("T_set", T_set), "T_upper": V("T_upper", 303.15),
        "T_in": V("T_in", 290.15), "q_T": V("q_T", 1.0), "q_mDot": V("q_mDot", 1.0),
        "mDot": V("mDot", 0.02, 0.0, 0.05),
        c.mean: V(c.mean, zb), c.multiplier: V(c.multiplier, lm),
        "penalty_factor": V("penalty_factor", rho),
    }
    prob = nlps.admm_room(N=N)
    oi = nlps.admm_room_inputs(prob, N=N, T0=T0, dist=dist, T_set=T_set, rho=rho,
                               zbar=np.array(zb), lam=np.array(lm))
    return Case(be, cv, prob, oi)


def admm_ahu(N=10, rho=0.4, zbar=0.01, lam=0.0) -> Case:
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": {"type": "agentlib_mpc_amd.models.examples.AirHandler"},
        "discretization_options": {"prediction_horizon": N, "time_step": 60},
        "solver": {"name": "ipopt", "options": {"ipopt": {"tol": 1e-10, "max_iter": 500}}},
    })
    coups = [adt.CouplingEntry(f"mDot_out_{i + 1}") for i in range(4)]
    vr = adt.VariableReference(states=[], controls=[f"mDot_{i + 1}" for i in range(4)], inputs=[],
                               parameters=["mDot_max"], outputs=[], couplings=coups)
    be.setup_optimization(vr)
    npts = len(be.coupling_grid)
    zb = np.broadcast_to(np.asarray(zbar, float), (4, npts)).copy() if np.ndim(zbar) < 2 else np.asarray(zbar)
    lm = np.broadcast_to(np.asarray(lam, float), (4, npts)).copy() if np.ndim(lam) < 2 else np.asarray(lam)
    cv = {f"mDot_{i + 1}": V(f"mDot_{i + 1}", 0.01, 0.0, 0.075) for i in range(4)}
    cv.update({"mDot_max": V("mDot_max", 0.1), "penalty_factor": V("penalty_factor", rho)})
    for i, c in enumerate(coups):
        cv[c.name] = V(c.name, 0.01)
        cv[c.mean] = V(c.mean, list(zb[i]))
        cv[c.multiplier] = V(c.multiplier, list(lm[i]))
    prob = nlps.admm_ahu(N=N)
    oi = nlps.admm_ahu_inputs(prob, N=N, rho=rho, zbar=zb, lam=lm)
    return Case(be, cv, prob, oi)


def exchange_room(N=10, T0=296.0, dist=150.0, rho=1e4, diff=0.0, lam=0.0, T_set=296.0) -> Case:
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": {"type": "agentlib_mpc_amd.models.examples.ExchangeRoom"},
        "discretization_options": {"method": "multiple_shooting", "integrator": "euler",
                                   "prediction_horizon": N, "time_step": 120},
        "solver": {"name": "ipopt", "options": {"ipopt": {"tol": 1e-10, "max_iter": 500}}},
    })
    e = adt.ExchangeEntry("mDot_out")
    vr = adt.VariableReference(states=["T"], controls=["mDot"], inputs=["d", "T_set", "T_upper", "T_in"],
                               parameters=["q_T", "q_mDot"], outputs=[], exchange=[e])
    be.setup_optimization(vr)
    npts = len(be.coupling_grid)
    df = [diff] * npts if np.isscalar(diff) else list(diff)
    lm = [lam] * npts if np.isscalar(lam) else list(lam)
    cv = {
        "T": V("T", T0, 288.15, 303.15), "mDot": V("mDot", 0.02, 0.0, 0.05),
        "d": V("d", dist), "T_set": V("T_set", T_set), "T_upper": V("T_upper", 296.15),
        "T_in": V("T_in", 290.15), "q_T": V("q_T", 1.0), "q_mDot": V("q_mDot", 0.0),
        "mDot_out": V("mDot_out", 0.02, 0.0, 0.05),
        e.mean_diff: V(e.mean_diff, df), e.multiplier: V(e.multiplier, lm),
        "penalty_factor": V("penalty_factor", rho),
    }
    prob = nlps.exchange_room(N=N)
    oi = nlps.exchange_room_inputs(prob, N=N, T0=T0, dist=dist, rho=rho, diff=np.array(df),
                                   lam=np.array(lm), T_set=T_set)
    return Case(be, cv, prob, oi)


def exchange_supply(N=10, rho=1e4, diff=0.0, lam=0.0, penalty=0.1) -> Case:
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": {"type": "agentlib_mpc_amd.models.examples.ExchangeSupply"},
        "discretization_options": {"method": "multiple_shooting", "integrator": "euler",
                                   "prediction_horizon": N, "time_step": 120},
        "solver": {"name": "ipopt", "options": {"ipopt": {"tol": 1e-10, "max_iter": 500}}},
    })
    e = adt.ExchangeEntry("mDot_out")
    vr = adt.VariableReference(states=[], controls=["mDot"], inputs=[], parameters=["penalty"],
                               outputs=[], exchange=[e])
    be.setup_optimization(vr)
    npts = len(be.coupling_grid)
    df = [diff] * npts if np.isscalar(diff) else list(diff)
    lm = [lam] * npts if np.isscalar(lam) else list(lam)
    cv = {
        "mDot": V("mDot", 0.01, 0.0, 0.1), "penalty": V("penalty", penalty),
        "mDot_out": V("mDot_out", 0.02, -0.1, 0.0),
        e.mean_diff: V(e.mean_diff, df), e.multiplier: V(e.multiplier, lm),
        "penalty_factor": V("penalty_factor", rho),
    }
    prob = nlps.exchange_supply(N=N)
    oi = nlps.exchange_supply_inputs(prob, N=N, penalty=penalty, rho=rho, diff=np.array(df),
                                     lam=np.array(lm))
    return Case(be, cv, prob, oi)


CASES: Dict[str, Callable[..., Case]] = {
    "one_room": one_room,
    "admm_room": admm_room,
    "admm_ahu": admm_ahu,
    "exchange_room": exchange_room,
    "exchange_supply": exchange_supply,
}


def product_nlp_inputs(case: Case, now: float = 0.0):
    prob = case.backend.problem
    mi = prob.mpc_inputs(case.current_vars, now)
    mi.update(prob.initial_guess(mi))
    return prob.nlp_inputs(mi), mi
