"""Backends of the benchmark configurations (BASELINE.json ``configs``).

* ``one_room``        C1/C3 — `examples/one_room_mpc/physical/simple_mpc.py:141-187`
* ``admm_room``       C2 room agent — `examples/4_Room_ADMM_Coordinator/configs/room_*_admm.json`
* ``admm_ahu``        C2 air handler — `examples/4_Room_ADMM_Coordinator/configs/rlt_admm.json`
* ``exchange_room``   C4 room agent — `examples/exchange_admm/configs/room_1_admm.json`
* ``exchange_supply`` C4 supply agent — `examples/exchange_admm/configs/rlt_admm.json`

Each builder returns ``(backend, current_vars)`` with the example's values;
keyword arguments override the per-agent values used for synthetic fleets.
"""

from __future__ import annotations

from typing import Callable, Dict, Tuple

import numpy as np

from agentlib_mpc_amd.data_structures import admm_datatypes as adt
from agentlib_mpc_amd.data_structures.mpc_datamodels import MPCVariable, VariableReference
from agentlib_mpc_amd.optimization_backends import create_optimization_backend

TIGHT = {"ipopt": {"tol": 1e-10, "max_iter": 500}}


def V(name, value=None, lb=-np.inf, ub=np.inf):
    return MPCVariable(name=name, value=value, lb=lb, ub=ub)


def one_room(N=15, T0=298.16, load=150.0, T_in=290.15, T_upper=295.15, u_prev=0.02,
             s_T=0.001, r_mDot=0.01, d=2, solver_options=TIGHT):
    be = create_optimization_backend({
        "type": "mi355x",
        "model": {"type": "agentlib_mpc_amd.models.examples.OneRoom"},
        "discretization_options": {"collocation_order": d, "collocation_method": "legendre",
                                   "prediction_horizon": N, "time_step": 300},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    be.setup_optimization(VariableReference(
        states=["T"], controls=["mDot"], inputs=["T_in", "load", "T_upper"],
        parameters=["s_T", "r_mDot"], outputs=["T_out"]))
    cv = {
        "T": V("T", T0, 288.15, 303.15), "mDot": V("mDot", u_prev, 0.0, 0.05),
        "T_in": V("T_in", T_in), "load": V("load", load), "T_upper": V("T_upper", T_upper),
        "s_T": V("s_T", s_T), "r_mDot": V("r_mDot", r_mDot), "T_out": V("T_out"),
    }
    return be, cv


def _vals(v, n):
    return [v] * n if np.isscalar(v) else list(v)


def admm_room(N=10, T0=296.0, dist=150.0, T_set=296.0, rho=0.4, zbar=0.02, lam=0.0,
              solver_options=TIGHT):
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": {"type": "agentlib_mpc_amd.models.examples.CooledRoom"},
        "discretization_options": {"prediction_horizon": N, "time_step": 60},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    c = adt.CouplingEntry("mDot")
    be.setup_optimization(adt.VariableReference(
        states=["T"], controls=[], inputs=["d", "T_set", "T_upper", "T_in"],
        parameters=["q_T", "q_mDot"], outputs=[], couplings=[c]))
    n = len(be.coupling_grid)
    cv = {
        "T": V("T", T0, 288.15, 303.15), "d": V("d", dist), "T_set": V("T_set", T_set),
        "T_upper": V("T_upper", 303.15), "T_in": V("T_in", 290.15), "q_T": V("q_T", 1.0),
        "q_mDot": V("q_mDot", 1.0), "mDot": V("mDot", 0.02, 0.0, 0.05),
        c.mean: V(c.mean, _vals(zbar, n)), c.multiplier: V(c.multiplier, _vals(lam, n)),
        "penalty_factor": V("penalty_factor", rho),
    }
    return be, cv


def admm_ahu(N=10, rho=0.4, zbar=0.01, lam=0.0, solver_options=TIGHT):
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": {"type": "agentlib_mpc_amd.models.examples.AirHandler"},
        "discretization_options": {"prediction_horizon": N, "time_step": 60},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    coups = [adt.CouplingEntry(f"mDot_out_{i + 1}") for i in range(4)]
    be.setup_optimization(adt.VariableReference(
        states=[], controls=[f"mDot_{i + 1}" for i in range(4)], inputs=[],
        parameters=["mDot_max"], outputs=[], couplings=coups))
    n = len(be.coupling_grid)
    zb = np.broadcast_to(np.asarray(zbar, float), (4, n)) if np.ndim(zbar) < 2 else np.asarray(zbar)
    lm = np.broadcast_to(np.asarray(lam, float), (4, n)) if np.ndim(lam) < 2 else np.asarray(lam)
    cv = {f"mDot_{i + 1}": V(f"mDot_{i + 1}", 0.01, 0.0, 0.075) for i in range(4)}
    cv.update({"mDot_max": V("mDot_max", 0.1), "penalty_factor": V("penalty_factor", rho)})
    for i, c in enumerate(coups):
        cv[c.name] = V(c.name, 0.01)
        cv[c.mean] = V(c.mean, list(zb[i]))
        cv[c.multiplier] = V(c.multiplier, list(lm[i]))
    return be, cv


def exchange_room(N=10, T0=296.0, dist=150.0, rho=1e4, diff=0.0, lam=0.0, T_set=296.0,
                  solver_options=TIGHT):
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": {"type": "agentlib_mpc_amd.models.examples.ExchangeRoom"},
        "discretization_options": {"method": "multiple_shooting", "integrator": "euler",
                                   "prediction_horizon": N, "time_step": 120},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    e = adt.ExchangeEntry("mDot_out")
    be.setup_optimization(adt.VariableReference(
        states=["T"], controls=["mDot"], inputs=["d", "T_set", "T_upper", "T_in"],
        parameters=["q_T", "q_mDot"], outputs=[], exchange=[e]))
    n = len(be.coupling_grid)
    cv = {
        "T": V("T", T0, 288.15, 303.15), "mDot": V("mDot", 0.02, 0.0, 0.05),
        "d": V("d", dist), "T_set": V("T_set", T_set), "T_upper": V("T_upper", 296.15),
        "T_in": V("T_in", 290.15), "q_T": V("q_T", 1.0), "q_mDot": V("q_mDot", 0.0),
        "mDot_out": V("mDot_out", 0.02, 0.0, 0.05),
        e.mean_diff: V(e.mean_diff, _vals(diff, n)), e.multiplier: V(e.multiplier, _vals(lam, n)),
        "penalty_factor": V("penalty_factor", rho),
    }
    return be, cv


def exchange_supply(N=10, rho=1e4, diff=0.0, lam=0.0, penalty=0.1, solver_options=TIGHT):
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": {"type": "agentlib_mpc_amd.models.examples.ExchangeSupply"},
        "discretization_options": {"method": "multiple_shooting", "integrator": "euler",
                                   "prediction_horizon": N, "time_step": 120},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    e = adt.ExchangeEntry("mDot_out")
    be.setup_optimization(adt.VariableReference(
        states=[], controls=["mDot"], inputs=[], parameters=["penalty"], outputs=[], exchange=[e]))
    n = len(be.coupling_grid)
    cv = {
        "mDot": V("mDot", 0.01, 0.0, 0.1), "penalty": V("penalty", penalty),
        "mDot_out": V("mDot_out", 0.02, -0.1, 0.0),
        e.mean_diff: V(e.mean_diff, _vals(diff, n)), e.multiplier: V(e.multiplier, _vals(lam, n)),
        "penalty_factor": V("penalty_factor", rho),
    }
    return be, cv


BUILDERS: Dict[str, Callable[..., Tuple[object, dict]]] = {
    "one_room": one_room,
    "admm_room": admm_room,
    "admm_ahu": admm_ahu,
    "exchange_room": exchange_room,
    "exchange_supply": exchange_supply,
}


def compile_all(verbose: bool = False):
    """Generate and compile the code objects of all benchmark structures."""
    from agentlib_mpc_amd.runtime import native

    current = native._kernel_deps_hash()
    if native.KERNEL_DIR.exists():  # drop code objects of older kernel sources
        for f in native.KERNEL_DIR.iterdir():
            if current not in f.name:
                f.unlink()
    paths = {}
    for name, fn in BUILDERS.items():
        be, _ = fn()
        paths[name] = be.problem.compile()
        if verbose:
            print(f"[mpcx] {name}: {paths[name].name}")
    return paths
