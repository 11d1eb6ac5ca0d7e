"""Backends of the benchmark configurations (BASELINE.json ``configs``).

* ``one_room``        C1/C3 — `examples/one_room_mpc/physical/simple_mpc.py:141-187`
* ``admm_room``       C2 room agent — `examples/4_Room_ADMM_Coordinator/configs/room_*_admm.json`
* ``admm_ahu``        C2 air handler — `examples/4_Room_ADMM_Coordinator/configs/rlt_admm.json`
* ``exchange_room``   C4 room agent — `examples/exchange_admm/configs/room_1_admm.json`
* ``exchange_supply`` C4 supply agent — `examples/exchange_admm/configs/rlt_admm.json`
* ``room_nn``         C5 zone agent (NARX ANNs) — `examples/three_zone_datadriven_admm/configs/mpc/Room_1.json`
* ``mhe_room``        moving horizon estimator — `examples/Estimators/mhe_example.py:188-228`

Each builder returns ``(backend, current_vars)`` with the example's values;
keyword arguments override the per-agent values used for synthetic fleets.
"""

from __future__ import annotations

from typing import Callable, Dict, Tuple

import os

import numpy as np

from agentlib_mpc_amd.data_structures import admm_datatypes as adt
from agentlib_mpc_amd.data_structures.mpc_datamodels import MPCVariable, VariableReference
from agentlib_mpc_amd.optimization_backends import create_optimization_backend

#: parity settings: a tight tolerance and no acceptable-level stop, so that two solvers are
#: compared at (nearly) exact solutions of the same NLP
TIGHT = {"ipopt": {"tol": 1e-10, "max_iter": 500, "acceptable_iter": 0}}
#: the reference's solver settings (`casadi_utils.py:197-206`; the backend applies them)
REFERENCE = {"ipopt": {}}


def V(name, value=None, lb=-np.inf, ub=np.inf):
    return MPCVariable(name=name, value=value, lb=lb, ub=ub)


def one_room(N=15, T0=298.16, load=150.0, T_in=290.15, T_upper=295.15, u_prev=0.02,
             s_T=0.001, r_mDot=0.01, d=2, solver_options=TIGHT, method="legendre", r_delta_mDot=None, model=None):
    """``r_delta_mDot``: use the change-penalty model (`with_change_control_penalty.py`)."""
    be = create_optimization_backend({
        "type": "mi355x",
        "model": model or {"type": "agentlib_mpc_amd.models.examples."
                          + ("OneRoom" if r_delta_mDot is None else "OneRoomDU")},
        "discretization_options": {"collocation_order": d, "collocation_method": method,
                                   "prediction_horizon": N, "time_step": 300},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    pars = ["s_T", "r_mDot"] + ([] if r_delta_mDot is None else ["r_delta_mDot"])
    be.setup_optimization(VariableReference(
        states=["T"], controls=["mDot"], inputs=["T_in", "load", "T_upper"],
        parameters=pars, outputs=["T_out"]))
    cv = {
        "T": V("T", T0, 288.15, 303.15), "mDot": V("mDot", u_prev, 0.0, 0.05),
        "T_in": V("T_in", T_in), "load": V("load", load), "T_upper": V("T_upper", T_upper),
        "s_T": V("s_T", s_T), "r_mDot": V("r_mDot", r_mDot), "T_out": V("T_out"),
    }
    if r_delta_mDot is not None:
        cv["r_delta_mDot"] = V("r_delta_mDot", r_delta_mDot)
    return be, cv


def _vals(v, n):
    return [v] * n if np.isscalar(v) else list(v)


def admm_room(N=10, T0=296.0, dist=150.0, T_set=296.0, rho=0.4, zbar=0.02, lam=0.0,
              solver_options=TIGHT, model=None):
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": model or {"type": "agentlib_mpc_amd.models.examples.CooledRoom"},
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


def admm_ahu(N=10, rho=0.4, zbar=0.01, lam=0.0, solver_options=TIGHT, model=None):
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": model or {"type": "agentlib_mpc_amd.models.examples.AirHandler"},
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
                  solver_options=TIGHT, integrator="euler", model=None):
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": model or {"type": "agentlib_mpc_amd.models.examples.ExchangeRoom"},
        "discretization_options": {"method": "multiple_shooting", "integrator": integrator,
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


def exchange_supply(N=10, rho=1e4, diff=0.0, lam=0.0, penalty=0.1, solver_options=TIGHT, model=None):
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": model or {"type": "agentlib_mpc_amd.models.examples.ExchangeSupply"},
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


def one_room_switch(N=15, T0=298.16, load=150.0, T_in=290.15, T_upper=295.15, u_prev=0.02, s_T=3.0,
                    r_mDot=1.0, r_mDot2=5.0, switch=600.0, integrator="euler", solver_options=TIGHT):
    """`examples/one_room_mpc/physical/simple_mpc_time_dependent_obj.py` (conditional
    objective switching at ``switch`` seconds), backend "casadi", multiple shooting
    (the example keeps the cvodes default; Euler / "rk" here)."""
    be = create_optimization_backend({
        "type": "mi355x",
        "model": {"type": "agentlib_mpc_amd.models.examples.SwitchRoom"},
        "discretization_options": {"method": "multiple_shooting", "integrator": integrator,
                                   "prediction_horizon": N, "time_step": 300},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    be.setup_optimization(VariableReference(
        states=["T"], controls=["mDot"], inputs=["T_in", "load", "T_upper"],
        parameters=["s_T", "r_mDot", "r_mDot2", "switch"], outputs=["T_out", "switch_test"]))
    cv = {
        "T": V("T", T0, 288.15, 303.15), "mDot": V("mDot", u_prev, 0.0, 0.05),
        "T_in": V("T_in", T_in), "load": V("load", load), "T_upper": V("T_upper", T_upper),
        "s_T": V("s_T", s_T), "r_mDot": V("r_mDot", r_mDot), "r_mDot2": V("r_mDot2", r_mDot2),
        "switch": V("switch", switch), "T_out": V("T_out"), "switch_test": V("switch_test"),
    }
    return be, cv


MHE_KNOWN_INPUTS = {"mDot": 0.22, "load": 0.0, "T_in": 17.0, "T_ambient": 28.0, "T_upper": 22.0}


def mhe_measurements(N=15, ts=200.0, d=2, theta=5.5, T0=25.0, T_wall0=27.0, noise=0.0, seed=0,
                     inputs=None):
    """Synthetic measurements of the estimator example: the RNGRoom model
    (`examples/Estimators/mhe_example.py:142-170`) simulated with the true
    capacity factor ``theta`` (RK4, 50 steps per interval), sampled at the
    collocation times of the past horizon ``[-N ts, 0]``.  Returns
    ``(measured T, measured T_wall)`` on the collocation grid (N*d points)."""
    from agentlib_mpc_amd.optimization_backends.discretization import collocation_polynomial

    u = dict(MHE_KNOWN_INPUTS, **(inputs or {}))
    cp, rho, Cw, Rzw, Rha, Vz = 1005.0, 1.2, 4_569_348.0, 0.0129, 0.1128, 59.0

    def f(x):
        T, Tw = x
        pw = (Tw - T) / Rzw
        dT = (u["load"] + cp * u["mDot"] * (u["T_in"] - T) + pw) / (rho * cp * Vz * theta)
        return np.array([dT, -((Tw - u["T_ambient"]) / Rha + pw) / Cw])

    def advance(x, dt, steps=50):
        h = dt / steps
        for _ in range(steps):
            k1 = f(x); k2 = f(x + h / 2 * k1); k3 = f(x + h / 2 * k2); k4 = f(x + h * k3)
            x = x + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
        return x

    roots = collocation_polynomial(d, "legendre").root[1:]
    x = np.array([T0, T_wall0], float)
    out = []
    for k in range(N):
        for r in roots:
            out.append(advance(x, r * ts))
        x = advance(x, ts)
    meas = np.array(out).T
    if noise:
        meas = meas + np.random.default_rng(seed).normal(scale=noise, size=meas.shape)
    return meas[0], meas[1]


def mhe_room(N=15, ts=200.0, d=2, theta_lb=5.0, theta_ub=6.0, theta_guess=None, w_T=1.0, w_T_wall=0.0,
             measured=None, inputs=None, model="RNGRoomMHE", estimate="theta", mDot_lb=0.0, mDot_ub=1.0,
             solver_options=TIGHT):
    """`examples/Estimators/mhe_example.py:188-228`: backend ``casadi_mhe`` on the
    RNGRoom model, estimating ``full_capacity_from_volume_factor`` (bounds 5..6)
    from zone temperature measurements (state weights T: 1, T_wall: 0).  The
    default model bounds the (cost-free) slack, see :class:`examples.RNGRoomMHE`.
    ``estimate="mDot"`` estimates the supply mass flow per interval instead
    (``estimated_inputs``, `mhe.py:163`) with the capacity factor known."""
    from agentlib_mpc_amd.data_structures.mpc_datamodels import MHEVariableReference

    be = create_optimization_backend({
        "type": "casadi_mhe",
        "model": {"type": f"agentlib_mpc_amd.models.examples.{model}"},
        "discretization_options": {"collocation_order": d, "collocation_method": "legendre",
                                   "prediction_horizon": N, "time_step": ts},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    est_u = estimate == "mDot"
    known = [n for n in MHE_KNOWN_INPUTS if not (est_u and n == "mDot")]
    be.setup_optimization(MHEVariableReference(
        states=["T", "T_wall"], measured_states=["measured_T", "measured_T_wall"],
        weights_states=["weight_T", "weight_T_wall"], estimated_inputs=["mDot"] if est_u else [],
        estimated_parameters=[] if est_u else ["full_capacity_from_volume_factor"], known_inputs=known,
        known_parameters=[], outputs=[]))
    if measured is None:
        measured = mhe_measurements(N=N, ts=ts, d=d)
    u = dict(MHE_KNOWN_INPUTS, **(inputs or {}))
    th = 0.5 * (theta_lb + theta_ub) if theta_guess is None else theta_guess
    cv = {
        "T": V("T", 25.0), "T_wall": V("T_wall", 27.0),
        "full_capacity_from_volume_factor": V("full_capacity_from_volume_factor", th, theta_lb, theta_ub),
        "mDot": V("mDot", u["mDot"], mDot_lb, mDot_ub),
        "measured_T": V("measured_T", [float(v) for v in measured[0]]),
        "measured_T_wall": V("measured_T_wall", [float(v) for v in measured[1]]),
        "weight_T": V("weight_T", w_T), "weight_T_wall": V("weight_T_wall", w_T_wall),
    }
    cv.update({n: V(n, u[n]) for n in known})
    if est_u:
        del cv["full_capacity_from_volume_factor"]
    return be, cv


def rng_room_mpc(N=15, T0=25.0, T_wall0=27.0, u_prev=0.02, T_upper=23.0, load=0.0, solver_options=TIGHT):
    """The MPC module of `examples/Estimators/mhe_example.py:230-268`: backend
    ``casadi`` on the two-state RNGRoom (zone + wall, one control: nx > nu, so
    the kernel factors it with the block chain), N=15, ts=200, Legendre d=2."""
    be = create_optimization_backend({
        "type": "casadi",
        "model": {"type": "agentlib_mpc_amd.models.examples.RNGRoom"},
        "discretization_options": {"collocation_order": 2, "collocation_method": "legendre",
                                   "prediction_horizon": N, "time_step": 200},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    be.setup_optimization(VariableReference(
        states=["T", "T_wall"], controls=["mDot"], inputs=["load", "T_in", "T_ambient", "T_upper"],
        parameters=["full_capacity_from_volume_factor"], outputs=[]))
    cv = {
        "T": V("T", T0, 15.0, 30.0), "T_wall": V("T_wall", T_wall0), "mDot": V("mDot", u_prev, 0.0, 0.1),
        "load": V("load", load), "T_in": V("T_in", 17.0), "T_ambient": V("T_ambient", 28.0),
        "T_upper": V("T_upper", T_upper),
        "full_capacity_from_volume_factor": V("full_capacity_from_volume_factor", 5.5, 1.0, 50.0),
    }
    return be, cv


ROOM_NN_COUPLINGS = (("T_v", 294.15, 285.0, 308.0), ("T_ahu", 295.0, 285.0, 308.0),
                     ("T_CCA_out", 294.15, 285.0, 310.0), ("T_air_out", 294.0, 285.0, 310.0))


def room_nn(N=24, T_air=294.0, T_CCA=294.15, load=100.0, T_amb=299.0, Q_rad=50.0, T_set=295.0,
            T_upper=301.15, T_lower=290.15, q_T=0.0, s_T=1.0, rho=1.0, zbar=None, lam=0.0,
            past_couplings=None, anns=None, solver_options=TIGHT):
    """C5 zone agent: ``RoomCCA`` with two NARX ANNs, backend ``casadi_admm_nn``
    (`examples/three_zone_datadriven_admm/configs/mpc/Room_1.json`: N=24, ts=1800,
    q_T=0, s_T=1, couplings T_v/T_ahu/T_CCA_out/T_air_out).  ``zbar`` / ``lam``
    are per coupling (scalar or length-N trajectory); the synthetic ANNs come
    from :func:`examples.room_cca_anns`."""
    from agentlib_mpc_amd.models import examples as ex

    be = create_optimization_backend({
        "type": "casadi_admm_nn",
        "model": {"type": "agentlib_mpc_amd.models.examples.RoomCCA",
                  "ml_model_sources": anns if anns is not None else ex.room_cca_anns(), "dt": 1800},
        "discretization_options": {"method": "multiple_shooting", "prediction_horizon": N, "time_step": 1800},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    coups = [adt.CouplingEntry(c[0]) for c in ROOM_NN_COUPLINGS]
    be.setup_optimization(adt.VariableReference(
        states=["T_air", "T_CCA_0"], controls=[],
        inputs=["mDot", "mDot_ahu", "d", "T_amb", "Q_rad", "T_set", "T_upper", "T_lower"],
        parameters=["q_T", "s_T"], outputs=[], couplings=coups))
    n = len(be.coupling_grid)
    cv = {
        "T_air": V("T_air", T_air, 280.15, 303.15), "T_CCA_0": V("T_CCA_0", T_CCA, 280.15, 303.15),
        "mDot": V("mDot", 0.1), "mDot_ahu": V("mDot_ahu", 0.025), "d": V("d", load),
        "T_amb": V("T_amb", T_amb), "Q_rad": V("Q_rad", Q_rad), "T_set": V("T_set", T_set),
        "T_upper": V("T_upper", T_upper), "T_lower": V("T_lower", T_lower),
        "q_T": V("q_T", q_T), "s_T": V("s_T", s_T), "penalty_factor": V("penalty_factor", rho),
    }
    for i, (c, (name, init, lb, ub)) in enumerate(zip(coups, ROOM_NN_COUPLINGS)):
        cv[name] = V(name, init, lb, ub)
        zb = init if zbar is None else (zbar[i] if np.ndim(zbar) > 0 else zbar)
        lm = lam[i] if np.ndim(lam) > 0 else lam
        cv[c.mean] = V(c.mean, _vals(zb, n))
        cv[c.multiplier] = V(c.multiplier, _vals(lm, n))
        past = init if past_couplings is None else past_couplings[i]
        cv[c.lagged] = V(c.lagged, past)
    return be, cv


TZ_AHU_COUPLINGS = ("T_ahu_out1", "T_room1", "T_ahu_out2", "T_room2", "T_ahu_out3", "T_room3")
TZ_CCA_COUPLINGS = ("T_v_out", "T_r1", "T_v_out2", "T_r2", "T_v_out3", "T_r3")


def tz_ahu(N=24, rho=1.0, zbar=295.0, lam=0.0, mDot_0=0.025, T_amb=299.0, r_T_v=1.0,
           solver_options=TIGHT):
    """C5 air handling unit: `three_zone_datadriven_admm/configs/mpc/ahu_controller.json`
    (casadi_admm, multiple shooting, N=24, ts=1800; controls T_ahu1..3 in [285, 308],
    outputs W1..3 in [-500, 500]).  ``zbar``/``lam``: scalar or [6][N] per coupling."""
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": {"type": "agentlib_mpc_amd.models.examples.ThreeZoneAHU"},
        "discretization_options": {"method": "multiple_shooting", "prediction_horizon": N, "time_step": 1800},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    coups = [adt.CouplingEntry(n) for n in TZ_AHU_COUPLINGS]
    be.setup_optimization(adt.VariableReference(
        states=[], controls=["T_ahu1", "T_ahu2", "T_ahu3"], inputs=["mDot_0", "T_amb"],
        parameters=["r_T_v"], outputs=["W1", "W2", "W3"], couplings=coups))
    n = len(be.coupling_grid)
    cv = {f"T_ahu{i}": V(f"T_ahu{i}", 295.0, 285.0, 308.0) for i in (1, 2, 3)}
    cv.update({f"W{i}": V(f"W{i}", 0.0, -500.0, 500.0) for i in (1, 2, 3)})
    cv.update({"mDot_0": V("mDot_0", mDot_0), "T_amb": V("T_amb", T_amb), "r_T_v": V("r_T_v", r_T_v),
               "penalty_factor": V("penalty_factor", rho)})
    zb = np.broadcast_to(np.asarray(zbar, float).reshape(-1, 1) if np.ndim(zbar) == 1 else zbar, (6, n))
    lm = np.broadcast_to(np.asarray(lam, float).reshape(-1, 1) if np.ndim(lam) == 1 else lam, (6, n))
    for i, c in enumerate(coups):
        cv[c.name] = V(c.name, 295.0)
        cv[c.mean] = V(c.mean, list(zb[i]))
        cv[c.multiplier] = V(c.multiplier, list(lm[i]))
    return be, cv


def tz_cca(N=24, rho=1.0, zbar=294.15, lam=0.0, mDot_0=0.1, r_T_v=1.0, solver_options=TIGHT):
    """C5 concrete-core supply: `three_zone_datadriven_admm/configs/mpc/cca_controller.json`
    (control T_v in [285, 308], outputs W1..3 in [-1e5, 1e5])."""
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": {"type": "agentlib_mpc_amd.models.examples.TempController"},
        "discretization_options": {"method": "multiple_shooting", "prediction_horizon": N, "time_step": 1800},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    coups = [adt.CouplingEntry(n) for n in TZ_CCA_COUPLINGS]
    be.setup_optimization(adt.VariableReference(
        states=[], controls=["T_v"], inputs=["mDot_0"], parameters=["r_T_v"],
        outputs=["W1", "W2", "W3"], couplings=coups))
    n = len(be.coupling_grid)
    cv = {"T_v": V("T_v", 294.15, 285.0, 308.0), "mDot_0": V("mDot_0", mDot_0), "r_T_v": V("r_T_v", r_T_v),
          "penalty_factor": V("penalty_factor", rho)}
    cv.update({f"W{i}": V(f"W{i}", 0.0, -1e5, 1e5) for i in (1, 2, 3)})
    zb = np.broadcast_to(np.asarray(zbar, float).reshape(-1, 1) if np.ndim(zbar) == 1 else zbar, (6, n))
    lm = np.broadcast_to(np.asarray(lam, float).reshape(-1, 1) if np.ndim(lam) == 1 else lam, (6, n))
    for i, c in enumerate(coups):
        cv[c.name] = V(c.name, 294.15)
        cv[c.mean] = V(c.mean, list(zb[i]))
        cv[c.multiplier] = V(c.multiplier, list(lm[i]))
    return be, cv


def fixture_mpc(N=5, T0=298.16, disturbance=270.0, u_prev=0.02, solver_options=TIGHT, model=None,
                backend="mi355x", T_lb=-np.inf, T_ub=np.inf):
    """The reference's MPC module test (`tests/test_mpc.py:121-146`): backend ``casadi``
    with default discretization options (collocation, Legendre d=3), time step 900 s,
    horizon 5, on the test-suite model (`tests/fixtures/casadi_test_model.py`); the module
    config declares state, control and disturbance only (parameters at model defaults).
    ``T_lb`` / ``T_ub``: bounds on the (unstable) state -- tight ones make the NLP infeasible,
    the restoration-phase cases of the parity tests."""
    be = create_optimization_backend({
        "type": backend,
        "model": model or {"type": "agentlib_mpc_amd.models.examples.FixtureModel"},
        "discretization_options": {"prediction_horizon": N, "time_step": 900},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    be.setup_optimization(VariableReference(states=["state"], controls=["myctrl"], inputs=["disturbance"],
                                            parameters=[], outputs=[]))
    cv = {"state": V("state", T0, T_lb, T_ub), "myctrl": V("myctrl", u_prev, 0.0, 1.0),
          "disturbance": V("disturbance", disturbance)}
    return be, cv


def fixture_admm(N=5, T0=298.16, disturbance=270.0, rho=10.0, zbar=298.16, lam=0.0, coupling=298.16,
                 solver_options=TIGHT, model=None):
    """The reference's ADMM module test (`tests/test_admm.py:24-58`): backend ``casadi_admm``
    on the test-suite model with ``myout`` as consensus coupling (value 298.16 for the first
    agent, 295 for the second), penalty factor 10 (`modules/dmpc/admm/admm.py:72-77`)."""
    be = create_optimization_backend({
        "type": "mi355x_admm",
        "model": model or {"type": "agentlib_mpc_amd.models.examples.FixtureModel"},
        "discretization_options": {"prediction_horizon": N, "time_step": 900},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    c = adt.CouplingEntry("myout")
    be.setup_optimization(adt.VariableReference(
        states=["state"], controls=["myctrl"], inputs=["disturbance"], parameters=[], outputs=[],
        couplings=[c]))
    n = len(be.coupling_grid)
    cv = {"state": V("state", T0), "myctrl": V("myctrl", 0.02, 0.0, 1.0),
          "disturbance": V("disturbance", disturbance), "myout": V("myout", coupling),
          c.mean: V(c.mean, _vals(zbar, n)), c.multiplier: V(c.multiplier, _vals(lam, n)),
          "penalty_factor": V("penalty_factor", rho)}
    return be, cv


def cubic_room(N=4, T0=295.0, solver_options=TIGHT):
    """Restoration-phase case (``models/examples.CubicRoom``): backend ``casadi``, collocation
    Legendre d=2, N=4, ts=10; the cubic rows start at the middle of their variable's bounds,
    in the basin of the local infeasibility minimum z = -1, so the filter line search fails
    and the feasibility restoration phase moves them to the root z = 2.279."""
    be = create_optimization_backend({
        "type": "mi355x",
        "model": {"type": "agentlib_mpc_amd.models.examples.CubicRoom"},
        "discretization_options": {"collocation_order": 2, "prediction_horizon": N, "time_step": 10},
        "solver": {"name": "ipopt", "options": solver_options},
    })
    be.setup_optimization(VariableReference(states=["T"], controls=["u"], inputs=[], parameters=[], outputs=[]))
    cv = {"T": V("T", T0), "u": V("u", 0.0, 0.0, 1.0)}
    return be, cv


BUILDERS: Dict[str, Callable[..., Tuple[object, dict]]] = {
    "one_room": one_room,
    "admm_room": admm_room,
    "admm_ahu": admm_ahu,
    "exchange_room": exchange_room,
    "exchange_supply": exchange_supply,
    "room_nn": room_nn,
    "tz_ahu": tz_ahu,
    "tz_cca": tz_cca,
    "fixture_mpc": fixture_mpc,
    "fixture_admm": fixture_admm,
    "cubic_room": cubic_room,
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
    # the benchmark structures plus the test-only variants (copy-lifted NARX, N=23)
    variants = dict(BUILDERS)
    variants["room_nn_n23"] = lambda: room_nn(N=23)
    variants["exchange_room_rk"] = lambda: exchange_room(integrator="rk")
    variants["one_room_radau3"] = lambda: one_room(d=3, method="radau")
    variants["one_room_du"] = lambda: one_room(r_delta_mDot=0.1)
    variants["one_room_switch"] = lambda: one_room_switch()
    variants["room_nn_n8"] = lambda: room_nn(N=8)      # C5 ADMM fixture (tests/golden/c5_admm_N8.json)
    variants["tz_ahu_n8"] = lambda: tz_ahu(N=8)
    variants["tz_cca_n8"] = lambda: tz_cca(N=8)
    variants["mhe_room"] = lambda: mhe_room()
    variants["mhe_room_u"] = lambda: mhe_room(estimate="mDot")
    variants["rng_room_mpc"] = lambda: rng_room_mpc()
    from concurrent.futures import ThreadPoolExecutor

    probs = {name: fn()[0].problem for name, fn in variants.items()}
    jobs = int(os.environ.get("MPCX_BUILD_JOBS", "4"))
    label = {None: "", native.SMALL_FLEET: " small-fleet", native.MID_FLEET: " one-wave-per-SIMD",
             native.WIDE_FLEET: " 20-agents-per-CU"}
    with ThreadPoolExecutor(max_workers=jobs) as ex:  # hipcc processes: one per code object
        # the one-wave-per-SIMD and 20-agents-per-CU builds after the main ones (they read the main
        # build's occupancy)
        for group in ((None, native.SMALL_FLEET), (native.MID_FLEET, native.WIDE_FLEET)):
            futs = {(name, v): ex.submit(native.compile_model, pr.gen, False, v)
                    for name, pr in probs.items() for v in group}
            for (name, v), fut in futs.items():
                path = fut.result()
                if v is None:
                    paths[name] = path
                if verbose:
                    print(f"[mpcx] {name}{label[v]}: {path.name if path else '-'}")
    # test builds of the filter (tests/test_gpu_ipm.py::test_gpu_filter_matches_oracle): a small LDS
    # part, so that the cubic_room case spills, and a small total capacity, so that it overflows
    saved = os.environ.get("MPCX_DEFINES")
    try:
        gen = cubic_room()[0].problem.gen
        for defines, _cap in FILTER_TEST_BUILDS.values():
            os.environ["MPCX_DEFINES"] = defines
            for v in (None, native.SMALL_FLEET, native.MID_FLEET, native.WIDE_FLEET):
                path = native.compile_model(gen, False, v)
                if verbose:
                    print(f"[mpcx] cubic_room {defines}{label[v]}: {path.name if path else '-'}")
    finally:
        if saved is None:
            os.environ.pop("MPCX_DEFINES", None)
        else:
            os.environ["MPCX_DEFINES"] = saved
    return paths


#: the filter's capacity (csrc/mpcx_ipm.hip MAXF + FSPILL; oracle/ipm.py max_filter)
FILTER_CAPACITY = 1024
#: filter test builds (MPCX_DEFINES) and the oracle cap each matches: "spill" keeps 8 entries in LDS
#: and the rest in the spill list (capacity unchanged), "capped" holds 12 in all (8 + 4)
FILTER_TEST_BUILDS = {"spill": ("MPCX_MAXF=8", FILTER_CAPACITY), "capped": ("MPCX_MAXF=8,MPCX_FSPILL=4", 12)}


# ---------------------------------------------------------------------------
# ADMM fleets (C2 scaled, C4)
# ---------------------------------------------------------------------------
C2_ROOMS = [  # (d, T0) of examples/4_Room_ADMM_Coordinator/configs/room_{1..4}_admm.json
    (150.0, 296.0), (100.0, 298.0), (50.0, 301.0), (10.0, 303.0)]
C4_ROOMS = C2_ROOMS  # examples/exchange_admm/configs/room_{1..4}_admm.json


def _class_inputs(be, cv, overrides, n):
    from agentlib_mpc_amd.optimization_backends.problem import fleet_nlp_inputs

    if not overrides:
        overrides = {next(iter(cv)): np.full(n, cv[next(iter(cv))].value, float)}
    return fleet_nlp_inputs(be.problem, cv, {k: np.asarray(v, float) for k, v in overrides.items()})


def c2_fleet_classes(n_blocks=1, N=10, rho=0.4, seed=None, block_offset=0, solver_options=TIGHT):
    """Coordinated consensus fleet: ``n_blocks`` x (4 rooms + 1 air handler) of
    `examples/4_Room_ADMM_Coordinator` (block 0 = the example's values; further
    blocks d~U(10,150), T0~U(296,303) from ``default_rng([seed, block])``).
    Returns the FleetClass list [rooms, air handlers]."""
    from agentlib_mpc_amd.admm.fleet import FleetClass

    d, T0, aliases = [], [], []
    for b in range(block_offset, block_offset + n_blocks):
        rng = np.random.default_rng([seed, b]) if seed is not None else None
        for i, (d_i, t_i) in enumerate(C2_ROOMS):
            if b == 0 or rng is None:
                d.append(d_i); T0.append(t_i)
            else:
                d.append(rng.uniform(10.0, 150.0)); T0.append(rng.uniform(296.0, 303.0))
            aliases.append(f"mDot{i + 1}_coupling_b{b}")
    be_r, cv_r = admm_room(N=N, rho=rho, solver_options=solver_options)
    nr = 4 * n_blocks
    rooms = FleetClass("room", be_r, _class_inputs(be_r, cv_r, {"T": T0, "d": d}, nr),
                       aliases={"mDot": aliases}, initial={"mDot": 0.02})
    rooms.plant = (cv_r, {"T": list(T0), "d": list(d)}, ("T",))  # closed-loop measurement update
    be_a, cv_a = admm_ahu(N=N, rho=rho, solver_options=solver_options)
    blocks = range(block_offset, block_offset + n_blocks)
    ahu = FleetClass("ahu", be_a, _class_inputs(be_a, cv_a, {}, n_blocks),
                     aliases={f"mDot_out_{i + 1}": [f"mDot{i + 1}_coupling_b{b}" for b in blocks]
                              for i in range(4)},
                     initial={f"mDot_out_{i + 1}": 0.01 for i in range(4)})
    return [rooms, ahu]


def value_at(problem, w: np.ndarray, var: str, t: float) -> np.ndarray:
    """Every agent's value of variable ``var`` at grid time ``t`` from reference-layout
    solutions ``w`` [n, nw] (the predicted state one control interval ahead: the measurement
    of a synthetic plant that follows the model)."""
    for _, grid, rows, index in problem.marshal.vars:
        if index is None:
            continue
        for row in rows:
            if row[1] == var:
                j = next(k for k, g in enumerate(grid) if abs(float(g) - t) <= 1e-9 * max(1.0, abs(t)))
                return w[:, index[row[0]][j]]
    raise KeyError(var)


def advance_plant(fleet, t: float):
    """Closed loop of a coordinated fleet (the reference's agents re-measuring before the next
    control step): every class built with a ``plant`` (template variables, measured values,
    state names) takes its states' predicted values at ``t`` as the next measurements and
    uploads the new NLP inputs (``ADMMFleet.set_inputs``); the warm starts, means and
    multipliers stay resident (the coordinator shifts the latter at the start of the round)."""
    for c in fleet.classes:
        plant = getattr(c, "plant", None)
        if plant is None:
            continue
        cv, vals, states = plant
        w = fleet.solutions(c.name)
        for name in states:
            vals[name] = list(value_at(c.backend.problem, w, name, t))
        p, lbw, ubw, _ = _class_inputs(c.backend, cv, vals, c.n)
        fleet.set_inputs(c.name, p, lbw, ubw)


def split_range(total: int, rank: int, world: int):
    """[lo, hi) of rank's contiguous share of ``total`` items (the first total % world ranks
    hold one more)."""
    base, extra = divmod(int(total), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def c4_fleet_classes(n_rooms=4, n_supply=1, N=10, rho=1e4, seed=None, solver_options=TIGHT, rank=0, world=1):
    """Exchange fleet of `examples/exchange_admm` (one alias ``mDot_coupling``):
    rooms (first four = the example's values, further d~U(10,150), T0~U(296,303))
    and supply units (penalty 0.1).  With ``world`` > 1 the fleet of ``n_rooms`` rooms and
    ``n_supply`` supply units is split over the ranks and this returns ``rank``'s share
    (the same agents as the one-rank fleet, for strong scaling)."""
    from agentlib_mpc_amd.admm.fleet import FleetClass

    rng = np.random.default_rng(seed)
    d, T0 = [], []
    for i in range(n_rooms):
        if i < 4 and seed is None:
            d.append(C4_ROOMS[i][0]); T0.append(C4_ROOMS[i][1])
        else:
            d.append(rng.uniform(10.0, 150.0)); T0.append(rng.uniform(296.0, 303.0))
    if world > 1:
        lo, hi = split_range(n_rooms, rank, world)
        d, T0, n_rooms = d[lo:hi], T0[lo:hi], hi - lo
        lo, hi = split_range(n_supply, rank, world)
        n_supply = hi - lo
    classes = []
    if n_rooms:
        be_r, cv_r = exchange_room(N=N, rho=rho, solver_options=solver_options)
        classes.append(FleetClass("room", be_r, _class_inputs(be_r, cv_r, {"T": T0, "d": d}, n_rooms),
                                  aliases={"mDot_out": "mDot_coupling"}, initial={"mDot_out": 0.02}))
    if n_supply:
        be_s, cv_s = exchange_supply(N=N, rho=rho, solver_options=solver_options)
        classes.append(FleetClass("supply", be_s, _class_inputs(be_s, cv_s, {}, n_supply),
                                  aliases={"mDot_out": "mDot_coupling"}, initial={"mDot_out": 0.02}))
    return classes


def c5_fleet_classes(n_blocks=1, N=24, rho=1.0, seed=None, block_offset=0, solver_options=TIGHT):
    """Coordinated consensus fleet of `examples/three_zone_datadriven_admm`:
    ``n_blocks`` x (3 NARX zones + 1 AHU + 1 CCA supply).  Couplings per zone i
    of block b (`configs/mpc/Room_{i}.json`, `ahu_controller.json`,
    `cca_controller.json`): T_v <-> CCA T_v_out{i} (alias T_coupling{i}), T_ahu <->
    AHU T_ahu_out{i} (T_coupling_ahu{i}), T_CCA_out <-> CCA T_r{i} (T_rucklauf{i}),
    T_air_out <-> AHU T_room{i} (T_airin{i}).  Block 0 = the example's values;
    further blocks draw T_air~U(292,297), d~U(50,200), T_amb~U(295,303),
    Q_rad~U(0,50) from ``default_rng([seed, block])``.  (With the trained networks a
    zone is infeasible -- its air temperature leaves the state bounds -- once the solar
    gain reaches ~100-200 W/m2 on a warm day, so the solar input stays below that.)"""
    from agentlib_mpc_amd.admm.fleet import FleetClass

    blocks = list(range(block_offset, block_offset + n_blocks))
    vals = {"T_air": [], "d": [], "T_amb": [], "Q_rad": []}
    for b in blocks:
        rng = np.random.default_rng([seed, b]) if seed is not None else None
        for _ in range(3):
            if b == 0 or rng is None:
                vals["T_air"].append(294.0); vals["d"].append(100.0)
                vals["T_amb"].append(299.0); vals["Q_rad"].append(50.0)
            else:
                vals["T_air"].append(rng.uniform(292.0, 297.0)); vals["d"].append(rng.uniform(50.0, 200.0))
                vals["T_amb"].append(rng.uniform(295.0, 303.0)); vals["Q_rad"].append(rng.uniform(0.0, 50.0))
    be_r, cv_r = room_nn(N=N, rho=rho, solver_options=solver_options)
    nz = 3 * n_blocks
    zone_alias = lambda pre: [f"{pre}{i + 1}_b{b}" for b in blocks for i in range(3)]  # noqa: E731
    rooms = FleetClass("zone", be_r, _class_inputs(be_r, cv_r, vals, nz),
                       aliases={"T_v": zone_alias("T_coupling"), "T_ahu": zone_alias("T_coupling_ahu"),
                                "T_CCA_out": zone_alias("T_rucklauf"), "T_air_out": zone_alias("T_airin")},
                       initial={"T_v": 294.15, "T_ahu": 295.0, "T_CCA_out": 294.15, "T_air_out": 294.0})
    rooms.plant = (cv_r, {k: list(v) for k, v in vals.items()}, ("T_air",))
    be_a, cv_a = tz_ahu(N=N, rho=rho, solver_options=solver_options)
    ahu_al = {}
    for i in range(3):
        ahu_al[f"T_ahu_out{i + 1}"] = [f"T_coupling_ahu{i + 1}_b{b}" for b in blocks]
        ahu_al[f"T_room{i + 1}"] = [f"T_airin{i + 1}_b{b}" for b in blocks]
    ahu = FleetClass("ahu", be_a, _class_inputs(be_a, cv_a, {}, n_blocks), aliases=ahu_al,
                     initial={k: 295.0 for k in ahu_al})
    be_c, cv_c = tz_cca(N=N, rho=rho, solver_options=solver_options)
    cca_al = {}
    for i, (vo, tr) in enumerate((("T_v_out", "T_r1"), ("T_v_out2", "T_r2"), ("T_v_out3", "T_r3"))):
        cca_al[vo] = [f"T_coupling{i + 1}_b{b}" for b in blocks]
        cca_al[tr] = [f"T_rucklauf{i + 1}_b{b}" for b in blocks]
    cca = FleetClass("cca", be_c, _class_inputs(be_c, cv_c, {}, n_blocks), aliases=cca_al,
                     initial={k: 294.15 for k in cca_al})
    return [rooms, ahu, cca]
