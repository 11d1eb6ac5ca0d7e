"""Deterministic result files written by the product writers (CPU, no solve): the
backend results + stats files (`core/casadi_backend.py:263-323`), the ADMM backend's
per-iteration files (`casadi_/admm.py:364-424`) and the coordinator's residual file
(`admm_coordinator.py:437-465`).  `tests/golden/make_reader_goldens.py` reads them with
the reference's own readers; `tests/test_result_files.py` pins the writers to the
committed copies under `tests/golden/result_files/`."""

from __future__ import annotations

import pathlib

from agentlib_mpc_amd import benchmarks as bm
from agentlib_mpc_amd.admm.fleet import ADMMFleet, IterationRecord

FILES = ("mpc/room.csv", "mpc/stats_room.csv", "admm/admm.csv", "admm/stats_admm.csv", "residuals.csv")
MPC_STEPS = (100.0, 400.0)
ADMM_STEPS = ((0.0, 3), (120.0, 2), (240.0, 1))


def _results(be, cv, now=0.0):
    prob = be.problem
    mi = prob.mpc_inputs(cv, now)
    mi.update(prob.initial_guess(mi))
    p, lbw, ubw, w0 = prob.nlp_inputs(mi)
    stats = {"success": True, "return_status": "Solve_Succeeded", "iter_count": 7, "obj": 1.5}
    return prob.make_results(mi, w0, stats)


def write_all(root) -> pathlib.Path:
    root = pathlib.Path(root)
    (root / "mpc").mkdir(parents=True, exist_ok=True)
    (root / "admm").mkdir(parents=True, exist_ok=True)
    be, cv = bm.one_room(N=4)
    be.config.results_file, be.config.save_results = root / "mpc" / "room.csv", True
    for now in MPC_STEPS:
        be.save_result_df(_results(be, cv, now), now)
    be, cv = bm.exchange_room(N=4)
    be.config.results_file, be.config.save_results = root / "admm" / "admm.csv", True
    r = _results(be, cv)
    for now, n_it in ADMM_STEPS:
        for _ in range(n_it):
            be.save_result_df(r, now)
    recs = [IterationRecord(1.0, 2.0, 0.4, wall_time=0.01), IterationRecord(0.5, 0.25, 0.8, wall_time=0.02)]
    ADMMFleet.save_stats(None, root / "residuals.csv", 0.0, recs)
    ADMMFleet.save_stats(None, root / "residuals.csv", 60.0, recs[:1])
    return root
