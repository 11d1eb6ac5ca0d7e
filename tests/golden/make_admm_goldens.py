"""Generate the coordinated-ADMM oracle fixtures read by tests/test_gpu_admm.py:

* ``c2_admm_N10.json`` — examples/4_Room_ADMM_Coordinator (4 rooms + air handler, collocation
  d=3, N=10, ts=60, rho=0.4, absolute criterion 0.002 / 0.1, admm_iter_max 40;
  `configs/coordinator.json:7-18`) run to its stopping rule;
* ``c5_admm_N24.json`` — examples/three_zone_datadriven_admm (3 NARX zones + AHU + CCA,
  N=24, ts=1800, rho=1, absolute criterion 0.04 / 0.04, admm_iter_max 50;
  `configs/coordinator.json:5-20`) at the config horizon.

Both are computed by the ORACLE only: hand restatements `oracle/nlps.py`, the oracle IPM
(tight tolerance, no acceptable stop: the product side runs with the same settings) and the
coordinator-loop restatement ``oracle.admm.coordinated_round``.  The agents of one ADMM
iteration are solved in parallel, one worker process per agent (each keeps its own warm
start, as the reference backend does).  Minutes of CPU, hence committed fixtures.

Run from the repository root: ``python tests/golden/make_admm_goldens.py [c2] [c5]``.
"""
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def _make_oracle(kind, N):
    from tests.admm_cases import C2Oracle, C5Oracle
    from agentlib_mpc_amd import benchmarks as bm

    if kind == "c2":
        return C2Oracle(N, bm.C2_ROOMS)
    from agentlib_mpc_amd.models import examples as ex

    orc = C5Oracle(N, ex.room_cca_anns())
    orc.allow_failed = True  # a supply agent's local solve may stop unsuccessfully; the round goes on
    return orc


def _worker(kind, N, conn):
    orc = _make_oracle(kind, N)
    while True:
        msg = conn.recv()
        if msg is None:
            conn.send(orc.failed)  # local solves that stopped unsuccessfully
            break
        ag, inp, rho = msg
        conn.send(orc(ag, inp, rho))


def run(kind, N, rho, iters, **crit):
    orc = _make_oracle(kind, N)
    agents = list(orc.participation)
    pipes = {}
    procs = []
    for ag in agents:
        a, b = mp.Pipe()
        p = mp.Process(target=_worker, args=(kind, N, b), daemon=True)
        p.start()
        pipes[ag] = a
        procs.append(p)

    def solve_batch(reqs, rho_):
        for ag, inp in reqs:
            pipes[ag].send((ag, inp, rho_))
        return [pipes[ag].recv() for ag, _ in reqs]

    from oracle import admm as oadmm

    t0 = time.time()
    T = 3 * N if kind == "c2" else N
    state, hist, it, conv = oadmm.coordinated_round(orc.participation, orc.initial, None, rho, N, iters,
                                                    T=T, solve_batch=solve_batch, **crit)
    failed = {}
    for ag in agents:
        pipes[ag].send(None)
        failed[ag] = pipes[ag].recv()
    for p in procs:
        p.join()
    out = {"N": N, "iterations": it, "converged": conv, "rho": rho, "admm_iter_max": iters, "criterion": crit,
           "solver": {"tol": orc.tol, "acceptable_iter": 0, "max_iter": 500},
           "failed_local_solves": failed,
           "history": [[float(a), float(b), float(c)] for a, b, c in hist],
           "means": {al: list(map(float, v.mean)) for al, v in state["vars"].items()}}
    path = os.path.join(HERE, f"{kind}_admm_N{N}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, f"{it} iterations, converged={conv}, {time.time() - t0:.0f}s", flush=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["c2", "c5"]
    if "c2" in which:
        run("c2", 10, 0.4, 40, primal_tol=0.002, dual_tol=0.1, use_relative_tolerances=False)
    if "c5" in which:
        run("c5", 24, 1.0, 50, primal_tol=0.04, dual_tol=0.04, use_relative_tolerances=False)
