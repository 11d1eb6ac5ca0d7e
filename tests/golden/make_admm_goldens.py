"""Generate the coordinated-ADMM oracle fixtures read by tests/test_gpu_admm.py:

* ``c2_admm_N10.json`` — examples/4_Room_ADMM_Coordinator (4 rooms + air handler, collocation
  d=3, N=10, ts=60, rho=0.4, absolute criterion 0.002 / 0.1, admm_iter_max 40;
  `configs/coordinator.json:7-18`) run to its stopping rule;
* ``c5_admm_N8.json`` / ``c5_admm_N24.json`` — examples/three_zone_datadriven_admm (3 NARX zones + AHU + CCA,
  N=8 and the config horizon N=24, ts=1800, rho=1, absolute criterion 0.04 / 0.04, admm_iter_max 50;
  `configs/coordinator.json:5-20`);
* ``c2_admm_N10_b3.json`` — block 3 of the bench's scaled C2 fleet (synthetic rooms drawn as
  ``benchmarks.c2_fleet_classes(seed=20261015 + 1)`` draws them), same coordinator settings,
  local solves at the reference's IPOPT settings (tol 1e-4, acceptable level 0.1 over 5
  iterations) as in the bench leg: a block that stops at the iteration cap.

All are computed by the ORACLE only: hand restatements `oracle/nlps.py`, the oracle IPM
(tight tolerance, no acceptable stop, unless stated: the product side runs with the same settings) and the
coordinator-loop restatement ``oracle.admm.coordinated_round``.  The agents of one ADMM
iteration are solved in parallel, one worker process per agent (each keeps its own warm
start, as the reference backend does).  Minutes of CPU, hence committed fixtures.

Run from the repository root: ``python tests/golden/make_admm_goldens.py [c2] [c5n8] [c5] [c2b3]``.
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


#: the reference's IPOPT settings (`casadi_utils.py:197-206`), as tests/test_gpu_ipm.py
REFERENCE_OPTS = dict(tol=1e-4, max_iter=100, acceptable_tol=0.1, acceptable_iter=5,
                      acceptable_constr_viol_tol=1.0, acceptable_compl_inf_tol=1.0)
#: the bench's scaled C2 fleet (bench.py c2_admm leg: seed 20261015 + 1)
C2_FLEET_SEED = 20261015 + 1


def c2_block_rooms(seed, block):
    """(d, T0) of the four rooms of synthetic block ``block`` of
    ``benchmarks.c2_fleet_classes(seed=seed)`` (same generator, same draw order)."""
    rng = np.random.default_rng([seed, block])
    out = []
    for _ in range(4):
        d = rng.uniform(10.0, 150.0)
        out.append((d, rng.uniform(296.0, 303.0)))
    return out


def _make_oracle(kind, N, block=None):
    from tests.admm_cases import C2Oracle, C5Oracle
    from agentlib_mpc_amd import benchmarks as bm

    if kind == "c2":
        if block is None:
            return C2Oracle(N, bm.C2_ROOMS)
        orc = C2Oracle(N, c2_block_rooms(C2_FLEET_SEED, block))
        orc.options = REFERENCE_OPTS  # the bench leg's local solves
        orc.allow_failed = True
        return orc
    from agentlib_mpc_amd.models import examples as ex

    orc = C5Oracle(N, ex.room_cca_anns())
    orc.allow_failed = True  # a supply agent's local solve may stop unsuccessfully; the round goes on
    return orc


def _worker(kind, N, conn, block=None):
    orc = _make_oracle(kind, N, block)
    while True:
        msg = conn.recv()
        if msg is None:
            conn.send(orc.failed)  # local solves that stopped unsuccessfully
            break
        ag, inp, rho = msg
        out = orc(ag, inp, rho)
        conn.send((out, orc.log[-1][1:]))


def run(kind, N, rho, iters, block=None, **crit):
    orc = _make_oracle(kind, N, block)
    agents = list(orc.participation)
    pipes = {}
    procs = []
    for ag in agents:
        a, b = mp.Pipe()
        p = mp.Process(target=_worker, args=(kind, N, b, block), daemon=True)
        p.start()
        pipes[ag] = a
        procs.append(p)

    solves = []  # per ADMM iteration: {agent: [status, IPM iterations]}

    def solve_batch(reqs, rho_):
        for ag, inp in reqs:
            pipes[ag].send((ag, inp, rho_))
        got = [pipes[ag].recv() for ag, _ in reqs]
        solves.append({ag: list(r[1]) for (ag, _), r in zip(reqs, got)})
        return [r[0] for r in got]

    from oracle import admm as oadmm

    t0 = time.time()
    T = 3 * N if kind == "c2" else N
    trace = []
    state, hist, it, conv = oadmm.coordinated_round(orc.participation, orc.initial, None, rho, N, iters,
                                                    T=T, solve_batch=solve_batch, trace=trace, **crit)
    failed = {}
    for ag in agents:
        pipes[ag].send(None)
        failed[ag] = pipes[ag].recv()
    for p in procs:
        p.join()
    out = {"N": N, "iterations": it, "converged": conv, "rho": rho, "admm_iter_max": iters, "criterion": crit,
           "solver": dict(orc.options) if orc.options else {"tol": orc.tol, "acceptable_iter": 0, "max_iter": 500},
           "failed_local_solves": failed,
           "history": [[float(a), float(b), float(c)] for a, b, c in hist],
           "means": {al: list(map(float, v.mean)) for al, v in state["vars"].items()},
           # per iteration: every agent's local solve (status, IPM iterations) and the means after it
           "local_solves": solves, "mean_history": trace}
    if block is not None:
        out["block"], out["seed"] = block, C2_FLEET_SEED
    path = os.path.join(HERE, f"{kind}_admm_N{N}" + (f"_b{block}" if block is not None else "") + ".json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(path, f"{it} iterations, converged={conv}, {time.time() - t0:.0f}s", flush=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["c2", "c5"]
    if "c2" in which:
        run("c2", 10, 0.4, 40, primal_tol=0.002, dual_tol=0.1, use_relative_tolerances=False)
    if "c2b3" in which:  # a block of the bench's scaled fleet that stalls above the primal tolerance
        run("c2", 10, 0.4, 40, block=3, primal_tol=0.002, dual_tol=0.1, use_relative_tolerances=False)
    if "c5n8" in which:
        run("c5", 8, 1.0, 50, primal_tol=0.04, dual_tol=0.04, use_relative_tolerances=False)
    if "c5" in which:
        run("c5", 24, 1.0, 50, primal_tol=0.04, dual_tol=0.04, use_relative_tolerances=False)
