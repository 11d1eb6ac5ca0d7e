"""Generate tests/golden/c5_admm_N<N>.json (N = 8, and the example's horizon N = 24 with
``python tests/golden/make_c5_admm_golden.py 24``): the coordinated ADMM round of one
three-zone block (3 NARX zones + AHU + CCA) computed by the ORACLE (hand
restatements `oracle/nlps.py` + oracle IPM + the coordinator-loop restatement
`oracle/admm.py`), N=8, rho=1, to the stopping rule of
`three_zone_datadriven_admm/configs/coordinator.json` (admm_iter_max 50, absolute
criterion primal_tol = dual_tol = 0.04), with the trained networks of `models/data/`.
The oracle takes minutes on a CPU, so the GPU test reads this fixture.

Run from the repository root: ``python tests/golden/make_c5_admm_golden.py``.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]

import numpy as np  # noqa: E402

from agentlib_mpc_amd.models import examples as ex  # noqa: E402
from oracle import admm as oadmm  # noqa: E402
from tests.admm_cases import C5Oracle  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 50  # the example's admm_iter_max
RHO = 1.0


def main():
    orc = C5Oracle(N, ex.room_cca_anns())
    state, hist, it, conv = oadmm.coordinated_round(
        orc.participation, orc.initial, orc, RHO, N, ITERS, primal_tol=0.04, dual_tol=0.04,
        use_relative_tolerances=False, T=N)
    out = {"N": N, "iterations": it, "converged": conv, "rho": RHO, "admm_iter_max": ITERS,
           "history": [[float(a), float(b)] for a, b, _ in hist],
           "means": {al: list(map(float, v.mean)) for al, v in state["vars"].items()},
           "mult_ahu": {al: list(map(float, state["vars"][al].mult["ahu"])) for al in orc.ahu_al}}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"c5_admm_N{N}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, hist)


if __name__ == "__main__":
    main()
