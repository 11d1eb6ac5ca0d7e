"""Diagnostic: C5 coordinated ADMM on a small random fleet — residual history,
per-class solve statuses and non-finite trajectories."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from agentlib_mpc_amd import benchmarks as bm  # noqa: E402
from agentlib_mpc_amd.admm.fleet import ADMMFleet  # noqa: E402
from agentlib_mpc_amd.runtime.native import stats_to_dicts  # noqa: E402


def main():
    nb = int(os.environ.get("BLOCKS", "32"))
    iters = int(os.environ.get("ITERS", "50"))
    tol = float(os.environ.get("TOL", "1e-4"))
    opts = {"ipopt": {"tol": tol, "max_iter": int(os.environ.get("MAXIT", "100"))}}
    classes = bm.c5_fleet_classes(n_blocks=nb, N=24, seed=20261015 + 5, solver_options=opts)
    fl = ADMMFleet(classes, device=torch.device("cuda"))
    out = fl.run_coordinated(1.0, admm_iter_max=iters, use_relative_tolerances=False, primal_tol=0.04,
                             dual_tol=0.04)
    for i, r in enumerate(out["records"]):
        print(i, r.primal_residual, r.dual_residual, flush=True)
    print("iterations", out["iterations"], "converged", out["converged"], "ok", out["converged_solves"])
    for c in classes:
        st = stats_to_dicts(c.ST.cpu().numpy().tobytes())
        codes = {}
        for s in st:
            codes[s["return_status"]] = codes.get(s["return_status"], 0) + 1
        w = c.W.cpu().numpy()
        print(c.name, codes, "max iters", max(s["iter_count"] for s in st),
              "non-finite agents", int((~np.isfinite(w)).any(axis=1).sum()))
    tr = fl.trajectories()
    bad = [k for k, v in tr.items() if not np.all(np.isfinite(v))]
    print("non-finite means", len(bad), bad[:5])


if __name__ == "__main__":
    main()
