"""Diagnostic: where the C5 coordinated-ADMM iteration time goes (per class solve)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]
import numpy as np
import torch


def main():
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.admm.fleet import ADMMFleet
    from agentlib_mpc_amd.admm.ops import NativeADMMOps
    from agentlib_mpc_amd.runtime.native import stats_to_dicts

    nb = int(os.environ.get("BLOCKS", "342"))
    classes = bm.c5_fleet_classes(n_blocks=nb, N=24, seed=20261015 + 5, solver_options={"ipopt": {}})
    times = {c.name: [] for c in classes}

    class TimedOps(NativeADMMOps):
        def solve(self, cls, active=None):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            super().solve(cls, active)
            torch.cuda.synchronize()
            times[cls.name].append(time.perf_counter() - t0)

    fl = ADMMFleet(classes, ops=TimedOps())
    t0 = time.perf_counter()
    out = fl.run_coordinated(1.0, admm_iter_max=int(os.environ.get("ITERS", "10")), use_relative_tolerances=False,
                             primal_tol=0.04, dual_tol=0.04)
    wall = time.perf_counter() - t0
    print("iterations", out["iterations"], "wall s", wall)
    for c in classes:
        st = stats_to_dicts(c.ST.cpu().numpy().tobytes())
        it = np.array([s["iter_count"] for s in st])
        tr = np.array([s["n_trials"] for s in st])
        sts = sorted({s["return_status"] for s in st})
        print(f"{c.name:5s} n={c.n} ms/solve-launch p50={1e3*np.median(times[c.name]):.2f} max={1e3*max(times[c.name]):.2f} "
              f"iters p50={np.median(it)} max={it.max()} trials max={tr.max()} statuses={sts} "
              f"gen={c.backend.problem.gen.dims} bordered={c.backend.problem.gen.bordered_rows}")
    rec = out["records"]
    print("residuals", [(round(r.primal_residual, 4), round(r.dual_residual, 4)) for r in rec])


if __name__ == "__main__":
    main()
