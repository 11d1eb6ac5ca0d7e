"""Diagnostic: C2 coordinated leg wall time, fleet driver before/after the participation
change (fleet_old.py = the previous driver), alternating, same process."""
import importlib
import sys
import time

sys.path[:0] = [".", "agentlib-mpc_amd"]
import torch  # noqa: E402

from agentlib_mpc_amd import benchmarks as bm  # noqa: E402

dev = torch.device("cuda:0")
for rep in range(2):
    for name in ("fleet_old", "fleet"):
        mod = importlib.import_module(f"agentlib_mpc_amd.admm.{name}")
        classes = bm.c2_fleet_classes(n_blocks=1024, N=10, seed=20261015 + 1, block_offset=0,
                                      solver_options={"ipopt": {}})
        fl = mod.ADMMFleet(classes, device=dev)
        for c in classes:
            c.native.reserve(c.n)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        out = fl.run_coordinated(0.4, admm_iter_max=40, use_relative_tolerances=False, primal_tol=0.002, dual_tol=0.1)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        out2 = fl.run_coordinated(0.4, admm_iter_max=40, use_relative_tolerances=False, primal_tol=0.002, dual_tol=0.1)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        print(f"{name:10s} rep {rep}: first {t1 - t0:.4f} s ({out['iterations']} it), second {t2 - t1:.4f} s "
              f"({out2['iterations']} it)", flush=True)
