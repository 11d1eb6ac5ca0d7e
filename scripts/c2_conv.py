"""Diagnostic (GPU): per-block convergence of a scaled C2 fleet (bench.py c2_admm leg blocks)
under the reference's IPOPT defaults and under tight local solves, same coordinator
settings (rho 0.4, abs tol 0.002 / 0.1, 40 iterations).  ``python scripts/c2_conv.py [n_blocks]``"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]


def main(nb):
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.admm.fleet import ADMMFleet

    kw = dict(admm_iter_max=40, use_relative_tolerances=False, primal_tol=0.002, dual_tol=0.1)
    for name, opts in (("reference", {"ipopt": {}}), ("tight", bm.TIGHT)):
        fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=nb, N=10, seed=20261015 + 1, solver_options=opts))
        out = fl.run_coordinated(0.4, **kw)
        its = np.asarray(out["block_iterations"])
        conv = np.asarray(out["block_converged"])
        last = [out["block_records"][k][-1] for k in range(nb)]
        prim = np.array([r.primal_residual for r in last])
        dual = np.array([r.dual_residual for r in last])
        print(f"{name}: converged {conv.mean():.3f} of {nb} blocks, iterations p50 {np.median(its):.0f} max {its.max()}")
        bad = np.flatnonzero(~conv)
        print(f"  not converged blocks (first 20): {bad[:20].tolist()}")
        if bad.size:
            print(f"  their final primal residual p50 {np.median(prim[bad]):.4g} (tol 0.002), dual p50 {np.median(dual[bad]):.4g} (tol 0.1)")
            k = int(bad[0])
            print(f"  block {k} history (primal, dual):")
            for i, r in enumerate(out["block_records"][k]):
                print(f"    {i + 1:2d} {r.primal_residual:.6g} {r.dual_residual:.6g}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 128)
