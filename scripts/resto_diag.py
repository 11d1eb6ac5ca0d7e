"""Diagnostic (GPU): where does a restoration-phase case leave the oracle's path?

Solves the case with max_iter = 1, 2, ... on the GPU and with the oracle IPM and prints,
per truncation, both statuses / counters and the largest relative difference of the
objectives: the first row that differs names the iteration (and the phase) to look at.
``python scripts/resto_diag.py <case index into tests.test_gpu_ipm.RESTO_CASES> [max]``.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]

import numpy as np  # noqa: E402


def main():
    from agentlib_mpc_amd import benchmarks as bm
    from oracle import ipm
    from tests import configs
    from tests.test_gpu_ipm import REFERENCE_OPTS, RESTO_CASES

    name, kw, setting = RESTO_CASES[int(sys.argv[1])]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 80
    tight = setting == "tight"
    base = dict(tol=1e-10, max_iter=500, acceptable_iter=0) if tight else dict(REFERENCE_OPTS)
    print(name, kw, setting, flush=True)
    differs = 0
    for m in range(1, top + 1):
        o = dict(base, max_iter=m)
        case = configs.CASES[name](solver_options={"ipopt": dict(o)}, **kw)
        p, lbw, ubw, w0 = case.oracle_inputs
        ref = ipm.solve(case.oracle.functions(p), w0, lbw, ubw, case.oracle.lbg(p), case.oracle.ubg(p),
                        ipm.IPMOptions(**o))
        r = case.backend.solve_batch(0.0, [case.current_vars])[0]
        st = r.stats
        got = (st["return_status"], st["iter_count"], st["n_soft_restorations"], st["n_restorations"],
               st["n_restoration_iters"])
        want = (ref.status, ref.iterations, ref.n_soft_resto, ref.n_resto, ref.resto_iterations)
        dobj = abs(st["obj"] - ref.f) / max(1.0, abs(ref.f))
        print(f"m={m:3d} gpu={got} oracle={want} obj {st['obj']:.14g} / {ref.f:.14g} rel {dobj:.2e}"
              f"{'' if got == want else '   <-- differs'}", flush=True)
        differs += got != want or dobj > 1e-9
        if differs >= 3 or (got[0] != "Maximum_Iterations_Exceeded" and want[0] != "Maximum_Iterations_Exceeded"):
            break


if __name__ == "__main__":
    main()
