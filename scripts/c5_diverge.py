"""Diagnostic: per-agent local-solve outcomes of the C5 N=8 coordinated ADMM round around the
iteration where the GPU fleet and the oracle part (tests/test_gpu_admm.py three-zone case).
``python scripts/c5_diverge.py oracle 13`` (CPU) / ``python scripts/c5_diverge.py gpu 13`` (GPU)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]

import numpy as np  # noqa: E402


def oracle(K):
    from agentlib_mpc_amd.models import examples as ex
    from oracle import admm as oadmm, ipm
    from tests.admm_cases import C5Oracle

    class Rec(C5Oracle):
        calls = {}

        def _run(self, key, prob, p, lbw, ubw, w0):
            guess = self.last.get(key)
            if guess is not None:
                w0 = guess.copy()
                fixed = lbw == ubw
                w0[fixed] = lbw[fixed]
            r = ipm.solve(prob.functions(p), w0, lbw, ubw, prob.lbg(p), prob.ubg(p),
                          ipm.IPMOptions(tol=self.tol, max_iter=500, acceptable_iter=0))
            n = self.calls[key] = self.calls.get(key, 0) + 1
            print(f"it {n:2d} {key:6s} {r.status:28s} iters {r.iterations:3d} soft {r.n_soft_resto} "
                  f"resto {r.n_resto} f {r.f:.12e}", flush=True)
            self.last[key] = r.x
            return r.x

    orc = Rec(8, ex.room_cca_anns())
    oadmm.coordinated_round(orc.participation, orc.initial, orc, 1.0, 8, K, primal_tol=0.04, dual_tol=0.04,
                            use_relative_tolerances=False, T=8)


def gpu(K):
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.admm.fleet import ADMMFleet

    opts = {"ipopt": {"tol": 1e-8, "max_iter": 500, "acceptable_iter": 0}}
    for k in range(max(1, K - 3), K + 1):
        fl = ADMMFleet(bm.c5_fleet_classes(n_blocks=1, N=8, solver_options=opts))
        fl.run_coordinated(1.0, admm_iter_max=k, use_relative_tolerances=False, primal_tol=0.04, dual_tol=0.04)
        for c in ("zone", "ahu", "cca"):
            for i, s in enumerate(fl.stats(c)):
                print(f"it {k:2d} {c}{i} {s['return_status']:28s} iters {s['iter_count']:3d} "
                      f"soft {s['n_soft_restorations']} resto {s['n_restorations']} f {s['obj']:.12e}", flush=True)


if __name__ == "__main__":
    {"oracle": oracle, "gpu": gpu}[sys.argv[1]](int(sys.argv[2]))
