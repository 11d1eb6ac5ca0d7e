"""Diagnostic (GPU): host-side profile (cProfile) of the coordinated C2 and the LocalADMM C4
fleet legs of bench.py, after an untimed warm-up round: where the per-iteration host time
goes besides the kernels.  ``python scripts/host_prof.py [c2|c4]``."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]


def main(which):
    import torch

    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.admm.fleet import ADMMFleet

    dev = torch.device("cuda")
    if which == "c1":  # one agent through the plugin API, as the reference MPC module calls it
        be, cv = bm.one_room(solver_options={"ipopt": {}})
        for _ in range(5):
            be.solve(0.0, cv)
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        for _ in range(100):
            r = be.solve(0.0, cv)
        pr.disable()
        wall = time.perf_counter() - t0
        print(f"c1: {wall * 10:.3f} ms per solve, status {r.stats['return_status']}")
        pstats.Stats(pr).sort_stats("tottime").print_stats(30)
        return
    if which == "c2":
        make = lambda: bm.c2_fleet_classes(n_blocks=1024, N=10, seed=20261015 + 1, solver_options={"ipopt": {}})  # noqa: E731
        run = lambda fl: fl.run_coordinated(0.4, admm_iter_max=40, use_relative_tolerances=False,  # noqa: E731
                                            primal_tol=0.002, dual_tol=0.1)
    else:
        make = lambda: bm.c4_fleet_classes(n_rooms=13108, n_supply=3276, N=10, seed=20261015 + 4,  # noqa: E731
                                           solver_options={"ipopt": {}})
        run = lambda fl: fl.run_local(1e4, max_iterations=15, record_residuals=False)  # noqa: E731
    warm = ADMMFleet(make(), device=dev)
    run(warm)
    fleet = ADMMFleet(make(), device=dev)
    for c in fleet.classes:
        c.native.reserve(c.n)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    out = run(fleet)
    torch.cuda.synchronize()
    pr.disable()
    wall = time.perf_counter() - t0
    print(f"{which}: {out['iterations']} iterations in {wall * 1e3:.1f} ms ({wall / out['iterations'] * 1e3:.3f} ms each)")
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "c2")
