"""Diagnostic (GPU): the single agent (C1, simple_mpc) through ``backend.solve`` -- end to end
per call, cold (``reset_warm_start``: the reference's first solve, what bench.py times) and warm
(the closed loop), the kernel alone (HIP events), and a cProfile of the host side of 200 warm
calls.  ``python scripts/c1_prof.py``."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]


def main():
    import torch

    from agentlib_mpc_amd import benchmarks as bm

    be, cv = bm.one_room(solver_options={"ipopt": {}})
    for _ in range(5):
        be.reset_warm_start()
        be.solve(0.0, cv)
    for label, cold in (("cold", True), ("warm", False)):
        ts = []
        for _ in range(100):
            if cold:
                be.reset_warm_start()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = be.solve(0.0, cv)
            ts.append(time.perf_counter() - t0)
        print(f"{label}: median {np.median(ts) * 1e3:.3f} ms  p10 {np.percentile(ts, 10) * 1e3:.3f}  "
              f"iters {r.stats['iter_count']}", flush=True)
    rb = be._resident
    launch = rb.native.bind(rb.P, rb.L, rb.U, rb.W, lam_g=rb.lam_g, stats=rb.ST)
    s = torch.cuda.current_stream()
    ks = []
    for _ in range(50):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        launch()
        e1.record(s)
        torch.cuda.synchronize()
        ks.append(e0.elapsed_time(e1))
    print(f"kernel (warm, resident buffers): median {np.median(ks):.3f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        be.solve(0.0, cv)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
