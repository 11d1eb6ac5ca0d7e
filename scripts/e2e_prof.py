"""Diagnostic (GPU): where the time of one 4096-agent C3 plugin-API step goes
(``MI355XBackend.solve_batch``, bench.py ``e2e`` leg): reading the agents' variables, the
column upload / scatter, the kernel (HIP events on the launch stream), the solution and
stats read-back, and the first-control extraction -- each bracketed by a device
synchronisation -- next to the resident FleetSession step, with the IPM iteration counts
of both.  ``python scripts/e2e_prof.py [n_agents]``."""
import copy
import cProfile
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]


def main(n):
    import torch

    import bench
    from agentlib_mpc_amd import benchmarks as bm

    dev = torch.device("cuda")
    be, cv = bm.one_room(solver_options=bm.REFERENCE)  # the bench e2e leg's settings
    vals = bench.fleet_values(n, 20261015 + 2)
    agents = []
    for a in range(n):
        c = copy.deepcopy(cv)
        for k in ("T", "load", "T_in", "T_upper", "mDot"):
            c[k].value = float(vals[k][a])
        agents.append(c)
    rng = np.random.default_rng(7)
    be.solve_batch(0.0, agents)
    rb = be._resident
    sync = torch.cuda.synchronize
    t_read = []
    read0 = rb.read

    def timed_read(*a, **k):
        t0 = time.perf_counter()
        out = read0(*a, **k)
        t_read.append(time.perf_counter() - t0)
        return out

    rb.read = timed_read
    rows = []
    for k in range(1, 8):
        drift = rng.normal(0.0, 0.05, n)
        for a, c in enumerate(agents):
            c["T"].value = float(vals["T"][a] + drift[a])
        sync()
        t = [time.perf_counter()]
        be._native()
        snap = rb.update(agents, 300.0 * k)
        sync(); t.append(time.perf_counter())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rb.native.solve(rb.P, rb.L, rb.U, rb.W, lam_g=rb.lam_g, stats=rb.ST)
        e1.record()
        sync(); t.append(time.perf_counter())
        w = torch.empty((rb.n, rb.W.shape[1]), dtype=torch.float64, pin_memory=True)
        sync(); t.append(time.perf_counter())
        w.copy_(rb.W, non_blocking=True)
        raw = rb.ST.cpu().numpy()
        sync(); t.append(time.perf_counter())
        from agentlib_mpc_amd.runtime.native import stats_array
        st = stats_array(raw)
        from agentlib_mpc_amd.optimization_backends.plugin_batch import RowSource
        from agentlib_mpc_amd.optimization_backends.problem import FleetResults
        from agentlib_mpc_amd.runtime.native import StatsView
        res = FleetResults(be.problem, be.problem.marshal, None, None, None, w.numpy(), StatsView(st), rows=RowSource(rb, snap))
        u0 = res.first_values("mDot")
        t.append(time.perf_counter())
        d = np.diff(t) * 1e3
        rows.append((d, e0.elapsed_time(e1), float(st["iter_count"].mean()), int(st["iter_count"].max())))
    print("plugin step pieces (ms): update (of which read) | launch+kernel | pinned alloc | D2H w+stats | "
          "results+first_values ; kernel(events) ; mean/max it")
    for (d, km, mi, mx), tr in zip(rows, t_read):
        print(f"  {d[0]:7.3f} ({tr * 1e3:6.3f}) | " + " | ".join(f"{x:7.3f}" for x in d[1:]) + f" ; {km:7.3f} ; {mi:.2f}/{mx}")
    # the full call, profiled
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for k in range(8, 13):
        for a, c in enumerate(agents):
            c["T"].value = float(vals["T"][a] + rng.normal(0.0, 0.05))
        res = be.solve_batch(300.0 * k, agents)
        res.first_values("mDot")
    pr.disable()
    print(f"solve_batch: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms per call (incl. the untimed agent updates)")
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)
    # resident session
    from agentlib_mpc_amd.optimization_backends.fleet_session import FleetSession
    sess = FleetSession(be, agents, now=0.0)
    sess.solve()
    for k in range(5):
        sess.update("T", vals["T"] + rng.normal(0.0, 0.05, n))
        sync()
        t0 = time.perf_counter()
        sess.solve()
        sync()
        ts = time.perf_counter() - t0
        s = sess.stats().array
        print(f"session solve {ts * 1e3:.3f} ms, mean/max it {s['iter_count'].mean():.2f}/{s['iter_count'].max()}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4096)
