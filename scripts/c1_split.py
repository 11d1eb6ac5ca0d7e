"""Diagnostic (GPU): where the single agent's (C1) end-to-end time goes -- the host steps of
``backend.solve`` (cold start) timed one by one: input update (host mirrors), the staged round
trip (upload, kernel, read-back, wait: one native call), the host post-processing and the result
object; the kernel alone by HIP events.  ``python scripts/c1_split.py``."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]


def main():
    import torch

    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.optimization_backends.plugin_batch import RowSource  # noqa: F401
    from agentlib_mpc_amd.optimization_backends.problem import FleetResults
    from agentlib_mpc_amd.runtime.native import StatsView, stats_array

    be, cv = bm.one_room(solver_options={"ipopt": {}})
    for _ in range(5):
        be.reset_warm_start()
        be.solve(0.0, cv)
    rb = be._resident
    prob = be.problem
    pc = time.perf_counter
    rows = []
    rb.solve()  # binds the staged round trip
    for _ in range(200):
        be.reset_warm_start()
        torch.cuda.synchronize()
        t0 = pc()
        be._native()
        snap = rb.update([cv], 0.0)
        t1 = pc()
        rb._roundtrip()
        t2 = pc()
        out = rb._pin_out.numpy()
        nw = rb.hW.size
        w = out[:nw].reshape(rb.hW.shape).copy()
        raw = out[nw:].view(np.uint8)[:rb.ST.numel()].copy()
        rb.hW[:] = w
        bad = np.flatnonzero(np.isnan(w.sum(axis=1)))
        rb.cold_rows = bad if bad.size else None
        t3 = pc()
        stats = StatsView(stats_array(raw), {"t_wall_total": t3 - t0})
        FleetResults(prob, prob.marshal, None, None, None, w, stats, rows=RowSource(rb, snap))
        t4 = pc()
        rows.append([t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0])
    med = np.median(np.array(rows), axis=0) * 1e6
    names = ["update (host mirrors)", "staged round trip", "post-process", "results object", "total"]
    for n, v in zip(names, med):
        print(f"{n:28s} {v:8.1f} us")
    launch = rb.native.bind(rb.P, rb.L, rb.U, rb.W, lam_g=rb.lam_g, stats=rb.ST)
    s = torch.cuda.current_stream()
    ks = []
    for _ in range(50):
        be.reset_warm_start()
        be._native()
        rb.update([cv], 0.0)
        rb._buf_in.copy_(rb._hbuf_in)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        launch()
        e1.record(s)
        torch.cuda.synchronize()
        ks.append(e0.elapsed_time(e1) * 1e3)
    print(f"{'kernel (HIP events, cold)':28s} {np.median(ks):8.1f} us")
    # fixed cost of a launch + read-back round trip: an empty torch op on the same buffers
    ts = []
    for _ in range(200):
        t0 = pc()
        rb.W.add_(0.0)
        rb._pin_out.copy_(rb.BUF[rb._out_off:], non_blocking=True)
        torch.cuda.current_stream().synchronize()
        ts.append(pc() - t0)
    print(f"{'empty op + read-back':28s} {np.median(ts) * 1e6:8.1f} us")


if __name__ == "__main__":
    main()
