"""Diagnostic (GPU): single-agent and 256-agent kernel time of each benchmark structure on the
small-fleet build (workspace hot part in LDS, one agent per CU) vs the HBM build, HIP events
on the launch stream, same inputs; statuses / iteration counts must agree.
``python scripts/small_fleet_ab.py``"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]


def main():
    import torch

    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.runtime.native import STATS_BYTES, stats_to_dicts

    dev = torch.device("cuda")
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    for name in ("one_room", "admm_room", "admm_ahu", "exchange_room", "room_nn", "tz_ahu", "tz_cca",
                 "mhe_room", "rng_room_mpc"):
        fn = {**bm.BUILDERS, "mhe_room": bm.mhe_room, "rng_room_mpc": bm.rng_room_mpc}[name]
        be, cv = fn(solver_options=bm.REFERENCE)
        native = be._native()
        prob = be.problem
        for n in (1, 256):
            p, lbw, ubw, w0 = prob.to_kernel(*prob.marshal.inputs([cv] * n, 0.0))
            res = {}
            for mode, mx in (("lds", -1), ("hbm", 0)):
                native.set_small_fleet_max(mx)
                ts = []
                for _ in range(6):
                    tw = T(w0)
                    st = torch.zeros(n * STATS_BYTES, dtype=torch.uint8, device=dev)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    native.solve(T(p), T(lbw), T(ubw), tw, stats=st)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1))
                s = stats_to_dicts(st.cpu().numpy().tobytes())
                res[mode] = (float(np.median(ts[1:])), [x["status"] for x in s], [x["iter_count"] for x in s],
                             tw.cpu().numpy())
            native.set_small_fleet_max(-1)
            same = res["lds"][1] == res["hbm"][1] and res["lds"][2] == res["hbm"][2]
            dw = float(np.max(np.abs(res["lds"][3] - res["hbm"][3]) / (1.0 + np.abs(res["hbm"][3]))))
            print(f"{name:14s} n={n:3d}  hbm {res['hbm'][0]:7.3f} ms  lds {res['lds'][0]:7.3f} ms  "
                  f"({res['lds'][0] / res['hbm'][0]:.2f}x)  status/iters equal: {same}  max rel dw {dw:.1e}  "
                  f"iters {res['lds'][2][0]}", flush=True)


if __name__ == "__main__":
    main()
