"""Diagnostic (GPU): kernel time of one fleet launch against the number of agents a CU holds at
once, lowered by dynamic LDS padding (``MPCX_LDS_PAD``, mpcx_runtime.cpp) -- does a fleet that
takes two generations anyway (C4 rooms: 13108 agents, 29 per CU by LDS) run faster with fewer,
less contended waves per SIMD?

usage: MODEL=exchange_room N=13108 LDS=5632 PER_CU=29,26,22,20 python scripts/occ_scan.py
(LDS: the code object's static LDS per workgroup, from a kernel trace; PER_CU 0 = no padding)
Every setting solves the same fleet (the template's values, the first parameter spread by
+-1 %) at the reference's IPOPT settings on the main build; statuses / iteration counts are
compared with the first setting.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]
LDS_CU = 160 * 1024


def main():
    import numpy as np
    import torch

    import bench
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.optimization_backends.problem import fleet_nlp_inputs
    from agentlib_mpc_amd.runtime.native import STATS_BYTES, stats_array

    model = os.environ.get("MODEL", "exchange_room")
    n = int(os.environ.get("N", "13108"))
    per_cu = [int(v) for v in os.environ.get("PER_CU", "0").split(",")]
    reps = int(os.environ.get("REPS", "5"))
    be, cv = getattr(bm, model)(solver_options=bm.REFERENCE)
    prob = be.problem
    native = be._native()
    native.set_small_fleet_max(0)
    native.set_mid_fleet_max(0)
    lds = int(os.environ["LDS"])
    dev = torch.device("cuda")
    if model == "one_room":
        vals = bench.fleet_values(n, 20261015 + 2)
    else:
        first = next(k for q in prob.system.parameters for k in q.ref_names if k in cv)
        rng = np.random.default_rng(5)
        vals = {first: cv[first].value * (1.0 + 0.01 * rng.uniform(-1, 1, n))}
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    p, lbw, ubw, w0 = prob.to_kernel(*fleet_nlp_inputs(prob, cv, vals))
    tp, tl, tu, tw0 = T(p), T(lbw), T(ubw), T(w0)
    native.reserve(n)
    ref = None
    for k in per_cu:
        pad = 0 if k <= 0 or lds is None else max(0, LDS_CU // k - lds)
        os.environ["MPCX_LDS_PAD"] = str(pad)
        tw = tw0.clone()
        st = torch.zeros(n * STATS_BYTES, dtype=torch.uint8, device=dev)
        s = torch.cuda.current_stream()
        for _ in range(2):
            tw.copy_(tw0)
            native.solve(tp, tl, tu, tw, stats=st, stream=s.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            tw.copy_(tw0)
            native.solve(tp, tl, tu, tw, stats=st, stream=s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        arr = stats_array(st.cpu().numpy())
        key = (arr["status"].tolist(), arr["iter_count"].tolist())
        same = None if ref is None else key == ref
        ref = ref or key
        print(json.dumps({"model": model, "agents": n, "static_lds": lds, "pad": pad,
                          "agents_per_cu": LDS_CU // (lds + pad) if lds else None,
                          "kernel_ms": e0.elapsed_time(e1) / reps, "mean_iter": float(arr["iter_count"].mean()),
                          "same_status_iters_as_first": same}), flush=True)
    os.environ.pop("MPCX_LDS_PAD", None)


if __name__ == "__main__":
    main()
