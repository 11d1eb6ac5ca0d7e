"""Summarise the FETCH_SIZE / WRITE_SIZE passes of scripts/gpu_final.sh into
profiles/<round>/<session>/pmc_traffic_c3.json (read by bench.py ``pmc_traffic``).

Only ``mpcx_ipm_solve`` dispatches of the C3 fleet (grid = 4096 workgroups x 64
lanes) are averaged; FETCH_SIZE is doubled (gfx950 note of MI355X_MICROARCH.md);
counters are in KB."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]


def per_dispatch(counter_dir, name):
    files = glob.glob(os.path.join(counter_dir, "**", "*counter_collection.csv"), recursive=True)
    tot = {}
    for fn in files:
        for r in csv.DictReader(open(fn)):
            if "mpcx_ipm_solve" not in r["Kernel_Name"] or r["Counter_Name"] != name:
                continue
            if int(r["Grid_Size"]) != 4096 * 64:
                continue
            tot[r["Dispatch_Id"]] = tot.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return tot


def main(out_dir):
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.runtime.native import code_object_path

    be, _ = bm.one_room(solver_options={"ipopt": {"tol": 1e-8, "max_iter": 500}})
    fetch = per_dispatch(os.path.join(ROOT, "gpurun_out", "pmc", "fetch"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(ROOT, "gpurun_out", "pmc", "write"), "WRITE_SIZE")
    f_kb = sum(fetch.values()) / len(fetch)
    w_kb = sum(write.values()) / len(write)
    d = {
        "kernel": "mpcx_ipm_solve",
        "code_object": code_object_path(be.problem.gen.key).name,
        "workload": "bench.py C3 leg (4096 one_room agents, reference IPOPT settings): --steps 2 --warmup 1 --admm-agents 0 "
                    "--nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0",
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in two separate runs; per-dispatch mean over "
                  "the mpcx_ipm_solve dispatches with grid 4096x64; FETCH_SIZE doubled per MI355X_MICROARCH.md "
                  "(gfx950 reports half of wide reads); KB->bytes x1024",
        "counters_kb": {"FETCH_SIZE": f_kb, "WRITE_SIZE": w_kb},
        "FETCH_SIZE_dispatches": len(fetch),
        "WRITE_SIZE_dispatches": len(write),
        "hbm_bytes_per_launch": (2 * f_kb + w_kb) * 1024,
    }
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "pmc_traffic_c3.json"), "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
