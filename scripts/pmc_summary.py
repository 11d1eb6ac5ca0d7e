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
    fp64_dir = os.path.join(ROOT, "gpurun_out", "pmc", "fp64")
    if os.path.isdir(fp64_dir):
        u = fp64_summary(fp64_dir, os.path.join(ROOT, "gpurun_out", "pmc", "issue"))
        u["code_object"] = d["code_object"]
        with open(os.path.join(out_dir, "pmc_fp64_c3.json"), "w") as f:
            json.dump(u, f, indent=1)
        print(json.dumps(u, indent=1))


def fp64_summary(fp64_dir, issue_dir):
    """FP64 utilisation of mpcx_ipm_solve from the instruction counters.  SQ_INSTS_* count
    wave instructions; a wave-wide FP64 op is 64 lane-ops (an FMA two flops), so
    64 x (ADD + MUL + 2 FMA + TRANS) is the issued-FLOP count with every lane active -- an
    upper bound, since lanes masked off by divergence still take the issue slot.  An
    FP64 MFMA op counts 512 flops per MOPS unit (rocprofv3 MfmaFlopsF64).  Peak: 78.6
    TFLOP/s vector FP64 (MI355X_MICROARCH.md); the issue share is SQ_ACTIVE_INST_VALU /
    SQ_WAVE_CYCLES (quad-cycle units both)."""
    names = ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64",
             "SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_SALU",
             "GRBM_GUI_ACTIVE"]
    c = {n: _mean(per_dispatch(fp64_dir, n)) for n in names}
    issue = ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
             "SQ_ACTIVE_INST_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"]
    if os.path.isdir(issue_dir):
        c.update({n: _mean(per_dispatch(issue_dir, n)) for n in issue})
    vflops = 64.0 * (c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + 2.0 * c["SQ_INSTS_VALU_FMA_F64"]
                     + c["SQ_INSTS_VALU_TRANS_F64"])
    mflops = 512.0 * c["SQ_INSTS_VALU_MFMA_MOPS_F64"]
    out = {"kernel": "mpcx_ipm_solve", "counters_per_dispatch": c,
           "fp64_valu_flops_per_launch_upper": vflops, "fp64_mfma_flops_per_launch": mflops,
           "fp64_share_of_valu_insts": (c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] +
                                        c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_TRANS_F64"]) /
                                       max(1.0, c["SQ_INSTS_VALU"]),
           "method": fp64_summary.__doc__.strip()}
    if "SQ_WAVE_CYCLES" in c:
        wc = max(1.0, c["SQ_WAVE_CYCLES"])
        out["wave_cycle_split"] = {"valu_issue": c["SQ_ACTIVE_INST_VALU"] / wc, "any_issue": c["SQ_ACTIVE_INST_ANY"] / wc,
                                   "wait_any": c["SQ_WAIT_ANY"] / wc, "wait_inst_any": c["SQ_WAIT_INST_ANY"] / wc}
    return out


def _mean(d):
    return sum(d.values()) / max(1, len(d))


if __name__ == "__main__":
    main(sys.argv[1])
