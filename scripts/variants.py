"""Diagnostic: time compile-time variants of mpcx_ipm_solve on the C3 fleet.

``python scripts/variants.py build`` (CPU) compiles every variant below into
``_build/variants/``; ``python scripts/variants.py run`` (GPU) times them on the
bench fleet and checks each against the default build's solution.
A variant = extra -D defines and/or a source transform of mpcx_ipm.hip.
"""
import json
import os
import pathlib
import subprocess
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "agentlib-mpc_amd")]

VARIANTS = {
    "base": ([], None),
    "nofence": (["-DMPCX_ELIM_FENCE=(void)0"], None),
    "inline_log": ([], ("return log(x); }", "return log(x); }\n#define log_ool(x) log(x)")),
    "nofence_ipra": (["-DMPCX_ELIM_FENCE=(void)0", "-mllvm", "-enable-ipra"], None),
    "lds20k": (["-DMPCX_LDS_TARGET_OVERRIDE=20000"], None),
    "lds14k": (["-DMPCX_LDS_TARGET_OVERRIDE=14000"], None),
    "lds24k_w2": (["-DMPCX_LDS_TARGET_OVERRIDE=24000", "-DMPCX_MIN_WAVES=2"], None),
    "lds14k_w2": (["-DMPCX_LDS_TARGET_OVERRIDE=14000", "-DMPCX_MIN_WAVES=2"], None),
    "lds24k": (["-DMPCX_LDS_TARGET_OVERRIDE=24000"], None),
    "w2": (["-DMPCX_MIN_WAVES=2"], None),
    "w3": (["-DMPCX_MIN_WAVES=3"], None),
    # 8 agents per CU: LDS share 160 KB / 8 and at most 256 VGPRs (2 waves per SIMD)
    "apc8_w2": (["-DMPCX_LDS_TARGET_OVERRIDE=20224", "-DMPCX_MIN_WAVES=2"], None),
    # 5 / 6 agents per CU with <= 256 registers: some SIMDs hold two waves
    "apc5_w2": (["-DMPCX_LDS_TARGET_OVERRIDE=32512", "-DMPCX_MIN_WAVES=2"], None),
    "apc6_w2": (["-DMPCX_LDS_TARGET_OVERRIDE=27050", "-DMPCX_MIN_WAVES=2"], None),
    "apc5": (["-DMPCX_LDS_TARGET_OVERRIDE=32512"], None),
    "apc8": (["-DMPCX_LDS_TARGET_OVERRIDE=20224"], None),
    "w1": (["-DMPCX_MIN_WAVES=1"], None),
    "inl_w2": (["-DMPCX_MIN_WAVES=2"], ("__noinline__", "__attribute__((always_inline))")),
    "inl_w4": ([], ("__noinline__", "__attribute__((always_inline))")),
    # interprocedural register allocation: callers only save what callees clobber
    "ipra": (["-mllvm", "-enable-ipra"], None),
    "nounroll": (["-fno-unroll-loops"], None),
    "ipra_nounroll": (["-mllvm", "-enable-ipra", "-fno-unroll-loops"], None),
    "o2": (["-O2"], None),
    # the kernel source of the last commit (A/B against the working tree)
    "head": ([], "HEAD"),
    # the round-3 record kernel (b34f043) against the working tree (same headers)
    "r03": ([], "REV:b34f043"),
    # r04: the filter cap of round 3 (LDS share 512 B smaller)
    "maxf32": (["-DMPCX_MAXF=32"], None),
    # r04: the hot phases inlined into the fleet build too
    "hot_inline": ([], ("#define MPCX_HOT __noinline__", "#define MPCX_HOT __attribute__((always_inline))")),
    # small-fleet (workspace-in-LDS) builds, loaded through mpcx_problem_small_fleet (AGENTS <= CUs):
    # r04 default (hot phases inlined) and with the phases out of line as in r03
    "lds_base": (["-DMPCX_WS_LDS"], None),
    "lds_noinl": (["-DMPCX_WS_LDS"], ("#define MPCX_HOT __attribute__((always_inline))", "#define MPCX_HOT __noinline__")),
    "lds_r03": (["-DMPCX_WS_LDS"], "REV:b34f043"),
    # wave reductions as the __shfl_xor (ds_bpermute) butterfly instead of DPP + readlane
    "shfl": (["-DMPCX_SHFL_REDUCE=1"], None),
    # leaf phases inlined into the kernel body: no callee-saved VGPR saves per call
    "inl_gj": ([], ("__device__ __noinline__ void eval_gj_lds(", "__device__ __attribute__((always_inline)) void eval_gj_lds(")),
    "inl_head": ([], ("__device__ __noinline__ int iter_head(const Agent a)", "__device__ __attribute__((always_inline)) int iter_head(const Agent a)")),
    # r04: the static elimination on a register image of the stage in the fleet build too
    "elimreg": (["-DMPCX_ELIM_FORCE_REG"], None),
    "elimreg_w1": (["-DMPCX_ELIM_FORCE_REG", "-DMPCX_MIN_WAVES=1"], None),
    "lds_noreg": (["-DMPCX_WS_LDS", "-DMPCX_ELIM_NOREG"], None),
    # r04: the register image loaded from the LDS image the GC lanes assembled (no assemble_reg)
    "asm_noreg": (["-DMPCX_ASM_NOREG"], None),
    "noreg": (["-DMPCX_ELIM_NOREG"], None),
    # r04: the one-sided state chain instead of the twisted one
    "chain_seq": (["-DMPCX_CHAIN_SEQ"], None),
    "lds_nofence": (["-DMPCX_WS_LDS", "-DMPCX_ELIM_FENCE=(void)0"], None),
    # r04: more than 16 agents per CU for structures with a small LDS share and register need
    "apc12": (["-DMPCX_APC=12"], None),
    "apc16": (["-DMPCX_APC=16"], None),
    "apc20": (["-DMPCX_APC=20"], None),
    "apc24": (["-DMPCX_APC=24"], None),
    "apc32": (["-DMPCX_APC=32"], None),
    "lds_asm_noreg": (["-DMPCX_WS_LDS", "-DMPCX_ASM_NOREG"], None),
    # r05: the kernel source of any revision (REV=<sha>) against the working tree, fleet and
    # small-fleet builds
    "rev": ([], "REV:" + os.environ.get("REV", "HEAD")),
    "lds_rev": (["-DMPCX_WS_LDS"], "REV:" + os.environ.get("REV", "HEAD")),
    # r05: IEEE divisions instead of the refined reciprocals (MPCX_RCP) in the generated elimination,
    # alone and with a revision's kernel
    "ieee": (["-DMPCX_IEEE_DIV"], None),
    "rev_ieee": (["-DMPCX_IEEE_DIV"], "REV:" + os.environ.get("REV", "HEAD")),
    "lds_ieee": (["-DMPCX_WS_LDS", "-DMPCX_IEEE_DIV"], None),
    "lds_rev_ieee": (["-DMPCX_WS_LDS", "-DMPCX_IEEE_DIV"], "REV:" + os.environ.get("REV", "HEAD")),
    # r05: interprocedural register allocation on the current kernel, fleet and small-fleet builds
    "lds_ipra": (["-DMPCX_WS_LDS", "-mllvm", "-enable-ipra"], None),
    "lds_nounroll": (["-DMPCX_WS_LDS", "-fno-unroll-loops"], None),
    "lds_o2": (["-DMPCX_WS_LDS", "-O2"], None),
    "lds_maxnsa": (["-DMPCX_WS_LDS", "-mllvm", "-amdgpu-schedule-metric-bias=100"], None),
    # r05/s26: the least-squares multiplier system through the LDS image (MPCX_LSQ_NOREG) in the
    # kernel of 9a47260 (assemble_reg_lsq; not kept: MHE 8.97 ms against 8.12, scratch 1776 B)
    "lsq_noreg": (["-DMPCX_LSQ_NOREG"], "REV:9a47260"),
    # r05/s28: the LDS pivot sweep (MPCX_SWEEP_LDS) in the kernel of 1bfd8f5, whose default swept the
    # twisted chain's pivots on register images (not kept: MHE 10.44 ms against 8.09 ms)
    "sweep_lds": (["-DMPCX_SWEEP_LDS"], "REV:1bfd8f5"),
    "sweep_reg": ([], "REV:1bfd8f5"),
    "lds_lsq_noreg": (["-DMPCX_WS_LDS", "-DMPCX_LSQ_NOREG"], "REV:9a47260"),
    # r06: a revision's small-fleet build with the working tree's filter size (48 in LDS), so that its
    # workspace matches the main build it is loaded beside (mpcx_problem_small_fleet checks it)
    "lds_rev48": (["-DMPCX_WS_LDS", "-DMPCX_MAXF=48"], "REV:" + os.environ.get("REV", "HEAD")),
    # r06: the vector phases' operands as the compiler places them (no MPCX_PIN batches)
    "nopin": (["-DMPCX_NO_PIN"], None),
    "lds_nopin": (["-DMPCX_WS_LDS", "-DMPCX_NO_PIN"], None),
    "pin_head": (["-DMPCX_PIN_HEAD_BATCH"], None),
    "lds_pin_head": (["-DMPCX_WS_LDS", "-DMPCX_PIN_HEAD_BATCH"], None),
    # r06: agents per CU past the one-round rule (MHE: 4 -> 5, two stage rounds)
    "apc5": (["-DMPCX_APC=5"], None),
    "apc20": (["-DMPCX_APC=20"], None),
    "apc24": (["-DMPCX_APC=24"], None),
    "apc28": (["-DMPCX_APC=28"], None),
    # r06: the main build's stage elimination / assembly without the register image (MHE)
    "noreg": (["-DMPCX_ELIM_NOREG"], None),
    "asm_noreg": (["-DMPCX_ASM_NOREG"], None),
}


def vdir():
    from agentlib_mpc_amd.runtime import native
    return native.KERNEL_DIR.parent / "variants" / os.environ.get("MODEL", "one_room")


def build(names):
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.runtime import native
    be, _ = getattr(bm, os.environ.get("MODEL", "one_room"))()
    gen = be.problem.gen
    d = vdir()
    d.mkdir(parents=True, exist_ok=True)
    for name in names:
        defs, tr = VARIANTS[name]
        kern = native.CSRC / "mpcx_ipm.hip"
        src_text = gen.source
        if tr is not None:
            if isinstance(tr, str):
                rev = "HEAD" if tr == "HEAD" else tr.split(":", 1)[1]
                ktxt = subprocess.run(["git", "-C", str(ROOT), "show", f"{rev}:agentlib-mpc_amd/csrc/mpcx_ipm.hip"],
                                      capture_output=True, text=True, check=True).stdout
            else:
                ktxt = kern.read_text()
                for pair in (tr if isinstance(tr, list) else [tr]):
                    assert pair[0] in ktxt, f"{name}: pattern not found"
                    ktxt = ktxt.replace(*pair)
            kp = d / f"mpcx_ipm_{name}.hip"
            kp.write_text(ktxt)
            src_text = src_text.replace('#include "mpcx_ipm.hip"', f'#include "{kp}"')
            assert str(kp) in src_text, "kernel include not found in generated source"
        src = d / f"{name}.hip"
        src.write_text(src_text)
        out = d / f"{name}.hsaco"
        cmd = [native._hipcc(), "--genco", "--offload-arch=gfx950", "-O3", "-std=c++17", *defs,
               f"-I{native.INCLUDE}", f"-I{native.CSRC}", str(src), "-o", str(out),
               "-Rpass-analysis=kernel-resource-usage"]
        r = subprocess.run(cmd, capture_output=True, text=True, check=True)
        info = [l.split("remark:")[1].strip() for l in r.stderr.splitlines()
                if "remark:" in l and any(k in l for k in ("VGPRs:", "Scratch", "Occupancy"))][:4]
        print(name, info)


def run(names):
    import numpy as np
    import torch
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.optimization_backends.problem import fleet_nlp_inputs
    from agentlib_mpc_amd.runtime.native import NativeProblem, STATS_BYTES, stats_to_dicts
    import bench
    model = os.environ.get("MODEL", "one_room")
    be, cv = getattr(bm, model)(solver_options={"ipopt": {"tol": 1e-8, "max_iter": 500}})
    n = int(os.environ.get("AGENTS", "4096"))
    if model == "one_room":
        vals = bench.fleet_values(n, 20261017)
    else:
        first = next(k for q in be.problem.system.parameters for k in q.ref_names if k in cv)
        vals = {first: np.full(n, cv[first].value, float)}
    p, lbw, ubw, w0 = be.problem.to_kernel(*fleet_nlp_inputs(be.problem, cv, vals))
    dev = torch.device("cuda")
    T = lambda a: torch.as_tensor(a, device=dev).contiguous()
    tp, tl, tu, tw0 = T(p), T(lbw), T(ubw), T(w0)
    ref = None
    res = {}
    for name in names:
        if name.startswith("lds"):  # a small-fleet build: loaded beside the default code object
            nat = NativeProblem(be.problem.gen)
            rc = nat.lib.mpcx_problem_small_fleet(nat.handle, str(vdir() / f"{name}.hsaco").encode(), -1)
            assert rc == 0, (name, rc)
        else:
            nat = NativeProblem(be.problem.gen, hsaco=vdir() / f"{name}.hsaco")
        nat.set_options(tol=1e-8, max_iter=500)
        nat.reserve(n)
        tw = tw0.clone()
        st = torch.zeros(n * STATS_BYTES, dtype=torch.uint8, device=dev)
        s = torch.cuda.current_stream()
        for _ in range(2):
            tw.copy_(tw0)
            nat.solve(tp, tl, tu, tw, stats=st, stream=s.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        e0.record(s)
        for _ in range(reps):
            tw.copy_(tw0)
            nat.solve(tp, tl, tu, tw, stats=st, stream=s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        w = tw.cpu().numpy()
        stats = stats_to_dicts(st.cpu().numpy().tobytes())
        ok = sum(x["success"] for x in stats)
        if ref is None:
            ref = w
        dev_max = float(np.max(np.abs(w - ref) / (1 + np.abs(ref))))
        its = [x["iter_count"] for x in stats]
        res[name] = {"ms": ms, "solves_per_s": ok / ms * 1e3, "ok": ok, "maxdev_vs_first": dev_max,
                     "iters_mean_max": [float(np.mean(its)), int(np.max(its))],
                     "statuses": sorted({x["status"] for x in stats}),
                     "restorations": int(sum(x["n_restorations"] for x in stats)),
                     "dense_stages": int(sum(x["n_dense_stages"] for x in stats))}
        print(name, json.dumps(res[name]), flush=True)
        del nat
    return res


if __name__ == "__main__":
    cmd = sys.argv[1]
    names = sys.argv[2:] or list(VARIANTS)
    {"build": build, "run": run}[cmd](names)
