"""Diagnostic (GPU): solve one MHE case with the default kernel and with the
block-chain-only build; print the kernel statistics of both."""
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "agentlib-mpc_amd")]


def build(case_name):
    from tests import configs
    from agentlib_mpc_amd.runtime import native
    case = configs.CASES[case_name]()
    gen = case.backend.problem.gen
    d = native.KERNEL_DIR.parent / "diag"
    d.mkdir(parents=True, exist_ok=True)
    prefix = os.environ.get("DIAG_PREFIX", "")
    src = d / f"{prefix}{case_name}.hip"
    src.write_text(gen.source.replace("#define MPCX_FORCE_BLOCK_CHAIN 1", ""))
    for tag, defs in (("default", []), ("chain", ["-DMPCX_FORCE_BLOCK_CHAIN"])):
        out = d / f"{prefix}{case_name}_{tag}.hsaco"
        subprocess.run([native._hipcc(), "--genco", "--offload-arch=gfx950", "-O3", "-std=c++17", *defs,
                        f"-I{native.INCLUDE}", f"-I{native.CSRC}", str(src), "-o", str(out)], check=True)
        print("built", out)


def run(case_name):
    import numpy as np
    import torch
    from tests import configs
    from agentlib_mpc_amd.runtime import native
    from agentlib_mpc_amd.runtime.native import NativeProblem, STATS_BYTES, stats_to_dicts
    case = configs.CASES[case_name]()
    prob = case.backend.problem
    (p, lbw, ubw, w0), _ = configs.product_nlp_inputs(case)
    kp, kl, ku, kw = prob.to_kernel(p[None], lbw[None], ubw[None], w0[None])
    dev = torch.device("cuda")
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)
    d = native.KERNEL_DIR.parent / "diag"
    for hs in sorted(d.glob(f"*{case_name}_*.hsaco")):
        tag = hs.stem
        nat = NativeProblem(prob.gen, hsaco=hs)
        nat.set_options(tol=1e-10, max_iter=500)
        tw = T(kw)
        st = torch.zeros(STATS_BYTES, dtype=torch.uint8, device=dev)
        nat.solve(T(kp), T(kl), T(ku), tw, stats=st)
        torch.cuda.synchronize()
        s = stats_to_dicts(st.cpu().numpy().tobytes())[0]
        print(tag, {k: s[k] for k in s if k in ("success", "return_status", "iter_count", "obj", "n_block_chain",
                                                "dual_inf", "constr_viol", "compl_inf", "mu")}, flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]](sys.argv[2])
