"""Diagnostic: per-phase cycle breakdown of mpcx_ipm_solve (MPCX_PROFILE build)."""
import os, sys, subprocess, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]
import numpy as np

CHAIN_PATCH = [
    ("SPROF(6);  // loads and the per-element terms", "(void)0;"),
    ("SPROF(7);  // reductions", "(void)0;"),
    ("SPROF(8);  // termination tests, barrier update", "(void)0;"),
    ("SPROF(9);  // rhs / diagonal stores and the barrier", "(void)0;"),
    ("  constexpr int NCX = NC * NX;\n#pragma unroll 1\n  for (int s = 0; s <= CSTEPS; ++s) {",
     "  constexpr int NCX = NC * NX;\n  SPROF_DECL\n#pragma unroll 1\n  for (int s = 0; s <= CSTEPS; ++s) {"),
    ("    wsync();\n    // the pivots, assembled in their Dinv slots", "    wsync();\n    SPROF(6);\n    // the pivots, assembled in their Dinv slots"),
    ("      L.Dinv[j * NCC + ee] = v;\n    }\n    wsync();\n", "      L.Dinv[j * NCC + ee] = v;\n    }\n    wsync();\n    SPROF(7);\n"),
    ("    in.pos += bi.pos; in.neg += bi.neg; in.zero += bi.zero;\n  }\n  wsync();\n  return in;\n}\n\n// The twisted chain's solve",
     "    in.pos += bi.pos; in.neg += bi.neg; in.zero += bi.zero;\n    SPROF(8);\n  }\n  wsync();\n  return in;\n}\n\n// The twisted chain's solve"),
]


def build_profile_hsaco(gen, wslds=False):
    from agentlib_mpc_amd.runtime import native
    src = native.KERNEL_DIR / f"prof_{gen.key}{'_wslds' if wslds else ''}.hip"
    out = src.with_suffix(".hsaco")
    src.parent.mkdir(parents=True, exist_ok=True)
    text = gen.source
    if os.environ.get("CHAIN_PROF", "0") == "1":
        # the twisted chain's three phases in the iteration head's profile slots (6-8), on a
        # patched copy of the kernel source (the shipped source stays as it is)
        k = (native.CSRC / "mpcx_ipm.hip").read_text()
        for a, b in CHAIN_PATCH:
            assert k.count(a) == 1, a
            k = k.replace(a, b)
        kp = src.with_name(src.stem + "_chainprof_ipm.hip")
        kp.write_text(k)
        text = text.replace('#include "mpcx_ipm.hip"', f'#include "{kp}"')
        assert str(kp) in text
    src.write_text("#define MPCX_PROFILE 1\n" + ("#define MPCX_WS_LDS 1\n" if wslds else "") + text)
    subprocess.run([native._hipcc(), "--genco", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    f"-I{native.INCLUDE}", f"-I{native.CSRC}", str(src), "-o", str(out)], check=True)
    return out

def main():
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.optimization_backends.problem import fleet_nlp_inputs
    from agentlib_mpc_amd.runtime.native import NativeProblem
    import bench
    model = os.environ.get("MODEL", "one_room")
    from agentlib_mpc_amd.optimization_backends.mi355x import ipopt_options_to_kernel
    sopts = bm.REFERENCE if os.environ.get("SOLVER", "reference") == "reference" else bm.TIGHT
    kopts = ipopt_options_to_kernel(sopts)
    be, cv = {**bm.BUILDERS, "mhe_room": bm.mhe_room, "rng_room_mpc": bm.rng_room_mpc}[model](solver_options=sopts)
    path = build_profile_hsaco(be.problem.gen)
    # WSLDS=1: the small-fleet build (workspace in LDS) for batches of <= one agent per CU
    wslds = os.environ.get("WSLDS", "0") == "1"
    lpath = build_profile_hsaco(be.problem.gen, wslds=True) if wslds else None
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        print(path, lpath); return
    import torch
    n = int(os.environ.get("AGENTS", "4096"))
    if model == "one_room":
        vals = bench.fleet_values(n, 20261015 + 2)
    else:
        first = next(k for q in be.problem.system.parameters for k in q.ref_names if k in cv)
        vals = {first: np.full(n, cv[first].value, float)}
    p, lbw, ubw, w0 = be.problem.to_kernel(*fleet_nlp_inputs(be.problem, cv, vals))
    nat = NativeProblem(be.problem.gen, hsaco=path)
    nat.set_options(**kopts)
    nat.reserve(n)
    if lpath is not None:
        assert nat.lib.mpcx_problem_small_fleet(nat.handle, str(lpath).encode(), -1) == 0
    d = torch.device("cuda")
    T = lambda a: torch.as_tensor(a, device=d).contiguous()
    tp, tl, tu, tw = T(p), T(lbw), T(ubw), T(w0)
    lw = torch.zeros_like(tw)
    from agentlib_mpc_amd.runtime.native import STATS_BYTES, stats_to_dicts, NativeProblem as NP
    st = torch.zeros(n * STATS_BYTES, dtype=torch.uint8, device=d)
    tw0 = T(w0)
    for _ in range(2):
        tw.copy_(tw0); nat.solve(tp, tl, tu, tw, lam_w=lw, stats=st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); tw.copy_(tw0); nat.solve(tp, tl, tu, tw, lam_w=lw, stats=st); e1.record()
    torch.cuda.synchronize()
    stats = stats_to_dicts(st.cpu().numpy().tobytes())
    print("profile build: kernel ms", e0.elapsed_time(e1), "mean iters", np.mean([x["iter_count"] for x in stats]),
          "mean fact", np.mean([x["n_factorizations"] for x in stats]))
    plain = NP(be.problem.gen)
    plain.set_options(**kopts)
    plain.reserve(n)
    for _ in range(2):
        tw.copy_(tw0); plain.solve(tp, tl, tu, tw, stats=st)
    torch.cuda.synchronize()
    e0.record(); tw.copy_(tw0); plain.solve(tp, tl, tu, tw, stats=st); e1.record()
    torch.cuda.synchronize()
    print("plain build: kernel ms", e0.elapsed_time(e1))
    prof = lw[:, :22].cpu().numpy()
    names = ["init", "ls_mult", "opt_err+mu", "hess", "rhs_x", "factor", "solve", "recover", "linesearch", "accept+gj",
             "f:assemble", "f:interior_bk", "f:schur+store", "f:chain", "s:forward", "s:chain+back"]
    tot = prof[:, :10].sum(axis=1).mean()
    print(json.dumps({k: float(v) for k, v in zip(names, prof.mean(axis=0))}))
    for k, v in zip(names, prof.mean(axis=0)):
        print(f"{k:12s} {v/1e3:10.1f} kcyc  {100*v/tot:5.1f}%")
    print("total kcycles/agent", tot / 1e3)
    if prof.shape[1] >= 22:
        head = lw[:, 18:22].cpu().numpy().mean(axis=0)
        labels = (["c:cw+cy", "c:assemble", "c:sweep", "-"] if os.environ.get("CHAIN_PROF", "0") == "1"
                  else ["h:loads+terms", "h:reductions", "h:tests+mu", "h:stores+sync"])
        for k, v in zip(labels, head):
            print(f"{k:14s} {v/1e3:10.1f} kcyc")
    seen = lw[:, 16].cpu().numpy().astype(np.int64) | (lw[:, 17].cpu().numpy().astype(np.int64) << 32)
    hist = [int(((seen >> k) & 1).sum()) for k in range(be.problem.gen.dims["N"])]
    print("agents with stage k ever on the dense path:", hist)

if __name__ == "__main__":
    main()
