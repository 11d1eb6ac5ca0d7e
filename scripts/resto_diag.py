"""Diagnostic (GPU): where does a restoration-phase case leave the oracle's path?

Solves the case with max_iter = 1, 2, ... on the GPU and with the oracle IPM and prints,
per truncation, both statuses / counters and the largest relative difference of the
objectives: the first row that differs names the iteration (and the phase) to look at.
``python scripts/resto_diag.py <case index into tests.test_gpu_ipm.RESTO_CASES> [max]``.

``python scripts/resto_diag.py trace <case> <m>``: the last line search of the solve truncated
at m iterations, from a -DMPCX_TRACE_LS build of the kernel and from the oracle's LS_TRACE hook
(header: theta, phi, gphi'd, alpha_min, theta_min, theta_max, mu, filter; then the trials).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]

import numpy as np  # noqa: E402


def main():
    from agentlib_mpc_amd import benchmarks as bm
    from oracle import ipm
    from tests import configs
    from tests.test_gpu_ipm import REFERENCE_OPTS, RESTO_CASES

    name, kw, setting = getattr(RESTO_CASES[int(sys.argv[1])], "values", RESTO_CASES[int(sys.argv[1])])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 80
    tight = setting == "tight"
    base = dict(tol=1e-10, max_iter=500, acceptable_iter=0) if tight else dict(REFERENCE_OPTS)
    print(name, kw, setting, flush=True)
    differs = 0
    for m in range(1, top + 1):
        o = dict(base, max_iter=m)
        case = configs.CASES[name](solver_options={"ipopt": dict(o)}, **kw)
        p, lbw, ubw, w0 = case.oracle_inputs
        ref = ipm.solve(case.oracle.functions(p), w0, lbw, ubw, case.oracle.lbg(p), case.oracle.ubg(p),
                        ipm.IPMOptions(**o))
        r = case.backend.solve_batch(0.0, [case.current_vars])[0]
        st = r.stats
        got = (st["return_status"], st["iter_count"], st["n_soft_restorations"], st["n_restorations"],
               st["n_restoration_iters"])
        want = (ref.status, ref.iterations, ref.n_soft_resto, ref.n_resto, ref.resto_iterations)
        dobj = abs(st["obj"] - ref.f) / max(1.0, abs(ref.f))
        print(f"m={m:3d} gpu={got} oracle={want} obj {st['obj']:.14g} / {ref.f:.14g} rel {dobj:.2e}"
              f"{'' if got == want else '   <-- differs'}", flush=True)
        differs += got != want or dobj > 1e-9
        if differs >= 3 or (got[0] != "Maximum_Iterations_Exceeded" and want[0] != "Maximum_Iterations_Exceeded"):
            break


def trace():
    from tests.test_gpu_ipm import RESTO_CASES

    name, kw, setting = getattr(RESTO_CASES[int(sys.argv[2])], "values", RESTO_CASES[int(sys.argv[2])])
    ms = [int(v) for v in sys.argv[3].split(":")]
    if len(ms) == 2:  # a range: only the headers of the last line search per truncation
        for m in range(ms[0], ms[1] + 1):
            trace_one(name, kw, setting, m, brief=True)
        return
    if len(sys.argv) > 4 and sys.argv[4] == "build":
        trace_one(name, kw, setting, ms[0], build_only=True)
        return
    trace_one(name, kw, setting, ms[0])


def trace_one(name, kw, setting, m, brief=False, build_only=False):
    import subprocess

    import torch

    from agentlib_mpc_amd.optimization_backends.mi355x import ipopt_options_to_kernel
    from agentlib_mpc_amd.runtime import native
    from oracle import ipm
    from tests import configs
    from tests.test_gpu_ipm import REFERENCE_OPTS

    base = dict(tol=1e-10, max_iter=500, acceptable_iter=0) if setting == "tight" else dict(REFERENCE_OPTS)
    o = dict(base, max_iter=m)
    case = configs.CASES[name](solver_options={"ipopt": dict(o)}, **kw)
    gen = case.backend.problem.gen
    # TRACE_TAG / TRACE_DEFS: extra -D flags (e.g. -DMPCX_ELIM_GROWTH=1e3); TRACE_NOSTATIC=1: no
    # static stage elimination (every stage on the dense Bunch-Kaufman path)
    tag = os.environ.get("TRACE_TAG", "")
    src = native.KERNEL_DIR / f"trace{tag}_{gen.key}.hip"
    out = src.with_suffix(".hsaco")
    if not out.exists() or build_only:
        text = gen.source
        if os.environ.get("TRACE_NOSTATIC"):
            text = text.replace("#define MPCX_STATIC_ELIM 1", "")
        src.write_text("#define MPCX_TRACE_LS 1\n" + text)
        subprocess.run([native._hipcc(), "--genco", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        *os.environ.get("TRACE_DEFS", "").split(),
                        f"-I{native.INCLUDE}", f"-I{native.CSRC}", str(src), "-o", str(out)], check=True)
    if build_only:
        print(out)
        return
    prob = case.backend.problem
    (p, lbw, ubw, w0), _ = configs.product_nlp_inputs(case)
    kp, kl, ku, kw0 = prob.to_kernel(p[None], lbw[None], ubw[None], w0[None])
    nat = native.NativeProblem(gen, hsaco=out)
    nat.set_options(**ipopt_options_to_kernel({"ipopt": o}))
    nat.reserve(1)
    d = torch.device("cuda")
    T = lambda a: torch.as_tensor(a, device=d).contiguous()  # noqa: E731
    tp, tl, tu, tw = T(kp), T(kl), T(ku), T(kw0)
    lg = torch.zeros((1, prob.nlp.kernel_ng), dtype=torch.float64, device=d)
    lw = torch.zeros_like(tw)
    st = torch.zeros(native.STATS_BYTES, dtype=torch.uint8, device=d)
    nat.solve(tp, tl, tu, tw, lam_g=lg, lam_w=lw, stats=st)
    torch.cuda.synchronize()
    h, g = lw[0].cpu().numpy(), lg[0].cpu().numpy()
    nf = int(h[7])
    if brief:
        sd = native.stats_to_dicts(st.cpu().numpy().tobytes())[0]
        ipm.LS_TRACE = []
        pp, l2, u2, w2 = case.oracle_inputs
        ref = ipm.solve(case.oracle.functions(pp), w2, l2, u2, case.oracle.lbg(pp), case.oracle.ubg(pp),
                        ipm.IPMOptions(**o))
        hd = ipm.LS_TRACE[0] if ipm.LS_TRACE else ("none",) + (float("nan"),) * 7 + ([], 0.0, 0.0)
        print(f"m={m:3d} GPU th {h[0]:.10e} phi {h[1]:.10e} mu {h[6]:.3e} dw {h[8]:.2e} dc {h[9]:.2e} nf {nf:2d} "
              f"{sd['return_status'][:12]} | ORC th {hd[1]:.10e} phi {hd[2]:.10e} mu {hd[7]:.3e} dw {hd[9]:.2e} "
              f"dc {hd[10]:.2e} nf {len(hd[8]):2d} {ref.status[:12]}", flush=True)
        ipm.LS_TRACE = None
        return
    print("GPU head", h[:8].tolist())
    print("GPU dw dc", h[8], h[9])
    print("GPU filter", [(h[10 + 2 * j], h[11 + 2 * j]) for j in range(nf)])
    for t in range(len(g) // 6):
        row = g[6 * t:6 * t + 6]
        if row[0] == 0.0:
            break
        print("GPU trial", row.tolist())
    print("GPU stats", native.stats_to_dicts(st.cpu().numpy().tobytes())[0])
    ipm.LS_TRACE = []
    pp, l2, u2, w2 = case.oracle_inputs
    ref = ipm.solve(case.oracle.functions(pp), w2, l2, u2, case.oracle.lbg(pp), case.oracle.ubg(pp), ipm.IPMOptions(**o))
    head = ipm.LS_TRACE[0]
    print("ORC head", list(head[1:8]), "nfilt", len(head[8]))
    print("ORC filter", head[8])
    for row in ipm.LS_TRACE[1:]:
        print("ORC trial", list(row))
    print("ORC", ref.status, ref.iterations, ref.n_resto, ref.resto_iterations)


if __name__ == "__main__":
    if sys.argv[1] == "trace":
        trace()
    else:
        main()
