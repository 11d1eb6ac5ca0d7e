"""Where does a long restoration run leave the oracle's path?  For the infeasible fixture_mpc case of
tests/test_gpu_ipm.py::test_gpu_long_restoration_run_follows_the_oracle (reference options), the
small-fleet build of several kernel revisions is run to max_iter = k for a range of k and compared
with the oracle's run to the same k (status, iterations, objective, max relative point deviation).

``python scripts/resto_ab.py build [name ...]`` (CPU: compiles the variants of this case's generated
source into <kernel dir>/../variants/resto/), ``python scripts/resto_ab.py run [name ...]`` (GPU).
Variants: ``cur`` (working tree), ``nopin`` (MPCX_NO_PIN), ``rev`` (REV=<sha>, default d394363), ``trace``
(MPCX_TRACE_IT: one line per iteration, the restoration starts and line searches).
``dist`` (GPU): the in-tree builds' final statuses on seeded perturbed starts; ``trace <draws>`` (GPU):
kernel and oracle iteration traces; ``kkt [draw] [it]`` (CPU): the oracle's inertia tests of one
iteration against the eigenvalues of the same matrix (profiles/r06/resto/)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]

KW = {"T_lb": 255.0, "T_ub": 302.0, "disturbance": 270.0, "T0": 290.0}
REF = dict(tol=1e-4, max_iter=100, acceptable_tol=0.1, acceptable_iter=5,
           acceptable_constr_viol_tol=1.0, acceptable_compl_inf_tol=1.0)
VARIANTS = {
    "cur": ([], None),
    "nopin": (["-DMPCX_NO_PIN"], None),
    "rev": ([], os.environ.get("REV", "d394363")),
    "trace": (["-DMPCX_TRACE_IT"], None),
}
BUILD = os.environ.get("BUILD", "lds")  # lds: -DMPCX_WS_LDS small-fleet object; main: the HBM build


def case_of(opts):
    from tests import configs
    return configs.CASES["fixture_mpc"](solver_options={"ipopt": dict(opts)}, **KW)


def vdir():
    from agentlib_mpc_amd.runtime import native
    return native.KERNEL_DIR.parent / "variants" / "resto"


def build(names):
    from agentlib_mpc_amd.runtime import native
    gen = case_of(REF).backend.problem.gen
    d = vdir()
    d.mkdir(parents=True, exist_ok=True)
    for name in names:
        defs, rev = VARIANTS[name]
        src_text = gen.source
        if rev is not None:
            ktxt = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:agentlib-mpc_amd/csrc/mpcx_ipm.hip"],
                                  capture_output=True, text=True, check=True).stdout
            kp = d / f"mpcx_ipm_{name}.hip"
            kp.write_text(ktxt)
            src_text = src_text.replace('#include "mpcx_ipm.hip"', f'#include "{kp}"')
            assert str(kp) in src_text
        src = d / f"{BUILD}_{name}.hip"
        src.write_text(src_text)
        out = d / f"{BUILD}_{name}.hsaco"
        extra = ["-DMPCX_WS_LDS"] if BUILD == "lds" else []
        subprocess.run([native._hipcc(), "--genco", "--offload-arch=gfx950", "-O3", "-std=c++17", *extra, *defs,
                        f"-I{native.INCLUDE}", f"-I{native.CSRC}", str(src), "-o", str(out)], check=True)
        print("built", out, flush=True)


def run(names):
    from oracle import ipm
    from tests.test_gpu_ipm import _w_of
    ks = [int(x) for x in os.environ.get("KS", "10,15,20,25,30,35,40,45,50,55,60,65,70,100").split(",")]
    for k in ks:
        opts = dict(REF, max_iter=k)
        case = case_of(opts)
        p, lbw, ubw, w0 = case.oracle_inputs
        ref = ipm.solve(case.oracle.functions(p), w0, lbw, ubw, case.oracle.lbg(p), case.oracle.ubg(p),
                        ipm.IPMOptions(**opts))
        line = [f"k={k:3d} oracle {ref.status[:12]:12s} it {ref.iterations:3d} resto {ref.n_resto:2d} f {ref.f:.10e}"]
        for name in names:
            case = case_of(opts)
            nat = case.backend._native()
            rc = nat.lib.mpcx_problem_small_fleet(nat.handle, str(vdir() / f"{BUILD}_{name}.hsaco").encode(), -1)
            assert rc == 0, (name, rc)
            nat.set_small_fleet_max(1 << 30)
            nat.set_mid_fleet_max(0)
            nat.set_wide_fleet_min(0)
            r = case.backend.solve_batch(0.0, [case.current_vars])[0]
            st = r.stats
            w = _w_of(case, r)
            dev = float(np.max(np.abs(w - ref.x) / (1.0 + np.abs(ref.x))))
            line.append(f"  {name}: {st['return_status'][:12]:12s} it {st['iter_count']:3d} resto {st['n_restorations']:2d} "
                        f"f {st['obj']:.10e} dev {dev:.1e}")
        print("\n".join(line), flush=True)


def dist(builds):
    """The kernel's final statuses on the seeded perturbed starts of scripts/resto_chaos.py (one
    launch of 1 + ND agents per in-tree build: lds / mid / main), against the oracle's
    (profiles/r06/resto_chaos.txt)."""
    import torch
    from agentlib_mpc_amd.runtime.native import STATS_BYTES, stats_to_dicts
    from tests.test_multi_minima import perturbed
    nd = int(os.environ.get("ND", "16"))
    case = case_of(REF)
    p, lbw, ubw, w0 = case.oracle_inputs
    ws = np.stack([w0] + [perturbed(w0, seed=0, k=d) for d in range(nd)])
    n = ws.shape[0]
    rep = lambda a: np.ascontiguousarray(np.broadcast_to(a, (n,) + a.shape))  # noqa: E731
    kp, kl, ku, kw = case.backend.problem.to_kernel(rep(p), rep(lbw), rep(ubw), ws)
    dev = torch.device("cuda")
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    nat = case.backend._native()
    for b in builds or ["lds", "mid", "main"]:
        nat.set_small_fleet_max(1 << 30 if b == "lds" else 0)
        nat.set_mid_fleet_max(1 << 30 if b == "mid" else 0)
        nat.set_wide_fleet_min(0)
        nat.set_options(**REF)
        nat.reserve(n)
        tw = T(kw)
        st = torch.zeros(n * STATS_BYTES, dtype=torch.uint8, device=dev)
        nat.solve(T(kp), T(kl), T(ku), tw, stats=st, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        stats = stats_to_dicts(st.cpu().numpy().tobytes())
        out = {}
        for d, x in enumerate(stats):
            out.setdefault(x["return_status"], []).append(("w0" if d == 0 else d - 1, x["iter_count"], x["n_restorations"]))
        print(b, {k: v for k, v in out.items()}, flush=True)


def trace(draws):
    """Per-iteration trace of the kernel (the ``trace`` variant, small-fleet build, one agent) and
    of the oracle on the perturbed starts ``draws`` (-1: w0): mu, objective, step sizes and
    line-search trials (kernel), refinement steps (both)."""
    import torch
    from oracle import ipm
    from agentlib_mpc_amd.runtime.native import STATS_BYTES, stats_to_dicts
    from tests.test_multi_minima import perturbed
    case = case_of(REF)
    p, lbw, ubw, w0 = case.oracle_inputs
    dev = torch.device("cuda")
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a)[None], device=dev)  # noqa: E731
    nat = case.backend._native()
    rc = nat.lib.mpcx_problem_small_fleet(nat.handle, str(vdir() / "lds_trace.hsaco").encode(), -1)
    assert rc == 0, rc
    nat.set_small_fleet_max(1 << 30)
    nat.set_options(**REF)
    nat.reserve(1)
    for d in [int(x) for x in draws]:
        w = w0 if d < 0 else perturbed(w0, seed=0, k=d)
        ipm.IT_TRACE = []
        r = ipm.solve(case.oracle.functions(p), w, lbw, ubw, case.oracle.lbg(p), case.oracle.ubg(p), ipm.IPMOptions(**REF))
        print(f"=== draw {d}: oracle {r.status} it {r.iterations} resto {r.n_resto}", flush=True)
        for row in ipm.IT_TRACE:
            if row[0] == "ls":
                print("oracle resto-ls it=%d acc=%d mu=%.6e theta=%.6e phi=%.14e gphid=%.6e amin=%.3e amax=%.3e "
                      "alpha=%.3e thmin=%.3e thmax=%.3e" % row[1:], flush=True)
            else:
                print("oracle it=%d inner=%d mu=%.6e fx=%.14e refine=%d" % row, flush=True)
        ipm.IT_TRACE = None
        kp, kl, ku, kw = case.backend.problem.to_kernel(p, lbw, ubw, w)
        st = torch.zeros(STATS_BYTES, dtype=torch.uint8, device=dev)
        tw = T(kw)
        print(f"=== draw {d}: kernel", flush=True)
        nat.solve(T(kp), T(kl), T(ku), tw, stats=st, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        x = stats_to_dicts(st.cpu().numpy().tobytes())[0]
        print(f"=== draw {d}: kernel {x['return_status']} it {x['iter_count']} resto {x['n_restorations']}", flush=True)


def kkt(args):
    """CPU, oracle only: the inertia tests of outer iteration IT (default 35) on perturbed start D
    (default 6): each tried dw with the LDL^T inertia the oracle uses and the eigenvalue count of
    the same matrix, its norm and its eigenvalues nearest zero -- is the inertia decision there
    above rounding?  Then the oracle's nonzero inertia shifts of the whole run."""
    from oracle import ipm
    from tests.test_multi_minima import perturbed
    d = int(args[0]) if args else 6
    it_ = int(args[1]) if len(args) > 1 else 35
    case = case_of(REF)
    p, lbw, ubw, w0 = case.oracle_inputs
    w = w0 if d < 0 else perturbed(w0, seed=0, k=d)
    got = []

    def hook(it, inner, dw, dc, K, npos, nneg, nzero):
        if it == it_ and not inner:
            got.append((dw, npos, nneg, nzero, np.linalg.eigvalsh(K)))
    ipm.KKT_HOOK, ipm.IT_TRACE = hook, []
    r = ipm.solve(case.oracle.functions(p), w, lbw, ubw, case.oracle.lbg(p), case.oracle.ubg(p), ipm.IPMOptions(**REF))
    print(f"draw {d}: oracle {r.status} at {r.iterations} iterations; inertia wanted: pos {len(w)} neg "
          f"{len(case.oracle.lbg(p))}")
    for dw, npos, nneg, nzero, ev in got:
        print(f"it {it_} dw={dw:g}: LDL^T pos {npos} neg {nneg} zero {nzero}; eigvalsh pos {(ev > 0).sum()} neg {(ev < 0).sum()}; "
              f"max|eig| {np.abs(ev).max():.3e} (eps x max|eig| = {np.finfo(float).eps * np.abs(ev).max():.1e}); "
              f"eigs in (-10, 10): {np.round(np.sort(ev[np.abs(ev) < 10])[:6], 3)}")
    print("oracle inertia shifts (iteration, in restoration, dw, dc):",
          [row[1:] for row in ipm.IT_TRACE if row[0] == "dw" and row[3] != 0.0])
    ipm.KKT_HOOK = ipm.IT_TRACE = None


if __name__ == "__main__":
    if sys.argv[1] == "kkt":
        kkt(sys.argv[2:])
        sys.exit(0)
    if sys.argv[1] == "trace":
        trace(sys.argv[2:])
        sys.exit(0)
    if sys.argv[1] == "dist":
        dist(sys.argv[2:])
        sys.exit(0)
    {"build": build, "run": run}[sys.argv[1]](sys.argv[2:] or list(VARIANTS))
