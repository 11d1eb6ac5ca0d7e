"""Diagnostic: per-case solver statistics of the kernel (current build or, with
MPCX_DEFINES=MPCX_NO_STATIC, the dense-only variant) next to the oracle IPM.
usage: python scripts/static_diag.py [--build-only]"""
import sys

sys.path[:0] = [".", "agentlib-mpc_amd"]
import numpy as np  # noqa: E402

from tests import configs  # noqa: E402

CASES = [("one_room", {}), ("mhe_room", {}), ("mhe_room", {"theta": 5.8, "noise": 0.05, "seed": 3, "w_T_wall": 0.5}),
         ("mhe_room", {"theta": 7.0}), ("mhe_room_u", {}), ("rng_room_mpc", {}), ("room_nn", {})]

if __name__ == "__main__":
    build_only = "--build-only" in sys.argv
    for name, kw in CASES:
        case = configs.CASES[name](**kw)
        if build_only:
            case.backend.problem.compile()
            continue
        from oracle import ipm

        p, lbw, ubw, w0 = case.oracle_inputs
        ref = ipm.solve(case.oracle.functions(p), w0, lbw, ubw, case.oracle.lbg(p), case.oracle.ubg(p),
                        ipm.IPMOptions(tol=1e-10, max_iter=500, acceptable_iter=0))
        r = case.backend.solve_batch(0.0, [case.current_vars])[0]
        st = r.stats
        print(f"{name} {kw}: kernel {st['return_status']} it {st['iter_count']} obj {st['obj']:.8f} "
              f"ic {st.get('n_inertia_corrections')} fact {st.get('n_factorizations')} chain {st.get('n_block_chain')} dense {st.get('n_dense_stages')}"
              f" | oracle {ref.status} it {ref.iterations} obj {ref.f:.8f}", flush=True)
