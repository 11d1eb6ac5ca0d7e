"""Diagnostic (GPU): per ADMM iteration, every agent's local-solve IPM iteration count and status
on the C5 N=8 fixture round, kernel fleet vs the oracle fixture (tests/golden/c5_admm_N8.json)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]


def main():
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.admm.fleet import ADMMFleet

    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", f"c5_admm_N{N}.json")))
    opts = {"ipopt": {"tol": 1e-8, "max_iter": 500, "acceptable_iter": 0}}
    fl = ADMMFleet(bm.c5_fleet_classes(n_blocks=1, N=N, solver_options=opts))
    fl.solve_trace = []
    out = fl.run_coordinated(gold["rho"], admm_iter_max=gold["admm_iter_max"], use_relative_tolerances=False,
                             primal_tol=0.04, dual_tol=0.04, check_every=1)
    k = len(fl.classes)
    print("classes", [c.name for c in fl.classes], "trace", len(fl.solve_trace))
    for it in range(out["iterations"]):
        row = []
        for name, w in fl.solve_trace[it * k:(it + 1) * k]:
            row += [f"{name}:{int(x[0])}/{int(x[1])}" for x in w.cpu().numpy()]
        o = gold["local_solves"][it]
        print(it + 1, " ".join(row), "| oracle", " ".join(f"{a}:{v[1]}/{v[0][:6]}" for a, v in o.items()),
              "| prim %.6e %.6e" % (out["records"][it].primal_residual, gold["history"][it][0]))


if __name__ == "__main__":
    main()
