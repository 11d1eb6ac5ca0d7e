"""The infeasible fixture_mpc case of test_gpu_long_restoration_run_follows_the_oracle (reference
IPOPT options): how far does the oracle's own restoration path carry a 1e-12 relative change of the
starting point?  For seeded perturbations w = w0 * (1 + 1e-12 N(0,1)) (tests/test_multi_minima.py
perturbed), the oracle is run to max_iter = k for a few k and to the end; printed: status, iterations,
restorations, objective and the point's max relative deviation from the unperturbed run at that k.
CPU only, oracle only.  usage: python scripts/resto_chaos.py [n_perturbations] > profiles/r06/resto_chaos.txt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "agentlib-mpc_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

from oracle import ipm  # noqa: E402
from tests import configs  # noqa: E402
from tests.test_multi_minima import perturbed  # noqa: E402

KW = {"T_lb": 255.0, "T_ub": 302.0, "disturbance": 270.0, "T0": 290.0}
REF = dict(tol=1e-4, max_iter=100, acceptable_tol=0.1, acceptable_iter=5,
           acceptable_constr_viol_tol=1.0, acceptable_compl_inf_tol=1.0)
KS = (30, 35, 40, 100)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
case = configs.CASES["fixture_mpc"](**KW)
p, lbw, ubw, w0 = case.oracle_inputs
fns, lbg, ubg = case.oracle.functions(p), case.oracle.lbg(p), case.oracle.ubg(p)
print(f"fixture_mpc {KW}, oracle IPM (oracle/ipm.py), reference options {REF}; w = w0 * (1 + 1e-12 N(0,1)), seed 0")
print("per max_iter k: status iterations restorations objective max|x - x_base|/(1 + |x_base|)")
base = {}
outcomes = {}
for d in range(-1, n):
    w = w0 if d < 0 else perturbed(w0, seed=0, k=d)
    cols = []
    for k in KS:
        r = ipm.solve(fns, w, lbw, ubw, lbg, ubg, ipm.IPMOptions(**dict(REF, max_iter=k)))
        base.setdefault(k, r)
        dev = float(np.max(np.abs(r.x - base[k].x) / (1.0 + np.abs(base[k].x))))
        cols.append(f"k={k}: {r.status[:14]:14s} {r.iterations:3d} {r.n_resto:2d} {r.f:.8e} {dev:.1e}")
        if k == KS[-1]:
            outcomes.setdefault(r.status, []).append(d)
    print(f"{'w0' if d < 0 else d:>3} | " + " | ".join(cols), flush=True)
print("final statuses (draws):", outcomes)
