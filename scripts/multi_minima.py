"""Scan of the oracle's local minima on one_room_switch (tight options) under seeded relative
1e-12 perturbations of the starting point (CPU only, oracle only).
usage: python scripts/multi_minima.py [n_perturbations] > profiles/r06/multi_minima.txt"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "agentlib-mpc_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

from oracle import ipm  # noqa: E402
from tests import configs  # noqa: E402
from tests.test_multi_minima import TIGHT, perturbed  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
case = configs.CASES["one_room_switch"]()
p, lbw, ubw, w0 = case.oracle_inputs
fns, lbg, ubg = case.oracle.functions(p), case.oracle.lbg(p), case.oracle.ubg(p)
print("one_room_switch, oracle IPM (oracle/ipm.py), tol 1e-10, acceptable_iter 0; w = w0 * (1 + 1e-12 N(0,1)), seed 0")
print(f"{'draw':>5} {'status':<18} {'iters':>5} {'objective':>22} {'|x - x_base|_inf':>17} {'s':>5}")
base = None
seen = {}
for k in range(-1, n):
    w = w0 if k < 0 else perturbed(w0, seed=0, k=k)
    t = time.time()
    r = ipm.solve(fns, w, lbw, ubw, lbg, ubg, TIGHT)
    if base is None:
        base = r
    dx = float(np.max(np.abs(r.x - base.x)))
    seen.setdefault(round(float(r.f), 3), []).append(k)
    print(f"{'w0' if k < 0 else k:>5} {r.status:<18} {r.iterations:>5} {r.f:>22.12f} {dx:>17.3e} {time.time() - t:>5.1f}",
          flush=True)
print("minima reached (objective rounded to 1e-3: draws):", seen)
