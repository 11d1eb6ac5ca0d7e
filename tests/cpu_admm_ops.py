"""Test-side CPU implementation of the fleet driver's device interface
(`agentlib_mpc_amd/admm/ops.py`), used to exercise the driver's host logic —
partitioning, the single all-reduce per iteration, stopping rules — on CPU
(`gloo`) without a GPU: the numpy restatement of every ADMM kernel
(`oracle/cpu_fleet.py`) with ``solve`` running the oracle IPM per agent
(independent derivatives, `oracle/nlps.py`).  This is test infrastructure: the product
path uses NativeADMMOps only.
"""

from __future__ import annotations

import numpy as np
import torch

from oracle import ipm
from oracle.cpu_fleet import CpuFleetOps, NMOM, TOTALS  # noqa: F401


class CpuADMMOps(CpuFleetOps):
    def __init__(self, oracle_problems: dict, tol: float = 1e-10):
        super().__init__()
        self.oracle_problems = oracle_problems  # class name -> oracle.nlps.OracleProblem
        self.tol = tol

    def solve(self, cls, active=None, agent_map=None, n_launch=None):
        prob = self.oracle_problems[cls.name]
        P, LB, UB, W = (t.numpy() for t in (cls.P, cls.LB, cls.UB, cls.W))
        st = cls.ST.view(torch.int32).view(cls.n, -1).numpy()
        act = np.ones(cls.n, bool) if active is None else active.numpy() != 0
        if agent_map is not None:  # the mapped launch: only the first n_launch map entries run
            m = agent_map.numpy()[:int(n_launch)]
            sel = np.zeros(cls.n, bool)
            sel[m[m >= 0]] = True
            act &= sel
        for a in np.flatnonzero(act):
            p = P[a]
            r = ipm.solve(prob.functions(p), W[a].copy(), LB[a], UB[a], prob.lbg(p), prob.ubg(p),
                          ipm.IPMOptions(tol=self.tol, max_iter=500, acceptable_iter=0))
            W[a] = r.x
            st[a, 13] = {"Solve_Succeeded": 0, "Solved_To_Acceptable_Level": 1}.get(r.status, -1)
