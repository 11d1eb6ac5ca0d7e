"""Test-side CPU implementation of the fleet driver's device interface
(`agentlib_mpc_amd/admm/ops.py`), used to exercise the driver's host logic —
partitioning, the single all-reduce per iteration, stopping rules — on CPU
(`gloo`) without a GPU.  Every op restates its HIP kernel
(`csrc/admm_kernels.hip`) in numpy; ``solve`` runs the oracle IPM per agent.
This is test infrastructure: the product path uses NativeADMMOps only.
"""

from __future__ import annotations

import numpy as np
import torch

from oracle import ipm

NMOM = 5
TOTALS = 8


class CpuADMMOps:
    def __init__(self, oracle_problems: dict, tol: float = 1e-10):
        self.oracle_problems = oracle_problems  # class name -> oracle.nlps.OracleProblem
        self.tol = tol

    def solve(self, cls, active=None):
        prob = self.oracle_problems[cls.name]
        P, LB, UB, W = (t.numpy() for t in (cls.P, cls.LB, cls.UB, cls.W))
        st = cls.ST.view(torch.int32).view(cls.n, -1).numpy()
        act = np.ones(cls.n, bool) if active is None else active.numpy() != 0
        for a in np.flatnonzero(act):
            p = P[a]
            r = ipm.solve(prob.functions(p), W[a].copy(), LB[a], UB[a], prob.lbg(p), prob.ubg(p),
                          ipm.IPMOptions(tol=self.tol, max_iter=500, acceptable_iter=0))
            W[a] = r.x
            st[a, 13] = {"Solve_Succeeded": 0, "Solved_To_Acceptable_Level": 1}.get(r.status, -1)

    def gather_rows(self, T, src, cols, dst, dst_rows):
        dst.numpy()[dst_rows.numpy()] = src.numpy()[:, cols.numpy()]

    def scatter_rows(self, T, src, src_rows, dst, cols):
        s = src.numpy()
        rows = np.arange(dst.shape[0]) if src_rows is None else src_rows.numpy()
        d = dst.numpy()
        d[:, cols.numpy()] = s[rows]

    def fill_column(self, dst, col, value):
        dst.numpy()[:, col] = value

    def moments_size(self, n_groups, n_blocks, T):
        return n_groups * (NMOM * T + 1) + TOTALS * n_blocks

    @staticmethod
    def _off(g, n_global, n_blocks, T):
        return g * (NMOM * T + 1) + (TOTALS * n_blocks if g >= n_global else 0)

    def moments(self, n_groups, n_global, n_blocks, T, gstart, max_rows, X, LAM, center, out):
        gs, x, c, o = gstart.numpy(), X.numpy(), center.numpy(), out.numpy()
        lam = None if LAM is None else LAM.numpy()
        for g in range(n_groups):
            r0, r1 = gs[g], gs[g + 1]
            if r1 <= r0:
                continue
            b = self._off(g, n_global, n_blocks, T)
            d = x[r0:r1] - c[g]
            o[b:b + T] += d.sum(0)
            o[b + T:b + 2 * T] += (d * d).sum(0)
            if lam is not None:
                l = lam[r0:r1]
                o[b + 2 * T:b + 3 * T] += l.sum(0)
                o[b + 3 * T:b + 4 * T] += (l * l).sum(0)
                o[b + 4 * T:b + 5 * T] += (l * d).sum(0)
            o[b + NMOM * T] += r1 - r0

    @staticmethod
    def _g(rho, rho_g, active_g, g):
        on = active_g is None or active_g.numpy()[g] != 0
        return on, (rho if rho_g is None else float(rho_g.numpy()[g]))

    def finalize(self, g0, g1, n_global, n_blocks, T, mom, exchange, gmult, rho_s, rho_g, active_g, block_g,
                 mean, dmean, totals):
        o, m, dm, tot_all = mom.numpy(), mean.numpy(), dmean.numpy(), totals.numpy().reshape(-1)
        ex = None if exchange is None else exchange.numpy()
        gm = None if gmult is None else gmult.numpy()
        for g in range(g0, g1):
            on, rho = self._g(rho_s, rho_g, active_g, g)
            if not on:
                continue
            b = self._off(g, n_global, n_blocks, T)
            n = o[b + NMOM * T]
            if n <= 0:
                continue
            s1, s2 = o[b:b + T], o[b + T:b + 2 * T]
            c = m[g].copy()
            d = s1 / n
            new = c + d
            var = np.maximum(s2 - s1 * d, 0.0)
            m[g] = new
            dm[g] = c - new
            is_ex = ex is not None and ex[g]
            prim = (new * new).sum() if is_ex else var.sum()
            if is_ex:
                ls = ((gm[g] + rho * new) ** 2).sum()
            else:
                sl, sl2, slx = o[b + 2 * T:b + 3 * T], o[b + 3 * T:b + 4 * T], o[b + 4 * T:b + 5 * T]
                ls = (sl2 + 2 * rho * (slx - d * sl) + rho * rho * var).sum()
            k = 0 if block_g is None else int(block_g.numpy()[g])
            tot_all[k * TOTALS:(k + 1) * TOTALS] += [
                prim, ((rho * (c - new)) ** 2).sum(), (s2 + 2 * c * s1 + n * c * c).sum(),
                (new * new).sum(), ls, n, T if is_ex else n, 1.0]

    def consensus_multipliers(self, n_groups, T, gstart, max_rows, X, mean, rho_s, rho_g, active_g, LAM):
        gs, x, m, lam = gstart.numpy(), X.numpy(), mean.numpy(), LAM.numpy()
        for g in range(n_groups):
            on, rho = self._g(rho_s, rho_g, active_g, g)
            if on:
                lam[gs[g]:gs[g + 1]] -= rho * (m[g] - x[gs[g]:gs[g + 1]])

    def exchange_update(self, n_groups, T, gstart, max_rows, X, mean, diff, gmult, update, rho_s, rho_g,
                        active_g):
        gs, x, m, df = gstart.numpy(), X.numpy(), mean.numpy(), diff.numpy()
        for g in range(n_groups):
            on, rho = self._g(rho_s, rho_g, active_g, g)
            if not on:
                continue
            df[gs[g]:gs[g + 1]] = x[gs[g]:gs[g + 1]] - m[g]
            if update:
                gmult.numpy()[g] += rho * m[g]

    def shift(self, T, shift, x):
        a = x.numpy()
        if shift:
            a[:, :T - shift] = a[:, shift:].copy()
