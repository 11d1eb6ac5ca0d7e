"""ORACLE (test infrastructure only) — the fleet driver's device interface on the CPU.

``CpuFleetOps`` restates every ADMM kernel of `agentlib-mpc_amd/csrc/admm_kernels.hip` in
numpy (moments, finalize with per-block totals, multiplier / diff updates, shifts, row
moves) and solves each class's agents with the C IPM restatement over the class's
generated model compiled for the host (`oracle/c/gen_model.cpp`, OpenMP over the host
cores).  With it, :class:`agentlib_mpc_amd.admm.fleet.ADMMFleet` runs unchanged on the
CPU: the CPU baseline of the ADMM legs in bench.py.  ``tests/cpu_admm_ops.py`` reuses the
arithmetic with the numpy oracle IPM for the CPU tests of the driver.
"""

from __future__ import annotations

import os

import numpy as np
import torch

NMOM = 5
TOTALS = 8
STATUS_WORD = 13   # int32 index of mpcx_stats.status


class CpuFleetOps:
    """ADMM arithmetic in numpy; ``solve`` through the host build of the generated model."""

    def __init__(self, ipopt: dict = None, threads: int = 0):
        self.ipopt = dict(ipopt or {"tol": 1e-8, "max_iter": 500, "acceptable_iter": 0})
        self.threads = threads or int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)

    def active_map(self, n, active, amap, count):
        """numpy restatement of ``mpcx_active_map`` (admm_kernels.hip k_active_map)."""
        idx = np.flatnonzero(active.numpy()[:n] != 0)
        m = amap.numpy()
        m[:idx.size] = idx
        m[idx.size:n] = -1
        count.numpy()[0] = idx.size

    def solve(self, cls, active=None, agent_map=None, n_launch=None):
        from oracle import cbuild

        P, LB, UB, W = (t.numpy() for t in (cls.P, cls.LB, cls.UB, cls.W))
        st = cls.ST.view(torch.int32).view(cls.n, -1).numpy()
        act = np.ones(cls.n, bool) if active is None else active.numpy() != 0
        if agent_map is not None:  # the mapped launch: only the first n_launch map entries run
            m = agent_map.numpy()[:int(n_launch)]
            sel = np.zeros(cls.n, bool)
            sel[m[m >= 0]] = True
            act &= sel
        idx = np.flatnonzero(act)
        if idx.size == 0:
            return
        opts = dict(self.ipopt)
        tol, mi = opts.pop("tol"), opts.pop("max_iter")
        w, stats, _ = cbuild.solve_generated_fleet(cls.backend.problem.gen, P[idx], LB[idx], UB[idx], W[idx],
                                                   threads=self.threads, tol=tol, max_iter=mi, **opts)
        W[idx] = w
        st[idx, STATUS_WORD] = [s["status"] for s in stats]

    def gather_rows(self, T, src, cols, dst, dst_rows):
        dst.numpy()[dst_rows.numpy()] = src.numpy()[:, cols.numpy()]

    def scatter_rows(self, T, src, src_rows, dst, cols):
        s = src.numpy()
        rows = np.arange(dst.shape[0]) if src_rows is None else src_rows.numpy()
        d = dst.numpy()
        d[:, cols.numpy()] = s[rows]

    def scatter_plan(self, moves, dst):
        return ("s", list(moves), dst)

    def gather_plan(self, T, src, moves):
        return ("g", T, src, list(moves))

    def run_plan(self, plan):
        if plan[0] == "s":
            for T, src, rows, cols in plan[1]:
                self.scatter_rows(T, src, rows, plan[2], cols)
        else:
            _, T, src, moves = plan
            for cols, dst, rows in moves:
                self.gather_rows(T, src, cols, dst, rows)

    def fill_column(self, dst, col, value):
        dst.numpy()[:, col] = value

    def moments_size(self, n_groups, n_blocks, T):
        return n_groups * (NMOM * T + 1) + TOTALS * n_blocks

    @staticmethod
    def _off(g, n_global, n_blocks, T):
        return g * (NMOM * T + 1) + (TOTALS * n_blocks if g >= n_global else 0)

    def moments(self, n_groups, n_global, n_blocks, T, gstart, max_rows, X, LAM, center, out, row_on=None):
        gs, x, c, o = gstart.numpy(), X.numpy(), center.numpy(), out.numpy()
        lam = None if LAM is None else LAM.numpy()
        on = np.ones(x.shape[0], bool) if row_on is None else row_on.numpy() != 0
        for g in range(n_groups):
            rows = np.arange(gs[g], gs[g + 1])
            rows = rows[on[rows]]
            if rows.size == 0:
                continue
            b = self._off(g, n_global, n_blocks, T)
            d = x[rows] - c[g]
            o[b:b + T] += d.sum(0)
            o[b + T:b + 2 * T] += (d * d).sum(0)
            if lam is not None:
                l = lam[rows]
                o[b + 2 * T:b + 3 * T] += l.sum(0)
                o[b + 3 * T:b + 4 * T] += (l * l).sum(0)
                o[b + 4 * T:b + 5 * T] += (l * d).sum(0)
            o[b + NMOM * T] += rows.size

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

    def consensus_multipliers(self, n_groups, T, gstart, max_rows, X, mean, rho_s, rho_g, active_g, LAM,
                              row_on=None):
        gs, x, m, lam = gstart.numpy(), X.numpy(), mean.numpy(), LAM.numpy()
        ron = np.ones(x.shape[0], bool) if row_on is None else row_on.numpy() != 0
        for g in range(n_groups):
            on, rho = self._g(rho_s, rho_g, active_g, g)
            if on:
                rows = np.arange(gs[g], gs[g + 1])
                rows = rows[ron[rows]]
                lam[rows] -= rho * (m[g] - x[rows])

    def exchange_update(self, n_groups, T, gstart, max_rows, X, mean, diff, gmult, update, rho_s, rho_g,
                        active_g, row_on=None):
        gs, x, m, df = gstart.numpy(), X.numpy(), mean.numpy(), diff.numpy()
        ron = np.ones(x.shape[0], bool) if row_on is None else row_on.numpy() != 0
        for g in range(n_groups):
            on, rho = self._g(rho_s, rho_g, active_g, g)
            if not on:
                continue
            rows = np.arange(gs[g], gs[g + 1])
            rows = rows[ron[rows]]
            df[rows] = x[rows] - m[g]
            if update:
                gmult.numpy()[g] += rho * m[g]

    def shift(self, T, shift, x):
        a = x.numpy()
        if shift:
            a[:, :T - shift] = a[:, shift:].copy()

    # -- the coordinators' stopping test (restates admm_kernels.hip k_block_stop / _expand) ----
    def block_stop(self, it, totals, crit, rho_b, active_b, iters_b, record, n_active, clock, control=None):
        import time

        if clock is not None:
            clock.numpy()[it] = int(time.perf_counter() * 1e9)
        if it == 0:
            if n_active is not None and active_b is not None:
                n_active.numpy()[0] += int((active_b.numpy() != 0).sum())
            if control is not None:
                control.numpy()[0] = float(n_active.numpy()[0])
            return
        use_rel, abs_tol, rel_tol, primal_tol, dual_tol, thr, fac = crit
        t = totals.numpy().reshape(-1, TOTALS)
        prim = np.sqrt(np.maximum(t[:, 0], 0.0))
        dual = np.sqrt(np.maximum(t[:, 1], 0.0))
        if use_rel:
            scale_p = np.maximum(np.sqrt(np.maximum(t[:, 2], 0.0)), np.sqrt(np.maximum(t[:, 3], 0.0)))
            conv = (prim < np.sqrt(t[:, 6]) * abs_tol + rel_tol * scale_p) & \
                   (dual < np.sqrt(t[:, 5]) * abs_tol + rel_tol * np.sqrt(np.maximum(t[:, 4], 0.0)))
        else:
            conv = (prim < primal_tol) & (dual < dual_tol)
        act = active_b.numpy() != 0
        rho = rho_b.numpy().reshape(-1)
        if thr > 1.0:
            up = act & (prim > thr * dual)
            down = act & ~up & (dual > thr * prim)
            rho[:] = np.where(up, rho * fac, np.where(down, rho / fac, rho))
        rec = record.numpy().reshape(-1, t.shape[0], 4)
        rec[it - 1] = np.stack([prim, dual, rho, act.astype(float)], axis=1)
        done = act & conv
        active_b.numpy()[done] = 0
        iters_b.numpy()[done] = it
        if n_active is not None:
            n_active.numpy()[it] += int((act & ~conv).sum())
        if control is not None:  # the control slot of the next all-reduce (C ABI v10)
            control.numpy()[0] = float(n_active.numpy()[it])

    def block_expand(self, idx, active_b, rho_b, part, out_active, out_rho):
        i = idx.numpy()
        if out_active is not None:
            a = active_b.numpy()[i] != 0
            if part is not None:
                a &= part.numpy() != 0
            out_active.numpy()[:] = a.astype(np.int32)
        if out_rho is not None:
            out_rho.numpy().reshape(-1)[:] = rho_b.numpy().reshape(-1)[i]

    def stats_count(self, n, stats, active, counts):
        """numpy restatement of ``mpcx_stats_count`` (admm_kernels.hip k_stats_count)."""
        from agentlib_mpc_amd.runtime.native import STATS_BYTES

        w = stats.numpy().view(np.int32).reshape(n, STATS_BYTES // 4)
        on = np.ones(n, bool) if active is None else active.numpy() != 0
        st = w[:, 13]
        c = counts.numpy()
        c[0] += int((((st == 0) | (st == 1)) & on).sum())
        c[1] += int(w[:, 15][on].sum())

    def clock_hz(self) -> float:
        return 1e9
