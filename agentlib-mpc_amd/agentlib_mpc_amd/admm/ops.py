"""Device operations of the ADMM fleet driver: the C-ABI kernels of `libmpcx.so`.

:class:`NativeADMMOps` is the product implementation — every call is one
stream-ordered launch through `include/mpcx.h` on device tensors (torch is
only the allocator).  The fleet driver (`admm/fleet.py`) is written against
this small interface so that its host-side orchestration (partitioning,
collectives, stopping rules) can also be exercised by CPU tests with a
test-side implementation; there is no CPU implementation in the package.
"""

from __future__ import annotations

import ctypes
from typing import Optional

from agentlib_mpc_amd.runtime import native


def _p(t) -> Optional[ctypes.c_void_p]:
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class NativeADMMOps:
    """ADMM arithmetic + NLP solves on the GPU (C ABI, HIP kernels)."""

    def __init__(self, stream=None):
        self.lib = native.load_library()
        self._stream = stream

    @property
    def stream(self):
        import torch

        s = self._stream if self._stream is not None else torch.cuda.current_stream()
        return ctypes.c_void_p(s.cuda_stream)

    def _chk(self, rc, name):
        if rc != 0:
            raise native.NativeError(f"{name} failed ({rc})")

    # -- NLP solves ---------------------------------------------------------------------
    def solve(self, cls, active=None, agent_map=None, n_launch=None) -> None:
        """Batched solve of one class; ``active`` (int32 [n] device tensor or None) skips the
        agents of converged blocks; ``agent_map`` + ``n_launch`` (mpcx_active_map's output and a
        bound on its count) launch only that many workgroups (``mpcx_batch_solve_mapped``)."""
        cls.native.solve(cls.P, cls.LB, cls.UB, cls.W, lam_g=cls.LAMG, stats=cls.ST, active=active,
                         stream=self.stream.value, agent_map=agent_map, n_launch=n_launch)

    def active_map(self, n, active, amap, count):
        """``mpcx_active_map``: the active agents' indices first (increasing), then -1; count[0]."""
        self._chk(self.lib.mpcx_active_map(n, _p(active), _p(amap), _p(count), self.stream), "mpcx_active_map")

    # -- moves ---------------------------------------------------------------------------
    def gather_rows(self, T, src, cols, dst, dst_rows):
        self._chk(self.lib.mpcx_gather_rows(src.shape[0], T, _p(src), src.shape[1], _p(cols), _p(dst),
                                            _p(dst_rows), self.stream), "mpcx_gather_rows")

    def scatter_rows(self, T, src, src_rows, dst, cols):
        self._chk(self.lib.mpcx_scatter_rows(dst.shape[0], T, _p(src), _p(src_rows), _p(dst), dst.shape[1],
                                             _p(cols), self.stream), "mpcx_scatter_rows")

    def scatter_plan(self, moves, dst):
        """A prepared ``mpcx_scatter_rows_multi`` launch of several ``scatter_rows`` into one
        destination (``moves`` = [(T, src, src_rows, cols)], not writing the same element): the
        descriptor table is built once on the device; :meth:`run_plan` issues it."""
        import torch

        words = []
        for T, src, rows, cols in moves:
            words += [src.data_ptr(), 0 if rows is None else rows.data_ptr(), cols.data_ptr(), int(T)]
        desc = torch.tensor(words, dtype=torch.int64, device=dst.device)
        args = (dst.shape[0], len(moves), _p(desc), max(int(m[0]) for m in moves), _p(dst), dst.shape[1])
        return (self.lib.mpcx_scatter_rows_multi, args, desc, "mpcx_scatter_rows_multi")

    def gather_plan(self, T, src, moves):
        """A prepared ``mpcx_gather_rows_multi`` launch of several ``gather_rows`` from one source
        (``moves`` = [(cols, dst, dst_rows)], each of ``T`` columns)."""
        import torch

        words = []
        for cols, dst, rows in moves:
            words += [dst.data_ptr(), rows.data_ptr(), cols.data_ptr(), int(T)]
        desc = torch.tensor(words, dtype=torch.int64, device=src.device)
        args = (src.shape[0], len(moves), _p(desc), int(T), _p(src), src.shape[1])
        return (self.lib.mpcx_gather_rows_multi, args, desc, "mpcx_gather_rows_multi")

    def run_plan(self, plan):
        """Issue a prepared fused move on the current stream (one launch, no host allocation)."""
        fn, args, _desc, name = plan
        self._chk(fn(*args, self.stream), name)

    def fill_column(self, dst, col, value):
        self._chk(self.lib.mpcx_fill_column(dst.shape[0], _p(dst), dst.shape[1], col, float(value),
                                            self.stream), "mpcx_fill_column")

    # -- ADMM arithmetic -------------------------------------------------------------------
    # rho_g / active_g / block_g: per-group penalty, freeze mask and block index (device
    # tensors, or None for one block with the scalar rho), see include/mpcx.h
    def moments_size(self, n_groups, n_blocks, T) -> int:
        return int(self.lib.mpcx_admm_moments_size(n_groups, n_blocks, T))

    # row_on: participation mask of the rows (device int32 [n_rows], None = every row),
    # the reference coordinator's active agents (include/mpcx.h, *_masked)
    def moments(self, n_groups, n_global, n_blocks, T, gstart, max_rows, X, LAM, center, out, row_on=None):
        self._chk(self.lib.mpcx_admm_moments_masked(n_groups, n_global, n_blocks, T, _p(gstart), max_rows, _p(X),
                                                    _p(LAM), _p(center), _p(row_on), _p(out), self.stream),
                  "mpcx_admm_moments_masked")

    def finalize(self, g0, g1, n_global, n_blocks, T, mom, exchange, gmult, rho, rho_g, active_g, block_g,
                 mean, dmean, totals):
        self._chk(self.lib.mpcx_admm_finalize(g0, g1, n_global, n_blocks, T, _p(mom), _p(exchange), _p(gmult),
                                              float(rho), _p(rho_g), _p(active_g), _p(block_g), _p(mean),
                                              _p(dmean), _p(totals), self.stream),
                  "mpcx_admm_finalize")

    def consensus_multipliers(self, n_groups, T, gstart, max_rows, X, mean, rho, rho_g, active_g, LAM,
                              row_on=None):
        self._chk(self.lib.mpcx_admm_consensus_multipliers_masked(n_groups, T, _p(gstart), max_rows, _p(X),
                                                                  _p(mean), float(rho), _p(rho_g), _p(active_g),
                                                                  _p(row_on), _p(LAM), None, self.stream),
                  "mpcx_admm_consensus_multipliers_masked")

    def exchange_update(self, n_groups, T, gstart, max_rows, X, mean, diff, gmult, update, rho, rho_g,
                        active_g, row_on=None):
        self._chk(self.lib.mpcx_admm_exchange_update_masked(n_groups, T, _p(gstart), max_rows, _p(X), _p(mean),
                                                            _p(diff), _p(gmult), int(bool(update)), float(rho),
                                                            _p(rho_g), _p(active_g), _p(row_on), self.stream),
                  "mpcx_admm_exchange_update_masked")

    # -- the coordinators' stopping test (include/mpcx.h mpcx_admm_block_stop / _expand) ----
    def block_stop(self, it, totals, crit, rho_b, active_b, iters_b, record, n_active, clock, control=None):
        """``crit`` = (use_relative, abs_tol, rel_tol, primal_tol, dual_tol, change_threshold,
        change_factor); device state tensors updated in place.  ``control``: the all-reduce's
        control slot (float64 [1]), receives n_active[it] (C ABI v10)."""
        nb = active_b.shape[0]
        self._chk(self.lib.mpcx_admm_block_stop(nb, it, _p(totals), int(crit[0]), *[float(v) for v in crit[1:]],
                                                _p(rho_b), _p(active_b), _p(iters_b), _p(record), _p(n_active),
                                                _p(clock), _p(control), self.stream), "mpcx_admm_block_stop")

    def block_expand(self, idx, active_b, rho_b, part, out_active, out_rho):
        self._chk(self.lib.mpcx_admm_block_expand(idx.shape[0], _p(idx), _p(active_b), _p(rho_b), _p(part),
                                                  _p(out_active), _p(out_rho), self.stream),
                  "mpcx_admm_block_expand")

    def expand_plan(self, entries, active_b, rho_b):
        """A prepared ``mpcx_admm_block_expand_multi`` launch (C ABI v15): ``entries`` =
        [(idx, part, out_active, out_rho)] -- each what :meth:`block_expand` would do, in one launch;
        :meth:`run_plan` issues it."""
        import torch

        words = []
        for idx, part, oa, orho in entries:
            words += [idx.shape[0]] + [0 if x is None else x.data_ptr() for x in (idx, part, oa, orho)]
        desc = torch.tensor(words, dtype=torch.int64, device=active_b.device)
        args = (len(entries), _p(desc), max(e[0].shape[0] for e in entries), _p(active_b), _p(rho_b))
        return (self.lib.mpcx_admm_block_expand_multi, args, desc, "mpcx_admm_block_expand_multi")

    def stats_plan(self, entries, counts):
        """A prepared ``mpcx_stats_count_multi`` launch (C ABI v15): ``entries`` = [(n, stats,
        active)] counted into ``counts`` in one launch."""
        import torch

        words = []
        for n, st, act in entries:
            words += [int(n), st.data_ptr(), 0 if act is None else act.data_ptr()]
        desc = torch.tensor(words, dtype=torch.int64, device=counts.device)
        args = (len(entries), _p(desc), max(int(e[0]) for e in entries), _p(counts))
        return (self.lib.mpcx_stats_count_multi, args, desc, "mpcx_stats_count_multi")

    def stats_count(self, n, stats, active, counts):
        """counts[0] += converged agents, counts[1] += their restoration calls (one launch)."""
        self._chk(self.lib.mpcx_stats_count(n, _p(stats), _p(active), _p(counts), self.stream), "mpcx_stats_count")

    def clock_hz(self) -> float:
        khz = int(self.lib.mpcx_device_clock_khz())
        if khz <= 0:
            raise native.NativeError(f"mpcx_device_clock_khz failed ({khz})")
        return 1e3 * khz

    def shift(self, T, shift, x):
        self._chk(self.lib.mpcx_admm_shift(x.shape[0], T, shift, _p(x), self.stream), "mpcx_admm_shift")
