"""Device-resident closed loop for a fleet of same-structure agents.

The plugin API (`MI355XBackend.solve_batch`, the drop-in for
`OptimizationBackend.solve` of every agent, `core/casadi_backend.py:133-139`)
re-marshals every agent's ``MPCVariable`` dict on each control step -- a Python
walk over agents x variables that costs far more than the kernel at fleet sizes.
A fleet that runs one structure in closed loop changes only a few scalar inputs
per step (the new measurement of each agent's states, `modules/mpc/mpc.py:
300-341`), so :class:`FleetSession` keeps the NLP inputs and the warm start
resident in HBM and moves only those per-agent columns across PCIe:

* ``update(name, values)``: host [n] -> device, scattered into every parameter /
  bound column that the marshalling derives from ``name`` (found once by probing
  the marshalling, so the mapping is the reference's own: initial-state
  parameter, the x_0 bounds it overrides, constant parameters on their grid);
* ``solve()``: one kernel launch on the resident arrays; the solution vector is
  updated in place and is the next step's initial guess -- the reference's
  remembered previous optimum (`core/discretization.py:221-223`, `247-251`);
* ``first_values(name)``: the actuation of every agent (first grid value >= 0,
  `modules/mpc/mpc.py:342-357`), device gather, n doubles back.
"""

from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np


class FleetSession:
    def __init__(self, backend, batch_vars: Sequence[dict], now: float = 0.0, device: str = "cuda"):
        import torch

        self.backend = backend
        self.prob = prob = backend.problem
        self.n = n = len(batch_vars)
        self.template = batch_vars[0]
        self.now = now
        p, lbw, ubw, w0 = prob.marshal.inputs(batch_vars, now)
        kp, kl, ku, kw = prob.to_kernel(p, lbw, ubw, w0)
        dev = torch.device(device)
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)  # noqa: E731
        self.p, self.lbw, self.ubw, self.w = T(kp), T(kl), T(ku), T(kw)
        self.lbw_ref = np.array(lbw, dtype=np.float64)  # reference-layout bounds (fixed variables the kernel NLP drops)
        self.dev = dev
        self._maps: Dict[str, List[Tuple[str, np.ndarray]]] = {}
        self._lam_g = self._stats = None

    # -- input columns ----------------------------------------------------------------
    def columns_of(self, name: str) -> List[Tuple[str, np.ndarray]]:
        """Kernel-order (array, columns) that the marshalling fills with the scalar value
        of ``name``: two probe agents that differ only in that value; every column that
        changes must equal the probed value (a copy), else the input is not a scalar
        column input and :meth:`update` refuses it."""
        if name in self._maps:
            return self._maps[name]
        import copy

        prob = self.prob
        base = self.template[name].value
        if not isinstance(base, (int, float, np.floating, np.integer)):
            raise TypeError(f"{name}: only scalar inputs can be updated in place (got {type(base).__name__})")
        probe = []
        for v in (float(base), float(base) + 1.2345):
            cv = copy.copy(self.template)
            cv[name] = copy.copy(self.template[name])
            cv[name].value = v
            probe.append(cv)
        ref = prob.marshal.inputs(probe, self.now)
        outs = prob.to_kernel(*ref)
        maps = []
        # reference-layout lower bounds: solution() rebuilds the variables the kernel NLP
        # drops (fixed past values of lifted NARX problems) from them
        outs = tuple(outs[:3]) + (ref[1],)
        for key, arr in zip(("p", "lbw", "ubw", "lbw_ref"), outs):
            a0, a1 = arr[0], arr[1]
            changed = np.flatnonzero(~((a0 == a1) | (np.isnan(a0) & np.isnan(a1))))
            if changed.size:
                if not np.all(a1[changed] == float(base) + 1.2345):
                    raise ValueError(f"{name}: derived (not copied) inputs in {key}; re-marshal instead")
                maps.append((key, changed))
        self._maps[name] = maps
        return maps

    def update(self, name: str, values) -> None:
        """New per-agent values [n] of the scalar input ``name`` (stream-ordered)."""
        import torch

        v = torch.as_tensor(np.ascontiguousarray(values, dtype=np.float64)).to(self.dev, non_blocking=True)
        if v.shape != (self.n,):
            raise ValueError(f"{name}: expected {self.n} values, got shape {tuple(v.shape)}")
        for key, cols in self.columns_of(name):
            if key == "lbw_ref":
                self.lbw_ref[:, cols] = np.asarray(values, dtype=np.float64)[:, None]
                continue
            arr = getattr(self, key)
            idx = torch.as_tensor(cols, device=self.dev)
            arr[:, idx] = v[:, None].expand(-1, idx.numel())

    # -- solve ----------------------------------------------------------------------------
    def solve(self) -> None:
        """One batched solve on the resident inputs; the solution replaces the guess."""
        import torch

        from agentlib_mpc_amd.runtime.native import STATS_BYTES

        if self._stats is None:
            self._lam_g = torch.empty((self.n, self.prob.nlp.kernel_ng), dtype=torch.float64, device=self.dev)
            self._stats = torch.zeros(self.n * STATS_BYTES, dtype=torch.uint8, device=self.dev)
        self.backend._native().solve(self.p, self.lbw, self.ubw, self.w, lam_g=self._lam_g, stats=self._stats)

    def first_values(self, name: str) -> np.ndarray:
        """First control/state value (grid time >= 0) of ``name`` for every agent."""
        nlp = self.prob.nlp
        for gname, lay in nlp.var_groups.items():
            full = self.prob.system_group_names.get(gname, [])
            if name in full:
                comp = full.index(name)
                j = next(j for j, t in enumerate(lay.grid) if t >= 0)
                ref_col = int(lay.index[comp, j])
                lift = nlp.lift
                col = ref_col if lift is None else int(lift.w_primary[ref_col])
                return self.w[:, col].cpu().numpy()
        raise KeyError(name)

    def stats(self):
        """Per-agent solver statistics of the last solve (structured array view)."""
        from agentlib_mpc_amd.runtime.native import StatsView, stats_array

        return StatsView(stats_array(self._stats.cpu().numpy()), {})

    def solution(self) -> np.ndarray:
        """Reference-layout solution vectors [n, nw] of the last solve."""
        return self.prob.from_kernel(self.w.cpu().numpy(), self.lbw_ref)
