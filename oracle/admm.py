"""ORACLE (test infrastructure only) — batched numpy restatement of the ADMM arithmetic.

Restates, over a segmented [rows][T] layout (participants of one alias are
contiguous rows), the reference updates:

* consensus mean / delta mean — ``ConsensusVariable.update_mean_trajectory``
  (`agentlib_mpc/data_structures/admm_datatypes.py:221-236`)
* consensus multipliers / primal residual — ``update_multipliers`` (:238-267)
* exchange mean, diffs, multiplier — ``ExchangeVariable`` (:292-324)
* residual norms — ``ADMMCoordinator._check_convergence``
  (`modules/dmpc/admm/admm_coordinator.py:354-435`)
* shift — ``shift_values_by_one`` (:275-282, :326-331)

Pinned against ``tests/golden/admm_golden.json`` (produced by executing the
reference module itself, see ``tests/golden/make_golden.py``).
"""

from __future__ import annotations

import numpy as np


def group_means(x, group_start, active=None, old_mean=None):
    """Returns (mean[g][T], delta_mean[g][T]); groups without active rows keep old values."""
    x = np.asarray(x, float)
    G = len(group_start) - 1
    T = x.shape[1]
    mean = np.zeros((G, T)) if old_mean is None else np.array(old_mean, float)
    dmean = np.zeros((G, T))
    act = np.ones(x.shape[0], bool) if active is None else np.asarray(active, bool)
    for g in range(G):
        rows = np.arange(group_start[g], group_start[g + 1])
        rows = rows[act[rows]]
        if rows.size == 0:
            continue
        m = x[rows].mean(axis=0)
        dmean[g] = mean[g] - m
        mean[g] = m
    return mean, dmean


def consensus_multipliers(x, lam, mean, group_start, rho, active=None):
    x = np.asarray(x, float)
    lam = np.array(lam, float)
    res = np.zeros_like(x)
    act = np.ones(x.shape[0], bool) if active is None else np.asarray(active, bool)
    for g in range(len(group_start) - 1):
        for r in range(group_start[g], group_start[g + 1]):
            if act[r]:
                res[r] = mean[g] - x[r]
                lam[r] = lam[r] - rho * res[r]
    return lam, res


def exchange_update(x, mean, group_start, lam_group, rho, active=None, diff=None):
    x = np.asarray(x, float)
    diff = np.zeros_like(x) if diff is None else np.array(diff, float)
    act = np.ones(x.shape[0], bool) if active is None else np.asarray(active, bool)
    for g in range(len(group_start) - 1):
        for r in range(group_start[g], group_start[g + 1]):
            if act[r]:
                diff[r] = x[r] - mean[g]
    lam = np.array(lam_group, float) + rho * np.asarray(mean, float)
    return diff, lam, np.array(mean, float)


def residual_norms(primal_residual, delta_mean, rho):
    """Primal / dual residual 2-norms as `admm_coordinator.py:389-394`."""
    return float(np.linalg.norm(np.ravel(primal_residual))), float(np.linalg.norm(rho * np.ravel(delta_mean)))


def shift(x, shift_by):
    x = np.asarray(x, float)
    return np.concatenate([x[:, shift_by:], x[:, x.shape[1] - shift_by:]], axis=1)


# ---------------------------------------------------------------------------
# Loop restatements (per-agent dictionaries, the reference's own formulas)
# ---------------------------------------------------------------------------

class _Consensus:
    """`admm_datatypes.py:160-282` (CouplingVariable + ConsensusVariable)."""

    def __init__(self):
        self.local = {}
        self.mean = [0]
        self.delta_mean = np.array([0.0])
        self.primal_residual = np.array([0.0])
        self.mult = {}

    def sources(self, active):
        # CouplingVariable._relevant_sources (`admm_datatypes.py:171-177`)
        return list(self.local) if active is None else [s for s in self.local if s in active]

    def update_mean(self, active=None):
        srcs = self.sources(active)
        if not srcs:
            return
        arr = np.array([self.local[s] for s in srcs])
        mean = np.mean(arr, axis=0)
        self.delta_mean = self.mean - mean
        self.mean = list(mean)

    def update_multipliers(self, rho, active=None):
        srcs = self.sources(active)
        if not srcs:
            return
        traj = np.array([self.local[s] for s in srcs])
        mul = np.array([self.mult[s] for s in srcs])
        self.primal_residual = np.array(self.mean) - traj
        new = mul - rho * self.primal_residual
        for i, s in enumerate(srcs):
            self.mult[s] = list(new[i])

    def shift(self, horizon):
        k = int(len(self.mean) / horizon)
        self.mean = self.mean[k:] + self.mean[-k:]
        for s, m in self.mult.items():
            self.mult[s] = m[k:] + m[-k:]


class _Exchange:
    """`admm_datatypes.py:285-331` (ExchangeVariable)."""

    def __init__(self):
        self.local = {}
        self.mean = [0]
        self.delta_mean = np.array([0.0])
        self.primal_residual = np.array([0.0])
        self.diff = {}
        self.mult = []

    def sources(self, active):
        return list(self.local) if active is None else [s for s in self.local if s in active]

    def update_mean(self, active=None):
        srcs = self.sources(active)
        if not srcs:
            return
        arr = np.array([self.local[s] for s in srcs])
        mean = np.mean(arr, axis=0)
        self.delta_mean = self.mean - mean
        self.mean = list(mean)
        for s in srcs:
            self.diff[s] = list(np.asarray(self.local[s]) - mean)

    def update_multipliers(self, rho, active=None):  # every round, whatever the sources (:311-324)
        self.primal_residual = np.array(self.mean)
        self.mult = list(self.mult + rho * self.primal_residual)

    def shift(self, horizon):
        k = int(len(self.mult) / horizon)
        self.mult = self.mult[k:] + self.mult[-k:]
        for s, d in self.diff.items():
            self.diff[s] = d[k:] + d[-k:]


def coordinated_round(participation, initial, solve, rho, horizon, admm_iter_max, primal_tol=1e-3,
                      dual_tol=1e-3, use_relative_tolerances=True, abs_tol=1e-3, rel_tol=1e-3,
                      penalty_change_threshold=-1.0, penalty_change_factor=2.0, T=None, state=None,
                      solve_batch=None, active=None, trace=None):
    """One round of ``ADMMCoordinator._fast_process`` (`admm_coordinator.py:259-321`).

    participation: {agent: {alias: "consensus"|"exchange"}}; initial: {agent: {alias: value}}
    solve(agent, {alias: (mean_or_diff, multiplier)}, rho) -> {alias: local trajectory}
    solve_batch (optional): [(agent, inputs)], rho -> [outputs] — the same solves of one
    iteration at once (they are independent; the fixture generators run them in parallel).
    active (optional): the agents with status ``ready`` this round (`admm_coordinator.py:
    323-353`); only they are solved and enter means, multiplier updates and the residual
    scalings (``sources=active_agents``); None: every registered agent.
    trace (optional list): gets {alias: mean} after every iteration's mean update.
    Returns (state, history [(primal, dual, rho after the variation)], iterations, converged).
    """
    if state is None:  # registration (`admm_coordinator.py:528-560`)
        state = {"vars": {}, "order": []}
        for ag, coups in participation.items():
            for al, kind in coups.items():
                v = state["vars"].setdefault(al, _Consensus() if kind == "consensus" else _Exchange())
                traj = [float(initial[ag][al])] * T
                v.local[ag] = traj
                if kind == "consensus":
                    v.mult[ag] = [0] * T
                else:
                    v.mult = [0] * T
    vars_ = state["vars"]
    for v in vars_.values():
        v.update_mean(active)
    for v in vars_.values():
        v.shift(horizon)
    hist = []
    converged = False
    it = 0
    for it in range(1, admm_iter_max + 1):
        reqs = []
        for ag, coups in participation.items():
            if active is not None and ag not in active:
                continue
            inp = {}
            for al, kind in coups.items():
                v = vars_[al]
                inp[al] = (np.array(v.mean), np.array(v.mult[ag])) if kind == "consensus" else \
                    (np.array(v.diff[ag]), np.array(v.mult))
            reqs.append((ag, inp))
        outs = solve_batch(reqs, rho) if solve_batch is not None else [solve(ag, inp, rho) for ag, inp in reqs]
        for (ag, _), out in zip(reqs, outs):
            for al in participation[ag]:
                vars_[al].local[ag] = list(np.ravel(out[al]))
        for v in vars_.values():
            v.update_mean(active)
        for v in vars_.values():
            v.update_multipliers(rho, active)
        if trace is not None:
            trace.append({al: [float(x) for x in v.mean] for al, v in vars_.items()})
        prim, dual, flat_locals, flat_means, flat_mult = [], [], [], [], []
        for v in vars_.values():
            prim.extend(v.primal_residual.flatten())
            dual.extend((rho * v.delta_mean).flatten())
            flat_locals.extend([v.local[s] for s in v.sources(active)])
            flat_means.extend(v.mean)
            if isinstance(v, _Consensus):
                flat_mult.extend([v.mult[s] for s in v.sources(active)])
            else:
                flat_mult.extend(v.mult)
        pn, dn = float(np.linalg.norm(prim)), float(np.linalg.norm(dual))
        # _check_convergence varies the penalty first and records it afterwards
        # (`admm_coordinator.py:396-397`)
        if penalty_change_threshold > 1:
            if pn > penalty_change_threshold * dn:
                rho = rho * penalty_change_factor
            elif dn > penalty_change_threshold * pn:
                rho = rho / penalty_change_factor
        hist.append((pn, dn, rho))
        if use_relative_tolerances:
            sp = max(_norm_lists(flat_locals), float(np.linalg.norm(flat_means)))
            sd = _norm_lists(flat_mult)
            eps_pri = np.sqrt(len(flat_mult)) * abs_tol + rel_tol * sp
            eps_dual = np.sqrt(len(flat_locals)) * abs_tol + rel_tol * sd
            conv = pn < eps_pri and dn < eps_dual
        else:
            conv = pn < primal_tol and dn < dual_tol
        if conv:
            converged = True
            break
    return state, hist, it, converged


def register(state, agent, coups, initial, T):
    """``ADMMCoordinator.register_agent`` (`admm_coordinator.py:527-560`): the agent's local
    trajectories start from its initial value, its consensus multipliers from zero, and the
    multiplier of an exchange alias it joins is reset to zero."""
    for al, kind in coups.items():
        v = state["vars"].setdefault(al, _Consensus() if kind == "consensus" else _Exchange())
        v.local[agent] = [float(initial[al])] * T
        if kind == "consensus":
            v.mult[agent] = [0] * T
        else:
            v.mult = [0] * T


def _norm_lists(items):
    return float(np.sqrt(sum(float(np.sum(np.square(np.asarray(x, float)))) for x in items)))


def local_round(participation, initial, solve, rho, shift_by, max_iterations, T=None, state=None):
    """One control step of ``LocalADMM.process`` (`modules/dmpc/admm/admm.py:873-937`) for
    all agents at once. Returns (state, per-iteration {alias: mean})."""
    if state is None:
        state = {"local": {}, "mult": {}}
        for ag, coups in participation.items():
            for al in coups:
                state["local"][(ag, al)] = [float(initial[ag][al])] * T
                state["mult"][(ag, al)] = [0] * T
    loc, mult = state["local"], state["mult"]

    def sh(seq):
        return list(seq[shift_by:]) + list(seq[-shift_by:])

    for k in list(loc):
        loc[k] = sh(loc[k])
        mult[k] = sh(mult[k])
    aliases = sorted({al for coups in participation.values() for al in coups})

    def means():
        out = {}
        for al in aliases:
            out[al] = np.mean(np.array([loc[(ag, al)] for ag, c in participation.items() if al in c]), axis=0)
        return out

    mean = means()
    hist = []
    for _ in range(max_iterations):
        for ag, coups in participation.items():
            inp = {}
            for al, kind in coups.items():
                own = np.array(loc[(ag, al)])
                inp[al] = (mean[al], np.array(mult[(ag, al)])) if kind == "consensus" else \
                    (own - mean[al], np.array(mult[(ag, al)]))
            out = solve(ag, inp, rho)
            for al in coups:
                loc[(ag, al)] = list(np.ravel(out[al]))
        mean = means()
        for ag, coups in participation.items():
            for al, kind in coups.items():
                own = np.array(loc[(ag, al)])
                lam = np.array(mult[(ag, al)])
                if kind == "consensus":
                    mult[(ag, al)] = list(lam - rho * (mean[al] - own))
                else:
                    diff = own - mean[al]
                    mult[(ag, al)] = list(lam - rho * (diff - own))
        hist.append({al: mean[al].copy() for al in aliases})
    return state, hist
