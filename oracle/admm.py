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
