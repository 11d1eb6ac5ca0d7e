"""The state chain's twisted factorisation (csrc/mpcx_ipm.hip ``chain_factor_tw`` /
``chain_solve_tw``, r04): pivots from both ends of the block-tridiagonal chain at once, the
middle pivot last.  Host restatement with the kernel's block layout -- S11(j) (NC x NC, c_j =
[mu_j, x_{j+1}]), S00(j+1) (NX x NX, added on the x part), S10(j) (NC x NX, coupling c_j with the
x part of c_{j-1}), fixed states as identity rows -- and the kernel's ``bk_sweep`` restatement
for every pivot inverse, checked against the assembled chain matrix: inertia (what the inertia
correction reads) against its eigenvalues, solution against a dense solve, and against the
one-sided chain (``chain_factor`` / ``chain_solve``)."""

import numpy as np
import pytest

from tests.test_chain_sweep import sweep


def make_chain(rng, N, NX, NMU, fixed=()):
    NC = NX + NMU
    S11 = [rng.normal(size=(NC, NC)) for _ in range(N)]
    S11 = [a + a.T for a in S11]
    for a in S11:
        a[:NMU, :NMU] = 0.0  # bordered multipliers: zero leading block
        a[NMU:, NMU:] += 2.0 * NX * np.eye(NX)  # states: Hessian-like, mostly positive
    S00 = [None] + [(lambda b: b + b.T + 2.0 * NX * np.eye(NX))(rng.normal(size=(NX, NX))) for _ in range(1, N)]
    S10 = [None] + [0.5 * rng.normal(size=(NC, NX)) for _ in range(1, N)]
    fix = {j: set() for j in range(N)}
    for j, i in fixed:  # state i of x_{j+1} fixed: an identity row, no coupling through it
        fix[j].add(i)
        if j + 1 < N:
            S10[j + 1][:, i] = 0.0
        if j > 0:
            S10[j][NMU + i, :] = 0.0
    return S11, S00, S10, fix


def block(S11, S00, fix, j, NX, NMU):
    N = len(S11)
    C = S11[j].copy()
    if j + 1 < N:
        C[NMU:, NMU:] += S00[j + 1]
    return C


def override(C, fix_j, NMU):
    for i in fix_j:
        C[NMU + i, :] = 0.0
        C[:, NMU + i] = 0.0
        C[NMU + i, NMU + i] = 1.0
    return C


def full_matrix(S11, S00, S10, fix, NX, NMU):
    N, NC = len(S11), NX + NMU
    T = np.zeros((N * NC, N * NC))
    for j in range(N):
        T[j * NC:(j + 1) * NC, j * NC:(j + 1) * NC] = override(block(S11, S00, fix, j, NX, NMU), fix[j], NMU)
        if j > 0:
            T[j * NC:(j + 1) * NC, (j - 1) * NC + NMU:j * NC] = S10[j]
            T[(j - 1) * NC + NMU:j * NC, j * NC:(j + 1) * NC] = S10[j].T
    return T


def one_sided(S11, S00, S10, fix, NX, NMU, rhs):
    N = len(S11)
    Dinv, inert = [], np.zeros(3, int)
    for j in range(N):
        C = block(S11, S00, fix, j, NX, NMU)
        if j > 0:
            C -= S10[j] @ Dinv[j - 1][NMU:, NMU:] @ S10[j].T
        inv, i3 = sweep(override(C, fix[j], NMU))
        Dinv.append(inv)
        inert += i3
    y = [rhs[0]]
    for j in range(1, N):
        y.append(rhs[j] - S10[j] @ (Dinv[j - 1] @ y[j - 1])[NMU:])
    c = [None] * N
    for j in range(N - 1, -1, -1):
        t = y[j].copy()
        if j + 1 < N:
            t[NMU:] -= S10[j + 1].T @ c[j + 1]
        c[j] = Dinv[j] @ t
    return np.concatenate(c), tuple(inert)


def twisted(S11, S00, S10, fix, NX, NMU, rhs):
    """Line by line chain_factor_tw / chain_solve_tw (their step order: forward pivot jf = s and
    backward pivot jb = N-1-s together, the middle pivot CMID = N // 2 at step CSTEPS)."""
    N = len(S11)
    CMID = N // 2
    CSTEPS = max(CMID, N - 1 - CMID)
    Dinv, inert = [None] * N, np.zeros(3, int)
    for s in range(CSTEPS + 1):
        mid = s == CSTEPS
        jf, jb = (CMID if mid else s), N - 1 - s
        hf, hb = mid or s < CMID, (not mid) and jb > CMID
        jt = CMID if mid else jb
        bw = (CMID + 1 < N) if mid else (hb and jb + 1 < N)
        todo = []
        if hf:
            C = block(S11, S00, fix, jf, NX, NMU)
            if jf > 0:
                C -= S10[jf] @ Dinv[jf - 1][NMU:, NMU:] @ S10[jf].T
            if mid and bw:
                C[NMU:, NMU:] -= S10[jt + 1].T @ Dinv[jt + 1] @ S10[jt + 1]
            todo.append((jf, override(C, fix[jf], NMU)))
        if hb:
            C = block(S11, S00, fix, jb, NX, NMU)
            if bw:
                C[NMU:, NMU:] -= S10[jt + 1].T @ Dinv[jt + 1] @ S10[jt + 1]
            todo.append((jb, override(C, fix[jb], NMU)))
        for j, C in todo:
            Dinv[j], i3 = sweep(C)
            inert += i3
    xs = [None] * N
    if CMID > 0:
        xs[0] = rhs[0].copy()
    if N - 1 > CMID:
        xs[N - 1] = rhs[N - 1].copy()
    for s in range(1, CSTEPS + 1):
        mid = s == CSTEPS
        jf, jb = (CMID, CMID) if mid else (s, N - 1 - s)
        hf = (mid or jf < CMID) and jf > 0
        hb = (mid or jb > CMID) and jb + 1 < N
        CY = (Dinv[jf - 1] @ xs[jf - 1])[NMU:] if hf else None
        CW = Dinv[jb + 1] @ xs[jb + 1] if hb else None
        if mid:
            v = rhs[CMID].copy()
            if hf:
                v -= S10[jf] @ CY
            if hb:
                v[NMU:] -= S10[jb + 1].T @ CW
            xs[CMID] = v
            continue
        if jf < CMID:
            xs[jf] = rhs[jf] - S10[jf] @ CY
        if jb > CMID:
            v = rhs[jb].copy()
            v[NMU:] -= S10[jb + 1].T @ CW
            xs[jb] = v
    if CSTEPS == 0:
        xs[0] = rhs[0].copy()
    for s in range(CSTEPS + 1):
        jf, jb = CMID - s, CMID + s
        new = {}
        if jf >= 0:
            t = xs[jf].copy()
            if s > 0:
                t[NMU:] -= S10[jf + 1].T @ xs[jf + 1]
            new[jf] = Dinv[jf] @ t
        if s > 0 and jb < N:
            new[jb] = Dinv[jb] @ (xs[jb] - S10[jb] @ xs[jb - 1][NMU:])
        for j, v in new.items():
            xs[j] = v
    return np.concatenate(xs), tuple(inert)


CASES = [(15, 3, 3), (24, 4, 3), (10, 2, 2), (12, 2, 2), (11, 4, 0), (3, 2, 1), (2, 2, 2), (1, 3, 1)]


@pytest.mark.parametrize("N,NX,NMU", CASES)
def test_twisted_chain_matches_dense_and_one_sided(N, NX, NMU):
    rng = np.random.default_rng(N * 100 + NX * 10 + NMU)
    NC = NX + NMU
    checked = 0
    for t in range(20):
        fixed = [(int(rng.integers(N)), int(rng.integers(NX)))] if t % 4 == 3 else []
        S11, S00, S10, fix = make_chain(rng, N, NX, NMU, fixed)
        T = full_matrix(S11, S00, S10, fix, NX, NMU)
        rhs = [rng.normal(size=NC) for _ in range(N)]
        for j in range(N):
            for i in fix[j]:
                rhs[j][NMU + i] = 0.0
        x_tw, in_tw = twisted(S11, S00, S10, fix, NX, NMU, rhs)
        x_os, in_os = one_sided(S11, S00, S10, fix, NX, NMU, rhs)
        ev = np.linalg.eigvalsh(T)
        if np.abs(ev).min() < 1e-8 * np.abs(ev).max():
            continue  # (nearly) singular draw: fixing a state can strand a multiplier row
        checked += 1
        assert in_tw == ((ev > 0).sum(), (ev < 0).sum(), 0) == in_os
        b = np.concatenate(rhs)
        # backward errors (random chains can be ill-conditioned): both orders solve T x = b
        for x in (x_tw, x_os):
            res = np.linalg.norm(T @ x - b) / (np.linalg.norm(T, 2) * np.linalg.norm(x) + np.linalg.norm(b))
            assert res < 1e-10, res
    assert checked >= 10
