"""Oracle-side solve callbacks for the ADMM loop restatements (`oracle/admm.py`).

Each callback builds the agent's NLP with the oracle's hand restatement
(`oracle/nlps.py`), solves it with the oracle IPM (warm-started from the
agent's previous solution, as the reference backend does,
`core/discretization.py:212-251`) and returns the coupling trajectories the
agent would send (``Results[coupling.name]``, t >= 0).
"""

from __future__ import annotations

import numpy as np

from oracle import ipm, nlps


class _Solver:
    def __init__(self):
        self.last = {}

    def _run(self, key, prob, p, lbw, ubw, w0):
        guess = self.last.get(key)
        if guess is not None:
            w0 = guess.copy()
            fixed = lbw == ubw
            w0[fixed] = lbw[fixed]
        r = ipm.solve(prob.functions(p), w0, lbw, ubw, prob.lbg(p), prob.ubg(p),
                      ipm.IPMOptions(tol=1e-10, max_iter=500))
        assert r.success, (key, r.status)
        self.last[key] = r.x
        return r.x


def _pick(prob, x, prefix):
    idx = [i for i, n in enumerate(prob.w_names) if n.split("@")[0] == prefix]
    return np.asarray(x)[idx]


class C4Oracle(_Solver):
    """examples/exchange_admm rooms + supply (multiple shooting, Euler)."""

    def __init__(self, N, rooms, n_supply=1):
        super().__init__()
        self.N = N
        self.rooms = rooms  # list of (d, T0)
        self.room = nlps.exchange_room(N=N)
        self.supply = nlps.exchange_supply(N=N)
        self.participation = {f"room{i}": {"mDot_coupling": "exchange"} for i in range(len(rooms))}
        self.participation.update({f"supply{i}": {"mDot_coupling": "exchange"} for i in range(n_supply)})
        self.initial = {ag: {"mDot_coupling": 0.02} for ag in self.participation}

    def __call__(self, ag, inp, rho):
        diff, lam = inp["mDot_coupling"]
        if ag.startswith("room"):
            d, T0 = self.rooms[int(ag[4:])]
            p, lbw, ubw, w0 = nlps.exchange_room_inputs(self.room, N=self.N, T0=T0, dist=d, rho=rho,
                                                        diff=diff, lam=lam)
            x = self._run(ag, self.room, p, lbw, ubw, w0)
            return {"mDot_coupling": _pick(self.room, x, "mDot_out")}
        p, lbw, ubw, w0 = nlps.exchange_supply_inputs(self.supply, N=self.N, rho=rho, diff=diff, lam=lam)
        x = self._run(ag, self.supply, p, lbw, ubw, w0)
        return {"mDot_coupling": _pick(self.supply, x, "mDot_out")}


class C2Oracle(_Solver):
    """examples/4_Room_ADMM_Coordinator: 4 rooms + air handler (collocation d=3), one block."""

    def __init__(self, N, rooms):
        super().__init__()
        self.N = N
        self.rooms = rooms
        self.room = nlps.admm_room(N=N)
        self.ahu = nlps.admm_ahu(N=N)
        self.participation = {f"room{i}": {f"mDot{i + 1}_coupling_b0": "consensus"} for i in range(4)}
        self.participation["ahu"] = {f"mDot{i + 1}_coupling_b0": "consensus" for i in range(4)}
        self.initial = {f"room{i}": {f"mDot{i + 1}_coupling_b0": 0.02} for i in range(4)}
        self.initial["ahu"] = {f"mDot{i + 1}_coupling_b0": 0.01 for i in range(4)}

    def __call__(self, ag, inp, rho):
        if ag.startswith("room"):
            i = int(ag[4:])
            al = f"mDot{i + 1}_coupling_b0"
            zbar, lam = inp[al]
            d, T0 = self.rooms[i]
            p, lbw, ubw, w0 = nlps.admm_room_inputs(self.room, N=self.N, T0=T0, dist=d, rho=rho, zbar=zbar, lam=lam)
            x = self._run(ag, self.room, p, lbw, ubw, w0)
            return {al: _pick(self.room, x, "mDot")}
        als = [f"mDot{i + 1}_coupling_b0" for i in range(4)]
        zbar = np.stack([inp[a][0] for a in als])
        lam = np.stack([inp[a][1] for a in als])
        p, lbw, ubw, w0 = nlps.admm_ahu_inputs(self.ahu, N=self.N, rho=rho, zbar=zbar, lam=lam)
        x = self._run(ag, self.ahu, p, lbw, ubw, w0)
        return {a: _pick(self.ahu, x, f"mDot_out_{i + 1}") for i, a in enumerate(als)}
