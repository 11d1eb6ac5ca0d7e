"""ORACLE (test infrastructure only) — build + ctypes binding of oracle/c/ipm_oracle.c.

The C restatement is the CPU baseline of bench.py (all host cores, OpenMP,
one agent NLP per thread) and is cross-checked against oracle/ipm.py in
tests/test_oracle.py.  Built with gcc -O3 -march=native -fopenmp into
oracle/c/build/ (git-ignored; travels to the GPU box with the snapshot).
"""

from __future__ import annotations

import ctypes
import os
import pathlib
import subprocess

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
SRC = HERE / "c" / "ipm_oracle.c"
OUT = HERE / "c" / "build" / "liboracle_ipm.so"

MAXD = 9


class RoomT(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("N", "d", "nx", "nv", "ng", "nps", "npg")] + [
        ("ts", ctypes.c_double),
        ("B", ctypes.c_double * (MAXD + 1)),
        ("C", (ctypes.c_double * (MAXD + 1)) * (MAXD + 1)),
        ("D", ctypes.c_double * (MAXD + 1)),
    ]


class OOpts(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        "tol", "dual_inf_tol", "constr_viol_tol", "compl_inf_tol", "acceptable_tol",
        "acceptable_dual_inf_tol", "acceptable_constr_viol_tol", "acceptable_compl_inf_tol",
        "acceptable_obj_change_tol")] + [("max_iter", ctypes.c_int), ("acceptable_iter", ctypes.c_int)]


def options(**kw) -> OOpts:
    """IPOPT termination options; defaults are IPOPT's own (acceptable_iter 15 ...)."""
    from oracle.ipm import IPMOptions

    d = IPMOptions(**kw)
    return OOpts(**{n: getattr(d, n) for n, _ in OOpts._fields_})


_OSTATS_INTS = ("iter", "status", "n_fact", "n_trials", "n_soft", "n_resto", "n_resto_iters", "n_filter_over",
                "n_refine")


class OStats(ctypes.Structure):
    _fields_ = [("obj", ctypes.c_double)] + [(n, ctypes.c_int) for n in _OSTATS_INTS]


def _stats_dicts(st):
    return [dict(obj=s.obj, **{n: getattr(s, n) for n in _OSTATS_INTS}) for s in st]


HDR = HERE / "c" / "ipm_oracle.h"
GEN_SRC = HERE / "c" / "gen_model.cpp"


def build(force: bool = False, march: str = "native") -> pathlib.Path:
    OUT.parent.mkdir(parents=True, exist_ok=True)
    if OUT.exists() and not force and OUT.stat().st_mtime >= max(SRC.stat().st_mtime, HDR.stat().st_mtime):
        return OUT
    cmd = ["gcc", "-O3", f"-march={march}", "-fopenmp", "-shared", "-fPIC", "-std=c11", str(SRC),
           "-o", str(OUT) + ".tmp", "-lm"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0 and march == "native":
        return build(force=True, march="x86-64-v2")
    if res.returncode != 0:
        raise RuntimeError(res.stderr)
    os.replace(str(OUT) + ".tmp", OUT)
    return OUT


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not OUT.exists():
            build()
        _lib = ctypes.CDLL(str(OUT))
        vp = ctypes.c_void_p
        _lib.oracle_room_init.argtypes = [ctypes.POINTER(RoomT), ctypes.c_int, ctypes.c_int, ctypes.c_double, vp, vp, vp]
        _lib.oracle_room_solve_fleet.argtypes = [ctypes.POINTER(RoomT), ctypes.c_int, vp, vp, vp, vp,
                                                 ctypes.POINTER(OStats), ctypes.POINTER(OOpts), ctypes.c_int]
        _lib.oracle_room_solve_fleet.restype = ctypes.c_int
        assert _lib.oracle_room_sizeof() == ctypes.sizeof(RoomT)
        assert _lib.oracle_opts_sizeof() == ctypes.sizeof(OOpts)
    return _lib


def room_model(N=15, d=2, ts=300.0) -> RoomT:
    from oracle.nlps import collocation

    _, B, C, D = collocation(d)
    m = RoomT()
    Bc = np.ascontiguousarray(B, dtype=np.float64)
    Cc = np.ascontiguousarray(C, dtype=np.float64)
    Dc = np.ascontiguousarray(D, dtype=np.float64)
    lib().oracle_room_init(ctypes.byref(m), N, d, ts, Bc.ctypes.data, Cc.ctypes.data, Dc.ctypes.data)
    return m


def solve_room_fleet(p, lbw, ubw, w0, N=15, d=2, tol=1e-8, max_iter=500, threads=0, **ipopt):
    """Returns (w, stats list of dicts, n_converged).  ``ipopt``: further IPOPT termination
    options (acceptable_*); without them IPOPT's defaults apply."""
    m = room_model(N, d)
    opts = options(tol=tol, max_iter=max_iter, **ipopt)
    p = np.ascontiguousarray(p, dtype=np.float64)
    lbw = np.ascontiguousarray(lbw, dtype=np.float64)
    ubw = np.ascontiguousarray(ubw, dtype=np.float64)
    w = np.array(w0, dtype=np.float64, order="C", copy=True)
    n = p.shape[0]
    st = (OStats * n)()
    ok = lib().oracle_room_solve_fleet(ctypes.byref(m), n, p.ctypes.data, lbw.ctypes.data, ubw.ctypes.data,
                                       w.ctypes.data, st, ctypes.byref(opts), threads)
    stats = _stats_dicts(st)
    return w, stats, ok


# ---------------------------------------------------------------------------
# generated stage models on the host (CPU baselines of C2 / C4 / C5, bench.py)
# ---------------------------------------------------------------------------
_gen_libs = {}


def build_generated(gen, march: str = "native") -> pathlib.Path:
    """Compile the C IPM with one generated model (``codegen.GeneratedModel``) for the host:
    the generated stage functions with the HIP qualifiers defined away (no kernel code)."""
    import hashlib

    key = hashlib.sha1((gen.source + SRC.read_text() + HDR.read_text() + GEN_SRC.read_text()).encode()).hexdigest()[:12]
    out = OUT.parent / f"libgen_{key}.so"
    if out.exists():
        return out
    OUT.parent.mkdir(parents=True, exist_ok=True)
    body, device_only = [], False
    for ln in gen.source.splitlines():  # the kernel's device-only section (static elimination) is dropped
        if ln.startswith("// >>> device only"):
            device_only = True
        if not device_only and not ln.startswith("#include <hip/") and not ln.startswith('#include "mpcx_ipm.hip"'):
            body.append(ln)
        if ln.startswith("// <<< device only"):
            device_only = False
    src = OUT.parent / f"gen_{key}.inc"
    src.write_text("\n".join(body) + "\n")
    core_o = OUT.parent / f"core_{key}.o"
    model_o = OUT.parent / f"model_{key}.o"
    for cmd in (["gcc", "-O3", f"-march={march}", "-fopenmp", "-fPIC", "-std=c11", "-c", str(SRC), "-o", str(core_o)],
                ["g++", "-O3", f"-march={march}", "-fopenmp", "-fPIC", "-std=c++17", f"-I{HERE / 'c'}",
                 f'-DMPCX_GEN_SOURCE="{src}"', "-c", str(GEN_SRC), "-o", str(model_o)],
                ["g++", "-shared", "-fopenmp", str(core_o), str(model_o), "-o", str(out) + ".tmp", "-lm"]):
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            if march == "native":
                return build_generated(gen, march="x86-64-v2")
            raise RuntimeError(res.stderr[-4000:])
    os.replace(str(out) + ".tmp", out)
    return out


def _gen_lib(gen):
    path = build_generated(gen)
    if path not in _gen_libs:
        lib = ctypes.CDLL(str(path))
        vp = ctypes.c_void_p
        lib.oracle_gen_solve_fleet.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.POINTER(OStats),
                                               ctypes.POINTER(OOpts), ctypes.c_int]
        lib.oracle_gen_solve_fleet.restype = ctypes.c_int
        _gen_libs[path] = lib
    return _gen_libs[path]


def solve_generated_fleet(gen, p, lbw, ubw, w0, threads=0, tol=1e-8, max_iter=500, **ipopt):
    """Solve kernel-layout NLP inputs [n, .] of one generated model on the host cores.
    Returns (w, stats list of dicts, n_succeeded)."""
    p = np.ascontiguousarray(p, dtype=np.float64)
    lbw = np.ascontiguousarray(lbw, dtype=np.float64)
    ubw = np.ascontiguousarray(ubw, dtype=np.float64)
    w = np.array(w0, dtype=np.float64, order="C", copy=True)
    n = p.shape[0]
    st = (OStats * n)()
    opts = options(tol=tol, max_iter=max_iter, **ipopt)
    ok = _gen_lib(gen).oracle_gen_solve_fleet(n, p.ctypes.data, lbw.ctypes.data, ubw.ctypes.data, w.ctypes.data,
                                              st, ctypes.byref(opts), threads)
    stats = _stats_dicts(st)
    return w, stats, ok
