"""ctypes binding of ``libmpcx.so`` (include/mpcx.h) and the code-object cache.

The product path is native only: if the shared library or a model's code
object cannot be loaded on a GPU box this module raises — there is no CPU
fallback.  Device memory and streams come from PyTorch (plumbing only): all
arrays passed to the C ABI are ``torch.float64`` CUDA(HIP) tensors.
"""

from __future__ import annotations

import ctypes
import hashlib
import os
import pathlib
import re
import shutil
import subprocess
import threading
import warnings
from typing import List, Dict, Optional

PKG_DIR = pathlib.Path(__file__).resolve().parents[1]          # agentlib_mpc_amd/
ROOT_DIR = PKG_DIR.parent                                       # agentlib-mpc_amd/
REPO_DIR = ROOT_DIR.parent
CSRC = ROOT_DIR / "csrc"
INCLUDE = REPO_DIR / "include"
BUILD_DIR = PKG_DIR / "_build"
KERNEL_DIR = BUILD_DIR / "kernels"
LIB_PATH = BUILD_DIR / "libmpcx.so"
OFFLOAD_ARCH = os.environ.get("MPCX_OFFLOAD_ARCH", "gfx950")

STATUS_NAMES = {
    0: "Solve_Succeeded",
    1: "Solved_To_Acceptable_Level",
    -1: "Maximum_Iterations_Exceeded",
    -2: "Restoration_Failed",
    -3: "Error_In_Step_Computation",
    -4: "Invalid_Number_Detected",
    -5: "Infeasible_Problem_Detected",
}


class NativeError(RuntimeError):
    pass


# ---------------------------------------------------------------------------
# C structs (must match include/mpcx.h)
# ---------------------------------------------------------------------------
class ProblemDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("n_stages", "nx", "nv", "ng", "nps", "npg", "abi", "reserved")]


_OPT_DOUBLES = [
    "tol", "dual_inf_tol", "constr_viol_tol", "compl_inf_tol", "acceptable_tol",
    "acceptable_dual_inf_tol", "acceptable_constr_viol_tol", "acceptable_compl_inf_tol",
    "acceptable_obj_change_tol",
    "mu_init", "mu_min", "kappa_eps", "kappa_mu", "theta_mu", "tau_min",
    "bound_push", "bound_frac", "bound_relax_factor", "bound_mult_init_val",
    "constr_mult_init_max", "kappa_sigma", "nlp_scaling_max_gradient", "nlp_scaling_min_value",
    "delta_w_first", "delta_w_min", "delta_w_max", "kappa_w_plus_bar", "kappa_w_plus",
    "kappa_w_minus", "delta_c_bar", "kappa_c", "theta_max_fact", "theta_min_fact", "eta_phi",
    "delta", "s_phi", "s_theta", "gamma_phi", "gamma_theta", "alpha_min_frac",
]
_OPT_INTS = ["max_iter", "acceptable_iter", "warm_start_mult", "reserved"]


class Options(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in _OPT_DOUBLES] + [(n, ctypes.c_int32) for n in _OPT_INTS]


_STATS_INTS = ("iter_count", "status", "n_inertia_corrections", "n_restorations", "n_factorizations", "n_trials",
               "n_block_chain", "n_dense_stages", "n_soft_restorations", "n_restoration_iters",
               "n_filter_overflows", "n_refinement_steps")


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in ("obj", "primal_inf", "dual_inf", "compl_inf", "mu", "obj_scale")] + \
               [(n, ctypes.c_int32) for n in _STATS_INTS]


STATS_BYTES = ctypes.sizeof(Stats)
EXPORTED_SYMBOLS = [
    "mpcx_version", "mpcx_default_options", "mpcx_problem_create", "mpcx_problem_destroy",
    "mpcx_set_options", "mpcx_reserve", "mpcx_workspace_bytes_per_agent", "mpcx_problem_small_fleet",
    "mpcx_problem_mid_fleet", "mpcx_problem_wide_fleet",
    "mpcx_batch_solve", "mpcx_batch_solve_staged", "mpcx_batch_solve_mapped", "mpcx_active_map",
    "mpcx_admm_moments_size", "mpcx_admm_reduce_count", "mpcx_admm_moments", "mpcx_admm_finalize",
    "mpcx_admm_moments_masked", "mpcx_admm_consensus_multipliers_masked", "mpcx_admm_exchange_update_masked",
    "mpcx_admm_consensus_multipliers", "mpcx_admm_exchange_update", "mpcx_admm_shift",
    "mpcx_gather_rows", "mpcx_scatter_rows", "mpcx_fill_column",
    "mpcx_admm_block_stop", "mpcx_admm_block_expand", "mpcx_device_clock_khz", "mpcx_stats_count",
    "mpcx_scatter_rows_multi", "mpcx_gather_rows_multi",
    "mpcx_allreduce_register", "mpcx_allreduce_register_fn", "mpcx_allreduce_unregister", "mpcx_allreduce_kind",
    "mpcx_admm_allreduce", "mpcx_allreduce_calls", "mpcx_rccl_unique_id", "mpcx_rccl_comm_init",
    "mpcx_rccl_comm_init_file", "mpcx_rccl_comm_destroy", "mpcx_stream_create_dedicated", "mpcx_stream_destroy",
    "mpcx_lds_bytes_per_agent", "mpcx_admm_block_expand_multi", "mpcx_stats_count_multi",
]
MOVE_DESC = 4  # MPCX_MOVE_DESC: int64 words per descriptor of the fused row moves (C ABI v12)
ADMM_TOTALS = 8  # MPCX_ADMM_TOTALS
ADMM_CONTROL = 1  # MPCX_ADMM_CONTROL: control doubles before the moments buffer (C ABI v10)
RCCL_ID_BYTES = 128  # MPCX_RCCL_ID_BYTES
COLLECTIVE_NONE, COLLECTIVE_RCCL, COLLECTIVE_FN = 0, 1, 2  # mpcx_allreduce_kind
ERR_ARG, ERR_COMM = -1, -6  # MPCX_ERR_ARG, MPCX_ERR_COMM
#: mpcx_allreduce_fn: int (*)(void* ctx, double* buf, int64_t count, void* stream)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)
KERNEL_ABI = 8  # MPCX_KERNEL_ABI (csrc/mpcx_internal.h)

_lib = None
_lib_lock = threading.Lock()


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise NativeError("hipcc not found; cannot build MI355X kernels")


def build_library(force: bool = False) -> pathlib.Path:
    """Compile libmpcx.so (host runtime + ADMM kernels) for gfx950, in-tree."""
    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    srcs = [CSRC / "mpcx_runtime.cpp", CSRC / "admm_kernels.hip", CSRC / "mpcx_collective.cpp"]
    deps = srcs + [INCLUDE / "mpcx.h", CSRC / "mpcx_internal.h"]
    if LIB_PATH.exists() and not force:
        if LIB_PATH.stat().st_mtime >= max(p.stat().st_mtime for p in deps):
            return LIB_PATH
    tmp = LIB_PATH.with_suffix(".so.tmp")
    cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={OFFLOAD_ARCH}", "-O3", "-std=c++17",
           "-Wno-unused-result", "-Wno-unused-value", f"-I{INCLUDE}", f"-I{CSRC}",
           *map(str, srcs), "-ldl", "-o", str(tmp)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise NativeError(f"building libmpcx.so failed:\n{res.stderr[-4000:]}")
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


PYREAD_PATH = BUILD_DIR / "_mpcx_pyread.so"
_pyread = None


def build_pyread(force: bool = False) -> pathlib.Path:
    """Compile the host-side attribute reader of the plugin batch (csrc/mpcx_pyread.c, a
    CPython extension; gcc), in-tree."""
    import sysconfig

    BUILD_DIR.mkdir(parents=True, exist_ok=True)
    src = CSRC / "mpcx_pyread.c"
    if PYREAD_PATH.exists() and not force and PYREAD_PATH.stat().st_mtime >= src.stat().st_mtime:
        return PYREAD_PATH
    tmp = PYREAD_PATH.with_suffix(".so.tmp")
    cc = os.environ.get("CC") or shutil.which("gcc") or "cc"
    cmd = [cc, "-O2", "-shared", "-fPIC", "-Wall", f"-I{sysconfig.get_paths()['include']}", str(src), "-o", str(tmp)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise NativeError(f"building {PYREAD_PATH.name} failed:\n{res.stderr[-4000:]}")
    os.replace(tmp, PYREAD_PATH)
    return PYREAD_PATH


def load_pyread():
    """The attribute reader module (raises NativeError when it was not built)."""
    global _pyread
    if _pyread is None:
        import importlib.machinery
        import importlib.util

        if not PYREAD_PATH.exists():
            raise NativeError(f"{PYREAD_PATH} is missing: run __graft_entry__.build() (or "
                              "agentlib_mpc_amd.runtime.native.build_pyread()) first.")
        loader = importlib.machinery.ExtensionFileLoader("_mpcx_pyread", str(PYREAD_PATH))
        spec = importlib.util.spec_from_file_location("_mpcx_pyread", str(PYREAD_PATH), loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _pyread = mod
    return _pyread


def load_library():
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists():
            raise NativeError(
                f"{LIB_PATH} is missing: run __graft_entry__.build() (or "
                "agentlib_mpc_amd.runtime.native.build_library()) first. There is no CPU fallback.")
        lib = ctypes.CDLL(str(LIB_PATH))
        vp, i32, f64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_double
        lib.mpcx_version.restype = ctypes.c_int
        lib.mpcx_default_options.argtypes = [ctypes.POINTER(Options)]
        lib.mpcx_default_options.restype = None
        lib.mpcx_problem_create.argtypes = [ctypes.POINTER(ProblemDesc), ctypes.c_char_p, ctypes.POINTER(vp)]
        lib.mpcx_problem_destroy.argtypes = [vp]
        lib.mpcx_set_options.argtypes = [vp, ctypes.POINTER(Options)]
        lib.mpcx_reserve.argtypes = [vp, i32]
        lib.mpcx_workspace_bytes_per_agent.argtypes = [vp]
        lib.mpcx_problem_small_fleet.argtypes = [vp, ctypes.c_char_p, i32]
        lib.mpcx_problem_mid_fleet.argtypes = [vp, ctypes.c_char_p, i32]
        lib.mpcx_problem_wide_fleet.argtypes = [vp, ctypes.c_char_p, i32]
        lib.mpcx_workspace_bytes_per_agent.restype = ctypes.c_int64
        lib.mpcx_admm_block_expand_multi.argtypes = [i32, vp, i32, vp, vp, vp]
        lib.mpcx_stats_count_multi.argtypes = [i32, vp, i32, vp, vp]
        lib.mpcx_lds_bytes_per_agent.argtypes = [vp]
        lib.mpcx_lds_bytes_per_agent.restype = ctypes.c_int64
        lib.mpcx_batch_solve.argtypes = [vp, i32] + [vp] * 9 + [vp, vp]
        lib.mpcx_batch_solve_mapped.argtypes = [vp, i32, i32, vp] + [vp] * 9 + [vp, vp]
        lib.mpcx_active_map.argtypes = [i32, vp, vp, vp, vp]
        i64 = ctypes.c_int64
        lib.mpcx_batch_solve_staged.argtypes = [vp, i32, vp, vp, i64, vp, vp, i64] + [vp] * 6 + [vp]
        lib.mpcx_admm_moments_size.argtypes = [i32, i32, i32]
        lib.mpcx_admm_moments_size.restype = i64
        lib.mpcx_admm_reduce_count.argtypes = [i32, i32, i32]
        lib.mpcx_admm_reduce_count.restype = i64
        lib.mpcx_admm_moments.argtypes = [i32, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp]
        lib.mpcx_admm_finalize.argtypes = [i32, i32, i32, i32, i32, vp, vp, vp, f64, vp, vp, vp, vp, vp, vp,
                                           vp]
        lib.mpcx_admm_consensus_multipliers.argtypes = [i32, i32, vp, i32, vp, vp, f64, vp, vp, vp, vp, vp]
        lib.mpcx_admm_exchange_update.argtypes = [i32, i32, vp, i32, vp, vp, vp, vp, i32, f64, vp, vp, vp]
        lib.mpcx_admm_shift.argtypes = [i32, i32, i32, vp, vp]
        lib.mpcx_admm_moments_masked.argtypes = [i32, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp, vp]
        lib.mpcx_admm_consensus_multipliers_masked.argtypes = [i32, i32, vp, i32, vp, vp, f64, vp, vp, vp, vp,
                                                               vp, vp]
        lib.mpcx_admm_exchange_update_masked.argtypes = [i32, i32, vp, i32, vp, vp, vp, vp, i32, f64, vp, vp,
                                                         vp, vp]
        lib.mpcx_gather_rows.argtypes = [i32, i32, vp, i64, vp, vp, vp, vp]
        lib.mpcx_scatter_rows.argtypes = [i32, i32, vp, vp, vp, i64, vp, vp]
        lib.mpcx_fill_column.argtypes = [i32, vp, i64, i32, f64, vp]
        lib.mpcx_scatter_rows_multi.argtypes = [i32, i32, vp, i32, vp, i64, vp]
        lib.mpcx_gather_rows_multi.argtypes = [i32, i32, vp, i32, vp, i64, vp]
        lib.mpcx_admm_block_stop.argtypes = [i32, i32, vp, i32, f64, f64, f64, f64, f64, f64, vp, vp, vp, vp, vp,
                                             vp, vp, vp]
        lib.mpcx_admm_block_expand.argtypes = [i32, vp, vp, vp, vp, vp, vp, vp]
        lib.mpcx_device_clock_khz.restype = i64
        lib.mpcx_stats_count.argtypes = [i32, vp, vp, vp, vp]
        # the collective of an ADMM iteration (C ABI v14, runtime/collective.py)
        lib.mpcx_allreduce_register.argtypes = [vp, ctypes.c_char_p]
        lib.mpcx_allreduce_register_fn.argtypes = [ALLREDUCE_FN, vp]
        lib.mpcx_admm_allreduce.argtypes = [vp, i64, vp]
        lib.mpcx_allreduce_calls.restype = i64
        lib.mpcx_rccl_unique_id.argtypes = [ctypes.c_char_p, vp]
        lib.mpcx_rccl_comm_init.argtypes = [ctypes.c_char_p, i32, i32, vp, ctypes.POINTER(vp)]
        lib.mpcx_rccl_comm_init_file.argtypes = [ctypes.c_char_p, ctypes.c_char_p, i32, i32, i32, ctypes.POINTER(vp)]
        lib.mpcx_rccl_comm_destroy.argtypes = [ctypes.c_char_p, vp]
        # streams with a hardware queue of their own (C ABI v15): the fleet's class streams
        lib.mpcx_stream_create_dedicated.argtypes = [ctypes.POINTER(vp)]
        lib.mpcx_stream_destroy.argtypes = [vp]
        for name in EXPORTED_SYMBOLS:
            getattr(lib, name)  # raises AttributeError if a symbol is missing
        _lib = lib
        return lib


_DEDICATED: dict = {}


def dedicated_streams(n: int, device) -> list:
    """``n`` HIP streams with a hardware queue of their own each (C ABI v15,
    ``mpcx_stream_create_dedicated``), as ``torch.cuda.ExternalStream``.  Ordinary streams share
    the runtime's few hardware queues, and two classes' solves on one queue run one after the
    other.  A per-device pool for the process: a fleet takes the first ``n``, so the process holds
    as many dedicated queues as its widest fleet has classes (fleets of one process run one at a
    time; sharing a stream only orders their launches).  The streams live as long as the process."""
    import torch

    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    pool = _DEDICATED.setdefault(idx, [])
    lib = load_library()
    with torch.cuda.device(idx):
        while len(pool) < n:
            s = ctypes.c_void_p()
            rc = lib.mpcx_stream_create_dedicated(ctypes.byref(s))
            if rc != 0:
                raise NativeError(f"mpcx_stream_create_dedicated failed ({rc})")
            pool.append(torch.cuda.ExternalStream(s.value, device=torch.device("cuda", idx)))
    return pool[:n]


def admm_reduce_count(n_global: int, n_global_blocks: int, T: int) -> int:
    """Doubles all-reduced over the ranks per ADMM iteration, from the control slot before the
    moments buffer on (``mpcx_admm_reduce_count``, host arithmetic of the C ABI: no GPU call)."""
    n = int(load_library().mpcx_admm_reduce_count(int(n_global), int(n_global_blocks), int(T)))
    if n < 0:
        raise NativeError(f"mpcx_admm_reduce_count({n_global}, {n_global_blocks}, {T}) failed ({n})")
    return n


def default_options() -> Options:
    opts = Options()
    load_library().mpcx_default_options(ctypes.byref(opts))
    return opts


# ---------------------------------------------------------------------------
# code objects
# ---------------------------------------------------------------------------
def _kernel_deps_hash() -> str:
    h = hashlib.sha1()
    for p in (CSRC / "mpcx_ipm.hip", CSRC / "mpcx_internal.h", INCLUDE / "mpcx.h"):
        h.update(p.read_bytes())
    return h.hexdigest()[:10]


def _extra_defines() -> List[str]:
    """Diagnostic kernel variants: ``MPCX_DEFINES="A,B=1"`` adds ``-DA -DB=1`` (e.g.
    ``MPCX_NO_STATIC`` forces the dense Bunch-Kaufman path); part of the code-object name."""
    return [d for d in os.environ.get("MPCX_DEFINES", "").split(",") if d]


#: small-fleet variant (workspace in LDS, one agent per CU; ``mpcx_problem_small_fleet``)
SMALL_FLEET = "wslds"
#: mid-fleet variant (one wave per SIMD, up to 512 registers; ``mpcx_problem_mid_fleet``)
MID_FLEET = "w1"
#: wide-fleet variant (20 agents per CU where the main build holds 16; ``mpcx_problem_wide_fleet``)
WIDE_FLEET = "apc20"
#: largest call-frame scratch (B/lane) a wide build may have: its register budget (96) spills more
#: than the main build's, and a structure whose stage code needs the registers loses more than
#: the extra agents per CU give (C4 room 92 B: 4 % faster at 13108 agents; C2 room 740 B)
WIDE_SCRATCH_MAX = 128
#: compiler messages of the kernel's own static_asserts that mean "this structure does not fit
#: the variant" (permanent for the code object's source hash)
_NOFIT_MESSAGES = ("workspace does not fit LDS", "LDS share per agent exceeded")
_VARIANT_DEFINES = {None: [], SMALL_FLEET: ["MPCX_WS_LDS"], MID_FLEET: ["MPCX_MIN_WAVES=1"],
                    WIDE_FLEET: ["MPCX_APC=20"]}


def code_object_path(gen_key: str, variant: Optional[str] = None) -> pathlib.Path:
    extra = _extra_defines()
    tag = ("_" + hashlib.sha1(",".join(extra).encode()).hexdigest()[:6]) if extra else ""
    vtag = f"_{variant}" if variant else ""
    return KERNEL_DIR / f"mpcx_{gen_key}_{_kernel_deps_hash()}{tag}{vtag}_{OFFLOAD_ARCH}.hsaco"


def compile_model(gen, verbose: bool = False, variant: Optional[str] = None) -> Optional[pathlib.Path]:
    """Compile a generated model source to a gfx950 code object (cached).  ``variant``
    SMALL_FLEET: the workspace-in-LDS build; None (and a ``.nofit`` marker) when the
    structure's workspace does not fit a CU's LDS."""
    KERNEL_DIR.mkdir(parents=True, exist_ok=True)
    out = code_object_path(gen.key, variant)
    if out.exists():
        return out
    nofit = out.with_suffix(".nofit")
    if variant is not None and nofit.exists():
        return None
    if variant in (MID_FLEET, WIDE_FLEET):
        # MID_FLEET only where the main build's register budget is tighter than one wave per SIMD,
        # WIDE_FLEET only where the main build holds 16 agents per CU (four waves per SIMD)
        base = compile_model(gen, verbose)
        occ = base.with_suffix(".occ")
        if not occ.exists():
            # the main build's occupancy is unknown (its resource remark was not found): no
            # marker, so the decision is taken again once the occupancy is known
            warnings.warn(f"occupancy of {base.name} unknown; no one-wave-per-SIMD build this time")
            return None
        if variant == MID_FLEET and int(occ.read_text() or "1") <= 1:
            nofit.write_text("the main build already runs one wave per SIMD")
            return None
        if variant == WIDE_FLEET and int(occ.read_text() or "0") != 4:
            nofit.write_text("the main build does not hold 16 agents per CU")
            return None
    src = out.with_suffix(".hip")
    src.write_text(gen.source)
    tmp = out.with_suffix(".tmp")
    defs = _extra_defines() + _VARIANT_DEFINES[variant]
    cmd = [_hipcc(), "--genco", f"--offload-arch={OFFLOAD_ARCH}", "-O3", "-std=c++17",
           f"-I{INCLUDE}", f"-I{CSRC}", *[f"-D{d}" for d in defs], str(src), "-o", str(tmp),
           "-Rpass-analysis=kernel-resource-usage"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        if variant is not None:
            # an optional build: any failure means "no such build this time", the main code
            # object serves every batch size.  Only a structural misfit (a static_assert of the
            # LDS / register budgets) is recorded as permanent (.nofit); a transient failure
            # (hipcc killed, out of memory, interrupted) is retried by the next process.
            if any(m in res.stderr for m in _NOFIT_MESSAGES):
                nofit.write_text(res.stderr[-4000:])
            else:
                name = {SMALL_FLEET: "small-fleet", MID_FLEET: "one-wave-per-SIMD",
                        WIDE_FLEET: "20-agents-per-CU"}.get(variant, variant)
                warnings.warn(f"{name} build of {gen.key} failed; the main build serves every batch:\n"
                              f"{res.stderr[-800:]}")
            tmp.unlink(missing_ok=True)
            return None
        raise NativeError(f"compiling {src} failed:\n{res.stderr[-4000:]}")
    if verbose and res.stderr:
        print(res.stderr)
    if variant is None:  # the register budget's occupancy (mpcx_ipm_solve), for the w1 decision
        occ = re.search(r"Function Name: mpcx_ipm_solve.*?Occupancy \[waves/SIMD\]: (\d+)", res.stderr, re.S)
        if occ:
            out.with_suffix(".occ").write_text(occ.group(1))
        else:  # remark format changed: leave the decision open rather than never building w1
            warnings.warn(f"no occupancy remark for mpcx_ipm_solve in the build of {out.name}")
    if variant == WIDE_FLEET:
        scr = re.search(r"Function Name: mpcx_ipm_solve.*?ScratchSize \[bytes/lane\]: (\d+)", res.stderr, re.S)
        if scr is None or int(scr.group(1)) > WIDE_SCRATCH_MAX:
            # permanent for this source hash when measured; an unreadable remark is retried
            if scr is not None:
                nofit.write_text(f"scratch {scr.group(1)} B/lane > {WIDE_SCRATCH_MAX}")
            else:
                warnings.warn(f"no scratch remark for mpcx_ipm_solve in the build of {out.name}")
            tmp.unlink(missing_ok=True)
            return None
    os.replace(tmp, out)
    return out


class NativeProblem:
    """Owns one ``mpcx_handle`` (code object + workspace) for a problem structure."""

    def __init__(self, gen, hsaco: Optional[pathlib.Path] = None):
        self.lib = load_library()
        self.gen = gen
        d = gen.dims
        self.desc = ProblemDesc(n_stages=d["N"], nx=d["NX"], nv=d["NV"], ng=d["NG"],
                                nps=d["NPS"], npg=d["NPG"], abi=KERNEL_ABI, reserved=0)
        path = hsaco or code_object_path(gen.key)
        if not pathlib.Path(path).exists():
            path = compile_model(gen)
        handle = ctypes.c_void_p()
        rc = self.lib.mpcx_problem_create(ctypes.byref(self.desc), str(path).encode(), ctypes.byref(handle))
        if rc != 0:
            raise NativeError(f"mpcx_problem_create failed ({rc}) for {path}")
        self.handle = handle
        self.small_fleet_path = None
        if hsaco is None and os.environ.get("MPCX_SMALL_FLEET", "1") != "0":
            # small fleets (<= one agent per CU) run the workspace-in-LDS build when the
            # structure's workspace fits a CU's LDS (compiled by build(), else here)
            sp = compile_model(gen, variant=SMALL_FLEET)
            if sp is not None:
                rc = self.lib.mpcx_problem_small_fleet(handle, str(sp).encode(), -1)
                if rc != 0:  # optional: the HBM build (loaded above) serves every batch size
                    warnings.warn(f"mpcx_problem_small_fleet failed ({rc}) for {sp}; using the HBM build")
                else:
                    self.small_fleet_path = sp
        self.mid_fleet_path = None
        if hsaco is None and os.environ.get("MPCX_MID_FLEET", "1") != "0":
            # fleets of at most one agent per SIMD run the build with that register budget
            mp = compile_model(gen, variant=MID_FLEET)
            if mp is not None:
                rc = self.lib.mpcx_problem_mid_fleet(handle, str(mp).encode(), -1)
                if rc != 0:  # optional, as the small-fleet build
                    warnings.warn(f"mpcx_problem_mid_fleet failed ({rc}) for {mp}; using the main build")
                else:
                    self.mid_fleet_path = mp
        self.wide_fleet_path = None
        if hsaco is None and os.environ.get("MPCX_WIDE_FLEET", "1") != "0":
            # fleets of more than one generation of a 16-agents-per-CU main build run the
            # 20-agents-per-CU build where its spills stay small
            wp = compile_model(gen, variant=WIDE_FLEET)
            if wp is not None:
                rc = self.lib.mpcx_problem_wide_fleet(handle, str(wp).encode(), -1)
                if rc != 0:  # optional, as the other builds
                    warnings.warn(f"mpcx_problem_wide_fleet failed ({rc}) for {wp}; using the main build")
                else:
                    self.wide_fleet_path = wp
        self.options = default_options()
        self.nw = d["NX"] + d["N"] * (d["NV"] + d["NX"])
        self.ng_total = d["N"] * d["NG"]
        self.npar = d["NPG"] + d["N"] * d["NPS"]

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                self.lib.mpcx_problem_destroy(h)
            except Exception:  # pragma: no cover - interpreter shutdown
                pass
            self.handle = None

    def set_options(self, **kw):
        self.options_key = None  # set_options may be called directly: the backend's cache is stale
        for k, v in kw.items():
            if not hasattr(self.options, k):
                raise KeyError(f"unknown solver option {k!r}")
            setattr(self.options, k, v)
        rc = self.lib.mpcx_set_options(self.handle, ctypes.byref(self.options))
        if rc != 0:
            raise NativeError(f"mpcx_set_options failed ({rc})")

    def set_small_fleet_max(self, max_agents: int):
        """Largest batch launched on the small-fleet (workspace-in-LDS) build: -1 one generation
        (the CU count times the agents a CU's LDS holds of that build, at most four; default),
        0 never."""
        rc = self.lib.mpcx_problem_small_fleet(self.handle, None, int(max_agents))
        if rc != 0:
            raise NativeError(f"mpcx_problem_small_fleet failed ({rc})")

    def set_mid_fleet_max(self, max_agents: int):
        """Largest batch launched on the one-wave-per-SIMD build: -1 four per CU (default), 0 never."""
        rc = self.lib.mpcx_problem_mid_fleet(self.handle, None, int(max_agents))
        if rc != 0:
            raise NativeError(f"mpcx_problem_mid_fleet failed ({rc})")

    def set_wide_fleet_min(self, min_agents: int):
        """Smallest batch launched on the 20-agents-per-CU build: -1 more than one generation of
        the main build (default), 0 never."""
        rc = self.lib.mpcx_problem_wide_fleet(self.handle, None, int(min_agents))
        if rc != 0:
            raise NativeError(f"mpcx_problem_wide_fleet failed ({rc})")

    def workspace_bytes_per_agent(self) -> int:
        return int(self.lib.mpcx_workspace_bytes_per_agent(self.handle))

    def lds_bytes_per_agent(self) -> int:
        """LDS bytes of one agent's workgroup on the main build (C ABI v15)."""
        return int(self.lib.mpcx_lds_bytes_per_agent(self.handle))

    def reserve(self, n_agents: int):
        rc = self.lib.mpcx_reserve(self.handle, int(n_agents))
        if rc != 0:
            raise NativeError(f"mpcx_reserve failed ({rc})")

    def solve(self, p, lbw, ubw, w, lbg=None, ubg=None, lam_g=None, lam_w=None, stats=None,
              active=None, stream=None, agent_map=None, n_launch=None):
        """Launch the batched solve on device tensors (stream-ordered, async).

        ``agent_map`` (int32 [n] device tensor, with ``n_launch``): launch ``n_launch``
        workgroups, workgroup i solving agent ``agent_map[i]`` (-1: none) --
        ``mpcx_batch_solve_mapped``, the code object chosen by ``n_launch``.

        Every buffer the kernel reads or writes is checked here (dtype, device, contiguity,
        size): an undersized or host buffer would otherwise become an out-of-bounds device
        access instead of a Python error."""
        import torch

        n = int(p.shape[0])

        def check(name, t, shape, dtype=torch.float64):
            if t.dtype != dtype or not t.is_cuda or not t.is_contiguous() or tuple(t.shape) != shape:
                raise ValueError(f"{name} must be a contiguous {dtype} device tensor of shape {shape}, "
                                 f"got {tuple(t.shape)} {t.dtype} on {t.device}")

        for name, t, cols in (("p", p, self.npar), ("lbw", lbw, self.nw), ("ubw", ubw, self.nw),
                              ("w", w, self.nw)):
            check(name, t, (n, cols))
        if (lbg is None) != (ubg is None):
            raise ValueError("lbg and ubg must be given together")
        for name, t, cols in (("lbg", lbg, self.ng_total), ("ubg", ubg, self.ng_total),
                              ("lam_g", lam_g, self.ng_total), ("lam_w", lam_w, self.nw)):
            if t is not None:
                check(name, t, (n, cols))
        if stats is not None:
            check("stats", stats, (n * STATS_BYTES,), torch.uint8)
        if active is not None:
            check("active", active, (n,), torch.int32)
        if stream is None:
            stream = torch.cuda.current_stream().cuda_stream
        ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        if agent_map is not None:
            check("agent_map", agent_map, (n,), torch.int32)
            n_launch = int(n_launch)
            if not 0 <= n_launch <= n:
                raise ValueError(f"n_launch {n_launch} outside [0, {n}]")
            rc = self.lib.mpcx_batch_solve_mapped(self.handle, n, n_launch, ptr(agent_map), ptr(p), ptr(lbw),
                                                  ptr(ubw), ptr(lbg), ptr(ubg), ptr(w), ptr(lam_g), ptr(lam_w),
                                                  ptr(stats), ptr(active), ctypes.c_void_p(stream))
            if rc != 0:
                raise NativeError(f"mpcx_batch_solve_mapped failed ({rc})")
            return
        rc = self.lib.mpcx_batch_solve(self.handle, n, ptr(p), ptr(lbw), ptr(ubw), ptr(lbg), ptr(ubg),
                                       ptr(w), ptr(lam_g), ptr(lam_w), ptr(stats), ptr(active),
                                       ctypes.c_void_p(stream))
        if rc != 0:
            raise NativeError(f"mpcx_batch_solve failed ({rc})")

    def bind(self, p, lbw, ubw, w, lam_g=None, stats=None):
        """A launcher for buffers that stay where they are (the resident plugin batch): they
        are checked once here, the call then only passes the pre-built pointer arguments and
        the current stream (the per-call checks and pointer extraction cost ~25 us, a tenth of
        a single agent's kernel).  Keep the tensors alive while the launcher is used."""
        import torch

        n = int(p.shape[0])
        for name, t, cols in (("p", p, self.npar), ("lbw", lbw, self.nw), ("ubw", ubw, self.nw), ("w", w, self.nw),
                              ("lam_g", lam_g, self.ng_total)):
            if t is not None and (t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous()
                                  or tuple(t.shape) != (n, cols)):
                raise ValueError(f"{name}: contiguous float64 device tensor of shape {(n, cols)} expected")
        if stats is not None and (stats.dtype != torch.uint8 or tuple(stats.shape) != (n * STATS_BYTES,)):
            raise ValueError("stats: uint8 device tensor of n * STATS_BYTES expected")
        ptr = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        head = (self.handle, n, ptr(p), ptr(lbw), ptr(ubw), None, None, ptr(w), ptr(lam_g), None, ptr(stats), None)
        fn = self.lib.mpcx_batch_solve

        def launch(stream=None):
            s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
            rc = fn(*head, ctypes.c_void_p(s))
            if rc != 0:
                raise NativeError(f"mpcx_batch_solve failed ({rc})")
        return launch

    def bind_staged(self, p, lbw, ubw, w, lam_g, stats, host_in, dev_in, host_out, dev_out):
        """:meth:`bind` for the small-batch host round trip (``mpcx_batch_solve_staged``): the
        returned call uploads ``host_in`` (pinned) into ``dev_in``, solves, reads ``dev_out``
        back into ``host_out`` (pinned) and returns when both are done -- one native call."""
        import torch

        self.bind(p, lbw, ubw, w, lam_g=lam_g, stats=stats)  # the same argument checks
        for name, t, dev in (("host_in", host_in, False), ("dev_in", dev_in, True),
                             ("host_out", host_out, False), ("dev_out", dev_out, True)):
            if not t.is_contiguous() or t.is_cuda != dev or (not dev and not t.is_pinned()):
                raise ValueError(f"{name}: contiguous {'device' if dev else 'pinned host'} tensor expected")
        nin, nout = host_in.numel() * host_in.element_size(), host_out.numel() * host_out.element_size()
        if dev_in.numel() * dev_in.element_size() != nin or dev_out.numel() * dev_out.element_size() != nout:
            raise ValueError("staged buffers: host and device sizes differ")
        vp = ctypes.c_void_p
        args = (self.handle, int(p.shape[0]), vp(host_in.data_ptr()), vp(dev_in.data_ptr()), nin,
                vp(host_out.data_ptr()), vp(dev_out.data_ptr()), nout, vp(p.data_ptr()), vp(lbw.data_ptr()),
                vp(ubw.data_ptr()), vp(w.data_ptr()), None if lam_g is None else vp(lam_g.data_ptr()),
                None if stats is None else vp(stats.data_ptr()))
        fn = self.lib.mpcx_batch_solve_staged

        def roundtrip(stream=None):
            s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
            rc = fn(*args, vp(s))
            if rc != 0:
                raise NativeError(f"mpcx_batch_solve_staged failed ({rc})")
        return roundtrip


_STATS_DOUBLES = ("obj", "primal_inf", "dual_inf", "compl_inf", "mu", "obj_scale")


_STATS_DTYPE = None


def stats_array(raw_bytes):
    """``mpcx_stats`` records as a numpy structured array (no per-agent objects); a contiguous
    uint8 array is viewed in place, anything else copied."""
    import numpy as np

    global _STATS_DTYPE
    if _STATS_DTYPE is None:
        _STATS_DTYPE = np.dtype([(n, "<f8") for n in _STATS_DOUBLES] + [(n, "<i4") for n in _STATS_INTS])
        assert _STATS_DTYPE.itemsize == STATS_BYTES
    if isinstance(raw_bytes, np.ndarray) and raw_bytes.dtype == np.uint8 and raw_bytes.ndim == 1 \
            and raw_bytes.flags.c_contiguous and raw_bytes.size % STATS_BYTES == 0:
        return raw_bytes.view(_STATS_DTYPE)
    return np.frombuffer(bytes(raw_bytes), dtype=_STATS_DTYPE)


class StatsView:
    """Per-agent stats dicts (IPOPT ``stats()`` keys, `core/discretization.py:41-47`) built
    on access from the structured array; ``array`` holds all agents' fields."""

    def __init__(self, arr, extra: Optional[dict] = None):
        self.array = arr
        self.extra = extra or {}

    def __len__(self):
        return len(self.array)

    def __iter__(self):
        return (self[i] for i in range(len(self)))

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        # one conversion of the record to Python numbers (float / int per field), keys in the
        # order of the result files' stats columns
        v = dict(zip(self.array.dtype.names, self.array[i].tolist()))
        st = v["status"]
        d = {k: v[k] for k in _STATS_DOUBLES}
        d["status"] = st
        d["return_status"] = STATUS_NAMES.get(st, str(st))
        d["success"] = st in (0, 1)
        for k in _STATS_INTS:
            if k != "status":
                d[k] = v[k]
        d.update(self.extra)
        return d

    @property
    def success(self):
        return (self.array["status"] == 0) | (self.array["status"] == 1)


def stats_to_dicts(raw_bytes) -> list:
    """Decode a uint8 tensor/bytes of n * sizeof(mpcx_stats) into dicts."""
    buf = bytes(raw_bytes)
    n = len(buf) // STATS_BYTES
    arr = (Stats * n).from_buffer_copy(buf)
    out = []
    for s in arr:
        d = {"obj": s.obj, "primal_inf": s.primal_inf, "dual_inf": s.dual_inf,
             "compl_inf": s.compl_inf, "mu": s.mu, "obj_scale": s.obj_scale,
             "status": s.status, "return_status": STATUS_NAMES.get(s.status, str(s.status)),
             "success": s.status in (0, 1)}
        for k in _STATS_INTS:
            d[k] = getattr(s, k)
        out.append(d)
    return out
