"""The C-ABI library (CPU, no GPU calls): it builds for gfx950, loads, and exports
every entry point declared in include/mpcx.h; generated kernels compile."""

import ctypes
import pathlib
import re

import pytest

from agentlib_mpc_amd.runtime import native

HEADER = pathlib.Path(__file__).resolve().parents[1] / "include" / "mpcx.h"


def declared_functions():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|void|int64_t)\s+(mpcx_\w+)\s*\(", text, re.M)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    assert "mpcx_batch_solve" in names and "mpcx_problem_create" in names
    assert set(names) == set(native.EXPORTED_SYMBOLS)


def test_library_builds_loads_and_exports_all_symbols():
    path = native.build_library()
    lib = ctypes.CDLL(str(path))
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.mpcx_version() == 15


def test_v15_entry_points_check_their_arguments():
    """C ABI v15 without a GPU: the LDS query answers -1 for no handle, the stream functions reject
    a null pointer before any HIP call (the GPU side: test_gpu_dedicated_streams_overlap)."""
    lib = native.load_library()
    assert lib.mpcx_lds_bytes_per_agent(None) == -1
    assert lib.mpcx_stream_create_dedicated(None) == native.ERR_ARG
    assert lib.mpcx_stream_destroy(None) == native.ERR_ARG


def test_collective_goes_through_the_registered_transport():
    """C ABI v14: mpcx_admm_allreduce issues the ADMM iteration's one all-reduce on the
    transport registered with the library.  A stub transport (a C-callable function that "sums" over
    two identical ranks by doubling) through the ABI: every call reaches it once with the buffer and
    length, the library counts the calls, and without a transport the call fails (MPCX_ERR_COMM).
    No GPU: host buffers, null stream."""
    import numpy as np

    lib = native.load_library()
    seen = []

    def stub(ctx, buf, count, stream):
        a = np.ctypeslib.as_array((ctypes.c_double * count).from_address(buf))
        a *= 2.0  # two ranks holding the same values
        seen.append((buf, count, ctx))
        return 0

    fn = native.ALLREDUCE_FN(stub)
    x = np.arange(1.0, 8.0)
    ptr = ctypes.c_void_p(x.ctypes.data)
    try:
        assert lib.mpcx_allreduce_register_fn(fn, ctypes.c_void_p(1234)) == 0
        assert lib.mpcx_allreduce_kind() == native.COLLECTIVE_FN
        c0 = lib.mpcx_allreduce_calls()
        for _ in range(3):
            assert lib.mpcx_admm_allreduce(ptr, 5, None) == 0
        assert lib.mpcx_allreduce_calls() - c0 == 3
        assert seen == [(x.ctypes.data, 5, 1234)] * 3
        np.testing.assert_array_equal(x, np.r_[8.0 * np.arange(1.0, 6.0), 6.0, 7.0])
        assert lib.mpcx_admm_allreduce(ptr, -1, None) == native.ERR_ARG
    finally:
        lib.mpcx_allreduce_unregister()
    assert lib.mpcx_allreduce_kind() == native.COLLECTIVE_NONE
    assert lib.mpcx_admm_allreduce(ptr, 5, None) == native.ERR_COMM
    # the RCCL transport's argument checks (no communicator is made here)
    assert lib.mpcx_allreduce_register(None, None) == native.ERR_ARG
    comm = ctypes.c_void_p()
    assert lib.mpcx_rccl_comm_init(None, 2, 2, ctypes.create_string_buffer(128), ctypes.byref(comm)) == native.ERR_ARG


def test_struct_sizes_match_header():
    # mpcx_options: 40 doubles + 4 int32; mpcx_stats: 6 doubles + 12 int32
    assert ctypes.sizeof(native.Options) == 40 * 8 + 4 * 4
    assert ctypes.sizeof(native.Stats) == 6 * 8 + 12 * 4
    assert ctypes.sizeof(native.ProblemDesc) == 8 * 4


def test_default_options_are_ipopt_defaults():
    o = native.default_options()
    assert o.mu_init == 0.1 and o.kappa_mu == 0.2 and o.theta_mu == 1.5
    assert o.bound_push == 1e-2 and o.kappa_sigma == 1e10 and o.tau_min == 0.99
    # IPOPT's acceptable-level defaults (the backend applies the reference's overrides)
    assert o.acceptable_tol == 1e-6 and o.acceptable_iter == 15 and o.acceptable_dual_inf_tol == 1e10
    assert o.acceptable_constr_viol_tol == 1e-2 and o.acceptable_compl_inf_tol == 1e-2
    assert o.acceptable_obj_change_tol == 1e20


def test_generated_kernel_compiles(tmp_path, monkeypatch):
    from agentlib_mpc_amd import benchmarks as bm

    be, _ = bm.exchange_supply()
    path = be.problem.compile()
    assert path.exists() and path.stat().st_size > 0
    # the small-fleet build (workspace hot part in LDS) of the same structure
    sp = native.compile_model(be.problem.gen, variant=native.SMALL_FLEET)
    assert sp is not None and sp.exists() and sp != path


def test_small_fleet_build_keeps_hbm_addressing_off_the_lds_workspace(tmp_path):
    """In the small-fleet build the only global-memory stores are the kernel's outputs and the
    workspace's cold part: the phases that run every iteration (evaluators, elimination,
    line search, iteration head) address the LDS workspace with LDS instructions (a pointer
    cast from the LDS workspace to an HBM type was a wild address on the GPU).  The build inlines
    those phases into the kernel body; compiled out of line here (MPCX_HOT) they can be told
    apart by function."""
    import re
    import subprocess

    from agentlib_mpc_amd import benchmarks as bm

    be, _ = bm.one_room()
    src = tmp_path / "wslds_isa.hip"
    src.write_text(be.problem.gen.source)
    out = src.with_suffix(".s")
    subprocess.run([native._hipcc(), "--cuda-device-only", "-S", f"--offload-arch={native.OFFLOAD_ARCH}", "-O3",
                    "-std=c++17", f"-I{native.INCLUDE}", f"-I{native.CSRC}", "-DMPCX_WS_LDS", "-DMPCX_HOT=__noinline__",
                    str(src), "-o", str(out)],
                   check=True, capture_output=True)
    fn, stores = None, {}
    for line in out.read_text().splitlines():
        m = re.match(r"^(_Z\S+|mpcx_ipm_solve):", line)
        if m:
            fn = m.group(1)
        elif "global_store" in line or "flat_store" in line:
            stores[fn] = stores.get(fn, 0) + 1
    hot = ("line_search", "recover_step", "accept_step", "local_assemble", "chain_factor", "eval_fg")
    bad = {f: c for f, c in stores.items() if f and any(h in f for h in hot) and "resto" not in f}
    assert not bad, bad
    assert stores.get("mpcx_ipm_solve", 0) <= 40, stores.get("mpcx_ipm_solve")


def test_product_path_has_no_cpu_fallback(monkeypatch):
    monkeypatch.setattr(native, "LIB_PATH", pathlib.Path("/nonexistent/libmpcx.so"))
    monkeypatch.setattr(native, "_lib", None)
    with pytest.raises(native.NativeError):
        native.load_library()


def test_kernel_abi_versions_agree():
    """The code objects report MPCX_KERNEL_ABI (csrc/mpcx_internal.h); the Python binding and
    the generated sources must use the same number (mpcx_problem_create rejects a mismatch)."""
    import re

    from agentlib_mpc_amd.runtime import codegen, native

    text = (native.CSRC / "mpcx_internal.h").read_text()
    abi = int(re.search(r"#define MPCX_KERNEL_ABI (\d+)", text).group(1))
    assert native.KERNEL_ABI == abi == codegen.KERNEL_ABI_VERSION


def test_small_fleet_variant_failure_is_not_fatal(tmp_path, monkeypatch):
    """The small-fleet build is optional: ANY failure of its compile means "no
    small-fleet build this time" (the HBM build serves every batch), while a failure of the main
    code object stays fatal.  Only a structural misfit (the kernel's LDS static_asserts) leaves a
    permanent .nofit marker; a transient failure (hipcc killed, out of memory) warns and is
    retried by the next compile."""
    from agentlib_mpc_amd import benchmarks as bm

    be, _ = bm.one_room()
    gen = be.problem.gen
    monkeypatch.setattr(native, "KERNEL_DIR", tmp_path)
    monkeypatch.setattr(native, "_hipcc", lambda: "/bin/false")
    nofit = native.code_object_path(gen.key, native.SMALL_FLEET).with_suffix(".nofit")
    with pytest.warns(UserWarning, match="small-fleet build"):
        assert native.compile_model(gen, variant=native.SMALL_FLEET) is None
    assert not nofit.exists()                 # transient: no marker, retried
    fake = tmp_path / "fake_hipcc.sh"         # a compiler that reports the static_assert
    fake.write_text("#!/bin/sh\necho 'error: static assertion failed: MPCX_WS_LDS: workspace does not fit LDS' >&2\n"
                    "exit 1\n")
    fake.chmod(0o755)
    monkeypatch.setattr(native, "_hipcc", lambda: str(fake))
    assert native.compile_model(gen, variant=native.SMALL_FLEET) is None
    assert nofit.exists()
    monkeypatch.setattr(native, "_hipcc", lambda: "/bin/false")
    assert native.compile_model(gen, variant=native.SMALL_FLEET) is None  # marker: no retry
    with pytest.raises(native.NativeError):
        native.compile_model(gen)


def test_one_wave_per_simd_build_only_where_the_main_build_is_tighter():
    """The mid-fleet variant (``mpcx_problem_mid_fleet``, C ABI v9) is compiled only when the main
    build's register budget allows more than one wave per SIMD (read from the compiler's resource
    report into the ``.occ`` file next to the main code object): one_room (16 agents per CU, 4
    waves per SIMD) gets it, the MHE (4 agents per CU, already one wave per SIMD) does not."""
    from agentlib_mpc_amd import benchmarks as bm

    gen = bm.one_room()[0].problem.gen
    assert native.compile_model(gen, variant=native.MID_FLEET) is not None
    assert int(native.code_object_path(gen.key).with_suffix(".occ").read_text()) == 4
    gen = bm.mhe_room()[0].problem.gen
    assert native.compile_model(gen, variant=native.MID_FLEET) is None
    assert int(native.code_object_path(gen.key).with_suffix(".occ").read_text()) == 1
