"""The NARX networks are evaluated on the FP64 matrix cores (CPU checks of the generated
code; the numerics are checked on the GPU by the room_nn / C5 parity cases in
tests/test_gpu_ipm.py and tests/test_gpu_admm.py).

Reference: the serialized ANN evaluated by CasADi inside IPOPT
(`agentlib_mpc/models/casadi_predictor.py:306-336`); here one batched
``[stages x call sites, inputs] x [inputs, hidden]`` product per wavefront and network
(csrc/mpcx_net_mfma.h).
"""

import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from agentlib_mpc_amd import benchmarks as bm
from agentlib_mpc_amd import symbolic as sx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gen(N=None):
    be, _ = bm.room_nn() if N is None else bm.room_nn(N=N)
    return be.problem.gen


def test_network_section_is_generated():
    src = _gen().source
    assert "#define MPCX_NET_MFMA 1" in src
    # every network is evaluated over all stages x call sites in one call per evaluation kind
    calls = re.findall(r"mpcx_net::eval<(\d+), (\d+), (\d+), (\d+), (\w+), (\d+), (\d+)>", src)
    assert len(calls) == 6   # 2 networks x (fg, gj, hess)
    n = int(re.search(r"#define MPCX_N (\d+)", src).group(1))
    for R, nin, H, act, wv, nd1, nd2 in calls:
        assert int(R) % n == 0 and int(H) == 32 and int(act) == sx.ACT_CODE["sigmoid"]
    # the stage functions of the kernel read the network entries instead of looping
    body = src[src.index("gen_stage_fg_m("):src.index("// <<< device only")]
    assert "for (int j = 0; j < 32; ++j)" not in body


def test_second_derivative_tables_are_pair_products():
    src = _gen().source
    m = re.search(r"__constant__ double ANN0_PWhess\[(\d+)\] = \{([^}]*)\}", src)
    d1 = re.search(r"__constant__ int ANN0_D1gj\[\d+\] = \{([^}]*)\}", src)
    assert m and d1
    rows = np.array([float(v) for v in m.group(2).split(",")]).reshape(-1, 32)

    def pair_products(w1):   # every row is W1[a] * W1[b] for some input pair (a >= b)
        return all(any(np.array_equal(r, w1[a] * w1[b]) for a in range(len(w1)) for b in range(a + 1))
                   for r in rows)

    assert any(pair_products(sx.network(i).W1) for i in range(len(sx._NETWORKS)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_code_object_issues_fp64_mfma(tmp_path):
    gen = _gen()
    src = tmp_path / "m.hip"
    src.write_text(gen.source)
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    out = tmp_path / "m.s"
    subprocess.run([hipcc, "--cuda-device-only", "-S", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    f"-I{ROOT}/include", f"-I{ROOT}/agentlib-mpc_amd/csrc", str(src), "-o", str(out)],
                   check=True, capture_output=True)
    asm = out.read_text()
    assert asm.count("v_mfma_f64_16x16x4") >= 6
