"""Drop-in model loading (CPU, build container only): the reference's OWN example model
files load unchanged through the backend's ``{"file", "class_name"}`` model injection
(`modules/mpc/mpc.py:110-143`, `optimization_backends/backend.py:94-100`), their
``agentlib_mpc.models.casadi_model`` imports resolving to this package
(`agentlib_mpc_amd/compat.py`), and yield exactly the NLP the package's restated example
models (`models/examples.py`) give: identical generated stage code, hence identical
variables, constraints, objective and derivatives.

The files are read from /root/reference (absent on the GPU box, hence skipped there).
`simple_mpc.py` is a script: its module-level imports of the agentlib runtime and the
plotting dashboard (`simple_mpc.py:16-17`) are stubbed; the model classes are untouched."""

import pathlib
import sys
import types

import pytest

from agentlib_mpc_amd import benchmarks as bm

REF = pathlib.Path("/root/reference/examples")
pytestmark = pytest.mark.skipif(not REF.is_dir(), reason="reference examples not present")


@pytest.fixture(scope="module", autouse=True)
def _script_imports():
    """Only what simple_mpc.py's script part imports at module level."""
    stubs = {}
    for name in ("agentlib", "agentlib.utils", "agentlib.utils.multi_agent_system",
                 "agentlib_mpc.utils", "agentlib_mpc.utils.plotting", "agentlib_mpc.utils.plotting.interactive"):
        if name not in sys.modules:
            stubs[name] = sys.modules[name] = types.ModuleType(name)
    sys.modules["agentlib.utils.multi_agent_system"].LocalMASAgency = object
    sys.modules["agentlib_mpc.utils.plotting.interactive"].show_dashboard = None
    from agentlib_mpc_amd.compat import install_reference_aliases

    assert install_reference_aliases()
    for name in ("agentlib_mpc.utils", "agentlib_mpc.utils.plotting"):
        sys.modules[name].__path__ = []
    yield
    for name in stubs:
        sys.modules.pop(name, None)


CASES = [
    ("one_room", "one_room_mpc/physical/simple_mpc.py", "MyCasadiModel"),
    ("admm_room", "4_Room_ADMM_Coordinator/models/room_model.py", "CaCooledRoom"),
    ("admm_ahu", "4_Room_ADMM_Coordinator/models/rlt_model.py", "RLT"),
    ("exchange_room", "exchange_admm/models/room_model.py", "CaCooledRoom"),
    ("exchange_supply", "exchange_admm/models/rlt_model.py", "RLT"),
]


@pytest.mark.parametrize("builder,rel,cls", CASES)
def test_reference_model_file_gives_the_same_nlp(builder, rel, cls):
    ours, _ = bm.BUILDERS[builder]()
    theirs, _ = bm.BUILDERS[builder](model={"type": {"file": str(REF / rel), "class_name": cls}})
    assert type(theirs.model).__module__.startswith("_mpcx_injected_")
    a, b = ours.problem, theirs.problem
    assert a.nlp.nlp_dims() == b.nlp.nlp_dims()
    assert list(a.layout.columns) == list(b.layout.columns)
    assert a.gen.source == b.gen.source
