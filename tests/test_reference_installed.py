"""Drop-in with the reference INSTALLED (CPU, build container only).

In a real deployment ``agentlib_mpc`` (with agentlib and casadi) is importable, so a model
file's ``from agentlib_mpc.models.casadi_model import ...`` binds the reference's CasADi
classes, which the MI355X backend cannot trace (`optimization_backends/backend.py:94-100`
would then reject them).  This test puts a stand-in ``agentlib_mpc`` package on
``sys.path`` (so ``compat.reference_available()`` is True and nothing is aliased
globally), whose model classes refuse to be instantiated as the CasADi ones would here,
and checks in a fresh interpreter that

* the reference's own example model files, injected as ``{"file", "class_name"}``
  (`modules/mpc/mpc.py:110-143`), give exactly the NLP of the non-installed mode;
* a model class imported normally from such a file (config ``type`` given as the class)
  is re-read against this package's model API and gives the same NLP;
* the backends are instances of the installed reference's ``OptimizationBackend`` /
  ``ADMMBackend`` (the ``create_optimization_backend`` assertion, `mpc.py:142`);
* the reference's module names in ``sys.modules`` still belong to the reference.
"""

import hashlib
import json
import pathlib
import subprocess
import sys
import textwrap

import pytest

from agentlib_mpc_amd import benchmarks as bm

REPO = pathlib.Path(__file__).resolve().parents[1]
REF = pathlib.Path("/root/reference/examples")
pytestmark = pytest.mark.skipif(not REF.is_dir(), reason="reference examples not present")

CASES = [
    ("one_room", "one_room_mpc/physical/simple_mpc.py", "MyCasadiModel"),
    ("admm_room", "4_Room_ADMM_Coordinator/models/room_model.py", "CaCooledRoom"),
    ("admm_ahu", "4_Room_ADMM_Coordinator/models/rlt_model.py", "RLT"),
    ("exchange_room", "exchange_admm/models/room_model.py", "CaCooledRoom"),
    ("exchange_supply", "exchange_admm/models/rlt_model.py", "RLT"),
]

STUB_MODEL_API = '''
"""Stand-in for the installed reference model API: CasADi classes that cannot be traced."""
from typing import List, Optional, Union, Dict


class _Var:
    def __init__(self, **kw):
        self.__dict__.update(kw)


class CasadiVariable(_Var):
    pass


class CasadiState(CasadiVariable):
    pass


class CasadiInput(CasadiVariable):
    pass


class CasadiOutput(CasadiVariable):
    pass


class CasadiParameter(CasadiVariable):
    pass


class CasadiModelConfig:
    pass


class CasadiModel:
    def __init__(self, **kw):
        raise RuntimeError("reference CasadiModel instantiated (needs casadi)")
'''

STUB_BACKEND = '''
import abc


class OptimizationBackend(abc.ABC):
    @abc.abstractmethod
    def setup_optimization(self, var_ref):
        ...

    @abc.abstractmethod
    def solve(self, now, current_vars):
        ...


class ADMMBackend(OptimizationBackend):
    pass
'''


def _write_stub(root: pathlib.Path):
    files = {
        "agentlib/__init__.py": "",
        "agentlib/utils/__init__.py": "",
        "agentlib/utils/multi_agent_system.py": "class LocalMASAgency:\n    pass\n",
        "agentlib_mpc/__init__.py": "",
        "agentlib_mpc/models/__init__.py": "",
        "agentlib_mpc/models/casadi_model.py": STUB_MODEL_API,
        "agentlib_mpc/optimization_backends/__init__.py": "",
        "agentlib_mpc/optimization_backends/backend.py": STUB_BACKEND,
        "agentlib_mpc/utils/__init__.py": "",
        "agentlib_mpc/utils/plotting/__init__.py": "",
        "agentlib_mpc/utils/plotting/interactive.py": "def show_dashboard(*a, **k):\n    pass\n",
    }
    for rel, text in files.items():
        p = root / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(text)


CHILD = textwrap.dedent('''
    import hashlib, importlib.util, json, sys
    from agentlib_mpc_amd import compat
    assert compat.reference_available()
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc.optimization_backends import backend as refbe
    import agentlib_mpc.models.casadi_model as ref_api
    cases, ref = json.loads(sys.argv[1]), sys.argv[2]
    out = {}
    for builder, rel, cls in cases:
        be, _ = bm.BUILDERS[builder](model={"type": {"file": ref + "/" + rel, "class_name": cls}})
        assert isinstance(be, refbe.OptimizationBackend), type(be).__mro__
        assert not isinstance(be.model, ref_api.CasadiModel)
        out[builder] = hashlib.sha1(be.problem.gen.source.encode()).hexdigest()
    # a class imported normally: it derives from the reference's CasadiModel
    spec = importlib.util.spec_from_file_location(
        "user_room_model", ref + "/4_Room_ADMM_Coordinator/models/room_model.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules["user_room_model"] = mod
    spec.loader.exec_module(mod)
    assert issubclass(mod.CaCooledRoom, ref_api.CasadiModel)
    assert compat.is_reference_model_class(mod.CaCooledRoom)
    be, _ = bm.BUILDERS["admm_room"](model={"type": mod.CaCooledRoom})
    assert isinstance(be, refbe.ADMMBackend)
    out["admm_room_class"] = hashlib.sha1(be.problem.gen.source.encode()).hexdigest()
    assert sys.modules["agentlib_mpc.models.casadi_model"] is ref_api
    print("RESULT " + json.dumps(out))
''')


def test_reference_models_trace_with_the_reference_installed(tmp_path):
    _write_stub(tmp_path)
    want = {}
    for builder, _, _ in CASES:
        be, _ = bm.BUILDERS[builder]()
        want[builder] = hashlib.sha1(be.problem.gen.source.encode()).hexdigest()
    want["admm_room_class"] = want["admm_room"]
    env_path = [str(tmp_path), str(REPO / "agentlib-mpc_amd"), str(REPO)]
    proc = subprocess.run(
        [sys.executable, "-c", CHILD, json.dumps(CASES), str(REF)], capture_output=True, text=True,
        env={"PYTHONPATH": ":".join(env_path), "PATH": "/usr/bin:/bin", "HOME": str(tmp_path)}, timeout=600)
    assert proc.returncode == 0, proc.stderr[-4000:]
    line = next(ln for ln in proc.stdout.splitlines() if ln.startswith("RESULT "))
    got = json.loads(line[len("RESULT "):])
    assert got == want
