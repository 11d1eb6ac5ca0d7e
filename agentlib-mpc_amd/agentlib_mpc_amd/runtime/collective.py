"""The one collective of an ADMM iteration, issued through the C ABI (``mpcx_admm_allreduce``, v14).

SURVEY §8b: the library issues the fleet's per-iteration all-reduce on its registered transport
(`include/mpcx.h`, ``mpcx_allreduce_register``); the Python fleet driver calls that entry point
like a C caller would, so both go through the same hook.  Transport chosen per
process group (``MPCX_COLLECTIVE``):

* ``auto`` (default) -- an ``nccl`` (= RCCL) process group: a communicator of the library's own,
  made once per process with ``mpcx_rccl_comm_init`` from the RCCL copy PyTorch already loaded
  (the unique id travels once, at set-up, with ``broadcast_object_list``); the library then calls
  ``ncclAllReduce`` on the fleet's stream.  Its own communicator keeps the fleet's collectives out
  of the order of PyTorch's (a communicator's operations must be issued in the same order on every
  rank).  Any other backend (``gloo``): the function transport below.
* ``torch`` -- the function transport for every backend: ``mpcx_allreduce_register_fn`` with a
  callback that runs ``torch.distributed.all_reduce`` on the registered buffer.

The reference exchange this serves: the coordinator's gather of the locals and broadcast of the
means (`modules/dmpc/admm/admm_coordinator.py:284-314`).
"""

from __future__ import annotations

import ctypes
import os
import weakref
from typing import Dict, Optional, Tuple

from agentlib_mpc_amd.runtime import native

_state: Dict[str, object] = {"key": None, "kind": None, "comm": None, "path": None}
_buffers: Dict[int, Tuple[object, object]] = {}   # data_ptr -> (weak ref of the tensor, process group)
_callback = None                                    # the registered ctypes function (kept alive)


def loaded_rccl_path() -> Optional[str]:
    """Path of the RCCL library already mapped into this process (PyTorch's copy), or None."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 6 and "librccl" in os.path.basename(parts[-1]):
                    return parts[-1]
    except OSError:
        pass
    return None


def _fn_transport(ctx, buf, count, stream):
    """mpcx_allreduce_fn over torch.distributed: the buffer is looked up by its address (the
    fleets register theirs), summed over the ranks in place."""
    try:
        ent = _buffers.get(int(buf or 0))
        if ent is None:
            return 1
        ref, group = ent
        t = ref()
        if t is None:
            return 1
        import torch.distributed as dist

        dist.all_reduce(t[:int(count)], group=group)
        return 0
    except Exception:  # nothing may propagate through the C frame
        return 1


def _register_fn():
    global _callback
    lib = native.load_library()
    if _callback is None:
        _callback = native.ALLREDUCE_FN(_fn_transport)
    rc = lib.mpcx_allreduce_register_fn(_callback, None)
    if rc != 0:
        raise native.NativeError(f"mpcx_allreduce_register_fn failed ({rc})")


def _register_rccl(dist, group, world: int, rank: int):
    """A library-owned RCCL communicator over the ranks of ``group`` (made once per process)."""
    lib = native.load_library()
    path = loaded_rccl_path()
    cpath = path.encode() if path else None
    uid = ctypes.create_string_buffer(native.RCCL_ID_BYTES)
    if rank == 0:
        rc = lib.mpcx_rccl_unique_id(cpath, uid)
        if rc != 0:
            raise native.NativeError(f"mpcx_rccl_unique_id failed ({rc})")
    box = [uid.raw if rank == 0 else None]
    dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    ctypes.memmove(uid, box[0], native.RCCL_ID_BYTES)
    comm = ctypes.c_void_p()
    rc = lib.mpcx_rccl_comm_init(cpath, int(world), int(rank), uid, ctypes.byref(comm))
    if rc != 0:
        raise native.NativeError(f"mpcx_rccl_comm_init failed ({rc})")
    rc = lib.mpcx_allreduce_register(comm, cpath)
    if rc != 0:
        raise native.NativeError(f"mpcx_allreduce_register failed ({rc})")
    return comm, path


class Collective:
    """The fleet's handle on the library's collective: ``bind`` a buffer once, then
    ``allreduce(n)`` sums its first ``n`` doubles over the ranks through ``mpcx_admm_allreduce``."""

    def __init__(self, dist, group, device):
        self.dist, self.group, self.device = dist, group, device
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        mode = os.environ.get("MPCX_COLLECTIVE", "auto")
        if mode not in ("auto", "torch", "rccl"):
            raise ValueError(f"MPCX_COLLECTIVE={mode!r}: auto, torch or rccl")
        backend = str(dist.get_backend(group)).lower()
        want = "rccl" if (mode == "rccl" or (mode == "auto" and backend == "nccl")) else "fn"
        if want == "rccl" and getattr(device, "type", "cuda") != "cuda":
            raise ValueError("the RCCL transport needs device buffers")
        key = (want, id(group), self.world, self.rank)
        if _state["key"] != key:
            if want == "rccl":
                comm, path = _register_rccl(dist, group, self.world, self.rank)
                _state.update(comm=comm, path=path)
            else:
                _register_fn()
            _state.update(key=key, kind=want)
        self.kind = want
        self.lib = native.load_library()
        self.buf = None

    def bind(self, tensor):
        """The buffer the iterations reduce (contiguous float64; its address must not change)."""
        if tensor.dtype.itemsize != 8 or not tensor.is_contiguous():
            raise ValueError("the collective's buffer must be a contiguous float64 tensor")
        self.buf = tensor
        _buffers[int(tensor.data_ptr())] = (weakref.ref(tensor), self.group)

    def allreduce(self, count: int):
        """Sum the first ``count`` doubles of the bound buffer over the ranks (in place,
        stream-ordered on the current stream): ONE ``mpcx_admm_allreduce`` call."""
        t = self.buf
        if t is None or not 0 <= count <= t.numel():
            raise ValueError(f"allreduce of {count} doubles: bind a buffer that holds them first")
        stream = None
        if t.is_cuda:
            import torch

            stream = torch.cuda.current_stream(t.device).cuda_stream
        rc = self.lib.mpcx_admm_allreduce(ctypes.c_void_p(t.data_ptr()), int(count),
                                          ctypes.c_void_p(stream) if stream else None)
        if rc != 0:
            raise native.NativeError(f"mpcx_admm_allreduce failed ({rc}, transport {self.kind})")


def calls() -> int:
    """Collectives issued through ``mpcx_admm_allreduce`` in this process."""
    return int(native.load_library().mpcx_allreduce_calls())


def kind() -> int:
    """The registered transport (native.COLLECTIVE_NONE / _RCCL / _FN)."""
    return int(native.load_library().mpcx_allreduce_kind())
