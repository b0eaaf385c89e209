"""Device context: one process per GPU, optionally one RCCL rank of a node-wide job.

The reference is a single CPU process (code.py has no distribution).  Here a
context binds one HIP device and, for world > 1, one RCCL rank; operators built
on it own a contiguous slab of layers.
"""
from __future__ import annotations

import ctypes
import os

from . import _ffi
from ._ffi import check, lib

_default = None


class Context:
    """A device (+ RCCL rank).  ``virtual_slabs`` > 1 splits this rank's rows into
    that many slabs on the same device (tests the decomposition on one GPU)."""

    def __init__(self, device: int = 0, rank: int = 0, world: int = 1, nccl_id: bytes | None = None,
                 virtual_slabs: int = 1, transport: str = "rccl"):
        """transport: "rccl" (production: one GPU per rank, RCCL over xGMI) or "shm"
        (host-staged shared memory; ranks may share one GPU -- test rehearsal)."""
        self.device, self.rank, self.world, self.virtual_slabs = device, rank, world, virtual_slabs
        self.transport = transport
        kinds = {"rccl": _ffi.HH_TRANSPORT_RCCL, "shm": _ffi.HH_TRANSPORT_SHM}
        if transport not in kinds:
            raise ValueError(f"unknown transport {transport!r}")
        h = ctypes.c_void_p()
        idbuf = None
        if world > 1:
            if nccl_id is None or len(nccl_id) != 128:
                raise ValueError("world > 1 needs the 128-byte communicator id from rank 0")
            idbuf = (ctypes.c_ubyte * 128).from_buffer_copy(nccl_id)
        check(lib.hh_ctx_create_ex(device, rank, world, idbuf, virtual_slabs, kinds[transport],
                                   ctypes.byref(h)))
        self._h = h
        _ffi.track(self, 2)

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("context destroyed")
        return self._h

    def allreduce_max(self, values):
        import numpy as np
        a = np.ascontiguousarray(values, dtype=np.float64).copy()
        check(lib.hh_ctx_allreduce_max(self.handle, _ffi.dptr(a), a.size))
        return a

    def allreduce_sum(self, values):
        import numpy as np
        a = np.ascontiguousarray(values, dtype=np.float64).copy()
        check(lib.hh_ctx_allreduce_sum(self.handle, _ffi.dptr(a), a.size))
        return a

    def barrier(self):
        check(lib.hh_ctx_barrier(self.handle))

    def synchronize(self):
        check(lib.hh_ctx_synchronize(self.handle))

    def collectives(self) -> int:
        """Collectives (halo exchanges + allreduces) this rank has entered (hh_ctx_progress);
        safe to call from another thread while this one is blocked inside a collective."""
        n = ctypes.c_long()
        check(lib.hh_ctx_progress(self.handle, ctypes.byref(n)))
        return n.value

    def close(self):
        if getattr(self, "_h", None) is not None:
            lib.hh_ctx_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass


def unique_id() -> bytes:
    buf = (ctypes.c_ubyte * 128)()
    check(lib.hh_comm_unique_id(buf))
    return bytes(buf)


def knobs(only_changed: bool = True) -> dict:
    """The library's HH_* knobs (hh_knobs_json): {name: {"value", "default"}} -- only those that
    differ from the shipped path by default, so a default run reports {}."""
    import json
    need = ctypes.c_int()
    check(lib.hh_knobs_json(int(only_changed), None, 0, ctypes.byref(need)))
    buf = ctypes.create_string_buffer(need.value)
    check(lib.hh_knobs_json(int(only_changed), buf, need.value, None))
    return json.loads(buf.value.decode())


def device_count() -> int:
    n = ctypes.c_int()
    check(lib.hh_device_count(ctypes.byref(n)))
    return n.value


def default_context() -> Context:
    """Single-rank context on LOCAL_RANK's device (0 when unset)."""
    global _default
    if _default is None:
        _default = Context(device=int(os.environ.get("HH_DEVICE", os.environ.get("LOCAL_RANK", "0"))))
    return _default


def set_default_context(ctx: Context | None) -> None:
    global _default
    _default = ctx
