"""One process per GPU on one node: rendezvous and row-slab bookkeeping.

The launcher (``python -m torch.distributed.run --nproc-per-node N ...``) sets
RANK / WORLD_SIZE / LOCAL_RANK.  Rank 0 creates the RCCL unique id and hands it
to the other ranks through a file in the node-local temp directory keyed by the
launcher's PID and MASTER_PORT (every rank is a child of the same launcher); each
rank then joins the RCCL communicator inside the C library.  No torch import is
needed on the product path.

Row slabs: rank r of P owns layers [floor(r n / P), floor((r+1) n / P)) -- the
same formula the C runtime uses (runtime.cpp, hh_op_create).
"""
from __future__ import annotations

import os
import tempfile
import time

from .context import Context, unique_id


def slab_bounds(n: int, world: int, rank: int):
    """0-based layer range [j0, j1) owned by `rank` (matches the C runtime)."""
    return (rank * n) // world, ((rank + 1) * n) // world


def env_rank_world():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))))


def job_key() -> str:
    """A key every rank of this launch computes alike (the launcher's PID, MASTER_PORT and run
    id): names the node-local files the ranks share (rendezvous id, watchdog state)."""
    return f"{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}_" \
           f"{os.environ.get('TORCHELASTIC_RUN_ID', 'none')}"


def job_file(kind: str, suffix: str, key: str | None = None) -> str:
    return os.path.join(os.environ.get("TMPDIR", tempfile.gettempdir()),
                        f"hh_{kind}_{key or job_key()}{suffix}")


def _rdzv_path(key: str | None):
    return job_file("rdzv", ".id", key)


def exchange_unique_id(rank: int, world: int, key: str | None = None, timeout: float = 300.0,
                       make_id=unique_id) -> bytes:
    """Rank 0 publishes a 128-byte id; the others wait for it (single node)."""
    path = _rdzv_path(key)
    if rank == 0:
        uid = make_id()
        tmp = path + f".tmp{os.getpid()}"
        with open(tmp, "wb") as fh:
            fh.write(uid)
        os.replace(tmp, path)
        return uid
    t0 = time.monotonic()
    while True:
        try:
            with open(path, "rb") as fh:
                data = fh.read()
            if len(data) == 128:
                return data
        except FileNotFoundError:
            pass
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(f"rank {rank}: no rendezvous file {path} after {timeout}s")
        time.sleep(0.02)


def cleanup_rendezvous(key: str | None = None):
    try:
        os.unlink(_rdzv_path(key))
    except FileNotFoundError:
        pass


def init_from_env(virtual_slabs: int = 1) -> Context:
    """Context for this process: its LOCAL_RANK's GPU, joined to the node-wide RCCL
    communicator when WORLD_SIZE > 1.

    Test rehearsal knobs (single-GPU machine): HH_TRANSPORT=shm selects the host-staged
    shared-memory transport, HH_FORCE_DEVICE=0 puts every rank on device 0, and
    HH_RCCL_HOSTID_PER_RANK=1 lets RCCL itself run with every rank on that one device.
    """
    rank, world, local = env_rank_world()
    device = int(os.environ.get("HH_FORCE_DEVICE", local if "LOCAL_RANK" in os.environ else 0))
    transport = os.environ.get("HH_TRANSPORT", "rccl")
    if world > 1 and transport == "rccl" and os.environ.get("HH_RCCL_HOSTID_PER_RANK") == "1":
        # RCCL rehearsal with every rank on one GPU (HH_FORCE_DEVICE): RCCL refuses two ranks
        # on one device of one host, so each rank poses as its own host and the ranks talk
        # through RCCL's socket transport over loopback.  Set before the first RCCL call.
        os.environ["NCCL_HOSTID"] = f"hh-rank-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    if world == 1:
        return Context(device=device, virtual_slabs=virtual_slabs)
    make_id = unique_id if transport == "rccl" else (lambda: os.urandom(128))
    uid = exchange_unique_id(rank, world, make_id=make_id)
    ctx = Context(device=device, rank=rank, world=world, nccl_id=uid, virtual_slabs=virtual_slabs,
                  transport=transport)
    ctx.barrier()
    if rank == 0:
        cleanup_rendezvous()
    return ctx
