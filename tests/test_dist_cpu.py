"""CPU tier, N > 1: the row-slab decomposition over torch.distributed gloo (world 2, 3, 4, 8).

* slab ownership (dist.slab_bounds == the C runtime's formula) tiles [0, n);
* the file rendezvous hands rank 0's 128-byte id to every rank;
* a numpy restatement of the distributed algorithm (tests/dist_mirror.py: halo exchange +
  allreduced inner products + scipy's control flow) reproduces the single-process
  reference solve (scipy gmres on the oracle CSR, golden-pinned) to 1e-10.
"""
import multiprocessing as mp
import os
import socket
import tempfile

import numpy as np
import pytest

from conftest import ROOT, load_golden, medium
from helmholtz_preconditioner_amd import dist as hdist
from oracle import helmholtz_oracle as O


def test_slab_bounds_tile_the_grid():
    for n in (1, 7, 100, 4096, 11584):
        for world in range(1, 9):
            if world > n:
                continue
            b = [hdist.slab_bounds(n, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(x[1] == y[0] for x, y in zip(b, b[1:]))
            sizes = [e - s for s, e in b]
            assert max(sizes) - min(sizes) <= 1 and min(sizes) >= 1


def _rdzv_worker(rank, world, key, q):
    uid = hdist.exchange_unique_id(rank, world, key=key, make_id=lambda: bytes(range(128)),
                                   timeout=60)
    q.put((rank, uid))


def test_file_rendezvous_two_processes():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    key = f"test_{os.getpid()}_{np.random.default_rng().integers(1 << 30)}"
    ps = [ctx.Process(target=_rdzv_worker, args=(r, 3, key, q)) for r in (1, 2, 0)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    hdist.cleanup_rendezvous(key)
    assert all(v == bytes(range(128)) for v in got.values()) and len(got) == 3


def _gloo_worker(rank, world, port, case, out, lagged=False):
    """lagged: False (two allreduces per iteration), True (one), or "onepass" (the one-pass
    iteration's order: one halo exchange of u_K's edge rows and one allreduce per pass)"""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from oracle import helmholtz_oracle as O
    import dist_mirror as DM
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = np.load(os.path.join(ROOT, "tests", "golden", case), allow_pickle=False)
    n = int(z["n"])
    j0, j1 = hdist.slab_bounds(n, world, rank)
    om = complex(z["omega"])
    op = DM.SlabOperator(float(z["C"]), float(z["eta"]), om, float(z["h"]), n,
                         medium(str(z["medium"]), n), j0, j1,
                         jacobi=str(z["precond"]) == "jacobi")
    f = O.init_f1_mat(.5, .125, om, n)[j0:j1].ravel()
    halo_it = 1.0
    if lagged == "onepass":
        x, info, hist, per_it, halo_it = DM.gmres_dist_onepass(op, f, 1e-3, 20, int(z["K"]))
    elif lagged:
        x, info, hist, per_it = DM.gmres_dist_lagged(op, f, 1e-3, 20, int(z["K"]))
    else:
        x, info, hist = DM.gmres_dist(op, f, 1e-3, 20, int(z["K"]))
        per_it = 2.0
    np.savez(out, x=x, info=info, hist=hist, j0=j0, j1=j1, per_it=per_it, halo_it=halo_it)
    dist.destroy_process_group()


@pytest.mark.parametrize("case,world,lagged", [("gmres_n64_c1_none.npz", 2, False),
                                               ("gmres_n128_jacobi.npz", 3, False),
                                               ("gmres_n64_c1_none.npz", 2, True),
                                               ("gmres_n128_jacobi.npz", 3, True),
                                               ("gmres_n64_c1_none.npz", 2, "onepass"),
                                               ("gmres_n128_jacobi.npz", 3, "onepass"),
                                               ("gmres_n128_none.npz", 4, "onepass"),
                                               ("gmres_n128_none.npz", 8, "onepass"),
                                               ("gmres_n128_jacobi.npz", 8, True)])
def test_distributed_gmres_mirror_matches_reference(case, world, lagged):
    """lagged: the one-allreduce iteration (the runtime's lagged path across ranks) -- the
    golden histories to 1e-9, with ONE allreduce per inner iteration inside the restart cycles
    (plus one per cycle for the last column's norm).  "onepass": the one-pass iteration's order
    (runtime.cpp run_fused, the default across ranks from n = 1024) -- ONE allreduce and ONE halo
    exchange (u_K's edge rows) per pass."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as td:
        outs = [os.path.join(td, f"r{r}.npz") for r in range(world)]
        ps = [ctx.Process(target=_gloo_worker, args=(r, world, port, case, outs[r], lagged))
              for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(timeout=300)
            assert p.exitcode == 0
        parts = [np.load(o) for o in outs]
        z = load_golden(case)
        x = np.concatenate([p["x"] for p in parts])
        for p in parts:
            assert int(p["info"]) == int(z["info"]) and len(p["hist"]) == len(z["history"])
            assert np.max(np.abs(p["hist"] - z["history"]) / z["history"]) < 1e-9
            if lagged:  # one allreduce per inner iteration inside the cycles
                assert float(p["per_it"]) == 1.0
            if lagged == "onepass":  # and one halo exchange, of u_K's edge rows
                assert float(p["halo_it"]) == 1.0
        assert np.linalg.norm(x - z["x"]) / np.linalg.norm(z["x"]) < 1e-9


def _gloo_worker9(rank, world, port, out):
    import torch.distributed as dist
    import dist_mirror as DM
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 48
    om, h, eta = O.problem_params(n, 6, 4.0, 2.0)
    j0, j1 = hdist.slab_bounds(n, world, rank)
    op = DM.SlabOperator(81.0, eta, om, h, n, medium("c1", n), j0, j1, jacobi=True, stencil=9)
    xg = np.random.default_rng(3).standard_normal(n * n) + 0j
    y = op.apply(xg[j0 * n:j1 * n])
    f = O.init_f1_mat(.5, .125, om, n)[j0:j1].ravel()
    x, info, hist = DM.gmres_dist(op, f, 1e-3, 20, 60)
    np.savez(out, x=x, info=info, hist=hist, y=y)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_9pt_mirror_matches_single_domain(world):
    """SURVEY row F4 over the N > 1 path: the 9-point operator's slab apply (one-row halo) and
    Jacobi-GMRES over gloo against the single-domain oracle CSR and scipy gmres."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as td:
        outs = [os.path.join(td, f"r{r}.npz") for r in range(world)]
        ps = [ctx.Process(target=_gloo_worker9, args=(r, world, port, outs[r])) for r in range(world)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(timeout=300)
            assert p.exitcode == 0
        parts = [np.load(o) for o in outs]
    n = 48
    om, h, eta = O.problem_params(n, 6, 4.0, 2.0)
    R = O.build_A9_matrix(6, 81.0, eta, om, h, n, medium("c1", n))
    xg = np.random.default_rng(3).standard_normal(n * n) + 0j
    y = np.concatenate([p["y"] for p in parts])
    assert np.linalg.norm(y - R @ xg) <= 1e-14 * np.linalg.norm(R @ xg)
    f = O.init_f1_mat(.5, .125, om, n).ravel()
    xr, infor, histr, _ = O.gmres_reference(R, f, M=O.jacobi_preconditioner(R), rtol=1e-3,
                                            restart=20, maxiter=60)
    x = np.concatenate([p["x"] for p in parts])
    for p in parts:
        assert int(p["info"]) == infor and len(p["hist"]) == len(histr)
        assert np.max(np.abs(p["hist"] - histr) / histr) < 1e-9
    assert np.linalg.norm(x - xr) / np.linalg.norm(xr) < 1e-9
