"""GPU tier, N > 1: row-slab decomposition across processes.

The box has one GPU, so these tests run W processes on device 0, over the host-staged
shared-memory transport (csrc/comm.cpp ShmComm) and over the production RCCL transport
(RcclComm; one NCCL_HOSTID per rank, see rccl_rank_env) -- slab ownership, the halo
exchange, rank-ordered global reductions -- checked against the single-domain result on
the same GPU:
  * the operator apply: bit-identical slabs;
  * GMRES (none / Jacobi / shifted-Laplace): residual history and field to 1e-8 (the
    reductions sum partials in a different order; the contract is 1e-6);
  * both the reference's 5-point operator and the 9-point one.
It also rehearses `bench.py --gpus 2` end to end under torch.distributed.run.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import helmholtz_preconditioner_amd as H
from conftest import ROOT

pytestmark = pytest.mark.gpu
WORKER = os.path.join(ROOT, "tests", "dist_worker.py")


def rccl_rank_env(rank):
    """RCCL on one GPU: a distinct NCCL_HOSTID per rank makes every rank its own "host"
    (RCCL refuses two ranks on one device of one host), connected by RCCL's socket
    transport over loopback."""
    return dict(NCCL_HOSTID=f"hh-rank-{rank}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                HH_FORCE_DEVICE="0")


def wait_ranks(procs, timeout):
    """Wait for the rank processes (stdout piped): the first rank that fails ends the run at
    once -- its peers would otherwise wait for it in a collective until their own transport
    timeout -- and its output is reported."""
    import time
    t0 = time.monotonic()
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [r for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r = bad[0]
                for q in procs:
                    if q.poll() is None:
                        q.kill()
                out = procs[r].stdout.read().decode(errors="replace")
                raise AssertionError(f"rank {r} of {len(procs)} exited with {codes[r]}:\n"
                                     f"{out[-3000:]}")
            if all(c == 0 for c in codes):
                return
            if time.monotonic() - t0 > timeout:
                raise subprocess.TimeoutExpired("rank processes", timeout)
            time.sleep(0.05)
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()


def _run_workers(tmp_path, world, n, extra=(), transport="shm", timeout=240, env_extra=None):
    tok = os.urandom(128).hex()
    procs = []
    for r in range(world):
        out = tmp_path / f"r{r}.npz"
        env = dict(os.environ, **(rccl_rank_env(r) if transport == "rccl" else {}),
                   TMPDIR=str(tmp_path), **(env_extra or {}))
        procs.append((subprocess.Popen([sys.executable, WORKER, "--rank", str(r), "--world",
                                        str(world), "--id", tok, "--out", str(out), "--n", str(n),
                                        "--transport", transport] + list(extra),
                                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env),
                      out))
    wait_ranks([p for p, _ in procs], timeout)
    return [np.load(o) for _, o in procs]


def _single_domain(n, stencil=5, default_limits=False, krylov="one"):
    ctx = H.Context(device=0)
    om, h, eta = H.problem_params(n, 12, 6.0, 2.0)
    A = H.build_A_matrix(12, 81.0, eta, om, h, n, H.init_c1_mat(.5, .5, n), context=ctx,
                         stencil=stencil)
    # like with like: the ranks' mode ("one": the lagged iteration, their default below n = 1024;
    # "fused": the one-pass iteration)
    A.krylov_mode(krylov)
    rng = np.random.default_rng(5)
    xg = rng.standard_normal(n * n) + 1j * rng.standard_normal(n * n)
    res = dict(y=A @ xg)
    M = H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7)
    M.configure()
    res["ysl"] = A._apply_host(xg, H._ffi.HH_APPLY_PREC_A)
    f = H.init_f1_mat(.5, .125, om, n).ravel()
    for name, M in (("none", None), ("jacobi", "jacobi"),
                    ("sl", H.ShiftedLaplace(A, beta=0.5, sweeps=2, damping=0.7))):
        x, info, hist = H.gmres(A, f, rtol=1e-3, restart=20, maxiter=50, M=M,
                                callback=lambda r: None, callback_type="legacy",
                                return_history=True)
        res[f"x_{name}"], res[f"info_{name}"], res[f"hist_{name}"] = x, info, hist
        res[f"path_{name}"] = A.last_solve_path()
    if default_limits:
        res["x_default"], res["info_default"] = H.gmres(A, f, rtol=1e-3, M="jacobi")
    return res


@pytest.mark.parametrize("world,slabs,stencil", [(2, 1, 5), (3, 1, 5), (2, 2, 5), (4, 1, 5),
                                                (3, 2, 5), (3, 1, 9), (2, 2, 9)])
def test_multiprocess_slabs_match_single_domain(tmp_path, world, slabs, stencil):
    _check_against_single_domain(
        _run_workers(tmp_path, world, 150, ["--slabs", str(slabs), "--stencil", str(stencil)]),
        _single_domain(150, stencil), world, 150)


def _check_against_single_domain(parts, ref, world, n, tol=1e-8):
    assert parts[0]["j0"] == 0 and parts[-1]["j1"] == n
    for a, b in zip(parts, parts[1:]):
        assert a["j1"] == b["j0"]
    y = np.concatenate([p["y"] for p in parts])
    np.testing.assert_array_equal(y, ref["y"])
    ysl = np.concatenate([p["ysl"] for p in parts])
    np.testing.assert_array_equal(ysl, ref["ysl"])  # fused M A across ranks
    errs = []
    for name in ("none", "jacobi", "sl"):
        x = np.concatenate([p[f"x_{name}"] for p in parts])
        href = ref[f"hist_{name}"]
        for r, p in enumerate(parts):
            h = p[f"hist_{name}"]
            herr = (np.max(np.abs(h - href) / href) if len(h) == len(href) else np.inf)
            errs.append((name, r, int(p[f"info_{name}"]), int(ref[f"info_{name}"]), len(h),
                         len(href), float(herr)))
        xerr = np.linalg.norm(x - ref[f"x_{name}"]) / np.linalg.norm(ref[f"x_{name}"])
        errs.append((name, "x", 0, 0, 0, 0, float(xerr)))
    bad = [e for e in errs if e[2] != e[3] or e[4] != e[5] or not e[6] < tol]
    assert not bad, "\n".join(map(str, errs))
    assert all(float(p["maxrank"]) == world - 1 for p in parts)
    if "x_default" in ref:
        x = np.concatenate([p["x_default"] for p in parts])
        assert all(int(p["info_default"]) == int(ref["info_default"]) for p in parts)
        # (a converging run of hundreds of iterations: past the 1e-8 reproducibility horizon of
        # reordered reductions)
        assert np.linalg.norm(x - ref["x_default"]) <= 1e-6 * np.linalg.norm(ref["x_default"])


def test_uneven_slabs_default_limits(tmp_path):
    """n = 151 over 3 ranks (50 / 50 / 51 layers) with scipy's default restart and maxiter:
    the defaults come from the global N = n^2 on every rank (a rank-local N would give the
    ranks different maxiter and desynchronise their collectives)."""
    n = 151
    _check_against_single_domain(_run_workers(tmp_path, 3, n, ["--default-limits"]),
                                 _single_domain(n, default_limits=True), 3, n)


@pytest.mark.parametrize("world,slabs,transport", [(2, 1, "shm"), (3, 2, "shm"), (4, 1, "shm"),
                                                  (8, 1, "shm"), (8, 2, "shm"),
                                                  (2, 1, "rccl"), (3, 1, "rccl"),
                                                  (4, 2, "rccl"), (8, 1, "rccl")])
def test_fused_pass_ranks_match_single_domain(tmp_path, world, slabs, transport):
    """The one-pass iteration across ranks (runtime.cpp run_fused: u_K's edge rows formed
    first, exchanged on the halo stream while the interior rows run, the boundary rows behind
    the exchange; one allreduce per pass) for none / Jacobi / the two-sweep shifted Laplace
    (two edge rows), over both transports, with and without virtual slabs inside the ranks, up
    to the node's 8 ranks (n = 150: 18-19 rows a rank, 9-10 a virtual slab -- the shifted
    Laplace's two edge rows and the bands' four halo rows all inside a neighbour): every rank
    reports the one-pass path, and matches the single domain's one-pass solve to 1e-8."""
    n = 150
    parts = _run_workers(tmp_path, world, n, ["--slabs", str(slabs), "--krylov", "fused"],
                         transport=transport, timeout=240)
    ref = _single_domain(n, krylov="fused")
    for name in ("none", "jacobi", "sl"):
        assert ref[f"path_{name}"] == "one-pass"
        assert all(str(p[f"path_{name}"]) == "one-pass" for p in parts), name
    # 16 slabs (8 ranks x 2): the Jacobi field lands 1.2e-8 from the single domain after 50
    # iterations -- the summation order alone does that: the numpy mirror of this solve on 1 vs
    # 16 slabs differs by 1.7e-8 in the field, 1.2e-9 in the history, and scipy on f vs
    # f (1 + 1e-15) by 7.7e-6 (tools/slab_drift.py --n 150 --slabs 16 --restart 20 --iters 50,
    # profiles/r05/r05_slab_drift_cpu_150_16slabs_jacobi.log)
    _check_against_single_domain(parts, ref, world, n, tol=1e-7 if world * slabs >= 16 else 1e-8)


@pytest.mark.parametrize("world,transport", [(3, "shm"), (3, "rccl"), (8, "shm")])
def test_fused_pass_guarded_halo_buffers(tmp_path, world, transport):
    """The round-5 8-rank RCCL fault: the shifted-Laplace pass's boundary rows read
    u_K of row -3 -- one row BEFORE the received halo -- at halo_lo - n.  The value was never
    used, so every parity test passed; whether the read faulted depended on what the allocator
    had mapped there (it did at 11584^2 / 8 ranks under RCCL's layout, in every rank).  Here
    every halo receive buffer sits against an unmapped guard granule (HH_GUARD_HALO=1,
    runtime.cpp dalloc_guarded): a read one row beyond a received halo on either side faults
    at the smallest shape, on either transport.  The one-pass path (none / Jacobi / the
    two-sweep shifted Laplace), the fused M A and the apply then run clean and still match the
    single domain."""
    n = 150
    parts = _run_workers(tmp_path, world, n, ["--krylov", "fused"], transport=transport,
                         timeout=240, env_extra={"HH_GUARD_HALO": "1", "HH_CHECK_HALO": "1"})
    ref = _single_domain(n, krylov="fused")
    for name in ("none", "jacobi", "sl"):
        assert all(str(p[f"path_{name}"]) == "one-pass" for p in parts), name
    _check_against_single_domain(parts, ref, world, n)


@pytest.mark.parametrize("world", [2, 3])
def test_rccl_transport_ranks_match_single_domain(tmp_path, world):
    """The production RCCL transport (RcclComm) with world > 1: ncclCommInitRank across
    processes, the grouped halo send/recv on the highest-priority stream overlapped with the
    interior launch, and the in-solve allreduces -- apply and fused M A bit-identical to the
    single domain, GMRES (none / Jacobi / shifted-Laplace) to 1e-8.  All ranks share device 0
    (see rccl_rank_env)."""
    n = 150
    _check_against_single_domain(_run_workers(tmp_path, world, n, transport="rccl", timeout=180),
                                 _single_domain(n), world, n)


def _torchrun_bench(tmp_path, world, bench_args, env_extra, timeout=400):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HH_FORCE_DEVICE="0", TMPDIR=str(tmp_path), **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", str(world)] + bench_args
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)


BENCH_SMALL = ["--grid", "768", "--steps", "10", "--warmup", "2", "--gmres-iters", "6",
               "--no-cpu-baseline", "--same-n", "1024", "--same-n-steps", "10"]


@pytest.mark.parametrize("transport", ["shm", "rccl"])
def test_bench_two_ranks_rehearsal(tmp_path, transport):
    """`bench.py --gpus 2` end to end under torch.distributed.run (both ranks on device 0):
    one JSON line with the weak-scaling aggregate, the same-N strong-scaling block (the grid
    on 2 ranks and on rank 0 alone) and the transport actually used in `parallelism`."""
    extra = {"HH_TRANSPORT": transport}
    if transport == "rccl":  # RCCL's own per-rank env (NCCL_HOSTID ...) is per process here:
        extra["HH_RCCL_HOSTID_PER_RANK"] = "1"  # bench sets it from LOCAL_RANK
    out = _torchrun_bench(tmp_path, 2, BENCH_SMALL, extra)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["n"] == 768 and res["value"] > 0
    assert ("RCCL" if transport == "rccl" else "SHM") in res["config"]["parallelism"]
    assert res["gmres"]["iterations"] == 6
    assert res["spmv_constant_medium"]["value"] > 0
    assert res["spmv_constant_medium"]["bytes_per_unknown"] == 32
    sn = res["same_n"]
    assert sn["n"] == 1024 and sn["spmv"]["speedup_same_n"] > 0
    assert sn["spmv"]["single_gpu_value"] > 0 and 0 < sn["spmv"]["per_gpu_frac"] < 1
    assert sn["gmres"]["speedup_same_n"] > 0
    # where the time goes on N ranks: per-span HIP-event times, max over ranks, all >= 0
    bd = sn["breakdown"]
    sp, gi = bd["spmv_per_apply"], bd["gmres_per_iteration"]
    assert set(sp) == {"halo", "boundary", "interior", "halo_wait"}
    assert all(v >= 0 for v in sp.values()) and all(v >= 0 for v in gi.values())
    assert sp["interior"] > 0 and sp["halo"] > 0 and sp["boundary"] > 0
    for k in ("allreduce", "column", "multidot", "update", "interior", "halo"):
        assert gi[k] > 0, (k, gi)
    assert 1 <= gi["allreduces"] <= 3  # one per inner iteration (+ per-cycle extras)


@pytest.mark.parametrize("world,stall", [(2, 1), (3, 2)])
def test_bench_stalled_rank_exits_with_the_phase_named(tmp_path, world, stall):
    """A rank that stalls (simulated: HH_BENCH_STALL makes it hang when its first applies start)
    must end the job with a non-zero status, the stalled phase named and the STALLED rank named
    -- not the rank waiting for it.  Both enter the phase together under the same bound, so
    either watchdog may fire first (the waiting rank's did once, round 5); whichever fires reads
    every rank's published progress (collectives entered, bench.py Watchdog) and names the rank
    with the fewest."""
    import re
    out = _torchrun_bench(tmp_path, world, BENCH_SMALL,
                          {"HH_TRANSPORT": "shm", "HH_WATCHDOG_SCALE": "0.1",
                           "HH_BENCH_STALL": f"{stall}:first applies"}, timeout=180)
    assert out.returncode != 0
    assert re.search(r"\[bench watchdog\] rank \d: phase 'first applies", out.stderr), \
        out.stderr[-3000:]
    named = re.findall(r"\[bench watchdog\] stalled rank\(s\): ([0-9,]+|undetermined)",
                       out.stderr)
    assert named and all(n == str(stall) for n in named), out.stderr[-3000:]


@pytest.mark.parametrize("world", [2, 3])
def test_multiprocess_apply_large_grid(tmp_path, world):
    """n = 2100: every rank's interior rows take the non-marching tile kernel (the default
    standalone apply from n = 2048), the cross-rank halo rows the marching one; the slabs
    together are bit-identical to the single domain."""
    n = 2100
    ctx = H.Context(device=0)
    om, h, eta = H.problem_params(n, 12, 6.0, 2.0)
    A = H.build_A_matrix(12, 81.0, eta, om, h, n, H.init_c1_mat(.5, .5, n), context=ctx)
    rng = np.random.default_rng(5)
    yref = A @ (rng.standard_normal(n * n) + 1j * rng.standard_normal(n * n))
    parts = _run_workers(tmp_path, world, n, ["--apply-only"])
    np.testing.assert_array_equal(np.concatenate([p["y"] for p in parts]), yref)


def test_rccl_calls_in_one_process():
    """The RCCL calls the production transport makes (RcclComm), on this box's RCCL: a 1-rank
    communicator, an in-place allreduce and the grouped send/recv on the halo stream.  (Two
    ranks cannot share one GPU under RCCL; the N > 1 orchestration is covered above with the
    SHM transport.)"""
    import ctypes
    from helmholtz_preconditioner_amd import _ffi
    ea, ep = ctypes.c_double(-1.0), ctypes.c_double(-1.0)
    _ffi.check(_ffi.lib.hh_comm_selftest(0, ctypes.byref(ea), ctypes.byref(ep)))
    assert ea.value == 0.0 and ep.value == 0.0
