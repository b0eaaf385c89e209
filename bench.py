#!/usr/bin/env python3
"""Headline benchmark: complex stencil SpMV GB/s (% of HBM peak) + GMRES iters/s.

BASELINE.json metric: "complex stencil SpMV GB/s (% HBM peak) + GMRES iters/sec,
N=4096^2".  Workload at N=1 = BASELINE config 3: 4096 x 4096 Marmousi-like
heterogeneous velocity, wave_num 100 (>= 20.5 points per wavelength), b=12, C=81,
alpha=2, shifted-Laplace (beta=0.5) preconditioned GMRES(20).

A "step" is one operator apply (y = A x) over the whole grid, inputs resident in
HBM; the steps cycle through 3 distinct (x, y) pairs so that, as in a solve, every apply
reads an input no earlier launch left in the Infinity Cache.  value = algorithmic bytes of all steps on all ranks / wall time of the timed
region (max over ranks); algorithmic bytes = 40 B per unknown (read u 16 + write y
16 + read 1/c^2 8).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
one process per GPU, row-slab decomposition with RCCL halo exchange overlapped
with the interior stencil; weak scaling -- the grid grows to n = 4096 sqrt(N)
(rounded to 32) so every GPU keeps ~4096^2 unknowns.  The same job then also runs the
fixed BASELINE grid (4096^2, or 16384^2 under --config 5) on all N ranks and, on rank 0
alone, on one GPU: the `same_n` block carries the same-N speedup and per-GPU fraction of
HBM peak the north star grades (strong scaling).

Every rank runs a watchdog thread: each phase (communicator init, first halo exchange,
first allreduce, first GMRES cycle, ...) has a time bound, and a phase that overruns it
prints the phase and rank and ends the process with status 3 -- a stalled collective
becomes a diagnosable non-zero exit instead of a hang.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]


class Watchdog:
    """Per-rank phase timer: `phase(name, bound_s)` starts a phase; a
    daemon thread ends the process with status 3 (os._exit: no re-exec, no cleanup that could
    block on the stalled collective) when the current phase overruns its bound.  ctypes releases
    the GIL inside the native calls, so the thread runs while the main thread is blocked in RCCL
    or a stream synchronize.

    Naming the stalled rank: the rank that stops and the ranks that wait for
    it in its next collective enter the phase together and overrun its bound together, so the
    first watchdog to fire may well be a waiting one.  Every rank's thread therefore publishes,
    twice a second, its phase and the collectives it has entered (hh_ctx_progress: halo
    exchanges + allreduces, the same sequence on every rank) to a node-local file next to the
    rendezvous file; the watchdog that fires reads all of them and names the rank(s) with the
    fewest collectives entered -- the one(s) the others are waiting for -- or, with equal counts,
    the earliest phase; a rank with no state file never started.
    HH_WATCHDOG_SCALE multiplies every bound (tests shorten them); HH_BENCH_STALL=rank:phase
    makes that rank hang at the start of the phase whose name starts with `phase` (the
    stalled-rank rehearsal)."""

    def __init__(self, rank, world=1):
        from helmholtz_preconditioner_amd import dist
        self.rank, self.world = rank, world
        self.scale = float(os.environ.get("HH_WATCHDOG_SCALE", "1"))
        self.name, self.deadline, self.t0 = "startup", None, time.monotonic()
        self.seq = 0  # phases entered
        self.ctx = None
        self.lock = threading.Lock()
        self.paths = [dist.job_file("wd", f"_r{r}.json") for r in range(world)]
        stall = os.environ.get("HH_BENCH_STALL", "")
        self.stall = tuple(stall.split(":", 1)) if ":" in stall else None
        threading.Thread(target=self._run, daemon=True).start()

    def attach(self, ctx):
        """the context whose collectives count as this rank's progress"""
        self.ctx = ctx

    def phase(self, name, bound_s):
        with self.lock:
            self.name, self.t0 = name, time.monotonic()
            self.deadline = self.t0 + bound_s * self.scale
            self.seq += 1
        self._publish()
        if self.stall and int(self.stall[0]) == self.rank and name.startswith(self.stall[1]):
            while True:  # simulated stalled rank: only the watchdog ends it
                time.sleep(1)

    def done(self):
        with self.lock:
            self.name, self.deadline = "done", None
        try:
            os.unlink(self.paths[self.rank])
        except OSError:
            pass

    def _collectives(self):
        try:
            return self.ctx.collectives() if self.ctx is not None else -1
        except Exception:  # (a closed context)
            return -1

    def _publish(self):
        if self.world == 1:
            return
        with self.lock:
            st = {"rank": self.rank, "phase": self.name, "seq": self.seq,
                  "in_phase_s": round(time.monotonic() - self.t0, 1)}
        st["collectives"] = self._collectives()
        path = self.paths[self.rank]
        try:
            with open(path + ".tmp", "w") as fh:
                json.dump(st, fh)
            os.replace(path + ".tmp", path)
        except OSError:
            pass

    def stalled_ranks(self):
        """(stalled ranks, per-rank states) from the ranks' published states"""
        states = {}
        for r, path in enumerate(self.paths):
            try:
                with open(path) as fh:
                    states[r] = json.load(fh)
            except (OSError, ValueError):
                pass
        missing = [r for r in range(self.world) if r not in states]
        if missing:
            return missing, states
        calls = {r: s["collectives"] for r, s in states.items() if s["collectives"] >= 0}
        if calls and min(calls.values()) < max(calls.values()):
            lo = min(calls.values())
            return sorted(r for r, c in calls.items() if c == lo), states
        seqs = {r: s["seq"] for r, s in states.items()}
        if min(seqs.values()) < max(seqs.values()):
            lo = min(seqs.values())
            return sorted(r for r, q in seqs.items() if q == lo), states
        return [], states

    def _run(self):
        while True:
            time.sleep(0.5)
            self._publish()
            with self.lock:
                late = self.deadline is not None and time.monotonic() > self.deadline
                name, el = self.name, time.monotonic() - self.t0
            if late:
                msg = (f"[bench watchdog] rank {self.rank}: phase '{name}' stalled for {el:.0f} s "
                       f"(bound exceeded); exiting with status 3")
                if self.world > 1:
                    stalled, states = self.stalled_ranks()
                    rows = "; ".join(f"rank {r}: '{s['phase'][:40]}' {s['in_phase_s']} s, "
                                     f"{s['collectives']} collectives" for r, s in sorted(states.items()))
                    who = ",".join(map(str, stalled)) if stalled else "undetermined"
                    msg += f"\n[bench watchdog] stalled rank(s): {who} -- {rows}"
                print(msg, file=sys.stderr, flush=True)
                os._exit(3)


def parse():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200, help="timed operator applies")
    p.add_argument("--warmup", type=int, default=200,
                   help="untimed applies before each timed leg: the GPU's clocks ramp up over "
                        "the first ~tens of ms of load (4096^2: 121 us per apply after 20 "
                        "warm-up applies, 116 us after 200 or 1000, profiles/r01z3_warmup.log)")
    p.add_argument("--grid", type=int, default=0, help="global grid size n (default 4096*sqrt(N))")
    p.add_argument("--medium", default="marmousi", choices=["marmousi", "const", "c1"])
    p.add_argument("--wave-num", type=float, default=100.0)
    p.add_argument("--pml-b", dest="b", type=int, default=12)
    p.add_argument("--pml-C", dest="C", type=float, default=81.0)
    p.add_argument("--alpha", type=float, default=2.0)
    p.add_argument("--precond", default="sl", choices=["sl", "jacobi", "none"])
    p.add_argument("--sl-sweeps", type=int, default=2)
    p.add_argument("--variant", type=int, default=-1,
                   help="force a stencil kernel shape (hh_op_tune; -1 = the built-in choice)")
    p.add_argument("--stencil", type=int, default=5, choices=[5, 9],
                   help="5 = the reference's operator; 9 = the 9-point operator (SURVEY row F4)")
    p.add_argument("--gmres-iters", type=int, default=40, help="timed inner GMRES iterations")
    p.add_argument("--restart", type=int, default=20)
    p.add_argument("--krylov", default="auto", choices=["auto", "two", "one", "fused"],
                   help="GMRES inner-iteration form (hh_op_set_krylov_mode; A/B studies)")
    p.add_argument("--no-gmres", action="store_true")
    p.add_argument("--const-steps", type=int, default=200,
                   help="timed applies of the same grid with a constant medium (reported as "
                        "spmv_constant_medium; 0 = skip; not run when --medium const)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-gmres-iters", type=int, default=0,
                   help="inner iterations of the CPU GMRES baseline (0 = one restart cycle, "
                        "BASELINE.md 2: --restart iterations)")
    p.add_argument("--virtual-slabs", type=int, default=1)
    p.add_argument("--rotate", type=int, default=3,
                   help="distinct (x, y) vector pairs the timed applies cycle through: like the "
                        "applies of a solve, none re-reads lines an earlier one left in the "
                        "256 MiB Infinity Cache (1 = the same x every step)")
    p.add_argument("--same-n", type=int, default=-1,
                   help="N > 1: also time this fixed grid on all ranks and on one GPU (rank 0) "
                        "for the same-N speedup (-1 = 4096, or 16384 under --config 5; 0 = skip)")
    p.add_argument("--same-n-steps", type=int, default=100)
    p.add_argument("--config", type=int, default=0, choices=[0, 1, 2, 3, 4, 5],
                   help="BASELINE.json config preset (fixed grid => strong scaling); "
                        "0 = config 3 workload with weak scaling (default)")
    a = p.parse_args()
    if a.config:  # SURVEY.md 8d concrete inputs
        grid, medium, wn, pc, its = {1: (128, "const", 8.0, "none", 200),
                                     2: (1024, "const", 64.0, "jacobi", 100),
                                     3: (4096, "marmousi", 100.0, "sl", 20),
                                     4: (8192, "const", 256.0, "jacobi", 20),
                                     5: (16384, "const", 800.0, "jacobi", 20)}[a.config]
        a.grid, a.medium, a.wave_num, a.precond = a.grid or grid, medium, wn, pc
        if a.gmres_iters == 40:
            a.gmres_iters = its
    return a


def relaunch_distributed(args):
    """`python bench.py --gpus N` without a launcher: start torch.distributed.run as a
    child (nothing here has touched the GPU) and exit with its status."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def local_f1(omega, n, j0, j1, r1=.5, r2=.125):
    """rows [j0, j1) of init_f1_mat(r1, r2, omega, n) (code.py:53-58), flattened."""
    import helmholtz_preconditioner_amd as H
    return H.init_f1_rows(r1, r2, omega, n, j0, j1).ravel()


TRAFFIC_DB = "profiles/r05_pmc_traffic.json"
TRAFFIC_DB_R03 = "profiles/r03_pmc_traffic.json"


def measured_traffic(n, medium, rows, stencil=5):
    """HBM traffic of the apply kernel per launch, as a ratio to its algorithmic bytes, from the
    rocprofv3 PMC passes committed under profiles/ (FETCH_SIZE x2 + WRITE_SIZE in separate
    passes, the gfx950 correction of MI355X_MICROARCH.md; tools/pmc_traffic.py --merge) for this
    grid width, slab height (`rows`: the whole grid on one rank, a rank's slab at N > 1 --
    measured on one GPU as a virtual slab of the same shape), medium and stencil.  PMC counters
    cannot be read inside the timed run, so this is the committed measurement of the same kernel
    and workload: (ratio, source), or Nones for a shape without a record."""
    kind = "const" if medium == "const" else medium
    import helmholtz_preconditioner_amd as H
    if "HH_TILE_XCD" in H.knobs():
        return None, None  # (the records are of the default tile order)
    for db, key in ((TRAFFIC_DB, f"n{n}_rows{rows}_{kind}_s{stencil}"),
                    (TRAFFIC_DB_R03, f"n{n}_{kind}_s{stencil}" if rows == n else None)):
        path = os.path.join(ROOT, db)
        rec = json.load(open(path)).get(key) if key and os.path.exists(path) else None
        if rec:
            return (round(rec["ratio"], 4),
                    f"{db}[{key}]: FETCH_SIZE x2 + WRITE_SIZE per launch of "
                    f"{rec['kernel'][:60]}..., same grid width / slab rows / medium / stencil")
    return None, None


def make_medium(kind, n, cols):
    import helmholtz_preconditioner_amd as H
    if kind == "marmousi":
        return H.marmousi_like_c_mat(n, cols=cols)
    if kind == "const":
        return H.constant_c_mat(n)
    return H.init_c1_mat(.5, .5, n)


def cpu_baseline(args, n, omega, h, eta, c_mat):
    """Reference CPU path on this host (rank 0, N=1): the oracle's CSR (identical to
    build_A_matrix, pinned by tests/golden) with scipy csr_matvec (single-threaded) and
    scipy gmres with the same preconditioner (OpenBLAS threads)."""
    import numpy as np
    from oracle import helmholtz_oracle as O
    t0 = time.perf_counter()
    if args.stencil == 9:
        A = O.build_A9_matrix(args.b, args.C, eta, omega, h, n, c_mat)
    else:
        A = O.build_A_matrix(args.b, args.C, eta, omega, h, n, c_mat)
    t_build = time.perf_counter() - t0
    rng = np.random.default_rng(0)
    x = rng.standard_normal(n * n) + 1j * rng.standard_normal(n * n)
    A @ x
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        A @ x
    t_spmv = (time.perf_counter() - t0) / reps
    bpp = 32 if args.medium == "const" else 40
    out = {"value": round(bpp * n * n / t_spmv / 1e9, 3), "unit": "GB/s", "cores": 1,
           "kind": "port",
           "sample": f"{reps} scipy csr_matvec applies of the identical {n}x{n} operator "
                     f"(oracle CSR, {A.nnz} nnz), {t_spmv * 1e3:.1f} ms each; CSR build "
                     f"{t_build:.1f} s untimed"}
    if not args.no_gmres and args.cpu_gmres_iters >= 0:
        if args.precond == "sl" and args.stencil == 9:
            import scipy.sparse.linalg
            Ab = O.build_A9_matrix(args.b, args.C, eta, omega, h, n, c_mat / np.sqrt(1 + 0.5j))
            dinv = 1.0 / Ab.diagonal()

            def mv(r, sweeps=args.sl_sweeps):
                r = np.ravel(r)
                z = 0.7 * dinv * r
                for _ in range(sweeps - 1):
                    z = z + 0.7 * dinv * (r - Ab @ z)
                return z
            M = scipy.sparse.linalg.LinearOperator(A.shape, matvec=mv, dtype=np.complex128)
        elif args.precond == "sl":
            M, _ = O.shifted_laplace_jacobi(args.b, args.C, eta, omega, h, n, c_mat, beta=0.5,
                                            sweeps=args.sl_sweeps, damping=0.7)
        elif args.precond == "jacobi":
            M = O.jacobi_preconditioner(A)
        else:
            M = None
        f = local_f1(omega, n, 0, n)
        its = args.cpu_gmres_iters or args.restart
        # OpenBLAS (scipy's level-1 BLAS in gmres) on the CPUs this process may use
        ncpu = host_cpu_share()
        try:
            from threadpoolctl import threadpool_info, threadpool_limits
            lim = threadpool_limits(limits=ncpu, user_api="blas")
            thr = ",".join(f"{d.get('internal_api')}={d.get('num_threads')}"
                           for d in threadpool_info() if d.get("user_api") == "blas") or str(ncpu)
        except ImportError:
            lim, thr = None, os.environ.get("OPENBLAS_NUM_THREADS", "default")
        t0 = time.perf_counter()
        O.gmres_reference(A, f, M=M, rtol=1e-14, restart=args.restart, maxiter=its)
        t_g = time.perf_counter() - t0
        if lim is not None:
            lim.restore_original_limits()
        out["gmres_iters_per_s"] = round(its / t_g, 4)
        cyc = " (one restart cycle)" if its == args.restart else ""
        out["gmres_sample"] = (f"{its} scipy gmres inner iterations{cyc}, GMRES({args.restart}), "
                               f"{args.precond} preconditioner, {t_g:.1f} s; OpenBLAS threads="
                               f"{thr} (the CPUs this process may use: {ncpu})")
        out["gmres_threads"] = ncpu
    out["host"] = host_description()
    return out


def host_cpu_share():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota (a GPU box's
    share of a larger host: os.cpu_count() shows every CPU of the machine)."""
    n = len(os.sched_getaffinity(0))
    try:  # cgroup v2, then v1
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
    except (OSError, ValueError):
        try:
            quota = open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read().strip()
            period = open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read().strip()
        except OSError:
            quota, period = "max", "1"
    if quota not in ("max", "-1"):
        n = min(n, max(1, int(int(quota) / int(period))))
    return n


def host_description():
    """CPU model and logical CPUs of the host the CPU baseline ran on."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return f"{model}, {os.cpu_count()} logical CPUs (process affinity: " \
           f"{len(os.sched_getaffinity(0))}, CPU share incl. cgroup quota: {host_cpu_share()})"


def timed_applies(A, ctx, R, steps, warmup):
    """`steps` timed applies over R rotating (x, y) pairs after `warmup` untimed ones:
    (wall s of the timed region, max over ranks; device ms; average interior-kernel ms)."""
    x, y = [A.vector() for _ in range(R)], [A.vector() for _ in range(R)]
    for k, v in enumerate(x):
        v.fill_hash(2024 + k)
    if warmup > 0:
        A.time_apply(x, y, warmup)
    ctx.barrier()
    t0 = time.perf_counter()
    dev_ms, kern_ms = A.time_apply(x, y, steps)
    ctx.barrier()
    elapsed = float(ctx.allreduce_max([time.perf_counter() - t0])[0])
    for v in x + y:
        v.close()
    return elapsed, dev_ms, kern_ms


def make_precond(H, A, kind, sweeps):
    if kind == "sl":
        return H.ShiftedLaplace(A, beta=0.5, sweeps=sweeps, damping=0.7)
    return H.Jacobi(A) if kind == "jacobi" else None


def timed_gmres(H, A, ctx, f_host, args, iters, wd=None):
    """Warm-up (full restart cycles, at least 0.1 s of them: first allreduces, and enough load
    that the clocks have ramped), then `iters` timed legacy-counted inner iterations:
    (iterations, wall s max over ranks, history)."""
    f = A.vector(f_host)
    M = make_precond(H, A, args.precond, args.sl_sweeps)
    if wd:
        wd.phase("gmres warm-up (first restart cycle, first in-solve allreduces)", 180)
    # one full restart cycle, repeated until >= 0.1 s of warm-up (a cycle of a small grid is ~1
    # ms: the clocks would still be ramping in the timed solve -- config 2's first run read 10 %
    # low, profiles/r05/r05x_spread_c2_5runs.log); the repeat count from the slowest rank, so
    # every rank runs the same collectives
    def warm():
        t = time.perf_counter()
        H.gmres(A, f, rtol=1e-14, restart=args.restart, maxiter=max(2, args.restart), M=M,
                callback=lambda r: None, callback_type="legacy")
        ctx.barrier()
        return float(ctx.allreduce_max([time.perf_counter() - t])[0])
    dt = warm()
    for _ in range(min(20, max(0, int(0.1 / max(dt, 1e-6))))):
        warm()
    if wd:
        wd.phase("timed gmres", 120 + 0.5 * iters)
    t0 = time.perf_counter()
    xs, info, hist = H.gmres(A, f, rtol=1e-14, restart=args.restart, maxiter=iters,
                             M=M, callback=lambda r: None, callback_type="legacy",
                             return_history=True)
    ctx.barrier()
    tg = float(ctx.allreduce_max([time.perf_counter() - t0])[0])
    f.close()
    xs.close()
    return len(hist), tg, hist


def gmres_bytes(args, its, bpp, N):
    """algorithmic bytes of `its` GMRES inner iterations (CGS, lazy normalisation): SpMV 40N +
    projection 16(j+2)N + update 16(j+3)N (SURVEY 8d style), + the preconditioner's own
    traffic: none for Jacobi (fused into the SpMV) and for the two-sweep shifted-Laplace M
    (M A in one launch, csrc/sl_fused.hip: 40 B/unknown in all); otherwise the stencil + sweep
    launches, 16 + 56 B per further sweep."""
    js = [i % args.restart for i in range(its)]
    fused = args.sl_sweeps == 2
    sl_extra = 0 if fused else bpp + 16 + 56 * (args.sl_sweeps - 1)
    pre = {"sl": sl_extra, "jacobi": 0, "none": 0}[args.precond]
    return sum((bpp + pre) * N + 16 * (j + 2) * N + 16 * (j + 3) * N for j in js), fused


FUSED_TRAFFIC_DB = "profiles/r05_pmc_fused.json"
# the environment knobs that change the one-pass kernels' traffic: a record applies only to a run
# with the same values (unset = the build's default)
FUSED_KNOBS = ("HH_FUSED_ITER", "HH_FUSED_KEEP", "HH_FUSED_ROWS", "HH_BASIS_PAD", "HH_SLK",
               "HH_SLV", "HH_SLK_ROWS", "HH_CYCLE_MERGE", "HH_FUSED_ALT")
SL_ONLY_KNOBS = ("HH_SLK", "HH_SLV", "HH_SLK_ROWS")


def fused_knobs(rec_knobs=None, precond="sl"):
    """FUSED_KNOBS with their effective values (the library's reading, hh_knobs_json): this
    run's, or -- rec_knobs given -- a record's (knobs it does not name at their default); the
    shifted-Laplace-only knobs are dropped for the other preconditioners"""
    import helmholtz_preconditioner_amd as H
    allk = H.knobs(only_changed=False)
    if rec_knobs is None:
        eff = {k: str(allk[k]["value"]) for k in FUSED_KNOBS}
    else:
        eff = {k: str(rec_knobs.get(k, allk[k]["default"])) for k in FUSED_KNOBS}
    return {k: v for k, v in eff.items() if precond == "sl" or k not in SL_ONLY_KNOBS}


def fused_pass_traffic(n, rows, medium, precond, restart):
    """Measured HBM traffic of the one-pass iteration's pass kernels over a restart cycle, as a
    ratio to their algorithmic bytes (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes, separate
    runs; tools/pmc_fused.py --merge), for this grid width, slab height (a rank's slab at N > 1,
    recorded as a virtual slab on one GPU), medium, preconditioner and restart, recorded with
    the same kernel knobs (FUSED_KNOBS) as this run: (ratio, per-K ratios, source), or Nones for
    a workload without a record."""
    path = os.path.join(ROOT, FUSED_TRAFFIC_DB)
    if not os.path.exists(path):
        return None, None, None
    key = f"n{n}_rows{rows}_{medium}_{precond}_r{restart}"
    rec = json.load(open(path)).get(key)
    if not rec or fused_knobs(rec.get("knobs", {}), precond) != fused_knobs(None, precond):
        return None, None, None
    return rec["ratio"], rec["per_K"], f"{FUSED_TRAFFIC_DB}[{key}]: {rec['source']}"


def gmres_path_bytes(args, its, bpp, N, path):
    """algorithmic bytes of `its` inner iterations on the path the solve actually ran, per
    unknown: the one-pass iteration moves, at iteration j of a cycle, j = 0: the
    cycle's first M A (bpp) + its projection (u_0, w_0: 32 B); j >= 1: ONE pass, w_{j-1} and
    the j basis vectors read, u_j and w_j written -- 16 (j + 3) B, + 8 B of 1/c^2 for a
    non-constant medium (the operator's bpp is 32 + 8 then) --; the end of the cycle, in which
    the last update's norm and the x update share one pass (fused.hip cycle_end_kernel: R basis
    vectors, w and x read, x and V b written; then x += y V b), adds 16 (R + 4 + 3) B.  The
    regular and lagged cycles move the CGS bytes of gmres_bytes (the SpMV, then the basis
    twice; their x update is left out, as is every cycle's residual).  (PMC counters cannot run inside the timed solve: the pass's measured
    traffic per K is in profiles/r04_pmc_fused.json.)"""
    if path != "one-pass":
        return gmres_bytes(args, its, bpp, N)[0]
    R = args.restart
    ic = bpp - 32 if args.stencil == 5 else 0
    total = 0.0
    for i in range(its):
        j = i % R
        total += (bpp + 32) * N if j == 0 else (16 * (j + 3) + ic) * N
        if j == R - 1:
            total += 16 * (R + 7) * N
    return total


def span_breakdown(H, A, ctx, args, its, f_host, R, applies=20):
    """Where an N-rank apply / GMRES iteration spends its time, per rank (diagnostic, after
    the timed legs, so the timed numbers carry no event overhead): HIP events around the halo
    exchange, boundary and interior kernels, allreduces and Krylov kernels on the streams they
    run on (hh_op_read_timing), as microseconds per apply and per inner iteration, max over
    ranks (the slowest rank sets the pace of every collective)."""
    import numpy as np
    from helmholtz_preconditioner_amd import _ffi
    names = _ffi.SPAN_NAMES
    x, y = [A.vector() for _ in range(R)], [A.vector() for _ in range(R)]
    for k, v in enumerate(x):
        v.fill_hash(7 + k)
    A.set_timing(True)
    A.time_apply(x, y, applies)
    ap = A.read_timing()
    for v in x + y:
        v.close()
    out = {"source": "HIP events per span on each rank's own streams (hh_op_read_timing), one "
                     "extra untimed run after the timed legs; max over ranks",
           "unit": "us"}
    vec = [1e3 * ap[k][0] / applies for k in names]
    gm = None
    if not args.no_gmres and its > 0:
        f = A.vector(f_host)
        M = make_precond(H, A, args.precond, args.sl_sweeps)
        A.read_timing()
        _, _, hist = H.gmres(A, f, rtol=1e-14, restart=args.restart, maxiter=its, M=M,
                             callback=lambda r: None, callback_type="legacy",
                             return_history=True)
        gm = A.read_timing()
        f.close()
        k = max(1, len(hist))
        vec += [1e3 * gm[n][0] / k for n in names] + [gm["allreduce"][1] / k]
    A.set_timing(False)
    mx = ctx.allreduce_max(np.asarray(vec, dtype=np.float64))
    out["spmv_per_apply"] = {k: round(float(mx[i]), 3) for i, k in enumerate(names)
                             if k in ("halo", "boundary", "interior", "halo_wait")}
    if gm is not None:
        m = len(names)
        out["gmres_per_iteration"] = {k: round(float(mx[m + i]), 3) for i, k in enumerate(names)}
        out["gmres_per_iteration"]["allreduces"] = round(float(mx[2 * m]), 3)
    return out


def same_n_leg(H, dist, args, ctx, rank, world, wd):
    """Strong scaling at the fixed BASELINE grid in the same job: the grid on all `world`
    ranks, then on rank 0 alone with a world-1 context on its own GPU (the other ranks wait at
    a barrier).  Returns the `same_n` block (rank 0) -- speedups are 1-GPU time / N-GPU time
    of the same work."""
    import numpy as np
    n = args.same_n
    omega, h, eta = H.problem_params(n, args.b, args.wave_num, args.alpha)
    R = max(1, args.rotate)
    steps = args.same_n_steps
    its = min(args.gmres_iters, 20)

    def measure(c, r, w):
        j0, j1 = dist.slab_bounds(n, w, r)
        c_mat = make_medium(args.medium, n, (j0 - 2, j1 + 2))
        A = H.build_A_matrix(args.b, args.C, eta, omega, h, n, c_mat, context=c,
                             stencil=args.stencil)
        del c_mat
        el, _, kern = timed_applies(A, c, R, steps, min(args.warmup, 100))
        out = {"spmv_ms_per_step": el * 1e3 / steps, "kernel_ms": kern,
               "bytes_per_unknown": A.bytes_per_point}
        if not args.no_gmres and its > 0:
            k, tg, _ = timed_gmres(H, A, c, local_f1(omega, n, j0, j1), args, its)
            out["gmres_iters_per_s"] = k / tg
        if w > 1:
            wd.phase(f"same-N leg: span breakdown on {w} ranks", 300)
            out["breakdown"] = span_breakdown(H, A, c, args, its, local_f1(omega, n, j0, j1), R)
        A.close()
        return out

    wd.phase(f"same-N leg: {n}^2 on {world} ranks", 600)
    multi = measure(ctx, rank, world)
    single = None
    wd.phase(f"same-N leg: {n}^2 on rank 0's GPU alone (other ranks wait)", 900)
    if rank == 0:
        c1 = H.Context(device=ctx.device)
        single = measure(c1, 0, 1)
        c1.close()
    ctx.barrier()
    if rank != 0:
        return None
    bpp = multi["bytes_per_unknown"]
    agg = bpp * float(n) * n / (multi["spmv_ms_per_step"] * 1e-3) / 1e9
    one = bpp * float(n) * n / (single["spmv_ms_per_step"] * 1e-3) / 1e9
    block = {
        "n": n, "medium": args.medium, "steps": steps, "scaling": "strong",
        "spmv": {"value": round(agg, 2), "unit": "GB/s",
                 "ms_per_step": round(multi["spmv_ms_per_step"], 5),
                 "per_gpu_frac": round(agg / (HBM_PEAK_GBPS * world), 4),
                 "single_gpu_value": round(one, 2),
                 "single_gpu_ms_per_step": round(single["spmv_ms_per_step"], 5),
                 "speedup_same_n": round(single["spmv_ms_per_step"] / multi["spmv_ms_per_step"], 3)},
    }
    if "breakdown" in multi:
        block["breakdown"] = multi["breakdown"]
    if "gmres_iters_per_s" in multi:
        block["gmres"] = {"iterations": its, "precond": args.precond,
                          "iters_per_s": round(multi["gmres_iters_per_s"], 3),
                          "single_gpu_iters_per_s": round(single["gmres_iters_per_s"], 3),
                          "speedup_same_n": round(multi["gmres_iters_per_s"]
                                                  / single["gmres_iters_per_s"], 3)}
    return block


def main():
    args = parse()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world_env == 1:
        sys.exit(relaunch_distributed(args))

    import numpy as np
    import helmholtz_preconditioner_amd as H
    from helmholtz_preconditioner_amd import dist

    rank, world, _ = dist.env_rank_world()
    wd = Watchdog(rank, world)
    transport = os.environ.get("HH_TRANSPORT", "rccl") if world > 1 else "none"
    wd.phase("context + communicator init (ncclCommInitRank)", 240)
    ctx = dist.init_from_env(virtual_slabs=args.virtual_slabs)
    wd.attach(ctx)
    H.set_default_context(ctx)

    n = args.grid or int(round(4096 * math.sqrt(world) / 32) * 32)
    omega, h, eta = H.problem_params(n, args.b, args.wave_num, args.alpha)
    j0, j1 = dist.slab_bounds(n, world, rank)
    wd.phase("operator build", 300)
    t0 = time.perf_counter()
    # this rank's layers plus two on each side (the fused shifted-Laplace M A evaluates the
    # first sweep on the neighbouring ranks' boundary layers)
    c_mat = make_medium(args.medium, n, (j0 - 2, j1 + 2))
    A = H.build_A_matrix(args.b, args.C, eta, omega, h, n, c_mat, context=ctx,
                         stencil=args.stencil)
    t_init = time.perf_counter() - t0
    assert (A.row_begin, A.row_end) == (j0, j1)
    if args.variant >= 0:
        A.tune(args.variant)
    A.krylov_mode(args.krylov)
    bpp = A.bytes_per_point

    # ---------------- GMRES(restart): timed inner iterations ----------------
    # Run BEFORE the timed applies: the solve is the workload the apply serves, and its run
    # leaves the GPU at the clocks an apply inside a solve sees (from idle, the clocks ramp over
    # the first tens of ms of load: profiles/r01z3_warmup.log).  The timed region below is
    # still exactly `--warmup` untimed + `--steps` timed applies.
    gmres_block = None
    if not args.no_gmres and args.gmres_iters > 0:
        its, tg, hist = timed_gmres(H, A, ctx, local_f1(omega, n, j0, j1), args,
                                    args.gmres_iters, wd)
        gbytes, fused = gmres_bytes(args, its, bpp, float(n) * n)
        gmres_block = {
            "iters_per_s": round(its / tg, 3),
            "iterations": its,
            "restart": args.restart,
            "precond": {"sl": f"shifted-Laplace(beta=0.5, {args.sl_sweeps} damped-Jacobi sweeps"
                              f"{', fused with the SpMV' if fused else ''})",
                        "jacobi": "Jacobi", "none": "none"}[args.precond],
            "ms_per_iter": round(tg * 1e3 / its, 4),
            # the CGS-minimal bytes of SURVEY 8d (SpMV + the basis streamed twice) per second: a
            # CGS-equivalent credit for the work, NOT a bandwidth -- the one-pass path moves ~half
            # of these bytes, so on that path it can pass the HBM peak
            "cgs_equivalent_GBps": round(gbytes / tg / 1e9, 1),
            # the bytes the path it ran actually has to move (gmres_path_bytes) per second: the
            # rate to hold against the 8 TB/s peak (pass_frac_of_peak)
            "pass_GBps": round(gmres_path_bytes(args, its, bpp, float(n) * n,
                                                A.last_solve_path()) / tg / 1e9, 1),
            "final_rel_presid": float(hist[-1]) if its else None,
            # cycle form (hh_op_last_solve_path): "one-pass" = update + next M A + projections in
            # one pass over the basis (fused.hip fused_iter_kernel)
            "solve_path": A.last_solve_path(),
        }
        # pass_GBps counts the bytes of the whole n^2 grid (all ranks): the fraction is of the
        # peak of the `world` devices the ranks run on (one per rank; a one-GPU rehearsal of N
        # ranks shares one device, so its fraction reads N times low)
        gmres_block["pass_frac_of_peak"] = round(gmres_block["pass_GBps"] /
                                                 (HBM_PEAK_GBPS * world), 4)
        gmres_block["peak_devices"] = world
        if gmres_block["solve_path"] == "one-pass":
            # the passes' measured HBM traffic per algorithmic byte over a cycle (PMC counters
            # cannot run inside the timed solve: the committed record of the same workload)
            ratio, per_k, src = fused_pass_traffic(n, j1 - j0, args.medium, args.precond,
                                                   args.restart)
            gmres_block["pass_traffic_vs_algorithmic"] = ratio
            gmres_block["pass_traffic_source"] = src

    R = max(1, args.rotate)
    const_block = None
    # ---------------- the same apply on a constant medium (same grid and ranks) ----------------
    # The north star reports constant-k next to Marmousi-like grids at every GPU count: one
    # extra operator (no 1/c^2 stream: 32 B per unknown), timed exactly like the headline
    # applies -- and run before them, so that those start from the clocks of a running stream.
    if args.medium != "const" and args.const_steps > 0:
        wd.phase("constant-medium applies", 180 + 0.05 * (args.warmup + args.const_steps))
        Ac = H.build_A_matrix(args.b, args.C, eta, omega, h, n,
                              np.broadcast_to(1.0, (n + 2, n + 2)), context=ctx,
                              stencil=args.stencil)
        if args.variant >= 0:
            Ac.tune(args.variant)
        tc, _, _ = timed_applies(Ac, ctx, R, args.const_steps, args.warmup)
        vc = Ac.bytes_per_point * float(n) * n * args.const_steps / tc / 1e9
        const_block = {
            "value": round(vc, 2), "unit": "GB/s", "steps": args.const_steps,
            "ms_per_step": round(tc * 1e3 / args.const_steps, 5),
            "bytes_per_unknown": Ac.bytes_per_point,
            "pct_hbm_peak": round(100.0 * vc / (HBM_PEAK_GBPS * world), 2)}
        cr, _ = measured_traffic(n, "const", j1 - j0, args.stencil)
        const_block.update(traffic=None if cr is None else round(cr * Ac.bytes_per_point *
                                                                 (j1 - j0) * n),
                           traffic_vs_algorithmic=cr)
        Ac.close()
        del Ac

    # ---------------- SpMV: K timed steps, inputs resident in HBM ----------------
    # Step k maps x[k % R] -> y[k % R]: R pairs (R x 32 B/unknown, 1.6 GB at 4096^2 for R = 3)
    # are far above the Infinity Cache, so every step streams its input from HBM, as in a
    # solve.  (The same x every step lets part of it survive on the die between launches:
    # +13 % at 4096^2, profiles/r01l_*.)
    R = max(1, args.rotate)
    wd.phase("first applies (first halo exchange) + warm-up", 120 + 0.05 * args.warmup)
    x, y = [A.vector() for _ in range(R)], [A.vector() for _ in range(R)]
    for k, v in enumerate(x):
        v.fill_hash(2024 + k)
    if args.warmup > 0:
        A.time_apply(x, y, args.warmup)
    wd.phase("first host allreduce (barrier)", 60)
    ctx.barrier()
    wd.phase("timed applies", 120 + 0.05 * args.steps)
    t0 = time.perf_counter()
    dev_ms, kern_ms = A.time_apply(x, y, args.steps)
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = float(ctx.allreduce_max([elapsed])[0])
    value = bpp * float(n) * n * args.steps / elapsed / 1e9
    # roofline of the dominant kernel (the interior stencil launch on this rank)
    interior_rows = (j1 - j0) - (1 if (world > 1 and rank > 0) else 0) \
        - (1 if (world > 1 and rank < world - 1) else 0)
    achieved = bpp * float(interior_rows) * n / (kern_ms * 1e-3) / 1e9
    achieved_min = float(ctx.allreduce_max([-achieved])[0]) * -1.0
    medium_desc = {"marmousi": "Marmousi-like layered velocity (seeded generator)",
                   "const": "constant velocity c = 1", "c1": "init_c1_mat(.5, .5) velocity"}

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
        "higher_is_better": True,
        "scaling": "strong" if args.config and world > 1 else "weak",
        "vs_baseline": None,
        "dtype": "complex128",
        "data": f"synthetic: {medium_desc[args.medium]}, hash-filled complex input, "
                f"{R} rotating vector pairs",
        "config": {
            "workload": f"config{args.config or 3}: {n}x{n} {args.medium} velocity, matrix-free "
                        f"{args.stencil}-point PML stencil apply "
                        f"(+ GMRES({args.restart}) {args.precond}-preconditioned)",
            "n": n, "unknowns": n * n, "wave_num": args.wave_num, "b": args.b, "C": args.C,
            "alpha": args.alpha, "bytes_per_unknown": bpp, "stencil_points": args.stencil,
            # the library's HH_* knobs that differ from the shipped path ({} = the default path)
            "knobs": H.knobs(),
            "parallelism": (f"row-slab x{world} ({'RCCL' if transport == 'rccl' else 'host-staged SHM'}"
                            f" halo{', all ranks on one GPU' if os.environ.get('HH_FORCE_DEVICE') else ''})"
                            if world > 1 else "single GPU"),
        },
        "pct_hbm_peak": round(100.0 * value / (HBM_PEAK_GBPS * world), 2),
        "device_ms_per_step": round(dev_ms / args.steps, 5),
        "init_s": round(t_init, 3),
    }
    # (ratio measured per launch over the slab's rows; traffic = that ratio x this launch's bytes)
    traffic_ratio, traffic_src = measured_traffic(n, args.medium, j1 - j0, args.stencil)
    traffic = None if traffic_ratio is None else int(round(traffic_ratio * bpp * interior_rows * n))
    result["roofline"] = {
        "bound": "hbm",
        "achieved": round(achieved_min, 1),
        "peak": HBM_PEAK_GBPS,
        "unit": "GB/s",
        "frac": round(achieved_min / HBM_PEAK_GBPS, 4),
        "traffic": traffic,
        "traffic_vs_algorithmic": traffic_ratio,
        "traffic_source": traffic_src,
        "kernel": (f"tile_kernel<EPI_AX,{'true' if A.constant_medium else 'false'},"
                   f"{(8 if A.constant_medium else 6) if n > 4608 else (6 if A.constant_medium else 4)}"
                   " rows> "
                   "(interior rows)") if (args.stencil == 5 and n >= 2048 and args.variant < 0) else
                  (f"stencil_kernel<EPI_AX,{'true' if A.constant_medium else 'false'},"
                   f"S9={'true' if args.stencil == 9 else 'false'}> (interior rows)"),
        "kernel_ms": round(kern_ms, 5),
        "bytes_per_launch": bpp * interior_rows * n,
    }
    for v in x + y:
        v.close()
    del x, y
    if gmres_block is not None:
        result["gmres"] = gmres_block
    if const_block is not None:
        result["spmv_constant_medium"] = const_block

    A.close()

    # ---------------- same-N strong scaling (N > 1): the north star's speedup ----------------
    if world > 1:
        if args.same_n < 0:
            args.same_n = 16384 if args.config == 5 else 4096
        if args.same_n > 0:
            block = same_n_leg(H, dist, args, ctx, rank, world, wd)
            if rank == 0:
                result["same_n"] = block

    # ---------------- CPU baseline (rank 0, N=1) ----------------
    if world == 1 and not args.no_cpu_baseline and n <= 4096:
        wd.phase("cpu baseline", 900)
        # N=1: c_mat holds the full field (plus two layers beyond the grid on each side)
        result["cpu_baseline"] = cpu_baseline(args, n, omega, h, eta, c_mat)
    elif world > 1:
        result["cpu_baseline"] = None

    if rank == 0:
        print(json.dumps(result), flush=True)
    wd.phase("final barrier", 120)
    ctx.barrier()
    wd.done()


if __name__ == "__main__":
    main()
