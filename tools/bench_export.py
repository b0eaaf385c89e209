"""CSR export (row F2) timing: device assembly kernel vs the CPU assembly of the same CSR.

Algorithmic bytes per unknown of the export kernel: writes 5 entries x (16 B value + 4 B
int32 index) + 8 B row pointer, reads 8 B of 1/c^2 -> 116 B (nnz = 5n^2 - 4n; the edge
rows write fewer).  The D2H copy of the result is timed separately (PCIe-bound).
usage: python tools/bench_export.py [n ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import helmholtz_preconditioner_amd as H  # noqa: E402

ns = [int(v) for v in sys.argv[1:]] or [1024, 4096]
for n in ns:
    om, h, eta = H.problem_params(n, 12, 100.0, 2.0)
    cm = H.marmousi_like_c_mat(n)
    A = H.build_A_matrix(12, 81.0, eta, om, h, n, cm)
    A.to_csr()  # warm-up (allocations, first launch)
    best = 1e9
    t0 = time.perf_counter()
    for _ in range(3):
        M, ms = A.to_csr(return_kernel_ms=True)
        best = min(best, ms)
    wall = (time.perf_counter() - t0) / 3
    nnz = M.nnz
    alg = nnz * 20 + (n * n + 1) * 8 + n * n * 8
    line = (f"n={n}: nnz={nnz} export kernel {best:.3f} ms = {alg / best / 1e6:.0f} GB/s "
            f"algorithmic ({alg / 1e9:.2f} GB); to_csr wall incl. D2H {wall * 1e3:.0f} ms")
    if n <= 4096 and os.path.isdir(os.path.join(ROOT, "oracle")):
        from oracle import helmholtz_oracle as O
        t0 = time.perf_counter()
        R = O.build_A_matrix(12, 81.0, eta, om, h, n, cm).tocsr()
        cpu = time.perf_counter() - t0
        line += f" | CPU numpy/scipy assembly of the same CSR: {cpu:.2f} s"
        del R
    print(line, flush=True)
    del A, M
