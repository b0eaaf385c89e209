"""Times one GMRES case repeatedly (for A/B of two library builds via HH_LIB_PATH).
usage: python tools/time_case.py [n] [restart] [maxiter] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import helmholtz_preconditioner_amd as H  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
restart = int(sys.argv[2]) if len(sys.argv) > 2 else 7
K = int(sys.argv[3]) if len(sys.argv) > 3 else 40
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 8
om, h, eta = H.problem_params(n, 12, max(3.0, n / 40.0), 2.0)
A = H.build_A_matrix(12, 81.0, eta, om, h, n, H.constant_c_mat(n))
f = H.init_f1_mat(.5, .125, om, n).ravel()
for r in range(reps):
    t0 = time.perf_counter()
    H.gmres(A, f, rtol=1e-12, restart=restart, maxiter=K, callback=lambda r: None,
            callback_type="legacy")
    dt = time.perf_counter() - t0
    print(f"{os.environ.get('HH_LIB_PATH', 'new')} n={n} restart={restart}: {K / dt:9.1f} it/s",
          flush=True)
