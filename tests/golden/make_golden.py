"""Generate the golden vectors in tests/golden/ from the REFERENCE itself.

Run in the build container only (the reference is not on the GPU box):
    python tests/golden/make_golden.py

It imports /root/reference/code.py (bocchs/helmholtz-preconditioner) with an
identity ``numba.jit`` stub (numba is not installed; SURVEY.md 8c recipe) and
records the outputs of the reference's own functions:

  inputs.npz          init_c1_mat / init_c2_mat / init_f1_mat / init_f2_mat (code.py:39-66)
  coef_<case>.npz     CSR of build_A_matrix (code.py:202-219)
  spmv_<case>.npz     y = A @ x, x = complex standard normal from default_rng(0)
  gmres_<case>.npz    scipy gmres(A, f, M, rtol=1e-3, restart=20, maxiter=K,
                      callback_type='legacy') on the reference A (code.py:516;
                      ``tol=`` -> ``rtol=`` because scipy >= 1.14 removed it)
  shift_n64.npz       build_A_matrix with c_mat / sqrt(1 + 0.5i)  (shifted Laplace operator)
  sweep_<case>.npz    the sweeping moving-PML preconditioner as the reference runs it:
                      algo2_3 + algo2_4 (code.py:345-385) applied to f and to a random x
                      (quirks Q1/Q2 included), two T_m = lu_Hm.solve([0..0, v])[-n:]
                      probes, the CSR of one H_m (get_Hm, code.py:283-290), and scipy gmres
                      with the reference's M (code.py:510-516)

Only data is committed (inputs and expected outputs); no reference source.
"""
import importlib.util
import os
import sys
import types

import numpy as np
import scipy
import scipy.sparse.linalg

HERE = os.path.dirname(os.path.abspath(__file__))
REF = '/root/reference/code.py'


def load_reference():
    os.environ.setdefault('MPLBACKEND', 'Agg')
    nb = types.ModuleType('numba')
    nb.jit = lambda *a, **k: (a[0] if a and callable(a[0]) and not k else (lambda f: f))
    sys.modules['numba'] = nb
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location('helm_ref', REF)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    return ref


def rand_complex(n_total, seed=0):
    rng = np.random.default_rng(seed)
    return rng.standard_normal(n_total) + 1j * rng.standard_normal(n_total)


def params(n, b, wn, alpha):
    omega = 2 * np.pi * wn + 1j * alpha
    h = 1 / (n + 1)
    return omega, h, b * h


def medium(ref, kind, n):
    if kind == 'c1':
        return ref.init_c1_mat(.5, .5, n)
    if kind == 'c2':
        return ref.init_c2_mat(n)
    if kind == 'const':
        return np.ones((n + 2, n + 2))
    raise ValueError(kind)


def csr_arrays(A):
    A = A.tocsr()
    A.sort_indices()
    return dict(data=A.data, indices=A.indices.astype(np.int32), indptr=A.indptr.astype(np.int64))


COEF_CASES = [  # name, n, medium, b, C, wave_num, alpha
    ('n16_c1', 16, 'c1', 6, 61.0, 4.0, 2.0),
    ('n33_c2', 33, 'c2', 12, 81.0, 8.0, 2.0),
    ('n64_const', 64, 'const', 12, 81.0, 8.0, 2.0),
    ('n64_c1', 64, 'c1', 12, 81.0, 8.0, 2.0),
]
SPMV_CASES = [
    ('n128_const', 128, 'const', 12, 81.0, 8.0, 2.0),
    ('n257_c1', 257, 'c1', 12, 81.0, 16.0, 2.0),
]
GMRES_CASES = [  # name, n, medium, b, C, wn, alpha, precond, K
    ('n128_none', 128, 'const', 12, 81.0, 8.0, 2.0, 'none', 200),
    ('n128_jacobi', 128, 'const', 12, 81.0, 8.0, 2.0, 'jacobi', 200),
    ('n64_c1_none', 64, 'c1', 12, 81.0, 4.0, 2.0, 'none', 120),
]


def main():
    ref = load_reference()
    meta = dict(scipy=scipy.__version__, numpy=np.__version__)
    print('reference loaded; scipy', meta['scipy'], 'numpy', meta['numpy'])

    omega = 2 * np.pi * 4 + 2j
    np.savez_compressed(os.path.join(HERE, 'inputs.npz'),
                        c1=ref.init_c1_mat(.5, .5, 20), c1_off=ref.init_c1_mat(.3, .6, 20),
                        c2=ref.init_c2_mat(20), f1=ref.init_f1_mat(.5, .125, omega, 20),
                        f2=ref.init_f2_mat(.125, .125, 1 / 2 ** .5, 1 / 2 ** .5, omega, 20),
                        omega=omega, n=20)

    for name, n, med, b, C, wn, al in COEF_CASES:
        om, h, eta = params(n, b, wn, al)
        A = ref.build_A_matrix(b, C, eta, om, h, n, medium(ref, med, n))
        np.savez_compressed(os.path.join(HERE, f'coef_{name}.npz'), n=n, b=b, C=C,
                            omega=om, h=h, eta=eta, medium=med, **csr_arrays(A))
        print('coef', name, A.nnz)

    for name, n, med, b, C, wn, al in SPMV_CASES:
        om, h, eta = params(n, b, wn, al)
        A = ref.build_A_matrix(b, C, eta, om, h, n, medium(ref, med, n)).tocsr()
        x = rand_complex(n * n, 0)
        y = A @ x
        np.savez_compressed(os.path.join(HERE, f'spmv_{name}.npz'), n=n, b=b, C=C, omega=om,
                            h=h, eta=eta, medium=med, y=y, x_head=x[:64],
                            x_sum=np.sum(x))
        print('spmv', name, np.linalg.norm(y))

    for name, n, med, b, C, wn, al, pc, K in GMRES_CASES:
        om, h, eta = params(n, b, wn, al)
        A = ref.build_A_matrix(b, C, eta, om, h, n, medium(ref, med, n)).tocsr()
        f = ref.init_f1_mat(.5, .125, om, n).flatten()
        M = None
        if pc == 'jacobi':
            dinv = 1.0 / A.diagonal()
            M = scipy.sparse.linalg.LinearOperator(A.shape, matvec=lambda v: dinv * np.ravel(v),
                                                   dtype=np.complex128)
        cnt = ref.gmres_counter(False)
        hist = []

        def cb(rk, cnt=cnt, hist=hist):
            cnt(rk)
            hist.append(float(rk))
        x, info = scipy.sparse.linalg.gmres(A, f, M=M, rtol=1e-3, restart=20, maxiter=K,
                                            callback=cb, callback_type='legacy')
        relres = np.linalg.norm(f - A @ x) / np.linalg.norm(f)
        np.savez_compressed(os.path.join(HERE, f'gmres_{name}.npz'), n=n, b=b, C=C, omega=om,
                            h=h, eta=eta, medium=med, precond=pc, K=K, x=x, info=info,
                            history=np.array(hist), niter=cnt.niter, relres=relres)
        print('gmres', name, 'iters', cnt.niter, 'info', info, 'relres', relres)

    n, b, C, wn, al = 64, 12, 81.0, 8.0, 2.0
    om, h, eta = params(n, b, wn, al)
    cm = ref.init_c1_mat(.5, .5, n) / np.sqrt(1 + 0.5j)
    A = ref.build_A_matrix(b, C, eta, om, h, n, cm)
    np.savez_compressed(os.path.join(HERE, 'shift_n64.npz'), n=n, b=b, C=C, omega=om, h=h,
                        eta=eta, beta=0.5, medium='c1', **csr_arrays(A))
    # F1: the sweeping moving-PML preconditioner (algo2_3 / algo2_4, code.py:345-385), as-is
    # (including quirks Q1/Q2), on the reference's own blocks (run_solver code.py:496-511)
    for name, n, med, b, C, wn, al in (('n48_c1', 48, 'c1', 12, 81.0, 4.0, 2.0),
                                       ('n37_c2', 37, 'c2', 6, 61.0, 3.0, 2.0)):
        om, h, eta = params(n, b, wn, al)
        cm = medium(ref, med, n)
        A = ref.build_A_matrix(b, C, eta, om, h, n, cm).tocsr()
        f = ref.init_f1_mat(.5, .125, om, n).flatten()
        lu_HF, lu_Hm_ra = ref.algo2_3(b, C, eta, om, h, n, cm)
        A_b1F = ref.get_A_b1F_block(b, C, eta, om, h, n, cm)
        A_Fb1 = ref.get_A_Fb1_block(b, C, eta, om, h, n, cm)
        up, lo = [], []
        for i in range(1, n):
            up.append(ref.get_A_block(i, i + 1, b, C, eta, om, h, n, cm))
            lo.append(ref.get_A_block(i + 1, i, b, C, eta, om, h, n, cm))
        u_f = ref.algo2_4(f, b, n, lu_HF, A_b1F, A_Fb1, up, lo, lu_Hm_ra)
        x = rand_complex(n * n, 3)
        u_x = ref.algo2_4(x, b, n, lu_HF, A_b1F, A_Fb1, up, lo, lu_Hm_ra)
        # T_m blocks for two m (1-based): last-layer block of Hm^-1 applied to unit-ish v
        v = rand_complex(n, 4)
        T = {}
        for m in (b + 1, n):
            tmp = np.zeros(b * n, complex)
            tmp[-n:] = v
            T[f'T_{m}'] = lu_Hm_ra[m - b - 1].solve(tmp)[-n:]
        Hm = ref.get_Hm(b + 3, b, C, eta, om, h, n, cm).tocsr()
        Hm.sort_indices()
        M = scipy.sparse.linalg.LinearOperator(A.shape, matvec=lambda xx: ref.algo2_4(
            f, b, n, lu_HF, A_b1F, A_Fb1, up, lo, lu_Hm_ra), dtype=np.complex128)
        hist = []
        xs, info = scipy.sparse.linalg.gmres(A, f, M=M, rtol=1e-3, callback=hist.append,
                                             callback_type='legacy')
        np.savez_compressed(os.path.join(HERE, f'sweep_{name}.npz'), n=n, b=b, C=C, omega=om,
                            h=h, eta=eta, medium=med, u_f=u_f.ravel(), u_x=u_x.ravel(), v=v,
                            Hm_m=b + 3, Hm_data=Hm.data, Hm_indices=Hm.indices.astype(np.int32),
                            Hm_indptr=Hm.indptr.astype(np.int64), gmres_hist=np.array(hist),
                            gmres_info=info, gmres_x=xs, **T)
        print('sweep', name, 'gmres callbacks', len(hist), 'info', info,
              'max|u|', np.abs(u_f).max())
    with open(os.path.join(HERE, 'VERSIONS.txt'), 'w') as fh:
        fh.write(f"generated from /root/reference/code.py with scipy {meta['scipy']} "
                 f"numpy {meta['numpy']} (numba absent: identity jit stub)\n")
    print('done')


if __name__ == '__main__':
    main()
