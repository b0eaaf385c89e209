/*
 * stencil_oracle.c -- TEST INFRASTRUCTURE ONLY (the CPU checker; nothing in the product package
 * links or loads it; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may).
 *
 * A plain-C restatement of the reference's operator for grids too large to assemble as a
 * numpy/scipy CSR on the host (BASELINE configs 4 and 5: 8192^2 and 16384^2 unknowns, 7 and
 * 28 GB of CSR): y = A x row by row, exactly the five entries build_A_matrix stores per row
 * (code.py:202-219: S = c3 of the layer below, W = c1, D = c5, E = c2, N = c4 of the layer
 * above; the +-1 entries are absent at layer boundaries, the +-n ones at the grid edge), each
 * coefficient from the formulas of get_A_diag_block_coeffs / get_upper / get_lower_A_block
 * (code.py:70-115, 130-154) with the PML profiles sigma1 / sigma2 / s1 / s2 of code.py:11-33
 * (sigma2 one-sided: quirk Q4) and the velocity read as c_mat[i-1, j-1] (quirk Q3: the caller
 * passes cc[j-1][i-1] = c_mat[i-1, j-1], see oracle/stencil_oracle.py).
 *
 * The row sum runs in scipy csr_matvec's order (code.py:516 -> sparsetools csr_matvec: sum over
 * the row's entries in column order S, W, D, E, N, then y[p] = sum), with the complex products
 * written out as (ac - bd, ad + bc) and no FMA contraction (-ffp-contract=off).  The coefficients
 * are formed with C99 complex division where numpy uses its own division algorithm, so values
 * agree with oracle.helmholtz_oracle.build_A_matrix to rounding (pinned in tests/test_oracle.py
 * against that CSR and the golden CSR / SpMV vectors made from the reference itself).
 *
 * Threads: OpenMP over layers; every output is computed by one thread in a fixed order, so the
 * result does not depend on the thread count.
 */
#include <complex.h>
#include <math.h>
#include <stdlib.h>

typedef double complex cplx;

static double sigma1(double x, double C, double eta) {   /* code.py:11-18 */
  if (x <= eta) return C / eta * ((x - eta) / eta) * ((x - eta) / eta);
  if (x >= 1 - eta) return C / eta * ((x - 1 + eta) / eta) * ((x - 1 + eta) / eta);
  return 0.0;
}
static double sigma2(double x, double C, double eta) {   /* code.py:20-25 (Q4) */
  if (x <= eta) return C / eta * ((x - eta) / eta) * ((x - eta) / eta);
  return 0.0;
}
static cplx s1(double x, double C, double eta, cplx om) { /* code.py:27-29 */
  return 1.0 / (1.0 + I * sigma1(x, C, eta) / om);
}
static cplx s2(double x, double C, double eta, cplx om) { /* code.py:31-33 */
  return 1.0 / (1.0 + I * sigma2(x, C, eta) / om);
}

typedef struct {
  int n;
  cplx *s1m, *s1p, *s1c;  /* s1((i -+ .5) h), s1(i h), i = 1..n */
  cplx *s2m, *s2p, *s2c;  /* s2((j -+ .5) h), s2(j h), j = 1..n */
  cplx om2;               /* omega^2 * mass scale */
  double ih2;
} Tables;

static int tables_make(Tables* t, int n, double C, double eta, cplx om, cplx mscale, double h) {
  t->n = n;
  cplx* buf = (cplx*)malloc(6 * (size_t)n * sizeof(cplx));
  if (!buf) return -1;
  t->s1m = buf; t->s1p = buf + n; t->s1c = buf + 2 * (size_t)n;
  t->s2m = buf + 3 * (size_t)n; t->s2p = buf + 4 * (size_t)n; t->s2c = buf + 5 * (size_t)n;
  for (int k = 0; k < n; ++k) {
    const double v = k + 1;
    t->s1m[k] = s1((v - .5) * h, C, eta, om);
    t->s1p[k] = s1((v + .5) * h, C, eta, om);
    t->s1c[k] = s1(v * h, C, eta, om);
    t->s2m[k] = s2((v - .5) * h, C, eta, om);
    t->s2p[k] = s2((v + .5) * h, C, eta, om);
    t->s2c[k] = s2(v * h, C, eta, om);
  }
  t->om2 = om * om * mscale;
  t->ih2 = 1.0 / (h * h);
  return 0;
}

/* W, E, S, N, D at 0-based (i, j), velocity c there (code.py:83-109) */
static void coeffs(const Tables* t, int i, int j, double c, cplx* W, cplx* E, cplx* S, cplx* N,
                   cplx* D) {
  *W = t->ih2 * (t->s1m[i] / t->s2c[j]);
  *E = t->ih2 * (t->s1p[i] / t->s2c[j]);
  *S = t->ih2 * (t->s2m[j] / t->s1c[i]);
  *N = t->ih2 * (t->s2p[j] / t->s1c[i]);
  *D = t->om2 / (t->s1c[i] * t->s2c[j] * (c * c)) - (*W + *E + *S + *N);
}

static inline void acc(double* sr, double* si, cplx a, const double* x) {
  const double ar = creal(a), ai = cimag(a);
  *sr += ar * x[0] - ai * x[1];
  *si += ar * x[1] + ai * x[0];
}

/* mode 0: y = A x;  mode 1: y = diag(A) (x unused).
 * cc: n*n doubles [j][i] = c_mat[i-1, j-1] (quirk Q3), or NULL for the constant c_const.
 * x, y: interleaved complex, index p = j n + i (0-based; code.py:448 f_mat.flatten()). */
int hho_apply(int n, double C, double eta, double om_re, double om_im, double h,
              const double* cc, double c_const, double ms_re, double ms_im, const double* x,
              double* y, int mode) {
  if (n < 1 || !y || (mode == 0 && !x) || (!cc && !(c_const > 0))) return -1;
  Tables t;
  if (tables_make(&t, n, C, eta, om_re + I * om_im, ms_re + I * ms_im, h)) return -2;
  const size_t nn = (size_t)n;
#pragma omp parallel for schedule(static)
  for (int j = 0; j < n; ++j) {
    for (int i = 0; i < n; ++i) {
      const size_t p = (size_t)j * nn + i;
      cplx W, E, S, N, D;
      coeffs(&t, i, j, cc ? cc[p] : c_const, &W, &E, &S, &N, &D);
      if (mode == 1) {
        y[2 * p] = creal(D);
        y[2 * p + 1] = cimag(D);
        continue;
      }
      double sr = 0.0, si = 0.0;  /* csr_matvec: entries in column order */
      if (j > 0) acc(&sr, &si, S, x + 2 * (p - nn));
      if (i > 0) acc(&sr, &si, W, x + 2 * (p - 1));
      acc(&sr, &si, D, x + 2 * p);
      if (i < n - 1) acc(&sr, &si, E, x + 2 * (p + 1));
      if (j < n - 1) acc(&sr, &si, N, x + 2 * (p + nn));
      y[2 * p] = sr;
      y[2 * p + 1] = si;
    }
  }
  free(t.s1m);
  return 0;
}
