// Coefficients of the 9-point operator at one point, shared by the stencil
// kernels (stencil.hip) and the CSR export (assemble.hip) so that the exported matrix is the
// applied operator bit for bit.  See stencil.hip for the scheme.
#pragma once
#include "hh_complex.hpp"
#include "hh_internal.hpp"

namespace hh {

// Row factors R2 (this row), R2m / R2p (rows j-1 / j+1), BS, BN; column factors AW, AE, R1m /
// R1p (columns i-1 / i+1).  M is the unshifted mass ω² R1 R2 / c² at the centre, Mo the mass
// of the operator being applied (M, or M x mshift for A_beta).  The centre coefficient is
// not produced here (the callers form c M - alpha (W + E + S + N) themselves).
// Output order: the CSR column order SW, S, SE, W, E, NW, N, NE.
struct Coef9 {
  double2 sw, s, se, w, e, nw, n, ne;
};

__device__ __forceinline__ Coef9 stencil9_offdiag(double2 W, double2 E, double2 S, double2 N,
                                                  double2 AW, double2 AE, double2 BS, double2 BN,
                                                  double2 R1m, double2 R1p, double2 R2m,
                                                  double2 R2p, double2 Mo, const Stencil9W w) {
  const double2 md = cscale(Mo, w.d), me = cscale(Mo, w.e);
  const double2 Wm = cmul(AW, R2m), Em = cmul(AE, R2m);
  const double2 Wp = cmul(AW, R2p), Ep = cmul(AE, R2p);
  const double2 Sm = cmul(BS, R1m), Nm = cmul(BN, R1m);
  const double2 Sp = cmul(BS, R1p), Np = cmul(BN, R1p);
  Coef9 c;
  c.sw = cadd(cscale(cadd(Wm, Sm), w.g), me);
  c.se = cadd(cscale(cadd(Em, Sp), w.g), me);
  c.nw = cadd(cscale(cadd(Wp, Nm), w.g), me);
  c.ne = cadd(cscale(cadd(Ep, Np), w.g), me);
  c.s = cadd(csub(cscale(S, w.alpha), cscale(cadd(Wm, Em), w.g)), md);
  c.n = cadd(csub(cscale(N, w.alpha), cscale(cadd(Wp, Ep), w.g)), md);
  c.w = cadd(csub(cscale(W, w.alpha), cscale(cadd(Sm, Nm), w.g)), md);
  c.e = cadd(csub(cscale(E, w.alpha), cscale(cadd(Sp, Np), w.g)), md);
  return c;
}

// centre coefficient c M - alpha (W + E + S + N), sum4 = ((W + E) + S) + N
__device__ __forceinline__ double2 stencil9_diag(double2 M, double2 sum4, const Stencil9W w) {
  return csub(cscale(M, w.c), cscale(sum4, w.alpha));
}

}  // namespace hh
