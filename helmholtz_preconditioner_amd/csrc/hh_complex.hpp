// complex128 arithmetic on double2 (x = re, y = im) for gfx950 device code.
#pragma once
#include <hip/hip_runtime.h>

namespace hh {

__device__ __forceinline__ double2 cadd(double2 a, double2 b) {
  return make_double2(a.x + b.x, a.y + b.y);
}
__device__ __forceinline__ double2 csub(double2 a, double2 b) {
  return make_double2(a.x - b.x, a.y - b.y);
}
__device__ __forceinline__ double2 cneg(double2 a) { return make_double2(-a.x, -a.y); }
__device__ __forceinline__ double2 cscale(double2 a, double s) {
  return make_double2(a.x * s, a.y * s);
}
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
// a * b + c
__device__ __forceinline__ double2 cfma(double2 a, double2 b, double2 c) {
  return make_double2(fma(a.x, b.x, fma(-a.y, b.y, c.x)), fma(a.x, b.y, fma(a.y, b.x, c.y)));
}
// conj(a) * b + c
__device__ __forceinline__ double2 cfma_conj(double2 a, double2 b, double2 c) {
  return make_double2(fma(a.x, b.x, fma(a.y, b.y, c.x)), fma(a.x, b.y, fma(-a.y, b.x, c.y)));
}
__device__ __forceinline__ double cabs2(double2 a) { return fma(a.x, a.x, a.y * a.y); }
__device__ __forceinline__ double2 cconj(double2 a) { return make_double2(a.x, -a.y); }
// a / b for well-scaled stencil diagonals (|b| ~ 1e2 .. 1e10): one reciprocal.
__device__ __forceinline__ double2 cdiv(double2 a, double2 b) {
  const double inv = 1.0 / fma(b.x, b.x, b.y * b.y);
  return make_double2(fma(a.x, b.x, a.y * b.y) * inv, fma(a.y, b.x, -a.x * b.y) * inv);
}
// Smith's algorithm (the one numpy uses) for the small Hessenberg arithmetic.
__device__ __forceinline__ double2 cdiv_smith(double2 a, double2 b) {
  if (fabs(b.x) >= fabs(b.y)) {
    if (b.x == 0.0 && b.y == 0.0) return make_double2(a.x / 0.0, a.y / 0.0);
    const double rat = b.y / b.x;
    const double scl = 1.0 / (b.x + b.y * rat);
    return make_double2((a.x + a.y * rat) * scl, (a.y - a.x * rat) * scl);
  } else {
    const double rat = b.x / b.y;
    const double scl = 1.0 / (b.y + b.x * rat);
    return make_double2((a.x * rat + a.y) * scl, (a.y * rat - a.x) * scl);
  }
}

// cdiv_smith split in two: the divisor's factors (its two divisions, independent of the
// dividend: computed for every diagonal at once, off a back-substitution's serial chain) and
// their application (multiplies only).  smith_apply(a, smith_of(b)) is cdiv_smith(a, b).
struct Smith {
  double rat, scl;
  int mode;  // 0: |b.x| >= |b.y|, 1: |b.x| < |b.y|, 2: b == 0
};
__device__ __forceinline__ Smith smith_of(double2 b) {
  if (fabs(b.x) >= fabs(b.y)) {
    if (b.x == 0.0 && b.y == 0.0) return Smith{0.0, 0.0, 2};
    const double rat = b.y / b.x;
    return Smith{rat, 1.0 / (b.x + b.y * rat), 0};
  }
  const double rat = b.x / b.y;
  return Smith{rat, 1.0 / (b.y + b.x * rat), 1};
}
__device__ __forceinline__ double2 smith_apply(double2 a, Smith f) {
  if (f.mode == 0) return make_double2((a.x + a.y * f.rat) * f.scl, (a.y - a.x * f.rat) * f.scl);
  if (f.mode == 1) return make_double2((a.x * f.rat + a.y) * f.scl, (a.y * f.rat - a.x) * f.scl);
  return make_double2(a.x / 0.0, a.y / 0.0);
}


// A 16-byte write-through store (global_store_dwordx4 sc1): the line leaves the XCD's L2 at once
// instead of staying there dirty (plain and NT stores keep it, MI355X_MICROARCH.md's store
// table), so a streaming kernel's outputs do not push out the lines it re-reads -- the apply's
// halo rows, a pass's projection rows.  Vector store; the compiler does not count it in its
// vmcnt bookkeeping, which only makes its later waits conservative.
__device__ __forceinline__ void st_wt(double2* p, double2 v) {
  typedef double d2wt __attribute__((ext_vector_type(2)));
  const d2wt x = {v.x, v.y};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
}

}  // namespace hh
