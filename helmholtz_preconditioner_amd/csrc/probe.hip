// Streaming roofline probes (diagnostics only; not on any solve path).
// They move the stencil's byte mix -- 16 B of u and 8 B of 1/c^2 read, 16 B of y written per
// point -- in different access shapes, to establish what HBM rate this mix can reach on
// MI355X and which load/store shapes the stencil kernel should use.
#include "hh_internal.hpp"
#include "hh_complex.hpp"

namespace hh {
namespace {

constexpr int kT = 256;

// P0: one point per lane: u dwordx4, ic dwordx2, y dwordx4.
__global__ __launch_bounds__(kT) void p0(const double2* __restrict__ u, const double* __restrict__ ic,
                                         double2* __restrict__ y, size_t len) {
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t p = (size_t)blockIdx.x * kT + threadIdx.x; p < len; p += stride)
    y[p] = cscale(u[p], ic[p]);
}

// P1: two adjacent points per lane: ic as one dwordx4; u, y as two dwordx4 (32-B lane stride).
__global__ __launch_bounds__(kT) void p1(const double2* __restrict__ u, const double* __restrict__ ic,
                                         double2* __restrict__ y, size_t len) {
  const size_t stride = (size_t)gridDim.x * kT;
  const size_t half = len / 2;
  for (size_t q = (size_t)blockIdx.x * kT + threadIdx.x; q < half; q += stride) {
    const double2 c = reinterpret_cast<const double2*>(ic)[q];
    const double2 a = u[2 * q], b = u[2 * q + 1];
    y[2 * q] = cscale(a, c.x);
    y[2 * q + 1] = cscale(b, c.y);
  }
}

// P2: two points per lane, wave-strided (p, p+64): u, y contiguous dwordx4; ic 2x dwordx2.
__global__ __launch_bounds__(kT) void p2(const double2* __restrict__ u, const double* __restrict__ ic,
                                         double2* __restrict__ y, size_t len) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t chunk = 128;  // points per wave per iteration
  const size_t nwaves = (size_t)gridDim.x * (kT / 64);
  for (size_t c = (size_t)blockIdx.x * (kT / 64) + wave; c * chunk < len; c += nwaves) {
    const size_t p = c * chunk + lane;
    const double2 a = u[p], b = u[p + 64];
    const double ca = ic[p], cb = ic[p + 64];
    y[p] = cscale(a, ca);
    y[p + 64] = cscale(b, cb);
  }
}

// P3: pure copy y = u (32 B per point).
__global__ __launch_bounds__(kT) void p3(const double2* __restrict__ u, const double* __restrict__ ic,
                                         double2* __restrict__ y, size_t len) {
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t p = (size_t)blockIdx.x * kT + threadIdx.x; p < len; p += stride) y[p] = u[p];
}

// P4: read-only (u and ic), one store per block to keep it live (24 B per point).
__global__ __launch_bounds__(kT) void p4(const double2* __restrict__ u, const double* __restrict__ ic,
                                         double2* __restrict__ y, size_t len) {
  const size_t stride = (size_t)gridDim.x * kT;
  double2 acc = make_double2(0.0, 0.0);
  for (size_t p = (size_t)blockIdx.x * kT + threadIdx.x; p < len; p += stride)
    acc = cadd(acc, cscale(u[p], ic[p]));
  if (acc.x == 12345.678) y[0] = acc;  // practically never taken
}

// P5: P0 with non-temporal loads and stores.
__global__ __launch_bounds__(kT) void p5(const double2* __restrict__ u, const double* __restrict__ ic,
                                         double2* __restrict__ y, size_t len) {
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t p = (size_t)blockIdx.x * kT + threadIdx.x; p < len; p += stride) {
    const double ux = __builtin_nontemporal_load(&u[p].x);
    const double uy = __builtin_nontemporal_load(&u[p].y);
    const double c = __builtin_nontemporal_load(&ic[p]);
    __builtin_nontemporal_store(ux * c, &y[p].x);
    __builtin_nontemporal_store(uy * c, &y[p].y);
  }
}

// P6: P1 with the ic stream replaced by nothing (u, y only: 32 B per point, two per lane).
__global__ __launch_bounds__(kT) void p6(const double2* __restrict__ u, const double* __restrict__ ic,
                                         double2* __restrict__ y, size_t len) {
  const size_t stride = (size_t)gridDim.x * kT;
  const size_t half = len / 2;
  for (size_t q = (size_t)blockIdx.x * kT + threadIdx.x; q < half; q += stride) {
    const double2 a = u[2 * q], b = u[2 * q + 1];
    y[2 * q] = a;
    y[2 * q + 1] = b;
  }
}

}  // namespace

int launch_probe_kind(int kind, int blocks, const double2* u, const double* ic, double2* y,
                      size_t len, hipStream_t s) {
  dim3 g(blocks), b(kT);
  switch (kind) {
    case 0: hipLaunchKernelGGL(p0, g, b, 0, s, u, ic, y, len); return 40;
    case 1: hipLaunchKernelGGL(p1, g, b, 0, s, u, ic, y, len); return 40;
    case 2: hipLaunchKernelGGL(p2, g, b, 0, s, u, ic, y, len); return 40;
    case 3: hipLaunchKernelGGL(p3, g, b, 0, s, u, ic, y, len); return 32;
    case 4: hipLaunchKernelGGL(p4, g, b, 0, s, u, ic, y, len); return 24;
    case 5: hipLaunchKernelGGL(p5, g, b, 0, s, u, ic, y, len); return 40;
    case 6: hipLaunchKernelGGL(p6, g, b, 0, s, u, ic, y, len); return 32;
    default: return 0;
  }
}

}  // namespace hh
