// Streaming roofline probes (diagnostics only; not on any solve path).
// They move the stencil's byte mix -- 16 B of u and 8 B of 1/c^2 read, 16 B of y written per
// point -- in different access shapes, to establish what HBM rate this mix can reach on
// MI355X and which load/store shapes the stencil kernel should use.
#include "hh_internal.hpp"
#include "hh_complex.hpp"

#include <cmath>

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

// P15 / P16: the copy y = u (32 B per point, the constant medium's byte mix) with NT loads and
// stores (P15) and with cached loads and NT stores (P16, the tile kernel's constant-medium form).
template <bool NTL>
__global__ __launch_bounds__(kT) void pcopy_nt(const double2* __restrict__ u,
                                               double2* __restrict__ y, size_t len) {
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t p = (size_t)blockIdx.x * kT + threadIdx.x; p < len; p += stride) {
    const double ux = NTL ? __builtin_nontemporal_load(&u[p].x) : u[p].x;
    const double uy = NTL ? __builtin_nontemporal_load(&u[p].y) : u[p].y;
    __builtin_nontemporal_store(ux, &y[p].x);
    __builtin_nontemporal_store(uy, &y[p].y);
  }
}

// P17 .. P21: the constant-medium tile kernel's access shape without its arithmetic (32 B per
// point): a 256-thread block owns a 256-wide x R-row tile (plain tile order), loads its R rows
// through the cache -- plus (HALO) the row above and below it, (EDGE) one broadcast load per row
// for the wave's W/E edge column, (TAB) three per-column table loads -- and stores R rows NT.
// Isolates what the tile shape itself costs against the streaming copy (P16).
template <int R, bool HALO, bool EDGE, bool TAB>
__global__ __launch_bounds__(kT) void ptile(const double2* __restrict__ u,
                                            double2* __restrict__ y, int n) {
  const int tiles_x = (n + kT - 1) / kT;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
  const int i = min(tx * kT + (int)threadIdx.x, n - 1), lane = threadIdx.x & 63;
  const int rb = ty * R, re = min(rb + R, n);
  if (rb >= n) return;
  double2 U[R + 2], EG[R];
  const double2 z = make_double2(0.0, 0.0);
#pragma unroll
  for (int m = 0; m < R + 2; ++m) {
    const int r = rb - 1 + m;
    const bool want = HALO ? (r >= 0 && r < n) : (m >= 1 && r < re);
    U[m] = want ? u[(size_t)r * n + i] : z;
  }
  const int iw = min(max(lane < 32 ? i - lane - 1 : i - lane + 64, 0), n - 1);
#pragma unroll
  for (int m = 0; m < R; ++m) EG[m] = EDGE ? u[(size_t)min(rb + m, re - 1) * n + iw] : z;
  double2 t0 = z, t1 = z, t2 = z;
  if (TAB) {
    t0 = u[i];
    t1 = u[(size_t)n + i];
    t2 = u[(size_t)2 * n + i];
  }
#pragma unroll
  for (int m = 0; m < R; ++m) {
    const int r = rb + m;
    if (r < re) {
      double vx = U[m + 1].x + 0.25 * (U[m].x + U[m + 2].x) + EG[m].x + t0.x + t1.x + t2.x;
      double vy = U[m + 1].y + 0.25 * (U[m].y + U[m + 2].y) + EG[m].y + t0.y + t1.y + t2.y;
      __builtin_nontemporal_store(vx, &y[(size_t)r * n + i].x);
      __builtin_nontemporal_store(vy, &y[(size_t)r * n + i].y);
    }
  }
}

// P7/P8: the stencil's traversal without its arithmetic or neighbours.  A 512-thread block
// owns a 512-wide strip x 32-row band and marches it with one row of prefetch (NT loads and
// stores, 40 B/point).  P7 deals tiles to XCDs in contiguous ranges as the stencil does; P8
// takes tiles in plain blockIdx order.
template <bool XCD, int RB>
__global__ __launch_bounds__(512) void pmarch(const double2* __restrict__ u,
                                              const double* __restrict__ ic,
                                              double2* __restrict__ y, int n) {
  constexpr int TW = 512;
  const int tiles_x = (n + TW - 1) / TW, tiles_y = (n + RB - 1) / RB;
  const int ntiles = tiles_x * tiles_y;
  int t = blockIdx.x;
  if (XCD) {
    const int per = (ntiles + 7) / 8;
    t = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  }
  if (t >= ntiles) return;
  const int i = min((t % tiles_x) * TW + (int)threadIdx.x, n - 1);
  const int r0 = (t / tiles_x) * RB, r1 = min(r0 + RB, n);
  auto ld = [&](int r, double2& uv, double& c) {
    const size_t p = (size_t)r * n + i;
    uv = make_double2(__builtin_nontemporal_load(&u[p].x), __builtin_nontemporal_load(&u[p].y));
    c = __builtin_nontemporal_load(&ic[p]);
  };
  double2 ua, ub;
  double ca, cb;
  ld(r0, ua, ca);
  for (int r = r0; r < r1; r += 2) {
    ld(min(r + 1, r1 - 1), ub, cb);
    double2* q = y + (size_t)r * n + i;
    __builtin_nontemporal_store(ua.x * ca, &q->x);
    __builtin_nontemporal_store(ua.y * ca, &q->y);
    ld(min(r + 2, r1 - 1), ua, ca);
    if (r + 1 < r1) {
      q += n;
      __builtin_nontemporal_store(ub.x * cb, &q->x);
      __builtin_nontemporal_store(ub.y * cb, &q->y);
    }
  }
}

// P13/P14: a naive 5-point gather -- one point per thread, no marching: u at (i, j), (i +- 1,
// j), (i, j +- 1) through the cache (the neighbours' lines are L2 / Infinity-Cache hits of
// the blocks working on the adjacent rows at the same time), 1/c^2 and y non-temporal; one
// block per 256 points in address order.  P13: blockIdx order (consecutive blocks on
// different XCDs); P14: XCD k takes a contiguous range of rows.
template <bool XCD>
__global__ __launch_bounds__(256) void pnaive(const double2* __restrict__ u,
                                              const double* __restrict__ ic,
                                              double2* __restrict__ y, int n) {
  const long nb = ((long)n * n + 255) / 256;
  long b = blockIdx.x;
  if (XCD) {
    const long per = (nb + 7) / 8;
    b = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  }
  const long p = b * 256 + threadIdx.x;
  if (b >= nb || p >= (long)n * n) return;
  const int i = (int)(p % n), j = (int)(p / n);
  const double2 z = make_double2(0.0, 0.0);
  const double2 c = u[p];
  const double2 w = i > 0 ? u[p - 1] : z;
  const double2 e = i + 1 < n ? u[p + 1] : z;
  const double2 sv = j > 0 ? u[p - n] : z;
  const double2 nv = j + 1 < n ? u[p + n] : z;
  const double k = __builtin_nontemporal_load(&ic[p]);
  const double2 r = make_double2(k * c.x + w.x + e.x + sv.x + nv.x, k * c.y + w.y + e.y + sv.y + nv.y);
  __builtin_nontemporal_store(r.x, &y[p].x);
  __builtin_nontemporal_store(r.y, &y[p].y);
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
    case 7: case 8: case 9: case 10: case 11: case 12: {
      // marching tiles over the n x n grid (len = n^2); `blocks` is ignored.  7: 32-row bands
      // XCD map; 8: 32-row bands blockIdx order; 9 / 10 / 11 / 12: 8 / 16 / 64 / 128-row
      // bands, XCD map
      const int n = (int)llround(std::sqrt((double)len));
      if ((size_t)n * n != len) return 0;
      const int rb = kind == 9 ? 8 : kind == 10 ? 16 : kind == 11 ? 64 : kind == 12 ? 128 : 32;
      const int tiles = ((n + 511) / 512) * ((n + rb - 1) / rb);
      const dim3 gm((tiles + 7) / 8 * 8), bm(512);
      switch (kind) {
        case 7: hipLaunchKernelGGL((pmarch<true, 32>), gm, bm, 0, s, u, ic, y, n); break;
        case 8: hipLaunchKernelGGL((pmarch<false, 32>), gm, bm, 0, s, u, ic, y, n); break;
        case 9: hipLaunchKernelGGL((pmarch<true, 8>), gm, bm, 0, s, u, ic, y, n); break;
        case 10: hipLaunchKernelGGL((pmarch<true, 16>), gm, bm, 0, s, u, ic, y, n); break;
        case 11: hipLaunchKernelGGL((pmarch<true, 64>), gm, bm, 0, s, u, ic, y, n); break;
        default: hipLaunchKernelGGL((pmarch<true, 128>), gm, bm, 0, s, u, ic, y, n); break;
      }
      return 40;
    }
    case 13:
    case 14: {
      const int n = (int)llround(std::sqrt((double)len));
      if ((size_t)n * n != len) return 0;
      const long nb = ((long)len + 255) / 256;
      const dim3 gn((unsigned)((nb + 7) / 8 * 8)), bn(256);
      if (kind == 13) hipLaunchKernelGGL(pnaive<false>, gn, bn, 0, s, u, ic, y, n);
      else hipLaunchKernelGGL(pnaive<true>, gn, bn, 0, s, u, ic, y, n);
      return 40;
    }
    case 17: case 18: case 19: case 20: case 21: {
      const int n = (int)llround(std::sqrt((double)len));
      if ((size_t)n * n != len) return 0;
      const int R = kind == 21 ? 12 : 6;
      const dim3 gt((unsigned)(((n + kT - 1) / kT) * ((n + R - 1) / R))), bt(kT);
      switch (kind) {
        case 17: hipLaunchKernelGGL((ptile<6, false, false, false>), gt, bt, 0, s, u, y, n); break;
        case 18: hipLaunchKernelGGL((ptile<6, true, false, false>), gt, bt, 0, s, u, y, n); break;
        case 19: hipLaunchKernelGGL((ptile<6, true, true, false>), gt, bt, 0, s, u, y, n); break;
        case 20: hipLaunchKernelGGL((ptile<6, true, true, true>), gt, bt, 0, s, u, y, n); break;
        default: hipLaunchKernelGGL((ptile<12, false, false, false>), gt, bt, 0, s, u, y, n); break;
      }
      return 32;
    }
    case 15: hipLaunchKernelGGL(pcopy_nt<true>, g, b, 0, s, u, y, len); return 32;
    case 16: hipLaunchKernelGGL(pcopy_nt<false>, g, b, 0, s, u, y, len); return 32;
    default: return 0;
  }
}

}  // namespace hh
