// Device helpers shared by the one-pass GMRES iteration kernels (fused.hip: M none / Jacobi and
// the two-sweep shifted Laplace at two blocks per CU; fused_slk.hip: the shifted-Laplace pass
// that keeps its whole basis window on chip at one block per CU).  DESIGN 3g.
#pragma once
#include <cstddef>

#include "hh_internal.hpp"
#include "hh_complex.hpp"
#include "hh_wave.hpp"
#include "hh_givens.hpp"

namespace hh {
namespace fusedk {

constexpr int kT = 256;  // threads per block = columns per strip

struct double2x2 {
  double2 a, b;
};
__device__ __forceinline__ double2x2 make_double2x2(double2 a, double2 b) { return {a, b}; }

// by-value select (a select of lvalues would become a select of addresses)
__device__ __forceinline__ double2 csel(bool c, double2 a, double2 b) {
  return make_double2(c ? a.x : b.x, c ? a.y : b.y);
}

// Global-address-space views: a row pointer made opaque to the optimiser (asm "+s", so neither
// per-vector address registers nor strength-reduced pointers appear) must stay a GLOBAL pointer,
// or every load through it becomes a flat load with a 64-bit VGPR address.
typedef double d2v __attribute__((ext_vector_type(2)));
using gd2 = const __attribute__((address_space(1))) d2v;
__device__ __forceinline__ gd2* gptr(const double2* p) { return (gd2*)p; }
// *(row + byte offset): `row` uniform (scalar registers), `boff` the lane's 32-bit byte offset --
// the global_load saddr form: one VGPR of address for every vector of a row instead of a 64-bit
// address per vector
__device__ __forceinline__ double2 ld_at(gd2* row, unsigned boff) {
  using gc = const __attribute__((address_space(1))) char;
  const d2v v = *(gd2*)((gc*)row + boff);
  return make_double2(v.x, v.y);
}

// Row tables through the constant address space: loads of a uniform address become scalar
// loads (s_load, waited for by lgkmcnt).  Through a plain pointer they were vector loads, and
// the vmcnt wait for them also waited for every load issued earlier -- the next row's prefetch.
using cdouble_p = const __attribute__((address_space(4))) double*;
__device__ __forceinline__ cdouble_p crow(const double2* tab, ptrdiff_t r) {
  return (cdouble_p)(reinterpret_cast<const double*>(tab) + 8 * r);
}

// Sum over the 32 lanes of this lane's half-wave, fixed order, the same bits on every lane of
// the half: pairs, quads, 8 and 16 by DPP lane moves (hh_wave.hpp), then the half's two rows
// by permlane16_swap -- VALU only, where an xor-shuffle tree is 5 dependent ds_bpermute
// rounds (the edge waves' critical path in the one-pass kernels)
__device__ __forceinline__ double half_sum(double v) {
  v += dpp_mov<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141, 0xf>(v);  // row_half_mirror
  v += dpp_mov<0x140, 0xf>(v);  // row_mirror
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(h16[0], l16[0]) + __hiloint2double(h16[1], l16[1]);
}
__device__ __forceinline__ double2 half_sum2(double2 v) {
  return make_double2(half_sum(v.x), half_sum(v.y));
}

// The band of this block: tiles dealt to XCDs in contiguous runs (block b -> XCD b % 8).
struct Band {
  bool live;
  int tx, ty, rb, re;  // strip, band index, rows [rb, re)
};
__device__ __forceinline__ Band band_of(const FusedArgs& a) {
  const int tiles_x = (a.n + kT - 1) / kT, T = tiles_x * a.bands;
  const int per_xcd = (T + 7) / 8;
  const int tile = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
  Band b;
  b.live = tile < T;
  b.tx = b.live ? tile % tiles_x : 0;
  const int ty = b.live ? tile / tiles_x : 0;
  const int step = a.row_step > 0 ? a.row_step : a.rows;
  b.ty = ty;
  b.rb = a.row_begin + ty * step;
  b.re = min(b.rb + a.rows, a.row_end);
  return b;
}

// u_K at row r (uniform), column col, given the value formed from the (clamped) row: rows inside
// [rlo, rhi) are formed from memory; the others are zero (FROW_ZERO) or the neighbour rank's
// received rows (FROW_HALO; H halo rows per side: rows -H .. -1 and nl .. nl+H-1).
// A march also asks for rows just beyond those (the shifted-Laplace pass's edge waves form u_K
// one row behind the band's first ring row: row -3 in a band starting at row 0).  Those values
// feed only rows the pass never outputs, and there is no received row to read: they are zero.
// (Until round 6 row -3 was read at halo_lo - n -- one row BEFORE the receive buffer.  Where
// that address was mapped by another allocation the value was discarded unnoticed; under
// RCCL's allocation layout at 11584^2 / 8 ranks it was unmapped and every rank faulted in the
// first pass's boundary rows.  DESIGN 4, tests/test_gpu_dist.py guarded-halo tests.)
template <int H>
__device__ __forceinline__ double2 row_value(const FusedArgs& a, int rlo, int rhi, int r, int col,
                                             double2 formed) {
  if (r >= rlo && r < rhi) return formed;
  if (r < 0)
    return (a.lo_mode == FROW_HALO && r >= -H) ? a.halo_lo[(size_t)(r + H) * a.n + col]
                                               : make_double2(0.0, 0.0);
  return (a.hi_mode == FROW_HALO && r < a.nl + H) ? a.halo_hi[(size_t)(r - a.nl) * a.n + col]
                                                  : make_double2(0.0, 0.0);
}

// the update coefficients c_k = raw_k s_k^2 (update_kernel's expression), k < K, into LDS
template <int K>
__device__ __forceinline__ void load_coef(const FusedArgs& a, double2* coef) {
  const int t = threadIdx.x;
  if (t < K) {
    const double sk = a.vscale[t];
    const double2 hk = cscale(make_double2(a.raw[2 * t], a.raw[2 * t + 1]), sk);
    coef[t] = cscale(hk, sk);
  }
}

// ---- the in-pass column (PassFold, HH_LAG_RED=2): after every block stored its partial row
// write-through (block_reduce_vec<SC1>), the pass's own blocks reduce the rows in EXACTLY
// reduce_kernel's order -- so the sums, the column and the whole history are bit-identical to
// HH_LAG_RED=1 / 0 (gmres_lag_red_kernel, reduce_kernel + gmres_lag_kernel):
//   reduce_kernel's thread t (< 256) sums rows t, t + 256, ... ascending from 0.0 (S_t); its tree
//   then forms U_r = (S_r + S_{r+128}) + (S_{r+64} + S_{r+192}) for r < 64 and sums the U_r by
//   shuffles (off = 32 .. 1).
//   Here the blocks b = r (mod 64) are one class: the last of them to arrive runs the four
//   S_{r + 64 q} of its class (its rows ascending, row j of the class into S_{j mod 4}) and
//   stores U_r; the last class to finish runs the shuffle tree of every column (one wave a
//   column, U_r on lane r) and the lag step (gmres_lag_kernel's arithmetic) on its first wave.
// Hand-offs (MI355X_MICROARCH.md's sc1 hand-off table, first row): every byte handed over is
// stored sc1 (write-through) and every storing wave drains its stores (vmcnt(0)) before a
// workgroup barrier; then ONE lane adds to the class's counter with a RELAXED agent-scope
// atomic; the block whose add returns the last ticket reads the bytes with sc1 loads only
// (global_load sc1), after a barrier.  No release/acquire fence: an acq_rel ticket lowers to
// buffer_wbl2 sc1 + buffer_inv sc1 in EVERY block -- a write-back of the XCD's L2, dirty with
// the pass's w / u stores -- and made the in-pass column slower than the launches it replaces
// (config 2 58.2 -> 67.8 us per iteration, profiles/r06/r06l_*).  Lines of the partial rows are
// never read earlier in the launch, and a kernel start invalidates the L2s, so a reader's L2 has
// no stale copy.  Counters re-armed by the block that finished with them; the next launch starts
// after a kernel boundary.
using gu32f = __attribute__((address_space(1))) unsigned;
using gu64f = __attribute__((address_space(1))) unsigned long long;
__device__ __forceinline__ double ld_agent(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load((gu64f*)p, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_agent(double* p, double v) {
  __hip_atomic_store((gu64f*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool fold_ticket(unsigned* counter, unsigned last) {
  __shared__ int is_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores landed
  __syncthreads();
  if (threadIdx.x == 0)
    is_last = __hip_atomic_fetch_add((gu32f*)counter, 1u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT) == last;
  __syncthreads();
  return is_last;
}
// The fold over `cols` columns of partial rows `width` apart, then the lag step of column f.j:
// gmres_lag_kernel's (final_step: only the subdiagonal's |w|^2 = the reduced column 0, as
// gmres_lag_red_kernel's final-step mode).  Used by the passes (pass_fold) and, on one rank, by
// the one-pass cycle's first dots and its end (fused.hip cycle_start_dots_kernel,
// cycle_end_kernel).
__device__ __forceinline__ void fold_reduce_lag(const PassFold& f, const double* partials,
                                                int width, int cols, bool final_step) {
  const int nb = gridDim.x, r = blockIdx.x % kFoldClasses;
  const int ncls = min(nb, kFoldClasses);
  const int cnt = (nb - r + kFoldClasses - 1) / kFoldClasses;  // blocks r, r + 64, ... < nb
  const int t = threadIdx.x;
  if (!fold_ticket(f.tickets + 1 + r, (unsigned)cnt - 1)) return;
  if (t < cols) {  // U_r of column t
    double S[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j0 = 0; j0 < cnt; j0 += 16) {  // (16 row loads in flight)
      double v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q)
        v[q] = ld_agent(partials +
                        (size_t)(r + kFoldClasses * min(j0 + q, cnt - 1)) * width + t);
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (j0 + q < cnt) S[q & 3] += v[q];  // (j0 a multiple of 4: row j0 + q into S_{q mod 4})
    }
    st_agent(f.gpart + (size_t)t * kFoldClasses + r, (S[0] + S[2]) + (S[1] + S[3]));
  }
  if (t == 0) f.tickets[1 + r] = 0u;  // (re-armed: every block of the class has arrived)
  if (!fold_ticket(f.tickets, (unsigned)ncls - 1)) return;
  __shared__ double sred[64];
  const int lane = t & (kWave - 1), w = t / kWave;
  constexpr int kCols = 64 / (kT / kWave);  // columns per wave
  double u[kCols];
#pragma unroll
  for (int k = 0; k < kCols; ++k) {
    const int c = w + (kT / kWave) * k;
    u[k] = (c < cols && lane < ncls) ? ld_agent(f.gpart + (size_t)c * kFoldClasses + lane) : 0.0;
  }
#pragma unroll
  for (int k = 0; k < kCols; ++k) {
    const int c = w + (kT / kWave) * k;
    if (c < cols) {  // (wave-uniform)
      double x = u[k];
#pragma unroll
      for (int off = kWave / 2; off > 0; off >>= 1) x += __shfl_down(x, off);
      if (lane == 0) {
        sred[c] = x;
        f.red[c] = x;
      }
    }
  }
  if (t == 0) f.tickets[0] = 0u;
  __syncthreads();
  if (t < kWave) {  // the lag step, one wave (gmres_lag_red_kernel's second half)
    using namespace givens;
    const LagIn L = lag_load(f.g, f.j);
    if (!L.stopped) {
      if (final_step) {
        lag_compute(f.g, f.j, L, make_double2(0.0, 0.0), 0.0, sred[0], 1, f.eps, f.ptol,
                    f.stop_col);
      } else {
        const int kj = min(t, f.j);
        const int is = 2 * (f.j + 1) + 1;  // (the first column's sig: not read at j = 0)
        lag_compute(f.g, f.j, L, make_double2(sred[2 * kj], sred[2 * kj + 1]), sred[2 * (f.j + 1)],
                    is < cols ? sred[is] : 0.0, 0, f.eps, f.ptol, f.stop_col);
      }
    }
  }
}
__device__ __forceinline__ void pass_fold(const FusedArgs& a, int width) {
  fold_reduce_lag(a.fold, a.partials, width, width, false);
}
// the pass's partial row: plain stores, or write-through stores + the in-pass column
template <int NV>
__device__ __forceinline__ void pass_epilogue(double (&v)[NV], const FusedArgs& a) {
  if (a.fold.tickets) {
    block_reduce_vec<NV, true>(v, a.partials, NV);
    pass_fold(a, NV);
  } else {
    block_reduce_vec<NV>(v, a.partials, NV);
  }
}

}  // namespace fusedk
}  // namespace hh
