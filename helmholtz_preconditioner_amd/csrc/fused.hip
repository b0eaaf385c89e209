// One pass over the Krylov basis per GMRES inner iteration (`hh_op_set_krylov_mode`
// 3): the update of iteration K-1 of the lagged-normalisation iteration (krylov.hip
// gmres_lag_kernel), the next M A and the next projections in ONE streaming kernel.
//
// Replaces, per inner iteration of scipy.sparse.linalg.gmres (scipy 1.15.3
// _isolve/iterative.py:748-800, which code.py:516 runs): the axpy loop of the orthogonalisation,
// the psolve(matvec(v)) of the next iteration (code.py:510-516: A @ x and the M slot) and the
// np.vdot projections of the next iteration -- three sweeps over the basis and the grid in one.
//
// A 256-thread block marches a 256-column strip of a band of rows.  Per row r it forms u_K on
// row r + 1 (w_{K-1} and the K basis rows: the iteration's only HBM read of them), applies the
// stencil (+ M) to row r from a three-row register ring (W/E neighbours through a
// double-buffered LDS row; the strip's two edge columns' u_K formed by the two edge waves,
// lane-parallel), stores u_K and w_K of row r and adds row r's <u_k, w_K>.  The projections
// need the basis row r one step after the update read it: the first KEEP vectors come from a
// one-row LDS copy of the thread's own column (written after row r's projections from the
// registers that held row r + 1 since its load -- the same lane writes and reads, so no
// barrier), the rest from the memory system.  A band re-forms its halo rows of u_K (never
// stored: each is a neighbouring band's own row); across slabs of one rank it forms them in
// place (FROW_MEM), across ranks it reads the neighbour's rows from the halo exchange
// (FROW_HALO, formed by fused_edge_kernel before the exchange).  Tiles are dealt to XCDs in
// contiguous runs (block b -> XCD b % 8), so a band's halo rows are mostly read on the XCD that
// owns them.  Arithmetic per point: update_kernel's coefficient and term order, stencil.hip's
// operator; only the inner products' summation order differs from the separate launches, and
// the strip edge columns' u_K (halo values, summed by a shuffle tree) agree with the stored u_K
// (k order) to rounding.
#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <string>

#include "hh_internal.hpp"
#include "hh_complex.hpp"
#include "hh_wave.hpp"
#include "hh_fused.hpp"
#include "hh_error.hpp"

namespace hh {
namespace {
using namespace fusedk;

// shifted-Laplace pass: basis vectors kept in its three-row LDS ring (HH_SL_KEEP at build time
// for A/B builds)
#ifndef HH_SL_KEEP
#define HH_SL_KEEP 5
#endif
constexpr int kSlKeep = HH_SL_KEEP;


// ------------------------------------------------------------------ M = none / Jacobi
template <int K, bool CONSTC, int KEEP>
__global__ __launch_bounds__(kT) void fused_iter_kernel(const FusedArgs a) {
  if (a.stop && *a.stop) return;
  constexpr int KL = KEEP < K ? KEEP : K;  // kept (LDS-served) projection re-reads
  // the next KR vectors' re-reads served from registers: their row r + 1 (loaded for the
  // update) and row r (the previous step's) both held -- 8 VGPRs each (K = 18, 19: every
  // re-read on chip within two waves per SIMD)
  constexpr int KR = KL > 0 ? (K - KL < 2 ? K - KL : 2) : 0;
  constexpr int kB = KL > 0 ? 4 : 8;       // batch of the remaining vectors' loads
  __shared__ double2 coef[K];
  __shared__ double2 urow[2][kT + 2];
  __shared__ double2 vkeep[KL > 0 ? KL : 1][kT];  // basis row r, k < KL, [k][lane]
  const int n = a.n, nl = a.nl;
  const Band bd = band_of(a);
  const int t = threadIdx.x, lane = t & (kWave - 1), wv = t / kWave;
  const int i0 = bd.tx * kT, i = i0 + t;
  const bool act = i < n;
  const int ic = min(i, n - 1);
  const int rb = bd.rb, re = bd.re;
  // rows whose u_K is formed from memory: the slab, and the neighbouring slab's row on a
  // FROW_MEM side
  const int rlo = a.lo_mode == FROW_MEM ? -1 : 0, rhi = a.hi_mode == FROW_MEM ? nl + 1 : nl;
  // the strip's edge columns: wave 0 forms u_K at i0 - 1, the last wave at i0 + kT
  const bool ew = wv == 0, ee = wv == kT / kWave - 1;
  const int ie = min(max(ew ? i0 - 1 : i0 + kT, 0), n - 1);
  const bool ehas = (ew && i0 > 0) || (ee && i0 + kT < n);
  load_coef<K>(a, coef);
  __syncthreads();
  const double sin = *a.sin;
  const double2 z = make_double2(0.0, 0.0);
  // kz: an opaque zero redefined every row, so neither the coefficients' LDS reads nor the
  // per-vector addresses become loop-invariant / strength-reduced registers (4 + 2-6 VGPRs per
  // basis vector otherwise)
  int kz = 0;
  // basis row r + 1 of the first KL vectors, held from the update's load until row r's
  // projections are done, then copied to vkeep for row r + 1's projections
  double2 hold[KL > 0 ? KL : 1];
  double2 rnext[KR > 0 ? KR : 1], rcur[KR > 0 ? KR : 1];  // rows r + 1 and r, k in [KL, KL + KR)
  // u_K at (r, col): w_{K-1} - sum_k c_k u_k in k order; the first KL loads issued together
  // (one memory round trip), the rest in batches of kB in a runtime loop (a fully unrolled
  // loop keeps ~16 VGPRs per vector live)
  // (addresses: a row pointer + k ldv, uniform -- scalar registers --, plus the lane's 32-bit
  // column offset: one VGPR for all K loads instead of a 64-bit address per vector)
  auto unew = [&](int r, unsigned col) {
    __builtin_amdgcn_sched_barrier(0);  // (calls and batches do not interleave: registers)
    const int rc = min(max(r, rlo), rhi - 1);
    gd2* vrow = gptr(a.V + (ptrdiff_t)rc * n);
    gd2* wrow = gptr(a.win + (ptrdiff_t)rc * n);
    // (opaque scalar row pointers: no per-vector strength-reduced address registers)
    asm volatile("" : "+s"(vrow), "+s"(wrow));
    const unsigned bo = col * (unsigned)sizeof(double2);
    double2 w = ld_at(wrow, bo);
    if constexpr (KL > 0) {
#pragma unroll
      for (int q = 0; q < KL; ++q) hold[q] = ld_at(vrow + (size_t)q * a.ldv, bo);
      // (the coefficients' LDS reads in batches of 4: all KL in flight would hold 4 KL VGPRs
      // next to the held row and the accumulators)
#pragma unroll
      for (int q0 = 0; q0 < KL; q0 += 4) {
        double2 c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) c[q] = coef[min(q0 + q, KL - 1) + kz];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (q0 + q < KL) w = csub(w, cmul(c[q], hold[q0 + q]));
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (KR > 0) {
#pragma unroll
      for (int q = 0; q < KR; ++q) rnext[q] = ld_at(vrow + (size_t)(KL + q) * a.ldv, bo);
#pragma unroll
      for (int q = 0; q < KR; ++q) w = csub(w, cmul(coef[KL + q + kz], rnext[q]));
    }
#pragma unroll 1
    for (int k0 = KL + KR; k0 < K; k0 += kB) {
      double2 v[kB];
#pragma unroll
      for (int q = 0; q < kB; ++q)
        v[q] = ld_at(vrow + (size_t)min(k0 + q, K - 1) * a.ldv, bo);
#pragma unroll
      for (int q = 0; q < kB; ++q)
        if (k0 + q < K) w = csub(w, cmul(coef[k0 + q + kz], v[q]));
    }
    // (w complete here: the update must not sink into row_value's branch, where its operands
    // -- the held row and every coefficient -- would all be live at once)
    asm volatile("" : "+v"(w.x), "+v"(w.y));
    return row_value<1>(a, rlo, rhi, r, col, w);
  };
  // u_K at one point, lane-parallel (the edge waves: lane k of each half takes the term
  // c_k u_k, summed by shuffles -- one load round trip instead of ceil(K / kB) batches).  Its
  // two loads are issued before the strip's own row (unew), so that both round trips overlap:
  // the edge waves otherwise waited on a second one every row, and the block's barrier with them
  struct EdgeLd {
    double2 wv, vk;
  };
  auto unew1_issue = [&](int r, int c) {
    const int k = lane & 31;
    const int rc = min(max(r, rlo), rhi - 1);
    const ptrdiff_t p = (ptrdiff_t)rc * n + c;
    EdgeLd e;
    e.wv = a.win[p];
    e.vk = (a.V + p)[(size_t)min(k, K - 1) * a.ldv];
    return e;
  };
  auto unew1_finish = [&](int r, int c, const EdgeLd& e) {
    const int k = lane & 31;
    const double2 tk = half_sum2(csel(k < K, cmul(coef[min(k, K - 1)], e.vk), z));
    return row_value<1>(a, rlo, rhi, r, c, csub(e.wv, tk));
  };
  const double2 AW = a.tab_i[ic], AE = a.tab_i[n + ic], R1 = a.tab_i[2 * n + ic];
  double2 acc[K + 1];
#pragma unroll
  for (int k = 0; k <= K; ++k) acc[k] = z;
  double nw = 0.0, nu = 0.0;
  if (bd.live) {
    // direction: odd bands march downwards (a.alt), so that neighbouring bands, which start
    // together, reach their shared boundary rows at the same time -- the halo rows a band
    // re-forms from the basis are then read while the owning band reads them (L2 hits), where
    // bands all marching up read them a band's length apart (round 4: 1.13-1.27x the pass's
    // bytes at 1024^2, 8-row bands).  Per point the same arithmetic; only the order in which a
    // band's rows add into its partial row changes.
    const bool dn = a.alt && (bd.ty & 1);
    const int d = dn ? -1 : 1;
    const int r_first = dn ? re - 1 : rb;
    double2 uB = unew(r_first - d, (unsigned)ic);  // the row behind the march
    double2 uC = unew(r_first, (unsigned)ic);
    if constexpr (KL > 0) {
#pragma unroll
      for (int q = 0; q < KL; ++q) vkeep[q][t] = hold[q];
    }
#pragma unroll
    for (int q = 0; q < KR; ++q) rcur[q] = rnext[q];
    int buf = 0;
    for (int s0 = 0; s0 < re - rb; ++s0) {
      int r = r_first + d * s0;
      asm volatile("" : "+s"(r), "+s"(kz));
      EdgeLd el{z, z};
      if (ew || ee) el = unew1_issue(r, ie);  // (wave-uniform: the two edge waves only)
      const double2 uA = unew(r + d, (unsigned)ic);  // the row ahead
      const double2 uS = csel(dn, uA, uB), uN = csel(dn, uB, uA);
      double2 ue = z;
      if (ew || ee) ue = unew1_finish(r, ie, el);
      urow[buf][1 + t] = csel(act, uC, z);
      if (ew && lane == 0) urow[buf][0] = csel(ehas, ue, z);
      if (ee && lane == kWave - 1) urow[buf][kT + 1] = csel(ehas, ue, z);
      __syncthreads();
      const double2 uW = urow[buf][t], uE = urow[buf][t + 2];
      const cdouble_p q = crow(a.tab_j, r);
      const double2 R2 = make_double2(q[0], q[1]), BS = make_double2(q[2], q[3]);
      const double2 BN = make_double2(q[4], q[5]), OM = make_double2(q[6], q[7]);
      const size_t p = (size_t)r * n + ic;
      const double icv = CONSTC ? a.invc2_const : a.invc2[p];
      const double2 W = cmul(AW, R2);
      const double2 E = cmul(AE, R2);
      const double2 S = cmul(BS, R1);
      const double2 N = cmul(BN, R1);
      const double2 M = cscale(cmul(OM, R1), icv);
      const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
      const double2 D = csub(M, sum4);
      double2 Au = cmul(S, uS);
      Au = cfma(W, uW, Au);
      Au = cfma(D, uC, Au);
      Au = cfma(E, uE, Au);
      Au = cfma(N, uN, Au);
      const double2 w = csel(act, a.jac ? cscale(cdiv(Au, D), sin) : cscale(Au, sin), z);
      if (act) {
        a.wout[p] = w;
        a.uout[p] = uC;
      }
      const double2 uo = csel(act, uC, z);
      nu = fma(uo.x, uo.x, fma(uo.y, uo.y, nu));
      nw = fma(w.x, w.x, fma(w.y, w.y, nw));
      if constexpr (KL > 0) {
        // (in batches of 4: all KL LDS reads in flight at once would hold 4 KL more VGPRs next
        // to the held row and the accumulators)
#pragma unroll
        for (int k0 = 0; k0 < KL; k0 += 4) {
          double2 v[4];
#pragma unroll
          for (int q2 = 0; q2 < 4; ++q2) v[q2] = vkeep[min(k0 + q2, KL - 1)][t];
#pragma unroll
          for (int q2 = 0; q2 < 4; ++q2)
            if (k0 + q2 < KL) acc[k0 + q2] = cfma_conj(v[q2], w, acc[k0 + q2]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int q2 = 0; q2 < KR; ++q2) acc[KL + q2] = cfma_conj(rcur[q2], w, acc[KL + q2]);
      // the remaining re-reads from the memory system, kB in flight
      gd2* vr = gptr(a.V + (size_t)r * n);
      asm volatile("" : "+s"(vr));
#pragma unroll
      for (int k0 = KL + KR; k0 < K; k0 += kB) {
        double2 v[kB];
#pragma unroll
        for (int q2 = 0; q2 < kB; ++q2)
          v[q2] = ld_at(vr + (size_t)min(k0 + q2, K - 1) * a.ldv, (unsigned)ic * 16u);
#pragma unroll
        for (int q2 = 0; q2 < kB; ++q2)
          if (k0 + q2 < K) acc[k0 + q2] = cfma_conj(v[q2], w, acc[k0 + q2]);
        __builtin_amdgcn_sched_barrier(0);
      }
      acc[K] = cfma_conj(uo, w, acc[K]);
      if constexpr (KL > 0) {  // (row r + d's basis for the next step's projections)
#pragma unroll
        for (int q2 = 0; q2 < KL; ++q2) vkeep[q2][t] = hold[q2];
      }
#pragma unroll
      for (int q2 = 0; q2 < KR; ++q2) rcur[q2] = rnext[q2];
      uB = uC;
      uC = uA;
      buf ^= 1;
    }
  }
  // one partial row: the K + 1 dots, |w_K|^2, then |u_K|^2 -- one reduce launch lands the last
  // exactly where gmres_lag_kernel reads sigma_K^2 (red + 16 + 2 (K + 1) + 1)
  double v[2 * (K + 1) + 2];
#pragma unroll
  for (int k = 0; k <= K; ++k) {
    v[2 * k] = acc[k].x;
    v[2 * k + 1] = acc[k].y;
  }
  v[2 * (K + 1)] = nw;
  v[2 * (K + 1) + 1] = nu;
  pass_epilogue<2 * (K + 1) + 2>(v, a);
}

// ------------------------------------------------------- M = two-sweep shifted Laplace
// The same pass with M = the two-sweep shifted-Laplace smoother (stencil.hip EPI_SL_FIRST then
// EPI_SL_SWEEP): T = s A u, z1 = damp T / D_beta, w = z1 + damp (T - A_beta z1) / D_beta.
// Output row r needs z1 on rows r-1 .. r+1, i.e. u_K on rows r-2 .. r+2 and on two columns
// beyond the strip on each side: per step L the block forms u_K on row L (own columns; the
// edge waves also on the edge column and, one row behind, the outer column), T and z1 on row
// L-1 (own columns; the edge waves on the edge column) and w on row L-2 -- rings of three u,
// two T and three z1 rows, W/E neighbours of u (row L-1) and z1 (row L-2) through two
// double-buffered LDS rows.  Rows and columns off the grid are zero for u, T and z1 alike
// (the two-launch path's Dirichlet neighbours); the slab's tables hold rows -2 .. nl+1 and
// invc2_halo the medium of rows -2, -1, nl, nl+1.
template <int K, bool CONSTC>
__global__ __launch_bounds__(kT) void fused_sl_iter_kernel(const FusedArgs a) {
  if (a.stop && *a.stop) return;
  // the projections of row r run two steps after its basis row was loaded for the update (w on
  // row r needs u_K two rows further): the first KS vectors' rows r .. r + 2 are kept in a
  // three-row LDS ring (written from the update's first load batch, read by the same lane),
  // the rest re-read from the memory system.  (KS = 5: 60 KB, the most that keeps two blocks
  // per CU beside the exchange rows)
  constexpr int KS = K < kSlKeep ? K : kSlKeep;
  constexpr bool kCarry = K <= 16;  // (the carried coefficients' 16 VGPRs: spills from K = 19)
  __shared__ double2 coef[K];
  __shared__ double2 urow[2][kT + 2], zrow[2][kT + 2];
  __shared__ double2 vkeep[3][KS][kT];
  const int n = a.n, nl = a.nl;
  const Band bd = band_of(a);
  const int t = threadIdx.x, lane = t & (kWave - 1), wv = t / kWave;
  const int i0 = bd.tx * kT, i = i0 + t;
  const bool act = i < n;
  const int ic = min(i, n - 1);
  const int rb = bd.rb, re = bd.re;
  const int rlo = a.lo_mode == FROW_MEM ? -2 : 0, rhi = a.hi_mode == FROW_MEM ? nl + 2 : nl;
  // edge waves: wave 0 the W edge column i0-1 (outer i0-2, inner i0 = LDS slot 1), the last
  // wave the E edge column i0+kT (outer i0+kT+1, inner i0+kT-1 = LDS slot kT)
  const bool ew = wv == 0, ee = wv == kT / kWave - 1;
  const int ie_raw = ew ? i0 - 1 : i0 + kT, io_raw = ew ? i0 - 2 : i0 + kT + 1;
  const bool ehas = (ew || ee) && ie_raw >= 0 && ie_raw < n;
  const bool ohas = (ew || ee) && io_raw >= 0 && io_raw < n;
  const int ie = min(max(ie_raw, 0), n - 1), io = min(max(io_raw, 0), n - 1);
  const int islot = ew ? 1 : kT;  // LDS slot of the edge column's inner neighbour
  load_coef<K>(a, coef);
  __syncthreads();
  const double sin = *a.sin;
  const double damp = a.damping;
  const double2 mshift = a.mshift;
  const double2 z = make_double2(0.0, 0.0);
  int kz = 0;
  // (scalar row pointers + the lane's 32-bit offset, coefficient reads in batches of 4, the
  // update kept out of row_value's branch: fused_iter_kernel's register economies)
  auto unew = [&](int r, unsigned col) {
    __builtin_amdgcn_sched_barrier(0);
    const int rc = min(max(r, rlo), rhi - 1);
    gd2* vrow = gptr(a.V + (ptrdiff_t)rc * n);
    gd2* wrow = gptr(a.win + (ptrdiff_t)rc * n);
    asm volatile("" : "+s"(vrow), "+s"(wrow));
    const unsigned bo = col * (unsigned)sizeof(double2);
    double2 w = ld_at(wrow, bo);
    const int slot = (r % 3 + 3) % 3;
    constexpr int kB = 8;
#pragma unroll 1
    for (int k0 = 0; k0 < K; k0 += kB) {
      double2 v[kB];
#pragma unroll
      for (int q = 0; q < kB; ++q) v[q] = ld_at(vrow + (size_t)min(k0 + q, K - 1) * a.ldv, bo);
      if (k0 == 0) {
#pragma unroll
        for (int q = 0; q < KS; ++q) vkeep[slot][q][threadIdx.x] = v[q];
      }
#pragma unroll
      for (int q0 = 0; q0 < kB; q0 += 4) {
        double2 c[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) c[q] = coef[min(k0 + q0 + q, K - 1) + kz];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (k0 + q0 + q < K) w = csub(w, cmul(c[q], v[q0 + q]));
      }
    }
    asm volatile("" : "+v"(w.x), "+v"(w.y));
    return row_value<2>(a, rlo, rhi, r, col, w);
  };
  // u_K at two points at once, lane-parallel (the edge waves): half h of the wave takes point
  // h, lane k of the half the term c_k u_k, the 32 terms summed by shuffles -- one load round
  // trip instead of two chains of ceil(K / 8) batches (terms in a tree order: the strip that
  // owns the column forms it in k order, so halo values agree to rounding).  The two loads are
  // issued before the strip's own row (so both round trips overlap), the sum after it.
  struct EdgeLd {
    double2 wv, vk;
  };
  auto unew2_issue = [&](int r1, int c1, int r2, int c2) {
    const int h = lane >> 5, k = lane & 31;
    const int r = h ? r2 : r1, c = h ? c2 : c1;
    const int rc = min(max(r, rlo), rhi - 1);
    const ptrdiff_t p = (ptrdiff_t)rc * n + c;
    EdgeLd e;
    e.wv = a.win[p];
    e.vk = (a.V + p)[(size_t)min(k, K - 1) * a.ldv];
    return e;
  };
  auto unew2_finish = [&](int r1, int c1, int r2, int c2, const EdgeLd& e) {
    const int k = lane & 31;
    const double2 tk = half_sum2(csel(k < K, cmul(coef[min(k, K - 1)], e.vk), z));
    const double2 ua = rlane2(tk, 0), ub = rlane2(tk, 32);
    const double2 wa = rlane2(e.wv, 0), wb = rlane2(e.wv, 32);
    return make_double2x2(row_value<2>(a, rlo, rhi, r1, c1, csub(wa, ua)),
                          row_value<2>(a, rlo, rhi, r2, c2, csub(wb, ub)));
  };
  // row r of the grid?  (the slab, or a neighbour's row on a side that is not the boundary)
  auto on_grid = [&](int r) {
    return (r >= 0 && r < nl) || (r < 0 && a.lo_mode != FROW_ZERO) ||
           (r >= nl && a.hi_mode != FROW_ZERO);
  };
  // the operator's coefficients at (row r, column c): W, E, S, N, D, D_beta (stencil.hip order)
  struct Co {
    double2 W, E, S, N, D, Db;
  };
  auto coefs = [&](int r, int c, double icv) {
    const cdouble_p q = crow(a.tab_j, min(max(r, -2), nl + 1));
    const double2 R2 = make_double2(q[0], q[1]), BS = make_double2(q[2], q[3]);
    const double2 BN = make_double2(q[4], q[5]), OM = make_double2(q[6], q[7]);
    const double2 AW = a.tab_i[c], AE = a.tab_i[n + c], R1 = a.tab_i[2 * n + c];
    Co o;
    o.W = cmul(AW, R2);
    o.E = cmul(AE, R2);
    o.S = cmul(BS, R1);
    o.N = cmul(BN, R1);
    const double2 M = cscale(cmul(OM, R1), icv);
    const double2 sum4 = cadd(cadd(cadd(o.W, o.E), o.S), o.N);
    o.D = csub(M, sum4);
    o.Db = csub(cmul(M, mshift), sum4);
    return o;
  };
  // 1/c^2 at (row r, column c): the slab's rows, or the two rows beyond each side
  auto icv_at = [&](int r, int c) {
    if constexpr (CONSTC) {
      return a.invc2_const;
    } else {
      const int rc = min(max(r, -2), nl + 1);
      const double* row = rc < 0 ? a.invc2_halo + (size_t)(rc + 2) * n
                                 : (rc >= nl ? a.invc2_halo + (size_t)(rc - nl + 2) * n
                                             : a.invc2 + (size_t)rc * n);
      return row[c];
    }
  };
  double2 acc[K + 1];
#pragma unroll
  for (int k = 0; k <= K; ++k) acc[k] = z;
  double nw = 0.0, nu = 0.0;
  if (bd.live) {
    // rings (own column): u(L-2), u(L-1); T(L-2); z1(L-3), z1(L-2).  Edge waves: u(L-2, ie),
    // u(L-1, ie), z1(L-2, ie).
    double2 uP = z, uC = z, Tm = z, z1a = z, z1b = z;
    double2 euP = z, euC = z, ez1b = z;
    // row L-1's shifted diagonal and the reciprocal of its |.|^2 (cdiv's one division), handed
    // to the second sweep of the next step, whose row it is
    double2 Dbm = make_double2(1.0, 0.0);
    double invm = 1.0;
    double2 Wm = z, Em = z, Sm = z, Nm = z;
    int buf = 0;
    for (int L0 = rb - 2; L0 <= re + 1; ++L0) {
      int L = L0;
      asm volatile("" : "+s"(L), "+s"(kz));
      EdgeLd el{z, z};
      if (ew || ee) el = unew2_issue(L, ie, L - 1, io);  // (wave-uniform)
      const double2 uN = unew(L, (unsigned)ic);
      double2 euN = z, eo = z;
      if (ew || ee) {
        const auto pr = unew2_finish(L, ie, L - 1, io, el);
        euN = csel(ehas, pr.a, z);
        eo = csel(ohas, pr.b, z);
      }
      urow[buf][1 + t] = csel(act, uC, z);
      zrow[buf][1 + t] = csel(act, z1b, z);
      if (ew && lane == 0) {
        urow[buf][0] = euC;
        zrow[buf][0] = ez1b;
      }
      if (ee && lane == kWave - 1) {
        urow[buf][kT + 1] = euC;
        zrow[buf][kT + 1] = ez1b;
      }
      __syncthreads();
      const double2 uW = urow[buf][t], uE = urow[buf][t + 2];
      const double2 zW = zrow[buf][t], zE = zrow[buf][t + 2];
      const bool v1 = on_grid(L - 1);  // row L-1 on the grid
      // T and z1 on row L-1 (own column)
      const double ic1 = icv_at(L - 1, ic);
      const Co c1 = coefs(L - 1, ic, ic1);
      double2 Au = cmul(c1.S, uP);
      Au = cfma(c1.W, uW, Au);
      Au = cfma(c1.D, uC, Au);
      Au = cfma(c1.E, uE, Au);
      Au = cfma(c1.N, uN, Au);
      const double2 T1 = csel(act && v1, cscale(Au, sin), z);
      const double inv1 = 1.0 / fma(c1.Db.x, c1.Db.x, c1.Db.y * c1.Db.y);
      auto cdivr = [](double2 x, double2 b, double inv) {  // cdiv with the reciprocal given
        return make_double2(fma(x.x, b.x, x.y * b.y) * inv, fma(x.y, b.x, -x.x * b.y) * inv);
      };
      const double2 z1c = csel(act && v1, cscale(cdivr(T1, c1.Db, inv1), damp), z);
      // the same at the edge column (edge waves; broadcast values)
      double2 ez1c = z;
      if (ew || ee) {
        const double2 uin = urow[buf][islot];
        const double2 eW = ew ? eo : uin, eE = ew ? uin : eo;
        const Co ce = coefs(L - 1, ie, icv_at(L - 1, ie));
        double2 Ae = cmul(ce.S, euP);
        Ae = cfma(ce.W, eW, Ae);
        Ae = cfma(ce.D, euC, Ae);
        Ae = cfma(ce.E, eE, Ae);
        Ae = cfma(ce.N, euN, Ae);
        const double2 eT = cscale(Ae, sin);
        ez1c = csel(ehas && v1, cscale(cdiv(eT, ce.Db), damp), z);
      }
      // w on row r = L-2: the second sweep (A_beta on z1)
      const int r = L - 2;
      if (r >= rb && r < re) {  // (block-uniform)
        const size_t p = (size_t)r * n + ic;
        // row r's W, E, S, N: the last step's row L-1 coefficients, carried (the same
        // expressions on the same operands) while registers allow, else formed again; its
        // D_beta and the reciprocal of |D_beta|^2 always carried
        double2 W2 = Wm, E2 = Em, S2 = Sm, N2 = Nm;
        if constexpr (!kCarry) {
          const cdouble_p q = crow(a.tab_j, r);
          const double2 R2 = make_double2(q[0], q[1]), BS = make_double2(q[2], q[3]);
          const double2 BN = make_double2(q[4], q[5]);
          const double2 AW = a.tab_i[ic], AE = a.tab_i[n + ic], R1 = a.tab_i[2 * n + ic];
          W2 = cmul(AW, R2);
          E2 = cmul(AE, R2);
          S2 = cmul(BS, R1);
          N2 = cmul(BN, R1);
        }
        double2 Az = cmul(S2, z1a);
        Az = cfma(W2, zW, Az);
        Az = cfma(Dbm, z1b, Az);
        Az = cfma(E2, zE, Az);
        Az = cfma(N2, z1c, Az);
        const double2 w = csel(act, cadd(z1b, cscale(cdivr(csub(Tm, Az), Dbm, invm), damp)), z);
        if (act) {
          a.wout[p] = w;
          a.uout[p] = uP;
        }
        const double2 uo = csel(act, uP, z);
        nu = fma(uo.x, uo.x, fma(uo.y, uo.y, nu));
        nw = fma(w.x, w.x, fma(w.y, w.y, nw));
        const int slot = r % 3;  // (r >= 0)
#pragma unroll
        for (int k = 0; k < KS; ++k) acc[k] = cfma_conj(vkeep[slot][k][t], w, acc[k]);
        gd2* vr = gptr(a.V + (size_t)r * n);
        asm volatile("" : "+s"(vr));
#pragma unroll
        for (int k0 = KS; k0 < K; k0 += 8) {
          double2 v[8];
#pragma unroll
          for (int q2 = 0; q2 < 8; ++q2)
            v[q2] = ld_at(vr + (size_t)min(k0 + q2, K - 1) * a.ldv, (unsigned)ic * 16u);
#pragma unroll
          for (int q2 = 0; q2 < 8; ++q2)
            if (k0 + q2 < K) acc[k0 + q2] = cfma_conj(v[q2], w, acc[k0 + q2]);
          __builtin_amdgcn_sched_barrier(0);
        }
        acc[K] = cfma_conj(uo, w, acc[K]);
      }
      uP = uC;
      uC = uN;
      Tm = T1;
      z1a = z1b;
      z1b = z1c;
      euP = euC;
      euC = euN;
      ez1b = ez1c;
      Dbm = c1.Db;
      invm = inv1;
      if constexpr (kCarry) {
        Wm = c1.W;
        Em = c1.E;
        Sm = c1.S;
        Nm = c1.N;
      }
      buf ^= 1;
    }
  }
  double v[2 * (K + 1) + 2];
#pragma unroll
  for (int k = 0; k <= K; ++k) {
    v[2 * k] = acc[k].x;
    v[2 * k + 1] = acc[k].y;
  }
  v[2 * (K + 1)] = nw;
  v[2 * (K + 1) + 1] = nu;
  pass_epilogue<2 * (K + 1) + 2>(v, a);
}

// ----------------------------------------------------------------- edge rows (across ranks)
// u_K on rows [r0, r0 + c0) and [r1, r1 + c1) of the rank-local vectors (a.V, a.win at the
// rank's first row), written to a.uout: the rows the neighbouring ranks' passes read as their
// halo.  The pass's own k-order arithmetic (csub(w, cmul(c_k, u_k)), explicit fmas): the value
// a rank stores for its boundary row and the value its neighbour reads are the same bits.
template <int K>
__global__ __launch_bounds__(kT) void fused_edge_kernel(const FusedArgs a, int r0, int c0, int r1) {
  if (a.stop && *a.stop) return;
  __shared__ double2 coef[K];
  load_coef<K>(a, coef);
  __syncthreads();
  const int tiles_x = (a.n + kT - 1) / kT;
  const int row_i = blockIdx.x / tiles_x;
  const int i = (blockIdx.x % tiles_x) * kT + threadIdx.x;
  if (i >= a.n) return;
  const int r = row_i < c0 ? r0 + row_i : r1 + (row_i - c0);
  const size_t p = (size_t)r * a.n + i;
  double2 w = a.win[p];
#pragma unroll
  for (int k = 0; k < K; ++k) w = csub(w, cmul(coef[k], a.V[(size_t)k * a.ldv + p]));
  a.uout[p] = w;
}

// ------------------------------------------------------------ the end of a full cycle
// A one-pass cycle that reaches its last column (col = stop_col) still owes: the last update
// u_{col+1} = w_col - sum_k c_k u_k, whose norm is the Hessenberg subdiagonal h1 of column col;
// then the triangular solve for y and x += sum_k y_k v_k (scipy iterative.py:817-824) -- two
// more passes over the K = col + 1 basis vectors (update_kernel, then xupdate_kernel).  y
// depends on h1 only through its last entry: with the rotations of columns < col known, the
// back-substitution is affine in y_col, y = a + y_col b (a: y_col = 0, b: the response to
// y_col = 1).  So ONE pass forms |u_{col+1}|^2 and, from the same loads, x + sum a_k v_k
// (in place) and vb = sum b_k v_k (into V[K], the vector u_{col+1} would have occupied); once
// the last column is finished, x += y_col vb.  K + 2 vector reads and 2 writes, then 2 + 1,
// instead of 2 K + 2 and 2.

// a, b of y = a + y_col b, scaled by the basis scales (x += sum (a_k + y_col b_k) v_k / sigma_k):
// ab[k] = a_k vscale_k, ab[kMaxProj + k] = b_k vscale_k, k <= col.  Column col as started by
// gmres_lag_kernel (unrotated); the previous columns final.  One wave (once per cycle), lane
// m holding row m: the rotation chain of column col run by every lane (uniform; lane k keeps
// entry k), then a column-oriented back-substitution -- y_m = s_m / R_mm by lane m (the Smith
// factors of every diagonal formed up front, in parallel), broadcast, and lanes k < m take
// s_k -= y_m R_km -- so the serial chain is col steps of a few dependent multiplies.  The
// row-oriented serial form (lane 0 alone, divisions on the chain) took 25 us per cycle even on
// LDS operands, 58-60 us on global ones (profiles/r05/r05f_rocprof_c2_kernel_stats.csv,
// r05i_rocprof_c2_kernel_stats.csv).  The subtraction order is gmres_solve_kernel's (m
// descending), so a merged cycle end and the separate solve agree to rounding.
__global__ void cycle_coef_kernel(GivensState g, int col, double2* ab) {
  __shared__ double2 sH[(kFusedMaxK + 1) * (kFusedMaxK + 2)];  // H(c, k), c <= col, k <= col + 1
  __shared__ double2 sG[2 * (kFusedMaxK + 1)];
  if (g.ctrl[0]) return;  // (the cycle stopped before its last column)
  const int R1 = g.restart + 1;
  const int lane = threadIdx.x, me = min(lane, col);
  for (int e = lane; e < (col + 1) * R1; e += kWave) sH[e] = g.H[e];
  for (int e = lane; e < 2 * col; e += kWave) sG[e] = g.G[e];
  const double2 s0 = g.S[me];
  const double sv = g.vscale[me];
  __syncthreads();
  auto H = [&](int c, int k) { return sH[c * R1 + k]; };
  // column col's rows < col after the previous rotations (gmres_finish_column's chain)
  double2 n0 = H(col, 0), hc = make_double2(0.0, 0.0);
  for (int k = 0; k < col; ++k) {
    const double c = sG[2 * k].x;
    const double2 sk = sG[2 * k + 1], n1 = H(col, k + 1);
    const double2 v = cadd(cscale(n0, c), cmul(sk, n1));
    if (lane == k) hc = v;
    n0 = cadd(cmul(make_double2(-sk.x, sk.y), n0), cscale(n1, c));
  }
  const Smith f = smith_of(H(me, me));
  // y = a + y_col b: a solves R a = S (a_col = 0), b solves R b = -hc (b_col = 1)
  double2 sa = s0, sb = cneg(hc);
  for (int m = col - 1; m >= 0; --m) {
    if (lane == m) {
      sa = smith_apply(sa, f);
      sb = smith_apply(sb, f);
    }
    const double2 ta = rlane2(sa, m), tb = rlane2(sb, m);
    if (lane < m) {
      const double2 h = H(m, lane);
      sa = csub(sa, cmul(ta, h));
      sb = csub(sb, cmul(tb, h));
    }
  }
  if (lane <= col) {
    const bool last = lane == col;
    ab[lane] = cscale(last ? make_double2(0.0, 0.0) : sa, sv);
    ab[kMaxProj + lane] = cscale(last ? make_double2(1.0, 0.0) : sb, sv);
  }
}

// |w - sum_k c_k V_k|^2 block partials (update_kernel's coefficients and term order), x += sum
// a_k V_k in place, vb = sum b_k V_k.  Coefficients in LDS (3 K complex: registers would not
// hold them), the K loads in batches of 8.
template <int K>
__global__ __launch_bounds__(kT) void cycle_end_kernel(const double2* __restrict__ V, size_t ldv,
                                                       const double* __restrict__ raw,
                                                       const double* __restrict__ vscale,
                                                       const double2* __restrict__ ab,
                                                       const double2* w, double2* x, double2* vb,
                                                       size_t len, double* partials,
                                                       const int* stop, const PassFold fold) {
  if (stop && *stop) return;
  __shared__ double2 cu[K], ca[K], cb[K];
  const int t = threadIdx.x;
  if (t < K) {
    const double sk = vscale[t];
    cu[t] = cscale(cscale(make_double2(raw[2 * t], raw[2 * t + 1]), sk), sk);
    ca[t] = ab[t];
    cb[t] = ab[kMaxProj + t];
  }
  __syncthreads();
  double nrm = 0.0;
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t p = (size_t)blockIdx.x * kT + t; p < len; p += stride) {
    double2 u = w[p], xa = x[p], b = make_double2(0.0, 0.0);
#pragma unroll
    for (int k0 = 0; k0 < K; k0 += 8) {
      double2 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = V[(size_t)min(k0 + q, K - 1) * ldv + p];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (k0 + q < K) {
          u = csub(u, cmul(cu[k0 + q], v[q]));
          xa = cfma(ca[k0 + q], v[q], xa);
          b = cfma(cb[k0 + q], v[q], b);
        }
    }
    nrm = fma(u.x, u.x, fma(u.y, u.y, nrm));
    x[p] = xa;
    vb[p] = b;
  }
  double v1[1] = {nrm};
  if (fold.tickets) {  // one rank: the norm's reduce and the final lag step in this launch
    block_reduce_vec<1, true>(v1, partials, kMaxNorms);
    fold_reduce_lag(fold, partials, kMaxNorms, 1, true);
  } else {
    block_reduce_vec<1>(v1, partials, kMaxNorms);
  }
}

// The one-pass cycle's first dots (u_0^H w_0 and |w_0|^2: multidot_kernel<1, NT>'s loop and
// partial row, bit for bit) with the reduce and the first lag step folded in (one rank).
template <bool NT>
__global__ __launch_bounds__(kT) void cycle_start_dots_kernel(const double2* __restrict__ V,
                                                              const double2* __restrict__ w,
                                                              size_t len, double* partials,
                                                              const int* stop,
                                                              const PassFold fold) {
  if (stop && *stop) return;
  double2 acc = make_double2(0.0, 0.0);
  double nrm = 0.0;
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t p = (size_t)blockIdx.x * kT + threadIdx.x; p < len; p += stride) {
    const double2 wv = w[p];
    nrm = fma(wv.x, wv.x, fma(wv.y, wv.y, nrm));
    const double2 vv = NT ? make_double2(__builtin_nontemporal_load(&V[p].x),
                                         __builtin_nontemporal_load(&V[p].y))
                          : V[p];
    acc = cfma_conj(vv, wv, acc);
  }
  double v[3] = {acc.x, acc.y, nrm};
  block_reduce_vec<3, true>(v, partials, 4);
  fold_reduce_lag(fold, partials, 4, 3, false);
}

// x += y_col vb once column col is finished: y_col = S[col] / H[col][col] (scipy's rule: S[col]
// = 0 when H[col][col] == 0, iterative.py:815-816)
// (a cycle that stopped before its last column col takes the solve + xupdate instead: decided
// here, from the last column it executed, so the host need not read it first)
// Its first block also does gmres_solve_kernel's work (the merged form, one launch fewer per
// cycle): ctl[2] raised when the cycle reached `col` (xupdate_kernel then skips), else the
// triangular solve of the columns it executed.
__global__ __launch_bounds__(kT) void cycle_finish_kernel(GivensState g, int col,
                                                          const double2* vb, double2* x,
                                                          size_t len) {
  __shared__ double2 sH[(kMaxProj + 1) * (kMaxProj + 2)];
  const int c1 = g.ctrl[1];
  if (blockIdx.x == 0) {
    const int cs = min(max(c1, 0), col);  // (gmres_solve_kernel's column)
    const bool skip = cs == col;
    if (threadIdx.x == 0) g.ctrl[2] = skip;
    if (!skip) {
      const int R1 = g.restart + 1;
      for (int e = threadIdx.x; e < (cs + 1) * R1; e += kT) sH[e] = g.H[e];
      __syncthreads();
      if (threadIdx.x < kWave) givens::solve_columns_wave(g, cs, sH);
      return;
    }
  }
  if (c1 != col) return;
  const int R1 = g.restart + 1;
  const double2 hcc = g.H[(size_t)col * R1 + col];
  const double2 sc = g.S[col];
  const double2 y = (hcc.x == 0.0 && hcc.y == 0.0) ? make_double2(0.0, 0.0) : cdiv_smith(sc, hcc);
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t p = (size_t)blockIdx.x * kT + threadIdx.x; p < len; p += stride)
    x[p] = cfma(y, vb[p], x[p]);
}

template <int K>
void cycle_end_launch(const double2* V, size_t ldv, const double* raw, const double* vscale,
                      const double2* ab, const double2* w, double2* x, double2* vb, size_t len,
                      double* partials, int blocks, hipStream_t s, const int* stop,
                      const PassFold& fold) {
  hipLaunchKernelGGL((cycle_end_kernel<K>), dim3(blocks), dim3(kT), 0, s, V, ldv, raw, vscale,
                     ab, w, x, vb, len, partials, stop, fold);
}
template <int... Ks>
struct CTable {
  using FN = void (*)(const double2*, size_t, const double*, const double*, const double2*,
                      const double2*, double2*, double2*, size_t, double*, int, hipStream_t,
                      const int*, const PassFold&);
  static constexpr FN f[] = {cycle_end_launch<Ks>...};
};
using CycleTable = CTable<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21>;

// basis vectors whose re-read comes from the LDS copy: HH_FUSED_KEEP = 0 turns the copy off
// (every re-read from the memory system), 17 (= kFusedKeepDefault, the only kept count built)
// keeps it; any other value is refused when the knobs are read (knobs.cpp).
int fused_keep() { return (int)knobs().fused_keep; }
template <int K>
void fused_launch(const FusedArgs& a, int blocks, hipStream_t s) {
  if (a.sl) {
    if (a.invc2)
      hipLaunchKernelGGL((fused_sl_iter_kernel<K, false>), dim3(blocks), dim3(kT), 0, s, a);
    else
      hipLaunchKernelGGL((fused_sl_iter_kernel<K, true>), dim3(blocks), dim3(kT), 0, s, a);
    return;
  }
  if (fused_keep() > 0) {
    if (a.invc2)
      hipLaunchKernelGGL((fused_iter_kernel<K, false, kFusedKeepDefault>), dim3(blocks), dim3(kT),
                         0, s, a);
    else
      hipLaunchKernelGGL((fused_iter_kernel<K, true, kFusedKeepDefault>), dim3(blocks), dim3(kT),
                         0, s, a);
  } else {
    if (a.invc2)
      hipLaunchKernelGGL((fused_iter_kernel<K, false, 0>), dim3(blocks), dim3(kT), 0, s, a);
    else
      hipLaunchKernelGGL((fused_iter_kernel<K, true, 0>), dim3(blocks), dim3(kT), 0, s, a);
  }
}
template <int K>
void edge_launch(const FusedArgs& a, int r0, int c0, int r1, int c1, hipStream_t s) {
  const int tiles_x = (a.n + kT - 1) / kT;
  hipLaunchKernelGGL((fused_edge_kernel<K>), dim3(tiles_x * (c0 + c1)), dim3(kT), 0, s, a, r0,
                     c0, r1);
}
template <int... Ks>
struct FTable {
  using FN = void (*)(const FusedArgs&, int, hipStream_t);
  using EN = void (*)(const FusedArgs&, int, int, int, int, hipStream_t);
  static constexpr FN f[] = {fused_launch<Ks>...};
  static constexpr EN e[] = {edge_launch<Ks>...};
};
using FusedTable = FTable<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20>;
static_assert(kFusedMaxK == 20, "table covers 1..kFusedMaxK");

}  // namespace

// HH_FUSED_ALT=0 turns the alternating march off (A/B; on by default -- config 2: +3.6 %,
// profiles/r05/r05b_ab_alt.log)
bool fused_alt_dir() { return knobs().fused_alt != 0; }

// One-pass column on one rank: the partial-row reduce and the lag step in one launch
// (gmres_lag_red_kernel); HH_LAG_RED=0 keeps the two launches (A/B).
bool lag_red_merge() { return knobs().lag_red != 0; }

// Band height: 8 rows at 1024^2, 32 at 4096^2 (profiles/r03t/r03s_ab_rows*), 64 from 8192^2;
// HH_FUSED_ROWS overrides.  The partial rows (one per block) stay within kMaxStreamBlocks.
int fused_iter_rows(int n, int rows) {
  const int env = (int)knobs().fused_rows;
  const long tiles_x = (n + kT - 1) / kT;
  // (64 rows from n = 8192: 3 % fewer halo-row re-formations, +1.5 % at 8192^2,
  // profiles/r04/r04g_ab_rows_8192.log; at 4096^2 64-row bands leave too few tiles per CU)
  int R = env > 0 ? env
                  : (n >= 8192 ? 64
                               : (int)std::min<long>(32, std::max<long>(8, tiles_x * n / 1024)));
  while ((long)tiles_x * ((rows + R - 1) / R) > kMaxStreamBlocks) R *= 2;
  return R;
}
int fused_iter_blocks(int n, int bands) {
  const int T = (n + kT - 1) / kT * bands;
  return (T + 7) / 8 * 8;
}
void launch_fused_iter(int K, const FusedArgs& a, int blocks, hipStream_t stream) {
  FusedTable::f[K - 1](a, blocks, stream);
}
void launch_fused_edge(int K, const FusedArgs& a, int r0, int c0, int r1, int c1,
                       hipStream_t stream) {
  if (c0 + c1 > 0) FusedTable::e[K - 1](a, r0, c0, r1, c1, stream);
}
void launch_cycle_coef(const GivensState& g, int col, double2* ab, hipStream_t stream) {
  hipLaunchKernelGGL(cycle_coef_kernel, dim3(1), dim3(kWave), 0, stream, g, col, ab);
}
void launch_cycle_end(int K, const double2* V, size_t ldv, const double* raw, const double* vscale,
                      const double2* ab, const double2* w, double2* x, double2* vb, size_t len,
                      double* partials, int blocks, hipStream_t stream, const int* stop,
                      const PassFold* fold) {
  const PassFold none{};
  CycleTable::f[K - 1](V, ldv, raw, vscale, ab, w, x, vb, len, partials, blocks, stream, stop,
                       fold ? *fold : none);
}
void launch_cycle_start_dots(const double2* V, const double2* w, size_t len, double* partials,
                             int blocks, bool nt, hipStream_t stream, const int* stop,
                             const PassFold& fold) {
  if (nt)
    hipLaunchKernelGGL((cycle_start_dots_kernel<true>), dim3(blocks), dim3(kT), 0, stream, V, w,
                       len, partials, stop, fold);
  else
    hipLaunchKernelGGL((cycle_start_dots_kernel<false>), dim3(blocks), dim3(kT), 0, stream, V, w,
                       len, partials, stop, fold);
}
void launch_cycle_finish(const GivensState& g, int col, const double2* vb, double2* x, size_t len,
                         int blocks, hipStream_t stream) {
  hipLaunchKernelGGL(cycle_finish_kernel, dim3(blocks), dim3(kT), 0, stream, g, col, vb, x, len);
}

}  // namespace hh
