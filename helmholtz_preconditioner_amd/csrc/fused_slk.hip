// The one-pass GMRES iteration with the two-sweep shifted-Laplace M, with the whole
// basis window its projections re-read kept on chip: one 256-thread block per CU, up to 512
// registers per lane (VGPRs + AGPRs) and all of the CU's LDS.
//
// Replaces, per inner iteration of scipy.sparse.linalg.gmres (scipy 1.15.3
// _isolve/iterative.py:748-800, which code.py:516 runs with M = code.py:510-511's slot): the
// orthogonalisation's axpy loop, the next psolve(matvec(v)) and the next np.vdot projections --
// the same pass as fused.hip fused_sl_iter_kernel, bit for bit (same tiles, same arithmetic, same
// accumulation order); what differs is where the projections' basis rows come from.
//
// The projections of row r run two steps after the update loaded the basis row r (w on row r
// needs u_K two rows further), so rows r, r + 1, r + 2 of every basis vector must stay on chip.
// fused_sl_iter_kernel (two blocks per CU) keeps 5 vectors in a three-row LDS ring and re-reads
// the rest: 1.83x its algorithmic bytes at K = 19 (profiles/r04_pmc_fused.json).  Here:
//   * the first KS = min(K, 11) vectors: a three-row LDS ring (3 x 11 x 4 KiB = 132 KiB);
//   * the rest (K = 12 .. 20: up to 9 vectors): a four-slot register ring (rows L - 2 .. L and
//     the row L + 1 in flight), the slot of a row fixed by the step's position in a four-step
//     unrolled loop (no register copies: copying a register an in-flight load targets drains it);
//   * every load of row L + 1 -- w_{K-1}, the K basis rows, 1/c^2, the edge columns -- is issued
//     right after row L's update consumed the previous ones, so one row's memory round trip
//     overlaps the stencil, second sweep and projections of the step (a one-block-per-CU kernel
//     has no second block to hide it);
//   * one band per CU where the grid allows (256 tiles at 4096^2: 256-row bands), so the four
//     halo rows a band re-forms cost 1.6 % instead of 12.5 % (32-row bands).
// A band runs a multiple of four steps; the steps past its last row recompute the last row's
// values (clamped rows) and store nothing.
#include <algorithm>
#include <cstddef>
#include <cstdlib>

#include "hh_internal.hpp"
#include "hh_complex.hpp"
#include "hh_wave.hpp"
#include "hh_fused.hpp"

namespace hh {
namespace {
using namespace fusedk;

// vectors kept in the three-row LDS ring (HH_SLK_LDS at build time for A/B builds)
#ifndef HH_SLK_LDS
#define HH_SLK_LDS 11
#endif
constexpr int kLdsKeep = HH_SLK_LDS;

template <int K, bool CONSTC>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(1, 1)))
void fused_slk_kernel(const FusedArgs a) {
  if (a.stop && *a.stop) return;
  constexpr int KS = K < kLdsKeep ? K : kLdsKeep;  // LDS ring
  constexpr int KR = K - KS;                       // register ring
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
  // The strip's two edge columns, W: i0-1 (outer i0-2, inner i0 = LDS slot 1) and E: i0+kT
  // (outer i0+kT+1, inner i0+kT-1 = LDS slot kT), take work from all four waves: waves 0 (W)
  // and 3 (E) form u_K at (L, edge) and (L-1, outer) by lane-parallel sums before the row's
  // barrier and publish them in LDS; waves 1 (W) and 2 (E) form the edge column's T and z1
  // after it.  (fused_sl_iter_kernel keeps both on waves 0 and 3, whose extra ~130 instructions
  // per step the other waves then waited for at every barrier -- at one wave per SIMD that idle
  // time is the SIMD's.)  The same values by the same arithmetic.
  const bool west = wv < 2;                           // this wave's side
  const bool eu = wv == 0 || wv == 3, ez = wv == 1 || wv == 2;
  const int ie_raw = west ? i0 - 1 : i0 + kT, io_raw = west ? i0 - 2 : i0 + kT + 1;
  const bool ehas = ie_raw >= 0 && ie_raw < n;
  const bool ohas = io_raw >= 0 && io_raw < n;
  const int ie = min(max(ie_raw, 0), n - 1), io = min(max(io_raw, 0), n - 1);
  const int islot = west ? 1 : kT;  // LDS slot of the edge column's inner neighbour
  const int eslot = west ? 0 : kT + 1;  // LDS slot of the edge column
  __shared__ double2 eus[2][2][2];  // [buf][side][u_K(L, edge), u_K(L-1, outer)]
  load_coef<K>(a, coef);
  __syncthreads();
  const double sin = *a.sin;
  const double damp = a.damping;
  const double2 mshift = a.mshift;
  const double2 z = make_double2(0.0, 0.0);
  int kz = 0;  // opaque zero (coefficient reads stay in the loop: registers)
  // the column tables of the own and the edge column (loop-invariant)
  const double2 AWo = a.tab_i[ic], AEo = a.tab_i[n + ic], R1o = a.tab_i[2 * n + ic];
  const double2 AWe = a.tab_i[ie], AEe = a.tab_i[n + ie], R1e = a.tab_i[2 * n + ie];
  struct Co {
    double2 W, E, S, N, D, Db;
  };
  // the operator's coefficients at row r (clamped to the slab's tables), column tables given
  // (stencil.hip's expressions and order)
  auto coefs = [&](int r, double2 AW, double2 AE, double2 R1, double icv) {
    const cdouble_p q = crow(a.tab_j, min(max(r, -2), nl + 1));
    const double2 R2 = make_double2(q[0], q[1]), BS = make_double2(q[2], q[3]);
    const double2 BN = make_double2(q[4], q[5]), OM = make_double2(q[6], q[7]);
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
  auto on_grid = [&](int r) {
    return (r >= 0 && r < nl) || (r < 0 && a.lo_mode != FROW_ZERO) ||
           (r >= nl && a.hi_mode != FROW_ZERO);
  };
  // u_K of a row outside the slab (rows -2, -1 and nl, nl + 1): received from the neighbour
  // rank (FROW_HALO) or zero (FROW_ZERO) -- fused.hip row_value as selects over a value loaded
  // unconditionally with the row's other loads (a load under a branch makes every later use
  // of any load wait for all of them: vmcnt(0) at the join)
  const bool lo_halo = a.lo_mode == FROW_HALO, hi_halo = a.hi_mode == FROW_HALO;
  const double2* h_lo = lo_halo ? a.halo_lo : a.win;  // (a valid address either way)
  const double2* h_hi = hi_halo ? a.halo_hi : a.win;
  auto halo_ld = [&](int r, int col) {
    const bool lo = r < 0;
    const double2* base = lo ? h_lo : h_hi;
    const int idx = lo ? min(max(r + 2, 0), 1) : min(max(r - nl, 0), 1);
    return base[(size_t)idx * n + col];
  };
  auto row_sel = [&](int r, double2 formed, double2 hv) {
    const bool halo = r < 0 ? lo_halo : hi_halo;
    return csel(r >= rlo && r < rhi, formed, csel(halo, hv, z));
  };
  // ---- the loads of one row (issued a step ahead; all unconditional)
  double2 pw, pv[KS];                      // w_{K-1} and the LDS-ring vectors of row L
  double2 rg[4][KR > 0 ? KR : 1];          // register ring: rows (slot = step mod 4)
  double pic[2], pice[2];                  // 1/c^2 of row L - 1 (own, edge column), by parity
  double2 pe_w = z, pe_v = z;              // edge waves: w and c_k u_k terms (unew2)
  double2 ph = z, peh = z;                 // halo values of the own point and the edge point
  auto issue = [&](int L, int s_ring, int s_par) {
    const int Lc = min(L, re + 1);
    // first the edge terms (fused.hip unew2: the other waves load the same in-cache addresses,
    // so no load sits under a branch) and the halo values -- the loads a step waits for last
    // are then the row's basis, and no wait for them also waits for the step's stores
    {
      const int h = lane >> 5, k = lane & 31;
      const int r = h ? Lc - 1 : Lc, c = h ? io : ie;
      const int rr = min(max(r, rlo), rhi - 1);
      const ptrdiff_t p = (ptrdiff_t)rr * n + c;
      pe_w = a.win[p];
      pe_v = (a.V + p)[(size_t)min(k, K - 1) * a.ldv];
      peh = halo_ld(r, c);
    }
    pice[s_par] = icv_at(Lc - 1, ie);
    pic[s_par] = icv_at(Lc - 1, ic);
    ph = halo_ld(Lc, ic);
    const int rc = min(max(L, rlo), rhi - 1);
    gd2* vrow = gptr(a.V + (ptrdiff_t)rc * n);
    gd2* wrow = gptr(a.win + (ptrdiff_t)rc * n);
    asm volatile("" : "+s"(vrow), "+s"(wrow));
    const unsigned bo = (unsigned)ic * (unsigned)sizeof(double2);
    pw = ld_at(wrow, bo);
#pragma unroll
    for (int q = 0; q < KS; ++q) pv[q] = ld_at(vrow + (size_t)q * a.ldv, bo);
#pragma unroll
    for (int q = 0; q < KR; ++q) rg[s_ring][q] = ld_at(vrow + (size_t)(KS + q) * a.ldv, bo);
  };
  double2 acc[K + 1];
#pragma unroll
  for (int k = 0; k <= K; ++k) acc[k] = z;
  double nw = 0.0, nu = 0.0;
  if (bd.live) {
    double2 uP = z, uC = z, Tm = z, z1a = z, z1b = z;
    double2 euP = z, euC = z, ez1b = z;
    double2 Dbm = make_double2(1.0, 0.0);
    double invm = 1.0;
    double2 Wm = z, Em = z, Sm = z, Nm = z;
    int buf = 0;
    // row r's w_K and u_K are stored one step later, before that step's prefetch: a store
    // issued between the prefetch and its use (under the branch that skips rows outside the
    // band) made the compiler wait for every load at the next use (vmcnt(0) at the join)
    double2 sw = z, su = z;
    int sr = -1;  // (uniform) the row pending, or -1
    issue(rb - 2, 0, 0);
    for (int L0 = rb - 2; L0 <= re + 1; L0 += 4) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        int L = L0 + s;
        asm volatile("" : "+s"(L), "+s"(kz));
        const bool real = L <= re + 1;  // (block-uniform)
        const int Lc = min(L, re + 1);
        // u_K on row L, own column: w_{K-1} - sum_k c_k u_k in k order
        double2 uN;
        {
          double2 w = pw;
#pragma unroll
          for (int q0 = 0; q0 < K; q0 += 4) {
            double2 c[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) c[q] = coef[min(q0 + q, K - 1) + kz];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int k = q0 + q;
              if (k < KS) w = csub(w, cmul(c[q], pv[k < KS ? k : 0]));
              else if (k < K) w = csub(w, cmul(c[q], rg[s][k - KS < KR ? k - KS : 0]));
            }
          }
          asm volatile("" : "+v"(w.x), "+v"(w.y));
          uN = row_sel(Lc, w, ph);
        }
        {
          const int slot = (Lc % 3 + 3) % 3;
#pragma unroll
          for (int q = 0; q < KS; ++q) vkeep[slot][q][t] = pv[q];
        }
        if (sr >= 0 && act) {  // (the last step's row)
          const size_t p = (size_t)sr * n + ic;
          a.wout[p] = sw;
          a.uout[p] = su;
        }
        sr = -1;
        // waves 0 / 3: u_K at (L, ie) and (L - 1, io), the terms summed across the half-waves
        double2 euN = z, eo = z;
        if (eu) {
          const int k = lane & 31;
          const double2 tk = half_sum2(csel(k < K, cmul(coef[min(k, K - 1)], pe_v), z));
          const double2 ua = rlane2(tk, 0), ub = rlane2(tk, 32);
          const double2 wa = rlane2(pe_w, 0), wb = rlane2(pe_w, 32);
          const double2 ha = rlane2(peh, 0), hb = rlane2(peh, 32);
          euN = csel(ehas, row_sel(Lc, csub(wa, ua), ha), z);
          eo = csel(ohas, row_sel(Lc - 1, csub(wb, ub), hb), z);
        }
        // row L + 1's loads, in flight during the rest of the step
        issue(L + 1, (s + 1) & 3, (s + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
        urow[buf][1 + t] = csel(act, uC, z);
        zrow[buf][1 + t] = csel(act, z1b, z);
        if (eu && lane == 0) {
          urow[buf][eslot] = euC;
          eus[buf][west ? 0 : 1][0] = euN;
          eus[buf][west ? 0 : 1][1] = eo;
        }
        if (ez && lane == 0) zrow[buf][eslot] = ez1b;
        __syncthreads();
        const double2 uW = urow[buf][t], uE = urow[buf][t + 2];
        const double2 zW = zrow[buf][t], zE = zrow[buf][t + 2];
        const bool v1 = on_grid(Lc - 1);
        // T and z1 on row L-1 (own column)
        const Co c1 = coefs(Lc - 1, AWo, AEo, R1o, pic[s & 1]);
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
        // waves 1 / 2: the same at the edge column (broadcast values; u_K of the edge and outer
        // columns from waves 0 / 3 through LDS)
        double2 ez1c = z;
        if (ez) {
          euN = eus[buf][west ? 0 : 1][0];
          eo = eus[buf][west ? 0 : 1][1];
          const double2 uin = urow[buf][islot];
          const double2 eW = west ? eo : uin, eE = west ? uin : eo;
          const Co ce = coefs(Lc - 1, AWe, AEe, R1e, pice[s & 1]);
          double2 Ae = cmul(ce.S, euP);
          Ae = cfma(ce.W, eW, Ae);
          Ae = cfma(ce.D, euC, Ae);
          Ae = cfma(ce.E, eE, Ae);
          Ae = cfma(ce.N, euN, Ae);
          const double2 eT = cscale(Ae, sin);
          ez1c = csel(ehas && v1, cscale(cdiv(eT, ce.Db), damp), z);
        }
        // w on row r = L-2: the second sweep (A_beta on z1), row r's W, E, S, N, D_beta and
        // 1/|D_beta|^2 carried from the last step
        const int r = Lc - 2;
        if (real && r >= rb && r < re) {  // (block-uniform)
          double2 Az = cmul(Sm, z1a);
          Az = cfma(Wm, zW, Az);
          Az = cfma(Dbm, z1b, Az);
          Az = cfma(Em, zE, Az);
          Az = cfma(Nm, z1c, Az);
          const double2 w = csel(act, cadd(z1b, cscale(cdivr(csub(Tm, Az), Dbm, invm), damp)), z);
          sw = w;
          su = uP;
          sr = r;
          const double2 uo = csel(act, uP, z);
          nu = fma(uo.x, uo.x, fma(uo.y, uo.y, nu));
          nw = fma(w.x, w.x, fma(w.y, w.y, nw));
          const int slot = r % 3;  // (r >= 0)
#pragma unroll
          for (int k = 0; k < KS; ++k) acc[k] = cfma_conj(vkeep[slot][k][t], w, acc[k]);
#pragma unroll
          for (int q = 0; q < KR; ++q) acc[KS + q] = cfma_conj(rg[(s + 2) & 3][q], w, acc[KS + q]);
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
        Wm = c1.W;
        Em = c1.E;
        Sm = c1.S;
        Nm = c1.N;
        buf ^= 1;
      }
    }
    if (sr >= 0 && act) {
      const size_t p = (size_t)sr * n + ic;
      a.wout[p] = sw;
      a.uout[p] = su;
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

template <int K>
void slk_launch(const FusedArgs& a, int blocks, hipStream_t s) {
  if (a.invc2)
    hipLaunchKernelGGL((fused_slk_kernel<K, false>), dim3(blocks), dim3(kT), 0, s, a);
  else
    hipLaunchKernelGGL((fused_slk_kernel<K, true>), dim3(blocks), dim3(kT), 0, s, a);
}
template <int... Ks>
struct STable {
  using FN = void (*)(const FusedArgs&, int, hipStream_t);
  static constexpr FN f[] = {slk_launch<Ks>...};
};
using SlkTable = STable<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20>;
static_assert(kFusedMaxK == 20, "table covers 1..kFusedMaxK");

}  // namespace

// HH_SLK (knobs.cpp): the smallest K that takes this kernel (0 = never).  Default 2: at K = 1
// (two vectors) fused_sl_iter_kernel's two blocks per CU win, 336 vs 412 us at 4096^2; from
// K = 4 this kernel does, 478 vs 493 us ... 1240 vs 1862 us at K = 19
// (profiles/r05/r05e_slk0_tbps.txt, r05e_slk1_tbps.txt)
int fused_slk_min_k() {
  return (int)knobs().slk_min_k;
}
bool fused_slk_use(int K) {
  const int m = fused_slk_min_k();
  return m > 0 && K >= m;
}
// Band height: one band per CU where the grid allows (tiles_x * bands <= 256), at least 16
// rows; HH_SLK_ROWS overrides.
int fused_slk_rows(int n, int rows) {
  const int env = (int)knobs().slk_rows;
  const long tiles_x = (n + kT - 1) / kT;
  const long bands = std::max<long>(1, 256 / tiles_x);
  int R = env > 0 ? env : (int)std::max<long>(16, (rows + bands - 1) / bands);
  while (tiles_x * ((rows + R - 1) / R) > kMaxStreamBlocks) R *= 2;
  return R;
}
void launch_fused_slk(int K, const FusedArgs& a, int blocks, hipStream_t stream) {
  SlkTable::f[K - 1](a, blocks, stream);
}

}  // namespace hh
