// Fused shifted-Laplace preconditioned operator apply, w = M A v, for gfx950 (MI355X).
//
// M is two damped-Jacobi sweeps on the shifted operator A_beta (the build's BASELINE config-3
// preconditioner; A_beta = build_A_matrix(..., c_mat / sqrt(1 + i beta)), code.py:202-219):
//   T  = A v                                   (stencil, unshifted diagonal D)
//   z1 = damp T / Db                           (first sweep from z0 = 0)
//   w  = z1 + damp (T - A_beta z1) / Db        (second sweep)
// Unfused this is two stencil launches (EPI_SL_FIRST writes T and z1, EPI_SL_SWEEP reads them
// back): 56 + 56 B per unknown.  Here one launch marches each tile's rows with the second
// sweep one row behind the first, so T and z1 live only in registers and LDS: 40 B per unknown
// (v 16 + 1/c^2 8 + w 16), the plain apply's traffic.
//
// Shape: as stencil.hip's marching tile (XCD-aware band map, register rings, unconditional
// clamped loads), with two changes.  (1) The second sweep needs z1 one row above and below,
// so every band also computes the first sweep on its two halo rows (rows rb-1 and re; v rows
// rb-2 .. re+1) -- for a band at a slab edge that is the neighbouring slab's (or rank's)
// boundary row, with its 1/c^2 and PML tables (two halo rows per side, runtime.cpp run_sl2);
// z1 vanishes only off the grid.  (2) It needs z1 one column to each side, so strips overlap:
// a block of TPB threads computes the first sweep on TPB columns and writes w on the TPB-2
// inner ones.  The arithmetic is stencil.hip's, term for term (coefficients, FMA order), so w
// is bit-identical to the two-launch path on any slab decomposition.
#include "hh_internal.hpp"
#include "hh_complex.hpp"
#include "hh_stencil9.hpp"
#include "hh_wave.hpp"

#include <algorithm>
#include <type_traits>

namespace hh {
namespace {

using cdouble_p = const __attribute__((address_space(4))) double*;

template <int K, int N, class F>
__device__ __forceinline__ void unroll(F&& f) {
  if constexpr (K < N) {
    f(std::integral_constant<int, K>{});
    unroll<K + 1, N>(f);
  }
}

// by-value select: `c ? arr[q].e : z` on an lvalue compiles to a select of stack addresses
// (the whole ring then lives in scratch)
__device__ __forceinline__ double2 csel(bool c, double2 a, double2 b) {
  return make_double2(c ? a.x : b.x, c ? a.y : b.y);
}

struct RowTab {
  double2 R2, BS, BN, OM;
};
struct RowIn {
  double ic;
  double2 e;  // v at this strip's halo columns (lanes 0-31: i0-2, lanes 32-63: i0+TPB-1)
  double2 b;  // (sl2_res_kernel) b at the lane's column
};

template <bool CONSTC, bool NTU, int TPB>
__device__ __forceinline__ void sl2_tile(const StencilArgs& a, const int t) {
  constexpr int WO = TPB - 2;  // output columns per strip
  __shared__ double2 lv[2][TPB + 2];
  __shared__ double2 lz[TPB + 2];
  const int tx = t % a.tiles_x;
  const int ty = t / a.tiles_x;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int n = a.n, nl = a.nl;
  const int i0 = tx * WO;
  const int c = i0 + tid - 1;  // this lane's column
  const bool cin = c >= 0 && c < n;
  const int cc = min(max(c, 0), n - 1);
  const bool outl = tid >= 1 && tid <= TPB - 2 && cin;
  const int rb = __builtin_amdgcn_readfirstlane(a.row_begin + ty * a.row_step);
  const int re = __builtin_amdgcn_readfirstlane(min(rb + a.rows_per_block, a.row_end));
  int ie = lane < kWave / 2 ? i0 - 2 : i0 + TPB - 1;
  const bool lw = tid == 0 && i0 - 2 >= 0;
  const bool le = tid == TPB - 1 && i0 + TPB - 1 < n;
  ie = min(max(ie, 0), n - 1);
  const double2 z2 = make_double2(0.0, 0.0);

  // rows -2 .. nl+1: two halo rows on each side (StencilArgs, fused SL fields)
  auto rowp = [&](int r) -> const double2* {
    return r < 0 ? a.halo_lo + (size_t)(r + 2) * n
                 : (r >= nl ? a.halo_hi + (size_t)(r - nl) * n : a.u + (size_t)r * n);
  };
  auto load_v = [&](int r) -> double2 {
    const double2* p = rowp(r) + cc;
    if constexpr (NTU)
      return make_double2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
    else
      return *p;
  };
  auto load_in = [&](int r, RowIn& v) {
    if constexpr (!CONSTC) {
      const double* q = r < 0 ? a.invc2_halo + (size_t)(r + 2) * n
                              : (r >= nl ? a.invc2_halo + (size_t)(r - nl + 2) * n
                                         : a.invc2 + (size_t)r * n);
      v.ic = __builtin_nontemporal_load(q + cc);
    } else {
      v.ic = a.invc2_const;
    }
    v.e = rowp(r)[ie];
  };
  const cdouble_p tabj = (cdouble_p)(a.tab_j);
  auto load_tab = [&](int r, RowTab& tb) {
    const int ru = __builtin_amdgcn_readfirstlane(min(max(r, -2), nl + 1));  // tab_j_ext rows
    const cdouble_p q = tabj + 8 * ru;
    tb.R2 = make_double2(q[0], q[1]);
    tb.BS = make_double2(q[2], q[3]);
    tb.BN = make_double2(q[4], q[5]);
    tb.OM = make_double2(q[6], q[7]);
  };
  const double2 AW = a.tab_i[cc], AE = a.tab_i[n + cc], R1 = a.tab_i[2 * n + cc];
  const double sin = a.in_scale ? *a.in_scale : 1.0;

  // first sweep on row s: T = s A v, z1 = damp T / Db (zero off the slab and off the grid)
  auto stage1 = [&](int s, int buf, double2 uS, double2 uC, double2 uN, const RowIn& in,
                    const RowTab& tb, double2& T, double2& z1) __attribute__((always_inline)) {
    double2* l = lv[buf];
    l[tid + 1] = csel(cin, uC, z2);
    if (tid == 0) l[0] = csel(lw, in.e, z2);
    if (tid == TPB - 1) l[TPB + 1] = csel(le, in.e, z2);
    __syncthreads();
    const double2 uW = l[tid], uE = l[tid + 2];
    const double2 W = cmul(AW, tb.R2);
    const double2 E = cmul(AE, tb.R2);
    const double2 S = cmul(tb.BS, R1);
    const double2 N = cmul(tb.BN, R1);
    const double2 M = cscale(cmul(tb.OM, R1), in.ic);
    const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
    const double2 D = csub(M, sum4);
    const double2 Db = csub(cmul(M, a.mshift), sum4);
    double2 Au = cmul(S, uS);
    Au = cfma(W, uW, Au);
    Au = cfma(D, uC, Au);
    Au = cfma(E, uE, Au);
    Au = cfma(N, uN, Au);
    T = cscale(Au, sin);
    z1 = csel(cin && a.j0 + s >= 0 && a.j0 + s < n, cscale(cdiv(T, Db), a.damping), z2);
  };
  // second sweep on row r: w = z1 + damp (T - A_beta z1) / Db
  auto stage2 = [&](double2 zS, double2 zC, double2 zN, double2 T, const RowIn& in,
                    const RowTab& tb) __attribute__((always_inline)) -> double2 {
    lz[tid + 1] = zC;
    __syncthreads();
    const double2 zW = lz[tid], zE = lz[tid + 2];
    const double2 W = cmul(AW, tb.R2);
    const double2 E = cmul(AE, tb.R2);
    const double2 S = cmul(tb.BS, R1);
    const double2 N = cmul(tb.BN, R1);
    const double2 M = cscale(cmul(tb.OM, R1), in.ic);
    const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
    const double2 Db = csub(cmul(M, a.mshift), sum4);
    double2 Au = cmul(S, zS);
    Au = cfma(W, zW, Au);
    Au = cfma(Db, zC, Au);
    Au = cfma(E, zE, Au);
    Au = cfma(N, zN, Au);
    return cadd(zC, cscale(cdiv(csub(T, Au), Db), a.damping));
  };

  // Rings of four, slot(row) = (row - rb + 2) & 3: v rows r .. r+2 (+ r+3 in flight), z1 rows
  // r-1 .. r+1, T rows r, r+1, the row inputs of rows r .. r+2.
  double2 V[4], Z[4], TT[4];
  RowIn IN[4];
  RowTab TB[4];
  if (tid == 0) lz[0] = z2;  // never-written halo slots of the z1 row (their lanes store
  if (tid == 0) lz[TPB + 1] = z2;  // nothing; keep the reads defined)
  V[0] = load_v(rb - 2);
  V[1] = load_v(rb - 1);
  V[2] = load_v(rb);
  V[3] = load_v(rb + 1);
  load_in(rb - 1, IN[1]);
  load_in(rb, IN[2]);
  load_in(rb + 1, IN[3]);
  load_tab(rb - 1, TB[1]);
  load_tab(rb, TB[2]);
  load_tab(rb + 1, TB[3]);
  stage1(rb - 1, 1, V[0], V[1], V[2], IN[1], TB[1], TT[1], Z[1]);
  V[0] = load_v(rb + 2);
  stage1(rb, 0, V[1], V[2], V[3], IN[2], TB[2], TT[2], Z[2]);

  for (int r0 = rb; r0 < re; r0 += 4) {
    unroll<0, 4>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const int r = r0 + k;
      const bool live = r < re;  // uniform; steps past the band end keep the rings going
      V[(k + 1) & 3] = load_v(min(r + 3, re + 1));
      load_in(min(r + 2, re), IN[k & 3]);
      load_tab(min(r + 2, re), TB[k & 3]);
      stage1(r + 1, (k + 1) & 1, V[(k + 2) & 3], V[(k + 3) & 3], V[k & 3], IN[(k + 3) & 3],
             TB[(k + 3) & 3], TT[(k + 3) & 3], Z[(k + 3) & 3]);
      const double2 w = stage2(Z[(k + 1) & 3], Z[(k + 2) & 3], Z[(k + 3) & 3], TT[(k + 2) & 3],
                               IN[(k + 2) & 3], TB[(k + 2) & 3]);
      if (outl && live) {
        double2* p = a.out0 + (size_t)r * n + c;
        __builtin_nontemporal_store(w.x, &p->x);
        __builtin_nontemporal_store(w.y, &p->y);
      }
    });
  }
  __syncthreads();  // LDS reuse by the block's next tile
}

// sl2_tile with ONE barrier per row instead of two.  Iteration r publishes v row r+1 (the
// first sweep's W/E input) and z1 row r (the second sweep's, computed one iteration earlier)
// into the LDS buffers of parity r, then a single barrier, then both stages.  Double buffering
// makes this safe: a thread writing parity p at iteration r+2 has passed the barrier of r+1,
// which every thread reaches only after its reads of iteration r.  Same arithmetic: bit-identical.
template <bool CONSTC, bool NTU, int TPB>
__device__ __forceinline__ void sl2_tile_1b(const StencilArgs& a, const int t) {
  constexpr int WO = TPB - 2;  // output columns per strip
  __shared__ double2 lv[2][TPB + 2];
  __shared__ double2 lz[2][TPB + 2];
  const int tx = t % a.tiles_x;
  const int ty = t / a.tiles_x;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int n = a.n, nl = a.nl;
  const int i0 = tx * WO;
  const int c = i0 + tid - 1;  // this lane's column
  const bool cin = c >= 0 && c < n;
  const int cc = min(max(c, 0), n - 1);
  const bool outl = tid >= 1 && tid <= TPB - 2 && cin;
  const int rb = __builtin_amdgcn_readfirstlane(a.row_begin + ty * a.row_step);
  const int re = __builtin_amdgcn_readfirstlane(min(rb + a.rows_per_block, a.row_end));
  int ie = lane < kWave / 2 ? i0 - 2 : i0 + TPB - 1;
  const bool lw = tid == 0 && i0 - 2 >= 0;
  const bool le = tid == TPB - 1 && i0 + TPB - 1 < n;
  ie = min(max(ie, 0), n - 1);
  const double2 z2 = make_double2(0.0, 0.0);

  auto rowp = [&](int r) -> const double2* {
    return r < 0 ? a.halo_lo + (size_t)(r + 2) * n
                 : (r >= nl ? a.halo_hi + (size_t)(r - nl) * n : a.u + (size_t)r * n);
  };
  auto load_v = [&](int r) -> double2 {
    const double2* p = rowp(r) + cc;
    if constexpr (NTU)
      return make_double2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
    else
      return *p;
  };
  auto load_in = [&](int r, RowIn& v) {
    if constexpr (!CONSTC) {
      const double* q = r < 0 ? a.invc2_halo + (size_t)(r + 2) * n
                              : (r >= nl ? a.invc2_halo + (size_t)(r - nl + 2) * n
                                         : a.invc2 + (size_t)r * n);
      v.ic = __builtin_nontemporal_load(q + cc);
    } else {
      v.ic = a.invc2_const;
    }
    v.e = rowp(r)[ie];
  };
  const cdouble_p tabj = (cdouble_p)(a.tab_j);
  auto load_tab = [&](int r, RowTab& tb) {
    const int ru = __builtin_amdgcn_readfirstlane(min(max(r, -2), nl + 1));  // tab_j_ext rows
    const cdouble_p q = tabj + 8 * ru;
    tb.R2 = make_double2(q[0], q[1]);
    tb.BS = make_double2(q[2], q[3]);
    tb.BN = make_double2(q[4], q[5]);
    tb.OM = make_double2(q[6], q[7]);
  };
  const double2 AW = a.tab_i[cc], AE = a.tab_i[n + cc], R1 = a.tab_i[2 * n + cc];
  const double sin = a.in_scale ? *a.in_scale : 1.0;

  // v row (centre + the strip's halo columns) into LDS buffer p
  auto put_v = [&](int p, double2 uC, const RowIn& in) __attribute__((always_inline)) {
    lv[p][tid + 1] = csel(cin, uC, z2);
    if (tid == 0) lv[p][0] = csel(lw, in.e, z2);
    if (tid == TPB - 1) lv[p][TPB + 1] = csel(le, in.e, z2);
  };
  // first sweep on row s from LDS buffer p (same arithmetic as sl2_tile's stage1)
  // The shifted diagonal Db of a row and the reciprocal 1/|Db|^2 of cdiv (hh_complex.hpp) are
  // formed once, by the first sweep, and kept for the second sweep on the same row one
  // iteration later: the same values cdiv would recompute, so the result is unchanged bit for
  // bit, with one IEEE division per point instead of two and no second mass term.
  auto stage1 = [&](int s, int p, double2 uS, double2 uC, double2 uN, const RowIn& in,
                    const RowTab& tb, double2& T, double2& z1, double2& Dbo, double& invo)
      __attribute__((always_inline)) {
    const double2 uW = lv[p][tid], uE = lv[p][tid + 2];
    const double2 W = cmul(AW, tb.R2);
    const double2 E = cmul(AE, tb.R2);
    const double2 S = cmul(tb.BS, R1);
    const double2 N = cmul(tb.BN, R1);
    const double2 M = cscale(cmul(tb.OM, R1), in.ic);
    const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
    const double2 D = csub(M, sum4);
    const double2 Db = csub(cmul(M, a.mshift), sum4);
    double2 Au = cmul(S, uS);
    Au = cfma(W, uW, Au);
    Au = cfma(D, uC, Au);
    Au = cfma(E, uE, Au);
    Au = cfma(N, uN, Au);
    T = cscale(Au, sin);
    const double inv = 1.0 / fma(Db.x, Db.x, Db.y * Db.y);  // = cdiv(T, Db), split
    const double2 q = make_double2(fma(T.x, Db.x, T.y * Db.y) * inv,
                                   fma(T.y, Db.x, -T.x * Db.y) * inv);
    z1 = csel(cin && a.j0 + s >= 0 && a.j0 + s < n, cscale(q, a.damping), z2);
    Dbo = Db;
    invo = inv;
  };
  auto stage2 = [&](int p, double2 zS, double2 zC, double2 zN, double2 T, double2 Db, double inv,
                    const RowTab& tb) __attribute__((always_inline)) -> double2 {
    const double2 zW = lz[p][tid], zE = lz[p][tid + 2];
    const double2 W = cmul(AW, tb.R2);
    const double2 E = cmul(AE, tb.R2);
    const double2 S = cmul(tb.BS, R1);
    const double2 N = cmul(tb.BN, R1);
    double2 Au = cmul(S, zS);
    Au = cfma(W, zW, Au);
    Au = cfma(Db, zC, Au);
    Au = cfma(E, zE, Au);
    Au = cfma(N, zN, Au);
    const double2 d = csub(T, Au);
    const double2 q = make_double2(fma(d.x, Db.x, d.y * Db.y) * inv,
                                   fma(d.y, Db.x, -d.x * Db.y) * inv);
    return cadd(zC, cscale(q, a.damping));
  };

  double2 V[4], Z[4], TT[4], DB[4];
  double INV[4];
  RowIn IN[4];
  RowTab TB[4];
  if (tid == 0) {  // z1 halo slots: never stored by a lane (outputs there are not written)
    lz[0][0] = z2;
    lz[1][0] = z2;
  }
  if (tid == TPB - 1) {
    lz[0][TPB + 1] = z2;
    lz[1][TPB + 1] = z2;
  }
  V[0] = load_v(rb - 2);
  V[1] = load_v(rb - 1);
  V[2] = load_v(rb);
  V[3] = load_v(rb + 1);
  load_in(rb - 1, IN[1]);
  load_in(rb, IN[2]);
  load_in(rb + 1, IN[3]);
  load_tab(rb - 1, TB[1]);
  load_tab(rb, TB[2]);
  load_tab(rb + 1, TB[3]);
  // prologue: first sweep on rows rb-1 (buffer 1) and rb (buffer 0), one barrier each
  put_v(1, V[1], IN[1]);
  __syncthreads();
  stage1(rb - 1, 1, V[0], V[1], V[2], IN[1], TB[1], TT[1], Z[1], DB[1], INV[1]);
  V[0] = load_v(rb + 2);
  put_v(0, V[2], IN[2]);
  __syncthreads();
  stage1(rb, 0, V[1], V[2], V[3], IN[2], TB[2], TT[2], Z[2], DB[2], INV[2]);

  for (int r0 = rb; r0 < re; r0 += 4) {
    unroll<0, 4>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      constexpr int p = (k + 1) & 1;  // parity of this iteration's buffers
      const int r = r0 + k;
      const bool live = r < re;
      V[(k + 1) & 3] = load_v(min(r + 3, re + 1));
      load_in(min(r + 2, re), IN[k & 3]);
      load_tab(min(r + 2, re), TB[k & 3]);
      put_v(p, V[(k + 3) & 3], IN[(k + 3) & 3]);  // v row r+1
      lz[p][tid + 1] = Z[(k + 2) & 3];            // z1 row r
      __syncthreads();
      stage1(r + 1, p, V[(k + 2) & 3], V[(k + 3) & 3], V[k & 3], IN[(k + 3) & 3],
             TB[(k + 3) & 3], TT[(k + 3) & 3], Z[(k + 3) & 3], DB[(k + 3) & 3], INV[(k + 3) & 3]);
      const double2 w = stage2(p, Z[(k + 1) & 3], Z[(k + 2) & 3], Z[(k + 3) & 3], TT[(k + 2) & 3],
                               DB[(k + 2) & 3], INV[(k + 2) & 3], TB[(k + 2) & 3]);
      if (outl && live) {
        double2* q = a.out0 + (size_t)r * n + c;
        __builtin_nontemporal_store(w.x, &q->x);
        __builtin_nontemporal_store(w.y, &q->y);
      }
    });
  }
  __syncthreads();  // LDS reuse by the block's next tile
}

// sl2_tile_1b with the instruction count cut (the kernel is VALU-issue-bound: ~200 vector
// instructions per point-row against ~80 for the plain stencil):
//  * the band's PML row tables (rows rb-2 .. re+1) are staged in LDS once per tile and read
//    with broadcast ds_read_b128 right before use -- no four-row ring of table values in SGPRs
//    (which spilled to VGPR lanes: ~130 v_readlane / v_writelane per four rows);
//  * Db and 1/|Db|^2 of a row come from its first sweep into the second (one division per
//    point, no second mass term) -- the values cdiv would recompute, so nothing changes;
//  * tiles whose columns and rows all lie on the grid (all but the strips at the two side
//    edges and the bands at the top / bottom of the grid) skip every mask (EDGE = false).
// Same arithmetic, term for term: bit-identical to the two-launch path.
constexpr int kSl2MaxBand = 60;  // band rows per tile for this shape (LDS table capacity)
struct Sl2Lds {  // one LDS block shared by both instantiations of sl2_tile_v2
  double2 lv[2][kStencilThreads + 2];
  double2 lz[2][kStencilThreads + 2];
  double2 ltab[kSl2MaxBand + 4][4];
};
// PF: rows of prefetch distance of the v and 1/c^2 streams (1, or 2 with rings of 8 and the
// row loop unrolled by 8): more bytes in flight per wave.
// RES (sl2_res_kernel): the first sweep's input is the residual r = b - A x instead of s A v
// (stencil.hip EPI_RES_SL's r, term for term), and acc[0] / acc[1] gather |r|^2 / |w|^2 of the
// tile's output points.
template <bool CONSTC, bool NTU, bool EDGE, int PF, bool RES = false>
__device__ __forceinline__ void sl2_tile_v2(const StencilArgs& a, const int t, Sl2Lds& L,
                                            double* acc = nullptr) {
  constexpr int RS = PF == 1 ? 4 : 8;  // ring slots: slot(row) = (row - rb + 2) % RS
  constexpr int TPB = kStencilThreads;
  constexpr int WO = TPB - 2;
  auto& lv = L.lv;
  auto& lz = L.lz;
  auto& ltab = L.ltab;
  const int tx = t % a.tiles_x;
  const int ty = t / a.tiles_x;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int n = a.n, nl = a.nl;
  const int i0 = tx * WO;
  const int c = i0 + tid - 1;
  const bool cin = !EDGE || (c >= 0 && c < n);
  const int cc = EDGE ? min(max(c, 0), n - 1) : c;
  const bool outl = tid >= 1 && tid <= TPB - 2 && cin;
  const int rb = __builtin_amdgcn_readfirstlane(a.row_begin + ty * a.row_step);
  const int re = __builtin_amdgcn_readfirstlane(min(rb + a.rows_per_block, a.row_end));
  int ie = lane < kWave / 2 ? i0 - 2 : i0 + TPB - 1;
  const bool lw = !EDGE || i0 - 2 >= 0;
  const bool le = !EDGE || i0 + TPB - 1 < n;
  if constexpr (EDGE) ie = min(max(ie, 0), n - 1);
  const double2 z2 = make_double2(0.0, 0.0);

  auto rowp = [&](int r) -> const double2* {
    return r < 0 ? a.halo_lo + (size_t)(r + 2) * n
                 : (r >= nl ? a.halo_hi + (size_t)(r - nl) * n : a.u + (size_t)r * n);
  };
  auto load_v = [&](int r) -> double2 {
    const double2* p = rowp(r) + cc;
    if constexpr (NTU)
      return make_double2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
    else
      return *p;
  };
  auto load_in = [&](int r, RowIn& v) {
    if constexpr (!CONSTC) {
      const double* q = r < 0 ? a.invc2_halo + (size_t)(r + 2) * n
                              : (r >= nl ? a.invc2_halo + (size_t)(r - nl + 2) * n
                                         : a.invc2 + (size_t)r * n);
      v.ic = __builtin_nontemporal_load(q + cc);
    } else {
      v.ic = a.invc2_const;
    }
    v.e = rowp(r)[ie];
    if constexpr (RES) {
      const double2* bp = r < 0 ? a.in1_lo + (size_t)(r + 2) * n
                                : (r >= nl ? a.in1_hi + (size_t)(r - nl) * n
                                           : a.in1 + (size_t)r * n);
      v.b = bp[cc];
    }
  };
  // PML row tables of the band (tab_j_ext rows rb-2 .. re+1) into LDS
  {
    const int cnt = (re - rb + 4) * 4;
    for (int k = tid; k < cnt; k += TPB) {
      const int rr = min(rb - 2 + k / 4, nl + 1);
      (&ltab[0][0])[k] = a.tab_j[4 * rr + (k & 3)];
    }
  }
  auto tab = [&](int r) -> const double2* { return ltab[r - rb + 2]; };
  const double2 AW = a.tab_i[cc], AE = a.tab_i[n + cc], R1 = a.tab_i[2 * n + cc];
  const double sin = a.in_scale ? *a.in_scale : 1.0;

  auto put_v = [&](int p, double2 uC, const RowIn& in) __attribute__((always_inline)) {
    lv[p][tid + 1] = EDGE ? csel(cin, uC, z2) : uC;
    if (tid == 0) lv[p][0] = EDGE ? csel(lw, in.e, z2) : in.e;
    if (tid == TPB - 1) lv[p][TPB + 1] = EDGE ? csel(le, in.e, z2) : in.e;
  };
  auto stage1 = [&](int s, int p, double2 uS, double2 uC, double2 uN, const RowIn& in,
                    double2& T, double2& z1, double2& Dbo, double& invo)
      __attribute__((always_inline)) {
    const double2* tb = tab(s);
    const double2 R2 = tb[0], BS = tb[1], BN = tb[2], OM = tb[3];
    const double2 uW = lv[p][tid], uE = lv[p][tid + 2];
    const double2 W = cmul(AW, R2);
    const double2 E = cmul(AE, R2);
    const double2 S = cmul(BS, R1);
    const double2 N = cmul(BN, R1);
    const double2 M = cscale(cmul(OM, R1), in.ic);
    const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
    const double2 D = csub(M, sum4);
    const double2 Db = csub(cmul(M, a.mshift), sum4);
    double2 Au = cmul(S, uS);
    Au = cfma(W, uW, Au);
    Au = cfma(D, uC, Au);
    Au = cfma(E, uE, Au);
    Au = cfma(N, uN, Au);
    if constexpr (RES) T = csub(in.b, Au);
    else T = cscale(Au, sin);
    const double inv = 1.0 / fma(Db.x, Db.x, Db.y * Db.y);  // = cdiv(T, Db), split
    const double2 q = cscale(make_double2(fma(T.x, Db.x, T.y * Db.y) * inv,
                                          fma(T.y, Db.x, -T.x * Db.y) * inv), a.damping);
    if constexpr (EDGE) z1 = csel(cin && a.j0 + s >= 0 && a.j0 + s < n, q, z2);
    else z1 = q;
    Dbo = Db;
    invo = inv;
  };
  auto stage2 = [&](int r, int p, double2 zS, double2 zC, double2 zN, double2 T, double2 Db,
                    double inv) __attribute__((always_inline)) -> double2 {
    const double2* tb = tab(r);
    const double2 R2 = tb[0], BS = tb[1], BN = tb[2];
    const double2 zW = lz[p][tid], zE = lz[p][tid + 2];
    const double2 W = cmul(AW, R2);
    const double2 E = cmul(AE, R2);
    const double2 S = cmul(BS, R1);
    const double2 N = cmul(BN, R1);
    double2 Au = cmul(S, zS);
    Au = cfma(W, zW, Au);
    Au = cfma(Db, zC, Au);
    Au = cfma(E, zE, Au);
    Au = cfma(N, zN, Au);
    const double2 d = csub(T, Au);
    const double2 q = make_double2(fma(d.x, Db.x, d.y * Db.y) * inv,
                                   fma(d.y, Db.x, -d.x * Db.y) * inv);
    return cadd(zC, cscale(q, a.damping));
  };

  double2 V[RS], Z[RS], TT[RS], DB[RS];
  double INV[RS];
  RowIn IN[RS];
  if (tid == 0) {
    lz[0][0] = z2;
    lz[1][0] = z2;
  }
  if (tid == TPB - 1) {
    lz[0][TPB + 1] = z2;
    lz[1][TPB + 1] = z2;
  }
  // rows rb-2 .. rb+1+PF of v and rb-1 .. rb+PF of 1/c^2 (slot = (row - rb + 2) % RS; with
  // PF 1 row rb+2 reuses the slot of row rb-2, so it is loaded once that row is consumed)
  unroll<0, 4>([&](auto kc) {
    constexpr int m = decltype(kc)::value;
    V[m] = load_v(min(rb - 2 + m, re + 1));
  });
  unroll<1, 2 + PF + 1>([&](auto kc) {
    constexpr int m = decltype(kc)::value;
    load_in(min(rb - 2 + m, re), IN[m]);
  });
  put_v(1, V[1], IN[1]);
  __syncthreads();  // (also publishes the table rows)
  stage1(rb - 1, 1, V[0], V[1], V[2], IN[1], TT[1], Z[1], DB[1], INV[1]);
  unroll<4, 4 + PF>([&](auto kc) {
    constexpr int m = decltype(kc)::value;
    V[m % RS] = load_v(min(rb - 2 + m, re + 1));
  });
  put_v(0, V[2], IN[2]);
  __syncthreads();
  stage1(rb, 0, V[1], V[2], V[3], IN[2], TT[2], Z[2], DB[2], INV[2]);

  for (int r0 = rb; r0 < re; r0 += RS) {
    unroll<0, RS>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      constexpr int p = (k + 1) & 1;
      // slot of row r + d at iteration k
      constexpr int s0 = (k + 2) % RS, s1 = (k + 3) % RS, s2 = (k + 4) % RS;
      constexpr int sm1 = (k + 1) % RS;
      constexpr int sv = (k + 4 + PF) % RS, si = (k + 3 + PF) % RS;
      const int r = r0 + k;
      const bool live = r < re;
      V[sv] = load_v(min(r + 2 + PF, re + 1));
      load_in(min(r + 1 + PF, re), IN[si]);
      put_v(p, V[s1], IN[s1]);  // v row r+1
      lz[p][tid + 1] = Z[s0];   // z1 row r
      __syncthreads();
      stage1(min(r + 1, re), p, V[s0], V[s1], V[s2], IN[s1], TT[s1], Z[s1], DB[s1], INV[s1]);
      const double2 w = stage2(min(r, re), p, Z[sm1], Z[s0], Z[s1], TT[s0], DB[s0], INV[s0]);
      if (outl && live) {
        double2* q = a.out0 + (size_t)r * n + c;
        __builtin_nontemporal_store(w.x, &q->x);
        __builtin_nontemporal_store(w.y, &q->y);
        if constexpr (RES) {
          acc[0] += cabs2(TT[s0]);
          acc[1] += cabs2(w);
        }
      }
    });
  }
  __syncthreads();  // LDS reuse by the block's next tile
}

// Barrier-free form: every WAVE is an independent overlapping strip -- its 64 lanes compute the
// first sweep on 64 columns and write w on the inner 62 -- so all W/E exchanges are wave
// shuffles (no LDS, no barrier: a wave never waits for another).  The two v columns beyond the
// strip come from one broadcast load per row (lanes 0-31: column i0-2, lanes 32-63: i0+63).
// Costs 64/62 lanes of arithmetic; same per-point arithmetic as sl2_tile: bit-identical.
template <bool CONSTC, bool NTU>
__device__ __forceinline__ void sl2_wave(const StencilArgs& a, const int t) {
  constexpr int WO = kWave - 2;
  const int wave = threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int n = a.n, nl = a.nl;
  const int strips = (n + WO - 1) / WO;
  const int tx = t % a.tiles_x;
  const int ty = t / a.tiles_x;
  const int strip = tx * (kStencilThreads / kWave) + wave;
  if (strip >= strips) return;  // (wave-uniform; no barrier in this shape)
  const int i0 = strip * WO;
  const int c = i0 + lane - 1;
  const bool cin = c >= 0 && c < n;
  const int cc = min(max(c, 0), n - 1);
  const bool outl = lane >= 1 && lane <= kWave - 2 && cin;
  const int rb = __builtin_amdgcn_readfirstlane(a.row_begin + ty * a.row_step);
  const int re = __builtin_amdgcn_readfirstlane(min(rb + a.rows_per_block, a.row_end));
  int ie = lane < kWave / 2 ? i0 - 2 : i0 + kWave - 1;
  const bool lw = lane == 0 && i0 - 2 >= 0;
  const bool le = lane == kWave - 1 && i0 + kWave - 1 < n;
  ie = min(max(ie, 0), n - 1);
  const double2 z2 = make_double2(0.0, 0.0);

  auto rowp = [&](int r) -> const double2* {
    return r < 0 ? a.halo_lo + (size_t)(r + 2) * n
                 : (r >= nl ? a.halo_hi + (size_t)(r - nl) * n : a.u + (size_t)r * n);
  };
  auto load_v = [&](int r) -> double2 {
    const double2* p = rowp(r) + cc;
    if constexpr (NTU)
      return make_double2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
    else
      return *p;
  };
  auto load_in = [&](int r, RowIn& v) {
    if constexpr (!CONSTC) {
      const double* q = r < 0 ? a.invc2_halo + (size_t)(r + 2) * n
                              : (r >= nl ? a.invc2_halo + (size_t)(r - nl + 2) * n
                                         : a.invc2 + (size_t)r * n);
      v.ic = __builtin_nontemporal_load(q + cc);
    } else {
      v.ic = a.invc2_const;
    }
    v.e = rowp(r)[ie];
  };
  const cdouble_p tabj = (cdouble_p)(a.tab_j);
  auto load_tab = [&](int r, RowTab& tb) {
    const int ru = __builtin_amdgcn_readfirstlane(min(max(r, -2), nl + 1));
    const cdouble_p q = tabj + 8 * ru;
    tb.R2 = make_double2(q[0], q[1]);
    tb.BS = make_double2(q[2], q[3]);
    tb.BN = make_double2(q[4], q[5]);
    tb.OM = make_double2(q[6], q[7]);
  };
  const double2 AW = a.tab_i[cc], AE = a.tab_i[n + cc], R1 = a.tab_i[2 * n + cc];
  const double sin = a.in_scale ? *a.in_scale : 1.0;
  auto shup = [](double2 v) { return make_double2(__shfl_up(v.x, 1), __shfl_up(v.y, 1)); };
  auto shdn = [](double2 v) { return make_double2(__shfl_down(v.x, 1), __shfl_down(v.y, 1)); };

  auto stage1 = [&](int s, double2 uS, double2 uC, double2 uN, const RowIn& in,
                    const RowTab& tb, double2& T, double2& z1) __attribute__((always_inline)) {
    const double2 uCm = csel(cin, uC, z2);
    const double2 sw = shup(uCm), se = shdn(uCm);
    const double2 uW = lane == 0 ? csel(lw, in.e, z2) : sw;
    const double2 uE = lane == kWave - 1 ? csel(le, in.e, z2) : se;
    const double2 W = cmul(AW, tb.R2);
    const double2 E = cmul(AE, tb.R2);
    const double2 S = cmul(tb.BS, R1);
    const double2 N = cmul(tb.BN, R1);
    const double2 M = cscale(cmul(tb.OM, R1), in.ic);
    const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
    const double2 D = csub(M, sum4);
    const double2 Db = csub(cmul(M, a.mshift), sum4);
    double2 Au = cmul(S, uS);
    Au = cfma(W, uW, Au);
    Au = cfma(D, uC, Au);
    Au = cfma(E, uE, Au);
    Au = cfma(N, uN, Au);
    T = cscale(Au, sin);
    z1 = csel(cin && a.j0 + s >= 0 && a.j0 + s < n, cscale(cdiv(T, Db), a.damping), z2);
  };
  auto stage2 = [&](double2 zS, double2 zC, double2 zN, double2 T, const RowIn& in,
                    const RowTab& tb) __attribute__((always_inline)) -> double2 {
    const double2 zW = shup(zC), zE = shdn(zC);  // (lanes 0 and 63 write no output)
    const double2 W = cmul(AW, tb.R2);
    const double2 E = cmul(AE, tb.R2);
    const double2 S = cmul(tb.BS, R1);
    const double2 N = cmul(tb.BN, R1);
    const double2 M = cscale(cmul(tb.OM, R1), in.ic);
    const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
    const double2 Db = csub(cmul(M, a.mshift), sum4);
    double2 Au = cmul(S, zS);
    Au = cfma(W, zW, Au);
    Au = cfma(Db, zC, Au);
    Au = cfma(E, zE, Au);
    Au = cfma(N, zN, Au);
    return cadd(zC, cscale(cdiv(csub(T, Au), Db), a.damping));
  };

  double2 V[4], Z[4], TT[4];
  RowIn IN[4];
  RowTab TB[4];
  V[0] = load_v(rb - 2);
  V[1] = load_v(rb - 1);
  V[2] = load_v(rb);
  V[3] = load_v(rb + 1);
  load_in(rb - 1, IN[1]);
  load_in(rb, IN[2]);
  load_in(rb + 1, IN[3]);
  load_tab(rb - 1, TB[1]);
  load_tab(rb, TB[2]);
  load_tab(rb + 1, TB[3]);
  stage1(rb - 1, V[0], V[1], V[2], IN[1], TB[1], TT[1], Z[1]);
  V[0] = load_v(rb + 2);
  stage1(rb, V[1], V[2], V[3], IN[2], TB[2], TT[2], Z[2]);

  for (int r0 = rb; r0 < re; r0 += 4) {
    unroll<0, 4>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const int r = r0 + k;
      const bool live = r < re;
      V[(k + 1) & 3] = load_v(min(r + 3, re + 1));
      load_in(min(r + 2, re), IN[k & 3]);
      load_tab(min(r + 2, re), TB[k & 3]);
      stage1(r + 1, V[(k + 2) & 3], V[(k + 3) & 3], V[k & 3], IN[(k + 3) & 3], TB[(k + 3) & 3],
             TT[(k + 3) & 3], Z[(k + 3) & 3]);
      const double2 w = stage2(Z[(k + 1) & 3], Z[(k + 2) & 3], Z[(k + 3) & 3], TT[(k + 2) & 3],
                               IN[(k + 2) & 3], TB[(k + 2) & 3]);
      if (outl && live) {
        double2* q = a.out0 + (size_t)r * n + c;
        __builtin_nontemporal_store(w.x, &q->x);
        __builtin_nontemporal_store(w.y, &q->y);
      }
    });
  }
}

// The same fused M A for the 9-point operator, in stencil.hip's separable form
// term for term (so w is bit-identical to the two-launch path): with X(r) the x second
// difference of row r, Y(i) the y one of column i and H(r) = u_W + u_E of row r,
//   A u = alpha (X(r) + Y(i)) + g (X(r-1) + X(r+1) + Y(i-1) + Y(i+1)) + M (c u_C + d edges + e corners).
// Each stage (first sweep on row s = r+1, second sweep on row r) brings one new row into LDS
// (v row s+1 / z1 row r+1) and exchanges its Y through LDS: one barrier per stage.  X and H of
// the two previous rows stay in registers.  The strip's edge lanes add Y of the v halo columns
// (i0-2, i0+TPB-1) from the v ring's halo slots; z1 needs no halo (the strips overlap).
// Row inputs (1/c^2, edges, tables) are prefetched three rows ahead: the first sweep on row s
// needs the edges and 1/s2 of row s+1.
template <bool CONSTC, bool NTU, int TPB>
__device__ __forceinline__ void sl2_tile9(const StencilArgs& a, const int t) {
  constexpr int WO = TPB - 2;
  __shared__ double2 lv[4][TPB + 2];  // v rows, slot(row) = (row - rb + 2) & 3
  __shared__ double2 lyv[TPB + 2];    // Y of v on the first-sweep row
  __shared__ double2 lz[TPB + 2];     // z1 row entering the second sweep
  __shared__ double2 lyz[TPB + 2];    // Y of z1 on the second-sweep row
  const int tx = t % a.tiles_x;
  const int ty = t / a.tiles_x;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int n = a.n, nl = a.nl;
  const int i0 = tx * WO;
  const int c = i0 + tid - 1;
  const bool cin = c >= 0 && c < n;
  const int cc = min(max(c, 0), n - 1);
  const bool outl = tid >= 1 && tid <= TPB - 2 && cin;
  const int rb = __builtin_amdgcn_readfirstlane(a.row_begin + ty * a.row_step);
  const int re = __builtin_amdgcn_readfirstlane(min(rb + a.rows_per_block, a.row_end));
  int ie = lane < kWave / 2 ? i0 - 2 : i0 + TPB - 1;
  const bool lw = tid == 0 && i0 - 2 >= 0;
  const bool le = tid == TPB - 1 && i0 + TPB - 1 < n;
  ie = min(max(ie, 0), n - 1);
  const double2 z2 = make_double2(0.0, 0.0);
  const Stencil9W w = a.w9;

  // rows -2 .. nl+1: two halo rows on each side (StencilArgs, fused SL fields)
  auto rowp = [&](int r) -> const double2* {
    return r < 0 ? a.halo_lo + (size_t)(r + 2) * n
                 : (r >= nl ? a.halo_hi + (size_t)(r - nl) * n : a.u + (size_t)r * n);
  };
  auto load_v = [&](int r) -> double2 {
    const double2* p = rowp(r) + cc;
    if constexpr (NTU)
      return make_double2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
    else
      return *p;
  };
  auto load_in = [&](int r, RowIn& v) {
    if constexpr (!CONSTC) {
      const double* q = r < 0 ? a.invc2_halo + (size_t)(r + 2) * n
                              : (r >= nl ? a.invc2_halo + (size_t)(r - nl + 2) * n
                                         : a.invc2 + (size_t)r * n);
      v.ic = __builtin_nontemporal_load(q + cc);
    } else {
      v.ic = a.invc2_const;
    }
    v.e = rowp(r)[ie];
  };
  const cdouble_p tabj = (cdouble_p)(a.tab_j);
  auto load_tab = [&](int r, RowTab& tb) {
    const int ru = __builtin_amdgcn_readfirstlane(min(max(r, -2), nl + 1));  // tab_j_ext rows
    const cdouble_p q = tabj + 8 * ru;
    tb.R2 = make_double2(q[0], q[1]);
    tb.BS = make_double2(q[2], q[3]);
    tb.BN = make_double2(q[4], q[5]);
    tb.OM = make_double2(q[6], q[7]);
  };
  const double2 AW = a.tab_i[cc], AE = a.tab_i[n + cc], R1 = a.tab_i[2 * n + cc];
  const double2 R1e = a.tab_i[2 * n + ie];  // the edge lanes' halo column
  const double sin = a.in_scale ? *a.in_scale : 1.0;
  auto xdiff = [&](double2 R2, double2 uW, double2 uC, double2 uE) {
    return cmul(R2, cfma(AE, csub(uE, uC), cmul(AW, csub(uW, uC))));
  };
  auto ydiff = [&](double2 R, const RowTab& tb, double2 uS, double2 uC, double2 uN) {
    return cmul(R, cfma(tb.BN, csub(uN, uC), cmul(tb.BS, csub(uS, uC))));
  };
  // the 9-point product from the separable terms (stencil.hip, S9 step, same association)
  auto op9 = [&](double2 Mo, double2 Xm, double2 Xc, double2 Xp, double2 Yc, double2 Yw,
                 double2 Ye, double2 Hm, double2 Hc, double2 Hp, double2 uS, double2 uC,
                 double2 uN) {
    const double2 lap = cadd(Xc, Yc);
    const double2 avg = cadd(cadd(Xm, Xp), cadd(Yw, Ye));
    const double2 edges = cadd(Hc, cadd(uS, uN));
    const double2 corners = cadd(Hm, Hp);
    const double2 mix = cadd(cadd(cscale(uC, w.c), cscale(edges, w.d)), cscale(corners, w.e));
    return cfma(Mo, mix, cadd(cscale(lap, w.alpha), cscale(avg, w.g)));
  };
  auto sum4_of = [&](const RowTab& tb) {
    const double2 W = cmul(AW, tb.R2);
    const double2 E = cmul(AE, tb.R2);
    const double2 S = cmul(tb.BS, R1);
    const double2 N = cmul(tb.BN, R1);
    return cadd(cadd(cadd(W, E), S), N);
  };

  double2 Xvm, Xvc, Hvm, Hvc;  // v: X, H of rows s-1, s
  double2 Xzm, Xzc, Hzm, Hzc;  // z1: X, H of rows r-1, r
  // first sweep on row s: row s+1 (vN, its edge eN, tables tbN) enters the v ring
  auto stage1 = [&](int s, double2 vS, double2 vC, double2 vN, double2 eN, const RowIn& in,
                    const RowTab& tb, const RowTab& tbN, double2& T, double2& z1)
      __attribute__((always_inline)) {
    double2* lS = lv[(s - 1 - rb + 2) & 3];
    double2* lC = lv[(s - rb + 2) & 3];
    double2* lN = lv[(s + 1 - rb + 2) & 3];
    const double2 Yc = ydiff(R1, tb, vS, vC, vN);
    lN[tid + 1] = csel(cin, vN, z2);
    lyv[tid + 1] = csel(cin, Yc, z2);
    if (tid == 0) {
      const double2 e = csel(lw, eN, z2);
      lN[0] = e;
      lyv[0] = ydiff(R1e, tb, lS[0], lC[0], e);
    }
    if (tid == TPB - 1) {
      const double2 e = csel(le, eN, z2);
      lN[TPB + 1] = e;
      lyv[TPB + 1] = ydiff(R1e, tb, lS[TPB + 1], lC[TPB + 1], e);
    }
    __syncthreads();
    const double2 vNW = lN[tid], vNE = lN[tid + 2];
    const double2 Yw = lyv[tid], Ye = lyv[tid + 2];
    const double2 Xp = xdiff(tbN.R2, vNW, vN, vNE);
    const double2 Hp = cadd(vNW, vNE);
    const double2 M = cscale(cmul(tb.OM, R1), in.ic);
    const double2 Db = stencil9_diag(cmul(M, a.mshift), sum4_of(tb), w);
    T = cscale(op9(M, Xvm, Xvc, Xp, Yc, Yw, Ye, Hvm, Hvc, Hp, vS, vC, vN), sin);
    z1 = csel(cin && a.j0 + s >= 0 && a.j0 + s < n, cscale(cdiv(T, Db), a.damping), z2);
    Xvm = Xvc;
    Xvc = Xp;
    Hvm = Hvc;
    Hvc = Hp;
  };
  // second sweep on row r: w = z1 + damp (T - A_beta z1) / Db; z1 row r+1 enters
  auto stage2 = [&](double2 zS, double2 zC, double2 zN, double2 T, const RowIn& in,
                    const RowTab& tb, const RowTab& tbN) __attribute__((always_inline)) -> double2 {
    const double2 Yc = ydiff(R1, tb, zS, zC, zN);
    lz[tid + 1] = zN;
    lyz[tid + 1] = Yc;
    __syncthreads();
    const double2 zNW = lz[tid], zNE = lz[tid + 2];
    const double2 Yw = lyz[tid], Ye = lyz[tid + 2];
    const double2 Xp = xdiff(tbN.R2, zNW, zN, zNE);
    const double2 Hp = cadd(zNW, zNE);
    const double2 M = cscale(cmul(tb.OM, R1), in.ic);
    const double2 Mb = cmul(M, a.mshift);
    const double2 Db = stencil9_diag(Mb, sum4_of(tb), w);
    const double2 Au = op9(Mb, Xzm, Xzc, Xp, Yc, Yw, Ye, Hzm, Hzc, Hp, zS, zC, zN);
    Xzm = Xzc;
    Xzc = Xp;
    Hzm = Hzc;
    Hzc = Hp;
    return cadd(zC, cscale(cdiv(csub(T, Au), Db), a.damping));
  };

  // rings of four by row, slot(row) = (row - rb + 2) & 3: v rows r .. r+3, z1 / T rows
  // r-1 .. r+1, row inputs and tables rows r .. r+3 (r+3 in flight)
  double2 V[4], Z[4], TT[4];
  RowIn IN[4];
  RowTab TB[4];
  if (tid == 0) {  // halo slots of the z1 rows: only lanes 0 / TPB-1 read them, for outputs
    lz[0] = z2;    // nobody stores
    lyz[0] = z2;
  }
  if (tid == TPB - 1) {
    lz[TPB + 1] = z2;
    lyz[TPB + 1] = z2;
  }
  V[0] = load_v(rb - 2);
  V[1] = load_v(rb - 1);
  V[2] = load_v(rb);
  V[3] = load_v(rb + 1);
  RowIn inm2;
  load_in(rb - 2, inm2);  // edges of row rb-2 (the ring's first row)
  load_in(rb - 1, IN[1]);
  load_in(rb, IN[2]);
  load_in(rb + 1, IN[3]);
  load_in(rb + 2, IN[0]);
  RowTab tbm2;
  load_tab(rb - 2, tbm2);
  load_tab(rb - 1, TB[1]);
  load_tab(rb, TB[2]);
  load_tab(rb + 1, TB[3]);
  load_tab(rb + 2, TB[0]);
  // rows rb-2 and rb-1 enter the v ring; X, H of both from it
  lv[0][tid + 1] = csel(cin, V[0], z2);
  lv[1][tid + 1] = csel(cin, V[1], z2);
  if (tid == 0) {
    lv[0][0] = csel(lw, inm2.e, z2);
    lv[1][0] = csel(lw, IN[1].e, z2);
  }
  if (tid == TPB - 1) {
    lv[0][TPB + 1] = csel(le, inm2.e, z2);
    lv[1][TPB + 1] = csel(le, IN[1].e, z2);
  }
  __syncthreads();
  Xvm = xdiff(tbm2.R2, lv[0][tid], V[0], lv[0][tid + 2]);
  Hvm = cadd(lv[0][tid], lv[0][tid + 2]);
  Xvc = xdiff(TB[1].R2, lv[1][tid], V[1], lv[1][tid + 2]);
  Hvc = cadd(lv[1][tid], lv[1][tid + 2]);
  stage1(rb - 1, V[0], V[1], V[2], IN[2].e, IN[1], TB[1], TB[2], TT[1], Z[1]);
  V[0] = load_v(rb + 2);
  __syncthreads();  // lyv is rewritten by the next first sweep
  stage1(rb, V[1], V[2], V[3], IN[3].e, IN[2], TB[2], TB[3], TT[2], Z[2]);
  // the second sweep's register ring starts with X, H of z1 rows rb-1 and rb
  lz[tid + 1] = Z[1];
  lyz[tid + 1] = Z[2];
  __syncthreads();
  Xzm = xdiff(TB[1].R2, lz[tid], Z[1], lz[tid + 2]);
  Hzm = cadd(lz[tid], lz[tid + 2]);
  Xzc = xdiff(TB[2].R2, lyz[tid], Z[2], lyz[tid + 2]);
  Hzc = cadd(lyz[tid], lyz[tid + 2]);
  __syncthreads();

  for (int r0 = rb; r0 < re; r0 += 4) {
    unroll<0, 4>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const int r = r0 + k;
      const bool live = r < re;
      V[(k + 1) & 3] = load_v(min(r + 3, re + 1));
      load_in(min(r + 3, re + 1), IN[(k + 1) & 3]);
      load_tab(min(r + 3, re + 1), TB[(k + 1) & 3]);
      stage1(r + 1, V[(k + 2) & 3], V[(k + 3) & 3], V[k & 3], IN[k & 3].e, IN[(k + 3) & 3],
             TB[(k + 3) & 3], TB[k & 3], TT[(k + 3) & 3], Z[(k + 3) & 3]);
      const double2 wv = stage2(Z[(k + 1) & 3], Z[(k + 2) & 3], Z[(k + 3) & 3], TT[(k + 2) & 3],
                                IN[(k + 2) & 3], TB[(k + 2) & 3], TB[(k + 3) & 3]);
      if (outl && live) {
        double2* p = a.out0 + (size_t)r * n + c;
        __builtin_nontemporal_store(wv.x, &p->x);
        __builtin_nontemporal_store(wv.y, &p->y);
      }
    });
  }
  __syncthreads();  // LDS reuse by the block's next tile
}

// sl2_tile9 with sl2_tile_v2's instruction cuts (the round-1 form is VALU-issue-bound: ~400
// vector instructions per point-row, a third of them v_readlane of a four-row ring of PML table
// values spilled from SGPRs):
//  * the band's row tables (rows rb-2 .. re+1) staged in LDS once per tile, read by broadcast;
//  * the second sweep takes the shifted mass Mb, the shifted diagonal Db and 1/|Db|^2 of its
//    row from the first sweep (the values it would recompute: one IEEE division per point,
//    no second mass / diagonal / four-coefficient sum);
//  * interior tiles run without masks (EDGE = false).
// Same separable arithmetic term for term: bit-identical to the two-launch path.
// T and z1 reach the second sweep as plain values, as in the two-launch path (where they make a
// round trip through HBM): without the empty asm, a mask-free tile lets the compiler fuse the
// multiply that produced them into their consumers (e.g. zN - zC -> fma), one rounding fewer
__device__ __forceinline__ double2 opaque(double2 v) {
  asm volatile("" : "+v"(v.x), "+v"(v.y));
  return v;
}
struct Sl9Lds {
  double2 lv[4][kStencilThreads + 2];  // v rows, slot(row) = (row - rb + 2) & 3
  double2 lyv[kStencilThreads + 2];    // Y of v on the first-sweep row
  double2 lz[kStencilThreads + 2];     // z1 row entering the second sweep
  double2 lyz[kStencilThreads + 2];    // Y of z1 on the second-sweep row
  double2 ltab[kSl2MaxBand + 4][4];
};
template <bool CONSTC, bool NTU, bool EDGE>
__device__ __forceinline__ void sl2_tile9_v2(const StencilArgs& a, const int t, Sl9Lds& L) {
  constexpr int TPB = kStencilThreads;
  constexpr int WO = TPB - 2;
  auto& lv = L.lv;
  auto& lyv = L.lyv;
  auto& lz = L.lz;
  auto& lyz = L.lyz;
  auto& ltab = L.ltab;
  const int tx = t % a.tiles_x;
  const int ty = t / a.tiles_x;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int n = a.n, nl = a.nl;
  const int i0 = tx * WO;
  const int c = i0 + tid - 1;
  const bool cin = !EDGE || (c >= 0 && c < n);
  const int cc = EDGE ? min(max(c, 0), n - 1) : c;
  const bool outl = tid >= 1 && tid <= TPB - 2 && cin;
  const int rb = __builtin_amdgcn_readfirstlane(a.row_begin + ty * a.row_step);
  const int re = __builtin_amdgcn_readfirstlane(min(rb + a.rows_per_block, a.row_end));
  int ie = lane < kWave / 2 ? i0 - 2 : i0 + TPB - 1;
  const bool lw = !EDGE || i0 - 2 >= 0;
  const bool le = !EDGE || i0 + TPB - 1 < n;
  if constexpr (EDGE) ie = min(max(ie, 0), n - 1);
  const double2 z2 = make_double2(0.0, 0.0);
  const Stencil9W w = a.w9;

  auto rowp = [&](int r) -> const double2* {
    return r < 0 ? a.halo_lo + (size_t)(r + 2) * n
                 : (r >= nl ? a.halo_hi + (size_t)(r - nl) * n : a.u + (size_t)r * n);
  };
  auto load_v = [&](int r) -> double2 {
    const double2* p = rowp(r) + cc;
    if constexpr (NTU)
      return make_double2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
    else
      return *p;
  };
  auto load_in = [&](int r, RowIn& v) {
    if constexpr (!CONSTC) {
      const double* q = r < 0 ? a.invc2_halo + (size_t)(r + 2) * n
                              : (r >= nl ? a.invc2_halo + (size_t)(r - nl + 2) * n
                                         : a.invc2 + (size_t)r * n);
      v.ic = __builtin_nontemporal_load(q + cc);
    } else {
      v.ic = a.invc2_const;
    }
    v.e = rowp(r)[ie];
  };
  {  // PML row tables of the band (tab_j_ext rows rb-2 .. re+1) into LDS
    const int cnt = (re - rb + 4) * 4;
    for (int k = tid; k < cnt; k += TPB) {
      const int rr = min(rb - 2 + k / 4, nl + 1);
      (&ltab[0][0])[k] = a.tab_j[4 * rr + (k & 3)];
    }
  }
  auto tab = [&](int r) -> const double2* { return ltab[r - rb + 2]; };
  const double2 AW = a.tab_i[cc], AE = a.tab_i[n + cc], R1 = a.tab_i[2 * n + cc];
  const double2 R1e = a.tab_i[2 * n + ie];  // the edge lanes' halo column
  const double sin = a.in_scale ? *a.in_scale : 1.0;
  auto xdiff = [&](double2 R2, double2 uW, double2 uC, double2 uE) {
    return cmul(R2, cfma(AE, csub(uE, uC), cmul(AW, csub(uW, uC))));
  };
  auto ydiff = [&](double2 R, double2 BS, double2 BN, double2 uS, double2 uC, double2 uN) {
    return cmul(R, cfma(BN, csub(uN, uC), cmul(BS, csub(uS, uC))));
  };
  auto op9 = [&](double2 Mo, double2 Xm, double2 Xc, double2 Xp, double2 Yc, double2 Yw,
                 double2 Ye, double2 Hm, double2 Hc, double2 Hp, double2 uS, double2 uC,
                 double2 uN) {
    const double2 lap = cadd(Xc, Yc);
    const double2 avg = cadd(cadd(Xm, Xp), cadd(Yw, Ye));
    const double2 edges = cadd(Hc, cadd(uS, uN));
    const double2 corners = cadd(Hm, Hp);
    const double2 mix = cadd(cadd(cscale(uC, w.c), cscale(edges, w.d)), cscale(corners, w.e));
    return cfma(Mo, mix, cadd(cscale(lap, w.alpha), cscale(avg, w.g)));
  };

  double2 Xvm, Xvc, Hvm, Hvc;  // v: X, H of rows s-1, s
  double2 Xzm, Xzc, Hzm, Hzc;  // z1: X, H of rows r-1, r
  // first sweep on row s: row s+1 (vN, its edge eN) enters the v ring; T, z1 and the row's
  // shifted mass, diagonal and 1/|Db|^2 out
  auto stage1 = [&](int s, double2 vS, double2 vC, double2 vN, double2 eN, const RowIn& in,
                    double2& T, double2& z1, double2& Mbo, double2& Dbo, double& invo)
      __attribute__((always_inline)) {
    const double2* tb = tab(s);
    const double2 BS = tb[1], BN = tb[2];
    double2* lS = lv[(s - 1 - rb + 2) & 3];
    double2* lC = lv[(s - rb + 2) & 3];
    double2* lN = lv[(s + 1 - rb + 2) & 3];
    const double2 Yc = ydiff(R1, BS, BN, vS, vC, vN);
    lN[tid + 1] = EDGE ? csel(cin, vN, z2) : vN;
    lyv[tid + 1] = EDGE ? csel(cin, Yc, z2) : Yc;
    if (tid == 0) {
      const double2 e = EDGE ? csel(lw, eN, z2) : eN;
      lN[0] = e;
      lyv[0] = ydiff(R1e, BS, BN, lS[0], lC[0], e);
    }
    if (tid == TPB - 1) {
      const double2 e = EDGE ? csel(le, eN, z2) : eN;
      lN[TPB + 1] = e;
      lyv[TPB + 1] = ydiff(R1e, BS, BN, lS[TPB + 1], lC[TPB + 1], e);
    }
    __syncthreads();
    const double2 vNW = lN[tid], vNE = lN[tid + 2];
    const double2 Yw = lyv[tid], Ye = lyv[tid + 2];
    const double2 Xp = xdiff(tab(s + 1)[0], vNW, vN, vNE);
    const double2 Hp = cadd(vNW, vNE);
    const double2 R2 = tb[0], OM = tb[3];
    const double2 W = cmul(AW, R2);
    const double2 E = cmul(AE, R2);
    const double2 S = cmul(BS, R1);
    const double2 N = cmul(BN, R1);
    const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
    const double2 M = cscale(cmul(OM, R1), in.ic);
    const double2 Mb = cmul(M, a.mshift);
    const double2 Db = stencil9_diag(Mb, sum4, w);
    T = opaque(cscale(op9(M, Xvm, Xvc, Xp, Yc, Yw, Ye, Hvm, Hvc, Hp, vS, vC, vN), sin));
    const double inv = 1.0 / fma(Db.x, Db.x, Db.y * Db.y);  // = cdiv(T, Db), split
    const double2 q = cscale(make_double2(fma(T.x, Db.x, T.y * Db.y) * inv,
                                          fma(T.y, Db.x, -T.x * Db.y) * inv), a.damping);
    if constexpr (EDGE) z1 = opaque(csel(cin && a.j0 + s >= 0 && a.j0 + s < n, q, z2));
    else z1 = opaque(q);
    Xvm = Xvc;
    Xvc = Xp;
    Hvm = Hvc;
    Hvc = Hp;
    Mbo = Mb;
    Dbo = Db;
    invo = inv;
  };
  // second sweep on row r: w = z1 + damp (T - A_beta z1) / Db; z1 row r+1 enters
  auto stage2 = [&](int r, double2 zS, double2 zC, double2 zN, double2 T, double2 Mb,
                    double2 Db, double inv) __attribute__((always_inline)) -> double2 {
    const double2* tb = tab(r);
    const double2 Yc = ydiff(R1, tb[1], tb[2], zS, zC, zN);
    lz[tid + 1] = zN;
    lyz[tid + 1] = Yc;
    __syncthreads();
    const double2 zNW = lz[tid], zNE = lz[tid + 2];
    const double2 Yw = lyz[tid], Ye = lyz[tid + 2];
    const double2 Xp = xdiff(tab(r + 1)[0], zNW, zN, zNE);
    const double2 Hp = cadd(zNW, zNE);
    const double2 Au = op9(Mb, Xzm, Xzc, Xp, Yc, Yw, Ye, Hzm, Hzc, Hp, zS, zC, zN);
    Xzm = Xzc;
    Xzc = Xp;
    Hzm = Hzc;
    Hzc = Hp;
    const double2 d = csub(T, Au);
    const double2 q = make_double2(fma(d.x, Db.x, d.y * Db.y) * inv,
                                   fma(d.y, Db.x, -d.x * Db.y) * inv);
    return cadd(zC, cscale(q, a.damping));
  };

  // rings of four by row, slot(row) = (row - rb + 2) & 3: v rows r .. r+3, z1 rows r-1 .. r+1,
  // T / Mb / Db / 1/|Db|^2 rows r, r+1, row inputs rows r .. r+3 (r+3 in flight)
  double2 V[4], Z[4], TT[4], MB[4], DB[4];
  double INV[4];
  RowIn IN[4];
  if (tid == 0) {  // halo slots of the z1 rows: only lanes 0 / TPB-1 read them, for outputs
    lz[0] = z2;    // nobody stores
    lyz[0] = z2;
  }
  if (tid == TPB - 1) {
    lz[TPB + 1] = z2;
    lyz[TPB + 1] = z2;
  }
  V[0] = load_v(rb - 2);
  V[1] = load_v(rb - 1);
  V[2] = load_v(rb);
  V[3] = load_v(rb + 1);
  RowIn inm2;
  load_in(rb - 2, inm2);  // edges of row rb-2 (the ring's first row)
  load_in(rb - 1, IN[1]);
  load_in(rb, IN[2]);
  load_in(rb + 1, IN[3]);
  load_in(rb + 2, IN[0]);
  // rows rb-2 and rb-1 enter the v ring; X, H of both from it
  lv[0][tid + 1] = EDGE ? csel(cin, V[0], z2) : V[0];
  lv[1][tid + 1] = EDGE ? csel(cin, V[1], z2) : V[1];
  if (tid == 0) {
    lv[0][0] = EDGE ? csel(lw, inm2.e, z2) : inm2.e;
    lv[1][0] = EDGE ? csel(lw, IN[1].e, z2) : IN[1].e;
  }
  if (tid == TPB - 1) {
    lv[0][TPB + 1] = EDGE ? csel(le, inm2.e, z2) : inm2.e;
    lv[1][TPB + 1] = EDGE ? csel(le, IN[1].e, z2) : IN[1].e;
  }
  __syncthreads();  // (also publishes the table rows)
  Xvm = xdiff(tab(rb - 2)[0], lv[0][tid], V[0], lv[0][tid + 2]);
  Hvm = cadd(lv[0][tid], lv[0][tid + 2]);
  Xvc = xdiff(tab(rb - 1)[0], lv[1][tid], V[1], lv[1][tid + 2]);
  Hvc = cadd(lv[1][tid], lv[1][tid + 2]);
  stage1(rb - 1, V[0], V[1], V[2], IN[2].e, IN[1], TT[1], Z[1], MB[1], DB[1], INV[1]);
  V[0] = load_v(rb + 2);
  __syncthreads();  // lyv is rewritten by the next first sweep
  stage1(rb, V[1], V[2], V[3], IN[3].e, IN[2], TT[2], Z[2], MB[2], DB[2], INV[2]);
  // the second sweep's register ring starts with X, H of z1 rows rb-1 and rb
  lz[tid + 1] = Z[1];
  lyz[tid + 1] = Z[2];
  __syncthreads();
  Xzm = xdiff(tab(rb - 1)[0], lz[tid], Z[1], lz[tid + 2]);
  Hzm = cadd(lz[tid], lz[tid + 2]);
  Xzc = xdiff(tab(rb)[0], lyz[tid], Z[2], lyz[tid + 2]);
  Hzc = cadd(lyz[tid], lyz[tid + 2]);
  __syncthreads();

  for (int r0 = rb; r0 < re; r0 += 4) {
    unroll<0, 4>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const int r = r0 + k;
      const bool live = r < re;
      V[(k + 1) & 3] = load_v(min(r + 3, re + 1));
      load_in(min(r + 3, re + 1), IN[(k + 1) & 3]);
      stage1(min(r + 1, re), V[(k + 2) & 3], V[(k + 3) & 3], V[k & 3], IN[k & 3].e,
             IN[(k + 3) & 3], TT[(k + 3) & 3], Z[(k + 3) & 3], MB[(k + 3) & 3], DB[(k + 3) & 3],
             INV[(k + 3) & 3]);
      const double2 wv = stage2(min(r, re), Z[(k + 1) & 3], Z[(k + 2) & 3], Z[(k + 3) & 3],
                                TT[(k + 2) & 3], MB[(k + 2) & 3], DB[(k + 2) & 3],
                                INV[(k + 2) & 3]);
      if (outl && live) {
        double2* p = a.out0 + (size_t)r * n + c;
        __builtin_nontemporal_store(wv.x, &p->x);
        __builtin_nontemporal_store(wv.y, &p->y);
      }
    });
  }
  __syncthreads();  // LDS reuse by the block's next tile
}

// SHAPE (5-point): 0 = sl2_tile (two barriers per row), 1 = sl2_tile_1b (one barrier per row),
// 2 = sl2_wave (wave strips, no barrier), 3 = sl2_tile_v2 (one barrier, LDS tables, mask-free
// interior tiles).  The 9-point operator has sl2_tile9 only.
template <bool CONSTC, bool NTU, int TPB, bool S9, int SHAPE = 0, int PF = 1>
__global__ __launch_bounds__(TPB, (S9 && SHAPE == 4) ? 3 : 1) void sl2_kernel(const StencilArgs a) {
  if (a.stop && *a.stop) return;  // queued GMRES cycle already stopped
  const int L = blockIdx.x;
  const int q = L >> 3, Q = gridDim.x >> 3;
  const int ntiles = a.tiles_x * a.tiles_y;
  for (int tt = q; tt < a.tiles_per_xcd; tt += Q) {
    const int t = (L & 7) * a.tiles_per_xcd + tt;
    if (t >= ntiles) break;  // uniform per block
    if constexpr (S9 && (SHAPE == 3 || SHAPE == 4)) {  // (4: at 3 waves per SIMD)
      const int tx = t % a.tiles_x, ty = t / a.tiles_x;
      const int i0 = tx * (TPB - 2);
      const int rb = a.row_begin + ty * a.row_step;
      const int re = min(rb + a.rows_per_block, a.row_end);
      const bool interior = i0 - 2 >= 0 && i0 + TPB - 1 < a.n && a.j0 + rb - 1 >= 0 &&
                            a.j0 + re < a.n;
      __shared__ Sl9Lds lds9;
      if (interior) sl2_tile9_v2<CONSTC, NTU, false>(a, t, lds9);
      else sl2_tile9_v2<CONSTC, NTU, true>(a, t, lds9);
    } else if constexpr (S9) sl2_tile9<CONSTC, NTU, TPB>(a, t);
    else if constexpr (SHAPE == 1) sl2_tile_1b<CONSTC, NTU, TPB>(a, t);
    else if constexpr (SHAPE == 2) sl2_wave<CONSTC, NTU>(a, t);
    else if constexpr (SHAPE == 3) {
      // interior tile: every column c = i0-1 .. i0+TPB-2 (+ the halo columns) and every first-
      // sweep row rb-1 .. re on the grid -> the mask-free instantiation (block-uniform branch)
      const int tx = t % a.tiles_x, ty = t / a.tiles_x;
      const int i0 = tx * (TPB - 2);
      const int rb = a.row_begin + ty * a.row_step;
      const int re = min(rb + a.rows_per_block, a.row_end);
      const bool interior = i0 - 2 >= 0 && i0 + TPB - 1 < a.n && a.j0 + rb - 1 >= 0 &&
                            a.j0 + re < a.n;
      __shared__ Sl2Lds lds;
      if (interior) sl2_tile_v2<CONSTC, NTU, false, PF>(a, t, lds);
      else sl2_tile_v2<CONSTC, NTU, true, PF>(a, t, lds);
    }
    else sl2_tile<CONSTC, NTU, TPB>(a, t);
  }
}

// v0 = M (b - A x) in one pass: sl2_tile_v2 with the residual as the first sweep's input (the
// unfused form is EPI_RES_SL's stencil launch writing r and z1, the second sweep's stencil
// launch reading them back and a norm pass over v0: 16 + 16 + 8 + 16 + 16 B, then 16 + 16 +
// 8 + 16 and 16 per unknown -- here x 16 + b 16 + 1/c^2 8 + v0 16).  v0 bit-identical to the
// unfused form; the two norms summed in another order (per block, then reduce_kernel).
template <bool CONSTC, int PF>
__global__ __launch_bounds__(kStencilThreads) void sl2_res_kernel(const StencilArgs a) {
  double acc[2] = {0.0, 0.0};
  const int L = blockIdx.x;
  const int q = L >> 3, Q = gridDim.x >> 3;
  const int ntiles = a.tiles_x * a.tiles_y;
  __shared__ Sl2Lds lds;
  for (int tt = q; tt < a.tiles_per_xcd; tt += Q) {
    const int t = (L & 7) * a.tiles_per_xcd + tt;
    if (t >= ntiles) break;  // uniform per block
    const int tx = t % a.tiles_x, ty = t / a.tiles_x;
    const int i0 = tx * (kStencilThreads - 2);
    const int rb = a.row_begin + ty * a.row_step;
    const int re = min(rb + a.rows_per_block, a.row_end);
    const bool interior = i0 - 2 >= 0 && i0 + kStencilThreads - 1 < a.n && a.j0 + rb - 1 >= 0 &&
                          a.j0 + re < a.n;
    if (interior) sl2_tile_v2<CONSTC, false, false, PF, true>(a, t, lds, acc);
    else sl2_tile_v2<CONSTC, false, true, PF, true>(a, t, lds, acc);
  }
  block_reduce_vec<2>(acc, a.partials, kMaxNorms);
}

template <int TPB, bool NTU, int SHAPE = 0, int PF = 1>
void launch_t(bool const_c, const StencilArgs& a, int blocks, hipStream_t s) {
  const bool s9 = a.tab_r2x != nullptr;  // 9-point operator (the tables themselves are unused)
  if (const_c) {
    if (s9) hipLaunchKernelGGL((sl2_kernel<true, NTU, TPB, true, SHAPE == 3 ? (PF == 2 ? 4 : 3) : 0>), dim3(blocks), dim3(TPB), 0, s, a);
    else hipLaunchKernelGGL((sl2_kernel<true, NTU, TPB, false, SHAPE, PF>), dim3(blocks), dim3(TPB), 0, s, a);
  } else {
    if (s9) hipLaunchKernelGGL((sl2_kernel<false, NTU, TPB, true, SHAPE == 3 ? (PF == 2 ? 4 : 3) : 0>), dim3(blocks), dim3(TPB), 0, s, a);
    else hipLaunchKernelGGL((sl2_kernel<false, NTU, TPB, false, SHAPE, PF>), dim3(blocks), dim3(TPB), 0, s, a);
  }
}

}  // namespace

void launch_sl2(bool const_c, const StencilArgs& a_in, hipStream_t stream, int variant) {
  StencilArgs a = a_in;
  const int n = a.n;
  // Round-1 shape (0, two barriers per row; still the 9-point one): 256-wide strips (126 VGPRs:
  // 4 blocks per CU instead of 2 at 512), non-temporal v on rows up to 4608 points; a stencil
  // tuning variant of the LDS family (6/18/30/42) selects it with its strip width (>= 24: 512)
  // and NT v loads (% 24 >= 12); kSl2Variant + ... selects any shape (hh_internal.hpp).
  // Default: shape 3 (one barrier per row, LDS row tables, mask-free interior tiles) with
  // prefetch distance 2 and v loaded through the cache.  Inside GMRES(20) at 4096^2 it averages
  // 118.7 us against 133.2 us for the two-barrier shape (rocprofv3, profiles/r02f_*); cold
  // standalone applies 141.8 vs 146.8 us (profiles/r02e_tune_sl2.log).
  int tpb = 256;
  bool ntu = false;
  int shape = 3;
  bool pf2 = true;
  if (variant == 6 || variant == 18 || variant == 30 || variant == 42) {  // (lds_family)
    tpb = variant >= 24 ? 512 : 256;
    ntu = variant % 24 >= 12;
    shape = 0;  // the round-1 two-barrier shape
    pf2 = false;
  } else if (sl2_variant(variant)) {  // kSl2Variant + shape (0..3) + 4 NT v loads + 8 PF 2
    shape = (variant - kSl2Variant) & 3;
    ntu = ((variant - kSl2Variant) & 4) != 0;
    pf2 = shape == 3 && ((variant - kSl2Variant) & 8) != 0;
  }
  const bool lds_family = variant == 6 || variant == 18 || variant == 30 || variant == 42;
  if (a.tab_r2x) {  // the 9-point operator: shape 3 = sl2_tile9_v2 with v through the cache
    // (the PF-2 bit, set by default, selects its instantiation held to 3 waves per SIMD:
    // 163-167 VGPRs, no scratch; without it 167-171, 2 waves), any other shape = the round-1
    // two-barrier form (sl2_tile9; NT v on rows up to 4608 points unless the variant says)
    if (lds_family || (sl2_variant(variant) && shape != 3)) {
      if (!sl2_variant(variant)) ntu = n <= 4608;
      shape = 0;
    }
  }
  const int rows = a.row_end - a.row_begin;
  if (shape == 3 && a.rows_per_block > kSl2MaxBand) {  // LDS table capacity of the shape
    if (a.row_step <= 0 || a.row_step == a.rows_per_block) {
      a.rows_per_block = kSl2MaxBand;
      a.row_step = 0;
    } else {
      shape = 1;  // (spaced bands taller than the table: the one-barrier shape)
    }
  }
  if (a.row_step <= 0) a.row_step = a.rows_per_block;  // (> 0: spaced boundary bands)
  // output columns per tile: TPB - 2 (strip shapes) or 4 wave strips of 62 (shape 2)
  const int wo = shape == 2 ? (kWave - 2) * (kStencilThreads / kWave) : tpb - 2;
  if (shape == 2) {
    const int strips = (n + kWave - 3) / (kWave - 2);
    a.tiles_x = (strips + 3) / 4;
  } else {
    a.tiles_x = (n + wo - 1) / wo;
  }
  a.tiles_y = stencil_bands(rows, a.rows_per_block, a.row_step);
  a.tiles_per_xcd = (a.tiles_x * a.tiles_y + 7) / 8;
  const int blocks = a.tiles_per_xcd * 8;
  if (shape == 1) {
    if (ntu) launch_t<256, true, 1>(const_c, a, blocks, stream);
    else launch_t<256, false, 1>(const_c, a, blocks, stream);
  } else if (shape == 3) {
    if (pf2) {
      if (ntu) launch_t<256, true, 3, 2>(const_c, a, blocks, stream);
      else launch_t<256, false, 3, 2>(const_c, a, blocks, stream);
    } else {
      if (ntu) launch_t<256, true, 3>(const_c, a, blocks, stream);
      else launch_t<256, false, 3>(const_c, a, blocks, stream);
    }
  } else if (shape == 2) {
    if (ntu) launch_t<256, true, 2>(const_c, a, blocks, stream);
    else launch_t<256, false, 2>(const_c, a, blocks, stream);
  } else if (tpb == 256) {
    if (ntu) launch_t<256, true>(const_c, a, blocks, stream);
    else launch_t<256, false>(const_c, a, blocks, stream);
  } else {
    if (ntu) launch_t<512, true>(const_c, a, blocks, stream);
    else launch_t<512, false>(const_c, a, blocks, stream);
  }
}

int sl2_res_blocks(int n, int rows, int rows_per_block) {
  const int tiles_x = (n + kStencilThreads - 3) / (kStencilThreads - 2);
  const int tiles = tiles_x * stencil_bands(rows, std::min(rows_per_block, kSl2MaxBand), 0);
  return (tiles + 7) / 8 * 8;
}

int launch_sl2_res(bool const_c, const StencilArgs& a_in, hipStream_t stream) {
  StencilArgs a = a_in;
  const int rows = a.row_end - a.row_begin;
  a.rows_per_block = std::min(a.rows_per_block, kSl2MaxBand);  // (the LDS row-table capacity)
  a.row_step = a.rows_per_block;
  a.tiles_x = (a.n + kStencilThreads - 3) / (kStencilThreads - 2);
  a.tiles_y = stencil_bands(rows, a.rows_per_block, 0);
  a.tiles_per_xcd = (a.tiles_x * a.tiles_y + 7) / 8;
  const int blocks = a.tiles_per_xcd * 8;
  if (const_c) hipLaunchKernelGGL((sl2_res_kernel<true, 2>), dim3(blocks), dim3(kStencilThreads), 0, stream, a);
  else hipLaunchKernelGGL((sl2_res_kernel<false, 2>), dim3(blocks), dim3(kStencilThreads), 0, stream, a);
  return blocks;
}

}  // namespace hh
