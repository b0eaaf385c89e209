// Matrix-free complex 5-point (and 9-point) PML Helmholtz stencil for gfx950 (MI355X).
//
// Replaces the reference's assembled CSR operator and its scipy csr_matvec:
//   coefficients  get_A_diag_block_coeffs  code.py:70-115 (W=c1, E=c2, S=c3, N=c4, D=c5)
//                 get_upper/lower_A_block   code.py:130-154
//   assembly      build_A_matrix            code.py:202-219
//   apply         A @ x  (scipy csr_matvec, A handed to gmres at code.py:516)
//
// Per point (i fast, j slow; p = j*n + i, 0-based):
//   W = AW[i]*R2[j]  E = AE[i]*R2[j]  S = BS[j]*R1[i]  N = BN[j]*R1[i]
//   D = OM[j]*R1[i]*(1/c^2)[j][i] - (W + E + S + N)          (code.py:107-109)
//   (A u)_p = S u_{j-1} + W u_{i-1} + D u + E u_{i+1} + N u_{j+1}  (CSR column order)
// The separable 1-D tables hold every PML factor; the only 2-D stream besides u and y
// is 1/c^2 (absent for a constant medium).  Algorithmic HBM bytes per point:
// 16 (read u) + 16 (write y) + 8 (read 1/c^2) = 40 B (32 B for constant c).
//
// 9-point operator (no reference counterpart, the reference is 5-point only,
// code.py:216-218): alpha x the 5-point operator above + (1 - alpha) x its line-averaged form
// (each second difference averaged over the two neighbouring lines, with those lines' PML
// factors) + the mass term spread over the 9 points with weights c, d, e (c + 4d + 4e = 1):
//   SW: g (Wm + Sm) + e M   S: alpha S - g (Wm + Em) + d M   SE: g (Em + Sp) + e M
//   W : alpha W - g (Sm + Nm) + d M   C: c M - alpha (W + E + S + N)   E: alpha E - g (Sp + Np) + d M
//   NW: g (Wp + Nm) + e M   N: alpha N - g (Wp + Ep) + d M   NE: g (Ep + Np) + e M
// with g = (1 - alpha) / 2, M = OM R1 / c^2 at the centre, Wm/Em/Wp/Ep = AW/AE x R2 of rows
// j-1 / j+1 and Sm/Nm/Sp/Np = BS/BN x R1 of columns i-1 / i+1 (hh_stencil9.hpp).  The kernels
// evaluate it in a separable form (see the S9 step of stencil_tile).  Same HBM bytes as the
// 5-point apply (40 B/pt).
//
// Two kernel shapes, bit-identical (the same per-point arithmetic):
// * marching (stencil_tile): a block owns a 256- or 512-wide strip of i and marches a band of
//   rows in j with a three-row register window (u_{j-1}, u_j, u_{j+1}) plus a one-row
//   prefetch, so every u is read from HBM once; W/E neighbours go through a double-buffered
//   LDS row (a 4-row ring for 9 points) with a one-point halo at each side (one barrier per
//   row).  Tiles are dealt to XCDs in contiguous bands.  Every epilogue (Jacobi, residual,
//   shifted-Laplace sweeps, norms); the shape used inside GMRES.
// * non-marching tiles (tile_kernel / tile9_kernel): R rows x 256 columns per block, every
//   load issued up front, wave-shuffle exchange, blocks in plain order -- the default
//   standalone apply on large grids (see stencil_resolve_variant).
#include "hh_internal.hpp"
#include "hh_complex.hpp"
#include "hh_stencil9.hpp"
#include "hh_error.hpp"
#include <algorithm>
#include <cstdlib>

#include <type_traits>

namespace hh {
namespace {

template <int EPI>
struct EpiTraits {
  static constexpr bool scaled_in = (EPI == EPI_AX || EPI == EPI_JAC || EPI == EPI_SL_FIRST);
  static constexpr bool reads_in1 = (EPI == EPI_RES || EPI == EPI_RES_JAC || EPI == EPI_RES_SL ||
                                     EPI == EPI_SL_SWEEP);
  static constexpr int nacc = (EPI == EPI_RES || EPI == EPI_RES_SL) ? 1 : (EPI == EPI_RES_JAC ? 2 : 0);
  static constexpr bool shifted = (EPI == EPI_RES_SL || EPI == EPI_SL_FIRST || EPI == EPI_SL_SWEEP);
};

template <int NACC, int TPB = kStencilThreads>
__device__ __forceinline__ void block_reduce_store(double (&acc)[kMaxNorms], double* partials,
                                                   int slot) {
  if constexpr (NACC > 0) {
    __shared__ double red[kMaxNorms][TPB / kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
#pragma unroll
    for (int k = 0; k < NACC; ++k) {
      double v = acc[k];
#pragma unroll
      for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0) red[k][wave] = v;
    }
    __syncthreads();
    if (threadIdx.x < NACC) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < TPB / kWave; ++w) s += red[threadIdx.x][w];
      partials[(size_t)slot * kMaxNorms + threadIdx.x] = s;
    }
  }
}

__device__ __forceinline__ double2 csel(bool c, double2 a, double2 b) {
  return make_double2(c ? a.x : b.x, c ? a.y : b.y);
}

__device__ __forceinline__ void store2(double2* p, double2 v, bool nt) {
  if (nt) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
  } else {
    *p = v;
  }
}

// Per-row operands a thread needs besides the centre column: 1/c^2 and its W/E inputs
// (block-edge values for XM_LDS, wave-edge values for XM_SHFL, both neighbours for
// XM_DIRECT).  Loaded unconditionally from clamped (always valid) addresses and masked
// at use: an exec-masked load makes hipcc drain vmcnt at the join, which would serialise
// the prefetch pipeline.
struct RowIn {
  double ic;
  double2 eW, eE;
  double2 b;  // the once-read second input (b or r) of the EPI_RES* / EPI_SL_SWEEP epilogues
};

template <bool NTL>
__device__ __forceinline__ double2 ld2(const double2* p) {
  if constexpr (NTL) {
    return make_double2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
  } else {
    return *p;
  }
}
template <bool NTL>
__device__ __forceinline__ double ld1(const double* p) {
  if constexpr (NTL) return __builtin_nontemporal_load(p);
  else return *p;
}

template <int K, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (K < N) {
    f(std::integral_constant<int, K>{});
    static_for<K + 1, N>(f);
  }
}

// Per-row PML factors (wave-uniform): read through the constant address space so hipcc
// issues scalar loads into SGPRs (the generic pointer would force vector loads because the
// kernel also stores through generic pointers).
using cdouble_p = const __attribute__((address_space(4))) double*;

// XM  : how W/E neighbours are exchanged -- XM_LDS (double-buffered LDS row, one barrier
//       per row), XM_DIRECT (each lane loads u[i-1], u[i+1]; the lines are L1/L2 hits of
//       the neighbouring lanes' loads), XM_SHFL (ds_bpermute within the wave, wave-edge
//       lanes load one extra value).
// PF  : rows of prefetch distance (1 or 2) for u, 1/c^2 and the edge values.
// NT  : non-temporal loads of the once-read 1/c^2 stream and stores of the outputs.
//
// The row loop is unrolled by the register-ring length: ring slot m always holds row
// rb-1+m (mod ring), so no value is copied between registers -- a copy of a register with
// a load still in flight would make hipcc drain vmcnt and serialise the prefetch.
template <int EPI, bool CONSTC, int XM, int PF, bool NT, bool NTU, int TPB, bool S9>
__device__ __forceinline__ void stencil_tile(const StencilArgs& a, const int t);

// Grid: either one block per tile, or a persistent grid of `gridDim.x` blocks (a multiple
// of 8) in which block L works through the tiles of XCD L % 8 in order, so at any moment
// each XCD streams one contiguous band window (L2 reuse of band-edge rows).
template <int EPI, bool CONSTC, int XM, int PF, bool NT, bool NTU, int TPB, bool S9>
__global__ __launch_bounds__(TPB) void stencil_kernel(const StencilArgs a) {
  if (a.stop && *a.stop) return;  // queued GMRES cycle already stopped
  const int L = blockIdx.x;
  const int q = L >> 3, Q = gridDim.x >> 3;
  const int ntiles = a.tiles_x * a.tiles_y;
  for (int tt = q; tt < a.tiles_per_xcd; tt += Q) {
    const int t = (L & 7) * a.tiles_per_xcd + tt;
    if (t >= ntiles) break;  // uniform per block
    stencil_tile<EPI, CONSTC, XM, PF, NT, NTU, TPB, S9>(a, t);
  }
}

template <int EPI, bool CONSTC, int XM, int PF, bool NT, bool NTU, int TPB, bool S9>
__device__ __forceinline__ void stencil_tile(const StencilArgs& a, const int t) {
  using T = EpiTraits<EPI>;
  static_assert(!S9 || (XM == XM_LDS && PF == 1), "9-point stencil: LDS row ring, prefetch 1");
  constexpr int UR = (PF == 1) ? 4 : 6;  // u ring: u_{r-1} .. u_{r+1+PF}
  constexpr int IR = PF + 1;             // per-row input ring
  constexpr int UNR = UR;                // unroll (multiple of UR, IR and 2)
  static_assert(UNR % IR == 0 && UNR % 2 == 0, "ring sizes");
  // LDS rows: double-buffered centre row (5-point); ring of 4 rows (9-point: rows r-1, r, r+1
  // are read at row r while row r+2's slot is free to be written one barrier later)
  constexpr int NLROW = S9 ? 4 : 2;
  __shared__ double2 lrow[NLROW][XM == XM_LDS ? TPB + 2 : 1];
  // 9-point: the y second difference of the current row, double-buffered (see the S9 step)
  __shared__ double2 ly[2][S9 ? TPB + 2 : 1];

  // XCD-aware tile map (see stencil_kernel): tile t is a 256-wide strip x one row band.
  const int tx = t % a.tiles_x;
  const int ty = t / a.tiles_x;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int n = a.n;
  const int i0 = tx * TPB;
  const int i = i0 + tid;
  const bool act = i < n;
  const int ic_ = min(i, n - 1);  // clamped column for loads
  // row band (wave-uniform; readfirstlane keeps the row loop and its prefetch branches on
  // the scalar unit)
  const int rb = __builtin_amdgcn_readfirstlane(a.row_begin + ty * a.row_step);
  const int re = __builtin_amdgcn_readfirstlane(min(rb + a.rows_per_block, a.row_end));

  auto rowp = [&](int r) -> const double2* {
    return r < 0 ? a.halo_lo : (r >= a.nl ? a.halo_hi : a.u + (size_t)r * n);
  };
  // which column each lane reads for its W / E inputs, and whether that value is real
  int iw, ie;
  bool lw, le;
  if constexpr (XM == XM_LDS) {
    // One broadcast load per wave and row serves both strip edges: lanes 0-31 read the W
    // halo column, lanes 32-63 the E halo column (two cache lines per wave; tid 0 keeps W,
    // tid TPB-1 keeps E).  Re-reading each lane's own column instead would cost a full row
    // of line requests per load, and miss entirely once u is loaded non-temporally.
    iw = ie = lane < kWave / 2 ? i0 - 1 : i0 + TPB;
    lw = tid == 0; le = tid == TPB - 1;
  } else if constexpr (XM == XM_SHFL) {
    // the same broadcast per wave: its W halo column for lanes 0-31, its E one for 32-63;
    // lane 0 keeps W, lane 63 keeps E (no block barrier: waves run independently)
    iw = ie = lane < kWave / 2 ? i - lane - 1 : i - lane + kWave;
    lw = lane == 0; le = lane == kWave - 1;
  } else {
    iw = i - 1; ie = i + 1; lw = act; le = act;
  }
  lw = lw && iw >= 0;
  le = le && ie < n;
  iw = min(max(iw, 0), n - 1);
  ie = min(max(ie, 0), n - 1);

  const double2 z2 = make_double2(0.0, 0.0);
  auto load_row_in = [&](int r, RowIn& v) {
    if constexpr (!CONSTC) v.ic = ld1<NT>(a.invc2 + (size_t)r * n + ic_);
    else v.ic = a.invc2_const;
    const double2* rp = rowp(S9 ? r + 1 : r);  // 9-point: edges of the row entering the ring
    v.eW = rp[iw];
    if constexpr (XM == XM_DIRECT) v.eE = rp[ie];  // else eW holds both edges (see above)
    if constexpr (T::reads_in1) v.b = ld2<NT>(a.in1 + (size_t)r * n + ic_);
  };
  auto load_u = [&](int r) { return ld2<NTU>(rowp(r) + ic_); };
  const cdouble_p tabj = (cdouble_p)(a.tab_j);
  struct Tab {
    double2 R2, BS, BN, OM;
    double2 R2m, R2p;  // 9-point: R2 of rows r-1 and r+1
  };
  const cdouble_p tabx = (cdouble_p)(a.tab_r2x);
  auto load_tab = [&](int r, Tab& tb) {
    const int ru = __builtin_amdgcn_readfirstlane(r);
    const cdouble_p q = tabj + 8 * ru;
    tb.R2 = make_double2(q[0], q[1]);
    tb.BS = make_double2(q[2], q[3]);
    tb.BN = make_double2(q[4], q[5]);
    tb.OM = make_double2(q[6], q[7]);
    if constexpr (S9) {
      const cdouble_p x = tabx + 2 * ru;  // entry r + 1 is row r: rows r-1, r+1 at r, r + 2
      tb.R2m = make_double2(x[0], x[1]);
      tb.R2p = make_double2(x[4], x[5]);
    }
  };

  const double2 AW = a.tab_i[ic_], AE = a.tab_i[n + ic_], R1 = a.tab_i[2 * n + ic_];
  // 9-point: R1 of the neighbouring columns (clamped at the grid edge, where they multiply
  // the zero Dirichlet values only)
  // 9-point: R1 of the strip's halo column for the two edge lanes (it only ever multiplies
  // zeros off the grid, so the clamped column is fine there)
  double2 R1e = R1;
  if constexpr (S9) {
    const int ce = tid == 0 ? i0 - 1 : i0 + TPB;
    R1e = a.tab_i[2 * n + min(max(ce, 0), n - 1)];
  }

  double2 U[UR];
  RowIn IN[IR];
  Tab TB[2];
  // Every load below is unconditional, with its row clamped into rows this band needs
  // anyway: hipcc's vmcnt bookkeeping takes the minimum over control-flow paths, so a
  // load under a (even uniform) branch would turn the next wait into vmcnt(0).
  U[0] = load_u(rb - 1);
  U[1] = load_u(rb);
  U[2] = load_u(rb + 1);
  load_row_in(rb, IN[0]);
  if constexpr (PF == 2) {
    U[3] = load_u(min(rb + 2, re));
    load_row_in(min(rb + 1, re - 1), IN[1]);
  }
  load_tab(rb, TB[0]);
  if constexpr (S9) {
    // rows rb-1 and rb enter the LDS ring before the loop (slot of row r: (r - rb + 1) & 3)
    // (selects by value: `c ? U[0] : z2` on lvalues selects stack addresses and moves the
    // whole register ring to scratch)
    const double2 em = rowp(rb - 1)[iw], ec = rowp(rb)[iw];
    lrow[0][tid + 1] = csel(act, U[0], z2);
    lrow[1][tid + 1] = csel(act, U[1], z2);
    if (tid == 0) {
      lrow[0][0] = csel(lw, em, z2);
      lrow[1][0] = csel(lw, ec, z2);
    }
    if (tid == TPB - 1) {
      lrow[0][TPB + 1] = csel(le, em, z2);
      lrow[1][TPB + 1] = csel(le, ec, z2);
    }
  }
  // 9-point register ring: x second differences X and W+E sums H of rows r-1 (m) and r (c)
  double2 Xm = z2, Xc = z2, Hm = z2, Hc = z2;
  if constexpr (S9) {
    __syncthreads();
    const cdouble_p x = tabx + 2 * __builtin_amdgcn_readfirstlane(rb);  // R2 of rows rb-1, rb
    const double2 R2a = make_double2(x[0], x[1]), R2b = make_double2(x[2], x[3]);
    const double2 w0 = lrow[0][tid], e0 = lrow[0][tid + 2];
    const double2 w1 = lrow[1][tid], e1 = lrow[1][tid + 2];
    Xm = cmul(R2a, cfma(AE, csub(e0, U[0]), cmul(AW, csub(w0, U[0]))));
    Xc = cmul(R2b, cfma(AE, csub(e1, U[1]), cmul(AW, csub(w1, U[1]))));
    Hm = cadd(w0, e0);
    Hc = cadd(w1, e1);
  }

  double sin = 1.0;
  if constexpr (T::scaled_in) {
    if (a.in_scale) sin = *a.in_scale;
  }
  double acc[kMaxNorms] = {0.0, 0.0};

  for (int r0 = rb; r0 < re; r0 += UNR) {
    static_for<0, UNR>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const int r = r0 + k;
      const bool live = r < re;  // uniform; steps past the band end only keep the ring going
      // ---- prefetch (distance PF rows) into ring slots that are dead by now ----
      U[(k + 2 + PF) % UR] = load_u(min(r + 1 + PF, re));
      load_row_in(min(r + PF, re - 1), IN[(k + PF) % IR]);
      load_tab(min(r + 1, re - 1), TB[(k + 1) % 2]);
      const double2 uS = U[k % UR], uC = U[(k + 1) % UR], uN = U[(k + 2) % UR];
      const RowIn& in = IN[k % IR];
      const Tab& tb = TB[k % 2];
      const size_t p = (size_t)min(r, re - 1) * n + ic_;
      const double2 bin = T::reads_in1 ? in.b : z2;  // prefetched with the row's inputs

      // ---- W/E neighbours ----
      const double2 uCm = act ? uC : z2;  // columns past n contribute zero (Dirichlet)
      const double2 eW = lw ? in.eW : z2;
      const double2 eE = le ? (XM == XM_DIRECT ? in.eE : in.eW) : z2;
      double2 uW = z2, uE = z2;
      double2 Yc = z2, Yw = z2, Ye = z2, Xp = z2, Hp = z2;
      if constexpr (S9) {
        // Separable form: with X(r') = R2(r') (AW (uW - uC) + AE (uE - uC)) the x second
        // difference of row r' and Y(i') = R1(i') (BS (uS - uC) + BN (uN - uC)) the y one of
        // column i' (this row's BS, BN), the operator is
        //   alpha (X(r) + Y(i)) + g (X(r-1) + X(r+1) + Y(i-1) + Y(i+1)) + M (c uC + d edges + e corners)
        // -- each X and each Y computed once.  Row r+1 enters the LDS ring (its edges arrived
        // with this row's inputs) and Y(i) of row r goes to LDS for the neighbouring columns;
        // the edge lanes add Y of the strip's halo columns from the ring's halo slots.
        double2* bS = lrow[k & 3];
        double2* bC = lrow[(k + 1) & 3];
        double2* bN = lrow[(k + 2) & 3];
        double2* yb = ly[k & 1];
        Yc = cmul(R1, cfma(tb.BN, csub(uN, uC), cmul(tb.BS, csub(uS, uC))));
        bN[tid + 1] = csel(act, uN, z2);
        yb[tid + 1] = csel(act, Yc, z2);
        if (tid == 0) {
          bN[0] = eW;
          const double2 hS = bS[0], hC = bC[0];
          yb[0] = cmul(R1e, cfma(tb.BN, csub(eW, hC), cmul(tb.BS, csub(hS, hC))));
        }
        if (tid == TPB - 1) {
          bN[TPB + 1] = eE;
          const double2 hS = bS[TPB + 1], hC = bC[TPB + 1];
          yb[TPB + 1] = cmul(R1e, cfma(tb.BN, csub(eE, hC), cmul(tb.BS, csub(hS, hC))));
        }
        __syncthreads();
        const double2 uNW = bN[tid], uNE = bN[tid + 2];
        Yw = yb[tid];
        Ye = yb[tid + 2];
        Xp = cmul(tb.R2p, cfma(AE, csub(uNE, uN), cmul(AW, csub(uNW, uN))));
        Hp = cadd(uNW, uNE);
      } else if constexpr (XM == XM_LDS) {
        double2* buf = lrow[k & 1];
        buf[tid + 1] = uCm;
        if (tid == 0) buf[0] = eW;
        if (tid == TPB - 1) buf[TPB + 1] = eE;
        __syncthreads();
        uW = buf[tid];
        uE = buf[tid + 2];
      } else if constexpr (XM == XM_SHFL) {
        const double2 sw = make_double2(__shfl_up(uCm.x, 1), __shfl_up(uCm.y, 1));
        const double2 se = make_double2(__shfl_down(uCm.x, 1), __shfl_down(uCm.y, 1));
        uW = lane == 0 ? eW : sw;
        uE = lane == kWave - 1 ? eE : se;
      } else {
        uW = eW;
        uE = eE;
      }

      // ---- coefficients (code.py:83-109) and the five-point product ----
      const double2 W = cmul(AW, tb.R2);
      const double2 E = cmul(AE, tb.R2);
      const double2 S = cmul(tb.BS, R1);
      const double2 N = cmul(tb.BN, R1);
      const double2 M = cscale(cmul(tb.OM, R1), in.ic);
      const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
      double2 D, Db, Au;
      if constexpr (!S9) {
        D = csub(M, sum4);
        Db = D;
        if constexpr (T::shifted) Db = csub(cmul(M, a.mshift), sum4);
        const double2 Dc = (EPI == EPI_SL_SWEEP) ? Db : D;
        Au = cmul(S, uS);
        Au = cfma(W, uW, Au);
        Au = cfma(Dc, uC, Au);
        Au = cfma(E, uE, Au);
        Au = cfma(N, uN, Au);
      } else {
        const Stencil9W w = a.w9;
        const double2 Mb = T::shifted ? cmul(M, a.mshift) : M;
        D = stencil9_diag(M, sum4, w);
        Db = stencil9_diag(Mb, sum4, w);
        // the applied operator: A_beta in the second sweep, A everywhere else
        const double2 Dc = (EPI == EPI_SL_SWEEP) ? Db : D;
        const double2 Mo = (EPI == EPI_SL_SWEEP) ? Mb : M;
        const double2 lap = cadd(Xc, Yc);
        const double2 avg = cadd(cadd(Xm, Xp), cadd(Yw, Ye));
        const double2 edges = cadd(Hc, cadd(uS, uN));
        const double2 corners = cadd(Hm, Hp);
        const double2 mix = cadd(cadd(cscale(uC, w.c), cscale(edges, w.d)), cscale(corners, w.e));
        Au = cfma(Mo, mix, cadd(cscale(lap, w.alpha), cscale(avg, w.g)));
        (void)Dc;
        Xm = Xc;
        Xc = Xp;
        Hm = Hc;
        Hc = Hp;
      }

      if (act && live) {
        if constexpr (EPI == EPI_AX) {
          store2(a.out0 + p, cscale(Au, sin), NT);
        } else if constexpr (EPI == EPI_JAC) {
          store2(a.out0 + p, cscale(cdiv(Au, D), sin), NT);
        } else if constexpr (EPI == EPI_RES) {
          const double2 rr = csub(bin, Au);
          store2(a.out0 + p, rr, NT);
          acc[0] += cabs2(rr);
        } else if constexpr (EPI == EPI_RES_JAC) {
          const double2 rr = csub(bin, Au);
          const double2 zz = cdiv(rr, D);
          store2(a.out0 + p, zz, NT);
          acc[0] += cabs2(rr);
          acc[1] += cabs2(zz);
        } else if constexpr (EPI == EPI_RES_SL) {
          const double2 rr = csub(bin, Au);
          store2(a.out0 + p, rr, NT);
          store2(a.out1 + p, cscale(cdiv(rr, Db), a.damping), NT);
          acc[0] += cabs2(rr);
        } else if constexpr (EPI == EPI_SL_FIRST) {
          const double2 tt = cscale(Au, sin);
          store2(a.out0 + p, tt, NT);
          store2(a.out1 + p, cscale(cdiv(tt, Db), a.damping), NT);
        } else if constexpr (EPI == EPI_SL_SWEEP) {
          store2(a.out0 + p, cadd(uC, cscale(cdiv(csub(bin, Au), Db), a.damping)), NT);
        }
      }
    });
  }
  block_reduce_store<T::nacc, TPB>(acc, a.partials, t);
  if constexpr (T::nacc > 0 || XM == XM_LDS) __syncthreads();  // LDS reuse by the next tile
}

// Non-marching tile shape (tuning variants kTileVariant + R, plain apply of the 5-point
// operator only): a 256-thread block computes an R-row x 256-column tile in one shot -- every
// load of its R + 2 input rows, R 1/c^2 rows and R broadcast edge values is issued up front --
// and exchanges W/E neighbours by wave shuffles (no LDS, no barrier).  Blocks run in plain
// order, so the concurrently resident tiles cover one narrow address window of the grid (the
// flat stream's access pattern); the two halo rows a tile shares with each vertical
// neighbour come mostly from L2 / the Infinity Cache.  Same per-point arithmetic as
// stencil_tile: bit-identical results.
// One tile t of tile_kernel (and of the persistent tile_persist_kernel, which loops over tiles)
// NTU: 0 u through the cache, 1 every u row non-temporal, 2 only the tile's private rows
// non-temporal (rows rb+1 .. re-2: no other tile reads them; the four rows a tile shares with
// its vertical neighbours stay cached for them)
template <int EPI, bool CONSTC, int R, bool NT, int NTU>
__device__ __forceinline__ void tile_do(const StencilArgs& a, const int t) {
  static_assert(EPI == EPI_AX || EPI == EPI_JAC, "tile shape: plain and Jacobi-fused apply");
  constexpr int TPB = kStencilThreads;
  const int n = a.n;
  const int tiles_x = a.tiles_x;
  const int tx = t % tiles_x, ty = t / tiles_x;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int i = tx * TPB + tid;
  const bool act = i < n;
  const int ic_ = min(i, n - 1);
  const int rb = __builtin_amdgcn_readfirstlane(a.row_begin + ty * R);
  const int re = __builtin_amdgcn_readfirstlane(min(rb + R, a.row_end));
  auto rowp = [&](int r) -> const double2* {
    return r < 0 ? a.halo_lo : (r >= a.nl ? a.halo_hi : a.u + (size_t)r * n);
  };
  // wave-edge lanes: lanes 0-31 load the wave's W halo column, 32-63 its E one (broadcast)
  int iw = lane < kWave / 2 ? i - lane - 1 : i - lane + kWave;
  const bool lw = lane == 0 && iw >= 0;
  const bool le = lane == kWave - 1 && iw < n;
  iw = min(max(iw, 0), n - 1);
  const double2 z2 = make_double2(0.0, 0.0);
  double2 U[R + 2], EG[R];
  double IC[R];
  #pragma unroll
  for (int m = 0; m < R + 2; ++m) {
    const double2* q = rowp(min(rb - 1 + m, re)) + ic_;
    U[m] = (NTU == 1 || (NTU == 2 && m >= 2 && m < R)) ? ld2<true>(q) : ld2<false>(q);
  }
  #pragma unroll
  for (int m = 0; m < R; ++m) {
    const int r = min(rb + m, re - 1);
    IC[m] = CONSTC ? a.invc2_const : ld1<NT>(a.invc2 + (size_t)r * n + ic_);
    EG[m] = rowp(r)[iw];
  }
  const cdouble_p tabj = (cdouble_p)(a.tab_j);
  const double2 AW = a.tab_i[ic_], AE = a.tab_i[n + ic_], R1 = a.tab_i[2 * n + ic_];
  double sin = 1.0;
  if (a.in_scale) sin = *a.in_scale;
  #pragma unroll
  for (int m = 0; m < R; ++m) {
    const int r = rb + m;
    const int ru = __builtin_amdgcn_readfirstlane(min(r, re - 1));
    const cdouble_p q = tabj + 8 * ru;
    const double2 R2 = make_double2(q[0], q[1]), BS = make_double2(q[2], q[3]);
    const double2 BN = make_double2(q[4], q[5]), OM = make_double2(q[6], q[7]);
    const double2 uS = U[m], uC = U[m + 1], uN = U[m + 2];
    const double2 uCm = act ? uC : z2;
    const double2 sw = make_double2(__shfl_up(uCm.x, 1), __shfl_up(uCm.y, 1));
    const double2 se = make_double2(__shfl_down(uCm.x, 1), __shfl_down(uCm.y, 1));
    const double2 e = EG[m];
    const double2 uW = lane == 0 ? (lw ? e : z2) : sw;
    const double2 uE = lane == kWave - 1 ? (le ? e : z2) : se;
    const double2 W = cmul(AW, R2);
    const double2 E = cmul(AE, R2);
    const double2 S = cmul(BS, R1);
    const double2 N = cmul(BN, R1);
    const double2 M = cscale(cmul(OM, R1), IC[m]);
    const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
    const double2 D = csub(M, sum4);
    double2 Au = cmul(S, uS);
    Au = cfma(W, uW, Au);
    Au = cfma(D, uC, Au);
    Au = cfma(E, uE, Au);
    Au = cfma(N, uN, Au);
    if (act && r < re) {
      // NT tiles: write-through stores -- the outputs leave L2 at once, so the halo rows the
      // next tiles re-read stay there (4096^2: 98.3-99.2 vs 100.8-100.9 us constant medium,
      // 116.7-117.5 vs 118.6-118.7 Marmousi-like; profiles/r06/r06v_ab_tile_sc1_stores.log)
      const double2 o = EPI == EPI_AX ? cscale(Au, sin) : cscale(cdiv(Au, D), sin);
#ifndef HH_AB_NT_STORE
      if constexpr (NT) st_wt(a.out0 + (size_t)r * n + ic_, o);
      else store2(a.out0 + (size_t)r * n + ic_, o, false);
#else
      store2(a.out0 + (size_t)r * n + ic_, o, NT);
#endif
    }
  }
}

// a.tiles_per_xcd > 0: XCD-contiguous tile runs -- block b runs on XCD b % 8 and takes tile
// (b % 8) tiles_per_xcd + b / 8, so each XCD sweeps its own contiguous run of tiles and a tile's
// vertical neighbours (tiles_x apart) share its L2.  In plain order they do only when tiles_x
// is a multiple of 8 (4096^2, 8192^2); at 5792^2 / 11584^2 (the 2- and 8-GPU weak-scaling
// slabs) every halo row goes to another XCD's L2: 1.23-1.29x the algorithmic fetch
// (profiles/r05/r05n_pmc_shapes.log) against 1.03x -- from the Infinity Cache: the map is the
// slower one (tile_xcd_map).
template <int EPI, bool CONSTC, int R, bool NT, int NTU>
__global__ __launch_bounds__(kStencilThreads) void tile_kernel(const StencilArgs a) {
  if (a.stop && *a.stop) return;  // queued GMRES cycle already stopped
  int t = blockIdx.x;
  if (a.tiles_per_xcd > 0) {
    t = (blockIdx.x & 7) * a.tiles_per_xcd + (blockIdx.x >> 3);
    if (t >= a.tiles_x * a.tiles_y) return;
  }
  tile_do<EPI, CONSTC, R, NT, NTU>(a, t);
}

// The same tiles from a persistent grid (a.grid_blocks blocks, as many as are resident at
// once): block b takes tiles b, b + G, b + 2 G, ... -- the resident blocks still sweep one
// contiguous window of tiles, without the dispatch of tiles_x * tiles_y blocks and with a
// tail of at most one tile per block (tuning variants kTilePersist + R).  Bit-identical.
template <int EPI, bool CONSTC, int R, bool NT, int NTU>
__global__ __launch_bounds__(kStencilThreads) void tile_persist_kernel(const StencilArgs a,
                                                                       int tiles) {
  if (a.stop && *a.stop) return;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) tile_do<EPI, CONSTC, R, NT, NTU>(a, t);
}

// The tile shape for the 9-point operator (stencil_tile's separable S9 form, same association,
// bit-identical): every row of the tile and its two halo rows gets its x second difference X
// and W+E sum H from wave shuffles (+ the broadcast edge values at the wave edges); the y
// second difference Y of each output row is exchanged by shuffles too, the wave-edge lanes
// computing Y of the halo column from the edge values of the three rows.
template <int EPI, bool CONSTC, int R, bool NT, bool NTU>
__global__ __launch_bounds__(kStencilThreads) void tile9_kernel(const StencilArgs a) {
  static_assert(EPI == EPI_AX || EPI == EPI_JAC, "tile shape: plain and Jacobi-fused apply");
  if (a.stop && *a.stop) return;
  constexpr int TPB = kStencilThreads;
  const int n = a.n;
  const int tiles_x = a.tiles_x;
  const int t = blockIdx.x;
  const int tx = t % tiles_x, ty = t / tiles_x;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int i = tx * TPB + tid;
  const bool act = i < n;
  const int ic_ = min(i, n - 1);
  const int rb = __builtin_amdgcn_readfirstlane(a.row_begin + ty * R);
  const int re = __builtin_amdgcn_readfirstlane(min(rb + R, a.row_end));
  auto rowp = [&](int r) -> const double2* {
    return r < 0 ? a.halo_lo : (r >= a.nl ? a.halo_hi : a.u + (size_t)r * n);
  };
  int iw = lane < kWave / 2 ? i - lane - 1 : i - lane + kWave;
  const bool lw = lane == 0 && iw >= 0;
  const bool le = lane == kWave - 1 && iw < n;
  iw = min(max(iw, 0), n - 1);
  const double2 z2 = make_double2(0.0, 0.0);
  double2 U[R + 2], EG[R + 2];
  double IC[R];
  #pragma unroll
  for (int m = 0; m < R + 2; ++m) {
    const double2* rp = rowp(min(rb - 1 + m, re));
    U[m] = ld2<NTU>(rp + ic_);
    EG[m] = rp[iw];
  }
  #pragma unroll
  for (int m = 0; m < R; ++m) {
    const int r = min(rb + m, re - 1);
    IC[m] = CONSTC ? a.invc2_const : ld1<NT>(a.invc2 + (size_t)r * n + ic_);
  }
  const cdouble_p tabj = (cdouble_p)(a.tab_j);
  const cdouble_p tabx = (cdouble_p)(a.tab_r2x);
  const double2 AW = a.tab_i[ic_], AE = a.tab_i[n + ic_], R1 = a.tab_i[2 * n + ic_];
  const double2 R1e = a.tab_i[2 * n + iw];  // the wave-edge lanes' halo column
  const Stencil9W w = a.w9;
  double sin = 1.0;
  if (a.in_scale) sin = *a.in_scale;
  auto shfl_up = [&](double2 v) { return make_double2(__shfl_up(v.x, 1), __shfl_up(v.y, 1)); };
  auto shfl_dn = [&](double2 v) { return make_double2(__shfl_down(v.x, 1), __shfl_down(v.y, 1)); };
  // X and H of tile row m (0 .. R+1 <-> rows rb-1 .. rb+R)
  auto xh = [&](int m, double2& X, double2& Hs) {
    const int ru = __builtin_amdgcn_readfirstlane(min(rb - 1 + m, re) + 1);  // tab_r2x entry
    const double2 R2 = make_double2(tabx[2 * ru], tabx[2 * ru + 1]);
    const double2 uC = U[m];
    const double2 uCm = act ? uC : z2;
    const double2 sw = shfl_up(uCm), se = shfl_dn(uCm);
    const double2 e = EG[m];
    const double2 uW = lane == 0 ? (lw ? e : z2) : sw;
    const double2 uE = lane == kWave - 1 ? (le ? e : z2) : se;
    X = cmul(R2, cfma(AE, csub(uE, uC), cmul(AW, csub(uW, uC))));
    Hs = cadd(uW, uE);
  };
  double2 Xm, Xc, Hm, Hc;
  xh(0, Xm, Hm);
  xh(1, Xc, Hc);
  #pragma unroll
  for (int m = 1; m <= R; ++m) {
    const int r = rb + m - 1;
    const int ru = __builtin_amdgcn_readfirstlane(min(r, re - 1));
    const cdouble_p q = tabj + 8 * ru;
    const double2 R2 = make_double2(q[0], q[1]), BS = make_double2(q[2], q[3]);
    const double2 BN = make_double2(q[4], q[5]), OM = make_double2(q[6], q[7]);
    double2 Xp, Hp;
    xh(m + 1, Xp, Hp);
    const double2 uS = U[m - 1], uC = U[m], uN = U[m + 1];
    const double2 Yc = cmul(R1, cfma(BN, csub(uN, uC), cmul(BS, csub(uS, uC))));
    const double2 Ycm = act ? Yc : z2;
    // Y of the wave's halo column from the edge values of rows r-1, r, r+1 (zero off the grid)
    const double2 eS = EG[m - 1], eC = EG[m], eN = EG[m + 1];
    const double2 Yh = cmul(R1e, cfma(BN, csub(eN, eC), cmul(BS, csub(eS, eC))));
    const double2 sw = shfl_up(Ycm), se = shfl_dn(Ycm);
    const double2 Yw = lane == 0 ? (lw ? Yh : z2) : sw;
    const double2 Ye = lane == kWave - 1 ? (le ? Yh : z2) : se;
    const double2 W = cmul(AW, R2);
    const double2 E = cmul(AE, R2);
    const double2 S = cmul(BS, R1);
    const double2 N = cmul(BN, R1);
    const double2 M = cscale(cmul(OM, R1), IC[m - 1]);
    const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
    const double2 lap = cadd(Xc, Yc);
    const double2 avg = cadd(cadd(Xm, Xp), cadd(Yw, Ye));
    const double2 edges = cadd(Hc, cadd(uS, uN));
    const double2 corners = cadd(Hm, Hp);
    const double2 mix = cadd(cadd(cscale(uC, w.c), cscale(edges, w.d)), cscale(corners, w.e));
    const double2 Au = cfma(M, mix, cadd(cscale(lap, w.alpha), cscale(avg, w.g)));
    if (act && r < re) {
      if constexpr (EPI == EPI_AX) store2(a.out0 + (size_t)r * n + ic_, cscale(Au, sin), NT);
      else store2(a.out0 + (size_t)r * n + ic_, cscale(cdiv(Au, stencil9_diag(M, sum4, w)), sin), NT);
    }
    Xm = Xc;
    Xc = Xp;
    Hm = Hc;
    Hc = Hp;
  }
}

// Pointwise operations needing only the diagonal D (or D_beta) of a point.
template <int OP, bool CONSTC>
__global__ __launch_bounds__(kStencilThreads) void point_kernel(const PointArgs a) {
  if (a.stop && *a.stop) return;
  const int n = a.n;
  const int tiles_x = (n + kStencilThreads - 1) / kStencilThreads;
  const long ntiles = (long)tiles_x * a.nl;
  double acc[kMaxNorms] = {0.0, 0.0};
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int r = (int)(t / tiles_x);
    const int i = (int)(t % tiles_x) * kStencilThreads + threadIdx.x;
    if (i >= n) continue;
    const size_t p = (size_t)r * n + i;
    if constexpr (OP == PT_COPY_NORM) {
      const double2 v = a.in0[p];
      if (a.out0 && a.out0 != a.in0) a.out0[p] = v;
      acc[0] += cabs2(v);
      continue;
    } else {
      const double2* tj = a.tab_j + 4 * r;
      const double2 R2 = tj[0], BS = tj[1], BN = tj[2], OM = tj[3];
      const double2 AW = a.tab_i[i], AE = a.tab_i[n + i], R1 = a.tab_i[2 * n + i];
      const double ic = CONSTC ? a.invc2_const : a.invc2[p];
      const double2 W = cmul(AW, R2);
      const double2 E = cmul(AE, R2);
      const double2 S = cmul(BS, R1);
      const double2 N = cmul(BN, R1);
      const double2 M = cscale(cmul(OM, R1), ic);
      const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
      // 9-point diagonal: c M - alpha (W + E + S + N)  (hh_stencil9.hpp)
      if constexpr (OP == PT_DIAG) {
        a.out0[p] = a.s9 ? stencil9_diag(M, sum4, a.w9) : csub(M, sum4);
      } else if constexpr (OP == PT_JAC) {
        const double2 z = cdiv(a.in0[p], a.s9 ? stencil9_diag(M, sum4, a.w9) : csub(M, sum4));
        a.out0[p] = z;
        acc[0] += cabs2(z);
      } else if constexpr (OP == PT_SL_FIRST) {
        const double2 Mb = cmul(M, a.mshift);
        const double2 Db = a.s9 ? stencil9_diag(Mb, sum4, a.w9) : csub(Mb, sum4);
        a.out0[p] = cscale(cdiv(a.in0[p], Db), a.damping);
      }
    }
  }
  if constexpr (OP == PT_JAC || OP == PT_COPY_NORM) {
    block_reduce_store<1>(acc, a.partials, blockIdx.x);
  }
}

// Default exchange/prefetch/store variant for every epilogue (tuned on MI355X, see
// DESIGN.md "stencil variants"); the benchmark kernel (EPI_AX) can run all 12 variants.
constexpr int kDefaultVariant = 30;  // XM_LDS, PF 1, NT stores + NT 1/c^2 loads, cached u, 512-wide
constexpr int kSmallVariant = 18;    // 256-wide strips, NT u loads (grids below 2048)
constexpr int kSmallCachedVariant = 8;  // 256-wide strips, wave-shuffle exchange, cached u
                                        // (plain apply below 2048: 8.2 vs 8.5 us for the LDS
                                        // exchange at 1024^2, profiles/r01w_tune_const_1024.log)
constexpr int kSolveVariant = 42;    // kDefaultVariant with NT u loads: solve epilogues, rows <= kLongRow
constexpr int kLongRow = 4608;
// Non-marching tile variants (plain 5-point apply): kTileVariant + 0/16 (NT u loads: + 16) +
// R rows per tile.
constexpr int kTileVariant = 96;
constexpr int kTileDefault = kTileVariant + 4;  // 4-row tiles, cached u, NT 1/c^2 and stores
// + 64: the same tiles from a persistent grid (tile_persist_kernel; cached u, NT 1/c^2 and
// stores; R rows per tile): kTilePersist + R
[[maybe_unused]] constexpr int kTilePersist = kTileVariant + 64;
// + 96: NT stores and 1/c^2, u non-temporal on the tile's private rows only (tile_do NTU = 2):
// kTilePrivNT + R.  Not a default: 4096^2 constant medium R = 6 97.3 vs 97.4 us, Marmousi-like
// R = 4 115.7 vs 114.8 (profiles/r06/r06o_tune_*_privnt.log).  (Also measured and not kept,
// round 6: the two edge-column loads restricted to the two lanes that use them, and interior
// strips taking the column tables as kernel arguments instead of three loads per lane -- each
// 0-4 % SLOWER, profiles/r06/r06r_*; the access-shape probe behind them: r06p_probe_tile_shape.log)
constexpr int kTilePrivNT = kTileVariant + 96;
constexpr bool tile_variant_known(int v) {
  const int w = v - kTileVariant, R = w % 16;
  return w >= 0 && (w < 80 || (w >= 96 && w < 112)) && R >= 2 && R <= 8 && R != 7;
}
// The 9-point operator instantiates the four LDS-exchange shapes below and takes the 5-point
// defaults: in its separable form (101-109 VGPRs, 4 waves per SIMD) it runs at the 5-point
// kernel's speed (4096^2 cold: 119.3 vs 119.6 us, profiles/r01v_tune_stencil9.log).
constexpr int kStencil9Variant = kSmallVariant;
bool stencil9_variant_valid(int v) {
  return v == 6 || v == kSmallVariant || v == kDefaultVariant || v == kSolveVariant ||
         (v >= kTileVariant && tile_variant_known(v));
}

// Variant table: V = XM + 3 (PF - 1) + 6 NT + 12 NTU + 24 (512-wide strips)  (0..47).
template <int V>
constexpr int variant_tpb() { return V >= 24 ? 512 : 256; }
template <int EPI, bool C, int V, bool S9 = false>
struct VariantLaunch {
  static void go(const StencilArgs& a, int blocks, hipStream_t s) {
    constexpr int W = V % 24;
    constexpr int XM = W % 3, PF = (W / 3) % 2 + 1;
    constexpr bool NT = (W / 6) % 2 == 1, NTU = W >= 12;
    constexpr int TPB = variant_tpb<V>();
    hipLaunchKernelGGL((stencil_kernel<EPI, C, XM, PF, NT, NTU, TPB, S9>), dim3(blocks), dim3(TPB),
                       0, s, a);
  }
};

template <int EPI, int V, bool S9 = false>
void launch_v(bool const_c, const StencilArgs& a, int blocks, hipStream_t s) {
  if (const_c) VariantLaunch<EPI, true, V, S9>::go(a, blocks, s);
  else VariantLaunch<EPI, false, V, S9>::go(a, blocks, s);
}

template <int EPI, int... Vs>
void launch_any(int v, bool const_c, const StencilArgs& a, int blocks, hipStream_t s) {
  bool done = false;
  ((v == Vs ? (launch_v<EPI, Vs>(const_c, a, blocks, s), done = true) : false), ...);
  if (!done) launch_v<EPI, kDefaultVariant>(const_c, a, blocks, s);
}

template <int EPI>
void launch_stencil_t(bool const_c, const StencilArgs& a, int blocks, hipStream_t s, int v) {
  if (a.tab_r2x) {
    // 9-point operator: LDS exchange, prefetch 1; 256- or 512-wide strips, NT or cached u
    if (v == 6) launch_v<EPI, 6, true>(const_c, a, blocks, s);
    else if (v == kDefaultVariant) launch_v<EPI, kDefaultVariant, true>(const_c, a, blocks, s);
    else if (v == kSolveVariant) launch_v<EPI, kSolveVariant, true>(const_c, a, blocks, s);
    else launch_v<EPI, kStencil9Variant, true>(const_c, a, blocks, s);
  } else if constexpr (EPI == EPI_AX) {
    launch_any<EPI, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21,
               22, 23, 24, 25, 26, 27, 30, 31, 32, 33, 42, 43, 44, 45>(v, const_c, a, blocks, s);
  } else {
    // every epilogue has the two default shapes: 256-wide (small grids) and 512-wide strips
    if (v == kSmallVariant) launch_v<EPI, kSmallVariant>(const_c, a, blocks, s);
    else if (v == kSolveVariant) launch_v<EPI, kSolveVariant>(const_c, a, blocks, s);
    else launch_v<EPI, kDefaultVariant>(const_c, a, blocks, s);
  }
}

template <int OP>
void launch_point_t(bool const_c, const PointArgs& a, int blocks, hipStream_t s) {
  if (const_c)
    hipLaunchKernelGGL((point_kernel<OP, true>), dim3(blocks), dim3(kStencilThreads), 0, s, a);
  else
    hipLaunchKernelGGL((point_kernel<OP, false>), dim3(blocks), dim3(kStencilThreads), 0, s, a);
}

}  // namespace

int stencil_rows_per_block(int n, int rows) {
  // Rows of 4608 points or fewer: ~2048 tiles (8 per CU) counted in 256-wide strips -- 32-row
  // bands at 4096^2; short bands keep small grids busy.  Longer rows: 16-row bands (measured
  // best at n = 5792 .. 16384 for both media, profiles/r01j_*, r01k_*).  A multiple of the
  // 4-row unroll.
  int rpb;
  if (n > kLongRow) {
    rpb = 16;
  } else {
    const int tiles_x = (n + kStencilThreads - 1) / kStencilThreads;
    long want_y = 2048 / tiles_x;
    if (want_y < 1) want_y = 1;
    rpb = (int)((rows + want_y - 1) / want_y);
    rpb = (rpb + 3) / 4 * 4;
  }
  if (rpb < 4) rpb = 4;
  if (rpb > 256) rpb = 256;
  if (rpb > rows) rpb = rows > 0 ? rows : 1;
  return rpb;
}

int stencil_resolve_variant(int epi, int requested, int n) {
  // 256-wide strips below n = 2048.  Above, the plain apply (EPI_AX) loads u through the
  // cache: on inputs no earlier launch left on the die -- every apply of a solve -- that is
  // the fastest shape at every size measured (n = 4096 .. 16384, profiles/r01l_* .. r01p_*).
  // The solve epilogues, whose input the previous kernel has just written, gain ~1 % from
  // NT u loads on rows up to kLongRow (tools/tune_gmres_variant.py,
  // profiles/r01i_tune_gmres_variant.log) and lose 4-8 % beyond.
  //   Below n = 2048 a grid's vectors fit the 256 MiB Infinity Cache: the plain apply then
  // loads u through the cache as well (1024^2: 8.6 vs 9.6 us with NT u loads,
  // profiles/r01w_tune_const_1024.log).
  //   A standalone plain apply (requested == -1) on n >= 2048 takes the non-marching tile
  // shape (tile_kernel, 4-row tiles): on cold inputs 5.84 vs 5.54 TB/s at 4096^2 and 5.8-6.0
  // vs 5.2-5.7 TB/s at 8192 .. 16384 (profiles/r01y_tune_tile*.log).  Inside a GMRES cycle
  // (requested == kVariantInSolve) the marching shape is kept: there the tile shape measured
  // 3-4 % slower (profiles/r01y_tune_tile_gmres.log).
  int autov = kDefaultVariant;
  if (n < 2048) autov = epi == EPI_AX ? kSmallCachedVariant : kSmallVariant;
  else if (epi != EPI_AX && n <= kLongRow) autov = kSolveVariant;
  else if (epi == EPI_AX && requested != kVariantInSolve) autov = kTileDefault;
  if (requested < 0 || sl2_variant(requested)) return autov;
  if (epi == EPI_AX) return stencil_variant_valid(requested) ? requested : autov;
  if (epi == EPI_JAC && requested >= kTileVariant && stencil_variant_valid(requested))
    return requested;  // the tile shape has the Jacobi-fused apply too
  return (requested == kSmallVariant || requested == kDefaultVariant || requested == kSolveVariant)
             ? requested
             : autov;
}

// The 5-point tile kernel's XCD-contiguous tile map (tile_kernel), HH_TILE_XCD=1; off by
// default.  It does what it is for -- the fetch of the 5792^2 / 11584^2 slabs falls from
// 1.23-1.29x to 1.006-1.021x the algorithmic bytes (profiles/r05/r05o_pmc_shapes_xcd.log) --
// but every shape runs 1-6 % SLOWER (r05o_ab_xcd_*.log: 11584^2 constant medium 5.55 -> 5.21
// TB/s): the plain order's cross-XCD halo re-reads are served by the Infinity Cache, not HBM
// (FETCH_SIZE counts both), while eight separate per-XCD streams cost DRAM locality.
bool tile_xcd_map(int tiles_x) {
  const bool on = knobs().tile_xcd == 1;
  (void)tiles_x;
  return on;
}

int stencil_bands(int rows, int rows_per_block, int row_step) {
  if (row_step <= 0) row_step = rows_per_block;
  return rows <= rows_per_block ? 1 : (rows - rows_per_block + row_step - 1) / row_step + 1;
}

int stencil_grid_blocks(int n, int rows, int rows_per_block, int row_step) {
  const int tiles_x = (n + kStencilThreads - 1) / kStencilThreads;
  const int tiles_y = stencil_bands(rows, rows_per_block, row_step);
  const int tiles = tiles_x * tiles_y;
  const int per_xcd = (tiles + 7) / 8;
  return per_xcd * 8;
}


int stencil_default_variant() { return kDefaultVariant; }
bool stencil_variant_valid(int v) {
  return (v >= 0 && v <= 27) || (v >= 30 && v <= 33) || (v >= 42 && v <= 45) || sl2_variant(v) ||
         (v >= kTileVariant && v < kTileVariant + 112 && tile_variant_known(v));
}

void launch_stencil(int epi, bool const_c, const StencilArgs& a_in, int nblocks_out[1],
                    hipStream_t stream, int variant) {
  StencilArgs a = a_in;
  const int rows = a.row_end - a.row_begin;
  int v = stencil_resolve_variant(epi, variant, a.n);
  // the 9-point operator has a subset of the shapes (launch_stencil_t): others take the default
  // 9-point standalone apply: 5-row tiles on long rows only (4096^2: tile 127.7 vs marching
  // 121.8 us; 8192^2: 479.9 vs 507.6 us; profiles/r01y_tune_tile9.log)
  if (a.tab_r2x && variant == -1 && v >= kTileVariant)
    v = a.n > kLongRow ? kTileVariant + 5 : kDefaultVariant;
  if (a.tab_r2x && !stencil9_variant_valid(v)) {
    v = stencil_resolve_variant(epi, -1, a.n);
    if (!stencil9_variant_valid(v))  // (the non-marching tile default is 5-point only)
      v = a.n < 2048 ? (epi == EPI_AX ? 6 : kSmallVariant)  // 6: LDS exchange, cached u
                     : (epi != EPI_AX && a.n <= kLongRow ? kSolveVariant : kDefaultVariant);
  }
  if (v >= kTileVariant && a.row_step > 0)  // spaced bands (halo rows): marching shape
    v = stencil_resolve_variant(epi, kVariantInSolve, a.n);
  // Taller tiles where they pay (the halo rows' share of the u loads (R + 2) / R): the constant
  // medium (no 1/c^2 stream, 32 B per unknown) 6 rows, 8 on rows longer than kLongRow; the
  // Marmousi-like medium 4 rows, 6 on rows longer than kLongRow.  With the write-through
  // stores (round 6): constant 4096^2 R5 / R6 / R8 95.2 / 95.3-95.9 / 98.2 us, 8192^2 R6 / R8
  // 358.5 / 354.5, 16384^2 1428 / 1380; Marmousi 4096^2 R4 / R6 113.7 / 114.7, 5792^2 232.2 /
  // 229.9, 8192^2 443.0 / 442.8, 11584^2 948.7 / 926.2 (profiles/r06/r06x_*, r06y_*; round 5:
  // r05s_tune_ntu_*.log)
  if (variant == -1 && v == kTileDefault && !a.tab_r2x) {
    if (const_c) v = kTileVariant + (a.n > kLongRow ? 8 : 6);
    else if (a.n > kLongRow) v = kTileVariant + 6;
  }
  if (v >= kTileVariant) {  // non-marching tiles (plain / Jacobi 5-point apply, tile_kernel)
    const int w = v - kTileVariant, R = w % 16;
    const bool ntu = (w / 16) % 2 == 1 && w < 64, nt = w < 32 || w >= 64;
    const bool priv = v >= kTilePrivNT;  // (5-point only; the 9-point tiles take NT stores)
    // (padding tiles_x to a multiple of 8, which would put vertically adjacent tiles on one
    // XCD, measured 3-7 % SLOWER at n = 5792 and 11584: profiles/r01y_tune_tile_pad.log)
    a.tiles_x = (a.n + kStencilThreads - 1) / kStencilThreads;
    a.tiles_y = (rows + R - 1) / R;
    const int tiles = a.tiles_x * a.tiles_y;
    const bool pers = w >= 64 && w < 80 && !a.tab_r2x;  // (5-point only)
    const bool xcd = !a.tab_r2x && !pers && tile_xcd_map(a.tiles_x);
    a.tiles_per_xcd = xcd ? (tiles + 7) / 8 : 0;
    nblocks_out[0] = 0;
    auto go = [&](auto ke, auto kr) {
      constexpr int E = decltype(ke)::value;
      constexpr int RR = decltype(kr)::value;
      const dim3 g(xcd ? 8 * a.tiles_per_xcd : tiles), b(kStencilThreads);
      if (pers) {  // persistent grid: every resident slot once
        static int slots = 0;
        if (slots == 0) {
          int dev = 0, cus = 0, per = 0;
          HIPC(hipGetDevice(&dev));
          HIPC(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
          HIPC(hipOccupancyMaxActiveBlocksPerMultiprocessor(
              &per, reinterpret_cast<const void*>(&tile_persist_kernel<E, false, RR, true, false>),
              kStencilThreads, 0));
          slots = std::max(1, cus * per);
        }
        const dim3 gp(std::min(tiles, slots));
        if (const_c)
          hipLaunchKernelGGL((tile_persist_kernel<E, true, RR, true, false>), gp, b, 0, stream, a,
                             tiles);
        else
          hipLaunchKernelGGL((tile_persist_kernel<E, false, RR, true, false>), gp, b, 0, stream,
                             a, tiles);
        return;
      }
      if (a.tab_r2x) {  // 9-point operator
        if (const_c) {
          if (!nt) hipLaunchKernelGGL((tile9_kernel<E, true, RR, false, false>), g, b, 0, stream, a);
          else if (ntu) hipLaunchKernelGGL((tile9_kernel<E, true, RR, true, true>), g, b, 0, stream, a);
          else hipLaunchKernelGGL((tile9_kernel<E, true, RR, true, false>), g, b, 0, stream, a);
        } else {
          if (!nt) hipLaunchKernelGGL((tile9_kernel<E, false, RR, false, false>), g, b, 0, stream, a);
          else if (ntu) hipLaunchKernelGGL((tile9_kernel<E, false, RR, true, true>), g, b, 0, stream, a);
          else hipLaunchKernelGGL((tile9_kernel<E, false, RR, true, false>), g, b, 0, stream, a);
        }
      } else if (const_c) {
        if (!nt) hipLaunchKernelGGL((tile_kernel<E, true, RR, false, false>), g, b, 0, stream, a);
        else if (priv) hipLaunchKernelGGL((tile_kernel<E, true, RR, true, 2>), g, b, 0, stream, a);
        else if (ntu) hipLaunchKernelGGL((tile_kernel<E, true, RR, true, true>), g, b, 0, stream, a);
        else hipLaunchKernelGGL((tile_kernel<E, true, RR, true, false>), g, b, 0, stream, a);
      } else {
        if (!nt) hipLaunchKernelGGL((tile_kernel<E, false, RR, false, false>), g, b, 0, stream, a);
        else if (priv) hipLaunchKernelGGL((tile_kernel<E, false, RR, true, 2>), g, b, 0, stream, a);
        else if (ntu) hipLaunchKernelGGL((tile_kernel<E, false, RR, true, true>), g, b, 0, stream, a);
        else hipLaunchKernelGGL((tile_kernel<E, false, RR, true, false>), g, b, 0, stream, a);
      }
    };
    auto go_r = [&](auto ke) {
      switch (R) {
        case 2: go(ke, std::integral_constant<int, 2>{}); break;
        case 3: go(ke, std::integral_constant<int, 3>{}); break;
        case 4: go(ke, std::integral_constant<int, 4>{}); break;
        case 5: go(ke, std::integral_constant<int, 5>{}); break;
        case 6: go(ke, std::integral_constant<int, 6>{}); break;
        default: go(ke, std::integral_constant<int, 8>{}); break;
      }
    };
    if (epi == EPI_JAC) go_r(std::integral_constant<int, EPI_JAC>{});
    else go_r(std::integral_constant<int, EPI_AX>{});
    return;
  }
  const int tpb = v >= 24 ? 512 : 256;
  a.tiles_x = (a.n + tpb - 1) / tpb;
  // bands start every row_step rows (spaced out only by the halo-row launch of a rank inside
  // the decomposition: rows 0 and nl-1 in one launch)
  if (a.row_step <= 0) a.row_step = a.rows_per_block;
  a.tiles_y = stencil_bands(rows, a.rows_per_block, a.row_step);
  a.tiles_per_xcd = (a.tiles_x * a.tiles_y + 7) / 8;
  int blocks = a.tiles_per_xcd * 8;
  if (a.grid_blocks > 0 && a.grid_blocks < blocks) blocks = (a.grid_blocks + 7) / 8 * 8;
  nblocks_out[0] = a.tiles_x * a.tiles_y;  // partial slots written (one per tile)
  switch (epi) {
    case EPI_AX: launch_stencil_t<EPI_AX>(const_c, a, blocks, stream, v); break;
    case EPI_JAC: launch_stencil_t<EPI_JAC>(const_c, a, blocks, stream, v); break;
    case EPI_RES: launch_stencil_t<EPI_RES>(const_c, a, blocks, stream, v); break;
    case EPI_RES_JAC: launch_stencil_t<EPI_RES_JAC>(const_c, a, blocks, stream, v); break;
    case EPI_RES_SL: launch_stencil_t<EPI_RES_SL>(const_c, a, blocks, stream, v); break;
    case EPI_SL_FIRST: launch_stencil_t<EPI_SL_FIRST>(const_c, a, blocks, stream, v); break;
    case EPI_SL_SWEEP: launch_stencil_t<EPI_SL_SWEEP>(const_c, a, blocks, stream, v); break;
    default: break;
  }
}

int point_blocks(size_t len) {
  size_t b = (len + kStencilThreads - 1) / kStencilThreads;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

void launch_point(int op, bool const_c, const PointArgs& a, int blocks, hipStream_t stream) {
  switch (op) {
    case PT_DIAG: launch_point_t<PT_DIAG>(const_c, a, blocks, stream); break;
    case PT_JAC: launch_point_t<PT_JAC>(const_c, a, blocks, stream); break;
    case PT_SL_FIRST: launch_point_t<PT_SL_FIRST>(const_c, a, blocks, stream); break;
    case PT_COPY_NORM: launch_point_t<PT_COPY_NORM>(const_c, a, blocks, stream); break;
    default: break;
  }
}

}  // namespace hh
