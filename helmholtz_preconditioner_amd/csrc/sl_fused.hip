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
// rb-2 .. re+1).  (2) It needs z1 one column to each side, so strips overlap: a block of TPB
// threads computes the first sweep on TPB columns and writes w on the TPB-2 inner ones.  The
// arithmetic is stencil.hip's, term for term (coefficients, FMA order), so w is bit-identical
// to the two-launch path.
#include "hh_internal.hpp"
#include "hh_complex.hpp"

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

  auto rowp = [&](int r) -> const double2* {
    return r < 0 ? a.halo_lo : (r >= nl ? a.halo_hi : a.u + (size_t)r * n);
  };
  auto load_v = [&](int r) -> double2 {
    const double2* p = rowp(r) + cc;
    if constexpr (NTU)
      return make_double2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
    else
      return *p;
  };
  auto load_in = [&](int r, RowIn& v) {
    const int rc = min(max(r, 0), nl - 1);
    if constexpr (!CONSTC) v.ic = __builtin_nontemporal_load(a.invc2 + (size_t)rc * n + cc);
    else v.ic = a.invc2_const;
    v.e = rowp(r)[ie];
  };
  const cdouble_p tabj = (cdouble_p)(a.tab_j);
  auto load_tab = [&](int r, RowTab& tb) {
    const int ru = __builtin_amdgcn_readfirstlane(min(max(r, 0), nl - 1));
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
    z1 = csel(cin && s >= 0 && s < nl, cscale(cdiv(T, Db), a.damping), z2);
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

template <bool CONSTC, bool NTU, int TPB>
__global__ __launch_bounds__(TPB) void sl2_kernel(const StencilArgs a) {
  if (a.stop && *a.stop) return;  // queued GMRES cycle already stopped
  const int L = blockIdx.x;
  const int q = L >> 3, Q = gridDim.x >> 3;
  const int ntiles = a.tiles_x * a.tiles_y;
  for (int tt = q; tt < a.tiles_per_xcd; tt += Q) {
    const int t = (L & 7) * a.tiles_per_xcd + tt;
    if (t >= ntiles) break;  // uniform per block
    sl2_tile<CONSTC, NTU, TPB>(a, t);
  }
}

template <int TPB, bool NTU>
void launch_t(bool const_c, const StencilArgs& a, int blocks, hipStream_t s) {
  if (const_c) hipLaunchKernelGGL((sl2_kernel<true, NTU, TPB>), dim3(blocks), dim3(TPB), 0, s, a);
  else hipLaunchKernelGGL((sl2_kernel<false, NTU, TPB>), dim3(blocks), dim3(TPB), 0, s, a);
}

}  // namespace

void launch_sl2(bool const_c, const StencilArgs& a_in, hipStream_t stream, int variant) {
  StencilArgs a = a_in;
  const int n = a.n;
  // 256-wide strips (126 VGPRs: 4 blocks per CU instead of 2 at 512; 4096^2 inside GMRES(20):
  // 768 vs 754 it/s, profiles/r01v_tune_sl2*.log), non-temporal v (just written by the previous
  // kernel) on rows up to 4608 points; a stencil tuning variant (hh_op_tune) of the LDS family
  // picks the strip width (>= 24: 512) and NT v loads (% 24 >= 12)
  int tpb = 256;
  bool ntu = n <= 4608;
  if (variant == 6 || variant == 18 || variant == 30 || variant == 42) {
    tpb = variant >= 24 ? 512 : 256;
    ntu = variant % 24 >= 12;
  }
  const int rows = a.row_end - a.row_begin;
  a.row_step = a.rows_per_block;
  a.tiles_x = (n + (tpb - 2) - 1) / (tpb - 2);
  a.tiles_y = stencil_bands(rows, a.rows_per_block, a.row_step);
  a.tiles_per_xcd = (a.tiles_x * a.tiles_y + 7) / 8;
  const int blocks = a.tiles_per_xcd * 8;
  if (tpb == 256) {
    if (ntu) launch_t<256, true>(const_c, a, blocks, stream);
    else launch_t<256, false>(const_c, a, blocks, stream);
  } else {
    if (ntu) launch_t<512, true>(const_c, a, blocks, stream);
    else launch_t<512, false>(const_c, a, blocks, stream);
  }
}

}  // namespace hh
