// The one-pass GMRES iteration with the two-sweep shifted-Laplace M for the first basis sizes
// (DESIGN 3g, round 6): fused_sl_iter_kernel's pass -- u_K = w_{K-1} - sum_k c_k u_k, w_K =
// M A (s u_K), <u_k, w_K> (k <= K), |w_K|^2, |u_K|^2 -- in the shape of the standalone fused M A
// (sl_fused.hip sl2_tile_v2), which streams its 40 B per unknown at 5.65 TB/s:
//   * overlapping strips instead of edge waves: thread t of a 256-thread block owns column
//     i0 - 2 + t, forms u_K there itself (k order: the stored value, bit for bit), takes the
//     first sweep on the inner 254 columns and writes w on the inner 252.  No lane-parallel sum,
//     no wave does more work than another, so nothing waits at the row's barrier for the edge
//     waves' ~130 extra instructions per step;
//   * one barrier per step (u of row L-1 and z1 of row L-2 published together into
//     double-buffered LDS rows, sl2_tile_1b's argument), row L-1's coefficients and its D_beta,
//     1/|D_beta|^2 carried into row L-2's second sweep;
//   * the projections' basis rows re-read one step ahead (L2: a block re-reads the rows it loaded
//     two steps before), so the kernel keeps no three-row ring and stays at four waves per SIMD;
//   * mask-free interior tiles (EDGE = false): every column and every row the band touches on
//     the grid and formed from memory.
// The operator and preconditioner arithmetic is fused_slk_kernel's term for term (stencil.hip's
// coefficients and FMA order); only the strip-edge columns' u_K (the old kernels' halo values,
// summed by a shuffle tree) and the order in which the projections' partial sums add differ, so
// histories agree with the older passes to rounding.  Used for K <= HH_SLV (knobs.cpp).
#include <algorithm>
#include <cstddef>

#include "hh_internal.hpp"
#include "hh_complex.hpp"
#include "hh_wave.hpp"
#include "hh_fused.hpp"

namespace hh {
namespace {
using namespace fusedk;

constexpr int kWO = kT - 4;  // output columns per strip

// the band of this block: tiles dealt to XCDs in contiguous runs (block b -> XCD b % 8)
struct BandV {
  bool live;
  int tx, rb, re;
};
__device__ __forceinline__ BandV band_v(const FusedArgs& a) {
  const int tiles_x = (a.n + kWO - 1) / kWO, T = tiles_x * a.bands;
  const int per_xcd = (T + 7) / 8;
  const int tile = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
  BandV b;
  b.live = tile < T;
  b.tx = b.live ? tile % tiles_x : 0;
  const int ty = b.live ? tile / tiles_x : 0;
  const int step = a.row_step > 0 ? a.row_step : a.rows;
  b.rb = a.row_begin + ty * step;
  b.re = min(b.rb + a.rows, a.row_end);
  return b;
}

// KEEP: the projections' basis rows from a three-row LDS ring each thread writes for its own
// column when it forms u_K (12 KiB per vector per block; no barrier: the same lane reads it two
// steps later) instead of a re-read from L2 -- no registers for the re-read in flight
template <int K, bool CONSTC, bool EDGE, bool KEEP>
__device__ __forceinline__ void slv_band(const FusedArgs& a, const BandV bd, double2 (&acc)[K + 1],
                                         double& nw, double& nu, double2 (*lu)[kT + 2],
                                         double2 (*lz)[kT + 2], const double2* coef,
                                         double2 (*vk)[K][kT]) {
  const int n = a.n, nl = a.nl;
  const int t = threadIdx.x;
  const int c = bd.tx * kWO - 2 + t;  // this thread's column
  const bool cin = !EDGE || (c >= 0 && c < n);
  const int cc = EDGE ? min(max(c, 0), n - 1) : c;
  const bool outc = t >= 2 && t < kT - 2 && cin;  // an output column of this strip
  const int rb = bd.rb, re = bd.re;
  const int rlo = a.lo_mode == FROW_MEM ? -2 : 0, rhi = a.hi_mode == FROW_MEM ? nl + 2 : nl;
  const double sin = *a.sin;
  const double damp = a.damping;
  const double2 mshift = a.mshift;
  const double2 z = make_double2(0.0, 0.0);
  const double2 AW = a.tab_i[cc], AE = a.tab_i[n + cc], R1 = a.tab_i[2 * n + cc];
  const bool lo_halo = a.lo_mode == FROW_HALO, hi_halo = a.hi_mode == FROW_HALO;
  const double2* h_lo = lo_halo ? a.halo_lo : a.win;  // (a valid address either way)
  const double2* h_hi = hi_halo ? a.halo_hi : a.win;
  const unsigned bo = (unsigned)cc * (unsigned)sizeof(double2);
  int kz = 0;  // opaque zero: the coefficients' LDS reads stay in the loop
  // 1/c^2 at (row r, own column): the slab's rows, or the two rows beyond each side
  auto icv_at = [&](int r) {
    if constexpr (CONSTC) {
      return a.invc2_const;
    } else {
      const int rc = min(max(r, -2), nl + 1);
      const double* row = rc < 0 ? a.invc2_halo + (size_t)(rc + 2) * n
                                 : (rc >= nl ? a.invc2_halo + (size_t)(rc - nl + 2) * n
                                             : a.invc2 + (size_t)rc * n);
      return __builtin_nontemporal_load(row + cc);
    }
  };
  // ---- row L's loads (issued a step ahead): w_{K-1}, the K basis rows, the halo value, and
  // 1/c^2 of row L - 1
  double2 pw, pv[K], ph = z, pr[KEEP ? 1 : K];  // pr: basis rows of the step's output row
  double pic;
  auto issue = [&](int L) {
    const int Lc = min(L, re + 1);
    const int rr = min(max(Lc, rlo), rhi - 1);
    gd2* vrow = gptr(a.V + (ptrdiff_t)rr * n);
    gd2* wrow = gptr(a.win + (ptrdiff_t)rr * n);
    asm volatile("" : "+s"(vrow), "+s"(wrow));
    pw = ld_at(wrow, bo);
#pragma unroll
    for (int q = 0; q < K; ++q) pv[q] = ld_at(vrow + (size_t)q * a.ldv, bo);
    if constexpr (EDGE) {
      const bool lo = Lc < 0;
      const double2* base = lo ? h_lo : h_hi;
      const int idx = lo ? min(max(Lc + 2, 0), 1) : min(max(Lc - nl, 0), 1);
      ph = base[(size_t)idx * n + cc];
    }
    pic = icv_at(Lc - 1);
  };
  // the projections' basis rows of output row L - 2 (a clamped in-band row otherwise), issued at
  // the end of step L - 1, after the step's own uses of the previous ones
  auto issue_proj = [&](int L) {
    if constexpr (KEEP) return;
    const int rp = min(max(L - 2, rb), re - 1);
    gd2* prow = gptr(a.V + (ptrdiff_t)rp * n);
    asm volatile("" : "+s"(prow));
#pragma unroll
    for (int q = 0; q < (KEEP ? 0 : K); ++q) pr[q] = ld_at(prow + (size_t)q * a.ldv, bo);
  };
  double2 uP = z, uC = z, Tm = z, z1a = z, z1b = z;
  double2 Dbm = make_double2(1.0, 0.0);
  double invm = 1.0;
  issue(rb - 2);
  issue_proj(rb - 2);
  int buf = 0;
  for (int L0 = rb - 2; L0 <= re + 1; ++L0) {
    int L = L0;
    asm volatile("" : "+s"(L), "+s"(kz));
    // u_K on row L, own column: w_{K-1} - sum_k c_k u_k in k order (fused_slk_kernel's
    // expression), or the received / zero row outside the rows formed from memory
    double2 uN;
    {
      double2 w = pw;
#pragma unroll
      for (int q0 = 0; q0 < K; q0 += 4) {
        double2 cq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) cq[q] = coef[min(q0 + q, K - 1) + kz];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (q0 + q < K) w = csub(w, cmul(cq[q], pv[q0 + q < K ? q0 + q : 0]));
      }
      asm volatile("" : "+v"(w.x), "+v"(w.y));
      if constexpr (EDGE) {
        const bool halo = L < 0 ? lo_halo : hi_halo;
        uN = csel(cin, csel(L >= rlo && L < rhi, w, csel(halo, ph, z)), z);
      } else {
        uN = w;
      }
    }
    const double icv = pic;
    if constexpr (KEEP) {  // basis row L for the projections of step L + 2
      const int slot = (L % 3 + 3) % 3;
#pragma unroll
      for (int q = 0; q < K; ++q) vk[slot][q][t] = pv[q];
    }
    // row L + 1's loads, in flight during the rest of the step
    issue(L + 1);
    __builtin_amdgcn_sched_barrier(0);
    // u of row L - 1 and z1 of row L - 2 for the W / E neighbours
    lu[buf][1 + t] = uC;
    lz[buf][1 + t] = z1b;
    __syncthreads();
    const double2 uW = lu[buf][t], uE = lu[buf][t + 2];
    const double2 zW = lz[buf][t], zE = lz[buf][t + 2];
    // first sweep on row s = L - 1 (T = s A u, z1 = damp T / D_beta), own column
    const int s = L - 1;
    const cdouble_p q = crow(a.tab_j, min(max(s, -2), nl + 1));
    const double2 R2 = make_double2(q[0], q[1]), BS = make_double2(q[2], q[3]);
    const double2 BN = make_double2(q[4], q[5]), OM = make_double2(q[6], q[7]);
    const double2 W1 = cmul(AW, R2);
    const double2 E1 = cmul(AE, R2);
    const double2 S1 = cmul(BS, R1);
    const double2 N1 = cmul(BN, R1);
    const double2 M1 = cscale(cmul(OM, R1), icv);
    const double2 sum4 = cadd(cadd(cadd(W1, E1), S1), N1);
    const double2 D1 = csub(M1, sum4);
    const double2 Db1 = csub(cmul(M1, mshift), sum4);
    double2 Au = cmul(S1, uP);
    Au = cfma(W1, uW, Au);
    Au = cfma(D1, uC, Au);
    Au = cfma(E1, uE, Au);
    Au = cfma(N1, uN, Au);
    const double inv1 = 1.0 / fma(Db1.x, Db1.x, Db1.y * Db1.y);
    auto cdivr = [](double2 x, double2 b, double inv) {  // cdiv with the reciprocal given
      return make_double2(fma(x.x, b.x, x.y * b.y) * inv, fma(x.y, b.x, -x.x * b.y) * inv);
    };
    double2 T1, z1c;
    if constexpr (EDGE) {
      const bool v1 = cin && ((s >= 0 && s < nl) || (s < 0 && a.lo_mode != FROW_ZERO) ||
                              (s >= nl && a.hi_mode != FROW_ZERO));
      T1 = csel(v1, cscale(Au, sin), z);
      z1c = csel(v1, cscale(cdivr(T1, Db1, inv1), damp), z);
    } else {
      T1 = cscale(Au, sin);
      z1c = cscale(cdivr(T1, Db1, inv1), damp);
    }
    // second sweep on row r = L - 2 (A_beta on z1): its W, E, S, N formed again from the row
    // tables (the same expressions on the same operands), D_beta and 1/|D_beta|^2 carried
    const int r = L - 2;
    if (r >= rb && r < re) {  // (block-uniform)
      const cdouble_p q2 = crow(a.tab_j, r);
      const double2 R2r = make_double2(q2[0], q2[1]), BSr = make_double2(q2[2], q2[3]);
      const double2 BNr = make_double2(q2[4], q2[5]);
      const double2 Wm = cmul(AW, R2r), Em = cmul(AE, R2r);
      const double2 Sm = cmul(BSr, R1), Nm = cmul(BNr, R1);
      double2 Az = cmul(Sm, z1a);
      Az = cfma(Wm, zW, Az);
      Az = cfma(Dbm, z1b, Az);
      Az = cfma(Em, zE, Az);
      Az = cfma(Nm, z1c, Az);
      const double2 w = csel(outc, cadd(z1b, cscale(cdivr(csub(Tm, Az), Dbm, invm), damp)), z);
      const double2 uo = csel(outc, uP, z);
      if (outc) {
        const size_t p = (size_t)r * n + c;
        a.wout[p] = w;
        a.uout[p] = uP;
      }
      nu = fma(uo.x, uo.x, fma(uo.y, uo.y, nu));
      nw = fma(w.x, w.x, fma(w.y, w.y, nw));
#pragma unroll
      for (int k = 0; k < K; ++k)
        acc[k] = cfma_conj(KEEP ? vk[r % 3][k][t] : pr[KEEP ? 0 : k], w, acc[k]);
      acc[K] = cfma_conj(uo, w, acc[K]);
    }
    issue_proj(L + 1);  // (row L - 1's, for the next step)
    uP = uC;
    uC = uN;
    Tm = T1;
    z1a = z1b;
    z1b = z1c;
    Dbm = Db1;
    invm = inv1;
    buf ^= 1;
  }
}

// (Holding the allocation to four waves per SIMD at K <= 2 -- 128 VGPRs, 10-16 of them spilled
// -- measured slower: K = 1 291 vs 242 us, K = 2 479 vs 331 us; profiles/r06/r06i_*)
template <int K, bool CONSTC, bool KEEP>
__global__ __launch_bounds__(kT) void fused_slv_kernel(const FusedArgs a) {
  if (a.stop && *a.stop) return;
  __shared__ double2 coef[K];
  __shared__ double2 lu[2][kT + 2], lz[2][kT + 2];
  __shared__ double2 vk[KEEP ? 3 : 1][K][kT];
  const BandV bd = band_v(a);
  load_coef<K>(a, coef);
  if (threadIdx.x < 2) {  // (the pads only feed columns that are never output)
    lu[threadIdx.x][0] = lu[threadIdx.x][kT + 1] = make_double2(0.0, 0.0);
    lz[threadIdx.x][0] = lz[threadIdx.x][kT + 1] = make_double2(0.0, 0.0);
  }
  __syncthreads();
  double2 acc[K + 1];
#pragma unroll
  for (int k = 0; k <= K; ++k) acc[k] = make_double2(0.0, 0.0);
  double nw = 0.0, nu = 0.0;
  if (bd.live) {
    // interior tile: every column of the strip on the grid and every row of the band's march
    // (rb - 2 .. re + 2: the loads run one row ahead) formed from memory
    const int rlo = a.lo_mode == FROW_MEM ? -2 : 0, rhi = a.hi_mode == FROW_MEM ? a.nl + 2 : a.nl;
    const int i0 = bd.tx * kWO;
    const bool interior = i0 - 2 >= 0 && i0 + kT - 2 <= a.n && bd.rb - 2 >= rlo && bd.re + 1 < rhi;
    if (interior)
      slv_band<K, CONSTC, false, KEEP>(a, bd, acc, nw, nu, lu, lz, coef, vk);
    else
      slv_band<K, CONSTC, true, KEEP>(a, bd, acc, nw, nu, lu, lz, coef, vk);
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
void slv_launch(const FusedArgs& a, int blocks, hipStream_t s) {
  const bool keep = K <= knobs().slv_keep_max;
  if (a.invc2) {
    if (keep) hipLaunchKernelGGL((fused_slv_kernel<K, false, true>), dim3(blocks), dim3(kT), 0, s, a);
    else hipLaunchKernelGGL((fused_slv_kernel<K, false, false>), dim3(blocks), dim3(kT), 0, s, a);
  } else {
    if (keep) hipLaunchKernelGGL((fused_slv_kernel<K, true, true>), dim3(blocks), dim3(kT), 0, s, a);
    else hipLaunchKernelGGL((fused_slv_kernel<K, true, false>), dim3(blocks), dim3(kT), 0, s, a);
  }
}
template <int... Ks>
struct VTable {
  using FN = void (*)(const FusedArgs&, int, hipStream_t);
  static constexpr FN f[] = {slv_launch<Ks>...};
};
using SlvTable = VTable<1, 2, 3, 4, 5, 6>;

}  // namespace

constexpr int kSlvMaxK = 6;
// HH_SLV (knobs.cpp): the largest K that takes this kernel (0 = never; at most kSlvMaxK)
bool fused_slv_use(int K) { return K <= std::min<long>(knobs().slv_max_k, kSlvMaxK); }
int fused_slv_blocks(int n, int bands) {
  const int T = (n + kWO - 1) / kWO * bands;
  return (T + 7) / 8 * 8;
}
void launch_fused_slv(int K, const FusedArgs& a, int blocks, hipStream_t stream) {
  SlvTable::f[K - 1](a, blocks, stream);
}

}  // namespace hh
