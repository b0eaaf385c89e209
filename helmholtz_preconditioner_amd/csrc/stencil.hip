// Matrix-free complex 5-point PML Helmholtz stencil for gfx950 (MI355X).
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
// Kernel shape: a block owns a 256-wide strip of i and marches a band of rows in j with a
// three-row register window (u_{j-1}, u_j, u_{j+1}) plus a one-row prefetch, so every u is
// read from HBM once; the W/E neighbours are exchanged through a double-buffered LDS row
// with a one-point halo at each side (one barrier per row).  Tiles are dealt to XCDs in
// contiguous bands so the band-edge halo rows of vertically adjacent tiles hit the same L2.
#include "hh_internal.hpp"
#include "hh_complex.hpp"

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

template <int NACC>
__device__ __forceinline__ void block_reduce_store(double (&acc)[kMaxNorms], double* partials,
                                                   int slot) {
  if constexpr (NACC > 0) {
    __shared__ double red[kMaxNorms][kStencilThreads / kWave];
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
      for (int w = 0; w < kStencilThreads / kWave; ++w) s += red[threadIdx.x][w];
      partials[(size_t)slot * kMaxNorms + threadIdx.x] = s;
    }
  }
}

template <int EPI, bool CONSTC>
__global__ __launch_bounds__(kStencilThreads) void stencil_kernel(const StencilArgs a) {
  using T = EpiTraits<EPI>;
  __shared__ double2 lrow[2][kStencilThreads + 2];

  // XCD-aware tile map: consecutive blocks go round-robin over the 8 XCDs, so give each XCD
  // a contiguous range of tiles (row-band major) -> vertically adjacent tiles share an L2.
  const int L = blockIdx.x;
  const int t = (L & 7) * a.tiles_per_xcd + (L >> 3);
  if (t >= a.tiles_x * a.tiles_y) return;  // uniform per block, before any barrier
  const int tx = t % a.tiles_x;
  const int ty = t / a.tiles_x;
  const int tid = threadIdx.x;
  const int n = a.n;
  const int i0 = tx * kStencilThreads;
  const int i = i0 + tid;
  const bool act = i < n;
  const int rb = a.row_begin + ty * a.rows_per_block;
  const int re = min(rb + a.rows_per_block, a.row_end);

  auto rowp = [&](int r) -> const double2* {
    return r < 0 ? a.halo_lo : (r >= a.nl ? a.halo_hi : a.u + (size_t)r * n);
  };

  const double2 z2 = make_double2(0.0, 0.0);
  double2 AW = z2, AE = z2, R1 = z2;
  if (act) {
    AW = a.tab_i[i];
    AE = a.tab_i[n + i];
    R1 = a.tab_i[2 * n + i];
  }
  const bool west_lane = tid == 0;
  const bool east_lane = tid == kStencilThreads - 1;
  const int iw = i0 - 1;
  const int ie = i0 + kStencilThreads;
  const bool has_w = iw >= 0;
  const bool has_e = ie < n;

  double2 uS = z2, uC = z2, uN = z2;
  double icC = a.invc2_const, icN = a.invc2_const;
  double2 eWc = z2, eEc = z2, eWn = z2, eEn = z2;
  if (act) {
    uS = rowp(rb - 1)[i];
    uC = rowp(rb)[i];
    uN = rowp(rb + 1)[i];
    if constexpr (!CONSTC) icC = a.invc2[(size_t)rb * n + i];
  }
  if (west_lane && has_w) eWc = rowp(rb)[iw];
  if (east_lane && has_e) eEc = rowp(rb)[ie];
  const double2* tj = a.tab_j + 4 * rb;
  double2 R2 = tj[0], BS = tj[1], BN = tj[2], OM = tj[3];

  double sin = 1.0;
  if constexpr (T::scaled_in) {
    if (a.in_scale) sin = *a.in_scale;
  }
  double acc[kMaxNorms] = {0.0, 0.0};

  for (int r = rb; r < re; ++r) {
    // ---- prefetch row r+1's operands (used next iteration) ----
    double2 uNN = z2;
    double2 R2n = R2, BSn = BS, BNn = BN, OMn = OM;
    const bool more = (r + 1) < re;
    if (more) {
      if (act) {
        uNN = rowp(r + 2)[i];
        if constexpr (!CONSTC) icN = a.invc2[(size_t)(r + 1) * n + i];
      }
      if (west_lane && has_w) eWn = rowp(r + 1)[iw];
      if (east_lane && has_e) eEn = rowp(r + 1)[ie];
      const double2* tn = a.tab_j + 4 * (r + 1);
      R2n = tn[0];
      BSn = tn[1];
      BNn = tn[2];
      OMn = tn[3];
    }
    double2 bin = z2;
    const size_t p = (size_t)r * n + i;
    if constexpr (T::reads_in1) {
      if (act) bin = a.in1[p];
    }

    // ---- W/E neighbours through LDS (double-buffered: one barrier per row) ----
    double2* buf = lrow[(r - rb) & 1];
    buf[tid + 1] = uC;
    if (west_lane) buf[0] = eWc;
    if (east_lane) buf[kStencilThreads + 1] = eEc;
    __syncthreads();
    const double2 uW = buf[tid];
    const double2 uE = buf[tid + 2];

    // ---- coefficients (code.py:83-109) and the five-point product ----
    const double2 W = cmul(AW, R2);
    const double2 E = cmul(AE, R2);
    const double2 S = cmul(BS, R1);
    const double2 N = cmul(BN, R1);
    const double2 M = cscale(cmul(OM, R1), icC);
    const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
    const double2 D = csub(M, sum4);
    double2 Db = D;
    if constexpr (T::shifted) Db = csub(cmul(M, a.mshift), sum4);
    const double2 Dc = (EPI == EPI_SL_SWEEP) ? Db : D;

    double2 Au = cmul(S, uS);
    Au = cfma(W, uW, Au);
    Au = cfma(Dc, uC, Au);
    Au = cfma(E, uE, Au);
    Au = cfma(N, uN, Au);

    if (act) {
      if constexpr (EPI == EPI_AX) {
        a.out0[p] = cscale(Au, sin);
      } else if constexpr (EPI == EPI_JAC) {
        a.out0[p] = cscale(cdiv(Au, D), sin);
      } else if constexpr (EPI == EPI_RES) {
        const double2 rr = csub(bin, Au);
        a.out0[p] = rr;
        acc[0] += cabs2(rr);
      } else if constexpr (EPI == EPI_RES_JAC) {
        const double2 rr = csub(bin, Au);
        const double2 zz = cdiv(rr, D);
        a.out0[p] = zz;
        acc[0] += cabs2(rr);
        acc[1] += cabs2(zz);
      } else if constexpr (EPI == EPI_RES_SL) {
        const double2 rr = csub(bin, Au);
        a.out0[p] = rr;
        a.out1[p] = cscale(cdiv(rr, Db), a.damping);
        acc[0] += cabs2(rr);
      } else if constexpr (EPI == EPI_SL_FIRST) {
        const double2 tt = cscale(Au, sin);
        a.out0[p] = tt;
        a.out1[p] = cscale(cdiv(tt, Db), a.damping);
      } else if constexpr (EPI == EPI_SL_SWEEP) {
        a.out0[p] = cadd(uC, cscale(cdiv(csub(bin, Au), Db), a.damping));
      }
    }

    // ---- rotate the register window ----
    uS = uC;
    uC = uN;
    uN = uNN;
    icC = icN;
    eWc = eWn;
    eEc = eEn;
    R2 = R2n;
    BS = BSn;
    BN = BNn;
    OM = OMn;
  }
  block_reduce_store<T::nacc>(acc, a.partials, t);
}

// Pointwise operations needing only the diagonal D (or D_beta) of a point.
template <int OP, bool CONSTC>
__global__ __launch_bounds__(kStencilThreads) void point_kernel(const PointArgs a) {
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
      if constexpr (OP == PT_DIAG) {
        a.out0[p] = csub(M, sum4);
      } else if constexpr (OP == PT_JAC) {
        const double2 z = cdiv(a.in0[p], csub(M, sum4));
        a.out0[p] = z;
        acc[0] += cabs2(z);
      } else if constexpr (OP == PT_SL_FIRST) {
        const double2 Db = csub(cmul(M, a.mshift), sum4);
        a.out0[p] = cscale(cdiv(a.in0[p], Db), a.damping);
      }
    }
  }
  if constexpr (OP == PT_JAC || OP == PT_COPY_NORM) {
    block_reduce_store<1>(acc, a.partials, blockIdx.x);
  }
}

template <int EPI>
void launch_stencil_t(bool const_c, const StencilArgs& a, int blocks, hipStream_t s) {
  if (const_c)
    hipLaunchKernelGGL((stencil_kernel<EPI, true>), dim3(blocks), dim3(kStencilThreads), 0, s, a);
  else
    hipLaunchKernelGGL((stencil_kernel<EPI, false>), dim3(blocks), dim3(kStencilThreads), 0, s, a);
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
  // Aim for ~4096 tiles (16 blocks per CU over 256 CUs) so the chip stays full while each
  // block marches a band long enough to amortise its two halo rows.
  const int tiles_x = (n + kStencilThreads - 1) / kStencilThreads;
  long want_y = 4096 / tiles_x;
  if (want_y < 1) want_y = 1;
  int rpb = (int)((rows + want_y - 1) / want_y);
  if (rpb < 16) rpb = 16;
  if (rpb > 256) rpb = 256;
  if (rpb > rows) rpb = rows > 0 ? rows : 1;
  return rpb;
}

int stencil_grid_blocks(int n, int rows, int rows_per_block) {
  const int tiles_x = (n + kStencilThreads - 1) / kStencilThreads;
  const int tiles_y = (rows + rows_per_block - 1) / rows_per_block;
  const int tiles = tiles_x * tiles_y;
  const int per_xcd = (tiles + 7) / 8;
  return per_xcd * 8;
}

void launch_stencil(int epi, bool const_c, const StencilArgs& a_in, int nblocks_out[1],
                    hipStream_t stream) {
  StencilArgs a = a_in;
  const int rows = a.row_end - a.row_begin;
  a.tiles_x = (a.n + kStencilThreads - 1) / kStencilThreads;
  a.tiles_y = (rows + a.rows_per_block - 1) / a.rows_per_block;
  a.tiles_per_xcd = (a.tiles_x * a.tiles_y + 7) / 8;
  const int blocks = a.tiles_per_xcd * 8;
  nblocks_out[0] = a.tiles_x * a.tiles_y;  // partial slots written (one per tile)
  switch (epi) {
    case EPI_AX: launch_stencil_t<EPI_AX>(const_c, a, blocks, stream); break;
    case EPI_JAC: launch_stencil_t<EPI_JAC>(const_c, a, blocks, stream); break;
    case EPI_RES: launch_stencil_t<EPI_RES>(const_c, a, blocks, stream); break;
    case EPI_RES_JAC: launch_stencil_t<EPI_RES_JAC>(const_c, a, blocks, stream); break;
    case EPI_RES_SL: launch_stencil_t<EPI_RES_SL>(const_c, a, blocks, stream); break;
    case EPI_SL_FIRST: launch_stencil_t<EPI_SL_FIRST>(const_c, a, blocks, stream); break;
    case EPI_SL_SWEEP: launch_stencil_t<EPI_SL_SWEEP>(const_c, a, blocks, stream); break;
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
