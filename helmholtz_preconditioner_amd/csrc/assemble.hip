// Operator export: the CSR matrix build_A_matrix returns, written on the
// device from the same 1-D PML tables and 1/c^2 field the matrix-free stencil applies.
//
// Reference: get_A_diag_block code.py:118-126 (diags(c5) + diags(c1,-1) + diags(c2,1)),
// get_upper/lower_A_block code.py:130-154 (c4 / c3 on the +-n diagonals), build_A_matrix
// code.py:202-219 (block_diag + diags(up, n) + diags(lo, -n) -> canonical CSR).  Row
// p = j n + i (0-based) holds, in column order, S (p-n), W (p-1), D (p), E (p+1), N (p+n);
// a neighbour outside the grid has no entry (its coefficient still enters D).
// nnz(A) = 5 n^2 - 4 n.
//
// One thread per row (staged through LDS, see the kernel).  The row start is closed-form (no scan): with
//   rownnz(i, j) = 1 + [i>0] + [i<n-1] + [j>0] + [j<n-1],
// the entries before global layer j are j (3n-2) + n (max(j-1, 0) + min(j, n-1)) and the
// entries before column i inside layer j are i (1 + [j>0] + [j<n-1]) + max(i-1, 0) + min(i, n-1).
// Values are computed with exactly the stencil's operation order (stencil.hip), so the
// exported matrix is the operator the kernels apply, bit for bit.
//
// 9-point operator: row p holds SW, S, SE, W, C, E, NW, N, NE (those inside
// the grid), rownnz = (1 + [i>0] + [i<n-1]) (1 + [j>0] + [j<n-1]); entries before layer j are
// (3n-2) (j + max(j-1, 0) + min(j, n-1)), before column i inside layer j
// (1 + [j>0] + [j<n-1]) (i + max(i-1, 0) + min(i, n-1)).  nnz = (3n-2)^2.
#include "hh_internal.hpp"
#include "hh_complex.hpp"
#include "hh_stencil9.hpp"

#include <algorithm>

namespace hh {
namespace {

__host__ __device__ __forceinline__ long long lines_before(long long n, long long j) {
  return j + (j > 0 ? j - 1 : 0) + (j < n - 1 ? j : n - 1);
}
template <bool S9>
__host__ __device__ __forceinline__ long long layer_start(long long n, long long j) {
  if constexpr (S9) return (3 * n - 2) * lines_before(n, j);
  else return j * (3 * n - 2) + n * ((j > 0 ? j - 1 : 0) + (j < n - 1 ? j : n - 1));
}

// A block owns 256 consecutive rows, whose entries are one contiguous range of the output:
// every thread stages its row's <= 5 entries in LDS at (row start - block start), then the
// block writes the range out with consecutive lanes on consecutive entries (coalesced
// 16-B value / 4- or 8-B index stores; a thread's own entries would be 80 B apart per lane).
constexpr int kCsrRows = 256;

template <class IDX, bool S9>
__global__ __launch_bounds__(kCsrRows) void csr_export_kernel(const CsrArgs a, IDX* indices) {
  constexpr int kCsrMax = (S9 ? 9 : 5) * kCsrRows;
  __shared__ double2 sval[kCsrMax];
  __shared__ IDX sidx[kCsrMax];
  __shared__ long long sfirst, send;
  const long long n = a.n;
  const long long base = layer_start<S9>(n, a.rank_j0);  // first entry of this rank's rows
  const size_t len = (size_t)a.nl * a.n;
  const size_t nblk = (len + kCsrRows - 1) / kCsrRows;
  for (size_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {  // uniform per block
    const size_t t = blk * kCsrRows + threadIdx.x;
    const bool live = t < len;
    const size_t tc = live ? t : len - 1;
    const int jl = (int)(tc / a.n);
    const int i = (int)(tc % a.n);
    const long long j = a.j0 + jl;  // global layer
    const int up = j > 0, dn = j < n - 1;
    const int lt = i > 0, rt = i < n - 1;
    long long start;
    int cnt;
    if constexpr (S9) {
      start = layer_start<true>(n, j) + (1 + up + dn) * lines_before(n, i) - base;
      cnt = (1 + up + dn) * (1 + lt + rt);
    } else {
      start = layer_start<false>(n, j) + (long long)i * (1 + up + dn) + (i > 0 ? i - 1 : 0) +
              (i < n - 1 ? i : n - 1) - base;
      cnt = 1 + up + dn + lt + rt;
    }
    if (threadIdx.x == 0) sfirst = start;
    if (live && (threadIdx.x == kCsrRows - 1 || t == len - 1)) send = start + cnt;
    __syncthreads();
    const double2* tj = a.tab_j + 4 * jl;
    const double2 R2 = tj[0], BS = tj[1], BN = tj[2], OM = tj[3];
    const double2 AW = a.tab_i[i], AE = a.tab_i[n + i], R1 = a.tab_i[2 * n + i];
    const double ic = a.invc2 ? a.invc2[tc] : a.invc2_const;
    const double2 W = cmul(AW, R2);
    const double2 E = cmul(AE, R2);
    const double2 S = cmul(BS, R1);
    const double2 N = cmul(BN, R1);
    const double2 M = cscale(cmul(OM, R1), ic);
    const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
    if (live) {
      const long long p = j * n + i;  // global row = global diagonal column
      int q = (int)(start - sfirst);
      auto put = [&](bool in, double2 v, long long col) {
        if (in) { sval[q] = v; sidx[q] = (IDX)col; ++q; }
      };
      if constexpr (S9) {
        const double2 R2m = a.tab_r2x[jl], R2p = a.tab_r2x[jl + 2];
        const double2 R1m = a.tab_i[2 * n + (i > 0 ? i - 1 : 0)];
        const double2 R1p = a.tab_i[2 * n + (i < n - 1 ? i + 1 : n - 1)];
        const Coef9 c = stencil9_offdiag(W, E, S, N, AW, AE, BS, BN, R1m, R1p, R2m, R2p, M, a.w9);
        put(up && lt, c.sw, p - n - 1);
        put(up, c.s, p - n);
        put(up && rt, c.se, p - n + 1);
        put(lt, c.w, p - 1);
        put(true, stencil9_diag(M, sum4, a.w9), p);
        put(rt, c.e, p + 1);
        put(dn && lt, c.nw, p + n - 1);
        put(dn, c.n, p + n);
        put(dn && rt, c.ne, p + n + 1);
      } else {
        put(up, S, p - n);
        put(lt, W, p - 1);
        put(true, csub(M, sum4), p);
        put(rt, E, p + 1);
        put(dn, N, p + n);
      }
      a.indptr[a.row_off + t] = start;
      if (a.last && t == len - 1) a.indptr[a.row_off + len] = start + cnt;
    }
    __syncthreads();
    const long long first = sfirst;
    const int total = (int)(send - first);
    for (int k = threadIdx.x; k < total; k += kCsrRows) {
      __builtin_nontemporal_store(sval[k].x, &a.data[first + k].x);
      __builtin_nontemporal_store(sval[k].y, &a.data[first + k].y);
      indices[first + k] = sidx[k];
    }
    __syncthreads();  // LDS reuse by the next row block
  }
}

}  // namespace

long long csr_rank_nnz(int n, int j0, int j1, int points) {
  if (points == 9) return layer_start<true>(n, j1) - layer_start<true>(n, j0);
  return layer_start<false>(n, j1) - layer_start<false>(n, j0);
}

void launch_csr_export(const CsrArgs& a, int index_bytes, hipStream_t stream) {
  const size_t len = (size_t)a.nl * a.n;
  const int blocks = (int)std::min<size_t>((len + kCsrRows - 1) / kCsrRows, 16384);
  const bool s9 = a.tab_r2x != nullptr;
  if (index_bytes == 8) {
    long long* idx = static_cast<long long*>(a.indices);
    if (s9) hipLaunchKernelGGL((csr_export_kernel<long long, true>), dim3(blocks), dim3(256), 0, stream, a, idx);
    else hipLaunchKernelGGL((csr_export_kernel<long long, false>), dim3(blocks), dim3(256), 0, stream, a, idx);
  } else {
    int* idx = static_cast<int*>(a.indices);
    if (s9) hipLaunchKernelGGL((csr_export_kernel<int, true>), dim3(blocks), dim3(256), 0, stream, a, idx);
    else hipLaunchKernelGGL((csr_export_kernel<int, false>), dim3(blocks), dim3(256), 0, stream, a, idx);
  }
}

}  // namespace hh
