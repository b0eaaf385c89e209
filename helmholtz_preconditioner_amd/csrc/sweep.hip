// Sweeping moving-PML preconditioner (Engquist-Ying) for gfx950.
//
// Reference: get_Hm_coeffs / get_Hm code.py:222-290, get_A_FF/Fb1/b1F code.py:177-199,
// algo2_3 code.py:345-353 (SuperLU of H_F and of n-b sub-problems H_m), algo2_4
// code.py:356-385 (forward sweep, middle sweep, backward sweep, F-block correction).
//
// Every solve the sweep performs is lu_Hm.solve([0 .. 0, v])[-n:] = T_m v, the last-layer
// block of H_m^-1.  H_m covers b layers x n columns; ordered column-major (i slow, layer k
// fast) it is block-tridiagonal with b x b blocks:
//   D_i = tridiag over layers (c5 diagonal, c3 / c4 couplings between layers),
//   L_i = diag(c1) (column i-1),  U_i = diag(c2) (column i+1).
// Block Thomas replaces SuperLU: Lambda_0 = D_0, Lambda_i = D_i - L_i P_{i-1} U_{i-1},
// P_i = Lambda_i^-1 (Gauss-Jordan, partial pivoting), stored per (system, i).  A solve is
// then y_i = P_i (r_i - L_i y_{i-1}) forward and x_i = y_i - P_i U_i x_{i+1} backward.
// H_F = block_diag(A_11 .. A_bb) (code.py:178-183: no inter-layer blocks) is the same
// machinery with the inter-layer couplings switched off.
//
// Parallel shape: factorisation -- one wave per system (all n-b+1 in parallel); middle
// sweep -- one wave per layer (independent solves); forward / backward sweeps -- inherently
// sequential in the layer index, one persistent wave walking all layers (no per-layer
// launches).  Solve shape: see bt_solve.
#include "hh_internal.hpp"
#include "hh_complex.hpp"
#include "sweep.hpp"

#include <type_traits>

namespace hh {
namespace {

constexpr int kSW = 64;  // one wave per workgroup

template <int K, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (K < N) {
    f(std::integral_constant<int, K>{});
    sfor<K + 1, N>(f);
  }
}

// Per-lane view of the coefficients of system s at column i, row (layer) j.
struct RowCoef {
  double2 W, E, S, N, D;  // S/N: couplings to layers j-1 / j+1 inside the sub-problem
};

__device__ __forceinline__ RowCoef row_coef(const SweepArgs& a, int s, int i, int j) {
  RowCoef c;
  const double2 z = make_double2(0.0, 0.0);
  if (j >= a.b) {
    c.W = c.E = c.S = c.N = z;
    c.D = make_double2(1.0, 0.0);  // identity padding of the b x b blocks
    return c;
  }
  const int n = a.n;
  const double2 AW = a.tab_i[i], AE = a.tab_i[n + i], R1 = a.tab_i[2 * n + i];
  const double2* tk = a.tab_k + 4 * j;  // local-layer PML: s2 at (j+1) h (moving PML)
  const double2 R2 = tk[0], BS = tk[1], BN = tk[2], OM = tk[3];
  const int layer = (s == 0 ? 0 : s) + j;  // global 0-based layer of this row
  const double ic = a.invc2 ? a.invc2[(size_t)layer * n + i] : a.invc2_const;
  const double2 W = cmul(AW, R2), E = cmul(AE, R2), S = cmul(BS, R1), N = cmul(BN, R1);
  c.D = csub(cscale(cmul(OM, R1), ic), cadd(cadd(cadd(W, E), S), N));
  c.W = i > 0 ? W : z;
  c.E = i + 1 < n ? E : z;
  const bool coupled = s > 0;  // H_F has no inter-layer blocks (code.py:178-183)
  c.S = (coupled && j > 0) ? S : z;
  c.N = (coupled && j + 1 < a.b) ? N : z;
  return c;
}

// ------------------------------------------------------------------ factorisation
template <int B>
__global__ __launch_bounds__(kSW) void sweep_factor_kernel(const SweepArgs a) {
  if (a.stop && *a.stop) return;
  __shared__ double2 prow[2 * B];
  __shared__ double2 bufU[B];
  __shared__ double2 perm[B][B];
  __shared__ double2 bufS[B], bufN[B];
  const int s = blockIdx.x;
  const int lane = threadIdx.x;
  const bool row = lane < B;
  const int n = a.n;
  double2 prev[B];  // P_{i-1}, row `lane`
  sfor<0, B>([&](auto kc) { prev[decltype(kc)::value] = make_double2(0.0, 0.0); });
  double2 Uprev = make_double2(0.0, 0.0);  // U_{i-1}[lane]
  double2* P = a.P + (size_t)s * n * B * B;

  for (int i = 0; i < n; ++i) {
    const RowCoef c = row_coef(a, s, i, row ? lane : a.b);
    // U_{i-1} of every row, for the column scaling of P_{i-1}
    if (row) bufU[lane] = Uprev;
    if (row) bufS[lane] = c.S;
    if (row) bufN[lane] = c.N;
    __syncthreads();
    // Lambda row `lane` | identity row `lane`
    double2 A[B], R[B];
    sfor<0, B>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      double2 d = make_double2(0.0, 0.0);
      if (k == lane) d = c.D;
      if (k + 1 == lane) d = c.S;  // row lane couples to layer lane-1
      if (k == lane + 1) d = c.N;  // row lane couples to layer lane+1
      // - L_i[lane] * P_{i-1}[lane][k] * U_{i-1}[k]
      A[k] = csub(d, cmul(c.W, cmul(prev[k], bufU[k])));
      R[k] = make_double2(k == lane ? 1.0 : 0.0, 0.0);
    });
    __syncthreads();
    // Gauss-Jordan with partial pivoting over the B lanes (implicit row permutation)
    bool used = !row;
    int my_col = -1;
    sfor<0, B>([&](auto cc) {
      constexpr int col = decltype(cc)::value;
      double mag = used ? -1.0 : cabs2(A[col]);
      int idx = lane;
      for (int off = 32; off > 0; off >>= 1) {
        const double om = __shfl_xor(mag, off);
        const int oi = __shfl_xor(idx, off);
        if (om > mag || (om == mag && oi < idx)) {
          mag = om;
          idx = oi;
        }
      }
      const int p = idx;  // pivot row for column `col`
      if (lane == p) {
        const double2 inv = cdiv_smith(make_double2(1.0, 0.0), A[col]);
        sfor<0, B>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          A[k] = cmul(A[k], inv);
          R[k] = cmul(R[k], inv);
          prow[k] = A[k];
          prow[B + k] = R[k];
        });
        used = true;
        my_col = col;
      }
      __syncthreads();
      if (row && lane != p) {
        const double2 fct = A[col];
        sfor<0, B>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          A[k] = csub(A[k], cmul(fct, prow[k]));
          R[k] = csub(R[k], cmul(fct, prow[B + k]));
        });
      }
      __syncthreads();
    });
    // lane with pivot column c holds row c of Lambda^-1: undo the permutation via LDS
    if (row) {
      sfor<0, B>([&](auto kc) { perm[my_col][decltype(kc)::value] = R[decltype(kc)::value]; });
    }
    __syncthreads();
    if (row) {
      double2* out = P + ((size_t)i * B + lane) * B;
      sfor<0, B>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        prev[k] = perm[lane][k];
        out[k] = prev[k];
      });
    }
    Uprev = c.E;
    __syncthreads();
  }
}

// ------------------------------------------------------------------------- solve
// A solve is 2n dependent steps, each a b x b complex product: latency, not bandwidth, is
// the bound (the P_i stream of one system is n B^2 16 B, read once).  Shape of a step:
// lanes (g, j) = (lane / 16, lane % 16) -- row j of the block, columns [g KG, (g+1) KG) --
// so all 64 lanes share the product and each holds only KG = B/4 entries of a P row.  That
// leaves the registers for a D-deep ring of prefetched steps (P entries, PML factor, right-
// hand side / y / old output), issued unconditionally from clamped addresses D steps ahead
// (HBM-miss latency ~900 cycles covers several steps).  Partial sums meet through the
// gfx950 permlane16/32 swaps (same summation order on every lane, so all four copies of y_j
// are bit-identical); the b-vector each step needs is broadcast through LDS.  Stores are
// unconditional too (masked lanes write a per-wave dummy slot), so the loop body has no
// divergent memory operation for the waitcnt pass to drain on.
constexpr int kGroups = 4;
constexpr int kMaxRing = 8;
template <int B>
constexpr int ring_depth() { return B <= 8 ? 8 : 6; }

// by-value select: `c ? arr[q] : z` on lvalues becomes a select of stack addresses (scratch)
__device__ __forceinline__ double2 csel(bool c, double2 a, double2 b) {
  return make_double2(c ? a.x : b.x, c ? a.y : b.y);
}

__device__ __forceinline__ double sum4(double v) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const double s = __hiloint2double(h16[0], l16[0]) + __hiloint2double(h16[1], l16[1]);
  lo = __double2loint(s);
  hi = __double2hiint(s);
  const auto l32 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto h32 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double(h32[0], l32[0]) + __hiloint2double(h32[1], l32[1]);
}

// Where a solve reads its right-hand side and writes its result.  Layer j (0-based inside
// the system) of the rhs is rhs + (j - rhs_first) rhs_ld for j >= rhs_first (else 0); with
// SR it is scaled by rmul * R1[i] (a sweep's S/N coupling, code.py:131-153).  Layers j >=
// out_first are written as out = alpha_old out + omul (R1[i] if SO) x.
struct SolveIO {
  const double2* rhs;
  int rhs_first;
  size_t rhs_ld;
  double2 rmul;
  double2* out;
  int out_first;
  size_t out_ld;
  double alpha_old;
  double2 omul;
};

template <int B, bool SR, bool SO>
__device__ __forceinline__ void bt_solve(const SweepArgs& a, int s, const SolveIO& io, double2* ys) {
  constexpr int KG = B / kGroups;
  constexpr int D = ring_depth<B>();
  constexpr size_t PS = (size_t)B * B;
  __shared__ double2 tl[2][kGroups][16];
  const int lane = threadIdx.x, g = lane >> 4, j = lane & 15;
  const int n = a.n;
  const bool row = j < B && j < a.b;
  const int jl = j < B ? j : B - 1;
  const bool has_rhs = row && j >= io.rhs_first;
  const bool has_out = row && j >= io.out_first;
  const double2* rb = io.rhs + (size_t)(has_rhs ? j - io.rhs_first : 0) * io.rhs_ld;
  double2* ob = io.out + (size_t)(has_out ? j - io.out_first : 0) * io.out_ld;
  double2* dummy = ys + (size_t)(n + kMaxRing) * 16 + lane;
  const double2* P = a.P + (size_t)s * n * PS + (size_t)jl * B + g * KG;
  const double2 z = make_double2(0.0, 0.0);
  const double2 R2 = csel(row, a.tab_k[4 * jl], z);  // local-layer 1/s2: c1 = AW R2, c2 = AE R2
  const double2* AW = a.tab_i;
  const double2* AE = a.tab_i + n;
  const double2* R1 = a.tab_i + 2 * n;
  const bool ystore = g == 0 && j < B;

  // ---- forward: y_i = P_i (r_i - L_i y_{i-1}) ----
  double2 Pf[D][KG], cf[D], rf[D], sf[SR ? D : 1];
  auto load_f = [&](auto qc, int i) {
    constexpr int q = decltype(qc)::value;
    sfor<0, KG>([&](auto cc) { Pf[q][decltype(cc)::value] = P[(size_t)i * PS + decltype(cc)::value]; });
    cf[q] = AW[i];
    rf[q] = rb[i];
    if constexpr (SR) sf[q] = R1[i];
  };
  sfor<0, D>([&](auto qc) { load_f(qc, min((int)decltype(qc)::value, n - 1)); });
  double2 y = z, ylast = z;
  for (int i0 = 0; i0 < n; i0 += D) {  // steps past n - 1 run on clamped data, results unused
    sfor<0, D>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      // keep each step's work inside its step: hoisting slot q's loaded-operand products
      // to the top of the unrolled body would wait on loads issued one step earlier
      __builtin_amdgcn_sched_barrier(0);
      const int i = i0 + q;
      double2 r = csel(has_rhs, rf[q], z);
      if constexpr (SR) r = cmul(r, cmul(io.rmul, sf[q]));
      tl[q & 1][g][j] = csub(r, cmul(cmul(cf[q], R2), y));  // y_{-1} = 0 covers i = 0
      __syncthreads();
      double2 acc = z;
      sfor<0, KG>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        acc = cfma(Pf[q][c], tl[q & 1][0][g * KG + c], acc);
      });
      y = make_double2(sum4(acc.x), sum4(acc.y));
      ylast = csel(i == n - 1, y, ylast);
      *(ystore ? ys + (size_t)i * 16 + j : dummy) = y;
      load_f(qc, min(i + D, n - 1));
    });
  }
  __syncthreads();

  // ---- backward: x_{n-1} = y_{n-1}; x_i = y_i - P_i (U_i x_{i+1}) ----
  double2 x = ylast;
  {
    const double2 old = ob[n - 1];
    double2 xo = x;
    if constexpr (SO) xo = cmul(x, R1[n - 1]);
    const double2 o = csel(io.alpha_old != 0.0, cscale(old, io.alpha_old), z);
    *(has_out ? ob + (n - 1) : dummy) = cadd(o, cmul(io.omul, xo));
  }
  double2 Pb[D][KG], cb[D], yb[D], obv[D], sb[SO ? D : 1];
  auto load_b = [&](auto qc, int i) {
    constexpr int q = decltype(qc)::value;
    sfor<0, KG>([&](auto cc) { Pb[q][decltype(cc)::value] = P[(size_t)i * PS + decltype(cc)::value]; });
    cb[q] = AE[i];
    yb[q] = ys[(size_t)i * 16 + jl];
    obv[q] = ob[i];
    if constexpr (SO) sb[q] = R1[i];
  };
  sfor<0, D>([&](auto qc) { load_b(qc, max(n - 2 - (int)decltype(qc)::value, 0)); });
  for (int i0 = n - 2; i0 >= 0; i0 -= D) {  // steps below 0 run on clamped data, stores to dummy
    sfor<0, D>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      __builtin_amdgcn_sched_barrier(0);
      const int i = i0 - q;
      tl[q & 1][g][j] = cmul(cmul(cb[q], R2), x);
      __syncthreads();
      double2 acc = z;
      sfor<0, KG>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        acc = cfma(Pb[q][c], tl[q & 1][0][g * KG + c], acc);
      });
      x = csub(yb[q], make_double2(sum4(acc.x), sum4(acc.y)));
      double2 xo = x;
      if constexpr (SO) xo = cmul(x, sb[q]);
      const double2 o = csel(io.alpha_old != 0.0, cscale(obv[q], io.alpha_old), z);
      *((has_out && i >= 0) ? ob + i : dummy) = cadd(o, cmul(io.omul, xo));
      load_b(qc, max(i - D, 0));
    });
  }
  __syncthreads();
}

__device__ __forceinline__ SolveIO solve_io(const double2* rhs, int rhs_first, double2 rmul,
                                            double2* out, int out_first, double alpha_old,
                                            double2 omul, size_t ld) {
  SolveIO io;
  io.rhs = rhs;
  io.rhs_first = rhs_first;
  io.rhs_ld = ld;
  io.rmul = rmul;
  io.out = out;
  io.out_first = out_first;
  io.out_ld = ld;
  io.alpha_old = alpha_old;
  io.omul = omul;
  return io;
}

// Algorithm 2.4 pieces.  u: layer-major [n][n] (layer j at u + j n).
// forward sweep (code.py:363-370): TFuF = HF^-1 u[0:b] -> uF; u[b] -= S_b * TFuF[b-1];
// for m = b+1..n-1: u[m] -= S_m * T_m u[m-1]  (S_m = BS_m R1[i], folded into the solve).
template <int B>
__global__ __launch_bounds__(kSW) void sweep_forward_kernel(const SweepArgs a, double2* u,
                                                            double2* uF) {
  if (a.stop && *a.stop) return;
  const int n = a.n, b = a.b;
  const double2 one = make_double2(1.0, 0.0);
  double2* ys = a.yscr;
  bt_solve<B, false, false>(a, 0, solve_io(u, 0, one, uF, 0, 0.0, one, n), ys);
  const double2* R1 = a.tab_i + 2 * n;
  {
    const double2 BS = a.tab_glob[4 * b + 1];  // c3 of global layer b (code.py:150-153)
    for (int i = threadIdx.x; i < n; i += kSW)
      u[(size_t)b * n + i] = csub(u[(size_t)b * n + i], cmul(cmul(BS, R1[i]), uF[(size_t)(b - 1) * n + i]));
  }
  __syncthreads();
  for (int m = b + 1; m < n; ++m) {  // system s = m - b covers layers m-b .. m-1
    const double2 BS = a.tab_glob[4 * m + 1];
    bt_solve<B, false, true>(a, m - b, solve_io(u + (size_t)(m - 1) * n, b - 1, one,
                                               u + (size_t)m * n, b - 1, 1.0, cneg(BS), n), ys);
  }
}

// middle sweep (code.py:372-375): for m = b+1..n: u[m-1] = T_m u[m-1] (corrected) or
// u[m-1] - T_m u[m-1] (as-is, quirk Q2).  One wave per m, all independent.
template <int B>
__global__ __launch_bounds__(kSW) void sweep_middle_kernel(const SweepArgs a, double2* u,
                                                           int asis) {
  if (a.stop && *a.stop) return;
  const int n = a.n, b = a.b;
  const int s = blockIdx.x + 1;  // system s <-> 1-based m = b + s, last layer m-1 = b+s-1
  double2* layer = u + (size_t)(b + s - 1) * n;
  double2* ys = a.yscr + (size_t)blockIdx.x * a.ystride;
  const double2 one = make_double2(1.0, 0.0);
  // in place: every forward-pass read of the layer precedes the backward-pass writes, and
  // the backward pass prefetches index i - D only after index i - D + 1.. were consumed
  bt_solve<B, false, false>(a, s, solve_io(layer, b - 1, one, layer, b - 1, asis ? 1.0 : 0.0,
                                           asis ? make_double2(-1.0, 0.0) : one, n), ys);
}

// backward sweep (code.py:376-380): for m = n-1..b+1: u[m-1] -= T_m (N_{m-1} u[m]);
// F correction (code.py:381-384): uF -= HF^-1 [0 .. 0, N_{b-1} u[b]]; u[0:b] = uF.
// N_{m-1} = BN_{m-1} R1[i] is folded into the solve's right-hand-side load.
template <int B>
__global__ __launch_bounds__(kSW) void sweep_backward_kernel(const SweepArgs a, double2* u,
                                                             double2* uF) {
  if (a.stop && *a.stop) return;
  const int n = a.n, b = a.b;
  double2* ys = a.yscr;
  const double2 mone = make_double2(-1.0, 0.0);
  for (int m = n - 1; m >= b + 1; --m) {
    const double2 BN = a.tab_glob[4 * (m - 1) + 2];  // c4 of global layer m-1 (code.py:131-140)
    bt_solve<B, true, false>(a, m - b, solve_io(u + (size_t)m * n, b - 1, BN,
                                               u + (size_t)(m - 1) * n, b - 1, 1.0, mone, n), ys);
  }
  // H_F is block diagonal: only its last layer sees the (last-layer-only) right-hand side
  const double2 BN = a.tab_glob[4 * (b - 1) + 2];
  bt_solve<B, true, false>(a, 0, solve_io(u + (size_t)b * n, b - 1, BN, uF + (size_t)(b - 1) * n,
                                          b - 1, 1.0, mone, n), ys);
  for (size_t p = threadIdx.x; p < (size_t)b * n; p += kSW) u[p] = uF[p];
}

template <int B>
void launch_all(const SweepArgs& a, int what, double2* u, double2* uF, int asis, hipStream_t st) {
  switch (what) {
    case 0:
      hipLaunchKernelGGL((sweep_factor_kernel<B>), dim3(a.nsys), dim3(kSW), 0, st, a);
      break;
    case 1:
      hipLaunchKernelGGL((sweep_forward_kernel<B>), dim3(1), dim3(kSW), 0, st, a, u, uF);
      break;
    case 2:
      hipLaunchKernelGGL((sweep_middle_kernel<B>), dim3(a.nsys - 1), dim3(kSW), 0, st, a, u,
                         asis);
      break;
    case 3:
      hipLaunchKernelGGL((sweep_backward_kernel<B>), dim3(1), dim3(kSW), 0, st, a, u, uF);
      break;
    default:
      break;
  }
}

}  // namespace

size_t sweep_scratch_per_wave(int n) { return (size_t)(n + kMaxRing) * 16 + 64; }

int sweep_block(int b) { return b <= 4 ? 4 : (b <= 8 ? 8 : (b <= 12 ? 12 : (b <= 16 ? 16 : 0))); }

void launch_sweep(const SweepArgs& a, int what, double2* u, double2* uF, int asis,
                  hipStream_t st) {
  switch (sweep_block(a.b)) {
    case 4: launch_all<4>(a, what, u, uF, asis, st); break;
    case 8: launch_all<8>(a, what, u, uF, asis, st); break;
    case 12: launch_all<12>(a, what, u, uF, asis, st); break;
    case 16: launch_all<16>(a, what, u, uF, asis, st); break;
    default: break;
  }
}

}  // namespace hh
