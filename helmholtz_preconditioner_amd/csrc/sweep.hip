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
#include <cstdlib>

#include "sweep.hpp"
#include "hh_error.hpp"

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
      double2* out = P + (size_t)i * B * B;
      sfor<0, B>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        prev[k] = perm[lane][k];
        out[pidx<B>(lane, k)] = prev[k];
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
  int s_next;  // the launch's next partitioned solve's system (prefetched), or -1
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
  const double2* P = a.P + (size_t)s * n * PS;
  int po[KG];  // this lane's entries (row jl, columns g KG + c) in the pidx order
  sfor<0, KG>([&](auto cc) { po[decltype(cc)::value] = pidx<B>(jl, g * KG + decltype(cc)::value); });
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
    sfor<0, KG>([&](auto cc) { Pf[q][decltype(cc)::value] = P[(size_t)i * PS + po[decltype(cc)::value]]; });
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
    sfor<0, KG>([&](auto cc) { Pb[q][decltype(cc)::value] = P[(size_t)i * PS + po[decltype(cc)::value]]; });
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

// ------------------------------------------------------- partitioned (chunked) solves
// The forward recurrence y_i = P_i (r_i - L_i y_{i-1}) = c_i + M_i y_{i-1} and the backward one
// x_i = y_i + N_i x_{i+1} (M_i = -P_i L_i, N_i = -P_i U_i) are affine in the carried vector, so
// with the columns split into K chunks [lo_k, hi_k):
//   y_i = yL_i + Psi_f[i] y_{lo_k - 1},   Psi_f[i] = M_i M_{i-1} .. M_{lo_k}
//   x_i = xL_i + Psi_b[i] x_{hi_k},       Psi_b[i] = N_i N_{i+1} .. N_{hi_k - 1}
// where yL / xL run the recurrence inside the chunk from a zero carry.  The chunks are grouped
// kSweepChunks to a workgroup and G workgroups share a solve; the chunk-end maps compose into
// one map per workgroup, Phi_f(g) = Psi_f[end_15] .. Psi_f[end_0] (Phi_b likewise), so a
// carry crosses a workgroup in one B x B step.  A solve is then: every chunk's local
// recurrence at once, a chain over the workgroup's 16 chunk boundaries, ONE exchange of the
// workgroups' zero-carry end vectors, a chain over the other workgroups' maps, one step per
// chunk through the workgroup's prefix map, and a parallel fix-up of every column --
// dependent depth ~2 (n / K + kSweepChunks + G) steps instead of 2 n.  Psi and the workgroup
// maps are operator data, formed once at setup.
__device__ __forceinline__ int chunk_lo(int n, int K, int k) { return n * k / K; }  // n K < 2^31

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Setup: Psi_f and Psi_b of one (system, chunk) per wave (K = a.chunks chunks per system).
// Lanes (g, j): row j, columns [g KG, (g+1) KG) of the running product, which every lane
// reads whole from LDS.
template <int B>
__global__ __launch_bounds__(kSW) void sweep_chunk_setup_kernel(const SweepArgs a) {
  constexpr int KG = B / kGroups;
  constexpr size_t PS = (size_t)B * B;
  __shared__ double2 Q[2][B][B];
  const int K = a.chunks;
  const int n = a.n;
  const int s = blockIdx.x / K, k = blockIdx.x % K;
  const int lo = chunk_lo(n, K, k), hi = chunk_lo(n, K, k + 1);
  const int lane = threadIdx.x, g = lane >> 4, j = lane & 15;
  const bool row = j < B;
  const int jl = row ? j : B - 1;
  const double2 z = make_double2(0.0, 0.0);
  const double2* P = a.P + (size_t)s * n * PS;
  for (int dir = 0; dir < 2; ++dir) {  // 0: Psi_f (i = lo .. hi-1), 1: Psi_b (i = hi-1 .. lo)
    double2* out = (dir == 0 ? a.Pf : a.Pb) + (size_t)s * n * PS;
    const double2* cpl = a.tab_i + (dir == 0 ? 0 : n);  // AW (L_i) or AE (U_i)
    for (int q = 0; q < hi - lo; ++q) {
      const int i = dir == 0 ? lo + q : hi - 1 - q;
      const double2 cc = cpl[i];
      double2 prow[B];  // row j of M_i = -P_i L_i (or N_i = -P_i U_i): -P_i[j][m] cc R2[m]
      sfor<0, B>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        const double2 r2 = m < a.b ? a.tab_k[4 * m] : z;  // 0 on padding layers
        prow[m] = cneg(cmul(P[(size_t)i * PS + pidx<B>(jl, m)], cmul(cc, r2)));
      });
      double2 v[KG];
      sfor<0, KG>([&](auto c2) {
        constexpr int c = decltype(c2)::value;
        const int col = g * KG + c;
        double2 acc = z;
        if (q == 0) {  // the first factor alone
          sfor<0, B>([&](auto mc) {
            constexpr int m = decltype(mc)::value;
            acc = csel(m == col, prow[m], acc);
          });
        } else {
          sfor<0, B>([&](auto mc) {
            constexpr int m = decltype(mc)::value;
            acc = cfma(prow[m], Q[(q - 1) & 1][m][col], acc);
          });
        }
        v[c] = acc;
      });
      if (row) {
        sfor<0, KG>([&](auto c2) {
          constexpr int c = decltype(c2)::value;
          Q[q & 1][j][g * KG + c] = v[c];
          out[(size_t)i * PS + pidx<B>(j, g * KG + c)] = v[c];
        });
      }
      wave_sync();
    }
  }
}

// Setup: the workgroup maps of one (system, workgroup) per wave (after the chunk products),
// with F_k = Psi_f[end_k], B_k = Psi_b[lo_k] the chunk maps (end_k / lo_k: the chunk's last /
// first column): forward Pw[..][0][q] = F_q .. F_0 (the map from the workgroup's carry to the
// end of chunk q), backward Pw[..][1][q] = B_{15-q} .. B_15 (from the carry past the workgroup
// to the start of chunk 15 - q); [15] is the whole workgroup's map Phi.
template <int B>
__global__ __launch_bounds__(kSW) void sweep_wg_setup_kernel(const SweepArgs a) {
  constexpr int KG = B / kGroups;
  constexpr size_t PS = (size_t)B * B;
  __shared__ double2 Q[2][B][B];
  const int n = a.n, G = a.G, K = a.chunks;
  const int s = blockIdx.x / G, wg = blockIdx.x % G;
  const int lane = threadIdx.x, g = lane >> 4, j = lane & 15;
  const bool row = j < B;
  const int jl = row ? j : B - 1;
  const double2 z = make_double2(0.0, 0.0);
  for (int dir = 0; dir < 2; ++dir) {
    const double2* src = (dir == 0 ? a.Pf : a.Pb) + (size_t)s * n * PS;
    double2* out = a.Pw + (((size_t)s * G + wg) * 2 + dir) * kSweepChunks * PS;
    for (int q = 0; q < kSweepChunks; ++q) {  // forward: chunks in order; backward: from the last
      const int k = kSweepChunks * wg + (dir == 0 ? q : kSweepChunks - 1 - q);
      const int col = dir == 0 ? chunk_lo(n, K, k + 1) - 1 : chunk_lo(n, K, k);
      double2 prow[B];
      sfor<0, B>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        prow[m] = src[(size_t)col * PS + pidx<B>(jl, m)];
      });
      double2 v[KG];
      sfor<0, KG>([&](auto c2) {
        constexpr int c = decltype(c2)::value;
        const int cx = g * KG + c;
        double2 acc = z;
        if (q == 0) {
          sfor<0, B>([&](auto mc) {
            constexpr int m = decltype(mc)::value;
            acc = csel(m == cx, prow[m], acc);
          });
        } else {
          sfor<0, B>([&](auto mc) {
            constexpr int m = decltype(mc)::value;
            acc = cfma(prow[m], Q[(q - 1) & 1][m][cx], acc);
          });
        }
        v[c] = acc;
      });
      if (row) {
        sfor<0, KG>([&](auto c2) {
          constexpr int c = decltype(c2)::value;
          Q[q & 1][j][g * KG + c] = v[c];
          out[(size_t)q * PS + pidx<B>(j, g * KG + c)] = v[c];
        });
      }
      wave_sync();
    }
  }
}

// Setup: the grid maps (SweepArgs::Tm), after the workgroup maps.  One wave per (system,
// direction, upstream workgroup u) walks the downstream workgroups by left products:
// T(u+2, u) = Phi_{u+1}, T(w+1, u) = Phi_w T(w, u) (backward mirrored: T(u-2, u) = Phi_{u-1},
// T(w-1, u) = Phi_w T(w, u)), Phi_w = Pw[s][w][dir][15].  Same lane split as above.
template <int B>
__global__ __launch_bounds__(kSW) void sweep_grid_setup_kernel(const SweepArgs a) {
  constexpr int KG = B / kGroups;
  constexpr size_t PS = (size_t)B * B;
  __shared__ double2 Q[2][B][B];
  const int G = a.G;
  const int s = blockIdx.x / (2 * G), dir = (blockIdx.x / G) & 1, u = blockIdx.x % G;
  const int steps = dir == 0 ? G - 2 - u : u - 1;  // downstream workgroups at distance >= 2
  const int lane = threadIdx.x, g = lane >> 4, j = lane & 15;
  const bool row = j < B;
  const int jl = row ? j : B - 1;
  const double2 z = make_double2(0.0, 0.0);
  double2* tbase = a.Tm + (size_t)(s * 2 + dir) * sweep_grid_tri(G) * PS;
  for (int q = 0; q < steps; ++q) {
    const int w = dir == 0 ? u + 1 + q : u - 1 - q;  // the new left factor's workgroup
    const int cnt = dir == 0 ? w + 1 : G - w;          // upstream count of the map's workgroup
    const double2* phi =
        a.Pw + ((((size_t)s * a.G + w) * 2 + dir) * kSweepChunks + kSweepChunks - 1) * PS;
    double2* out = tbase + (sweep_grid_tri(cnt) + (size_t)q) * PS;  // distance d = q + 2
    double2 prow[B];
    sfor<0, B>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      prow[m] = phi[pidx<B>(jl, m)];
    });
    double2 v[KG];
    sfor<0, KG>([&](auto c2) {
      constexpr int c = decltype(c2)::value;
      const int cx = g * KG + c;
      double2 acc = z;
      if (q == 0) {
        sfor<0, B>([&](auto mc) {
          constexpr int m = decltype(mc)::value;
          acc = csel(m == cx, prow[m], acc);
        });
      } else {
        sfor<0, B>([&](auto mc) {
          constexpr int m = decltype(mc)::value;
          acc = cfma(prow[m], Q[(q - 1) & 1][m][cx], acc);
        });
      }
      v[c] = acc;
    });
    if (row) {
      sfor<0, KG>([&](auto c2) {
        constexpr int c = decltype(c2)::value;
        Q[q & 1][j][g * KG + c] = v[c];
        out[pidx<B>(j, g * KG + c)] = v[c];
      });
    }
    wave_sync();
  }
}

#ifndef HH_SWEEP_TOUCH
#define HH_SWEEP_TOUCH 1
#endif
template <int B>
constexpr int chunk_ring() { return B <= 4 ? 4 : (B == 8 ? 3 : 2); }  // (no spills at 256 VGPRs)
template <int B>
constexpr int part_max_wgs() { return kSweepMaxWgs; }  // (each half holds kSweepGridMaps maps)
constexpr int kPartThreads = kSweepChunks / 2 * kSW;      // 8 waves, two chunks each
constexpr unsigned kPartSpin = 1u << 20;                   // ~1 s of polling per wait
// dynamic LDS of a partitioned solve: the chunk chain's maps [kSweepChunks][B B], then the
// other workgroups' published vectors [G][16]
// the most columns one workgroup owns (n K < 2^31: chunk_lo exact) + 1
__host__ __device__ inline int part_ys_cols(int n, int G) { return (n + G - 1) / G + 1; }
// double2 of the fixed part (tl, bf, bb, yvl of bt_solve_chunked)
constexpr int kPartFixedLds = kSweepChunks * 2 * 16 + 2 * (kSweepChunks + 2) * 16 +
                              kSweepChunks * 16;
template <int B>
size_t part_lds_bytes(int G, int n, bool ly) {
  return ((size_t)kPartFixedLds + (size_t)kSweepChunks * B * B + kSW + (size_t)G * 16 +
          (ly ? (size_t)part_ys_cols(n, G) * B + kSW : 0)) * sizeof(double2);
}
constexpr size_t kPartStaticLds = 256;  // (anything the compiler adds beside the dynamic block)
constexpr size_t kPartLdsBudget = 160 * 1024;

// wait until at most N of this wave's vector-memory operations are outstanding (vmcnt only;
// they complete in issue order).  After an LDS DMA and N later loads: waits for the DMA alone,
// where the compiler's own wait before the next LDS access would take every load with it.
// The count N is hand-derived from the loads issued after the DMA (the sfor ring); it is right
// only while the compiler emits exactly those after it.  tools/check_sweep_waitcnt.py checks the
// built ISA (every LDS read after an LDS DMA is covered by a wait that retires the DMA);
// -DHH_SWEEP_WAIT_ALL builds every such wait as vmcnt(0) (make waitall) for A/B runs of the
// linearity / determinism tests.
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
#ifdef HH_SWEEP_WAIT_ALL
  __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));
#else
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
#endif
}

// base[byte offset]: a scalar base plus a 32-bit lane offset in bytes is the form the
// global_load/store saddr addressing takes (no 64-bit address pair per lane)
template <class T>
__device__ __forceinline__ T& at(T* base, unsigned byte_off) {
  return *reinterpret_cast<T*>(reinterpret_cast<
      std::conditional_t<std::is_const<T>::value, const char, char>*>(base) + byte_off);
}

// sum of v over the two 16-lane rows of this lane's 32-lane half (same order on every lane)
__device__ __forceinline__ double sum2(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(h16[0], l16[0]) + __hiloint2double(h16[1], l16[1]);
}

// Granule tags of the grid exchange: launch sequence number, solve (round) and direction.  A
// slot [dir][round & 1][g] is rewritten two rounds later at the earliest, which no reader of it
// can reach first (each round's backward exchange needs every later workgroup past the forward
// one, and the next round's forward exchange every earlier workgroup past this backward one).
__device__ __forceinline__ unsigned part_tag(unsigned seq, int round, int dir) {
  return (seq << 15) | ((unsigned)(round & 0x3fff) << 1) | (unsigned)dir;
}
using gu64p = __attribute__((address_space(1))) unsigned long long*;
__device__ __forceinline__ void st_gran4(unsigned long long* p, unsigned tag, double2 v) {
  const unsigned long long tt = (unsigned long long)tag << 32;
  const unsigned long long hx = (unsigned long long)__double_as_longlong(v.x);
  const unsigned long long hy = (unsigned long long)__double_as_longlong(v.y);
  __hip_atomic_store((gu64p)p, tt | (hx >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((gu64p)(p + 1), tt | (hx & 0xffffffffull), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((gu64p)(p + 2), tt | (hy >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((gu64p)(p + 3), tt | (hy & 0xffffffffull), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// One partitioned solve, with the SolveIO contract of bt_solve, by workgroup wg = blockIdx.x of
// a.G (all co-resident).  Each 32-lane half of a wave owns one chunk (local chunk cl = 2 w + h,
// global chunk kSweepChunks wg + cl): lanes (g, j) of the half -- row j of the block, columns
// [g KG, (g+1) KG), KG = B / 2 -- so the two chunks of a wave step in lockstep (their lengths
// differ by at most one column: the shorter one's last step runs on clamped data and is not
// stored).  Half-wave chunks give 16 chunks with 8 waves, i.e. 256 VGPRs per lane.  ys:
// sweep_chunk_scratch.  Per direction (forward shown; backward mirrors it from the right):
//   1. chunk-local (every half): yL_i = P_i (r_i - L_i yL_{i-1}), from yL_{lo-1} = 0
//   2. the chain maps staged in LDS (chunk ends' Psi_f, earlier workgroups' Phi_f); wave 0:
//      chunk boundaries from a zero workgroup carry, y_end_k = yL_end_k + Psi_f y_end_{k-1},
//      the last one published as granules; waves 1..7 meanwhile poll the earlier workgroups'
//   3. the workgroup's carry y_in = sum over the earlier workgroups u of T(wg, u) y_end_u (the
//      grid maps, SweepArgs::Tm; identity for u = wg - 1): every half applies up to
//      kSweepGridMaps of them (their rows requested before step 2, so they wait in registers),
//      wave 0 sums the halves' partials in a fixed order -- one step after the last arrival
//      instead of a chain of G - 1 (G = 1: step 2 alone)
//   4. every half: its chunk's carry y_{lo-1} = the zero-carry chain's value + the workgroup's
//      prefix map (Pw) applied to y_in; fix-up (rows independent): y_i = yL_i + Psi_f[i] y_{lo-1};
//      then backward, chunk-local:
//      xL_i = y_i - P_i U_i xL_{i+1} (a wave reads back only its own rows); 2-3 backward; then
//   5. fix-up + output (rows independent, prefetched like 1 / 4): x_i = xL_i + Psi_b[i] x_{hi}
// (chunk 0 in 4 and chunk 15 in 5 multiply their Psi rows by the workgroup carry, zero for the
// first / last workgroup, instead of branching: both halves run one instruction stream.)  A
// ring slot of KG = 6 double2 is 24 VGPRs at B = 12, so no phase keeps two matrix rings.  ok:
// false once a grid wait of this workgroup timed out (no further waits; garbage output and
// a.timeout set for the host).
template <int B, bool SR, bool SO, bool LY>
__device__ __forceinline__ void bt_solve_chunked(const SweepArgs& a, int s, int round,
                                                 const SolveIO& io, const double2 R2,
                                                 double2* ys, bool& ok,
                                                 unsigned long long (&tk)[kSweepProfSlots]) {
  constexpr int KG = B / 2;
  constexpr int D = chunk_ring<B>();
  constexpr int KL = kSweepChunks;
  constexpr int PS = B * B;
  constexpr unsigned PSB = (unsigned)PS * 16u;  // bytes of one B x B matrix
  constexpr int NQ = 4 * B;                     // granules of one published vector
  // all LDS is carved from the dynamic block (one copy however many instantiations a kernel
  // calls): the per-chunk step vectors tl (in step 3 the halves' partial sums), the chunk
  // boundaries bf / bb ([KL]: workgroup carry, [KL + 1]: zeros), the chunk-end (forward) /
  // chunk-start (backward) vectors yvl, then the chain maps, the grid vectors and (LY) the
  // B-vectors
  extern __shared__ double2 part_lds[];
  auto tl = reinterpret_cast<double2 (*)[2][16]>(part_lds);
  auto bf = reinterpret_cast<double2 (*)[16]>(part_lds + KL * 2 * 16);
  auto bb = bf + (KL + 2);
  auto yvl = bb + (KL + 2);
  const int tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, h = lane >> 5, g = (lane >> 4) & 1, j = lane & 15;
  const int n = a.n, G = a.G, wg = blockIdx.x, K = KL * G;
  double2* mats = part_lds + kPartFixedLds;   // [KL][PS]
  double2* gin = mats + (size_t)KL * PS + kSW;  // [G][16] (after the DMA slack)
  // LY: the workgroup's B-vectors (y, then x) in LDS, [column - c0w][B] + a junk slot per
  // lane: no global store in the dependent loops (a wait for a ring load would also wait for
  // every older store, and a store takes ~1 us to retire)
  double2* ysl = gin + (size_t)G * 16;
  const int c0w = chunk_lo(n, K, KL * wg);
  const int cl = 2 * w + h;  // this half's local chunk
  const int c = KL * wg + cl;
  const int lo = chunk_lo(n, K, c), hi = chunk_lo(n, K, c + 1), len = hi - lo;
  const int m0 = chunk_lo(n, K, KL * wg + 2 * w + 1);
  const int lenw = max(m0 - chunk_lo(n, K, KL * wg + 2 * w),
                       chunk_lo(n, K, KL * wg + 2 * w + 2) - m0);  // both halves
  const int last = len - 1;  // (n >= 2 K: every chunk has >= 2 columns)
  const bool row = j < B && j < a.b;
  const int jl = j < B ? j : B - 1;
  const bool has_rhs = row && j >= io.rhs_first;
  const bool has_out = row && j >= io.out_first && g == 0;
  // byte offsets of this lane from scalar bases
  const unsigned roff = has_rhs ? (unsigned)((j - io.rhs_first) * io.rhs_ld) * 16u : 0u;
  const unsigned ooff =
      (row && j >= io.out_first) ? (unsigned)((j - io.out_first) * io.out_ld) * 16u : 0u;
  const unsigned lofs = (unsigned)pidx<B>(jl, g * KG) * 16u;  // row jl, this lane's columns
  constexpr unsigned QS = 2u * B * 16u;  // byte step between a lane's consecutive entries
  const unsigned dofs =
      ((unsigned)(n * 16) + (unsigned)wg * kPartThreads + (unsigned)tid) * 16u;  // dummy slot
  const size_t sbase = (size_t)s * n * PS;
  const double2* P = a.P + sbase;
  const double2* Pf = a.Pf + sbase;
  const double2* Pb = a.Pb + sbase;
  const double2 z = make_double2(0.0, 0.0);
  const double2* AW = a.tab_i;
  const double2* AE = a.tab_i + n;
  const double2* R1 = a.tab_i + 2 * n;
  const bool ystore = g == 0 && j < B;
  auto ld_row = [&](double2 (&m)[KG], const double2* base, int i) {
    const unsigned o = (unsigned)i * PSB + lofs;
    sfor<0, KG>([&](auto cc) { m[decltype(cc)::value] = at(base, o + QS * decltype(cc)::value); });
  };
  auto yget = [&](int i) {
    if constexpr (LY) return ysl[(i - c0w) * B + jl];
    else return at(ys, ((unsigned)i * 16u + (unsigned)jl) * 16u);
  };
  auto yput = [&](bool ok_, int i, double2 v) {
    if constexpr (LY) ysl[ok_ ? (i - c0w) * B + j : part_ys_cols(n, G) * B + lane] = v;
    else at(ys, ok_ ? ((unsigned)i * 16u + (unsigned)j) * 16u : dofs) = v;
  };
  // this lane's KG entries against entries [g KG, (g+1) KG) of an LDS 16-vector, summed over
  // the half's two lane groups
  auto rowdot = [&](const double2 (&m)[KG], const double2* vec) {
    double2 acc = z;
    sfor<0, KG>([&](auto cc) {
      constexpr int q = decltype(cc)::value;
      acc = cfma(m[q], vec[g * KG + q], acc);
    });
    return make_double2(sum2(acc.x), sum2(acc.y));
  };
  // the chain maps of direction dir into LDS: map k is local chunk k's end map (forward:
  // Psi_f at its last column; backward: Psi_b at its first).  By LDS DMA (global_load_lds: no
  // registers, lane-linear 1 KB per wave instruction, per-lane sources), issued at the start
  // of a chunk-local phase so its latency overlaps that phase's first ring loads; the barrier
  // before the maps are read waits for it.  (The last instruction may write up to 63 entries
  // past the maps: the region has that slack.)
  auto stage = [&](int dir) {
    constexpr int tot = KL * PS;
    constexpr int NI = (tot + kPartThreads - 1) / kPartThreads;  // (a fixed count: exact vmcnt)
    const double2* cp = dir == 0 ? Pf : Pb;
    sfor<0, NI>([&](auto ic) {
      const int e0 = w * kSW + (int)decltype(ic)::value * kPartThreads;
      const int e = min(e0 + lane, tot - 1);
      const int mi = e / PS, off = e - mi * PS;
      const int k = KL * wg + mi;
      const double2* src =
          cp + (size_t)(dir == 0 ? chunk_lo(n, K, k + 1) - 1 : chunk_lo(n, K, k)) * PS + off;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(mats +
                                                                                 min(e0, tot)),
                                       16, 0, 0);
    });
  };
  // waves 1..7: wait for the vectors the grid step needs (forward: workgroups 0 .. wg-1,
  // backward: wg+1 .. G-1) and unpack them into gin (PQ granules per lane at a time)
  auto poll = [&](int dir) {
    const int first = dir == 0 ? 0 : wg + 1;
    const int nq = (dir == 0 ? wg : G - 1 - wg) * NQ;
    constexpr int PQ = 4;
    constexpr int STEP = kPartThreads - kSW;
    const unsigned tg = part_tag(a.seq, round, dir);
    const unsigned long long* gb =
        a.gran + (size_t)(dir * 2 + (round & 1)) * G * kSweepGranStride;
    for (int q0 = tid - kSW; q0 < nq && ok; q0 += PQ * STEP) {
      unsigned long long v[PQ];
      unsigned spins = 0;
      for (;;) {
        sfor<0, PQ>([&](auto pc) {
          const int q = min(q0 + (int)decltype(pc)::value * STEP, nq - 1);
          v[decltype(pc)::value] = __hip_atomic_load(
              (gu64p)(gb + (size_t)(first + q / NQ) * kSweepGranStride + q % NQ), __ATOMIC_RELAXED,
              __HIP_MEMORY_SCOPE_AGENT);
        });
        bool all = true;
        sfor<0, PQ>([&](auto pc) {
          const int q = q0 + (int)decltype(pc)::value * STEP;
          all = all && (q >= nq || (unsigned)(v[decltype(pc)::value] >> 32) == tg);
        });
        if (all) break;
        if (++spins > kPartSpin) {
          ok = false;
          __hip_atomic_store((__attribute__((address_space(1))) unsigned*)a.timeout, 1u,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      unsigned* g32 = reinterpret_cast<unsigned*>(gin);
      sfor<0, PQ>([&](auto pc) {
        const int q = q0 + (int)decltype(pc)::value * STEP;
        if (q < nq) {  // granule r of a vector: row r / 4, part r % 4 = x hi, x lo, y hi, y lo
          const int gi = q / NQ, r = q % NQ;
          g32[(gi * 16 + (r >> 2)) * 4 + ((r & 3) ^ 1)] = (unsigned)v[decltype(pc)::value];
        }
      });
    }
  };
  // wave 0: chain over the local chunk boundaries, bv[k] = yv[k] + map_k bv[prev], prev = the
  // neighbour chunk (forward k - 1, backward k + 1) or `start` for the first step
  // (a staged map's row entries into registers: issued a step ahead of their use, so a step
  // waits only on the vector it depends on)
  auto ldm = [&](double2 (&m)[KG], int mi) {
    const double2* mr = mats + mi * PS + pidx<B>(jl, g * KG);
    sfor<0, KG>([&](auto cc) { m[decltype(cc)::value] = mr[decltype(cc)::value * 2 * B]; });
  };
  // (the step's chunk-end value is read a step ahead too, and the row sum runs as two
  // interleaved FMA chains: the step's dependent span is the LDS round trip of bv, half the
  // row's FMAs and the half-wave sum)
  auto chain = [&](auto fwdc, double2 (*bv)[16], int start) {
    constexpr bool fwd = decltype(fwdc)::value;
    double2 v = z;
    double2 mq[2][KG], yq[2];
    ldm(mq[0], fwd ? 0 : KL - 1);
    yq[0] = yvl[fwd ? 0 : KL - 1][jl];
    sfor<0, KL>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      constexpr int k = fwd ? q : KL - 1 - q;
      if constexpr (q + 1 < KL) {
        ldm(mq[(q + 1) & 1], fwd ? k + 1 : k - 1);
        yq[(q + 1) & 1] = yvl[fwd ? k + 1 : k - 1][jl];
      }
      const int prev = q == 0 ? start : (fwd ? k - 1 : k + 1);
      const double2* vec = &bv[prev][0];
      double2 a0 = z, a1 = z;
      sfor<0, KG>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        if constexpr (c % 2 == 0) a0 = cfma(mq[q & 1][c], vec[g * KG + c], a0);
        else a1 = cfma(mq[q & 1][c], vec[g * KG + c], a1);
      });
      const double2 acc = cadd(a0, a1);
      v = cadd(yq[q & 1], make_double2(sum2(acc.x), sum2(acc.y)));
      if (lane < 16) bv[k][lane] = v;
      wave_sync();
    });
    return v;
  };
  // phase timing (diagnostic): thread 0's wall clock at phase ends, into tk[slot]
  const bool prof = a.prof != nullptr && tid == 0;
  unsigned long long tmark = prof ? wall_clock64() : 0;
  auto mark = [&](int slot) {
    if (prof) {
      const unsigned long long now = wall_clock64();
      tk[slot] += now - tmark;
      tmark = now;
    }
  };
  // the workgroup-map selector of this (system, workgroup, direction)
  auto wsel = [&](int dir) { return ((size_t)s * G + wg) * 2 + dir; };
  // waves 1..7 before their polls: L2 prefetch of what every chunk loads first after this
  // exchange -- forward: its fix-up ring's first Psi_f and backward ring's first P matrices,
  // its workgroup-map row; backward: its fix-up ring's first Psi_b, its map row and the next
  // solve's first P matrices.  One 4-byte LDS-DMA load per 128-byte line into the slack after
  // the maps (no register held; the first poll's wait, which these waves pay anyway, covers
  // it -- the wave that runs the chain issues none, its LDS reads would wait for them).
  auto touch_next = [&](int dir, int s_next) {
    constexpr int LN = (int)((PSB + 127u) / 128u);  // lines of one B x B matrix
    constexpr int NMAT = 5;                         // matrices per chunk
    constexpr int TOT = KL * NMAT * LN;
    constexpr int STEP = kPartThreads - kSW;
    constexpr int NIT = (TOT + STEP - 1) / STEP;
    const bool has_in = dir == 0 ? wg > 0 : wg < G - 1;
#pragma unroll 1
    for (int it = 0; it < NIT; ++it) {  // (not unrolled: registers; the polls wait anyway)
      const int idx = min(tid - kSW + it * STEP, TOT - 1);
      const int c = idx / (NMAT * LN), r = idx - c * (NMAT * LN);
      const int m = r / LN, l = r - m * LN;
      const int k = KL * wg + c;
      const int clo = chunk_lo(n, K, k), chi = chunk_lo(n, K, k + 1);
      const double2* base;
      int i;
      if (m < 2) {  // the fix-up ring's first two
        base = dir == 0 ? Pf : Pb;
        i = clo + min(m, chi - clo - 1);
      } else if (m == 2) {  // the carry's workgroup-map row (none for an edge workgroup)
        base = has_in ? a.Pw + wsel(dir) * KL * PS : (dir == 0 ? Pf : Pb);
        i = has_in ? (dir == 0 ? max(c - 1, 0) : max(KL - 2 - c, 0)) : clo;
      } else if (dir == 0) {  // the backward chunk-local ring's first two
        base = P;
        i = chi - 1 - min(m - 3, chi - clo - 1);
      } else {  // the next solve's forward ring
        base = s_next >= 0 ? a.P + (size_t)s_next * n * PS : P;
        i = clo + min(m - 3, chi - clo - 1);
      }
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(reinterpret_cast<const char*>(base) +
                                                          (size_t)i * PSB + (unsigned)l * 128u),
          (__attribute__((address_space(3))) void*)(mats + KL * PS), 4, 0, 0);
    }
  };
  // steps 2-3 of one direction (after the chunk-local pass and its barrier)
  auto boundaries = [&](auto dirc, double2 (*bv)[16]) {
    constexpr int dir = decltype(dirc)::value;
    constexpr bool fwd = dir == 0;
    const auto fwdc = std::integral_constant<bool, fwd>{};
    if (tid < KL * 16) {  // (rows j >= B: copies of row B - 1, never used)
      const int k = tid >> 4;
      const int col = fwd ? chunk_lo(n, K, KL * wg + k + 1) - 1 : chunk_lo(n, K, KL * wg + k);
      const int row = min(tid & 15, B - 1);
      if constexpr (LY) yvl[k][tid & 15] = ysl[(col - c0w) * B + row];
      else yvl[k][tid & 15] = at(ys, ((unsigned)col * 16u + (unsigned)row) * 16u);
    }
    if (tid < 16) {
      bv[KL][tid] = z;
      bv[KL + 1][tid] = z;
    }
    __syncthreads();
    mark(fwd ? 1 : 5);  // chunk-end vectors + barrier (the maps' DMA already waited for)
    if (G == 1) {
      if (w == 0) chain(fwdc, bv, KL + 1);
    } else {
      const int cnt = fwd ? wg : G - 1 - wg;  // (block-uniform) upstream workgroups
      // this half's grid maps, distances d = 2 + cl + KL t: the first TM requested now (used in
      // step 3), any beyond the next T2 (G > 2 + (TM + T2) KL) loaded in step 3
      constexpr int TM = B >= 16 ? 1 : kSweepGridMapsHeld;  // (B = 16: registers)
      double2 tm[TM][KG];
      const double2* Tb = a.Tm + ((size_t)(s * 2 + dir) * sweep_grid_tri(G) +
                                  sweep_grid_tri(cnt)) * PS;
      sfor<0, TM>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        const int d = 2 + cl + KL * t;
        if (d <= cnt) ld_row(tm[t], Tb, d - 2);
      });
      // the next T2 of them (G > 2 + TM KL): waves 1..7 request theirs before polling, wave 0
      // after its chain (held through the polls, not through the chain: registers)
      constexpr int T2 = 1;
      double2 tm2[T2][KG];
      auto load_tm2 = [&]() {
        if (2 + KL * TM <= cnt)
          sfor<0, T2>([&](auto tc) {
            const int d = 2 + cl + KL * (TM + (int)decltype(tc)::value);
            if (d <= cnt) ld_row(tm2[decltype(tc)::value], Tb, d - 2);
          });
      };
      if (w == 0) {
        const double2 v = chain(fwdc, bv, KL + 1);
        const bool other = fwd ? wg + 1 < G : wg > 0;  // someone reads it
        if (other && lane < B)
          st_gran4(a.gran + ((size_t)(dir * 2 + (round & 1)) * G + wg) * kSweepGranStride +
                       4 * lane, part_tag(a.seq, round, dir), v);
        load_tm2();
      } else {
#if HH_SWEEP_TOUCH
        touch_next(dir, io.s_next);
#endif
        load_tm2();
        poll(dir);
      }
      ok = __syncthreads_and(ok);
      mark(fwd ? 2 : 6);  // zero-carry chain + publish | polls
      if (cnt > 0) {
        // 3. the halves' partials sum_t T(wg, u_d) y_end(u_d), u_d = wg -+ d (unused slots: a
        // select, so both halves of a wave run one instruction stream), then wave 0 adds them
        // to the nearest workgroup's vector (d = 1, identity map) in the halves' order
        double2 acc = z;
        sfor<0, TM>([&](auto tc) {
          constexpr int t = decltype(tc)::value;
          if (2 + KL * t <= cnt) {
            const int d = 2 + cl + KL * t;
            const int gi = fwd ? max(wg - d, 0) : min(d - 1, G - 1);  // (gin slot of u_d)
            acc = csel(d <= cnt, cadd(acc, rowdot(tm[t], &gin[gi * 16])), acc);
          }
        });
        sfor<0, T2>([&](auto tc) {
          constexpr int t = TM + decltype(tc)::value;
          if (2 + KL * t <= cnt) {
            const int d = 2 + cl + KL * t;
            const int gi = fwd ? max(wg - d, 0) : min(d - 1, G - 1);
            acc = csel(d <= cnt, cadd(acc, rowdot(tm2[decltype(tc)::value], &gin[gi * 16])), acc);
          }
        });
        for (int t = TM + T2; 2 + KL * t <= cnt; ++t) {
          const int d = 2 + cl + KL * t;
          const int gi = fwd ? max(wg - d, 0) : min(d - 1, G - 1);
          double2 m[KG];
          ld_row(m, Tb, min(d, cnt) - 2);
          acc = csel(d <= cnt, cadd(acc, rowdot(m, &gin[gi * 16])), acc);
        }
        if (g == 0) tl[cl][0][j] = acc;
        __syncthreads();
        if (tid < 16) {  // (every half wrote a partial, zero if it had no map)
          double2 p[KL];
          sfor<0, KL>([&](auto hc) { p[decltype(hc)::value] = tl[decltype(hc)::value][0][tid]; });
          double2 v = gin[(fwd ? wg - 1 : 0) * 16 + tid];
          sfor<0, KL>([&](auto hc) { v = cadd(v, p[decltype(hc)::value]); });
          bv[KL][tid] = v;
        }
      }
    }
    __syncthreads();
    mark(fwd ? 3 : 7);  // grid step
  };
  // the true carry into this half's chunk (forward: y at the end of chunk cl - 1; backward: x
  // at the start of chunk cl + 1) -- the zero-carry chain's value plus the workgroup carry
  // bv[KL] through the workgroup's prefix / suffix map, Pw[s][wg][dir][idx]: one B x B step per
  // chunk instead of the chain again.  Chunk 0 (forward) / 15 (backward) takes bv[KL] itself.
  // Returns the LDS vector to use (tl[cl][0] when it had to be formed).
  auto carry_in = [&](auto dirc, double2 (*bv)[16]) -> const double2* {
    constexpr int dir = decltype(dirc)::value;
    const bool edge = dir == 0 ? cl == 0 : cl == KL - 1;  // (per half)
    const int nb = dir == 0 ? cl - 1 : cl + 1;            // neighbour chunk
    const bool has_in = dir == 0 ? wg > 0 : wg < G - 1;   // (block-uniform) nonzero bv[KL]
    if (!has_in) return &bv[edge ? KL : nb][0];
    const int idx = dir == 0 ? max(cl - 1, 0) : max(KL - 2 - cl, 0);  // (edge: unused, clamped)
    double2 m[KG];
    ld_row(m, a.Pw + wsel(dir) * KL * PS, idx);
    const double2 v = cadd(bv[edge ? KL + 1 : nb][jl], rowdot(m, &bv[KL][0]));
    if (g == 0) tl[cl][0][j] = csel(edge, bv[KL][jl], v);
    wave_sync();
    __builtin_amdgcn_sched_barrier(0);  // (keep the next ring's loads out of this step's span)
    return &tl[cl][0][0];
  };

  // ---- 1. forward, chunk-local (the forward chain maps on their way to LDS meanwhile) ----
  stage(0);
  {
    double2 Pq[D][KG], cq[D], rq[D], sq[SR ? D : 1];
    auto ld = [&](auto qc, int q) {
      constexpr int r = decltype(qc)::value;
      const int i = lo + min(q, last);
      ld_row(Pq[r], P, i);
      cq[r] = AW[i];
      rq[r] = at(io.rhs, (unsigned)i * 16u + roff);
      if constexpr (SR) sq[r] = R1[i];
    };
    sfor<0, D>([&](auto qc) { ld(qc, decltype(qc)::value); });
    wait_vm<D * (KG + 2 + (SR ? 1 : 0))>();  // the maps' DMA (its LDS writes), not the ring
    double2 y = z;
    for (int q0 = 0; q0 < lenw; q0 += D) {  // steps past the half's last column: unstored
      sfor<0, D>([&](auto qc) {
        constexpr int r = decltype(qc)::value;
        __builtin_amdgcn_sched_barrier(0);
        const int q = q0 + r;
        double2 rr = csel(has_rhs, rq[r], z);
        if constexpr (SR) rr = cmul(rr, cmul(io.rmul, sq[r]));
        tl[cl][r & 1][j] = csub(rr, cmul(cmul(cq[r], R2), y));
        wave_sync();
        y = rowdot(Pq[r], &tl[cl][r & 1][0]);
        yput(ystore && q < len, lo + q, y);
        ld(qc, q + D);
      });
    }
  }
  __syncthreads();
  mark(0);  // chunk-local forward
  // ---- 2-3. forward boundaries ----
  boundaries(std::integral_constant<int, 0>{}, bf);
  // ---- 4. forward fix-up (rows independent): y_i = yL_i + Psi_f[i] y_{lo-1} ----
  {
    double2 mq[D][KG], yq[D];
    auto ld = [&](auto qc, int q) {
      constexpr int r = decltype(qc)::value;
      const int i = lo + min(q, last);
      ld_row(mq[r], Pf, i);
      yq[r] = yget(i);
    };
    // the ring's first loads ahead of the carry's map row (B = 16: after it -- registers)
    const double2* carry = nullptr;
    if constexpr (B >= 16) carry = carry_in(std::integral_constant<int, 0>{}, bf);
    stage(1);  // the backward chain maps, overlapping this phase
    sfor<0, D>([&](auto qc) { ld(qc, decltype(qc)::value); });
    if constexpr (B < 16) carry = carry_in(std::integral_constant<int, 0>{}, bf);
    else wait_vm<D * (KG + (LY ? 0 : 1))>();  // the DMA, not the ring
    for (int q0 = 0; q0 < lenw; q0 += D) {
      sfor<0, D>([&](auto qc) {
        constexpr int r = decltype(qc)::value;
        const int q = q0 + r;
        const double2 y = cadd(yq[r], rowdot(mq[r], carry));
        yput(ystore && q < len, lo + q, y);
        ld(qc, q + D);
      });
    }
  }
  // ---- 4b. backward, chunk-local: xL_i = y_i - P_i U_i xL_{i+1} (own rows: no barrier) ----
  {
    double2 Pq[D][KG], cq[D], yq[D];
    auto ld = [&](auto qc, int q) {
      constexpr int r = decltype(qc)::value;
      const int i = hi - 1 - min(q, last);
      ld_row(Pq[r], P, i);
      cq[r] = AE[i];
      yq[r] = yget(i);
    };
    sfor<0, D>([&](auto qc) { ld(qc, decltype(qc)::value); });
    double2 x = z;
    for (int q0 = 0; q0 < lenw; q0 += D) {
      sfor<0, D>([&](auto qc) {
        constexpr int r = decltype(qc)::value;
        __builtin_amdgcn_sched_barrier(0);
        const int q = q0 + r;
        tl[cl][r & 1][j] = cmul(cmul(cq[r], R2), x);
        wave_sync();
        x = csub(yq[r], rowdot(Pq[r], &tl[cl][r & 1][0]));
        yput(ystore && q < len, hi - 1 - q, x);
        ld(qc, q + D);
      });
    }
  }
  __syncthreads();
  mark(4);  // forward fix-up + chunk-local backward
  // ---- 2-3. backward boundaries ----
  boundaries(std::integral_constant<int, 1>{}, bb);
  // ---- 5. fix-up + output ----
  {
    double2 mq[D][KG], xq[D], oq[D], sq[SO ? D : 1];
    auto ld = [&](auto qc, int q) {
      constexpr int r = decltype(qc)::value;
      const int i = lo + min(q, last);
      ld_row(mq[r], Pb, i);
      xq[r] = yget(i);
      oq[r] = at(io.out, (unsigned)i * 16u + ooff);
      if constexpr (SO) sq[r] = R1[i];
    };
    const double2* carry = nullptr;
    if constexpr (B >= 16) carry = carry_in(std::integral_constant<int, 1>{}, bb);
    sfor<0, D>([&](auto qc) { ld(qc, decltype(qc)::value); });
    if constexpr (B < 16) carry = carry_in(std::integral_constant<int, 1>{}, bb);
    for (int q0 = 0; q0 < lenw; q0 += D) {
      sfor<0, D>([&](auto qc) {
        constexpr int r = decltype(qc)::value;
        const int q = q0 + r;
        const double2 x = cadd(xq[r], rowdot(mq[r], carry));
        double2 xo = x;
        if constexpr (SO) xo = cmul(x, sq[r]);
        const double2 o = csel(io.alpha_old != 0.0, cscale(oq[r], io.alpha_old), z);
        if (has_out && q < len) at(io.out, (unsigned)(lo + q) * 16u + ooff) = cadd(o, cmul(io.omul, xo));
        ld(qc, q + D);
      });
    }
  }
  __syncthreads();
  mark(8);  // fix-up + output
}

__device__ __forceinline__ SolveIO solve_io(const double2* rhs, int rhs_first, double2 rmul,
                                            double2* out, int out_first, double alpha_old,
                                            double2 omul, size_t ld, int s_next = -1) {
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
  io.s_next = s_next;
  return io;
}

// this lane's local-layer 1/s2 in a partitioned solve (row j = lane mod 16 of the block; 0 on
// padding rows), loaded once per launch: a load inside a solve would sit before the chain
// maps' LDS DMA and its use would wait for the DMA too
template <int B>
__device__ __forceinline__ double2 part_r2(const SweepArgs& a) {
  const int j = threadIdx.x & 15;
  return csel(j < B && j < a.b, a.tab_k[4 * min(j, B - 1)], make_double2(0.0, 0.0));
}

// the sequential sweeps' solves: one wave walking the columns, or (CH) the partitioned solve
// of a.G workgroups of kSweepChunks / 2 waves (round: the solve's index in the launch)
template <int B, bool SR, bool SO, bool CH, bool LY>
__device__ __forceinline__ void solve(const SweepArgs& a, int s, int round, const SolveIO& io,
                                      const double2 R2, double2* ys, bool& ok,
                                      unsigned long long (&tk)[kSweepProfSlots]) {
  if constexpr (CH)
    bt_solve_chunked<B, SR, SO, LY>(a, s, round, io, R2, ys, ok, tk);
  else
    bt_solve<B, SR, SO>(a, s, io, ys);
}

// diagnostic phase ticks of a partitioned launch: thread 0 of each workgroup adds its sums
template <bool CH>
__device__ __forceinline__ void prof_flush(const SweepArgs& a, const unsigned long long (&tk)[kSweepProfSlots]) {
  if constexpr (CH) {
    if (a.prof != nullptr && threadIdx.x == 0)
      for (int q = 0; q < 9; ++q) a.prof[(size_t)blockIdx.x * kSweepProfSlots + q] += tk[q];
  }
}

// the columns a workgroup of a partitioned launch owns (all n for the sequential one)
template <bool CH>
__device__ __forceinline__ void own_columns(const SweepArgs& a, int& c0, int& c1) {
  c0 = 0;
  c1 = a.n;
  if constexpr (CH) {
    const int K = kSweepChunks * a.G;
    c0 = chunk_lo(a.n, K, kSweepChunks * (int)blockIdx.x);
    c1 = chunk_lo(a.n, K, kSweepChunks * ((int)blockIdx.x + 1));
  }
}

// Algorithm 2.4 pieces.  u: layer-major [n][n] (layer j at u + j n).
// forward sweep (code.py:363-370): TFuF = HF^-1 u[0:b] -> uF; u[b] -= S_b * TFuF[b-1];
// for m = b+1..n-1: u[m] -= S_m * T_m u[m-1]  (S_m = BS_m R1[i], folded into the solve).
// Partitioned: a workgroup reads and writes only its own columns of u and uF between solves.
template <int B, bool CH, bool LY = false>
__global__ __launch_bounds__(CH ? kPartThreads : kSW) void sweep_forward_kernel(
    const SweepArgs a, double2* u, double2* uF) {
  if (a.stop && *a.stop) return;
  const int n = a.n, b = a.b;
  const double2 one = make_double2(1.0, 0.0);
  double2* ys = a.yscr;
  bool ok = true;
  int round = 0;
  unsigned long long tk[kSweepProfSlots] = {};
  const double2 R2 = part_r2<B>(a);
  solve<B, false, false, CH, LY>(a, 0, round++,
                                 solve_io(u, 0, one, uF, 0, 0.0, one, n, b + 1 < n ? 1 : -1),
                                 R2, ys, ok, tk);
  const double2* R1 = a.tab_i + 2 * n;
  int c0, c1;
  own_columns<CH>(a, c0, c1);
  {
    const double2 BS = a.tab_glob[4 * b + 1];  // c3 of global layer b (code.py:150-153)
    for (int i = c0 + threadIdx.x; i < c1; i += blockDim.x)
      u[(size_t)b * n + i] = csub(u[(size_t)b * n + i], cmul(cmul(BS, R1[i]), uF[(size_t)(b - 1) * n + i]));
  }
  __syncthreads();
  for (int m = b + 1; m < n; ++m) {  // system s = m - b covers layers m-b .. m-1
    const double2 BS = a.tab_glob[4 * m + 1];
    solve<B, false, true, CH, LY>(a, m - b, round++,
                              solve_io(u + (size_t)(m - 1) * n, b - 1, one, u + (size_t)m * n,
                                       b - 1, 1.0, cneg(BS), n, m + 1 < n ? m + 1 - b : -1),
                              R2, ys, ok, tk);
  }
  prof_flush<CH>(a, tk);
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
template <int B, bool CH, bool LY = false>
__global__ __launch_bounds__(CH ? kPartThreads : kSW) void sweep_backward_kernel(
    const SweepArgs a, double2* u, double2* uF) {
  if (a.stop && *a.stop) return;
  const int n = a.n, b = a.b;
  double2* ys = a.yscr;
  const double2 mone = make_double2(-1.0, 0.0);
  bool ok = true;
  int round = 0;
  unsigned long long tk[kSweepProfSlots] = {};
  const double2 R2 = part_r2<B>(a);
  for (int m = n - 1; m >= b + 1; --m) {
    const double2 BN = a.tab_glob[4 * (m - 1) + 2];  // c4 of global layer m-1 (code.py:131-140)
    solve<B, true, false, CH, LY>(a, m - b, round++,
                              solve_io(u + (size_t)m * n, b - 1, BN, u + (size_t)(m - 1) * n,
                                       b - 1, 1.0, mone, n, m - 1 - b),
                              R2, ys, ok, tk);
  }
  // H_F is block diagonal: only its last layer sees the (last-layer-only) right-hand side
  const double2 BN = a.tab_glob[4 * (b - 1) + 2];
  solve<B, true, false, CH, LY>(a, 0, round++,
                            solve_io(u + (size_t)b * n, b - 1, BN, uF + (size_t)(b - 1) * n, b - 1,
                                     1.0, mone, n),
                            R2, ys, ok, tk);
  prof_flush<CH>(a, tk);
  int c0, c1;
  own_columns<CH>(a, c0, c1);
  for (int l = 0; l < b; ++l)
    for (int i = c0 + threadIdx.x; i < c1; i += blockDim.x)
      u[(size_t)l * n + i] = uF[(size_t)l * n + i];
}

// a partitioned sweep: G workgroups of kPartThreads, all co-resident (a cooperative launch
// when G > 1, so a grid that cannot be placed fails at launch instead of waiting forever)
template <int B>
void launch_part(const void* fn, const SweepArgs& a, double2* u, double2* uF, hipStream_t st,
                 bool ly) {
  const size_t lds = part_lds_bytes<B>(a.G, a.n, ly);
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess) {
    SweepArgs arg = a;
    void* params[] = {&arg, &u, &uF};
    e = a.G > 1 && sweep_coop_launch()
            ? hipLaunchCooperativeKernel(fn, dim3(a.G), dim3(kPartThreads), params,
                                         (unsigned)lds, st)
            : hipLaunchKernel(fn, dim3(a.G), dim3(kPartThreads), params, lds, st);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    fail(HH_ERR_HIP, "sweeping preconditioner: launch of the partitioned sweep over %d "
                     "workgroups (%zu B of LDS each) failed (%s)",
         a.G, lds, hipGetErrorString(e));
  }
}

// the B-vectors of a partitioned solve in LDS when they fit beside the chain maps
template <int B>
bool part_ys_lds(int G, int n) {
  return part_lds_bytes<B>(G, n, true) + kPartStaticLds <= kPartLdsBudget;
}

template <int B>
void launch_all(const SweepArgs& a, int what, double2* u, double2* uF, int asis, hipStream_t st) {
  switch (what) {
    case 0:
      hipLaunchKernelGGL((sweep_factor_kernel<B>), dim3(a.nsys), dim3(kSW), 0, st, a);
      break;
    case 1:
      if (a.chunks > 0 && part_ys_lds<B>(a.G, a.n))
        launch_part<B>(reinterpret_cast<const void*>(&sweep_forward_kernel<B, true, true>), a, u,
                       uF, st, true);
      else if (a.chunks > 0)
        launch_part<B>(reinterpret_cast<const void*>(&sweep_forward_kernel<B, true, false>), a, u,
                       uF, st, false);
      else
        hipLaunchKernelGGL((sweep_forward_kernel<B, false>), dim3(1), dim3(kSW), 0, st, a, u, uF);
      break;
    case 2:
      hipLaunchKernelGGL((sweep_middle_kernel<B>), dim3(a.nsys - 1), dim3(kSW), 0, st, a, u,
                         asis);
      break;
    case 3:
      if (a.chunks > 0 && part_ys_lds<B>(a.G, a.n))
        launch_part<B>(reinterpret_cast<const void*>(&sweep_backward_kernel<B, true, true>), a, u,
                       uF, st, true);
      else if (a.chunks > 0)
        launch_part<B>(reinterpret_cast<const void*>(&sweep_backward_kernel<B, true, false>), a, u,
                       uF, st, false);
      else
        hipLaunchKernelGGL((sweep_backward_kernel<B, false>), dim3(1), dim3(kSW), 0, st, a, u, uF);
      break;
    case 4:
      hipLaunchKernelGGL((sweep_chunk_setup_kernel<B>), dim3(a.nsys * a.chunks), dim3(kSW), 0,
                         st, a);
      hipLaunchKernelGGL((sweep_wg_setup_kernel<B>), dim3(a.nsys * a.G), dim3(kSW), 0, st, a);
      if (a.G > 2)
        hipLaunchKernelGGL((sweep_grid_setup_kernel<B>), dim3(a.nsys * 2 * a.G), dim3(kSW), 0,
                           st, a);
      break;
    default:
      break;
  }
}

}  // namespace

size_t sweep_scratch_per_wave(int n) { return (size_t)(n + kMaxRing) * 16 + 64; }
size_t sweep_chunk_scratch(int n) { return (size_t)n * 16 + (size_t)32 * kPartThreads; }
int sweep_part_max_wgs(int B) {
  return B == 4 ? part_max_wgs<4>() : B == 8 ? part_max_wgs<8>() : B == 12 ? part_max_wgs<12>()
                                                                          : part_max_wgs<16>();
}
bool sweep_part_ys_lds(int B, int G, int n) {
  return B == 4 ? part_ys_lds<4>(G, n) : B == 8 ? part_ys_lds<8>(G, n)
       : B == 12 ? part_ys_lds<12>(G, n) : part_ys_lds<16>(G, n);
}
size_t sweep_part_granules(int G) { return (size_t)2 * 2 * G * kSweepGranStride; }

bool sweep_coop_launch() {
  static const bool coop = knobs().sweep_coop != 0 && !under_profiler();
  return coop;
}

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
