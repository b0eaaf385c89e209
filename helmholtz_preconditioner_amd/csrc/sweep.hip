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

// ------------------------------------------------------- partitioned (chunked) solves
// The forward recurrence y_i = P_i (r_i - L_i y_{i-1}) = c_i + M_i y_{i-1} and the backward one
// x_i = y_i + N_i x_{i+1} (M_i = -P_i L_i, N_i = -P_i U_i) are linear in the carried vector, so
// with the columns split into K chunks [lo_k, hi_k):
//   y_i = yL_i + Psi_f[i] y_{lo_k - 1},   Psi_f[i] = M_i M_{i-1} .. M_{lo_k}
//   x_i = xL_i + Psi_b[i] x_{hi_k},       Psi_b[i] = N_i N_{i+1} .. N_{hi_k - 1}
// where yL / xL run the recurrence inside the chunk from a zero carry.  A solve is then: every
// chunk's local recurrence at once (one wave per chunk), the K chunk boundaries in sequence
// (one B x B matvec each), and a parallel fix-up of every column -- dependent depth ~2 (n / K +
// K) steps instead of 2 n.  The Psi products are operator data, formed once at setup.
__device__ __forceinline__ int chunk_lo(int n, int K, int k) { return n * k / K; }  // n K < 2^31

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Setup: Psi_f and Psi_b of one (system, chunk) per wave.  Lanes (g, j): row j, columns
// [g KG, (g+1) KG) of the running product, which every lane reads whole from LDS.
template <int B>
__global__ __launch_bounds__(kSW) void sweep_chunk_setup_kernel(const SweepArgs a) {
  constexpr int KG = B / kGroups;
  constexpr size_t PS = (size_t)B * B;
  __shared__ double2 Q[2][B][B];
  constexpr int K = kSweepChunks;
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
        prow[m] = cneg(cmul(P[((size_t)i * B + jl) * B + m], cmul(cc, r2)));
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
          out[((size_t)i * B + j) * B + g * KG + c] = v[c];
        });
      }
      wave_sync();
    }
  }
}

template <int B>
constexpr int chunk_ring() { return B <= 8 ? 4 : (B == 12 ? 2 : 3); }  // (no spills at 256 VGPRs)

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

// One partitioned solve by a block of kSweepChunks / 2 waves, with the SolveIO contract of
// bt_solve.  Each 32-lane half of a wave owns one chunk (chunk c = 2 w + h): lanes (g, j) of
// the half -- row j of the block, columns [g KG, (g+1) KG), KG = B / 2 -- so the two chunks of
// a wave step in lockstep (their lengths differ by at most one column: the shorter one's last
// step runs on clamped data and is not stored).  Half-wave chunks give 16 chunks with 8 waves,
// i.e. 256 VGPRs per lane instead of the 128 a 16-wave block allows.  ys: sweep_chunk_scratch.
//   1. forward, chunk-local (every half): yL_i = P_i (r_i - L_i yL_{i-1}), from yL_{lo-1} = 0
//   2. forward boundaries (wave 0, K - 1 steps): y_{hi_k - 1} = yL + Psi_f y_{hi_{k-1} - 1}
//   3. forward fix-up (rows independent): y_i = yL_i + Psi_f[i] y_{lo-1}; then backward,
//      chunk-local: xL_i = y_i - P_i U_i xL_{i+1} (a wave reads back only its own rows)
//   4. backward boundaries (wave 0): x_{lo_k} = xL_{lo_k} + Psi_b x_{lo_{k+1}}
//   5. fix-up + output (rows independent, prefetched like 1 / 3): x_i = xL_i + Psi_b[i] x_{hi}
// (chunk 0 in 3 and chunk K-1 in 5 multiply their Psi rows by an LDS zero vector instead of
// branching: both halves run one instruction stream.)  A ring slot of KG = 6 double2 is 24
// VGPRs at B = 12, so no phase keeps two matrix rings.
template <int B, bool SR, bool SO>
__device__ __forceinline__ void bt_solve_chunked(const SweepArgs& a, int s, const SolveIO& io,
                                                 double2* ys) {
  constexpr int KG = B / 2;
  constexpr int D = chunk_ring<B>();
  constexpr int K = kSweepChunks;
  constexpr size_t PS = (size_t)B * B;
  constexpr unsigned PSB = (unsigned)PS * 16u;  // bytes of one B x B matrix
  __shared__ double2 tl[K][2][16];
  __shared__ double2 bf[K + 1][16], bb[K + 1][16];  // [K]: zeros
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, h = lane >> 5, g = (lane >> 4) & 1, j = lane & 15;
  const int c = 2 * w + h;  // this half's chunk
  const int n = a.n;
  const int lo = chunk_lo(n, K, c), hi = chunk_lo(n, K, c + 1), len = hi - lo;
  const int m0 = chunk_lo(n, K, 2 * w + 1);
  const int lenw = max(m0 - chunk_lo(n, K, 2 * w), chunk_lo(n, K, 2 * w + 2) - m0);  // both halves
  const int last = len - 1;  // (n >= 2 K: every chunk has >= 2 columns)
  const bool row = j < B && j < a.b;
  const int jl = j < B ? j : B - 1;
  const bool has_rhs = row && j >= io.rhs_first;
  const bool has_out = row && j >= io.out_first && g == 0;
  // byte offsets of this lane from scalar bases
  const unsigned roff = has_rhs ? (unsigned)((j - io.rhs_first) * io.rhs_ld) * 16u : 0u;
  const unsigned ooff =
      (row && j >= io.out_first) ? (unsigned)((j - io.out_first) * io.out_ld) * 16u : 0u;
  const unsigned lofs = (unsigned)(jl * B + g * KG) * 16u;  // row jl, this lane's columns
  const unsigned dofs = ((unsigned)(n * 16) + threadIdx.x) * 16u;  // this lane's dummy slot
  const size_t sbase = (size_t)s * n * PS;
  const double2* P = a.P + sbase;
  const double2* Pf = a.Pf + sbase;
  const double2* Pb = a.Pb + sbase;
  const double2 z = make_double2(0.0, 0.0);
  const double2 R2 = csel(row, a.tab_k[4 * jl], z);
  const double2* AW = a.tab_i;
  const double2* AE = a.tab_i + n;
  const double2* R1 = a.tab_i + 2 * n;
  const bool ystore = g == 0 && j < B;
  auto ld_row = [&](double2 (&m)[KG], const double2* base, int i) {
    const unsigned o = (unsigned)i * PSB + lofs;
    sfor<0, KG>([&](auto cc) { m[decltype(cc)::value] = at(base, o + 16u * decltype(cc)::value); });
  };
  auto yget = [&](int i) { return at(ys, ((unsigned)i * 16u + (unsigned)jl) * 16u); };
  auto yput = [&](bool ok, int i, double2 v) {
    at(ys, ok ? ((unsigned)i * 16u + (unsigned)j) * 16u : dofs) = v;
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
  if (threadIdx.x < 16) {
    bf[K][threadIdx.x] = z;
    bb[K][threadIdx.x] = z;
  }

  // ---- 1. forward, chunk-local ----
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
    double2 y = z;
    for (int q0 = 0; q0 < lenw; q0 += D) {  // steps past the half's last column: unstored
      sfor<0, D>([&](auto qc) {
        constexpr int r = decltype(qc)::value;
        __builtin_amdgcn_sched_barrier(0);
        const int q = q0 + r;
        double2 rr = csel(has_rhs, rq[r], z);
        if constexpr (SR) rr = cmul(rr, cmul(io.rmul, sq[r]));
        tl[c][r & 1][j] = csub(rr, cmul(cmul(cq[r], R2), y));
        wave_sync();
        y = rowdot(Pq[r], &tl[c][r & 1][0]);
        yput(ystore && q < len, lo + q, y);
        ld(qc, q + D);
      });
    }
  }
  __syncthreads();
  // ---- 2. forward boundaries (wave 0; both halves compute the same values) ----
  if (w == 0) {
    double2 v = yget(chunk_lo(n, K, 1) - 1);
    if (lane < 16) bf[0][j] = v;
    double2 mq[D][KG], yq[D];
    auto ld = [&](auto qc, int k) {
      constexpr int r = decltype(qc)::value;
      const int e = chunk_lo(n, K, min(k, K - 1) + 1) - 1;
      ld_row(mq[r], Pf, e);
      yq[r] = yget(e);
    };
    sfor<0, D>([&](auto qc) { ld(qc, 1 + decltype(qc)::value); });
    wave_sync();
#pragma unroll 1
    for (int k0 = 1; k0 < K; k0 += D) {
      sfor<0, D>([&](auto qc) {
        constexpr int r = decltype(qc)::value;
        const int k = k0 + r;
        if (k < K) {  // (wave-uniform)
          v = cadd(yq[r], rowdot(mq[r], &bf[k - 1][0]));
          if (lane < 16) bf[k][j] = v;
          wave_sync();
        }
        ld(qc, k + D);
      });
    }
  }
  __syncthreads();
  // ---- 3. forward fix-up (rows independent): y_i = yL_i + Psi_f[i] y_{lo-1} ----
  {
    double2 mq[D][KG], yq[D];
    auto ld = [&](auto qc, int q) {
      constexpr int r = decltype(qc)::value;
      const int i = lo + min(q, last);
      ld_row(mq[r], Pf, i);
      yq[r] = yget(i);
    };
    sfor<0, D>([&](auto qc) { ld(qc, decltype(qc)::value); });
    const double2* carry = &bf[c > 0 ? c - 1 : K][0];
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
  // ---- 3b. backward, chunk-local: xL_i = y_i - P_i U_i xL_{i+1} (own rows: no barrier) ----
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
        tl[c][r & 1][j] = cmul(cmul(cq[r], R2), x);
        wave_sync();
        x = csub(yq[r], rowdot(Pq[r], &tl[c][r & 1][0]));
        yput(ystore && q < len, hi - 1 - q, x);
        ld(qc, q + D);
      });
    }
  }
  __syncthreads();
  // ---- 4. backward boundaries (wave 0) ----
  if (w == 0) {
    double2 v = yget(chunk_lo(n, K, K - 1));
    if (lane < 16) bb[K - 1][j] = v;
    double2 mq[D][KG], yq[D];
    auto ld = [&](auto qc, int t) {  // t = 1 .. K-1: chunk k = K - 1 - t
      constexpr int r = decltype(qc)::value;
      const int e = chunk_lo(n, K, max(K - 1 - t, 0));
      ld_row(mq[r], Pb, e);
      yq[r] = yget(e);
    };
    sfor<0, D>([&](auto qc) { ld(qc, 1 + decltype(qc)::value); });
    wave_sync();
#pragma unroll 1
    for (int t0 = 1; t0 < K; t0 += D) {
      sfor<0, D>([&](auto qc) {
        constexpr int r = decltype(qc)::value;
        const int t = t0 + r, k = K - 1 - t;
        if (t < K) {
          v = cadd(yq[r], rowdot(mq[r], &bb[k + 1][0]));
          if (lane < 16) bb[k][j] = v;
          wave_sync();
        }
        ld(qc, t + D);
      });
    }
  }
  __syncthreads();
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
    sfor<0, D>([&](auto qc) { ld(qc, decltype(qc)::value); });
    const double2* carry = &bb[c < K - 1 ? c + 1 : K][0];
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

// the sequential sweeps' solves: one wave walking the columns, or (CH) the partitioned solve
// of one workgroup of kSweepChunks / 2 waves
template <int B, bool SR, bool SO, bool CH>
__device__ __forceinline__ void solve(const SweepArgs& a, int s, const SolveIO& io, double2* ys) {
  if constexpr (CH)
    bt_solve_chunked<B, SR, SO>(a, s, io, ys);
  else
    bt_solve<B, SR, SO>(a, s, io, ys);
}

// Algorithm 2.4 pieces.  u: layer-major [n][n] (layer j at u + j n).
// forward sweep (code.py:363-370): TFuF = HF^-1 u[0:b] -> uF; u[b] -= S_b * TFuF[b-1];
// for m = b+1..n-1: u[m] -= S_m * T_m u[m-1]  (S_m = BS_m R1[i], folded into the solve).
template <int B, bool CH>
__global__ __launch_bounds__(CH ? kSweepChunks / 2 * kSW : kSW) void sweep_forward_kernel(
    const SweepArgs a, double2* u, double2* uF) {
  if (a.stop && *a.stop) return;
  const int n = a.n, b = a.b;
  const double2 one = make_double2(1.0, 0.0);
  double2* ys = a.yscr;
  solve<B, false, false, CH>(a, 0, solve_io(u, 0, one, uF, 0, 0.0, one, n), ys);
  const double2* R1 = a.tab_i + 2 * n;
  {
    const double2 BS = a.tab_glob[4 * b + 1];  // c3 of global layer b (code.py:150-153)
    for (int i = threadIdx.x; i < n; i += blockDim.x)
      u[(size_t)b * n + i] = csub(u[(size_t)b * n + i], cmul(cmul(BS, R1[i]), uF[(size_t)(b - 1) * n + i]));
  }
  __syncthreads();
  for (int m = b + 1; m < n; ++m) {  // system s = m - b covers layers m-b .. m-1
    const double2 BS = a.tab_glob[4 * m + 1];
    solve<B, false, true, CH>(a, m - b, solve_io(u + (size_t)(m - 1) * n, b - 1, one,
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
template <int B, bool CH>
__global__ __launch_bounds__(CH ? kSweepChunks / 2 * kSW : kSW) void sweep_backward_kernel(
    const SweepArgs a, double2* u, double2* uF) {
  if (a.stop && *a.stop) return;
  const int n = a.n, b = a.b;
  double2* ys = a.yscr;
  const double2 mone = make_double2(-1.0, 0.0);
  for (int m = n - 1; m >= b + 1; --m) {
    const double2 BN = a.tab_glob[4 * (m - 1) + 2];  // c4 of global layer m-1 (code.py:131-140)
    solve<B, true, false, CH>(a, m - b, solve_io(u + (size_t)m * n, b - 1, BN,
                                               u + (size_t)(m - 1) * n, b - 1, 1.0, mone, n), ys);
  }
  // H_F is block diagonal: only its last layer sees the (last-layer-only) right-hand side
  const double2 BN = a.tab_glob[4 * (b - 1) + 2];
  solve<B, true, false, CH>(a, 0, solve_io(u + (size_t)b * n, b - 1, BN, uF + (size_t)(b - 1) * n,
                                          b - 1, 1.0, mone, n), ys);
  for (size_t p = threadIdx.x; p < (size_t)b * n; p += blockDim.x) u[p] = uF[p];
}

template <int B>
void launch_all(const SweepArgs& a, int what, double2* u, double2* uF, int asis, hipStream_t st) {
  switch (what) {
    case 0:
      hipLaunchKernelGGL((sweep_factor_kernel<B>), dim3(a.nsys), dim3(kSW), 0, st, a);
      break;
    case 1:
      if (a.chunks > 0)
        hipLaunchKernelGGL((sweep_forward_kernel<B, true>), dim3(1), dim3(kSweepChunks / 2 * kSW), 0, st,
                           a, u, uF);
      else
        hipLaunchKernelGGL((sweep_forward_kernel<B, false>), dim3(1), dim3(kSW), 0, st, a, u, uF);
      break;
    case 2:
      hipLaunchKernelGGL((sweep_middle_kernel<B>), dim3(a.nsys - 1), dim3(kSW), 0, st, a, u,
                         asis);
      break;
    case 3:
      if (a.chunks > 0)
        hipLaunchKernelGGL((sweep_backward_kernel<B, true>), dim3(1), dim3(kSweepChunks / 2 * kSW), 0, st,
                           a, u, uF);
      else
        hipLaunchKernelGGL((sweep_backward_kernel<B, false>), dim3(1), dim3(kSW), 0, st, a, u, uF);
      break;
    case 4:
      hipLaunchKernelGGL((sweep_chunk_setup_kernel<B>), dim3(a.nsys * kSweepChunks), dim3(kSW), 0, st,
                         a);
      break;
    default:
      break;
  }
}

}  // namespace

size_t sweep_scratch_per_wave(int n) { return (size_t)(n + kMaxRing) * 16 + 64; }
size_t sweep_chunk_scratch(int n) { return (size_t)n * 16 + kSweepChunks * kSW; }

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
