// Sweeping preconditioner, dense-transfer form for gfx950.
//
// Every solve algo2_4 (code.py:356-385) performs is v -> lu_Hm.solve([0 .. 0, v])[-n:], i.e.
// the n x n matrix T_m = E^T H_m^-1 E (E = the last layer of the moving-PML sub-problem H_m,
// code.py:282-290), and the H_F solves are the n x n inverses A_ll^-1 of its b diagonal blocks
// (code.py:177-183: H_F has no inter-layer blocks).  When the n matrices fit in HBM
// (n^3 x 16 B: 17 GB at n = 1023, 137 GB at n = 2047) they are formed once at setup and the
// apply becomes a chain of 2 (n - b) + 1 dense complex GEMVs -- HBM-streaming kernels -- in
// place of 2 (n - b) latency-bound block-Thomas solves of 2n dependent steps each (sweep.hip).
//
// Setup: the block-Thomas factors P_i = Lambda_i^-1 of every system (sweep.hip) applied to
// all n unit right-hand sides at once, one RHS column per lane:
//   forward  y_i = P_i (r_i - W_i y_{i-1}),   r_i = e (the RHS layer(s)) at i == k, else 0
//   backward x_i = y_i - P_i (U_i x_{i+1})
// with W_i = diag(AW_i R2_l), U_i = diag(AE_i R2_l) over the b layers l (the in-layer
// couplings c1 / c2 of code.py:238-251 under the moving PML s2m).  T[i][k] = x_i[last layer]
// (H_m) or x_i[l] for every layer l (H_F, whose layers are independent).  y_i is zero for
// i < k, so a block of RHS columns starting at k0 begins its forward pass at i = k0.
//
// Apply (sweep order of algo2_4, with the forward and middle sweeps fused: the middle sweep's
// T_m u_{m-1} is the very product the forward step m computes, on the same u_{m-1}):
//   F0   w_l = A_ll^-1 r_l (l < b);      u_b = r_b - S_b . w_{b-1}                (code.py:362-364)
//   FWD  t = T_m u_{m-1};  w_{m-1} = t (corrected) | u_{m-1} - t (as-is, Q2);
//        u_m = r_m - S_m . t                                                   (m = b+1 .. n-1)
//   MID  w_{n-1} = T_n u_{n-1}  (| u_{n-1} - T_n u_{n-1})                        (code.py:372-375)
//   BWD  w_{m-1} -= T_m (N_{m-1} . w_m)                                        (m = n-1 .. b+1)
//   FC   w_{b-1} -= A_bb^-1 (N_{b-1} . w_b)                                      (code.py:381-384)
// with S_m = BS_m R1_i, N_m = BN_m R1_i (c3 / c4 of code.py:130-154).  w is the result.
#include "hh_internal.hpp"
#include "hh_complex.hpp"
#include "sweep.hpp"

#include <algorithm>
#include <type_traits>

namespace hh {
namespace {

template <int K, int N, class F>
__device__ __forceinline__ void ufor(F&& f) {
  if constexpr (K < N) {
    f(std::integral_constant<int, K>{});
    ufor<K + 1, N>(f);
  }
}

constexpr int kSetupThreads = 256;  // RHS columns per setup block

// ------------------------------------------------------------------------------- setup
template <int B>
__global__ __launch_bounds__(kSetupThreads) void dense_setup_kernel(const SweepArgs a, int s_base,
                                                                    double2* yscr,
                                                                    size_t yscr_block,
                                                                    double2* T) {
  __shared__ double2 Pl[2][B * B];
  const int n = a.n, b = a.b;
  const int s = s_base + blockIdx.y;
  const int tid = threadIdx.x;
  const int k0 = blockIdx.x * kSetupThreads;
  const int k = k0 + tid;
  const bool live = k < n;
  double2* Y = yscr + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * yscr_block;  // [n][B][256]
  const double2* Ps = a.P + (size_t)s * n * B * B;
  const double2 z = make_double2(0.0, 0.0);
  __shared__ double2 R2[B];  // local-layer 1/s2 (moving PML), zero in the padded rows
  if (tid < B) R2[tid] = tid < b ? a.tab_k[4 * tid] : z;
  // right-hand side rows: the last layer (H_m), or every layer (H_F: independent layers)
  auto rhs_row = [&](int l) { return s == 0 ? l < b : l == b - 1; };

  double2 y[B];  // y_i in the forward pass, then x_i in the backward pass
  ufor<0, B>([&](auto lc) { y[decltype(lc)::value] = z; });
  // ---- forward, from the block's first RHS column on (rows above it are zero) ----
  for (int i = k0; i < n; ++i) {
    double2* pl = Pl[i & 1];
    for (int q = tid; q < B * B; q += kSetupThreads) pl[q] = Ps[(size_t)i * B * B + q];
    __syncthreads();
    const double2 AW = a.tab_i[i];
    double2 t[B];
    ufor<0, B>([&](auto lc) {
      constexpr int l = decltype(lc)::value;
      t[l] = cneg(cmul(cmul(AW, R2[l]), y[l]));
      if (i == k && rhs_row(l)) t[l].x += 1.0;
    });
    double2* Yi = Y + (size_t)i * B * kSetupThreads + tid;
    ufor<0, B>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      double2 acc = z;
      ufor<0, B>([&](auto lc) {
        constexpr int l = decltype(lc)::value;
        acc = cfma(pl[j * B + l], t[l], acc);
      });
      y[j] = acc;
      Yi[(size_t)j * kSetupThreads] = acc;
    });
  }
  // ---- backward: x_{n-1} = y_{n-1}; x_i = y_i - P_i (U_i x_{i+1}) ----
  // T_m (matrix b + s - 1) keeps the last layer; H_F (s = 0) keeps every layer l < b
  // (matrix l = A_ll^-1).
  for (int i = n - 1; i >= 0; --i) {
    if (i < n - 1) {
      double2* pl = Pl[i & 1];
      for (int q = tid; q < B * B; q += kSetupThreads) pl[q] = Ps[(size_t)i * B * B + q];
      __syncthreads();
      const double2 AE = a.tab_i[n + i];
      double2 t[B];
      ufor<0, B>([&](auto lc) {
        constexpr int l = decltype(lc)::value;
        t[l] = cmul(cmul(AE, R2[l]), y[l]);
      });
      const bool below = i < k0;  // uniform: y_i = 0 for every column of this block
      const double2* Yi = Y + (size_t)i * B * kSetupThreads + tid;
      ufor<0, B>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        double2 acc = z;
        ufor<0, B>([&](auto lc) {
          constexpr int l = decltype(lc)::value;
          acc = cfma(pl[j * B + l], t[l], acc);
        });
        const double2 yi = below ? z : Yi[(size_t)j * kSetupThreads];
        y[j] = csub(yi, acc);
      });
    }
    if (live) {
      ufor<0, B>([&](auto lc) {
        constexpr int l = decltype(lc)::value;
        if (s == 0) {
          if (l < b) T[((size_t)l * n + i) * n + k] = y[l];
        } else if (l == b - 1) {
          T[((size_t)(b + s - 1) * n + i) * n + k] = y[l];
        }
      });
    }
  }
}

// ------------------------------------------------------------------------------- apply
// One dense GEMV t = T_mat x (n x n, row-major) with the fused sweep epilogue; four rows per
// 256-thread block (one wave per row), x staged in LDS (optionally scaled by in_c * R1[k]).
// blockIdx.y batches independent GEMVs (the b layers of F0), stepping mat / in / out by one.
struct GemvStep {
  const double2* T;       // matrix 0; matrix (mat + y) is used
  int mat;
  const double2* in;      // x = in (+ y n)
  int in_scaled;          // x_k *= in_c * R1[k]
  double2 in_c;
  double2* out;           // out (+ y n)[i] = a_old out + a_in in_raw[i] + a_t t
  double a_old, a_in, a_t;
  double2* unext;         // if set (and y == next_y): unext[i] = rnext[i] - (S_c R1[i]) t
  const double2* rnext;
  double2 S_c;
  int next_y;
};

template <int J>
__global__ __launch_bounds__(256) void dense_gemv_kernel(const GemvStep g, const int n,
                                                         const double2* R1, const int* stop) {
  if (stop && *stop) return;
  __shared__ double2 xs[J * 64];
  const int y = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int i = min(blockIdx.x * 4 + (threadIdx.x >> 6), n - 1);  // rows past n: clamped, unused
  // the matrix row does not depend on x: its loads go out first (unconditional, clamped
  // columns, masked at use: xs is 0 there) and stream while x is staged in LDS
  const double2* Trow = g.T + ((size_t)(g.mat + y) * n + i) * n;
  double2 tv[J];
  ufor<0, J>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const int k = min(lane + 64 * j, n - 1);
    tv[j] = make_double2(__builtin_nontemporal_load(&Trow[k].x), __builtin_nontemporal_load(&Trow[k].y));
  });
  const double2* in = g.in + (size_t)y * n;
  for (int k = threadIdx.x; k < J * 64; k += 256) {
    double2 v = make_double2(0.0, 0.0);
    if (k < n) {
      v = in[k];
      if (g.in_scaled) v = cmul(v, cmul(g.in_c, R1[k]));
    }
    xs[k] = v;
  }
  __syncthreads();
  if (blockIdx.x * 4 + (threadIdx.x >> 6) >= n) return;
  double2 acc = make_double2(0.0, 0.0);
  ufor<0, J>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    acc = cfma(tv[j], xs[lane + 64 * j], acc);
  });
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    acc.x += __shfl_xor(acc.x, off);
    acc.y += __shfl_xor(acc.y, off);
  }
  if (lane == 0) {
    double2* out = g.out + (size_t)y * n;
    double2 o = cscale(acc, g.a_t);
    if (g.a_in != 0.0) o = cadd(o, cscale(g.in[(size_t)y * n + i], g.a_in));
    if (g.a_old != 0.0) o = cadd(o, cscale(out[i], g.a_old));
    out[i] = o;
    if (g.unext && y == g.next_y) g.unext[i] = csub(g.rnext[i], cmul(cmul(g.S_c, R1[i]), acc));
  }
}

void launch_gemv(const GemvStep& g, int batch, int n, const double2* R1, const int* stop,
                 hipStream_t st) {
  const dim3 grid((n + 3) / 4, batch);
  if (n <= 512)
    hipLaunchKernelGGL(dense_gemv_kernel<8>, grid, dim3(256), 0, st, g, n, R1, stop);
  else if (n <= 1024)
    hipLaunchKernelGGL(dense_gemv_kernel<16>, grid, dim3(256), 0, st, g, n, R1, stop);
  else
    hipLaunchKernelGGL(dense_gemv_kernel<32>, grid, dim3(256), 0, st, g, n, R1, stop);
}

template <int B>
void launch_setup_t(const SweepArgs& a, int s_base, int batch, double2* yscr, size_t yscr_block,
                    double2* T, hipStream_t st) {
  const dim3 grid((a.n + kSetupThreads - 1) / kSetupThreads, batch);
  hipLaunchKernelGGL((dense_setup_kernel<B>), grid, dim3(kSetupThreads), 0, st, a, s_base, yscr,
                     yscr_block, T);
}

}  // namespace

size_t sweep_dense_bytes(int n) { return (size_t)n * n * n * sizeof(double2); }

size_t sweep_dense_scratch_per_block(int n, int b) {
  return (size_t)n * sweep_block(b) * kSetupThreads;  // double2 elements
}
int sweep_dense_chunks(int n) { return (n + kSetupThreads - 1) / kSetupThreads; }

void launch_sweep_dense_setup(const SweepArgs& a, int s_base, int batch, double2* yscr,
                              double2* T, hipStream_t st) {
  const size_t yb = sweep_dense_scratch_per_block(a.n, a.b);
  switch (sweep_block(a.b)) {
    case 4: launch_setup_t<4>(a, s_base, batch, yscr, yb, T, st); break;
    case 8: launch_setup_t<8>(a, s_base, batch, yscr, yb, T, st); break;
    case 12: launch_setup_t<12>(a, s_base, batch, yscr, yb, T, st); break;
    case 16: launch_setup_t<16>(a, s_base, batch, yscr, yb, T, st); break;
    default: break;
  }
}

void launch_sweep_dense_apply(const SweepArgs& a, const double2* T, const double2* r, double2* w,
                              double2* u, int asis, hipStream_t st) {
  const int n = a.n, b = a.b;
  const size_t N = n;
  const double2* R1 = a.tab_i + 2 * n;
  auto BS = [&](int layer) { return a.tab_glob[4 * layer + 1]; };  // c3 of a global layer
  auto BN = [&](int layer) { return a.tab_glob[4 * layer + 2]; };  // c4 of a global layer
  const double t_sign = asis ? -1.0 : 1.0, in_w = asis ? 1.0 : 0.0;
  // F0: w_l = A_ll^-1 r_l (l < b); u_b = r_b - S_b w_{b-1}
  {
    GemvStep g{};
    g.T = T; g.mat = 0; g.in = r; g.out = w;
    g.a_old = 0.0; g.a_in = 0.0; g.a_t = 1.0;
    g.unext = u + (size_t)b * N; g.rnext = r + (size_t)b * N; g.S_c = BS(b); g.next_y = b - 1;
    launch_gemv(g, b, n, R1, a.stop, st);
  }
  // FWD (m = b+1 .. n-1, 1-based) fused with the middle sweep; MID for m = n
  for (int m = b + 1; m <= n; ++m) {
    GemvStep g{};
    g.T = T; g.mat = m - 1;                    // matrix b + s - 1, s = m - b
    g.in = u + (size_t)(m - 1) * N;            // u_{m-1} (0-based layer m-1)
    g.out = w + (size_t)(m - 1) * N;
    g.a_old = 0.0; g.a_in = in_w; g.a_t = t_sign;
    if (m < n) {
      g.unext = u + (size_t)m * N; g.rnext = r + (size_t)m * N; g.S_c = BS(m); g.next_y = 0;
    }
    launch_gemv(g, 1, n, R1, a.stop, st);
  }
  // BWD (m = n-1 .. b+1): w_{m-1} -= T_m (N_{m-1} w_m);  FC: w_{b-1} -= A_bb^-1 (N_{b-1} w_b)
  for (int m = n - 1; m >= b; --m) {
    GemvStep g{};
    g.T = T; g.mat = m - 1;                    // m == b: matrix b - 1 = A_bb^-1 of H_F
    g.in = w + (size_t)m * N; g.in_scaled = 1; g.in_c = BN(m - 1);
    g.out = w + (size_t)(m - 1) * N;
    g.a_old = 1.0; g.a_in = 0.0; g.a_t = -1.0;
    launch_gemv(g, 1, n, R1, a.stop, st);
  }
}

}  // namespace hh
