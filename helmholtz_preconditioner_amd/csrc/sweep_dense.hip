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
#include "hh_wave.hpp"
#include "sweep.hpp"
#include "hh_error.hpp"

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
        acc = cfma(pl[pidx<B>(j, l)], t[l], acc);
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
          acc = cfma(pl[pidx<B>(j, l)], t[l], acc);
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
  acc.x = wave_sum_to_63(acc.x);
  acc.y = wave_sum_to_63(acc.y);
  if (lane == 63) {
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

// ---------------------------------------------------------------- persistent apply chain
// The FWD+MID and BWD sweeps as ONE cooperative launch (2 (n - b) dependent GEMVs) instead of
// one launch per GEMV: a launch boundary costs about as much as streaming a whole matrix.
// Workgroup w owns rows 4w .. 4w+3 of every GEMV (one compute wave per row, the same lane
// partition, FMA order and DPP reduction as dense_gemv_kernel: bit-identical results); four
// loader waves stream the NEXT step's matrix rows into the other LDS slot while the compute
// waves wait for the current input.  Step s's outputs are handed to every workgroup as tagged
// 8-byte granules {tag, 32-bit half} (MI355X_MICROARCH.md: the data is the flag -- no counter,
// no fence); the tag carries the launch's sequence number and the step.  Two workgroup barriers
// per step: A(s) -- slot s loaded, input s staged; B(s) -- every compute wave done with input s
// (so the next input may overwrite it).  Every wait is bounded: on timeout the timeout word is
// set and the grid drains.
constexpr int kChainRows = 4;       // rows (compute waves) per workgroup
// + two groups of loader waves (group g loads the steps of parity g, two steps ahead)
constexpr int kChainThreads = 3 * kChainRows * 64;
constexpr unsigned kChainSpin = 1u << 22;

// by-value select (a select of two lvalues would become a select of addresses: flat accesses)
__device__ __forceinline__ double2 csel2(bool c, double2 a, double2 b) {
  return make_double2(c ? a.x : b.x, c ? a.y : b.y);
}

__device__ __forceinline__ unsigned chain_tag(unsigned seq, int step) {
  return (seq << 12) | ((unsigned)step & 0xfffu);
}

template <int J>
__global__ __launch_bounds__(kChainThreads) void sweep_chain_kernel(const ChainArgs a) {
  if (a.stop && *a.stop) return;
  constexpr int PAD = 64 * J;  // padded row length (n <= PAD)
  constexpr int PER = PAD / (kChainRows * 64);  // input elements per compute thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double2* slots = reinterpret_cast<double2*>(smem);  // [2][kChainRows][PAD]
  double2* xs = slots + 2 * kChainRows * PAD;         // [PAD]
  using gu64 = __attribute__((address_space(1))) unsigned long long;
  const int n = a.n, b = a.b, S = 2 * (n - b);
  const int t = threadIdx.x;
  const bool loader = t >= kChainRows * 64;
  const int lgrp = loader ? (t - kChainRows * 64) / (kChainRows * 64) : 0;  // loader group
  const int lt = (t - kChainRows * 64) % (kChainRows * 64);                // index in group
  const int wv = t >> 6, lane = t & 63;
  const int row0 = blockIdx.x * kChainRows;
  const double2 z = make_double2(0.0, 0.0);
  auto mat_of = [&](int s) { return s < n - b ? b + s : n - 2 - (s - (n - b)); };

  // loader: this step's matrix rows -> registers (issued together), then -> LDS slot
  double2 lv[PER * 4];
  auto load_rows = [&](int s) {
    if (a.diag == 1 || a.diag == 3) return;
    const double2* Tm = a.T + (size_t)mat_of(s) * n * n;
#pragma unroll
    for (int q = 0; q < PER * 4; ++q) {
      const int e = lt + kChainRows * 64 * q;
      const int r = e / PAD, k = e % PAD;
      const double2* p = Tm + (size_t)min(row0 + r, n - 1) * n + min(k, n - 1);
      lv[q] = make_double2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
    }
  };
  auto store_rows = [&](int s) {
    if (a.diag == 1 || a.diag == 3) return;
    double2* sl = slots + (size_t)(s & 1) * kChainRows * PAD;
#pragma unroll
    for (int q = 0; q < PER * 4; ++q) sl[lt + kChainRows * 64 * q] = lv[q];
  };
  // loader group g owns the steps of parity g: step s's rows are requested two steps ahead (at
  // B(s-3)), stored into slot s & 1 at B(s-1) and read after A(s) -- two steps of load latency
  // hidden, 2 x 64 KB per CU in flight
  if (loader) {
    if (lgrp == 0) {
      load_rows(0);
      store_rows(0);
      if (S > 2) load_rows(2);
    } else if (S > 1) {
      load_rows(1);
    }
  }
  // compute threads: R1 of this thread's input elements (the backward sweep's scaling)
  double2 r1v[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) r1v[q] = a.R1[min(t + kChainRows * 64 * q, n - 1)];
  // compute threads: step 0's input u_b was written by the F0 launch before this one
  if (!loader) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + kChainRows * 64 * q;
      xs[e] = csel2(e < n, a.u[(size_t)b * n + min(e, n - 1)], z);
    }
  }
  // The two roles run their own loops (disjoint register live ranges) through the same
  // barrier sequence per step: A(s), B(s), S1(s) (not after the last step).  The barriers
  // are bare s_barrier after the wave's LDS operations (no memory fence: a workgroup fence would
  // make every wave wait for its outstanding global loads -- the loader's two-steps-ahead
  // matrix rows -- at every barrier); the abort decision travels through an LDS word.
  auto bar = [] {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
  __shared__ int abort_word;  // (accessed directly: a pointer to it would be a flat pointer)
  if (t == 0) abort_word = 0;
  __syncthreads();
  bool ok = true;
  if (loader) {
    for (int s = 0; s < S; ++s) {
      bar();  // A(s)
      if (__builtin_nontemporal_load(&abort_word)) break;
      bar();  // B(s)
      if (s + 1 >= S) break;
      if (((s + 1) & 1) == lgrp) {
        store_rows(s + 1);
        if (s + 3 < S) load_rows(s + 3);
      }
      bar();  // S1(s)
    }
  } else {
    const int i = row0 + wv;
    const int ic = min(i, n - 1);
    const double2 R1i = a.R1[ic];
    // the epilogue's operands of a step (independent of the chain): requested one step ahead
    // (valid addresses always, selected by value)
    auto epi_ops = [&](int s, double2& r_i, double2& BSm, double2& w_old) {
      const bool bw = s >= n - b;
      const int mm = bw ? n - 1 - (s - (n - b)) : b + 1 + s;
      const int mc = min(mm, n - 1);
      r_i = csel2(!bw && mm < n, a.r[(size_t)mc * n + ic], z);
      BSm = csel2(!bw && mm < n, a.tab_glob[4 * mc + 1], z);
      w_old = csel2(bw, a.w[(size_t)(mm - 1) * n + ic], z);
    };
    double2 r_i, BSm, w_old;
    epi_ops(0, r_i, BSm, w_old);
    for (int s = 0; s < S; ++s) {
      if (!ok) abort_word = 1;
      bar();  // A(s)
      if (__builtin_nontemporal_load(&abort_word)) break;
      const bool bwd = s >= n - b;
      const int m = bwd ? n - 1 - (s - (n - b)) : b + 1 + s;  // 1-based sweep index of the step
      const double2* sl = slots + ((size_t)(s & 1) * kChainRows + wv) * PAD;
      double2 acc = z;
#pragma unroll 4
      for (int j = 0; j < J; ++j) acc = cfma(sl[lane + 64 * j], xs[lane + 64 * j], acc);
      acc.x = wave_sum_to_63(acc.x);
      acc.y = wave_sum_to_63(acc.y);
      if (lane == 63 && i < n) {
        double2 o, next;
        if (!bwd) {  // FWD (m < n) / MID (m == n): w_{m-1} = t | u_{m-1} - t
          o = cscale(acc, a.t_sign);
          if (a.a_in != 0.0) o = cadd(o, cscale(xs[i], a.a_in));
          a.w[(size_t)(m - 1) * n + i] = o;
          if (m < n) {  // u_m = r_m - S_m t
            next = csub(r_i, cmul(cmul(BSm, R1i), acc));
            a.u[(size_t)m * n + i] = next;
          } else {
            next = o;  // the backward sweep starts from w_{n-1}
          }
        } else {  // BWD: w_{m-1} -= T_m (N_{m-1} w_m)
          o = cadd(cscale(acc, -1.0), cscale(w_old, 1.0));
          a.w[(size_t)(m - 1) * n + i] = o;
          next = o;
        }
        if (s + 1 < S) {
          const unsigned tg = chain_tag(a.seq, s + 1);
          unsigned long long* gp = a.gbuf + ((size_t)((s + 1) & 1) * PAD + i) * 4;
          const unsigned long long hx = (unsigned long long)__double_as_longlong(next.x);
          const unsigned long long hy = (unsigned long long)__double_as_longlong(next.y);
          const unsigned long long tt = (unsigned long long)tg << 32;
          __hip_atomic_store((gu64*)gp, tt | (hx >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store((gu64*)(gp + 1), tt | (hx & 0xffffffffull), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store((gu64*)(gp + 2), tt | (hy >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store((gu64*)(gp + 3), tt | (hy & 0xffffffffull), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      bar();  // B(s): input s no longer read
      if (s + 1 >= S) break;
      // (w_old of a BWD step: written by this very lane in an earlier FWD step)
      epi_ops(s + 1, r_i, BSm, w_old);
      // input of step s+1 (BWD: scaled N R1): every row's granules, in flight together, polled
      // until all carry the step's tag
      const bool nb = s + 1 >= n - b;
      const int mn = nb ? n - 1 - (s + 1 - (n - b)) : 1;
      const double2 inc = a.tab_glob[4 * (mn - 1) + 2];
      const unsigned tg = chain_tag(a.seq, s + 1);
      const unsigned long long* gb = a.gbuf + (size_t)((s + 1) & 1) * PAD * 4;
      unsigned spins = 0;
      // S1(s): the input polls start after the loader has issued its next rows (measured: 10.0
      // vs 14.8 ms per n = 1023 apply without this barrier -- polls issued first, then stuck
      // behind the rows in the CU's memory queue, repeat)
      bar();
      unsigned long long v[PER][4];
      for (;;) {
        if (a.diag >= 3) {  // (diagnostic: no input read at all)
#pragma unroll
          for (int q = 0; q < PER; ++q)
#pragma unroll
            for (int h = 0; h < 4; ++h) v[q][h] = 0;
          break;
        }
        bool all = true;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
          const int e = min(t + kChainRows * 64 * q, n - 1);
          const unsigned long long* gp = gb + (size_t)e * 4;
#pragma unroll
          for (int h = 0; h < 4; ++h)
            v[q][h] = __hip_atomic_load((gu64*)(gp + h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int q = 0; q < PER; ++q)
#pragma unroll
          for (int h = 0; h < 4; ++h) all = all && (unsigned)(v[q][h] >> 32) == tg;
        if (all || !ok || a.diag == 2) break;
        if (++spins > kChainSpin) {
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int e = t + kChainRows * 64 * q;
        double2 x = make_double2(
            __longlong_as_double((long long)((v[q][0] << 32) | (v[q][1] & 0xffffffffull))),
            __longlong_as_double((long long)((v[q][2] << 32) | (v[q][3] & 0xffffffffull))));
        if (nb) x = cmul(x, cmul(inc, r1v[q]));
        xs[e] = csel2(e < n, x, z);
      }
    }
  }
  if (!ok && t == 0)
    __hip_atomic_store((__attribute__((address_space(1))) unsigned*)a.timeout, 1u,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

bool sweep_chain_fits(int n, int device_cus) {
  return n >= 2 && n <= 1024 && (n + kChainRows - 1) / kChainRows <= device_cus;
}
size_t sweep_chain_granules() { return 2 * 1024 * 4; }

template <int J>
void launch_chain_t(const ChainArgs& c, hipStream_t st) {
  constexpr int PAD = 64 * J;
  const size_t lds = (2 * kChainRows + 1) * (size_t)PAD * sizeof(double2);
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&sweep_chain_kernel<J>),
      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) {
    (void)hipGetLastError();
    fail(HH_ERR_HIP, "sweep chain: cannot enable %zu B of dynamic LDS (%s)", lds,
         hipGetErrorString(attr));
  }
  ChainArgs arg = c;
  void* params[] = {&arg};
  const dim3 grid((c.n + kChainRows - 1) / kChainRows), block(kChainThreads);
  // cooperative: the launch fails instead of hanging if the grid cannot be co-resident
  // (HH_SWEEP_COOP=0: a plain launch; the chain's waits are bounded either way)
  const void* fn = reinterpret_cast<const void*>(&sweep_chain_kernel<J>);
  const hipError_t e = sweep_coop_launch()
                           ? hipLaunchCooperativeKernel(fn, grid, block, params, (unsigned)lds, st)
                           : hipLaunchKernel(fn, grid, block, params, lds, st);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    fail(HH_ERR_HIP, "sweep chain: launch of %u workgroups failed (%s)", grid.x,
         hipGetErrorString(e));
  }
}

void launch_sweep_dense_apply(const SweepArgs& a, const double2* T, const double2* r, double2* w,
                              double2* u, int asis, hipStream_t st, const ChainArgs* chain) {
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
  if (chain) {  // FWD + MID + BWD as one persistent launch
    ChainArgs c = *chain;
    c.T = T;
    c.n = n;
    c.b = b;
    c.R1 = R1;
    c.tab_glob = a.tab_glob;
    c.r = r;
    c.u = u;
    c.w = w;
    c.a_in = in_w;
    c.t_sign = t_sign;
    c.stop = a.stop;
    if (n <= 512) launch_chain_t<8>(c, st);
    else launch_chain_t<16>(c, st);
    return;
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
