// Krylov (GMRES) kernels for gfx950: fused multi-dot projection, fused update + norm,
// solution update, fixed-order reductions and the single-wave Hessenberg/Givens step.
//
// Replaces the per-iteration Python/OpenBLAS work of scipy.sparse.linalg.gmres
// (scipy 1.15.3 _isolve/iterative.py:748-800) that code.py:516 runs:
//   MGS loop np.vdot / axpy over N-vectors  -> one multidot pass + one update pass (CGS),
//   np.linalg.norm(w) (h0, h1)               -> fused into those passes,
//   lartg + rotation of the Hessenberg column-> gmres_column_kernel (one lane),
//   triangular solve, x += y @ v             -> gmres_solve_kernel + xupdate.
// Every reduction is two-level and fixed-order (wave butterfly -> LDS -> per-block partial ->
// one block per output summing partials in index order), so results are reproducible
// run to run and identical on every rank after the RCCL allreduce.
#include <algorithm>
#include <cstdlib>

#include "hh_internal.hpp"
#include "hh_complex.hpp"
#include "hh_wave.hpp"
#include "hh_givens.hpp"

namespace hh {
namespace {
using namespace givens;

constexpr int kT = 256;  // threads per streaming block

template <bool NT>
__device__ __forceinline__ double2 ldnt(const double2* p) {
  if constexpr (NT) {
    return make_double2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
  } else {
    return *p;
  }
}

using gu64k = __attribute__((address_space(1))) unsigned long long;
using gu32k = __attribute__((address_space(1))) unsigned;


template <bool SC1 = false>
__device__ double wave_reduce_like_block(const double* partials, int count, int width);
__device__ void column_from_sums(const GivensState& g, int col, const double* rd, double rn0,
                                 double eps, double ptol, int stop_col);

// Last-block hand-off of a streaming kernel (single rank): every block has stored its partials;
// it releases them (device-scope fence) and takes a ticket; the block holding the last ticket
// acquires and does what the next, one-block kernel would have done -- one launch boundary
// and one kernel start fewer per GMRES iteration.  The ticket counter is re-armed by that block.
// The ticket is an agent-scope acq_rel RMW behind a workgroup barrier: the release publishes
// every wave's partial stores (the barrier orders them before thread 0's release), the acquire
// makes the last block see all of them -- a guarantee of the memory model, not an assumption
// about the multi-XCD hardware (HH_KRYLOV_FUSE only; no default path uses these kernels).
__device__ __forceinline__ bool last_block(unsigned* counter) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 partial stores landed
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add((gu32k*)counter, 1u, __ATOMIC_ACQ_REL,
                                  __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  return last;
}

// partials[blk][2K+2]: [2k, 2k+1] = sum_p conj(V_k[p]) w[p];  [2K] = sum |w|^2.
// FUSED: the last block also reduces the `cols` columns over all blocks into `out`, each column
// by one wave in reduce_kernel's exact order (bit-identical to the separate reduce launch).
template <int K, bool NT, bool FUSED>
__global__ __launch_bounds__(kT) void multidot_kernel(const double2* __restrict__ V, size_t ldv,
                                                      const double2* __restrict__ w, size_t len,
                                                      double* __restrict__ partials,
                                                      const int* stop, double* out, int cols,
                                                      unsigned* counter) {
  if (stop && *stop) return;
  double2 acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = make_double2(0.0, 0.0);
  double nrm = 0.0;
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t p = (size_t)blockIdx.x * kT + threadIdx.x; p < len; p += stride) {
    const double2 wv = w[p];
    nrm = fma(wv.x, wv.x, fma(wv.y, wv.y, nrm));
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = cfma_conj(ldnt<NT>(V + (size_t)k * ldv + p), wv, acc[k]);
  }
  double v[2 * K + 1];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    v[2 * k] = acc[k].x;
    v[2 * k + 1] = acc[k].y;
  }
  v[2 * K] = nrm;
  block_reduce_vec<2 * K + 1, FUSED>(v, partials, 2 * K + 2);
  if constexpr (FUSED) {
    if (last_block(counter)) {
      const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
      for (int c = wave; c < cols; c += kT / kWave) {
        const double r = wave_reduce_like_block<true>(partials + c, gridDim.x, 2 * K + 2);
        if (lane == 0) out[c] = r;
      }
      if (threadIdx.x == 0) *counter = 0u;
    }
  }
}

// w_out = w - sum_k (s_k * (s_k * raw_k)) V_k; partials[blk][kMaxNorms]: [0] = |w_out|^2.
// REV: the grid sweeps the vectors back to front.  The multidot before it swept them front to
// back, so on a basis that (partly) fits the 256 MB Infinity Cache the update starts on the
// lines the multidot left there last (and leaves the heads hot for the next multidot); each
// element's arithmetic is unchanged, only the norm partials add in the reverse order.
// FUSED (single rank): the last block also folds the norm partials and completes the Hessenberg
// column (gmres_column_kernel's work, bit-identical), one launch fewer per iteration.
struct ColumnFuse {
  GivensState g;
  int col, stop_col;
  const double* rd;
  double eps, ptol;
  unsigned* counter;
};
template <int K, bool NT, bool REV, bool FUSED>
__global__ __launch_bounds__(kT) void update_kernel(const double2* __restrict__ V, size_t ldv,
                                                    const double* __restrict__ raw,
                                                    const double* __restrict__ scale,
                                                    const double2* w, double2* w_out, size_t len,
                                                    double* __restrict__ partials,
                                                    const int* stop, const ColumnFuse cf) {
  if (stop && *stop) return;
  double2 coef[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double s = scale[k];
    const double2 hk = cscale(make_double2(raw[2 * k], raw[2 * k + 1]), s);  // H[col][k]
    coef[k] = cscale(hk, s);                                                    // h_k * s_k
  }
  double nrm = 0.0;
  const size_t stride = (size_t)gridDim.x * kT;
  const size_t p0 = (size_t)blockIdx.x * kT + threadIdx.x;
  auto point = [&](size_t p) {
    double2 wv = w[p];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double2 vk = ldnt<NT>(V + (size_t)k * ldv + p);
      wv = csub(wv, cmul(coef[k], vk));
    }
    w_out[p] = wv;
    nrm = fma(wv.x, wv.x, fma(wv.y, wv.y, nrm));
  };
  if constexpr (REV) {
    const size_t steps = (len + stride - 1) / stride;
    for (size_t i = steps; i-- > 0;) {
      const size_t p = i * stride + p0;
      if (p < len) point(p);
    }
  } else {
    // (the plain forward loop: the REV loop's form measured 4-8 % slower here for K >= 13)
    for (size_t p = p0; p < len; p += stride) point(p);
  }
  double v[1] = {nrm};
  block_reduce_vec<1, FUSED>(v, partials, kMaxNorms);
  if constexpr (FUSED) {
    if (last_block(cf.counter)) {
      if (threadIdx.x < kWave) {
        const double rn0 = wave_reduce_like_block<true>(partials, gridDim.x, kMaxNorms);
        column_from_sums(cf.g, cf.col, cf.rd, rlane(rn0, 0), cf.eps, cf.ptol, cf.stop_col);
      }
      if (threadIdx.x == 0) *cf.counter = 0u;
    }
  }
}

// x += sum_k y_k V_k (NT: the basis is dead after this pass; non-temporal loads at 4096^2).
// ctl (the cycle's control words, nullable): ctl[2] != 0 skips the update (the merged cycle end
// already applied it); otherwise only the ctl[1] + 1 vectors of the executed columns are read
// (a block-uniform bound: the vectors past an early stop may never have been written, and
// since round 6 they are not loaded at all -- ADVICE r05: the re-reads of the last counted
// vector with coefficient 0 cost up to K / kc times the bytes under NT loads), so the update of
// a cycle that stopped early needs no host round trip for its length.  Full cycles: kc == K.
template <int K, bool NT>
__global__ __launch_bounds__(kT) void xupdate_kernel(const double2* __restrict__ V, size_t ldv,
                                                     const double2* __restrict__ y,
                                                     double2* __restrict__ x, size_t len,
                                                     const int* ctl) {
  int kc = K;
  if (ctl) {
    if (ctl[2]) return;
    kc = __builtin_amdgcn_readfirstlane(min(max(ctl[1] + 1, 1), K));  // (uniform)
  }
  double2 c[K];
#pragma unroll
  for (int k = 0; k < K; ++k) c[k] = k < kc ? y[k] : make_double2(0.0, 0.0);
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t p = (size_t)blockIdx.x * kT + threadIdx.x; p < len; p += stride) {
    double2 t = make_double2(0.0, 0.0);
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < kc) t = cfma(c[k], ldnt<NT>(V + (size_t)k * ldv + p), t);
    x[p] = cadd(x[p], t);
  }
}

// One block per output column: out[k] = sum_b partials[b*width + k] in fixed order: each thread
// its b = t, t + 256, ... in ascending order (the loads of 8 of them issued together), then the
// pairwise tree sh[t] += sh[t + off], off = 128 .. 1 -- its last six levels by wave shuffles in the
// same operand order (two block barriers instead of eight; wave_reduce_like_block emulates it).
__global__ __launch_bounds__(kT) void reduce_kernel(const double* __restrict__ partials, int count,
                                                    int width, double* __restrict__ out,
                                                    const int* stop) {
  if (stop && *stop) return;
  __shared__ double sh[kT];
  const int k = blockIdx.x;
  const int t = threadIdx.x;
  constexpr int kChunk = 8;
  double s = 0.0;
  for (int b0 = t; b0 < count; b0 += kChunk * kT) {
    double v[kChunk];
#pragma unroll
    for (int i = 0; i < kChunk; ++i)
      v[i] = partials[(size_t)min(b0 + i * kT, count - 1) * width + k];
#pragma unroll
    for (int i = 0; i < kChunk; ++i)
      if (b0 + i * kT < count) s += v[i];
  }
  sh[t] = s;
  __syncthreads();
  if (t < kT / 2) sh[t] += sh[t + kT / 2];
  __syncthreads();
  if (t < kWave) {
    double x = sh[t] + sh[t + kWave];  // (off = 64)
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) x += __shfl_down(x, off);
    if (t == 0) out[k] = x;
  }
}

__global__ void add_small_kernel(const double* in, double* out, int count, const int* stop) {
  if (stop && *stop) return;
  for (int k = threadIdx.x; k < count; k += blockDim.x) out[k] += in[k];
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kT) void fill_hash_kernel(double2* v, size_t len, size_t goff,
                                                       uint64_t seed) {
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t p = (size_t)blockIdx.x * kT + threadIdx.x; p < len; p += stride) {
    const uint64_t g = (uint64_t)(goff + p);
    const uint64_t a = splitmix64(seed ^ (2 * g));
    const uint64_t b = splitmix64(seed ^ (2 * g + 1));
    // 53-bit uniforms in [-1, 1)
    const double re = (double)(a >> 11) * (2.0 / 9007199254740992.0) - 1.0;
    const double im = (double)(b >> 11) * (2.0 / 9007199254740992.0) - 1.0;
    v[p] = make_double2(re, im);
  }
}

__global__ __launch_bounds__(kT) void scale_copy_kernel(const double2* in, double2* out,
                                                        size_t len, double s, const int* stop) {
  if (stop && *stop) return;
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t p = (size_t)blockIdx.x * kT + threadIdx.x; p < len; p += stride)
    out[p] = cscale(in[p], s);
}


// |w|^2 from the update kernel's per-block partials (column 0 of `width`), summed by one
// wave in exactly reduce_kernel's order: the 256 strided partial sums of its threads, then its
// LDS tree (steps 128 and 64 inside each lane's four sums, 32 .. 1 by shuffles).  Every lane
// returns; lane 0's value is the result, bit-identical to reduce_kernel's out[0].
template <bool SC1>
__device__ double wave_reduce_like_block(const double* partials, int count, int width) {
  static_assert(kT == 4 * kWave, "four strided sums per lane emulate a 256-thread block");
  const int l = threadIdx.x & (kWave - 1);
  // the four strided sums, each in ascending b; the loads of a chunk of 8 x 256 blocks issued
  // together from clamped addresses (one memory latency per chunk: count <= 2048 is one chunk;
  // a load per iteration would wait a round trip each -- 11 us for 1024 partials)
  constexpr int kChunk = 8;
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  for (int b0 = l; b0 < count; b0 += kChunk * kT) {
    double v[4][kChunk];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < kChunk; ++i) {
        const int b = min(b0 + q * kWave + i * kT, count - 1);
        const double* p = partials + (size_t)b * width;
        v[q][i] = SC1 ? __longlong_as_double((long long)__hip_atomic_load(
                            (gu64k*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                      : *p;
      }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < kChunk; ++i)
        if (b0 + q * kWave + i * kT < count) s[q] += v[q][i];
  }
  s[0] += s[2];  // off = 128: threads l and l + 64
  s[1] += s[3];
  s[0] += s[1];  // off = 64
  double x = s[0];
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) x += __shfl_down(x, off);
  return x;
}


// column `col` from the reduced dots rd and |w_new|^2 = rn0 (one wave: entry k on lane k); rd,
// the scales and the finish's operands are loaded together
struct SumsIn {  // a column's reduced dots (entry `lane`), scale and |w|^2, loaded together
  double2 dk;
  double vk, h0sq;
  ColIn in;
};
__device__ __forceinline__ SumsIn load_sums_in(const GivensState& g, int col, const double* rd) {
  const int lane = threadIdx.x & (kWave - 1);
  const int kc = min(lane, col);
  SumsIn s;
  s.dk = make_double2(rd[2 * kc], rd[2 * kc + 1]);
  s.vk = g.vscale[kc];
  s.h0sq = rd[2 * (col + 1)];
  s.in = load_col_in(g, col);
  return s;
}
__device__ void column_from_sums(const GivensState& g, int col, const SumsIn& s, double rn0,
                                 double eps, double ptol, int stop_col) {
  const int lane = threadIdx.x & (kWave - 1);
  const double2 hk = lane <= col ? cscale(s.dk, s.vk) : make_double2(0.0, 0.0);
  const double h0 = sqrt(s.h0sq);
  const double h1 = sqrt(rn0);
  gmres_finish_column(g, col, hk, s.in, h0, h1, 1.0 / h1, eps, ptol, stop_col);
}
__device__ void column_from_sums(const GivensState& g, int col, const double* rd, double rn0,
                                 double eps, double ptol, int stop_col) {
  column_from_sums(g, col, load_sums_in(g, col, rd), rn0, eps, ptol, stop_col);
}

__global__ void gmres_column_kernel(GivensState g, int col, const double* rd, const double* rn,
                                    const double* npart, int ncount, double eps, double ptol,
                                    int stop_col) {
  // the column's operands and the stop flag requested before the norm's partials are summed
  // (one memory latency for all of them)
  const SumsIn s = load_sums_in(g, col, rd);
  const int stopped = g.ctrl[0];
  const double rn0 = npart ? wave_reduce_like_block(npart, ncount, kMaxNorms) : rn[0];
  if (stopped) return;
  // (wave_reduce_like_block leaves the sum in lane 0: broadcast it)
  column_from_sums(g, col, s, npart ? rlane(rn0, 0) : rn0, eps, ptol, stop_col);
}

// every operand loaded up front: one memory latency per launch
__device__ __forceinline__ void lag_body(const GivensState& g, int j, const double* rd,
                                         const double* sig2, int final_step, double eps,
                                         double ptol, int stop_col) {
  const int lane = threadIdx.x & (kWave - 1);
  const LagIn L = lag_load(g, j);
  const double sig = *sig2;
  const int kj = min(lane, j);
  const double* rdp = rd ? rd : sig2;  // (final step: rd unused, any valid words of red)
  const double2 d = make_double2(rdp[2 * kj], rdp[2 * kj + 1]);
  const double w2 = rdp[2 * (j + 1)];
  if (L.stopped) return;
  lag_compute(g, j, L, d, w2, sig, final_step, eps, ptol, stop_col);
}

__global__ void gmres_lag_kernel(GivensState g, int j, const double* rd, const double* sig2,
                                 int final_step, double eps, double ptol, int stop_col) {
  lag_body(g, j, rd, sig2, final_step, eps, ptol, stop_col);
}

// reduce_kernel + gmres_lag_kernel in ONE launch for a single rank (no allreduce between them),
// bit-identical to the two.  reduce_kernel sums column k with 256 threads t (rows t, t + 256,
// ... ascending, then the pairwise tree off = 128 .. 1); here lane c of wave w (8 waves) plays
// those threads t = w + 8 q (q < 32) for column c -- each row read coalesced across the
// columns, 32 loads in flight -- so the tree's levels 128 .. 8 pair two of its own sums (q,
// q + 2^l) and the last three (4, 2, 1) pair waves: wave 0's lane c finishes them from LDS.
// The sums land in `red` and LDS; wave 0 then runs the lag step on the LDS copy, its own
// operands requested before the partial rows (their latencies overlap).  One launch instead of
// two per one-pass inner iteration (~5 us each at 1024^2, where an iteration is ~60 us).
// (16 waves of 16 virtual threads each hold 128 VGPRs at most and spilled -- 10.1 / 14.1 us;
// a first version with reduce_kernel's strided per-column reads ran 13.9 us:
// profiles/r05/r05i_*, r05j_*, r05k_rocprof_c2_kernel_stats.csv.)
constexpr int kLagRedWaves = 8;
constexpr int kLagRedThreads = kLagRedWaves * kWave;
constexpr int kLagRedQ = kT / kLagRedWaves;  // virtual threads per lane
// final_step (the cycle end's norm, cols = 1): the reduced column is the subdiagonal's |w|^2 and
// the lag step only completes column j - 1 (gmres_lag_kernel with final_step, whose rd / w2
// operands that step never reads).
__global__ __launch_bounds__(kLagRedThreads) void gmres_lag_red_kernel(
    GivensState g, int j, const double* partials, int count, int width, int cols, double* red,
    double eps, double ptol, int stop_col, int final_step) {
  __shared__ double wsum[kLagRedWaves][kWave];
  __shared__ double sred[kWave];
  const int w = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  const int c = min(lane, cols - 1);
  // the lag step's own operands (and the stop flag) requested before the partial rows
  LagIn L;
  if (w == 0) L = lag_load(g, j);
  double s[kLagRedQ];
#pragma unroll
  for (int q = 0; q < kLagRedQ; ++q) s[q] = 0.0;
  for (int b0 = 0; b0 < count; b0 += kT) {
    double v[kLagRedQ];
#pragma unroll
    for (int q = 0; q < kLagRedQ; ++q)
      v[q] = partials[(size_t)min(b0 + w + kLagRedWaves * q, count - 1) * width + c];
#pragma unroll
    for (int q = 0; q < kLagRedQ; ++q)
      if (b0 + w + kLagRedWaves * q < count) s[q] += v[q];
  }
#pragma unroll
  for (int h = kLagRedQ / 2; h > 0; h >>= 1)  // tree levels off = 128 .. 8
#pragma unroll
    for (int q = 0; q < h; ++q) s[q] += s[q + h];
  wsum[w][lane] = s[0];
  __syncthreads();
  if (w == 0) {
    double x[kLagRedWaves];
#pragma unroll
    for (int q = 0; q < kLagRedWaves; ++q) x[q] = wsum[q][lane];
#pragma unroll
    for (int h = kLagRedWaves / 2; h > 0; h >>= 1)  // levels 4, 2, 1
#pragma unroll
      for (int q = 0; q < h; ++q) x[q] += x[q + h];
    // (the cycle stopped: reduce_kernel and gmres_lag_kernel leave red and the state alone)
    if (lane < cols && !L.stopped) {
      sred[lane] = x[0];
      red[lane] = x[0];
    }
  }
  __syncthreads();
  if (w == 0 && !L.stopped) {
    if (final_step) {
      lag_compute(g, j, L, make_double2(0.0, 0.0), 0.0, sred[0], 1, eps, ptol, stop_col);
    } else {
      const int kj = min(lane, j);
      lag_compute(g, j, L, make_double2(sred[2 * kj], sred[2 * kj + 1]), sred[2 * (j + 1)],
                  sred[2 * (j + 1) + 1], 0, eps, ptol, stop_col);
    }
  }
}

__global__ void gmres_start_kernel(GivensState g, const double* red, int idx_r, int idx_m) {
  if (threadIdx.x != 0) return;
  g.ctrl[0] = 0;
  g.ctrl[1] = -1;
  const double rn = sqrt(red[idx_r]);
  const double mn = sqrt(red[idx_m]);
  for (int k = 0; k <= g.restart; ++k) g.S[k] = make_double2(0.0, 0.0);
  g.S[0] = make_double2(mn, 0.0);
  g.vscale[0] = 1.0 / mn;
  g.sscale[0] = 1.0 / mn;
  g.status[4] = rn;
  g.status[5] = mn;
}

// The triangular solve, one wave, lane m holding y_m: H copied to LDS by the whole wave (one
// memory latency), the Smith factors of every diagonal formed at once, then the column-oriented
// back-substitution -- y_k /= R_kk by lane k, broadcast, lanes m < k take y_m -= y_k R_mk -- the
// same operations in the same order per y_m as the serial form (lane 0 alone, global operands:
// a dependent round trip per operand, both divisions of every step on the chain).
// The column comes from the device (ctl[1], the last one the cycle executed; the host learns it
// only from the cycle's report, read after the residual): with `merged`, a cycle that reached
// its last column `stop_col` already had its x update from cycle_end_kernel + cycle_finish_kernel
// -- the solve then only raises ctl[2], which skips xupdate_kernel.
__global__ void gmres_solve_kernel(GivensState g, int stop_col, int merged) {
  __shared__ double2 sH[(kMaxProj + 1) * (kMaxProj + 2)];
  const int col = min(max(g.ctrl[1], 0), stop_col);
  const bool skip = merged && col == stop_col;
  if (threadIdx.x == 0) g.ctrl[2] = skip;
  if (skip) return;
  const int R1 = g.restart + 1;
  for (int e = threadIdx.x; e < (col + 1) * R1; e += kWave) sH[e] = g.H[e];
  __syncthreads();
  solve_columns_wave(g, col, sH);
}

// Krylov tuning knobs (hh_tune_krylov): non-temporal basis loads, streaming grid size;
// -1 / 0 = by vector length.  Measured (GMRES(20) it/s, profiles/r01_tune_krylov.log and
// r01z3_tune_krylov_{1024,128}.log): at 4096^2 NT loads +7.7 % and 1024 blocks best; at
// 1024^2 (a 21-vector basis of 352 MB, partly served by the 256 MB Infinity Cache) cached
// loads +3 % and 512 blocks another +2 %; at 128^2 every setting within 1 % (launch-bound).
int g_krylov_nt = -1;
int g_krylov_blocks = 0;
constexpr size_t kSmallKrylovLen = (size_t)2 << 20;  // rank-local unknowns

bool krylov_nt(size_t len) { return g_krylov_nt < 0 ? len > kSmallKrylovLen : g_krylov_nt != 0; }
// back-to-front update sweeps with cached loads (HH_KRYLOV_REV=0 turns them off: diagnostic)
bool krylov_rev() {
  return knobs().krylov_rev != 0;
}

template <int K>
void md_launch(const double2* V, size_t ldv, const double2* w, size_t len, double* part,
               int blocks, hipStream_t s, const int* stop, double* out, int cols,
               unsigned* counter) {
  const bool nt = krylov_nt(len);
  if (counter) {
    if (nt)
      hipLaunchKernelGGL((multidot_kernel<K, true, true>), dim3(blocks), dim3(kT), 0, s, V, ldv,
                         w, len, part, stop, out, cols, counter);
    else
      hipLaunchKernelGGL((multidot_kernel<K, false, true>), dim3(blocks), dim3(kT), 0, s, V, ldv,
                         w, len, part, stop, out, cols, counter);
  } else {
    if (nt)
      hipLaunchKernelGGL((multidot_kernel<K, true, false>), dim3(blocks), dim3(kT), 0, s, V, ldv,
                         w, len, part, stop, out, cols, counter);
    else
      hipLaunchKernelGGL((multidot_kernel<K, false, false>), dim3(blocks), dim3(kT), 0, s, V,
                         ldv, w, len, part, stop, out, cols, counter);
  }
}
template <int K, bool FUSED>
void up_launch_t(const double2* V, size_t ldv, const double* raw, const double* scale,
                 const double2* w, double2* wo, size_t len, double* part, int blocks,
                 hipStream_t s, const int* stop, const ColumnFuse& cf) {
  if (krylov_nt(len))
    hipLaunchKernelGGL((update_kernel<K, true, false, FUSED>), dim3(blocks), dim3(kT), 0, s, V,
                       ldv, raw, scale, w, wo, len, part, stop, cf);
  else if (krylov_rev())
    hipLaunchKernelGGL((update_kernel<K, false, true, FUSED>), dim3(blocks), dim3(kT), 0, s, V,
                       ldv, raw, scale, w, wo, len, part, stop, cf);
  else
    hipLaunchKernelGGL((update_kernel<K, false, false, FUSED>), dim3(blocks), dim3(kT), 0, s, V,
                       ldv, raw, scale, w, wo, len, part, stop, cf);
}
template <int K>
void up_launch(const double2* V, size_t ldv, const double* raw, const double* scale,
               const double2* w, double2* wo, size_t len, double* part, int blocks,
               hipStream_t s, const int* stop, const ColumnFuse* cf) {
  if (cf) up_launch_t<K, true>(V, ldv, raw, scale, w, wo, len, part, blocks, s, stop, *cf);
  else up_launch_t<K, false>(V, ldv, raw, scale, w, wo, len, part, blocks, s, stop, ColumnFuse{});
}
template <int K>
void xu_launch(const double2* V, size_t ldv, const double2* y, double2* x, size_t len, int blocks,
               hipStream_t s, const int* ctl) {
  if (krylov_nt(len))
    hipLaunchKernelGGL((xupdate_kernel<K, true>), dim3(blocks), dim3(kT), 0, s, V, ldv, y, x, len,
                       ctl);
  else
    hipLaunchKernelGGL((xupdate_kernel<K, false>), dim3(blocks), dim3(kT), 0, s, V, ldv, y, x, len,
                       ctl);
}

template <int... Ks>
struct KTable {
  using MD = void (*)(const double2*, size_t, const double2*, size_t, double*, int, hipStream_t,
                      const int*, double*, int, unsigned*);
  using UP = void (*)(const double2*, size_t, const double*, const double*, const double2*,
                      double2*, size_t, double*, int, hipStream_t, const int*, const ColumnFuse*);
  using XU = void (*)(const double2*, size_t, const double2*, double2*, size_t, int, hipStream_t,
                     const int*);
  static constexpr MD md[] = {md_launch<Ks>...};
  static constexpr UP up[] = {up_launch<Ks>...};
  static constexpr XU xu[] = {xu_launch<Ks>...};
};
using Table = KTable<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21,
                     22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32>;
static_assert(kMaxProj == 32, "table covers 1..kMaxProj");

}  // namespace

bool krylov_nt_for(size_t len) { return krylov_nt(len); }

void tune_krylov(int nt, int blocks) {
  g_krylov_nt = nt < 0 ? -1 : (nt != 0);
  g_krylov_blocks = blocks > 0 ? (blocks < kMaxStreamBlocks ? blocks : kMaxStreamBlocks) : 0;
}

int stream_blocks(size_t len) {
  const size_t cap = g_krylov_blocks > 0 ? (size_t)g_krylov_blocks
                                         : (len <= kSmallKrylovLen ? 512 : 1024);
  size_t b = (len + kT - 1) / kT;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

void launch_multidot(const double2* V, size_t ldv, int K, const double2* w, size_t len,
                     double* partials, int blocks, hipStream_t stream, const int* stop) {
  Table::md[K - 1](V, ldv, w, len, partials, blocks, stream, stop, nullptr, 0, nullptr);
}

void launch_multidot_reduced(const double2* V, size_t ldv, int K, const double2* w, size_t len,
                             double* partials, int blocks, double* out, int cols,
                             unsigned* counter, hipStream_t stream, const int* stop) {
  Table::md[K - 1](V, ldv, w, len, partials, blocks, stream, stop, out, cols, counter);
}

void launch_update(const double2* V, size_t ldv, int K, const double* raw, const double* scale,
                   const double2* w, double2* w_out, size_t len, double* partials, int blocks,
                   hipStream_t stream, const int* stop) {
  Table::up[K - 1](V, ldv, raw, scale, w, w_out, len, partials, blocks, stream, stop, nullptr);
}

void launch_update_column(const double2* V, size_t ldv, int K, const double* raw,
                          const double* scale, const double2* w, double2* w_out, size_t len,
                          double* partials, int blocks, hipStream_t stream, const int* stop,
                          const GivensState& g, int col, const double* red_dots, double eps,
                          double ptol, int stop_col, unsigned* counter) {
  ColumnFuse cf{};
  cf.g = g;
  cf.col = col;
  cf.stop_col = stop_col;
  cf.rd = red_dots;
  cf.eps = eps;
  cf.ptol = ptol;
  cf.counter = counter;
  Table::up[K - 1](V, ldv, raw, scale, w, w_out, len, partials, blocks, stream, stop, &cf);
}

void launch_xupdate(const double2* V, size_t ldv, int K, const double2* y, double2* x,
                    size_t len, int blocks, hipStream_t stream, const int* ctl) {
  Table::xu[K - 1](V, ldv, y, x, len, blocks, stream, ctl);
}

void launch_reduce(const double* partials, int count, int width, int cols, double* out,
                   hipStream_t stream, const int* stop) {
  hipLaunchKernelGGL(reduce_kernel, dim3(cols), dim3(kT), 0, stream, partials, count, width, out,
                     stop);
}

void launch_add_small(const double* in, double* out, int count, hipStream_t stream,
                      const int* stop) {
  hipLaunchKernelGGL(add_small_kernel, dim3(1), dim3(kT), 0, stream, in, out, count, stop);
}

void launch_fill_hash(double2* v, size_t len, size_t goff, uint64_t seed, hipStream_t stream) {
  hipLaunchKernelGGL(fill_hash_kernel, dim3(stream_blocks(len)), dim3(kT), 0, stream, v, len, goff,
                     seed);
}

void launch_scale_copy(const double2* in, double2* out, size_t len, double s,
                       hipStream_t stream, const int* stop) {
  hipLaunchKernelGGL(scale_copy_kernel, dim3(stream_blocks(len)), dim3(kT), 0, stream, in, out,
                     len, s, stop);
}

void launch_gmres_column(const GivensState& g, int col, const double* red_dots,
                         const double* red_norm, const double* norm_partials, int norm_count,
                         double eps, double ptol, int stop_col, hipStream_t stream) {
  hipLaunchKernelGGL(gmres_column_kernel, dim3(1), dim3(kWave), 0, stream, g, col, red_dots,
                     red_norm, norm_partials, norm_count, eps, ptol, stop_col);
}

void launch_gmres_lag_red(const GivensState& g, int j, const double* partials, int count,
                          int width, int cols, double* red, double eps, double ptol, int stop_col,
                          hipStream_t stream, int final_step) {
  hipLaunchKernelGGL(gmres_lag_red_kernel, dim3(1), dim3(kLagRedThreads), 0, stream, g, j,
                     partials, count, width, cols, red, eps, ptol, stop_col, final_step);
}
void launch_gmres_lag(const GivensState& g, int j, const double* red_dots, const double* sig2,
                      bool final_step, double eps, double ptol, int stop_col, hipStream_t stream) {
  hipLaunchKernelGGL(gmres_lag_kernel, dim3(1), dim3(kWave), 0, stream, g, j, red_dots, sig2,
                     final_step ? 1 : 0, eps, ptol, stop_col);
}

void launch_gmres_start(const GivensState& g, const double* red, int idx_r, int idx_m,
                        hipStream_t stream) {
  hipLaunchKernelGGL(gmres_start_kernel, dim3(1), dim3(kWave), 0, stream, g, red, idx_r, idx_m);
}

void launch_gmres_solve(const GivensState& g, int stop_col, bool merged, hipStream_t stream) {
  hipLaunchKernelGGL(gmres_solve_kernel, dim3(1), dim3(kWave), 0, stream, g, stop_col,
                     (int)merged);
}

}  // namespace hh
