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

namespace hh {
namespace {

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

// Block-reduce NV doubles held per thread; lane results land in partials[blk*width + k].
// SC1: stored write-through at device scope (agent-scope relaxed atomic stores), for a last
// block that reads them in the same launch (MI355X_MICROARCH.md's hand-off form: sc1 stores,
// drained, then one lane's agent-scope ticket; no L2-writeback fence).
template <int NV, bool SC1 = false>
__device__ __forceinline__ void block_reduce_vec(double (&v)[NV], double* partials, int width) {
  __shared__ double red[NV][kT / kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  // wave sums by DPP lane moves (VALU only; the xor butterfly took 12 dependent ds_bpermute per
  // value: ~500 LDS permutes per wave for the 41 values of a 20-vector multidot)
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double x = wave_sum_to_63(v[k]);
    if (lane == kWave - 1) red[k][wave] = x;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < NV; k += kT) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kT / kWave; ++w) s += red[k][w];
    if constexpr (SC1)
      __hip_atomic_store((gu64k*)(partials + (size_t)blockIdx.x * width + k),
                         (unsigned long long)__double_as_longlong(s), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    else
      partials[(size_t)blockIdx.x * width + k] = s;
  }
}


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
template <int K, bool NT>
__global__ __launch_bounds__(kT) void xupdate_kernel(const double2* __restrict__ V, size_t ldv,
                                                     const double2* __restrict__ y,
                                                     double2* __restrict__ x, size_t len) {
  double2 c[K];
#pragma unroll
  for (int k = 0; k < K; ++k) c[k] = y[k];
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t p = (size_t)blockIdx.x * kT + threadIdx.x; p < len; p += stride) {
    double2 t = make_double2(0.0, 0.0);
#pragma unroll
    for (int k = 0; k < K; ++k) t = cfma(c[k], ldnt<NT>(V + (size_t)k * ldv + p), t);
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

// LAPACK (3.10+) zlartg main branch: [c s; -conj(s) c] [f; g] = [r; 0], c real >= 0.
__device__ void zlartg(double2 f, double2 g, double* c, double2* s, double2* r) {
  if (g.x == 0.0 && g.y == 0.0) {
    *c = 1.0;
    *s = make_double2(0.0, 0.0);
    *r = f;
    return;
  }
  if (f.x == 0.0 && f.y == 0.0) {
    const double d = hypot(g.x, g.y);
    *c = 0.0;
    *s = make_double2(g.x / d, -g.y / d);
    *r = make_double2(d, 0.0);
    return;
  }
  const double f2 = cabs2(f);
  const double g2 = cabs2(g);
  const double h2 = f2 + g2;
  const double cc = sqrt(f2 / h2);
  *c = cc;
  *r = make_double2(f.x / cc, f.y / cc);
  const double d = sqrt(f2 * h2);
  const double2 fd = make_double2(f.x / d, f.y / d);
  *s = cmul(cconj(g), fd);
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

// Second half of a Hessenberg column, by ONE wave (every lane computes the same values, lane 0
// stores them): subdiagonal h1 against h0 (scipy's breakdown test), the previous Givens
// rotations, a new one (zlartg), the residual estimate and the inner exit test
// (iterative.py:767-795).  hk = entry `lane` of the column (lanes 0 .. col).  Lane k loads
// rotation k, so the chain of previous rotations takes its operands by readlane: one global
// load latency per column instead of one per rotation (the one-lane form waited on a dependent
// G load per step: 14 us per column at col ~ 19).  Same operations in the same order as the
// one-lane form: bit-identical.  Returns the exit decision (uniform; also in g.ctrl[0]).
// The finish's memory operands (lane k: rotation k; S[col] on every lane), loaded unconditionally
// from clamped addresses so that a caller can issue them with its own loads: one memory latency
// per launch (a load under a branch makes hipcc wait for every load at the join).
struct ColIn {
  double ck;
  double2 sk, Sc;
};
__device__ __forceinline__ ColIn load_col_in(const GivensState& g, int col) {
  const int lane = threadIdx.x & (kWave - 1);
  const int kr = min(lane, max(col - 1, 0));
  ColIn in;
  in.ck = g.G[2 * kr].x;
  in.sk = g.G[2 * kr + 1];
  in.Sc = g.S[col];
  return in;
}
__device__ bool gmres_finish_column(const GivensState& g, int col, double2 hk, const ColIn& in,
                                    double h0, double h1, double inv_sigma_next, double eps,
                                    double ptol, int stop_col) {
  const int lane = threadIdx.x & (kWave - 1);
  const bool l0 = lane == 0;
  const int R1 = g.restart + 1;
  double2* h = g.H + (size_t)col * R1;
  double2 hsub = make_double2(h1, 0.0);
  double brk = 0.0;
  if (h1 <= eps * h0) {
    hsub = make_double2(0.0, 0.0);
    brk = 1.0;
  } else if (l0) {
    g.vscale[col + 1] = inv_sigma_next;
  }
  const double ck = in.ck;
  const double2 sk = in.sk;
  double2 n0 = rlane2(hk, 0);
  for (int k = 0; k < col; ++k) {
    const double c = rlane(ck, k);
    const double2 s = rlane2(sk, k), n1 = rlane2(hk, k + 1);
    const double2 hn = cadd(cscale(n0, c), cmul(s, n1));
    if (l0) h[k] = hn;
    n0 = cadd(cmul(make_double2(-s.x, s.y), n0), cscale(n1, c));  // -conj(s)*n0 + c*n1
  }
  double c;
  double2 s, r;
  zlartg(n0, hsub, &c, &s, &r);
  const double2 Sc = in.Sc;
  const double2 tmp = cmul(make_double2(-s.x, s.y), Sc);  // -conj(s) * S[col]
  const double presid = hypot(tmp.x, tmp.y);
  const bool stop = presid <= ptol || brk != 0.0 || col >= stop_col;
  if (l0) {
    g.G[2 * col] = make_double2(c, 0.0);
    g.G[2 * col + 1] = s;
    h[col] = r;
    h[col + 1] = make_double2(0.0, 0.0);
    g.S[col] = cscale(Sc, c);
    g.S[col + 1] = tmp;
    g.status[0] = presid;
    g.status[1] = brk;
    g.status[2] = h0;
    g.status[3] = h1;
    double* st = g.status_it + 4 * col;
    st[0] = presid;
    st[1] = brk;
    st[2] = h0;
    st[3] = h1;
    g.ctrl[1] = col;
    if (stop) g.ctrl[0] = 1;
  }
  return stop;
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

// One-allreduce iteration j (lagged normalisation, world > 1; see runtime.cpp hh_gmres).  The
// basis is stored raw: u_k with exact norms sigma_k (vscale[k] = 1/sigma_k once known) and the
// SpMV of iteration j ran on sscale[j] u_j, sscale[j] an estimate of 1/sigma_j.  With raw dots
// d_k = <u_k, w> (rd[2k], rd[2k+1], k <= j), |w|^2 = rd[2j+2] and |u_j|^2 = rd[2j+3] (j >= 1), all
// from the iteration's single allreduce:
//   (a) vscale[j] = 1/sigma_j;
//   (b) column j-1 is finished: h1 = sigma_j vscale[j-1] / sscale[j-1] (the Hessenberg
//       subdiagonal the previous iteration could not know), rotations, presid, exit test;
//   (c) column j is started: h_kj = d_k vscale[k] f, h0 = |w| f with f = vscale[j] / sscale[j]
//       (the true <v_k, M A v_j> and |M A v_j| of scipy's normalised basis);
//   (d) sscale[j+1] = 1 / sqrt(|w|^2 - sum_k |d_k|^2 vscale[k]^2) (Pythagoras, floored): only
//       the scale of the next SpMV's input -- never part of H -- so cancellation in it cannot
//       reach the solve.
// The update (w -= sum_k d_k vscale[k]^2 u_k) follows with the exact vscale.  `final` (after the
// cycle's last iteration): rd is unused and sig2 holds |u_j|^2 -- steps (a), (b) only.
// One wave: entry k of a column on lane k (the sum of (d) in k order by readlane).
__global__ void gmres_lag_kernel(GivensState g, int j, const double* rd, const double* sig2,
                                 int final_step, double eps, double ptol, int stop_col) {
  const int lane = threadIdx.x & (kWave - 1);
  const int R1 = g.restart + 1;
  // every operand loaded up front, from clamped addresses (the finish of column j-1 and the start
  // of column j read disjoint words: the finish writes only vscale[j], which the start takes
  // from vj): one memory latency per launch
  const int col = max(j - 1, 0);
  const int stopped = g.ctrl[0];
  const double sig = *sig2;
  const double vs0 = g.vscale[0], vcol = g.vscale[col], scol = g.sscale[col], sj_ = g.sscale[j];
  const double h0c = g.status_it[4 * col + 2];  // stored when the column was started
  const double2 hk0 = g.H[(size_t)col * R1 + min(lane, col)];  // (previous launch)
  const ColIn in = load_col_in(g, col);
  const int kj = min(lane, j);
  const double vkj = g.vscale[kj];
  const double* rdp = rd ? rd : sig2;  // (final step: rd unused, any valid words of red)
  const double2 d = make_double2(rdp[2 * kj], rdp[2 * kj + 1]);
  const double w2 = rdp[2 * (j + 1)];
  if (stopped) return;
  double vj = vs0;
  if (j >= 1) {
    const double sj = sqrt(sig);
    vj = 1.0 / sj;
    const double f = vcol / scol;
    const double h1 = sj * f;
    const double2 hk = lane <= col ? hk0 : make_double2(0.0, 0.0);
    const bool stop = gmres_finish_column(g, col, hk, in, h0c, h1, vj, eps, ptol, stop_col);
    if (stop || final_step) return;
  }
  const double f = vj / sj_;
  double2* h = g.H + (size_t)j * R1;
  double tv = 0.0, tw = 0.0;
  if (lane <= j) {
    const double vk = lane == j ? vj : vkj;
    h[lane] = cscale(cscale(d, vk), f);
    tv = cabs2(d) * vk;
    tw = vk;
  }
  // rest -= |d_k|^2 v_k^2 in k order, the last multiply fused as the one-lane loop's compiled
  // form fused it (fp-contract), explicitly here
  double rest = w2;
  for (int k = 0; k <= j; ++k) rest = fma(-rlane(tv, k), rlane(tw, k), rest);
  if (lane == 0) {
    g.status_it[4 * j + 2] = sqrt(w2) * f;
    const double floor2 = fmax(w2 * 1e-28, 1e-300);
    g.sscale[j + 1] = 1.0 / sqrt(fmax(rest, floor2));
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

__global__ void gmres_solve_kernel(GivensState g, int col) {
  if (threadIdx.x != 0) return;
  const int R1 = g.restart + 1;
  auto H = [&](int c, int k) -> double2& { return g.H[(size_t)c * R1 + k]; };
  if (H(col, col).x == 0.0 && H(col, col).y == 0.0) g.S[col] = make_double2(0.0, 0.0);
  double2 y[kMaxProj];
  for (int k = 0; k <= col; ++k) y[k] = g.S[k];
  for (int k = col; k > 0; --k) {
    if (y[k].x != 0.0 || y[k].y != 0.0) {
      y[k] = cdiv_smith(y[k], H(k, k));
      const double2 t = y[k];
      for (int m = 0; m < k; ++m) y[m] = csub(y[m], cmul(t, H(k, m)));
    }
  }
  if (y[0].x != 0.0 || y[0].y != 0.0) y[0] = cdiv_smith(y[0], H(0, 0));
  for (int k = 0; k <= col; ++k) g.ycoef[k] = cscale(y[k], g.vscale[k]);
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
  static const bool rev = [] {
    const char* e = std::getenv("HH_KRYLOV_REV");
    return !(e && e[0] == '0');
  }();
  return rev;
}

// One-pass lagged GMRES iteration (FusedArgs, hh_internal.hpp).  A 256-thread block owns a
// 256-column strip of a band of `rows` grid rows and marches it: per row r it forms u_K on row
// r + 1 (w_{K-1} and the K basis vectors of that row: the iteration's only HBM read of them),
// applies the stencil (+ Jacobi) to row r from a three-row register ring (W/E neighbours through
// a double-buffered LDS row; the strip's two edge columns' u_K formed by the edge waves from
// broadcast loads), stores u_K and w_K of row r and adds row r's <u_k, w_K> -- the u_k re-read
// one row after the first read: the first KEEP of them from a two-row LDS copy each thread made
// of its own column (no barrier: the same lane writes and reads), the rest from the memory
// system (at 8192^2 the re-reads miss the L2: PMC FETCH ~2x the algorithmic reads,
// profiles/r03zc/).  The band's two halo rows of u_K are formed, never
// stored (each is a neighbouring band's own row): (rows + 2) / rows of the basis rows are read.
// Tiles are dealt to XCDs in contiguous runs (block b -> XCD b % 8), so a band's halo rows are
// mostly read on the XCD that owns them.  Arithmetic per point: update_kernel's coefficient
// and term order, stencil.hip's operator (bit-identical to the three launches it replaces,
// except the inner products' summation order).
struct double2x2 {
  double2 a, b;
};
__device__ __forceinline__ double2x2 make_double2x2(double2 a, double2 b) { return {a, b}; }

// by-value select (a select of lvalues would become a select of addresses)
__device__ __forceinline__ double2 csel(bool c, double2 a, double2 b) {
  return make_double2(c ? a.x : b.x, c ? a.y : b.y);
}

template <int K, bool CONSTC, int KEEP>
__global__ __launch_bounds__(kT) void fused_iter_kernel(const FusedArgs a) {
  if (a.stop && *a.stop) return;
  constexpr int KL = KEEP < K ? KEEP : K;  // (<= the update's batch of 8: its first batch)
  static_assert(KL <= 8, "kept vectors come from the update's first batch");
  __shared__ double2 coef[K];
  __shared__ double2 urow[2][kT + 2];
  __shared__ double2 vkeep[KL > 0 ? 2 : 1][KL > 0 ? KL : 1][kT];  // [row & 1][k][lane]
  const int n = a.n, R = a.rows;
  const int tiles_x = (n + kT - 1) / kT, bands = (n + R - 1) / R, T = tiles_x * bands;
  const int per_xcd = (T + 7) / 8;
  const int tile = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
  const bool live = tile < T;
  const int tx = live ? tile % tiles_x : 0, ty = live ? tile / tiles_x : 0;
  const int t = threadIdx.x, lane = t & (kWave - 1), wv = t / kWave;
  const int i0 = tx * kT, i = i0 + t;
  const bool act = i < n;
  const int ic = min(i, n - 1);
  const int rb = ty * R, re = min(rb + R, n);
  // the strip's edge columns: wave 0 forms u_K at i0 - 1, the last wave at i0 + kT
  const bool ew = wv == 0, ee = wv == kT / kWave - 1;
  const int ie = min(max(ew ? i0 - 1 : i0 + kT, 0), n - 1);
  const bool ehas = (ew && i0 > 0) || (ee && i0 + kT < n);
  if (t < K) {
    const double sk = a.vscale[t];
    const double2 hk = cscale(make_double2(a.raw[2 * t], a.raw[2 * t + 1]), sk);
    coef[t] = cscale(hk, sk);
  }
  __syncthreads();
  const double sin = *a.sin;
  const double2 z = make_double2(0.0, 0.0);
  // u_K at (r, col); rows off the grid are zero (loads from clamped rows, selected by value).
  // kz: an opaque zero redefined every row, so neither the coefficients' LDS reads nor the
  // per-vector addresses become loop-invariant / strength-reduced registers (4 + 2-6 VGPRs per
  // basis vector otherwise, i.e. one wave per SIMD at K >= 11)
  int kz = 0;
  auto unew = [&](int r, int col, bool keep) {
    __builtin_amdgcn_sched_barrier(0);  // (calls and batches do not interleave: registers)
    const size_t p = (size_t)min(max(r, 0), n - 1) * n + col;
    double2 w = a.win[p];
    constexpr int kB = 8;
    // a runtime loop over batches (an unrolled one kept ~16 VGPRs per basis vector live:
    // one wave per SIMD from K = 11)
#pragma unroll 1
    for (int k0 = 0; k0 < K; k0 += kB) {
      double2 v[kB];
#pragma unroll
      for (int q = 0; q < kB; ++q) v[q] = a.V[(size_t)min(k0 + q, K - 1) * a.ldv + p];
      if (KL > 0 && keep && k0 == 0) {
#pragma unroll
        for (int q = 0; q < KL; ++q) vkeep[r & 1][q][threadIdx.x] = v[q];
      }
#pragma unroll
      for (int q = 0; q < kB; ++q)
        if (k0 + q < K) w = csub(w, cmul(coef[k0 + q + kz], v[q]));
    }
    return csel(r >= 0 && r < n, w, z);
  };
  // u_K at one point, lane-parallel (the edge waves: lane k of each half takes the term
  // c_k u_k, summed by shuffles -- one load round trip instead of ceil(K / 8) batches)
  auto unew1 = [&](int r, int c) {
    const int k = lane & 31;
    const size_t p = (size_t)min(max(r, 0), n - 1) * n + c;
    const double2 wv = a.win[p];
    const double2 vk = a.V[(size_t)min(k, K - 1) * a.ldv + p];
    double2 tk = csel(k < K, cmul(coef[min(k, K - 1)], vk), z);
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) {
      tk.x += __shfl_xor(tk.x, off);
      tk.y += __shfl_xor(tk.y, off);
    }
    return csel(r >= 0 && r < n, csub(wv, tk), z);
  };
  const double2 AW = a.tab_i[ic], AE = a.tab_i[n + ic], R1 = a.tab_i[2 * n + ic];
  double2 acc[K + 1];
#pragma unroll
  for (int k = 0; k <= K; ++k) acc[k] = z;
  double nw = 0.0, nu = 0.0;
  if (live) {
    double2 uS = unew(rb - 1, ic, false), uC = unew(rb, ic, true);
    int buf = 0;
    for (int r0 = rb; r0 < re; ++r0) {
      int r = r0;
      asm volatile("" : "+s"(r), "+s"(kz));
      const double2 uN = unew(r + 1, ic, true);
      double2 ue = z;
      if (ew || ee) ue = unew1(r, ie);  // (wave-uniform: the two edge waves only)
      urow[buf][1 + t] = csel(act, uC, z);
      if (ew && lane == 0) urow[buf][0] = csel(ehas, ue, z);
      if (ee && lane == kWave - 1) urow[buf][kT + 1] = csel(ehas, ue, z);
      __syncthreads();
      const double2 uW = urow[buf][t], uE = urow[buf][t + 2];
      const double* q = reinterpret_cast<const double*>(a.tab_j) + 8 * (size_t)r;
      const double2 R2 = make_double2(q[0], q[1]), BS = make_double2(q[2], q[3]);
      const double2 BN = make_double2(q[4], q[5]), OM = make_double2(q[6], q[7]);
      const size_t p = (size_t)r * n + ic;
      const double icv = CONSTC ? a.invc2_const : a.invc2[p];
      const double2 W = cmul(AW, R2);
      const double2 E = cmul(AE, R2);
      const double2 S = cmul(BS, R1);
      const double2 N = cmul(BN, R1);
      const double2 M = cscale(cmul(OM, R1), icv);
      const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
      const double2 D = csub(M, sum4);
      double2 Au = cmul(S, uS);
      Au = cfma(W, uW, Au);
      Au = cfma(D, uC, Au);
      Au = cfma(E, uE, Au);
      Au = cfma(N, uN, Au);
      const double2 w = csel(act, a.jac ? cscale(cdiv(Au, D), sin) : cscale(Au, sin), z);
      if (act) {
        a.wout[p] = w;
        a.uout[p] = uC;
      }
      const double2 uo = csel(act, uC, z);
      nu = fma(uo.x, uo.x, fma(uo.y, uo.y, nu));
      nw = fma(w.x, w.x, fma(w.y, w.y, nw));
      // (batches of 8 re-reads in flight: all K at once would hold 4 K more VGPRs)
#pragma unroll
      for (int k0 = 0; k0 < K; k0 += 8) {
        double2 v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q)
          v[q] = k0 + q < KL ? vkeep[r & 1][k0 + q][t]
                             : a.V[(size_t)min(k0 + q, K - 1) * a.ldv + p];
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (k0 + q < K) acc[k0 + q] = cfma_conj(v[q], w, acc[k0 + q]);
        __builtin_amdgcn_sched_barrier(0);
      }
      acc[K] = cfma_conj(uo, w, acc[K]);
      uS = uC;
      uC = uN;
      buf ^= 1;
    }
  }
  // one partial row: the K + 1 dots, |w_K|^2, then |u_K|^2 -- one reduce launch lands the last
  // exactly where gmres_lag_kernel reads sigma_K^2 (red + 16 + 2 (K + 1) + 1)
  double v[2 * (K + 1) + 2];
#pragma unroll
  for (int k = 0; k <= K; ++k) {
    v[2 * k] = acc[k].x;
    v[2 * k + 1] = acc[k].y;
  }
  v[2 * (K + 1)] = nw;
  v[2 * (K + 1) + 1] = nu;
  block_reduce_vec<2 * (K + 1) + 2>(v, a.partials, 2 * (K + 1) + 2);
}

// The same pass with M = the two-sweep shifted-Laplace smoother (stencil.hip EPI_SL_FIRST then
// EPI_SL_SWEEP): T = s A u, z1 = damp T / D_beta, w = z1 + damp (T - A_beta z1) / D_beta.
// Output row r needs z1 on rows r-1 .. r+1, i.e. u_K on rows r-2 .. r+2 and on two columns
// beyond the strip on each side: per step L the block forms u_K on row L (own columns; the
// edge waves also on the edge column and, one row behind, the outer column), T and z1 on row
// L-1 (own columns; the edge waves on the edge column) and w on row L-2 -- rings of three u,
// two T and three z1 rows, W/E neighbours of u (row L-1) and z1 (row L-2) through two
// double-buffered LDS rows.  Rows and columns off the grid are zero for u, T and z1 alike
// (the two-launch path's Dirichlet neighbours).
template <int K, bool CONSTC>
__global__ __launch_bounds__(kT) void fused_sl_iter_kernel(const FusedArgs a) {
  if (a.stop && *a.stop) return;
  __shared__ double2 coef[K];
  __shared__ double2 urow[2][kT + 2], zrow[2][kT + 2];
  const int n = a.n, R = a.rows;
  const int tiles_x = (n + kT - 1) / kT, bands = (n + R - 1) / R, T_ = tiles_x * bands;
  const int per_xcd = (T_ + 7) / 8;
  const int tile = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
  const bool live = tile < T_;
  const int tx = live ? tile % tiles_x : 0, ty = live ? tile / tiles_x : 0;
  const int t = threadIdx.x, lane = t & (kWave - 1), wv = t / kWave;
  const int i0 = tx * kT, i = i0 + t;
  const bool act = i < n;
  const int ic = min(i, n - 1);
  const int rb = ty * R, re = min(rb + R, n);
  // edge waves: wave 0 the W edge column i0-1 (outer i0-2, inner i0 = LDS slot 1), the last
  // wave the E edge column i0+kT (outer i0+kT+1, inner i0+kT-1 = LDS slot kT)
  const bool ew = wv == 0, ee = wv == kT / kWave - 1;
  const int ie_raw = ew ? i0 - 1 : i0 + kT, io_raw = ew ? i0 - 2 : i0 + kT + 1;
  const bool ehas = (ew || ee) && ie_raw >= 0 && ie_raw < n;
  const bool ohas = (ew || ee) && io_raw >= 0 && io_raw < n;
  const int ie = min(max(ie_raw, 0), n - 1), io = min(max(io_raw, 0), n - 1);
  const int islot = ew ? 1 : kT;  // LDS slot of the edge column's inner neighbour
  if (t < K) {
    const double sk = a.vscale[t];
    const double2 hk = cscale(make_double2(a.raw[2 * t], a.raw[2 * t + 1]), sk);
    coef[t] = cscale(hk, sk);
  }
  __syncthreads();
  const double sin = *a.sin;
  const double damp = a.damping;
  const double2 mshift = a.mshift;
  const double2 z = make_double2(0.0, 0.0);
  int kz = 0;
  auto unew = [&](int r, int col) {
    __builtin_amdgcn_sched_barrier(0);
    const size_t p = (size_t)min(max(r, 0), n - 1) * n + col;
    double2 w = a.win[p];
    constexpr int kB = 8;
#pragma unroll 1
    for (int k0 = 0; k0 < K; k0 += kB) {
      double2 v[kB];
#pragma unroll
      for (int q = 0; q < kB; ++q) v[q] = a.V[(size_t)min(k0 + q, K - 1) * a.ldv + p];
#pragma unroll
      for (int q = 0; q < kB; ++q)
        if (k0 + q < K) w = csub(w, cmul(coef[k0 + q + kz], v[q]));
    }
    return csel(r >= 0 && r < n, w, z);
  };
  // u_K at two points at once, lane-parallel (the edge waves): half h of the wave takes point
  // h, lane k of the half the term c_k u_k, the 32 terms summed by shuffles -- one load round
  // trip instead of two chains of ceil(K / 8) batches (terms in a tree order: the strip that
  // owns the column forms it in k order, so halo values agree to rounding)
  auto unew2 = [&](int r1, int c1, int r2, int c2) {
    const int h = lane >> 5, k = lane & 31;
    const int r = h ? r2 : r1, c = h ? c2 : c1;
    const size_t p = (size_t)min(max(r, 0), n - 1) * n + c;
    const double2 wv = a.win[p];
    const double2 vk = a.V[(size_t)min(k, K - 1) * a.ldv + p];
    double2 tk = csel(k < K, cmul(coef[min(k, K - 1)], vk), z);
#pragma unroll
    for (int off = 16; off > 0; off >>= 1) {
      tk.x += __shfl_xor(tk.x, off);
      tk.y += __shfl_xor(tk.y, off);
    }
    const double2 u = csel(r >= 0 && r < n, csub(wv, tk), z);
    const double2 ua = make_double2(__shfl(u.x, 0), __shfl(u.y, 0));
    const double2 ub = make_double2(__shfl(u.x, 32), __shfl(u.y, 32));
    return make_double2x2(ua, ub);
  };
  // the operator's coefficients at (row r, column c): W, E, S, N, D, D_beta (stencil.hip order)
  struct Co {
    double2 W, E, S, N, D, Db;
  };
  auto coefs = [&](int r, int c, double icv) {
    const double* q = reinterpret_cast<const double*>(a.tab_j) + 8 * (size_t)min(max(r, 0), n - 1);
    const double2 R2 = make_double2(q[0], q[1]), BS = make_double2(q[2], q[3]);
    const double2 BN = make_double2(q[4], q[5]), OM = make_double2(q[6], q[7]);
    const double2 AW = a.tab_i[c], AE = a.tab_i[n + c], R1 = a.tab_i[2 * n + c];
    Co o;
    o.W = cmul(AW, R2);
    o.E = cmul(AE, R2);
    o.S = cmul(BS, R1);
    o.N = cmul(BN, R1);
    const double2 M = cscale(cmul(OM, R1), icv);
    const double2 sum4 = cadd(cadd(cadd(o.W, o.E), o.S), o.N);
    o.D = csub(M, sum4);
    o.Db = csub(cmul(M, mshift), sum4);
    return o;
  };
  auto icv_at = [&](int r, int c) {
    return CONSTC ? a.invc2_const : a.invc2[(size_t)min(max(r, 0), n - 1) * n + c];
  };
  double2 acc[K + 1];
#pragma unroll
  for (int k = 0; k <= K; ++k) acc[k] = z;
  double nw = 0.0, nu = 0.0;
  if (live) {
    // rings (own column): u(L-2), u(L-1); T(L-2); z1(L-3), z1(L-2).  Edge waves: u(L-2, ie),
    // u(L-1, ie), z1(L-2, ie).
    double2 uP = z, uC = z, Tm = z, z1a = z, z1b = z;
    double2 euP = z, euC = z, ez1b = z;
    // row L-1's shifted diagonal and the reciprocal of its |.|^2 (cdiv's one division), handed
    // to the second sweep of the next step, whose row it is
    double2 Dbm = make_double2(1.0, 0.0);
    double invm = 1.0;
    int buf = 0;
    for (int L0 = rb - 2; L0 <= re + 1; ++L0) {
      int L = L0;
      asm volatile("" : "+s"(L), "+s"(kz));
      const double2 uN = unew(L, ic);
      double2 euN = z, eo = z;
      if (ew || ee) {  // (wave-uniform)
        const auto pr = unew2(L, ie, L - 1, io);
        euN = csel(ehas, pr.a, z);
        eo = csel(ohas, pr.b, z);
      }
      urow[buf][1 + t] = csel(act, uC, z);
      zrow[buf][1 + t] = csel(act, z1b, z);
      if (ew && lane == 0) {
        urow[buf][0] = euC;
        zrow[buf][0] = ez1b;
      }
      if (ee && lane == kWave - 1) {
        urow[buf][kT + 1] = euC;
        zrow[buf][kT + 1] = ez1b;
      }
      __syncthreads();
      const double2 uW = urow[buf][t], uE = urow[buf][t + 2];
      const double2 zW = zrow[buf][t], zE = zrow[buf][t + 2];
      const bool v1 = L - 1 >= 0 && L - 1 < n;  // row L-1 on the grid
      // T and z1 on row L-1 (own column)
      const double ic1 = icv_at(L - 1, ic);
      const Co c1 = coefs(L - 1, ic, ic1);
      double2 Au = cmul(c1.S, uP);
      Au = cfma(c1.W, uW, Au);
      Au = cfma(c1.D, uC, Au);
      Au = cfma(c1.E, uE, Au);
      Au = cfma(c1.N, uN, Au);
      const double2 T1 = csel(act && v1, cscale(Au, sin), z);
      const double inv1 = 1.0 / fma(c1.Db.x, c1.Db.x, c1.Db.y * c1.Db.y);
      auto cdivr = [](double2 x, double2 b, double inv) {  // cdiv with the reciprocal given
        return make_double2(fma(x.x, b.x, x.y * b.y) * inv, fma(x.y, b.x, -x.x * b.y) * inv);
      };
      const double2 z1c = csel(act && v1, cscale(cdivr(T1, c1.Db, inv1), damp), z);
      // the same at the edge column (edge waves; broadcast values)
      double2 ez1c = z;
      if (ew || ee) {
        const double2 uin = urow[buf][islot];
        const double2 eW = ew ? eo : uin, eE = ew ? uin : eo;
        const Co ce = coefs(L - 1, ie, icv_at(L - 1, ie));
        double2 Ae = cmul(ce.S, euP);
        Ae = cfma(ce.W, eW, Ae);
        Ae = cfma(ce.D, euC, Ae);
        Ae = cfma(ce.E, eE, Ae);
        Ae = cfma(ce.N, euN, Ae);
        const double2 eT = cscale(Ae, sin);
        ez1c = csel(ehas && v1, cscale(cdiv(eT, ce.Db), damp), z);
      }
      // w on row r = L-2: the second sweep (A_beta on z1)
      const int r = L - 2;
      if (r >= rb && r < re) {  // (block-uniform)
        const size_t p = (size_t)r * n + ic;
        // row r's W, E, S, N (no mass term: its D_beta and reciprocal come from the last step)
        const double* q = reinterpret_cast<const double*>(a.tab_j) + 8 * (size_t)r;
        const double2 R2 = make_double2(q[0], q[1]), BS = make_double2(q[2], q[3]);
        const double2 BN = make_double2(q[4], q[5]);
        const double2 AW = a.tab_i[ic], AE = a.tab_i[n + ic], R1 = a.tab_i[2 * n + ic];
        const double2 W2 = cmul(AW, R2), E2 = cmul(AE, R2), S2 = cmul(BS, R1), N2 = cmul(BN, R1);
        double2 Az = cmul(S2, z1a);
        Az = cfma(W2, zW, Az);
        Az = cfma(Dbm, z1b, Az);
        Az = cfma(E2, zE, Az);
        Az = cfma(N2, z1c, Az);
        const double2 w = csel(act, cadd(z1b, cscale(cdivr(csub(Tm, Az), Dbm, invm), damp)), z);
        if (act) {
          a.wout[p] = w;
          a.uout[p] = uP;
        }
        const double2 uo = csel(act, uP, z);
        nu = fma(uo.x, uo.x, fma(uo.y, uo.y, nu));
        nw = fma(w.x, w.x, fma(w.y, w.y, nw));
#pragma unroll
        for (int k0 = 0; k0 < K; k0 += 8) {
          double2 v[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = a.V[(size_t)min(k0 + q, K - 1) * a.ldv + p];
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if (k0 + q < K) acc[k0 + q] = cfma_conj(v[q], w, acc[k0 + q]);
          __builtin_amdgcn_sched_barrier(0);
        }
        acc[K] = cfma_conj(uo, w, acc[K]);
      }
      uP = uC;
      uC = uN;
      Tm = T1;
      z1a = z1b;
      z1b = z1c;
      euP = euC;
      euC = euN;
      ez1b = ez1c;
      Dbm = c1.Db;
      invm = inv1;
      buf ^= 1;
    }
  }
  double v[2 * (K + 1) + 2];
#pragma unroll
  for (int k = 0; k <= K; ++k) {
    v[2 * k] = acc[k].x;
    v[2 * k + 1] = acc[k].y;
  }
  v[2 * (K + 1)] = nw;
  v[2 * (K + 1) + 1] = nu;
  block_reduce_vec<2 * (K + 1) + 2>(v, a.partials, 2 * (K + 1) + 2);
}

// basis vectors whose re-read comes from the LDS copy (HH_FUSED_KEEP: 0, 4 or 8; read per
// launch so one process can A/B it)
int fused_keep() {
  const char* e = std::getenv("HH_FUSED_KEEP");
  return e ? std::atoi(e) : kFusedKeepDefault;
}
template <int K>
void fused_launch(const FusedArgs& a, int blocks, hipStream_t s) {
  if (a.sl) {
    if (a.invc2)
      hipLaunchKernelGGL((fused_sl_iter_kernel<K, false>), dim3(blocks), dim3(kT), 0, s, a);
    else
      hipLaunchKernelGGL((fused_sl_iter_kernel<K, true>), dim3(blocks), dim3(kT), 0, s, a);
    return;
  }
  const int keep = fused_keep();
  if (keep >= 8) {
    if (a.invc2)
      hipLaunchKernelGGL((fused_iter_kernel<K, false, 8>), dim3(blocks), dim3(kT), 0, s, a);
    else
      hipLaunchKernelGGL((fused_iter_kernel<K, true, 8>), dim3(blocks), dim3(kT), 0, s, a);
  } else if (keep >= 4) {
    if (a.invc2)
      hipLaunchKernelGGL((fused_iter_kernel<K, false, 4>), dim3(blocks), dim3(kT), 0, s, a);
    else
      hipLaunchKernelGGL((fused_iter_kernel<K, true, 4>), dim3(blocks), dim3(kT), 0, s, a);
  } else {
    if (a.invc2)
      hipLaunchKernelGGL((fused_iter_kernel<K, false, 0>), dim3(blocks), dim3(kT), 0, s, a);
    else
      hipLaunchKernelGGL((fused_iter_kernel<K, true, 0>), dim3(blocks), dim3(kT), 0, s, a);
  }
}
template <int... Ks>
struct FTable {
  using FN = void (*)(const FusedArgs&, int, hipStream_t);
  static constexpr FN f[] = {fused_launch<Ks>...};
};
using FusedTable = FTable<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20>;
static_assert(kFusedMaxK == 20, "table covers 1..kFusedMaxK");

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
               hipStream_t s) {
  if (krylov_nt(len))
    hipLaunchKernelGGL((xupdate_kernel<K, true>), dim3(blocks), dim3(kT), 0, s, V, ldv, y, x, len);
  else
    hipLaunchKernelGGL((xupdate_kernel<K, false>), dim3(blocks), dim3(kT), 0, s, V, ldv, y, x, len);
}

template <int... Ks>
struct KTable {
  using MD = void (*)(const double2*, size_t, const double2*, size_t, double*, int, hipStream_t,
                      const int*, double*, int, unsigned*);
  using UP = void (*)(const double2*, size_t, const double*, const double*, const double2*,
                      double2*, size_t, double*, int, hipStream_t, const int*, const ColumnFuse*);
  using XU = void (*)(const double2*, size_t, const double2*, double2*, size_t, int, hipStream_t);
  static constexpr MD md[] = {md_launch<Ks>...};
  static constexpr UP up[] = {up_launch<Ks>...};
  static constexpr XU xu[] = {xu_launch<Ks>...};
};
using Table = KTable<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21,
                     22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32>;
static_assert(kMaxProj == 32, "table covers 1..kMaxProj");

}  // namespace

int fused_iter_rows(int n) {
  static const int env = [] {
    const char* e = std::getenv("HH_FUSED_ROWS");
    return e ? std::atoi(e) : 0;
  }();
  const long tiles_x = (n + kT - 1) / kT;
  int R = env > 0 ? env : (int)std::min<long>(32, std::max<long>(8, tiles_x * n / 1024));
  // the partial rows (one per block) fit kMaxStreamBlocks
  while ((long)tiles_x * ((n + R - 1) / R) > kMaxStreamBlocks) R *= 2;
  return R;
}
int fused_iter_blocks(int n, int rows) {
  const int T = (n + kT - 1) / kT * ((n + rows - 1) / rows);
  return (T + 7) / 8 * 8;
}
void launch_fused_iter(int K, const FusedArgs& a, int blocks, hipStream_t stream) {
  FusedTable::f[K - 1](a, blocks, stream);
}

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
                    size_t len, int blocks, hipStream_t stream) {
  Table::xu[K - 1](V, ldv, y, x, len, blocks, stream);
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

void launch_gmres_lag(const GivensState& g, int j, const double* red_dots, const double* sig2,
                      bool final_step, double eps, double ptol, int stop_col, hipStream_t stream) {
  hipLaunchKernelGGL(gmres_lag_kernel, dim3(1), dim3(kWave), 0, stream, g, j, red_dots, sig2,
                     final_step ? 1 : 0, eps, ptol, stop_col);
}

void launch_gmres_start(const GivensState& g, const double* red, int idx_r, int idx_m,
                        hipStream_t stream) {
  hipLaunchKernelGGL(gmres_start_kernel, dim3(1), dim3(kWave), 0, stream, g, red, idx_r, idx_m);
}

void launch_gmres_solve(const GivensState& g, int col, hipStream_t stream) {
  hipLaunchKernelGGL(gmres_solve_kernel, dim3(1), dim3(kWave), 0, stream, g, col);
}

}  // namespace hh
