// A whole GMRES restart cycle in ONE launch, for small grids (BASELINE config 1: 128^2).
//
// The regular cycle (runtime.cpp hh_gmres) queues five launches per inner iteration (stencil,
// multidot, reduce, update, Givens column).  At N = n^2 = 16384 each launch moves ~0.5 MB and
// costs a kernel boundary (~4-5 us of GPU timeline), so the cycle is launch-bound at ~30 us per
// iteration.  Here the grid keeps the Krylov basis ON CHIP and meets once per inner iteration:
//
//  * workgroup g owns layer (row) g of the grid, thread t column t; its LDS holds, for every
//    basis vector u_k, its own row and copies of the two neighbouring rows ("ghost" rows);
//  * iteration j: z = M A (s_j u_j) on the own row (neighbours from LDS: the ghosts), partial
//    sums <u_k, z> (k <= j), |z|^2 and |u_j|^2 of the own row, then ONE grid barrier that also
//    hands every workgroup its neighbours' rows of z;
//  * after it every workgroup reduces all partials in the same fixed order (identical numbers
//    on every workgroup, no second collective), runs the lagged-normalisation step of
//    krylov.hip gmres_lag_kernel (the Hessenberg column j-1 completed with |u_j|, column j
//    started, the Pythagorean scale of the next input) redundantly on lane 0, and forms
//    u_{j+1} = z - sum_k c_k u_k on its own row AND on its two ghost rows -- the neighbours'
//    z rows arrived with the barrier and every ghost u_k is kept, so no second hand-off is
//    needed;
//  * after the last column: the triangular solve and x += sum y_k u_k on the own row.
// Inter-workgroup data follows MI355X_MICROARCH.md's valid hand-off form (every shared byte
// stored and loaded with agent-scope relaxed atomics = sc1 global accesses, each storing wave
// drains vmcnt before one lane's agent-scope counter add; one workgroup per CU); every spin is
// bounded and a timeout ends the launch with the timeout word set (the host raises an error).
//
// Arithmetic: the stencil and Jacobi epilogue are stencil.hip's term for term; dot products
// and the update follow krylov.hip; only the summation order of the inner products differs
// from the regular cycle (histories agree to rounding; tests/test_gpu_small_cycle.py).
#include "hh_internal.hpp"
#include "hh_complex.hpp"

namespace hh {
namespace {

using gu32 = __attribute__((address_space(1))) unsigned;
using gu64 = __attribute__((address_space(1))) unsigned long long;

__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

__device__ __forceinline__ double2 csel(bool c, double2 a, double2 b) {
  return make_double2(c ? a.x : b.x, c ? a.y : b.y);
}

constexpr int kSmallThreads = 256;    // block size cap for the grid's rows (n <= 256)
constexpr int kPStride = 2 * (kMaxProj + 1) + 2;  // partial-sum columns (global layout)
constexpr unsigned kSpinLimit = 1u << 22;  // ~1 s of polling: a barrier wait is microseconds

// LDS pointers carry address space 3 on the device (ds_ instructions, not flat ones); the host
// pass only parses this code, with plain pointers
#if defined(__HIP_DEVICE_COMPILE__)
#define HH_LDS __attribute__((address_space(3)))
#else
#define HH_LDS
#endif
using l2 = HH_LDS double2;
using l1 = HH_LDS double;
using li = HH_LDS int;
struct Shared {  // LDS layout (carved from dynamic shared memory; see small_cycle_lds_bytes)
  l2* U;     // [R1][3][n]: rows 0 = g-1 (ghost), 1 = g (own), 2 = g+1 (ghost)
  l2* zrow;  // [n] this iteration's z on the own row
  l2* H;     // [R][R1]
  l2* Gr;    // [R][2] Givens (c, s)
  l2* S;     // [R1]
  l2* coef;  // [R1] update / x-update coefficients
  l1* vs;    // [R1] exact 1 / |u_k|
  l1* ss;    // [R1] scale of each SpMV input
  l1* h0s;   // [R]
  l1* red;   // [kSmallThreads] chunk sums of the partial reduction
  l1* sum;   // [PSTRIDE] reduced sums
  li* ctl;   // [4]: 0 stop, 1 last column, 2 abort
};

// All-reduce of `cols` doubles per workgroup, one level (the words are zeroed before the
// launch; rows and sums are double-buffered by `par`, so a round never overwrites what a slower
// workgroup may still read from the round before):
//  1. every workgroup has published its row part[par][g][0 .. cols) (sc1 stores, drained by
//     every storing wave, then a workgroup barrier); thread 0 adds to the arrival counter;
//  2. the LAST arriver (told by the value its add returns) sums every column over all rows in
//     row order -- each thread a column x a contiguous chunk of rows, its loads in flight
//     together, the chunk sums added in chunk order -- into fsum[par], then raises the round's
//     flag;
//  3. everyone polls the flag (thread 0, relaxed sc1 loads, bounded) and reads fsum into LDS.
// The arithmetic order is fixed whichever workgroup is last: identical sums on every workgroup
// and every run.  Hand-offs in MI355X_MICROARCH.md's valid form (sc1 stores drained before one
// lane's agent-scope add or flag store; sc1 loads after the poll + a workgroup barrier).
// Returns false on timeout (every workgroup then leaves the kernel).
constexpr int kChunk = 32;  // rows one reducing thread loads in flight per batch
struct ArArgs {
  double* part;     // [2][G][kPStride]
  double* fsum;     // [2][kPStride]
  unsigned* words;  // [0] arrival counter, [1] timeout, [2] flag
};
__device__ bool allreduce_rows(const ArArgs& ar, int par, unsigned epoch, int cols, l1* out,
                               l1* red, li* ctl) {
  const unsigned G = gridDim.x;
  const int t = threadIdx.x, nt = blockDim.x;
  unsigned* cnt = ar.words;
  unsigned* tmo = ar.words + 1;
  unsigned* flag = ar.words + 2;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's row stores drained
  __syncthreads();
  if (t == 0) {
    const unsigned old =
        __hip_atomic_fetch_add((gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ctl[3] = old + 1 == epoch * G ? 1 : 0;
  }
  __syncthreads();
  if (ctl[3]) {  // the last arriver reduces
    const int hq = max(1, min(nt / cols, (int)G));
    const int chunk = ((int)G + hq - 1) / hq;
    const int c = t / hq, h = t % hq;
    if (c < cols) {
      const int q0 = h * chunk, q1 = min((int)G, q0 + chunk);
      double s = 0.0;
      for (int b = q0; b < q1; b += kChunk) {
        double v[kChunk];
#pragma unroll
        for (int i = 0; i < kChunk; ++i)
          v[i] = ld_sc1(ar.part + ((size_t)par * G + min(b + i, q1 - 1)) * kPStride + c);
#pragma unroll
        for (int i = 0; i < kChunk; ++i)
          if (b + i < q1) s += v[i];
      }
      red[t] = s;
    }
    __syncthreads();
    if (t < cols) {
      double r = 0.0;
      for (int q = 0; q < hq; ++q) r += red[t * hq + q];
      st_sc1(ar.fsum + (size_t)par * kPStride + t, r);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0)
      __hip_atomic_store((gu32*)flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (t == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load((gu32*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kSpinLimit) {
        __hip_atomic_store((gu32*)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ctl[2] = 1;
        break;
      }
    }
  }
  __syncthreads();
  if (ctl[2]) return false;
  if (t < cols) out[t] = ld_sc1(ar.fsum + (size_t)par * kPStride + t);
  __syncthreads();
  return true;
}

// LAPACK zlartg main branch (krylov.hip)
__device__ void zlartg_s(double2 f, double2 g, double* c, double2* s, double2* r) {
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

// lane 0: complete column `col` with its subdiagonal h1 (krylov.hip gmres_finish_column); the
// status of the column goes to status_it (workgroup 0 only).  Returns true when the cycle stops.
__device__ bool finish_column(const Shared& sh, const SmallCycleArgs& a, int col, double h1,
                              double inv_sigma_next) {
  const int R1 = a.restart + 1;
  l2* h = sh.H + (size_t)col * R1;
  const double h0 = sh.h0s[col];
  h[col + 1] = make_double2(h1, 0.0);
  double brk = 0.0;
  if (h1 <= a.eps * h0) {
    h[col + 1] = make_double2(0.0, 0.0);
    brk = 1.0;
  } else {
    sh.vs[col + 1] = inv_sigma_next;
  }
  // the previous rotations, in order; the running entry is carried in registers and the next
  // step's operands are loaded one step ahead (the chain never waits on an LDS round trip)
  if (col > 0) {
    double2 n0 = h[0];
    double c = sh.Gr[0].x;
    double2 s = sh.Gr[1], n1 = h[1];
    for (int k = 0; k < col; ++k) {
      const int kn = min(k + 1, col - 1);
      const double cn = sh.Gr[2 * kn].x;
      const double2 sn = sh.Gr[2 * kn + 1], n1n = h[kn + 1];
      h[k] = cadd(cscale(n0, c), cmul(s, n1));
      n0 = cadd(cmul(make_double2(-s.x, s.y), n0), cscale(n1, c));
      c = cn;
      s = sn;
      n1 = n1n;
    }
    h[col] = n0;
  }
  double c;
  double2 s, r;
  zlartg_s(h[col], h[col + 1], &c, &s, &r);
  sh.Gr[2 * col] = make_double2(c, 0.0);
  sh.Gr[2 * col + 1] = s;
  h[col] = r;
  h[col + 1] = make_double2(0.0, 0.0);
  const double2 Sc = sh.S[col];
  const double2 tmp = cmul(make_double2(-s.x, s.y), Sc);
  sh.S[col] = cscale(Sc, c);
  sh.S[col + 1] = tmp;
  const double presid = hypot(tmp.x, tmp.y);
  if (blockIdx.x == 0) {
    double* st = a.g.status_it + 4 * col;
    st[0] = presid;
    st[1] = brk;
    st[2] = h0;
    st[3] = h1;
  }
  sh.ctl[1] = col;
  return presid <= a.ptol || brk != 0.0 || col >= a.stop_col;
}


template <bool CONSTC, bool JAC>
__global__ __launch_bounds__(kSmallThreads + kWave) void gmres_small_cycle_kernel(SmallCycleArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = a.n, R = a.restart, R1 = R + 1;
  const int g = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
  // threads 0 .. nrow-1 own the row's columns; the last wave (lane `book`) keeps the books:
  // it completes the previous Hessenberg column while the others update the basis
  const int nrow = nt - kWave, book = nt - kWave;
  const bool act = t < n;
  const int tc = min(t, n - 1);
  const unsigned G = gridDim.x;
  Shared sh;
  {
    using lc = HH_LDS char;
    lc* p = (lc*)smem;
    auto take = [&](size_t bytes) {
      lc* q = p;
      p += (bytes + 15) / 16 * 16;
      return q;
    };
    sh.U = (l2*)take(sizeof(double2) * (size_t)R1 * 3 * n);
    sh.zrow = (l2*)take(sizeof(double2) * n);
    sh.H = (l2*)take(sizeof(double2) * (size_t)R * R1);
    sh.Gr = (l2*)take(sizeof(double2) * 2 * (size_t)R);
    sh.S = (l2*)take(sizeof(double2) * R1);
    sh.coef = (l2*)take(sizeof(double2) * R1);
    sh.vs = (l1*)take(sizeof(double) * R1);
    sh.ss = (l1*)take(sizeof(double) * R1);
    sh.h0s = (l1*)take(sizeof(double) * R);
    sh.red = (l1*)take(2 * sizeof(double) * (kSmallThreads + kWave));
    sh.sum = (l1*)take(sizeof(double) * kPStride);
    sh.ctl = (li*)take(sizeof(int) * 4);
  }
  auto Urow = [&](int k, int r) -> l2* { return sh.U + ((size_t)k * 3 + r) * n; };
  const double2 z2 = make_double2(0.0, 0.0);
  ArArgs ar;
  ar.part = a.part;
  ar.fsum = a.part + 2 * (size_t)G * kPStride;
  ar.words = a.bar;

  // operator coefficients of this thread's point (stencil.hip's formulas; row g, column t)
  const double2 AW = a.tab_i[tc], AE = a.tab_i[n + tc], R1c = a.tab_i[2 * n + tc];
  const double2 R2 = a.tab_j[4 * g], BS = a.tab_j[4 * g + 1], BN = a.tab_j[4 * g + 2];
  const double2 OM = a.tab_j[4 * g + 3];
  const double ic = CONSTC ? a.invc2_const : a.invc2[(size_t)g * n + tc];
  const double2 W = cmul(AW, R2);
  const double2 E = cmul(AE, R2);
  const double2 S = cmul(BS, R1c);
  const double2 N = cmul(BN, R1c);
  const double2 M = cscale(cmul(OM, R1c), ic);
  const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
  const double2 D = csub(M, sum4);

  // u_0 = the (unnormalised) V[0] = M r of the regular cycle, own and ghost rows
  for (int r = 0; r < 3; ++r) {
    const int gr = g - 1 + r;
    const double2 u0 = a.v0[(size_t)min(max(gr, 0), n - 1) * n + tc];
    if (act) Urow(0, r)[t] = csel(gr >= 0 && gr < n, u0, z2);
  }
  if (t == 0) {
    sh.vs[0] = a.g.vscale[0];
    sh.ss[0] = a.g.vscale[0];
    const double2 s0 = a.g.S[0];
    for (int k = 0; k < R1; ++k) sh.S[k] = csel(k == 0, s0, z2);
    sh.ctl[0] = sh.ctl[1] = sh.ctl[2] = sh.ctl[3] = 0;
  }
  __syncthreads();

  unsigned epoch = 0;
  // optional phase timing (workgroup 0, thread 0; s_memrealtime ticks): 0 stencil + partial
  // sums, 1 all-reduce, 2 (unused), 3 coefficients, 4 basis update + Givens
  const bool prof = a.phase_ticks != nullptr && g == 0 && t == 0;
  unsigned long long tk[5] = {0, 0, 0, 0, 0};
  unsigned long long tprev = prof ? wall_clock64() : 0;
  auto tick = [&](int ph) {
    if (prof) {
      const unsigned long long now = wall_clock64();
      tk[ph] += now - tprev;
      tprev = now;
    }
  };
  bool stopped = false;
  for (int j = 0; j <= a.stop_col; ++j) {
    const int K = j + 1;
    const int cols = 2 * K + 2;
    // z = M A (s_j u_j) on the own row (zero Dirichlet rows beyond the grid are zero ghosts)
    // (by-value selects of loads from clamped columns: a select of lvalues would become a
    // select of addresses, i.e. flat loads)
    const double2 uC = csel(act, Urow(j, 1)[tc], z2);
    const double2 uW = csel(act && t > 0, Urow(j, 1)[max(tc - 1, 0)], z2);
    const double2 uE = csel(act && t < n - 1, Urow(j, 1)[min(tc + 1, n - 1)], z2);
    const double2 uS = csel(act, Urow(j, 0)[tc], z2);
    const double2 uN = csel(act, Urow(j, 2)[tc], z2);
    double2 Au = cmul(S, uS);
    Au = cfma(W, uW, Au);
    Au = cfma(D, uC, Au);
    Au = cfma(E, uE, Au);
    Au = cfma(N, uN, Au);
    const double sj = sh.ss[j];
    const double2 z = csel(act, JAC ? cscale(cdiv(Au, D), sj) : cscale(Au, sj), z2);
    // hand the z row to the neighbours (sc1 stores); keep it in LDS for the partial sums
    const int par = epoch & 1;
    double* zout = a.zbuf + ((size_t)par * n + g) * 2 * n;
    if (act) {
      st_sc1(zout + 2 * t, z.x);
      st_sc1(zout + 2 * t + 1, z.y);
      sh.zrow[t] = z;
    }
    __syncthreads();
    // partial sums of the own row: K + 2 quantities (conj(u_k) z, k < K; |z|^2; |u_j|^2), each
    // split over `seg` threads taking contiguous point ranges, added in segment order
    {
      const int nq = K + 2;
      const int seg = max(1, min(nt / nq, 16));
      const int q = t / seg, sgi = t % seg;
      const int len = (n + seg - 1) / seg;
      const int p0 = sgi * len, p1 = min(n, p0 + len);
      double2 acc = z2;
      if (q < nq) {
        const l2* uk = Urow(min(q, j), 1);
        for (int p = p0; p < p1; ++p) {
          const double2 zp = sh.zrow[p];
          const double2 up = uk[p];
          if (q < K) acc = cfma_conj(up, zp, acc);
          else if (q == K) acc.x = fma(zp.x, zp.x, fma(zp.y, zp.y, acc.x));
          else acc.x = fma(up.x, up.x, fma(up.y, up.y, acc.x));
        }
        sh.red[2 * t] = acc.x;
        sh.red[2 * t + 1] = acc.y;
      }
      __syncthreads();
      if (t < nq) {
        double2 d = z2;
        for (int i = 0; i < seg; ++i)
          d = cadd(d, make_double2(sh.red[2 * (t * seg + i)], sh.red[2 * (t * seg + i) + 1]));
        double* pr = ar.part + ((size_t)par * G + g) * kPStride;
        if (t < K) {
          st_sc1(pr + 2 * t, d.x);
          st_sc1(pr + 2 * t + 1, d.y);
        } else if (t == K) {
          st_sc1(pr + 2 * K, d.x);
        } else {
          st_sc1(pr + 2 * K + 1, j > 0 ? d.x : 0.0);
        }
      }
    }
    tick(0);
    epoch++;
    // the neighbours' z rows are loaded after the all-reduce (whose flag orders them)
    if (!allreduce_rows(ar, par, epoch, cols, sh.sum, sh.red, sh.ctl)) return;
    tick(1);
    const int glo = min(max(g - 1, 0), n - 1), ghi = min(g + 1, n - 1);
    const double* zlo = a.zbuf + ((size_t)par * n + glo) * 2 * n + 2 * tc;
    const double* zhi = a.zbuf + ((size_t)par * n + ghi) * 2 * n + 2 * tc;
    const double2 zl = make_double2(ld_sc1(zlo), ld_sc1(zlo + 1));
    const double2 zh = make_double2(ld_sc1(zhi), ld_sc1(zhi + 1));
    // the lagged-normalisation step (krylov.hip gmres_lag_kernel), split: 1/|u_j| and the
    // update coefficients first (one thread per basis vector) ...
    const double vj = j >= 1 ? 1.0 / sqrt(sh.sum[2 * K + 1]) : sh.vs[0];
    if (t <= j) {
      const double vk = t == j ? vj : sh.vs[t];
      const double2 d = make_double2(sh.sum[2 * t], sh.sum[2 * t + 1]);
      sh.coef[t] = cscale(cscale(d, vk), vk);  // krylov.hip update_kernel's coefficient
      // column j of H (gmres_lag_kernel step (c)); the entries are untouched by the finishing
      // of column j-1 below
      sh.H[(size_t)j * R1 + t] = cscale(cscale(d, vk), vj / sh.ss[j]);
    }
    __syncthreads();
    tick(3);
    if (t < nrow) {
      // ... then u_{j+1} = z - sum_k c_k u_k on the own row and both ghost rows (neighbours'
      // z from the all-reduce's round; beyond the grid the ghost stays zero)
      if (act) {
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const int gr = g - 1 + r;
          double2 w = r == 0 ? zl : (r == 1 ? z : zh);
          for (int k = 0; k < K; ++k) w = csub(w, cmul(sh.coef[k], Urow(k, r)[t]));
          Urow(j + 1, r)[t] = csel(gr >= 0 && gr < n, w, z2);
        }
      }
    } else if (t == book) {
      // ... while the bookkeeping lane completes column j-1 (its subdiagonal from |u_j|,
      // rotations, presid, exit test) and starts column j
      bool stop = false;
      if (j >= 1) {
        const int col = j - 1;
        stop = finish_column(sh, a, col, (1.0 / vj) * sh.vs[col] / sh.ss[col], vj);
      }
      if (!stop) {
        sh.vs[j] = vj;
        const double f = vj / sh.ss[j];
        const double w2 = sh.sum[2 * K];
        double rest = w2;
        for (int k = 0; k <= j; ++k) {
          const double vk = k == j ? vj : sh.vs[k];
          rest -= cabs2(make_double2(sh.sum[2 * k], sh.sum[2 * k + 1])) * vk * vk;
        }
        sh.h0s[j] = sqrt(w2) * f;
        sh.ss[j + 1] = 1.0 / sqrt(fmax(rest, fmax(w2 * 1e-28, 1e-300)));
      }
      sh.ctl[0] = stop ? 1 : 0;
    }
    __syncthreads();
    tick(4);
    if (sh.ctl[0]) {
      stopped = true;
      break;
    }
  }
  if (prof)
    for (int q = 0; q < 5; ++q) a.phase_ticks[q] += tk[q];
  if (!stopped) {
    // the cycle's last column needs |u_{stop_col+1}|: one more reduction round
    const int last = a.stop_col + 1;
    const int par = epoch & 1;
    if (t == 0) {
      const l2* ul = Urow(last, 1);
      double s = 0.0;
      for (int p = 0; p < n; ++p) s = fma(ul[p].x, ul[p].x, fma(ul[p].y, ul[p].y, s));
      st_sc1(ar.part + ((size_t)par * G + g) * kPStride, s);
    }
    epoch++;
    if (!allreduce_rows(ar, par, epoch, 1, sh.sum, sh.red, sh.ctl)) return;
    if (t == 0) {
      const double sg = sqrt(sh.sum[0]);
      const int col = a.stop_col;
      finish_column(sh, a, col, sg * sh.vs[col] / sh.ss[col], 1.0 / sg);
    }
    __syncthreads();
  }
  // triangular solve (krylov.hip gmres_solve_kernel) on lane 0, then x += sum_k y_k v_k
  const int col = sh.ctl[1];
  if (t == 0) {
    auto Hc = [&](int c, int k) -> l2& { return sh.H[(size_t)c * R1 + k]; };
    if (Hc(col, col).x == 0.0 && Hc(col, col).y == 0.0) sh.S[col] = z2;
    double2 y[kMaxProj];
    for (int k = 0; k <= col; ++k) y[k] = sh.S[k];
    for (int k = col; k > 0; --k) {
      if (y[k].x != 0.0 || y[k].y != 0.0) {
        y[k] = cdiv_smith(y[k], Hc(k, k));
        const double2 tt = y[k];
        for (int m = 0; m < k; ++m) y[m] = csub(y[m], cmul(tt, Hc(k, m)));
      }
    }
    if (y[0].x != 0.0 || y[0].y != 0.0) y[0] = cdiv_smith(y[0], Hc(0, 0));
    for (int k = 0; k <= col; ++k) sh.coef[k] = cscale(y[k], sh.vs[k]);
    if (g == 0) {
      a.g.ctrl[1] = col;
      a.g.ctrl[0] = 1;
    }
  }
  __syncthreads();
  if (act) {
    double2 acc = z2;
    for (int k = 0; k <= col; ++k) acc = cfma(sh.coef[k], Urow(k, 1)[t], acc);
    double2* xp = a.x + (size_t)g * n + t;
    *xp = cadd(*xp, acc);
  }
}

}  // namespace

size_t small_cycle_lds_bytes(int n, int restart) {
  const size_t R1 = restart + 1;
  auto al = [](size_t b) { return (b + 15) / 16 * 16; };
  return al(16 * R1 * 3 * n) + al(16 * (size_t)n) + al(16 * (size_t)restart * R1) +
         al(32 * (size_t)restart) + 2 * al(16 * R1) + 2 * al(8 * R1) + al(8 * (size_t)restart) +
         al(16 * (size_t)(kSmallThreads + kWave)) + al(8 * kPStride) + al(16);
}

size_t small_cycle_scratch_doubles(int n) {
  // z rows [2][n][2n], then the all-reduce rows [2][n][kPStride] and sums [2][kPStride]
  return 2 * (size_t)n * 2 * n + 2 * (size_t)kPStride * (n + 1);
}

bool small_cycle_eligible(int n, int restart) {
  return n >= 1 && n <= kSmallThreads && restart >= 1 && restart < kMaxProj &&
         small_cycle_lds_bytes(n, restart) <= (size_t)150 * 1024;
}

template <bool C, bool J>
void launch_one(const SmallCycleArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t s) {
  // dynamic LDS above 64 KB (gfx950 has 160 KB per CU) must be allowed per kernel, once
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&gmres_small_cycle_kernel<C, J>),
      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)attr;
  hipLaunchKernelGGL((gmres_small_cycle_kernel<C, J>), grid, block, lds, s, a);
}

void launch_small_cycle(const SmallCycleArgs& a, bool const_c, bool jacobi, hipStream_t s) {
  const int threads = (a.n + kWave - 1) / kWave * kWave + kWave;  // + the bookkeeping wave
  const size_t lds = small_cycle_lds_bytes(a.n, a.restart);
  const dim3 grid(a.n), block(threads);
  if (const_c) {
    if (jacobi) launch_one<true, true>(a, grid, block, lds, s);
    else launch_one<true, false>(a, grid, block, lds, s);
  } else {
    if (jacobi) launch_one<false, true>(a, grid, block, lds, s);
    else launch_one<false, false>(a, grid, block, lds, s);
  }
}

}  // namespace hh
