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
#include "hh_cycle.hpp"

#include <algorithm>
#include <cstdlib>

namespace hh {
namespace {

template <bool CONSTC, bool JAC>
__global__ __launch_bounds__(kSmallBlock) void gmres_small_cycle_kernel(SmallCycleArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int n = a.n, R1 = a.restart + 1;
  const int g = blockIdx.x, t = threadIdx.x, nt = blockDim.x;
  const bool act = t < n;
  const int tc = min(t, n - 1);
  // row-split mode (block of >= 3 npad threads): thread (lrow, lcol) updates basis row lrow
  // (0 ghost g-1, 1 own, 2 ghost g+1) at column lcol
  const int npad = (n + kWave - 1) / kWave * kWave;
  const bool split = nt >= 3 * npad;
  const int lrow = t / npad, lcol = min(t - lrow * npad, n - 1);
  const bool ract = split && lrow < 3 && t - lrow * npad < n;
  const int G = n;  // row workgroups; workgroup n keeps the Givens books
  const bool prof = a.phase_ticks != nullptr && blockIdx.x == 0 && threadIdx.x == 0;
  const unsigned long long t_launch = prof ? wall_clock64() : 0;
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
    sh.H = (l2*)take(sizeof(double2) * (size_t)a.restart * R1);
    sh.Gr = (l2*)take(sizeof(double2) * 2 * (size_t)a.restart);
    sh.S = (l2*)take(sizeof(double2) * R1);
    sh.coef = (l2*)take(sizeof(double2) * R1);
    sh.vs = (l1*)take(sizeof(double) * R1);
    sh.ss = (l1*)take(sizeof(double) * R1);
    sh.h0s = (l1*)take(sizeof(double) * a.restart);
    sh.red = (l1*)take(sizeof(double) * (kRedRuns + kRuns));
    sh.sum = (l1*)take(sizeof(double) * kPStride);
    sh.ctl = (li*)take(sizeof(int) * 4);
    sh.gv = (l1*)take(sizeof(double) * 2);
    sh.st = (l1*)take(sizeof(double) * 4 * (size_t)a.restart);
    sh.tk = (HH_LDS unsigned long long*)take(sizeof(unsigned long long) * 16);
  }
  if (!coresidency_gate(a, G + 1, sh.ctl + 3)) return;
  auto Urow = [&](int k, int r) -> l2* { return sh.U + ((size_t)k * 3 + r) * n; };
  const double2 z2 = make_double2(0.0, 0.0);
  ArArgs ar;
  ar.part = a.part;
  ar.sums = a.sums;
  ar.timeout = a.timeout_word;
  ar.seq = a.seq;
  ar.G = G;
  auto raise_timeout = [&] {
    if (t == 0)
      __hip_atomic_store((gu32*)a.timeout_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  // Up to a.cycles restart cycles in this launch (one cooperative launch per host batch): cycle
  // `cyc` tags its granules with seq + cyc and reports into its own slot of the host mapping.
  // Between cycles, what the next launch would have read from global memory after the kernel
  // boundary travels as tagged granules instead: the restart-loop state (workgroup 0's decisions,
  // `obuf`) and the neighbours' rows of the new V[0] = M r (`mbuf`); the own row, x and |M r|^2
  // is kept.  Per-point state (coefficients, x, b, the own row of V[0]) is reloaded every cycle
  // (this thread wrote x and V[0] itself): nothing but |M r|^2 stays live across cycles.
  if (g == G) {  // the Givens workgroup: its first wave keeps the books of every cycle
    if (t >= kWave) return;
    for (int cyc = 0; cyc < a.cycles; ++cyc) {
      CycleView cv = cycle_view(a, cyc);
      const CycleHead hd = cycle_head<true>(a, cv, cyc);
      if (hd.bad) {
        raise_timeout();
        return;
      }
      if (hd.quit) return;  // (row workgroup 0 marks the skipped slots)
      cv.mn2 = hd.mn2;
      if (!givens_role(sh, a, cv, hd.stop_col, hd.ptol)) {  // (wave-uniform)
        raise_timeout();
        return;
      }
      const unsigned long long ts = a.phase_ticks != nullptr ? wall_clock64() : 0;
      solve_and_publish(sh, a, cv);
      givens_tail_tick(a, ts);
    }
    return;
  }
  double mn2 = 0.0;
  // scipy's restart-loop state (iterative.py's outer loop): ptol, ptol_max_factor, inner
  // iterations so far, done -- from `outer` at launch, then advanced by every row thread
  double rs_ptol = a.ptol, rs_pmf = 1.0, rs_inner = 0.0;
  bool rs_done = false;
  if (a.outer) {
    rs_ptol = a.outer[0];
    rs_pmf = a.outer[1];
    rs_inner = a.outer[3];
    rs_done = a.outer[6] != 0.0;
  }
  for (int cyc = 0; cyc < a.cycles; ++cyc) {
  const CycleView cv = cycle_view(a, cyc);
  ar.seq = cv.seq;
  // this cycle's stop column from the restart loop's state, which every row thread carries
  // itself (ptol only matters to the Givens workgroup, which polls it) (the same decisions from the same reduced numbers in the same order
  // everywhere: no hand-off on the critical path between cycles)
  if (cyc == 0) mn2 = *a.mnorm2;
  if (rs_done || *a.timeout_word != 0u) {  // the solve finished earlier: slots skipped
    if (g == 0 && t == 0)
      for (int q = cyc; q < a.cycles; ++q)
        reinterpret_cast<int*>(a.report + (size_t)q * kRedDoubles + kRedCtrl)[0] = 2;
    return;
  }
  int stop_col = a.stop_col;
  if (a.outer && a.outer[5] != 0.0) {  // legacy: maxiter caps the inner iterations
    const double left = a.outer[4] - rs_inner;
    stop_col = left >= (double)a.restart ? a.restart - 1 : (int)left - 1;
  }

  // operator coefficients of this thread's point (stencil.hip's formulas; row g, column t)
  const double2* tab_i = a.tab_i;
  const double2* tab_j = a.tab_j;
  const double* invc2 = a.invc2;
  const double2* bvec = a.b;
  const double2 AW = tab_i[tc], AE = tab_i[n + tc], R1c = tab_i[2 * n + tc];
  const double2 R2 = tab_j[4 * g], BS = tab_j[4 * g + 1], BN = tab_j[4 * g + 2];
  const double2 OM = tab_j[4 * g + 3];
  const double ic = CONSTC ? a.invc2_const : invc2[(size_t)g * n + tc];
  const double2 W = cmul(AW, R2);
  const double2 E = cmul(AE, R2);
  const double2 S = cmul(BS, R1c);
  const double2 N = cmul(BN, R1c);
  const double2 M = cscale(cmul(OM, R1c), ic);
  const double2 sum4 = cadd(cadd(cadd(W, E), S), N);
  const double2 D = csub(M, sum4);
  // this point's x and b, for the cycle's tail (x += V y, r = b - A x): loaded now, off the tail's
  // critical path (only this thread writes x[g][t])
  const double2 x_old = a.x[(size_t)g * n + tc];
  const double2 b_pt = bvec[(size_t)g * n + tc];

  // u_0 = the (unnormalised) V[0] = M r of the regular cycle, own and ghost rows: from global
  // memory in the launch's first cycle, afterwards the neighbours' rows from their tagged
  // granules (the own row: this thread's own store of the previous cycle)
  for (int r = 0; r < 3; ++r) {
    const int gr = g - 1 + r;
    if (cyc > 0 && r != 1) continue;
    const double2 u0 = a.v0[(size_t)min(max(gr, 0), n - 1) * n + tc];
    if (act) Urow(0, r)[t] = csel(gr >= 0 && gr < n, u0, z2);
  }
  bool mok = true;
  if (cyc > 0 && act) {
    const unsigned mtag = gran_tag(cv.seq - 1, 0xfe);
    double lo_x = 0.0, lo_y = 0.0, hi_x = 0.0, hi_y = 0.0;
    if (g > 0) {
      const unsigned long long* p = a.mbuf + (size_t)(g - 1) * 4 * n + 4 * t;
      mok = ld_gran(p, mtag, &lo_x) && ld_gran(p + 2, mtag, &lo_y);
    }
    if (g < n - 1 && mok) {
      const unsigned long long* p = a.mbuf + (size_t)(g + 1) * 4 * n + 4 * t;
      mok = ld_gran(p, mtag, &hi_x) && ld_gran(p + 2, mtag, &hi_y);
    }
    Urow(0, 0)[t] = make_double2(lo_x, lo_y);
    Urow(0, 2)[t] = make_double2(hi_x, hi_y);
  }
  // gmres_start_kernel's scaling of V[0], on every workgroup
  const double vs0 = 1.0 / sqrt(mn2);
  if (t == 0) {
    sh.vs[0] = vs0;
    sh.ctl[0] = 0;
  }
  if (__syncthreads_or(!mok)) {
    raise_timeout();
    return;
  }

  unsigned epoch = 0;
  // optional phase timing (workgroup 0, thread 0; s_memrealtime ticks): 0 stencil + z hand-off,
  // 5 partial sums, 6 their publication, 1 all-reduce, 3 the neighbours' z (+ the verdict),
  // 2 basis update (coefficients and the next scale inline), 4 the closing barrier
  // sh.tk: [0, 8) loop phases, [8, 12) head / tail spans, [12] the previous tick, [13] the
  // all-reduce's first hop (publish -> column 0 reduced here), [14] shader clock at loop start
  if (prof) {
    const unsigned long long now = wall_clock64();
    for (int q = 0; q < 16; ++q) sh.tk[q] = 0;
    sh.tk[8] = cyc == 0 ? now - t_launch : 0;
    sh.tk[12] = now;
    sh.tk[14] = __builtin_amdgcn_s_memtime();
  }
  auto tick = [&](int ph) {
    if (prof) {
      const unsigned long long now = wall_clock64();
      sh.tk[ph] += now - sh.tk[12];
      sh.tk[12] = now;
    }
  };
  bool stopped = false;
  double sj = vs0;  // scale of this iteration's SpMV input (every row thread holds it)
  for (int j = 0; j <= stop_col; ++j) {
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
    const double2 z = csel(act, JAC ? cscale(cdiv(Au, D), sj) : cscale(Au, sj), z2);
    // hand the z row to the neighbours (tagged granules: no drain, they poll them); keep it in
    // LDS for the partial sums
    const int par = epoch & 1;
    const unsigned rtag = gran_tag(cv.seq, epoch + 1);
    unsigned long long* zout = a.zbuf + ((size_t)par * n + g) * 4 * n;
    if (act) {
      st_gran(zout + 4 * t, rtag, z.x);
      st_gran(zout + 4 * t + 2, rtag, z.y);
      sh.zrow[t] = z;
    }
    __syncthreads();
    tick(0);
    // partial sums of the own row: K + 2 quantities (conj(u_k) z, k < K; |z|^2; |u_j|^2), each
    // split over `seg` threads taking every seg-th point (neighbouring lanes read neighbouring
    // points: no LDS bank conflicts), the segments added in segment order.  Branch-free: for
    // |z|^2 and |u_j|^2 both factors are the same vector (cfma_conj(v, v) = |v|^2 + 0 i).
    {
      const int nq = K + 2;
      const int seg = max(1, min(min(nt / nq, 16), kRedRuns / (2 * nq)));  // (sh.red holds them)
      const int q = t / seg, sgi = t % seg;
      const int len = (n - sgi + seg - 1) / seg;
      double2 acc = z2;
      if (q < nq) {
        const l2* uk = Urow(min(q, j), 1);
        const bool zz = q == K, uu = q == K + 1;
        for (int i0 = 0; i0 < len; i0 += kBatch) {
          double2 zp[kBatch], up[kBatch];
#pragma unroll
          for (int i = 0; i < kBatch; ++i) {  // loads in flight together
            const int pi = min(sgi + seg * (i0 + i), n - 1);
            zp[i] = sh.zrow[pi];
            up[i] = uk[pi];
          }
#pragma unroll
          for (int i = 0; i < kBatch; ++i) {
            const bool in = i0 + i < len;
            const double2 zv = csel(in, uu ? up[i] : zp[i], z2);
            const double2 uv = csel(in, zz ? zp[i] : up[i], z2);
            acc = cfma_conj(uv, zv, acc);
          }
        }
        sh.red[2 * (sgi * nq + q)] = acc.x;  // [segment][quantity]
        sh.red[2 * (sgi * nq + q) + 1] = acc.y;
      }
      __syncthreads();
      tick(5);
      // granules of the row's partial sums
      const unsigned tag = rtag;
      if (t < nq) {
        double2 d = z2;
        for (int i0 = 0; i0 < seg; i0 += kBatch) {
          double2 v[kBatch];
#pragma unroll
          for (int i = 0; i < kBatch; ++i) {
            const int ii = min(i0 + i, seg - 1) * nq + t;
            v[i] = make_double2(sh.red[2 * ii], sh.red[2 * ii + 1]);
          }
#pragma unroll
          for (int i = 0; i < kBatch; ++i)
            if (i0 + i < seg) d = cadd(d, v[i]);
        }
        unsigned long long* pr = ar.part + ((size_t)par * G + g) * 2 * kPStride;
        if (t < K) {
          st_gran(pr + 4 * t, tag, d.x);
          st_gran(pr + 4 * t + 2, tag, d.y);
        } else if (t == K) {
          st_gran(pr + 4 * K, tag, d.x);
        } else {
          st_gran(pr + 4 * K + 2, tag, j > 0 ? d.x : 0.0);
        }
      }
    }
    tick(6);
    epoch++;
    // the neighbours' z rows of this round: the eight granules are requested now, before the
    // all-reduce (their latency hides behind it), and checked after it -- as a rule they have
    // arrived (the all-reduce needed the neighbours' partial sums, stored after them); any that
    // have not are polled until they carry the round's tag
    // (row-split mode: the ghost-row threads load their own row's four granules only)
    const int glo = min(max(g - 1, 0), n - 1), ghi = min(g + 1, n - 1);
    const bool zwait = split ? ract && lrow != 1 : act;
    const int zc = split ? lcol : tc;
    const unsigned long long* zlo =
        a.zbuf + ((size_t)par * n + (split && lrow == 2 ? ghi : glo)) * 4 * n + 4 * zc;
    const unsigned long long* zhi = a.zbuf + ((size_t)par * n + ghi) * 4 * n + 4 * zc;
    unsigned long long zg[8];
    auto load_ghosts = [&] {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        zg[i] = __hip_atomic_load((gu64*)(zlo + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        zg[4 + i] = split ? zg[i]
                          : __hip_atomic_load((gu64*)(zhi + i), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
      }
    };
    if (zwait) load_ghosts();
    // (and thread 0 the Givens workgroup's verdict on column j-2, checked after the all-reduce)
    const unsigned long long* vp = a.verdict + 2 * max(j - 2, 0);
    unsigned long long vg[2] = {0, 0};
    if (t == 0 && j >= 2) {
      vg[0] = __hip_atomic_load((gu64*)vp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      vg[1] = __hip_atomic_load((gu64*)(vp + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    unsigned long long t_red = 0;
    const unsigned long long t_ar = prof ? sh.tk[12] : 0;
    if (!allreduce_rows(ar, par, epoch, cols, sh.sum, sh.red, prof ? &t_red : nullptr)) return;
    if (prof) sh.tk[13] += t_red - t_ar;
    tick(1);
    double2 zl = z2, zh = z2;
    bool zok = true;
    if (zwait) {
      unsigned spins = 0;
      for (;;) {
        bool all = true;
#pragma unroll
        for (int i = 0; i < 8; ++i) all = all && (unsigned)(zg[i] >> 32) == rtag;
        if (all) break;
        if (++spins > kSpinLimit) {
          zok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        load_ghosts();
      }
      auto dbl = [](unsigned long long hi, unsigned long long lo) {
        return __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
      };
      zl = make_double2(dbl(zg[0], zg[1]), dbl(zg[2], zg[3]));
      zh = make_double2(dbl(zg[4], zg[5]), dbl(zg[6], zg[7]));
    }
    // the Givens workgroup's verdict on column j-2 (published two iterations ago, as a rule;
    // every workgroup polls the same granule, so all stop at the same iteration)
    if (t == 0 && j >= 2) {
      const unsigned vtag = gran_tag(cv.seq, j - 1);
      double v = 0.0;
      if ((unsigned)(vg[0] >> 32) == vtag && (unsigned)(vg[1] >> 32) == vtag)
        v = __longlong_as_double((long long)((vg[0] << 32) | (vg[1] & 0xffffffffull)));
      else if (!ld_gran(vp, vtag, &v))
        zok = false;
      sh.ctl[0] = v != 0.0 ? 1 : 0;
    }
    // the lagged-normalisation step (krylov.hip gmres_lag_kernel / update_kernel) without a
    // barrier of its own: every row thread forms the coefficients c_k = d_k / sigma_k^2 and the
    // next input's Pythagorean scale (the same expressions, in the same order, on every thread)
    const double vj = j >= 1 ? 1.0 / sqrt(sh.sum[2 * K + 1]) : vs0;
    const double w2 = sh.sum[2 * K];
    double rest = w2;
    tick(3);
    if (split) {
      // one row per thread group: the same terms in the same order as the three-row form below
      // (identical bits), a quarter of the LDS loads and FMAs per thread
      if (ract) {
        constexpr int kStep = 8;
        double2 w = lrow == 1 ? sh.zrow[lcol] : zl;
        for (int k0 = 0; k0 < K; k0 += kStep) {
          double2 cv[kStep], uv[kStep];
          double tv[kStep], tw[kStep];
#pragma unroll
          for (int i = 0; i < kStep; ++i) {
            const int k = min(k0 + i, K - 1);
            const double vk = k == j ? vj : sh.vs[k];
            const double2 d = make_double2(sh.sum[2 * k], sh.sum[2 * k + 1]);
            cv[i] = cscale(cscale(d, vk), vk);
            tv[i] = cabs2(d) * vk;
            tw[i] = vk;
            uv[i] = Urow(k, lrow)[lcol];
          }
#pragma unroll
          for (int i = 0; i < kStep; ++i)
            if (k0 + i < K) {
              rest = fma(-tv[i], tw[i], rest);  // (|d_k|^2 v_k^2, explicitly fused)
              w = csub(w, cmul(cv[i], uv[i]));
            }
        }
        const int gr = g - 1 + lrow;
        Urow(j + 1, lrow)[lcol] = csel(gr >= 0 && gr < n, w, z2);
      }
    } else if (act) {
      // u_{j+1} = z - sum_k c_k u_k on the own row and both ghost rows (neighbours' z from the
      // all-reduce's round; beyond the grid the ghost stays zero); the three rows' chains
      // interleaved, the loads of kStep basis vectors in flight together, terms in k order
      constexpr int kStep = 4;
      double2 w[3] = {zl, z, zh};
      for (int k0 = 0; k0 < K; k0 += kStep) {
        double2 cv[kStep], uv[3][kStep];
        double tv[kStep], tw[kStep];
#pragma unroll
        for (int i = 0; i < kStep; ++i) {
          const int k = min(k0 + i, K - 1);
          const double vk = k == j ? vj : sh.vs[k];
          const double2 d = make_double2(sh.sum[2 * k], sh.sum[2 * k + 1]);
          cv[i] = cscale(cscale(d, vk), vk);
          tv[i] = cabs2(d) * vk;
          tw[i] = vk;
#pragma unroll
          for (int r = 0; r < 3; ++r) uv[r][i] = Urow(k, r)[t];
        }
#pragma unroll
        for (int i = 0; i < kStep; ++i)
          if (k0 + i < K) {
            rest = fma(-tv[i], tw[i], rest);
#pragma unroll
            for (int r = 0; r < 3; ++r) w[r] = csub(w[r], cmul(cv[i], uv[r][i]));
          }
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int gr = g - 1 + r;
        Urow(j + 1, r)[t] = csel(gr >= 0 && gr < n, w[r], z2);
      }
    }
    if (t == 0) sh.vs[j] = vj;
    sj = 1.0 / sqrt(fmax(rest, fmax(w2 * 1e-28, 1e-300)));
    tick(2);
    if (__syncthreads_or(!zok)) {  // (a neighbour's z or the verdict never arrived)
      raise_timeout();
      return;
    }
    tick(4);
    if (sh.ctl[0]) {
      stopped = true;
      break;
    }
  }
  // shader-clock cycles over the loop (the effective clock: slot 7 / sum of slots); every
  // counter is written at the end of the launch (no global round trip inside the timed spans)
  if (prof) sh.tk[7] = __builtin_amdgcn_s_memtime() - sh.tk[14];
  auto tail_tick = [&](int slot) {  // head / tail spans (slots 8 .. 11, written at the end)
    if (prof) {
      const unsigned long long now = wall_clock64();
      sh.tk[slot] += now - sh.tk[12];
      sh.tk[12] = now;
    }
  };
  if (!stopped) {
    // the cycle's last column needs |u_{stop_col+1}|: one more reduction round (for the Givens
    // workgroup)
    const int last = stop_col + 1;
    const int par = epoch & 1;
    if (t < kWave) {  // (wave 0: strided partial sums, then the butterfly)
      const l2* ul = Urow(last, 1);
      double s = 0.0;
      for (int p = t; p < n; p += kWave) s = fma(ul[p].x, ul[p].x, fma(ul[p].y, ul[p].y, s));
      s = wave_sum_to_63(s);
      if (t == kWave - 1)
        st_gran(ar.part + ((size_t)par * G + g) * 2 * kPStride, gran_tag(cv.seq, epoch + 1), s);
    }
    epoch++;
    if (!allreduce_rows(ar, par, epoch, 1, sh.sum, sh.red)) return;
  }
  // the column the cycle solved for and y_k / sigma_k, from the Givens workgroup
  {
    const unsigned ytag = gran_tag(cv.seq, 0xff);
    bool ok = true;
    if (t == 0) {
      double c = 0.0, pr = 0.0;
      ok = ld_gran(a.ycoef + 4 * kMaxProj, ytag, &c);
      if (ok) ok = ld_gran(a.ycoef + 4 * kMaxProj + 2, ytag, &pr);
      const int cb = (int)c;
      sh.ctl[1] = cb & 63;
      sh.gv[0] = pr;
      sh.gv[1] = cb >= 64 ? 1.0 : 0.0;
    }
    if (__syncthreads_or(!ok)) {
      raise_timeout();
      return;
    }
    const int col = sh.ctl[1];
    if (t <= col) {
      double cx = 0.0, cy = 0.0;
      ok = ld_gran(a.ycoef + 4 * t, ytag, &cx) && ld_gran(a.ycoef + 4 * t + 2, ytag, &cy);
      sh.coef[t] = make_double2(cx, cy);
    }
    if (__syncthreads_or(!ok)) {
      raise_timeout();
      return;
    }
  }
  tail_tick(9);
  const int col = sh.ctl[1];
  double2 xn = z2;
  if (act) {
    double2 acc = z2;
    for (int k0 = 0; k0 <= col; k0 += kBatch) {  // (loads in flight together, k order)
      double2 cv[kBatch], uv[kBatch];
#pragma unroll
      for (int i = 0; i < kBatch; ++i) {
        const int k = min(k0 + i, col);
        cv[i] = sh.coef[k];
        uv[i] = Urow(k, 1)[t];
      }
#pragma unroll
      for (int i = 0; i < kBatch; ++i)
        if (k0 + i <= col) acc = cfma(cv[i], uv[i], acc);
    }
    xn = cadd(x_old, acc);
    a.x[(size_t)g * n + t] = xn;
  }
  // The next cycle's start (runtime.cpp residual): r = b - A x, V[0] = M r, |r|^2 and |M r|^2,
  // in two more rounds -- the x rows to the neighbours (tagged granules), then a two-column
  // all-reduce -- instead of two launches and a copy after this one.
  const unsigned xtag = gran_tag(cv.seq, epoch + 1);
  if (act) {
    unsigned long long* xo = a.xbuf + (size_t)g * 4 * n + 4 * t;
    st_gran(xo, xtag, xn.x);
    st_gran(xo + 2, xtag, xn.y);
  }
  double2 xl = z2, xh = z2;
  bool xok = true;
  if (act) {
    const unsigned long long* xlo = a.xbuf + (size_t)min(max(g - 1, 0), n - 1) * 4 * n + 4 * tc;
    const unsigned long long* xhi = a.xbuf + (size_t)min(g + 1, n - 1) * 4 * n + 4 * tc;
    // the eight granules in flight together, polled until all carry the round's tag
    unsigned long long xg[8];
    unsigned spins = 0;
    for (;;) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        xg[i] = __hip_atomic_load((gu64*)(xlo + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        xg[4 + i] = __hip_atomic_load((gu64*)(xhi + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      bool all = true;
#pragma unroll
      for (int i = 0; i < 8; ++i) all = all && (unsigned)(xg[i] >> 32) == xtag;
      if (all) break;
      if (++spins > kSpinLimit) {
        xok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    auto dbl = [](unsigned long long hi, unsigned long long lo) {
      return __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
    };
    xl = make_double2(dbl(xg[0], xg[1]), dbl(xg[2], xg[3]));
    xh = make_double2(dbl(xg[4], xg[5]), dbl(xg[6], xg[7]));
    sh.zrow[t] = xn;
  }
  if (__syncthreads_or(!xok)) {
    raise_timeout();
    return;
  }
  tail_tick(10);
  double r2 = 0.0, m2 = 0.0;
  if (act) {
    const double2 xC = sh.zrow[tc];
    const double2 xW = csel(t > 0, sh.zrow[max(tc - 1, 0)], z2);
    const double2 xE = csel(t < n - 1, sh.zrow[min(tc + 1, n - 1)], z2);
    const double2 xS = csel(g > 0, xl, z2);
    const double2 xN = csel(g < n - 1, xh, z2);
    double2 Ax = cmul(S, xS);
    Ax = cfma(W, xW, Ax);
    Ax = cfma(D, xC, Ax);
    Ax = cfma(E, xE, Ax);
    Ax = cfma(N, xN, Ax);
    const double2 rr = csub(b_pt, Ax);
    const double2 mr = JAC ? cdiv(rr, D) : rr;
    a.v0[(size_t)g * n + t] = mr;
    if (cyc + 1 < a.cycles) {  // the next cycle's ghost rows of V[0]
      unsigned long long* mo = a.mbuf + (size_t)g * 4 * n + 4 * t;
      const unsigned mtag = gran_tag(cv.seq, 0xfe);
      st_gran(mo, mtag, mr.x);
      st_gran(mo + 2, mtag, mr.y);
    }
    r2 = cabs2(rr);
    m2 = cabs2(mr);
  }
  // row sums: per wave by DPP lane moves, then the waves in order
  {
    const double r2w = wave_sum_to_63(r2), m2w = wave_sum_to_63(m2);
    if ((t & (kWave - 1)) == kWave - 1) {
      sh.red[2 * (t / kWave)] = r2w;
      sh.red[2 * (t / kWave) + 1] = m2w;
    }
  }
  __syncthreads();
  const int par = epoch & 1;
  epoch++;
  if (t < 2) {
    double sacc = 0.0;
    for (int q = 0; q < (n + kWave - 1) / kWave; ++q) sacc += sh.red[2 * q + t];
    st_gran(ar.part + ((size_t)par * G + g) * 2 * kPStride + 2 * t, xtag, sacc);
  }
  if (!allreduce_rows(ar, par, epoch, 2, sh.sum, sh.red)) return;
  tail_tick(11);
  if (prof) {
    for (int q = 0; q < 12; ++q) a.phase_ticks[q] += sh.tk[q];
    a.phase_ticks[15] += sh.tk[13];
  }
  mn2 = sh.sum[1];  // (|M r|^2; = |r|^2 bit for bit without a preconditioner)
  // scipy's restart-loop decisions (the end of iterative.py's outer loop, exactly as runtime.cpp
  // hh_gmres takes them) for the next cycle, on every thread
  if (a.outer) {
    const double* o = a.outer;  // ([2] atol, [4] maxiter, [5] legacy: constant during the solve)
    const double presid = sh.gv[0];
    const double rn = sqrt(sh.sum[0]);
    rs_inner += (double)(col + 1);
    rs_done = (o[5] != 0.0 && rs_inner >= o[4]) || rn <= o[2] || sh.gv[1] != 0.0;
    if (!rs_done) {
      rs_pmf = presid <= rs_ptol ? fmax(a.eps, 0.25 * rs_pmf) : fmin(1.0, 1.5 * rs_pmf);
      rs_ptol = presid * fmin(rs_pmf, o[2] / rn);
    }
  } else {
    rs_done = true;  // (a single cycle as given)
  }
  if (g == 0 && t == 0) {
    a.red[4] = sh.sum[0];  // (device: the next cycle's |r|^2, |M r|^2)
    a.red[5] = sh.sum[1];
    cv.report[4] = sh.sum[0];  // (host: this cycle's report)
    cv.report[5] = sh.sum[1];
    if (a.outer) {  // for the launch queued behind this one, and the host
      double* o = a.outer;
      o[0] = rs_ptol;
      o[1] = rs_pmf;
      o[3] = rs_inner;
      o[6] = rs_done ? 1.0 : 0.0;
      cv.report[6] = o[6];
      cv.report[7] = o[0];
      if (cyc + 1 < a.cycles) {  // to the Givens workgroup's next cycle
        const unsigned otag = gran_tag(cv.seq, 0xfd);
        st_gran(a.obuf, otag, rs_ptol);
        st_gran(a.obuf + 2, otag, rs_inner);
        st_gran(a.obuf + 4, otag, rs_done ? 1.0 : 0.0);
        st_gran(a.obuf + 6, otag, sh.sum[1]);
      }
    }
    cv.ctrl[1] = col;
    cv.ctrl[0] = 1;
  }
  // (no barrier before the next cycle: its head writes only this thread's own LDS columns and
  // thread 0's sh.vs[0] / sh.ctl[0], which nothing in this tail reads after the last barrier)
  }  // cycles
}

}  // namespace

size_t small_cycle_lds_bytes(int n, int restart) {
  const size_t R1 = restart + 1;
  auto al = [](size_t b) { return (b + 15) / 16 * 16; };
  return al(16 * R1 * 3 * n) + al(16 * (size_t)n) + al(16 * (size_t)restart * R1) +
         al(32 * (size_t)restart) + 2 * al(16 * R1) + 2 * al(8 * R1) + al(8 * (size_t)restart) +
         al(8 * (size_t)(kRedRuns + kRuns)) + al(8 * kPStride) + al(16) + al(16) +
         al(32 * (size_t)restart) + al(8 * 16);
}

size_t small_cycle_scratch_doubles(int n) {
  // 8-byte granules: z rows [2][n][4n], x rows [n][4n], the all-reduce rows [2][n][2 kPStride],
  // the sums of every round [kSmallRounds][2 kPStride], verdicts [kMaxProj][2], y [kMaxProj+1][4],
  // the next cycle's V[0] rows [n][4n] and restart-loop state [8]
  return 12 * (size_t)n * n + 4 * (size_t)kPStride * n + 2 * (size_t)kPStride * kSmallRounds +
         2 * kMaxProj + 4 * (kMaxProj + 1) + 4 * (size_t)n * n + 8 +
         (kSmallThreads + 2) / 2 + 2;  // + the gate: arrival words (u32) and the decision
}

bool small_cycle_eligible(int n, int restart, int device_cus) {
  // n row workgroups + the Givens workgroup, one per CU (the LDS use allows no second)
  return n >= 1 && n <= kSmallThreads && n + 1 <= device_cus && restart >= 1 &&
         restart < kMaxProj && small_cycle_lds_bytes(n, restart) <= (size_t)150 * 1024;
}

template <bool C, bool J>
hipError_t launch_one(const SmallCycleArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t s) {
  // dynamic LDS above 64 KB (gfx950 has 160 KB per CU, the kernel's static LDS included) must
  // be allowed per kernel, once
  static const hipError_t attr = [] {
    const void* fn = reinterpret_cast<const void*>(&gmres_small_cycle_kernel<C, J>);
    hipFuncAttributes fa{};
    hipError_t e = hipFuncGetAttributes(&fa, fn);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                               160 * 1024 - (int)fa.sharedSizeBytes);
  }();
  if (attr != hipSuccess) {
    (void)hipGetLastError();  // (reported here, not by the next unrelated check)
    fail(HH_ERR_HIP, "small-grid GMRES cycle: cannot enable %zu B of dynamic LDS (%s)", lds,
         hipGetErrorString(attr));
  }
  // Plain launch: co-residency is checked by the kernel's own gate (coresidency_gate), which
  // refuses a grid that cannot be resident before any state changes.  HH_SMALL_COOP=1 launches
  // cooperatively instead (the runtime's own residency check; ~55 us per launch), for A/B timing.
  static const bool coop = knobs().small_coop == 1 && !under_profiler();
  if (!coop) {
    hipLaunchKernelGGL((gmres_small_cycle_kernel<C, J>), grid, block, lds, s, a);
    return hipGetLastError();
  }
  SmallCycleArgs arg = a;
  void* params[] = {&arg};
  const hipError_t e = hipLaunchCooperativeKernel(
      reinterpret_cast<const void*>(&gmres_small_cycle_kernel<C, J>), grid, block, params,
      (unsigned)lds, s);
  if (e != hipSuccess) (void)hipGetLastError();  // (reported by the caller, not a later check)
  return e;
}

hipError_t launch_small_cycle(const SmallCycleArgs& a, bool const_c, bool jacobi, hipStream_t s) {
  const int npad = (a.n + kWave - 1) / kWave * kWave;
  // at most 2 copies of the row's threads by default: 9.76-9.80 us/it at 128^2 against
  // 9.80-9.91 for 1 and 9.96-10.14 for 4 (the row-split update; block barriers of 8 waves)
  // (profiles/r02z_*); HH_SMALL_WIDE=c selects up to c copies, for A/B timing
  const int wide = (int)knobs().small_wide;
  const int threads = npad * std::max(1, std::min(wide, kSmallBlock / npad));
  const size_t lds = small_cycle_lds_bytes(a.n, a.restart);
  const dim3 grid(a.n + 1), block(threads);  // + the Givens workgroup
  if (const_c) return jacobi ? launch_one<true, true>(a, grid, block, lds, s)
                             : launch_one<true, false>(a, grid, block, lds, s);
  return jacobi ? launch_one<false, true>(a, grid, block, lds, s)
                : launch_one<false, false>(a, grid, block, lds, s);
}

}  // namespace hh
