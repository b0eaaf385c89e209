// Device helpers of the whole-cycle GMRES kernel (gmres_small.hip): tagged 8-byte granules (the
// data is the flag), the two-hop all-reduce of per-workgroup rows, the Givens workgroup's
// Hessenberg books and triangular solve, the co-residency gate, and the restart-loop state
// between the cycles of one launch.
#pragma once

#include "hh_internal.hpp"
#include "hh_complex.hpp"
#include "hh_error.hpp"
#include "hh_wave.hpp"

namespace hh {
namespace {

using gu32 = __attribute__((address_space(1))) unsigned;
using gu64 = __attribute__((address_space(1))) unsigned long long;

__device__ __forceinline__ double2 csel(bool c, double2 a, double2 b) {
  return make_double2(c ? a.x : b.x, c ? a.y : b.y);
}

constexpr int kSmallThreads = 256;    // grid rows at most (n <= 256)
// Block size: P copies of the row's npad threads (P = 2 by default, up to 4 = 512 / 128).  The
// stencil, x update and residual need one thread per column; the partial sums get P times the
// segments, and with P >= 3 the basis update gives each of the three rows (ghost, own, ghost) a
// thread group of its own (measured slower at 128^2: the block barriers of 8 waves).
constexpr int kSmallBlock = 512;
constexpr int kPStride = kSmallCols;  // partial-sum columns (global layout)
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
  l1* red;   // [kRedRuns + kRuns] segment sums of the partial sums, run sums of the reducer
  l1* sum;   // [PSTRIDE] reduced sums
  li* ctl;   // [4]: 0 stop, 1 last column, 2 abort
  l1* gv;    // [2]: presid and breakdown of the last finished column (Givens workgroup; then
             // workgroup 0, for the restart loop's decisions)
  HH_LDS unsigned long long* tk;  // [16] phase timing of workgroup 0's thread 0 (optional): kept
                                  // in LDS, not registers, so it costs the row path nothing
  l1* st;    // [R][4]: the columns' statuses (Givens workgroup), copied to the host-mapped
             // status_it only after y is published: a store to host memory holds the storing
             // wave's next vmcnt wait for a PCIe round trip (~3 us per column on the books)
};

// All-reduce of `cols` doubles per workgroup with NO counter and NO flag: every value travels
// as two 8-byte granules {tag, 32-bit half} (MI355X_MICROARCH.md's "the data is the flag" form
// for small payloads -- a granule is written by one 8-byte store, so a reader that sees the tag
// sees the half that came with it; nothing needs ordering or draining).  The tag is the launch's
// sequence number and the round (epoch), so granules of an earlier round or launch never match.
//  1. every workgroup has stored its row of partial sums as granules, part[par][g][.];
//  2. column c is reduced by workgroup c mod G, on its first wave: lane l polls the two
//     granules of rows l, l + 64, ... until all carry the round's tag, sums them in that order,
//     and the 64 lane sums are added by DPP lane moves in a fixed order (no barrier, no LDS);
//     the sum is stored as two granules;
//  3. every workgroup polls the `cols` sums' granules until tagged.
// Two hops (partials -> reducer -> everyone) and no serialised atomics.  The arithmetic order is
// fixed: identical sums on every workgroup and every run.  Rows and sums are double-buffered by
// `par`: a round's granules are only overwritten two rounds later, which no workgroup can reach
// before every workgroup has read them.  Returns false on timeout (every workgroup then leaves).
constexpr int kRuns = 32;
constexpr int kBatch = 8;  // LDS loads a thread keeps in flight in its reduction loops
constexpr int kRowsPerLane = (kSmallThreads + kWave - 1) / kWave;  // reducer rows per lane
// sh.red: [0, kRedRuns) the partial-sum segments of the caller, [kRedRuns, + kRuns) run sums
constexpr int kRedRuns = 2 * (kSmallThreads + kWave);
struct ArArgs {
  unsigned long long* part;  // [2][G][2 kPStride]
  unsigned long long* sums;  // [kSmallRounds][2 kPStride]: one slot per round (the Givens
                             // workgroup reads them at its own pace)
  unsigned* timeout;
  unsigned seq;
  int G;                     // participating (row) workgroups
};
__device__ __forceinline__ unsigned gran_tag(unsigned seq, unsigned epoch) {
  return (seq << 8) | (epoch & 0xffu);
}
__device__ __forceinline__ void st_gran(unsigned long long* p, unsigned tag, double v) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned long long tg = (unsigned long long)tag << 32;
  __hip_atomic_store((gu64*)p, tg | (u >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((gu64*)(p + 1), tg | (u & 0xffffffffull), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// polls the two granules of one double until both carry `tag`; false on timeout
__device__ __forceinline__ bool ld_gran(const unsigned long long* p, unsigned tag, double* v) {
  unsigned spins = 0;
  for (;;) {
    const unsigned long long hi =
        __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long lo =
        __hip_atomic_load((gu64*)(p + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((unsigned)(hi >> 32) == tag && (unsigned)(lo >> 32) == tag) {
      *v = __longlong_as_double((long long)((hi << 32) | (lo & 0xffffffffull)));
      return true;
    }
    if (++spins > kSpinLimit) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ bool allreduce_rows(const ArArgs& ar, int par, unsigned epoch, int cols, l1* out,
                               l1* red, unsigned long long* t_reduced = nullptr) {
  const int G = ar.G, g = blockIdx.x;
  const int t = threadIdx.x;
  const unsigned tag = gran_tag(ar.seq, epoch);
  bool ok = true;
  (void)red;
  for (int c = g; c < cols; c += G) {
    if (t < kWave) {
      // wave 0: lane l polls rows l, l + 64, ... (all granules in flight together) until
      // tagged, sums them in row order, then the 64 lane sums by DPP (fixed order, no barrier,
      // no LDS); lane 63 publishes the column's sum
      double s = 0.0;
      unsigned spins = 0;
      for (;;) {
        unsigned long long v[2 * kRowsPerLane];
#pragma unroll
        for (int i = 0; i < kRowsPerLane; ++i) {
          const int q = min(t + kWave * i, G - 1);
          const unsigned long long* p = ar.part + ((size_t)par * G + q) * 2 * kPStride + 2 * c;
          v[2 * i] = __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v[2 * i + 1] =
              __hip_atomic_load((gu64*)(p + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        bool all = true;
#pragma unroll
        for (int i = 0; i < kRowsPerLane; ++i)
          if (t + kWave * i < G)
            all = all && (unsigned)(v[2 * i] >> 32) == tag && (unsigned)(v[2 * i + 1] >> 32) == tag;
        if (all) {
#pragma unroll
          for (int i = 0; i < kRowsPerLane; ++i)
            if (t + kWave * i < G)
              s += __longlong_as_double(
                  (long long)((v[2 * i] << 32) | (v[2 * i + 1] & 0xffffffffull)));
          break;
        }
        if (++spins > kSpinLimit) {
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      s = wave_sum_to_63(s);
      if (t == kWave - 1) st_gran(ar.sums + (size_t)epoch * 2 * kPStride + 2 * c, tag, s);
      if (t_reduced && c == 0) *t_reduced = wall_clock64();  // (profiling: column 0 summed)
    }
  }
  if (t < cols) {
    double v = 0.0;
    ok = ld_gran(ar.sums + (size_t)epoch * 2 * kPStride + 2 * t, tag, &v) && ok;
    out[t] = v;
  }
  if (__syncthreads_or(!ok)) {
    if (t == 0)
      __hip_atomic_store((gu32*)ar.timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  return true;
}


// LAPACK zlartg main branch (krylov.hip), by value: each branch yields all three results (no
// output pointers -- a branch-selected store target would become a scratch slot)
struct Rot {
  double c;
  double2 s, r;
};
__device__ __forceinline__ Rot zlartg_s(double2 f, double2 g) {
  const bool gz = g.x == 0.0 && g.y == 0.0;
  const bool fz = f.x == 0.0 && f.y == 0.0;
  Rot o;
  if (gz) {
    o.c = 1.0;
    o.s = make_double2(0.0, 0.0);
    o.r = f;
  } else if (fz) {
    const double d = hypot(g.x, g.y);
    o.c = 0.0;
    o.s = make_double2(g.x / d, -g.y / d);
    o.r = make_double2(d, 0.0);
  } else {
    const double f2 = cabs2(f);
    const double g2 = cabs2(g);
    const double h2 = f2 + g2;
    const double cc = sqrt(f2 / h2);
    o.c = cc;
    o.r = make_double2(f.x / cc, f.y / cc);
    const double d = sqrt(f2 * h2);
    o.s = cmul(cconj(g), make_double2(f.x / d, f.y / d));
  }
  return o;
}


// What changes from one restart cycle to the next inside a multi-cycle launch: the tags' sequence
// number, the cycle's slot of the host-mapped report (statuses, control words) and |M r|^2.
struct CycleView {
  unsigned seq;
  double* report;     // [kRedDoubles]: [4..7] norms / decisions, statuses at kRedStatusOff
  double* status_it;  // report + kRedStatusOff
  int* ctrl;          // (int*)(report + kRedCtrlOff)
  double mn2;         // |M r|^2 of the cycle's start
};

// The Givens workgroup's wave: complete column `col` with its subdiagonal h1 (krylov.hip
// gmres_finish_column) -- every lane computes the same values, lane 0 stores them.  Lane k
// holds rotation k and entry k of the column, so the chain of previous rotations reads its
// operands by readlane instead of waiting on an LDS round trip per step.  The status of the
// column goes to sh.st.  Returns true (on every lane) when the cycle stops.
__device__ bool finish_column(const Shared& sh, const SmallCycleArgs& a, int col, double h1,
                              double inv_sigma_next, double ptol, int stop_col) {
  const int R1 = a.restart + 1;
  const int lane = threadIdx.x;
  const bool l0 = lane == 0;
  l2* h = sh.H + (size_t)col * R1;
  const double h0 = sh.h0s[col];
  double2 hsub = make_double2(h1, 0.0);
  double brk = 0.0;
  if (h1 <= a.eps * h0) {
    hsub = make_double2(0.0, 0.0);
    brk = 1.0;
  } else if (l0) {
    sh.vs[col + 1] = inv_sigma_next;
  }
  double ck = 0.0;
  double2 sk = make_double2(0.0, 0.0), hk = make_double2(0.0, 0.0);
  if (lane < col) {
    ck = sh.Gr[2 * lane].x;
    sk = sh.Gr[2 * lane + 1];
  }
  if (lane <= col) hk = h[lane];
  // the previous rotations, in order, the running entry carried
  double2 n0 = rlane2(hk, 0);
  for (int k = 0; k < col; ++k) {
    const double c = rlane(ck, k);
    const double2 s = rlane2(sk, k), n1 = rlane2(hk, k + 1);
    const double2 hn = cadd(cscale(n0, c), cmul(s, n1));
    if (l0) h[k] = hn;
    n0 = cadd(cmul(make_double2(-s.x, s.y), n0), cscale(n1, c));
  }
  const Rot rot = zlartg_s(n0, hsub);
  const double c = rot.c;
  const double2 s = rot.s;
  const double2 Sc = sh.S[col];
  const double2 tmp = cmul(make_double2(-s.x, s.y), Sc);
  const double presid = hypot(tmp.x, tmp.y);
  if (l0) {
    sh.Gr[2 * col] = make_double2(c, 0.0);
    sh.Gr[2 * col + 1] = s;
    h[col] = rot.r;
    h[col + 1] = make_double2(0.0, 0.0);
    sh.S[col] = cscale(Sc, c);
    sh.S[col + 1] = tmp;
    l1* st = sh.st + 4 * col;
    st[0] = presid;
    st[1] = brk;
    st[2] = h0;
    st[3] = h1;
    sh.ctl[1] = col;
    sh.gv[0] = presid;
    sh.gv[1] = brk;
  }
  return presid <= ptol || brk != 0.0 || col >= stop_col;
}



// Extra workgroup n ("Givens workgroup", its first wave): follows the rounds' sums at its own
// pace and keeps the Hessenberg books -- column j from the round-j sums, column j-1 completed
// with |u_j| (krylov.hip gmres_lag_kernel / gmres_finish_column), rotations, presid, scipy's
// exit tests -- so none of it sits on the row workgroups' critical path.  Per column it
// publishes a verdict granule (0 continue / 1 stop), at the end the column the cycle solved for
// and y_k / sigma_k.  A round's 2K + 2 sums are fetched by one lane each (one load latency per
// round, not one per column: the books then keep up with the rows, and the cycle's tail waits
// on one round trip); lane 0 does the arithmetic.  Returns false on timeout (wave-uniform).
__device__ bool givens_role(const Shared& sh, const SmallCycleArgs& a, const CycleView& cv,
                            int stop_col, double ptol) {
  const int R1 = a.restart + 1;
  const int lane = threadIdx.x;
  const bool l0 = lane == 0;
  // optional span timing (lane 0; slots 12 sum waits, 13 per-round work, 14 last column + solve)
  // (accumulated in registers, written once at the end: a read-modify-write of the counters
  // per span would itself wait on a global load)
  const bool prof = a.phase_ticks != nullptr && l0;
  unsigned long long tp = prof ? wall_clock64() : 0;
  unsigned long long acc[3] = {0, 0, 0};
  auto span = [&](int slot) {
    if (prof) {
      const unsigned long long now = wall_clock64();
      acc[slot - 12] += now - tp;
      tp = now;
    }
  };
  auto fetch = [&](unsigned epoch, int cols) {  // sums of round `epoch` into sh.sum[0 .. cols)
    span(13);
    bool ok = true;
    if (lane < cols) {
      double v = 0.0;
      ok = ld_gran(a.sums + (size_t)epoch * 2 * kPStride + 2 * lane, gran_tag(cv.seq, epoch), &v);
      sh.sum[lane] = v;
    }
    const bool all = __ballot(!ok) == 0;
    span(12);
    return all;
  };
  if (l0) {
    const double mn = sqrt(cv.mn2);
    sh.vs[0] = 1.0 / mn;
    sh.ss[0] = 1.0 / mn;
    for (int k = 0; k < R1; ++k) sh.S[k] = make_double2(k == 0 ? mn : 0.0, 0.0);
  }
  int col = -1;
  for (int j = 0; j <= stop_col && col < 0; ++j) {
    const int K = j + 1;
    const unsigned epoch = j + 1;
    if (!fetch(epoch, 2 * K + 2)) return false;  // dots, |z|^2, |u_j|^2
    // column j of H, entry k on lane k, and the Pythagorean terms (the row workgroups'
    // expressions; `rest` summed in their k order)
    const double w2 = sh.sum[2 * K], u2 = sh.sum[2 * K + 1];
    const double vj = j >= 1 ? 1.0 / sqrt(u2) : sh.vs[0];
    double tv = 0.0, tw = 0.0;
    if (lane <= j) {
      const double2 d = make_double2(sh.sum[2 * lane], sh.sum[2 * lane + 1]);
      const double vk = lane == j ? vj : sh.vs[lane];
      sh.H[(size_t)j * R1 + lane] = cscale(cscale(d, vk), vj / sh.ss[j]);
      tv = cabs2(d) * vk;
      tw = vk;
    }
    double rest = w2;
    for (int k = 0; k <= j; ++k) rest = fma(-rlane(tv, k), rlane(tw, k), rest);
    bool stop = false;
    if (j >= 1) {
      const int c = j - 1;
      stop = finish_column(sh, a, c, (1.0 / vj) * sh.vs[c] / sh.ss[c], vj, ptol, stop_col);
      if (l0) st_gran(a.verdict + 2 * c, gran_tag(cv.seq, c + 1), stop ? 1.0 : 0.0);
      if (stop) col = c;
    }
    if (l0) {
      if (!stop) {
        sh.vs[j] = vj;
        sh.h0s[j] = sqrt(w2) * (vj / sh.ss[j]);
        sh.ss[j + 1] = 1.0 / sqrt(fmax(rest, fmax(w2 * 1e-28, 1e-300)));
      }
    }
  }
  if (col < 0) {  // ran to stop_col: the last column needs |u_{stop_col+1}| (one more round)
    if (!fetch(stop_col + 2, 1)) return false;
    col = stop_col;
    const double sg = sqrt(sh.sum[0]);
    finish_column(sh, a, col, sg * sh.vs[col] / sh.ss[col], 1.0 / sg, ptol, stop_col);
  }
  if (l0) sh.ctl[1] = col;
  span(14);
  if (prof)
    for (int q = 0; q < 3; ++q) a.phase_ticks[12 + q] += acc[q];
  return true;
}
__device__ __forceinline__ void givens_tail_tick(const SmallCycleArgs& a, unsigned long long t0) {
  if (a.phase_ticks != nullptr && threadIdx.x == 0) a.phase_ticks[14] += wall_clock64() - t0;
}

// The triangular solve (krylov.hip gmres_solve_kernel) on the Givens workgroup's first wave,
// lane m holding y_m: for k = col .. 0, y_k *= 1 / H_kk (the reciprocals formed on all lanes at
// once, Smith's division: one division latency instead of one per step), then lanes m < k
// subtract y_k H_km in parallel (the next step's H entries loaded a step ahead) -- the
// sequential solve's order, one column step per iteration instead of one entry.
// y_k / sigma_k published for the x update.
__device__ void solve_and_publish(const Shared& sh, const SmallCycleArgs& a, const CycleView& cv) {
  const int R1 = a.restart + 1;
  const int lane = threadIdx.x;
  const int col = sh.ctl[1];
  auto Hc = [&](int c, int k) -> l2& { return sh.H[(size_t)c * R1 + k]; };
  const double2 hcc = Hc(col, col);
  double2 y = make_double2(0.0, 0.0);
  if (lane <= col) y = sh.S[lane];
  if (lane == col && hcc.x == 0.0 && hcc.y == 0.0) y = make_double2(0.0, 0.0);
  double2 rd = make_double2(0.0, 0.0);
  if (lane <= col) rd = cdiv_smith(make_double2(1.0, 0.0), Hc(lane, lane));
  double2 hk = Hc(col, min(lane, col));
  for (int k = col; k >= 0; --k) {
    const double2 hn = Hc(max(k - 1, 0), min(lane, max(k - 1, 0)));  // (next step's, ahead)
    double2 yk = make_double2(rlane(y.x, k), rlane(y.y, k));
    if (yk.x != 0.0 || yk.y != 0.0) {
      yk = cmul(yk, make_double2(rlane(rd.x, k), rlane(rd.y, k)));
      if (lane == k) y = yk;
      if (lane < k) y = csub(y, cmul(yk, hk));
    }
    hk = hn;
  }
  const unsigned ytag = gran_tag(cv.seq, 0xff);
  if (lane <= col) {
    const double2 c = cscale(y, sh.vs[lane]);
    st_gran(a.ycoef + 4 * lane, ytag, c.x);
    st_gran(a.ycoef + 4 * lane + 2, ytag, c.y);
  }
  // header: the column (+ 64 on a breakdown) and its presid, for the restart loop's decisions
  if (lane == 0) {
    st_gran(a.ycoef + 4 * kMaxProj, ytag, (double)(col + (sh.gv[1] != 0.0 ? 64 : 0)));
    st_gran(a.ycoef + 4 * kMaxProj + 2, ytag, sh.gv[0]);
  }
  // the columns' statuses to the host-mapped report, off the critical path now
  if (lane <= col) {
    double* st = cv.status_it + 4 * lane;
    for (int q = 0; q < 4; ++q) st[q] = sh.st[4 * lane + q];
  }
}

// Co-residency gate, instead of a cooperative launch (whose launch cost measured ~55 us: 3 % of a
// ten-cycle batch at 128^2, profiles/r03*_ab_c1.log).  The workgroups wait on each other, so all
// of them must be resident at once.  Every workgroup stores its arrival (a word tagged with the
// launch's sequence number); workgroup 0 polls all arrivals and decides GO; a workgroup whose
// co-residents did not come within its bound decides ABORT.  The decision is ONE word, set by
// compare-and-swap from any value not tagged with this launch: the first decision wins, so either
// every workgroup proceeds, or every workgroup leaves before touching any state (workgroup 0,
// which always runs eventually, then marks report slot 0 with ctrl = 3 and the host takes the
// regular cycle).  Returns true to proceed (block-uniform).
constexpr unsigned kGateSpins = 4000;  // ~ms: a resident grid arrives within microseconds
__device__ unsigned gate_decide(unsigned long long* decide, unsigned seq, unsigned state) {
  unsigned long long old =
      __hip_atomic_load((gu64*)decide, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    if ((unsigned)(old >> 2) == seq) return (unsigned)(old & 3u);  // decided already
    const unsigned long long want = ((unsigned long long)seq << 2) | state;
    if (__hip_atomic_compare_exchange_strong((gu64*)decide, &old, want, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      return state;
  }
}
__device__ bool coresidency_gate(const SmallCycleArgs& a, int nwg, HH_LDS int* flag) {
  const int g = blockIdx.x, t = threadIdx.x;
  if (t < kWave) {
    if (t == 0)
      __hip_atomic_store((gu32*)(a.gate_arrive + g), a.seq, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    unsigned st = 0;
    if (g == 0) {  // wave 0 polls every arrival word, one lane per word
      bool all = false;
      for (unsigned spins = 0; !all && spins < kGateSpins && !a.gate_force_abort; ++spins) {
        bool mine = true;
        for (int q = t; q < nwg; q += kWave)
          mine = mine && __hip_atomic_load((gu32*)(a.gate_arrive + q), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT) == a.seq;
        all = __all(mine);
        if (!all) __builtin_amdgcn_s_sleep(2);
      }
      if (t == 0) st = gate_decide(a.gate_decide, a.seq, all ? 1u : 2u);
    } else if (t == 0) {
      for (unsigned spins = 0;; ++spins) {
        const unsigned long long v =
            __hip_atomic_load((gu64*)a.gate_decide, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)(v >> 2) == a.seq) {
          st = (unsigned)(v & 3u);
          break;
        }
        if (spins > 2 * kGateSpins) {
          st = gate_decide(a.gate_decide, a.seq, 2u);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    if (t == 0) *flag = (int)st;
  }
  __syncthreads();
  const bool go = *flag == 1;
  if (!go && g == 0 && t == 0)  // (the refusal, for the host)
    reinterpret_cast<int*>(a.report + kRedCtrl)[0] = 3;
  return go;
}

__device__ __forceinline__ CycleView cycle_view(const SmallCycleArgs& a, int cyc) {
  CycleView cv;
  cv.seq = a.seq + (unsigned)cyc;
  cv.report = a.report + (size_t)cyc * kRedDoubles;
  cv.status_it = cv.report + kRedStatus;
  cv.ctrl = reinterpret_cast<int*>(cv.report + kRedCtrl);
  cv.mn2 = 0.0;
  return cv;
}

// The head of cycle `cyc`: its stop column and inner tolerance, as given, or from the restart
// loop's state that the previous cycle left -- in global memory for the launch's first cycle
// (written before the launch), afterwards from workgroup 0's granules {ptol, inner iterations,
// done, |M r|^2} (polled by every thread: the same four granules, cache hits after the first).
// quit: the solve already finished (or a wait timed out): nothing to do.  bad: a wait timed out
// here (WAVE: the Givens workgroup's single wave votes; otherwise the whole block).
struct CycleHead {
  int stop_col;
  double ptol, mn2;
  bool quit, bad;
};
template <bool WAVE>
__device__ __forceinline__ CycleHead cycle_head(const SmallCycleArgs& a, const CycleView& cv,
                                                int cyc) {
  CycleHead h{a.stop_col, a.ptol, 0.0, false, false};
  double inner = 0.0;
  if (cyc == 0) {
    h.mn2 = *a.mnorm2;
    if (!a.outer) return h;
    const double* o = a.outer;
    h.quit = o[6] != 0.0 || *a.timeout_word != 0u;
    h.ptol = o[0];
    inner = o[3];
  } else {
    const unsigned otag = gran_tag(cv.seq - 1, 0xfd);
    double ov[4];
    bool ok = true;
    for (int q = 0; q < 4; ++q) ok = ld_gran(a.obuf + 2 * q, otag, &ov[q]) && ok;
    h.bad = WAVE ? __any(!ok) : __syncthreads_or(!ok);
    h.ptol = ov[0];
    inner = ov[1];
    h.quit = ov[2] != 0.0 || *a.timeout_word != 0u;
    h.mn2 = ov[3];
  }
  const double* o = a.outer;
  if (o[5] != 0.0) {  // legacy: maxiter caps the inner iterations
    const double left = o[4] - inner;
    h.stop_col = left >= (double)a.restart ? a.restart - 1 : (int)left - 1;
  }
  return h;
}

}  // namespace
}  // namespace hh
