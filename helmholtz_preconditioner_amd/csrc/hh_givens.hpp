// Device helpers of the GMRES column (one wave): LAPACK's zlartg, the finish of a Hessenberg
// column (rotations, residual estimate, scipy's exit test -- iterative.py:767-795) and the
// lagged-normalisation step of the one-allreduce / one-pass iteration.  Shared by the Krylov
// kernels (krylov.hip) and the one-pass kernels' in-pass column (fused.hip, round 6).
#pragma once

#include "hh_internal.hpp"
#include "hh_complex.hpp"
#include "hh_wave.hpp"

namespace hh {
namespace givens {

// LAPACK (3.10+) zlartg main branch: [c s; -conj(s) c] [f; g] = [r; 0], c real >= 0.
// (by value: the pointer-output form kept c and r in scratch memory -- the branches' stores
// through pointers defeated register promotion, 24 bytes of scratch per lane)
struct Rot {
  double c;
  double2 s, r;
};
__device__ __forceinline__ Rot zlartg(double2 f, double2 g) {
  if (g.x == 0.0 && g.y == 0.0) return Rot{1.0, make_double2(0.0, 0.0), f};
  if (f.x == 0.0 && f.y == 0.0) {
    const double d = hypot(g.x, g.y);
    return Rot{0.0, make_double2(g.x / d, -g.y / d), make_double2(d, 0.0)};
  }
  const double f2 = cabs2(f);
  const double g2 = cabs2(g);
  const double h2 = f2 + g2;
  const double cc = sqrt(f2 / h2);
  const double d = sqrt(f2 * h2);
  const double2 fd = make_double2(f.x / d, f.y / d);
  return Rot{cc, cmul(cconj(g), fd), make_double2(f.x / cc, f.y / cc)};
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
__device__ __forceinline__ bool gmres_finish_column(const GivensState& g, int col, double2 hk,
                                                    const ColIn& in, double h0, double h1, double inv_sigma_next, double eps,
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
  const Rot rot = zlartg(n0, hsub);
  const double c = rot.c;
  const double2 s = rot.s, r = rot.r;
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
// lag_body's operands that do not come from the reductions (the finish of column j-1 and the
// start of column j read disjoint words: the finish writes only vscale[j], which the start takes
// from vj), loaded from clamped addresses -- one memory latency for all of them
struct LagIn {
  int stopped;
  double vs0, vcol, scol, sj, h0c, vkj;
  double2 hk0;
  ColIn in;
};
__device__ __forceinline__ LagIn lag_load(const GivensState& g, int j) {
  const int lane = threadIdx.x & (kWave - 1);
  const int R1 = g.restart + 1;
  const int col = max(j - 1, 0);
  LagIn L;
  L.stopped = g.ctrl[0];
  L.vs0 = g.vscale[0];
  L.vcol = g.vscale[col];
  L.scol = g.sscale[col];
  L.sj = g.sscale[j];
  L.h0c = g.status_it[4 * col + 2];                   // stored when the column was started
  L.hk0 = g.H[(size_t)col * R1 + min(lane, col)];     // (previous launch)
  L.in = load_col_in(g, col);
  L.vkj = g.vscale[min(lane, j)];
  return L;
}
// d = (rd[2k], rd[2k+1]) on lane k = min(lane, j), w2 = |w|^2, sig = |u_j|^2
__device__ __forceinline__ void lag_compute(const GivensState& g, int j, const LagIn& L,
                                            double2 d, double w2, double sig, int final_step,
                                            double eps, double ptol, int stop_col) {
  const int lane = threadIdx.x & (kWave - 1);
  const int R1 = g.restart + 1;
  const int col = max(j - 1, 0);
  double vj = L.vs0;
  if (j >= 1) {
    const double sj = sqrt(sig);
    vj = 1.0 / sj;
    const double f = L.vcol / L.scol;
    const double h1 = sj * f;
    const double2 hk = lane <= col ? L.hk0 : make_double2(0.0, 0.0);
    const bool stop = gmres_finish_column(g, col, hk, L.in, L.h0c, h1, vj, eps, ptol, stop_col);
    if (stop || final_step) return;
  }
  const double f = vj / L.sj;
  double2* h = g.H + (size_t)j * R1;
  double tv = 0.0, tw = 0.0;
  if (lane <= j) {
    const double vk = lane == j ? vj : L.vkj;
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

// The triangular solve H y = S of columns 0 .. col and y_k s_k into g.ycoef (lane k: y_k), on
// one wave, from H's columns already in LDS (sH, R1 = restart + 1 per column) -- gmres_solve
// _kernel's body, also run by cycle_finish_kernel's first block when a cycle stopped early.
__device__ __forceinline__ void solve_columns_wave(const GivensState& g, int col,
                                                   const double2* sH) {
  const int R1 = g.restart + 1;
  const int lane = threadIdx.x & (kWave - 1), me = min(lane, col);
  double2 y = g.S[me];
  const double sv = g.vscale[me];
  auto H = [&](int c, int k) { return sH[c * R1 + k]; };
  const double2 hcc = H(col, col);
  if (hcc.x == 0.0 && hcc.y == 0.0) {
    if (lane == 0) g.S[col] = make_double2(0.0, 0.0);
    if (lane == col) y = make_double2(0.0, 0.0);
  }
  const Smith f = smith_of(H(me, me));
  for (int k = col; k >= 0; --k) {
    const double2 t0 = rlane2(y, k);
    if (t0.x != 0.0 || t0.y != 0.0) {  // (uniform)
      if (lane == k) y = smith_apply(y, f);
      if (k == 0) break;
      const double2 t = rlane2(y, k);
      if (lane < k) y = csub(y, cmul(t, H(k, lane)));
    }
  }
  if (lane <= col) g.ycoef[lane] = cscale(y, sv);
}

}  // namespace givens
}  // namespace hh
