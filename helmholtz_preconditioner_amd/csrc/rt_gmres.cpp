// The one-pass GMRES iteration across slabs and ranks and hh_gmres, scipy 1.15.3's restarted
// GMRES control flow (iterative.py:582-840) as code.py:516 calls it (see hh_runtime.hpp for the
// runtime's layout).
#include "hh_runtime.hpp"

namespace hh {

// the one-pass iteration where it applies, unless HH_FUSED_ITER=0
bool fused_default() { return knobs().fused_iter != 0; }

// One pass of the one-pass GMRES iteration (fused.hip) over the rank's slabs: u_K = w_{K-1} -
// sum_k c_k u_k into V[K], w_K = M A (s_K u_K) into wout, and the partial rows of the next
// projections (width 2 (K + 1) + 2).  Slabs of one rank read each other's rows in place
// (FROW_MEM).  Across ranks the rows next to a rank boundary need the neighbour's u_K, which
// does not exist before the pass: the rank's own edge rows of it (H = 1, or 2 for the
// shifted Laplace) are formed first by a small launch, exchanged on the halo stream while the
// interior rows run on the compute stream, and the H boundary rows run behind the exchange on
// the halo stream (run_stencil's overlap).  Returns the number of partial rows written.
int run_fused(hh_op* op, int K, const double2* win, double2* wout, const double* raw,
              const double* sin, const PassFold* fold) {
  hh_ctx* c = op->ctx;
  const int n = op->n;
  const int S = (int)op->slabs.size();
  const bool sl = op->pkind == HH_PREC_SHIFTED_LAPLACE;
  const int H = sl ? 2 : 1;
  const bool lo_x = c->world > 1 && c->rank > 0;
  const bool hi_x = c->world > 1 && c->rank < c->world - 1;
  const size_t ldv = op->ldv;
  double2* uout = op->V + (size_t)K * ldv;
  const int width = 2 * (K + 1) + 2;
  const int rows_rank = op->je - op->jb;
  const bool slv = sl && fused_slv_use(K);
  const bool slk = sl && !slv && fused_slk_use(K);
  const int R = slk ? fused_slk_rows(n, rows_rank) : fused_iter_rows(n, rows_rank);
  FusedArgs base{};
  base.ldv = ldv;
  base.raw = raw;
  base.vscale = op->gs.vscale;
  base.sin = sin;
  base.tab_i = op->tab_i;
  base.invc2_const = op->invc2_const;
  base.n = n;
  base.jac = op->pkind == HH_PREC_JACOBI ? 1 : 0;
  base.sl = sl ? 1 : 0;
  base.mshift = op->mshift;
  base.damping = op->damping;
  base.stop = op->stop_flag;
  base.alt = (!sl && fused_alt_dir()) ? 1 : 0;
  if (fold) {  // (one launch covers every partial row: one slab of one rank)
    REQUIRE(c->world == 1 && S == 1, "the in-pass column needs one slab of one rank");
    REQUIRE(width <= 64, "in-pass column: %d partial-row columns (at most 64)", width);
    base.fold = *fold;
  }
  int nparts = 0;
  auto launch = [&](int si, int r0, int r1, int rows, int step, hipStream_t st) {
    if (r1 <= r0) return;
    const Slab& s = op->slabs[si];
    FusedArgs a = base;
    a.V = op->V + s.off;
    a.win = win + s.off;
    a.wout = wout + s.off;
    a.uout = uout + s.off;
    a.tab_j = s.tab_j;
    a.invc2 = op->const_c ? nullptr : s.invc2;
    a.invc2_halo = s.invc2_halo;
    a.nl = s.nl;
    a.lo_mode = si > 0 ? FROW_MEM : (lo_x ? FROW_HALO : FROW_ZERO);
    a.hi_mode = si < S - 1 ? FROW_MEM : (hi_x ? FROW_HALO : FROW_ZERO);
    a.halo_lo = sl ? s.halo2_lo : s.halo_lo_buf;
    a.halo_hi = sl ? s.halo2_hi : s.halo_hi_buf;
    a.row_begin = r0;
    a.row_end = r1;
    a.rows = rows;
    a.row_step = step;
    a.bands = step > 0 ? (r1 - r0 - 1) / step + 1 : (r1 - r0 + rows - 1) / rows;
    a.partials = op->partials + (size_t)nparts * width;
    const int blocks = slv ? fused_slv_blocks(n, a.bands) : fused_iter_blocks(n, a.bands);
    REQUIRE((size_t)(nparts + blocks) * width <= op->partials_cap,
            "partials workspace too small for the one-pass iteration (%d blocks)", nparts + blocks);
    if (slv)
      launch_fused_slv(K, a, blocks, st);
    else if (slk)
      launch_fused_slk(K, a, blocks, st);
    else
      launch_fused_iter(K, a, blocks, st);
    nparts += blocks;
  };
  hipEvent_t t_halo = nullptr;
  if (lo_x || hi_x) {
    FusedArgs e = base;  // (rank-local rows)
    e.V = op->V;
    e.win = win;
    e.uout = uout;
    if (rows_rank <= 2 * H)
      launch_fused_edge(K, e, 0, rows_rank, 0, 0, c->stream);
    else
      launch_fused_edge(K, e, 0, lo_x ? H : 0, rows_rank - H, hi_x ? H : 0, c->stream);
    check_site(c, "one-pass: edge rows of u_K", c->stream);
    const Slab& s0 = op->slabs[0];
    const Slab& sL = op->slabs[S - 1];
    hipEvent_t t_ready = tmark(op, c->stream);
    c->comm->halo(lo_x ? uout : nullptr, lo_x ? (sl ? s0.halo2_lo : s0.halo_lo_buf) : nullptr,
                  hi_x ? uout + (size_t)(rows_rank - H) * n : nullptr,
                  hi_x ? (sl ? sL.halo2_hi : sL.halo_hi_buf) : nullptr,
                  (size_t)H * n * sizeof(double2), c->stream, c->cstream, c->ev_in);
    t_halo = tmark(op, c->cstream);
    tspan(op, HH_SPAN_HALO, t_ready, t_halo);
    check_site(c, "one-pass: u_K halo exchange", c->cstream);
  }
  hipEvent_t t_int0 = tmark(op, c->stream);
  for (int si = 0; si < S; ++si) {
    const Slab& s = op->slabs[si];
    const int r0 = (si == 0 && lo_x) ? H : 0;
    const int r1 = (si == S - 1 && hi_x) ? s.nl - H : s.nl;
    launch(si, r0, r1, R, 0, c->stream);
  }
  hipEvent_t t_int1 = tmark(op, c->stream);
  tspan(op, HH_SPAN_INTERIOR, t_int0, t_int1);
  if (lo_x || hi_x) check_site(c, slk ? "one-pass (slk): interior rows" : "one-pass: interior rows",
                               c->stream);
  if (lo_x || hi_x) {
    hipStream_t hs = c->cstream;
    const Slab& s0 = op->slabs[0];
    const Slab& sL = op->slabs[S - 1];
    if (S == 1 && lo_x && hi_x) {
      if (s0.nl <= 2 * H) launch(0, 0, s0.nl, s0.nl, 0, hs);  // (no interior rows)
      else launch(0, 0, s0.nl, H, s0.nl - H, hs);             // rows [0, H) and [nl - H, nl)
    } else {
      if (lo_x) launch(0, 0, std::min(H, s0.nl), H, 0, hs);
      if (hi_x) launch(S - 1, std::max(0, sL.nl - H), sL.nl, H, 0, hs);
    }
    check_site(c, slk ? "one-pass (slk): boundary rows" : "one-pass: boundary rows", hs);
    hipEvent_t t_bnd = tmark(op, hs);
    tspan(op, HH_SPAN_BOUNDARY, t_halo, t_bnd);
    tspan(op, HH_SPAN_HALO_WAIT, t_int1, t_bnd, true);
    HIPC(hipEventRecord(c->ev_halo, hs));
    HIPC(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
  }
  HIPC(hipGetLastError());
  op->stats.spmv_count++;
  return nparts;
}

// Padding between consecutive basis vectors, in complex elements (HH_BASIS_PAD overrides).
// Unpadded, the K vectors a Krylov pass streams together sit exactly nloc * 16 B apart (1 GiB
// at 8192^2): 4 KiB + 256 B between them measured +3 % for the one-pass iteration at 8192^2
// (316.6 -> 326.0 it/s; 256 B +1.5 %, 2.3 / 8.3 / 64.3 KiB +1.5-2.5 %,
// profiles/r04/r04h_ab_pad_c4.log, r04i_ab_nt_c4.log)
size_t basis_pad() { return (size_t)knobs().basis_pad; }

void ensure_gmres(hh_op* op, int restart) {
  REQUIRE(restart >= 1 && restart <= kMaxProj - 1, "restart must be in [1, %d]", kMaxProj - 1);
  if (op->V && op->V_cols >= restart + 1) return;
  dfree(op->V);
  op->ldv = op->nloc + basis_pad();
  dfree(op->gbuf);
  op->V = dalloc<double2>(op->ldv * (size_t)(restart + 1));
  op->V_cols = restart + 1;
  const int R1 = restart + 1;
  const size_t nH = (size_t)restart * R1, nG = 2 * (size_t)restart, nS = R1, nY = restart;
  const size_t total2 = nH + nG + nS + nY + (R1 + 8 + 1) / 2 + 8 + 2 * (size_t)restart + 8 +
                        (R1 + 1) / 2 + 1;
  op->gbuf = dalloc<double2>(total2);
  HIPC(hipMemsetAsync(op->gbuf, 0, total2 * sizeof(double2), op->ctx->stream));
  GivensState& g = op->gs;
  g.H = op->gbuf;
  g.G = g.H + nH;
  g.S = g.G + nG;
  g.ycoef = g.S + nS;
  g.vscale = reinterpret_cast<double*>(g.ycoef + nY);
  g.status = g.vscale + R1 + 1;
  g.status_it = g.status + 8;
  g.sscale = g.status_it + 4 * (size_t)restart;
  if (!op->npart) op->npart = dalloc<double>((size_t)kMaxStreamBlocks * kMaxNorms);
  if (!op->kcount) {
    op->kcount = dalloc<unsigned>(4);
    HIPC(hipMemsetAsync(op->kcount, 0, 4 * sizeof(unsigned), op->ctx->stream));
  }
  // the per-iteration statuses and the cycle's control words live in the reduction buffer,
  // next to the residual norms: the end of a cycle reads them all with ONE copy (kRedReport)
  g.status_it = op->red + kRedStatus;
  g.ctrl = reinterpret_cast<int*>(op->red + kRedCtrl);
  HIPC(hipMemsetAsync(g.ctrl, 0, 8 * sizeof(int), op->ctx->stream));
  g.restart = restart;
}

}  // namespace hh

// ------------------------------------------------------------------- GMRES
// Control flow of scipy 1.15.3 gmres (iterative.py:582-840), which code.py:516 calls.
HH_API int hh_gmres(hh_op* op, const hh_vec* bv, hh_vec* xv, double rtol, double atol,
                    int restart, long maxiter, int legacy_maxiter, int reorth, double* hist,
                    long hist_cap, hh_gmres_callback cb, void* user, long* iters_out,
                    int* info_out, double* rnorm_out, double* bnorm_out) {
  GUARD_BEGIN
  REQUIRE(op && bv && xv && bv->op == op && xv->op == op && bv != xv, "bad vectors");
  REQUIRE(maxiter >= 1, "maxiter must be >= 1");
  REQUIRE(rtol >= 0 && atol >= 0, "tolerances must be non-negative");
  hh_ctx* c = op->ctx;
  HIPC(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const auto t_start = std::chrono::steady_clock::now();
  // In-solve state (the cycle's stop flag every queued kernel polls, the as-is sweep's
  // constant M b) must not outlive this call on ANY exit path -- an error, an SHM timeout or a
  // callback abort included: a later plain apply would otherwise poll a raised stop flag and
  // return a stale buffer.  The stream is drained first so no queued kernel still reads them.
  struct SolveScope {
    hh_op* op;
    ~SolveScope() {
      (void)hipStreamSynchronize(op->ctx->stream);
      op->stop_flag = nullptr;
      dfree(op->sw_const);
      op->sw_const = nullptr;
    }
  } scope{op};
  op->stats = hh_stats{};
  if (restart > (long)op->n * op->n) restart = (int)((long)op->n * op->n);
  ensure_gmres(op, restart);
  const size_t L = op->nloc;
  const size_t ldv = op->ldv;
  double2* V = op->V;
  const double2* b = bv->d;
  double2* x = xv->d;
  GivensState& g = op->gs;
  const double eps = std::numeric_limits<double>::epsilon();
  const int blocks = stream_blocks(L);
  REQUIRE((size_t)blocks * (2 * (restart + 1) + 2) <= op->partials_cap,
          "partials workspace too small for %d streaming blocks", blocks);
  double st[8];

  // red[4] = |b|^2 (= |r|^2 while x0 == 0), red[2] = |x0|^2; and (one host sync for all of
  // them) V[0] = M b, red[5] = |M b|^2 -- except for the as-is sweep, whose M needs b first
  norm2(op, b, 4);
  norm2(op, x, 2);
  const bool mb_early = op->pkind != HH_PREC_SWEEP_REF;
  if (mb_early) {
    apply_M(op, b, V);
    norm2(op, V, 5);
  }
  read_dev(op, op->red, st, 6);
  const double bnrm2 = std::sqrt(st[4]);
  const bool x_any = st[2] > 0.0;
  if (bnorm_out) *bnorm_out = bnrm2;
  atol = std::max(atol, rtol * bnrm2);
  auto finish = [&](long it, int info, double rn) {
    if (iters_out) *iters_out = it;
    if (info_out) *info_out = info;
    if (rnorm_out) *rnorm_out = rn;
    op->stats.inner_iterations = it;
    op->stats.solve_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
  };
  if (bnrm2 == 0.0) {
    launch_scale_copy(b, x, L, 1.0, s);
    HIPC(hipStreamSynchronize(s));
    finish(0, 0, 0.0);
    return HH_OK;
  }
  if (op->pkind == HH_PREC_SWEEP_REF) {
    // The constant map makes M A rank one: every w = M A v is the same vector c as v_0, and the
    // whole cycle hinges on scipy's breakdown test h1 <= eps h0 (iterative.py:767) applied to
    // the ~1-ulp residue of c - <v_0, c> v_0 -- rounding decides whether it fires (scipy: after
    // 1-3 cycles).  A second Gram-Schmidt pass takes the residue to the exact-arithmetic
    // answer (h1 ~ eps^2 h0): breakdown in the first cycle, never a 10 N-iteration crawl.
    reorth = 1;
    // run_solver's M (code.py:510-511, quirk Q1) is algo2_4 of the right-hand side f_vec,
    // whatever GMRES passes it: compute that constant once
    dfree(op->sw_const);
    op->sw_const = nullptr;
    double2* c = dalloc<double2>(L);
    sweep_apply(op, b, c, true);
    op->sw_const = c;
  }
  // Mb_nrm2 = ||psolve(b)||; V[0] = M b, red[5] = |M b|^2 (= |M r|^2 while x0 == 0)
  if (!mb_early) {
    apply_M(op, b, V);
    norm2(op, V, 5);
    read_dev(op, op->red + 5, st + 5, 1);
  }
  const double Mb_nrm2 = std::sqrt(st[5]);
  double ptol_max_factor = 1.0;
  double ptol = Mb_nrm2 * std::min(ptol_max_factor, atol / bnrm2);
  double presid = 0.0, rnorm = 0.0;
  long inner = 0;
  bool legacy = legacy_maxiter != 0;
  // collectives per inner iteration: one (lagged normalisation) by default across ranks, two on
  // one rank (no collective there; the exact-norm path keeps round 1's bit-for-bit results)
  // one pass over the basis per inner iteration (fused.hip fused_iter_kernel): the lagged
  // iteration with the update, the next M A and the next projection in one streaming kernel;
  // any slabs and ranks (run_fused: one halo exchange and one allreduce per inner iteration),
  // 5-point, M none / Jacobi / two-sweep shifted Laplace (mode 3, or by default where it applies)
  const bool fused_ok = !reorth && op->points == 5 &&
                        (op->pkind == HH_PREC_NONE || op->pkind == HH_PREC_JACOBI ||
                         (op->pkind == HH_PREC_SHIFTED_LAPLACE && op->sweeps == 2 &&
                          op->sl_ext_ok)) &&
                        restart <= kFusedMaxK + 1;
  // (by default from n = 1024: smaller grids give the pass too few tiles to stream at speed --
  // n = 300: 16-25k it/s against 29-30k for the regular cycle, profiles/r03q; the two-sweep
  // shifted-Laplace pass too since round 4: 889-894 vs 769-774 it/s for the regular cycle at
  // 4096^2, profiles/r04/r04q_ab_sl_fused_vs_regular_4096.log)
  const bool fused = fused_ok && (op->krylov_mode == 3 ||
                                  (op->krylov_mode == 0 && fused_default() && op->n >= 1024));
  const bool lagged = !reorth && !fused &&
                      (op->krylov_mode == 2 || (op->krylov_mode == 0 && c->world > 1));
  // small single-rank grids: the whole cycle in one launch (gmres_small.hip) -- launch-bound
  // otherwise (five kernel boundaries per inner iteration at ~0.5 MB each)
  const bool small = !reorth && op->small_cycle != 0 && c->world == 1 && op->slabs.size() == 1 &&
                     op->points == 5 &&
                     (op->pkind == HH_PREC_NONE || op->pkind == HH_PREC_JACOBI) &&
                     (op->krylov_mode != 1) && small_cycle_eligible(op->n, restart, device_cus(c)) &&
                     (op->small_cycle == 1 || (size_t)op->n * op->n <= ((size_t)1 << 18));
  // every sweep apply above (M b, the as-is constant) is checked before the word is re-armed
  check_sweep_chain(op);
  unsigned* small_timeout = reinterpret_cast<unsigned*>(op->red + kRedTimeout);
  HIPC(hipMemsetAsync(small_timeout, 0, sizeof(double), s));  // (the device wait-bound word)
  if (small) {
    if (!op->small_scr) {
      const size_t nd = small_cycle_scratch_doubles(op->n);
      op->small_scr = dalloc<double>(nd);
      HIPC(hipMemsetAsync(op->small_scr, 0, nd * sizeof(double), s));  // (no stale tags)
    }
  }

  if (fused && !op->fw) op->fw = dalloc<double2>(2 * L);
  if (fused && !op->cab) op->cab = dalloc<double2>(2 * kMaxProj);
  // the end of a full one-pass cycle in one pass over the basis (fused.hip cycle_end_kernel:
  // the last update's norm, x += V a and V b together; HH_CYCLE_MERGE=0: update, then the
  // triangular solve and xupdate)
  const bool merge_end = fused && knobs().cycle_merge != 0;
  double r0 = bnrm2;  // (x0 = 0: r = b)
  if (x_any) {
    residual(op, b, x, V, 4);  // V[0] = M (b - A x0); red[4..5]
    read_dev(op, op->red + 4, st, 1);
    r0 = std::sqrt(st[0]);
  }
  if (r0 < atol) {  // (scipy's test before the first cycle)
    finish(0, 0, r0);
    return HH_OK;
  }
  // replays one finished cycle's per-iteration statuses to the host callbacks (in order)
  auto replay = [&](const double* sth, int col) {
    double rel[kMaxProj];
    const long first = inner + 1;
    for (int k = 0; k <= col; ++k) {
      const double pr = sth[4 * k];
      inner += 1;
      rel[k] = pr / bnrm2;
      if (hist && inner - 1 < hist_cap) hist[inner - 1] = rel[k];
      if (cb && cb(user, inner, rel[k]) != 0) {
        finish(inner, -1, 0.0);
        fail(HH_ERR_ABORTED, "gmres stopped by the per-iteration callback at iteration %ld", inner);
      }
    }
    if (op->hist_cb) {
      const int r = op->hist_cb(op->hist_user, first, col + 1, rel);
      if (r != 0) {
        const long at = first - 1 + (r >= 1 && r <= col + 1 ? r : col + 1);
        finish(at, -1, 0.0);
        fail(HH_ERR_ABORTED, "gmres stopped by the history callback at iteration %ld", at);
      }
    }
  };
  bool small_refused = false;
  long cycles_done = 0;  // restart cycles the small-grid kernel completed before a refusal
  op->last_path = small ? 1 : (fused ? 3 : 0);
  if (small) {
    // Small grids: whole-cycle launches (gmres_small.hip), each running up to kSmallBatch restart
    // cycles -- scipy's restart-loop decisions are taken on the device from the state below
    // (bitwise the host's expressions), so a cycle starts right after the previous one inside
    // the same launch instead of after a host round trip.  One cooperative launch and one sync
    // per batch; the host then replays each cycle's report: callbacks in order, legacy maxiter,
    // the x callback (which limits a batch to one cycle, x being observed after every cycle).
    // The cycles after the one that finished the solve are skipped (ctrl = 2).  An exception
    // raised by a callback ends the solve after the batch (x is then up to kSmallBatch - 1
    // cycles further; the Python shim returns no x then).
    double* outer_h = op->status_h + kRedOuter;  // (pinned staging for the upload)
    outer_h[0] = ptol;
    outer_h[1] = ptol_max_factor;
    outer_h[2] = atol;
    outer_h[3] = 0.0;
    outer_h[4] = (double)maxiter;
    outer_h[5] = legacy ? 1.0 : 0.0;
    outer_h[6] = 0.0;
    outer_h[7] = 0.0;
    double* outer = op->red + kRedOuter;
    HIPC(hipMemcpyAsync(outer, outer_h, kOuterDoubles * sizeof(double), hipMemcpyHostToDevice, s));
    const int cap = op->cycle_cb ? 1 : kSmallBatch;
    const Slab& sl = op->slabs[0];
    long iteration = 0, launches = 0;
    bool done = false;
    while (!done && iteration < maxiter) {
      // (legacy: maxiter caps inner iterations, so no more cycles than those left can run)
      const long cycles_left =
          legacy ? (maxiter - inner + restart - 1) / restart : maxiter - iteration;
      const int P = (int)std::min<long>(cap, cycles_left);
      {
        // ONE cooperative launch runs the batch's P cycles (their restart-loop decisions taken
        // on the device); cycle i reports into slot 1 + i of the pinned host mirror
        double* rep = op->status_h + kRedDoubles;
        SmallCycleArgs sa{};
        sa.n = op->n;
        sa.restart = restart;
        sa.stop_col = restart - 1;  // (from `outer`)
        sa.tab_i = op->tab_i;
        sa.tab_j = sl.tab_j;
        sa.invc2 = op->const_c ? nullptr : sl.invc2;
        sa.invc2_const = op->invc2_const;
        sa.v0 = V;
        sa.mnorm2 = op->red + mnorm_slot(op, 4);
        sa.b = b;
        sa.x = x;
        sa.red = op->red;
        sa.report = rep;
        sa.g = g;
        for (int i = 0; i < P; ++i)  // (ctrl[0] = 1 marks a slot's cycle complete)
          reinterpret_cast<int*>(rep + (size_t)i * kRedDoubles + kRedCtrl)[0] = 0;
        sa.eps = eps;
        sa.ptol = ptol;  // (from `outer`)
        sa.zbuf = reinterpret_cast<unsigned long long*>(op->small_scr);
        sa.xbuf = sa.zbuf + 8 * (size_t)op->n * op->n;
        sa.part = sa.xbuf + 4 * (size_t)op->n * op->n;
        sa.sums = sa.part + 2 * (size_t)op->n * 2 * kSmallCols;
        sa.verdict = sa.sums + (size_t)kSmallRounds * 2 * kSmallCols;
        sa.ycoef = sa.verdict + 2 * kMaxProj;
        sa.mbuf = sa.ycoef + 4 * (kMaxProj + 1);
        sa.obuf = sa.mbuf + 4 * (size_t)op->n * op->n;
        sa.gate_decide = sa.obuf + 8;
        sa.gate_arrive = reinterpret_cast<unsigned*>(sa.gate_decide + 1);
        // test hooks: the gate refuses every launch (HH_SMALL_COOP_REFUSE=1), or only the
        // solve's launch number HH_SMALL_REFUSE_AT (1-based: 2 = the second batch)
        const bool force_abort = knobs().small_coop_refuse != 0;
        const long refuse_at = knobs().small_refuse_at;
        ++launches;
        sa.gate_force_abort = (force_abort || launches == refuse_at) ? 1 : 0;
        // P consecutive sequence numbers, none 0 (tag 0 is the zeroed scratch)
        if (((op->small_seq + (unsigned)P) & 0xffffffu) < (unsigned)P) op->small_seq = 0;
        sa.seq = (op->small_seq + 1) & 0xffffffu;
        op->small_seq += (unsigned)P;
        sa.cycles = P;
        sa.timeout_word = small_timeout;
        sa.phase_ticks = op->small_ticks;
        sa.outer = outer;
        const hipError_t le = launch_small_cycle(sa, op->const_c, op->pkind == HH_PREC_JACOBI, s);
        if (le != hipSuccess) {
          // refused before anything of the batch ran (cooperative launch: e.g. the grid cannot
          // be co-resident): the regular cycle takes over below, at this restart boundary
          small_refused = true;
        }
      }
      if (small_refused) break;
      HIPC(hipStreamSynchronize(s));
      if (reinterpret_cast<const int*>(op->status_h + kRedDoubles + kRedCtrl)[0] == 3) {
        // the kernel's co-residency gate refused the grid before any workgroup touched state
        // (the GPU shared with another process?): the regular cycle takes over below
        small_refused = true;
        break;
      }
      for (int i = 0; i < P && !done; ++i) {
        const double* rep = op->status_h + (size_t)(1 + i) * kRedDoubles;
        int ctl[2];
        std::memcpy(ctl, rep + kRedCtrl, 2 * sizeof(int));
        if (ctl[0] != 1) {
          double w = 0.0;
          read_dev(op, op->red + kRedTimeout, &w, 1);
          unsigned tmo = 0;
          std::memcpy(&tmo, &w, sizeof(unsigned));
          REQUIRE(tmo == 0, "small-grid GMRES cycle: a grid-wide wait timed out (workgroups not "
                            "co-resident?); hh_op_set_small_cycle(op, 0) selects the regular cycle");
          fail(HH_ERR_STATE, ctl[0] == 2 ? "small-grid GMRES: a queued cycle found the solve "
                                           "finished before the host did"
                                         : "small-grid GMRES cycle ended without its report");
        }
        const int col = ctl[1];
        REQUIRE(col >= 0 && col < restart, "GMRES cycle state corrupt (last column %d)", col);
        const double* sth = rep + kRedStatus;
        replay(sth, col);
        presid = sth[4 * col];
        op->stats.restarts++;
        ++iteration;
        rnorm = std::sqrt(rep[4]);
        if (legacy && inner == maxiter) {
          finish(inner, rnorm <= atol ? 0 : (int)std::min<long>(maxiter, 0x7fffffff), rnorm);
          return HH_OK;
        }
        if (op->cycle_cb && op->cycle_cb(op->cycle_user, op->stats.restarts) != 0) {
          finish(inner, -1, rnorm);
          fail(HH_ERR_ABORTED, "gmres stopped by the cycle callback after cycle %ld",
               op->stats.restarts);
        }
        done = rep[6] != 0.0;  // (rnorm <= atol, breakdown, or legacy maxiter)
      }
    }
    if (!small_refused) {
      finish(inner, rnorm <= atol ? 0 : (int)std::min<long>(maxiter, 0x7fffffff), rnorm);
      return HH_OK;
    }
    // Refused: the regular cycle below runs the rest of the solve.  A batch starts at a restart
    // boundary and a refusal leaves the cycle state untouched, so it resumes from exactly where
    // the last completed cycle left it: x, V[0] = M r and red[4..5] (|r|^2, |M r|^2) of the
    // current x -- each cycle's tail computes them for the next --, and scipy's restart-loop
    // state the kernel carried on the device (ptol, ptol_max_factor; `inner` and the cycle
    // count are the host's own, from the replayed reports).
    op->last_path = 2;
    cycles_done = iteration;
    if (iteration > 0) {
      double o[kOuterDoubles];
      read_dev(op, outer, o, kOuterDoubles);
      ptol = o[0];
      ptol_max_factor = o[1];
    }
  }

  for (long iteration = cycles_done; iteration < maxiter; ++iteration) {
    // v[0] = psolve(r) / ||psolve(r)||, S[0] = ||psolve(r)|| (lazy scale); clears the stop flag
    launch_gmres_start(g, op->red, 4, mnorm_slot(op, 4), s);
    // The whole cycle is queued at once: the column kernel evaluates scipy's inner exit test
    // (presid <= ptol, breakdown, legacy maxiter) and raises the stop flag, after which the
    // kernels still queued in this cycle return immediately.  One host sync per cycle.
    bool breakdown = false;
    int col = 0;
    const long left = legacy ? maxiter - inner : (long)restart;
    const int stop_col = (int)std::min<long>(restart - 1, left - 1);
    op->stop_flag = g.ctrl;
    if (fused) {
      // the lagged iteration (below) with update(c2), M A(c2 + 1) and multidot(c2 + 1) in ONE
      // pass over the basis (fused_iter_kernel): w_j lives in a ping-pong pair instead of V[j+1]
      // (the pass writes u_{j+1} there while other tiles still read their halo rows of w_j)
      const int* stp = g.ctrl;
      double2* Wb[2] = {op->fw, op->fw + L};
      // HH_LAG_RED=2, one slab of one rank: the pass's own blocks reduce its partial rows (in
      // reduce_kernel's order) and run the column (hh_fused.hpp pass_fold) -- no reduce / column
      // launch between two passes, nor after the cycle's first dots and its end
      const bool fold = c->world == 1 && op->slabs.size() == 1 && knobs().lag_red == 2;
      if (fold && !op->fold_tickets) {
        op->fold_tickets = dalloc<unsigned>(1 + kFoldClasses);
        op->fold_gpart = dalloc<double>((size_t)64 * kFoldClasses);
        HIPC(hipMemsetAsync(op->fold_tickets, 0, (1 + kFoldClasses) * sizeof(unsigned), s));
      }
      auto fold_at = [&](int j, double* red) {
        PassFold pf{};
        pf.tickets = op->fold_tickets;
        pf.gpart = op->fold_gpart;
        pf.red = red;
        pf.g = g;
        pf.j = j;
        pf.stop_col = stop_col;
        pf.eps = eps;
        pf.ptol = ptol;
        return pf;
      };
      apply_MA(op, V, g.sscale, Wb[0]);  // w_0 = M A (s_0 u_0)
      if (fold) {
        launch_cycle_start_dots(V, Wb[0], L, op->partials, blocks, krylov_nt_for(L), s, stp,
                                fold_at(0, op->red + 16));
      } else {
        launch_multidot(V, ldv, 1, Wb[0], L, op->partials, blocks, s, stp);
        if (c->world == 1 && lag_red_merge()) {  // (one rank: reduce + lag step in one launch)
          launch_gmres_lag_red(g, 0, op->partials, blocks, 4, 3, op->red + 16, eps, ptol, stop_col,
                               s);
        } else {
          launch_reduce(op->partials, blocks, 4, 3, op->red + 16, s, stp);
          allreduce_sum_dev(op, op->red + 16, 3);
          launch_gmres_lag(g, 0, op->red + 16, op->red + 16 + 3, false, eps, ptol, stop_col, s);
        }
      }
      check_site(c, "one-pass: first projection + column", s);
      for (int c2 = 0; c2 < stop_col; ++c2) {
        const int K = c2 + 1, K2 = K + 1;
        PassFold pf{};
        if (fold) pf = fold_at(c2 + 1, op->red + 16);
        const int np = run_fused(op, K, Wb[c2 & 1], Wb[(c2 + 1) & 1], op->red + 16, g.sscale + K,
                                 fold ? &pf : nullptr);
        // (dots, |w|^2 and |u|^2 in one partial row: one reduce, one allreduce; on one rank the
        // reduce and the column in one launch, or in the pass itself)
        if (fold) {
          // (the pass ran the column)
        } else if (c->world == 1 && 2 * K2 + 2 <= 64 && lag_red_merge()) {
          hipEvent_t k1 = tmark(op, s);
          launch_gmres_lag_red(g, c2 + 1, op->partials, np, 2 * K2 + 2, 2 * K2 + 2, op->red + 16,
                               eps, ptol, stop_col, s);
          tspan(op, HH_SPAN_COLUMN, k1, tmark(op, s));
        } else {
          hipEvent_t k0 = tmark(op, s);
          launch_reduce(op->partials, np, 2 * K2 + 2, 2 * K2 + 2, op->red + 16, s, stp);
          tspan(op, HH_SPAN_MULTIDOT, k0, tmark(op, s));
          allreduce_sum_dev(op, op->red + 16, 2 * K2 + 2);
          hipEvent_t k1 = tmark(op, s);
          launch_gmres_lag(g, c2 + 1, op->red + 16, op->red + 16 + 2 * K2 + 1, false, eps, ptol,
                           stop_col, s);
          tspan(op, HH_SPAN_COLUMN, k1, tmark(op, s));
        }
        HIPC(hipGetLastError());
        check_site(c, "one-pass: reduce + allreduce + column", s);
      }
      {  // the last column's update and the norm that completes it
        const int K = stop_col + 1;
        hipEvent_t k0 = tmark(op, s);
        const bool fold_end = fold && merge_end;
        if (merge_end) {  // (with x += V a, V b: see cycle_coef_kernel)
          launch_cycle_coef(g, stop_col, op->cab, s);
          const PassFold pe = fold_end ? fold_at(stop_col + 1, op->red + 8) : PassFold{};
          launch_cycle_end(K, V, ldv, op->red + 16, g.vscale, op->cab, Wb[stop_col & 1], x,
                           V + (size_t)K * ldv, L, op->npart, blocks, s, stp,
                           fold_end ? &pe : nullptr);
        } else {
          launch_update(V, ldv, K, op->red + 16, g.vscale, Wb[stop_col & 1],
                        V + (size_t)K * ldv, L, op->npart, blocks, s, stp);
        }
        tspan(op, HH_SPAN_UPDATE, k0, tmark(op, s));
        if (fold_end) {
          // (the cycle end's own blocks reduced the norm and ran the final lag step)
        } else if (c->world == 1 && lag_red_merge()) {  // (the norm's reduce + the final lag step)
          launch_gmres_lag_red(g, stop_col + 1, op->npart, blocks, kMaxNorms, 1, op->red + 8, eps,
                               ptol, stop_col, s, 1);
        } else {
          launch_reduce(op->npart, blocks, kMaxNorms, 1, op->red + 8, s, stp);
          allreduce_sum_dev(op, op->red + 8, 1);
          launch_gmres_lag(g, stop_col + 1, nullptr, op->red + 8, true, eps, ptol, stop_col, s);
        }
        HIPC(hipGetLastError());
        check_site(c, "one-pass: cycle end", s);
      }
    }
    for (int c2 = 0; c2 <= stop_col && lagged; ++c2) {
      // ONE allreduce per inner iteration (lagged normalisation, gmres_lag_kernel): the norm of
      // the vector the previous update wrote (u_c2, its partials kept in npart) travels with
      // this iteration's raw dots; the Hessenberg subdiagonal of column c2-1 is completed from
      // it, one iteration late, and the SpMV meanwhile runs on a Pythagorean estimate of the
      // scale.  Same Krylov space, same H to rounding, same exit decisions (one wasted SpMV +
      // projection when a column stops the cycle).
      double2* vcol = V + (size_t)c2 * ldv;
      double2* w = V + (size_t)(c2 + 1) * ldv;
      const int* stp = g.ctrl;
      apply_MA(op, vcol, g.sscale + c2, w);  // w = M A (s_c2 u_c2)
      const int K = c2 + 1;
      hipEvent_t k0 = tmark(op, s);
      launch_multidot(V, ldv, K, w, L, op->partials, blocks, s, stp);
      launch_reduce(op->partials, blocks, 2 * K + 2, 2 * K + 1, op->red + 16, s, stp);
      if (c2 > 0) launch_reduce(op->npart, blocks, kMaxNorms, 1, op->red + 16 + 2 * K + 1, s, stp);
      tspan(op, HH_SPAN_MULTIDOT, k0, tmark(op, s));
      allreduce_sum_dev(op, op->red + 16, 2 * K + (c2 > 0 ? 2 : 1));
      hipEvent_t k1 = tmark(op, s);
      launch_gmres_lag(g, c2, op->red + 16, op->red + 16 + 2 * K + 1, false, eps, ptol, stop_col, s);
      hipEvent_t k2 = tmark(op, s);
      tspan(op, HH_SPAN_COLUMN, k1, k2);
      launch_update(V, ldv, K, op->red + 16, g.vscale, w, w, L, op->npart, blocks, s, stp);
      tspan(op, HH_SPAN_UPDATE, k2, tmark(op, s));
      HIPC(hipGetLastError());
      if (c2 == stop_col) {  // the cycle's last column needs the norm of the last update
        launch_reduce(op->npart, blocks, kMaxNorms, 1, op->red + 8, s, stp);
        allreduce_sum_dev(op, op->red + 8, 1);
        launch_gmres_lag(g, c2 + 1, nullptr, op->red + 8, true, eps, ptol, stop_col, s);
      }
    }
    for (int c2 = 0; c2 <= stop_col && !lagged && !fused; ++c2) {
      double2* vcol = V + (size_t)c2 * ldv;
      double2* w = V + (size_t)(c2 + 1) * ldv;
      const int* stp = g.ctrl;
      apply_MA(op, vcol, g.vscale + c2, w);  // w = M A v_col
      const int K = c2 + 1;
      // classical Gram-Schmidt: raw dots u_k^H w (+ |w|^2), then w -= sum h_k v_k, |w|^2
      // single rank, no second pass, HH_KRYLOV_FUSE: the multidot's last block reduces the dots
      // and / or the update's last block folds the norm and completes the column (bit-identical
      // to the separate launches)
      const int fuse = c->world == 1 && !reorth ? op->fuse_krylov : 0;
      if (fuse) {
        if (fuse & 1) {
          launch_multidot_reduced(V, ldv, K, w, L, op->partials, blocks, op->red + 16, 2 * K + 1,
                                  op->kcount, s, stp);
        } else {
          launch_multidot(V, ldv, K, w, L, op->partials, blocks, s, stp);
          launch_reduce(op->partials, blocks, 2 * K + 2, 2 * K + 1, op->red + 16, s, stp);
        }
        if (fuse & 2) {
          launch_update_column(V, ldv, K, op->red + 16, g.vscale, w, w, L, op->partials, blocks,
                               s, stp, g, c2, op->red + 16, eps, ptol, stop_col, op->kcount + 1);
        } else {
          launch_update(V, ldv, K, op->red + 16, g.vscale, w, w, L, op->partials, blocks, s, stp);
          launch_gmres_column(g, c2, op->red + 16, op->red + 8, op->partials, blocks, eps, ptol,
                              stop_col, s);
        }
        HIPC(hipGetLastError());
        continue;
      }
      hipEvent_t k0 = tmark(op, s);
      launch_multidot(V, ldv, K, w, L, op->partials, blocks, s, stp);
      launch_reduce(op->partials, blocks, 2 * K + 2, 2 * K + 1, op->red + 16, s, stp);
      tspan(op, HH_SPAN_MULTIDOT, k0, tmark(op, s));
      allreduce_sum_dev(op, op->red + 16, 2 * K + 1);
      // single rank: the column kernel sums the update's norm partials itself (one launch
      // fewer per iteration); across ranks they are reduced and allreduced first
      const bool fold = c->world == 1;
      hipEvent_t k1 = tmark(op, s);
      launch_update(V, ldv, K, op->red + 16, g.vscale, w, w, L, op->partials, blocks, s, stp);
      tspan(op, HH_SPAN_UPDATE, k1, tmark(op, s));
      if (!fold) {  // (with reorth this norm is superseded by the second pass's)
        launch_reduce(op->partials, blocks, kMaxNorms, 1, op->red + 8, s, stp);
        allreduce_sum_dev(op, op->red + 8, 1);
      }
      if (reorth) {
        // CGS2: project once more; the H column is the sum of both passes' dots, h0 stays
        // the first pass's |w| (scipy's h0 is taken before orthogonalisation).
        launch_multidot(V, ldv, K, w, L, op->partials, blocks, s, stp);
        launch_reduce(op->partials, blocks, 2 * K + 2, 2 * K, op->red + 96, s, stp);
        allreduce_sum_dev(op, op->red + 96, 2 * K);
        launch_update(V, ldv, K, op->red + 96, g.vscale, w, w, L, op->partials, blocks, s, stp);
        if (!fold) {
          launch_reduce(op->partials, blocks, kMaxNorms, 1, op->red + 8, s, stp);
          allreduce_sum_dev(op, op->red + 8, 1);
        }
        launch_add_small(op->red + 96, op->red + 16, 2 * K, s, stp);
      }
      hipEvent_t k2 = tmark(op, s);
      launch_gmres_column(g, c2, op->red + 16, op->red + 8, fold ? op->partials : nullptr, blocks,
                          eps, ptol, stop_col, s);
      tspan(op, HH_SPAN_COLUMN, k2, tmark(op, s));
      HIPC(hipGetLastError());
    }
    op->stop_flag = nullptr;  // (the SolveScope also clears it if anything above throws)
    // The cycle's report (per-iteration statuses + the last column executed) is copied behind
    // it, and the x update of the columns it executed is queued without waiting for it: the
    // merged end's finish or the triangular solve + x update, chosen on the device from that
    // last column (cycle_finish_kernel, gmres_solve_kernel, xupdate_kernel's ctl).  The host's
    // one sync per cycle is the residual norm's, below; the report is read after it.
    HIPC(hipMemcpyAsync(op->status_h, op->red, kRedReport * sizeof(double), hipMemcpyDeviceToHost,
                        s));
    if (merge_end)  // (with the triangular solve's decision and work: gmres_solve_kernel's)
      launch_cycle_finish(g, stop_col, V + (size_t)(stop_col + 1) * ldv, x, L, blocks, s);
    else
      launch_gmres_solve(g, stop_col, false, s);
    launch_xupdate(V, ldv, stop_col + 1, g.ycoef, x, L, blocks, s, g.ctrl);
    check_site(c, "cycle finish + triangular solve + x update", s);
    residual(op, b, x, V, 4);  // r = b - A x; V[0] = M r for the next cycle
    read_dev(op, op->red + 4, st, 1);
    const double* sth = op->status_h + kRedStatus;
    int ctl[2];
    std::memcpy(ctl, op->status_h + kRedCtrl, 2 * sizeof(int));
    {  // (the persistent sweep chain's wait bound)
      unsigned tmo = 0;
      std::memcpy(&tmo, op->status_h + kRedTimeout, sizeof(unsigned));
      if (tmo != 0) {
        HIPC(hipMemset(op->red + kRedTimeout, 0, sizeof(double)));
        fail(HH_ERR_STATE, "sweeping preconditioner: the persistent apply chain timed out "
                           "(workgroups not co-resident?); HH_SWEEP_CHAIN=0 selects one launch "
                           "per GEMV");
      }
    }
    col = ctl[1];
    REQUIRE(col >= 0 && col <= stop_col, "GMRES cycle state corrupt (last column %d)", col);
    replay(sth, col);
    presid = sth[4 * col];
    breakdown = sth[4 * col + 1] != 0.0;
    op->stats.restarts++;
    check_sweep_chain(op);  // (the M r of the last cycle is never read by a cycle report)
    rnorm = std::sqrt(st[0]);
    if (legacy && inner == maxiter) {
      finish(inner, rnorm <= atol ? 0 : (int)std::min<long>(maxiter, 0x7fffffff), rnorm);
      return HH_OK;
    }
    if (op->cycle_cb && op->cycle_cb(op->cycle_user, op->stats.restarts) != 0) {
      finish(inner, -1, rnorm);
      fail(HH_ERR_ABORTED, "gmres stopped by the cycle callback after cycle %ld",
           op->stats.restarts);
    }
    if (rnorm <= atol) break;
    else if (breakdown) break;
    else if (presid <= ptol) ptol_max_factor = std::max(eps, 0.25 * ptol_max_factor);
    else ptol_max_factor = std::min(1.0, 1.5 * ptol_max_factor);
    ptol = presid * std::min(ptol_max_factor, atol / rnorm);
  }
  finish(inner, rnorm <= atol ? 0 : (int)std::min<long>(maxiter, 0x7fffffff), rnorm);
  GUARD_END
}

