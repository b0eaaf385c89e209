// The halo exchange and the stencil / fused shifted-Laplace launches over a rank's slabs and
// across ranks, the preconditioners' applies (code.py:510-511's M slot), residuals and their
// reductions (see hh_runtime.hpp for the runtime's layout).
#include "hh_runtime.hpp"

namespace hh {

// Guarded allocations (HH_GUARD_HALO=1, diagnostic): each cross-rank halo receive buffer gets
// its own reserved address range, [unmapped granule][mapped granules][unmapped granule], and
// sits against the guard on the side a stray read would cross: the rows BELOW the slab (rows
// -H .. -1) start where the mapping starts, so a read of row -H-1 faults; the rows ABOVE it
// (nl .. nl+H-1) end where the mapping ends (`at_end`), so a read of row nl+H faults.  A kernel
// that reads one row beyond a received halo then faults at that access on every transport and
// grid size, instead of only where the allocator happened to leave the neighbouring address
// unmapped (the round-5 RCCL fault at 11584^2 / 8 ranks: DESIGN 4).
namespace {
struct GuardMap {
  char* va;        // reserved range: [guard][mapped][guard]
  size_t total;    // reserved bytes
  size_t mapped;   // mapped bytes (a multiple of the granule)
  hipMemGenericAllocationHandle_t h;
};
std::vector<std::pair<void*, GuardMap>>& guard_registry() {
  static std::vector<std::pair<void*, GuardMap>> r;
  return r;
}
}  // namespace

void* dalloc_guarded_bytes(size_t bytes, int device, bool at_end) {
  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  size_t gran = 0;
  HIPC(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
  GuardMap g{};
  g.mapped = (bytes + gran - 1) / gran * gran;
  g.total = g.mapped + 2 * gran;
  void* va = nullptr;
  HIPC(hipMemAddressReserve(&va, g.total, gran, nullptr, 0));
  g.va = static_cast<char*>(va);
  HIPC(hipMemCreate(&g.h, g.mapped, &prop, 0));
  HIPC(hipMemMap(g.va + gran, g.mapped, 0, g.h, 0));
  hipMemAccessDesc acc{};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  HIPC(hipMemSetAccess(g.va + gran, g.mapped, &acc, 1));
  char* p = g.va + gran + (at_end ? g.mapped - bytes : 0);
  guard_registry().push_back({p, g});
  return p;
}

void dfree(void* p) {
  if (!p) return;
  auto& reg = guard_registry();
  for (size_t k = 0; k < reg.size(); ++k) {
    if (reg[k].first != p) continue;
    const GuardMap g = reg[k].second;
    reg.erase(reg.begin() + (ptrdiff_t)k);
    const size_t gran = (g.total - g.mapped) / 2;
    (void)hipDeviceSynchronize();
    (void)hipMemUnmap(g.va + gran, g.mapped);
    (void)hipMemRelease(g.h);
    (void)hipMemAddressFree(g.va, g.total);
    return;
  }
  (void)hipFree(p);
}

void ensure_scratch(hh_op* op) {
  if (!op->scrT) op->scrT = dalloc<double2>(op->nloc);
  if (!op->scrZ) op->scrZ = dalloc<double2>(op->nloc);
}

// timing marks (no-ops unless hh_op_set_timing enabled them)
hipEvent_t tmark(hh_op* op, hipStream_t s) { return op->timer.on ? op->timer.mark(s) : nullptr; }
void tspan(hh_op* op, int cat, hipEvent_t a, hipEvent_t b, bool clamp) {
  if (op->timer.on) op->timer.span(cat, a, b, clamp);
}

// HH_CHECK_HALO (diagnostic, off by default): after every halo exchange, launch group and
// collective of the multi-rank paths, synchronise the stream it was queued on and attribute a
// device fault to that site (rank, site, running check number) instead of to the next host sync
// far behind it.  1: check; 2: also trace every site to stderr.  The streams are serialised by
// it, so it also tells a hazard between the halo and compute streams (passes when checked) from
// a fault of one launch (reported at its own site).
void check_site(const hh_ctx* c, const char* site, hipStream_t s) {
  const long lvl = knobs().check_halo;
  if (lvl == 0) return;
  static thread_local long count = 0;
  ++count;
  const hipError_t e = hipStreamSynchronize(s);
  const char* sname = s == c->cstream ? "halo" : "compute";
  if (e != hipSuccess) {
    std::fprintf(stderr, "[HH_CHECK_HALO] rank %d/%d: FAULT at %s (check #%ld, %s stream): %s\n",
                 c->rank, c->world, site, count, sname, hipGetErrorString(e));
    std::fflush(stderr);
    fail(HH_ERR_HIP, "[HH_CHECK_HALO] rank %d: %s (check #%ld, %s stream) -> %s", c->rank, site,
         count, sname, hipGetErrorString(e));
  }
  if (lvl >= 2) {
    std::fprintf(stderr, "[HH_CHECK_HALO] rank %d: ok %s (#%ld, %s)\n", c->rank, site, count, sname);
    std::fflush(stderr);
  }
}

void allreduce_sum_dev(hh_op* op, double* d, int count) {
  hh_ctx* c = op->ctx;
  if (c->world > 1) {
    check_site(c, "before allreduce", c->stream);
    hipEvent_t a = tmark(op, c->stream);
    c->comm->allreduce(d, count, false, c->stream);
    tspan(op, HH_SPAN_ALLREDUCE, a, tmark(op, c->stream));
    check_site(c, "allreduce (RCCL kernel)", c->stream);
  }
}

// Halo exchange for rank-local vector `in` and stencil launch of `epi` over all slabs.
// Returns the number of partial rows written at op->partials.
int run_stencil(hh_op* op, int epi, const double2* in, const double* in_scale,
                const double2* in1, double2* out0, double2* out1, bool shifted) {
  hh_ctx* c = op->ctx;
  const int n = op->n;
  const int S = (int)op->slabs.size();
  const bool lo_x = c->world > 1 && c->rank > 0;             // cross-rank halo below
  const bool hi_x = c->world > 1 && c->rank < c->world - 1;  // cross-rank halo above
  hipEvent_t t_ready = nullptr, t_halo = nullptr, t_int1 = nullptr;
  if (lo_x || hi_x) {
    const Slab& s0 = op->slabs[0];
    const Slab& sl = op->slabs[S - 1];
    t_ready = tmark(op, c->stream);  // (the input is complete: the exchange may start)
    check_site(c, "stencil: work before the exchange", c->stream);
    c->comm->halo(lo_x ? in + s0.off : nullptr, lo_x ? s0.halo_lo_buf : nullptr,
                  hi_x ? in + sl.off + (size_t)(sl.nl - 1) * n : nullptr,
                  hi_x ? sl.halo_hi_buf : nullptr, 2 * sizeof(double) * (size_t)n, c->stream,
                  c->cstream, c->ev_in);
    t_halo = tmark(op, c->cstream);
    tspan(op, HH_SPAN_HALO, t_ready, t_halo);
    check_site(c, "stencil: one-row halo exchange", c->cstream);
  }

  auto make_args = [&](int si) {
    const Slab& s = op->slabs[si];
    StencilArgs a{};
    a.u = in + s.off;
    // Local neighbour slabs on the same device are read in place; cross-rank halos land in
    // the receive buffers; the global boundary reads a zero row (homogeneous Dirichlet).
    if (si > 0) a.halo_lo = in + op->slabs[si - 1].off + (size_t)(op->slabs[si - 1].nl - 1) * n;
    else a.halo_lo = lo_x ? s.halo_lo_buf : op->zero_row;
    if (si < S - 1) a.halo_hi = in + op->slabs[si + 1].off;
    else a.halo_hi = hi_x ? s.halo_hi_buf : op->zero_row;
    a.invc2 = op->const_c ? nullptr : s.invc2;
    a.invc2_const = op->invc2_const;
    a.tab_i = op->tab_i;
    a.tab_j = s.tab_j;
    a.n = n;
    a.nl = s.nl;
    a.mshift = shifted ? op->mshift : make_double2(1.0, 0.0);
    a.damping = op->damping;
    a.in_scale = in_scale;
    a.tab_r2x = op->points == 9 ? s.tab_r2x : nullptr;
    a.w9 = op->w9;
    a.in1 = in1 ? in1 + s.off : nullptr;
    a.out0 = out0 ? out0 + s.off : nullptr;
    a.out1 = out1 ? out1 + s.off : nullptr;
    a.stop = op->stop_flag;
    return a;
  };

  int nparts = 0;
  auto launch_rows = [&](int si, int r0, int r1, int rpb, int step = 0,
                         hipStream_t st = nullptr) {
    if (r1 <= r0) return;
    StencilArgs a = make_args(si);
    a.row_begin = r0;
    a.row_end = r1;
    a.row_step = step;
    a.rows_per_block = (op->rpb_override > 0 && rpb > 1) ? std::min(op->rpb_override, r1 - r0) : rpb;
    a.grid_blocks = op->grid_override;
    a.partials = op->partials + (size_t)nparts * kMaxNorms;
    REQUIRE((size_t)(nparts + stencil_grid_blocks(n, r1 - r0, a.rows_per_block, step)) * kMaxNorms <=
                op->partials_cap,
            "partials workspace too small for the stencil launch");
    int written = 0;
    const int variant = (op->variant < 0 && op->stop_flag) ? kVariantInSolve : op->variant;
    launch_stencil(epi, op->const_c, a, &written, st ? st : c->stream, variant);
    nparts += written;
  };

  // interior (independent of cross-rank halos) first, then the dependent boundary rows
  bool first = true;
  hipEvent_t t_int0 = tmark(op, c->stream);
  for (int si = 0; si < S; ++si) {
    const Slab& s = op->slabs[si];
    const int r0 = (si == 0 && lo_x) ? 1 : 0;
    const int r1 = (si == S - 1 && hi_x) ? s.nl - 1 : s.nl;
    if (first && op->tk0) HIPC(hipEventRecord(op->tk0, c->stream));
    launch_rows(si, r0, r1, s.rpb);
    if (first && op->tk1) HIPC(hipEventRecord(op->tk1, c->stream));
    first = false;
  }
  t_int1 = tmark(op, c->stream);
  tspan(op, HH_SPAN_INTERIOR, t_int0, t_int1);
  if (lo_x || hi_x) check_site(c, "stencil: interior rows", c->stream);
  if (lo_x || hi_x) {
    // The boundary rows run on the halo stream, right behind the exchange (which it ordered
    // after everything the compute stream had queued), concurrently with the interior launch;
    // they read the same input and write disjoint rows and partial slots.  The compute stream
    // then waits for them.
    hipStream_t hs = c->cstream;
    const Slab& s0 = op->slabs[0];
    const Slab& sl = op->slabs[S - 1];
    if (S == 1 && s0.nl == 1) {
      launch_rows(0, 0, 1, 1, 0, hs);
    } else if (S == 1 && lo_x && hi_x) {
      launch_rows(0, 0, s0.nl, 1, s0.nl - 1, hs);  // rows 0 and nl-1: one launch of two bands
    } else {
      if (lo_x) launch_rows(0, 0, 1, 1, 0, hs);
      if (hi_x) launch_rows(S - 1, sl.nl - 1, sl.nl, 1, 0, hs);
    }
    check_site(c, "stencil: boundary rows", hs);
    hipEvent_t t_bnd = tmark(op, hs);
    tspan(op, HH_SPAN_BOUNDARY, t_halo, t_bnd);
    tspan(op, HH_SPAN_HALO_WAIT, t_int1, t_bnd, true);  // compute stream idle behind the halo
    HIPC(hipEventRecord(c->ev_halo, hs));
    HIPC(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
  }
  HIPC(hipGetLastError());
  op->stats.spmv_count++;
  return nparts;
}

// w = M A (s v) for the two-sweep shifted-Laplace M in one launch per slab (sl_fused.hip): T
// and the first sweep never leave the chip.  A band reads v two rows beyond its own rows and
// evaluates the first sweep on its two halo rows, so the slab needs two halo rows per side
// (exchanged here across ranks; read in place from a neighbouring slab on the same device) and
// the medium and PML tables two layers beyond it (Slab::tab_j_ext, invc2_halo).
bool sl_fused_applies(const hh_op* op) {
  return op->sl_fuse && op->sweeps == 2 && op->sl_ext_ok;
}
void run_sl2(hh_op* op, const double2* v, const double* vs, double2* out) {
  hh_ctx* c = op->ctx;
  const int n = op->n;
  const int S = (int)op->slabs.size();
  const bool lo_x = c->world > 1 && c->rank > 0;
  const bool hi_x = c->world > 1 && c->rank < c->world - 1;
  hipEvent_t t_halo = nullptr;
  if (lo_x || hi_x) {
    const Slab& s0 = op->slabs[0];
    const Slab& sl = op->slabs[S - 1];
    hipEvent_t t_ready = tmark(op, c->stream);
    check_site(c, "sl2 (fused M A): work before the exchange", c->stream);
    c->comm->halo(lo_x ? v + s0.off : nullptr, lo_x ? s0.halo2_lo : nullptr,
                  hi_x ? v + sl.off + (size_t)(sl.nl - 2) * n : nullptr,
                  hi_x ? sl.halo2_hi : nullptr, 2 * 2 * sizeof(double) * (size_t)n, c->stream,
                  c->cstream, c->ev_in);
    t_halo = tmark(op, c->cstream);
    tspan(op, HH_SPAN_HALO, t_ready, t_halo);
    check_site(c, "sl2 (fused M A): two-row halo exchange", c->cstream);
  }
  auto launch_rows = [&](int si, int r0, int r1, int rpb, int step, hipStream_t st) {
    if (r1 <= r0) return;
    const Slab& s = op->slabs[si];
    StencilArgs a{};
    a.u = v + s.off;
    a.halo_lo = si > 0 ? v + op->slabs[si - 1].off + (size_t)(op->slabs[si - 1].nl - 2) * n
                       : (lo_x ? s.halo2_lo : op->zero_row);
    a.halo_hi = si < S - 1 ? v + op->slabs[si + 1].off : (hi_x ? s.halo2_hi : op->zero_row);
    a.invc2 = op->const_c ? nullptr : s.invc2;
    a.invc2_halo = s.invc2_halo;
    a.invc2_const = op->invc2_const;
    a.tab_i = op->tab_i;
    a.tab_j = s.tab_j;  // row 0 of tab_j_ext: rows -2 .. nl+1 are valid
    a.j0 = s.j0;
    a.n = n;
    a.nl = s.nl;
    a.row_begin = r0;
    a.row_end = r1;
    a.row_step = step;
    a.rows_per_block = (op->rpb_override > 0 && rpb > 2) ? std::min(op->rpb_override, r1 - r0) : rpb;
    a.mshift = op->mshift;
    a.damping = op->damping;
    a.in_scale = vs;
    a.out0 = out + s.off;
    a.stop = op->stop_flag;
    a.tab_r2x = op->points == 9 ? s.tab_r2x : nullptr;  // selects the 9-point kernel
    a.w9 = op->w9;
    launch_sl2(op->const_c, a, st, op->variant);
  };
  // interior rows (no cross-rank halo needed: a band reads two rows beyond itself) first
  hipEvent_t t_int0 = tmark(op, c->stream);
  for (int si = 0; si < S; ++si) {
    const Slab& s = op->slabs[si];
    const int r0 = (si == 0 && lo_x) ? 2 : 0;
    const int r1 = (si == S - 1 && hi_x) ? s.nl - 2 : s.nl;
    if (si == 0 && op->tk0) HIPC(hipEventRecord(op->tk0, c->stream));
    launch_rows(si, r0, r1, s.rpb, 0, c->stream);
    if (si == 0 && op->tk1) HIPC(hipEventRecord(op->tk1, c->stream));
  }
  hipEvent_t t_int1 = tmark(op, c->stream);
  tspan(op, HH_SPAN_INTERIOR, t_int0, t_int1);
  if (lo_x || hi_x) check_site(c, "sl2 (fused M A): interior rows", c->stream);
  if (lo_x || hi_x) {
    // the two rows next to each cross-rank boundary, on the halo stream behind the exchange
    hipStream_t hs = c->cstream;
    const Slab& s0 = op->slabs[0];
    const Slab& sl = op->slabs[S - 1];
    if (S == 1 && lo_x && hi_x) {
      if (s0.nl < 4) launch_rows(0, 0, s0.nl, s0.nl, 0, hs);     // (no interior rows)
      else launch_rows(0, 0, s0.nl, 2, s0.nl - 2, hs);          // rows 0-1 and nl-2 - nl-1
    } else {
      if (lo_x) launch_rows(0, 0, std::min(2, s0.nl), 2, 0, hs);
      if (hi_x) launch_rows(S - 1, std::max(0, sl.nl - 2), sl.nl, 2, 0, hs);
    }
    check_site(c, "sl2 (fused M A): boundary rows", hs);
    hipEvent_t t_bnd = tmark(op, hs);
    tspan(op, HH_SPAN_BOUNDARY, t_halo, t_bnd);
    tspan(op, HH_SPAN_HALO_WAIT, t_int1, t_bnd, true);
    HIPC(hipEventRecord(c->ev_halo, hs));
    HIPC(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
  }
  HIPC(hipGetLastError());
  op->stats.spmv_count++;
}

// Pointwise op over all local slabs; returns partial rows written.
int run_point(hh_op* op, int pt, const double2* in0, double2* out0, bool shifted) {
  hh_ctx* c = op->ctx;
  int nparts = 0;
  for (const Slab& s : op->slabs) {
    PointArgs a{};
    a.in0 = in0 ? in0 + s.off : nullptr;
    a.out0 = out0 ? out0 + s.off : nullptr;
    a.invc2 = op->const_c ? nullptr : s.invc2;
    a.invc2_const = op->invc2_const;
    a.tab_i = op->tab_i;
    a.tab_j = s.tab_j;
    a.n = op->n;
    a.nl = s.nl;
    a.mshift = shifted ? op->mshift : make_double2(1.0, 0.0);
    a.damping = op->damping;
    a.partials = op->partials + (size_t)nparts * kMaxNorms;
    a.stop = op->stop_flag;
    a.s9 = op->points == 9 ? 1 : 0;
    a.w9 = op->w9;
    const int blocks = point_blocks((size_t)s.nl * op->n);
    REQUIRE((size_t)(nparts + blocks) * kMaxNorms <= op->partials_cap,
            "partials workspace too small for the pointwise launch");
    launch_point(pt, op->const_c, a, blocks, c->stream);
    nparts += blocks;
  }
  HIPC(hipGetLastError());
  return nparts;
}

// reduce the first `cols` columns of `nparts` partial rows (row width kMaxNorms) into
// op->red[dst..dst+cols), then allreduce across ranks
void reduce_norms(hh_op* op, int nparts, int dst, int cols) {
  launch_reduce(op->partials, nparts, kMaxNorms, cols, op->red + dst, op->ctx->stream);
  check_site(op->ctx, "norm reduce", op->ctx->stream);
  allreduce_sum_dev(op, op->red + dst, cols);
}

// SL sweeps: z_1 already computed into `z1dst`; performs sweeps 2..s with r = T; the last
// iterate lands in `out`.  `z1dst` must be chosen by sl_first_dst().
void sl_sweeps(hh_op* op, const double2* T, double2* z1dst, double2* out) {
  double2* cur = z1dst;
  for (int k = 2; k <= op->sweeps; ++k) {
    double2* dst = ((op->sweeps - k) % 2 == 0) ? out : op->scrZ;
    if (dst == cur) dst = (cur == out) ? op->scrZ : out;
    run_stencil(op, EPI_SL_SWEEP, cur, nullptr, T, dst, nullptr, true);
    cur = dst;
  }
  if (cur != out) launch_scale_copy(cur, out, op->nloc, 1.0, op->ctx->stream, op->stop_flag);
}
double2* sl_first_dst(hh_op* op, double2* out) {
  return ((op->sweeps - 1) % 2 == 0) ? out : op->scrZ;
}


// out = M A (s * v)
void apply_MA(hh_op* op, const double2* v, const double* vs, double2* out) {
  switch (op->pkind) {
    case HH_PREC_NONE:
      run_stencil(op, EPI_AX, v, vs, nullptr, out, nullptr, false);
      break;
    case HH_PREC_JACOBI:
      run_stencil(op, EPI_JAC, v, vs, nullptr, out, nullptr, false);
      break;
    case HH_PREC_SHIFTED_LAPLACE: {
      if (sl_fused_applies(op)) {
        run_sl2(op, v, vs, out);
        break;
      }
      ensure_scratch(op);
      double2* z1 = sl_first_dst(op, out);
      run_stencil(op, EPI_SL_FIRST, v, vs, nullptr, op->scrT, z1, true);
      sl_sweeps(op, op->scrT, z1, out);
      break;
    }
    case HH_PREC_SWEEP:
      ensure_scratch(op);
      run_stencil(op, EPI_AX, v, vs, nullptr, op->scrT, nullptr, false);
      sweep_apply(op, op->scrT, out, false);
      break;
    case HH_PREC_SWEEP_REF:
      // code.py:510-511 (quirk Q1): the preconditioner ignores its argument
      REQUIRE(op->sw_const, "as-is sweeping preconditioner needs its right-hand side (hh_gmres)");
      launch_scale_copy(op->sw_const, out, op->nloc, 1.0, op->ctx->stream, op->stop_flag);
      break;
  }
}

// out = M r (no norms).  r and out must differ.
void apply_M(hh_op* op, const double2* r, double2* out) {
  switch (op->pkind) {
    case HH_PREC_NONE:
      launch_scale_copy(r, out, op->nloc, 1.0, op->ctx->stream);
      break;
    case HH_PREC_JACOBI:
      run_point(op, PT_JAC, r, out, false);
      break;
    case HH_PREC_SHIFTED_LAPLACE: {
      ensure_scratch(op);
      double2* z1 = sl_first_dst(op, out);
      run_point(op, PT_SL_FIRST, r, z1, true);
      sl_sweeps(op, r, z1, out);
      break;
    }
    case HH_PREC_SWEEP:
      sweep_apply(op, r, out, false);
      break;
    case HH_PREC_SWEEP_REF:
      if (op->sw_const)  // inside hh_gmres: constant map (quirk Q1)
        launch_scale_copy(op->sw_const, out, op->nloc, 1.0, op->ctx->stream, op->stop_flag);
      else               // plain apply: algo2_4 as-is (quirk Q2) on the given vector
        sweep_apply(op, r, out, true);
      break;
  }
}

// |v|^2 -> op->red[dst] (allreduced)
void norm2(hh_op* op, const double2* v, int dst) {
  const int np = run_point(op, PT_COPY_NORM, v, nullptr, false);
  reduce_norms(op, np, dst, 1);
}

// v0 = M (b - A x); red[dst] = |b - A x|^2, red[dst+1] = |v0|^2
// The shifted-Laplace residual v0 = M (b - A x) in one pass (sl_fused.hip sl2_res_kernel) where
// it applies: the 5-point operator, the two-sweep M with the medium known two layers beyond
// every slab (as for the fused M A, run_sl2); HH_SL_RES=0 keeps the three launches (r and z1,
// the second sweep, |M r|^2).  v0 is bit-identical either way; the norms are summed in another
// order.  Independent of the M A fusion switch (hh_op_set_sl_fusion: that A/B stays
// bit-identical).
bool sl_res_fused(const hh_op* op) {
  return knobs().sl_res != 0 && op->points == 5 && op->sweeps == 2 && op->sl_ext_ok;
}

// run_sl2's structure: a band reads x AND b two rows beyond itself -- in place from a
// neighbouring slab of the rank, from the two-row halo buffers across ranks (b's exchanged
// beside x's, every call: b may change between solves), zero rows off the grid; the rows next
// to a cross-rank boundary run on the halo stream after the exchange.
void run_sl2_res(hh_op* op, const double2* b, const double2* x, double2* v0, int dst) {
  hh_ctx* c = op->ctx;
  const int n = op->n;
  const int S = (int)op->slabs.size();
  const bool lo_x = c->world > 1 && c->rank > 0;
  const bool hi_x = c->world > 1 && c->rank < c->world - 1;
  const Slab& s0 = op->slabs[0];
  const Slab& sl = op->slabs[S - 1];
  if (lo_x || hi_x) {
    const size_t two = 2 * (size_t)n;
    if (!op->res_bh_lo) {
      op->res_bh_lo = dalloc_guarded<double2>(two, c->device, false);
      op->res_bh_hi = dalloc_guarded<double2>(two, c->device, true);
      HIPC(hipMemsetAsync(op->res_bh_lo, 0, two * sizeof(double2), c->stream));
      HIPC(hipMemsetAsync(op->res_bh_hi, 0, two * sizeof(double2), c->stream));
    }
    const size_t bytes = two * sizeof(double2);
    check_site(c, "sl2_res: work before the exchanges", c->stream);
    c->comm->halo(lo_x ? b + s0.off : nullptr, lo_x ? op->res_bh_lo : nullptr,
                  hi_x ? b + sl.off + (size_t)(sl.nl - 2) * n : nullptr,
                  hi_x ? op->res_bh_hi : nullptr, bytes, c->stream, c->cstream, c->ev_in);
    check_site(c, "sl2_res: b's two-row halo exchange", c->cstream);
    c->comm->halo(lo_x ? x + s0.off : nullptr, lo_x ? s0.halo2_lo : nullptr,
                  hi_x ? x + sl.off + (size_t)(sl.nl - 2) * n : nullptr,
                  hi_x ? sl.halo2_hi : nullptr, bytes, c->stream, c->cstream, c->ev_in);
    check_site(c, "sl2_res: x's two-row halo exchange", c->cstream);
  }
  int np = 0;
  auto launch_rows = [&](int si, int r0, int r1, int rpb, hipStream_t st) {
    if (r1 <= r0) return;
    const Slab& s = op->slabs[si];
    const size_t prev_tail =
        si > 0 ? op->slabs[si - 1].off + (size_t)(op->slabs[si - 1].nl - 2) * n : 0;
    const size_t next_head = si < S - 1 ? op->slabs[si + 1].off : 0;
    StencilArgs a{};
    a.u = x + s.off;
    a.halo_lo = si > 0 ? x + prev_tail : (lo_x ? s.halo2_lo : op->zero_row);
    a.halo_hi = si < S - 1 ? x + next_head : (hi_x ? s.halo2_hi : op->zero_row);
    a.in1 = b + s.off;
    a.in1_lo = si > 0 ? b + prev_tail : (lo_x ? op->res_bh_lo : op->zero_row);
    a.in1_hi = si < S - 1 ? b + next_head : (hi_x ? op->res_bh_hi : op->zero_row);
    a.invc2 = op->const_c ? nullptr : s.invc2;
    a.invc2_halo = s.invc2_halo;
    a.invc2_const = op->invc2_const;
    a.tab_i = op->tab_i;
    a.tab_j = s.tab_j;
    a.j0 = s.j0;
    a.n = n;
    a.nl = s.nl;
    a.row_begin = r0;
    a.row_end = r1;
    a.rows_per_block = rpb;
    a.mshift = op->mshift;
    a.damping = op->damping;
    a.out0 = v0 + s.off;
    a.partials = op->partials + (size_t)np * kMaxNorms;
    REQUIRE((size_t)(np + sl2_res_blocks(n, r1 - r0, rpb)) * kMaxNorms <= op->partials_cap,
            "partials workspace too small for the shifted-Laplace residual");
    np += launch_sl2_res(op->const_c, a, st);
  };
  // interior rows (no cross-rank halo needed) first
  for (int si = 0; si < S; ++si) {
    const Slab& s = op->slabs[si];
    const int r0 = (si == 0 && lo_x) ? std::min(2, s.nl) : 0;
    const int r1 = (si == S - 1 && hi_x) ? std::max(r0, s.nl - 2) : s.nl;
    launch_rows(si, r0, r1, s.rpb, c->stream);
  }
  if (lo_x || hi_x) check_site(c, "sl2_res: interior rows", c->stream);
  if (lo_x || hi_x) {
    // the two rows next to each cross-rank boundary, on the halo stream behind the exchange
    hipStream_t hs = c->cstream;
    if (S == 1 && lo_x && hi_x && s0.nl < 4) {
      launch_rows(0, 0, s0.nl, s0.nl, hs);  // (no interior rows)
    } else {
      if (lo_x) launch_rows(0, 0, std::min(2, s0.nl), 2, hs);
      if (hi_x) launch_rows(S - 1, std::max(0, sl.nl - 2), sl.nl, 2, hs);
    }
    check_site(c, "sl2_res: boundary rows", hs);
    HIPC(hipEventRecord(c->ev_halo, hs));
    HIPC(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
  }
  HIPC(hipGetLastError());
  reduce_norms(op, np, dst, 2);  // red[dst] = |r|^2, red[dst + 1] = |M r|^2
}

void residual(hh_op* op, const double2* b, const double2* x, double2* v0, int dst) {
  switch (op->pkind) {
    case HH_PREC_NONE: {
      const int np = run_stencil(op, EPI_RES, x, nullptr, b, v0, nullptr, false);
      reduce_norms(op, np, dst, 1);  // (|M r| = |r|: readers take red[dst], see mnorm_slot)
      break;
    }
    case HH_PREC_JACOBI: {
      const int np = run_stencil(op, EPI_RES_JAC, x, nullptr, b, v0, nullptr, false);
      reduce_norms(op, np, dst, 2);
      break;
    }
    case HH_PREC_SHIFTED_LAPLACE: {
      if (sl_res_fused(op)) {  // one pass: v0 = M r with |r|^2 and |M r|^2
        run_sl2_res(op, b, x, v0, dst);
        break;
      }
      ensure_scratch(op);
      // r must survive the sweeps: it lives in scrR, distinct from scrT/scrZ/v0.
      if (!op->scrR) op->scrR = dalloc<double2>(op->nloc);
      double2* z1 = sl_first_dst(op, v0);
      const int np = run_stencil(op, EPI_RES_SL, x, nullptr, b, op->scrR, z1, true);
      reduce_norms(op, np, dst, 1);  // red[dst] = |r|^2
      sl_sweeps(op, op->scrR, z1, v0);
      norm2(op, v0, dst + 1);
      break;
    }
    case HH_PREC_SWEEP:
    case HH_PREC_SWEEP_REF: {
      if (!op->scrR) op->scrR = dalloc<double2>(op->nloc);
      const int np = run_stencil(op, EPI_RES, x, nullptr, b, op->scrR, nullptr, false);
      reduce_norms(op, np, dst, 1);  // red[dst] = |r|^2
      apply_M(op, op->scrR, v0);
      norm2(op, v0, dst + 1);
      break;
    }
  }
}

int device_cus(hh_ctx* c) {
  static int cus = 0;  // (one device model per process)
  if (cus == 0) HIPC(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
  return cus;
}

// where residual(op, .., dst) left |M r|^2: red[dst + 1], or red[dst] itself for M = none
int mnorm_slot(const hh_op* op, int dst) { return op->pkind == HH_PREC_NONE ? dst : dst + 1; }

void read_dev(hh_op* op, const double* dsrc, double* hdst, int count) {
  check_site(op->ctx, "queued work before a host read", op->ctx->stream);
  HIPC(hipMemcpyAsync(op->status_h, dsrc, count * sizeof(double), hipMemcpyDeviceToHost,
                      op->ctx->stream));
  HIPC(hipStreamSynchronize(op->ctx->stream));
  std::memcpy(hdst, op->status_h, count * sizeof(double));
}

}  // namespace hh
