// Host runtime behind the C ABI (include/helmholtz_amd.h): device context + RCCL rank,
// the row-slab operator (PML tables, pre-transposed 1/c^2), halo exchange, apply modes,
// preconditioners and the restarted GMRES driver with scipy's control flow.
//
// Reference boundary (code.py, bocchs/helmholtz-preconditioner):
//   build_A_matrix(b, const, eta, omega, h, n, c_mat)  code.py:202   -> hh_op_create
//   A @ x (LinearOperator.matvec -> csr_matvec)          code.py:516   -> hh_op_apply(_dev)
//   scipy.sparse.linalg.gmres(A, f, M=M, tol=1e-3, ...)  code.py:516   -> hh_gmres
//   M slot LinearOperator(matvec=...)                    code.py:510   -> hh_op_set_precond
#include "hh_runtime.hpp"

namespace hh {

thread_local std::string g_err = "";

// --------------------------------------------------------------- PML profiles
// sigma1/sigma2/s1/s2 exactly as code.py:11-33 (s2 one-sided: quirk Q4).
static double sigma1(double x, double C, double eta) {
  if (x <= eta) return C / eta * ((x - eta) / eta) * ((x - eta) / eta);
  if (x >= 1 - eta) return C / eta * ((x - 1 + eta) / eta) * ((x - 1 + eta) / eta);
  return 0.0;
}
static double sigma2(double x, double C, double eta) {
  if (x <= eta) return C / eta * ((x - eta) / eta) * ((x - eta) / eta);
  return 0.0;
}
static cd s1(double x, double C, double eta, cd om) {
  return 1.0 / (1.0 + cd(0, 1) * sigma1(x, C, eta) / om);
}
static cd s2(double x, double C, double eta, cd om) {
  return 1.0 / (1.0 + cd(0, 1) * sigma2(x, C, eta) / om);
}
static double2 d2(cd z) { return make_double2(z.real(), z.imag()); }

bool under_profiler() {
  static const bool on = [] {
    const char* pre = std::getenv("LD_PRELOAD");
    const bool p = std::getenv("ROCPROFILER_LIBRARY_CTOR") || std::getenv("ROCPROF_OUTPUT_PATH") ||
                   (pre && std::strstr(pre, "rocprofiler"));
    if (p)
      std::fprintf(stderr, "[helmholtz_amd] rocprofv3 detected: grid-wide sweeps and the "
                           "small-grid cycle use plain launches (no cooperative launch: ROCm's "
                           "exit-time queue teardown after rocprofiler-sdk finalised, DESIGN 3b)\n");
    return p;
  }();
  return on;
}

}  // namespace hh

HH_API int hh_abi_version(void) { return HH_ABI_VERSION; }
HH_API const char* hh_last_error(void) { return g_err.c_str(); }

HH_API int hh_device_count(int* count) {
  GUARD_BEGIN
  REQUIRE(count, "null count");
  HIPC(hipGetDeviceCount(count));
  GUARD_END
}

HH_API int hh_comm_unique_id(unsigned char id_out[128]) {
  GUARD_BEGIN
  REQUIRE(id_out, "null id");
  rccl_unique_id(id_out);
  GUARD_END
}

HH_API int hh_comm_selftest(int device, double* allreduce_err, double* p2p_err) {
  GUARD_BEGIN
  REQUIRE(allreduce_err && p2p_err, "null output");
  int ndev = 0;
  HIPC(hipGetDeviceCount(&ndev));
  REQUIRE(device >= 0 && device < ndev, "device %d not present (%d devices)", device, ndev);
  rccl_selftest(device, allreduce_err, p2p_err);
  GUARD_END
}

HH_API int hh_ctx_create_ex(int device, int rank, int world, const unsigned char* id,
                            int virtual_slabs, int transport, hh_ctx** out) {
  GUARD_BEGIN
  REQUIRE(out, "null ctx out");
  REQUIRE(world >= 1 && rank >= 0 && rank < world, "bad rank %d / world %d", rank, world);
  REQUIRE(virtual_slabs >= 1 && virtual_slabs <= 64, "virtual_slabs must be in [1, 64]");
  REQUIRE(world == 1 || id, "world > 1 needs a communicator id from rank 0");
  REQUIRE(transport == TRANSPORT_RCCL || transport == TRANSPORT_SHM, "unknown transport %d",
          transport);
  (void)knobs();  // every HH_* knob read here, once per process (a malformed one fails here)
  int ndev = 0;
  HIPC(hipGetDeviceCount(&ndev));
  REQUIRE(device >= 0 && device < ndev, "device %d not present (%d devices)", device, ndev);
  HIPC(hipSetDevice(device));
  std::unique_ptr<hh_ctx> c(new hh_ctx());
  c->device = device;
  c->rank = rank;
  c->world = world;
  c->vslabs = virtual_slabs;
  c->transport = transport;
  try {
    HIPC(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    // The halo stream runs the exchange (RCCL send/recv kernels) and the boundary rows
    // concurrently with the interior stencil launch, which alone fills every CU: give it the
    // highest priority so the dispatcher places its few blocks first instead of behind the
    // interior grid.
    int prio_least = 0, prio_greatest = 0;
    HIPC(hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest));
    HIPC(hipStreamCreateWithPriority(&c->cstream, hipStreamNonBlocking, prio_greatest));
    HIPC(hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming));
    HIPC(hipEventCreateWithFlags(&c->ev_halo, hipEventDisableTiming));
    c->dscratch = dalloc<double>(256);
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&c->hpinned), 256 * sizeof(double)));
    if (world > 1)
      c->comm = transport == TRANSPORT_RCCL ? make_rccl_comm(rank, world, id)
                                            : make_shm_comm(rank, world, id);
  } catch (...) {
    if (c->ev_in) (void)hipEventDestroy(c->ev_in);
    if (c->ev_halo) (void)hipEventDestroy(c->ev_halo);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    dfree(c->dscratch);
    if (c->hpinned) (void)hipHostFree(c->hpinned);
    throw;
  }
  *out = c.release();
  GUARD_END
}

HH_API int hh_ctx_create(int device, int rank, int world, const unsigned char* nccl_id,
                         int virtual_slabs, hh_ctx** out) {
  return hh_ctx_create_ex(device, rank, world, nccl_id, virtual_slabs, TRANSPORT_RCCL, out);
}

// Lifetimes: hh_*_destroy releases the caller's handle; an object is freed when its last
// dependent is gone too (a context outlives its operators, an operator its vectors), so no
// destroy order -- e.g. a garbage collector's -- can leave a dangling context or operator.
static void ctx_release(hh_ctx* c) {
  if (--c->refs > 0) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  c->comm.reset();
  (void)hipEventDestroy(c->ev_in);
  (void)hipEventDestroy(c->ev_halo);
  (void)hipStreamDestroy(c->stream);
  (void)hipStreamDestroy(c->cstream);
  dfree(c->dscratch);
  if (c->hpinned) (void)hipHostFree(c->hpinned);
  (void)hipGetLastError();  // teardown errors are not reported to a later call
  delete c;
}

HH_API int hh_ctx_destroy(hh_ctx* c) {
  GUARD_BEGIN
  if (!c) return HH_OK;
  ctx_release(c);
  GUARD_END
}

static void host_allreduce(hh_ctx* c, double* v, int count, bool max) {
  REQUIRE(v && count >= 0 && count <= 256, "bad allreduce buffer");
  if (c->world == 1 || count == 0) return;
  HIPC(hipSetDevice(c->device));
  HIPC(hipMemcpyAsync(c->dscratch, v, count * sizeof(double), hipMemcpyHostToDevice, c->stream));
  c->comm->allreduce(c->dscratch, count, max, c->stream);
  HIPC(hipMemcpyAsync(c->hpinned, c->dscratch, count * sizeof(double), hipMemcpyDeviceToHost,
                      c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  std::memcpy(v, c->hpinned, count * sizeof(double));
}

HH_API int hh_ctx_allreduce_max(hh_ctx* c, double* v, int count) {
  GUARD_BEGIN
  REQUIRE(c, "null ctx");
  host_allreduce(c, v, count, true);
  GUARD_END
}

HH_API int hh_ctx_allreduce_sum(hh_ctx* c, double* v, int count) {
  GUARD_BEGIN
  REQUIRE(c, "null ctx");
  host_allreduce(c, v, count, false);
  GUARD_END
}

HH_API int hh_ctx_barrier(hh_ctx* c) {
  GUARD_BEGIN
  REQUIRE(c, "null ctx");
  HIPC(hipSetDevice(c->device));
  HIPC(hipStreamSynchronize(c->stream));
  double one = 1.0;
  host_allreduce(c, &one, 1, false);
  HIPC(hipDeviceSynchronize());
  GUARD_END
}

HH_API int hh_ctx_progress(hh_ctx* c, long* collectives) {
  GUARD_BEGIN
  REQUIRE(c && collectives, "null argument");
  *collectives = c->comm ? c->comm->entered() : 0;
  GUARD_END
}

HH_API int hh_ctx_synchronize(hh_ctx* c) {
  GUARD_BEGIN
  REQUIRE(c, "null ctx");
  HIPC(hipSetDevice(c->device));
  HIPC(hipDeviceSynchronize());
  GUARD_END
}

// ------------------------------------------------------------------ operator
HH_API int hh_op_create(hh_ctx* c, int n, int b, double cconst, double eta, double omega_re,
                        double omega_im, double h, const double* c_mat, double c_const,
                        double mass_scale_re, double mass_scale_im, hh_op** out) {
  GUARD_BEGIN
  REQUIRE(c && out, "null ctx/op");
  REQUIRE(n >= 1, "n must be >= 1 (got %d)", n);
  REQUIRE(n >= c->world * c->vslabs, "n=%d too small for %d ranks x %d slabs", n, c->world,
          c->vslabs);
  REQUIRE(h > 0 && eta > 0, "h and eta must be positive");
  REQUIRE(c_mat || c_const > 0, "constant medium needs c_const > 0");
  HIPC(hipSetDevice(c->device));
  hh_op* op = new hh_op();
  try {
    op->ctx = c;
    op->n = n;
    op->b = b;
    op->C = cconst;
    op->eta = eta;
    op->h = h;
    op->omega = cd(omega_re, omega_im);
    op->mscale = cd(mass_scale_re, mass_scale_im);
    op->const_c = (c_mat == nullptr);
    op->invc2_const = op->const_c ? 1.0 / (c_const * c_const) : 1.0;
    // rank slab: balanced contiguous split of the n layers
    op->jb = (int)((long)c->rank * n / c->world);
    op->je = (int)((long)(c->rank + 1) * n / c->world);
    op->nloc = (size_t)(op->je - op->jb) * n;
    const cd om = op->omega;
    const cd om2 = om * om * op->mscale;
    const double ih2 = 1.0 / (h * h);
    // per-i table (fast axis): AW, AE, R1
    std::vector<double2> ti(3 * (size_t)n);
    for (int ii = 0; ii < n; ++ii) {
      const double i = ii + 1;
      ti[ii] = d2(s1((i - .5) * h, cconst, eta, om) * ih2);
      ti[n + ii] = d2(s1((i + .5) * h, cconst, eta, om) * ih2);
      ti[2 * n + ii] = d2(1.0 / s1(i * h, cconst, eta, om));
    }
    op->tab_i = dalloc<double2>(3 * (size_t)n);
    HIPC(hipMemcpy(op->tab_i, ti.data(), ti.size() * sizeof(double2), hipMemcpyHostToDevice));
    op->zero_row = dalloc<double2>(2 * (size_t)n);
    HIPC(hipMemsetAsync(op->zero_row, 0, 2 * n * sizeof(double2), c->stream));
    // local slabs
    const int rows = op->je - op->jb;
    size_t off = 0;
    std::vector<double> col;
    for (int s = 0; s < c->vslabs; ++s) {
      Slab sl;
      sl.j0 = op->jb + (int)((long)s * rows / c->vslabs);
      sl.j1 = op->jb + (int)((long)(s + 1) * rows / c->vslabs);
      sl.nl = sl.j1 - sl.j0;
      sl.off = off;
      off += (size_t)sl.nl * n;
      sl.rpb = stencil_rows_per_block(n, sl.nl);
      // per-layer table of local rows -2 .. nl+1 (the fused SL kernel reads two rows beyond
      // the slab); tab_j proper is rows 0 .. nl-1 of it
      std::vector<double2> tj(4 * ((size_t)sl.nl + 4));
      for (int jl = -2; jl < sl.nl + 2; ++jl) {
        const double j = sl.j0 + jl + 1;
        const cd r2 = 1.0 / s2(j * h, cconst, eta, om);
        double2* t = &tj[4 * (size_t)(jl + 2)];
        t[0] = d2(r2);
        t[1] = d2(s2((j - .5) * h, cconst, eta, om) * ih2);
        t[2] = d2(s2((j + .5) * h, cconst, eta, om) * ih2);
        t[3] = d2(om2 * r2);
      }
      sl.tab_j_ext = dalloc<double2>(tj.size());
      HIPC(hipMemcpy(sl.tab_j_ext, tj.data(), tj.size() * sizeof(double2), hipMemcpyHostToDevice));
      sl.tab_j = sl.tab_j_ext + 8;  // row 0
      if (!op->const_c) {
        // invc2[jl][ii] = 1 / c_mat[ii, j-1]^2  (c_mat read as c_mat[i-1, j-1]: quirk Q3),
        // transposed once here so the kernel streams it along i with unit stride.
        std::vector<double> buf((size_t)sl.nl * n);
        const size_t ld = (size_t)n + 2;
        constexpr int TB = 64;
        for (int ib = 0; ib < n; ib += TB)
          for (int jb2 = 0; jb2 < sl.nl; jb2 += TB)
            for (int ii = ib; ii < std::min(n, ib + TB); ++ii) {
              const double* src = c_mat + (size_t)ii * ld + sl.j0;
              for (int jl = jb2; jl < std::min(sl.nl, jb2 + TB); ++jl) {
                const double cv = src[jl];
                buf[(size_t)jl * n + ii] = 1.0 / (cv * cv);
              }
            }
        sl.invc2 = dalloc<double>(buf.size());
        HIPC(hipMemcpy(sl.invc2, buf.data(), buf.size() * sizeof(double), hipMemcpyHostToDevice));
        // 1/c^2 of the two layers on each side of the slab (0 off the grid): the fused SL
        // kernel's first sweep on the neighbours' boundary rows.  A caller that filled only its
        // own columns of c_mat (zero elsewhere) gets the two-launch path instead.
        std::vector<double> hb(4 * (size_t)n, 0.0);
        const int rows4[4] = {sl.j0 - 2, sl.j0 - 1, sl.j1, sl.j1 + 1};
        for (int q = 0; q < 4; ++q) {
          const int j = rows4[q];
          if (j < 0 || j >= n) continue;
          for (int ii = 0; ii < n; ++ii) {
            const double cv = c_mat[(size_t)ii * ld + j];
            if (!(cv > 0.0) || !std::isfinite(cv)) {
              op->sl_ext_ok = false;
              break;
            }
            hb[(size_t)q * n + ii] = 1.0 / (cv * cv);
          }
        }
        sl.invc2_halo = dalloc<double>(hb.size());
        HIPC(hipMemcpy(sl.invc2_halo, hb.data(), hb.size() * sizeof(double), hipMemcpyHostToDevice));
      }
      sl.halo2_lo = dalloc_guarded<double2>(2 * (size_t)n, c->device, false);
      sl.halo2_hi = dalloc_guarded<double2>(2 * (size_t)n, c->device, true);
      HIPC(hipMemsetAsync(sl.halo2_lo, 0, 2 * n * sizeof(double2), c->stream));
      HIPC(hipMemsetAsync(sl.halo2_hi, 0, 2 * n * sizeof(double2), c->stream));
      sl.halo_lo_buf = dalloc_guarded<double2>(n, c->device, false);
      sl.halo_hi_buf = dalloc_guarded<double2>(n, c->device, true);
      HIPC(hipMemsetAsync(sl.halo_lo_buf, 0, n * sizeof(double2), c->stream));
      HIPC(hipMemsetAsync(sl.halo_hi_buf, 0, n * sizeof(double2), c->stream));
      op->slabs.push_back(sl);
    }
    // The fused SL path exchanges two halo rows, the two-launch path one: every rank must take
    // the same path, so the condition (medium known two layers beyond every slab, slabs of at
    // least two layers) is agreed on by all ranks.
    {
      bool ok = op->sl_ext_ok;
      for (const Slab& sl : op->slabs) ok = ok && sl.nl >= 2;
      if (c->world > 1) {
        double bad = ok ? 0.0 : 1.0;
        host_allreduce(c, &bad, 1, true);
        ok = bad == 0.0;
      }
      op->sl_ext_ok = ok;
    }
    // partial-sum workspace: stencil tiles (+ boundary rows) of every slab, or streaming blocks
    size_t tiles = 0;
    for (const Slab& sl : op->slabs) {
      tiles += (size_t)stencil_grid_blocks(n, sl.nl, std::min(sl.rpb, 4)) +
               2 * (size_t)((n + kStencilThreads - 1) / kStencilThreads) + 8;
    }
    size_t cap = std::max(tiles * kMaxNorms, (size_t)kMaxStreamBlocks * (2 * kMaxProj + 2));
    cap = std::max(cap, (size_t)c->vslabs * 2048 * kMaxNorms);
    op->partials = dalloc<double>(cap);
    op->partials_cap = cap;
    op->red = dalloc<double>(kRedDoubles);
    HIPC(hipMemset(op->red, 0, kRedDoubles * sizeof(double)));
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&op->status_h),
                       (1 + kSmallBatch) * kRedDoubles * sizeof(double)));
    HIPC(hipDeviceSynchronize());
  } catch (...) {
    delete op;  // device memory of a failed create is reclaimed at process exit
    throw;
  }
  c->refs++;  // the operator keeps its context alive
  *out = op;
  GUARD_END
}

static void op_release(hh_op* op) {
  if (--op->refs > 0) return;
  hh_ctx* c = op->ctx;
  (void)hipSetDevice(op->ctx->device);
  (void)hipStreamSynchronize(op->ctx->stream);
  for (Slab& s : op->slabs) {
    dfree(s.invc2);
    dfree(s.tab_j_ext);  // (tab_j points into it)
    dfree(s.tab_r2x);
    dfree(s.invc2_halo);
    dfree(s.halo2_lo);
    dfree(s.halo2_hi);
    dfree(s.halo_lo_buf);
    dfree(s.halo_hi_buf);
  }
  dfree(op->tab_i);
  dfree(op->zero_row);
  dfree(op->partials);
  dfree(op->red);
  dfree(op->hx);
  dfree(op->hy);
  dfree(op->scrT);
  dfree(op->scrZ);
  dfree(op->scrR);
  dfree(op->res_bh_lo);
  dfree(op->res_bh_hi);
  dfree(op->V);
  dfree(op->gbuf);
  dfree(op->npart);
  dfree(op->fw);
  dfree(op->cab);
  dfree(op->small_scr);
  dfree(op->small_ticks);
  dfree(op->kcount);
  dfree(op->fold_tickets);
  dfree(op->fold_gpart);
  dfree(op->sw_P);
  dfree(op->sw_Pf);
  dfree(op->sw_Pb);
  dfree(op->sw_Pw);
  dfree(op->sw_Tm);
  dfree(op->sw_gran);
  dfree(op->sw_prof);
  dfree(op->sw_y);
  dfree(op->sw_uF);
  dfree(op->sw_const);
  sweep_dense_release(op);
  if (op->status_h) (void)hipHostFree(op->status_h);
  (void)hipGetLastError();
  delete op;
  ctx_release(c);
}

HH_API int hh_op_destroy(hh_op* op) {
  GUARD_BEGIN
  if (!op) return HH_OK;
  op_release(op);
  GUARD_END
}

HH_API int hh_op_local_rows(hh_op* op, int* j_begin, int* j_end) {
  GUARD_BEGIN
  REQUIRE(op && j_begin && j_end, "null argument");
  *j_begin = op->jb;
  *j_end = op->je;
  GUARD_END
}

HH_API int hh_op_set_precond(hh_op* op, int kind, double beta, int sweeps, double damping) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  REQUIRE(kind == HH_PREC_NONE || kind == HH_PREC_JACOBI || kind == HH_PREC_SHIFTED_LAPLACE ||
              is_sweep(kind),
          "unknown preconditioner kind %d", kind);
  if (kind == HH_PREC_SHIFTED_LAPLACE) {
    REQUIRE(sweeps >= 1 && sweeps <= 64, "sweeps must be in [1, 64]");
    REQUIRE(damping > 0, "damping must be positive");
  }
  if (is_sweep(kind)) {
    REQUIRE(op->points == 5, "the sweeping preconditioner is built for the 5-point operator");
    // sequential in the layer index: no row-slab sharding (SURVEY 8e -> replicas only)
    REQUIRE(op->ctx->world == 1 && op->slabs.size() == 1,
            "the sweeping preconditioner needs the whole grid on one rank and one slab");
    REQUIRE(op->b >= 1 && op->b < op->n, "sweeping needs 1 <= b < n (b = %d, n = %d)", op->b,
            op->n);
    REQUIRE(sweep_block(op->b) > 0, "sweeping supports b <= 16 (b = %d)", op->b);
    if (!op->sw_P) {
      HIPC(hipSetDevice(op->ctx->device));
      const int n = op->n, b = op->b, B = sweep_block(b);
      SweepArgs& a = op->sweep;
      a.n = n;
      a.b = b;
      a.nsys = 1 + (n - b);
      op->sw_P = dalloc<double2>((size_t)a.nsys * n * B * B);
      a.ystride = sweep_scratch_per_wave(n);
      op->sw_y = dalloc<double2>(std::max((size_t)std::max(1, a.nsys - 1) * a.ystride,
                                          sweep_chunk_scratch(n)));
      op->sw_uF = dalloc<double2>((size_t)b * n);
      a.P = op->sw_P;
      a.yscr = op->sw_y;
      a.tab_i = op->tab_i;
      a.tab_k = op->slabs[0].tab_j;      // layers 0..b-1: the local PML of every H_m
      a.tab_glob = op->slabs[0].tab_j;
      a.invc2 = op->const_c ? nullptr : op->slabs[0].invc2;
      a.invc2_const = op->invc2_const;
      a.stop = nullptr;
      a.chunks = 0;
      a.Pf = a.Pb = nullptr;
      // algo2_3 (code.py:345-353): factor H_F and every H_m, all in parallel
      launch_sweep(a, 0, nullptr, nullptr, 0, op->ctx->stream);
      HIPC(hipGetLastError());
      HIPC(hipStreamSynchronize(op->ctx->stream));
    }
    sweep_dense_configure(op);
    sweep_chunk_configure(op);
  }
  op->pkind = kind;
  op->beta = beta;
  op->sweeps = kind == HH_PREC_SHIFTED_LAPLACE ? sweeps : 1;
  op->damping = kind == HH_PREC_SHIFTED_LAPLACE ? damping : 1.0;
  // A_beta mass term: omega^2 (1 + i beta) / (s1 s2 c^2) == build_A_matrix(c / sqrt(1 + i beta))
  op->mshift = make_double2(1.0, beta);
  GUARD_END
}

static void apply_mode(hh_op* op, const double2* x, double2* y, int mode) {
  switch (mode) {
    case HH_APPLY_A: run_stencil(op, EPI_AX, x, nullptr, nullptr, y, nullptr, false); break;
    case HH_APPLY_JACOBI_A: run_stencil(op, EPI_JAC, x, nullptr, nullptr, y, nullptr, false); break;
    case HH_APPLY_PREC:
      REQUIRE(x != y, "in-place preconditioner apply not supported");
      apply_M(op, x, y);
      break;
    case HH_APPLY_PREC_A: apply_MA(op, x, nullptr, y); break;
    default: fail(HH_ERR_INVALID, "unknown apply mode %d", mode);
  }
}

HH_API int hh_op_apply(hh_op* op, const double* x, double* y, int mode) {
  GUARD_BEGIN
  REQUIRE(op && x && y, "null argument");
  HIPC(hipSetDevice(op->ctx->device));
  if (!op->hx) op->hx = dalloc<double2>(op->nloc);
  if (!op->hy) op->hy = dalloc<double2>(op->nloc);
  hipStream_t s = op->ctx->stream;
  HIPC(hipMemcpyAsync(op->hx, x, op->nloc * sizeof(double2), hipMemcpyHostToDevice, s));
  // hy doubles as residual scratch for the SL preconditioner: use a fresh target buffer
  double2* dst = op->hy;
  apply_mode(op, op->hx, dst, mode);
  HIPC(hipMemcpyAsync(y, dst, op->nloc * sizeof(double2), hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  if (mode == HH_APPLY_PREC || mode == HH_APPLY_PREC_A) check_sweep_chain(op);
  GUARD_END
}

HH_API int hh_op_diagonal(hh_op* op, double* d) {
  GUARD_BEGIN
  REQUIRE(op && d, "null argument");
  HIPC(hipSetDevice(op->ctx->device));
  if (!op->hy) op->hy = dalloc<double2>(op->nloc);
  run_point(op, PT_DIAG, nullptr, op->hy, false);
  HIPC(hipMemcpyAsync(d, op->hy, op->nloc * sizeof(double2), hipMemcpyDeviceToHost,
                      op->ctx->stream));
  HIPC(hipStreamSynchronize(op->ctx->stream));
  GUARD_END
}

// ------------------------------------------------------------- CSR export (F2)
HH_API int hh_op_csr_nnz(hh_op* op, int64_t* nnz) {
  GUARD_BEGIN
  REQUIRE(op && nnz, "null argument");
  *nnz = csr_rank_nnz(op->n, op->jb, op->je, op->points);
  GUARD_END
}

HH_API int hh_op_export_csr(hh_op* op, int64_t* indptr, void* indices, int index_bytes,
                            double* data, double* kernel_ms) {
  GUARD_BEGIN
  REQUIRE(op && indptr && indices && data, "null argument");
  REQUIRE(index_bytes == 4 || index_bytes == 8, "index_bytes must be 4 or 8");
  REQUIRE(index_bytes == 8 || (long long)op->n * op->n < (1LL << 31),
          "n^2 >= 2^31: int32 column indices overflow (use index_bytes = 8)");
  HIPC(hipSetDevice(op->ctx->device));
  hipStream_t s = op->ctx->stream;
  const long long nnz = csr_rank_nnz(op->n, op->jb, op->je, op->points);
  const size_t rows = op->nloc;
  long long* d_ptr = dalloc<long long>(rows + 1);
  void* d_idx = nullptr;
  double2* d_val = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  try {
    d_idx = dalloc<char>((size_t)nnz * index_bytes);
    d_val = dalloc<double2>((size_t)nnz);
    HIPC(hipEventCreate(&e0));
    HIPC(hipEventCreate(&e1));
    HIPC(hipEventRecord(e0, s));
    for (size_t si = 0; si < op->slabs.size(); ++si) {
      const Slab& sl = op->slabs[si];
      CsrArgs a{};
      a.tab_i = op->tab_i;
      a.tab_j = sl.tab_j;
      a.invc2 = op->const_c ? nullptr : sl.invc2;
      a.invc2_const = op->invc2_const;
      a.n = op->n;
      a.nl = sl.nl;
      a.j0 = sl.j0;
      a.rank_j0 = op->jb;
      a.row_off = sl.off;
      a.last = si + 1 == op->slabs.size();
      a.indptr = d_ptr;
      a.indices = d_idx;
      a.data = d_val;
      a.tab_r2x = op->points == 9 ? sl.tab_r2x : nullptr;
      a.w9 = op->w9;
      if (sl.nl > 0) launch_csr_export(a, index_bytes, s);
    }
    HIPC(hipGetLastError());
    HIPC(hipEventRecord(e1, s));
    HIPC(hipMemcpyAsync(indptr, d_ptr, (rows + 1) * sizeof(long long), hipMemcpyDeviceToHost, s));
    HIPC(hipMemcpyAsync(indices, d_idx, (size_t)nnz * index_bytes, hipMemcpyDeviceToHost, s));
    HIPC(hipMemcpyAsync(data, d_val, (size_t)nnz * sizeof(double2), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, e0, e1));
    if (kernel_ms) *kernel_ms = ms;
  } catch (...) {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    dfree(d_ptr);
    dfree(d_idx);
    dfree(d_val);
    throw;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  dfree(d_ptr);
  dfree(d_idx);
  dfree(d_val);
  GUARD_END
}

// ------------------------------------------------------------------ vectors
HH_API int hh_vec_create(hh_op* op, hh_vec** v) {
  GUARD_BEGIN
  REQUIRE(op && v, "null argument");
  HIPC(hipSetDevice(op->ctx->device));
  hh_vec* x = new hh_vec();
  x->op = op;
  try {
    x->d = dalloc<double2>(op->nloc);
    HIPC(hipMemsetAsync(x->d, 0, op->nloc * sizeof(double2), op->ctx->stream));
  } catch (...) {
    delete x;
    throw;
  }
  op->refs++;  // the vector keeps its operator alive
  *v = x;
  GUARD_END
}

HH_API int hh_vec_destroy(hh_vec* v) {
  GUARD_BEGIN
  if (!v) return HH_OK;
  hh_op* op = v->op;
  (void)hipSetDevice(op->ctx->device);
  (void)hipStreamSynchronize(op->ctx->stream);
  dfree(v->d);
  delete v;
  op_release(op);
  GUARD_END
}

HH_API int hh_vec_upload(hh_vec* v, const double* host) {
  GUARD_BEGIN
  REQUIRE(v && host, "null argument");
  HIPC(hipSetDevice(v->op->ctx->device));
  HIPC(hipMemcpyAsync(v->d, host, v->op->nloc * sizeof(double2), hipMemcpyHostToDevice,
                      v->op->ctx->stream));
  HIPC(hipStreamSynchronize(v->op->ctx->stream));
  GUARD_END
}

HH_API int hh_vec_download(hh_vec* v, double* host) {
  GUARD_BEGIN
  REQUIRE(v && host, "null argument");
  HIPC(hipSetDevice(v->op->ctx->device));
  HIPC(hipMemcpyAsync(host, v->d, v->op->nloc * sizeof(double2), hipMemcpyDeviceToHost,
                      v->op->ctx->stream));
  HIPC(hipStreamSynchronize(v->op->ctx->stream));
  GUARD_END
}

HH_API int hh_vec_fill_hash(hh_vec* v, uint64_t seed) {
  GUARD_BEGIN
  REQUIRE(v, "null vec");
  hh_op* op = v->op;
  HIPC(hipSetDevice(op->ctx->device));
  launch_fill_hash(v->d, op->nloc, (size_t)op->jb * op->n, seed, op->ctx->stream);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(op->ctx->stream));
  GUARD_END
}

HH_API int hh_op_apply_dev(hh_op* op, const hh_vec* x, hh_vec* y, int mode) {
  GUARD_BEGIN
  REQUIRE(op && x && y && x->op == op && y->op == op, "vectors must belong to this operator");
  REQUIRE(x != y, "in-place apply not supported (the stencil reads neighbours)");
  HIPC(hipSetDevice(op->ctx->device));
  apply_mode(op, x->d, y->d, mode);
  HIPC(hipStreamSynchronize(op->ctx->stream));
  if (mode == HH_APPLY_PREC || mode == HH_APPLY_PREC_A) check_sweep_chain(op);
  GUARD_END
}

HH_API int hh_op_time_apply(hh_op* op, const hh_vec* x, hh_vec* y, int mode, int iters,
                            double* total_ms, double* kernel_ms) {
  return hh_op_time_apply_set(op, &x, &y, 1, mode, iters, total_ms, kernel_ms);
}

HH_API int hh_op_time_apply_set(hh_op* op, const hh_vec* const* xs, hh_vec* const* ys, int nvec,
                                int mode, int iters, double* total_ms, double* kernel_ms) {
  GUARD_BEGIN
  REQUIRE(op && xs && ys && nvec >= 1 && iters >= 1 && total_ms && kernel_ms, "bad arguments");
  for (int k = 0; k < nvec; ++k)
    REQUIRE(xs[k] && ys[k] && xs[k] != ys[k] && xs[k]->op == op && ys[k]->op == op,
            "pair %d: vectors must be distinct and belong to this operator", k);
  HIPC(hipSetDevice(op->ctx->device));
  hipStream_t s = op->ctx->stream;
  // A plain apply on one slab of one rank is exactly one stencil launch: then the events
  // bracketing the back-to-back launches give the kernel's average duration directly, and
  // no per-launch event is inserted between them.  Otherwise (halo exchange, several
  // launches) events are recorded around the interior stencil launch of every apply.
  const bool single = mode == HH_APPLY_A && op->ctx->world == 1 && op->slabs.size() == 1;
  // every event is released on every exit path (a failing call must not leak them)
  struct Events {
    std::vector<hipEvent_t> ev;
    hipEvent_t make() {
      hipEvent_t e = nullptr;
      HIPC(hipEventCreate(&e));
      ev.push_back(e);
      return e;
    }
    ~Events() {
      for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    }
  } events;
  struct TimingHooks {  // the operator's timing hooks never outlive this call
    hh_op* op;
    ~TimingHooks() { op->tk0 = op->tk1 = nullptr; }
  } hooks{op};
  std::vector<hipEvent_t> k0, k1;
  if (!single) {
    k0.resize(iters);
    k1.resize(iters);
    for (int i = 0; i < iters; ++i) {
      k0[i] = events.make();
      k1[i] = events.make();
    }
  }
  hipEvent_t t0 = events.make(), t1 = events.make();
  HIPC(hipStreamSynchronize(s));
  HIPC(hipEventRecord(t0, s));
  for (int i = 0; i < iters; ++i) {
    if (!single) {
      op->tk0 = k0[i];
      op->tk1 = k1[i];
    }
    apply_mode(op, xs[i % nvec]->d, ys[i % nvec]->d, mode);
  }
  op->tk0 = op->tk1 = nullptr;
  HIPC(hipEventRecord(t1, s));
  HIPC(hipEventSynchronize(t1));
  if (mode == HH_APPLY_PREC || mode == HH_APPLY_PREC_A) check_sweep_chain(op);
  float ms = 0.f;
  HIPC(hipEventElapsedTime(&ms, t0, t1));
  *total_ms = ms;
  if (single) {
    *kernel_ms = ms / iters;
  } else {
    double ksum = 0.0;
    for (int i = 0; i < iters; ++i) {
      float km = 0.f;
      HIPC(hipEventElapsedTime(&km, k0[i], k1[i]));
      ksum += km;
    }
    *kernel_ms = ksum / iters;
  }
  GUARD_END
}

HH_API int hh_op_set_cycle_callback(hh_op* op, hh_gmres_cycle_callback cb, void* user) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  op->cycle_cb = cb;
  op->cycle_user = user;
  GUARD_END
}

HH_API int hh_op_set_history_callback(hh_op* op, hh_gmres_history_callback cb, void* user) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  op->hist_cb = cb;
  op->hist_user = user;
  GUARD_END
}

HH_API int hh_op_set_stencil(hh_op* op, int points, double alpha, double c, double d) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  REQUIRE(points == 5 || points == 9, "points must be 5 or 9 (got %d)", points);
  REQUIRE(points == 5 || !is_sweep(op->pkind),
          "the sweeping preconditioner is built for the 5-point operator");
  HIPC(hipSetDevice(op->ctx->device));
  if (points == 9) {
    REQUIRE(std::isfinite(alpha) && std::isfinite(c) && std::isfinite(d), "non-finite weights");
    // R2 = 1/s2(jh) of every local row and the two beyond the slab (1-based j = j0 .. j1 + 1;
    // at the grid edges they multiply the zero Dirichlet rows only)
    for (Slab& sl : op->slabs) {
      if (sl.tab_r2x) continue;
      std::vector<double2> t((size_t)sl.nl + 2);
      for (int k = 0; k < sl.nl + 2; ++k) {
        const double j = sl.j0 + k;  // local row k - 1 -> 1-based j0 + k
        t[k] = d2(1.0 / s2(j * op->h, op->C, op->eta, op->omega));
      }
      sl.tab_r2x = dalloc<double2>(t.size());
      HIPC(hipMemcpy(sl.tab_r2x, t.data(), t.size() * sizeof(double2), hipMemcpyHostToDevice));
    }
    op->w9 = Stencil9W{alpha, (1.0 - alpha) / 2.0, c, d, (1.0 - c - 4.0 * d) / 4.0};
  } else {
    op->w9 = Stencil9W{1.0, 0.0, 1.0, 0.0, 0.0};
  }
  op->points = points;
  GUARD_END
}

HH_API int hh_op_set_krylov_mode(hh_op* op, int mode) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  REQUIRE(mode >= 0 && mode <= 3,
          "krylov mode must be 0 (auto), 1 (two reductions), 2 (one) or 3 (one, one pass)");
  op->krylov_mode = mode;
  GUARD_END
}

HH_API int hh_op_set_small_cycle(hh_op* op, int mode) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  REQUIRE(mode >= -1 && mode <= 1, "small-cycle mode must be -1 (auto), 0 (off) or 1 (on)");
  op->small_cycle = mode;
  GUARD_END
}

HH_API int hh_op_small_cycle_profile(hh_op* op, int enable, double* phase_us) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  HIPC(hipSetDevice(op->ctx->device));
  if (phase_us && op->small_ticks) {
    unsigned long long t[8];
    HIPC(hipMemcpy(t, op->small_ticks, sizeof(t), hipMemcpyDeviceToHost));
    int mhz = 100;  // s_memrealtime: a constant 100 MHz clock on gfx9
    (void)hipDeviceGetAttribute(&mhz, hipDeviceAttributeWallClockRate, op->ctx->device);
    const double khz = mhz > 0 ? (double)mhz : 100000.0;  // (the attribute is in kHz)
    for (int q = 0; q < 7; ++q) phase_us[q] = t[q] * 1e3 / khz;
    phase_us[7] = (double)t[7];  // shader-clock cycles over the same span (s_memtime)
  }
  if (enable && !op->small_ticks) op->small_ticks = dalloc<unsigned long long>(kSmallTicks);
  if (op->small_ticks)
    HIPC(hipMemset(op->small_ticks, 0, kSmallTicks * sizeof(unsigned long long)));
  if (!enable) {
    dfree(op->small_ticks);
    op->small_ticks = nullptr;
  }
  GUARD_END
}

HH_API int hh_op_small_cycle_tail_profile(hh_op* op, double* tail_us) {
  GUARD_BEGIN
  REQUIRE(op && tail_us, "null argument");
  REQUIRE(op->small_ticks, "small-cycle profiling is not enabled (hh_op_small_cycle_profile)");
  HIPC(hipSetDevice(op->ctx->device));
  unsigned long long t[kSmallTicks];
  HIPC(hipMemcpy(t, op->small_ticks, sizeof(t), hipMemcpyDeviceToHost));
  int khz = 100000;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, op->ctx->device);
  for (int q = 0; q < 8; ++q) tail_us[q] = t[8 + q] * 1e3 / (khz > 0 ? khz : 100000);
  GUARD_END
}

HH_API int hh_op_sl_fusion(hh_op* op, int enable) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  op->sl_fuse = enable != 0;
  GUARD_END
}

HH_API int hh_op_tune(hh_op* op, int variant, int rows_per_block, int grid_blocks) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  REQUIRE(grid_blocks >= 0, "grid_blocks must be >= 0");
  op->grid_override = grid_blocks;
  REQUIRE(variant == -1 || stencil_variant_valid(variant), "variant %d not instantiated", variant);
  REQUIRE(rows_per_block == 0 || (rows_per_block >= 4 && rows_per_block <= 4096),
          "rows_per_block must be 0 or in [4, 4096]");
  op->variant = variant;
  op->rpb_override = rows_per_block;
  GUARD_END
}
HH_API int hh_tune_krylov(int nt_loads, int blocks) {
  GUARD_BEGIN
  REQUIRE(blocks >= 0 && blocks <= (1 << 20), "blocks out of range");
  tune_krylov(nt_loads, blocks);
  GUARD_END
}

HH_API int hh_op_probe_stream(hh_op* op, int kind, int blocks, const hh_vec* x, hh_vec* y,
                              int iters, double* kernel_ms, int* bytes_per_point) {
  return hh_op_probe_stream_set(op, kind, blocks, &x, &y, 1, iters, kernel_ms, bytes_per_point);
}

HH_API int hh_op_probe_stream_set(hh_op* op, int kind, int blocks, const hh_vec* const* xs,
                                  hh_vec* const* ys, int nvec, int iters, double* kernel_ms,
                                  int* bytes_per_point) {
  GUARD_BEGIN
  REQUIRE(op && xs && ys && nvec >= 1 && iters >= 1 && kernel_ms && bytes_per_point,
          "bad arguments");
  for (int k = 0; k < nvec; ++k)
    REQUIRE(xs[k] && ys[k] && xs[k] != ys[k] && xs[k]->op == op && ys[k]->op == op,
            "pair %d: vectors must be distinct and belong to this operator", k);
  REQUIRE(!op->const_c && op->slabs.size() == 1, "probe needs a heterogeneous single-slab operator");
  REQUIRE(blocks >= 1 && blocks <= (1 << 20), "blocks out of range");
  HIPC(hipSetDevice(op->ctx->device));
  hipStream_t s = op->ctx->stream;
  hipEvent_t t0, t1;
  HIPC(hipEventCreate(&t0));
  HIPC(hipEventCreate(&t1));
  int bpp = 0;
  for (int k = 0; k < nvec; ++k)  // warm-up, one launch per pair
    bpp = launch_probe_kind(kind, blocks, xs[k]->d, op->slabs[0].invc2, ys[k]->d, op->nloc, s);
  REQUIRE(bpp > 0, "unknown probe kind %d", kind);
  HIPC(hipEventRecord(t0, s));
  for (int i = 0; i < iters; ++i)
    launch_probe_kind(kind, blocks, xs[i % nvec]->d, op->slabs[0].invc2, ys[i % nvec]->d,
                      op->nloc, s);
  HIPC(hipEventRecord(t1, s));
  HIPC(hipEventSynchronize(t1));
  float ms = 0.f;
  HIPC(hipEventElapsedTime(&ms, t0, t1));
  *kernel_ms = ms / iters;
  *bytes_per_point = bpp;
  (void)hipEventDestroy(t0);
  (void)hipEventDestroy(t1);
  GUARD_END
}

HH_API int hh_op_set_timing(hh_op* op, int enable) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  HIPC(hipSetDevice(op->ctx->device));
  HIPC(hipStreamSynchronize(op->ctx->stream));
  op->timer.reset();
  op->timer.on = enable != 0;
  GUARD_END
}

HH_API int hh_op_read_timing(hh_op* op, double* ms, long* counts) {
  GUARD_BEGIN
  REQUIRE(op && ms && counts, "null argument");
  HIPC(hipSetDevice(op->ctx->device));
  HIPC(hipDeviceSynchronize());  // (the halo stream's events too)
  for (int k = 0; k < HH_SPAN_COUNT; ++k) {
    ms[k] = 0.0;
    counts[k] = 0;
  }
  for (const auto& sp : op->timer.spans) {
    float t = 0.f;
    HIPC(hipEventElapsedTime(&t, sp.a, sp.b));
    if (sp.clamp && t < 0.f) t = 0.f;
    ms[sp.cat] += t;
    counts[sp.cat] += 1;
  }
  op->timer.reset();  // (timing stays enabled; the next read covers what follows)
  GUARD_END
}

HH_API int hh_op_last_solve_path(hh_op* op, int* path) {
  GUARD_BEGIN
  REQUIRE(op && path, "null argument");
  *path = op->last_path;
  GUARD_END
}

HH_API int hh_op_last_stats(hh_op* op, hh_stats* st) {
  GUARD_BEGIN
  REQUIRE(op && st, "null argument");
  *st = op->stats;
  GUARD_END
}
