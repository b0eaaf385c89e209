// The sweeping moving-PML preconditioner (code.py:290-385 algo2_3 / algo2_4):
// its apply on the device, the choice and formation of its dense / partitioned forms, and its
// tuning ABI (see hh_runtime.hpp for the runtime's layout).
#include "hh_runtime.hpp"

namespace hh {

void sweep_dense_release(hh_op* op) {
  for (auto& g : op->sw_graphs) (void)hipGraphExecDestroy(g.exec);
  op->sw_graphs.clear();
  dfree(op->sw_T);
  dfree(op->sw_chain);
  op->sw_chain = nullptr;
  dfree(op->sw_u);
  dfree(op->sw_in);
  dfree(op->sw_out);
  op->sw_T = op->sw_u = op->sw_in = op->sw_out = nullptr;
}

// algo2_4 (code.py:356-385) on r -> out: forward, middle (as-is: u -= T u, quirk Q2;
// corrected: u = T u), backward sweeps.  r and out must differ.
void sweep_apply(hh_op* op, const double2* r, double2* out, bool asis) {
  hipStream_t s = op->ctx->stream;
  if (op->sw_T && op->sw_chain) {
    // F0 (one batched launch) + the persistent chain (one cooperative launch): no graph needed
    SweepArgs a = op->sweep;
    a.stop = op->stop_flag;
    ChainArgs c{};
    c.gbuf = op->sw_chain;
    c.timeout = reinterpret_cast<unsigned*>(op->red + kRedTimeout);
    c.diag = (int)knobs().sweep_diag;
    c.seq = (++op->sw_seq) & 0xfffffu;
    if (c.seq == 0) c.seq = op->sw_seq = 1;  // (tag 0 is the zeroed buffer)
    launch_sweep_dense_apply(a, op->sw_T, r, out, op->sw_u, asis ? 1 : 0, s, &c);
    HIPC(hipGetLastError());
    return;
  }
  if (op->sw_T) {
    // The chain is 2 (n - b) + 1 dependent GEMV launches: replayed from a graph captured once
    // per (mode, stop flag) on fixed buffers, so the host does not pay a launch per GEMV.
    const int am = asis ? 1 : 0;
    // HH_SWEEP_GRAPH=0: eager launches of the same kernels (profilers that cannot follow
    // graph replays)
    if (knobs().sweep_graph == 0) {
      SweepArgs a = op->sweep;
      a.stop = op->stop_flag;
      launch_sweep_dense_apply(a, op->sw_T, r, out, op->sw_u, am, s);
      HIPC(hipGetLastError());
      return;
    }
    hipGraphExec_t exec = nullptr;
    for (auto& g : op->sw_graphs)
      if (g.asis == am && g.stop == op->stop_flag) exec = g.exec;
    if (!exec) {
      SweepArgs a = op->sweep;
      a.stop = op->stop_flag;
      hipGraph_t graph = nullptr;
      HIPC(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      launch_sweep_dense_apply(a, op->sw_T, op->sw_in, op->sw_out, op->sw_u, am, s);
      const hipError_t le = hipGetLastError();
      HIPC(hipStreamEndCapture(s, &graph));
      if (le != hipSuccess) {
        (void)hipGraphDestroy(graph);
        HIPC(le);
      }
      const hipError_t ie = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
      (void)hipGraphDestroy(graph);
      HIPC(ie);
      if (op->sw_graphs.size() >= 4) {  // stale stop flags (a reallocated GMRES workspace)
        (void)hipGraphExecDestroy(op->sw_graphs.front().exec);
        op->sw_graphs.erase(op->sw_graphs.begin());
      }
      op->sw_graphs.push_back({am, op->stop_flag, exec});
    }
    const size_t bytes = (size_t)op->n * op->n * sizeof(double2);
    HIPC(hipMemcpyAsync(op->sw_in, r, bytes, hipMemcpyDeviceToDevice, s));
    HIPC(hipGraphLaunch(exec, s));
    HIPC(hipMemcpyAsync(out, op->sw_out, bytes, hipMemcpyDeviceToDevice, s));
    return;
  }
  launch_scale_copy(r, out, op->nloc, 1.0, s, op->stop_flag);
  SweepArgs a = op->sweep;
  a.stop = op->stop_flag;
  // the partitioned sweeps tag their grid exchange with a per-launch sequence number
  auto next_seq = [&] {
    a.seq = (++op->sw_seq) & 0x1ffffu;
    if (a.seq == 0) a.seq = op->sw_seq = 1;  // (tag 0 is the zeroed buffer)
  };
  next_seq();
  launch_sweep(a, 1, out, op->sw_uF, 0, s);
  launch_sweep(a, 2, out, op->sw_uF, asis ? 1 : 0, s);
  next_seq();
  launch_sweep(a, 3, out, op->sw_uF, 0, s);
  HIPC(hipGetLastError());
}

// The persistent sweep chain (sweep_dense.hip) bounds its grid-wide waits and reports a
// timeout in red[kRedTimeout] instead of hanging; its output is then garbage.  Every path that
// ran a chained sweep apply checks the word here (one synchronising read; nothing for the other
// preconditioners) and clears it only after the check, so no timeout is lost or reported twice.
void check_sweep_chain(hh_op* op) {
  const bool grid = op->sw_chain || (!op->sw_T && op->sweep.chunks > 0 && op->sweep.G > 1);
  if (!grid || !is_sweep(op->pkind)) return;
  double w = 0.0;
  read_dev(op, op->red + kRedTimeout, &w, 1);
  unsigned tmo = 0;
  std::memcpy(&tmo, &w, sizeof(unsigned));
  if (tmo != 0) {
    HIPC(hipMemset(op->red + kRedTimeout, 0, sizeof(double)));
    fail(HH_ERR_STATE, "sweeping preconditioner: a grid-wide wait of the persistent apply "
                       "chain or of the partitioned solves timed out (workgroups not "
                       "co-resident?); HH_SWEEP_CHAIN=0 / hh_op_sweep_workgroups(op, 1) select "
                       "forms without grid waits");
  }
}

// The persistent apply chain of the dense form (sweep_dense.hip sweep_chain_kernel) where it
// fits, unless mode 2 (one launch per GEMV, replayed from a graph) or HH_SWEEP_CHAIN=0.
void sweep_chain_configure(hh_op* op) {
  const bool chain_env = knobs().sweep_chain != 0;
  int cus = 0;
  HIPC(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, op->ctx->device));
  const bool want = op->sw_T && op->sw_mode != 2 && chain_env && sweep_chain_fits(op->n, cus);
  if (!want) {
    dfree(op->sw_chain);
    op->sw_chain = nullptr;
  } else if (!op->sw_chain) {
    op->sw_chain = dalloc<unsigned long long>(sweep_chain_granules());
    HIPC(hipMemset(op->sw_chain, 0, sweep_chain_granules() * sizeof(unsigned long long)));
  }
}

// Dense-transfer form of the sweeping preconditioner (sweep_dense.hip): decide, allocate, form.
void sweep_dense_configure(hh_op* op) {
  const int n = op->n, b = op->b;
  if (op->sw_mode == 0 || op->sw_mode == 3) {
    sweep_dense_release(op);
    return;
  }
  if (op->sw_T) {
    sweep_chain_configure(op);
    return;
  }
  size_t free_b = 0, total_b = 0;
  HIPC(hipMemGetInfo(&free_b, &total_b));
  const size_t tbytes = sweep_dense_bytes(n);
  const size_t blk = sweep_dense_scratch_per_block(n, b) * sizeof(double2);
  const int chunks = sweep_dense_chunks(n);
  const bool fits = tbytes + (size_t)chunks * blk + (size_t)n * n * 16 < free_b / 10 * 7;
  if (op->sw_mode < 0 && (n > 2048 || !fits)) return;  // auto: keep the block-Thomas solves
  REQUIRE(fits, "dense sweeping needs %.1f GB for n = %d (%.1f GB free)", tbytes / 1e9, n,
          free_b / 1e9);
  REQUIRE(n <= 2048, "dense sweeping supports n <= 2048 (n = %d)", n);
  hipStream_t s = op->ctx->stream;
  op->sw_T = dalloc<double2>(tbytes / sizeof(double2));
  double2* scr = nullptr;
  try {
    op->sw_u = dalloc<double2>((size_t)n * n);
    HIPC(hipMemsetAsync(op->sw_u, 0, (size_t)n * n * sizeof(double2), op->ctx->stream));
    // concurrency: ~1024 setup blocks, within a scratch budget of the remaining memory
    const size_t left = free_b - tbytes - (size_t)n * n * 16;
    const size_t budget = std::min(left / 4, (size_t)32 << 30);
    const int nsys = op->sweep.nsys;
    int batch = std::max(1, std::min(nsys, 1024 / chunks));
    while (batch > 1 && (size_t)batch * chunks * blk > budget) batch /= 2;
    scr = dalloc<double2>((size_t)batch * chunks * blk / sizeof(double2));
    for (int s0 = 0; s0 < nsys; s0 += batch)
      launch_sweep_dense_setup(op->sweep, s0, std::min(batch, nsys - s0), scr, op->sw_T, s);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(s));
    op->sw_in = dalloc<double2>((size_t)n * n);
    op->sw_out = dalloc<double2>((size_t)n * n);
  } catch (...) {
    dfree(scr);
    sweep_dense_release(op);
    throw;
  }
  dfree(scr);
  sweep_chain_configure(op);
}

// Partitioned block-Thomas solves (sweep.hip bt_solve_chunked) for the forward / backward
// sweeps when the block-Thomas form is in use: G workgroups of kSweepChunks chunks each share
// every solve (G by n: 2 columns per chunk, at most sweep_part_max_wgs(B) and the CU count;
// hh_op_sweep_workgroups overrides it).  The chunk products Psi_f / Psi_b (2 x the factors'
// memory) and the workgroup maps are formed once here.  Mode 3, the dense form, n < 2 columns
// per chunk or a lack of memory keep the sequential solves.
void sweep_part_release(hh_op* op) {
  dfree(op->sw_Pf);
  dfree(op->sw_Pb);
  dfree(op->sw_Pw);
  dfree(op->sw_Tm);
  dfree(op->sw_gran);
  op->sw_Pf = op->sw_Pb = op->sw_Pw = op->sw_Tm = nullptr;
  op->sw_gran = nullptr;
  SweepArgs& a = op->sweep;
  a.chunks = 0;
  a.G = 0;
  a.Pf = a.Pb = a.Pw = a.Tm = nullptr;
  a.gran = nullptr;
}

int sweep_part_wgs(hh_op* op) {
  const int n = op->n, B = sweep_block(op->b);
  int cus = 0;
  HIPC(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, op->ctx->device));
  // by n: 2 columns per chunk (the chunk-local passes are per-CU latency / bandwidth bound, the
  // grid step is one B x B step per half-wave whatever G: profiles/r04/r04sw3_*)
  int G = op->sw_wgs > 0 ? op->sw_wgs : n / (2 * kSweepChunks);
  G = std::max(1, std::min({G, sweep_part_max_wgs(B), cus, n / (2 * kSweepChunks)}));
  if (op->sw_wgs == 0)  // by n: the largest G <= that whose B-vectors fit in LDS, if any
    for (int g2 = G; g2 >= 1; --g2)
      if (sweep_part_ys_lds(B, g2, n)) return g2;
  return G;
}

void sweep_chunk_configure(hh_op* op) {
  SweepArgs& a = op->sweep;
  const int n = op->n, B = sweep_block(op->b);
  const bool want = !op->sw_T && (op->sw_mode == -1 || op->sw_mode == 0) &&
                    n >= 2 * kSweepChunks;
  if (!want) {
    sweep_part_release(op);
    return;
  }
  const int G = sweep_part_wgs(op);
  if (op->sw_Pf && a.G == G) return;
  sweep_part_release(op);
  const size_t elems = (size_t)a.nsys * n * B * B;
  const size_t welems = (size_t)a.nsys * G * 2 * kSweepChunks * B * B;
  const size_t telems = (size_t)a.nsys * 2 * sweep_grid_tri(G) * B * B;
  size_t free_b = 0, total_b = 0;
  HIPC(hipMemGetInfo(&free_b, &total_b));
  if ((2 * elems + welems + telems) * sizeof(double2) > free_b / 10 * 8) return;  // sequential
  try {
    op->sw_Pf = dalloc<double2>(elems);
    op->sw_Pb = dalloc<double2>(elems);
    op->sw_Pw = dalloc<double2>(welems);
    op->sw_Tm = dalloc<double2>(std::max<size_t>(telems, 1));
    op->sw_gran = dalloc<unsigned long long>(sweep_part_granules(G));
  } catch (...) {
    sweep_part_release(op);
    throw;
  }
  HIPC(hipMemset(op->sw_gran, 0, sweep_part_granules(G) * sizeof(unsigned long long)));
  a.chunks = kSweepChunks * G;
  a.G = G;
  a.Pf = op->sw_Pf;
  a.Pb = op->sw_Pb;
  a.Pw = op->sw_Pw;
  a.Tm = op->sw_Tm;
  a.gran = op->sw_gran;
  a.timeout = reinterpret_cast<unsigned*>(op->red + kRedTimeout);
  launch_sweep(a, 4, nullptr, nullptr, 0, op->ctx->stream);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(op->ctx->stream));
}

}  // namespace hh

HH_API int hh_op_sweep_mode(hh_op* op, int mode, int* active) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  REQUIRE(mode >= -1 && mode <= 3, "mode must be -1, 0, 1, 2 or 3");
  HIPC(hipSetDevice(op->ctx->device));
  op->sw_mode = mode;
  if (op->sw_P) {  // already factored: switch now
    if (mode == 1 || mode == 2) sweep_chunk_configure(op);  // release before the dense setup
    sweep_dense_configure(op);
    sweep_chunk_configure(op);
  }
  if (active) *active = op->sw_T ? 1 : (op->sweep.chunks > 0 ? 2 : 0);
  GUARD_END
}

HH_API int hh_op_sweep_profile(hh_op* op, int enable, double* phase_us, int cap) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  HIPC(hipSetDevice(op->ctx->device));
  const size_t slots = (size_t)kSweepMaxWgs * kSweepProfSlots;  // (one row per workgroup)
  if (phase_us && op->sw_prof) {
    std::vector<unsigned long long> t(slots);
    HIPC(hipMemcpy(t.data(), op->sw_prof, slots * sizeof(unsigned long long),
                   hipMemcpyDeviceToHost));
    int khz = 100000;  // s_memrealtime: a constant 100 MHz clock on gfx9 (attribute in kHz)
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, op->ctx->device);
    for (int q = 0; q < cap && q < (int)slots; ++q) phase_us[q] = t[q] * 1e3 / (khz > 0 ? khz : 100000);
  }
  if (enable && !op->sw_prof) op->sw_prof = dalloc<unsigned long long>(slots);
  if (op->sw_prof) HIPC(hipMemset(op->sw_prof, 0, slots * sizeof(unsigned long long)));
  if (!enable) {
    dfree(op->sw_prof);
    op->sw_prof = nullptr;
  }
  op->sweep.prof = op->sw_prof;
  GUARD_END
}

HH_API int hh_op_sweep_workgroups(hh_op* op, int workgroups, int* active) {
  GUARD_BEGIN
  REQUIRE(op, "null op");
  REQUIRE(workgroups >= 0 && workgroups <= 1024, "workgroups must be in [0, 1024]");
  HIPC(hipSetDevice(op->ctx->device));
  op->sw_wgs = workgroups;
  if (op->sw_P) sweep_chunk_configure(op);
  if (active) *active = (!op->sw_T && op->sweep.chunks > 0) ? op->sweep.G : 0;
  GUARD_END
}

