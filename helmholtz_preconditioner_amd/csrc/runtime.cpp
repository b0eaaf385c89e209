// Host runtime behind the C ABI (include/helmholtz_amd.h): device context + RCCL rank,
// the row-slab operator (PML tables, pre-transposed 1/c^2), halo exchange, apply modes,
// preconditioners and the restarted GMRES driver with scipy's control flow.
//
// Reference boundary (code.py, bocchs/helmholtz-preconditioner):
//   build_A_matrix(b, const, eta, omega, h, n, c_mat)  code.py:202   -> hh_op_create
//   A @ x (LinearOperator.matvec -> csr_matvec)          code.py:516   -> hh_op_apply(_dev)
//   scipy.sparse.linalg.gmres(A, f, M=M, tol=1e-3, ...)  code.py:516   -> hh_gmres
//   M slot LinearOperator(matvec=...)                    code.py:510   -> hh_op_set_precond
#include <algorithm>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <string>
#include <vector>

#include "../../include/helmholtz_amd.h"
#include "comm.hpp"
#include "hh_error.hpp"
#include "hh_internal.hpp"
#include "sweep.hpp"

using cd = std::complex<double>;

namespace hh {

thread_local std::string g_err = "";

template <class T>
static T* dalloc(size_t count) {
  if (count == 0) count = 1;
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, count * sizeof(T));
  if (e != hipSuccess)
    fail(HH_ERR_ALLOC, "hipMalloc(%zu bytes) failed: %s", count * sizeof(T), hipGetErrorString(e));
  return static_cast<T*>(p);
}

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

template <class T>
static T* dalloc_guarded(size_t count, int device, bool at_end) {
  if (knobs().guard_halo == 0) return dalloc<T>(count);
  const size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
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
  return reinterpret_cast<T*>(p);
}

static void dfree(void* p) {
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

using namespace hh;

struct hh_ctx {
  int refs = 1;  // the caller's handle + one per live operator (freed at zero)
  int device = 0, rank = 0, world = 1, vslabs = 1, transport = 0;
  std::unique_ptr<hh::Comm> comm;  // null at world == 1
  hipStream_t stream = nullptr;   // compute
  hipStream_t cstream = nullptr;  // halo exchange + boundary rows (highest priority)
  hipEvent_t ev_in = nullptr, ev_halo = nullptr;
  double* dscratch = nullptr;     // device scratch for host collectives
  double* hpinned = nullptr;      // pinned host staging
};

namespace {
// layout of the per-operator reduction buffer `red` (device) and its host mirror status_h:
// [0, 256) reductions (norms at 0..15, dots from 16), [256, 384) the cycle's per-iteration
// statuses (4 x restart), [384, 388) the cycle's control words (ints), [388] the small cycle's
// timeout word; the end of a cycle copies [0, kRedReport) once
constexpr int kRedTimeout = 388;
constexpr int kRedReport = 389;
constexpr int kRedOuter = 400;  // [400, 408): the small cycle's restart-loop state (device only)
// restart cycles per whole-cycle launch (gmres_small.hip: one cooperative launch runs a batch,
// one host sync per batch); cycle i reports into its own slot of the host mirror,
// status_h + (1 + i) kRedDoubles
constexpr int kSmallBatch = 16;
static_assert(kRedOuter >= kRedReport && kRedOuter + kOuterDoubles <= kRedDoubles, "red layout");
}  // namespace

namespace {
struct Slab {
  int j0 = 0, j1 = 0, nl = 0;  // global 0-based layers [j0, j1)
  size_t off = 0;              // element offset inside the rank-local vector
  double* invc2 = nullptr;     // [nl][n]
  double2* tab_j = nullptr;    // [nl][4]
  double2* tab_r2x = nullptr;  // 9-point only: R2 = 1/s2 of local rows -1 .. nl ([nl + 2])
  double2* halo_lo_buf = nullptr;
  double2* halo_hi_buf = nullptr;
  // for the fused shifted-Laplace M A (sl_fused.hip) across slabs / ranks, which reads v two
  // rows beyond the slab and evaluates the first sweep on the neighbours' boundary rows:
  double2* tab_j_ext = nullptr;  // [nl + 4][4]: the tab_j rows of local rows -2 .. nl+1
  double* invc2_halo = nullptr;  // [4][n]: 1/c^2 of local rows -2, -1, nl, nl+1 (0 off-grid)
  double2* halo2_lo = nullptr;   // [2][n]: cross-rank v rows -2, -1
  double2* halo2_hi = nullptr;   // [2][n]: cross-rank v rows nl, nl+1
  int rpb = 16;
};
}  // namespace

namespace {
// Diagnostic span timing (hh_op_set_timing / hh_op_read_timing): HIP events recorded around the
// pieces of an apply / GMRES iteration on the streams they run on, summed per category when
// read.  Off by default (no event is recorded then); the N > 1 bench turns it on for one extra,
// untimed solve to say where a rank's time goes.
struct SpanTimer {
  bool on = false;
  std::vector<hipEvent_t> pool;  // created lazily, reused after each read
  size_t used = 0;
  struct Span {
    int cat;
    hipEvent_t a, b;
    bool clamp;  // a wait: max(0, b - a) (b may complete before a)
  };
  std::vector<Span> spans;
  hipEvent_t mark(hipStream_t s) {
    if (used == pool.size()) {
      hipEvent_t e = nullptr;
      HIPC(hipEventCreate(&e));
      pool.push_back(e);
    }
    hipEvent_t e = pool[used++];
    HIPC(hipEventRecord(e, s));
    return e;
  }
  void span(int cat, hipEvent_t a, hipEvent_t b, bool clamp = false) {
    if (a && b) spans.push_back({cat, a, b, clamp});
  }
  void reset() {
    spans.clear();
    used = 0;
  }
  ~SpanTimer() {
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
  }
};
}  // namespace

struct hh_op {
  int refs = 1;  // the caller's handle + one per live vector (freed at zero)
  hh_ctx* ctx = nullptr;
  int n = 0, b = 0;
  double C = 0, eta = 0, h = 0;
  cd omega, mscale;
  bool const_c = false;
  double invc2_const = 1.0;
  int jb = 0, je = 0;
  size_t nloc = 0;
  std::vector<Slab> slabs;
  double2* tab_i = nullptr;
  double2* zero_row = nullptr;   // two zero rows (the fused SL kernel reads two halo rows)
  bool sl_ext_ok = true;          // every rank holds the medium two layers beyond its slab
  // preconditioner
  int pkind = HH_PREC_NONE;
  double beta = 0.5, damping = 1.0;
  int sweeps = 1;
  double2 mshift = make_double2(1.0, 0.0);
  bool sl_fuse = true;  // two-sweep M A in one launch (sl_fused.hip) where it applies
  // stencil: 5 (the reference's operator) or 9 (hh_op_set_stencil)
  int points = 5;
  Stencil9W w9{1.0, 0.0, 1.0, 0.0, 0.0};
  // reductions
  double* partials = nullptr;
  size_t partials_cap = 0;  // doubles
  double* red = nullptr;    // 256 doubles
  // scratch
  double2* hx = nullptr;
  double2* hy = nullptr;
  double2* scrT = nullptr;
  double2* scrZ = nullptr;
  double2* scrR = nullptr;
  double2* res_bh_lo = nullptr;  // b's two rows beyond the rank's slab, per side (run_sl2_res)
  double2* res_bh_hi = nullptr;
  // GMRES workspace
  double2* V = nullptr;
  int V_cols = 0;
  size_t ldv = 0;  // distance between consecutive basis vectors (nloc + basis_pad())
  double2* gbuf = nullptr;
  GivensState gs{};
  double* status_h = nullptr;
  // in-solve reductions per inner iteration (hh_op_set_krylov_mode): 0 auto (two allreduces on
  // one rank -- where they are free --, one across ranks), 1 two, 2 one (lagged normalisation)
  int krylov_mode = 0;
  double* npart = nullptr;  // update-kernel norm partials, kept one iteration (one-allreduce mode)
  // whole-cycle kernel for small grids (gmres_small.hip): hand-off scratch and barrier words
  int small_cycle = -1;     // -1 auto, 0 off, 1 on where eligible (hh_op_set_small_cycle)
  double* small_scr = nullptr;
  unsigned small_seq = 0;          // launch sequence number (the tags of its hand-off granules)
  unsigned long long* small_ticks = nullptr;  // phase timing of the small cycle (diagnostic)
  // fused single-rank Krylov kernels (last-block reductions): their ticket counters
  unsigned* kcount = nullptr;
  // HH_KRYLOV_FUSE bit 0: multidot + reduce, bit 1: update + Givens column as last-block fused
  // kernels.  Off by default: measured no faster at 1024^2 (update+column 8 975-9 077 vs 8 878-
  // 9 105 it/s unfused; multidot+reduce 8 219 -- its last block's reduction is a serial chain
  // of device-scope loads; profiles/r02c2e_fuse_ab.log)
  int fuse_krylov = (int)knobs().krylov_fuse;
  // timing hooks
  hipEvent_t tk0 = nullptr, tk1 = nullptr;
  // device stop flag of the GMRES cycle being queued (nullptr outside hh_gmres)
  const int* stop_flag = nullptr;
  // sweeping preconditioner (HH_PREC_SWEEP / HH_PREC_SWEEP_REF)
  SweepArgs sweep{};
  double2* sw_P = nullptr;
  double2* sw_y = nullptr;
  double2* sw_uF = nullptr;
  double2* sw_const = nullptr;  // as-is (quirk Q1): M x = algo2_4(b) for every x
  double2* sw_T = nullptr;      // dense transfer matrices (sweep_dense.hip), or null
  double2* sw_Pf = nullptr;     // chunk products of the partitioned solves, or null
  double2* sw_Pb = nullptr;
  double2* sw_Pw = nullptr;     // workgroup maps of the multi-workgroup partitioned solves
  double2* sw_Tm = nullptr;     // their grid maps
  unsigned long long* sw_gran = nullptr;  // their grid-exchange granules
  int sw_wgs = 0;               // requested workgroups per partitioned solve (0: by n)
  unsigned long long* sw_prof = nullptr;  // diagnostic phase ticks (hh_op_sweep_profile)
  unsigned long long* sw_chain = nullptr;  // granules of the persistent apply chain, or null
  double2* fw = nullptr;        // one-pass GMRES iteration: the w_j ping-pong pair [2][nloc]
  double2* cab = nullptr;       // its cycle end: y = a + y_col b coefficients [2][kMaxProj]
  unsigned sw_seq = 0;                     // its launch sequence number
  double2* sw_u = nullptr;      // dense apply scratch (n^2)
  double2* sw_in = nullptr;     // dense apply: fixed input / output the captured graphs use
  double2* sw_out = nullptr;
  struct SweepGraph {
    int asis;
    const int* stop;
    hipGraphExec_t exec;
  };
  std::vector<SweepGraph> sw_graphs;  // the 2 (n - b) + 1 GEMV launches, captured once
  int sw_mode = -1;  // -1 auto, 0 block-Thomas solves (partitioned where the chunk products
                     // fit), 1 dense transfer matrices, 2 dense with one launch per GEMV (no
                     // persistent chain), 3 block-Thomas sequential solves
  // tuning (hh_op_tune): stencil variant for the plain apply, rows per block override
  int variant = -1;
  int rpb_override = 0;
  // hh_op_set_cycle_callback: scipy's callback_type='x' hook, once per restart cycle
  hh_gmres_cycle_callback cycle_cb = nullptr;
  void* cycle_user = nullptr;
  // hh_op_set_history_callback: the per-iteration statuses of a cycle in one call
  hh_gmres_history_callback hist_cb = nullptr;
  void* hist_user = nullptr;
  int grid_override = 0;
  hh_stats stats{};
  SpanTimer timer;
  int last_path = 0;  // the last hh_gmres: 0 regular cycle, 1 small-grid cycle kernel, 2 small
                      // cycle refused at launch -> regular cycle, 3 one-pass regular cycle
                      // (hh_op_last_solve_path)
};

struct hh_vec {
  hh_op* op = nullptr;
  double2* d = nullptr;
};

namespace {

void ensure_scratch(hh_op* op) {
  if (!op->scrT) op->scrT = dalloc<double2>(op->nloc);
  if (!op->scrZ) op->scrZ = dalloc<double2>(op->nloc);
}

// timing marks (no-ops unless hh_op_set_timing enabled them)
hipEvent_t tmark(hh_op* op, hipStream_t s) { return op->timer.on ? op->timer.mark(s) : nullptr; }
void tspan(hh_op* op, int cat, hipEvent_t a, hipEvent_t b, bool clamp = false) {
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

bool is_sweep(int kind) { return kind == HH_PREC_SWEEP || kind == HH_PREC_SWEEP_REF; }

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
              const double* sin) {
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
  const bool slk = sl && fused_slk_use(K);
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
    const int blocks = fused_iter_blocks(n, a.bands);
    REQUIRE((size_t)(nparts + blocks) * width <= op->partials_cap,
            "partials workspace too small for the one-pass iteration (%d blocks)", nparts + blocks);
    if (slk)
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

}  // namespace

// ======================================================================== C ABI
#define HH_API extern "C" __attribute__((visibility("default")))
#define GUARD_BEGIN try {
#define GUARD_END                                  \
  }                                                \
  catch (const Error& e) {                         \
    return e.code;                                 \
  }                                                \
  catch (const std::exception& e) {                \
    g_err = e.what();                              \
    return HH_ERR_STATE;                           \
  }                                                \
  return HH_OK;

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

// The persistent apply chain of the dense form (sweep_dense.hip sweep_chain_kernel) where it
// fits, unless mode 2 (one launch per GEMV, replayed from a graph) or HH_SWEEP_CHAIN=0.
static void sweep_chain_configure(hh_op* op) {
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
static void sweep_dense_configure(hh_op* op) {
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
static void sweep_part_release(hh_op* op) {
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

static int sweep_part_wgs(hh_op* op) {
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

static void sweep_chunk_configure(hh_op* op) {
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
      apply_MA(op, V, g.sscale, Wb[0]);  // w_0 = M A (s_0 u_0)
      launch_multidot(V, ldv, 1, Wb[0], L, op->partials, blocks, s, stp);
      launch_reduce(op->partials, blocks, 4, 3, op->red + 16, s, stp);
      allreduce_sum_dev(op, op->red + 16, 3);
      launch_gmres_lag(g, 0, op->red + 16, op->red + 16 + 3, false, eps, ptol, stop_col, s);
      check_site(c, "one-pass: first projection + column", s);
      for (int c2 = 0; c2 < stop_col; ++c2) {
        const int K = c2 + 1, K2 = K + 1;
        const int np = run_fused(op, K, Wb[c2 & 1], Wb[(c2 + 1) & 1], op->red + 16, g.sscale + K);
        // (dots, |w|^2 and |u|^2 in one partial row: one reduce, one allreduce; on one rank the
        // reduce and the column in one launch)
        if (c->world == 1 && 2 * K2 + 2 <= 64 && lag_red_merge()) {
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
        if (merge_end) {  // (with x += V a, V b: see cycle_coef_kernel)
          launch_cycle_coef(g, stop_col, op->cab, s);
          launch_cycle_end(K, V, ldv, op->red + 16, g.vscale, op->cab, Wb[stop_col & 1], x,
                           V + (size_t)K * ldv, L, op->npart, blocks, s, stp);
        } else {
          launch_update(V, ldv, K, op->red + 16, g.vscale, Wb[stop_col & 1],
                        V + (size_t)K * ldv, L, op->npart, blocks, s, stp);
        }
        tspan(op, HH_SPAN_UPDATE, k0, tmark(op, s));
        launch_reduce(op->npart, blocks, kMaxNorms, 1, op->red + 8, s, stp);
        allreduce_sum_dev(op, op->red + 8, 1);
        launch_gmres_lag(g, stop_col + 1, nullptr, op->red + 8, true, eps, ptol, stop_col, s);
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
    if (merge_end)
      launch_cycle_finish(g, stop_col, V + (size_t)(stop_col + 1) * ldv, x, L, blocks, s);
    launch_gmres_solve(g, stop_col, merge_end, s);
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
