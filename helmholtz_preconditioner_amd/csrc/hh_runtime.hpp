// Internal host-runtime declarations shared by the runtime's translation units (the C ABI of
// include/helmholtz_amd.h is implemented across them):
//   runtime.cpp   contexts, operators (build_A_matrix, code.py:202), vectors, apply / tuning ABI
//   rt_apply.cpp  the halo exchange + stencil / fused M A launches over slabs and ranks, the
//                 preconditioners' applies, residuals, reductions, guarded halo allocations
//   rt_gmres.cpp  the one-pass GMRES iteration across slabs / ranks and hh_gmres (scipy's control
//                 flow, code.py:516)
//   rt_sweep.cpp  the sweeping preconditioner's apply, its configuration and ABI (row F1)
#pragma once

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

template <class T>
inline T* dalloc(size_t count) {
  if (count == 0) count = 1;
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, count * sizeof(T));
  if (e != hipSuccess)
    fail(HH_ERR_ALLOC, "hipMalloc(%zu bytes) failed: %s", count * sizeof(T), hipGetErrorString(e));
  return static_cast<T*>(p);
}
// a halo receive buffer against an unmapped guard granule when HH_GUARD_HALO=1 (rt_apply.cpp)
void* dalloc_guarded_bytes(size_t bytes, int device, bool at_end);
template <class T>
inline T* dalloc_guarded(size_t count, int device, bool at_end) {
  if (knobs().guard_halo == 0) return dalloc<T>(count);
  return static_cast<T*>(dalloc_guarded_bytes(std::max<size_t>(count, 1) * sizeof(T), device, at_end));
}
void dfree(void* p);  // hipFree, or the guarded mapping's release

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

namespace hh {
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
}  // namespace hh

namespace hh {
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
}  // namespace hh

namespace hh {
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
}  // namespace hh

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
  // the one-pass iteration's in-pass column (HH_LAG_RED=2): ticket counters and group rows
  unsigned* fold_tickets = nullptr;
  double* fold_gpart = nullptr;
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

namespace hh {

inline bool is_sweep(int kind) { return kind == HH_PREC_SWEEP || kind == HH_PREC_SWEEP_REF; }
void ensure_scratch(hh_op* op);
hipEvent_t tmark(hh_op* op, hipStream_t s);
void tspan(hh_op* op, int cat, hipEvent_t a, hipEvent_t b, bool clamp = false);
void check_site(const hh_ctx* c, const char* site, hipStream_t s);
void allreduce_sum_dev(hh_op* op, double* d, int count);
int run_stencil(hh_op* op, int epi, const double2* in, const double* in_scale,
                const double2* in1, double2* out0, double2* out1, bool shifted);
bool sl_fused_applies(const hh_op* op);
void run_sl2(hh_op* op, const double2* v, const double* vs, double2* out);
int run_point(hh_op* op, int pt, const double2* in0, double2* out0, bool shifted);
void reduce_norms(hh_op* op, int nparts, int dst, int cols);
void sl_sweeps(hh_op* op, const double2* T, double2* z1dst, double2* out);
double2* sl_first_dst(hh_op* op, double2* out);
void sweep_dense_release(hh_op* op);
void sweep_apply(hh_op* op, const double2* r, double2* out, bool asis);
void apply_MA(hh_op* op, const double2* v, const double* vs, double2* out);
void apply_M(hh_op* op, const double2* r, double2* out);
void norm2(hh_op* op, const double2* v, int dst);
bool sl_res_fused(const hh_op* op);
void run_sl2_res(hh_op* op, const double2* b, const double2* x, double2* v0, int dst);
void residual(hh_op* op, const double2* b, const double2* x, double2* v0, int dst);
int device_cus(hh_ctx* c);
int mnorm_slot(const hh_op* op, int dst);
void read_dev(hh_op* op, const double* dsrc, double* hdst, int count);
bool fused_default();
int run_fused(hh_op* op, int K, const double2* win, double2* wout, const double* raw,
              const double* sin, const PassFold* fold = nullptr);
void check_sweep_chain(hh_op* op);
size_t basis_pad();
void ensure_gmres(hh_op* op, int restart);
void sweep_chain_configure(hh_op* op);
void sweep_dense_configure(hh_op* op);
void sweep_part_release(hh_op* op);
int sweep_part_wgs(hh_op* op);
void sweep_chunk_configure(hh_op* op);

}  // namespace hh
