// Internal declarations shared by the HIP kernels and the host runtime.
// gfx950 (MI355X) only: 64-wide wavefronts, double2 = one 16-byte complex128.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace hh {

constexpr int kWave = 64;
constexpr int kStencilThreads = 256;   // one 256-wide strip of the fast axis i per block
constexpr int kReduceThreads = 256;
constexpr int kMaxProj = 32;           // max basis vectors per multidot/update launch
constexpr int kMaxNorms = 2;           // norm accumulators a stencil epilogue may produce
constexpr int kMaxStreamBlocks = 8192; // upper bound of the Krylov streaming grid

// Stencil epilogues (what the kernel writes after computing (A u) at a point).
enum Epi : int {
  EPI_AX = 0,        // out0 = s * A u
  EPI_JAC = 1,       // out0 = s * A u / D
  EPI_RES = 2,       // r = b - A u; out0 = r                    acc0 = |r|^2
  EPI_RES_JAC = 3,   // r = b - A u; out0 = r / D                acc0 = |r|^2, acc1 = |r/D|^2
  EPI_RES_SL = 4,    // r = b - A u; out0 = r; out1 = damp r / Dbeta   acc0 = |r|^2
  EPI_SL_FIRST = 5,  // t = s * A u; out0 = t; out1 = damp t / Dbeta
  EPI_SL_SWEEP = 6,  // z' = z + damp (r - Abeta z) / Dbeta   (u = z, in1 = r)
};

// W/E neighbour exchange of the stencil kernel (see stencil.hip).
enum XMode : int { XM_LDS = 0, XM_DIRECT = 1, XM_SHFL = 2 };
// Tuning variant of the marching kernel = XM + 3 * (PF - 1) + 6 * NT + 12 * NTU + 24 * (512-wide
// strips)  (0..47; the 512-wide set is instantiated for 24..27 and 30..33).  Variants 96 + R
// (+ 16: NT u loads, + 32: cached 1/c^2 and plain stores) select the non-marching R-row tile
// kernel (plain and Jacobi-fused apply; stencil.hip, tile_kernel / tile9_kernel).
constexpr int kNumVariants = 48;
// Shapes of the fused two-sweep shifted-Laplace M A (sl_fused.hip, hh_op_tune): kSl2Variant +
// shape (0: two barriers per row, 1: one barrier per row, 2: barrier-free wave strips, 3:
// sl2_tile_v2) + 4 (NT v
// loads; shape 3: one barrier per row, LDS tables, mask-free interior tiles).  The plain stencil
// launches ignore them (they take their default shape).
constexpr int kSl2Variant = 160;
constexpr bool sl2_variant(int v) {  // (+ 8: prefetch distance 2, shape 3 only)
  return v >= kSl2Variant && v < kSl2Variant + 16 && (v < kSl2Variant + 8 || (v & 3) == 3);
}

// Pointwise (no-neighbour) operations that need only the diagonal.
enum PointOp : int {
  PT_DIAG = 0,       // out0 = D
  PT_JAC = 1,        // out0 = in0 / D                       acc0 = |out0|^2
  PT_SL_FIRST = 2,   // out0 = damp in0 / Dbeta
  PT_COPY_NORM = 3,  // out0 = in0 (if distinct)             acc0 = |out0|^2
};

// Weights of the 9-point operator: Cartesian share alpha (g = (1 - alpha) / 2 on the
// line-averaged part) and mass weights c (centre), d (edges), e (corners), c + 4d + 4e = 1.
struct Stencil9W {
  double alpha, g, c, d, e;
};

struct StencilArgs {
  const double2* u;        // input slab [nl][n]
  const double2* halo_lo;  // global row j0-1 (zero row at the bottom boundary)
  const double2* halo_hi;  // global row j1   (zero row at the top boundary)
  const double* invc2;     // 1/c^2 [nl][n] (row j, column i), or nullptr
  double invc2_const;      // used when invc2 == nullptr
  const double2* tab_i;    // [3][n]: AW = s1((i-1/2)h)/h^2, AE = s1((i+1/2)h)/h^2, R1 = 1/s1(ih)
  const double2* tab_j;    // [nl][4]: R2 = 1/s2(jh), BS = s2((j-1/2)h)/h^2, BN = s2((j+1/2)h)/h^2,
                           //          OM = omega^2 * R2
  int n, nl;
  int row_begin, row_end;  // local rows computed by this launch
  int rows_per_block;      // strip height marched by one block
  int row_step;            // first-row distance of consecutive bands (0: rows_per_block)
  int tiles_x, tiles_y, tiles_per_xcd;  // XCD-aware tile map
  int grid_blocks;         // 0: one block per tile; >0: persistent grid of this many blocks
  double2 mshift;          // mass-term multiplier for the shifted operator (EPI_SL_*)
  double damping;          // damped-Jacobi weight (EPI_SL_*)
  const double* in_scale;  // lazily-normalised input: A (s u) = s (A u); nullptr -> 1
  const double2* in1;      // b (EPI_RES*) or r (EPI_SL_SWEEP)
  double2* out0;
  double2* out1;
  double* partials;        // [blocks][kMaxNorms] when the epilogue accumulates norms
  const int* stop;         // GMRES cycle stop flag: the launch is a no-op once *stop != 0
  // 9-point operator, selected by tab_r2x != nullptr: R2 = 1/s2 of the local
  // rows -1 .. nl ([nl + 2], entry r + 1 for row r) and the stencil weights (see stencil.hip)
  const double2* tab_r2x;
  Stencil9W w9;
  // fused SL kernel only (sl_fused.hip): halo_lo / halo_hi point at TWO rows each (rows -2, -1
  // and nl, nl+1), tab_j is valid for rows -2 .. nl+1, invc2_halo holds 1/c^2 of rows -2, -1,
  // nl, nl+1, and j0 is the slab's first global layer (z1 vanishes only off the grid)
  const double* invc2_halo;
  int j0;
  // fused shifted-Laplace residual (sl_fused.hip sl2_res_kernel): in1 = b over the slab, and
  // its two rows beyond each side (the neighbouring slab's, or zero rows off the grid)
  const double2* in1_lo;
  const double2* in1_hi;
};

struct PointArgs {
  const double2* in0;
  double2* out0;
  const double* invc2;
  double invc2_const;
  const double2* tab_i;
  const double2* tab_j;
  int n, nl;
  double2 mshift;
  double damping;
  double* partials;        // [blocks][kMaxNorms]
  const int* stop;         // as StencilArgs::stop
  int s9;                  // 1: 9-point operator, diagonal c M - alpha (W + E + S + N)
  Stencil9W w9;
};

// CSR export of one slab (assemble.hip).
struct CsrArgs {
  const double2* tab_i;    // as StencilArgs
  const double2* tab_j;    // this slab's [nl][4]
  const double* invc2;     // this slab's [nl][n], or nullptr
  double invc2_const;
  int n, nl;
  int j0;                  // global first layer of the slab
  int rank_j0;             // global first layer of the rank (indptr origin)
  size_t row_off;          // local row offset of the slab inside the rank
  int last;                // 1: also write indptr[row_off + nl n]
  long long* indptr;       // [local rows + 1], relative to the rank's first entry
  void* indices;           // int32 or int64 global column indices
  double2* data;
  const double2* tab_r2x;  // 9-point operator (as StencilArgs), or nullptr
  Stencil9W w9;
};
long long csr_rank_nnz(int n, int j0, int j1, int points = 5);
void launch_csr_export(const CsrArgs& a, int index_bytes, hipStream_t stream);

// Kernel launchers (kernels.hip).  All are asynchronous on `stream`.
void launch_stencil(int epi, bool const_c, const StencilArgs& a, int nblocks_out[1],
                    hipStream_t stream, int variant = -1);
int stencil_default_variant();
bool stencil_variant_valid(int v);  // instantiated for the plain apply
// the variant a launch really uses (requested < 0: size-dependent default; kVariantInSolve:
// the default inside a GMRES cycle, whose inputs the previous kernel has just written)
constexpr int kVariantInSolve = -2;
int stencil_resolve_variant(int epi, int requested, int n);
// Streaming roofline probes (probe.hip); returns the probe's bytes per point (0: unknown kind).
int launch_probe_kind(int kind, int blocks, const double2* u, const double* ic, double2* y,
                      size_t len, hipStream_t s);
int stencil_grid_blocks(int n, int rows, int rows_per_block, int row_step = 0);
int stencil_bands(int rows, int rows_per_block, int row_step);  // tiles along j
// Fused M A for the two-sweep shifted-Laplace M (sl_fused.hip): a.u = v, a.out0 = w; two halo
// rows per side and the extended tables (StencilArgs, fused SL fields); a.tab_r2x != nullptr
// selects the 9-point operator.
void launch_sl2(bool const_c, const StencilArgs& a, hipStream_t stream, int variant = -1);
// v0 = M (b - A x) for the two-sweep shifted Laplace in one pass (5-point; one slab's rows -- across
// slabs and ranks runtime's run_sl2_res supplies b's and x's two rows beyond it): a.u = x,
// a.in1 / in1_lo / in1_hi = b, a.out0 = v0; per block |r|^2 and |M r|^2 into a.partials
// (width kMaxNorms).  Returns the blocks launched (the partial rows written).
int launch_sl2_res(bool const_c, const StencilArgs& a, hipStream_t stream);
int sl2_res_blocks(int n, int rows, int rows_per_block);
int stencil_rows_per_block(int n, int rows);
void launch_point(int op, bool const_c, const PointArgs& a, int blocks, hipStream_t stream);
int point_blocks(size_t len);

// Krylov kernels.
//   multidot: partials[blk][2K+2] = sum conj(V_k) w (K vectors, stride ldv), |w|^2 at [2K]
// `stop` (optional): device flag of a queued GMRES cycle; kernels return at once when set.
void launch_multidot(const double2* V, size_t ldv, int K, const double2* w, size_t len,
                     double* partials, int blocks, hipStream_t stream, const int* stop = nullptr);
//   update: w_out = w - sum_k coef_k V_k, coef_k = scale_k^2 * raw_k (raw from reduced dots);
//   acc |w_out|^2 into partials[blk][0]
// Single-rank fused forms (one launch fewer each): the multidot whose last block also reduces
// the `cols` partial columns into `out` (bit-identical to launch_reduce), and the update whose
// last block also folds the norm partials and completes Hessenberg column `col` (bit-identical
// to launch_gmres_column with norm partials).  `counter`: a zeroed device word per kernel,
// re-armed by the kernel itself.
void launch_multidot_reduced(const double2* V, size_t ldv, int K, const double2* w, size_t len,
                             double* partials, int blocks, double* out, int cols,
                             unsigned* counter, hipStream_t stream, const int* stop);
void launch_update(const double2* V, size_t ldv, int K, const double* raw, const double* scale,
                   const double2* w, double2* w_out, size_t len, double* partials, int blocks,
                   hipStream_t stream, const int* stop = nullptr);
//   xupdate: x += sum_k y_k V_k  (y complex, device, already including scales); ctl (nullable):
//   the cycle's control words -- ctl[2] skips, k > ctl[1] count zero (krylov.hip xupdate_kernel)
void launch_xupdate(const double2* V, size_t ldv, int K, const double2* y, double2* x,
                    size_t len, int blocks, hipStream_t stream, const int* ctl = nullptr);
int stream_blocks(size_t len);
void tune_krylov(int nt, int blocks);  // global knobs (tuning studies only)
// Deterministic reduction of `count` partial rows of width `width` (fixed order):
// out[k] = sum_b partials[b*width + k] for k < cols.  One block per column.
void launch_reduce(const double* partials, int count, int width, int cols, double* out,
                   hipStream_t stream, const int* stop = nullptr);
// out[k] += in[k], k < count (tiny, one block).
void launch_add_small(const double* in, double* out, int count, hipStream_t stream,
                      const int* stop = nullptr);
// Hash fill of a slab vector (global element offset `goff`).
void launch_fill_hash(double2* v, size_t len, size_t goff, uint64_t seed, hipStream_t stream);
void launch_scale_copy(const double2* in, double2* out, size_t len, double s, hipStream_t stream,
                       const int* stop = nullptr);

// GMRES device state machine step (single wave, krylov.hip).
struct GivensState {
  // Device buffers (complex as double2).
  double2* H;      // [restart][restart+1]   H[col*(restart+1) + k]
  double2* G;      // [restart][2] (c, s)
  double2* S;      // [restart+1]
  double* vscale;  // [restart+1] real scales of the stored basis vectors (1 / their norms)
  double* sscale;  // [restart+1] scale of each SpMV input: = vscale (two-allreduce mode), or
                   // its Pythagorean estimate (one-allreduce mode, gmres_lag_kernel)
  double2* ycoef;  // [restart] x-update coefficients y_k * vscale_k
  double* status;  // [8]: 0 presid, 1 breakdown, 2 h0, 3 h1, 4 rnorm, 5 mnorm
  double* status_it;  // [restart][4]: presid, breakdown, h0, h1 of every inner iteration
  int* ctrl;          // [0] stop flag of the queued cycle, [1] last column executed
  int restart;
};
// One pass over the Krylov basis per lagged GMRES inner iteration (fused.hip
// fused_iter_kernel; 5-point operator, M = none, Jacobi or the two-sweep shifted Laplace): the
// update of iteration K-1, u_K = w_{K-1} - sum_{k<K} c_k u_k (c_k = d_k s_k^2 from the raw dots
// and the basis scales, as update_kernel), written to V + K ldv; then w_K = M A (s_K u_K) into
// wout; per block ONE partial row (width 2 (K + 1) + 2): <u_k, w_K> for k <= K and |w_K|^2 --
// multidot_kernel's quantities -- then |u_K|^2.  Every basis vector is read from HBM once per
// iteration instead of twice.  One launch covers rows [row_begin, row_end) of one slab; the
// rows just outside the slab (u_K of rows -H .. -1 and nl .. nl+H-1, H = 1, or 2 for the
// shifted Laplace) come from `lo_mode` / `hi_mode`.
enum FusedRow : int {
  FROW_ZERO = 0,  // off the grid: u_K = 0 (homogeneous Dirichlet)
  FROW_MEM = 1,   // a neighbouring slab of the same rank, contiguous in memory: formed in place
  FROW_HALO = 2,  // a neighbouring rank's rows of u_K, received into halo_lo / halo_hi
};
// The in-pass column of the one-pass iteration on one rank (HH_LAG_RED=2, round 6): the pass's
// own blocks reduce its partial rows in reduce_kernel's exact order (the blocks of each residue
// class mod kFoldClasses, then the classes: hh_fused.hpp pass_fold) and the last one runs the
// lag step (gmres_lag_kernel's arithmetic) -- no reduce / lag launch, no launch boundary
// between two passes; bit-identical to them.  tickets == nullptr: off.
constexpr int kFoldClasses = 64;
struct PassFold {
  unsigned* tickets;  // [1 + kFoldClasses] zeroed counters, re-armed by the kernel
  double* gpart;      // [64 columns][kFoldClasses] the classes' tree sums U_r
  double* red;        // the reduced row (red + 16: gmres_lag_kernel's operands)
  GivensState g;
  int j, stop_col;
  double eps, ptol;
};
struct FusedArgs {
  const double2* V;        // basis, at the slab's first row (negative row offsets: FROW_MEM)
  size_t ldv;
  const double2* win;      // w_{K-1}, at the slab's first row
  double2* wout;           // w_K
  double2* uout;           // u_K (= V + K ldv)
  const double* raw;       // raw dots d_k (2 K doubles) of w_{K-1}
  const double* vscale;    // s_k, k < K
  const double* sin;       // s_K, the scale of the SpMV input (gmres_lag_kernel's estimate)
  const double2* tab_i;
  const double2* tab_j;    // the slab's rows (shifted Laplace: rows -2 .. nl+1 valid)
  const double* invc2;     // the slab's [nl][n], or nullptr (constant medium)
  double invc2_const;
  const double* invc2_halo;  // shifted Laplace: 1/c^2 of rows -2, -1, nl, nl+1 (Slab)
  int n;                   // row length
  int nl;                  // rows of the slab
  int row_begin, row_end;  // rows of this launch
  int rows;                // rows per band
  int row_step;            // first-row distance of consecutive bands (0: rows)
  int bands;               // bands of this launch (grid: fused_iter_blocks)
  int lo_mode, hi_mode;    // FusedRow of the rows below / above the slab
  const double2* halo_lo;  // FROW_HALO: u_K of rows -H .. -1, [H][n]
  const double2* halo_hi;  //            u_K of rows nl .. nl+H-1
  int jac;                 // 1: Jacobi M
  int sl;                  // 1: the two-sweep shifted-Laplace M (fused_sl_iter_kernel)
  double2 mshift;          // SL: mass-term multiplier of A_beta
  double damping;          // SL: damped-Jacobi weight
  double* partials;        // this launch's partial rows
  const int* stop;
  int alt;                 // fused_iter_kernel: odd bands march downwards (fused_alt_dir)
  PassFold fold;           // the in-pass column (single rank), or fold.tickets == nullptr
};
// Running under rocprofv3 (its preloaded rocprofiler-sdk: ROCPROFILER_LIBRARY_CTOR /
// ROCPROF_OUTPUT_PATH in the environment, or a rocprofiler library in LD_PRELOAD)?  ROCm 7.2:
// a process that made any cooperative launch dies with SIGSEGV inside exit() once
// rocprofiler-sdk has finalised (tools/exit_probe.py), so the grid-wide sweeps and
// the small-grid cycle then launch plainly (their waits are bounded either way); logged once.
bool under_profiler();
constexpr int kFusedMaxK = 20;  // K <= this (restart <= kFusedMaxK + 1)
// basis vectors whose projection re-read is served from the pass's own LDS copy (HH_FUSED_KEEP:
// 0 = every re-read from the memory system, for A/B)
constexpr int kFusedKeepDefault = 17;
int fused_iter_rows(int n, int rows);  // band height for a slab of `rows` rows
int fused_iter_blocks(int n, int bands);
void launch_fused_iter(int K, const FusedArgs& a, int blocks, hipStream_t stream);
// the shifted-Laplace pass with the whole basis window on chip (fused_slk.hip; one block per
// CU): used for K >= HH_SLK (default 2; 0 = never) above fused_slv's range, with its own band
// height
bool fused_slk_use(int K);
// fused_iter_kernel's odd bands march downwards (HH_FUSED_ALT, read once), so the halo rows a
// band re-forms are read while their owners read them too (fused.hip)
bool fused_alt_dir();
bool lag_red_merge();  // HH_LAG_RED != 0 (default 2: in the pass where it can, else merged)
int fused_slk_rows(int n, int rows);
void launch_fused_slk(int K, const FusedArgs& a, int blocks, hipStream_t stream);
// the shifted-Laplace pass in the standalone fused M A's shape (fused_slv.hip: overlapping
// strips, no edge waves, four waves per SIMD, the projections' basis rows re-read from L2): used
// for K <= HH_SLV; its grid (252 output columns per strip)
bool fused_slv_use(int K);
int fused_slv_blocks(int n, int bands);
void launch_fused_slv(int K, const FusedArgs& a, int blocks, hipStream_t stream);
// u_K on rows [r0, r0 + c0) and [r1, r1 + c1) of a.V / a.win (rank-local), written to a.uout:
// the rows a neighbouring rank's pass reads as its halo (fused_iter_kernel's arithmetic)
void launch_fused_edge(int K, const FusedArgs& a, int r0, int c0, int r1, int c1,
                       hipStream_t stream);

// The end of a one-pass cycle that reaches its last column col (fused.hip): cycle_coef writes
// ab[k] = a_k s_k, ab[kMaxProj + k] = b_k s_k (y = a + y_col b, k <= col; a no-op once the
// stop flag is up); cycle_end forms the last update's |u|^2 partials (partials[blk][kMaxNorms])
// and, from the same loads, x += sum a_k s_k V_k in place and vb = sum b_k s_k V_k over K =
// col + 1 vectors; after the last column is finished, cycle_finish does x += y_col vb.
void launch_cycle_coef(const GivensState& g, int col, double2* ab, hipStream_t stream);
void launch_cycle_end(int K, const double2* V, size_t ldv, const double* raw, const double* vscale,
                      const double2* ab, const double2* w, double2* x, double2* vb, size_t len,
                      double* partials, int blocks, hipStream_t stream, const int* stop,
                      const PassFold* fold = nullptr);
// the one-pass cycle's first dots (multidot_kernel<1>'s partial row) with the reduce and the
// first lag step folded in (one rank; fold_reduce_lag)
void launch_cycle_start_dots(const double2* V, const double2* w, size_t len, double* partials,
                             int blocks, bool nt, hipStream_t stream, const int* stop,
                             const PassFold& fold);
bool krylov_nt_for(size_t len);  // the Krylov kernels' NT basis loads at this length
// x += y_col vb, only if the cycle reached its last column col (g.ctrl[1] == col)
void launch_cycle_finish(const GivensState& g, int col, const double2* vb, double2* x, size_t len,
                         int blocks, hipStream_t stream);

// After multidot+update reductions: column `col` of H from raw dots (red_dots, 2*(col+1)
// doubles + |w|^2 at [2*(col+1)]) and |w_new|^2 (red_norm[0]).  Then scipy's inner-loop
// exit test (iterative.py:792-795) on the device: presid <= ptol, breakdown, or
// col == stop_col (the legacy maxiter cap) raises ctrl[0], which turns every kernel queued
// after it in this cycle into a no-op.
// With norm_partials non-null, |w_new|^2 is instead summed from the update kernel's
// `norm_count` block partials inside this launch (bit-identical to launch_reduce; single rank
// only -- across ranks the norm needs the allreduce in between).
void launch_update_column(const double2* V, size_t ldv, int K, const double* raw,
                          const double* scale, const double2* w, double2* w_out, size_t len,
                          double* partials, int blocks, hipStream_t stream, const int* stop,
                          const GivensState& g, int col, const double* red_dots, double eps,
                          double ptol, int stop_col, unsigned* counter);
void launch_gmres_column(const GivensState& g, int col, const double* red_dots,
                         const double* red_norm, const double* norm_partials, int norm_count,
                         double eps, double ptol, int stop_col, hipStream_t stream);
// One-allreduce iteration j (lagged normalisation; krylov.hip gmres_lag_kernel): finishes column
// j-1 with |u_j|^2 = *sig2, starts column j from the raw dots red_dots (2(j+1) doubles, |w|^2
// after them) and estimates the next SpMV input scale.  final_step: only finish column j-1.
// launch_reduce + launch_gmres_lag in one launch (single rank: no allreduce between them)
void launch_gmres_lag_red(const GivensState& g, int j, const double* partials, int count,
                          int width, int cols, double* red, double eps, double ptol, int stop_col,
                          hipStream_t stream, int final_step = 0);
void launch_gmres_lag(const GivensState& g, int j, const double* red_dots, const double* sig2,
                      bool final_step, double eps, double ptol, int stop_col, hipStream_t stream);
// Start of a cycle: S[0] = ||Mr||, vscale[0] = 1/||Mr|| from red[idx_m]; status[4] = ||r||.
void launch_gmres_start(const GivensState& g, const double* red, int idx_r, int idx_m,
                        hipStream_t stream);
// A whole restart cycle in one launch for small single-rank grids (gmres_small.hip): workgroup g
// owns row g with the basis on chip, one grid barrier per inner iteration (lagged
// normalisation, as gmres_lag_kernel), then the triangular solve and x += V y.
struct SmallCycleArgs {
  int n, restart, stop_col;
  const double2* tab_i;    // as StencilArgs (single slab: rows 0 .. n-1)
  const double2* tab_j;
  const double* invc2;     // or nullptr (constant medium)
  double invc2_const;
  double2* v0;             // V[0] = M r, unnormalised: in, and out for the next cycle
  const double* mnorm2;    // |M r|^2 (the residual's reduction; gmres_start_kernel's input)
  const double2* b;        // right-hand side (the next cycle's residual)
  double2* x;              // x += V y at the end of the cycle
  double* red;             // device: red[4] = |r|^2, red[5] = |M r|^2 of the new x
  double* report;          // host-mapped: report[4..5] the same, for the host's outer loop
  GivensState g;           // status_it, ctrl[0..1] out (host-mapped: no copy after the cycle)
  double eps, ptol;
  unsigned long long* zbuf;  // [2][n][4n] tagged granules of the z rows handed to the neighbours
  unsigned long long* xbuf;  // [n][4n] tagged granules of the new x rows (the residual)
  unsigned long long* part;  // [2][n][2 kSmallCols] tagged granules of the partial sums
  unsigned long long* sums;  // [kSmallRounds][2 kSmallCols] tagged granules of the reduced sums
  unsigned long long* verdict;  // [kMaxProj][2] the Givens workgroup's per-column exit verdicts
  unsigned long long* ycoef;    // [kMaxProj + 1][4] y_k / sigma_k, then the solved column
  unsigned seq;            // launch sequence number: the tags of this launch's granules
  unsigned* timeout_word;  // set when a wait gives up (zeroed at the start of a solve)
  unsigned long long* phase_ticks;  // optional [kSmallTicks]: workgroup 0's wall-clock ticks
  // optional (device) scipy's restart-loop state, so that several cycles can be queued behind
  // each other: [0] ptol, [1] ptol_max_factor, [2] atol, [3] inner iterations so far,
  // [4] maxiter, [5] legacy (maxiter caps inner iterations), [6] done.  A launch that finds
  // `done` (or the timeout word) set returns at once with ctrl[0] = 2; otherwise it takes
  // stop_col / ptol from here and, after its residual, takes scipy's decisions for the next
  // cycle (report[6] = done, report[7] = the next ptol).  nullptr: stop_col / ptol as given.
  double* outer;
  // cycles in this launch (>= 1; > 1 needs `outer`): cycle c tags with seq + c and reports into
  // report + c kRedDoubles (statuses at + kRedStatus, control words at + kRedCtrl)
  int cycles;
  unsigned long long* obuf;  // [8] granules: the restart-loop state handed to the next cycle
  unsigned long long* mbuf;  // [n][4n] granules: the next cycle's V[0] rows for the neighbours
  unsigned* gate_arrive;     // [n + 1] co-residency gate: each workgroup's arrival (seq)
  unsigned long long* gate_decide;  // the gate's decision word ((seq << 2) | 1 go / 2 abort)
  int gate_force_abort;      // test hook: workgroup 0 decides ABORT (HH_SMALL_COOP_REFUSE=1)
};
constexpr int kOuterDoubles = 8;
// layout of an operator's reduction buffer `red` and of each slot of its host mirror: [0, 256)
// reductions, [256, 384) the cycle's per-iteration statuses, [384, 388) control words
constexpr int kRedDoubles = 512;
constexpr int kRedStatus = 256;
constexpr int kRedCtrl = 384;
constexpr int kSmallTicks = 16;  // phase_ticks: 7 loop phases, shader clock, 4 head / tail spans,
                                 // 3 Givens-workgroup spans
// columns of the small cycle's all-reduce rows: 2 K dot halves, |z|^2, |u_j|^2 (K <= kMaxProj)
constexpr int kSmallCols = 2 * (kMaxProj + 1) + 2;
constexpr int kSmallRounds = kMaxProj + 8;  // all-reduce rounds per launch (<= restart + 3)
bool small_cycle_eligible(int n, int restart, int device_cus);
size_t small_cycle_lds_bytes(int n, int restart);
size_t small_cycle_scratch_doubles(int n);
// returns a launch error instead of throwing; a grid that cannot be co-resident is refused on the
// device (report slot 0: ctrl = 3) before any state changed, so the caller can take the regular
// cycle
hipError_t launch_small_cycle(const SmallCycleArgs& a, bool const_c, bool jacobi, hipStream_t s);
// End of a cycle: triangular solve for y, ycoef_k = y_k * vscale_k, over the columns the cycle
// executed (g.ctrl[1] <= stop_col, read on the device); `merged`: a cycle that reached stop_col
// was completed by the merged end instead (g.ctrl[2] = 1: the xupdate skips).
void launch_gmres_solve(const GivensState& g, int stop_col, bool merged, hipStream_t stream);

// Every HH_* environment knob, read once per process (knobs.cpp; the table there gives each
// one's default -- the shipped path -- and meaning).  hh_ctx_create reads them first, so a
// malformed value fails there; hh_knobs_json reports them.
struct Knobs {
  long fused_iter, sl_res, slk_min_k, slv_max_k, slv_keep_max, slk_rows, fused_rows, fused_keep, fused_alt, lag_red,
      cycle_merge, basis_pad, krylov_fuse, krylov_rev, tile_xcd;
  long sweep_chain, sweep_graph, sweep_coop, sweep_diag;
  long small_coop, small_wide, small_coop_refuse, small_refuse_at;
  long check_halo, guard_halo;
};
const Knobs& knobs();

}  // namespace hh
