/*
 * helmholtz_amd.h -- C ABI of the MI355X-native Helmholtz operator apply and
 * GMRES solve (hot path of bocchs/helmholtz-preconditioner, code.py).
 *
 * Library: helmholtz_preconditioner_amd/libhelmholtz_amd.so (hipcc, gfx950).
 * Plain C types only: ints, doubles, host pointers and opaque handles.  No
 * torch types, no CUDA-compat headers.  Complex vectors are interleaved
 * (re, im) doubles -- the memory layout of a numpy complex128 array -- with the
 * reference's unknown ordering p = (j-1)*n + (i-1), i the fast axis
 * (code.py:81-113, f_vec = f_mat.flatten() at code.py:448).
 *
 * Error convention: every int-returning call returns HH_OK (0) or a negative
 * hh_err; hh_last_error() returns a thread-local message for the last failure.
 * The reference raises Python exceptions instead; the ctypes shim
 * (helmholtz_preconditioner_amd/_ffi.py) turns a negative code into an
 * exception carrying that message.
 *
 * Threading: a context is bound to the host thread that created it.  Calls are
 * synchronous on return (work is stream-ordered inside).
 */
#ifndef HELMHOLTZ_AMD_H
#define HELMHOLTZ_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HH_ABI_VERSION 2

typedef enum {
  HH_OK = 0,
  HH_ERR_INVALID = -1,   /* bad argument (shape, size, null pointer)           */
  HH_ERR_HIP = -2,       /* HIP runtime failure                                 */
  HH_ERR_RCCL = -3,      /* RCCL failure                                        */
  HH_ERR_ALLOC = -4,     /* device / host allocation failure                    */
  HH_ERR_STATE = -5,     /* call not valid in this state (e.g. wrong context)   */
  HH_ERR_ABORTED = -6    /* a hh_gmres callback returned non-zero: solve stopped */
} hh_err;

/* Preconditioner kinds filling the reference's M slot (code.py:510-511). */
typedef enum {
  HH_PREC_NONE = 0,            /* M = I                                          */
  HH_PREC_JACOBI = 1,          /* M = diag(A)^-1, fused into the stencil          */
  HH_PREC_SHIFTED_LAPLACE = 2, /* M ~= A_beta^-1 by damped-Jacobi sweeps on the   */
                               /* shifted operator build_A_matrix(c/sqrt(1+i*b))  */
  HH_PREC_SWEEP = 3,           /* sweeping moving-PML preconditioner, Engquist-Ying */
                               /* Alg. 2.4 (algo2_3/algo2_4, code.py:345-385) with  */
                               /* quirks Q1/Q2 corrected: M x = sweep(x)             */
  HH_PREC_SWEEP_REF = 4        /* the reference as run_solver runs it: inside        */
                               /* hh_gmres M x = algo2_4(b) for every x (Q1), middle  */
                               /* sweep u -= T u (Q2); plain applies use algo2_4(x)   */
} hh_precond_kind;

/* Operator-apply modes for hh_op_apply*. */
typedef enum {
  HH_APPLY_A = 0,        /* y = A x                         (code.py:516: A @ x) */
  HH_APPLY_JACOBI_A = 1, /* y = diag(A)^-1 A x                                   */
  HH_APPLY_PREC = 2,     /* y = M x   with the operator's configured M           */
  HH_APPLY_PREC_A = 3    /* y = M A x                                            */
} hh_apply_mode;

typedef struct hh_ctx hh_ctx; /* one device + (optionally) one RCCL rank        */
typedef struct hh_op hh_op;   /* one Helmholtz operator, sharded by row slab    */
typedef struct hh_vec hh_vec; /* a device-resident complex vector on an hh_op   */

/* ---------------------------------------------------------------- context */
int hh_abi_version(void);
const char* hh_last_error(void);
int hh_device_count(int* count);

/* RCCL bootstrap: rank 0 calls this and ships the 128 bytes to the others. */
int hh_comm_unique_id(unsigned char id_out[128]);

/* Diagnostic (no reference counterpart): the RCCL calls of the row-slab transport in one
 * process on `device` -- a 1-rank communicator, an in-place allreduce and a grouped
 * send/recv to itself on a second stream ordered by an event.  Writes the max abs error of
 * each (0 when RCCL works). */
int hh_comm_selftest(int device, double* allreduce_err, double* p2p_err);

/* Create a context on HIP device `device` as rank `rank` of `world` ranks
 * (one process per GPU).  world == 1: nccl_id may be NULL.  `virtual_slabs`
 * >= 1 splits this rank's rows into that many slabs on the same device, with
 * explicit halo copies between them (test mode for the slab decomposition;
 * production uses 1). */
int hh_ctx_create(int device, int rank, int world, const unsigned char* nccl_id,
                  int virtual_slabs, hh_ctx** ctx);
/* Same, choosing the inter-rank transport: HH_TRANSPORT_RCCL (production, one GPU per
 * rank) or HH_TRANSPORT_SHM (host-staged POSIX shared memory; several ranks may share one
 * GPU -- the test rehearsal of the N > 1 path on a single-GPU machine).  For SHM the 128
 * id bytes are any random token shared by all ranks. */
#define HH_TRANSPORT_RCCL 0
#define HH_TRANSPORT_SHM 1
int hh_ctx_create_ex(int device, int rank, int world, const unsigned char* id,
                     int virtual_slabs, int transport, hh_ctx** ctx);
int hh_ctx_destroy(hh_ctx* ctx);
/* Host-side collectives for harness timing (RCCL allreduce; no-op at world 1). */
int hh_ctx_allreduce_max(hh_ctx* ctx, double* values, int count);
int hh_ctx_allreduce_sum(hh_ctx* ctx, double* values, int count);
int hh_ctx_barrier(hh_ctx* ctx);
int hh_ctx_synchronize(hh_ctx* ctx);
/* Collectives (halo exchanges + allreduces) this rank has entered so far, 0 at world 1.  Every
 * rank of a job enters the same sequence, so when a job stalls the rank with the fewest is the
 * one that stopped (bench.py's watchdog reads it from its own thread while the main thread may
 * be blocked inside a collective: the read takes no lock and touches no device). */
int hh_ctx_progress(hh_ctx* ctx, long* collectives);
/* The library's HH_* environment knobs (A/B switches and diagnostics), read once per process,
 * as a JSON object {"HH_X": {"value": v, "default": d}, ...}: all of them, or (only_changed)
 * those that differ from the shipped path -- an empty object for a default run.  Writes at most
 * cap bytes (NUL-terminated); *needed (nullable) receives the full size. */
int hh_knobs_json(int only_changed, char* buf, int cap, int* needed);

/* --------------------------------------------------------------- operator */
/* Replaces build_A_matrix(b, const, eta, omega, h, n, c_mat), code.py:202-219
 * (coefficients: get_A_diag_block_coeffs code.py:70-115, get_upper/lower_A_block
 * code.py:130-154, PML profiles sigma1/sigma2/s1/s2 code.py:11-33).  The matrix
 * is never assembled: the operator keeps 1-D PML tables and the pre-transposed
 * 1/c^2 field of this rank's row slab.
 *   c_mat: (n+2)*(n+2) row-major doubles as the reference holds it, read as
 *          c_mat[i-1, j-1] (reference quirk Q3); NULL selects a constant medium
 *          c == c_const (no 2-D field is stored or streamed).
 *   mass_scale_re/im: multiplies omega^2 in the mass term (1 for A itself;
 *          1+i*beta gives the shifted-Laplace operator A_beta, identical to
 *          build_A_matrix(..., c_mat / sqrt(1+i*beta))).
 *   Rows are sharded over ranks in contiguous layer slabs. */
int hh_op_create(hh_ctx* ctx, int n, int b, double cconst, double eta,
                 double omega_re, double omega_im, double h, const double* c_mat,
                 double c_const, double mass_scale_re, double mass_scale_im,
                 hh_op** op);
int hh_op_destroy(hh_op* op);
/* Layers owned by this rank: global 0-based [j_begin, j_end); local length =
 * (j_end - j_begin) * n complex values. */
int hh_op_local_rows(hh_op* op, int* j_begin, int* j_end);
/* Configure the preconditioner used by HH_APPLY_PREC* and hh_gmres.  The sweeping kinds
 * factor every moving-PML sub-problem on the first call (algo2_3, code.py:345-353; b is the
 * PML width given to hh_op_create) and need a single-rank, single-slab operator. */
int hh_op_set_precond(hh_op* op, int kind, double beta, int sweeps, double damping);

/* Host-buffer apply, the LinearOperator.matvec path (scipy _interface.py:227):
 * x, y: this rank's local slab, 2*len doubles.  Does H2D, halo exchange, the
 * stencil kernel and D2H. */
int hh_op_apply(hh_op* op, const double* x, double* y, int mode);
/* diag(A) of the local slab (A.diagonal()), 2*len doubles. */
int hh_op_diagonal(hh_op* op, double* d);

/* Operator export: the CSR matrix build_A_matrix returns (code.py:202-219,
 * canonical scipy CSR: per row S, W, D, E, N in column order, nnz = 5n^2 - 4n; for the
 * 9-point operator SW, S, SE, W, C, E, NW, N, NE, nnz = (3n-2)^2), restricted
 * to this rank's rows, with global column indices.  Written on the device from the same
 * tables the stencil applies (the exported values are the applied operator, bit for bit),
 * then copied to the caller's host arrays.
 *   nnz:      entries in this rank's rows (hh_op_csr_nnz).
 *   indptr:   local rows + 1 int64 offsets (indptr[0] = 0).
 *   indices:  nnz column indices, int32 (index_bytes 4; needs n^2 < 2^31) or int64 (8).
 *   data:     2*nnz doubles (interleaved complex).
 *   kernel_ms (optional): duration of the device export kernels. */
int hh_op_csr_nnz(hh_op* op, int64_t* nnz);
int hh_op_export_csr(hh_op* op, int64_t* indptr, void* indices, int index_bytes, double* data,
                     double* kernel_ms);

/* ------------------------------------------------------------ device vecs */
int hh_vec_create(hh_op* op, hh_vec** v);
int hh_vec_destroy(hh_vec* v);
int hh_vec_upload(hh_vec* v, const double* host);
int hh_vec_download(hh_vec* v, double* host);
/* Deterministic synthetic fill: re, im uniform in [-1, 1) from a counter hash of
 * (seed, global index) -- identical for any slab decomposition. */
int hh_vec_fill_hash(hh_vec* v, uint64_t seed);
/* Device-resident apply: y = mode(A) x, including the halo exchange. */
int hh_op_apply_dev(hh_op* op, const hh_vec* x, hh_vec* y, int mode);

/* Timing harness: `iters` back-to-back device applies (x -> y) on the stream the
 * stencil runs on.  total_ms: HIP events bracketing the whole timed region.
 * kernel_ms: average stencil-kernel duration -- total / iters when one apply is one
 * launch (single rank, single slab, HH_APPLY_A); otherwise the average of events
 * recorded around the interior stencil launch of every apply. */
int hh_op_time_apply(hh_op* op, const hh_vec* x, hh_vec* y, int mode, int iters,
                     double* total_ms, double* kernel_ms);
/* The same over `nvec` distinct (x, y) pairs taken round-robin (apply i: xs[i % nvec] ->
 * ys[i % nvec]): with nvec * 32 B/unknown well above the 256 MiB Infinity Cache no apply can
 * reuse lines an earlier one left on the die, as in a solve, where each apply reads a new
 * vector. */
int hh_op_time_apply_set(hh_op* op, const hh_vec* const* xs, hh_vec* const* ys, int nvec,
                         int mode, int iters, double* total_ms, double* kernel_ms);

/* ------------------------------------------------------------------ solve */
/* Replaces scipy.sparse.linalg.gmres(A, f_vec, M=M, tol=1e-3, callback=...)
 * as called at code.py:516 (scipy 1.15.3 iterative.py:582-840): restarted,
 * left-preconditioned GMRES with scipy's control flow -- restart cycles,
 * legacy callback counting (maxiter caps inner iterations when
 * legacy_maxiter != 0, else restart cycles), the gh-8400 inner tolerance
 * ptol, the true-residual outer test ||b - A x|| <= max(rtol*||b||, atol),
 * breakdown test h1 <= eps*h0 and info = 0 / maxiter.  Orthogonalisation is
 * classical Gram-Schmidt (reorth != 0: CGS2) with fixed-order reductions.
 *   b, x: device vectors (x holds x0 on entry, the solution on exit).
 *   hist: optional host array of length >= maxiter*restart (legacy: maxiter)
 *         receiving presid/||b|| per inner iteration.
 *   cb:   optional per-iteration callback(user, iteration, presid/||b||); returns 0 to
 *         continue, non-zero to stop the solve at once (hh_gmres then returns
 *         HH_ERR_ABORTED; scipy propagates a callback's exception the same way).
 *         After HH_ERR_ABORTED the contents of x are unspecified: the small-grid cycle kernel
 *         (hh_op_set_small_cycle) queues up to 16 restart cycles per host synchronisation, so
 *         x may be up to 15 cycles past the iteration the callback stopped at (scipy's callers
 *         never see x in that case either: the exception propagates).
 *   x after HH_ERR_STATE is unspecified too: a cycle's end (the x update and the next
 *         residual) is queued before the host reads the cycle's report, so a grid-wide wait of
 *         the sweeping preconditioner that timed out (reported as HH_ERR_STATE) is detected
 *         after x has been updated from that cycle's garbage.
 * On every exit path -- success, error or abort -- the operator is left ready for plain
 * applies (no stale in-solve state). */
typedef int (*hh_gmres_callback)(void* user, long iteration, double rel_presid);
int hh_gmres(hh_op* op, const hh_vec* b, hh_vec* x, double rtol, double atol,
             int restart, long maxiter, int legacy_maxiter, int reorth,
             double* hist, long hist_cap, hh_gmres_callback cb, void* user,
             long* iters_out, int* info_out, double* rnorm_out, double* bnorm_out);
/* Per-restart-cycle hook of the following hh_gmres calls on `op` (NULL removes it): called
 * after each cycle's x update and true residual, where scipy calls callback(x) for
 * callback_type='x' (iterative.py, after `r = b - matvec(x)`; not after the legacy exit);
 * x is complete on the device, so the hook may download it (hh_vec_download).  Returns 0
 * to continue, non-zero to stop (HH_ERR_ABORTED). */
typedef int (*hh_gmres_cycle_callback)(void* user, long cycle);
int hh_op_set_cycle_callback(hh_op* op, hh_gmres_cycle_callback cb, void* user);
/* Batched form of hh_gmres's per-iteration callback for the following hh_gmres calls on `op`
 * (NULL removes it): called once per restart cycle, when that cycle's statuses reach the host
 * (the same point the per-iteration callback is called at), with the cycle's `count` values
 * presid/||b|| of iterations first_iteration .. first_iteration + count - 1.  One call per
 * cycle instead of one per iteration (a foreign-function caller such as ctypes pays its call
 * overhead once).  Returns 0 to continue, or r in [1, count] when the caller stopped after the
 * r-th value (any other non-zero value: after the last one); the solve then ends with
 * HH_ERR_ABORTED and iterations = first_iteration - 1 + r. */
typedef int (*hh_gmres_history_callback)(void* user, long first_iteration, int count,
                                         const double* rel_presid);
int hh_op_set_history_callback(hh_op* op, hh_gmres_history_callback cb, void* user);

/* Global reductions per GMRES inner iteration (no reference counterpart: scipy runs on one
 * process).  mode 1: classical Gram-Schmidt with two -- the projections (+ |w|^2), then the norm
 * of the updated vector (the round-1 path, bit-for-bit).  mode 2: ONE -- the norm of the vector
 * the previous iteration's update wrote travels with the projections (lagged normalisation: the
 * Hessenberg subdiagonal of column j is completed in iteration j+1, the SpMV input is scaled by a
 * Pythagorean estimate meanwhile; H, the residual history and x agree to rounding, one extra
 * collective per restart cycle).  mode 3: mode 2 with the update of iteration j, the M A of
 * iteration j+1 and its projections in ONE pass over the basis (each basis vector read from HBM
 * once per iteration instead of twice; single rank and slab, 5-point operator, M none or
 * Jacobi, restart <= 21; elsewhere as mode 0).  mode 0 (default): mode 3 where it applies
 * (HH_FUSED_ITER=0: not), else one reduction (mode 2) across ranks and two (mode 1) on a single
 * rank.  CGS2 (reorth) always uses mode 1. */
int hh_op_set_krylov_mode(hh_op* op, int mode);
/* Whole-cycle GMRES kernel for small grids (no reference counterpart): a restart cycle of
 * hh_gmres as ONE launch whose workgroups keep the Krylov basis on chip and meet once per inner
 * iteration (lagged normalisation as krylov mode 2), instead of five launches per iteration.
 * Applies on a single rank and slab, 5-point operator, M = none or Jacobi, without reorth, when
 * n <= 255 (n + 1 workgroups, one per CU, all resident at once: the kernel's own gate checks
 * it and refuses the grid before touching any state otherwise) and the basis fits the LDS
 * (3 n (restart + 1) x 16 B <= ~150 KB); up to 16 restart cycles run per launch.  mode -1 (default):
 * used when it applies and n^2 <= 2^18; 1: whenever it applies; 0: never.  Results agree with the
 * regular cycle to rounding. */
int hh_op_set_small_cycle(hh_op* op, int mode);
/* Which cycle form the last hh_gmres on `op` ran: 0 the regular per-launch cycle, 1 the
 * small-grid whole-cycle kernel, 2 the small-grid kernel refused at its first launch -- its
 * n + 1 workgroups could not be co-resident -- so the regular cycle ran the whole solve
 * instead (same results to rounding; no partial state), 3 the regular cycle with the one-pass
 * iteration (hh_op_set_krylov_mode 3). */
int hh_op_last_solve_path(hh_op* op, int* path);
/* Diagnostic: phase timing of the small-grid cycle kernel (workgroup 0's wall clock summed over
 * the following solves): phase_us (optional, 8 doubles) receives the totals so far in us
 * (0 stencil + z hand-off, 5 partial sums, 6 their publication, 1 all-reduce, 3 coefficients +
 * the neighbours' z, 2 basis update, 4 wait for the Givens step) and in [7] the shader-clock
 * cycles over the same span; then the counters restart (enable = 1) or stop (enable = 0). */
int hh_op_small_cycle_profile(hh_op* op, int enable, double* phase_us);
/* Diagnostic, with hh_op_small_cycle_profile enabled: workgroup 0's wall clock outside the
 * inner iterations, summed over the cycles so far, in us: [0] launch start
 * to the first iteration, [1] the last column's round + the Givens workgroup's solve (y received),
 * [2] the x update and the x rows' hand-off, [3] the next cycle's residual and its all-reduce;
 * the Givens workgroup's [4] waits for the rounds' sums, [5] per-round Hessenberg work, [6] last
 * column, triangular solve and publication of y; [7] the all-reduces' first hop as workgroup 0
 * sees it: its publication to column 0 reduced on it, i.e. the rows' arrival skew + one hop
 * (tail_us: 8 doubles). */
int hh_op_small_cycle_tail_profile(hh_op* op, double* tail_us);
/* Performance tuning of the stencil kernel used by HH_APPLY_A: variant in [0, 48) selects the
 * marching kernel's W/E exchange (LDS row / direct cached loads / wave shuffle), prefetch depth,
 * load/store cache policy and strip width, 96 + R (R = 2 .. 8 rows, + 16 / + 32 cache-policy
 * bits) the non-marching tile kernel (-1 = built-in default: tiles for standalone applies on
 * n >= 2048, marching inside hh_gmres and below); rows_per_block overrides
 * the band height one workgroup marches (0 = automatic); grid_blocks > 0 runs a
 * persistent grid of that many workgroups (0 = one per tile).  Results are identical
 * for every setting; only speed changes. */
int hh_op_tune(hh_op* op, int variant, int rows_per_block, int grid_blocks);
/* Stencil of the operator (the reference itself is 5-point only,
 * code.py:216-218, so this has no reference counterpart).  points = 5: the reference's
 * operator (default).  points = 9: alpha x the 5-point operator + (1 - alpha) x its
 * line-averaged form (each second difference averaged over the two neighbouring lines, with
 * those lines' PML factors) + the mass term spread over the 3x3 points with weights c (centre),
 * d (edges), e = (1 - c - 4d) / 4 (corners) -- the optimal 9-point PML scheme family
 * (Chen, Cheng, Feng & Wu 2013).  Second order for any weights with alpha, c, d finite;
 * tools/optimize_9pt.py derives the dispersion-optimal defaults the Python layer passes
 * (alpha 0.7910350, c 0.6276117, d 0.0948567: phase-velocity error <= 0.42 % at >= 4 points
 * per wavelength vs 10 % for 5 points).  Same HBM bytes per apply (40 B/unknown).  Every
 * apply, preconditioner (none / Jacobi / shifted-Laplace), GMRES and the CSR export
 * (nnz = (3n-2)^2) follow the selected stencil; the sweeping preconditioner needs 5 points. */
int hh_op_set_stencil(hh_op* op, int points, double alpha, double c, double d);
/* Two-sweep shifted-Laplace M: apply M A in one fused launch (default 1) or as the stencil
 * + sweep pair (0).  Same results bit for bit; the fused form moves 40 instead of 112 B per
 * unknown.  Any slab / rank layout (ranks exchange two halo rows for it); it needs the medium
 * two layers beyond every slab in the c_mat given to hh_op_create, else the pair runs. */
int hh_op_sl_fusion(hh_op* op, int enable);
/* Sweeping preconditioner form (speed / memory only; results agree to rounding):
 *   mode -1 (default) dense transfer matrices when n <= 2048 and the n^3 x 16 B fit in HBM,
 *           else as mode 0;  0 block-Thomas solves, the forward / backward sweeps' solves
 *           partitioned over 16 column chunks per workgroup and G workgroups (chunk products:
 *           2 x the factors' O(n^2 b^2) memory; dependent depth ~2 (n/16G + 32 + G) steps per
 *           solve; hh_op_sweep_workgroups) when n >= 32 and they fit,
 *           else sequential;  1 dense transfer matrices (error if they do not fit), their
 *           GEMV chain as ONE persistent cooperative launch when n <= 1024 (else one launch per
 *           GEMV);  2 dense, one launch per GEMV always (HH_SWEEP_CHAIN=0 does the same for
 *           modes -1 and 1);  3 block-Thomas sequential solves (2n dependent steps each).  The
 *           dense forms give the same results bit for bit, the others agree to rounding.
 * Applies at the next sweeping setup, or at once if the operator is already factored.
 * active (optional) receives 1 when the dense form is in use, 2 for partitioned solves,
 * 0 for sequential ones. */
int hh_op_sweep_mode(hh_op* op, int mode, int* active);
/* Workgroups sharing each partitioned block-Thomas solve (speed only; results agree to
 * rounding): 0 (default) by n (2 columns per chunk, at most 64 and the CU count, fewer when
 * the solve's vectors would not fit LDS), else that many, clamped to 64, the CU count and 2
 * columns per chunk.  G > 1 runs each forward / backward sweep as one cooperative launch of G
 * workgroups that exchange the solves' chunk carries through device memory.  Applies at the
 * next sweeping setup, or at once if the operator is already factored.  active (optional)
 * receives the workgroup count in use, 0 when the solves are not partitioned. */
int hh_op_sweep_workgroups(hh_op* op, int workgroups, int* active);
/* Diagnostic: phase timing of the partitioned solves.  enable = 1 starts (and zeroes) the
 * per-workgroup accumulators, 0 stops; phase_us (optional, cap entries) first receives the
 * sums so far, in microseconds of workgroup w's thread-0 wall clock: phase_us[16 w + k], k =
 * 0 chunk-local forward, 1 / 5 map staging, 2 / 6 zero-carry chunk chain + publish | polls,
 * 3 / 7 grid step, 4 fix-up + chunk-local backward, 8 fix-up + output (k = 1-3 forward
 * recurrence, 5-7 backward), summed over every solve of every sweep since enabled; up to 64
 * workgroups (w < 64). */
int hh_op_sweep_profile(hh_op* op, int enable, double* phase_us, int cap);
/* Process-wide tuning of the Krylov streaming kernels (multidot / update): non-temporal
 * basis loads on (1) / off (0) / by vector length (-1, default: on above 2^21 rank-local
 * unknowns) and the streaming grid size (0 = by vector length: 512 blocks up to 2^21
 * unknowns, 1024 above).  Speed only. */
int hh_tune_krylov(int nt_loads, int blocks);
/* Streaming roofline probes (diagnostic only): the stencil's byte mix without neighbour
 * traffic in different access shapes (`kind`, see csrc/probe.hip), `blocks` workgroups,
 * `iters` launches; outputs the average kernel ms and the probe's bytes per point. */
int hh_op_probe_stream(hh_op* op, int kind, int blocks, const hh_vec* x, hh_vec* y, int iters,
                       double* kernel_ms, int* bytes_per_point);
/* The same over `nvec` (x, y) pairs taken round-robin (cold inputs, as hh_op_time_apply_set). */
int hh_op_probe_stream_set(hh_op* op, int kind, int blocks, const hh_vec* const* xs,
                           hh_vec* const* ys, int nvec, int iters, double* kernel_ms,
                           int* bytes_per_point);

/* Diagnostic span timing (no reference counterpart): with timing enabled, the operator records
 * HIP events around the pieces of every apply and GMRES inner iteration on the streams they run
 * on; hh_op_read_timing synchronises the device, sums the spans per category (ms; counts = spans
 * recorded) and restarts the sums.  Categories:
 *   HALO       input complete (compute stream) -> the halo exchange done (halo stream)
 *   BOUNDARY   the boundary-row kernel(s) behind the exchange (halo stream)
 *   INTERIOR   the interior stencil / fused M A launch (compute stream)
 *   HALO_WAIT  compute stream idle after the interior launch until the boundary rows are done
 *              (0 when the exchange hid behind the interior)
 *   ALLREDUCE  each in-solve device allreduce (RCCL / SHM; none on one rank)
 *   COLUMN     the Givens / Hessenberg column kernel of an inner iteration
 *   MULTIDOT   projections V^H w and their fixed-order block reduction
 *   UPDATE     w -= V h (+ the norm partials)
 * Events add ~1-2 us of queue work each: enable it for diagnostic runs, not timed ones.
 * enable = 0 stops recording (and clears); the whole-cycle small-grid kernel is not split. */
#define HH_SPAN_HALO 0
#define HH_SPAN_BOUNDARY 1
#define HH_SPAN_INTERIOR 2
#define HH_SPAN_HALO_WAIT 3
#define HH_SPAN_ALLREDUCE 4
#define HH_SPAN_COLUMN 5
#define HH_SPAN_MULTIDOT 6
#define HH_SPAN_UPDATE 7
#define HH_SPAN_COUNT 8
int hh_op_set_timing(hh_op* op, int enable);
int hh_op_read_timing(hh_op* op, double* ms /* [HH_SPAN_COUNT] */, long* counts /* [HH_SPAN_COUNT] */);

/* Optional per-call counters of the last hh_gmres / hh_op_time_apply. */
typedef struct {
  double solve_ms;        /* wall ms inside hh_gmres                      */
  long inner_iterations;  /* legacy callback count                        */
  long restarts;          /* restart cycles run                           */
  long spmv_count;        /* operator applies (incl. residuals)           */
  double algorithmic_bytes; /* sum of per-kernel algorithmic bytes (local) */
} hh_stats;
int hh_op_last_stats(hh_op* op, hh_stats* stats);

#ifdef __cplusplus
}
#endif
#endif /* HELMHOLTZ_AMD_H */
