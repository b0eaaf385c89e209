// Sweeping moving-PML preconditioner (sweep.hip) -- shared declarations.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace hh {

struct SweepArgs {
  int n, b;            // grid size, PML width in layers (= sub-problem height)
  int nsys;            // 1 (H_F) + (n - b) sub-problems H_m, m = b+1..n (1-based)
  double2* P;          // [nsys][n][B][B] block-Thomas inverses Lambda_i^-1
  const double2* tab_i;     // operator's per-column PML table [3][n]
  const double2* tab_k;     // per-layer PML table of layers 0..b-1 (local PML of every H_m)
  const double2* tab_glob;  // operator's per-layer table [n][4] (S/N couplings of the sweep)
  const double* invc2;      // 1/c^2 [n][n] (row = layer) or nullptr
  double invc2_const;
  double2* yscr;       // per-wave solve scratch, ystride double2 each (sweep_scratch_per_wave)
  size_t ystride;
  const int* stop;     // GMRES cycle stop flag (kernels return at once when set)
  // chunked solves (partitioned Thomas): chunks = kSweepChunks splits the columns of every
  // system into that many contiguous chunks (0: the sequential solves); per (system, column) the B x B
  // products of the recurrence matrices inside its chunk -- forward Psi_f[i] = M_i .. M_a,
  // M_i = -P_i L_i; backward Psi_b[i] = N_i .. N_{e-1}, N_i = -P_i U_i -- laid out as P
  int chunks;
  double2* Pf;
  double2* Pb;
  // multi-workgroup partitioned solves: G workgroups (one persistent cooperative launch per
  // sweep), kSweepChunks chunks each (chunks = kSweepChunks G).  Pw [nsys][G][2][16][B][B]:
  // per workgroup the prefix (forward, 0) / suffix (backward, 1) products of its chunk maps
  // (sweep_wg_setup_kernel).
  // Carries cross workgroups as tagged granules, gran [2 dir][2 parity][G][kSweepGranStride].
  // Tm [nsys][2][sweep_grid_tri(G)][B][B]: the grid maps of the product-form grid step,
  // T(w, u) = Phi_{w-1} .. Phi_{u+1} (forward; backward Phi_{w+1} .. Phi_{u-1}) for every
  // workgroup w and upstream workgroup u at distance d = |w - u| >= 2, at
  // sweep_grid_tri(cnt_w) + d - 2 (cnt_w: the workgroups upstream of w; sweep_grid_setup_kernel).
  int G;
  double2* Pw;
  double2* Tm;
  unsigned long long* gran;
  unsigned* timeout;  // set when a grid wait gives up (the output is then garbage)
  unsigned seq;       // launch sequence number of the granule tags (1 .. 2^17 - 1)
  // diagnostic (hh_op_sweep_profile): per workgroup [G][kSweepProfSlots] s_memrealtime ticks of
  // the partitioned solves' phases, accumulated by each workgroup's thread 0; null: off
  unsigned long long* prof;
};
constexpr int kSweepProfSlots = 16;

// Storage order of every B x B block-Thomas matrix (P, Psi_f, Psi_b, the workgroup maps):
// entry (row j, column c) at pidx<B>(j, c) = (c % (B/2)) 2B + (c / (B/2)) B + j.  A half-wave
// of the partitioned solve (lanes g 16 + j, row j, columns g B/2 + q) then loads, per q, 2B
// contiguous entries -- coalesced, where row-major rows made every load instruction touch all
// of the matrix's cache lines.
template <int B>
__host__ __device__ constexpr int pidx(int j, int c) {
  return (c % (B / 2)) * 2 * B + (c / (B / 2)) * B + j;
}
// Grid-wide sweeps (the partitioned block-Thomas solves over G > 1 workgroups, the dense
// form's persistent chain) are cooperative launches, so a grid that cannot be co-resident fails
// at launch; HH_SWEEP_COOP=0 launches them as plain kernels, whose grid-wide waits are bounded
// anyway (a timeout word the host checks).  (ROCm 7.2 + rocprofv3: a process that made ANY
// cooperative launch dies with SIGSEGV inside exit() -- libamdhip64's exit handler tearing down
// an HSA queue after rocprofiler-sdk finalised, tools/exit_probe.py, DESIGN 3b: under
// rocprofv3 the launches are plain automatically, hh_internal.hpp under_profiler.)
bool sweep_coop_launch();
int sweep_block(int b);
size_t sweep_scratch_per_wave(int n);  // padded block size B (4, 8, 12, 16) or 0 if b > 16
// what: 0 factor (one wave per system), 1 forward sweep, 2 middle sweep, 3 backward sweep,
// 4 the chunk products Psi_f / Psi_b, the workgroup products Pw and the grid maps Tm (after 0;
// needs a.chunks = kSweepChunks a.G > 0, Pf, Pb, Pw, Tm).  With a.chunks > 0 the forward and
// backward sweeps run every solve partitioned over the chunks: a.G workgroups of kSweepChunks
// / 2 waves (one cooperative launch per sweep when G > 1), dependent depth ~2 (n / chunks +
// kSweepChunks + 2) steps instead of 2 n.
void launch_sweep(const SweepArgs& a, int what, double2* u, double2* uF, int asis,
                  hipStream_t st);
constexpr int kSweepChunks = 16;  // chunks per workgroup of a partitioned solve (two per wave)
constexpr int kSweepGranStride = 64;  // u64 granules per (direction, parity, workgroup)
// grid maps per half-wave of the product-form grid step requested ahead of the grid exchange
// (held in registers; with more than 2 + kSweepChunks kSweepGridMapsHeld workgroups the rest
// is loaded after it); kSweepMaxWgs the cap of a launch
constexpr int kSweepGridMapsHeld = 2;
constexpr int kSweepMaxWgs = 64;
// grid maps of a workgroup with cnt upstream workgroups before its own (distances 2 .. cnt)
__host__ __device__ inline size_t sweep_grid_tri(int cnt) {
  return cnt >= 2 ? (size_t)(cnt - 1) * (size_t)(cnt - 2) / 2 : 0;
}
// scratch (double2) of one partitioned solve: the n B-vectors + per-thread dummy slots
size_t sweep_chunk_scratch(int n);
// largest workgroup count of a partitioned solve for block size B
int sweep_part_max_wgs(int B);
// whether a partitioned solve over G workgroups keeps its B-vectors in LDS (else in yscr)
bool sweep_part_ys_lds(int B, int G, int n);
// u64 granules of SweepArgs::gran for G workgroups
size_t sweep_part_granules(int G);

// Dense-transfer form (sweep_dense.hip): n matrices of n x n -- A_ll^-1 (l < b) of H_F, then
// T_m (m = b+1 .. n) -- formed at setup from the block-Thomas factors; the apply is a GEMV chain.
size_t sweep_dense_bytes(int n);                       // bytes of the n matrices
size_t sweep_dense_scratch_per_block(int n, int b);    // setup scratch (double2) per block
int sweep_dense_chunks(int n);                          // setup blocks per system
void launch_sweep_dense_setup(const SweepArgs& a, int s_base, int batch, double2* yscr,
                              double2* T, hipStream_t st);
// The persistent form of the apply chain (sweep_dense.hip sweep_chain_kernel): one cooperative
// launch for the 2 (n - b) dependent GEMVs after F0, when n <= 1024 and its ceil(n / 4)
// workgroups (one per CU: 80-160 KB of LDS each) fit the device.
struct ChainArgs {
  const double2* T;
  int n, b;
  const double2* R1;        // operator's R1 = 1/s1 per column
  const double2* tab_glob;  // per-layer table [n][4] (BS at 1, BN at 2)
  const double2* r;
  double2* u;               // u_m (u_b written by F0 before the launch)
  double2* w;               // the result
  double a_in, t_sign;      // FWD / MID epilogue: w = t_sign t + a_in u_{m-1}
  const int* stop;          // GMRES cycle stop flag or nullptr
  unsigned long long* gbuf;  // [2][pad][4] tagged granules of each step's output (zeroed once)
  unsigned* timeout;        // set when a wait gives up
  unsigned seq;             // launch sequence number (granule tags)
  int diag;                 // diagnostic (HH_SWEEP_DIAG): 1 no matrix loads, 2 no input waits,
                            // 3 neither loads nor input reads, 4 no input reads
};
bool sweep_chain_fits(int n, int device_cus);
size_t sweep_chain_granules();  // u64 elements of ChainArgs::gbuf
// out = M r (r and out distinct, u: n^2 scratch); asis: middle sweep u -= T u (quirk Q2).
// chain non-null: the FWD/MID/BWD chain runs as one persistent launch (its gbuf, timeout, seq
// taken from *chain); otherwise as one launch per GEMV.
void launch_sweep_dense_apply(const SweepArgs& a, const double2* T, const double2* r,
                              double2* out, double2* u, int asis, hipStream_t st,
                              const ChainArgs* chain = nullptr);

}  // namespace hh
