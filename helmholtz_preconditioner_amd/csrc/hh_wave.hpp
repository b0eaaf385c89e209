// Wave-level helpers for gfx950 device code (64-lane waves): broadcast of one lane's double by
// readlane, and a fixed-order sum over the 64 lanes by DPP lane moves.
#pragma once
#include <hip/hip_runtime.h>

namespace hh {

// lane k's double, on every lane of the wave (k uniform)
__device__ __forceinline__ double rlane(double v, int k) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffff), k);
  const int hi = __builtin_amdgcn_readlane((int)(u >> 32), k);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double2 rlane2(double2 v, int k) {
  return make_double2(rlane(v.x, k), rlane(v.y, k));
}

// Sum over the 64 lanes of a wave by DPP lane moves (no LDS round trips, unlike a shuffle
// butterfly: 12 dependent ds_bpermute per double), fixed order; the total lands in lane 63.
// Pairs, quads, 8 (half-row mirror), 16 (row mirror), then row 0 -> 1 and row 2 -> 3
// (row_bcast:15), rows 0-1 -> 2-3 (row_bcast:31).  Lanes a move does not write read 0.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_mov(double x) {
  const long long u = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(u & 0xffffffff), CTRL, ROWS, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTRL, ROWS, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum_to_63(double v) {
  v += dpp_mov<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141, 0xf>(v);  // row_half_mirror
  v += dpp_mov<0x140, 0xf>(v);  // row_mirror
  v += dpp_mov<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
  v += dpp_mov<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3
  return v;
}

// Block-reduce NV doubles held per thread (a 256-thread block); the block's results land in
// partials[blockIdx.x * width + k].  SC1: stored write-through at device scope (agent-scope
// relaxed atomic stores), for a last block that reads them in the same launch
// (MI355X_MICROARCH.md's hand-off form: sc1 stores, drained, then one lane's agent-scope
// ticket; no L2-writeback fence).
template <int NV, bool SC1 = false>
__device__ __forceinline__ void block_reduce_vec(double (&v)[NV], double* partials, int width) {
  constexpr int kBT = 256;
  __shared__ double red[NV][kBT / 64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x / 64;
  // wave sums by DPP lane moves (VALU only; the xor butterfly took 12 dependent ds_bpermute per
  // value: ~500 LDS permutes per wave for the 41 values of a 20-vector multidot)
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double x = wave_sum_to_63(v[k]);
    if (lane == 63) red[k][wave] = x;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < NV; k += kBT) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kBT / 64; ++w) s += red[k][w];
    if constexpr (SC1)
      __hip_atomic_store(
          (__attribute__((address_space(1))) unsigned long long*)(partials +
                                                                  (size_t)blockIdx.x * width + k),
          (unsigned long long)__double_as_longlong(s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      partials[(size_t)blockIdx.x * width + k] = s;
  }
}

}  // namespace hh
