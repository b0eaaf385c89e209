// Inter-rank transport for the row-slab decomposition: the one-row halo exchange with the
// neighbouring ranks and the small global reductions of GMRES.
//   RcclComm : production -- ncclSend/ncclRecv pairs in one group on the halo stream and
//              ncclAllReduce on the compute stream (RCCL over xGMI; one process per GPU).
//   ShmComm  : test transport -- host-staged through a POSIX shared-memory segment with a
//              process-shared barrier; lets N ranks share ONE GPU (RCCL refuses duplicate
//              devices), so the N > 1 orchestration is exercised on a single-GPU box.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <memory>

namespace hh {

enum Transport : int { TRANSPORT_RCCL = 0, TRANSPORT_SHM = 1 };

class Comm {
 public:
  virtual ~Comm() = default;
  // In-place sum (or max) of `count` doubles in device memory, ordered on `s`.  The result
  // is identical on every rank.
  void allreduce(double* d, int count, bool max, hipStream_t s) {
    calls.fetch_add(1, std::memory_order_relaxed);
    do_allreduce(d, count, max, s);
  }
  // One-row halo exchange, ordered after the work already queued on `compute`:
  // send_lo -> rank-1, send_hi -> rank+1; recv_lo <- rank-1, recv_hi <- rank+1 (nullptr
  // where there is no neighbour).  Work for it is queued on `halo` (RCCL) or done
  // synchronously (SHM); the caller records its completion event on `halo`.
  void halo(const void* send_lo, void* recv_lo, const void* send_hi, void* recv_hi, size_t bytes,
            hipStream_t compute, hipStream_t hs, hipEvent_t ready) {
    calls.fetch_add(1, std::memory_order_relaxed);
    do_halo(send_lo, recv_lo, send_hi, recv_hi, bytes, compute, hs, ready);
  }
  // collectives this rank has entered (halo exchanges + allreduces): every rank of a job runs
  // the same sequence, so after a stall the rank with the fewest is the one that stopped
  // (hh_ctx_progress; bench.py's watchdog)
  long entered() const { return calls.load(std::memory_order_relaxed); }
  int rank = 0, world = 1;

 protected:
  virtual void do_allreduce(double* d, int count, bool max, hipStream_t s) = 0;
  virtual void do_halo(const void* send_lo, void* recv_lo, const void* send_hi, void* recv_hi,
                       size_t bytes, hipStream_t compute, hipStream_t hs, hipEvent_t ready) = 0;

 private:
  std::atomic<long> calls{0};
};

std::unique_ptr<Comm> make_rccl_comm(int rank, int world, const unsigned char id[128]);
std::unique_ptr<Comm> make_shm_comm(int rank, int world, const unsigned char id[128]);
void rccl_unique_id(unsigned char out[128]);
void rccl_selftest(int device, double* allreduce_err, double* p2p_err);

}  // namespace hh
