// Inter-rank transports (see comm.hpp).
#include "comm.hpp"

#include <fcntl.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "hh_error.hpp"

namespace hh {

// ------------------------------------------------------------------------- RCCL
namespace {
class RcclComm final : public Comm {
 public:
  RcclComm(int r, int w, const unsigned char id[128]) {
    rank = r;
    world = w;
    ncclUniqueId uid;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    std::memcpy(&uid, id, 128);
    NCCLC(ncclCommInitRank(&comm_, w, uid, r));
  }
  ~RcclComm() override {
    if (comm_) ncclCommDestroy(comm_);
  }
  void do_allreduce(double* d, int count, bool max, hipStream_t s) override {
    NCCLC(ncclAllReduce(d, d, count, ncclFloat64, max ? ncclMax : ncclSum, comm_, s));
  }
  void do_halo(const void* send_lo, void* recv_lo, const void* send_hi, void* recv_hi,
               size_t bytes, hipStream_t compute, hipStream_t hs, hipEvent_t ready) override {
    // the halo stream starts once the input vector is complete on the compute stream
    HIPC(hipEventRecord(ready, compute));
    HIPC(hipStreamWaitEvent(hs, ready, 0));
    const size_t cnt = bytes / sizeof(double);
    NCCLC(ncclGroupStart());
    if (recv_lo) NCCLC(ncclRecv(recv_lo, cnt, ncclFloat64, rank - 1, comm_, hs));
    if (send_lo) NCCLC(ncclSend(send_lo, cnt, ncclFloat64, rank - 1, comm_, hs));
    if (recv_hi) NCCLC(ncclRecv(recv_hi, cnt, ncclFloat64, rank + 1, comm_, hs));
    if (send_hi) NCCLC(ncclSend(send_hi, cnt, ncclFloat64, rank + 1, comm_, hs));
    NCCLC(ncclGroupEnd());
  }

 private:
  ncclComm_t comm_ = nullptr;
};

// -------------------------------------------------------------------------- SHM
constexpr size_t kShmSlotDoubles = 256;          // allreduce slot per rank
// the fused shifted-Laplace M A exchanges TWO complex rows per side (run_sl2), the plain
// stencil one: slots hold two rows of up to n = 65536
constexpr size_t kShmMaxRow = 65536;
constexpr size_t kShmHaloBytes = 2 * kShmMaxRow * 16;
constexpr uint64_t kShmMagic = 0x48484d5348574d31ull;
constexpr double kShmTimeoutS = 300.0;

struct ShmHeader {
  std::atomic<uint64_t> magic;
  std::atomic<int> arrive;
  std::atomic<int> generation;
  std::atomic<int> detached;
  int world;
};

class ShmComm final : public Comm {
 public:
  ShmComm(int r, int w, const unsigned char id[128]) {
    rank = r;
    world = w;
    char hex[33];
    for (int k = 0; k < 16; ++k) snprintf(hex + 2 * k, 3, "%02x", id[k]);
    name_ = std::string("/hh_shm_") + hex;
    size_ = 4096 + (size_t)w * kShmSlotDoubles * sizeof(double) + (size_t)w * 2 * kShmHaloBytes;
    int fd = -1;
    if (r == 0) {
      fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) fail(HH_ERR_STATE, "shm_open(%s) create failed", name_.c_str());
      if (ftruncate(fd, (off_t)size_) != 0) fail(HH_ERR_ALLOC, "ftruncate shm failed");
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      while ((fd = shm_open(name_.c_str(), O_RDWR, 0600)) < 0) {
        if (elapsed(t0) > kShmTimeoutS) fail(HH_ERR_STATE, "rank %d: shm %s never appeared", r, name_.c_str());
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
      }
      struct stat st;
      const auto t1 = std::chrono::steady_clock::now();
      while (fstat(fd, &st) == 0 && (size_t)st.st_size < size_) {
        if (elapsed(t1) > kShmTimeoutS) fail(HH_ERR_STATE, "shm segment never sized");
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
      }
    }
    void* p = mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) fail(HH_ERR_ALLOC, "mmap shm failed");
    base_ = static_cast<char*>(p);
    hdr_ = reinterpret_cast<ShmHeader*>(base_);
    if (r == 0) {
      new (&hdr_->arrive) std::atomic<int>(0);
      new (&hdr_->generation) std::atomic<int>(0);
      new (&hdr_->detached) std::atomic<int>(0);
      hdr_->world = w;
      hdr_->magic.store(kShmMagic, std::memory_order_release);
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      while (hdr_->magic.load(std::memory_order_acquire) != kShmMagic) {
        if (elapsed(t0) > kShmTimeoutS) fail(HH_ERR_STATE, "shm header never initialised");
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
      if (hdr_->world != w) fail(HH_ERR_STATE, "shm world mismatch");
    }
    slots_ = reinterpret_cast<double*>(base_ + 4096);
    halo_ = base_ + 4096 + (size_t)w * kShmSlotDoubles * sizeof(double);
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&pin_), kShmSlotDoubles * sizeof(double)));
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&hpin_), 4 * kShmHaloBytes));
    barrier();
    // every rank has mapped the segment: drop its name now so nothing can leak in /dev/shm
    // (the mappings stay valid until each rank unmaps)
    if (r == 0) shm_unlink(name_.c_str());
  }
  ~ShmComm() override {
    // no barrier here: a peer may already have exited
    if (pin_) (void)hipHostFree(pin_);
    if (hpin_) (void)hipHostFree(hpin_);
    if (base_) munmap(base_, size_);
  }
  void do_allreduce(double* d, int count, bool max, hipStream_t s) override {
    REQUIRE(count <= (int)kShmSlotDoubles, "shm allreduce too large");
    HIPC(hipMemcpyAsync(pin_, d, count * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    std::memcpy(slots_ + (size_t)rank * kShmSlotDoubles, pin_, count * sizeof(double));
    barrier();
    for (int k = 0; k < count; ++k) {  // fixed rank order: identical result on every rank
      double acc = slots_[k];
      for (int q = 1; q < world; ++q) {
        const double v = slots_[(size_t)q * kShmSlotDoubles + k];
        acc = max ? std::max(acc, v) : acc + v;
      }
      pin_[k] = acc;
    }
    barrier();
    HIPC(hipMemcpyAsync(d, pin_, count * sizeof(double), hipMemcpyHostToDevice, s));
    HIPC(hipStreamSynchronize(s));
  }
  void do_halo(const void* send_lo, void* recv_lo, const void* send_hi, void* recv_hi,
               size_t bytes, hipStream_t compute, hipStream_t, hipEvent_t) override {
    REQUIRE(bytes <= kShmHaloBytes, "shm halo of %zu bytes exceeds the slot (two rows of n <= %zu)",
            bytes, kShmMaxRow);
    // Device <-> shared memory goes through this rank's pinned staging rows: DMA copies to /
    // from pinned memory on `compute` (ordered after the kernels that produced `send_*` and
    // before the boundary-row kernels that read `recv_*`), completed by a stream sync, and
    // plain CPU copies between the pinned rows and the shared segment.  Pageable (shm)
    // memory is never a DMA endpoint: its copy semantics are not stream-ordered.
    if (send_lo) HIPC(hipMemcpyAsync(hpin_, send_lo, bytes, hipMemcpyDeviceToHost, compute));
    if (send_hi) HIPC(hipMemcpyAsync(hpin_ + kShmHaloBytes, send_hi, bytes, hipMemcpyDeviceToHost, compute));
    HIPC(hipStreamSynchronize(compute));
    if (send_lo) std::memcpy(slot(rank, 0), hpin_, bytes);
    if (send_hi) std::memcpy(slot(rank, 1), hpin_ + kShmHaloBytes, bytes);
    barrier();
    if (recv_lo) std::memcpy(hpin_ + 2 * kShmHaloBytes, slot(rank - 1, 1), bytes);
    if (recv_hi) std::memcpy(hpin_ + 3 * kShmHaloBytes, slot(rank + 1, 0), bytes);
    barrier();  // the neighbours' slots may be refilled from here on
    if (recv_lo) HIPC(hipMemcpyAsync(recv_lo, hpin_ + 2 * kShmHaloBytes, bytes, hipMemcpyHostToDevice, compute));
    if (recv_hi) HIPC(hipMemcpyAsync(recv_hi, hpin_ + 3 * kShmHaloBytes, bytes, hipMemcpyHostToDevice, compute));
    HIPC(hipStreamSynchronize(compute));  // hpin_ is reused by the next exchange
  }

 private:
  static double elapsed(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  char* slot(int r, int side) { return halo_ + ((size_t)r * 2 + side) * kShmHaloBytes; }
  void barrier() {
    const int gen = hdr_->generation.load(std::memory_order_acquire);
    if (hdr_->arrive.fetch_add(1, std::memory_order_acq_rel) == world - 1) {
      hdr_->arrive.store(0, std::memory_order_relaxed);
      hdr_->generation.fetch_add(1, std::memory_order_acq_rel);
      return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    unsigned spins = 0;
    while (hdr_->generation.load(std::memory_order_acquire) == gen) {
      if (++spins > 1000) {
        sched_yield();
        if ((spins & 0xfff) == 0 && elapsed(t0) > kShmTimeoutS)
          fail(HH_ERR_STATE, "rank %d: shm barrier timed out", rank);
      }
    }
  }
  std::string name_;
  size_t size_ = 0;
  char* base_ = nullptr;
  ShmHeader* hdr_ = nullptr;
  double* slots_ = nullptr;
  char* halo_ = nullptr;
  double* pin_ = nullptr;
  char* hpin_ = nullptr;  // pinned halo staging: send lo, send hi, recv lo, recv hi
};
}  // namespace

std::unique_ptr<Comm> make_rccl_comm(int rank, int world, const unsigned char id[128]) {
  return std::make_unique<RcclComm>(rank, world, id);
}
std::unique_ptr<Comm> make_shm_comm(int rank, int world, const unsigned char id[128]) {
  return std::make_unique<ShmComm>(rank, world, id);
}
void rccl_selftest(int device, double* allreduce_err, double* p2p_err) {
  // The RCCL calls RcclComm makes, in one process: a 1-rank communicator, an in-place
  // float64 sum on the compute stream, and a grouped send/recv pair (to itself) on a second,
  // highest-priority stream ordered behind the compute stream by an event -- the halo pattern.
  constexpr int kCount = 4096;
  HIPC(hipSetDevice(device));
  struct Res {
    ncclComm_t comm = nullptr;
    hipStream_t s = nullptr, hs = nullptr;
    hipEvent_t ev = nullptr;
    double* d = nullptr;
    ~Res() {
      if (d) (void)hipFree(d);
      if (ev) (void)hipEventDestroy(ev);
      if (hs) (void)hipStreamDestroy(hs);
      if (s) (void)hipStreamDestroy(s);
      if (comm) ncclCommDestroy(comm);
    }
  } r;
  ncclUniqueId id;
  NCCLC(ncclGetUniqueId(&id));
  NCCLC(ncclCommInitRank(&r.comm, 1, id, 0));
  int lo = 0, hi = 0;
  HIPC(hipDeviceGetStreamPriorityRange(&lo, &hi));
  HIPC(hipStreamCreateWithFlags(&r.s, hipStreamNonBlocking));
  HIPC(hipStreamCreateWithPriority(&r.hs, hipStreamNonBlocking, hi));
  HIPC(hipEventCreateWithFlags(&r.ev, hipEventDisableTiming));
  HIPC(hipMalloc(reinterpret_cast<void**>(&r.d), 3 * kCount * sizeof(double)));
  std::vector<double> h(3 * kCount);
  for (int k = 0; k < kCount; ++k) h[k] = h[kCount + k] = 0.5 + k * 1e-3;
  for (int k = 0; k < kCount; ++k) h[2 * kCount + k] = -1.0;
  HIPC(hipMemcpyAsync(r.d, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, r.s));
  NCCLC(ncclAllReduce(r.d, r.d, kCount, ncclFloat64, ncclSum, r.comm, r.s));
  HIPC(hipEventRecord(r.ev, r.s));
  HIPC(hipStreamWaitEvent(r.hs, r.ev, 0));
  NCCLC(ncclGroupStart());
  NCCLC(ncclRecv(r.d + 2 * kCount, kCount, ncclFloat64, 0, r.comm, r.hs));
  NCCLC(ncclSend(r.d + kCount, kCount, ncclFloat64, 0, r.comm, r.hs));
  NCCLC(ncclGroupEnd());
  HIPC(hipStreamSynchronize(r.hs));
  std::vector<double> o(3 * kCount);
  HIPC(hipMemcpy(o.data(), r.d, o.size() * sizeof(double), hipMemcpyDeviceToHost));
  double ea = 0.0, ep = 0.0;
  for (int k = 0; k < kCount; ++k) {
    ea = std::max(ea, std::abs(o[k] - h[k]));
    ep = std::max(ep, std::abs(o[2 * kCount + k] - h[kCount + k]));
  }
  *allreduce_err = ea;
  *p2p_err = ep;
}

void rccl_unique_id(unsigned char out[128]) {
  ncclUniqueId id;
  NCCLC(ncclGetUniqueId(&id));
  std::memcpy(out, &id, 128);
}

}  // namespace hh
