// Intra-node shared-memory all-reduce for CPU ranks (the CPU / gloo path of BASELINE config 1:
// the reference's mpiexec ranks on one machine, ref.py:61-63,185-203).  MPI moves such tiny
// messages through shared memory; torch's gloo goes through loopback TCP, ~0.3-0.4 ms per
// all-reduce of the 13-parameter gradient -- ten times the whole native step.
//
// Segment: one cache line holding a monotonic arrival counter, then two parity banks of
// `world` fp32 slots of `cap` elements.  Call k: every rank copies its vector into slot
// [k & 1][rank], adds 1 to the counter (release) and waits until it reads (k + 1) * world
// (acquire); then every rank sums the `world` slots IN RANK ORDER into its own buffer, so all
// replicas get the same bits.  A rank can only write bank k & 1 again in call k + 2, after the
// wait of call k + 1, i.e. after every rank has finished reading call k: one wait per call.
// A stalled peer is detected by a timeout (the caller's watchdog then aborts the job).
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include "shm_comm.h"

namespace nnmpi {

namespace {
constexpr size_t kHeader = 128;
}

ShmComm::ShmComm(const std::string& name, int rank, int world, long long cap, bool create)
    : name_(name), rank_(rank), world_(world), cap_(cap) {
  if (world < 1 || rank < 0 || rank >= world || cap < 1)
    throw std::runtime_error("ShmComm: bad rank / world / capacity");
  bytes_ = kHeader + (size_t)2 * world * cap * sizeof(float);
  const int flags = create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR;
  const int fd = shm_open(name.c_str(), flags, 0600);
  if (fd < 0) throw std::runtime_error("ShmComm: shm_open(" + name + ") failed");
  if (create && ftruncate(fd, (off_t)bytes_) != 0) {
    close(fd);
    shm_unlink(name.c_str());
    throw std::runtime_error("ShmComm: ftruncate failed");
  }
  void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("ShmComm: mmap failed");
  base_ = static_cast<char*>(p);
  if (create) {
    std::memset(base_, 0, kHeader);
    new (base_) std::atomic<uint64_t>(0);
  }
}

ShmComm::~ShmComm() {
  if (base_) munmap(base_, bytes_);
}

void ShmComm::unlink() { shm_unlink(name_.c_str()); }

float* ShmComm::slot(int bank, int r) const {
  return reinterpret_cast<float*>(base_ + kHeader) + ((size_t)bank * world_ + r) * cap_;
}

int ShmComm::allreduce_sum(float* buf, long long n, double timeout_s) {
  if (n > cap_) return 2;
  const uint64_t k = calls_++;
  const int bank = (int)(k & 1);
  std::memcpy(slot(bank, rank_), buf, (size_t)n * sizeof(float));
  auto* ctr = reinterpret_cast<std::atomic<uint64_t>*>(base_);
  ctr->fetch_add(1, std::memory_order_acq_rel);
  const uint64_t target = (k + 1) * (uint64_t)world_;
  if (ctr->load(std::memory_order_acquire) < target) {
    const auto t0 = std::chrono::steady_clock::now();
    unsigned spins = 0;
    while (ctr->load(std::memory_order_acquire) < target) {
      if (++spins > 2000) {
        sched_yield();
        if ((spins & 1023) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
          return 1;
      }
    }
  }
  // every rank sums the same slots in the same (rank) order: identical bits everywhere
  const float* s0 = slot(bank, 0);
  for (long long i = 0; i < n; ++i) buf[i] = s0[i];
  for (int r = 1; r < world_; ++r) {
    const float* s = slot(bank, r);
    for (long long i = 0; i < n; ++i) buf[i] += s[i];
  }
  return 0;
}

}  // namespace nnmpi
