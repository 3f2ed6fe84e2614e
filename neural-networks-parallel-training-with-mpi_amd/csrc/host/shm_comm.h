// Intra-node shared-memory all-reduce for CPU ranks (see shm_comm.cpp).
#pragma once
#include <cstdint>
#include <string>

namespace nnmpi {

class ShmComm {
 public:
  // create = true on exactly one rank, before the others attach (the caller orders it with a
  // barrier of its own process group); cap = the largest vector (elements) a call reduces
  ShmComm(const std::string& name, int rank, int world, long long cap, bool create);
  ~ShmComm();
  ShmComm(const ShmComm&) = delete;
  ShmComm& operator=(const ShmComm&) = delete;
  // remove the name (once every rank has attached: the mapping lives on until the last unmap)
  void unlink();
  // in-place fp32 sum over the ranks; 0 ok, 1 timeout (a peer stalled), 2 n > capacity
  int allreduce_sum(float* buf, long long n, double timeout_s);
  int rank() const { return rank_; }
  int world() const { return world_; }

 private:
  float* slot(int bank, int r) const;
  std::string name_;
  int rank_, world_;
  long long cap_;
  size_t bytes_ = 0;
  char* base_ = nullptr;
  uint64_t calls_ = 0;
};

}  // namespace nnmpi
