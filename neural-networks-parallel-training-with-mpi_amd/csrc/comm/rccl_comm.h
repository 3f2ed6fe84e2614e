// Native communication runtime: one RCCL communicator per process/GPU plus a bucketed,
// stream-overlapped gradient synchroniser.
//
// Replaces the reference's pickle-over-MPI star exchange (ref.py:185 comm.gather of the gradient
// list, ref.py:190-197 root averaging, ref.py:199/203 serial send/recv) and the init
// broadcasts (ref.py:87,97) / row scatter (ref.py:108,138):
//   * allreduce  — ncclAllReduce(SUM) per contiguous gradient bucket on a dedicated comm stream,
//                  gated by a "bucket ready" event recorded on the compute stream after that
//                  layer's wgrad, joined back before the optimizer;
//   * broadcast  — initial parameters from rank 0 (ncclBroadcast);
//   * scatterv   — grouped ncclSend/ncclRecv with per-rank counts (uneven splits, fixes D1-D3);
//   * reduce_scatter / allgather — the sharded-optimizer (ZeRO-1) gradient and parameter legs.
// Every call is asynchronous and hipGraph-capturable (no host sync inside).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>
#include <vector>

namespace nnmpi {

class RcclComm {
 public:
  static std::string get_unique_id();
  RcclComm(const std::string& uid, int nranks, int rank, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int rank() const { return rank_; }
  int size() const { return nranks_; }
  ncclComm_t handle() const { return comm_; }

  void allreduce(void* buf, size_t count, int dtype, int op, hipStream_t s);
  void broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s);
  void reduce(void* buf, size_t count, int dtype, int op, int root, hipStream_t s);
  // root sends counts[r] elements starting at displs[r] of sendbuf to rank r (recvbuf on r)
  void scatterv(const void* sendbuf, const std::vector<long long>& counts,
                const std::vector<long long>& displs, void* recvbuf, int dtype, int root,
                hipStream_t s);
  void allgather(const void* sendbuf, void* recvbuf, size_t count, int dtype, hipStream_t s);
  // rank r receives the reduction of elements [r*recvcount, (r+1)*recvcount) of every sendbuf
  // (in place when recvbuf == sendbuf + r*recvcount)
  void reduce_scatter(const void* sendbuf, void* recvbuf, size_t recvcount, int dtype, int op,
                      hipStream_t s);
  // grouped in-place ncclBroadcast of pieces [base + offsets[i], + counts[i]) from roots[i]
  // (the sharded optimizer's fp32 refresh of the regions the kernels read from the master)
  void broadcast_pieces(void* base, const std::vector<long long>& offsets,
                        const std::vector<long long>& counts, const std::vector<int>& roots,
                        int dtype, hipStream_t s);
  // bf16 sum all-reduce with ONE rounding: [buf, buf + count) is cut into 64-aligned owner
  // slices; a grouped send/recv all-to-all delivers every rank's copy of slice r to rank r
  // (scratch: at least acc32_scratch_elems(count) bf16), the owner adds the P copies in fp32 in
  // rank order and rounds once, and a grouped all-gather returns the slices.  The same wire bytes
  // as a ring all-reduce in bf16 -- which rounds the partial sum at every hop, so its error grows
  // with P -- and every transfer takes the direct xGMI link between the two GPUs.
  void allreduce_bf16_acc32(void* buf, void* scratch, size_t count, hipStream_t s);
  size_t acc32_slice(size_t count) const;
  // fp32 all-reduce with a fixed per-element summation order (rank 0 + 1 + ... + P-1, on the
  // element's owner): the same all-to-all / owner sum / all-gather as the bf16 form, no rounding
  // step.  Bitwise independent of how a gradient is cut into buckets.  scratch: at least
  // acc32_scratch_elems(count) floats.
  void allreduce_f32_ordered(void* buf, void* scratch, size_t count, hipStream_t s);
  size_t acc32_scratch_elems(size_t count) const { return acc32_slice(count) * nranks_; }
  // Returns the RCCL async error code (0 = ok); aborts the communicator on error if asked.
  int poll_error(bool abort_on_error);
  void abort();

 private:
  ncclComm_t comm_ = nullptr;
  int nranks_ = 0, rank_ = 0, device_ = 0;
  bool aborted_ = false;
};

// Bucketed gradient all-reduce overlapped with backward on a side stream.
class GradSync {
 public:
  GradSync(RcclComm* comm, int n_buckets, int priority);
  ~GradSync();
  // compute stream -> (event) -> comm stream: all-reduce [ptr, ptr+count) of bucket b.
  void bucket_ready(int b, void* ptr, size_t count, int dtype, hipStream_t compute);
  // bf16 buckets use RcclComm::allreduce_bf16_acc32 with this scratch (nullptr: ncclAllReduce)
  void set_acc32_scratch(void* scratch) { acc32_scratch_ = scratch; }
  // fp32 buckets use RcclComm::allreduce_f32_ordered with this scratch (nullptr: ncclAllReduce)
  void set_f32_scratch(void* scratch) { f32_scratch_ = scratch; }
  // diagnostic: after each bucket's collective, hold `blocks` CUs on the comm stream for the
  // time the bucket would take at `gbps` bus bandwidth (kernels.h cu_hold; 0 blocks: off)
  void set_standin(int blocks, double gbps) { standin_blocks_ = blocks; standin_gbps_ = gbps; }
  // comm stream -> (event) -> compute stream: everything launched so far is complete.
  void join(hipStream_t compute);
  hipStream_t comm_stream() const { return comm_stream_; }

 private:
  RcclComm* comm_;
  void* acc32_scratch_ = nullptr;
  void* f32_scratch_ = nullptr;
  int standin_blocks_ = 0;
  double standin_gbps_ = 0.0;
  hipStream_t comm_stream_ = nullptr;
  std::vector<hipEvent_t> ready_;
  hipEvent_t done_ = nullptr;
};

// Minimal native stream-capture graph runner (hipStreamBeginCapture / hipGraphInstantiate).
class GraphRunner {
 public:
  GraphRunner() = default;
  ~GraphRunner();
  // mode: 0 global, 1 thread-local (default), 2 relaxed (hipStreamCaptureMode*)
  void begin(hipStream_t s, int mode = 1);
  void end();
  void launch(hipStream_t s);
  // abandon an in-progress capture (after a throw) and drop any partial graph
  void cancel();
  bool ready() const { return exec_ != nullptr; }
  size_t num_nodes() const;

 private:
  hipStream_t cap_ = nullptr;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
};

}  // namespace nnmpi
