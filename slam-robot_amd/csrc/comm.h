// comm.h — the landmark-shard communicator of the bundle adjuster (one rank per GPU, RCCL over xGMI).
//
// The only collective on the hot path: per LM iteration the camera-side normal
// equations (camera blocks + gradient + cost), the reduced camera system S and its right-hand side, and
// the step scalars are summed over the landmark shards; every rank then factors the identical S and takes
// the identical accept/reject decision.
//
// Two implementations of one interface:
//   RcclComm   ncclAllReduce on the solver's stream (the product path, one process per GPU);
//   LocalComm  an in-process group of ranks on one device, driven by one host thread per rank: each
//              all-reduce synchronises the rank's stream, meets the other ranks at a host barrier and sums
//              every rank's buffer in rank order with a device kernel.  It exists so that the sharded
//              device chain (envelope union, rank-0 assembly, packed S exchange, k_decide) runs on a
//              one-GPU box; the solver's compute path is the same for both.
#ifndef SG_COMM_H_
#define SG_COMM_H_

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstddef>
#include <memory>
#include <mutex>
#include <vector>

namespace sg {

class Comm {
 public:
  virtual ~Comm() = default;
  virtual void AllReduceSum(double* buf, size_t n, hipStream_t s) = 0;
  virtual void AllReduceMax(double* buf, size_t n, hipStream_t s) = 0;
  int nranks() const { return nranks_; }
  int rank() const { return rank_; }

 protected:
  int nranks_ = 1, rank_ = 0;
};

class RcclComm : public Comm {
 public:
  RcclComm(const void* id128, int nranks, int rank);
  ~RcclComm() override;
  static void UniqueId(void* id128);
  void AllReduceSum(double* buf, size_t n, hipStream_t s) override;
  void AllReduceMax(double* buf, size_t n, hipStream_t s) override;

 private:
  void* comm_ = nullptr;  // ncclComm_t
};

// A host transport behind a callback (sg_ba_comm_init_host): every all-reduce copies the device buffer to
// pinned host memory, calls fn(buf, n, op, user) (op 0 sum, 1 max; nonzero return = failure) and copies the
// result back, in the solver's stream order.  The same call sequence as RcclComm, so a multi-process run over
// any host collective (gloo in tests/test_multirank_gloo_gpu.py, MPI) exercises the solver's exchange path
// with one process per rank on a one-GPU box.
typedef int (*HostAllReduceFn)(double* buf, long long n, int op, void* user);
class HostComm : public Comm {
 public:
  HostComm(int nranks, int rank, HostAllReduceFn fn, void* user);
  ~HostComm() override;
  void AllReduceSum(double* buf, size_t n, hipStream_t s) override { Reduce(buf, n, s, 0); }
  void AllReduceMax(double* buf, size_t n, hipStream_t s) override { Reduce(buf, n, s, 1); }

 private:
  void Reduce(double* buf, size_t n, hipStream_t s, int op);
  HostAllReduceFn fn_;
  void* user_;
  double* host_ = nullptr;
  size_t cap_ = 0;
};

// Shared state of an in-process group (sg_comm_group in the C-ABI).
struct LocalGroup {
  static constexpr int kMaxRanks = 8;
  explicit LocalGroup(int n) : nranks(n), bufs(n, nullptr), lens(n, 0) {}
  void Barrier();   // throws SG_ECOMM after a timeout (a rank that failed never arrives)
  int nranks;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  long generation = 0;
  std::vector<double*> bufs;
  std::vector<size_t> lens;
};

class LocalComm : public Comm {
 public:
  LocalComm(std::shared_ptr<LocalGroup> g, int rank);
  ~LocalComm() override;
  void AllReduceSum(double* buf, size_t n, hipStream_t s) override { Reduce(buf, n, s, 0); }
  void AllReduceMax(double* buf, size_t n, hipStream_t s) override { Reduce(buf, n, s, 1); }

 private:
  void Reduce(double* buf, size_t n, hipStream_t s, int op);
  std::shared_ptr<LocalGroup> g_;
  double* tmp_ = nullptr;
  size_t cap_ = 0;
};

}  // namespace sg

#endif  // SG_COMM_H_
