// comm.h — RCCL communicator for landmark-sharded bundle adjustment (one process per GPU, xGMI).
//
// The only collective on the hot path: per LM iteration the camera-side normal
// equations (camera blocks + gradient + cost), the reduced camera system S and its right-hand side, and
// the step scalars are summed over the landmark shards with ncclAllReduce; every rank then factors the
// identical S and takes the identical accept/reject decision.
#ifndef SG_COMM_H_
#define SG_COMM_H_

#include <hip/hip_runtime.h>

#include <cstddef>

namespace sg {

class Comm {
 public:
  Comm(const void* id128, int nranks, int rank);
  ~Comm();
  static void UniqueId(void* id128);
  void AllReduceSum(double* buf, size_t n, hipStream_t s);
  void AllReduceMax(double* buf, size_t n, hipStream_t s);
  int nranks() const { return nranks_; }
  int rank() const { return rank_; }

 private:
  void* comm_ = nullptr;  // ncclComm_t
  int nranks_ = 1, rank_ = 0;
};

}  // namespace sg

#endif  // SG_COMM_H_
