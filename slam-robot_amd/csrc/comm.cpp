// comm.cpp — RCCL (NCCL API on ROCm) wrappers.
#include "comm.h"

#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "common.h"

namespace sg {

static void Check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw Error(SG_ECOMM, std::string(what) + ": " + ncclGetErrorString(r));
}

void Comm::UniqueId(void* id128) {
  ncclUniqueId id;
  Check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::memcpy(id128, &id, sizeof(id));
}

Comm::Comm(const void* id128, int nranks, int rank) : nranks_(nranks), rank_(rank) {
  SG_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, SG_EINVAL, "bad communicator rank/size");
  ncclUniqueId id;
  std::memcpy(&id, id128, sizeof(id));
  ncclComm_t c = nullptr;
  Check(ncclCommInitRank(&c, nranks, id, rank), "ncclCommInitRank");
  comm_ = c;
}

Comm::~Comm() {
  if (comm_) (void)ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void Comm::AllReduceSum(double* buf, size_t n, hipStream_t s) {
  Check(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, static_cast<ncclComm_t>(comm_), s), "ncclAllReduce(sum)");
}

void Comm::AllReduceMax(double* buf, size_t n, hipStream_t s) {
  Check(ncclAllReduce(buf, buf, n, ncclDouble, ncclMax, static_cast<ncclComm_t>(comm_), s), "ncclAllReduce(max)");
}

}  // namespace sg
