// comm.hip — the landmark-shard communicators (comm.h): RCCL for the product path, and the in-process
// group that runs the sharded device chain on one GPU (tests).
#include "comm.h"

#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <string>

#include "common.h"

namespace sg {

static void Check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw Error(SG_ECOMM, std::string(what) + ": " + ncclGetErrorString(r));
}

void RcclComm::UniqueId(void* id128) {
  ncclUniqueId id;
  Check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::memcpy(id128, &id, sizeof(id));
}

RcclComm::RcclComm(const void* id128, int nranks, int rank) {
  SG_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, SG_EINVAL, "bad communicator rank/size");
  nranks_ = nranks;
  rank_ = rank;
  ncclUniqueId id;
  std::memcpy(&id, id128, sizeof(id));
  ncclComm_t c = nullptr;
  Check(ncclCommInitRank(&c, nranks, id, rank), "ncclCommInitRank");
  comm_ = c;
}

RcclComm::~RcclComm() {
  if (comm_) (void)ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void RcclComm::AllReduceSum(double* buf, size_t n, hipStream_t s) {
  Check(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, static_cast<ncclComm_t>(comm_), s), "ncclAllReduce(sum)");
}

void RcclComm::AllReduceMax(double* buf, size_t n, hipStream_t s) {
  Check(ncclAllReduce(buf, buf, n, ncclDouble, ncclMax, static_cast<ncclComm_t>(comm_), s), "ncclAllReduce(max)");
}

// ------------------------------------------------------------------------------------------------
// Host-callback transport

HostComm::HostComm(int nranks, int rank, HostAllReduceFn fn, void* user) : fn_(fn), user_(user) {
  SG_REQUIRE(fn && nranks >= 1 && rank >= 0 && rank < nranks, SG_EINVAL, "bad host communicator");
  nranks_ = nranks;
  rank_ = rank;
}

HostComm::~HostComm() {
  if (host_) (void)hipHostFree(host_);
}

void HostComm::Reduce(double* buf, size_t n, hipStream_t s, int op) {
  if (n == 0) return;
  if (n > cap_) {
    SG_HIP_CHECK(hipStreamSynchronize(s));
    if (host_) (void)hipHostFree(host_);
    host_ = nullptr;
    cap_ = 0;
    SG_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&host_), n * sizeof(double), hipHostMallocDefault));
    cap_ = n;
  }
  SG_HIP_CHECK(hipMemcpyAsync(host_, buf, n * sizeof(double), hipMemcpyDeviceToHost, s));
  SG_HIP_CHECK(hipStreamSynchronize(s));
  const int rc = fn_(host_, (long long)n, op, user_);
  if (rc != 0) throw Error(SG_ECOMM, "host communicator callback failed (" + std::to_string(rc) + ")");
  SG_HIP_CHECK(hipMemcpyAsync(buf, host_, n * sizeof(double), hipMemcpyHostToDevice, s));
  SG_HIP_CHECK(hipStreamSynchronize(s));   // host_ is reused by the next all-reduce
}

// ------------------------------------------------------------------------------------------------
// In-process group

void LocalGroup::Barrier() {
  std::unique_lock<std::mutex> lk(mu);
  const long gen = generation;
  if (++arrived == nranks) {
    arrived = 0;
    ++generation;
    cv.notify_all();
    return;
  }
  if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return generation != gen; })) {
    --arrived;
    throw Error(SG_ECOMM, "in-process communicator: a rank did not reach the all-reduce (120 s)");
  }
}

LocalComm::LocalComm(std::shared_ptr<LocalGroup> g, int rank) : g_(std::move(g)) {
  SG_REQUIRE(g_ && g_->nranks >= 1 && g_->nranks <= LocalGroup::kMaxRanks && rank >= 0 && rank < g_->nranks,
             SG_EINVAL, "bad in-process communicator rank/size");
  nranks_ = g_->nranks;
  rank_ = rank;
}

LocalComm::~LocalComm() {
  if (tmp_) (void)hipFree(tmp_);
}

struct RankPtrs {
  const double* p[LocalGroup::kMaxRanks];
};

// out[i] = sum (or max) over ranks of their buffer's element i, in rank order: every rank computes the same bits.
__global__ void k_local_reduce(RankPtrs in, int nranks, size_t n, int op, double* out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    double v = in.p[0][i];
    for (int r = 1; r < nranks; ++r) v = op == 0 ? v + in.p[r][i] : fmax(v, in.p[r][i]);
    out[i] = v;
  }
}

void LocalComm::Reduce(double* buf, size_t n, hipStream_t s, int op) {
  if (nranks_ == 1 || n == 0) return;
  if (n > cap_) {
    if (tmp_) (void)hipFree(tmp_);
    tmp_ = nullptr;
    SG_HIP_CHECK(hipMalloc(&tmp_, n * sizeof(double)));
    cap_ = n;
  }
  SG_HIP_CHECK(hipStreamSynchronize(s));   // this rank's contribution is complete
  {
    std::lock_guard<std::mutex> lk(g_->mu);
    g_->bufs[rank_] = buf;
    g_->lens[rank_] = n;
  }
  g_->Barrier();   // every contribution complete and registered
  RankPtrs rp{};
  for (int r = 0; r < nranks_; ++r) {
    SG_REQUIRE(g_->lens[r] == n, SG_ECOMM, "in-process communicator: ranks disagree on the all-reduce size");
    rp.p[r] = g_->bufs[r];
  }
  const int blocks = (int)std::min<size_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(k_local_reduce, dim3(blocks), dim3(256), 0, s, rp, nranks_, n, op, tmp_);
  SG_HIP_CHECK(hipGetLastError());
  SG_HIP_CHECK(hipStreamSynchronize(s));
  g_->Barrier();   // every rank has read every input
  SG_HIP_CHECK(hipMemcpyAsync(buf, tmp_, n * sizeof(double), hipMemcpyDeviceToDevice, s));
  SG_HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace sg
