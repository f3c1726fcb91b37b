// hamming.hip — all-pairs 256-bit descriptor matching (BASELINE config 4, the brute-force descriptor
// distance of the north star).  distance = popcount(a XOR b) over 4 x u64; per query
// the argmin over the train set (ties -> lowest train index) and the second-smallest distance.
//
// Integer-VALU bound: each thread owns one query (8 dwords in registers) and streams a slice of the train
// set through LDS in 256-descriptor tiles (broadcast reads); v_bcnt_u32_b32 accumulates the popcounts.
// The train set is split into slices across workgroups for parallelism, and a second kernel merges the
// per-slice (best, index, second) triples in slice order, which keeps the lowest-index tie rule exact.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <memory>
#include <vector>

#include "common.h"
#include "dbuf.h"

namespace sg {

namespace {

constexpr int kHamThreads = 256;
constexpr int kHamTile = 256;

struct Best {
  int bd, bi, sd;
};

__global__ __launch_bounds__(kHamThreads) void k_hamming_slices(const uint4* __restrict__ q, int nq,
                                                                const uint4* __restrict__ t, int nt, int slice_len,
                                                                int3* __restrict__ part) {
  __shared__ uint4 tile[2 * kHamTile];
  const int i = blockIdx.x * kHamThreads + threadIdx.x;
  const int s = blockIdx.y;
  const int j0 = s * slice_len, j1 = min(nt, j0 + slice_len);
  uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
  if (i < nq) {
    a0 = q[2 * (size_t)i];
    a1 = q[2 * (size_t)i + 1];
  }
  int bd = 1 << 30, bi = -1, sd = 1 << 30;
  for (int base = j0; base < j1; base += kHamTile) {
    const int cnt = min(kHamTile, j1 - base);
    __syncthreads();
    for (int k = threadIdx.x; k < 2 * cnt; k += kHamThreads) tile[k] = t[2 * (size_t)base + k];
    __syncthreads();
    for (int k = 0; k < cnt; ++k) {
      const uint4 b0 = tile[2 * k], b1 = tile[2 * k + 1];
      const int d = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
          __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
      const bool better = d < bd;
      sd = better ? bd : min(sd, d);
      bi = better ? base + k : bi;
      bd = better ? d : bd;
    }
  }
  if (i < nq) part[(size_t)s * nq + i] = make_int3(bd, bi, sd);
}

__global__ void k_hamming_merge(const int3* __restrict__ part, int nq, int nslice, int nt, int32_t* best_idx,
                                int32_t* best_dist, int32_t* second_dist) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  int bd = 1 << 30, bi = -1, sd = 1 << 30;
  for (int s = 0; s < nslice; ++s) {   // slice order = train index order
    const int3 p = part[(size_t)s * nq + i];
    if (p.x < bd) {
      sd = min(bd, p.z);
      bd = p.x;
      bi = p.y;
    } else {
      sd = min(sd, p.x);
    }
  }
  best_idx[i] = bi;
  best_dist[i] = nt > 0 ? bd : -1;
  second_dist[i] = nt > 1 ? sd : -1;
}

}  // namespace

class HammingMatcher {
 public:
  explicit HammingMatcher(const sg_device_options& d) : dev_(d) {
    int ndev = 0;
    SG_HIP_CHECK(hipGetDeviceCount(&ndev));
    SG_REQUIRE(ndev > 0 && d.device >= 0 && d.device < ndev, SG_ENODEV, "no such HIP device");
    SG_HIP_CHECK(hipSetDevice(d.device));
    SG_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    SG_HIP_CHECK(hipEventCreate(&e0_));
    SG_HIP_CHECK(hipEventCreate(&e1_));
  }
  ~HammingMatcher() {
    (void)hipSetDevice(dev_.device);
    if (e0_) (void)hipEventDestroy(e0_);
    if (e1_) (void)hipEventDestroy(e1_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }

  void Load(const uint64_t* q, int nq, const uint64_t* t, int nt) {
    SG_REQUIRE(nq >= 0 && nt >= 0 && (nq == 0 || q) && (nt == 0 || t), SG_EINVAL, "bad descriptors");
    SG_HIP_CHECK(hipSetDevice(dev_.device));
    nq_ = nq;
    nt_ = nt;
    q_.Upload(std::vector<uint64_t>(q, q + 4 * (size_t)nq), stream_);
    t_.Upload(std::vector<uint64_t>(t, t + 4 * (size_t)nt), stream_);
    nslice_ = std::max(1, std::min(64, nt / kHamTile));
    slice_len_ = std::max(1, (nt + nslice_ - 1) / nslice_);
    part_.Resize((size_t)nslice_ * std::max(nq, 1) * 3);
    bi_.Resize(std::max(nq, 1));
    bd_.Resize(std::max(nq, 1));
    sd_.Resize(std::max(nq, 1));
  }

  void Run(int repeats) {
    SG_REQUIRE(repeats >= 1, SG_EINVAL, "repeats must be >= 1");
    SG_HIP_CHECK(hipSetDevice(dev_.device));
    SG_HIP_CHECK(hipEventRecord(e0_, stream_));
    if (nq_ > 0)
      for (int r = 0; r < repeats; ++r) {
        hipLaunchKernelGGL(k_hamming_slices, dim3((nq_ + kHamThreads - 1) / kHamThreads, nslice_), dim3(kHamThreads),
                           0, stream_, (const uint4*)q_.ptr, nq_, (const uint4*)t_.ptr, nt_, slice_len_,
                           (int3*)part_.ptr);
        hipLaunchKernelGGL(k_hamming_merge, dim3((nq_ + 255) / 256), dim3(256), 0, stream_, (const int3*)part_.ptr,
                           nq_, nslice_, nt_, bi_.ptr, bd_.ptr, sd_.ptr);
      }
    SG_HIP_CHECK(hipEventRecord(e1_, stream_));
    SG_HIP_CHECK(hipGetLastError());
    ran_ = true;
    repeats_ = repeats;
  }

  void Results(int32_t* bi, int32_t* bd, int32_t* sd, double* ms) {
    SG_REQUIRE(ran_, SG_EINVAL, "no matching run");
    SG_HIP_CHECK(hipSetDevice(dev_.device));
    if (nq_ > 0) {
      if (bi) SG_HIP_CHECK(hipMemcpyAsync(bi, bi_.ptr, 4 * (size_t)nq_, hipMemcpyDeviceToHost, stream_));
      if (bd) SG_HIP_CHECK(hipMemcpyAsync(bd, bd_.ptr, 4 * (size_t)nq_, hipMemcpyDeviceToHost, stream_));
      if (sd) SG_HIP_CHECK(hipMemcpyAsync(sd, sd_.ptr, 4 * (size_t)nq_, hipMemcpyDeviceToHost, stream_));
    }
    SG_HIP_CHECK(hipStreamSynchronize(stream_));
    float t = 0.f;
    SG_HIP_CHECK(hipEventElapsedTime(&t, e0_, e1_));
    if (ms) *ms = t / repeats_;
  }

 private:
  sg_device_options dev_;
  hipStream_t stream_ = nullptr;
  hipEvent_t e0_ = nullptr, e1_ = nullptr;
  DBuf<uint64_t> q_, t_;
  DBuf<int32_t> part_, bi_, bd_, sd_;
  int nq_ = 0, nt_ = 0, nslice_ = 1, slice_len_ = 1, repeats_ = 1;
  bool ran_ = false;
};

}  // namespace sg

struct sg_matcher {
  std::unique_ptr<sg::HammingMatcher> m;
};

extern "C" {

int sg_matcher_create(sg_matcher** out, const sg_device_options* dev) {
  SG_CAPI_BEGIN
  SG_REQUIRE(out, SG_EINVAL, "null output handle");
  sg_device_options d;
  sg_device_options_default(&d);
  if (dev) d = *dev;
  auto h = std::make_unique<sg_matcher>();
  h->m.reset(new sg::HammingMatcher(d));
  *out = h.release();
  SG_CAPI_END
}

void sg_matcher_destroy(sg_matcher* m) { delete m; }

int sg_hamming_load(sg_matcher* m, const uint64_t* query, int32_t nq, const uint64_t* train, int32_t nt) {
  SG_CAPI_BEGIN
  SG_REQUIRE(m, SG_EINVAL, "null handle");
  m->m->Load(query, nq, train, nt);
  SG_CAPI_END
}

int sg_hamming_run(sg_matcher* m, int32_t repeats) {
  SG_CAPI_BEGIN
  SG_REQUIRE(m, SG_EINVAL, "null handle");
  m->m->Run(repeats);
  SG_CAPI_END
}

int sg_hamming_results(sg_matcher* m, int32_t* best_idx, int32_t* best_dist, int32_t* second_dist, double* kernel_ms) {
  SG_CAPI_BEGIN
  SG_REQUIRE(m, SG_EINVAL, "null handle");
  m->m->Results(best_idx, best_dist, second_dist, kernel_ms);
  SG_CAPI_END
}

int sg_hamming_match(sg_matcher* m, const uint64_t* query, int32_t nq, const uint64_t* train, int32_t nt,
                     int32_t* best_idx, int32_t* best_dist, int32_t* second_dist) {
  SG_CAPI_BEGIN
  SG_REQUIRE(m && (nq == 0 || (best_idx && best_dist && second_dist)), SG_EINVAL, "null argument");
  m->m->Load(query, nq, train, nt);
  m->m->Run(1);
  m->m->Results(best_idx, best_dist, second_dist, nullptr);
  SG_CAPI_END
}

}  // extern "C"
