// stager.h — batched host-to-device upload of a solver's structure arrays.
//
// A full sg_ba_load uploads some forty index lists and value arrays.  Issued one hipMemcpyAsync each from
// pageable vectors, every copy is staged synchronously by the runtime, which dominated the load of the small
// problems main.cpp solves every frame (SolveFrames(2, 5): tools/e2e_replay.py).  The Stager packs them into
// one pinned, device-mapped host buffer (16-byte aligned pieces) and one kernel launch reads the pieces
// straight from host memory into their device buffers (zero-copy): no copy engine on the load's path.  (A
// hipMemcpyAsync into a device staging buffer went through the SDMA engine, whose copies stalled 13-28 ms in
// about one load in six of the main.cpp replay; HSA_ENABLE_SDMA=0 removed most of those stalls.)
#ifndef SG_STAGER_H_
#define SG_STAGER_H_

#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "common.h"
#include "dbuf.h"

namespace sg {

struct StagePiece {
  unsigned long long dst;   // device address
  unsigned long long off;   // byte offset in the staging buffer (16-aligned)
  unsigned long long bytes;
};

// A load may flush in several batches (the observation arrays early, so their DMA overlaps the host's work-list
// construction, then the lists): each batch occupies its own region of the pinned buffer and of the device
// staging buffer, at the same offsets, and the pinned buffer is only rewritten after Clear() (next load) has
// waited for the last batch's copy.
// One workgroup column per piece (blockIdx.y); 16-byte copies for the aligned body, bytes for the tail.
static __global__ __launch_bounds__(256) void k_stage_scatter(const StagePiece* __restrict__ pieces,
                                                       const unsigned char* __restrict__ stage) {
  const StagePiece pc = pieces[blockIdx.y];
  const unsigned char* src = stage + pc.off;
  unsigned char* dst = reinterpret_cast<unsigned char*>(pc.dst);
  const size_t n16 = pc.bytes / 16;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
  if (blockIdx.x == 0 && threadIdx.x < pc.bytes - 16 * n16) dst[16 * n16 + threadIdx.x] = src[16 * n16 + threadIdx.x];
}

class Stager {
 public:
  ~Stager() {
    WaitCopy();
    if (copied_) (void)hipEventDestroy(copied_);
    if (host_) (void)hipHostFree(host_);
  }

  // Pre-size the pinned buffer (a caller that knows its map's high-water mark): growing it later costs a
  // pinned allocation (milliseconds for tens of MB) on the load's critical path.
  bool ReserveBytes(size_t bytes) {
    if (bytes > cap_) Grow(bytes);
    return false;   // (no device buffer: the scatter reads host memory)
  }
  size_t staged_bytes() const { return last_bytes_; }

  // Resize dst to v.size() and queue v for it (the copy happens in Flush).
  template <typename T>
  void Add(DBuf<T>& dst, const std::vector<T>& v) {
    AddInto(dst, v.size(), v);
  }
  // Resize dst to n >= v.size() elements and queue v for its first v.size() elements.
  template <typename T>
  void AddInto(DBuf<T>& dst, size_t n, const std::vector<T>& v) {
    dst.Resize(n);
    if (v.empty()) return;
    const size_t bytes = v.size() * sizeof(T);
    const size_t off = Reserve(bytes);
    std::memcpy(host_ + off, v.data(), bytes);
    pieces_.push_back(StagePiece{(unsigned long long)(uintptr_t)dst.ptr, off, bytes});
    max_bytes_ = std::max(max_bytes_, bytes);
  }

  // Drop anything queued (a load that failed part way).  The previous batch's DMA may still read the pinned
  // buffer if that load threw between Flush and its stream synchronisation: wait for it first.
  void Clear() {
    WaitCopy();
    pieces_.clear();
    used_ = 0;
    batch0_ = 0;
    max_bytes_ = 0;
  }

  // One scatter launch on stream s reading this batch's pieces from the mapped pinned buffer.  The batch's
  // region is not rewritten before the next load's Clear() waits for the launch.
  void Flush(hipStream_t s) {
    if (pieces_.empty()) return;
    const size_t tbytes = pieces_.size() * sizeof(StagePiece);
    const size_t tbl_off = Reserve(tbytes);
    std::memcpy(host_ + tbl_off, pieces_.data(), tbytes);
    if (!copied_) SG_HIP_CHECK(hipEventCreateWithFlags(&copied_, hipEventDisableTiming));
    last_bytes_ += used_ - batch0_;
    const unsigned gx = (unsigned)std::min<size_t>(64, std::max<size_t>(1, (max_bytes_ / 16 + 255) / 256));
    hipLaunchKernelGGL(k_stage_scatter, dim3(gx, (unsigned)pieces_.size()), dim3(256), 0, s,
                       reinterpret_cast<const StagePiece*>(hdev_ + tbl_off), hdev_);
    SG_HIP_CHECK(hipGetLastError());
    SG_HIP_CHECK(hipEventRecord(copied_, s));
    pending_ = true;
    pieces_.clear();
    batch0_ = (used_ + 15) & ~(size_t)15;
    used_ = batch0_;
    max_bytes_ = 0;
  }
  void ResetBytes() { last_bytes_ = 0; }

 private:
  void WaitCopy() {
    if (pending_) {
      (void)hipEventSynchronize(copied_);
      pending_ = false;
    }
  }

  size_t Reserve(size_t bytes) {
    if (used_ == 0) WaitCopy();   // first piece of a load: the buffer is about to be rewritten
    const size_t off = (used_ + 15) & ~(size_t)15;
    const size_t need = off + bytes;
    if (need > cap_) Grow(std::max(need, 2 * cap_));   // geometric: a growing map re-pins O(log) times
    used_ = need;
    return off;
  }

  // Keeps what is queued (pieces_ hold offsets, not host pointers).  At least 8 MB, rounded to 1 MB.
  void Grow(size_t want) {
    WaitCopy();
    const size_t ncap = (std::max<size_t>(want, 8u << 20) + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
    unsigned char* nh = nullptr;
    SG_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&nh), ncap, hipHostMallocMapped));
    void* dp = nullptr;
    SG_HIP_CHECK(hipHostGetDevicePointer(&dp, nh, 0));
    if (host_) {
      std::memcpy(nh, host_, used_);
      (void)hipHostFree(host_);
    }
    host_ = nh;
    hdev_ = static_cast<unsigned char*>(dp);
    cap_ = ncap;
  }

  unsigned char* host_ = nullptr;   // pinned, mapped into the device's address space
  unsigned char* hdev_ = nullptr;   // its device-side address
  size_t cap_ = 0, used_ = 0, batch0_ = 0, max_bytes_ = 0, last_bytes_ = 0;
  hipEvent_t copied_ = nullptr;     // the last scatter launch (it reads host_)
  bool pending_ = false;
  std::vector<StagePiece> pieces_;
};

}  // namespace sg

#endif  // SG_STAGER_H_
