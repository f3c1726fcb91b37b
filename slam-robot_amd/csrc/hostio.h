// hostio.h — the per-call host <-> device transfers of the Slam facade's map passes (ReprojectMap, Clean,
// ApplyEpipolarConstraint, Normalize) without a copy engine and without the runtime's blocking wait.
//
// Uploads are packed into one pinned, device-mapped buffer and scattered by one kernel (stager.h); downloads are
// gathered by one kernel into a second mapped buffer, the host spins on an event (WaitEvent), then copies the
// pieces out.  Round 4's main.cpp replay (tools/e2e_replay.py) still saw a load in about fifty start 17-28 ms
// late; every BA load was already copy-engine free, but the map passes between the solves were not (about seventy
// pageable hipMemcpyAsync per frame through the SDMA engine, a second HIP stream, and hipStreamSynchronize).
#ifndef SG_HOSTIO_H_
#define SG_HOSTIO_H_

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

#include "common.h"
#include "dbuf.h"
#include "hostmirror.h"
#include "stager.h"

namespace sg {

// Wait for a recorded event by polling it (hipEventSynchronize's blocking wait returned 13-28 ms late in a few
// percent of the replay's calls, profiles/r3_v8_*), falling back to the blocking wait after `spin_ms`; `yield`
// between polls when other host threads share the cores (landmark shards).
inline void WaitEvent(hipEvent_t ev, double spin_ms = 200.0, bool yield = false) {
  const auto t0 = std::chrono::steady_clock::now();
  while (true) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) SG_HIP_CHECK(e);
    if (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() > spin_ms) break;
    if (yield) std::this_thread::yield();
  }
  SG_HIP_CHECK(hipEventSynchronize(ev));
}

// One workgroup column per piece (blockIdx.y): device bytes at pc.dst -> the mapped buffer at pc.off.  16-byte
// copies when both ends are 16-aligned, 8-byte words when 8-aligned, bytes otherwise.
static __global__ __launch_bounds__(256) void k_stage_gather(const StagePiece* __restrict__ pieces,
                                                      unsigned char* __restrict__ stage) {
  const StagePiece pc = pieces[blockIdx.y];
  const unsigned char* src = reinterpret_cast<const unsigned char*>(pc.dst);
  unsigned char* dst = stage + pc.off;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (size_t)gridDim.x * blockDim.x;
  const unsigned long long a = pc.dst | (unsigned long long)(uintptr_t)dst;
  if ((a & 15) == 0) {
    const size_t n16 = pc.bytes / 16;
    for (size_t i = t; i < n16; i += nt) reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    for (size_t i = 16 * n16 + t; i < pc.bytes; i += nt) dst[i] = src[i];
  } else if ((a & 7) == 0) {
    const size_t n8 = pc.bytes / 8;
    for (size_t i = t; i < n8; i += nt)
      reinterpret_cast<unsigned long long*>(dst)[i] = reinterpret_cast<const unsigned long long*>(src)[i];
    for (size_t i = 8 * n8 + t; i < pc.bytes; i += nt) dst[i] = src[i];
  } else {
    for (size_t i = t; i < pc.bytes; i += nt) dst[i] = src[i];
  }
}

class HostIo {
 public:
  HostIo() : up_(new Stager()) {}
  ~HostIo() {
    if (ev_) (void)hipEventDestroy(ev_);
  }

  // A new call: waits for the previous call's upload (its pinned region is rewritten) and drops queued pieces.
  void Begin() {
    up_->Clear();
    down_.clear();
    down_bytes_ = 0;
  }
  // dst resized to max(n, 1) elements; the first n filled from host memory src in Flush.
  template <typename T>
  void Up(DBuf<T>& dst, const T* src, size_t n) {
    up_->AddInto(dst, std::max<size_t>(n, 1), n ? std::vector<T>(src, src + n) : std::vector<T>{});
  }
  template <typename T>
  void Up(DBuf<T>& dst, const std::vector<T>& v) {
    up_->AddInto(dst, std::max<size_t>(v.size(), 1), v);
  }
  // dst resized to max(n, 1) elements, all zero.
  template <typename T>
  void UpZero(DBuf<T>& dst, size_t n) {
    up_->AddInto(dst, std::max<size_t>(n, 1), std::vector<T>(std::max<size_t>(n, 1), T{}));
  }
  void FlushUp(hipStream_t s) { up_->Flush(s); }

  // Queue `bytes` of device memory at src for the host array dst (copied out by FinishDown).
  void Down(void* dst, const void* src, size_t bytes) {
    if (!bytes) return;
    const size_t off = (down_bytes_ + 15) & ~(size_t)15;
    down_.push_back(Piece{dst, StagePiece{(unsigned long long)(uintptr_t)src, off, bytes}});
    down_bytes_ = off + bytes;
  }
  // Everything queued on s so far, then the gather, completes; the queued host arrays are filled.
  void FinishDown(hipStream_t s) {
    const size_t tbl = (down_bytes_ + 15) & ~(size_t)15;
    const size_t need = tbl + down_.size() * sizeof(StagePiece);
    mirror_.Reserve(std::max<size_t>(need, 4096));
    size_t maxb = 0;
    for (size_t i = 0; i < down_.size(); ++i) {
      std::memcpy(mirror_.h + tbl + i * sizeof(StagePiece), &down_[i].pc, sizeof(StagePiece));
      maxb = std::max<size_t>(maxb, down_[i].pc.bytes);
    }
    if (!down_.empty()) {
      const unsigned gx = (unsigned)std::min<size_t>(64, std::max<size_t>(1, (maxb / 16 + 255) / 256));
      hipLaunchKernelGGL(k_stage_gather, dim3(gx, (unsigned)down_.size()), dim3(256), 0, s,
                         reinterpret_cast<const StagePiece*>(mirror_.d + tbl), mirror_.d);
      SG_HIP_CHECK(hipGetLastError());
    }
    Wait(s);
    for (const Piece& p : down_) std::memcpy(p.host, mirror_.h + p.pc.off, p.pc.bytes);
    down_.clear();
    down_bytes_ = 0;
  }
  // Everything queued on s so far completes (event poll).
  void Wait(hipStream_t s) {
    if (!ev_) SG_HIP_CHECK(hipEventCreateWithFlags(&ev_, hipEventDisableTiming));
    SG_HIP_CHECK(hipEventRecord(ev_, s));
    WaitEvent(ev_);
  }

 private:
  struct Piece {
    void* host;
    StagePiece pc;   // dst = the device source address
  };
  std::unique_ptr<Stager> up_;
  HostMirror mirror_;
  std::vector<Piece> down_;
  size_t down_bytes_ = 0;
  hipEvent_t ev_ = nullptr;
};

}  // namespace sg

#endif  // SG_HOSTIO_H_
