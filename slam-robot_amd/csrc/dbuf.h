// dbuf.h — growable device buffer owned by a solver / tracker object.
#ifndef SG_DBUF_H_
#define SG_DBUF_H_

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <vector>

#include "common.h"

namespace sg {

// device allocations made by every DBuf of the process (SG_HOST_TIMING: reported per load)
inline std::atomic<long> g_dbuf_allocs{0};

template <typename T>
struct DBuf {
  T* ptr = nullptr;
  size_t cap = 0;
  size_t size = 0;
  void Resize(size_t n) {
    size = n;
    if (n <= cap) return;
    // grow geometrically: a map that grows by a frame per call (main.cpp's loop) would otherwise pay a
    // hipFree (a device synchronisation) and a hipMalloc on almost every load
    Reserve(cap ? std::max(n, 2 * cap) : n);
  }
  // Capacity for n elements without changing size (pre-sizing from a high-water mark: no reallocation, and
  // so no hipFree / hipMalloc, on a later load's critical path).  Contents are not preserved.
  bool Reserve(size_t ncap) {
    if (ncap <= cap) return false;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
    SG_HIP_CHECK(hipMalloc(&ptr, std::max<size_t>(ncap, 1) * sizeof(T)));
    g_dbuf_allocs.fetch_add(1, std::memory_order_relaxed);
    cap = ncap;
    return true;
  }
  void Upload(const std::vector<T>& v, hipStream_t s) {
    Resize(v.size());
    if (!v.empty()) SG_HIP_CHECK(hipMemcpyAsync(ptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
  }
  void Zero(hipStream_t s) {
    if (size) SG_HIP_CHECK(hipMemsetAsync(ptr, 0, size * sizeof(T), s));
  }
  ~DBuf() {
    if (ptr) (void)hipFree(ptr);
  }
};

}  // namespace sg

#endif  // SG_DBUF_H_
