// dbuf.h — growable device buffer owned by a solver / tracker object.
#ifndef SG_DBUF_H_
#define SG_DBUF_H_

#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "common.h"

namespace sg {

template <typename T>
struct DBuf {
  T* ptr = nullptr;
  size_t cap = 0;
  size_t size = 0;
  void Resize(size_t n) {
    size = n;
    if (n <= cap) return;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
    SG_HIP_CHECK(hipMalloc(&ptr, std::max<size_t>(n, 1) * sizeof(T)));
    cap = n;
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
