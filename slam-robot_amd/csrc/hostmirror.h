// hostmirror.h — pinned host memory mapped into the device's address space.  Kernels write results into it
// (and read inputs from it) directly, so the solver's small per-call transfers (the LM state polls, the
// solution download) never go through a copy engine: hipMemcpyAsync between pageable host memory and the
// device goes through the SDMA engine and a runtime staging buffer, and those copies stalled for 13-28 ms in
// a few percent of the calls of the main.cpp replay (tools/e2e_replay.py).
#ifndef SG_HOSTMIRROR_H_
#define SG_HOSTMIRROR_H_

#include <hip/hip_runtime.h>

#include "common.h"

namespace sg {

struct HostMirror {
  unsigned char* h = nullptr;   // host address
  unsigned char* d = nullptr;   // device address of the same memory
  size_t cap = 0;
  // At least `bytes` of capacity.  Contents are not preserved; call only while no launch uses the buffer.
  void Reserve(size_t bytes) {
    if (bytes <= cap) return;
    if (h) (void)hipHostFree(h);
    h = d = nullptr;
    cap = 0;
    const size_t nc = (bytes + 4095) & ~(size_t)4095;
    SG_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h), nc, hipHostMallocMapped));
    void* dp = nullptr;
    SG_HIP_CHECK(hipHostGetDevicePointer(&dp, h, 0));
    d = static_cast<unsigned char*>(dp);
    cap = nc;
  }
  ~HostMirror() {
    if (h) (void)hipHostFree(h);
  }
};

}  // namespace sg

#endif  // SG_HOSTMIRROR_H_
