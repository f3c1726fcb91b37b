// common.h — error plumbing shared by the libslamgpu.so translation units.
#ifndef SG_COMMON_H_
#define SG_COMMON_H_

#include <cstdio>
#include <stdexcept>
#include <string>

#include "slamgpu.h"

namespace sg {

// Thread-local message behind sg_last_error().
void SetError(const std::string& msg);

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

}  // namespace sg

#define SG_HIP_CHECK(expr)                                                                       \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess)                                                                        \
      throw ::sg::Error(SG_EDEVICE, std::string(#expr " -> ") + hipGetErrorString(e_) + " at " + \
                                         __FILE__ + ":" + std::to_string(__LINE__));             \
  } while (0)

#define SG_REQUIRE(cond, code, msg)                        \
  do {                                                     \
    if (!(cond)) throw ::sg::Error((code), (msg));         \
  } while (0)

// Wrap a C-ABI body: exceptions become error codes + sg_last_error().
#define SG_CAPI_BEGIN try {
#define SG_CAPI_END                                              \
  }                                                              \
  catch (const ::sg::Error& e) {                                 \
    ::sg::SetError(e.what());                                    \
    return e.code;                                               \
  }                                                              \
  catch (const std::bad_alloc&) {                                \
    ::sg::SetError("host allocation failed");                    \
    return SG_ENOMEM;                                            \
  }                                                              \
  catch (const std::exception& e) {                              \
    ::sg::SetError(e.what());                                    \
    return SG_EINVAL;                                            \
  }                                                              \
  return SG_OK;

#endif  // SG_COMMON_H_
