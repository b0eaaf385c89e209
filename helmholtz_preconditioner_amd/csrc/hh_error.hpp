// Error plumbing shared by the host-side translation units: internal C++ exceptions carry a
// negative hh_err code; the C ABI entry points catch them and return the code, with the
// message available from hh_last_error().
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/helmholtz_amd.h"

namespace hh {

extern thread_local std::string g_err;

struct Error {
  int code;
};

[[noreturn]] inline void fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  throw Error{code};
}

}  // namespace hh

#define HIPC(expr)                                                                        \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      ::hh::fail(HH_ERR_HIP, "%s:%d %s -> %s", __FILE__, __LINE__, #expr,                 \
                 hipGetErrorString(e_));                                                  \
  } while (0)

#define NCCLC(expr)                                                                       \
  do {                                                                                    \
    ncclResult_t r_ = (expr);                                                             \
    if (r_ != ncclSuccess)                                                                \
      ::hh::fail(HH_ERR_RCCL, "%s:%d %s -> %s (%s)", __FILE__, __LINE__, #expr,           \
                 ncclGetErrorString(r_), ncclGetLastError(nullptr));                      \
  } while (0)

#define REQUIRE(cond, ...)                                                                \
  do {                                                                                    \
    if (!(cond)) ::hh::fail(HH_ERR_INVALID, __VA_ARGS__);                                 \
  } while (0)
