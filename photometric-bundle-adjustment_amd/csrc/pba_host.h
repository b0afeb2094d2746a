// pba_host.h — host-only helpers shared by every translation unit of the engine library: the thread-local error
// message behind pba_last_error() and the status-returning fail().  No HIP: the host-only sources (pba_map.cpp,
// pba_outliers_host.cpp) include only this, so they also build with plain g++ (tests/test_host_sanitizers.py builds
// them with AddressSanitizer + UndefinedBehaviorSanitizer).
#pragma once

#include <string>

namespace pba {
namespace detail {

extern thread_local std::string g_last_error;

inline int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

}  // namespace detail
}  // namespace pba
