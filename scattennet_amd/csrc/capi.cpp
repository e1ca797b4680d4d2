// C ABI glue for libscatten_hip.so: error reporting and version (kernels live in *.hip).
#include <string.h>

#include "../../include/scatten.h"

namespace {
thread_local char g_err[256] = "";
}

extern "C" void sca_set_error(const char* msg) {
  strncpy(g_err, msg, sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = 0;
}

extern "C" const char* sca_last_error(void) { return g_err; }

extern "C" int sca_version(void) { return 1; }

#ifndef SCA_BUILD_DIGEST
#error "build through the Makefile: it passes SCA_BUILD_DIGEST (sha256 of the library sources)"
#endif
// sha256 (first 16 hex digits) of the sources this library was compiled from (Makefile)
extern "C" const char* sca_build_digest(void) { return SCA_BUILD_DIGEST; }

namespace {
const unsigned long long* g_drop_offset = nullptr;
}

extern "C" int sca_dropout_offset(const unsigned long long* counter) {
  g_drop_offset = counter;
  return SCA_OK;
}

// read by the launchers (host side) of every dropout-capable kernel
extern "C" const unsigned long long* sca_drop_offset_ptr(void) { return g_drop_offset; }
