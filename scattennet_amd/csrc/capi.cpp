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
