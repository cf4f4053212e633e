// Host-side C-ABI plumbing for liblci: error reporting, ABI version and build hash.
#include <stdarg.h>
#include <stdio.h>

#include "lci.h"

#ifndef LCI_BUILD_HASH
#define LCI_BUILD_HASH "unknown"
#endif

namespace lci {
static thread_local char g_err[1024] = {0};
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace lci

extern "C" const char* lci_last_error(void) { return lci::g_err; }
extern "C" int lci_abi_version(void) { return LCI_ABI_VERSION; }
extern "C" const char* lci_build_hash(void) { return LCI_BUILD_HASH; }
