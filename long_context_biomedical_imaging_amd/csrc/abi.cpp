// Host-side C-ABI plumbing for liblci: error reporting and version query.
#include <stdarg.h>
#include <stdio.h>

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
extern "C" int lci_abi_version(void) { return 2; }
