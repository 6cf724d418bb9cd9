// Thread-local last-error text for the C ABI (vad_last_error()).
#include <string>
#include "common.h"
namespace vad {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
const char* last_error() { return g_err.c_str(); }
KTimer& ktimer() {
  static thread_local KTimer t;
  return t;
}
}  // namespace vad
