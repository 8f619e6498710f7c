// Error plumbing and small utilities of the C-ABI (beast_hip.h).
#include <cstring>

#include "common.h"

namespace beast {

static thread_local char g_err[512] = "";
int64_t g_merge_lds_min = 4096;   // measured at K5: 65,536 -> 4,096 cut the merge loop 62.6 -> 58.8 ms
int g_bpe_encode_mode = 0;
int g_bpe_dedup_key_bits = 64;

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int hip_fail(hipError_t e, const char* what) {
  set_error("%s: %s (%d)", what, hipGetErrorString(e), static_cast<int>(e));
  return BEAST_E_HIP;
}

}  // namespace beast

extern "C" int beast_abi_version(void) { return BEAST_ABI_VERSION; }

extern "C" const char* beast_last_error(void) { return beast::g_err; }
