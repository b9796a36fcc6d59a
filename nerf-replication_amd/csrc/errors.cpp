// Error plumbing of the C-ABI: thread-local last-error string, hipError_t -> status.
#include <stdarg.h>
#include "common.h"

namespace nerf {

static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return -1000 - (int)e;
  }
  return 0;
}

}  // namespace nerf

extern "C" {

const char* nerf_last_error(void) { return nerf::g_last_error; }

// bumped whenever an exported signature changes
int nerf_abi_version(void) { return 4; }  // 3: dtype 3 (bf16x3f), nerf_composite_pdf, nerf_mse2_*; 4: nerf_composite_pdf_fragile

}  // extern "C"
