// C-ABI plumbing shared by every entry point: thread-local error message, launch checks.
#include "common.h"

namespace mhada {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(const std::string& msg) {
  set_error(msg);
  return MHADA_ERR_ARG;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return MHADA_ERR_LAUNCH;
  }
  return MHADA_OK;
}

}  // namespace mhada

extern "C" int mhada_abi_version(void) { return 2; }  // 2: mhada_fold_block takes kscale

extern "C" const char* mhada_last_error(void) { return mhada::g_last_error.c_str(); }
