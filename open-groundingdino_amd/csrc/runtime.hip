// Runtime entry points of the C-ABI: error reporting and build/device info.
// gd_runtime_info replaces the reference's get_cuda_version
// (models/GroundingDINO/csrc/vision.cpp:11-51, csrc/cuda_version.cu).
#include <cstring>
#include <string>

#include "gd_common.h"

namespace gd {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

}  // namespace gd

extern "C" const char* gd_last_error(void) { return gd::g_last_error.c_str(); }

extern "C" int gd_abi_version(void) { return 1; }

extern "C" const char* gd_runtime_info(void) {
  static thread_local std::string info;
  int rt = 0;
  if (hipRuntimeGetVersion(&rt) != hipSuccess) rt = -1;
  std::string arch = "none";
  int dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
    arch = prop.gcnArchName;
  info = "hip=" + std::to_string(rt) + ";arch=" + arch + ";build=" + std::to_string(HIP_VERSION) +
         ";target=gfx950";
  return info.c_str();
}
