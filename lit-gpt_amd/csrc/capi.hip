// C-ABI plumbing shared by every entry point: thread-local error string, version, device info.
#include <stdio.h>
#include <string.h>

#include "common.h"

static thread_local char g_err[512] = {0};

extern "C" void lga_set_error(const char* msg) {
  strncpy(g_err, msg ? msg : "", sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = 0;
}

extern "C" const char* lga_last_error_string(void) { return g_err; }

extern "C" int lga_version(void) { return 1; }

// builds the device objects of the prefill path's kernels now rather than at their first launch (common.h)
extern "C" int lga_preload_kernels(void) {
  const int bad = lga::preload_gemm_q4f() + lga::preload_attention() + lga::preload_norm_rope() +
                  lga::preload_sample() + lga::preload_gemv() + lga::preload_moe();
  if (bad) {
    lga_set_error("lga_preload_kernels: hipFuncGetAttributes failed");
    return 1;
  }
  return 0;
}

// fills *n_cu and *arch_major/minor for device `dev`; 0 on success
extern "C" int lga_device_info(int dev, int* n_cu, char* arch_name, int arch_len) {
  hipDeviceProp_t p;
  hipError_t e = hipGetDeviceProperties(&p, dev);
  if (e != hipSuccess) {
    lga_set_error(hipGetErrorString(e));
    return (int)e;
  }
  if (n_cu) *n_cu = p.multiProcessorCount;
  if (arch_name && arch_len > 0) {
    strncpy(arch_name, p.gcnArchName, arch_len - 1);
    arch_name[arch_len - 1] = 0;
  }
  return 0;
}
