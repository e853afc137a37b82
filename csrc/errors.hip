// Launch-error reporting (csrc/common.hpp ATE_LAUNCH / ATE_CHECK_LAUNCH) and the debug
// build's kernel resource check at library load.
#include "common.hpp"

#include <string.h>

using namespace ate;

static int copy_msg(const LaunchError& e, char* buf, int len) {
  if (buf && len > 0) {
    strncpy(buf, e.msg, (size_t)len - 1);
    buf[len - 1] = 0;
  }
  return e.code;
}

// The last failed launch of this thread: its HIP error code (0: none) and message.
ATE_API int ate_last_error(char* buf, int len) { return copy_msg(g_launch_error, buf, len); }

// The last error found pending BEFORE one of our launches (an earlier HIP call's), cleared
// there so that it is not reported as that launch's failure.
ATE_API int ate_last_stale_error(char* buf, int len) { return copy_msg(g_stale_error, buf, len); }

ATE_API int ate_clear_errors() {
  g_launch_error = LaunchError{};
  g_stale_error = LaunchError{};
  return 0;
}

__global__ void debug_noop_kernel(int* out) {
  if (out) out[threadIdx.x] = 0;
}

// A deliberately invalid launch (block of `threads` > 1024 work-items): the runtime refuses it
// before dispatch. tests/test_gpu.py checks that the named error reaches Python.
ATE_API int ate_debug_bad_launch(int threads, void* stream) {
  ATE_LAUNCH(debug_noop_kernel, dim3(1), dim3(threads), 0, (hipStream_t)stream, (int*)nullptr);
  ATE_CHECK_LAUNCH();
  return 0;
}

// Debug build (loaded with ATE_DEBUG=1): every registered kernel's compiled attributes against
// its launch shape -- the block size within the kernel's maximum (launch bounds, registers),
// static + dynamic LDS within the device's per-block limit. Writes one line per kernel to buf
// and returns the number of kernels that cannot launch as registered (-1: no device).
ATE_API int ate_check_kernel_resources(char* buf, int len) {
  int dev = 0, lds_max = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess)
    return -1;
  int bad = 0, off = 0;
  if (buf && len > 0) buf[0] = 0;
  for (const KernelShape& k : kernel_shapes()) {
    hipFuncAttributes a{};
    const hipError_t e = hipFuncGetAttributes(&a, k.fn);
    const char* why = "ok";
    if (e != hipSuccess) why = hipGetErrorName(e);
    else if (a.maxThreadsPerBlock < k.threads) why = "FAIL: block larger than the kernel allows";
    else if ((int)a.sharedSizeBytes + k.dyn_lds > lds_max) why = "FAIL: LDS over the per-block limit";
    if (why[0] != 'o') ++bad;
    if (buf && off < len - 1) {
      const int w = snprintf(buf + off, (size_t)(len - off),
                             "%s: threads %d (max %d), LDS %d + %d (max %d), VGPR %d, scratch %d B/lane: %s\n",
                             k.name, k.threads, a.maxThreadsPerBlock, (int)a.sharedSizeBytes,
                             k.dyn_lds, lds_max, a.numRegs, (int)a.localSizeBytes, why);
      off += w > 0 ? w : 0;
    }
  }
  (void)hipGetLastError();   // the attribute queries leave nothing pending
  return bad;
}
