// mx_runtime.hip -- process-level state, error mapping and device probes of
// libmx_kernels.so.  The buffer probe replaces the accelerator hooks the
// reference uses to route a buffer (opal/datatype/opal_datatype_cuda.c:70-90
// opal_cuda_check_bufs, opal/mca/common/cuda/common_cuda.c:1736-1857).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "mx_internal.h"
#include "mx_mem.hpp"

namespace mx {
int g_num_cus = 256;
int g_device = -1;

// Launches whose streams together touch at least this many bytes use
// non-temporal 16-byte accesses (mx_mem.hpp); MX_NT_MIN_BYTES overrides
// (0 = always, -1 = never).  384 MiB: above the 256 MiB Infinity Cache a
// re-used working set no longer stays on-die (measured crossover between
// 2 x 128 MiB, where default accesses win 7.36 vs 6.42 TB/s, and 2 x 512 MiB,
// where nt wins 6.32 vs 5.86 TB/s; profiles/r01/nt_policy_sizes.txt).
static long long nt_min_bytes() {
  static long long v = [] {
    const char *e = getenv("MX_NT_MIN_BYTES");
    return e ? atoll(e) : (384LL << 20);
  }();
  return v;
}
bool mx_nt_for(size_t bytes) {
  const long long t = nt_min_bytes();
  return t >= 0 && (long long)bytes >= t;
}
}  // namespace mx

using namespace mx;

int mx_hip_rc(hipError_t e) { return e == hipSuccess ? MX_SUCCESS : MX_ERR_HIP; }

int mx_check_launch(void) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    fprintf(stderr, "mx_kernels: launch failed: %s\n", hipGetErrorString(e));
    return MX_ERR_HIP;
  }
  return MX_SUCCESS;
}

extern "C" int mx_init(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MX_ERR_NOT_INIT;
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess) return MX_ERR_HIP;
  }
  if (device >= n) return MX_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return MX_ERR_HIP;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return MX_ERR_HIP;
  g_num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  g_device = device;
  return MX_SUCCESS;
}

int mx_ensure_init(void) {
  if (g_device >= 0) {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur == g_device) return MX_SUCCESS;
  }
  return mx_init(-1);
}

extern "C" int mx_finalize(void) {
  g_device = -1;
  return MX_SUCCESS;
}

extern "C" int mx_is_device_ptr(const void *p) {
  if (!p) return 0;
  hipPointerAttribute_t attr;
  memset(&attr, 0, sizeof attr);
  hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();  // unregistered host memory: clear the sticky error
    return 0;
  }
  return (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) ? 1 : 0;
}

extern "C" int mx_stream_sync(void *stream) {
  return mx_hip_rc(hipStreamSynchronize((hipStream_t)stream));
}

extern "C" int mx_copy(void *dst, const void *src, size_t bytes, void *stream) {
  if (bytes == 0) return MX_SUCCESS;
  if (!dst || !src) return MX_ERR_ARG;
  int rc = mx_ensure_init();
  if (rc) return rc;
  return copy_async(dst, src, bytes, (hipStream_t)stream);
}

extern "C" const char *mx_strerror(int rc) {
  switch (rc) {
    case MX_SUCCESS: return "success";
    case MX_ERR_ARG: return "invalid argument";
    case MX_ERR_UNSUPPORTED: return "operation not defined for this datatype";
    case MX_ERR_HIP: return "HIP runtime error";
    case MX_ERR_NOMEM: return "out of memory";
    case MX_ERR_TIMEOUT: return "timed out waiting for a peer";
    case MX_ERR_RCCL: return "RCCL error";
    case MX_ERR_NOT_INIT: return "not initialised / no device";
    case MX_ERR_STATE: return "invalid state";
    case MX_ERR_TRUNCATE: return "message truncated (longer than the receive buffer)";
    case MX_ERR_TAG: return "envelope tag differs from the receive's (channels match in order)";
    default: return "unknown error";
  }
}

extern "C" const char *mx_version(void) { return "mx_kernels gfx950 abi 1"; }
