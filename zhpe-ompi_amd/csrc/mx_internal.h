// mx_internal.h -- shared state of libmx_kernels.so (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/mx_kernels.h"

namespace mx {
extern int g_num_cus;      // CUs of the current device (256 on MI355X)
extern int g_device;       // device selected by mx_init
// 16-byte streaming device copy (mx_coll.hip), falls back to the runtime copy
int copy_async(void *dst, const void *src, size_t bytes, hipStream_t s);
}  // namespace mx

// Lazily performs mx_init(current device) if the caller did not.
int mx_ensure_init(void);
// Converts hipGetLastError() after a launch into an MX code.
int mx_check_launch(void);
int mx_hip_rc(hipError_t e);
