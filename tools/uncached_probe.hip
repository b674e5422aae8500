// uncached_probe -- copy bandwidth from / to the memory kinds the collectives
// use: ordinary device memory (hipMalloc), uncached device memory (the IPC
// staging and gather areas, hipExtMallocWithFlags(hipDeviceMallocUncached))
// and fine-grained device memory (hipDeviceMallocFinegrained).  The gather
// copy of every staged / zero-copy allreduce reads an uncached area.
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/uncached_probe tools/uncached_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__global__ void __launch_bounds__(256) k_copy16(const uint4 *__restrict__ s, uint4 *__restrict__ d, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) d[i] = s[i];
}

__global__ void __launch_bounds__(256) k_copy16_nt(const uint4 *__restrict__ s, uint4 *__restrict__ d, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    uint4 v;
    v.x = __builtin_nontemporal_load(&s[i].x);
    v.y = __builtin_nontemporal_load(&s[i].y);
    v.z = __builtin_nontemporal_load(&s[i].z);
    v.w = __builtin_nontemporal_load(&s[i].w);
    __builtin_nontemporal_store(v.x, &d[i].x);
    __builtin_nontemporal_store(v.y, &d[i].y);
    __builtin_nontemporal_store(v.z, &d[i].z);
    __builtin_nontemporal_store(v.w, &d[i].w);
  }
}

static int bench(const char *name, const void *src, void *dst, size_t bytes, bool nt) {
  const size_t n = bytes / 16;
  const unsigned g = (unsigned)((n + 255) / 256);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 2; w++) {
    if (nt) hipLaunchKernelGGL(k_copy16_nt, dim3(g), dim3(256), 0, 0, (const uint4 *)src, (uint4 *)dst, n);
    else hipLaunchKernelGGL(k_copy16, dim3(g), dim3(256), 0, 0, (const uint4 *)src, (uint4 *)dst, n);
  }
  const int reps = 10;
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; r++) {
    if (nt) hipLaunchKernelGGL(k_copy16_nt, dim3(g), dim3(256), 0, 0, (const uint4 *)src, (uint4 *)dst, n);
    else hipLaunchKernelGGL(k_copy16, dim3(g), dim3(256), 0, 0, (const uint4 *)src, (uint4 *)dst, n);
  }
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double t = ms / reps * 1e-3;
  printf("%-34s %s %7.1f us  %6.2f TB/s (read + write)\n", name, nt ? "nt " : "   ", t * 1e6, 2.0 * bytes / t / 1e12);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 0;
}

int main() {
  const size_t bytes = (size_t)224 << 20;   // the gather copy of a 256 MiB allreduce at n = 8
  CK(hipSetDevice(0));
  void *norm0, *norm1, *unc, *fine;
  CK(hipMalloc(&norm0, bytes));
  CK(hipMalloc(&norm1, bytes));
  CK(hipExtMallocWithFlags(&unc, bytes, hipDeviceMallocUncached));
  CK(hipExtMallocWithFlags(&fine, bytes, hipDeviceMallocFinegrained));
  CK(hipMemset(norm0, 1, bytes));
  CK(hipMemset(unc, 2, bytes));
  CK(hipMemset(fine, 3, bytes));
  CK(hipDeviceSynchronize());
  for (int nt = 0; nt < 2; nt++) {
    if (bench("ordinary -> ordinary", norm0, norm1, bytes, nt)) return 1;
    if (bench("uncached -> ordinary", unc, norm1, bytes, nt)) return 1;
    if (bench("fine-grained -> ordinary", fine, norm1, bytes, nt)) return 1;
    if (bench("ordinary -> uncached", norm0, unc, bytes, nt)) return 1;
    if (bench("ordinary -> fine-grained", norm0, fine, bytes, nt)) return 1;
  }
  CK(hipFree(norm0));
  CK(hipFree(norm1));
  CK(hipFree(unc));
  CK(hipFree(fine));
  return 0;
}
