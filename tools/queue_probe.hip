// queue_probe.hip -- diagnostic (not product): do kernels on different HIP
// streams of one process run concurrently once there are more streams than
// hardware queues (GPU_MAX_HW_QUEUES, 4 on the pool)?  The p2p engine keeps
// spinning kernels on several internal streams (send, receive, rendezvous),
// which is only deadlock-free if a spinning kernel never holds back a kernel
// of another stream.
//
// For S streams: a waiter kernel on each of streams 0..S-2 spins on its own
// flag (bounded: gives up after 2 s), then a setter kernel on stream S-1
// raises every flag.  Every waiter that saw its flag ran concurrently with
// the setter; a waiter that timed out was held behind it (shared queue).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void k_wait(unsigned *flag, int *result) {
  if (threadIdx.x != 0) return;
  const long long t0 = wall_clock64();
  const long long limit = 2LL * 100000000;   // wall_clock64 runs at 100 MHz
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
    __builtin_amdgcn_s_sleep(4);
    if (wall_clock64() - t0 > limit) {
      __hip_atomic_store(result, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
  __hip_atomic_store(result, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_set(unsigned *flags, int n) {
  if (threadIdx.x < n) __hip_atomic_store(flags + threadIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// mode 0: hipStreamCreateWithFlags; 1: hipExtStreamCreateWithCUMask (all
// CUs); 2: hipStreamCreateWithPriority (highest priority)
static int run(int S, bool with_null, int mode = 0) {
  unsigned *flags;
  int *res;
  hipMalloc(&flags, 64 * sizeof(unsigned));
  hipHostMalloc(&res, 64 * sizeof(int), hipHostMallocMapped);
  hipMemset(flags, 0, 64 * sizeof(unsigned));
  for (int i = 0; i < 64; i++) res[i] = 0;
  hipDeviceSynchronize();
  std::vector<hipStream_t> st(S);
  for (auto &s : st) {
    if (mode == 1 || mode == 3) {
      hipDeviceProp_t p;
      hipGetDeviceProperties(&p, 0);
      std::vector<uint32_t> mask((p.multiProcessorCount + 31) / 32, 0xffffffffu);
      hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
    } else if (mode == 2) {
      int lo, hi;
      hipDeviceGetStreamPriorityRange(&lo, &hi);
      hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi);
    } else {
      hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    }
  }
  if (with_null) {   // touch the null stream too, as torch-using processes do
    hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, nullptr, flags + 63, 1);
    hipDeviceSynchronize();
  }
  int *rdev;
  hipHostGetDevicePointer((void **)&rdev, res, 0);
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < S - 1; i++) hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, st[i], flags + i, rdev + i);
  // mode 3: CU-mask waiters, the setter on the legacy null stream (does the
  // null stream wait for a CU-masked stream, as for a blocking one?)
  hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, mode == 3 ? nullptr : st[S - 1], flags, S - 1);
  hipDeviceSynchronize();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  int ok = 0;
  printf("streams %2d%s%s: ", S, with_null ? " (+null)" : "        ",
         mode == 1 ? " cumask" : mode == 2 ? " hiprio" : mode == 3 ? " cm+nul" : "       ");
  for (int i = 0; i < S - 1; i++) {
    printf("%c", res[i] == 1 ? '+' : res[i] == 2 ? 'T' : '?');
    ok += res[i] == 1;
  }
  printf("  %d/%d waiters concurrent with the setter, %.1f ms\n", ok, S - 1, ms);
  fflush(stdout);
  for (auto &s : st) hipStreamDestroy(s);
  hipFree(flags);
  hipHostFree(res);
  return ok == S - 1 ? 0 : 1;
}

int main() {
  hipSetDevice(0);
  const char *q = getenv("GPU_MAX_HW_QUEUES");
  printf("GPU_MAX_HW_QUEUES=%s\n", q ? q : "(unset)");
  int bad = 0;
  for (int S : {2, 3, 4, 5, 6, 8, 12}) bad += run(S, false);
  for (int S : {4, 5, 8}) bad += run(S, true);
  for (int S : {4, 8, 12}) bad += run(S, false, 1);
  for (int S : {4, 8}) bad += run(S, false, 2);
  for (int S : {2, 4}) bad += run(S, false, 3);
  {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    std::vector<uint32_t> mask((p.multiProcessorCount + 31) / 32, 0xffffffffu);
    hipStream_t s;
    unsigned fl = 99;
    hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
    hipStreamGetFlags(s, &fl);
    printf("CU-mask stream flags: %u (hipStreamNonBlocking = %u)\n", fl, (unsigned)hipStreamNonBlocking);
    hipStreamDestroy(s);
  }
  printf("%s\n", bad ? "SOME WAITERS WERE HELD BEHIND THE SETTER" : "all concurrent");
  return 0;
}
