// svc_pingpong_probe.hip -- diagnostic (not product): what one host -> resident
// kernel -> host round trip costs on this box, piece by piece, to decide
// whether the op service (csrc/mx_service.hip) can beat a launch per call.
// One workgroup stays resident and serves `iters` commands; the host posts a
// sequence number and spins on the kernel's completion word (host memory).
//   mode 0  doorbell in coherent mapped host memory (the kernel polls over
//           PCIe); completion written at once
//   mode 1  0 + a system-scope acquire before and release after (the
//           service's fences)
//   mode 2  1 + a 4 KiB reduce (load two 4 KiB operands, add, store)
//   mode 3  doorbell in fine-grained device memory written by the host
//           (the kernel polls its own HBM/L2; the host's write is posted)
//   mode 4  3 + fences + the 4 KiB reduce
//   mode 5  2 + 63 more resident workgroups polling a word in uncached
//           device memory (the product service's idle takers)
//   mode 6  2 with the command read as four 16-byte nontemporal loads of
//           the 64-byte line (the product's read)
//   mode 7  5 with the pollers sleeping s_sleep(127) between polls
//   mode 8  2 with the command read as eight 8-byte system-scope loads
//           (the product's read since r4l)
//   mode 9  2 with a 1024-lane workgroup (the same 4 KiB reduce)
//   mode 10 2 with the command read by one instruction of wave 0 (lanes
//           0..7 one 8-byte system-scope load each, gathered by shuffles)
// Each kernel leaves after `iters` commands or 1 s without one.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(1024) k_serve(const uint64_t *bell, uint64_t *done, float *a, float *b, int mode,
                                               uint64_t iters, uint64_t idle_ticks, uint64_t *gate) {
  __shared__ uint64_t s_q;
  __shared__ int s_exit;
  if (blockIdx.x > 0) {                     // modes 5, 7: pollers until workgroup 0 leaves
    if (threadIdx.x == 0)
      while (__hip_atomic_load(gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        if (mode == 7) __builtin_amdgcn_s_sleep(127);
        else __builtin_amdgcn_s_sleep(1);
      }
    return;
  }
  for (uint64_t k = 1; k <= iters; k++) {
    if (mode == 10 && threadIdx.x < 64) {   // the whole of wave 0 polls
      const int lane = threadIdx.x;
      const uint64_t t0 = wall_clock64();
      int ex = 0;
      uint64_t v0 = 0;
      for (;;) {
        const uint64_t x = lane < 8 ? __hip_atomic_load(bell + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
        uint64_t acc = 0;
#pragma unroll
        for (int j = 1; j < 8; j++) acc ^= __shfl(x, j);
        v0 = __shfl(x, 0) + (acc & 0);
        if (v0 >= k) break;
        if (wall_clock64() - t0 > idle_ticks) { ex = 1; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      if (lane == 0) { s_q = v0; s_exit = ex; }
    } else if (mode != 10 && threadIdx.x == 0) {
      const uint64_t t0 = wall_clock64();
      s_exit = 0;
      for (;;) {
        uint64_t v;
        if (mode == 8) {
          uint64_t w[8];
#pragma unroll
          for (int j = 0; j < 8; j++) w[j] = __hip_atomic_load(bell + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          v = w[0] + ((w[1] ^ w[2] ^ w[3] ^ w[4] ^ w[5] ^ w[6] ^ w[7]) & 0);
        } else if (mode == 6) {
          const u64x2 *p = reinterpret_cast<const u64x2 *>(bell);
          u64x2 v0 = __builtin_nontemporal_load(p), v1 = __builtin_nontemporal_load(p + 1);
          u64x2 v2 = __builtin_nontemporal_load(p + 2), v3 = __builtin_nontemporal_load(p + 3);
          v = v0.x + ((v1.x ^ v2.y ^ v3.x ^ v0.y ^ v1.y ^ v2.x ^ v3.y) & 0);
        } else {
          v = __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (v >= k) { s_q = v; break; }
        if (wall_clock64() - t0 > idle_ticks) { s_exit = 1; break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    if (s_exit) break;
    const bool fences = mode != 0 && mode != 3;
    const bool work = fences && mode != 1;
    if (fences) __atomic_thread_fence(__ATOMIC_ACQUIRE);
    if (work && threadIdx.x < 256) {
      float4 x = reinterpret_cast<float4 *>(b)[threadIdx.x];
      const float4 y = reinterpret_cast<const float4 *>(a)[threadIdx.x];
      x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
      reinterpret_cast<float4 *>(b)[threadIdx.x] = x;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      if (fences) __threadfence_system();
      __hip_atomic_store(done, s_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(gate, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

int main(int argc, char **argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const uint64_t iters = argc > 1 ? strtoull(argv[1], nullptr, 10) : 20000;
  int rate_khz = 100000;
  (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
  const uint64_t idle = (uint64_t)rate_khz * 1000;   // 1 s
  uint64_t *hbell, *dbell_h, *hdone, *ddone;
  CK(hipHostMalloc((void **)&hbell, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void **)&dbell_h, hbell, 0));
  CK(hipHostMalloc((void **)&hdone, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void **)&ddone, hdone, 0));
  uint64_t *fbell = nullptr;   // fine-grained device memory
  const bool fg = hipExtMallocWithFlags((void **)&fbell, 64, hipDeviceMallocFinegrained) == hipSuccess;
  bool fg_host = false;
  if (fg) {
    CK(hipMemset(fbell, 0, 64));
    CK(hipDeviceSynchronize());
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, fbell) == hipSuccess) printf("fine-grained bell: type %d hostPointer %p devicePointer %p\n", (int)at.type, at.hostPointer, at.devicePointer);
    // the host touches it before any kernel runs: a fault here ends nothing on the GPU
    volatile uint64_t *p = fbell;
    *p = 7;
    fg_host = *p == 7;
    *p = 0;
    printf("fine-grained bell host access: %s\n", fg_host ? "ok" : "no");
  }
  printf("setup done\n");
  float *a, *b;
  CK(hipMalloc(&a, 4096));
  CK(hipMalloc(&b, 4096));
  CK(hipMemset(a, 0, 4096));
  CK(hipMemset(b, 0, 4096));
  uint64_t *gate;
  CK(hipExtMallocWithFlags((void **)&gate, 64, hipDeviceMallocUncached));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<int> modes;
  for (int i = 2; i < argc; i++) modes.push_back(atoi(argv[i]));
  if (modes.empty()) modes = {0, 1, 2, 5, 6, 7};   // 3 and 4 hung on the box (r4j): opt-in only
  for (int mode : modes) {
    if ((mode == 3 || mode == 4) && !fg_host) continue;
    uint64_t *bell_host = (mode == 3 || mode == 4) ? fbell : hbell;
    const uint64_t *bell_dev = (mode == 3 || mode == 4) ? fbell : dbell_h;
    printf("mode %d: start\n", mode);
    __atomic_store_n(bell_host, 0, __ATOMIC_RELEASE);
    __atomic_store_n(hdone, 0, __ATOMIC_RELEASE);
    CK(hipMemset(gate, 0, 8));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_serve, dim3(mode == 5 || mode == 7 ? 64 : 1), dim3(mode == 9 ? 1024 : 256), 0, s, bell_dev, ddone, a, b, mode, iters, idle, gate);
    CK(hipGetLastError());
    std::vector<double> t;
    t.reserve(iters);
    bool lost = false;
    for (uint64_t k = 1; k <= iters; k++) {
      const auto t0 = std::chrono::steady_clock::now();
      __atomic_store_n(bell_host, k, __ATOMIC_RELEASE);
      for (unsigned n = 0; __atomic_load_n(hdone, __ATOMIC_ACQUIRE) < k; n++) {
        __builtin_ia32_pause();
        if ((n & 4095) == 4095 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 0.5) {
          lost = true;
          break;
        }
      }
      if (lost) break;
      t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    printf("mode %d: %zu commands, joining\n", mode, t.size());
    CK(hipStreamSynchronize(s));   // the kernel leaves after iters commands or 1 s idle
    if (lost) { printf("mode %d: completion lost at %zu\n", mode, t.size()); continue; }
    std::sort(t.begin(), t.end());
    printf("mode %d  round trip: median %.2f us  p10 %.2f  p90 %.2f  p99 %.2f\n", mode, t[t.size() / 2],
           t[t.size() / 10], t[t.size() * 9 / 10], t[t.size() * 99 / 100]);
  }
  return 0;
}
