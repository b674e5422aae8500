// event_probe -- cost of ordering one stream after another with an event
// (hipEventRecord on A + hipStreamWaitEvent on B), per hand-off, for the
// stream kinds the library uses: the legacy default stream, ordinary
// blocking / non-blocking streams and high-priority non-blocking streams
// (the channel / request streams).  Each iteration runs a tiny
// kernel on A, hands off to B, runs a tiny kernel on B and hands back.
// build: hipcc --offload-arch=gfx950 -O2 -o /tmp/event_probe tools/event_probe.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <stdio.h>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__global__ void k_tiny(int *p) {
  if (threadIdx.x == 0 && p) p[0] += 1;
}

static int run(const char *name, hipStream_t a, hipStream_t b, int *buf, bool handoff) {
  hipEvent_t ea, eb;
  CK(hipEventCreateWithFlags(&ea, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
  const int iters = 2000;
  for (int pass = 0; pass < 2; pass++) {
    CK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; i++) {
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, a, buf);
      if (handoff) {
        CK(hipEventRecord(ea, a));
        CK(hipStreamWaitEvent(b, ea, 0));
      }
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, handoff ? b : a, buf + 16);
      if (handoff) {
        CK(hipEventRecord(eb, b));
        CK(hipStreamWaitEvent(a, eb, 0));
      }
    }
    CK(hipDeviceSynchronize());
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (pass) printf("%-52s %8.2f us per iteration (2 kernels%s)\n", name, us / iters, handoff ? ", 2 hand-offs" : "");
  }
  CK(hipEventDestroy(ea));
  CK(hipEventDestroy(eb));
  return 0;
}

int main() {
  CK(hipSetDevice(0));
  int *buf;
  CK(hipMalloc(&buf, 4096));
  CK(hipMemset(buf, 0, 4096));
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t blk, nb, hi1, hi2;
  CK(hipStreamCreateWithFlags(&blk, hipStreamDefault));
  CK(hipStreamCreateWithFlags(&nb, hipStreamNonBlocking));
  CK(hipStreamCreateWithPriority(&hi1, hipStreamNonBlocking, greatest));
  CK(hipStreamCreateWithPriority(&hi2, hipStreamNonBlocking, greatest));
  if (run("same stream (no hand-off), legacy default", 0, 0, buf, false)) return 1;
  if (run("same stream (no hand-off), high priority", hi1, hi1, buf, false)) return 1;
  if (run("legacy default <-> high-priority non-blocking", 0, hi1, buf, true)) return 1;
  if (run("blocking <-> high-priority non-blocking", blk, hi1, buf, true)) return 1;
  if (run("non-blocking <-> high-priority non-blocking", nb, hi1, buf, true)) return 1;
  if (run("high-priority <-> high-priority", hi1, hi2, buf, true)) return 1;
  if (run("legacy default <-> non-blocking", 0, nb, buf, true)) return 1;
  CK(hipFree(buf));
  return 0;
}
