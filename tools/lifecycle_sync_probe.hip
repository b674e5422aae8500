// lifecycle_sync_probe.hip -- which HIP runtime calls wait for a kernel
// spinning on another stream?  (communicator
// create / destroy / p2p setup must never wait for another communicator's
// spinning collective or receive.)
//
// For every call below: a one-wave kernel spins on a mapped host word on
// stream S (non-blocking high-priority like a p2p channel, or an ordinary
// blocking stream), a host thread releases it after kRelease ms, and the
// call is timed on the main thread.  A call that takes ~kRelease ms waited
// for the spinner.  The spinner also exits by itself after 5 s, so nothing
// can hang.  The IPC open / close rows use a buffer exported by a child
// process forked before any HIP call.
//
// build: hipcc --offload-arch=gfx950 -O2 -o tools/lifecycle_sync_probe tools/lifecycle_sync_probe.hip
#include <hip/hip_runtime.h>
#include <unistd.h>
#include <sys/wait.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <thread>

static const int kRelease = 800;   // ms

__global__ void spin(int *go, long long max_ticks) {
  const long long t0 = wall_clock64();
  while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 && wall_clock64() - t0 < max_ticks)
    __builtin_amdgcn_s_sleep(10);
}

__global__ void nop() {}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); } } while (0)

static int *g_go;
static hipStream_t g_spin_stream;

static double timed(const char *name, const std::function<hipError_t()> &fn) {
  *(volatile int *)g_go = 0;
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, g_spin_stream, g_go, 500000000LL);
  CK(hipGetLastError());
  std::this_thread::sleep_for(std::chrono::milliseconds(30));
  std::thread rel([] {
    std::this_thread::sleep_for(std::chrono::milliseconds(kRelease));
    __atomic_store_n(g_go, 1, __ATOMIC_SEQ_CST);
  });
  const auto t0 = std::chrono::steady_clock::now();
  const hipError_t e = fn();
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  rel.join();
  CK(hipStreamSynchronize(g_spin_stream));
  printf("  %-46s %9.2f ms  %s%s\n", name, ms, ms > 0.8 * kRelease ? "WAITS FOR THE SPINNER" : "independent",
         e == hipSuccess ? "" : "  (call failed)");
  fflush(stdout);
  return ms;
}

int main() {
  // child: exports one allocation, sends the handle, waits for "done"
  int h2c[2], c2h[2];
  if (pipe(h2c) || pipe(c2h)) return 1;
  const pid_t pid = fork();
  if (pid == 0) {
    void *b = nullptr;
    hipIpcMemHandle_t hd;
    memset(&hd, 0, sizeof hd);
    if (hipMalloc(&b, 4 << 20) != hipSuccess || hipIpcGetMemHandle(&hd, b) != hipSuccess) memset(&hd, 0, sizeof hd);
    if (write(c2h[1], &hd, sizeof hd) != (ssize_t)sizeof hd) _exit(1);
    char x;
    if (read(h2c[0], &x, 1) != 1) _exit(1);
    _exit(0);
  }
  hipIpcMemHandle_t peer;
  if (read(c2h[0], &peer, sizeof peer) != (ssize_t)sizeof peer) return 1;

  CK(hipSetDevice(0));
  CK(hipHostMalloc((void **)&g_go, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t priv;
  CK(hipStreamCreateWithFlags(&priv, hipStreamNonBlocking));
  hipLaunchKernelGGL(nop, dim3(1), dim3(64), 0, priv);
  CK(hipStreamSynchronize(priv));
  char *pre[8];
  for (auto &p : pre) CK(hipMalloc((void **)&p, 1 << 20));
  char *preu[2];
  for (auto &p : preu) CK(hipExtMallocWithFlags((void **)&p, 1 << 20, hipDeviceMallocUncached));
  int *preh[2];
  for (auto &p : preh) CK(hipHostMalloc((void **)&p, 4096, hipHostMallocMapped));

  for (int mode = 0; mode < 2; mode++) {
    if (mode == 0) {
      CK(hipStreamCreateWithPriority(&g_spin_stream, hipStreamNonBlocking, hi));
      printf("spinner on a non-blocking high-priority stream (p2p channel / request stream):\n");
    } else {
      CK(hipStreamCreateWithFlags(&g_spin_stream, hipStreamDefault));
      printf("spinner on an ordinary blocking stream:\n");
    }
    char *m = nullptr, *u = nullptr;
    int *h = nullptr;
    void *imp = nullptr;
    uint64_t v = 7;
    timed("hipDeviceSynchronize (control)", [] { return hipDeviceSynchronize(); });
    timed("hipMalloc 1 MiB", [&] { return hipMalloc((void **)&m, 1 << 20); });
    timed("hipFree (an idle 1 MiB buffer)", [&] { return hipFree(pre[mode * 2]); });
    timed("hipExtMallocWithFlags uncached 1 MiB", [&] { return hipExtMallocWithFlags((void **)&u, 1 << 20,
                                                                                      hipDeviceMallocUncached); });
    timed("hipFree (an idle uncached buffer)", [&] { return hipFree(preu[mode]); });
    timed("hipMemset 8 B (null stream)", [&] { return hipMemset(m, 0, 8); });
    timed("hipMemcpy H2D 8 B", [&] { return hipMemcpy(m, &v, 8, hipMemcpyHostToDevice); });
    timed("hipMemcpy D2H 8 B", [&] { return hipMemcpy(&v, m, 8, hipMemcpyDeviceToHost); });
    timed("hipMemsetAsync + sync, private nb stream", [&] {
      hipError_t e = hipMemsetAsync(m, 0, 8, priv);
      return e == hipSuccess ? hipStreamSynchronize(priv) : e;
    });
    timed("hipMemcpyAsync D2H + sync, private nb stream", [&] {
      hipError_t e = hipMemcpyAsync(&v, m, 8, hipMemcpyDeviceToHost, priv);
      return e == hipSuccess ? hipStreamSynchronize(priv) : e;
    });
    timed("kernel + sync, private nb stream", [&] {
      hipLaunchKernelGGL(nop, dim3(1), dim3(64), 0, priv);
      return hipStreamSynchronize(priv);
    });
    timed("kernel + sync, null stream", [&] {
      hipLaunchKernelGGL(nop, dim3(1), dim3(64), 0, nullptr);
      return hipStreamSynchronize(nullptr);
    });
    timed("hipHostMalloc mapped 4 KiB", [&] { return hipHostMalloc((void **)&h, 4096, hipHostMallocMapped); });
    timed("hipHostFree (an idle buffer)", [&] { return hipHostFree(preh[mode]); });
    timed("hipStreamCreate + hipStreamDestroy (idle)", [&] {
      hipStream_t s;
      hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
      return e == hipSuccess ? hipStreamDestroy(s) : e;
    });
    timed("hipEventCreate + hipEventDestroy", [&] {
      hipEvent_t ev;
      hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
      return e == hipSuccess ? hipEventDestroy(ev) : e;
    });
    timed("hipIpcGetMemHandle (fresh alloc)", [&] {
      hipIpcMemHandle_t hd;
      return hipIpcGetMemHandle(&hd, u);
    });
    timed("hipIpcOpenMemHandle (child's buffer)", [&] {
      return hipIpcOpenMemHandle(&imp, peer, hipIpcMemLazyEnablePeerAccess);
    });
    timed("hipIpcCloseMemHandle", [&] { return imp ? hipIpcCloseMemHandle(imp) : hipErrorInvalidValue; });
    timed("hipFree (the buffer hipMalloc'ed above)", [&] { return hipFree(m); });
    timed("hipFree (the uncached buffer above)", [&] { return hipFree(u); });
    timed("hipHostFree (the buffer above)", [&] { return hipHostFree(h); });
    CK(hipStreamDestroy(g_spin_stream));
  }
  char x = 1;
  if (write(h2c[1], &x, 1) != 1) return 1;
  waitpid(pid, nullptr, 0);
  return 0;
}
