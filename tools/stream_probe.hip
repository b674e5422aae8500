// stream_probe.hip -- diagnostic (not product): host cost of one small
// synchronous kernel call under the stream disciplines the op / coll
// components can use (profiles/r02/stream_probe.txt).
//   null      launch on the legacy default stream, hipStreamSynchronize(0)
//   nb        launch on a non-blocking stream, hipStreamSynchronize(s)
//   nb+order  hipEventRecord(ev, 0) + hipStreamWaitEvent(s, ev) + launch(s) + sync(s)
//   nb+evsync launch(s) + hipEventRecord(done, s) + hipEventSynchronize(done)
//   blocking  launch on a hipStreamDefault stream (implicitly ordered with 0) + sync(s)
//   nb+query  launch(s) + poll hipStreamQuery(s) until done
// and the host cost of single calls on an idle device (no wait):
//   query0    hipStreamQuery(0)        queryNB  hipStreamQuery(nb)
//   record    hipEventRecord(ev, nb)   launch64 a 64-workgroup kernel on nb
//   devptr    hipHostGetDevicePointer of a mapped host block
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_add(float *a, const float *b, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] += b[i];
}

int main() {
  const int n = 1024, iters = 2000;
  float *a, *b;
  hipMalloc(&a, n * 4);
  hipMalloc(&b, n * 4);
  hipStream_t nb, bl;
  hipStreamCreateWithFlags(&nb, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&bl, hipStreamDefault);
  hipEvent_t ev, done;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  hipEventCreateWithFlags(&done, hipEventDisableTiming);
  auto run = [&](const char *name, auto body) {
    for (int i = 0; i < 100; i++) body();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; i++) body();
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
    printf("%-10s %7.2f us per call\n", name, us);
  };
  run("null", [&] { hipLaunchKernelGGL(k_add, dim3(4), dim3(256), 0, 0, a, b, n); hipStreamSynchronize(0); });
  run("nb", [&] { hipLaunchKernelGGL(k_add, dim3(4), dim3(256), 0, nb, a, b, n); hipStreamSynchronize(nb); });
  run("nb+order", [&] {
    hipEventRecord(ev, 0);
    hipStreamWaitEvent(nb, ev, 0);
    hipLaunchKernelGGL(k_add, dim3(4), dim3(256), 0, nb, a, b, n);
    hipStreamSynchronize(nb);
  });
  run("nb+evsync", [&] {
    hipLaunchKernelGGL(k_add, dim3(4), dim3(256), 0, nb, a, b, n);
    hipEventRecord(done, nb);
    hipEventSynchronize(done);
  });
  run("blocking", [&] { hipLaunchKernelGGL(k_add, dim3(4), dim3(256), 0, bl, a, b, n); hipStreamSynchronize(bl); });
  run("nb+query", [&] {
    hipLaunchKernelGGL(k_add, dim3(4), dim3(256), 0, nb, a, b, n);
    while (hipStreamQuery(nb) == hipErrorNotReady) {
    }
  });
  run("null+query", [&] {
    hipLaunchKernelGGL(k_add, dim3(4), dim3(256), 0, 0, a, b, n);
    while (hipStreamQuery(0) == hipErrorNotReady) {
    }
  });
  hipDeviceSynchronize();
  auto cost = [&](const char *name, auto body) {
    for (int i = 0; i < 100; i++) body();
    hipDeviceSynchronize();
    double tot = 0;
    for (int i = 0; i < iters; i++) {
      const auto t0 = std::chrono::steady_clock::now();
      body();
      tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if ((i & 63) == 63) hipDeviceSynchronize();
    }
    printf("%-10s %7.2f us per call (host)\n", name, tot / iters);
  };
  int64_t *hb = nullptr, *db = nullptr;
  hipHostMalloc((void **)&hb, 64, hipHostMallocMapped);
  cost("query0", [&] { (void)hipStreamQuery(0); });
  cost("queryNB", [&] { (void)hipStreamQuery(nb); });
  cost("record", [&] { hipEventRecord(done, nb); });
  cost("launch64", [&] { hipLaunchKernelGGL(k_add, dim3(64), dim3(256), 0, nb, a, b, n); });
  cost("devptr", [&] { hipHostGetDevicePointer((void **)&db, hb, 0); });
  hipDeviceSynchronize();
  return 0;
}
