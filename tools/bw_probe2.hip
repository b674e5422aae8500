#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
template <int B, int U>
__global__ void __launch_bounds__(B) k_chunk(const f4 *__restrict__ a, f4 *__restrict__ b, size_t nvec) {
  size_t base = (size_t)blockIdx.x * B * U + threadIdx.x;
  f4 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; u++) { size_t i = base + u * B; if (i < nvec) { x[u] = b[i]; y[u] = a[i]; } }
#pragma unroll
  for (int u = 0; u < U; u++) { size_t i = base + u * B; if (i < nvec) b[i] = x[u] + y[u]; }
}
// persistent contiguous segments
template <int B, int U>
__global__ void __launch_bounds__(B) k_seg(const f4 *__restrict__ a, f4 *__restrict__ b, size_t nvec) {
  size_t per = (nvec + gridDim.x - 1) / gridDim.x;
  size_t lo = (size_t)blockIdx.x * per, hi = lo + per < nvec ? lo + per : nvec;
  for (size_t base = lo + threadIdx.x; base < hi; base += B * U) {
    f4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) { size_t i = base + u * B; if (i < hi) { x[u] = b[i]; y[u] = a[i]; } }
#pragma unroll
    for (int u = 0; u < U; u++) { size_t i = base + u * B; if (i < hi) b[i] = x[u] + y[u]; }
  }
}
template <int B>
__global__ void __launch_bounds__(B) k_gs(const f4 *__restrict__ a, f4 *__restrict__ b, size_t nvec) {
  for (size_t i = (size_t)blockIdx.x * B + threadIdx.x; i < nvec; i += (size_t)gridDim.x * B) b[i] = b[i] + a[i];
}
template <class F> float timeit(F f, int it) {
  hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
  f(); f(); hipDeviceSynchronize();
  hipEventRecord(s); for (int i = 0; i < it; i++) f(); hipEventRecord(e); hipEventSynchronize(e);
  float ms; hipEventElapsedTime(&ms, s, e); return ms / it;
}
int main() {
  for (size_t mib : {1024, 256, 64}) {
  size_t bytes = mib << 20, nvec = bytes / 16;
  f4 *a, *b; hipMalloc(&a, bytes); hipMalloc(&b, bytes); hipMemset(a, 0, bytes); hipMemset(b, 0, bytes);
  double algo = 3.0 * bytes;
  printf("== %zu MiB\n", mib);
  auto rep = [&](const char *n, float ms) { printf("%-30s %8.4f ms %8.1f GB/s\n", n, ms, algo / ms / 1e6); };
  rep("chunk B256 U1", timeit([&] { k_chunk<256, 1><<<(nvec + 255) / 256, 256>>>(a, b, nvec); }, 30));
  rep("chunk B512 U1", timeit([&] { k_chunk<512, 1><<<(nvec + 511) / 512, 512>>>(a, b, nvec); }, 30));
  rep("chunk B1024 U1", timeit([&] { k_chunk<1024, 1><<<(nvec + 1023) / 1024, 1024>>>(a, b, nvec); }, 30));
  rep("chunk B256 U2", timeit([&] { k_chunk<256, 2><<<(nvec + 511) / 512, 256>>>(a, b, nvec); }, 30));
  rep("chunk B512 U2", timeit([&] { k_chunk<512, 2><<<(nvec + 1023) / 1024, 512>>>(a, b, nvec); }, 30));
  for (unsigned g : {256u, 512u, 1024u, 2048u}) {
    char nm[64];
    sprintf(nm, "seg B256 U1 g%u", g); rep(nm, timeit([&] { k_seg<256, 1><<<g, 256>>>(a, b, nvec); }, 30));
    sprintf(nm, "seg B256 U4 g%u", g); rep(nm, timeit([&] { k_seg<256, 4><<<g, 256>>>(a, b, nvec); }, 30));
    sprintf(nm, "seg B512 U2 g%u", g); rep(nm, timeit([&] { k_seg<512, 2><<<g, 512>>>(a, b, nvec); }, 30));
  }
  for (unsigned g : {256u, 384u, 512u}) {
    char nm[64];
    sprintf(nm, "gs B256 g%u", g); rep(nm, timeit([&] { k_gs<256><<<g, 256>>>(a, b, nvec); }, 30));
    sprintf(nm, "gs B512 g%u", g); rep(nm, timeit([&] { k_gs<512><<<g, 512>>>(a, b, nvec); }, 30));
    sprintf(nm, "gs B1024 g%u", g); rep(nm, timeit([&] { k_gs<1024><<<g, 1024>>>(a, b, nvec); }, 30));
  }
  hipFree(a); hipFree(b);
  }
  return 0;
}
