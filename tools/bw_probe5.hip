// bw_probe5.hip -- K1 shape probe, round 3: the round-1b winner (dense grid,
// one 16-byte vector per lane, non-temporal loads AND store) combined with
// the other knobs round 1b measured only on the cached policy: XCD-contiguous
// block placement, workgroup size, and 2 vectors per lane (both loaded before
// either is stored).  1 GiB and 2 GiB per buffer, best of 2 x 30 launches.
// Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int SWZ, int B, int V, bool NT = true>
__global__ void __launch_bounds__(B) k_sum(const f4 *__restrict__ a, f4 *__restrict__ b, size_t nvec) {
  size_t blk = blockIdx.x;
  if (SWZ) {  // the blocks one XCD receives (blockIdx % 8 equal) cover one contiguous eighth
    const size_t G = gridDim.x, per = G / 8;
    if (blk < per * 8) blk = (blk % 8) * per + blk / 8;
  }
  const size_t i0 = blk * (B * V) + threadIdx.x;
  f4 x[V], y[V];
#pragma unroll
  for (int v = 0; v < V; v++) {
    const size_t i = i0 + (size_t)v * B;
    if (i < nvec) {
      if (NT) { x[v] = __builtin_nontemporal_load(&b[i]); y[v] = __builtin_nontemporal_load(&a[i]); }
      else { x[v] = b[i]; y[v] = a[i]; }
    }
  }
#pragma unroll
  for (int v = 0; v < V; v++) {
    const size_t i = i0 + (size_t)v * B;
    if (i < nvec) {
      if (NT) __builtin_nontemporal_store(x[v] + y[v], &b[i]);
      else b[i] = x[v] + y[v];
    }
  }
}

template <class F> float timeit(F f, int it) {
  hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
  f(); f(); hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 2; r++) {
    hipEventRecord(s); for (int i = 0; i < it; i++) f(); hipEventRecord(e); hipEventSynchronize(e);
    float ms; hipEventElapsedTime(&ms, s, e); ms /= it; best = ms < best ? ms : best;
  }
  return best;
}
int main(int argc, char **argv) {
  if (argc > 1 && argv[1][0] == 'c') {   // `bw_probe5 cached`: the default-policy instance below 384 MiB
    for (size_t mib : {4, 16, 64, 128}) {
      size_t bytes = mib << 20, nvec = bytes / 16;
      f4 *a, *b;
      if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
      hipMemset(a, 0, bytes); hipMemset(b, 0, bytes);
      const double algo = 3.0 * bytes;
      printf("== %zu MiB per buffer (cached policy)\n", mib);
      auto rep = [&](const char *n, float ms) { printf("%-30s %8.4f ms %8.1f GB/s\n", n, ms, algo / ms / 1e6); };
      for (int round = 0; round < 3; round++) {
        rep("B256", timeit([&] { k_sum<0, 256, 1, false><<<(unsigned)((nvec + 255) / 256), 256>>>(a, b, nvec); }, 50));
        rep("B128", timeit([&] { k_sum<0, 128, 1, false><<<(unsigned)((nvec + 127) / 128), 128>>>(a, b, nvec); }, 50));
        rep("B64", timeit([&] { k_sum<0, 64, 1, false><<<(unsigned)((nvec + 63) / 64), 64>>>(a, b, nvec); }, 50));
      }
      hipFree(a); hipFree(b);
    }
    return 0;
  }
  for (size_t mib : {4096, 1024}) {
    size_t bytes = mib << 20, nvec = bytes / 16;
    f4 *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    hipMemset(a, 0, bytes); hipMemset(b, 0, bytes);
    const double algo = 3.0 * bytes;
    printf("== %zu MiB per buffer\n", mib);
    auto rep = [&](const char *n, float ms) { printf("%-30s %8.4f ms %8.1f GB/s\n", n, ms, algo / ms / 1e6); };
#define RUN(NAME, SWZ, B, V) \
    rep(NAME, timeit([&] { k_sum<SWZ, B, V><<<(unsigned)((nvec + B * V - 1) / (B * V)), B>>>(a, b, nvec); }, 30))
    for (int round = 0; round < 3; round++) {
      RUN("nt B256 V1 (K1 today)", 0, 256, 1);
      RUN("nt B128 V1", 0, 128, 1);
      RUN("nt B64 V1", 0, 64, 1);
      RUN("nt B128 V1 xcd-swizzle", 1, 128, 1);
      RUN("nt B192 V1", 0, 192, 1);
    }
    hipFree(a); hipFree(b);
  }
  return 0;
}
