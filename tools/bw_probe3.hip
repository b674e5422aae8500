// bw_probe3.hip -- K1 shape probe, round 1b: cache-policy and XCD-placement
// variants of the dense one-vector-per-lane 2-buffer SUM (b = b + a), plus the
// copy / read-only ceilings on the same box.  Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int LNT, int SNT, int SWZ, int B>
__global__ void __launch_bounds__(B) k_sum(const f4 *__restrict__ a, f4 *__restrict__ b, size_t nvec) {
  size_t blk = blockIdx.x;
  if (SWZ) {  // XCD-contiguous: the blocks one XCD receives (b % 8 equal) cover one contiguous 1/8
    const size_t G = gridDim.x, per = G / 8;
    if (blk < per * 8) blk = (blk % 8) * per + blk / 8;
  }
  const size_t i = blk * B + threadIdx.x;
  if (i >= nvec) return;
  f4 x, y;
  if (LNT) { x = __builtin_nontemporal_load(&b[i]); y = __builtin_nontemporal_load(&a[i]); }
  else { x = b[i]; y = a[i]; }
  x += y;
  if (SNT) __builtin_nontemporal_store(x, &b[i]);
  else b[i] = x;
}
__global__ void __launch_bounds__(256) k_copy(const f4 *__restrict__ a, f4 *__restrict__ b, size_t nvec) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < nvec) b[i] = a[i];
}
__global__ void __launch_bounds__(256) k_read(const f4 *__restrict__ a, const f4 *__restrict__ b, float *out, size_t nvec) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < nvec) {
    f4 x = a[i] + b[i];
    if (x.x == 12345.f) out[0] = x.y;  // never true for the zero-filled input
  }
}
template <class F> float timeit(F f, int it) {
  hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
  f(); f(); hipDeviceSynchronize();
  hipEventRecord(s); for (int i = 0; i < it; i++) f(); hipEventRecord(e); hipEventSynchronize(e);
  float ms; hipEventElapsedTime(&ms, s, e); return ms / it;
}
int main() {
  for (size_t mib : {1024, 2048}) {
    size_t bytes = mib << 20, nvec = bytes / 16;
    f4 *a, *b; float *o;
    hipMalloc(&a, bytes); hipMalloc(&b, bytes); hipMalloc(&o, 64);
    hipMemset(a, 0, bytes); hipMemset(b, 0, bytes);
    const double algo = 3.0 * bytes;
    printf("== %zu MiB per buffer\n", mib);
    auto rep = [&](const char *n, float ms, double by) { printf("%-34s %8.4f ms %8.1f GB/s\n", n, ms, by / ms / 1e6); };
    const unsigned g = (unsigned)((nvec + 255) / 256);
    for (int r = 0; r < 2; r++) {
      rep("sum base", timeit([&] { k_sum<0, 0, 0, 256><<<g, 256>>>(a, b, nvec); }, 30), algo);
      rep("sum nt-store", timeit([&] { k_sum<0, 1, 0, 256><<<g, 256>>>(a, b, nvec); }, 30), algo);
      rep("sum nt-load", timeit([&] { k_sum<1, 0, 0, 256><<<g, 256>>>(a, b, nvec); }, 30), algo);
      rep("sum nt-both", timeit([&] { k_sum<1, 1, 0, 256><<<g, 256>>>(a, b, nvec); }, 30), algo);
      rep("sum xcd-swizzle", timeit([&] { k_sum<0, 0, 1, 256><<<g, 256>>>(a, b, nvec); }, 30), algo);
      rep("sum xcd-swizzle nt-store", timeit([&] { k_sum<0, 1, 1, 256><<<g, 256>>>(a, b, nvec); }, 30), algo);
      rep("sum B128", timeit([&] { k_sum<0, 0, 0, 128><<<(unsigned)((nvec + 127) / 128), 128>>>(a, b, nvec); }, 30), algo);
      rep("copy (2 streams)", timeit([&] { k_copy<<<g, 256>>>(a, b, nvec); }, 30), 2.0 * bytes);
      rep("read (2 streams)", timeit([&] { k_read<<<g, 256>>>(a, b, o, nvec); }, 30), 2.0 * bytes);
    }
    hipFree(a); hipFree(b); hipFree(o);
  }
  return 0;
}
