// bw_probe4.hip -- K1 probe, round 1c: XCD placement and block size on top
// of the nt-both policy that K1 ships (bw_probe3 measured swizzle only with
// default-policy loads).  b = b + a, fp32, 1 and 2 GiB per buffer.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int SWZ, int B>
__global__ void __launch_bounds__(B) k_sum(const f4 *__restrict__ a, f4 *__restrict__ b, size_t nvec) {
  size_t blk = blockIdx.x;
  if (SWZ == 1) {  // XCD-contiguous: the blocks one XCD receives (blk % 8 equal) cover one contiguous 1/8
    const size_t G = gridDim.x, per = G / 8;
    if (blk < per * 8) blk = (blk % 8) * per + blk / 8;
  } else if (SWZ == 2) {  // XCD-chunked: runs of 64 consecutive blocks stay on one XCD
    const size_t G = gridDim.x, grp = 64 * 8;
    if (blk < G / grp * grp) {
      const size_t g = blk / grp, r = blk % grp;
      blk = g * grp + (r % 8) * 64 + r / 8;
    }
  }
  const size_t i = blk * B + threadIdx.x;
  if (i >= nvec) return;
  f4 x = __builtin_nontemporal_load(&b[i]);
  f4 y = __builtin_nontemporal_load(&a[i]);
  x += y;
  __builtin_nontemporal_store(x, &b[i]);
}

template <class F> float timeit(F f, int it) {
  hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
  f(); hipDeviceSynchronize();
  hipEventRecord(s); for (int i = 0; i < it; i++) f(); hipEventRecord(e); hipEventSynchronize(e);
  float ms; hipEventElapsedTime(&ms, s, e); return ms / it;
}

int main() {
  for (size_t mib : {1024, 2048}) {
    size_t bytes = mib << 20, nvec = bytes / 16;
    f4 *a, *b;
    hipMalloc(&a, bytes); hipMalloc(&b, bytes);
    hipMemset(a, 0, bytes); hipMemset(b, 0, bytes);
    const double algo = 3.0 * bytes;
    printf("== %zu MiB per buffer\n", mib);
    auto rep = [&](const char *n, float ms) { printf("%-34s %8.4f ms %8.1f GB/s\n", n, ms, algo / ms / 1e6); };
    for (int r = 0; r < 4; r++) {
      rep("nt-both B256", timeit([&] { k_sum<0, 256><<<(unsigned)((nvec + 255) / 256), 256>>>(a, b, nvec); }, 30));
      rep("nt-both B256 xcd-contig", timeit([&] { k_sum<1, 256><<<(unsigned)((nvec + 255) / 256), 256>>>(a, b, nvec); }, 30));
      rep("nt-both B1024", timeit([&] { k_sum<0, 1024><<<(unsigned)((nvec + 1023) / 1024), 1024>>>(a, b, nvec); }, 30));
      rep("nt-both B1024 xcd-contig", timeit([&] { k_sum<1, 1024><<<(unsigned)((nvec + 1023) / 1024), 1024>>>(a, b, nvec); }, 30));
    }
    hipFree(a); hipFree(b);
  }
  return 0;
}
