// Tuning probe for the K1 streaming kernel shape (fp32 SUM, 2-buffer, 1 GiB).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4 add4(f4 a, f4 b) { return a + b; }

template <int U, bool NT>
__global__ void __launch_bounds__(256) k_gs(const f4 *__restrict__ a, f4 *__restrict__ b, size_t nvec) {
  size_t tid = (size_t)blockIdx.x * 256 + threadIdx.x, stride = (size_t)gridDim.x * 256;
  size_t i = tid;
  for (; i + (U - 1) * stride < nvec; i += U * stride) {
    f4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (NT) { x[u] = __builtin_nontemporal_load(&b[i + u * stride]); y[u] = __builtin_nontemporal_load(&a[i + u * stride]); }
      else { x[u] = b[i + u * stride]; y[u] = a[i + u * stride]; }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      f4 r = add4(x[u], y[u]);
      if (NT) __builtin_nontemporal_store(r, &b[i + u * stride]); else b[i + u * stride] = r;
    }
  }
  for (; i < nvec; i += stride) b[i] = add4(b[i], a[i]);
}
// contiguous chunk per block: block handles [blk*CH, (blk+1)*CH) vecs, U vecs per thread per iter
template <int U>
__global__ void __launch_bounds__(256) k_chunk(const f4 *__restrict__ a, f4 *__restrict__ b, size_t nvec) {
  size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  f4 x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; u++) { size_t i = base + u * 256; if (i < nvec) { x[u] = b[i]; y[u] = a[i]; } }
#pragma unroll
  for (int u = 0; u < U; u++) { size_t i = base + u * 256; if (i < nvec) b[i] = add4(x[u], y[u]); }
}
template <class F>
float timeit(F f, int it) {
  hipEvent_t s, e; hipEventCreate(&s); hipEventCreate(&e);
  f(); hipDeviceSynchronize();
  hipEventRecord(s); for (int i = 0; i < it; i++) f(); hipEventRecord(e); hipEventSynchronize(e);
  float ms; hipEventElapsedTime(&ms, s, e); return ms / it;
}
int main() {
  size_t bytes = 1ull << 30, nvec = bytes / 16;
  f4 *a, *b; CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0, bytes)); CK(hipMemset(b, 0, bytes));
  double algo = 3.0 * bytes;
  auto rep = [&](const char *n, float ms) { printf("%-34s %8.3f ms %8.1f GB/s\n", n, ms, algo / ms / 1e6); };
  for (int mult : {2, 4, 8, 16, 32}) {
    unsigned g = 256 * mult; char nm[64];
    sprintf(nm, "gs U1 grid %u", g); rep(nm, timeit([&] { k_gs<1, false><<<g, 256>>>(a, b, nvec); }, 20));
    sprintf(nm, "gs U2 grid %u", g); rep(nm, timeit([&] { k_gs<2, false><<<g, 256>>>(a, b, nvec); }, 20));
    sprintf(nm, "gs U4 grid %u", g); rep(nm, timeit([&] { k_gs<4, false><<<g, 256>>>(a, b, nvec); }, 20));
    sprintf(nm, "gs U8 grid %u", g); rep(nm, timeit([&] { k_gs<8, false><<<g, 256>>>(a, b, nvec); }, 20));
    sprintf(nm, "gs U4 NT grid %u", g); rep(nm, timeit([&] { k_gs<4, true><<<g, 256>>>(a, b, nvec); }, 20));
  }
  rep("chunk U1", timeit([&] { k_chunk<1><<<(nvec + 255) / 256, 256>>>(a, b, nvec); }, 20));
  rep("chunk U2", timeit([&] { k_chunk<2><<<(nvec + 511) / 512, 256>>>(a, b, nvec); }, 20));
  rep("chunk U4", timeit([&] { k_chunk<4><<<(nvec + 1023) / 1024, 256>>>(a, b, nvec); }, 20));
  rep("chunk U8", timeit([&] { k_chunk<8><<<(nvec + 2047) / 2048, 256>>>(a, b, nvec); }, 20));
  rep("hipMemcpy D2D 1GiB (2/3 algo)", timeit([&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice); }, 20) * 1.5f);
  return 0;
}
