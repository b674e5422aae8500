// sector_probe.hip -- diagnostic (not product): what HBM write traffic and
// time does a gapped store pattern cost on gfx950, independent of the
// convertor?  Each pattern stores into a span of a large destination buffer;
// run once for time (HIP events) and under `rocprofv3 --pmc WRITE_SIZE` for
// the bytes that leave L2 (profiles/r02/sector_probe.txt).
//   full         16 B per lane, contiguous                    (data = span)
//   dw_s8        4 B every 8 B, one store per lane             (data = span/2)
//   dw_s8_2pass  4 B at 8i, then 4 B at 8i+4, same lane       (data = span)
//   u4_s32       16 B every 32 B                               (data = span/2)
//   u4x2_s64     32 B every 64 B (two 16 B stores per lane)    (data = span/2)
//   struct48     char@0, 3 x u64 @8..31, u32 @32 every 48 B   (data = 29/48 span)
//   struct48_fm  the same bytes, field-major: a wave writes field f of 64
//                consecutive instances before field f+1
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kB = 256;

__global__ void k_full(uint4 *d, size_t n) {
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) d[i] = make_uint4(i, i, i, i);
}
__global__ void k_dw_s8(uint32_t *d, size_t n) {
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) d[2 * i] = (uint32_t)i;
}
__global__ void k_dw_s8_2pass(uint32_t *d, size_t n) {
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) {
    d[2 * i] = (uint32_t)i;
    __builtin_amdgcn_s_waitcnt(0);
    d[2 * i + 1] = (uint32_t)~i;
  }
}
__global__ void k_u4_s32(uint4 *d, size_t n) {
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) d[2 * i] = make_uint4(i, i, i, i);
}
__global__ void k_u4x2_s64(uint4 *d, size_t n) {
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) {
    d[4 * i] = make_uint4(i, i, i, i);
    d[4 * i + 1] = make_uint4(i, i, i, i);
  }
}
__global__ void k_struct48(char *d, size_t n) {
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) {
    char *p = d + 48 * i;
    p[0] = (char)i;
    reinterpret_cast<uint64_t *>(p + 8)[0] = i;
    reinterpret_cast<uint64_t *>(p + 8)[1] = i;
    reinterpret_cast<uint64_t *>(p + 8)[2] = i;
    reinterpret_cast<uint32_t *>(p + 32)[0] = (uint32_t)i;
  }
}
// field-major: lane l of a wave writes 8-byte piece l of 64/5 consecutive
// instances' [char | d0 | d1 | d2 | int] pieces, so one store instruction
// covers a contiguous stretch of pieces
__global__ void k_struct48_fm(char *d, size_t n) {
  const size_t w = ((size_t)blockIdx.x * kB + threadIdx.x) / 64;   // wave id
  const int l = threadIdx.x & 63;
  const size_t inst0 = w * 64;
  for (int k = 0; k < 5; k++) {               // piece p = k*64 + l of 320
    const int p = k * 64 + l;
    const size_t inst = inst0 + p / 5;
    if (inst >= n) continue;
    char *q = d + 48 * inst;
    switch (p % 5) {
      case 0: q[0] = (char)inst; break;
      case 1: reinterpret_cast<uint64_t *>(q + 8)[0] = inst; break;
      case 2: reinterpret_cast<uint64_t *>(q + 8)[1] = inst; break;
      case 3: reinterpret_cast<uint64_t *>(q + 8)[2] = inst; break;
      default: reinterpret_cast<uint32_t *>(q + 32)[0] = (uint32_t)inst; break;
    }
  }
}

int main() {
  const size_t span = (size_t)2 << 30;
  char *d;
  if (hipMalloc(&d, span) != hipSuccess) return 1;
  hipMemset(d, 0, span);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char *name, double data, double spanb, auto launch) {
    launch();
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      hipEventRecord(e0, 0);
      launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    printf("%-12s %8.1f us  data %6.3f GiB (%6.1f GB/s)  span %6.3f GiB (%6.1f GB/s)\n", name, best * 1e3,
           data / (1 << 30), data / (best * 1e-3) / 1e9, spanb / (1 << 30), spanb / (best * 1e-3) / 1e9);
  };
  const size_t nfull = span / 16, ndw = span / 8, nu4 = span / 32, nu42 = span / 64, ns = span / 48;
  auto g = [](size_t n) { return dim3((unsigned)((n + kB - 1) / kB)); };
  run("full", span, span, [&] { hipLaunchKernelGGL(k_full, g(nfull), dim3(kB), 0, 0, (uint4 *)d, nfull); });
  run("dw_s8", span / 2, span, [&] { hipLaunchKernelGGL(k_dw_s8, g(ndw), dim3(kB), 0, 0, (uint32_t *)d, ndw); });
  run("dw_s8_2pass", span, span,
      [&] { hipLaunchKernelGGL(k_dw_s8_2pass, g(ndw), dim3(kB), 0, 0, (uint32_t *)d, ndw); });
  run("u4_s32", span / 2, span, [&] { hipLaunchKernelGGL(k_u4_s32, g(nu4), dim3(kB), 0, 0, (uint4 *)d, nu4); });
  run("u4x2_s64", span / 2, span, [&] { hipLaunchKernelGGL(k_u4x2_s64, g(nu42), dim3(kB), 0, 0, (uint4 *)d, nu42); });
  run("struct48", ns * 29.0, ns * 48.0, [&] { hipLaunchKernelGGL(k_struct48, g(ns), dim3(kB), 0, 0, d, ns); });
  run("struct48_fm", ns * 29.0, ns * 48.0,
      [&] { hipLaunchKernelGGL(k_struct48_fm, g(ns * 5 / 5), dim3(kB), 0, 0, d, ns); });
  hipFree(d);
  return 0;
}
