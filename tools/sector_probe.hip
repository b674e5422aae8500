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
//   *_pf         round 3: the same stores, after each lane has loaded the
//                span it is about to write (coalesced loads, values kept
//                live): does a line that is valid in L2 leave as a whole?
//   sp48_1112    48 B (6 x u64) every 1112 B: the matrix-borders unpack
//                pattern (ref_matrix_borders_20_3), data 4.3 % of the span
//   sp48_1112_pfg  the same, the 16-byte granules under the block loaded first
//   sp48_1112_pfl  the same, the whole 128-byte line(s) under the block loaded first
//   sp48_1112_pf64 the same, the 64-byte granule(s) under the block loaded first
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

__device__ __forceinline__ void keep(uint32_t v) { asm volatile("" : : "v"(v)); }

__global__ void k_dw_s8_pf(uint32_t *d, size_t n) {
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) {
    const uint2 v = reinterpret_cast<const uint2 *>(d)[i];
    keep(v.x ^ v.y);
    d[2 * i] = (uint32_t)i;
  }
}
__global__ void k_u4_s32_pf(uint4 *d, size_t n) {
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) {
    const uint4 a = d[2 * i], b = d[2 * i + 1];
    keep(a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w);
    d[2 * i] = make_uint4(i, i, i, i);
  }
}
__global__ void k_struct48_pf(char *d, size_t n) {
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) {
    char *p = d + 48 * i;
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    const uint4 a = q[0], b = q[1], c = q[2];
    keep(a.x ^ a.w ^ b.y ^ b.z ^ c.x ^ c.w);
    p[0] = (char)i;
    reinterpret_cast<uint64_t *>(p + 8)[0] = i;
    reinterpret_cast<uint64_t *>(p + 8)[1] = i;
    reinterpret_cast<uint64_t *>(p + 8)[2] = i;
    reinterpret_cast<uint32_t *>(p + 32)[0] = (uint32_t)i;
  }
}
// MODE 0: stores only; 1: the 16-byte granules under the block loaded first;
// 2: the whole 128-byte lines under the block loaded first; 3: the 64-byte
// granules under the block loaded first
template <int MODE>
__global__ void k_sp48(char *d, size_t n) {
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) {
    uint64_t *p = reinterpret_cast<uint64_t *>(d + 1112 * i);
    if (MODE) {
      const uintptr_t a = (uintptr_t)p, e = a + 48;
      const uintptr_t m = MODE == 1 ? 15 : MODE == 2 ? 127 : 63;
      const uintptr_t lo = a & ~m, hi = (e + m) & ~m;
      uint32_t x = 0;
      for (uintptr_t g = lo; g < hi; g += 16) {
        const uint4 v = *reinterpret_cast<const uint4 *>(g);
        x ^= v.x ^ v.w;
      }
      keep(x);
    }
#pragma unroll
    for (int k = 0; k < 6; k++) p[k] = i + k;
  }
}

// the same 48-byte blocks every 1112 bytes, read instead of written (pack side)
__global__ void k_sp48_ld(const char *d, size_t n, uint32_t *sink) {
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) {
    const uint64_t *p = reinterpret_cast<const uint64_t *>(d + 1112 * i);
    uint64_t x = 0;
#pragma unroll
    for (int k = 0; k < 6; k++) x ^= p[k];
    if (x == 0x9e3779b97f4a7c15ull) sink[0] = 1;
  }
}

int main(int argc, char **argv) {
  // `sector_probe big`: a 24 GiB span (the user span of ref_matrix_borders_20_3
  // at 1 GiB packed is 23.2 GiB): full stores and the sparse patterns only
  const bool big = argc > 1 && argv[1][0] == 'b';
  const size_t span = big ? (size_t)24 << 30 : (size_t)2 << 30;
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
  const size_t nsp = (span - 256) / 1112;
  uint32_t *sink;
  if (hipMalloc(&sink, 4) != hipSuccess) return 1;
  if (big) {
    run("full", span, span, [&] { hipLaunchKernelGGL(k_full, g(nfull), dim3(kB), 0, 0, (uint4 *)d, nfull); });
    run("sp48_1112", nsp * 48.0, nsp * 1112.0, [&] { hipLaunchKernelGGL(k_sp48<0>, g(nsp), dim3(kB), 0, 0, d, nsp); });
    run("sp48_1112_ld", nsp * 48.0, nsp * 1112.0,
        [&] { hipLaunchKernelGGL(k_sp48_ld, g(nsp), dim3(kB), 0, 0, d, nsp, sink); });
    hipFree(d);
    return 0;
  }
  run("full", span, span, [&] { hipLaunchKernelGGL(k_full, g(nfull), dim3(kB), 0, 0, (uint4 *)d, nfull); });
  run("dw_s8", span / 2, span, [&] { hipLaunchKernelGGL(k_dw_s8, g(ndw), dim3(kB), 0, 0, (uint32_t *)d, ndw); });
  run("dw_s8_2pass", span, span,
      [&] { hipLaunchKernelGGL(k_dw_s8_2pass, g(ndw), dim3(kB), 0, 0, (uint32_t *)d, ndw); });
  run("u4_s32", span / 2, span, [&] { hipLaunchKernelGGL(k_u4_s32, g(nu4), dim3(kB), 0, 0, (uint4 *)d, nu4); });
  run("u4x2_s64", span / 2, span, [&] { hipLaunchKernelGGL(k_u4x2_s64, g(nu42), dim3(kB), 0, 0, (uint4 *)d, nu42); });
  run("struct48", ns * 29.0, ns * 48.0, [&] { hipLaunchKernelGGL(k_struct48, g(ns), dim3(kB), 0, 0, d, ns); });
  run("struct48_fm", ns * 29.0, ns * 48.0,
      [&] { hipLaunchKernelGGL(k_struct48_fm, g(ns * 5 / 5), dim3(kB), 0, 0, d, ns); });
  run("dw_s8_pf", span / 2, span, [&] { hipLaunchKernelGGL(k_dw_s8_pf, g(ndw), dim3(kB), 0, 0, (uint32_t *)d, ndw); });
  run("u4_s32_pf", span / 2, span, [&] { hipLaunchKernelGGL(k_u4_s32_pf, g(nu4), dim3(kB), 0, 0, (uint4 *)d, nu4); });
  run("struct48_pf", ns * 29.0, ns * 48.0, [&] { hipLaunchKernelGGL(k_struct48_pf, g(ns), dim3(kB), 0, 0, d, ns); });
  run("sp48_1112_ld", nsp * 48.0, nsp * 1112.0,
      [&] { hipLaunchKernelGGL(k_sp48_ld, g(nsp), dim3(kB), 0, 0, d, nsp, sink); });
  run("sp48_1112", nsp * 48.0, nsp * 1112.0, [&] { hipLaunchKernelGGL(k_sp48<0>, g(nsp), dim3(kB), 0, 0, d, nsp); });
  run("sp48_1112_pfg", nsp * 48.0, nsp * 1112.0, [&] { hipLaunchKernelGGL(k_sp48<1>, g(nsp), dim3(kB), 0, 0, d, nsp); });
  run("sp48_1112_pfl", nsp * 48.0, nsp * 1112.0, [&] { hipLaunchKernelGGL(k_sp48<2>, g(nsp), dim3(kB), 0, 0, d, nsp); });
  run("sp48_1112_pf64", nsp * 48.0, nsp * 1112.0, [&] { hipLaunchKernelGGL(k_sp48<3>, g(nsp), dim3(kB), 0, 0, d, nsp); });
  hipFree(d);
  return 0;
}
