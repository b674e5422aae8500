// pack_floor_probe.hip -- diagnostic (not product): the HBM floor of a PACK
// of a layout whose user span is `span` bytes for `packed` packed bytes
// (VERDICT r4 next 3).  A pack must read the user span (every line holding
// data; for the CFG-C types that is the whole span) and write the packed
// stream once.  The floor kernel does exactly that with no layout work:
// lane k writes packed granule k (16 B) and reads span granules
// [k*r, (k+1)*r) (r = span / packed, coalesced: a wave reads 64*r*16
// consecutive bytes), xor-folding them so no load is dead.
//   plain   cached loads and stores
//   nt      non-temporal loads and stores (the product's policy at >= 384 MiB)
// usage: pack_floor_probe NAME SPAN_BYTES PACKED_BYTES [NAME SPAN PACKED ...]
// Prints the median of 9 timed launches per variant (HIP events), the time,
// and GB/s as 2 x packed (algorithmic, the product's unit) and as
// span + packed (bytes moved).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int kB = 256;

template <bool NT>
__global__ void __launch_bounds__(kB) k_floor(const v4u *span, uint64_t nspan, v4u *packed, uint64_t npk,
                                              uint64_t r_num, uint64_t r_den) {
  const uint64_t k = (uint64_t)blockIdx.x * kB + threadIdx.x;
  if (k >= npk) return;
  uint64_t j0 = k * r_num / r_den, j1 = (k + 1) * r_num / r_den;
  if (j1 > nspan) j1 = nspan;
  v4u acc = {(uint32_t)k, 0, 0, 0};
  for (uint64_t j = j0; j < j1; j++) {
    const v4u v = NT ? __builtin_nontemporal_load(span + j) : span[j];
    acc ^= v;
  }
  if (NT) __builtin_nontemporal_store(acc, packed + k);
  else packed[k] = acc;
}

// split: the two streams each perfectly coalesced (consecutive lanes on
// consecutive granules, grid-stride), the span folded per thread into what
// it stores -- the plain streaming floor of reading `span` + writing `packed`
template <bool NT>
__global__ void __launch_bounds__(kB) k_floor_split(const v4u *span, uint64_t nspan, v4u *packed, uint64_t npk) {
  const uint64_t nth = (uint64_t)gridDim.x * kB, k0 = (uint64_t)blockIdx.x * kB + threadIdx.x;
  v4u acc = {(uint32_t)k0, 0, 0, 0};
  for (uint64_t j = k0; j < nspan; j += nth) acc ^= NT ? __builtin_nontemporal_load(span + j) : span[j];
  for (uint64_t k = k0; k < npk; k += nth) {
    const v4u v = acc + (uint32_t)k;
    if (NT) __builtin_nontemporal_store(v, packed + k);
    else packed[k] = v;
  }
}

int main(int argc, char **argv) {
  if (argc < 4 || (argc - 1) % 3) {
    printf("usage: %s NAME SPAN_BYTES PACKED_BYTES [...]\n", argv[0]);
    return 2;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int a = 1; a + 2 < argc; a += 3) {
    const char *name = argv[a];
    const uint64_t span = strtoull(argv[a + 1], nullptr, 0), pk = strtoull(argv[a + 2], nullptr, 0);
    const uint64_t nspan = (span + 15) / 16, npk = (pk + 15) / 16;
    v4u *s = nullptr, *p = nullptr;
    CK(hipMalloc(&s, nspan * 16));
    CK(hipMalloc(&p, npk * 16));
    CK(hipMemset(s, 1, nspan * 16));
    CK(hipMemset(p, 0, npk * 16));
    // PFP_SHIFT=16: the span starts 16 bytes past a 128-byte line (as a
    // product tile's 16-aligned span usually does)
    const uint64_t shift = getenv("PFP_SHIFT") ? strtoull(getenv("PFP_SHIFT"), nullptr, 0) / 16 : 0;
    const v4u *ss = s + shift;
    const uint64_t nss = nspan - shift;
    for (int mode = 0; mode < 4; mode++) {
      const int nt = mode & 1, split = mode >> 1;
      auto launch = [&] {
        const dim3 g((unsigned)((npk + kB - 1) / kB)), b(kB);
        const dim3 gs((unsigned)(256 * 8)), bs(kB);
        if (split && nt) hipLaunchKernelGGL(k_floor_split<true>, gs, bs, 0, 0, ss, nss, p, npk);
        else if (split) hipLaunchKernelGGL(k_floor_split<false>, gs, bs, 0, 0, ss, nss, p, npk);
        else if (nt) hipLaunchKernelGGL(k_floor<true>, g, b, 0, 0, ss, nss, p, npk, nss, npk);
        else hipLaunchKernelGGL(k_floor<false>, g, b, 0, 0, ss, nss, p, npk, nss, npk);
      };
      launch();
      CK(hipDeviceSynchronize());
      std::vector<float> ts;
      for (int r = 0; r < 9; r++) {
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const double us = ts[4] * 1e3;
      printf("%-32s %-11s span %12llu packed %12llu  %9.1f us  2x packed %7.1f GB/s  moved %7.1f GB/s\n", name,
             split ? (nt ? "split-nt" : "split-plain") : (nt ? "nt" : "plain"), (unsigned long long)span, (unsigned long long)pk, us, 2.0 * pk / us / 1e3,
             (double)(span + pk) / us / 1e3);
      fflush(stdout);
    }
    CK(hipFree(s));
    CK(hipFree(p));
  }
  return 0;
}
