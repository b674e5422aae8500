// pattern_floor_probe.hip -- diagnostic (not product): the write floor of a
// gapped UNPACK for the exact user layout of a datatype, independent of the
// convertor's kernels.  A type is given as (user offset, bytes) blocks of one
// instance + the extent; `count` instances cover 1 GiB of packed data.
//   full      every byte of the user span written (16 B per lane): the
//             no-gap reference
//   dw        each 4 B of data one store, lanes in stream order (a wave
//             writes 256 consecutive data bytes): store-only floor
//   piece     the data cut into naturally aligned 16/8/4-byte pieces (the
//             convertor's piece kernel's cut), one store per lane
//   piece_rd  piece + each lane first loads its packed bytes (coalesced
//             16-byte loads of the 1 GiB packed stream): reads + writes
// Types: blacs (ref_blacs_indexed: 6 x 52 B every 88 B, then 48..4 B every
// 92 B, extent 1548, 624 B of data), struct48 (char @0, 28 B @8, extent 48),
// u4s32 (16 B every 32 B: vector_f32_b4_s8's blocks without its instance
// seam), v97 (vector_f32_b4_s8 exactly: 97 x 16 B every 32 B, extent 3088).
// Prints the median of 7 timed launches per variant (HIP events).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kB = 256;

struct Piece { uint32_t uoff, soff; uint32_t lg; uint32_t pad; };
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ void k_full(uint4 *d, size_t n) {
  size_t i = (size_t)blockIdx.x * kB + threadIdx.x;
  if (i < n) d[i] = make_uint4(i, i, i, i);
}

// one dword per lane: dword k of instance i at user + i * ext + dw[k]
__global__ void k_dw(char *u, const uint32_t *dw, uint32_t ndw, int64_t ext, size_t n) {
  size_t t = (size_t)blockIdx.x * kB + threadIdx.x;
  if (t >= n) return;
  const size_t inst = t / ndw;
  const uint32_t k = (uint32_t)(t - inst * ndw);
  *reinterpret_cast<uint32_t *>(u + inst * ext + dw[k]) = (uint32_t)t;
}

// RD: 0 store only, 1 one aligned 16 B load of the piece's granule, 2 the
// one or two granules holding the piece's bytes + byte extraction (what a
// direct-load unpack kernel must do), 3 as 1 with a non-temporal load.
// NTS: non-temporal stores.
template <int RD, bool NTS>
__global__ void k_piece(char *u, const char *packed, const Piece *pc, uint32_t npi, int64_t ext, uint32_t S, size_t n) {
  size_t t = (size_t)blockIdx.x * kB + threadIdx.x;
  if (t >= n) return;
  const size_t inst = t / npi;
  const Piece p = pc[t - inst * npi];
  char *d = u + inst * ext + p.uoff;
  uint4 v = make_uint4((uint32_t)t, 1, 2, 3);
  const char *s = packed + inst * S + p.soff;
  const uint4 *g = reinterpret_cast<const uint4 *>((uintptr_t)s & ~(uintptr_t)15);
  if (RD == 1 || RD == 3) {   // the packed bytes of this piece (aligned as in the stream's 16 B granule)
    const v4u a = RD == 3 ? __builtin_nontemporal_load(reinterpret_cast<const v4u *>(g)) : *reinterpret_cast<const v4u *>(g);
    v.x ^= a.x; v.y ^= a.y; v.z ^= a.z; v.w ^= a.w;
  } else if (RD == 2) {
    const uint32_t sh = (uint32_t)((uintptr_t)s & 15), nb = 1u << p.lg;
    const uint4 a = g[0];
    const uint4 b = (sh + nb > 16) ? g[1] : make_uint4(0, 0, 0, 0);
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t q = sh >> 2, r8 = (sh & 3) * 8;
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t lo = w[(q + k) & 7], hi = w[(q + k + 1) & 7];
      o[k] = r8 ? (lo >> r8) | (hi << (32 - r8)) : lo;
    }
    v = make_uint4(o[0], o[1], o[2], o[3]);
  }
  switch (p.lg) {
    case 2: if (NTS) __builtin_nontemporal_store(v.x, reinterpret_cast<uint32_t *>(d)); else *reinterpret_cast<uint32_t *>(d) = v.x; break;
    case 3: if (NTS) { __builtin_nontemporal_store(v.x, reinterpret_cast<uint32_t *>(d)); __builtin_nontemporal_store(v.y, reinterpret_cast<uint32_t *>(d) + 1); }
            else *reinterpret_cast<uint2 *>(d) = make_uint2(v.x, v.y); break;
    default: {
      const v4u x = {v.x, v.y, v.z, v.w};
      if (NTS) __builtin_nontemporal_store(x, reinterpret_cast<v4u *>(d)); else *reinterpret_cast<uint4 *>(d) = v;
      break;
    }
  }
}

int main(int argc, char **argv) {
  const char *type = argc > 1 ? argv[1] : "blacs";
  std::vector<std::pair<uint32_t, uint32_t>> blocks;
  int64_t ext = 0;
  if (!strcmp(type, "blacs")) {
    for (int k = 0; k < 6; k++) blocks.push_back({(uint32_t)(88 * k), 52});
    for (int k = 0; k < 12; k++) blocks.push_back({(uint32_t)(532 + 92 * k), (uint32_t)(48 - 4 * k)});
    ext = 1548;
  } else if (!strcmp(type, "u4s32")) {   // vector_f32_b4_s8: 16 B every 32 B
    blocks.push_back({0, 16});
    ext = 32;
  } else if (!strcmp(type, "v97")) {     // vector_f32_b4_s8 as committed
    for (int k = 0; k < 97; k++) blocks.push_back({(uint32_t)(32 * k), 16});
    ext = 3088;
  } else if (!strcmp(type, "struct48")) {
    blocks.push_back({0, 1});
    blocks.push_back({8, 28});
    ext = 48;
  } else {
    printf("unknown type %s\n", type);
    return 2;
  }
  uint32_t S = 0;
  for (auto &b : blocks) S += b.second;
  const size_t count = ((size_t)1 << 30) / S;
  const size_t span = count * ext;
  // dwords (blacs: every block is 4-aligned, a multiple of 4)
  std::vector<uint32_t> dw;
  bool dw_ok = true;
  for (auto &b : blocks) {
    if (b.first % 4 || b.second % 4) dw_ok = false;
    for (uint32_t o = 0; o + 4 <= b.second; o += 4) dw.push_back(b.first + o);
  }
  // pieces: the user base is 16-aligned; cut each block at natural alignment
  std::vector<Piece> pc;
  uint32_t soff = 0;
  for (auto &b : blocks) {
    uint32_t o = b.first, left = b.second;
    while (left) {
      uint32_t lg = 4;
      while (lg > 0 && ((o % (1u << lg)) || (1u << lg) > left)) lg--;
      if (lg < 2) lg = 2;    // sub-dword pieces written as a dword (diagnostic only: same lines touched)
      const uint32_t n = std::min(1u << lg, left);
      pc.push_back({o, soff, lg, 0});
      o += n; soff += n; left -= n;
    }
  }
  char *u = nullptr, *packed = nullptr;
  uint32_t *ddw = nullptr;
  Piece *dpc = nullptr;
  CK(hipMalloc(&u, span + 64));
  CK(hipMalloc(&packed, count * S + 64));
  CK(hipMemset(u, 0, span + 64));
  CK(hipMemset(packed, 1, count * S + 64));
  CK(hipMalloc(&ddw, dw.size() * 4 + 4));
  CK(hipMalloc(&dpc, pc.size() * sizeof(Piece)));
  CK(hipMemcpy(ddw, dw.data(), dw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpc, pc.data(), pc.size() * sizeof(Piece), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char *name, auto launch) {
    launch();
    (void)hipDeviceSynchronize();
    std::vector<float> ts;
    for (int r = 0; r < 7; r++) {
      (void)hipEventRecord(e0, 0);
      launch();
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[3] * 1e3;
    printf("%-6s %-9s %9.1f us  data %.3f GiB  span %.3f GiB  (span %7.1f GB/s, 2x packed %7.1f GB/s)\n", type, name,
           us, (double)count * S / (1 << 30), (double)span / (1 << 30), span / us / 1e3, 2.0 * count * S / us / 1e3);
  };
  timeit("full", [&] { size_t n = span / 16; hipLaunchKernelGGL(k_full, dim3((n + kB - 1) / kB), dim3(kB), 0, 0, (uint4 *)u, n); });
  if (dw_ok)
    timeit("dw", [&] { size_t n = count * dw.size(); hipLaunchKernelGGL(k_dw, dim3((n + kB - 1) / kB), dim3(kB), 0, 0, u, ddw, (uint32_t)dw.size(), ext, n); });
#define PV(NAME, RD, NTS) timeit(NAME, [&] { size_t n = count * pc.size(); hipLaunchKernelGGL((k_piece<RD, NTS>), dim3((n + kB - 1) / kB), dim3(kB), 0, 0, u, packed, dpc, (uint32_t)pc.size(), ext, S, n); })
  PV("piece", 0, false);
  PV("piece_nts", 0, true);
  PV("piece_rd", 1, false);
  PV("piece_rdnt", 3, false);
  PV("piece_ld2", 2, false);
  PV("pc_ld2nts", 2, true);
  printf("%-6s pieces/instance %zu, dwords/instance %zu, %zu instances\n", type, pc.size(), dw.size(), count);
  return 0;
}
