// mx_convertor.hip -- K5/K6: derived-datatype pack/unpack on gfx950.
//
// The reference walks its description with an explicit stack and issues one
// memcpy per contiguous block (opal_datatype_pack.c:235-370,
// opal_datatype_pack.h:86-185; unpack :245-427), i.e. one cuMemcpy per block
// on the CUDA path.  Here the committed description is flattened once on the
// host into a table of strided RUNS, in pack order:
//     run = { disp, blen (bytes), cnt1, stride1, cnt2, stride2, poff }
//     block (l2, l1) of a run lives at  origin + disp + l2*stride2 + l1*stride1
// (an ELEM is a 1-level run; a LOOP whose body is one run becomes a 2-level
// run; other loops are unrolled).  One kernel launch then moves every
// 16-byte granule of the packed stream: the lane maps its packed offset to
// (instance, run, block, byte) with a binary search over the run table
// staged in LDS, gathers the granule with the widest access the layout
// allows (`UNIT` = 16/8/4/2/1 bytes, chosen on the host from the gcd of all
// displacements, strides and block sizes) into registers, and writes one
// coalesced 16-byte store (unpack: one 16-byte load, scattered stores).
// Algorithmic bytes per launch: 2 * packed bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>

#include "mx_internal.h"
#include "../../include/mx_convertor.h"

namespace mx {

struct DRun {
  int64_t disp;
  uint64_t blen;     // bytes per block
  uint64_t cnt1;     // inner block count
  int64_t stride1;
  uint64_t cnt2;     // outer repetition count
  int64_t stride2;
  uint64_t poff;     // packed offset of the run within one instance
  uint64_t bytes;    // blen * cnt1 * cnt2
};

constexpr int kCB = 256;
constexpr int kLdsRuns = 1024;   // 64 KiB of LDS

struct Pos {
  uint64_t inst, b, o;
  int r;
};

__device__ __forceinline__ int find_run(const DRun *runs, int n, uint64_t q) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (runs[mid].poff <= q) lo = mid; else hi = mid - 1;
  }
  return lo;
}

template <int UNIT> struct unit_t;
template <> struct unit_t<16> { using T = uint4; };
template <> struct unit_t<8> { using T = uint64_t; };
template <> struct unit_t<4> { using T = uint32_t; };
template <> struct unit_t<2> { using T = uint16_t; };
template <> struct unit_t<1> { using T = uint8_t; };

// One lane = one 16-byte granule of the packed buffer: granule g covers
// packed[g*16, g*16+16) = stream bytes [offset + g*16, ...).  The granule is
// staged in 16/UNIT registers (compile-time indexed, no scratch): PACK
// gathers UNIT-sized pieces from the user layout and stores the granule
// with one 16-byte access; UNPACK loads it with one access and scatters.
template <int UNIT, bool PACK>
__global__ void __launch_bounds__(kCB)
k_convert(const DRun *__restrict__ gruns, int nruns, uint64_t S, int64_t extent, char *user, char *packed,
          uint64_t offset, uint64_t len, int pk_vec) {
  using U = typename unit_t<UNIT>::T;
  constexpr int K = 16 / UNIT;
  __shared__ DRun sruns[kLdsRuns];
  const DRun *runs = gruns;
  if (nruns <= kLdsRuns) {
    for (int i = threadIdx.x; i < nruns; i += kCB) sruns[i] = gruns[i];
    __syncthreads();
    runs = sruns;
  }
  const uint64_t g = (uint64_t)blockIdx.x * kCB + threadIdx.x;
  const uint64_t rel0 = g * 16;
  if (rel0 >= len) return;
  const uint64_t n = (len - rel0) < 16 ? (len - rel0) : 16;
  const bool full = (n == 16) && pk_vec;
  const uint64_t p = offset + rel0;
  uint64_t inst = p / S;
  const uint64_t q = p - inst * S;
  int r = find_run(runs, nruns, q);
  DRun R = runs[r];
  const uint64_t w = q - R.poff;
  const uint64_t b = w / R.blen;
  uint64_t o = w - b * R.blen;
  uint64_t l2 = b / R.cnt1, l1 = b - l2 * R.cnt1;
  U regs[K];
  if (!PACK) {
    if (full) {
      const uint4 v = *reinterpret_cast<const uint4 *>(packed + rel0);
      memcpy(regs, &v, 16);
    } else {
#pragma unroll
      for (int k = 0; k < K; k++)
        if ((uint64_t)k * UNIT < n) regs[k] = *reinterpret_cast<const U *>(packed + rel0 + k * UNIT);
    }
  }
#pragma unroll
  for (int k = 0; k < K; k++) {
    if ((uint64_t)k * UNIT < n) {
      char *a = user + (int64_t)inst * extent + R.disp + (int64_t)l2 * R.stride2 + (int64_t)l1 * R.stride1 + o;
      if (PACK) regs[k] = *reinterpret_cast<const U *>(a);
      else *reinterpret_cast<U *>(a) = regs[k];
      o += UNIT;
      if (o == R.blen) {
        o = 0;
        if (++l1 == R.cnt1) {
          l1 = 0;
          if (++l2 == R.cnt2) {
            l2 = 0;
            if (++r == nruns) { r = 0; inst++; }
            R = runs[r];
          }
        }
      }
    }
  }
  if (PACK) {
    if (full) {
      uint4 v;
      memcpy(&v, regs, 16);
      *reinterpret_cast<uint4 *>(packed + rel0) = v;
    } else {
#pragma unroll
      for (int k = 0; k < K; k++)
        if ((uint64_t)k * UNIT < n) *reinterpret_cast<U *>(packed + rel0 + k * UNIT) = regs[k];
    }
  }
}

}  // namespace mx

using namespace mx;

struct mx_ddt {
  std::vector<DRun> host;
  DRun *dev;
  size_t size;
  int64_t lb, ub;
  uint64_t gcd_all;  // gcd of every disp/stride/blen/extent (access unit)
};

namespace {

// dt_elem_desc record views (opal_datatype_internal.h:146-196)
struct RecElem { uint16_t flags, type; uint32_t count; uint64_t blocklen; int64_t extent; int64_t disp; };
struct RecLoop { uint16_t flags, type; uint32_t items; uint32_t loops; uint32_t pad; uint64_t unused; int64_t extent; };
static_assert(sizeof(RecElem) == 32 && sizeof(RecLoop) == 32, "dt_elem_desc is 32 bytes");

constexpr uint16_t T_LOOP = 0, T_END_LOOP = 1, T_LB = 2, T_UB = 3;
constexpr uint16_t F_DATA = 0x0100;
constexpr size_t kMaxRuns = (size_t)1 << 22;

static const uint64_t kBasicLP64[MX_OPAL_NBASIC] = {
    0, 0, 0, 0,            // LOOP END_LOOP LB UB
    1, 2, 4, 8, 16,        // INT1 INT2 INT4 INT8 INT16
    1, 2, 4, 8, 16,        // UINT1 .. UINT16
    2, 4, 8, 16, 16,       // FLOAT2 FLOAT4 FLOAT8 FLOAT12 (long double: 16 B) FLOAT16
    4, 8, 16, 32,          // SHORT_FLOAT_COMPLEX FLOAT_COMPLEX DOUBLE_COMPLEX LONG_DOUBLE_COMPLEX
    1, 4, 0                // BOOL WCHAR UNAVAILABLE
};

static bool contiguous_single(const DRun &r) { return r.cnt1 == 1 && r.cnt2 == 1; }

static void push_run(std::vector<DRun> &out, DRun r) {
  if (r.bytes == 0) return;
  // a 1-level run whose blocks touch is one contiguous block
  if (r.cnt2 == 1 && r.cnt1 > 1 && r.stride1 == (int64_t)r.blen) { r.blen *= r.cnt1; r.cnt1 = 1; r.stride1 = 0; }
  if (!out.empty()) {
    DRun &p = out.back();
    if (contiguous_single(p) && contiguous_single(r) && p.disp + (int64_t)p.blen == r.disp) {
      p.blen += r.blen;
      p.bytes += r.bytes;
      return;
    }
  }
  out.push_back(r);
}

static int flatten(const uint8_t *recs, size_t lo, size_t hi, int64_t base, const uint64_t *bs,
                   std::vector<DRun> &out) {
  size_t i = lo;
  while (i < hi) {
    RecElem e;
    memcpy(&e, recs + 32 * i, 32);
    if (e.type == T_END_LOOP) return MX_SUCCESS;   // terminator of this level
    if (e.type == T_LOOP) {
      RecLoop L;
      memcpy(&L, recs + 32 * i, 32);
      if (L.items == 0 || i + L.items >= hi + 1) return MX_ERR_ARG;
      std::vector<DRun> body;
      int rc = flatten(recs, i + 1, i + L.items, 0, bs, body);
      if (rc) return rc;
      if (body.size() == 1 && body[0].cnt2 == 1) {
        DRun r = body[0];
        r.disp += base;
        if (contiguous_single(r)) {          // loop of one contiguous block
          r.cnt1 = L.loops;
          r.stride1 = L.extent;
        } else {
          r.cnt2 = L.loops;
          r.stride2 = L.extent;
        }
        r.bytes = r.blen * r.cnt1 * r.cnt2;
        push_run(out, r);
      } else {
        if (out.size() + body.size() * (size_t)L.loops > kMaxRuns) return MX_ERR_UNSUPPORTED;
        for (uint32_t l = 0; l < L.loops; l++)
          for (DRun r : body) {
            r.disp += base + (int64_t)l * L.extent;
            push_run(out, r);
          }
      }
      i += L.items + 1;
      continue;
    }
    if (e.type == T_LB || e.type == T_UB || !(e.flags & F_DATA)) { i++; continue; }
    if (e.type >= MX_OPAL_NBASIC || bs[e.type] == 0) return MX_ERR_ARG;
    DRun r;
    r.disp = base + e.disp;
    r.blen = e.blocklen * bs[e.type];
    r.cnt1 = e.count;
    r.stride1 = e.extent;
    r.cnt2 = 1;
    r.stride2 = 0;
    r.bytes = r.blen * r.cnt1;
    push_run(out, r);
    if (out.size() > kMaxRuns) return MX_ERR_UNSUPPORTED;
    i++;
  }
  return MX_SUCCESS;
}

static uint64_t gcd64(uint64_t a, uint64_t b) {
  while (b) { uint64_t t = a % b; a = b; b = t; }
  return a;
}
static uint64_t absg(int64_t v) { return v < 0 ? (uint64_t)(-v) : (uint64_t)v; }

}  // namespace

extern "C" int mx_ddt_create(const void *desc, size_t nrec, const uint64_t *basic_sizes, size_t size, int64_t lb,
                             int64_t ub, mx_ddt_t **out) {
  if (!desc || !nrec || !out) return MX_ERR_ARG;
  const uint64_t *bs = basic_sizes ? basic_sizes : kBasicLP64;
  mx_ddt *d = new (std::nothrow) mx_ddt();
  if (!d) return MX_ERR_NOMEM;
  int rc = flatten((const uint8_t *)desc, 0, nrec, 0, bs, d->host);
  if (rc) { delete d; return rc; }
  uint64_t poff = 0, g = 16;
  for (DRun &r : d->host) {
    r.poff = poff;
    poff += r.bytes;
    g = gcd64(g, absg(r.disp));
    g = gcd64(g, r.blen);
    if (r.cnt1 > 1) g = gcd64(g, absg(r.stride1));
    if (r.cnt2 > 1) g = gcd64(g, absg(r.stride2));
  }
  if (poff != size) { delete d; return MX_ERR_ARG; }   // description / size mismatch
  d->size = size;
  d->lb = lb;
  d->ub = ub;
  d->gcd_all = gcd64(g, absg(ub - lb));
  d->dev = nullptr;
  if (!d->host.empty()) {
    if ((rc = mx_ensure_init())) { delete d; return rc; }
    if (hipMalloc((void **)&d->dev, d->host.size() * sizeof(DRun)) != hipSuccess ||
        hipMemcpy(d->dev, d->host.data(), d->host.size() * sizeof(DRun), hipMemcpyHostToDevice) != hipSuccess) {
      if (d->dev) (void)hipFree(d->dev);
      delete d;
      return MX_ERR_HIP;
    }
  }
  *out = d;
  return MX_SUCCESS;
}

extern "C" int mx_ddt_destroy(mx_ddt_t *d) {
  if (!d) return MX_SUCCESS;
  if (d->dev) (void)hipFree(d->dev);
  delete d;
  return MX_SUCCESS;
}

extern "C" size_t mx_ddt_size(const mx_ddt_t *d) { return d ? d->size : 0; }
extern "C" int64_t mx_ddt_extent(const mx_ddt_t *d) { return d ? d->ub - d->lb : 0; }
extern "C" size_t mx_ddt_runs(const mx_ddt_t *d) { return d ? d->host.size() : 0; }

template <bool PACK>
static int convert(const mx_ddt_t *d, size_t count, char *user, char *packed, size_t offset, size_t len,
                   void *stream) {
  if (!d || !user || !packed) return MX_ERR_ARG;
  if (len == 0) return MX_SUCCESS;
  if (d->size == 0 || offset + len > d->size * count) return MX_ERR_ARG;
  int rc = mx_ensure_init();
  if (rc) return rc;
  // widest unit that every piece of every granule respects: layout gcd,
  // alignment of the user origin, and the stream offset of granule 0
  uint64_t u = gcd64(d->gcd_all, ((uintptr_t)user) & 15 ? ((uintptr_t)user & 15) : 16);
  u = gcd64(u, offset & 15 ? (offset & 15) : 16);
  u = gcd64(u, len & 15 ? (len & 15) : 16);
  if (((uintptr_t)packed & 15) != 0) u = gcd64(u, (uintptr_t)packed & 15);
  const int pk_vec = ((uintptr_t)packed & 15) == 0;
  const int nr = (int)d->host.size();
  const uint64_t g = (len + 15) / 16;
  const dim3 grid((unsigned)((g + kCB - 1) / kCB)), block(kCB);
  hipStream_t s = (hipStream_t)stream;
  const int64_t ext = d->ub - d->lb;
  switch (u) {
    case 16: hipLaunchKernelGGL((k_convert<16, PACK>), grid, block, 0, s, d->dev, nr, d->size, ext, user, packed, offset, len, pk_vec); break;
    case 8: hipLaunchKernelGGL((k_convert<8, PACK>), grid, block, 0, s, d->dev, nr, d->size, ext, user, packed, offset, len, pk_vec); break;
    case 4: hipLaunchKernelGGL((k_convert<4, PACK>), grid, block, 0, s, d->dev, nr, d->size, ext, user, packed, offset, len, pk_vec); break;
    case 2: hipLaunchKernelGGL((k_convert<2, PACK>), grid, block, 0, s, d->dev, nr, d->size, ext, user, packed, offset, len, pk_vec); break;
    default: hipLaunchKernelGGL((k_convert<1, PACK>), grid, block, 0, s, d->dev, nr, d->size, ext, user, packed, offset, len, pk_vec); break;
  }
  return mx_check_launch();
}

extern "C" int mx_pack(const mx_ddt_t *d, size_t count, const void *user, void *packed, size_t offset, size_t len,
                       void *stream) {
  return convert<true>(d, count, (char *)user, (char *)packed, offset, len, stream);
}

extern "C" int mx_unpack(const mx_ddt_t *d, size_t count, void *user, const void *packed, size_t offset,
                         size_t len, void *stream) {
  return convert<false>(d, count, (char *)user, (char *)packed, offset, len, stream);
}
