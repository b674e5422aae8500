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
#include <climits>
#include <algorithm>
#include <mutex>
#include <atomic>
#include <type_traits>

#include "mx_internal.h"
#include "mx_mem.hpp"
#include "../../include/mx_convertor.h"

namespace mx {

// Division by a run-time constant without a 64-bit divide: for numerators
// n < 2^48, floor(n / d) = floor(n * m / 2^k) with k = 48 + ceil(log2 d),
// m = ceil(2^k / d) (Granlund & Montgomery, PLDI'94, thm 4.2).
struct Magic { uint64_t m; uint32_t k; uint32_t pad; };
constexpr int kMagicBits = 48;

__host__ __device__ __forceinline__ uint64_t udiv(uint64_t n, const Magic &M) {
  return (uint64_t)(((unsigned __int128)n * M.m) >> M.k);
}

struct DRun {
  int64_t disp;
  uint64_t blen;     // bytes per block
  uint64_t cnt1;     // inner block count
  int64_t stride1;
  uint64_t cnt2;     // outer repetition count
  int64_t stride2;
  uint64_t poff;     // packed offset of the run within one instance
  uint64_t bytes;    // blen * cnt1 * cnt2
  Magic mblen, mcnt1;
};

constexpr int kCB = 256;
constexpr int kLdsRuns = 512;    // run tables up to 48 KiB are staged in LDS

struct Pos {
  uint64_t inst, l2, l1, o;
  int r;
};

struct ConvArgs {
  const DRun *runs;
  int nruns;
  uint64_t S;        // packed bytes per instance
  Magic mS;
  int64_t ext;       // instance extent
  char *user;
  char *packed;      // receives / holds stream bytes [offset, offset + len)
  uint64_t offset, len;
  int pk_vec;        // packed is 16-byte aligned
  int ntld;          // UNPACK: the packed stream read non-temporal (read once)
};

__device__ __forceinline__ int find_run(const DRun *runs, int n, uint64_t q) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (runs[mid].poff <= q) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// stream position p -> (instance, run, outer block, inner block, byte)
__device__ __forceinline__ Pos map_pos(const DRun *runs, int nruns, uint64_t S, const Magic &mS, uint64_t p) {
  Pos P;
  P.inst = udiv(p, mS);
  const uint64_t q = p - P.inst * S;
  P.r = find_run(runs, nruns, q);
  const DRun &R = runs[P.r];
  const uint64_t w = q - R.poff;
  const uint64_t b = udiv(w, R.mblen);
  P.o = w - b * R.blen;
  P.l2 = udiv(b, R.mcnt1);
  P.l1 = b - P.l2 * R.cnt1;
  return P;
}

__device__ __forceinline__ int64_t block_addr(const Pos &P, const DRun &R, int64_t ext) {
  return (int64_t)P.inst * ext + R.disp + (int64_t)P.l2 * R.stride2 + (int64_t)P.l1 * R.stride1;
}

// advance to the next block after finishing one
__device__ __forceinline__ void next_block(Pos &P, const DRun *runs, int nruns, DRun &R) {
  P.o = 0;
  if (++P.l1 == R.cnt1) {
    P.l1 = 0;
    if (++P.l2 == R.cnt2) {
      P.l2 = 0;
      if (++P.r == nruns) { P.r = 0; P.inst++; }
      R = runs[P.r];
    }
  }
}


template <int UNIT> struct unit_t;
template <> struct unit_t<16> { using T = uint4; };
template <> struct unit_t<8> { using T = uint64_t; };
template <> struct unit_t<4> { using T = uint32_t; };
template <> struct unit_t<2> { using T = uint16_t; };
template <> struct unit_t<1> { using T = uint8_t; };

// 16 bytes at dword alignment: one dwordx4 access where the user address
// is only 4-byte aligned (the compiler picks the instruction for align 4)
struct __attribute__((aligned(4))) W4 { uint32_t x, y, z, w; };

// loads through an explicitly global pointer: global_load (vmcnt only), not
// flat_load, whose lgkmcnt would tie a load in flight to every LDS wait
typedef uint32_t v4u_a16 __attribute__((ext_vector_type(4), aligned(16)));
typedef uint32_t v4u_a4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ uint4 gld16(const char *p) {        // 16-byte aligned
  const v4u_a16 v = *(const __attribute__((address_space(1))) v4u_a16 *)(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <bool NT>
__device__ __forceinline__ uint4 gld16p(const char *p) {       // 16-byte aligned, nt when NT
  if constexpr (NT) {
    const v4u_a16 v = __builtin_nontemporal_load((const __attribute__((address_space(1))) v4u_a16 *)(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return gld16(p);
  }
}
__device__ __forceinline__ W4 gld16a4(const char *p) {         // 4-byte aligned
  const v4u_a4 v = *(const __attribute__((address_space(1))) v4u_a4 *)(p);
  W4 w;
  w.x = v.x; w.y = v.y; w.z = v.z; w.w = v.w;
  return w;
}
__device__ __forceinline__ uint32_t gld4(const char *p) {
  return *(const __attribute__((address_space(1))) uint32_t *)(p);
}
// ... and stores / loads of any unit the same way (16-byte units as a plain
// vector: HIP's vector classes have no address-space-1 assignment)
template <class U>
__device__ __forceinline__ U gload(const char *p) {
  if constexpr (sizeof(U) == 16) {
    const v4u_a16 v = *(const __attribute__((address_space(1))) v4u_a16 *)(p);
    U r;
    __builtin_memcpy(&r, &v, 16);
    return r;
  } else if constexpr (std::is_scalar<U>::value) {
    return *(const __attribute__((address_space(1))) U *)(p);
  } else {   // a small struct: as the unsigned integer of its size
    static_assert(sizeof(U) == 8 || sizeof(U) == 4, "gload: 4, 8 or 16 bytes");
    using I = typename std::conditional<sizeof(U) == 8, uint64_t, uint32_t>::type;
    const I v = *(const __attribute__((address_space(1))) I *)(p);
    U r;
    __builtin_memcpy(&r, &v, sizeof(U));
    return r;
  }
}
template <class U>
__device__ __forceinline__ void gstore(char *p, const U &x) {
  if constexpr (sizeof(U) == 16) {
    v4u_a16 v;
    __builtin_memcpy(&v, &x, 16);
    *(__attribute__((address_space(1))) v4u_a16 *)(p) = v;
  } else {
    *(__attribute__((address_space(1))) U *)(p) = x;
  }
}

// ---------------------------------------------------------------------------
// GRANULE kernel: one lane = one 16-byte granule of the packed buffer
// (granule g = stream bytes [offset + 16g, +16)), staged in 16/UNIT
// registers (compile-time indexed, no scratch).  PACK gathers UNIT-sized
// pieces from the user layout and stores the granule with one 16-byte
// access; UNPACK loads it with one access and scatters.  Used when every
// piece is 16-byte aligned (UNIT = 16: whole-vector moves, no staging) and
// as the per-tile fallback of the TILE kernels.
// ---------------------------------------------------------------------------
template <int UNIT, bool PACK>
__device__ __forceinline__ void convert_granule(const ConvArgs &a, const DRun *runs, uint64_t g) {
  using U = typename unit_t<UNIT>::T;
  constexpr int K = 16 / UNIT;
  const uint64_t rel0 = g * 16;
  if (rel0 >= a.len) return;
  const uint64_t n = (a.len - rel0) < 16 ? (a.len - rel0) : 16;
  const bool full = (n == 16) && a.pk_vec;
  Pos P = map_pos(runs, a.nruns, a.S, a.mS, a.offset + rel0);
  DRun R = runs[P.r];
  U regs[K];
  if (!PACK) {
    if (full) {
      const uint4 v = a.ntld ? gld16p<true>(a.packed + rel0) : gld16(a.packed + rel0);
      memcpy(regs, &v, 16);
    } else {
#pragma unroll
      for (int k = 0; k < K; k++)
        if ((uint64_t)k * UNIT < n) regs[k] = gload<U>(a.packed + rel0 + k * UNIT);
    }
  }
#pragma unroll
  for (int k = 0; k < K; k++) {
    if ((uint64_t)k * UNIT < n) {
      char *p = a.user + block_addr(P, R, a.ext) + P.o;
      if (PACK) regs[k] = gload<U>(p);
      else gstore<U>(p, regs[k]);
      P.o += UNIT;
      if (P.o == R.blen) next_block(P, runs, a.nruns, R);
    }
  }
  if (PACK) {
    if (full) {
      uint4 v;
      memcpy(&v, regs, 16);
      gstore<uint4>(a.packed + rel0, v);
    } else {
#pragma unroll
      for (int k = 0; k < K; k++)
        if ((uint64_t)k * UNIT < n) gstore<U>(a.packed + rel0 + k * UNIT, regs[k]);
    }
  }
}

// RL: the run table staged in LDS (a.nruns <= kLdsRuns), read through the LDS
// array itself -- a pointer that may point at either memory is generic, and
// its flat loads would tie LDS waits to the global accesses in flight
template <int UNIT, bool PACK, bool RL>
__global__ void __launch_bounds__(kCB) k_convert(ConvArgs a) {
  extern __shared__ DRun sruns[];
  const uint64_t g = (uint64_t)blockIdx.x * kCB + threadIdx.x;
  if constexpr (RL) {
    static_assert(sizeof(DRun) % 8 == 0, "DRun is copied as 8-byte words");
    uint64_t *d = reinterpret_cast<uint64_t *>(sruns);
    const char *src = reinterpret_cast<const char *>(a.runs);
    for (uint32_t i = threadIdx.x; i < (uint32_t)a.nruns * (sizeof(DRun) / 8); i += kCB)
      d[i] = gload<uint64_t>(src + 8 * (size_t)i);
    __syncthreads();
    convert_granule<UNIT, PACK>(a, sruns, g);
  } else {
    convert_granule<UNIT, PACK>(a, a.runs, g);
  }
}

// ---------------------------------------------------------------------------
// VEC kernel: the layout is ONE strided 1-level run (what MPI_Type_vector /
// hvector and resized contiguous types flatten to): block l of instance i
// lives at  i*ext + disp + l*stride1, blen bytes, cnt1 blocks per instance,
// and every piece is a whole number of aligned W-byte words (W = 4 or 8).
// Consecutive lanes own consecutive W-byte words of a workgroup's stretch
// of the stream, so the packed side is one coalesced access per wave
// instruction and the user side touches only the lines holding data.  The
// stretch start is mapped once (two multiply-shift divisions); each word is
// mapped from it in 32-bit arithmetic (float-reciprocal quotient by blen,
// made exact by the remainder correction), with no LDS phase and no barrier.
// kVIt words per lane are loaded before any is stored.
// ---------------------------------------------------------------------------
constexpr int kVIt = 8;
constexpr uint64_t kVecMaxBlen = (uint64_t)1 << 22;   // keeps t / blen exact in fp32 + 1 correction

template <int W, bool PACK, bool NT = false>
__global__ void __launch_bounds__(kCB) k_convert_vec(ConvArgs a, DRun R, float rblen) {
  using U = typename unit_t<W>::T;
  const uint64_t nw = a.len / W;
  const uint64_t wbase = (uint64_t)blockIdx.x * (kCB * kVIt);
  const uint64_t p0 = a.offset + wbase * W;   // stream byte where this stretch starts
  const uint64_t B0 = udiv(p0, R.mblen);      // global block index (S = cnt1 * blen)
  const uint32_t o0 = (uint32_t)(p0 - B0 * R.blen);
  const uint64_t i0 = udiv(B0, R.mcnt1);
  const uint64_t l0 = B0 - i0 * R.cnt1;
  const uint32_t blen = (uint32_t)R.blen;
  U v[kVIt];
  U *ua[kVIt];
#pragma unroll
  for (int k = 0; k < kVIt; k++) {
    const uint32_t rel = (uint32_t)(k * kCB + threadIdx.x);
    if (wbase + rel < nw) {
      const uint32_t t = o0 + rel * W;
      uint32_t q = (uint32_t)((float)t * rblen);
      int32_t r = (int32_t)(t - q * blen);
      if (r < 0) { q--; r += (int32_t)blen; }
      if (r < 0) { q--; r += (int32_t)blen; }
      if (r >= (int32_t)blen) { q++; r -= (int32_t)blen; }
      if (r >= (int32_t)blen) { q++; r -= (int32_t)blen; }
      uint64_t l1 = l0 + q, inst = i0;
      if (l1 >= R.cnt1) {
        const uint64_t d = udiv(l1, R.mcnt1);
        inst += d;
        l1 -= d * R.cnt1;
      }
      ua[k] = reinterpret_cast<U *>(a.user + (int64_t)inst * a.ext + R.disp + (int64_t)l1 * R.stride1 + r);
      if (PACK && NT) v[k] = __builtin_nontemporal_load(ua[k]);
      else v[k] = PACK ? *ua[k] : reinterpret_cast<const U *>(a.packed)[wbase + rel];
    }
  }
#pragma unroll
  for (int k = 0; k < kVIt; k++) {
    const uint32_t rel = (uint32_t)(k * kCB + threadIdx.x);
    if (wbase + rel < nw) {
      if (PACK && NT) __builtin_nontemporal_store(v[k], reinterpret_cast<U *>(a.packed) + wbase + rel);
      else if (PACK) reinterpret_cast<U *>(a.packed)[wbase + rel] = v[k];
      else *ua[k] = v[k];
    }
  }
}

// PACK of a periodic strided layout with small blocks (round 3): one run of
// blen-byte blocks every stride bytes, instances continuing the period
// (extent = cnt1 * stride) or one instance, stride 8 or 16, the first block
// 16-byte aligned.  Lane q reads user chunk q (16 bytes, one aligned load: a wave
// streams 1 KiB of span) holding M = 16 / stride whole blocks, and writes
// their M * blen packed bytes with one store (a wave writes M * blen * 64
// contiguous bytes).  The run-walking VEC kernel reads the same lines as
// one 4-byte word per lane at the stride (twice the load instructions for
// 4-byte blocks every 8 bytes).
template <int STRIDE, int BLEN, bool NT = false>
__global__ void __launch_bounds__(kCB) k_pack_vec_span(const char *ubase, char *packed, uint64_t offset,
                                                       uint64_t len, uint64_t q0, uint64_t q1) {
  constexpr int M = 16 / STRIDE, OUT = M * BLEN;
  static_assert(16 % STRIDE == 0 && BLEN < STRIDE && (BLEN == 4 || BLEN == 8 || BLEN == 2 || BLEN == 1),
                "periodic small blocks");
  const uint64_t q = q0 + (uint64_t)blockIdx.x * kCB + threadIdx.x;
  if (q >= q1) return;
  const uint4 v = gld16p<NT>(ubase + 16 * q);
  const uint32_t d[4] = {v.x, v.y, v.z, v.w};
  uint8_t o[OUT];
#pragma unroll
  for (int k = 0; k < M; k++)
#pragma unroll
    for (int i = 0; i < BLEN; i++) {
      const int b = k * STRIDE + i;                          // byte of the chunk
      o[k * BLEN + i] = (uint8_t)(d[b >> 2] >> (8 * (b & 3)));
    }
  const uint64_t p = q * OUT;                                // stream offset of the chunk's first packed byte
  if (p >= offset && p + OUT <= offset + len) {
    char *dst = packed + (p - offset);
    if constexpr (OUT == 8) {
      uint32_t w0 = 0, w1 = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) { w0 |= (uint32_t)o[i] << (8 * i); w1 |= (uint32_t)o[4 + i] << (8 * i); }
      if constexpr (NT) __builtin_nontemporal_store((uint64_t)w0 | (uint64_t)w1 << 32, reinterpret_cast<uint64_t *>(dst));
      else *reinterpret_cast<uint2 *>(dst) = make_uint2(w0, w1);
    } else if constexpr (OUT == 4) {
      uint32_t w0 = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) w0 |= (uint32_t)o[i] << (8 * i);
      if constexpr (NT) __builtin_nontemporal_store(w0, reinterpret_cast<uint32_t *>(dst));
      else *reinterpret_cast<uint32_t *>(dst) = w0;
    } else {
#pragma unroll
      for (int i = 0; i < OUT; i++) dst[i] = (char)o[i];
    }
  } else {                                                   // window edge: the bytes inside only
#pragma unroll
    for (int i = 0; i < OUT; i++)
      if (p + i >= offset && p + i < offset + len) packed[p + i - offset] = (char)o[i];
  }
}

// ---------------------------------------------------------------------------
// TILE kernels (pieces narrower than 16 bytes): a workgroup owns kTP bytes
// of the stream.  PACK loads the user span the tile reads (monotonic
// layouts: [addr(first byte), addr(last byte)]) into LDS with 16-byte
// coalesced loads, every lane walks the pieces of its kChunk-byte stretch
// copying LDS -> LDS (4-byte words, v_alignbyte for misaligned pieces), and
// the packed tile leaves with 16-byte coalesced stores.  UNPACK stages the
// packed tile in LDS the same way and stores each piece straight to user
// memory with the widest aligned accesses (gap bytes are never written).
// One mapping (three multiply-shift divisions) per lane instead of one per
// byte; HBM sees only wide accesses.
// ---------------------------------------------------------------------------
// TP = stream bytes per tile (TP / kCB per lane); a PACK tile may stage up
// to 3 * TP user bytes.  Each piece's user address is advanced in place
// (next block: + stride1; next outer block / run / instance: from the
// instance base) instead of being recomputed with 64-bit multiplies.
template <int TP> struct TileGeom {
  static constexpr int kChunk = TP / kCB;
  static constexpr int kSpanCap = 3 * TP;
  static constexpr size_t lds(bool pack, size_t run_bytes) {
    return TP + 16 + (pack ? kSpanCap + 32 : 0) + run_bytes;
  }
};

__device__ __forceinline__ uint32_t lds_word(const char *s) {  // 4 bytes at any alignment
  const uintptr_t u = (uintptr_t)s;
  const uint32_t *w = reinterpret_cast<const uint32_t *>(u & ~(uintptr_t)3);
  const int sh = (int)(u & 3);
  return sh ? __builtin_amdgcn_alignbyte(w[1], w[0], sh) : w[0];
}

__device__ __forceinline__ void lds_copy(char *d, const char *s, uint64_t n) {
  while (n && ((uintptr_t)d & 3)) { *d++ = *s++; n--; }
  for (; n >= 4; n -= 4, d += 4, s += 4) *reinterpret_cast<uint32_t *>(d) = lds_word(s);
  while (n--) *d++ = *s++;
}

__device__ __forceinline__ void lds_to_global(char *g, const char *s, uint64_t n) {
  while (n && ((uintptr_t)g & 3)) { *g++ = *s++; n--; }
  while (n >= 4 && ((uintptr_t)g & 15)) {
    *reinterpret_cast<uint32_t *>(g) = lds_word(s);
    g += 4; s += 4; n -= 4;
  }
  for (; n >= 16; n -= 16, g += 16, s += 16)
    *reinterpret_cast<uint4 *>(g) = make_uint4(lds_word(s), lds_word(s + 4), lds_word(s + 8), lds_word(s + 12));
  for (; n >= 4; n -= 4, g += 4, s += 4) *reinterpret_cast<uint32_t *>(g) = lds_word(s);
  while (n--) *g++ = *s++;
}

// stream bytes [t0, t1) between global and LDS (16-byte accesses when aligned)
template <bool TO_LDS>
__device__ __forceinline__ void tile_move(char *lds, char *glob, uint64_t nbytes, int vec) {
  if (vec) {
    const uint64_t nv = nbytes / 16;
    for (uint64_t i = threadIdx.x; i < nv; i += kCB) {
      if (TO_LDS) reinterpret_cast<uint4 *>(lds)[i] = reinterpret_cast<const uint4 *>(glob)[i];
      else reinterpret_cast<uint4 *>(glob)[i] = reinterpret_cast<const uint4 *>(lds)[i];
    }
    for (uint64_t i = nv * 16 + threadIdx.x; i < nbytes; i += kCB) {
      if (TO_LDS) lds[i] = glob[i]; else glob[i] = lds[i];
    }
  } else {
    for (uint64_t i = threadIdx.x; i < nbytes; i += kCB) {
      if (TO_LDS) lds[i] = glob[i]; else glob[i] = lds[i];
    }
  }
}

// One lane's kChunk-byte stretch of tile [r0, r1): PACK copies pieces from
// the staged user span (LDS, origin `lo`) into the packed tile (LDS),
// UNPACK stores pieces from the packed tile straight to user memory.
template <bool PACK, int TP>
__device__ __forceinline__ void walk_chunk(const ConvArgs &a, const DRun *runs, char *pk, const char *span,
                                           uintptr_t lo, uint64_t r0, uint64_t r1) {
  constexpr int kChunk = TileGeom<TP>::kChunk;
  const uint64_t c0 = r0 + (uint64_t)threadIdx.x * kChunk;
  const uint64_t c1 = c0 + kChunk < r1 ? c0 + kChunk : r1;
  if (c0 < c1) {
    Pos P = map_pos(runs, a.nruns, a.S, a.mS, a.offset + c0);
    const DRun *R = &runs[P.r];
    int64_t ibase = (int64_t)P.inst * a.ext;                       // instance origin
    int64_t obase = ibase + R->disp + (int64_t)P.l2 * R->stride2;  // outer block origin
    int64_t ua = obase + (int64_t)P.l1 * R->stride1 + (int64_t)P.o;
    uint64_t pos = c0;
    while (pos < c1) {
      const uint64_t blen = R->blen;
      const uint64_t avail = blen - P.o, want = c1 - pos;
      const uint64_t n = avail < want ? avail : want;
      if (PACK) lds_copy(pk + (pos - r0), span + ((uintptr_t)a.user + ua - lo), n);
      else lds_to_global(a.user + ua, pk + (pos - r0), n);
      pos += n;
      P.o += n;
      ua += (int64_t)n;
      if (P.o == blen) {
        P.o = 0;
        if (++P.l1 < R->cnt1) {
          ua += R->stride1 - (int64_t)blen;
        } else {
          P.l1 = 0;
          if (++P.l2 < R->cnt2) {
            obase += R->stride2;
          } else {
            P.l2 = 0;
            if (++P.r == a.nruns) { P.r = 0; ibase += a.ext; }
            R = &runs[P.r];
            obase = ibase + R->disp;
          }
          ua = obase;
        }
      }
    }
  }
}

template <bool PACK, int TP>
__global__ void __launch_bounds__(kCB) k_convert_tile(ConvArgs a, int nruns_lds, int wordpar) {
  constexpr int kTP = TP, kSpanCap = TileGeom<TP>::kSpanCap;
  extern __shared__ __align__(16) char smem[];
  char *pk = smem;                                   // kTP (+16 slack)
  char *span = smem + kTP + 16;                      // kSpanCap (+32 slack), PACK only
  DRun *sruns = reinterpret_cast<DRun *>(smem + kTP + 16 + (PACK ? kSpanCap + 32 : 0));
  __shared__ int64_t s_first, s_last;
  const DRun *runs = a.runs;
  if (nruns_lds) {
    for (int i = threadIdx.x; i < a.nruns; i += kCB) sruns[i] = a.runs[i];
    runs = sruns;
  }
  const uint64_t r0 = (uint64_t)blockIdx.x * kTP;                 // relative to offset
  const uint64_t r1 = r0 + kTP < a.len ? r0 + kTP : a.len;
  const int vec = a.pk_vec;
  uintptr_t lo = 0;
  bool staged = true;
  if (PACK) {
    __syncthreads();
    if (threadIdx.x < 2) {
      const uint64_t p = a.offset + (threadIdx.x ? r1 - 1 : r0);
      const Pos P = map_pos(runs, a.nruns, a.S, a.mS, p);
      const int64_t ad = block_addr(P, runs[P.r], a.ext) + (int64_t)P.o;
      if (threadIdx.x) s_last = ad; else s_first = ad;
    }
    __syncthreads();
    lo = ((uintptr_t)a.user + s_first) & ~(uintptr_t)15;
    const uintptr_t hi = ((uintptr_t)a.user + s_last + 16) & ~(uintptr_t)15;
    staged = s_last >= s_first && hi - lo <= (uintptr_t)kSpanCap;
    if (staged) tile_move<true>(span, reinterpret_cast<char *>(lo), hi - lo, 1);
  } else {
    tile_move<true>(pk, a.packed + r0, r1 - r0, vec);
  }
  __syncthreads();
  if (PACK && !staged) {   // span too wide for LDS: per-granule gather
    const uint64_t g0 = r0 / 16, g1 = (r1 + 15) / 16;
    for (uint64_t g = g0 + threadIdx.x; g < g1; g += kCB) convert_granule<1, true>(a, runs, g);
    return;
  }
  if (!PACK && wordpar) {
    // word-parallel stores: consecutive lanes write consecutive stream
    // words, so a wave's stores land on neighbouring user blocks
    const uint64_t nb = r1 - r0;
    for (uint64_t w = threadIdx.x; w * 4 < nb; w += kCB) {
      const uint64_t nbytes = nb - w * 4 < 4 ? nb - w * 4 : 4;
      Pos P = map_pos(runs, a.nruns, a.S, a.mS, a.offset + r0 + w * 4);
      DRun R = runs[P.r];
      char *ua = a.user + block_addr(P, R, a.ext) + (int64_t)P.o;
      if (nbytes == 4 && P.o + 4 <= R.blen && ((uintptr_t)ua & 3) == 0) {
        *reinterpret_cast<uint32_t *>(ua) = *reinterpret_cast<const uint32_t *>(pk + w * 4);
      } else {
        for (uint64_t i = 0; i < nbytes; i++) {
          a.user[block_addr(P, R, a.ext) + (int64_t)P.o] = pk[w * 4 + i];
          if (++P.o == R.blen) next_block(P, runs, a.nruns, R);
        }
      }
    }
    return;
  }
  walk_chunk<PACK, TP>(a, runs, pk, span, lo, r0, r1);
  if (PACK) {
    __syncthreads();
    tile_move<false>(pk, a.packed + r0, r1 - r0, vec);
  }
}

// PACK, pipelined: persistent workgroups walk tiles t, t + grid, ...; while
// the lanes copy tile t's pieces out of LDS, the next tile's user span is
// already in flight into registers (SPAN / 16 / kCB uint4 per lane), and
// lands in LDS after the tile's packed bytes have left.  The one-tile
// kernel above idles the memory pipe during every LDS phase (SQ counters on
// the struct type: ~730 VALU instructions per 22.6k-cycle wave, i.e. waves
// mostly wait on the span load).
// Geometry (TP stream bytes per tile, SPAN bytes of user span staged): each
// lane owns TP / kCB consecutive stream bytes, so at every step of the walk
// the 64 lanes of a wave write the packed tile at a stride of TP / kCB
// bytes.  With 32-byte stretches (TP 8192) lane starts fall on only 8 of
// the 64 LDS banks (8-way conflicts, SQ_LDS_BANK_CONFLICT 2.7 cycles per LDS
// instruction on the struct type); 36-byte stretches (TP 9216, 9 dwords,
// coprime to 64) start every lane of a wave on its own bank.  A smaller span
// cap (16 KiB: the struct type reads 48/29 x TP) lets 6 instead of 4
// workgroups share a CU.
template <int TP, int SPAN>
struct PipeGeom {
  static constexpr int kSpanCap = SPAN;
  static constexpr int kPre = SPAN / 16 / kCB;   // uint4 per lane for a full span
  static constexpr size_t lds(size_t run_bytes) { return TP + 16 + SPAN + 32 + run_bytes; }
};

template <int TP, int SPAN>
__global__ void __launch_bounds__(kCB) k_pack_tile_pipe(ConvArgs a, int nruns_lds, uint64_t ntiles) {
  constexpr int kTP = TP, kSpanCap = SPAN, kPre = PipeGeom<TP, SPAN>::kPre;
  static_assert(kSpanCap % (16 * kCB) == 0, "span staging is whole vectors per lane");
  static_assert(kTP % (16 * 4) == 0 && kTP / kCB >= 16, "tiles are whole 16-byte vectors");
  extern __shared__ __align__(16) char smem[];
  char *pk = smem;
  char *span = smem + kTP + 16;
  DRun *sruns = reinterpret_cast<DRun *>(smem + kTP + 16 + kSpanCap + 32);
  __shared__ uintptr_t s_lo[2];
  __shared__ uint64_t s_nb[2];
  __shared__ int s_ok[2];
  const DRun *runs = a.runs;
  if (nruns_lds) {
    for (int i = threadIdx.x; i < a.nruns; i += kCB) sruns[i] = a.runs[i];
    runs = sruns;
  }
  auto bounds = [&](uint64_t t, int slot) {   // one thread: user span of tile t
    const uint64_t r0 = t * kTP, r1 = r0 + kTP < a.len ? r0 + kTP : a.len;
    const Pos P0 = map_pos(runs, a.nruns, a.S, a.mS, a.offset + r0);
    const Pos P1 = map_pos(runs, a.nruns, a.S, a.mS, a.offset + r1 - 1);
    const int64_t f = block_addr(P0, runs[P0.r], a.ext) + (int64_t)P0.o;
    const int64_t l = block_addr(P1, runs[P1.r], a.ext) + (int64_t)P1.o;
    const uintptr_t lo = ((uintptr_t)a.user + f) & ~(uintptr_t)15;
    const uintptr_t hi = ((uintptr_t)a.user + l + 16) & ~(uintptr_t)15;
    s_lo[slot] = lo;
    s_nb[slot] = hi - lo;
    s_ok[slot] = l >= f && hi - lo <= (uintptr_t)kSpanCap;
  };
  uint64_t t = blockIdx.x;
  if (t >= ntiles) return;
  __syncthreads();                                   // runs staged
  if (threadIdx.x == 0) bounds(t, 0);
  __syncthreads();
  if (s_ok[0]) tile_move<true>(span, reinterpret_cast<char *>(s_lo[0]), s_nb[0], 1);
  int cur = 0;
  for (;;) {
    const uint64_t tn = t + gridDim.x;
    const bool has_next = tn < ntiles;
    if (has_next && threadIdx.x == 0) bounds(tn, cur ^ 1);
    __syncthreads();                                 // span of t in LDS; bounds of tn visible
    uint4 pre[kPre];
    const bool pre_ok = has_next && s_ok[cur ^ 1];
    const uint32_t nvn = pre_ok ? (uint32_t)(s_nb[cur ^ 1] / 16) : 0;
    const uint32_t tx = threadIdx.x;
    {
      const uint4 *g = reinterpret_cast<const uint4 *>(s_lo[cur ^ 1]);
#pragma unroll
      for (int k = 0; k < kPre; k++)
        if (tx + k * kCB < nvn) pre[k] = g[tx + k * kCB];
    }
    const uint64_t r0 = t * kTP, r1 = r0 + kTP < a.len ? r0 + kTP : a.len;
    if (s_ok[cur]) {
      walk_chunk<true, TP>(a, runs, pk, span, s_lo[cur], r0, r1);
      __syncthreads();
      tile_move<false>(pk, a.packed + r0, r1 - r0, a.pk_vec);
    } else {                                         // span too wide for LDS: per-granule gather
      const uint64_t g0 = r0 / 16, g1 = (r1 + 15) / 16;
      for (uint64_t g = g0 + threadIdx.x; g < g1; g += kCB) convert_granule<1, true>(a, runs, g);
    }
    if (!has_next) break;
    __syncthreads();                                 // span and pk of t are free
    {
      uint4 *d = reinterpret_cast<uint4 *>(span);
#pragma unroll
      for (int k = 0; k < kPre; k++)
        if (tx + k * kCB < nvn) d[tx + k * kCB] = pre[k];
    }
    t = tn;
    cur ^= 1;
  }
}

// ---------------------------------------------------------------------------
// BYTE-MAP / PIECE kernels (instances of at most kBmapMaxS packed bytes,
// i.e. the struct-like types whose pieces are narrow and irregular).
//
// The run walk above serialises each lane on its own stretch of pieces (the
// struct type: ~3 divergent byte / word loops per lane per tile), so the
// tile kernels are instruction-bound, and their unpack stores leave a user
// line partially written for long enough that L2 writes it back more than
// once (WRITE_SIZE 3.1 x the span on the struct type,
// profiles/r02/convertor_r2.txt).  Here the instance layout is tabled once
// per type and every lane runs the same straight-line code:
//   PACK (byte map): bmap[b] = user offset of packed byte b of an instance.
//     A workgroup stages the user span of a tile of stream bytes in LDS
//     (16-byte coalesced loads), each lane assembles 16 packed bytes with 16
//     LDS byte reads through the map and leaves with one 16-byte store.
//   UNPACK (pieces): the instance is cut into naturally aligned pieces of
//     1/2/4/8/16 user bytes (per user-pointer alignment), in stream order.
//     A workgroup stages the packed bytes of a tile of pieces in LDS; lane l
//     takes piece l, reads its bytes with five dword LDS reads + byte
//     alignment and writes them with ONE store of the piece's width, so a
//     wave writes 64 consecutive pieces at once and every user line is
//     complete within a few instructions.  Gap bytes are never written.
// ---------------------------------------------------------------------------
constexpr uint32_t kBmapMaxS = 65535;      // packed bytes per instance (piece soff is 16-bit)
constexpr size_t kBmapLds = 20480;         // PACK: map bytes staged in LDS
constexpr int kBmapSpan = 24576;           // PACK: user span staged per tile
constexpr int kBmapSpans[3] = {12288, kBmapSpan, 49152};   // MX_CONV_BMAP_SPAN choices
constexpr int kPieceStage = 16384;         // UNPACK: packed bytes staged per tile

struct DPiece {
  int32_t uoff;       // user offset from the instance origin
  uint16_t soff;      // stream offset within the instance
  uint8_t lg;         // width = 1 << lg bytes (user address aligned to it)
  uint8_t pad;
};

struct BmapArgs {
  const void *map;         // M[S]: user offset of packed byte b minus umin
  uint32_t S;
  Magic mS;
  int64_t ext;
  int64_t umin, uspan;     // an instance touches user [umin, umin + uspan)
  int mono;                // monotonic layout: a tile's span is [addr(first), addr(last)]
  const char *user;
  char *packed;            // (packed - offset) is 16-byte aligned
  uint64_t offset, len;
  uint64_t g0;             // first absolute granule (offset / 16)
  uint64_t T;              // stream bytes per tile (multiple of 16)
  uint64_t ntiles;
  uint32_t adv_b;          // kCB * 4 stream bytes = adv_io / ext instances + adv_b bytes
  int64_t adv_io;
  uint64_t lo_mask;        // a tile's staged span starts at lo & ~lo_mask (15, or 127: whole lines)
  uint32_t qsh;            // 2: the map is staged as quads (entry b at [4b], its dword's bytes at [4b..4b+3])
  uint32_t cw;             // try one LDS dword read per packed dword (word-piece layouts)
  uint32_t unroll;         // kBmapU dwords per lane per step in the DW gather
  uint32_t word;           // word map: entries 4k only (S % 4 == 0, every packed dword user-contiguous)
};
constexpr int kBmapU = 4;

// M = uint16_t when the instance's user span is below 64 KiB, else uint32_t.
// PIPE (round 3): persistent workgroups keep the NEXT tile's user span in
// flight in registers (SPAN / 16 / kCB uint4 per lane) while the lanes
// gather the current tile out of LDS -- without it every tile's span load
// and gather run back to back inside the workgroup.
template <int SPAN, class M, bool DW, bool PIPE, bool NT>
// waves per SIMD the LDS allows (workgroups per CU: 6 at a 24 KiB span), so
// the register budget never lowers the occupancy below it
__global__ void __launch_bounds__(kCB, SPAN >= 49152 ? 3 : SPAN >= 24576 ? 6 : 7) k_pack_bmap(BmapArgs a) {
  extern __shared__ __align__(16) char smem[];
  char *span = smem;                                         // SPAN + 32
  // The map in LDS, entry x = user offset of packed byte x (x >= S: of the
  // next instance, + ext), so a dword at instance byte b reads its four
  // entries x = b..b+3 with no wrap test:
  //   qsh 0: entries 0 .. S+2 in a row -- one 8-byte LDS read when b is a
  //          multiple of 4 (S % 4 == 0);
  //   qsh 2: quads, [4b + j] = entry b + j -- every dword's four entries in
  //          one aligned 8-byte read for any S (a misaligned read of the row
  //          stalled the struct type's gather: SQ_WAIT_INST_LDS 388M vs 23M,
  //          profiles/r05/pmc_pack_r5j.jsonl).
  // bmap[x << qsh] is entry x either way.
  //   word (S % 4 == 0, every packed dword 4 user-contiguous bytes: word
  //          pieces): only entries 4k are staged, [k] = entry 4k, and entry
  //          x = [x >> 2] + (x & 3) -- a quarter of the LDS (indexed's 10 KiB
  //          map: 2.6 KiB, so the 24 KiB span keeps five workgroups per CU)
  //          and one byte-map read + one dword read per packed dword.
  M *bmap = reinterpret_cast<M *>(smem + SPAN + 32);
  __shared__ uintptr_t s_lo[2], s_hi[2];
  constexpr int kPre = SPAN / 16 / kCB;
  const uint32_t qsh = a.qsh;
  const bool word = a.word != 0;
  const uint32_t nent = word ? a.S / 4 : qsh ? 4 * a.S : a.S + 3;
  for (uint32_t i = threadIdx.x; i < nent; i += kCB) {
    const uint32_t x = word ? 4 * i : qsh ? (i >> 2) + (i & 3) : i;
    const uint32_t k = x / a.S;
    bmap[i] = (M)(reinterpret_cast<const M *>(a.map)[x - k * a.S] + k * (uint32_t)a.ext);
  }
  auto ent = [&](uint64_t x) -> int64_t {                    // entry x < S
    return word ? (int64_t)bmap[x >> 2] + (int64_t)(x & 3) : (int64_t)bmap[x << qsh];
  };
  const uint64_t wend = a.offset + a.len;
  // tile t: absolute stream bytes [s0, s1) (window-clipped from sa), instances ia..ib
  auto geom = [&](uint64_t t, uint64_t &s0, uint64_t &sa, uint64_t &s1, uint64_t &ia, uint64_t &ib) {
    s0 = a.g0 * 16 + t * a.T;
    sa = s0 < a.offset ? a.offset : s0;
    s1 = s0 + a.T < wend ? s0 + a.T : wend;
    ia = udiv(sa, a.mS);
    ib = udiv(s1 - 1, a.mS);
  };
  // one thread: the 16-aligned user span [lo, hi) tile t reads (bmap staged)
  auto bounds = [&](uint64_t t, int slot) {
    uint64_t s0, sa, s1, ia, ib;
    geom(t, s0, sa, s1, ia, ib);
    const uintptr_t ubase = (uintptr_t)a.user + (int64_t)ia * a.ext + a.umin;
    uintptr_t lo = ubase, hi = ubase + (int64_t)(ib - ia) * a.ext + a.uspan;
    if (a.mono) {
      lo = ubase + ent(sa - ia * a.S);
      hi = ubase + (int64_t)(ib - ia) * a.ext + ent(s1 - 1 - ib * a.S) + 1;
    }
    s_lo[slot] = lo & ~(uintptr_t)a.lo_mask;
    s_hi[slot] = (hi + 15) & ~(uintptr_t)15;
  };
  auto gather = [&](uint64_t t, uintptr_t lo) {
    uint64_t s0, sa, s1, ia, ib;
    geom(t, s0, sa, s1, ia, ib);
    const uintptr_t ubase = (uintptr_t)a.user + (int64_t)ia * a.ext + a.umin;   // instance ia, + umin
    const int64_t d0 = (int64_t)(ubase - lo);
    if (DW) {
      // lane = one packed dword per step, consecutive lanes consecutive
      // dwords: the map reads of a wave are 8 bytes apart (2-way bank
      // conflicts; 16-byte lanes read it 32 bytes apart, 8-way) and each
      // store instruction writes 256 contiguous bytes.  Everything inside the
      // tile is 32-bit: dword j of the tile is stream bytes s0 + 4j (the tile
      // is < 64 KiB of stream, its span < 64 KiB of LDS), so the loop is 4
      // map reads, 4 byte reads and ~16 VALU per dword (round 4's 64-bit
      // loop with a wrap test per byte took 55, PMC SQ_INSTS_VALU,
      // profiles/r05/pmc_pack_r5.jsonl)
      const uint32_t nq = (uint32_t)((s1 - s0 + 3) / 4);
      const uint32_t jlo = (uint32_t)((sa - s0 + 3) / 4);     // dwords [jlo, jhi) lie inside the window
      const uint32_t jhi = (uint32_t)((s1 - s0) / 4);
      char *const pk = a.packed + (int64_t)(s0 - a.offset);   // dword j at pk + 4j (j >= jlo)
      const uint64_t p0 = s0 + 4 * (uint64_t)threadIdx.x;
      const uint64_t inst = udiv(p0, a.mS);
      uint32_t b = (uint32_t)(p0 - inst * a.S);
      int32_t io = (int32_t)((int64_t)(inst - ia) * a.ext + d0);
      const int32_t adv_io = (int32_t)a.adv_io, ext = (int32_t)a.ext;
      uint32_t j = threadIdx.x;
      if (a.unroll) {
        // kBmapU dwords per lane per step (j, j + kCB, ...), all inside the
        // window: their map reads, then their byte reads, are independent and
        // in flight together (one dword per step waits out two LDS round
        // trips back to back)
        for (; j >= jlo && j + (kBmapU - 1) * kCB < jhi; j += kBmapU * kCB) {
          uint32_t bu[kBmapU];
          int32_t iu[kBmapU];
          bu[0] = b;
          iu[0] = io;
#pragma unroll
          for (int u = 1; u < kBmapU; u++) {
            uint32_t nb = bu[u - 1] + a.adv_b;
            int32_t ni = iu[u - 1] + adv_io;
            if (nb >= a.S) { nb -= a.S; ni += ext; }
            bu[u] = nb;
            iu[u] = ni;
          }
          uint32_t v[kBmapU];
          if (word) {                                         // b % 4 == 0 here (S % 4 == 0)
            int32_t w[kBmapU];
#pragma unroll
            for (int u = 0; u < kBmapU; u++) w[u] = bmap[bu[u] >> 2];
#pragma unroll
            for (int u = 0; u < kBmapU; u++) v[u] = *reinterpret_cast<const uint32_t *>(span + iu[u] + w[u]);
#pragma unroll
            for (int u = 0; u < kBmapU; u++) {
              uint32_t *q = reinterpret_cast<uint32_t *>(pk + 4 * (j + u * kCB));
              if (NT) __builtin_nontemporal_store(v[u], q);
              else *q = v[u];
            }
            b = bu[kBmapU - 1] + a.adv_b;
            io = iu[kBmapU - 1] + adv_io;
            if (b >= a.S) { b -= a.S; io += ext; }
            continue;
          }
          int32_t e[kBmapU][4];
#pragma unroll
          for (int u = 0; u < kBmapU; u++) {
            const M *m = bmap + (bu[u] << qsh);
#pragma unroll
            for (int k = 0; k < 4; k++) e[u][k] = m[k];
          }
          bool cont = a.cw != 0;
#pragma unroll
          for (int u = 0; u < kBmapU; u++)
            cont = cont && (e[u][1] == e[u][0] + 1) & (e[u][2] == e[u][0] + 2) & (e[u][3] == e[u][0] + 3);
          if (a.cw && __all(cont)) {
#pragma unroll
            for (int u = 0; u < kBmapU; u++) v[u] = *reinterpret_cast<const uint32_t *>(span + iu[u] + e[u][0]);
          } else {
#pragma unroll
            for (int u = 0; u < kBmapU; u++)
              v[u] = (uint32_t)(uint8_t)span[iu[u] + e[u][0]] | (uint32_t)(uint8_t)span[iu[u] + e[u][1]] << 8 |
                     (uint32_t)(uint8_t)span[iu[u] + e[u][2]] << 16 | (uint32_t)(uint8_t)span[iu[u] + e[u][3]] << 24;
          }
#pragma unroll
          for (int u = 0; u < kBmapU; u++) {
            uint32_t *q = reinterpret_cast<uint32_t *>(pk + 4 * (j + u * kCB));
            if (NT) __builtin_nontemporal_store(v[u], q);
            else *q = v[u];
          }
          b = bu[kBmapU - 1] + a.adv_b;
          io = iu[kBmapU - 1] + adv_io;
          if (b >= a.S) { b -= a.S; io += ext; }
        }
      }
      for (; j < nq; j += kCB) {
        if (j >= jlo && j < jhi && word) {
          const uint32_t v = *reinterpret_cast<const uint32_t *>(span + io + (int32_t)bmap[b >> 2]);
          if (NT) __builtin_nontemporal_store(v, reinterpret_cast<uint32_t *>(pk + 4 * j));
          else *reinterpret_cast<uint32_t *>(pk + 4 * j) = v;
        } else if (j >= jlo && j < jhi) {
          const M *m = bmap + (b << qsh);
          const int32_t e0 = m[0], e1 = m[1], e2 = m[2], e3 = m[3];
          uint32_t v;
          // a wave whose every dword is 4 user-contiguous bytes (word
          // pieces: indexed / BLACS) reads each with one LDS dword read
          if (a.cw && __all((e1 == e0 + 1) & (e2 == e0 + 2) & (e3 == e0 + 3))) {
            v = *reinterpret_cast<const uint32_t *>(span + io + e0);
          } else {
            v = (uint32_t)(uint8_t)span[io + e0] | (uint32_t)(uint8_t)span[io + e1] << 8 |
                (uint32_t)(uint8_t)span[io + e2] << 16 | (uint32_t)(uint8_t)span[io + e3] << 24;
          }
          if (NT) __builtin_nontemporal_store(v, reinterpret_cast<uint32_t *>(pk + 4 * j));
          else *reinterpret_cast<uint32_t *>(pk + 4 * j) = v;
        } else {                                              // window edge: the bytes inside only
          const uint64_t p = s0 + 4 * (uint64_t)j;
          for (uint64_t x = p < a.offset ? a.offset : p; x < p + 4 && x < wend; x++) {
            const uint64_t i = udiv(x, a.mS);
            a.packed[x - a.offset] = span[(int64_t)(i - ia) * a.ext + d0 + ent(x - i * a.S)];
          }
        }
        b += a.adv_b;                                         // next: kCB dwords further
        io += adv_io;
        if (b >= a.S) { b -= a.S; io += ext; }
      }
      return;
    }
    for (uint64_t g = s0 / 16 + threadIdx.x; g * 16 < s1; g += kCB) {
      const uint64_t p = g * 16;
      if (p < a.offset || p + 16 > wend) {                    // window edge: the bytes inside only
        for (uint64_t q = p < a.offset ? a.offset : p; q < p + 16 && q < wend; q++) {
          const uint64_t i = udiv(q, a.mS);
          a.packed[q - a.offset] = span[(int64_t)(i - ia) * a.ext + d0 + ent(q - i * a.S)];
        }
        continue;
      }
      uint64_t inst = udiv(p, a.mS);
      uint32_t b = (uint32_t)(p - inst * a.S);
      int64_t io = (int64_t)(inst - ia) * a.ext + d0;       // LDS offset of the instance origin (+ umin)
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          v |= (uint32_t)(uint8_t)span[io + ent(b)] << (8 * i);
          if (++b == a.S) { b = 0; io += a.ext; }
        }
        w[k] = v;
      }
      if (NT) {
        const v4u_a16 x = {w[0], w[1], w[2], w[3]};
        __builtin_nontemporal_store(x, reinterpret_cast<v4u_a16 *>(a.packed + (p - a.offset)));
      } else {
        *reinterpret_cast<uint4 *>(a.packed + (p - a.offset)) = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  };
  if (!PIPE) {
    for (uint64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
      __syncthreads();                                        // map staged; previous tile done with span
      if (threadIdx.x == 0) bounds(t, 0);
      __syncthreads();
      {
        const char *g = reinterpret_cast<const char *>(s_lo[0]);
        uint4 *d = reinterpret_cast<uint4 *>(span);
        const uint32_t nv = (uint32_t)((s_hi[0] - s_lo[0]) / 16);
        for (uint32_t i = threadIdx.x; i < nv; i += kCB) d[i] = gld16p<NT>(g + 16 * (size_t)i);
      }
      __syncthreads();
      gather(t, s_lo[0]);
    }
    return;
  }
  uint64_t t = blockIdx.x;
  if (t >= a.ntiles) return;
  __syncthreads();                                            // map staged
  if (threadIdx.x == 0) bounds(t, 0);
  __syncthreads();
  {
    const char *g = reinterpret_cast<const char *>(s_lo[0]);
    uint4 *d = reinterpret_cast<uint4 *>(span);
    const uint32_t nv = (uint32_t)((s_hi[0] - s_lo[0]) / 16);
    for (uint32_t i = threadIdx.x; i < nv; i += kCB) d[i] = gld16p<NT>(g + 16 * (size_t)i);
  }
  int cur = 0;
  for (;;) {
    const uint64_t tn = t + gridDim.x;
    const bool has_next = tn < a.ntiles;
    if (has_next && threadIdx.x == 0) bounds(tn, cur ^ 1);
    __syncthreads();                                          // span of t in LDS; bounds of tn visible
    uint4 pre[kPre];
    const uint32_t nvn = has_next ? (uint32_t)((s_hi[cur ^ 1] - s_lo[cur ^ 1]) / 16) : 0;
    {
      const char *g = reinterpret_cast<const char *>(s_lo[cur ^ 1]);
#pragma unroll
      for (int k = 0; k < kPre; k++)
        if (threadIdx.x + k * kCB < nvn) pre[k] = gld16p<NT>(g + 16 * (size_t)(threadIdx.x + k * kCB));
    }
    gather(t, s_lo[cur]);
    if (!has_next) break;
    __syncthreads();                                          // tile t's span is free
    {
      uint4 *d = reinterpret_cast<uint4 *>(span);
#pragma unroll
      for (int k = 0; k < kPre; k++)
        if (threadIdx.x + k * kCB < nvn) d[threadIdx.x + k * kCB] = pre[k];
    }
    t = tn;
    cur ^= 1;
  }
}

struct PieceArgs {
  const DPiece *pieces;
  uint32_t npi;
  Magic mnpi;
  uint64_t S;
  int64_t ext;
  char *user;
  char *packed;            // UNPACK reads it, PACK writes it
  uint64_t offset, len;
  uint64_t P0, P1;         // pieces overlapping [offset, offset + len)
  uint32_t K;              // pieces per tile (multiple of kCB)
  uint32_t dinst, dj;      // kCB pieces = dinst instances + dj pieces
  uint64_t ntiles;
  int tbl_lds;             // table staged in LDS
  int u32;                 // UNPACK: the tile's store loop in 32-bit LDS coordinates
  int ntld;                // UNPACK: the packed stream read non-temporal (read once)
};

__device__ __forceinline__ void piece_store(char *u, int lg, uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3) {
  switch (lg) {   // (global stores: gstore)
    case 0: gstore<uint8_t>(u, (uint8_t)v0); break;
    case 1: gstore<uint16_t>(u, (uint16_t)v0); break;
    case 2: gstore<uint32_t>(u, v0); break;
    case 3: gstore<uint64_t>(u, (uint64_t)v0 | ((uint64_t)v1 << 32)); break;
    default: gstore<uint4>(u, make_uint4(v0, v1, v2, v3)); break;
  }
}

// PIPE: the packed range of the workgroup's next tile is loaded into
// registers (kPieceStage / 16 / kCB 16-byte vectors per lane) while the
// lanes store the current tile from LDS.  Measured slower (round 4,
// interleaved A/B at 1 GiB, profiles/r04/unpack_pipe_ab.txt: BLACS 1540 ->
// 1577 us, struct 949 -> 1071 us): the unpack is bound by its partial-line
// stores, and loads kept in flight beside them only compete (64 more VGPRs
// per lane, fewer waves); so it is off (MX_CONV_UNPACK_PIPE=1 turns it on).
template <bool PIPE, bool TL>
__global__ void __launch_bounds__(kCB) k_unpack_piece(PieceArgs a) {
  extern __shared__ __align__(16) char smem[];
  char *stage = smem;                                        // kPieceStage + 48
  DPiece *stbl = reinterpret_cast<DPiece *>(smem + kPieceStage + 48);
  if (TL) {
    for (uint32_t i = threadIdx.x; i < a.npi; i += kCB) stbl[i] = gload<DPiece>(reinterpret_cast<const char *>(a.pieces + i));
    __syncthreads();
  }
  // the piece table from LDS (TL: a.tbl_lds) or from global memory, each
  // through a pointer of its own address space (one that may be either is
  // generic: flat loads, whose waits also wait for the stores in flight)
  auto piece_at = [&](uint64_t k) -> DPiece {
    if constexpr (TL) {
      return stbl[k];
    } else {
      return gload<DPiece>(reinterpret_cast<const char *>(a.pieces + k));
    }
  };
  const uint64_t wend = a.offset + a.len;
  // stream range of tile t: first byte of piece Pa .. last byte of Pb - 1,
  // as 16-byte aligned addresses of the packed buffer
  auto range = [&](uint64_t t, uintptr_t &lo, uintptr_t &hi) {
    const uint64_t Pa = a.P0 + t * a.K;
    const uint64_t Pb = Pa + a.K < a.P1 ? Pa + a.K : a.P1;
    const uint64_t ia = udiv(Pa, a.mnpi), ib = udiv(Pb - 1, a.mnpi);
    const DPiece fa = piece_at(Pa - ia * a.npi), fb = piece_at(Pb - 1 - ib * a.npi);
    uint64_t sa = ia * a.S + fa.soff, sb = ib * a.S + fb.soff + (1u << fb.lg);
    sa = sa < a.offset ? a.offset : sa;
    sb = sb < wend ? sb : wend;
    lo = (uintptr_t)(a.packed + (sa - a.offset)) & ~(uintptr_t)15;
    hi = ((uintptr_t)(a.packed + (sb - a.offset)) + 15) & ~(uintptr_t)15;
  };
  // the same loop with everything inside the tile 32-bit: instance origins
  // as LDS offsets (a tile's packed range is < kPieceStage), the window as
  // clamped LDS bounds, the user pointer advanced by whole instances
  auto store_tile32 = [&](uint64_t t, uintptr_t lo) {
    const uint64_t Pa = a.P0 + t * a.K;
    const uint64_t Pb = Pa + a.K < a.P1 ? Pa + a.K : a.P1;
    const uint64_t P = Pa + threadIdx.x;
    if (P >= Pb) return;
    const uint64_t inst = udiv(P, a.mnpi);
    uint32_t j = (uint32_t)(P - inst * a.npi);
    const int64_t base = (int64_t)((uintptr_t)a.packed - lo) - (int64_t)a.offset;   // LDS offset of stream byte 0
    int32_t ib = (int32_t)(base + (int64_t)(inst * a.S));
    char *ub = a.user + (int64_t)inst * a.ext;
    const int64_t w0 = (int64_t)((uintptr_t)a.packed - lo), w1 = w0 + (int64_t)a.len;
    const int32_t wlo = w0 < INT32_MIN ? INT32_MIN : (int32_t)w0, whi = w1 > INT32_MAX ? INT32_MAX : (int32_t)w1;
    const int32_t S32 = (int32_t)a.S, dS = (int32_t)(a.dinst * a.S);
    const int64_t dE = (int64_t)a.dinst * a.ext;
    const uint32_t iters = (uint32_t)((Pb - P + kCB - 1) / kCB);
    for (uint32_t it = 0; it < iters; it++) {
      const DPiece pc = piece_at(j);
      const int32_t li = ib + (int32_t)pc.soff;
      const int32_t n = 1 << pc.lg;
      char *u = ub + pc.uoff;
      if (li >= wlo && li + n <= whi) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(stage + (li & ~3));
        const int sh = li & 3;
        const uint32_t x0 = w[0], x1 = w[1], x2 = w[2], x3 = w[3], x4 = w[4];
        piece_store(u, pc.lg, __builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                    __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh));
      } else {                                                // piece cut by the window
        for (int32_t i = 0; i < n; i++)
          if (li + i >= wlo && li + i < whi) *gp(u + i) = stage[li + i];
      }
      j += a.dj;
      ib += dS;
      ub += dE;
      if (j >= a.npi) { j -= a.npi; ib += S32; ub += a.ext; }
    }
  };
  auto store_tile = [&](uint64_t t, uintptr_t lo) {
    if (a.u32) {
      store_tile32(t, lo);
      return;
    }
    const uint64_t Pa = a.P0 + t * a.K;
    const uint64_t Pb = Pa + a.K < a.P1 ? Pa + a.K : a.P1;
    uint64_t P = Pa + threadIdx.x;
    uint64_t inst = udiv(P, a.mnpi);
    uint32_t j = (uint32_t)(P - inst * a.npi);
    for (; P < Pb; P += kCB) {
      const DPiece pc = piece_at(j);
      const uint64_t sp = inst * a.S + pc.soff;
      const uint32_t n = 1u << pc.lg;
      char *u = a.user + (int64_t)inst * a.ext + pc.uoff;
      const int64_t li = (int64_t)((uintptr_t)(a.packed + (sp - a.offset)) - lo);
      if (sp >= a.offset && sp + n <= wend) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(stage + (li & ~(int64_t)3));
        const int sh = (int)(li & 3);
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
        piece_store(u, pc.lg, __builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                    __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
      } else {                                                // piece cut by the window
        for (uint32_t i = 0; i < n; i++)
          if (sp + i >= a.offset && sp + i < wend) *gp(u + i) = stage[li + i];
      }
      j += a.dj;
      inst += a.dinst;
      if (j >= a.npi) { j -= a.npi; inst++; }
    }
  };
  if constexpr (!PIPE) {
    for (uint64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
      uintptr_t lo, hi;
      range(t, lo, hi);
      __syncthreads();                                        // previous tile consumed
      {
        const uint4 *g = reinterpret_cast<const uint4 *>(lo);
        uint4 *d = reinterpret_cast<uint4 *>(stage);
        const uint32_t nv = (uint32_t)((hi - lo) / 16);
        if (a.ntld)
          for (uint32_t i = threadIdx.x; i < nv; i += kCB) d[i] = gld16p<true>(reinterpret_cast<const char *>(g + i));
        else
          for (uint32_t i = threadIdx.x; i < nv; i += kCB) d[i] = gld16(reinterpret_cast<const char *>(g + i));
      }
      __syncthreads();
      store_tile(t, lo);
    }
  } else {
    constexpr int kPre = kPieceStage / 16 / kCB;
    uint64_t t = blockIdx.x;
    if (t >= a.ntiles) return;
    uintptr_t lo, hi;
    range(t, lo, hi);
    {
      const uint4 *g = reinterpret_cast<const uint4 *>(lo);
      uint4 *d = reinterpret_cast<uint4 *>(stage);
      const uint32_t nv = (uint32_t)((hi - lo) / 16);
      for (uint32_t i = threadIdx.x; i < nv; i += kCB) d[i] = g[i];
    }
    for (;;) {
      const uint64_t tn = t + gridDim.x;
      const bool has_next = tn < a.ntiles;
      uintptr_t nlo = 0, nhi = 0;
      if (has_next) range(tn, nlo, nhi);
      uint4 pre[kPre];
      const uint32_t nvn = (uint32_t)((nhi - nlo) / 16);
#pragma unroll
      for (int k = 0; k < kPre; k++)
        if (threadIdx.x + k * kCB < nvn) pre[k] = reinterpret_cast<const uint4 *>(nlo)[threadIdx.x + k * kCB];
      __syncthreads();                                        // tile t staged
      store_tile(t, lo);
      if (!has_next) break;
      __syncthreads();                                        // tile t consumed
      {
        uint4 *d = reinterpret_cast<uint4 *>(stage);
#pragma unroll
        for (int k = 0; k < kPre; k++)
          if (threadIdx.x + k * kCB < nvn) d[threadIdx.x + k * kCB] = pre[k];
      }
      t = tn;
      lo = nlo;
    }
  }
}

// UNPACK, pieces, one piece per lane (round 6): lane P stores piece P of the
// window straight from the packed stream -- the one or two aligned 16-byte
// granules holding its bytes, loaded by the lane itself (the L2 merges the
// neighbours' overlapping loads) -- with no tile staging, no barrier and no
// persistent loop: the form of tools/pattern_floor_probe's `piece_ld2`,
// which runs at the layout's read + store floor.  Pieces cut
// by the window's ends move byte by byte.
template <bool NTLD>
__global__ void __launch_bounds__(kCB) k_unpack_piece_direct(PieceArgs a) {
  const uint64_t P = a.P0 + (uint64_t)blockIdx.x * kCB + threadIdx.x;
  if (P >= a.P1) return;
  const uint64_t inst = udiv(P, a.mnpi);
  const DPiece pc = gload<DPiece>(reinterpret_cast<const char *>(a.pieces + (P - inst * a.npi)));
  const uint64_t sp = inst * a.S + pc.soff;            // stream offset of the piece
  const uint32_t n = 1u << pc.lg;
  char *u = a.user + (int64_t)inst * a.ext + pc.uoff;
  const uint64_t wend = a.offset + a.len;
  if (sp >= a.offset && sp + n <= wend) {
    const uintptr_t src = (uintptr_t)(a.packed + (sp - a.offset));
    const char *g = reinterpret_cast<const char *>(src & ~(uintptr_t)15);
    const uint32_t sh = (uint32_t)(src & 15);
    // (a granule holding a byte of the window lies inside its 4 KiB page)
    const uint4 A = gld16p<NTLD>(g);
    const uint4 B = sh + n > 16 ? gld16p<NTLD>(g + 16) : make_uint4(0, 0, 0, 0);
    const uint32_t w[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
    const uint32_t q = sh >> 2, r = sh & 3;
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {   // w[q + k], w[q + k + 1] by selects (no indexed registers)
        lo = (uint32_t)i == q + k ? w[i] : lo;
        hi = (uint32_t)i == q + k + 1 ? w[i] : hi;
      }
      o[k] = __builtin_amdgcn_alignbyte(hi, lo, r);
    }
    piece_store(u, pc.lg, o[0], o[1], o[2], o[3]);
  } else {                                             // piece cut by the window
    for (uint32_t i = 0; i < n; i++)
      if (sp + i >= a.offset && sp + i < wend) u[i] = a.packed[sp + i - a.offset];
  }
}

// PACK, pieces: the mirror of k_unpack_piece for layouts the byte map does
// not take (instances whose map exceeds the LDS budget, sparse layouts that
// would stage mostly gaps).  Lane l loads piece l straight from user memory
// with one aligned load of the piece's width -- a wave reads 64 consecutive
// pieces, so only lines holding data are fetched -- and drops its bytes into
// the tile's packed image in LDS (whole words when the stream offset allows,
// bytes otherwise); the image leaves with 16-byte stores, the two edge
// granules a neighbouring tile shares byte by byte.
__device__ __forceinline__ void piece_load(const char *u, int lg, uint32_t &v0, uint32_t &v1, uint32_t &v2,
                                           uint32_t &v3) {
  v1 = v2 = v3 = 0;
  switch (lg) {
    case 0: v0 = *reinterpret_cast<const uint8_t *>(u); break;
    case 1: v0 = *reinterpret_cast<const uint16_t *>(u); break;
    case 2: v0 = *reinterpret_cast<const uint32_t *>(u); break;
    case 3: { const uint2 t = *reinterpret_cast<const uint2 *>(u); v0 = t.x; v1 = t.y; break; }
    default: { const uint4 t = *reinterpret_cast<const uint4 *>(u); v0 = t.x; v1 = t.y; v2 = t.z; v3 = t.w; break; }
  }
}

__global__ void __launch_bounds__(kCB) k_pack_piece(PieceArgs a) {
  extern __shared__ __align__(16) char smem[];
  char *stage = smem;                                        // kPieceStage + 48
  DPiece *stbl = reinterpret_cast<DPiece *>(smem + kPieceStage + 48);
  const DPiece *tbl = a.pieces;
  if (a.tbl_lds) {
    for (uint32_t i = threadIdx.x; i < a.npi; i += kCB) stbl[i] = a.pieces[i];
    tbl = stbl;
  }
  const uint64_t wend = a.offset + a.len;
  for (uint64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    const uint64_t Pa = a.P0 + t * a.K;
    const uint64_t Pb = Pa + a.K < a.P1 ? Pa + a.K : a.P1;
    __syncthreads();                                          // table staged / previous tile stored
    const uint64_t ia = udiv(Pa, a.mnpi), ib = udiv(Pb - 1, a.mnpi);
    const DPiece fa = tbl[Pa - ia * a.npi], fb = tbl[Pb - 1 - ib * a.npi];
    uint64_t sa = ia * a.S + fa.soff, sb = ib * a.S + fb.soff + (1u << fb.lg);
    sa = sa < a.offset ? a.offset : sa;
    sb = sb < wend ? sb : wend;
    const uintptr_t gA = (uintptr_t)(a.packed + (sa - a.offset)), gB = (uintptr_t)(a.packed + (sb - a.offset));
    const uintptr_t lo = gA & ~(uintptr_t)15;
    uint64_t P = Pa + threadIdx.x;
    uint64_t inst = udiv(P, a.mnpi);
    uint32_t j = (uint32_t)(P - inst * a.npi);
    for (; P < Pb; P += kCB) {
      const DPiece pc = tbl[j];
      const uint64_t sp = inst * a.S + pc.soff;
      const uint32_t n = 1u << pc.lg;
      const char *u = a.user + (int64_t)inst * a.ext + pc.uoff;
      const int64_t li = (int64_t)((uintptr_t)(a.packed + (sp - a.offset)) - lo);
      if (sp >= a.offset && sp + n <= wend) {
        uint32_t v[4];
        piece_load(u, pc.lg, v[0], v[1], v[2], v[3]);
        if (n >= 4 && (li & 3) == 0) {
          uint32_t *w = reinterpret_cast<uint32_t *>(stage + li);
#pragma unroll
          for (int k = 0; k < 4; k++)
            if ((uint32_t)k * 4 < n) w[k] = v[k];
        } else {
#pragma unroll
          for (int i = 0; i < 16; i++)
            if ((uint32_t)i < n) stage[li + i] = (char)(v[i >> 2] >> (8 * (i & 3)));
        }
      } else {                                                // piece cut by the window
        for (uint32_t i = 0; i < n; i++)
          if (sp + i >= a.offset && sp + i < wend) stage[li + i] = u[i];
      }
      j += a.dj;
      inst += a.dinst;
      if (j >= a.npi) { j -= a.npi; inst++; }
    }
    __syncthreads();
    const uint32_t ng = (uint32_t)((((gB + 15) & ~(uintptr_t)15) - lo) / 16);
    for (uint32_t g = threadIdx.x; g < ng; g += kCB) {
      const uintptr_t ga = lo + (uintptr_t)g * 16;
      if (ga >= gA && ga + 16 <= gB) {
        *reinterpret_cast<uint4 *>(ga) = reinterpret_cast<const uint4 *>(stage)[g];
      } else {
        for (int i = 0; i < 16; i++)
          if (ga + i >= gA && ga + i < gB) reinterpret_cast<char *>(ga)[i] = stage[g * 16 + i];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// BLOCK kernels (instances the byte map / piece tables do not take: more
// than kBmapMaxS packed bytes -- an indexed type with 10^5 blocks, a large
// triangle -- whose run tables are too long for the LDS search of the tile
// kernels; map_pos over 10^5 runs is 17 dependent global loads per lane).
// The instance is tabled once on the host as its contiguous user blocks in
// stream order (DBlk, 8 B), plus tfirst[k] = the block holding instance
// stream byte k*G (G = 256).  A workgroup owns T bytes of packed MEMORY
// (whole 16-byte granules, T <= 16 KiB chosen so that no T-byte stretch of
// the stream overlaps more than kBlkCap blocks); two lanes locate its first
// and last block (tfirst + a few-step search, L2-resident tables) and the
// workgroup stages the blocks between them -- across instance boundaries,
// user offsets relative to the first instance, stream offsets relative to
// the tile -- in LDS.  Lane l then takes granule l: one aligned 16-byte
// access on the packed side, an LDS search for its first block, and on the
// user side
//   UNPACK: the granule's bytes stored block part by block part, each part
//           cut into naturally aligned 1/2/4/8/16-byte stores (gap bytes are
//           never written);
//   PACK:   each part fetched with the one or two aligned 16-byte loads
//           under it (the loads of up to kBlkParts parts issued before any
//           is used), funnel-shifted into place; one 16-byte store.
// Only lines holding data are touched on the user side and no lane walks
// more than its own 16 bytes.
// ---------------------------------------------------------------------------
constexpr uint32_t kBlkCap = 1024;         // staged blocks per tile (16 KiB of LDS)
constexpr uint32_t kBlkG = 256;            // tfirst granularity (instance stream bytes)

// device block table entry (8 B): user offset from the instance origin and
// stream offset; a block's length is the next entry's soff minus its own
// (the table carries one sentinel entry with soff = the instance size)
struct DBlk { int32_t uoff; uint32_t soff; };
struct DBlkL { int32_t uoff; uint32_t soff, send; };   // an entry with its end, in registers
struct SBlk { int64_t u; int32_t s; uint32_t len; };   // u: from instance ia's origin; s: from the tile start

struct BlkArgs {
  const DBlk *blk;
  uint32_t nblk;
  Magic mnblk;
  const uint32_t *tfirst;  // tfirst[q / kBlkG]
  uint64_t S;
  Magic mS;
  int64_t ext;
  char *user;
  char *packed;            // window [offset, offset + len) of the stream
  uint64_t offset, len;
  uint64_t T;              // packed-memory bytes per tile (multiple of 16)
  uint64_t ntiles;
  int w4;                  // UNPACK: a granule inside one block at a 4-byte-aligned user address is one dwordx4 store
};

// block holding instance stream byte q
__device__ __forceinline__ uint32_t blk_find(const BlkArgs &a, uint64_t q) {
  const uint32_t k = (uint32_t)(q / kBlkG);
  uint32_t lo = a.tfirst[k], hi = a.tfirst[k + 1];
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (a.blk[mid].soff <= q) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// last staged block whose tile-relative start is <= x
__device__ __forceinline__ uint32_t sblk_find(const SBlk *sb, uint32_t n, int32_t x) {
  uint32_t lo = 0, hi = n - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (sb[mid].s <= x) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ unsigned __int128 u128(const uint4 v) {
  return (unsigned __int128)v.x | ((unsigned __int128)v.y << 32) | ((unsigned __int128)v.z << 64) |
         ((unsigned __int128)v.w << 96);
}

// widest naturally aligned store (<= 16 B, <= n bytes) at u, from the low bytes of w
__device__ __forceinline__ uint32_t store_piece(char *u, unsigned __int128 w, uint32_t n) {
  const uint32_t al = (uint32_t)__builtin_ctzll((uint64_t)(uintptr_t)u | 16);
  const uint32_t ln = 31u - (uint32_t)__builtin_clz(n);
  const uint32_t lg = al < ln ? al : ln;
  const uint64_t w0 = (uint64_t)w, w1 = (uint64_t)(w >> 64);
  switch (lg) {
    case 0: *reinterpret_cast<uint8_t *>(u) = (uint8_t)w0; break;
    case 1: *reinterpret_cast<uint16_t *>(u) = (uint16_t)w0; break;
    case 2: *reinterpret_cast<uint32_t *>(u) = (uint32_t)w0; break;
    case 3: *reinterpret_cast<uint64_t *>(u) = w0; break;
    default: *reinterpret_cast<uint4 *>(u) = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1,
                                                        (uint32_t)(w1 >> 32)); break;
  }
  return 1u << lg;
}

// staged block holding tile-relative stream position x
__device__ __forceinline__ uint32_t blk_search(const SBlk *sb, const uint16_t *smap, uint32_t n, uint32_t nmap,
                                               int32_t x0, int32_t x) {
  const uint32_t i = (uint32_t)(x - x0) >> 6;
  uint32_t lo = smap[i], hi = i + 1 < nmap ? smap[i + 1] : n - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (sb[mid].s <= x) lo = mid; else hi = mid - 1;
  }
  return lo;
}

constexpr int kBlkPre = 4;                         // block entries per lane (cap <= 1024)

struct SpanTile {          // what the pipeline knows of a tile before staging it
  uint64_t ia;             // first instance
  uint32_t ba, n;          // first block (instance ia), blocks overlapping
  uint32_t nv;             // 16-byte vectors of its user span
  int64_t lo;              // span start (16-aligned) as a byte offset from a.user
};

__device__ __forceinline__ void tile_geom(const BlkArgs &a, uint64_t t, uintptr_t &mlo, uintptr_t &mhi, uint64_t &tb,
                                          uint64_t &te, int32_t &x0) {
  const uintptr_t pbase = (uintptr_t)a.packed - a.offset;
  const uintptr_t wlo = (uintptr_t)a.packed, whi = wlo + a.len;
  mlo = (wlo & ~(uintptr_t)15) + t * a.T;
  mhi = mlo + a.T < whi ? mlo + a.T : whi;
  tb = (mlo > wlo ? mlo : wlo) - pbase;
  te = mhi - pbase;
  x0 = (int32_t)((int64_t)(mlo - pbase) - (int64_t)tb);
}

// lanes 2j and 2j + 1 of wave 0: the first / last byte of tile t ->
// instance, block, user offset; lane 2j returns the combined SpanTile
// (every lane of the wave must call it: the pair exchange is a shuffle)
__device__ __forceinline__ SpanTile span_search(const BlkArgs &a, uint64_t t) {
  uintptr_t mlo, mhi;
  uint64_t tb, te;
  int32_t x0;
  tile_geom(a, t, mlo, mhi, tb, te, x0);
  const uint32_t odd = threadIdx.x & 1;
  const uint64_t p = odd ? te - 1 : tb;
  const uint64_t i = udiv(p, a.mS);
  const uint64_t q = p - i * a.S;
  const uint32_t b = blk_find(a, q);
  const DBlk B = a.blk[b];
  const int64_t u = (int64_t)i * a.ext + B.uoff + (int64_t)(q - B.soff);   // user offset of byte p
  const int src = (int)(threadIdx.x | 1);
  const uint64_t i1 = __shfl(i, src);
  const uint32_t b1 = __shfl(b, src);
  const int64_t u1 = __shfl(u, src);
  SpanTile S;
  S.ia = i;
  S.ba = b;
  S.n = (uint32_t)((i1 - i) * a.nblk + b1 - b + 1);
  const uintptr_t lo = ((uintptr_t)a.user + u) & ~(uintptr_t)15;
  const uintptr_t hi = ((uintptr_t)a.user + u1 + 16) & ~(uintptr_t)15;
  S.lo = (int64_t)(lo - (uintptr_t)a.user);
  S.nv = (uint32_t)((hi - lo) / 16);
  return S;
}

// The tile directory: wave 0 searches the workgroup's next kSpanBatch tiles
// at once (one chain of dependent table loads per batch instead of per
// tile) into a ring of 2 * kSpanBatch SpanTiles.
constexpr int kSpanBatch = 32;

__device__ __forceinline__ void span_batch(const BlkArgs &a, SpanTile *dir, uint64_t i0) {
  if (threadIdx.x >= 64) return;
  const uint64_t j = i0 + threadIdx.x / 2;                    // the workgroup's j-th tile
  const uint64_t t = blockIdx.x + j * gridDim.x;
  const SpanTile S = span_search(a, t < a.ntiles ? t : blockIdx.x);
  if (!(threadIdx.x & 1) && t < a.ntiles) dir[j % (2 * kSpanBatch)] = S;
}

// The block-entry half of a tile's staging, shared by both BLOCK kernels:
// blk_prefetch issues the loads of tile U's block entries into registers
// (kBlkPre per lane), blk_commit writes them into LDS tile-relative once the
// previous tile is done with it, blk_map builds the 64-byte search map.
__device__ __forceinline__ void blk_prefetch(const BlkArgs &a, const SpanTile &U, DBlkL *pb) {
#pragma unroll
  for (int k = 0; k < kBlkPre; k++) {
    const uint32_t e = threadIdx.x + k * kCB;
    if (e < U.n) {
      const uint32_t L = U.ba + e;
      const uint32_t di = (uint32_t)udiv(L, a.mnblk);
      const DBlk *p = a.blk + (L - di * a.nblk);
      const DBlk b0 = p[0];
      pb[k].uoff = b0.uoff;
      pb[k].soff = b0.soff;
      pb[k].send = p[1].soff;
    }
  }
}

__device__ __forceinline__ void blk_commit(const BlkArgs &a, const SpanTile &U, uint64_t u, const DBlkL *pb, SBlk *sb) {
  uintptr_t mlo, mhi;
  uint64_t tb, te;
  int32_t x0;
  tile_geom(a, u, mlo, mhi, tb, te, x0);
#pragma unroll
  for (int k = 0; k < kBlkPre; k++) {
    const uint32_t e = threadIdx.x + k * kCB;
    if (e < U.n) {
      const uint32_t L = U.ba + e;
      const uint32_t di = (uint32_t)udiv(L, a.mnblk);
      SBlk x;
      x.u = (int64_t)di * a.ext + pb[k].uoff;
      x.s = (int32_t)((int64_t)((U.ia + di) * a.S + pb[k].soff) - (int64_t)tb);
      x.len = pb[k].send - pb[k].soff;
      sb[e] = x;
    }
  }
}

__device__ __forceinline__ void blk_map(const BlkArgs &a, uint32_t n, uint64_t u, const SBlk *sb, uint16_t *smap,
                                        uint32_t nmap) {
  uintptr_t mlo, mhi;
  uint64_t tb, te;
  int32_t x0;
  tile_geom(a, u, mlo, mhi, tb, te, x0);
  for (uint32_t i = threadIdx.x; i < nmap; i += kCB) {
    const int32_t x = x0 + 64 * (int32_t)i;
    smap[i] = (uint16_t)(x <= 0 ? 0 : sblk_find(sb, n, x));
  }
}

constexpr uint32_t kBlkMaxT = 65536;       // largest tile (packed-memory bytes)
constexpr uint32_t kBlkMaxMap = kBlkMaxT / 64;

// Lane l owns the 16-byte packed-memory granules l, l + kCB, ... of the
// tile, kBlkNG at a time: first every granule's block search and user
// address, then every granule's loads (unconditional: a granule with
// nothing to load reads g_blk_dummy, so no branch splits the batch), then
// the stores -- the loads of kBlkNG granules are in flight together, and
// the searches are LDS-only.  A granule inside one block (the common case
// for blocks >> 16 B) is
//   PACK:   one dwordx4 (+ one dword when the user address is not 4-byte
//           aligned, joined with alignbyte) and one 16-byte store;
//   UNPACK: one 16-byte load and one dwordx4 store (4-byte-aligned user
//           address) or naturally aligned pieces.
// A granule that straddles blocks or the window edge goes part by part:
// UNPACK stores each part in aligned pieces; PACK loads the (at most 5)
// dwords under each part, funnel-shifts them into place and ORs them in.
__device__ uint32_t g_blk_dummy[8];

template <bool PACK, int kBlkNG>
__global__ void __launch_bounds__(kCB) k_convert_blk(BlkArgs a) {
  __shared__ SBlk sb[kBlkCap];
  __shared__ uint16_t smap[kBlkMaxMap];
  __shared__ SpanTile s_t[2 * kSpanBatch];
  const uintptr_t pbase = (uintptr_t)a.packed - a.offset;   // memory address of stream byte 0
  const uintptr_t wlo = (uintptr_t)a.packed;
  const uintptr_t MA = wlo & ~(uintptr_t)15;
  char *const pk0 = a.packed - (wlo - MA);                    // MA as a (global) pointer
  const uint32_t nmap = (uint32_t)(a.T / 64);
  const char *const dummy = reinterpret_cast<const char *>(g_blk_dummy);
  const uint64_t g = gridDim.x;
  uint64_t t = blockIdx.x;
  if (t >= a.ntiles) return;
  uint64_t it = 0;                                            // t = blockIdx.x + it * g
  constexpr int kRing = 2 * kSpanBatch;
  DBlkL pb[kBlkPre];
  // the directory's first batch, tile t staged (prefetching the next
  // tile's block entries during this one's conversion measured no faster
  // here: profiles/r03/convertor_r3.txt)
  span_batch(a, s_t, 0);
  __syncthreads();
  blk_prefetch(a, s_t[0], pb);
  blk_commit(a, s_t[0], t, pb, sb);
  __syncthreads();
  blk_map(a, s_t[0].n, t, sb, smap, nmap);
  __syncthreads();
  for (;;) {
    const uint64_t u = t + g;
    const bool has_u = u < a.ntiles;
    const int cur = (int)(it % kRing), nxt = (int)((it + 1) % kRing);
    if (has_u && (it + 1) % kSpanBatch == 0) {               // tiles it + 1 .. it + kSpanBatch
      span_batch(a, s_t, it + 1);
      __syncthreads();
    }
    uintptr_t mlo, mhi;
    uint64_t tb, te;
    int32_t x0;
    tile_geom(a, t, mlo, mhi, tb, te, x0);
    const uint32_t n = s_t[cur].n;
    char *ubase = a.user + (int64_t)s_t[cur].ia * a.ext;
    for (uintptr_t gb = mlo + (uintptr_t)threadIdx.x * 16; gb < mhi; gb += (uintptr_t)kCB * 16 * kBlkNG) {
      int32_t xs[kBlkNG], xe[kBlkNG];
      uint32_t es[kBlkNG];
      int st[kBlkNG];                                         // 0 none, 1 inside one block, 2 part by part
      char *up[kBlkNG];
#pragma unroll
      for (int k = 0; k < kBlkNG; k++) {
        const uintptr_t ga = gb + (uintptr_t)k * kCB * 16;
        st[k] = 0;
        up[k] = nullptr;
        if (ga < mhi) {
          const uintptr_t m0 = ga > wlo ? ga : wlo, m1 = ga + 16 < mhi ? ga + 16 : mhi;
          xs[k] = (int32_t)(m0 - pbase - tb);                 // tile-relative stream positions
          xe[k] = (int32_t)(m1 - pbase - tb);
          es[k] = blk_search(sb, smap, n, nmap, x0, xs[k]);
          const SBlk B = sb[es[k]];
          up[k] = ubase + B.u + (xs[k] - B.s);
          st[k] = (m0 == ga && m1 == ga + 16 && xs[k] + 16 <= B.s + (int32_t)B.len) ? 1 : 2;
        }
      }
      if (!PACK) {
        uint4 v[kBlkNG];
#pragma unroll
        for (int k = 0; k < kBlkNG; k++) {
          const char *g = st[k] ? pk0 + (gb - MA) + (uintptr_t)k * kCB * 16 : dummy;
          v[k] = gld16(g);
        }
#pragma unroll
        for (int k = 0; k < kBlkNG; k++) {
          if (st[k] == 1 && ((uintptr_t)up[k] & 3) == 0 && a.w4) {
            W4 w;
            w.x = v[k].x; w.y = v[k].y; w.z = v[k].z; w.w = v[k].w;
            *reinterpret_cast<W4 *>(up[k]) = w;
          } else if (st[k]) {
            const int32_t xg = (int32_t)(gb + (uintptr_t)k * kCB * 16 - pbase - tb);
            const unsigned __int128 vv = u128(v[k]);
            int32_t x = xs[k];
            uint32_t e = es[k];
            while (x < xe[k]) {
              const SBlk B = sb[e++];
              const int32_t bend = B.s + (int32_t)B.len;
              const int32_t stop = bend < xe[k] ? bend : xe[k];
              char *u = ubase + B.u + (x - B.s);
              unsigned __int128 w = vv >> (8 * (x - xg));
              uint32_t left = (uint32_t)(stop - x);
              while (left) {
                const uint32_t q = store_piece(u, w, left);
                u += q;
                left -= q;
                w = q == 16 ? 0 : (w >> (8 * q));
              }
              x = stop;
            }
          }
        }
      } else {
        W4 l[kBlkNG];
        uint32_t h[kBlkNG];
#pragma unroll
        for (int k = 0; k < kBlkNG; k++) {
          const uint32_t sh = (uint32_t)((uintptr_t)up[k] & 3);
          const char *p4 = st[k] == 1 ? up[k] - sh : dummy;
          const char *ph = st[k] == 1 && sh ? up[k] - sh + 16 : dummy;
          l[k] = gld16a4(p4);
          h[k] = gld4(ph);
        }
#pragma unroll
        for (int k = 0; k < kBlkNG; k++) {
          char *gp = pk0 + (gb - MA) + (uintptr_t)k * kCB * 16;
          if (st[k] == 1) {
            const uint32_t sh = (uint32_t)((uintptr_t)up[k] & 3);
            *reinterpret_cast<uint4 *>(gp) =
                make_uint4(__builtin_amdgcn_alignbyte(l[k].y, l[k].x, sh), __builtin_amdgcn_alignbyte(l[k].z, l[k].y, sh),
                           __builtin_amdgcn_alignbyte(l[k].w, l[k].z, sh), __builtin_amdgcn_alignbyte(h[k], l[k].w, sh));
          } else if (st[k] == 2) {
            const int32_t xg = (int32_t)(gb + (uintptr_t)k * kCB * 16 - pbase - tb);
            unsigned __int128 acc = 0;
            int32_t x = xs[k];
            uint32_t e = es[k];
            while (x < xe[k]) {
              const SBlk B = sb[e++];
              const int32_t bend = B.s + (int32_t)B.len;
              const int32_t stop = bend < xe[k] ? bend : xe[k];
              const char *u = ubase + B.u + (x - B.s);
              const uint32_t pn = (uint32_t)(stop - x), sh = (uint32_t)((uintptr_t)u & 3);
              const char *u4 = u - sh;
              const uint32_t nd = (sh + pn + 3) / 4;            // dwords holding the part (<= 5)
              uint32_t d[5];
#pragma unroll
              for (int j = 0; j < 5; j++)
                d[j] = gld4((uint32_t)j < nd ? u4 + 4 * j : dummy);
              const uint32_t w0 = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
              const uint32_t w1 = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
              const uint32_t w2 = __builtin_amdgcn_alignbyte(d[3], d[2], sh);
              const uint32_t w3 = __builtin_amdgcn_alignbyte(d[4], d[3], sh);
              unsigned __int128 w = (unsigned __int128)w0 | ((unsigned __int128)w1 << 32) |
                                    ((unsigned __int128)w2 << 64) | ((unsigned __int128)w3 << 96);
              if (pn < 16) w &= (((unsigned __int128)1) << (8 * pn)) - 1;
              acc |= w << (8 * (x - xg));
              x = stop;
            }
            if (xs[k] == xg && xe[k] == xg + 16) {
              *reinterpret_cast<uint4 *>(gp) = make_uint4((uint32_t)acc, (uint32_t)(acc >> 32), (uint32_t)(acc >> 64),
                                                          (uint32_t)(acc >> 96));
            } else {                                          // window edge: the bytes inside only
              for (int32_t i = xs[k]; i < xe[k]; i++) gp[i - xg] = (char)(acc >> (8 * (i - xg)));
            }
          }
        }
      }
    }
    __syncthreads();                                          // tile t's LDS is free
    if (!has_u) break;
    blk_prefetch(a, s_t[nxt], pb);
    blk_commit(a, s_t[nxt], u, pb, sb);
    __syncthreads();
    blk_map(a, s_t[nxt].n, u, sb, smap, nmap);
    __syncthreads();
    t = u;
    it++;
  }
}

// PACK of monotonic layouts, span-staged: a tile's user bytes all lie in
// [addr(first byte), addr(last byte)] (at most kBlkSpan bytes: the host's
// choice of T), so the workgroup stages that span in LDS with coalesced
// 16-byte loads (every lane's loads in flight at once) and each lane then
// gathers its granule from LDS -- one 16-byte run of LDS dwords joined with
// alignbyte when the granule lies inside one block, part by part otherwise
// -- and leaves with one 16-byte store.  User lines are read once, whole;
// no lane waits on a dependent global load after the staging.
constexpr uint32_t kBlkSpan = 24576;
constexpr int kBlkSpanPer = kBlkSpan / 16 / kCB;   // uint4 per lane

// (pointer arithmetic, not an integer round trip: the compiler must keep
// seeing an LDS pointer -- a flat access would merge the dwords into one
// 16-byte load that LDS cannot serve at 4-byte alignment)
__device__ __forceinline__ unsigned __int128 lds16(const char *p) {   // 16 bytes at any LDS alignment
  const uint32_t *w = reinterpret_cast<const uint32_t *>(p - ((uintptr_t)p & 3));
  const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
  const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4];
  return (unsigned __int128)__builtin_amdgcn_alignbyte(d1, d0, sh) |
         ((unsigned __int128)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32) |
         ((unsigned __int128)__builtin_amdgcn_alignbyte(d3, d2, sh) << 64) |
         ((unsigned __int128)__builtin_amdgcn_alignbyte(d4, d3, sh) << 96);
}

// Software pipeline (persistent workgroups, tiles t, t + grid, ...): while
// the lanes gather tile t out of LDS, tile t + grid's block entries and user
// span are already in flight into registers, located through the tile
// directory (span_batch) -- no tile waits on a chain of dependent loads.
__global__ void __launch_bounds__(kCB) k_pack_blk_span(BlkArgs a, uint32_t cap) {
  extern __shared__ __align__(16) char smem[];
  char *span = smem;                                          // kBlkSpan + 32
  SBlk *sb = reinterpret_cast<SBlk *>(smem + kBlkSpan + 32);  // cap
  uint16_t *smap = reinterpret_cast<uint16_t *>(sb + cap);    // T / 64
  __shared__ SpanTile s_t[2 * kSpanBatch];
  const uintptr_t pbase = (uintptr_t)a.packed - a.offset;
  const uintptr_t wlo = (uintptr_t)a.packed;
  const uintptr_t MA = wlo & ~(uintptr_t)15;
  char *const pk0 = a.packed - (wlo - MA);
  const uint32_t nmap = (uint32_t)(a.T / 64);
  const uint64_t g = gridDim.x;
  uint64_t t = blockIdx.x;
  if (t >= a.ntiles) return;
  uint64_t it = 0;                                            // t = blockIdx.x + it * g
  constexpr int kRing = 2 * kSpanBatch;
  // registers of the tile in flight
  DBlkL pb[kBlkPre];
  uint4 ps[kBlkSpanPer];
  // issue the loads of tile u (its SpanTile in s_t[slot]) into pb / ps
  auto prefetch = [&](int slot) {
    const SpanTile U = s_t[slot];
    blk_prefetch(a, U, pb);
    const char *lo = a.user + U.lo;
#pragma unroll
    for (int k = 0; k < kBlkSpanPer; k++) {
      const uint32_t i = threadIdx.x + k * kCB;
      if (i < U.nv) ps[k] = gld16(lo + 16 * i);
    }
  };
  // move the registers of tile u into LDS (blocks tile-relative)
  auto commit = [&](int slot, uint64_t u) {
    const SpanTile U = s_t[slot];
    blk_commit(a, U, u, pb, sb);
#pragma unroll
    for (int k = 0; k < kBlkSpanPer; k++) {
      const uint32_t i = threadIdx.x + k * kCB;
      if (i < U.nv) reinterpret_cast<uint4 *>(span)[i] = ps[k];
    }
  };
  auto build_map = [&](int slot, uint64_t u) { blk_map(a, s_t[slot].n, u, sb, smap, nmap); };
  // prologue: the first batch of the directory, tile t staged
  span_batch(a, s_t, 0);
  __syncthreads();
  prefetch(0);
  commit(0, t);
  __syncthreads();
  build_map(0, t);
  __syncthreads();
  for (;;) {
    const uint64_t u = t + g;
    const bool has_u = u < a.ntiles;
    const int cur = (int)(it % kRing), nxt = (int)((it + 1) % kRing);
    if (has_u && (it + 1) % kSpanBatch == 0) {               // tiles it + 1 .. it + kSpanBatch
      span_batch(a, s_t, it + 1);
      __syncthreads();
    }
    if (has_u) prefetch(nxt);
    // gather tile t
    {
      const SpanTile T0 = s_t[cur];
      uintptr_t mlo, mhi;
      uint64_t tb, te;
      int32_t x0;
      tile_geom(a, t, mlo, mhi, tb, te, x0);
      const uint32_t n = T0.n;
      const char *ubase = a.user + (int64_t)T0.ia * a.ext;
      const int64_t d0 = (int64_t)(ubase - (a.user + T0.lo));   // LDS offset of user offset 0 of instance ia
      for (uintptr_t ga = mlo + (uintptr_t)threadIdx.x * 16; ga < mhi; ga += (uintptr_t)kCB * 16) {
        const uintptr_t m0 = ga > wlo ? ga : wlo, m1 = ga + 16 < mhi ? ga + 16 : mhi;
        const int32_t xs = (int32_t)(m0 - pbase - tb), xe = (int32_t)(m1 - pbase - tb);
        const int32_t xg = (int32_t)(ga - pbase - tb);
        uint32_t e = blk_search(sb, smap, n, nmap, x0, xs);
        char *gp = pk0 + (ga - MA);
        SBlk B = sb[e];
        if (xs == xg && xe == xg + 16 && xs + 16 <= B.s + (int32_t)B.len) {
          const unsigned __int128 v = lds16(span + d0 + B.u + (xs - B.s));
          *reinterpret_cast<uint4 *>(gp) =
              make_uint4((uint32_t)v, (uint32_t)(v >> 32), (uint32_t)(v >> 64), (uint32_t)(v >> 96));
          continue;
        }
        unsigned __int128 acc = 0;
        int32_t x = xs;
        while (x < xe) {
          B = sb[e++];
          const int32_t bend = B.s + (int32_t)B.len;
          const int32_t stop = bend < xe ? bend : xe;
          const uint32_t pn = (uint32_t)(stop - x);
          unsigned __int128 v = lds16(span + d0 + B.u + (x - B.s));
          if (pn < 16) v &= (((unsigned __int128)1) << (8 * pn)) - 1;
          acc |= v << (8 * (x - xg));
          x = stop;
        }
        if (xs == xg && xe == xg + 16) {
          *reinterpret_cast<uint4 *>(gp) =
              make_uint4((uint32_t)acc, (uint32_t)(acc >> 32), (uint32_t)(acc >> 64), (uint32_t)(acc >> 96));
        } else {
          for (int32_t i = xs; i < xe; i++) gp[i - xg] = (char)(acc >> (8 * (i - xg)));
        }
      }
    }
    __syncthreads();                                          // tile t's LDS is free
    if (!has_u) break;
    commit(nxt, u);
    __syncthreads();
    build_map(nxt, u);
    __syncthreads();
    t = u;
    it++;
  }
}

}  // namespace mx

using namespace mx;

struct HBlk { int64_t uoff; uint32_t soff; uint32_t len; };   // host side of the block table (blk_tab)

struct mx_ddt {
  std::vector<DRun> host;
  DRun *dev;
  size_t size;
  int64_t lb, ub;
  uint64_t gcd_all;  // gcd of every disp/stride/blen/extent (access unit)
  Magic mS;          // divide by size
  bool monotonic;    // user addresses strictly increase along the stream
  // byte map of one instance (size <= kBmapMaxS): bmap[b] = user offset of
  // packed byte b.  PACK kernel k_pack_bmap stages (bmap - umin) as 16-bit
  // (user span < 64 KiB) or 32-bit words when they fit kBmapLds.
  std::vector<int32_t> bmap;
  void *map_dev = nullptr;
  int map16 = 0;
  int64_t umin = 0, uspan = 0;
  uint64_t bmap_T = 0;             // stream bytes per PACK tile (0: no PACK kernel)
  uint64_t bmap_Ts[3] = {0, 0, 0}; // the same for staged spans kBmapSpans[0..2] (bmap_T = [1])
  bool bmap_quad = false;          // the PACK kernel stages the map as quads (BmapArgs::qsh)
  bool bmap_cw = false;            // >= 90 % of packed dwords are 4 user-contiguous bytes (BmapArgs::cw)
  bool bmap_word = false;          // every dword at a phase 4k is (BmapArgs::word)
  bool piece_pack = false;         // PACK takes the piece kernel (wide word-aligned pieces, build_bmap)
  // piece tables per user-origin alignment (address mod 16), built on first
  // use: UNPACK kernel k_unpack_piece
  struct PieceTab {
    std::vector<DPiece> host;
    DPiece *dev = nullptr;
    uint32_t K = 0;                // pieces per tile
    int built = 0;                 // 1 ok, -1 not applicable
  } ptab[16];
  // UNPACK through piece tables: the LDS-staged tile kernel or one piece per
  // lane, chosen per datatype by measurement (round 6: one piece per lane is
  // 0.83x the staged kernel's time for BLACS and 1.4-1.6x for `ref_struct` /
  // `ref_strange`, profiles/r06/unpack_direct_ab_r6x.txt).  The first two
  // unpacks of >= 4 MiB run one form each between HIP events; once both
  // have completed, the faster per byte is kept (0 undecided, 1 staged,
  // 2 one piece per lane).  Both forms write the same bytes.
  std::mutex up_mu;
  int up_choice = 0;
  int up_tried = 0;                // bit v: form v + 1 launched with events
  hipEvent_t up_ev[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  double up_bytes[2] = {0, 0};
  // contiguous user blocks of one instance in stream order + tfirst (BLOCK
  // kernels k_convert_blk), built on first use for instances the byte map
  // does not take
  struct BlkTab {
    std::vector<HBlk> host;        // the blocks (the device table adds the sentinel)
    DBlk *dev = nullptr;
    uint32_t *tfirst = nullptr;
    uint64_t T = 0;                // packed-memory bytes per tile
    uint64_t Tspan = 0;            // PACK through k_pack_blk_span: its tile (0: not applicable)
    uint32_t capspan = 0;          // most blocks one of its tiles overlaps
    int built = 0;                 // 1 ok, -1 not applicable
  } btab;
  int force_blk = 0;               // mx_ddt_set_path(MX_DDT_PATH_BLOCK)
  std::atomic<int> last_path{0};   // mx_ddt_last_path
  std::mutex mu;
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

static Magic make_magic(uint64_t d) {
  Magic M;
  int l = 0;
  while (l < 64 && (((unsigned __int128)1) << l) < d) l++;
  M.k = (uint32_t)(kMagicBits + l);
  const unsigned __int128 two_k = ((unsigned __int128)1) << M.k;
  M.m = (uint64_t)((two_k + d - 1) / d);
  M.pad = 0;
  return M;
}

// Every byte of the stream lies at a higher user address than the one
// before it (runs, blocks and instances in address order, no overlap):
// then a tile's bytes all lie in [addr(first), addr(last)].
static bool is_monotonic(const std::vector<DRun> &runs, int64_t ext) {
  if (runs.empty()) return false;
  int64_t prev_end = INT64_MIN;   // one past the last byte so far
  for (const DRun &r : runs) {
    if (r.cnt1 > 1 && r.stride1 < (int64_t)r.blen) return false;
    const int64_t inner = (int64_t)(r.cnt1 - 1) * r.stride1 + (int64_t)r.blen;
    if (r.cnt2 > 1 && r.stride2 < inner) return false;
    if (r.disp < prev_end) return false;
    prev_end = r.disp + (int64_t)(r.cnt2 - 1) * r.stride2 + inner;
  }
  return prev_end <= ext + runs[0].disp;   // next instance starts after
}

static uint64_t gcd64(uint64_t a, uint64_t b) {
  while (b) { uint64_t t = a % b; a = b; b = t; }
  return a;
}
static uint64_t absg(int64_t v) { return v < 0 ? (uint64_t)(-v) : (uint64_t)v; }

// Pieces of one instance for a user origin at address `al` mod 16: maximal
// contiguous user runs in stream order, cut into naturally aligned
// 1/2/4/8/16-byte pieces (aligned for every instance: the width also
// divides the extent).
static void cut_pieces(const mx_ddt *d, int al, std::vector<DPiece> &v) {
  const uint64_t A = gcd64(16, absg(d->ub - d->lb));
  const size_t S = d->bmap.size();
  for (size_t b = 0; b < S;) {
    size_t L = 1;
    while (b + L < S && d->bmap[b + L] == d->bmap[b] + (int32_t)L) L++;
    for (size_t pos = 0; pos < L;) {
      const int64_t x = (int64_t)d->bmap[b] + (int64_t)pos;
      const uint64_t addr = (uint64_t)(((al + x) % 16 + 16) % 16);
      uint64_t w = 16;
      while (w > 1 && (addr % w || w > L - pos || A % w)) w >>= 1;
      DPiece pc;
      pc.uoff = (int32_t)x;
      pc.soff = (uint16_t)(b + pos);
      pc.lg = (uint8_t)__builtin_ctzll(w);
      pc.pad = 0;
      v.push_back(pc);
      pos += w;
    }
    b += L;
  }
}

// Byte map of one instance: bmap[b] = user offset of packed byte b.  Also
// fixes the PACK tile: the largest multiple of 256 stream bytes (<= 16 KiB)
// whose user span, rounded out to 16 bytes, always fits kBmapSpan -- whole
// instances for a non-monotonic layout, [addr(first), addr(last)] for a
// monotonic one.
// MX_CONV_BMAP_INST=0: the byte-map PACK's tiles of non-monotonic layouts
// stay multiples of 256 stream bytes instead of whole instances (A/B switch;
// read at datatype creation)
static bool conv_bmap_inst_tiles() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_BMAP_INST");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

static void build_bmap(mx_ddt *d) {
  const int64_t ext = d->ub - d->lb;
  const uint64_t S = d->size;
  if (S == 0 || S > kBmapMaxS || ext <= 0) return;
  std::vector<int32_t> m;
  m.reserve(S);
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  for (const DRun &r : d->host)
    for (uint64_t l2 = 0; l2 < r.cnt2; l2++)
      for (uint64_t l1 = 0; l1 < r.cnt1; l1++)
        for (uint64_t o = 0; o < r.blen; o++) {
          const int64_t u = r.disp + (int64_t)l2 * r.stride2 + (int64_t)l1 * r.stride1 + (int64_t)o;
          if (u < INT32_MIN || u > INT32_MAX) return;
          m.push_back((int32_t)u);
          lo = std::min(lo, u);
          hi = std::max(hi, u + 1);
        }
  if (m.size() != S) return;
  d->bmap.swap(m);
  d->umin = lo;
  d->uspan = hi - lo;
  // 16-bit map entries when every entry of the kernel's wrapped table
  // (bmap + ext for the three bytes past an instance) fits
  d->map16 = d->uspan + (int64_t)((S + 2) / S) * ext <= 65536;
  // PACK kernel choice: pieces of >= 8 bytes on average that all land on
  // whole packed words move with few wide accesses through the piece kernel;
  // narrow or misaligned pieces go through the byte map, whose cost per
  // byte is flat.  Measured at 1 GiB (profiles/r02/convertor_r2.txt): lower
  // triangle (8-byte pieces) piece 3.58 vs byte map 2.28 TB/s; indexed /
  // BLACS (4-byte) 2.66 / 2.85 vs 3.40 / 3.05; struct (misaligned) 2.46 vs
  // 3.41; 8-byte struct types equal within 2 %.
  {
    std::vector<DPiece> v;
    cut_pieces(d, 0, v);
    bool words = true;
    for (const DPiece &p : v) words = words && p.lg >= 2 && (p.soff & 3) == 0;
    d->piece_pack = words && !v.empty() && S >= 8 * v.size();
  }
  // The byte map is staged only for dense layouts (<= 4 user bytes per
  // packed byte; a sparse one reads mostly gaps -- ref_matrix_borders at 23:
  // 0.83 -> 0.42 TB/s) and maps small enough for >= 3 workgroups per CU
  // (ref_upper_matrix_60's 29 KiB map: 1.32 -> 1.25 TB/s)
  if ((S + 3) * (d->map16 ? 2 : 4) > kBmapLds || ext > 4 * (int64_t)S || d->uspan > 4 * (int64_t)S) return;
  d->bmap_quad = S % 4 != 0 && 4 * S * (d->map16 ? 2 : 4) <= kBmapLds;
  {                                // packed dwords whose 4 bytes are user-contiguous, by instance phase
    auto Ux = [&](uint64_t x) { return (int64_t)(x / S) * ext + d->bmap[x % S]; };
    uint64_t c = 0;
    for (uint64_t b = 0; b < S; b++) c += Ux(b + 3) == Ux(b) + 3 && Ux(b + 1) == Ux(b) + 1 && Ux(b + 2) == Ux(b) + 2;
    d->bmap_cw = c * 10 >= 9 * S;
    uint64_t cwd = 0;                // at the phases a dword of a 16-aligned tile starts at
    for (uint64_t b = 0; b < S; b += 4)
      cwd += Ux(b + 3) == Ux(b) + 3 && Ux(b + 1) == Ux(b) + 1 && Ux(b + 2) == Ux(b) + 2;
    d->bmap_word = S % 4 == 0 && cwd == S / 4;
  }
  // user bytes a tile of T stream bytes starting at instance byte b touches
  auto U = [&](uint64_t x) { return (int64_t)(x / S) * ext + d->bmap[x % S]; };
  auto worst = [&](uint64_t T) {
    if (!d->monotonic) return (int64_t)(((T - 1) / S + 1) * (uint64_t)ext) + d->uspan;
    int64_t w = 0;
    for (uint64_t b = 0; b < S; b++) w = std::max<int64_t>(w, U(b + T - 1) - U(b) + 1);
    return w;
  };
  // the largest T (a multiple of 256, at most 2/3 of the span) whose worst
  // user span + 160 fits: the span staged from a 128-byte line start
  // (MX_CONV_BMAP_ALIGN) plus its 16-byte rounding up.  worst() grows with T.
  for (int k = 0; k < 3; k++) {
    const int64_t span = kBmapSpans[k];
    uint64_t lo = 0, hi = (uint64_t)span * 2 / 3 / 256;      // in units of 256
    while (lo < hi) {
      const uint64_t mid = (lo + hi + 1) / 2;
      if (worst(mid * 256) + 160 <= span) lo = mid;
      else hi = mid - 1;
    }
    d->bmap_Ts[k] = lo * 256;
    // a layout that is not monotonic stages whole instances per tile; when
    // S % 16 == 0 a tile of exactly k instances starts (from offset 0) on an
    // instance boundary and stages k of them, not the k + 1 a tile cut
    // mid-instance does (indexed: 12.9 instead of 19.3 KiB per 10 KiB of stream)
    if (!d->monotonic && S % 16 == 0) {
      const int64_t kk = (span - 160 - d->uspan) / ext;   // worst(kk * S) + 160 <= span
      if (kk >= 1 && (uint64_t)kk * S >= 256 && (uint64_t)kk * S <= (uint64_t)span * 2 / 3 &&
          worst((uint64_t)kk * S) + 160 <= span && conv_bmap_inst_tiles())
        d->bmap_Ts[k] = (uint64_t)kk * S;
    }
  }
  d->bmap_T = d->bmap_Ts[1];
}

// The piece table for a user origin at address `al` mod 16 (cut_pieces),
// uploaded, with its tile size.  Caller holds d->mu.
static mx_ddt::PieceTab *piece_tab(mx_ddt *d, int al) {
  mx_ddt::PieceTab &P = d->ptab[al];
  if (P.built) return P.built > 0 ? &P : nullptr;
  P.built = -1;
  const size_t S = d->bmap.size();
  std::vector<DPiece> v;
  cut_pieces(d, al, v);
  const uint32_t npi = (uint32_t)v.size();
  // pieces per tile: ~8 KiB of stream, staged bytes (+ alignment slop) <= kPieceStage
  auto window = [&](uint32_t K) {
    uint64_t mx = 0;
    for (uint32_t j = 0; j < npi; j++) {
      const uint64_t e = (uint64_t)j + K - 1;
      const DPiece &pe = v[e % npi];
      const uint64_t end = (e / npi) * S + pe.soff + (1u << pe.lg);
      mx = std::max<uint64_t>(mx, end - v[j].soff);
    }
    return mx;
  };
  uint64_t K = std::max<uint64_t>(kCB, std::min<uint64_t>(4096, (8192ull * npi / S) / kCB * kCB));
  while (K > kCB && window((uint32_t)K) + 32 > (uint64_t)kPieceStage) K -= kCB;
  if (window((uint32_t)K) + 32 > (uint64_t)kPieceStage) return nullptr;
  if (hipMalloc((void **)&P.dev, npi * sizeof(DPiece)) != hipSuccess) { P.dev = nullptr; return nullptr; }
  if (hipMemcpy(P.dev, v.data(), npi * sizeof(DPiece), hipMemcpyHostToDevice) != hipSuccess) {
    release_later(P.dev, REL_DEV);
    P.dev = nullptr;
    return nullptr;
  }
  P.host.swap(v);
  P.K = (uint32_t)K;
  P.built = 1;
  return &P;
}

// BLOCK kernel geometry (A/B switches; results are identical):
// MX_CONV_BLK_T = largest tile (4096 .. 65536 packed bytes, default 16384),
// MX_CONV_BLK_NG = granules per lane in flight (1, 2, 4; default 2 for
// PACK -- layouts the span kernel does not take -- and 4 for UNPACK:
// measured, profiles/r03/convertor_r3.txt),
// MX_CONV_BLK_W4=0 stores every UNPACK granule in naturally aligned pieces.
static uint64_t conv_blk_tmax() {
  static const uint64_t t = [] {
    const char *e = getenv("MX_CONV_BLK_T");
    const long v = e ? atol(e) : 16384;
    return (uint64_t)((v >= 4096 && v <= (long)kBlkMaxT && (v & (v - 1)) == 0) ? v : 16384);
  }();
  return t;
}
static int conv_blk_ng(bool pack) {
  static const int g = [] {
    const char *e = getenv("MX_CONV_BLK_NG");
    const int v = e ? atoi(e) : 0;
    return (v == 1 || v == 2 || v == 4) ? v : 0;
  }();
  return g ? g : (pack ? 2 : 4);
}
// MX_CONV_BLK_SPAN=0 keeps PACK of monotonic layouts on the granule
// kernel instead of the span-staged one (A/B switch).
static bool conv_blk_span() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_BLK_SPAN");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}
static int conv_blk_w4() {
  static const int w = [] {
    const char *e = getenv("MX_CONV_BLK_W4");
    return (e && *e == '0') ? 0 : 1;
  }();
  return w;
}

// The block table of k_convert_blk (caller holds d->mu): the instance's
// contiguous user blocks in stream order (touching blocks merged), tfirst[k]
// = the block holding instance stream byte k * kBlkG (one entry past the
// last stretch, so [tfirst[k], tfirst[k + 1]] always brackets the search),
// and the tile T: the largest of 16 KiB .. 512 B of packed memory whose
// stream stretch never overlaps more than kBlkCap blocks (a T-byte stretch
// overlaps at most the blocks from b to the one holding end(b) - 2 + T,
// over every block b, across instance boundaries).
static mx_ddt::BlkTab *blk_tab(mx_ddt *d) {
  mx_ddt::BlkTab &B = d->btab;
  if (B.built) return B.built > 0 ? &B : nullptr;
  B.built = -1;
  const uint64_t S = d->size;
  const int64_t ext = d->ub - d->lb;
  constexpr uint64_t kMaxBlocks = (uint64_t)1 << 22;
  if (S == 0 || S >= ((uint64_t)1 << 31) || ext <= 0) return nullptr;
  std::vector<HBlk> v;
  uint64_t soff = 0;
  for (const DRun &r : d->host) {
    if (v.size() + r.cnt1 * r.cnt2 > kMaxBlocks + 1) return nullptr;
    for (uint64_t l2 = 0; l2 < r.cnt2; l2++)
      for (uint64_t l1 = 0; l1 < r.cnt1; l1++) {
        const int64_t u = r.disp + (int64_t)l2 * r.stride2 + (int64_t)l1 * r.stride1;
        if (!v.empty() && v.back().uoff + (int64_t)v.back().len == u && v.back().len + r.blen < ((uint64_t)1 << 31)) {
          v.back().len += (uint32_t)r.blen;
        } else {
          HBlk b;
          b.uoff = u;
          b.soff = (uint32_t)soff;
          b.len = (uint32_t)r.blen;
          v.push_back(b);
        }
        soff += r.blen;
      }
  }
  if (v.empty() || v.size() > kMaxBlocks || soff != S) return nullptr;
  const uint64_t nb = v.size();
  auto max_overlap = [&](uint64_t T) {
    uint64_t mx = 0, j = 0;
    for (uint64_t b = 0; b < nb; b++) {
      const uint64_t last = (uint64_t)v[b].soff + v[b].len - 1 + T - 1;   // end(b) - 2 + T
      if (j < b) j = b;
      // advance j to the block holding `last` (monotonic in b)
      while (true) {
        const uint64_t jn = j + 1, i = jn / nb;
        const uint64_t start = i * S + v[jn - i * nb].soff;
        if (start > last) break;
        j = jn;
      }
      mx = std::max<uint64_t>(mx, j - b + 1);
    }
    return mx;
  };
  uint64_t T = conv_blk_tmax();
  while (T > 512 && max_overlap(T) > kBlkCap) T /= 2;
  if (max_overlap(T) > kBlkCap) return nullptr;
  // span PACK (k_pack_blk_span): monotonic blocks; the user span of a
  // T-byte stretch that starts in block b and ends in block j is
  // T + G(j) - G(b), G = user offset - stream offset (non-decreasing), so
  // its maximum over stretches starting in b is at the last j reachable
  bool mono = true;
  for (uint64_t b = 0; b + 1 < nb && mono; b++) mono = v[b].uoff + (int64_t)v[b].len <= v[b + 1].uoff;
  mono = mono && v[nb - 1].uoff + (int64_t)v[nb - 1].len <= v[0].uoff + ext;
  uint64_t Ts = 0, caps = 0;
  if (mono && conv_blk_span()) {
    auto G = [&](uint64_t j) {
      const uint64_t i = j / nb;
      return ((int64_t)i * ext + v[j - i * nb].uoff) - (int64_t)(i * S + v[j - i * nb].soff);
    };
    auto max_span = [&](uint64_t TT) {
      int64_t mx = 0;
      uint64_t j = 0;
      for (uint64_t b = 0; b < nb; b++) {
        const uint64_t last = (uint64_t)v[b].soff + v[b].len - 1 + TT - 1;
        if (j < b) j = b;
        while (true) {
          const uint64_t jn = j + 1, i = jn / nb;
          if (i * S + v[jn - i * nb].soff > last) break;
          j = jn;
        }
        mx = std::max<int64_t>(mx, G(j) - G(b));
      }
      return (int64_t)TT + mx;
    };
    for (uint64_t TT = 16384; TT >= 2048; TT /= 2) {
      if (max_overlap(TT) <= kBlkCap && max_span(TT) + 32 <= (int64_t)kBlkSpan) {
        Ts = TT;
        caps = max_overlap(TT) + 1;
        break;
      }
    }
  }
  const uint64_t nk = (S + kBlkG - 1) / kBlkG;
  std::vector<uint32_t> tf(nk + 1);
  for (uint64_t k = 0, b = 0; k < nk; k++) {
    while (b + 1 < nb && v[b + 1].soff <= k * kBlkG) b++;
    tf[k] = (uint32_t)b;
  }
  tf[nk] = (uint32_t)(nb - 1);
  std::vector<DBlk> dv(nb + 1);
  for (uint64_t b = 0; b < nb; b++) {
    if (v[b].uoff < INT32_MIN || v[b].uoff > INT32_MAX) return nullptr;   // instance offsets beyond +-2 GiB
    dv[b].uoff = (int32_t)v[b].uoff;
    dv[b].soff = v[b].soff;
  }
  dv[nb].uoff = 0;
  dv[nb].soff = (uint32_t)S;
  if (hipMalloc((void **)&B.dev, (nb + 1) * sizeof(DBlk)) != hipSuccess) { B.dev = nullptr; return nullptr; }
  if (hipMalloc((void **)&B.tfirst, (nk + 1) * sizeof(uint32_t)) != hipSuccess) {
    release_later(B.dev, REL_DEV);
    B.dev = nullptr;
    B.tfirst = nullptr;
    return nullptr;
  }
  if (hipMemcpy(B.dev, dv.data(), (nb + 1) * sizeof(DBlk), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(B.tfirst, tf.data(), (nk + 1) * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
    release_later(B.dev, REL_DEV);
    release_later(B.tfirst, REL_DEV);
    B.dev = nullptr;
    B.tfirst = nullptr;
    return nullptr;
  }
  B.host.swap(v);
  B.T = T;
  B.Tspan = Ts;
  B.capspan = (uint32_t)caps;
  B.built = 1;
  return &B;
}

// index of the piece holding packed byte b of an instance
static uint32_t piece_of(const std::vector<DPiece> &v, uint64_t b) {
  uint32_t lo = 0, hi = (uint32_t)v.size() - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) / 2;
    if (v[mid].soff <= b) lo = mid; else hi = mid - 1;
  }
  return lo;
}

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
  for (DRun &r : d->host) {
    r.mblen = make_magic(r.blen);
    r.mcnt1 = make_magic(r.cnt1);
  }
  d->size = size;
  d->lb = lb;
  d->ub = ub;
  d->gcd_all = gcd64(g, absg(ub - lb));
  d->mS = make_magic(size ? size : 1);
  d->monotonic = is_monotonic(d->host, ub - lb);
  d->dev = nullptr;
  if (!d->host.empty()) {
    if ((rc = mx_ensure_init())) { delete d; return rc; }
    if (hipMalloc((void **)&d->dev, d->host.size() * sizeof(DRun)) != hipSuccess ||
        hipMemcpy(d->dev, d->host.data(), d->host.size() * sizeof(DRun), hipMemcpyHostToDevice) != hipSuccess) {
      if (d->dev) release_later(d->dev, REL_DEV);
      delete d;
      return MX_ERR_HIP;
    }
  }
  build_bmap(d);
  if (d->bmap_T) {
    std::vector<uint16_t> m16;
    std::vector<uint32_t> m32;
    for (int32_t u : d->bmap) {
      if (d->map16) m16.push_back((uint16_t)(u - d->umin));
      else m32.push_back((uint32_t)(u - d->umin));
    }
    const size_t nb = d->map16 ? m16.size() * 2 : m32.size() * 4;
    const void *src = d->map16 ? (const void *)m16.data() : (const void *)m32.data();
    if (hipMalloc(&d->map_dev, nb) != hipSuccess || hipMemcpy(d->map_dev, src, nb, hipMemcpyHostToDevice) != hipSuccess) {
      if (d->map_dev) release_later(d->map_dev, REL_DEV);
      if (d->dev) release_later(d->dev, REL_DEV);
      delete d;
      return MX_ERR_HIP;
    }
  }
  *out = d;
  return MX_SUCCESS;
}

extern "C" int mx_ddt_destroy(mx_ddt_t *d) {
  if (!d) return MX_SUCCESS;
  if (d->dev) release_later(d->dev, REL_DEV);
  if (d->map_dev) release_later(d->map_dev, REL_DEV);
  for (auto &P : d->ptab)
    if (P.dev) release_later(P.dev, REL_DEV);
  if (d->btab.dev) release_later(d->btab.dev, REL_DEV);
  if (d->btab.tfirst) release_later(d->btab.tfirst, REL_DEV);
  for (auto &e : d->up_ev)
    for (hipEvent_t ev : e)
      if (ev) (void)hipEventDestroy(ev);
  delete d;
  return MX_SUCCESS;
}

extern "C" size_t mx_ddt_size(const mx_ddt_t *d) { return d ? d->size : 0; }
extern "C" int64_t mx_ddt_extent(const mx_ddt_t *d) { return d ? d->ub - d->lb : 0; }
extern "C" size_t mx_ddt_runs(const mx_ddt_t *d) { return d ? d->host.size() : 0; }

// Byte range [*lo, *hi) relative to `user` that `count` instances touch
// (the true extent; instance i is displaced by i * extent).
extern "C" int mx_ddt_span(const mx_ddt_t *d, size_t count, int64_t *lo, int64_t *hi) {
  if (!d || !lo || !hi) return MX_ERR_ARG;
  *lo = *hi = 0;
  if (!count || d->host.empty()) return MX_SUCCESS;
  int64_t a = INT64_MAX, b = INT64_MIN;
  for (const DRun &r : d->host) {
    if (!r.bytes) continue;
    const int64_t s1 = (int64_t)(r.cnt1 - 1) * r.stride1, s2 = (int64_t)(r.cnt2 - 1) * r.stride2;
    const int64_t first = r.disp + std::min<int64_t>(0, s1) + std::min<int64_t>(0, s2);
    const int64_t last = r.disp + std::max<int64_t>(0, s1) + std::max<int64_t>(0, s2) + (int64_t)r.blen;
    a = std::min(a, first);
    b = std::max(b, last);
  }
  if (a > b) return MX_SUCCESS;
  const int64_t ext = d->ub - d->lb, tail = (int64_t)(count - 1) * ext;
  *lo = a + std::min<int64_t>(0, tail);
  *hi = b + std::max<int64_t>(0, tail);
  return MX_SUCCESS;
}

// MX_CONV_VEC=0 sends single-run layouts to the general kernels instead
// (A/B measurement switch; results are identical).
static bool conv_vec_enabled() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_VEC");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_PIPE=0 sends PACK to the one-tile-per-workgroup kernel instead
// of the pipelined one (A/B switch; results are identical).
static bool conv_pipe_enabled() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_PIPE");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_BMAP=0 keeps small irregular instances on the run-walking tile
// kernels (A/B switch; results are identical).
static bool conv_bmap_enabled() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_BMAP");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_BMAP_PACK=0 sends PACK of small dense instances to the piece
// kernel instead of the byte-map kernel (A/B switch).
static bool conv_bmap_pack_enabled() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_BMAP_PACK");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_PPACK=0 keeps PACK of layouts the byte map does not take on the
// run-walking kernels instead of the piece kernel (A/B switch).
static bool conv_ppack_enabled() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_PPACK");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_BMAP_DW=0 gives each lane of the byte-map PACK kernel 16 packed
// bytes (one 16-byte store) instead of one dword per step (A/B switch).
static bool conv_bmap_dw() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_BMAP_DW");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_BLK: 0 keeps every layout off the BLOCK kernels, 1 (default)
// sends instances without a byte map (> kBmapMaxS packed bytes) to them,
// 2 also small instances (A/B against the byte-map / piece kernels; results
// are identical).
static int conv_blk_mode() {
  static const int m = [] {
    const char *e = getenv("MX_CONV_BLK");
    const int v = e ? atoi(e) : 1;
    return (v >= 0 && v <= 2) ? v : 1;
  }();
  return m;
}

// MX_CONV_BMAP_PIPE=0 runs the byte-map PACK kernel without the span
// prefetch of the next tile (A/B switch; results are identical).
static bool conv_bmap_pipe() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_BMAP_PIPE");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_BMAP_ALIGN=16|128: the byte-map PACK stages a tile's user span
// from its first 16-byte granule or from the start of that granule's
// 128-byte line, so that a wave's 1 KiB loads cover whole lines
static uint64_t conv_bmap_align() {
  static const uint64_t v = [] {
    const char *e = getenv("MX_CONV_BMAP_ALIGN");
    return (uint64_t)((e && atoi(e) == 16) ? 16 : 128);
  }();
  return v;
}

// MX_CONV_BMAP_QUAD=0 stages the byte-map PACK's map as one row also where
// S % 4 != 0 (A/B switch; results identical)
static bool conv_bmap_quad() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_BMAP_QUAD");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_BMAP_CW=0: the byte-map PACK reads every packed byte on its own
// also where whole waves of packed dwords are user-contiguous (A/B switch)
static bool conv_bmap_cw() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_BMAP_CW");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_BMAP_NT=0: the byte-map PACK reads the user span and writes the
// packed stream with ordinary accesses instead of non-temporal ones (A/B
// switch).  The span is staged with one coalesced 16-byte load per lane, the
// pattern whose floor is 1.23x faster non-temporal at 256 MiB
// (tools/pack_floor_probe split-nt vs split-plain, profiles/r05/pack_floor_r5j.txt)
static bool conv_bmap_nt() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_BMAP_NT");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_VEC_NT=0: the VEC and VEC-span PACK kernels keep ordinary accesses
// at the streaming sizes too (A/B switch)
static bool conv_vec_nt() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_VEC_NT");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_UNPACK_NTLD=1: the UNPACK kernels read the packed stream with
// non-temporal loads at the streaming sizes (A/B switch, off: -5 % / +5 %
// on indexed at 256 MiB / 1 GiB, within 1 % elsewhere, profiles/r05/conv_ab_r5y.txt;
// the unpack is bound by its partial-line stores)
static bool conv_unpack_ntld() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_UNPACK_NTLD");
    return (e && *e == '1') ? 1 : 0;
  }();
  return on != 0;
}

// MX_CONV_UNPACK_U32=0: the piece UNPACK kernel's store loop in 64-bit
// stream coordinates (round 4's form; A/B switch)
static bool conv_unpack_u32() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_UNPACK_U32");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_BMAP_WORD=1: the byte-map PACK stages a word map for word-piece
// layouts (A/B switch, off: indexed 112 -> 137 us at 256 MiB with it, BLACS
// equal, profiles/r05/conv_r5r.txt -- the gather gets shorter and the tile's
// span prefetch, which it hid, is waited for instead)
static bool conv_bmap_word() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_BMAP_WORD");
    return (e && *e == '1') ? 1 : 0;
  }();
  return on != 0;
}

// MX_CONV_BMAP_UNROLL=0: one packed dword per lane per step in the byte-map
// PACK's gather instead of kBmapU (A/B switch)
static bool conv_bmap_unroll() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_BMAP_UNROLL");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_CONV_BMAP_SPAN=12288|24576|49152: user span the byte-map PACK stages
// per tile (A/B switch; the tile's stream bytes follow from it; unset: 24 KiB
// where five workgroups fit a CU, else 12 KiB)
static int conv_bmap_span_idx() {
  static const int v = [] {
    const char *e = getenv("MX_CONV_BMAP_SPAN");
    if (!e) return -1;                                   // by the map's size
    const long x = atol(e);
    return x == kBmapSpans[0] ? 0 : x == kBmapSpans[2] ? 2 : 1;
  }();
  return v;
}

// MX_CONV_UNPACK_PIPE=1 runs the piece UNPACK kernel with the register
// prefetch of the next tile's packed range (A/B switch, off: measured
// slower; results are identical).
static bool conv_unpack_pipe() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_UNPACK_PIPE");
    return (e && *e == '1') ? 1 : 0;
  }();
  return on != 0;
}

// The piece UNPACK form: MX_CONV_UNPACK_DIRECT=0 always the LDS-staged tile
// kernel, =1 always one piece per lane, unset: measured per datatype
// (mx_ddt::up_choice).  Results are identical.
static int conv_unpack_direct() {
  static const int v = [] {
    const char *e = getenv("MX_CONV_UNPACK_DIRECT");
    return (e && *e == '0') ? 1 : (e && *e == '1') ? 2 : 0;
  }();
  return v;
}

// The form of this piece unpack (1 staged, 2 one piece per lane) and, during
// the trials, the events to bracket it with (null otherwise).
static int unpack_piece_form(mx_ddt *dm, uint64_t len, hipEvent_t *ev0, hipEvent_t *ev1) {
  *ev0 = *ev1 = nullptr;
  if (const int f = conv_unpack_direct()) return f;
  std::lock_guard<std::mutex> lk(dm->up_mu);
  if (dm->up_choice) return dm->up_choice;
  if (len < ((uint64_t)4 << 20)) return 1;
  for (int v = 0; v < 2; v++) {
    if (dm->up_tried & (1 << v)) continue;
    for (int k = 0; k < 2; k++)
      if (!dm->up_ev[v][k] && hipEventCreate(&dm->up_ev[v][k]) != hipSuccess) {
        (void)hipGetLastError();
        dm->up_choice = 1;   // no events: keep the staged form
        return 1;
      }
    dm->up_tried |= 1 << v;
    dm->up_bytes[v] = (double)len;
    *ev0 = dm->up_ev[v][0];
    *ev1 = dm->up_ev[v][1];
    return v + 1;
  }
  // both tried: decide once both have completed (never waits)
  float ms[2];
  for (int v = 0; v < 2; v++) {
    const hipError_t e = hipEventQuery(dm->up_ev[v][1]);
    if (e == hipErrorNotReady) {
      (void)hipGetLastError();
      return 1;
    }
    if (e != hipSuccess || hipEventElapsedTime(&ms[v], dm->up_ev[v][0], dm->up_ev[v][1]) != hipSuccess) {
      (void)hipGetLastError();
      dm->up_choice = 1;
      return 1;
    }
  }
  dm->up_choice = ms[1] / dm->up_bytes[1] < ms[0] / dm->up_bytes[0] ? 2 : 1;
  return dm->up_choice;
}

// MX_CONV_VEC_SPAN=0 packs periodic small-block vectors through the VEC
// kernel instead of k_pack_vec_span (A/B switch; results are identical).
static bool conv_vec_span() {
  static const int on = [] {
    const char *e = getenv("MX_CONV_VEC_SPAN");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

static int conv_pipe_geom() {
  static const int g = [] {
    const char *e = getenv("MX_CONV_PIPE_GEOM");
    const int v = e ? atoi(e) : 0;
    return (v >= 0 && v <= 3) ? v : 0;
  }();
  return g;
}

// Tile size of the TILE kernels (MX_CONV_TP = 2048 / 4096 / 8192 for
// measurement; results are identical).
static int conv_tile_bytes() {
  static const int tp = [] {
    const char *e = getenv("MX_CONV_TP");
    const int v = e ? atoi(e) : 0;
    return (v == 2048 || v == 4096 || v == 8192) ? v : 8192;
  }();
  return tp;
}

template <bool PACK>
static int convert(const mx_ddt_t *d, size_t count, char *user, char *packed, size_t offset, size_t len,
                   void *stream) {
  if (!d || !user || !packed) return MX_ERR_ARG;
  if (len == 0) return MX_SUCCESS;
  if (d->size == 0 || offset + len > d->size * count) return MX_ERR_ARG;
  if ((offset + len) >> kMagicBits) return MX_ERR_UNSUPPORTED;   // > 256 TiB streams
  int rc = mx_ensure_init();
  if (rc) return rc;
  ConvArgs a;
  a.runs = d->dev;
  a.nruns = (int)d->host.size();
  a.S = d->size;
  a.mS = d->mS;
  a.ext = d->ub - d->lb;
  a.user = user;
  a.packed = packed;
  a.offset = offset;
  a.len = len;
  a.pk_vec = ((uintptr_t)packed & 15) == 0;
  a.ntld = !PACK && conv_unpack_ntld() && mx_nt_for((size_t)(2 * len));
  hipStream_t s = (hipStream_t)stream;
  mx_ddt *dm = const_cast<mx_ddt *>(d);
  // a contiguous type (one block, extent = size): the stream is the user
  // bytes themselves -- one copy (ref_contiguous_int2_77 unpack 2.27 TB/s
  // through the piece kernel)
  if (a.nruns == 1 && d->host[0].cnt1 == 1 && d->host[0].cnt2 == 1 && d->host[0].blen == d->size &&
      a.ext == (int64_t)d->size) {
    char *u = user + d->host[0].disp + offset;
    dm->last_path.store(1, std::memory_order_relaxed);
    return PACK ? copy_async(packed, u, len, s) : copy_async(u, packed, len, s);
  }
  // widest unit that every piece of every granule respects: layout gcd,
  // alignment of the user origin, and the stream offset of granule 0
  uint64_t u = gcd64(d->gcd_all, ((uintptr_t)user) & 15 ? ((uintptr_t)user & 15) : 16);
  u = gcd64(u, offset & 15 ? (offset & 15) : 16);
  u = gcd64(u, len & 15 ? (len & 15) : 16);
  if (!a.pk_vec) u = gcd64(u, (uintptr_t)packed & 15);
  const size_t run_lds = a.nruns <= kLdsRuns ? (size_t)a.nruns * sizeof(DRun) : 0;
  // periodic small blocks, PACK: whole 16-byte chunks of the span (k_pack_vec_span)
  if (PACK && a.nruns == 1 && d->host[0].cnt2 == 1 && !d->force_blk && conv_vec_span()) {
    const DRun &R = d->host[0];
    // the period: the block stride, or the extent for one block per instance;
    // instances continue it when extent == cnt1 * period, or the window stays
    // inside instance 0 (one plain MPI vector)
    const int64_t st = R.cnt1 > 1 ? R.stride1 : a.ext;
    const char *ub = user + R.disp;
    const bool periodic = (st == 8 || st == 16) && (int64_t)R.blen < st &&
                          (a.ext == (int64_t)R.cnt1 * st || offset + len <= a.S) &&
                          ((uintptr_t)ub & 15) == 0 && (R.blen == 4 || R.blen == 8) &&
                          (((uintptr_t)packed - offset) & (16 / st * R.blen - 1)) == 0;
    if (periodic) {
      const uint64_t outb = (uint64_t)(16 / st) * R.blen;   // packed bytes per chunk
      const uint64_t q0 = offset / outb, q1 = (offset + len + outb - 1) / outb;
      const uint64_t nq = q1 - q0;
      const dim3 grid((unsigned)((nq + kCB - 1) / kCB)), block(kCB);
      dm->last_path.store(2, std::memory_order_relaxed);
      // non-temporal at the streaming sizes (span + stream >= MX_NT_MIN_BYTES)
      const bool nt = conv_vec_nt() && mx_nt_for((size_t)(len + len * (uint64_t)st / R.blen));
#define MX_VSPAN(S_, B_)                                                                                      \
  do {                                                                                                        \
    if (nt) hipLaunchKernelGGL((k_pack_vec_span<S_, B_, true>), grid, block, 0, s, ub, packed, offset, len, q0, q1); \
    else hipLaunchKernelGGL((k_pack_vec_span<S_, B_, false>), grid, block, 0, s, ub, packed, offset, len, q0, q1);   \
  } while (0)
      if (st == 8) MX_VSPAN(8, 4);
      else if (R.blen == 8) MX_VSPAN(16, 8);
      else MX_VSPAN(16, 4);
#undef MX_VSPAN
      return mx_check_launch();
    }
  }
  // one strided 1-level run of whole aligned 4/8-byte words: the VEC kernel
  // (16-byte-granular layouts stay on k_convert<16>: measured 3.9 vs 2.8 TB/s
  // for 16-byte blocks at 1 GiB, while 4-byte blocks go 2.1 -> 3.5 TB/s here;
  // profiles/r01/convertor_vec_ab.txt)
  if (a.nruns == 1 && d->host[0].cnt2 == 1 && u % 4 == 0 && u != 16 && d->host[0].blen <= kVecMaxBlen &&
      conv_vec_enabled() && !d->force_blk) {
    dm->last_path.store(2, std::memory_order_relaxed);
    const DRun &R = d->host[0];
    const uint64_t W = (u % 8 == 0) ? 8 : 4;
    const uint64_t nw = len / W;
    const dim3 grid((unsigned)((nw + kCB * kVIt - 1) / (kCB * kVIt))), block(kCB);
    const float rblen = 1.0f / (float)R.blen;
    // PACK: non-temporal at the streaming sizes (the user lines read + the
    // stream written >= MX_NT_MIN_BYTES); UNPACK keeps cached stores (its
    // partial-line writes)
    const bool nt = PACK && conv_vec_nt() && mx_nt_for((size_t)(len + len * (uint64_t)R.stride1 / R.blen));
    if (nt && W == 8) hipLaunchKernelGGL((k_convert_vec<8, PACK, true>), grid, block, 0, s, a, R, rblen);
    else if (nt) hipLaunchKernelGGL((k_convert_vec<4, PACK, true>), grid, block, 0, s, a, R, rblen);
    else if (W == 8) hipLaunchKernelGGL((k_convert_vec<8, PACK>), grid, block, 0, s, a, R, rblen);
    else hipLaunchKernelGGL((k_convert_vec<4, PACK>), grid, block, 0, s, a, R, rblen);
    return mx_check_launch();
  }
  const int blk = d->force_blk ? 2 : conv_blk_mode();
  if (blk && (blk == 2 || d->bmap.empty())) {
    mx_ddt::BlkTab *bt;
    {
      std::lock_guard<std::mutex> g(dm->mu);
      bt = blk_tab(dm);
    }
    if (bt) {
      BlkArgs b;
      b.blk = bt->dev;
      b.nblk = (uint32_t)bt->host.size();
      b.mnblk = make_magic(b.nblk);
      b.tfirst = bt->tfirst;
      b.S = d->size;
      b.mS = d->mS;
      b.ext = d->ub - d->lb;
      b.user = user;
      b.packed = packed;
      b.offset = offset;
      b.len = len;
      b.T = bt->T;
      const uintptr_t MA = (uintptr_t)packed & ~(uintptr_t)15;
      b.ntiles = ((uintptr_t)packed + len - MA + b.T - 1) / b.T;
      const uint64_t grid = std::min<uint64_t>(b.ntiles, (uint64_t)g_num_cus * 8);
      dm->last_path.store(6, std::memory_order_relaxed);
      b.w4 = conv_blk_w4();
      if (PACK && bt->Tspan) {
        b.T = bt->Tspan;
        b.ntiles = ((uintptr_t)packed + len - MA + b.T - 1) / b.T;
        const size_t lds = kBlkSpan + 32 + (size_t)bt->capspan * sizeof(SBlk) + (b.T / 64) * 2;
        const uint64_t per_cu = std::max<uint64_t>(1, std::min<uint64_t>(8, (160 * 1024) / (lds + 128)));
        const uint64_t gs = std::min<uint64_t>(b.ntiles, (uint64_t)g_num_cus * per_cu);
        hipLaunchKernelGGL(k_pack_blk_span, dim3((unsigned)gs), dim3(kCB), lds, s, b, bt->capspan);
        return mx_check_launch();
      }
      const int ng = conv_blk_ng(PACK);
      if (ng == 1) hipLaunchKernelGGL((k_convert_blk<PACK, 1>), dim3((unsigned)grid), dim3(kCB), 0, s, b);
      else if (ng == 2) hipLaunchKernelGGL((k_convert_blk<PACK, 2>), dim3((unsigned)grid), dim3(kCB), 0, s, b);
      else hipLaunchKernelGGL((k_convert_blk<PACK, 4>), dim3((unsigned)grid), dim3(kCB), 0, s, b);
      return mx_check_launch();
    }
  }
  if (u == 16) {
    dm->last_path.store(3, std::memory_order_relaxed);
    const uint64_t g = (len + 15) / 16;
    if (run_lds) hipLaunchKernelGGL((k_convert<16, PACK, true>), dim3((unsigned)((g + kCB - 1) / kCB)), dim3(kCB), run_lds, s, a);
    else hipLaunchKernelGGL((k_convert<16, PACK, false>), dim3((unsigned)((g + kCB - 1) / kCB)), dim3(kCB), 0, s, a);
    return mx_check_launch();
  }
  // small irregular instances: byte-map PACK / piece UNPACK (see the kernels)
  if (!d->bmap.empty() && conv_bmap_enabled()) {
    if (PACK && d->bmap_T && !d->piece_pack && (((uintptr_t)packed - offset) & 15) == 0 &&
        conv_bmap_pack_enabled()) {
      BmapArgs b;
      b.map = d->map_dev;
      b.mono = d->monotonic;
      b.S = (uint32_t)d->size;
      b.mS = d->mS;
      b.ext = d->ub - d->lb;
      b.umin = d->umin;
      b.uspan = d->uspan;
      b.user = user;
      b.packed = packed;
      b.offset = offset;
      b.len = len;
      b.g0 = offset / 16;
      const bool dw = conv_bmap_dw(), nt = conv_bmap_nt(), pipe = conv_bmap_pipe();
      int si = conv_bmap_span_idx();
      const bool word = d->bmap_word && conv_bmap_word() && dw;
      const size_t map_lds = (word ? d->size / 4 : d->bmap_quad && conv_bmap_quad() ? 4 * d->size : d->size + 3) *
                             (d->map16 ? 2 : 4);
      // default: the 24 KiB span where five or more workgroups fit a CU (a
      // small map), else 12 KiB, which keeps seven (indexed's 10 KiB map: four
      // at 24 KiB).  On one box against the floors (profiles/r05/conv_ab_r5q.txt,
      // pack_floor_r5q.txt), 256 MiB: struct 24 KiB 123 us / 12 KiB 159 /
      // 48 KiB 157 (floor 125); indexed 123 / 116 / 180 (floor 109)
      if (si < 0) si = (160 * 1024) / (kBmapSpans[1] + 32 + map_lds + 128) >= 5 ? 1 : 0;
      if (!d->bmap_Ts[si] || !(dw && nt && pipe) || kBmapSpans[si] + 32 + map_lds > 65536)
        si = 1;                                       // other spans: the default kernel shape only
      b.T = d->bmap_Ts[si];
      b.ntiles = ((offset + len + 15) / 16 * 16 - b.g0 * 16 + b.T - 1) / b.T;
      b.word = word;
      b.qsh = !word && d->bmap_quad && conv_bmap_quad() ? 2 : 0;
      b.cw = d->bmap_cw && conv_bmap_cw();
      b.unroll = conv_bmap_unroll();
      const size_t lds = kBmapSpans[si] + 32 + map_lds;
      const uint64_t per_cu = std::max<uint64_t>(1, std::min<uint64_t>(8, (160 * 1024) / lds));
      const uint64_t grid = std::min<uint64_t>(b.ntiles, (uint64_t)g_num_cus * per_cu);
      b.adv_b = (uint32_t)((kCB * 4) % d->size);
      b.adv_io = (int64_t)((kCB * 4) / d->size) * b.ext;
      b.lo_mask = conv_bmap_align() - 1;
      dm->last_path.store(4, std::memory_order_relaxed);
      if (si != 1) {
        if (d->map16) {
          if (si == 0) hipLaunchKernelGGL((k_pack_bmap<kBmapSpans[0], uint16_t, true, true, true>), dim3((unsigned)grid), dim3(kCB), lds, s, b);
          else hipLaunchKernelGGL((k_pack_bmap<kBmapSpans[2], uint16_t, true, true, true>), dim3((unsigned)grid), dim3(kCB), lds, s, b);
        } else {
          if (si == 0) hipLaunchKernelGGL((k_pack_bmap<kBmapSpans[0], uint32_t, true, true, true>), dim3((unsigned)grid), dim3(kCB), lds, s, b);
          else hipLaunchKernelGGL((k_pack_bmap<kBmapSpans[2], uint32_t, true, true, true>), dim3((unsigned)grid), dim3(kCB), lds, s, b);
        }
        return mx_check_launch();
      }
#define MX_BMAP_LAUNCH2(M, DW, NT)                                                                               \
  do {                                                                                                           \
    if (pipe)                                                                                                    \
      hipLaunchKernelGGL((k_pack_bmap<kBmapSpan, M, DW, true, NT>), dim3((unsigned)grid), dim3(kCB), lds, s, b); \
    else                                                                                                         \
      hipLaunchKernelGGL((k_pack_bmap<kBmapSpan, M, DW, false, NT>), dim3((unsigned)grid), dim3(kCB), lds, s, b);\
  } while (0)
#define MX_BMAP_LAUNCH(M, DW)                                                                                   \
  do {                                                                                                           \
    if (nt) MX_BMAP_LAUNCH2(M, DW, true);                                                                        \
    else MX_BMAP_LAUNCH2(M, DW, false);                                                                          \
  } while (0)
      if (d->map16) { if (dw) MX_BMAP_LAUNCH(uint16_t, true); else MX_BMAP_LAUNCH(uint16_t, false); }
      else { if (dw) MX_BMAP_LAUNCH(uint32_t, true); else MX_BMAP_LAUNCH(uint32_t, false); }
#undef MX_BMAP_LAUNCH
#undef MX_BMAP_LAUNCH2
      return mx_check_launch();
    }
    if (!PACK || conv_ppack_enabled()) {
      mx_ddt::PieceTab *pt;
      {
        std::lock_guard<std::mutex> g(dm->mu);
        pt = piece_tab(dm, (int)((uintptr_t)user & 15));
      }
      if (pt) {
        PieceArgs p;
        const uint32_t npi = (uint32_t)pt->host.size();
        p.pieces = pt->dev;
        p.npi = npi;
        p.mnpi = make_magic(npi);
        p.S = d->size;
        p.ext = d->ub - d->lb;
        p.user = user;
        p.packed = packed;
        p.offset = offset;
        p.len = len;
        const uint64_t i0 = offset / d->size, i1 = (offset + len - 1) / d->size;
        p.P0 = i0 * npi + piece_of(pt->host, offset - i0 * d->size);
        p.P1 = i1 * npi + piece_of(pt->host, offset + len - 1 - i1 * d->size) + 1;
        p.K = pt->K;
        p.dinst = (uint32_t)(kCB / npi);
        p.dj = (uint32_t)(kCB % npi);
        p.ntiles = (p.P1 - p.P0 + p.K - 1) / p.K;
        p.tbl_lds = npi * sizeof(DPiece) <= 16384;
        p.u32 = conv_unpack_u32();
        p.ntld = !PACK && conv_unpack_ntld() && mx_nt_for((size_t)(2 * len));
        const size_t lds = kPieceStage + 48 + (p.tbl_lds ? npi * sizeof(DPiece) : 0);
        const uint64_t per_cu = std::max<uint64_t>(1, std::min<uint64_t>(8, (160 * 1024) / lds));
        const uint64_t grid = std::min<uint64_t>(p.ntiles, (uint64_t)g_num_cus * per_cu);
        dm->last_path.store(5, std::memory_order_relaxed);
        const uint64_t npieces = p.P1 - p.P0;
        hipEvent_t ev0 = nullptr, ev1 = nullptr;
        const int form = PACK ? 1 : unpack_piece_form(dm, len, &ev0, &ev1);
        if (ev0 && hipEventRecord(ev0, s) != hipSuccess) (void)hipGetLastError();
        if (PACK) hipLaunchKernelGGL(k_pack_piece, dim3((unsigned)grid), dim3(kCB), lds, s, p);
        else if (form == 2 && npieces <= (uint64_t)UINT32_MAX * kCB) {
          const unsigned g2 = (unsigned)((npieces + kCB - 1) / kCB);
          if (p.ntld) hipLaunchKernelGGL(k_unpack_piece_direct<true>, dim3(g2), dim3(kCB), 0, s, p);
          else hipLaunchKernelGGL(k_unpack_piece_direct<false>, dim3(g2), dim3(kCB), 0, s, p);
        } else if (conv_unpack_pipe()) {
          if (p.tbl_lds) hipLaunchKernelGGL((k_unpack_piece<true, true>), dim3((unsigned)grid), dim3(kCB), lds, s, p);
          else hipLaunchKernelGGL((k_unpack_piece<true, false>), dim3((unsigned)grid), dim3(kCB), lds, s, p);
        } else if (p.tbl_lds) {
          hipLaunchKernelGGL((k_unpack_piece<false, true>), dim3((unsigned)grid), dim3(kCB), lds, s, p);
        } else {
          hipLaunchKernelGGL((k_unpack_piece<false, false>), dim3((unsigned)grid), dim3(kCB), lds, s, p);
        }
        const int lrc = mx_check_launch();
        if (ev1 && hipEventRecord(ev1, s) != hipSuccess) (void)hipGetLastError();
        return lrc;
      }
    }
  }
  // narrow pieces: tile kernels (PACK needs a monotonic layout so that a
  // tile's user bytes form one span)
  if (!PACK || d->monotonic) {
    dm->last_path.store(7, std::memory_order_relaxed);
    const int nlds = a.nruns <= 64 ? 1 : 0;
    const size_t rb = nlds ? (size_t)a.nruns * sizeof(DRun) : 0;
    if (PACK && conv_pipe_enabled()) {
      // MX_CONV_PIPE_GEOM selects the tile geometry (A/B measurement; results
      // are identical): 0 = 8192 x 24 KiB span, 1 = 9216 x 16 KiB,
      // 2 = 9216 x 28 KiB, 3 = 8192 x 16 KiB.  0 is fastest on every type
      // measured (profiles/r02/convertor_r2.txt): the bank-conflict-free
      // 36-byte stretches of 1 / 2 lose more to the tile / occupancy change
      // than the conflicts cost (20k of ~4M cycles per wave).
      const int geom = conv_pipe_geom();
#define MX_PIPE_LAUNCH(TPV, SPV, WGS)                                                                        \
  do {                                                                                                        \
    const uint64_t tiles = (len + TPV - 1) / TPV;                                                             \
    const uint64_t grid = std::min<uint64_t>(tiles, (uint64_t)g_num_cus * (WGS));                             \
    hipLaunchKernelGGL((k_pack_tile_pipe<TPV, SPV>), dim3((unsigned)grid), dim3(kCB),                          \
                       (PipeGeom<TPV, SPV>::lds(rb)), s, a, nlds, tiles);                                        \
  } while (0)
      if (geom == 2) MX_PIPE_LAUNCH(9216, 28672, 3);
      else if (geom == 3) MX_PIPE_LAUNCH(8192, 16384, 6);
      else if (geom == 1) MX_PIPE_LAUNCH(9216, 16384, 6);
      else MX_PIPE_LAUNCH(8192, 24576, 4);
#undef MX_PIPE_LAUNCH
      return mx_check_launch();
    }
    const int tp = conv_tile_bytes();
    // narrow 4-byte-aligned blocks: word-parallel stores (see the kernel)
    uint64_t maxblen = 0;
    for (const DRun &r : d->host) maxblen = std::max<uint64_t>(maxblen, r.blen);
    const int wordpar = !PACK && (u % 4) == 0 && maxblen <= 32;
#define MX_TILE_LAUNCH(TPV)                                                                          \
  hipLaunchKernelGGL((k_convert_tile<PACK, TPV>), dim3((unsigned)((len + TPV - 1) / TPV)), dim3(kCB),     \
                     TileGeom<TPV>::lds(PACK, rb), s, a, nlds, wordpar)
    if (tp == 2048) MX_TILE_LAUNCH(2048);
    else if (tp == 4096) MX_TILE_LAUNCH(4096);
    else MX_TILE_LAUNCH(8192);
#undef MX_TILE_LAUNCH
    return mx_check_launch();
  }
  const dim3 grid((unsigned)(((len + 15) / 16 + kCB - 1) / kCB)), block(kCB);
  dm->last_path.store(3, std::memory_order_relaxed);
#define MX_CONV_LAUNCH(U)                                                                   \
  do {                                                                                      \
    if (run_lds) hipLaunchKernelGGL((k_convert<U, PACK, true>), grid, block, run_lds, s, a); \
    else hipLaunchKernelGGL((k_convert<U, PACK, false>), grid, block, 0, s, a);              \
  } while (0)
  switch (u) {
    case 8: MX_CONV_LAUNCH(8); break;
    case 4: MX_CONV_LAUNCH(4); break;
    case 2: MX_CONV_LAUNCH(2); break;
    default: MX_CONV_LAUNCH(1); break;
  }
#undef MX_CONV_LAUNCH
  return mx_check_launch();
}

extern "C" int mx_ddt_set_path(mx_ddt_t *d, int path) {
  if (!d || (path != MX_DDT_PATH_AUTO && path != MX_DDT_PATH_BLOCK)) return MX_ERR_ARG;
  if (path == MX_DDT_PATH_BLOCK) {
    int rc = mx_ensure_init();
    if (rc) return rc;
    std::lock_guard<std::mutex> g(d->mu);
    if (!blk_tab(d)) return MX_ERR_UNSUPPORTED;
  }
  d->force_blk = path == MX_DDT_PATH_BLOCK;
  return MX_SUCCESS;
}

extern "C" int mx_ddt_last_path(const mx_ddt_t *d) { return d ? d->last_path.load(std::memory_order_relaxed) : 0; }

extern "C" int mx_pack(const mx_ddt_t *d, size_t count, const void *user, void *packed, size_t offset, size_t len,
                       void *stream) {
  return convert<true>(d, count, (char *)user, (char *)packed, offset, len, stream);
}

extern "C" int mx_unpack(const mx_ddt_t *d, size_t count, void *user, const void *packed, size_t offset,
                         size_t len, void *stream) {
  return convert<false>(d, count, (char *)user, (char *)packed, offset, len, stream);
}
