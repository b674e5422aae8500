// mx_reduce.hip -- K1..K4: the predefined MPI_Op element kernels on gfx950.
//
// Replaces the host loops of ompi/mca/op/base/op_base_functions.c
// (OP_FUNC :40-51, FUNC_FUNC :60-73, LOC_FUNC :88-104, 3-buffer :654-775)
// with HBM-streaming kernels:
//  * one 16-byte vector per lane (global_load/store_dwordx4) and a grid
//    that covers the buffer densely (no reuse => no LDS, no MFMA: the op
//    is <= 1 flop per element, ~0.08 flop/B -> HBM bound);
//  * head/tail elements that do not fill a 16-byte vector are handled by
//    the first lanes of the grid (ragged counts, unaligned sub-blocks of a
//    ring step);
//  * buffers whose misalignment differs mod 16 fall back to an
//    element-per-lane kernel (still coalesced);
//  * large launches (>= 384 MiB footprint) use non-temporal loads AND
//    stores in one-wave workgroups (mx_mem.hpp): 1 GiB fp32 SUM 0.475-0.483
//    ms per launch, 6.67-6.78 TB/s = 0.83-0.85 of 8 TB/s, PMC traffic =
//    the algorithmic bytes (profiles/r04/,
//    profiles/r05/reduce_local_kernel_stats_r5.csv).
// Algorithmic bytes per launch: 2-buffer 3*n*size (read in, read inout,
// write inout), 3-buffer 3*n*size.
#include <hip/hip_runtime.h>
#include <chrono>
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>

#include "mx_dispatch.hpp"
#include "mx_internal.h"
#include "mx_mem.hpp"

namespace mx {

constexpr int kBlock = 256;
// The non-temporal (>= 384 MiB) vector instances run one-wave (64-lane)
// workgroups: tools/bw_probe5.hip, 3 interleaved rounds per box (fp32 SUM,
// nt loads + store), 256 / 128 / 64 lanes in TB/s -- box A: 1 GiB 6.49 /
// 6.73 / 6.70, 2 GiB 6.45 / 6.64 / 6.71; box B: 1 GiB 6.17 / 6.44 / 6.75,
// 4 GiB 6.19 / 6.03 / 6.25 (profiles/r03/bw_probe5*.txt).  The cached
// instance keeps 256 lanes (64 lanes lose up to 25 % below 64 MiB,
// bw_probe5_cached.txt).
constexpr int kBlockNT = 64;

template <class T>
struct alignas(16) vec16 {
  static constexpr int N = 16 / sizeof(T);
  T e[N];
};

// Completion mark (mx_reduce2_sync): every workgroup, after its stores,
// releases them at system scope (its XCD's L2 written back, as a kernel's
// end would) and writes its own flag in mapped host memory -- no atomics,
// no counter (a counter's system-scope atomics serialise: 32 workgroups
// cost ~2.7 us, profiles/r04/op_call_cost_r4_flags.txt).  The host sees the
// flags instead of waiting for a second, marker kernel -- one dispatch less
// per blocking call (op/mi355x's handler, ompi_op_reduce op.h:547-610).
// mk.flags is a kernel argument, so the branch is uniform; without a mark it
// costs nothing.
__device__ __forceinline__ void mark_done(const Mark &mk) {
  if (mk.flags == nullptr) return;
  // every wave's stores have reached its L2 before thread 0's write-back:
  // the barrier alone orders issue, not completion, and the system fence
  // below waits only for thread 0's own wave
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x < kMarkFlags) {
    __threadfence_system();
    __hip_atomic_store(mk.flags + blockIdx.x, (mk.v << 12) | (uint64_t)(gridDim.x - 1), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Scalar per-element application, inout-form (x = b, y = a) or 3-buffer.
// Results are stored field by field (store_fields): bytes of the target
// outside the value fields (pair-type padding, x87 pad) keep their content,
// as the reference's member assignments leave them (LOC_FUNC :88-104).
template <class T, class OP>
__device__ __forceinline__ void red2_elem(const T *__restrict__ a, T *__restrict__ b, size_t i) {
  store_fields(&b[i], OP()(b[i], a[i]));
}

// 2-buffer, vector body: elements [head, head + nvec*N) as 16-B vectors,
// ONE vector per lane and a grid covering all of them (no grid-stride
// loop): measured on MI355X at 1 GiB this dense block->address mapping
// streams at ~5.9 TB/s vs 4.3-5.6 TB/s for grid-stride variants
// (tools/bw_probe*.hip).
template <class T, class OP, bool NT, int BS = NT ? kBlockNT : kBlock>
__global__ void __launch_bounds__(BS)
k_reduce2(const T *__restrict__ a, T *__restrict__ b, size_t n, size_t head, size_t nvec, Mark mk) {
  using V = vec16<T>;
  constexpr int N = V::N;
  const size_t tid = (size_t)blockIdx.x * BS + threadIdx.x;
  OP op;
  if (tid < nvec) {
    const V *__restrict__ av = reinterpret_cast<const V *>(a + head);
    V *__restrict__ bv = reinterpret_cast<V *>(b + head);
    V x, y;
    ld16<NT>(x, bv + tid);
    ld16<NT>(y, av + tid);
#pragma unroll
    for (int j = 0; j < N; j++) store_fields(&x.e[j], op(x.e[j], y.e[j]));
    st16<NT>(bv + tid, x);
  }
  // ragged head and tail
  const size_t tail0 = head + nvec * N;
  if (tid < head) red2_elem<T, OP>(a, b, tid);
  if (tid < n - tail0) red2_elem<T, OP>(a, b, tail0 + tid);
  mark_done(mk);
}

// 2-buffer, 32-byte elements (complex long double, long double + int):
// one element per lane moved as two raw 16-byte vectors, the result's value
// fields merged into the destination's own bytes (store_fields on the
// loaded copy), so its padding travels back unchanged and every 128-byte
// line is written whole -- field-by-field stores leave 12 of every 32
// bytes unwritten, which costs a partial-line write-back per line
// (tools/sector_probe.hip).  Both buffers 16-byte aligned.
template <class T, class OP, bool NT>
__device__ __forceinline__ void red2_w32(const T *__restrict__ a, T *__restrict__ b, size_t i) {
  const u32x4 *pa = reinterpret_cast<const u32x4 *>(a + i);
  u32x4 *pb = reinterpret_cast<u32x4 *>(b + i);
  u32x4 ra[2], rb[2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if constexpr (NT) { ra[k] = __builtin_nontemporal_load(pa + k); rb[k] = __builtin_nontemporal_load(pb + k); }
    else { ra[k] = pa[k]; rb[k] = pb[k]; }
  }
  T x, y;
  __builtin_memcpy(&x, rb, 32);
  __builtin_memcpy(&y, ra, 32);
  store_fields(&x, OP()(x, y));
  __builtin_memcpy(rb, &x, 32);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if constexpr (NT) __builtin_nontemporal_store(rb[k], pb + k);
    else pb[k] = rb[k];
  }
}

template <class T, class OP, bool NT, int BS>
__global__ void __launch_bounds__(BS) k_reduce2_w32(const T *__restrict__ a, T *__restrict__ b, size_t n, Mark mk) {
  static_assert(sizeof(T) == 32, "32-byte elements");
  const size_t i = (size_t)blockIdx.x * BS + threadIdx.x;
  if (i < n) red2_w32<T, OP, NT>(a, b, i);
  mark_done(mk);
}

// The same through LDS: the workgroup's BS elements (2*BS 16-byte vectors
// per operand) are loaded with consecutive lanes on consecutive vectors --
// every wave instruction reads / writes whole lines, where the per-element
// form's two accesses 32 bytes apart each touch half of every line -- then
// lane t takes element t from LDS.
template <class T, class OP, bool NT, int BS>
__global__ void __launch_bounds__(BS) k_reduce2_w32t(const T *__restrict__ a, T *__restrict__ b, size_t n, Mark mk) {
  static_assert(sizeof(T) == 32, "32-byte elements");
  __shared__ u32x4 sa[2 * BS], sb[2 * BS];
  const size_t e0 = (size_t)blockIdx.x * BS;
  const unsigned nel = (unsigned)(n - e0 < (size_t)BS ? n - e0 : (size_t)BS);
  const unsigned nv = 2 * nel;
  const u32x4 *pa = reinterpret_cast<const u32x4 *>(a + e0);
  u32x4 *pb = reinterpret_cast<u32x4 *>(b + e0);
  const unsigned t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const unsigned v = t + k * BS;
    if (v < nv) {
      if constexpr (NT) { sa[v] = __builtin_nontemporal_load(pa + v); sb[v] = __builtin_nontemporal_load(pb + v); }
      else { sa[v] = pa[v]; sb[v] = pb[v]; }
    }
  }
  __syncthreads();
  if (t < nel) {
    T x, y;
    __builtin_memcpy(&x, &sb[2 * t], 32);
    __builtin_memcpy(&y, &sa[2 * t], 32);
    store_fields(&x, OP()(x, y));
    __builtin_memcpy(&sb[2 * t], &x, 32);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const unsigned v = t + k * BS;
    if (v < nv) {
      if constexpr (NT) __builtin_nontemporal_store(sb[v], pb + v);
      else pb[v] = sb[v];
    }
  }
  mark_done(mk);
}

// 2-buffer, one element per lane (mismatched alignment, or element > 16 B).
template <class T, class OP>
__global__ void __launch_bounds__(kBlock)
k_reduce2_elem(const T *__restrict__ a, T *__restrict__ b, size_t n, Mark mk) {
  const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) red2_elem<T, OP>(a, b, i);
  mark_done(mk);
}

// PAD (element types with padding: pairs, x87): the results' value fields
// are merged into the destination's own loaded bytes, so its padding keeps
// its content (LOC_FUNC_3BUF's member stores) and every line is written
// whole -- a field-by-field store leaves holes in every line, a partial-line
// write-back each (tools/sector_probe.hip).
template <class T, class OP, bool NT, int BS = NT ? kBlockNT : kBlock, bool PAD = false>
__global__ void __launch_bounds__(BS)
k_reduce3(const T *__restrict__ a1, const T *__restrict__ a2, T *__restrict__ o, size_t n,
          size_t head, size_t nvec) {
  using V = vec16<T>;
  constexpr int N = V::N;
  const size_t tid = (size_t)blockIdx.x * BS + threadIdx.x;
  OP op;
  if (tid < nvec) {
    const V *__restrict__ p = reinterpret_cast<const V *>(a1 + head);
    const V *__restrict__ q = reinterpret_cast<const V *>(a2 + head);
    V *__restrict__ ov = reinterpret_cast<V *>(o + head);
    V x, y;
    ld16<NT>(x, p + tid);
    ld16<NT>(y, q + tid);
    if constexpr (PAD) {
      V z;
      ld16<NT>(z, ov + tid);
#pragma unroll
      for (int j = 0; j < N; j++) store_fields(&z.e[j], op(x.e[j], y.e[j]));
      st16<NT>(ov + tid, z);
    } else {
#pragma unroll
      for (int j = 0; j < N; j++) x.e[j] = op(x.e[j], y.e[j]);
      st16<NT>(ov + tid, x);
    }
  }
  const size_t tail0 = head + nvec * N;
  if constexpr (PAD) {
    if (tid < head) store_fields(&o[tid], op(a1[tid], a2[tid]));
    if (tid < n - tail0) store_fields(&o[tail0 + tid], op(a1[tail0 + tid], a2[tail0 + tid]));
  } else {
    if (tid < head) o[tid] = op(a1[tid], a2[tid]);
    if (tid < n - tail0) o[tail0 + tid] = op(a1[tail0 + tid], a2[tail0 + tid]);
  }
}

// 3-buffer, 32-byte elements (complex long double, long double + int): as
// k_reduce2_w32t, with the destination's own bytes loaded too so its
// padding travels back unchanged and every line is written whole.
template <class T, class OP, bool NT, int BS>
__global__ void __launch_bounds__(BS) k_reduce3_w32t(const T *__restrict__ a1, const T *__restrict__ a2,
                                                     T *__restrict__ o, size_t n) {
  static_assert(sizeof(T) == 32, "32-byte elements");
  __shared__ u32x4 s1[2 * BS], s2[2 * BS], so[2 * BS];
  const size_t e0 = (size_t)blockIdx.x * BS;
  const unsigned nel = (unsigned)(n - e0 < (size_t)BS ? n - e0 : (size_t)BS);
  const unsigned nv = 2 * nel;
  const u32x4 *p1 = reinterpret_cast<const u32x4 *>(a1 + e0);
  const u32x4 *p2 = reinterpret_cast<const u32x4 *>(a2 + e0);
  u32x4 *po = reinterpret_cast<u32x4 *>(o + e0);
  const unsigned t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const unsigned v = t + k * BS;
    if (v < nv) {
      if constexpr (NT) {
        s1[v] = __builtin_nontemporal_load(p1 + v);
        s2[v] = __builtin_nontemporal_load(p2 + v);
        so[v] = __builtin_nontemporal_load(po + v);
      } else {
        s1[v] = p1[v];
        s2[v] = p2[v];
        so[v] = po[v];
      }
    }
  }
  __syncthreads();
  if (t < nel) {
    T x, y, z;
    __builtin_memcpy(&x, &s1[2 * t], 32);
    __builtin_memcpy(&y, &s2[2 * t], 32);
    __builtin_memcpy(&z, &so[2 * t], 32);
    store_fields(&z, OP()(x, y));
    __builtin_memcpy(&so[2 * t], &z, 32);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const unsigned v = t + k * BS;
    if (v < nv) {
      if constexpr (NT) __builtin_nontemporal_store(so[v], po + v);
      else po[v] = so[v];
    }
  }
}

// 3-buffer results are stored field by field for element types with
// padding (pairs, x87): the reference's LOC_FUNC_3BUF / `*(b) = a1 op a2`
// write only the value fields, so the padding bytes of `out` must keep
// whatever they held.
template <class T, class OP>
__global__ void __launch_bounds__(kBlock)
k_reduce3_elem(const T *__restrict__ a1, const T *__restrict__ a2, T *__restrict__ o, size_t n) {
  const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  OP op;
  if (i < n) store_fields(&o[i], op(a1[i], a2[i]));
}

// One lane per work item; counts beyond 2^31 blocks x 256 lanes (> 8 TiB of
// fp32) are rejected by the callers' size check.
static inline unsigned grid_for(size_t work_items, size_t bs = kBlock) {
  size_t g = (work_items + bs - 1) / bs;
  return (unsigned)(g < 1 ? 1 : g);
}
static constexpr size_t kMaxItems = ((size_t)1 << 31) * kBlock - kBlock;
// one-wave workgroups while the grid fits 2^31 - 1 of them (vectors up to 2^37: 2 TiB)
static inline bool nt_small_wg(size_t work) { return work < ((size_t)1 << 31) * kBlockNT - kBlockNT; }

// MX_REDUCE_W32=0 keeps 32-byte elements on the field-by-field element
// kernel (A/B switch; results are identical)
static bool conv_w32() {
  static const int on = [] {
    const char *e = getenv("MX_REDUCE_W32");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// MX_REDUCE_W32T=0: 32-byte elements move per element (two accesses 32
// bytes apart) instead of through LDS (A/B switch; results are identical)
static bool w32_lds() {
  static const int on = [] {
    const char *e = getenv("MX_REDUCE_W32T");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// launches that carry their own completion mark: grids of at most
// kMarkFlags workgroups.  A 256-lane launch for count elements has at most
// ceil((count + 16) / 256) workgroups (one 16-byte vector, or one element,
// per lane), so counts up to this bound fit; the 64-lane non-temporal
// instances (from 384 MiB footprints unless MX_NT_MIN_BYTES says otherwise)
// may not, and mark_fit drops the mark for them.
constexpr size_t kFusedMarkMax = (size_t)kMarkFlags * 256 - 16;

// Launches mark themselves (default; MX_FUSED_MARK=0
// keeps the marker kernel).  Round 3 switched this off after an 8-process
// failure (one 5000-element block wrong at one rank) that was later traced
// to a different cause -- a freed communicator's flags recycled while a
// peer's trailing signals were still in flight (mx_coll.hip, the IPC region
// pool); that run never called this function.  The contract,
// inout complete for every agent on return (ompi/mca/op/op.h:258-273), is
// tested from another process: tests/test_op_consumer_gpu.py (8 processes,
// coll/base recursive doubling through op/mi355x, each step's result copied
// by the peer through an IPC mapping as soon as the handler returns).
static bool fused_mark() {
  static const int on = [] {
    const char *e = getenv("MX_FUSED_MARK");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// The mark rides on a launch only if its grid has a flag per workgroup
// (kMarkFlags); a larger grid -- e.g. a 64-lane non-temporal instance forced
// below its usual footprint by MX_NT_MIN_BYTES -- runs unmarked and `mk` is
// cleared, so the caller waits through the marker kernel instead (ADVICE r4:
// a mark over part of the grid would return before the rest had written).
static inline const Mark &mark_fit(Mark &mk, unsigned grid) {
  if (mk.flags && grid > kMarkFlags) mk = Mark{nullptr, nullptr, 0};
  return mk;
}

template <class T, class OP>
static int launch2(const void *in, void *inout, size_t n, hipStream_t s, Mark &mk) {
  const T *a = static_cast<const T *>(in);
  T *b = static_cast<T *>(inout);
  if (n == 0) return MX_SUCCESS;
  constexpr size_t N = (sizeof(T) <= 16 && 16 % sizeof(T) == 0) ? 16 / sizeof(T) : 0;
  const uintptr_t ma = (uintptr_t)a & 15, mb = (uintptr_t)b & 15;
  if constexpr (sizeof(T) == 32) {
    if (ma == 0 && mb == 0 && conv_w32()) {
      const bool nt = mx_nt_for(2 * n * sizeof(T)) && nt_small_wg(n);
      if (w32_lds()) {
        if (nt)
          hipLaunchKernelGGL((k_reduce2_w32t<T, OP, true, kBlockNT>), dim3(grid_for(n, kBlockNT)), dim3(kBlockNT), 0,
                             s, a, b, n, mark_fit(mk, grid_for(n, kBlockNT)));
        else
          hipLaunchKernelGGL((k_reduce2_w32t<T, OP, false, kBlock>), dim3(grid_for(n)), dim3(kBlock), 0, s, a, b, n,
                             mark_fit(mk, grid_for(n)));
      } else if (nt) {
        hipLaunchKernelGGL((k_reduce2_w32<T, OP, true, kBlockNT>), dim3(grid_for(n, kBlockNT)), dim3(kBlockNT), 0, s,
                           a, b, n, mark_fit(mk, grid_for(n, kBlockNT)));
      } else {
        hipLaunchKernelGGL((k_reduce2_w32<T, OP, false, kBlock>), dim3(grid_for(n)), dim3(kBlock), 0, s, a, b, n,
                           mark_fit(mk, grid_for(n)));
      }
      return mx_check_launch();
    }
  }
  if (N == 0 || ma != mb || (ma % sizeof(T)) != 0) {
    hipLaunchKernelGGL((k_reduce2_elem<T, OP>), dim3(grid_for(n)), dim3(kBlock), 0, s, a, b, n, mark_fit(mk, grid_for(n)));
    return mx_check_launch();
  }
  size_t head = ma ? (16 - ma) / sizeof(T) : 0;
  if (head > n) head = n;
  const size_t nvec = N ? (n - head) / N : 0;
  size_t work = nvec;
  if (work < head + N) work = head + N;  // enough lanes for head + tail
  if (mx_nt_for(2 * n * sizeof(T))) {
    if (nt_small_wg(work))
      hipLaunchKernelGGL((k_reduce2<T, OP, true>), dim3(grid_for(work, kBlockNT)), dim3(kBlockNT), 0, s, a, b, n, head,
                         nvec, mark_fit(mk, grid_for(work, kBlockNT)));
    else
      hipLaunchKernelGGL((k_reduce2<T, OP, true, kBlock>), dim3(grid_for(work)), dim3(kBlock), 0, s, a, b, n, head,
                         nvec, mark_fit(mk, grid_for(work)));
  } else {
    hipLaunchKernelGGL((k_reduce2<T, OP, false>), dim3(grid_for(work)), dim3(kBlock), 0, s, a, b, n, head, nvec,
                       mark_fit(mk, grid_for(work)));
  }
  return mx_check_launch();
}

template <class T, class OP>
static int launch3(const void *in1, const void *in2, void *out, size_t n, hipStream_t s) {
  const T *a1 = static_cast<const T *>(in1);
  const T *a2 = static_cast<const T *>(in2);
  T *o = static_cast<T *>(out);
  if (n == 0) return MX_SUCCESS;
  constexpr size_t N = (sizeof(T) <= 16 && 16 % sizeof(T) == 0) ? 16 / sizeof(T) : 0;
  constexpr bool PAD = has_pad<T>::value;
  const uintptr_t m1 = (uintptr_t)a1 & 15, m2 = (uintptr_t)a2 & 15, mo = (uintptr_t)o & 15;
  if constexpr (sizeof(T) == 32) {
    if (m1 == 0 && m2 == 0 && mo == 0 && w32_lds()) {
      if (mx_nt_for(3 * n * sizeof(T)) && nt_small_wg(n))
        hipLaunchKernelGGL((k_reduce3_w32t<T, OP, true, kBlockNT>), dim3(grid_for(n, kBlockNT)), dim3(kBlockNT), 0, s,
                           a1, a2, o, n);
      else
        hipLaunchKernelGGL((k_reduce3_w32t<T, OP, false, kBlock>), dim3(grid_for(n)), dim3(kBlock), 0, s, a1, a2, o,
                           n);
      return mx_check_launch();
    }
  }
  if (N == 0 || (PAD && !w32_lds()) || m1 != m2 || m1 != mo || (m1 % sizeof(T)) != 0) {
    hipLaunchKernelGGL((k_reduce3_elem<T, OP>), dim3(grid_for(n)), dim3(kBlock), 0, s, a1, a2, o, n);
    return mx_check_launch();
  }
  size_t head = m1 ? (16 - m1) / sizeof(T) : 0;
  if (head > n) head = n;
  const size_t nvec = N ? (n - head) / N : 0;
  size_t work = nvec;
  if (work < head + N) work = head + N;
  if (mx_nt_for(3 * n * sizeof(T))) {
    if (nt_small_wg(work))
      hipLaunchKernelGGL((k_reduce3<T, OP, true, kBlockNT, PAD>), dim3(grid_for(work, kBlockNT)), dim3(kBlockNT), 0, s,
                         a1, a2, o, n, head, nvec);
    else
      hipLaunchKernelGGL((k_reduce3<T, OP, true, kBlock, PAD>), dim3(grid_for(work)), dim3(kBlock), 0, s, a1, a2, o,
                         n, head, nvec);
  } else {
    hipLaunchKernelGGL((k_reduce3<T, OP, false, kBlock, PAD>), dim3(grid_for(work)), dim3(kBlock), 0, s, a1, a2, o, n,
                       head, nvec);
  }
  return mx_check_launch();
}

// ---- type-slot dispatch ---------------------------------------------------
typedef int (*launch2_fn)(const void *, void *, size_t, hipStream_t, Mark &);
typedef int (*launch3_fn)(const void *, const void *, void *, size_t, hipStream_t);

struct entry { launch2_fn f2; launch3_fn f3; };

struct EntryVisitor {
  template <class T, class OP2, class OP3> entry go() { return entry{&launch2<T, OP2>, &launch3<T, OP3>}; }
  entry none() { return entry{nullptr, nullptr}; }
};

static entry lookup(int op, int type) {
  EntryVisitor v;
  return dispatch(op, type, v);
}

}  // namespace mx

using namespace mx;

static bool is_fortran_slot(int t) {
  switch (t) {
    case MX_TYPE_INTEGER: case MX_TYPE_INTEGER1: case MX_TYPE_INTEGER2: case MX_TYPE_INTEGER4:
    case MX_TYPE_INTEGER8: case MX_TYPE_REAL: case MX_TYPE_REAL4: case MX_TYPE_REAL8:
    case MX_TYPE_DOUBLE_PRECISION: case MX_TYPE_LOGICAL: case MX_TYPE_2REAL:
    case MX_TYPE_2DOUBLE_PRECISION: case MX_TYPE_2INTEGER:
      return true;
    default:
      return false;
  }
}

extern "C" int mx_op_supported(int op, int type, int table_variant) {
  if (op < 0 || op >= MX_OP_COUNT || type < 0 || type >= MX_TYPE_COUNT) return 0;
  if (table_variant == MX_TABLE_C_ONLY && is_fortran_slot(type)) return 0;
  return lookup(op, type).f2 != nullptr;
}

extern "C" size_t mx_type_size(int t) {
  switch (t) {
    case MX_TYPE_INT8_T: case MX_TYPE_UINT8_T: case MX_TYPE_INTEGER1: case MX_TYPE_BOOL: case MX_TYPE_BYTE:
      return 1;
    case MX_TYPE_INT16_T: case MX_TYPE_UINT16_T: case MX_TYPE_INTEGER2:
      return 2;
    case MX_TYPE_INT32_T: case MX_TYPE_UINT32_T: case MX_TYPE_INTEGER: case MX_TYPE_INTEGER4:
    case MX_TYPE_FLOAT: case MX_TYPE_REAL: case MX_TYPE_REAL4: case MX_TYPE_LOGICAL:
      return 4;
    case MX_TYPE_INT64_T: case MX_TYPE_UINT64_T: case MX_TYPE_INTEGER8: case MX_TYPE_DOUBLE:
    case MX_TYPE_REAL8: case MX_TYPE_DOUBLE_PRECISION: case MX_TYPE_C_FLOAT_COMPLEX:
    case MX_TYPE_FLOAT_INT: case MX_TYPE_2INT: case MX_TYPE_SHORT_INT: case MX_TYPE_2REAL:
    case MX_TYPE_2INTEGER:
      return 8;
    case MX_TYPE_LONG_DOUBLE: case MX_TYPE_C_DOUBLE_COMPLEX: case MX_TYPE_DOUBLE_INT:
    case MX_TYPE_LONG_INT: case MX_TYPE_2DOUBLE_PRECISION:
      return 16;
    case MX_TYPE_C_LONG_DOUBLE_COMPLEX: case MX_TYPE_LONG_DOUBLE_INT:
      return 32;
    default:
      return 0;
  }
}

extern "C" int mx_reduce2(int op, int type, const void *in, void *inout, size_t count, void *stream) {
  if (op < 0 || op >= MX_OP_COUNT || type < 0 || type >= MX_TYPE_COUNT) return MX_ERR_ARG;
  entry e = lookup(op, type);
  if (!e.f2) return MX_ERR_UNSUPPORTED;
  if (count == 0) return MX_SUCCESS;
  if (!in || !inout || count > kMaxItems) return MX_ERR_ARG;
  int rc = mx_ensure_init();
  if (rc) return rc;
  Mark none{nullptr, nullptr, 0};
  return e.f2(in, inout, count, (hipStream_t)stream, none);
}

extern "C" int mx_reduce2_sync(int op, int type, const void *in, void *inout, size_t count, void *stream) {
  if (op < 0 || op >= MX_OP_COUNT || type < 0 || type >= MX_TYPE_COUNT) return MX_ERR_ARG;
  entry e = lookup(op, type);
  if (!e.f2) return MX_ERR_UNSUPPORTED;
  if (count == 0) return MX_SUCCESS;
  if (!in || !inout || count > kMaxItems) return MX_ERR_ARG;
  int rc = mx_ensure_init();
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  // the resident service (mx_service.hip) for calls on a non-default stream
  // that is idle, with the legacy default stream idle too (svc_reduce checks):
  // nothing the launch would be ordered after is pending, so the served call
  // keeps the launch path's order
  if (s) {
    rc = svc_reduce(op, type, in, nullptr, inout, count, s);
    if (rc) return rc < 0 ? rc : MX_SUCCESS;
  }
  Mark mk{nullptr, nullptr, 0};
  if (fused_mark() && count <= kFusedMarkMax) mark_arm(&mk, true);
  // no flags (or a grid too large for them, cleared by the launch): the marker kernel
  rc = e.f2(in, inout, count, s, mk);
  if (rc) return rc;
  return mk.flags ? mark_wait(mk, s) : mx_stream_sync_fast(stream);
}

// As mx_reduce3, returning with `out` complete for every agent: the op
// component's 3-buffer handler (ompi_3buff_op_reduce, op.h:618-660).  The
// resident service on an idle non-default stream (as mx_reduce2_sync), else
// the launch and the marker kernel.
extern "C" int mx_reduce3_sync(int op, int type, const void *in1, const void *in2, void *out, size_t count,
                               void *stream) {
  if (op < 0 || op >= MX_OP_COUNT || type < 0 || type >= MX_TYPE_COUNT) return MX_ERR_ARG;
  entry e = lookup(op, type);
  if (!e.f3) return MX_ERR_UNSUPPORTED;
  if (count == 0) return MX_SUCCESS;
  if (!in1 || !in2 || !out || count > kMaxItems) return MX_ERR_ARG;
  int rc = mx_ensure_init();
  if (rc) return rc;
  if (stream) {
    rc = svc_reduce(op, type, in1, in2, out, count, (hipStream_t)stream);
    if (rc) return rc < 0 ? rc : MX_SUCCESS;
  }
  rc = e.f3(in1, in2, out, count, (hipStream_t)stream);
  return rc ? rc : mx_stream_sync_fast(stream);
}

extern "C" int mx_reduce3(int op, int type, const void *in1, const void *in2, void *out, size_t count,
                          void *stream) {
  if (op < 0 || op >= MX_OP_COUNT || type < 0 || type >= MX_TYPE_COUNT) return MX_ERR_ARG;
  entry e = lookup(op, type);
  if (!e.f3) return MX_ERR_UNSUPPORTED;
  if (count == 0) return MX_SUCCESS;
  if (!in1 || !in2 || !out || count > kMaxItems) return MX_ERR_ARG;
  int rc = mx_ensure_init();
  if (rc) return rc;
  return e.f3(in1, in2, out, count, (hipStream_t)stream);
}
