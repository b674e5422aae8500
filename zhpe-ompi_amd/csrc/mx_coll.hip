// mx_coll.hip -- all-peer xGMI collectives with the reference's fold order.
//
// What the reference does (ompi/mca/coll/base/coll_base_allreduce.c et al.):
// n-1 neighbour exchanges through the PML, one host `ompi_op_reduce` per
// step.  What this file does on MI355X:
//
//   * a FOLD PROGRAM describes, for a range of elements, the exact reduction
//     tree the selected reference algorithm applies to the n contributions:
//       CHAIN      acc = x[o0]; acc = OP(x[oj], acc) (ring: local operand is
//                  the target, :471/:782) or OP(acc, x[oj]) (basic linear
//                  reduce, coll_base_reduce.c:62-81), for j = 1..n-1;
//       BUTTERFLY  a binary tree over p' = 2^D virtual ranks combined level
//                  by level; at each level the operand holding the `pref`
//                  side is the target.  Recursive doubling (:130-274) is
//                  pref = all ones (every rank computes OP(high, low)),
//                  Rabenseifner (:970-1243) and recursive halving
//                  (coll_base_reduce_scatter.c:132-) are pref = the final
//                  owner's virtual rank; leaves fold the non-power-of-two
//                  pairs (2v, 2v+1) first in the reference's order.
//   * ONE fused kernel per output part loads the n contributions (16-B
//     vectors), evaluates the program in registers (uniform control flow),
//     and stores the result to every destination (local rbuf and each
//     peer's gather area = the allgather push over all xGMI links at once).
//   * multi-process: contributions are pushed all-peer into IPC-mapped
//     staging (uncached device memory), ordered by generation-tagged
//     system-scope flags and bounded spins; local (1-process) communicators
//     read/write every rank's buffers directly.
//
// Work partition (who computes which elements) is COLL_BASE_COMPUTE_
// BLOCKCOUNT over each chunk (coll_base_functions.h:428-435); the FOLD
// partition (which tree an element gets) always follows the reference
// algorithm over the full count, so chunking never changes results.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>

#include "mx_dispatch.hpp"
#include "mx_internal.h"
#include "../../include/mx_coll.h"

namespace mx {

constexpr int MAXR = MX_MAX_RANKS;
constexpr int kFB = 256;  // fold / copy block size

// ---------------------------------------------------------------------------
// fold programs
// ---------------------------------------------------------------------------
enum { PROG_CHAIN = 0, PROG_BFLY = 1 };

struct FoldProg {
  int kind;
  int n;           // chain: number of operands; butterfly: p' leaves
  int D;           // butterfly depth (p' = 1 << D)
  int acc_first;   // chain: accumulator is the target (first operand)
  uint32_t pref;   // butterfly: bit s set -> upper half is the target at level s
  int8_t ord[MAXR];  // chain: source index per step
  int8_t la[MAXR];   // butterfly leaf slot i: first operand source
  int8_t lb[MAXR];   //   second operand source, -1 = plain leaf
};

struct FoldArgs {
  const char *src[MAXR];
  char *dst[MAXR];
  int ndst;
  size_t n, head, nvec;  // elements; scalar head; 16-B vectors after head
  FoldProg p;
};

template <class T> struct alignas(16) fvec {
  static constexpr int N = 16 / sizeof(T);
  T e[N];
};

template <class OP, class T>
__device__ __forceinline__ T comb(const T &x, const T &y) { return OP()(x, y); }
template <class OP, class T>
__device__ __forceinline__ fvec<T> comb(const fvec<T> &x, const fvec<T> &y) {
  fvec<T> r;
#pragma unroll
  for (int j = 0; j < fvec<T>::N; j++) r.e[j] = OP()(x.e[j], y.e[j]);
  return r;
}

// Evaluates the program; LD(j) returns operand j at this lane's position.
template <class OP, class V, class L>
__device__ __forceinline__ V eval_prog(const FoldProg &p, L LD) {
  if (p.kind == PROG_CHAIN) {
    V acc = LD(p.ord[0]);
#pragma unroll
    for (int j = 1; j < MAXR; j++) {
      if (j < p.n) {
        const V v = LD(p.ord[j]);
        acc = p.acc_first ? comb<OP>(acc, v) : comb<OP>(v, acc);
      }
    }
    return acc;
  }
  V R[MAXR];
#pragma unroll
  for (int i = 0; i < MAXR; i++) {
    if (i < p.n) {
      V a = LD(p.la[i]);
      if (p.lb[i] >= 0) a = comb<OP>(a, LD(p.lb[i]));
      R[i] = a;
    }
  }
#pragma unroll
  for (int s = 0; s < 4; s++) {
    if (s < p.D) {
      const int h = 1 << s;
      const bool hi_first = (p.pref >> s) & 1;
#pragma unroll
      for (int u = 0; u < MAXR; u += 2 << s) {
        if (u < p.n) R[u] = hi_first ? comb<OP>(R[u + h], R[u]) : comb<OP>(R[u], R[u + h]);
      }
    }
  }
  return R[0];
}

template <class T, class OP>
__global__ void __launch_bounds__(kFB) k_fold(FoldArgs a) {
  using V = fvec<T>;
  constexpr int N = V::N;
  const size_t tid = (size_t)blockIdx.x * kFB + threadIdx.x;
  if (N > 0 && tid < a.nvec) {
    const size_t off = a.head * sizeof(T) + tid * 16;
    const V r = eval_prog<OP, V>(a.p, [&](int j) { return *reinterpret_cast<const V *>(a.src[j] + off); });
#pragma unroll
    for (int d = 0; d < MAXR; d++)
      if (d < a.ndst) *reinterpret_cast<V *>(a.dst[d] + off) = r;
  }
  // scalar elements: the head, the tail, or everything (element path)
  const size_t tail0 = a.head + a.nvec * N;
  size_t e = (size_t)-1;
  if (tid < a.head) e = tid;
  else if (tid - a.head < a.n - tail0 && tid >= a.head) e = tail0 + (tid - a.head);
  if (e < a.n) {
    const size_t off = e * sizeof(T);
    const T r = eval_prog<OP, T>(a.p, [&](int j) { return *reinterpret_cast<const T *>(a.src[j] + off); });
#pragma unroll
    for (int d = 0; d < MAXR; d++)
      if (d < a.ndst) store_fields(reinterpret_cast<T *>(a.dst[d] + off), r);
  }
}

typedef int (*fold_launch_fn)(FoldArgs &, hipStream_t);

template <class T, class OP>
static int fold_launch(FoldArgs &a, hipStream_t s) {
  constexpr size_t N = (sizeof(T) <= 16 && 16 % sizeof(T) == 0) ? 16 / sizeof(T) : 0;
  bool vec = N > 0 && !has_pad<T>::value;   // padded types: field stores, element path
  uintptr_t m = (uintptr_t)a.src[0] & 15;
  for (int j = 0; j < MAXR; j++)
    if (a.src[j] && ((uintptr_t)a.src[j] & 15) != m) vec = false;
  for (int d = 0; d < a.ndst; d++)
    if (((uintptr_t)a.dst[d] & 15) != m) vec = false;
  if (vec && (m % sizeof(T)) != 0) vec = false;
  if (vec) {
    size_t head = m ? (16 - m) / sizeof(T) : 0;
    if (head > a.n) head = a.n;
    a.head = head;
    a.nvec = (a.n - head) / (N ? N : 1);
  } else {
    a.head = a.n;  // everything scalar (element per lane)
    a.nvec = 0;
  }
  size_t work = a.nvec + a.head + (N ? N : 1);
  if (!vec) work = a.n;
  const size_t g = (work + kFB - 1) / kFB;
  hipLaunchKernelGGL((k_fold<T, OP>), dim3((unsigned)(g ? g : 1)), dim3(kFB), 0, s, a);
  return mx_check_launch();
}

struct FoldVisitor {
  template <class T, class OP2, class OP3> fold_launch_fn go() { return &fold_launch<T, OP2>; }
  fold_launch_fn none() { return nullptr; }
};

// ---------------------------------------------------------------------------
// multi-job byte copy (scatter push, gather, allgather, bcast)
// ---------------------------------------------------------------------------
struct CopyJob { const char *src; char *dst; size_t bytes; };
struct CopyArgs { CopyJob j[MAXR]; int n; };

__global__ void __launch_bounds__(kFB) k_copy(CopyArgs a) {
  const CopyJob jb = a.j[blockIdx.y];
  const size_t tid = (size_t)blockIdx.x * kFB + threadIdx.x;
  const uintptr_t ms = (uintptr_t)jb.src & 15, md = (uintptr_t)jb.dst & 15;
  if (ms == md) {
    size_t head = ms ? 16 - ms : 0;
    if (head > jb.bytes) head = jb.bytes;
    const size_t nvec = (jb.bytes - head) / 16;
    if (tid < nvec)
      reinterpret_cast<uint4 *>(jb.dst + head)[tid] = reinterpret_cast<const uint4 *>(jb.src + head)[tid];
    const size_t tail0 = head + nvec * 16;
    if (tid < head) jb.dst[tid] = jb.src[tid];
    if (tid < jb.bytes - tail0) jb.dst[tail0 + tid] = jb.src[tail0 + tid];
  } else {
    for (size_t i = tid; i < jb.bytes; i += (size_t)gridDim.x * kFB) jb.dst[i] = jb.src[i];
  }
}

static int copy_launch(CopyArgs &a, hipStream_t s) {
  size_t maxw = 1;
  int k = 0;
  for (int i = 0; i < a.n; i++) {
    if (a.j[i].bytes == 0) continue;
    a.j[k++] = a.j[i];
    size_t w = a.j[i].bytes / 16 + 32;
    if (w > maxw) maxw = w;
  }
  a.n = k;
  if (k == 0) return MX_SUCCESS;
  const size_t g = (maxw + kFB - 1) / kFB;
  hipLaunchKernelGGL(k_copy, dim3((unsigned)g, (unsigned)k), dim3(kFB), 0, s, a);
  return mx_check_launch();
}

// ---------------------------------------------------------------------------
// cross-GPU flags: generation-tagged, system scope, bounded spin
// ---------------------------------------------------------------------------
enum { FLAG_READY = 0, FLAG_PUSHED = 1, FLAG_DONE = 2, NFLAGS = 3 };

// one-shot small-message allreduce: per (source rank, workgroup) READY flags
// after the NFLAGS x MAXR block, then one local completion counter.
constexpr int OSWG = 16;
constexpr size_t OS_FLAG_BASE = NFLAGS * MAXR;
constexpr size_t OS_COUNTER = OS_FLAG_BASE + (size_t)MAXR * OSWG;
constexpr size_t FLAG_WORDS = OS_COUNTER + 8;
constexpr size_t kOneShotMax = 64 << 10;   // bytes per rank
constexpr int OS_MAXSEG = 16;

struct SignalArgs { uint64_t *peer_flag[MAXR]; int n; uint64_t value; };

__global__ void k_signal(SignalArgs a) {
  const int j = threadIdx.x;
  __threadfence_system();  // everything this stream wrote is visible first
  if (j < a.n && a.peer_flag[j])
    __hip_atomic_store(a.peer_flag[j], a.value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Waits until flags[j] >= value for every j in `mask`.
__global__ void k_wait(const uint64_t *flags, uint32_t mask, uint64_t value, uint64_t timeout_ticks, int *err) {
  const int j = threadIdx.x;
  if (j < MAXR && ((mask >> j) & 1)) {
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(&flags[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < value) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > timeout_ticks) {
        __hip_atomic_store(err, MX_ERR_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
}

// ---------------------------------------------------------------------------
// one-shot allreduce for small messages: ONE launch per call.  Workgroup w
// owns element slice w: it pushes that slice of my contribution into every
// peer's one-shot slot (double-buffered by generation parity), raises READY
// (source=me, slice=w) at each peer, waits for every peer's READY for slice
// w, and folds the slice for the WHOLE vector from the n copies (every rank
// evaluates the same fold program per element, so all ranks agree bit for
// bit).  Reuse of a parity buffer needs the peer to have finished gen-2,
// i.e. DONE >= gen-2; the last workgroup to finish raises DONE(gen).
// ---------------------------------------------------------------------------
struct OsSeg { size_t lo, hi; FoldProg p; };
struct OneShotArgs {
  const char *sb;
  char *rb;
  char *peer_slot[MAXR];        // peer p's buffer (this parity) at my slot; null for me
  const char *src[MAXR];        // operand j: my buffer (this parity) slot j; src[rank] = sb
  uint64_t *peer_ready[MAXR];   // peer p's OS READY row for source = me
  uint64_t *peer_done[MAXR];    // peer p's DONE flag for source = me
  const uint64_t *my_ready;     // my OS READY rows [src][wg]
  const uint64_t *my_done;      // my DONE flags [src]
  uint64_t *counter;
  uint64_t counter_last, gen, timeout_ticks;
  int *err;
  int n, rank, nseg;
  size_t count, es, slice;
  OsSeg seg[OS_MAXSEG];
};

constexpr int kOSB = 256;

__device__ __forceinline__ void os_spin(const uint64_t *f, uint64_t v, uint64_t ticks, int *err) {
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < v) {
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > ticks) {
      __hip_atomic_store(err, MX_ERR_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
}

template <class T, class OP>
__global__ void __launch_bounds__(kOSB) k_oneshot(OneShotArgs a) {
  const int w = blockIdx.x, t = threadIdx.x;
  const size_t lo = (size_t)w * a.slice, hi = lo + a.slice < a.count ? lo + a.slice : a.count;
  // (1) every peer is past gen-2: its reads of this parity buffer are over
  if (t < a.n && t != a.rank && a.gen > 2) os_spin(a.my_done + t, a.gen - 2, a.timeout_ticks, a.err);
  __syncthreads();
  // (2) push my slice (bytes [lo*es, hi*es)) to every peer
  if (lo < hi) {
    const size_t b0 = lo * a.es, b1 = hi * a.es;
    const bool vec = (((uintptr_t)a.sb | b0 | b1) & 15) == 0;
    for (int p = 0; p < a.n; p++) {
      if (p == a.rank) continue;
      char *d = a.peer_slot[p];
      if (vec) {
        for (size_t i = b0 / 16 + t; i < b1 / 16; i += kOSB)
          reinterpret_cast<uint4 *>(d)[i] = reinterpret_cast<const uint4 *>(a.sb)[i];
      } else {
        for (size_t i = b0 + t; i < b1; i += kOSB) d[i] = a.sb[i];
      }
    }
  }
  __threadfence_system();
  __syncthreads();
  // (3) READY(me, w) at every peer; (4) wait READY(p, w) from every peer
  if (t < a.n && t != a.rank) {
    __hip_atomic_store(a.peer_ready[t] + w, a.gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    os_spin(a.my_ready + (size_t)t * OSWG + w, a.gen, a.timeout_ticks, a.err);
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  // (5) fold the slice
  int sidx = 0;
  for (size_t e = lo + t; e < hi; e += kOSB) {
    while (sidx + 1 < a.nseg && e >= a.seg[sidx].hi) sidx++;
    const size_t off = e * sizeof(T);
    const T r = eval_prog<OP, T>(a.seg[sidx].p, [&](int j) { return *reinterpret_cast<const T *>(a.src[j] + off); });
    store_fields(reinterpret_cast<T *>(a.rb + off), r);
  }
  // (6) the last workgroup out raises DONE(gen) at every peer
  __syncthreads();
  if (t == 0) {
    __threadfence();
    const uint64_t old = __hip_atomic_fetch_add(a.counter, (uint64_t)1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == a.counter_last) {
      __threadfence_system();
      for (int p = 0; p < a.n; p++)
        if (p != a.rank) __hip_atomic_store(a.peer_done[p], a.gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

typedef int (*oneshot_launch_fn)(OneShotArgs &, int nwg, hipStream_t);

template <class T, class OP>
static int oneshot_launch(OneShotArgs &a, int nwg, hipStream_t s) {
  hipLaunchKernelGGL((k_oneshot<T, OP>), dim3(nwg), dim3(kOSB), 0, s, a);
  return mx_check_launch();
}

struct OneShotVisitor {
  template <class T, class OP2, class OP3> oneshot_launch_fn go() { return &oneshot_launch<T, OP2>; }
  oneshot_launch_fn none() { return nullptr; }
};

}  // namespace mx

using namespace mx;

// ---------------------------------------------------------------------------
// communicator
// ---------------------------------------------------------------------------
struct mx_comm {
  int rank, size, device, local;
  int flags;
  size_t staging_bytes;
  size_t main_bytes;           // staging for the chunked paths: [0, main_bytes)
  size_t os_max, os_slot;      // one-shot: max bytes per rank, slot stride
  uint64_t os_count;           // one-shot workgroup completions so far
  char *staging;               // mine (uncached, IPC-exported)
  char *peer_staging[MAXR];    // mapped views (peer_staging[rank] = staging)
  uint64_t *flagmem;           // mine: [NFLAGS][MAXR]
  uint64_t *peer_flags[MAXR];  // mapped views
  int *err_host, *err_dev;
  uint64_t gen;
  double timeout_s;
  uint64_t timeout_ticks;
  ncclComm_t nccl;
  // profiling: event pairs recorded around kernels of the current call
  int prof;
  hipEvent_t ev[64];
  int nev;
  int ev_kind[32];   // 0 fold, 1 push, 2 gather
  double ev_bytes[32];
  mx_coll_stats_t st;
};

static uint64_t ticks_for(double seconds) {
  int rate_khz = 0;
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0) != hipSuccess || rate_khz <= 0)
    rate_khz = 100000;
  return (uint64_t)(seconds * rate_khz * 1000.0);
}

extern "C" int mx_comm_set_profiling(mx_comm_t *c, int on) {
  if (!c) return MX_ERR_ARG;
  if (on && !c->prof) {
    for (int i = 0; i < 64; i++)
      if (hipEventCreate(&c->ev[i]) != hipSuccess) return MX_ERR_HIP;
  }
  c->prof = on ? 1 : 0;
  c->nev = 0;
  return MX_SUCCESS;
}

extern "C" int mx_comm_get_stats(mx_comm_t *c, mx_coll_stats_t *st, int reset) {
  if (!c || !st) return MX_ERR_ARG;
  *st = c->st;
  if (reset) memset(&c->st, 0, sizeof c->st);
  return MX_SUCCESS;
}

// bracket a kernel with an event pair (no-op unless profiling)
static inline void prof_begin(mx_comm *c, hipStream_t s) {
  if (c && c->prof && c->nev + 2 <= 64) (void)hipEventRecord(c->ev[c->nev], s);
}
static inline void prof_end(mx_comm *c, hipStream_t s, int kind, double bytes) {
  if (c && c->prof && c->nev + 2 <= 64) {
    (void)hipEventRecord(c->ev[c->nev + 1], s);
    c->ev_kind[c->nev / 2] = kind;
    c->ev_bytes[c->nev / 2] = bytes;
    c->nev += 2;
  }
}
static void prof_collect(mx_comm *c) {
  if (!c || !c->prof) return;
  c->st.calls++;
  for (int i = 0; i < c->nev; i += 2) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, c->ev[i], c->ev[i + 1]);
    const int k = c->ev_kind[i / 2];
    if (k == 0) { c->st.fold_ms += ms; c->st.fold_launches++; c->st.fold_bytes += c->ev_bytes[i / 2]; }
    else if (k == 1) c->st.push_ms += ms;
    else c->st.gather_ms += ms;
  }
  if (c->nev >= 2) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[c->nev - 1]);
    c->st.total_ms += ms;
  }
  c->nev = 0;
}

extern "C" int mx_comm_set_timeout(mx_comm_t *c, double seconds) {
  if (!c || seconds <= 0) return MX_ERR_ARG;
  c->timeout_s = seconds;
  c->timeout_ticks = ticks_for(seconds);
  return MX_SUCCESS;
}

extern "C" int mx_comm_size(const mx_comm_t *c) { return c ? c->size : MX_ERR_ARG; }
extern "C" int mx_comm_rank(const mx_comm_t *c) { return c ? c->rank : MX_ERR_ARG; }

extern "C" int mx_comm_create_local(int size, int device, mx_comm_t **out) {
  if (!out || size < 1 || size > MAXR) return MX_ERR_ARG;
  int rc = mx_init(device);
  if (rc) return rc;
  mx_comm *c = (mx_comm *)calloc(1, sizeof(mx_comm));
  if (!c) return MX_ERR_NOMEM;
  c->rank = 0;
  c->size = size;
  c->device = g_device;
  c->local = 1;
  mx_comm_set_timeout(c, 60.0);
  *out = c;
  return MX_SUCCESS;
}

struct ipc_info {
  hipIpcMemHandle_t staging, flags;
  int rank, device;
  uint64_t staging_bytes;
};

extern "C" int mx_comm_create(int rank, int size, int device, size_t staging_bytes, int flags,
                              mx_allgather_fn ag, void *ctx, mx_comm_t **out) {
  if (!out || !ag || size < 1 || rank < 0 || rank >= size) return MX_ERR_ARG;
  if ((flags & MX_COMM_IPC) && size > MAXR) return MX_ERR_ARG;
  int rc = mx_init(device);
  if (rc) return rc;
  mx_comm *c = (mx_comm *)calloc(1, sizeof(mx_comm));
  if (!c) return MX_ERR_NOMEM;
  c->rank = rank;
  c->size = size;
  c->device = g_device;
  c->flags = flags;
  mx_comm_set_timeout(c, 60.0);
  if (hipHostMalloc((void **)&c->err_host, sizeof(int), hipHostMallocMapped) != hipSuccess) goto fail;
  *c->err_host = 0;
  if (hipHostGetDevicePointer((void **)&c->err_dev, c->err_host, 0) != hipSuccess) goto fail;

  if (flags & MX_COMM_IPC) {
    ipc_info mine, *all = (ipc_info *)calloc(size, sizeof(ipc_info));
    if (!all) goto fail;
    c->staging_bytes = staging_bytes ? staging_bytes : ((size_t)64 << 20);
    // one-shot region at the top of staging: 2 parities x n slots
    c->os_max = std::min<size_t>(kOneShotMax, c->staging_bytes / (8 * (size_t)size)) & ~(size_t)255;
    if (c->os_max < 1024) c->os_max = 0;
    c->os_slot = c->os_max ? c->os_max + 256 : 0;
    c->main_bytes = (c->staging_bytes - 2 * (size_t)size * c->os_slot) & ~(size_t)255;
    if (hipExtMallocWithFlags((void **)&c->staging, c->staging_bytes, hipDeviceMallocUncached) != hipSuccess ||
        hipExtMallocWithFlags((void **)&c->flagmem, FLAG_WORDS * sizeof(uint64_t), hipDeviceMallocUncached) !=
            hipSuccess ||
        hipMemset(c->flagmem, 0, FLAG_WORDS * sizeof(uint64_t)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
      free(all);
      goto fail;
    }
    memset(&mine, 0, sizeof mine);
    if (hipIpcGetMemHandle(&mine.staging, c->staging) != hipSuccess ||
        hipIpcGetMemHandle(&mine.flags, c->flagmem) != hipSuccess) {
      free(all);
      goto fail;
    }
    mine.rank = rank;
    mine.device = c->device;
    mine.staging_bytes = c->staging_bytes;
    if (ag(&mine, all, sizeof(ipc_info), ctx) != 0) { free(all); goto fail; }
    for (int p = 0; p < size; p++) {
      if (all[p].staging_bytes != c->staging_bytes) { free(all); goto fail; }
      if (p == rank) {
        c->peer_staging[p] = c->staging;
        c->peer_flags[p] = c->flagmem;
        continue;
      }
      if (hipIpcOpenMemHandle((void **)&c->peer_staging[p], all[p].staging, hipIpcMemLazyEnablePeerAccess) !=
              hipSuccess ||
          hipIpcOpenMemHandle((void **)&c->peer_flags[p], all[p].flags, hipIpcMemLazyEnablePeerAccess) !=
              hipSuccess) {
        fprintf(stderr, "mx_comm_create: rank %d cannot map rank %d's staging\n", rank, p);
        free(all);
        goto fail;
      }
    }
    free(all);
    // every rank mapped every peer before anyone signals
    int dummy = 0, *dummies = (int *)calloc(size, sizeof(int));
    int arc = dummies ? ag(&dummy, dummies, sizeof(int), ctx) : -1;
    free(dummies);
    if (arc) goto fail;
  }
  if (flags & MX_COMM_RCCL) {
    ncclUniqueId id, *ids = (ncclUniqueId *)calloc(size, sizeof(ncclUniqueId));
    if (!ids) goto fail;
    memset(&id, 0, sizeof id);
    if (rank == 0 && ncclGetUniqueId(&id) != ncclSuccess) { free(ids); goto fail; }
    if (ag(&id, ids, sizeof(id), ctx) != 0) { free(ids); goto fail; }
    id = ids[0];
    free(ids);
    if (ncclCommInitRank(&c->nccl, size, id, rank) != ncclSuccess) {
      c->nccl = nullptr;
      goto fail;
    }
  }
  *out = c;
  return MX_SUCCESS;
fail:
  mx_comm_destroy(c);
  return MX_ERR_HIP;
}

extern "C" int mx_comm_destroy(mx_comm_t *c) {
  if (!c) return MX_SUCCESS;
  (void)hipDeviceSynchronize();
  for (int p = 0; p < c->size && p < MAXR; p++) {
    if (p == c->rank) continue;
    if (c->peer_staging[p]) (void)hipIpcCloseMemHandle(c->peer_staging[p]);
    if (c->peer_flags[p]) (void)hipIpcCloseMemHandle(c->peer_flags[p]);
  }
  if (c->staging) (void)hipFree(c->staging);
  if (c->flagmem) (void)hipFree(c->flagmem);
  if (c->err_host) (void)hipHostFree(c->err_host);
  if (c->nccl) ncclCommDestroy(c->nccl);
  if (c->prof)
    for (int i = 0; i < 64; i++) (void)hipEventDestroy(c->ev[i]);
  free(c);
  return MX_SUCCESS;
}

// ---------------------------------------------------------------------------
// fold partitions: which tree each element gets (restating the reference)
// ---------------------------------------------------------------------------
namespace {

struct Seg { size_t lo, hi; FoldProg p; };

// COLL_BASE_COMPUTE_BLOCKCOUNT (coll_base_functions.h:428-435)
static void blockcount(size_t count, int nblocks, size_t *off, size_t *len) {
  const size_t late = count / nblocks, split = count % nblocks, early = late + (split ? 1 : 0);
  for (int b = 0; b < nblocks; b++) {
    off[b] = (size_t)b < split ? b * early : b * late + split;
    len[b] = (size_t)b < split ? early : late;
  }
}

static int ilog2(int v) { int d = 0; while ((1 << (d + 1)) <= v) d++; return d; }

static uint32_t bitrev(uint32_t v, int D) {
  uint32_t r = 0;
  for (int i = 0; i < D; i++) if (v & (1u << i)) r |= 1u << (D - 1 - i);
  return r;
}

static FoldProg chain(int n, int start, int step, bool acc_first) {
  FoldProg p;
  memset(&p, 0, sizeof p);
  p.kind = PROG_CHAIN;
  p.n = n;
  p.acc_first = acc_first;
  for (int j = 0; j < n; j++) p.ord[j] = (int8_t)(((start + step * j) % n + n) % n);
  return p;
}

// Butterfly over p' = 2^D virtual ranks.  asc: level s combines on bit s
// (recursive doubling / Rabenseifner: mask = 1, 2, 4, ...); !asc: level s
// combines on bit D-1-s (recursive halving: mask = p'/2, ..., 1).  pref: bit
// b set -> the side with bit b = 1 is the target at the level splitting b.
// Leaves: v < extra -> pair (2v, 2v+1) with the odd one first iff first_odd,
// else real rank v + extra.
static FoldProg butterfly(int n, bool asc, uint32_t pref, bool first_odd) {
  FoldProg p;
  memset(&p, 0, sizeof p);
  const int D = ilog2(n), P = 1 << D, extra = n - P;
  p.kind = PROG_BFLY;
  p.n = P;
  p.D = D;
  p.pref = asc ? pref : bitrev(pref, D);
  for (int i = 0; i < P; i++) {
    const int v = asc ? i : (int)bitrev(i, D);  // slot i holds leaf v
    if (v < extra) {
      p.la[i] = (int8_t)(first_odd ? 2 * v + 1 : 2 * v);
      p.lb[i] = (int8_t)(first_odd ? 2 * v : 2 * v + 1);
    } else {
      p.la[i] = (int8_t)(v + extra);
      p.lb[i] = -1;
    }
  }
  return p;
}

static void push_clip(std::vector<Seg> &out, size_t lo, size_t hi, size_t rlo, size_t rhi, const FoldProg &p) {
  const size_t a = std::max(lo, rlo), b = std::min(hi, rhi);
  if (a < b) out.push_back(Seg{a, b, p});
}

// Allreduce fold segments restricted to [rlo, rhi).
static int allreduce_segments(int alg, int n, size_t count, size_t es, size_t rlo, size_t rhi,
                              std::vector<Seg> &out) {
  if (alg == MX_ALLREDUCE_AUTO) alg = mx_allreduce_decision(n, count, -(int)es);
  if (alg == MX_ALLREDUCE_RING || alg == MX_ALLREDUCE_SEGMENTED_RING) {
    if (count < (size_t)n) alg = MX_ALLREDUCE_RECURSIVE_DOUBLING;  // :371-377 (segmented -> ring -> RD)
  }
  if (alg == MX_ALLREDUCE_RABENSEIFNER) {
    const int P = 1 << ilog2(n);
    if (count < (size_t)P) alg = MX_ALLREDUCE_BASIC_LINEAR;       // :988-995
  }
  switch (alg) {
    case MX_ALLREDUCE_RING:
    case MX_ALLREDUCE_SEGMENTED_RING: {
      // block b folds x_b, then OP(x_{b+1}, acc), ... (:407-482); segmenting
      // into phases (:702-811) only subdivides the blocks.
      size_t off[MAXR], len[MAXR];
      blockcount(count, n, off, len);
      for (int b = 0; b < n; b++) push_clip(out, off[b], off[b] + len[b], rlo, rhi, chain(n, b, +1, false));
      return MX_SUCCESS;
    }
    case MX_ALLREDUCE_RECURSIVE_DOUBLING:
      // every level computes OP(high, low) (:227-236); odd leaves of the
      // non-power-of-two fold compute OP(x_odd, x_even) (:191-193)
      push_clip(out, 0, count, rlo, rhi, butterfly(n, true, 0xffffffffu, true));
      return MX_SUCCESS;
    case MX_ALLREDUCE_BASIC_LINEAR:
      // reduce_intra_basic_linear: rbuf = x_{n-1}; rbuf = OP(rbuf, x_i), i = n-2..0
      push_clip(out, 0, count, rlo, rhi, chain(n, n - 1, -1, true));
      return MX_SUCCESS;
    case MX_ALLREDUCE_RABENSEIFNER: {
      // final window of each virtual rank from recursive halving
      // (:1110-1160): at mask m the lower rank keeps floor(w/2) on the left
      const int D = ilog2(n), P = 1 << D, rem = n - P;
      const size_t lhalf = count / 2;
      for (int v = 0; v < P; v++) {
        size_t lo = 0, w = count;
        for (int s = 0; s < D; s++) {
          const size_t left = w / 2;
          if (v & (1 << s)) { lo += left; w -= left; } else { w = left; }
        }
        // leaves of the non-power-of-two fold: left half OP(x_even, x_odd),
        // right half OP(x_odd, x_even) (:1050-1092)
        if (rem > 0) {
          push_clip(out, lo, std::min(lo + w, lhalf), rlo, rhi, butterfly(n, true, (uint32_t)v, false));
          push_clip(out, std::max(lo, lhalf), lo + w, rlo, rhi, butterfly(n, true, (uint32_t)v, true));
        } else {
          push_clip(out, lo, lo + w, rlo, rhi, butterfly(n, true, (uint32_t)v, false));
        }
      }
      std::sort(out.begin(), out.end(), [](const Seg &a, const Seg &b) { return a.lo < b.lo; });
      return MX_SUCCESS;
    }
    default:
      return MX_ERR_UNSUPPORTED;
  }
}

// Reduce-scatter fold segments for output block `blk` (elements relative to
// the full vector).
static int reduce_scatter_segments(int alg, int n, const size_t *rcounts, size_t es, int blk,
                                   std::vector<Seg> &out) {
  size_t total = 0, disp[MAXR];
  for (int i = 0; i < n; i++) { disp[i] = total; total += rcounts[i]; }
  if (alg == MX_RS_AUTO) alg = mx_reduce_scatter_decision(n, total, -(int)es);
  const size_t lo = disp[blk], hi = disp[blk] + rcounts[blk];
  if (alg == MX_RS_RING) {
    // block b starts at rank b+1 and ends at rank b (:520-604)
    push_clip(out, lo, hi, lo, hi, chain(n, blk + 1, +1, false));
    return MX_SUCCESS;
  }
  if (alg == MX_RS_RECURSIVE_HALVING) {
    // owner virtual rank of block blk (tmp_rcounts, :205-216); every level
    // computes OP(own, received) with masks p'/2 .. 1 (:218-290); leaves
    // of the non-power-of-two fold: odd rank computes OP(x_odd, x_even)
    const int D = ilog2(n), P = 1 << D, rem = n - P;
    int v = blk < 2 * rem ? blk / 2 : blk - rem;
    (void)P;
    push_clip(out, lo, hi, lo, hi, butterfly(n, false, (uint32_t)v, true));
    return MX_SUCCESS;
  }
  return MX_ERR_UNSUPPORTED;
}

static int finish(mx_comm *c, hipStream_t s) {
  if (hipStreamSynchronize(s) != hipSuccess) return MX_ERR_HIP;
  prof_collect(c);
  if (c->err_host && *(volatile int *)c->err_host) {
    int e = *(volatile int *)c->err_host;
    *c->err_host = 0;
    return e;
  }
  return MX_SUCCESS;
}

static int run_fold(mx_comm *c, fold_launch_fn fl, const Seg &sg, size_t part_lo, const char *const *src_base,
                    int nsrc, char *const *dst_base, int ndst, size_t es, hipStream_t s) {
  // src_base / dst_base point at element part_lo of each operand/destination
  FoldArgs a;
  memset(&a, 0, sizeof a);
  const size_t shift = (sg.lo - part_lo) * es;
  for (int j = 0; j < nsrc; j++) a.src[j] = src_base[j] + shift;
  for (int d = 0; d < ndst; d++) a.dst[d] = dst_base[d] + shift;
  a.ndst = ndst;
  a.n = sg.hi - sg.lo;
  a.p = sg.p;
  prof_begin(c, s);
  const int rc = fl(a, s);
  prof_end(c, s, 0, (double)(nsrc + ndst) * (double)a.n * (double)es);
  return rc;
}

}  // namespace

extern "C" int mx_allreduce_decision(int n, size_t count, int type) {
  // ompi_coll_tuned_allreduce_intra_dec_fixed (coll_tuned_decision_fixed.c:44-95);
  // every predefined op is commutative.  type < 0 passes -element_size.
  const size_t es = type < 0 ? (size_t)(-type) : mx_type_size(type);
  const size_t block_dsize = es * count;
  if (n <= 1) return MX_ALLREDUCE_RING;
  if (block_dsize < 10000) return MX_ALLREDUCE_RECURSIVE_DOUBLING;
  if (count > (size_t)n) {
    const size_t segment_size = 1 << 20;
    return (size_t)n * segment_size >= block_dsize ? MX_ALLREDUCE_RING : MX_ALLREDUCE_SEGMENTED_RING;
  }
  return MX_ALLREDUCE_NONOVERLAPPING;
}

extern "C" int mx_reduce_scatter_decision(int n, size_t total_count, int type) {
  // ompi_coll_tuned_reduce_scatter_intra_dec_fixed (:466-512)
  const size_t es = type < 0 ? (size_t)(-type) : mx_type_size(type);
  const double a = 0.0012, b = 8.0;
  const size_t small_message_size = 12 * 1024, large_message_size = 256 * 1024;
  const size_t total = total_count * es;
  int pow2 = 1;
  while (pow2 < n) pow2 <<= 1;
  if (total <= small_message_size || (total <= large_message_size && pow2 == n) ||
      (double)n >= a * (double)total + b)
    return MX_RS_RECURSIVE_HALVING;
  return MX_RS_RING;
}

// ---------------------------------------------------------------------------
// local communicators: all ranks' buffers in this process
// ---------------------------------------------------------------------------
extern "C" int mx_allreduce_local(mx_comm_t *c, const void *const *sbufs, void *const *rbufs, size_t count,
                                  int type, int op, int alg, void *stream) {
  if (!c || !c->local || !rbufs) return MX_ERR_ARG;
  FoldVisitor fv;
  fold_launch_fn fl = dispatch(op, type, fv);
  if (!fl) return MX_ERR_UNSUPPORTED;
  const size_t es = mx_type_size(type);
  const int n = c->size;
  hipStream_t s = (hipStream_t)stream;
  if (count == 0) return MX_SUCCESS;
  const char *src[MAXR];
  char *dst[MAXR];
  for (int j = 0; j < n; j++) {
    const void *sb = (sbufs && sbufs[j] != MX_IN_PLACE) ? sbufs[j] : rbufs[j];
    src[j] = (const char *)sb;
    dst[j] = (char *)rbufs[j];
  }
  if (n == 1) {
    if (src[0] != dst[0] && hipMemcpyAsync(dst[0], src[0], count * es, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return MX_ERR_HIP;
    return finish(c, s);
  }
  size_t off[MAXR], len[MAXR];
  blockcount(count, n, off, len);
  for (int p = 0; p < n; p++) {
    std::vector<Seg> segs;
    int rc = allreduce_segments(alg, n, count, es, off[p], off[p] + len[p], segs);
    if (rc) return rc;
    const char *sp[MAXR];
    char *dp[MAXR];
    for (int j = 0; j < n; j++) { sp[j] = src[j] + off[p] * es; dp[j] = dst[j] + off[p] * es; }
    for (const Seg &sg : segs) {
      rc = run_fold(c, fl, sg, off[p], sp, n, dp, n, es, s);
      if (rc) return rc;
    }
  }
  return finish(c, s);
}

extern "C" int mx_reduce_scatter_local(mx_comm_t *c, const void *const *sbufs, void *const *rbufs,
                                       const size_t *rcounts, int type, int op, int alg, void *stream) {
  if (!c || !c->local || !rbufs || !rcounts) return MX_ERR_ARG;
  FoldVisitor fv;
  fold_launch_fn fl = dispatch(op, type, fv);
  if (!fl) return MX_ERR_UNSUPPORTED;
  const size_t es = mx_type_size(type);
  const int n = c->size;
  hipStream_t s = (hipStream_t)stream;
  size_t disp[MAXR], total = 0;
  for (int j = 0; j < n; j++) { disp[j] = total; total += rcounts[j]; }
  const char *src[MAXR];
  for (int j = 0; j < n; j++) {
    const void *sb = (sbufs && sbufs[j] != MX_IN_PLACE) ? sbufs[j] : rbufs[j];
    src[j] = (const char *)sb;
  }
  if (n == 1) {
    if (src[0] != rbufs[0] && total &&
        hipMemcpyAsync(rbufs[0], src[0], total * es, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return MX_ERR_HIP;
    return finish(c, s);
  }
  // IN_PLACE (or rbuf aliasing sbuf): rank p's result lands at rbufs[p][0..)
  // while other blocks of rbufs[p] are still inputs, so results go to a
  // temporary laid out like the full vector and are copied back at the end.
  bool any_alias = false;
  for (int p = 0; p < n; p++)
    if ((const char *)rbufs[p] == src[p]) any_alias = true;
  char *tmp = nullptr;
  if (any_alias && hipMallocAsync((void **)&tmp, total * es + 16, s) != hipSuccess) return MX_ERR_NOMEM;
  for (int p = 0; p < n; p++) {
    if (!rcounts[p]) continue;
    std::vector<Seg> segs;
    int rc = reduce_scatter_segments(alg, n, rcounts, es, p, segs);
    if (rc) return rc;
    const char *sp[MAXR];
    for (int j = 0; j < n; j++) sp[j] = src[j] + disp[p] * es;
    char *dp[1] = {tmp ? tmp + disp[p] * es : (char *)rbufs[p]};
    for (const Seg &sg : segs)
      if ((rc = run_fold(c, fl, sg, disp[p], sp, n, dp, 1, es, s))) return rc;
  }
  if (tmp) {
    CopyArgs ca;
    memset(&ca, 0, sizeof ca);
    for (int p = 0; p < n; p++)
      if (rcounts[p]) ca.j[ca.n++] = CopyJob{tmp + disp[p] * es, (char *)rbufs[p], rcounts[p] * es};
    int rc = copy_launch(ca, s);
    (void)hipFreeAsync(tmp, s);
    if (rc) return rc;
  }
  return finish(c, s);
}

extern "C" int mx_allgather_local(mx_comm_t *c, const void *const *sbufs, void *const *rbufs, size_t bytes,
                                  void *stream) {
  if (!c || !c->local || !rbufs) return MX_ERR_ARG;
  const int n = c->size;
  hipStream_t s = (hipStream_t)stream;
  if (!bytes) return MX_SUCCESS;
  // all-peer: rank j's block goes to every rank in one launch per source
  for (int j = 0; j < n; j++) {
    const char *sb = (sbufs && sbufs[j] != MX_IN_PLACE) ? (const char *)sbufs[j]
                                                        : (const char *)rbufs[j] + (size_t)j * bytes;
    CopyArgs a;
    memset(&a, 0, sizeof a);
    for (int r = 0; r < n; r++) {
      char *d = (char *)rbufs[r] + (size_t)j * bytes;
      if (d == sb) continue;
      a.j[a.n++] = CopyJob{sb, d, bytes};
    }
    int rc = copy_launch(a, s);
    if (rc) return rc;
  }
  return finish(c, s);
}

extern "C" int mx_bcast_local(mx_comm_t *c, void *const *bufs, size_t bytes, int root, void *stream) {
  if (!c || !c->local || !bufs || root < 0 || root >= c->size) return MX_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (!bytes) return MX_SUCCESS;
  CopyArgs a;
  memset(&a, 0, sizeof a);
  for (int r = 0; r < c->size; r++)
    if (r != root) a.j[a.n++] = CopyJob{(const char *)bufs[root], (char *)bufs[r], bytes};
  int rc = copy_launch(a, s);
  if (rc) return rc;
  return finish(c, s);
}

// ---------------------------------------------------------------------------
// multi-process all-peer path (IPC staging + flags)
// ---------------------------------------------------------------------------
namespace {

static int signal_all(mx_comm *c, int kind, uint64_t value, hipStream_t s) {
  SignalArgs a;
  memset(&a, 0, sizeof a);
  a.n = c->size;
  a.value = value;
  for (int p = 0; p < c->size; p++)
    a.peer_flag[p] = (p == c->rank) ? nullptr : c->peer_flags[p] + kind * MAXR + c->rank;
  hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, s, a);
  return mx_check_launch();
}

static int wait_mask(mx_comm *c, int kind, uint32_t mask, uint64_t value, hipStream_t s) {
  hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, s, (const uint64_t *)(c->flagmem + kind * MAXR), mask, value,
                     c->timeout_ticks, c->err_dev);
  return mx_check_launch();
}
static int wait_all(mx_comm *c, int kind, uint64_t value, hipStream_t s) {
  const uint32_t all = (c->size >= 32) ? 0xffffffffu : ((1u << c->size) - 1);
  return wait_mask(c, kind, all & ~(1u << c->rank), value, s);
}

static inline size_t rup(size_t v, size_t a) { return (v + a - 1) / a * a; }

// staging layout for a chunk of `ce` elements of size es
struct Layout { size_t slot, gather_off; };
static Layout layout_for(int n, size_t ce, size_t es) {
  Layout L;
  L.slot = rup((ce + n - 1) / n * es + 16, 256);
  L.gather_off = rup(L.slot * n, 256);
  return L;
}
static size_t chunk_elems(const mx_comm *c, size_t count, size_t es) {
  const int n = c->size;
  size_t ce = count;
  while (ce > 1) {
    Layout L = layout_for(n, ce, es);
    if (L.gather_off + ce * es + 16 <= c->main_bytes) break;
    const size_t fit = (c->main_bytes > (size_t)(n + 2) * 512)
                           ? (c->main_bytes - (size_t)(n + 2) * 512) / (2 * es) : 1;
    ce = std::min(ce - 1, std::max<size_t>(fit, 1));
  }
  return ce;
}

// one-shot allreduce (small messages): one kernel, see k_oneshot
static int allreduce_oneshot(mx_comm *c, oneshot_launch_fn ol, const std::vector<Seg> &segs, const char *sb,
                             char *rb, size_t count, size_t es, hipStream_t s) {
  const int n = c->size, r = c->rank;
  const uint64_t g = ++c->gen;
  char *const region = c->staging + c->main_bytes + (g & 1) * (size_t)n * c->os_slot;
  OneShotArgs a;
  memset(&a, 0, sizeof a);
  a.sb = sb;
  a.rb = rb;
  for (int p = 0; p < n; p++) {
    const size_t peer_region = c->main_bytes + (g & 1) * (size_t)n * c->os_slot;
    a.peer_slot[p] = p == r ? nullptr : c->peer_staging[p] + peer_region + (size_t)r * c->os_slot;
    a.src[p] = p == r ? sb : region + (size_t)p * c->os_slot;
    a.peer_ready[p] = p == r ? nullptr : c->peer_flags[p] + OS_FLAG_BASE + (size_t)r * OSWG;
    a.peer_done[p] = p == r ? nullptr : c->peer_flags[p] + FLAG_DONE * MAXR + r;
  }
  a.my_ready = c->flagmem + OS_FLAG_BASE;
  a.my_done = c->flagmem + FLAG_DONE * MAXR;
  a.counter = c->flagmem + OS_COUNTER;
  a.gen = g;
  a.timeout_ticks = c->timeout_ticks;
  a.err = c->err_dev;
  a.n = n;
  a.rank = r;
  a.count = count;
  a.es = es;
  // slices of ~4 KiB, 16-byte aligned when the element size allows
  const size_t bytes = count * es;
  size_t nwg = std::min<size_t>(OSWG, std::max<size_t>(1, (bytes + 4095) / 4096));
  size_t slice = (count + nwg - 1) / nwg;
  if (16 % es == 0) slice = rup(slice, 16 / es);
  nwg = (count + slice - 1) / slice;
  a.slice = slice;
  a.counter_last = c->os_count + nwg - 1;
  c->os_count += nwg;
  a.nseg = (int)segs.size();
  for (size_t i = 0; i < segs.size(); i++) a.seg[i] = OsSeg{segs[i].lo, segs[i].hi, segs[i].p};
  prof_begin(c, s);
  int rc = ol(a, (int)nwg, s);
  prof_end(c, s, 0, (double)(n + 1) * (double)bytes);
  if (rc) return rc;
  return finish(c, s);
}

}  // namespace

extern "C" int mx_allreduce(mx_comm_t *c, const void *sbuf, void *rbuf, size_t count, int type, int op, int alg,
                            void *stream) {
  if (!c || !rbuf) return MX_ERR_ARG;
  if (c->local) {
    const void *sb[1] = {sbuf};
    void *rb[1] = {rbuf};
    if (c->size != 1) return MX_ERR_STATE;
    return mx_allreduce_local(c, sb, rb, count, type, op, alg, stream);
  }
  hipStream_t s = (hipStream_t)stream;
  const size_t es = mx_type_size(type);
  if (!es) return MX_ERR_ARG;
  const int n = c->size, r = c->rank;
  const char *sb = (sbuf == MX_IN_PLACE || !sbuf) ? (const char *)rbuf : (const char *)sbuf;
  char *rb = (char *)rbuf;
  if (count == 0) return MX_SUCCESS;
  if (alg == MX_ALLREDUCE_RCCL) {
    if (!c->nccl) return MX_ERR_STATE;
    ncclDataType_t dt;
    ncclRedOp_t ro;
    switch (type) {
      case MX_TYPE_INT8_T: case MX_TYPE_INTEGER1: dt = ncclInt8; break;
      case MX_TYPE_UINT8_T: dt = ncclUint8; break;
      case MX_TYPE_INT32_T: case MX_TYPE_INTEGER: case MX_TYPE_INTEGER4: dt = ncclInt32; break;
      case MX_TYPE_UINT32_T: dt = ncclUint32; break;
      case MX_TYPE_INT64_T: case MX_TYPE_INTEGER8: dt = ncclInt64; break;
      case MX_TYPE_UINT64_T: dt = ncclUint64; break;
      case MX_TYPE_FLOAT: case MX_TYPE_REAL: case MX_TYPE_REAL4: dt = ncclFloat32; break;
      case MX_TYPE_DOUBLE: case MX_TYPE_REAL8: case MX_TYPE_DOUBLE_PRECISION: dt = ncclFloat64; break;
      default: return MX_ERR_UNSUPPORTED;
    }
    switch (op) {
      case MX_OP_SUM: ro = ncclSum; break;
      case MX_OP_PROD: ro = ncclProd; break;
      case MX_OP_MAX: ro = ncclMax; break;
      case MX_OP_MIN: ro = ncclMin; break;
      default: return MX_ERR_UNSUPPORTED;
    }
    if (ncclAllReduce(sb, rb, count, dt, ro, c->nccl, s) != ncclSuccess) return MX_ERR_RCCL;
    return finish(c, s);
  }
  FoldVisitor fv;
  fold_launch_fn fl = dispatch(op, type, fv);
  if (!fl) return MX_ERR_UNSUPPORTED;
  if (n == 1) {
    if (sb != rb && hipMemcpyAsync(rb, sb, count * es, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return MX_ERR_HIP;
    return finish(c, s);
  }
  if (!(c->flags & MX_COMM_IPC)) return MX_ERR_STATE;
  if (c->os_max && count * es <= c->os_max) {
    std::vector<Seg> segs;
    int rc = allreduce_segments(alg, n, count, es, 0, count, segs);
    if (rc) return rc;
    OneShotVisitor ov;
    oneshot_launch_fn ol = dispatch(op, type, ov);
    if (ol && segs.size() <= (size_t)OS_MAXSEG) return allreduce_oneshot(c, ol, segs, sb, rb, count, es, s);
  }
  {  // validate the algorithm once for the whole vector
    std::vector<Seg> probe;
    int rc = allreduce_segments(alg, n, count, es, 0, 0, probe);
    if (rc) return rc;
  }
  const size_t ce = chunk_elems(c, count, es);
  for (size_t c0 = 0; c0 < count; c0 += ce) {
    const size_t cl = std::min(ce, count - c0);
    const Layout L = layout_for(n, ce, es);
    size_t off[MAXR], len[MAXR];
    blockcount(cl, n, off, len);
    const uint64_t g = ++c->gen;
    int rc;
    // (a) peers finished the previous round with their staging
    if ((rc = wait_all(c, FLAG_DONE, g - 1, s))) return rc;
    // (b) push my contribution for part p into rank p's slot `r`
    CopyArgs ca;
    memset(&ca, 0, sizeof ca);
    for (int p = 0; p < n; p++) {
      if (p == r || !len[p]) continue;
      const size_t e0 = c0 + off[p];
      ca.j[ca.n++] = CopyJob{sb + e0 * es, c->peer_staging[p] + (size_t)r * L.slot + ((e0 * es) & 15), len[p] * es};
    }
    prof_begin(c, s);
    if ((rc = copy_launch(ca, s))) return rc;
    prof_end(c, s, 1, 0);
    if ((rc = signal_all(c, FLAG_READY, g, s))) return rc;
    if ((rc = wait_all(c, FLAG_READY, g, s))) return rc;
    // (c) fold my part, store to my rbuf and every peer's gather area
    if (len[r]) {
      const size_t e0 = c0 + off[r];
      const size_t mis = (e0 * es) & 15;
      const char *sp[MAXR];
      char *dp[MAXR];
      int nd = 0;
      for (int j = 0; j < n; j++) sp[j] = (j == r) ? sb + e0 * es : c->staging + (size_t)j * L.slot + mis;
      dp[nd++] = rb + e0 * es;
      for (int p = 0; p < n; p++)
        if (p != r) dp[nd++] = c->peer_staging[p] + L.gather_off + ((c0 * es) & 15) + off[r] * es;
      std::vector<Seg> segs;
      if ((rc = allreduce_segments(alg, n, count, es, e0, e0 + len[r], segs))) return rc;
      for (const Seg &sg : segs)
        if ((rc = run_fold(c, fl, sg, e0, sp, n, dp, nd, es, s))) return rc;
    }
    if ((rc = signal_all(c, FLAG_PUSHED, g, s))) return rc;
    if ((rc = wait_all(c, FLAG_PUSHED, g, s))) return rc;
    // (d) copy the other parts from my gather area into rbuf
    memset(&ca, 0, sizeof ca);
    for (int p = 0; p < n; p++) {
      if (p == r || !len[p]) continue;
      ca.j[ca.n++] = CopyJob{c->staging + L.gather_off + ((c0 * es) & 15) + off[p] * es, rb + (c0 + off[p]) * es,
                             len[p] * es};
    }
    prof_begin(c, s);
    if ((rc = copy_launch(ca, s))) return rc;
    prof_end(c, s, 2, 0);
    if ((rc = signal_all(c, FLAG_DONE, g, s))) return rc;
  }
  return finish(c, s);
}

extern "C" int mx_reduce_scatter(mx_comm_t *c, const void *sbuf, void *rbuf, const size_t *rcounts, int type,
                                 int op, int alg, void *stream) {
  if (!c || !rbuf || !rcounts) return MX_ERR_ARG;
  if (c->local) {
    if (c->size != 1) return MX_ERR_STATE;
    const void *sb[1] = {sbuf};
    void *rb[1] = {rbuf};
    return mx_reduce_scatter_local(c, sb, rb, rcounts, type, op, alg, stream);
  }
  hipStream_t s = (hipStream_t)stream;
  const size_t es = mx_type_size(type);
  if (!es) return MX_ERR_ARG;
  const int n = c->size, r = c->rank;
  const char *sb = (sbuf == MX_IN_PLACE || !sbuf) ? (const char *)rbuf : (const char *)sbuf;
  size_t disp[MAXR], total = 0, maxc = 0;
  for (int j = 0; j < n; j++) { disp[j] = total; total += rcounts[j]; maxc = std::max(maxc, rcounts[j]); }
  if (total == 0) return MX_SUCCESS;
  FoldVisitor fv;
  fold_launch_fn fl = dispatch(op, type, fv);
  if (!fl) return MX_ERR_UNSUPPORTED;
  if (n == 1) {
    if (sb != rbuf && hipMemcpyAsync(rbuf, sb, total * es, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return MX_ERR_HIP;
    return finish(c, s);
  }
  if (!(c->flags & MX_COMM_IPC)) return MX_ERR_STATE;
  std::vector<Seg> segs;
  int rc = reduce_scatter_segments(alg, n, rcounts, es, r, segs);
  if (rc) return rc;
  const size_t slot = rup(maxc * es + 16, 256);
  if (slot * n > c->staging_bytes) return MX_ERR_NOMEM;  // TODO: chunk very large blocks
  const uint64_t g = ++c->gen;
  if ((rc = wait_all(c, FLAG_DONE, g - 1, s))) return rc;
  CopyArgs ca;
  memset(&ca, 0, sizeof ca);
  for (int p = 0; p < n; p++) {
    if (p == r || !rcounts[p]) continue;
    ca.j[ca.n++] = CopyJob{sb + disp[p] * es, c->peer_staging[p] + (size_t)r * slot + ((disp[p] * es) & 15),
                           rcounts[p] * es};
  }
  if ((rc = copy_launch(ca, s))) return rc;
  if ((rc = signal_all(c, FLAG_READY, g, s))) return rc;
  if ((rc = wait_all(c, FLAG_READY, g, s))) return rc;
  if (rcounts[r]) {
    const size_t mis = (disp[r] * es) & 15;
    const char *sp[MAXR];
    for (int j = 0; j < n; j++) sp[j] = (j == r) ? sb + disp[r] * es : c->staging + (size_t)j * slot + mis;
    // IN_PLACE with disp[r] != 0: the result goes to rbuf[0..] which may
    // overlap my own input still being read -> fold into the gather area
    // first, then copy.
    const bool overlap = (sb == (const char *)rbuf) && disp[r] != 0;
    char *dst = overlap ? c->staging + n * slot + mis : (char *)rbuf;
    if (overlap && n * slot + mis + rcounts[r] * es > c->staging_bytes) return MX_ERR_NOMEM;
    char *dp[1] = {dst};
    for (const Seg &sg : segs)
      if ((rc = run_fold(c, fl, sg, disp[r], sp, n, dp, 1, es, s))) return rc;
    if (overlap) {
      memset(&ca, 0, sizeof ca);
      ca.j[ca.n++] = CopyJob{dst, (char *)rbuf, rcounts[r] * es};
      if ((rc = copy_launch(ca, s))) return rc;
    }
  }
  if ((rc = signal_all(c, FLAG_DONE, g, s))) return rc;
  return finish(c, s);
}

extern "C" int mx_allgather(mx_comm_t *c, const void *sbuf, void *rbuf, size_t bytes, void *stream) {
  if (!c || !rbuf) return MX_ERR_ARG;
  if (c->local) {
    if (c->size != 1) return MX_ERR_STATE;
    const void *sb[1] = {sbuf};
    void *rb[1] = {rbuf};
    return mx_allgather_local(c, sb, rb, bytes, stream);
  }
  hipStream_t s = (hipStream_t)stream;
  const int n = c->size, r = c->rank;
  char *rb = (char *)rbuf;
  const char *sb = (sbuf == MX_IN_PLACE || !sbuf) ? rb + (size_t)r * bytes : (const char *)sbuf;
  if (!bytes) return MX_SUCCESS;
  if (n == 1) {
    if (sb != rb && hipMemcpyAsync(rb, sb, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess) return MX_ERR_HIP;
    return finish(c, s);
  }
  if (!(c->flags & MX_COMM_IPC)) return MX_ERR_STATE;
  // n slots of `slot` bytes; each round moves up to `cb` bytes per rank
  const size_t slot = (c->main_bytes / n) & ~(size_t)255;
  if (slot < 512) return MX_ERR_NOMEM;
  const size_t cb = slot - 256;
  for (size_t o = 0; o < bytes; o += cb) {
    const size_t l = std::min(cb, bytes - o);
    const uint64_t g = ++c->gen;
    int rc;
    if ((rc = wait_all(c, FLAG_DONE, g - 1, s))) return rc;
    CopyArgs ca;
    memset(&ca, 0, sizeof ca);
    for (int p = 0; p < n; p++)
      if (p != r) ca.j[ca.n++] = CopyJob{sb + o, c->peer_staging[p] + (size_t)r * slot + ((r * bytes + o) & 15), l};
    if (sb != rb + (size_t)r * bytes) ca.j[ca.n++] = CopyJob{sb + o, rb + (size_t)r * bytes + o, l};
    if ((rc = copy_launch(ca, s))) return rc;
    if ((rc = signal_all(c, FLAG_READY, g, s))) return rc;
    if ((rc = wait_all(c, FLAG_READY, g, s))) return rc;
    memset(&ca, 0, sizeof ca);
    for (int p = 0; p < n; p++)
      if (p != r)
        ca.j[ca.n++] = CopyJob{c->staging + (size_t)p * slot + ((p * bytes + o) & 15), rb + (size_t)p * bytes + o, l};
    if ((rc = copy_launch(ca, s))) return rc;
    if ((rc = signal_all(c, FLAG_DONE, g, s))) return rc;
  }
  return finish(c, s);
}

extern "C" int mx_bcast(mx_comm_t *c, void *buf, size_t bytes, int root, void *stream) {
  if (!c || !buf || root < 0 || root >= c->size) return MX_ERR_ARG;
  if (c->local) {
    if (c->size != 1) return MX_ERR_STATE;
    void *b[1] = {buf};
    return mx_bcast_local(c, b, bytes, root, stream);
  }
  hipStream_t s = (hipStream_t)stream;
  const int n = c->size, r = c->rank;
  if (!bytes || n == 1) return MX_SUCCESS;
  if (!(c->flags & MX_COMM_IPC)) return MX_ERR_STATE;
  const size_t cb = (c->main_bytes - 256) & ~(size_t)255;
  for (size_t o = 0; o < bytes; o += cb) {
    const size_t l = std::min(cb, bytes - o);
    const uint64_t g = ++c->gen;
    int rc;
    if ((rc = wait_all(c, FLAG_DONE, g - 1, s))) return rc;
    if (r == root) {
      CopyArgs ca;
      memset(&ca, 0, sizeof ca);
      for (int p = 0; p < n; p++)
        if (p != r) ca.j[ca.n++] = CopyJob{(const char *)buf + o, c->peer_staging[p] + (o & 15), l};
      if ((rc = copy_launch(ca, s))) return rc;
      if ((rc = signal_all(c, FLAG_READY, g, s))) return rc;
    } else {
      if ((rc = wait_mask(c, FLAG_READY, 1u << root, g, s))) return rc;
      CopyArgs ca;
      memset(&ca, 0, sizeof ca);
      ca.j[ca.n++] = CopyJob{c->staging + (o & 15), (char *)buf + o, l};
      if ((rc = copy_launch(ca, s))) return rc;
    }
    if ((rc = signal_all(c, FLAG_DONE, g, s))) return rc;
  }
  return finish(c, s);
}

// ---------------------------------------------------------------------------
// OpenSHMEM reductions through the allreduce (scoll/mpi, scoll_mpi_ops.c:212-275)
// ---------------------------------------------------------------------------
extern "C" int mx_shmem_to_mpi(int sop, int st, size_t dt_size, int *mx_op, int *mx_type) {
  if (!mx_op || !mx_type) return MX_ERR_ARG;
  switch (sop) {  // shmem_op_to_ompi_op
    case MX_SHMEM_AND: *mx_op = MX_OP_BAND; break;
    case MX_SHMEM_OR: *mx_op = MX_OP_BOR; break;
    case MX_SHMEM_XOR: *mx_op = MX_OP_BXOR; break;
    case MX_SHMEM_MAX: *mx_op = MX_OP_MAX; break;
    case MX_SHMEM_MIN: *mx_op = MX_OP_MIN; break;
    case MX_SHMEM_SUM: *mx_op = MX_OP_SUM; break;
    case MX_SHMEM_PROD: *mx_op = MX_OP_PROD; break;
    default: return MX_ERR_ARG;
  }
  switch (st) {  // shmem_dtype_to_ompi_dtype
    case MX_SHMEM_FLOAT: *mx_type = MX_TYPE_FLOAT; break;
    case MX_SHMEM_DOUBLE: *mx_type = MX_TYPE_DOUBLE; break;
    case MX_SHMEM_LDOUBLE: *mx_type = MX_TYPE_LONG_DOUBLE; break;
    case MX_SHMEM_FCOMPLEX: *mx_type = MX_TYPE_C_FLOAT_COMPLEX; break;
    case MX_SHMEM_DCOMPLEX: *mx_type = MX_TYPE_C_DOUBLE_COMPLEX; break;
    case MX_SHMEM_FINT4: *mx_type = MX_TYPE_INTEGER4; break;
    case MX_SHMEM_FINT8: *mx_type = MX_TYPE_INTEGER8; break;
    case MX_SHMEM_FREAL4: *mx_type = MX_TYPE_REAL4; break;
    case MX_SHMEM_FREAL8: *mx_type = MX_TYPE_REAL8; break;
    case MX_SHMEM_FREAL16: *mx_type = MX_TYPE_REAL16; break;   // no kernel (as in the reference)
    default:
      switch (dt_size * 8) {
        case 64: *mx_type = MX_TYPE_INT64_T; break;
        case 32: *mx_type = MX_TYPE_INT32_T; break;
        case 16: *mx_type = MX_TYPE_INT16_T; break;
        case 8: *mx_type = MX_TYPE_INT8_T; break;
        default: return MX_ERR_ARG;   // ompi_mpi_datatype_null
      }
  }
  return MX_SUCCESS;
}

extern "C" int mx_shmem_reduce(mx_comm_t *c, int sop, int st, size_t dt_size, void *target, const void *source,
                               size_t nreduce, void *stream) {
  int op, type;
  int rc = mx_shmem_to_mpi(sop, st, dt_size, &op, &type);
  if (rc) return rc;
  if (!mx_op_supported(op, type, MX_TABLE_WITH_FORTRAN)) return MX_ERR_UNSUPPORTED;
  if (nreduce == 0) return MX_SUCCESS;
  return mx_allreduce(c, source == target ? MX_IN_PLACE : source, target, nreduce, type, op, MX_ALLREDUCE_AUTO,
                      stream);
}
