// mx_runtime.hip -- process-level state, error mapping and device probes of
// libmx_kernels.so.  The buffer probe replaces the accelerator hooks the
// reference uses to route a buffer (opal/datatype/opal_datatype_cuda.c:70-90
// opal_cuda_check_bufs, opal/mca/common/cuda/common_cuda.c:1736-1857).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <mutex>
#include <vector>
#include "mx_internal.h"
#include "mx_mem.hpp"

namespace mx {
int g_num_cus = 256;
int g_device = -1;

// Launches whose streams together touch at least this many bytes use
// non-temporal 16-byte accesses (mx_mem.hpp); MX_NT_MIN_BYTES overrides
// (0 = always, -1 = never).  384 MiB: above the 256 MiB Infinity Cache a
// re-used working set no longer stays on-die (measured crossover between
// 2 x 128 MiB, where default accesses win 7.36 vs 6.42 TB/s, and 2 x 512 MiB,
// where nt wins 6.32 vs 5.86 TB/s; profiles/r01/nt_policy_sizes.txt).
static long long nt_min_bytes() {
  static long long v = [] {
    const char *e = getenv("MX_NT_MIN_BYTES");
    return e ? atoll(e) : (384LL << 20);
  }();
  return v;
}
bool mx_nt_for(size_t bytes) {
  const long long t = nt_min_bytes();
  return t >= 0 && (long long)bytes >= t;
}
}  // namespace mx

using namespace mx;

int mx_hip_rc(hipError_t e) { return e == hipSuccess ? MX_SUCCESS : MX_ERR_HIP; }

int mx_check_launch(void) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    fprintf(stderr, "mx_kernels: launch failed: %s\n", hipGetErrorString(e));
    return MX_ERR_HIP;
  }
  return MX_SUCCESS;
}

extern "C" int mx_init(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MX_ERR_NOT_INIT;
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess) return MX_ERR_HIP;
  }
  if (device >= n) return MX_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return MX_ERR_HIP;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return MX_ERR_HIP;
  g_num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  g_device = device;
  return MX_SUCCESS;
}

int mx_ensure_init(void) {
  if (g_device >= 0) {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur == g_device) return MX_SUCCESS;
  }
  return mx_init(-1);
}

extern "C" int mx_finalize(void) {
  g_device = -1;
  return MX_SUCCESS;
}

// Buffer classification is on every op-handler and coll-slot call (the
// framework's function tables are fixed at init), so device
// allocations are remembered as address ranges: a pointer inside a known
// range answers without a HIP call.  A miss asks the runtime once
// (hipPointerGetAttributes, then hipMemGetAddressRange for the allocation's
// extent) and replaces the least recently used entry.  Host pointers are not
// cached (a host page never turns into device memory; a freed device range
// can only come back as another device allocation from the same aperture).
namespace {
constexpr int kPtrCache = 64;
struct PtrRange { uintptr_t lo, hi; uint64_t used; };
PtrRange g_ranges[kPtrCache];
uint64_t g_ptr_clock;
pthread_mutex_t g_ptr_mu = PTHREAD_MUTEX_INITIALIZER;
}  // namespace

// MX_PTR_CACHE=0 disables the cache (the before/after measurement of
// profiles/r02/op_call_cost.txt)
static bool ptr_cache_on() {
  static const bool on = [] {
    const char *e = getenv("MX_PTR_CACHE");
    return !(e && e[0] == '0');
  }();
  return on;
}

extern "C" int mx_is_device_ptr(const void *p) {
  if (!p) return 0;
  const uintptr_t a = (uintptr_t)p;
  if (!ptr_cache_on()) {
    hipPointerAttribute_t attr;
    memset(&attr, 0, sizeof attr);
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    return (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) ? 1 : 0;
  }
  pthread_mutex_lock(&g_ptr_mu);
  for (int i = 0; i < kPtrCache; i++)
    if (a >= g_ranges[i].lo && a < g_ranges[i].hi) {
      g_ranges[i].used = ++g_ptr_clock;
      pthread_mutex_unlock(&g_ptr_mu);
      return 1;
    }
  pthread_mutex_unlock(&g_ptr_mu);
  hipPointerAttribute_t attr;
  memset(&attr, 0, sizeof attr);
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    // unregistered host memory: the runtime reports it as an error; take
    // back exactly that error so a later launch check does not see it
    (void)hipGetLastError();
    return 0;
  }
  if (attr.type != hipMemoryTypeDevice && attr.type != hipMemoryTypeManaged) return 0;
  void *base = nullptr;
  size_t bytes = 0;
  if (hipMemGetAddressRange(&base, &bytes, (void *)p) == hipSuccess && base && bytes) {
    pthread_mutex_lock(&g_ptr_mu);
    int victim = 0;
    for (int i = 1; i < kPtrCache; i++)
      if (g_ranges[i].used < g_ranges[victim].used) victim = i;
    g_ranges[victim] = PtrRange{(uintptr_t)base, (uintptr_t)base + bytes, ++g_ptr_clock};
    pthread_mutex_unlock(&g_ptr_mu);
  } else {
    (void)hipGetLastError();
  }
  return 1;
}

// Forget cached device ranges overlapping [p, p + bytes) (the allocation is
// being freed by a caller that knows it; mx_free does this itself).
extern "C" int mx_ptr_cache_forget(const void *p, size_t bytes) {
  const uintptr_t lo = (uintptr_t)p, hi = lo + (bytes ? bytes : 1);
  pthread_mutex_lock(&g_ptr_mu);
  for (int i = 0; i < kPtrCache; i++)
    if (g_ranges[i].lo < hi && lo < g_ranges[i].hi) g_ranges[i] = PtrRange{0, 0, 0};
  pthread_mutex_unlock(&g_ptr_mu);
  return MX_SUCCESS;
}

extern "C" int mx_alloc(size_t bytes, void **p) {
  if (!p) return MX_ERR_ARG;
  *p = nullptr;
  if (!bytes) return MX_SUCCESS;
  if (int rc = mx_ensure_init()) return rc;
  return hipMalloc(p, bytes) == hipSuccess ? MX_SUCCESS : MX_ERR_NOMEM;
}

extern "C" int mx_free(void *p) {
  if (!p) return MX_SUCCESS;
  void *base = nullptr;
  size_t bytes = 0;
  if (hipMemGetAddressRange(&base, &bytes, p) == hipSuccess) mx_ptr_cache_forget(base, bytes);
  else (void)hipGetLastError();
  release_later(p, REL_DEV);   // hipFree waits for every stream of the device
  return MX_SUCCESS;
}

extern "C" int mx_host_alloc(size_t bytes, void **p) {
  if (!p) return MX_ERR_ARG;
  *p = nullptr;
  if (!bytes) return MX_SUCCESS;
  if (int rc = mx_ensure_init()) return rc;
  return hipHostMalloc(p, bytes, hipHostMallocDefault) == hipSuccess ? MX_SUCCESS : MX_ERR_NOMEM;
}

extern "C" int mx_host_free(void *p) {
  if (!p) return MX_SUCCESS;
  release_later(p, REL_HOST);
  return MX_SUCCESS;
}

extern "C" int mx_memcpy(void *dst, const void *src, size_t bytes, void *stream) {
  if (!bytes) return MX_SUCCESS;
  if (!dst || !src) return MX_ERR_ARG;
  return mx_hip_rc(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, (hipStream_t)stream));
}

// A non-blocking stream at the highest priority: the collectives queued on
// it spin on their peers, and a spinning kernel holds back every kernel
// behind it on its hardware queue, whatever the stream; the highest
// priority's queues are not shared with the process's ordinary streams
// (profiles/r02/queue_probe.txt).
extern "C" int mx_stream_create(void **stream) {
  if (!stream) return MX_ERR_ARG;
  if (int rc = mx_ensure_init()) return rc;
  hipStream_t s = nullptr;
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
  if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest) != hipSuccess) return MX_ERR_HIP;
  *stream = s;
  return MX_SUCCESS;
}

// A blocking stream: implicitly after the legacy default stream's earlier
// work (and before its later work) with no event per call -- the same host
// cost as the default stream itself (profiles/r02/stream_probe.txt: 11.6 us
// per synchronous call vs 22.9 us for a non-blocking stream + explicit
// event order).
extern "C" int mx_stream_create_ordered(void **stream) {
  if (!stream) return MX_ERR_ARG;
  if (int rc = mx_ensure_init()) return rc;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamDefault) != hipSuccess) return MX_ERR_HIP;
  *stream = s;
  return MX_SUCCESS;
}

extern "C" int mx_stream_destroy(void *stream) {
  return stream ? mx_hip_rc(hipStreamDestroy((hipStream_t)stream)) : MX_SUCCESS;
}

// `stream` waits (on the device) for everything queued on `after` so far.
// A thread-local event per calling thread: the record and the wait are the
// only host work.
extern "C" int mx_stream_order(void *stream, void *after) {
  if (stream == after) return MX_SUCCESS;
  static thread_local hipEvent_t ev = nullptr;
  if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    ev = nullptr;
    return MX_ERR_HIP;
  }
  if (hipEventRecord(ev, (hipStream_t)after) != hipSuccess) return MX_ERR_HIP;
  return mx_hip_rc(hipStreamWaitEvent((hipStream_t)stream, ev, 0));
}

extern "C" int mx_stream_sync(void *stream) {
  return mx_hip_rc(hipStreamSynchronize((hipStream_t)stream));
}

namespace {
std::mutex g_life_mu;
struct PoolEnt { void *p; size_t bytes; bool host; };
std::vector<PoolEnt> *g_pool = nullptr;   // never destroyed: entries outlive static destructors
}  // namespace

// The legacy default stream.  tools/lifecycle_sync_probe.hip: its copies,
// memsets and kernels never wait for a kernel spinning on a NON-BLOCKING
// stream -- where every request collective (the coll component's request
// stream) and point-to-point channel of this library spins -- while
// hipDeviceSynchronize, hipFree, hipHostFree and hipIpcCloseMemHandle do.  A
// private stream was tried first: it is one more hardware queue per process,
// and with 8 processes sharing one GPU (the test pool's multi-rank setup) the
// extra queues made staged collectives time out waiting for peers whose
// kernels were not scheduled (profiles/r05/gpu_r5f_staged_push_timeout.txt).
hipStream_t mx::life_stream() { return nullptr; }

int mx::life_sync() { return mx_hip_rc(hipStreamSynchronize(life_stream())); }

static void *pool_get(size_t bytes, bool host) {
  {
    std::lock_guard<std::mutex> lk(g_life_mu);
    if (g_pool)
      for (size_t i = 0; i < g_pool->size(); i++)
        if ((*g_pool)[i].bytes == bytes && (*g_pool)[i].host == host) {
          void *p = (*g_pool)[i].p;
          (*g_pool)[i] = g_pool->back();
          g_pool->pop_back();
          return p;
        }
  }
  void *p = nullptr;
  const hipError_t e = host ? hipHostMalloc(&p, bytes, hipHostMallocMapped) : hipMalloc(&p, bytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}
static void pool_put(void *p, size_t bytes, bool host) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_life_mu);
  if (!g_pool) g_pool = new std::vector<PoolEnt>();
  g_pool->push_back(PoolEnt{p, bytes, host});
}
void *mx::pool_dev_get(size_t bytes) { return pool_get(bytes, false); }
void mx::pool_dev_put(void *p, size_t bytes) { pool_put(p, bytes, false); }
void *mx::pool_host_get(size_t bytes) { return pool_get(bytes, true); }
void mx::pool_host_put(void *p, size_t bytes) { pool_put(p, bytes, true); }

namespace {
// one thread's completion word: the marker kernel, last on the stream,
// raises it to the call's sequence number (system-scope store into mapped
// host memory after a system fence), the host polls it
__global__ void k_mark(uint64_t *w, uint64_t v) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
struct MarkWord {
  uint64_t *host = nullptr, *dev = nullptr;
  uint64_t *flags = nullptr, *flags_dev = nullptr;   // kMarkFlags per-workgroup flags (mapped host memory)
  uint64_t seq = 0;
  bool failed = false, flags_failed = false;
  ~MarkWord() {
    if (host) (void)hipHostFree(host);
    if (flags) (void)hipHostFree(flags);
  }
};
thread_local MarkWord t_mark;

MarkWord &mark_word() {
  MarkWord &m = t_mark;
  if (!m.host && !m.failed) {
    if (hipHostMalloc((void **)&m.host, 64, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void **)&m.dev, m.host, 0) != hipSuccess) {
      (void)hipGetLastError();
      if (m.host) (void)hipHostFree(m.host);
      m.host = nullptr;
      m.failed = true;
    } else {
      *(volatile uint64_t *)m.host = 0;
    }
  }
  return m;
}
}  // namespace

void mx::mark_arm(Mark *out, bool flags) {
  MarkWord &m = mark_word();
  *out = Mark{nullptr, nullptr, 0};
  if (!m.host) return;
  if (flags) {
    // made on first use only (the marker-kernel path never needs them); the
    // entries carry the call's sequence number, so they are never reset
    if (!m.flags && !m.flags_failed) {
      if (hipHostMalloc((void **)&m.flags, kMarkFlags * sizeof(uint64_t), hipHostMallocMapped) != hipSuccess ||
          hipHostGetDevicePointer((void **)&m.flags_dev, m.flags, 0) != hipSuccess) {
        (void)hipGetLastError();
        if (m.flags) (void)hipHostFree(m.flags);
        m.flags = nullptr;
        m.flags_failed = true;
      } else {
        memset(m.flags, 0, kMarkFlags * sizeof(uint64_t));
      }
    }
    if (!m.flags) return;
    *out = Mark{nullptr, m.flags_dev, ++m.seq};
    return;
  }
  *out = Mark{m.dev, nullptr, ++m.seq};
}

// every entry of the grid carries v: workgroup 0's entry gives the grid
// size; the rest are read with independent loads (the host overlaps the
// misses on lines the device rewrote)
static bool flags_done(const uint64_t *f, uint64_t v) {
  const uint64_t f0 = __atomic_load_n(f, __ATOMIC_RELAXED);
  if ((f0 >> 12) < v) return false;
  const unsigned n = (unsigned)(f0 & 4095) + 1;
  uint64_t lo = f0;
  for (unsigned b = 1; b < n && b < kMarkFlags; b++) {
    const uint64_t x = __atomic_load_n(f + b, __ATOMIC_RELAXED);
    lo = x < lo ? x : lo;
  }
  if ((lo >> 12) < v) return false;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  return true;
}

int mx::mark_wait(const Mark &mk, hipStream_t s) {
  MarkWord &m = t_mark;
  if ((!mk.word && !mk.flags) || !m.host) return mx_hip_rc(hipStreamSynchronize(s));
  static const long spins = [] {            // ~2 ms of polling; MX_FAST_SYNC_SPINS overrides (tests)
    const char *e = getenv("MX_FAST_SYNC_SPINS");
    return e && *e ? atol(e) : (1L << 16);
  }();
  if (mk.flags) {
    for (long i = 0; i < spins; i++) {
      if (flags_done(m.flags, mk.v)) return MX_SUCCESS;
      __builtin_ia32_pause();
    }
    return mx_hip_rc(hipStreamSynchronize(s));
  }
  for (long i = 0; i < spins; i++) {
    if (__atomic_load_n(m.host, __ATOMIC_ACQUIRE) >= mk.v) return MX_SUCCESS;
    __builtin_ia32_pause();
  }
  return mx_hip_rc(hipStreamSynchronize(s));
}

// hipStreamSynchronize wakes the host several microseconds after the GPU is
// done; a word in mapped host memory is seen as soon as the marker kernel
// writes it (the p2p completion path).  After ~2 ms without the
// word (a long kernel, or a fault) the call falls back to the runtime's wait,
// which also reports errors.
extern "C" int mx_stream_sync_fast(void *stream) {
  hipStream_t s = (hipStream_t)stream;
  Mark mk;
  mark_arm(&mk);
  if (!mk.word) return mx_hip_rc(hipStreamSynchronize(s));
  hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s, mk.word, mk.v);
  if (int rc = mx_check_launch()) return rc;
  return mark_wait(mk, s);
}

extern "C" int mx_copy(void *dst, const void *src, size_t bytes, void *stream) {
  if (bytes == 0) return MX_SUCCESS;
  if (!dst || !src) return MX_ERR_ARG;
  int rc = mx_ensure_init();
  if (rc) return rc;
  return copy_async(dst, src, bytes, (hipStream_t)stream);
}

extern "C" const char *mx_strerror(int rc) {
  switch (rc) {
    case MX_SUCCESS: return "success";
    case MX_ERR_ARG: return "invalid argument";
    case MX_ERR_UNSUPPORTED: return "operation not defined for this datatype";
    case MX_ERR_HIP: return "HIP runtime error";
    case MX_ERR_NOMEM: return "out of memory";
    case MX_ERR_TIMEOUT: return "timed out waiting for a peer";
    case MX_ERR_RCCL: return "RCCL error";
    case MX_ERR_NOT_INIT: return "not initialised / no device";
    case MX_ERR_STATE: return "invalid state";
    case MX_ERR_TRUNCATE: return "message truncated (longer than the receive buffer)";
    case MX_ERR_TAG: return "envelope tag differs from the receive's (channels match in order)";
    default: return "unknown error";
  }
}

extern "C" const char *mx_version(void) { return "mx_kernels gfx950 abi 1"; }
