// mx_service.hip -- a resident reduce service for the op component's
// synchronous calls (ompi_op_reduce on device buffers, ompi/op/op.h:547-610,
// op/mi355x's 2-buffer handler; round 4).
//
// A blocking ompi_op_reduce of a few KiB costs ~7.5 us with a launch per
// call (profiles/r04/op_call_cost_r4_fused_default.txt): the host's launch,
// the packet processor's dispatch and the wake-up, not the ~0.5 us of work.
// The service removes the launch and the dispatch: one kernel of kSvcWG
// workgroups stays resident on a stream of its own (highest priority, whose
// hardware queues the process's ordinary streams do not share)
// and serves commands the host writes into coherent mapped host memory:
//   * the host fills the command (operands, count) and raises its sequence
//     number (a release store); workgroup 0 polls that word over PCIe,
//     copies the command into device memory and raises a device word that
//     the other workgroups poll (L2, not PCIe);
//   * every workgroup takes a system-scope acquire (its XCD's L2 drops stale
//     lines of the operands: the service never passes a kernel boundary),
//     reduces its grid-stride share with the op kernels' element functors,
//     waits for its stores, releases at system scope and counts itself done;
//     the last one raises the done word in mapped host memory, which the
//     host polls -- the completion contract of mx_reduce2_sync (inout final
//     for every agent on return).
// One service per process, bound to one (op, type) at a time (a kernel per
// pair, like the op kernels); a call for another pair stops it and starts
// that pair's.  It leaves by itself after kSvcIdle of wall clock without a
// command, so it holds its CUs only while calls keep coming (the segmented
// ring's one ompi_op_reduce per segment); the host relaunches it on demand
// and, at exit, stops it (atexit), so the grid has drained before the
// process ends.  A command is taken only by a running kernel: if the kernel
// left (idle) before taking the posted one, the host sees the stream idle
// with the command undone and relaunches it from that sequence number --
// a command never runs twice.  Before the first command the host waits for
// the kernel to report itself running; a kernel that does not start within
// kSvcStartUs (its hardware queue held by another spinning kernel) is told
// to leave and the process falls back to launches for good.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <mutex>

#include "mx_dispatch.hpp"
#include "mx_internal.h"
#include "mx_mem.hpp"

namespace mx {

constexpr int kSvcWG = 64;                 // resident workgroups
constexpr int kSvcB = 256;                 // lanes per workgroup
constexpr size_t kSvcMaxBytes = 1 << 20;   // calls up to 1 MiB per buffer
constexpr double kSvcIdleS = 2e-3;         // leave after 2 ms without a command
constexpr double kSvcStartUs = 2000;       // a kernel not running after 2 ms: no service

struct alignas(64) SvcCmd {                // coherent mapped host memory, written by the host
  uint64_t seq;
  uint64_t in, inout, count;
  uint64_t exit;
  uint64_t in2;                            // 3-buffer commands: inout = in OP in2; 0: inout = inout OP in
};
struct alignas(64) SvcHost {               // mapped host memory, written by the kernel
  uint64_t done;                           // last command completed
  uint64_t running;                        // launch epoch the kernel reported at start
};
struct SvcDev {                            // device (uncached): workgroup 0 -> the others
  uint64_t tag;                            // (launch epoch << 32) | broadcast number of this launch
  uint64_t in, inout, count, exit, q, in2; // the command (q: its host sequence number)
  uint64_t done_tag;                       // (epoch << 32) | last broadcast every workgroup finished
  unsigned ctr;                            // workgroups done with the current broadcast
};

__device__ __forceinline__ uint64_t svc_ld(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Broadcasts are numbered per launch (k = 1, 2, ...) and tagged with the
// launch's epoch, so a tag left in device memory by an earlier launch never
// matches.  Workgroup 0 starts its idle clock only once every workgroup has
// finished the last broadcast (done_tag), so a workgroup that became resident
// late never misses a command.
template <class T, class OP, class OP3>
__global__ void __launch_bounds__(kSvcB) k_svc(const SvcCmd *cmd, SvcHost *host, SvcDev *dev, uint64_t last,
                                               uint64_t epoch, uint64_t idle_ticks) {
  __shared__ uint64_t s_in, s_inout, s_count, s_exit, s_q, s_in2;
  uint64_t seen = last;                    // host command sequence number taken last
  uint32_t k = 0;                          // broadcasts of this launch
  if (blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(&host->running, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    k++;
    if (threadIdx.x == 0) {
      if (blockIdx.x == 0) {
        uint64_t t0 = wall_clock64();
        uint64_t q;
        bool idle = false;
        while ((q = svc_ld(&cmd->seq)) <= seen) {
          if (k > 1 && __hip_atomic_load(&dev->done_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                           ((epoch << 32) | (k - 1)))
            t0 = wall_clock64();           // a broadcast still in progress: not idle
          else if (wall_clock64() - t0 > idle_ticks) { idle = true; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        if (idle) {
          s_exit = 1;                      // nothing taken: the others leave with it
        } else {
          __atomic_thread_fence(__ATOMIC_ACQUIRE);
          s_in = svc_ld(&cmd->in);
          s_inout = svc_ld(&cmd->inout);
          s_count = svc_ld(&cmd->count);
          s_exit = svc_ld(&cmd->exit);
          s_in2 = svc_ld(&cmd->in2);
          s_q = q;
          seen = q;
        }
        dev->in = s_in;
        dev->inout = s_inout;
        dev->count = s_count;
        dev->exit = s_exit;
        dev->q = s_q;
        dev->in2 = s_in2;
        __hip_atomic_store(&dev->tag, (epoch << 32) | k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        const uint64_t want = (epoch << 32) | k;
        while (__hip_atomic_load(&dev->tag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != want)
          __builtin_amdgcn_s_sleep(1);
        s_in = dev->in;
        s_inout = dev->inout;
        s_count = dev->count;
        s_exit = dev->exit;
        s_q = dev->q;
        s_in2 = dev->in2;
      }
    }
    __syncthreads();
    if (s_exit) return;                    // every workgroup leaves from here
    __atomic_thread_fence(__ATOMIC_ACQUIRE);   // system scope: stale operand lines of this XCD's L2 dropped
    const T *a = reinterpret_cast<const T *>(s_in);
    T *b = reinterpret_cast<T *>(s_inout);
    const size_t n = s_count;
    constexpr size_t N = 16 / sizeof(T);
    struct alignas(16) V { T e[N]; };
    const size_t nvec = n / N;
    const size_t stride = (size_t)gridDim.x * kSvcB;
    if (!s_in2) {                          // 2-buffer: inout = inout OP in (the op kernels' K1)
      OP op;
      for (size_t i = (size_t)blockIdx.x * kSvcB + threadIdx.x; i < nvec; i += stride) {
        V x, y;
        ld16<false>(x, reinterpret_cast<const V *>(b) + i);
        ld16<false>(y, reinterpret_cast<const V *>(a) + i);
#pragma unroll
        for (size_t j = 0; j < N; j++) store_fields(&x.e[j], op(x.e[j], y.e[j]));
        st16<false>(reinterpret_cast<V *>(b) + i, x);
      }
      for (size_t i = nvec * N + (size_t)blockIdx.x * kSvcB + threadIdx.x; i < n; i += stride)
        store_fields(&b[i], op(b[i], a[i]));
    } else {                               // 3-buffer: out = in1 OP in2 (K2)
      OP3 op;
      const T *a2 = reinterpret_cast<const T *>(s_in2);
      for (size_t i = (size_t)blockIdx.x * kSvcB + threadIdx.x; i < nvec; i += stride) {
        V x, y;
        ld16<false>(x, reinterpret_cast<const V *>(a) + i);
        ld16<false>(y, reinterpret_cast<const V *>(a2) + i);
#pragma unroll
        for (size_t j = 0; j < N; j++) x.e[j] = op(x.e[j], y.e[j]);
        st16<false>(reinterpret_cast<V *>(b) + i, x);
      }
      for (size_t i = nvec * N + (size_t)blockIdx.x * kSvcB + threadIdx.x; i < n; i += stride)
        b[i] = op(a[i], a2[i]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores reached L2
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence_system();              // release: this XCD's L2 written back
      const unsigned d = __hip_atomic_fetch_add(&dev->ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (d == gridDim.x - 1) {
        __hip_atomic_store(&dev->ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&dev->done_tag, (epoch << 32) | k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        __threadfence_system();
        __hip_atomic_store(&host->done, s_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

typedef void (*svc_launch_fn)(const SvcCmd *, SvcHost *, SvcDev *, uint64_t, uint64_t, uint64_t, hipStream_t);

template <class T, class OP, class OP3>
static void svc_launch(const SvcCmd *c, SvcHost *h, SvcDev *d, uint64_t last, uint64_t epoch, uint64_t idle,
                       hipStream_t s) {
  hipLaunchKernelGGL((k_svc<T, OP, OP3>), dim3(kSvcWG), dim3(kSvcB), 0, s, c, h, d, last, epoch, idle);
}

// pairs served: element types that tile 16-byte vectors with no bytes
// outside their value fields (no x87, no padded pair types)
struct SvcVisitor {
  template <class T, class OP2, class OP3> svc_launch_fn go() {
    if constexpr (sizeof(T) <= 16 && 16 % sizeof(T) == 0 && !has_pad<T>::value) return &svc_launch<T, OP2, OP3>;
    else return nullptr;
  }
  svc_launch_fn none() { return nullptr; }
};

namespace {
struct Service {
  std::mutex mu;
  int state = 0;          // 0 not set up, 1 usable, -1 off (disabled, setup failed or never started)
  SvcCmd *cmd = nullptr;  // host pointer
  SvcCmd *cmd_d = nullptr;
  SvcHost *host = nullptr, *host_d = nullptr;
  SvcDev *dev = nullptr;
  hipStream_t s = nullptr;
  uint64_t seq = 0;       // commands posted
  uint64_t epoch = 0;     // launches
  bool live = false;      // a kernel was launched and has not been seen to leave
  int op = -1, type = -1;
  uint64_t idle_ticks = 0;
  uint64_t served = 0;    // commands completed by the service
};
Service g_svc;

bool svc_enabled() {
  static const int on = [] {
    const char *e = getenv("MX_OP_SERVICE");
    return (e && *e == '0') ? 0 : 1;
  }();
  return on != 0;
}

// the kernel has left (its stream is idle)
bool svc_left(Service &v) {
  const hipError_t e = hipStreamQuery(v.s);
  if (e == hipErrorNotReady) return false;
  (void)hipGetLastError();
  return true;
}

void svc_stop_locked(Service &v) {
  if (!v.live) return;
  if (!svc_left(v)) {
    v.cmd->exit = 1;
    __atomic_store_n(&v.cmd->seq, ++v.seq, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(v.s);
    v.cmd->exit = 0;
    // the EXIT command counts as done: later kernels start after it
    __atomic_store_n(&v.host->done, v.seq, __ATOMIC_RELEASE);
  }
  v.live = false;
}

void svc_atexit() {
  Service &v = g_svc;
  std::lock_guard<std::mutex> lk(v.mu);
  if (v.state == 1) svc_stop_locked(v);
}

int svc_setup(Service &v) {
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
  int rate_khz = 0;
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, g_device < 0 ? 0 : g_device) != hipSuccess ||
      rate_khz <= 0)
    rate_khz = 100000;
  v.idle_ticks = (uint64_t)(kSvcIdleS * rate_khz * 1000.0);
  if (hipHostMalloc((void **)&v.cmd, sizeof(SvcCmd), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&v.cmd_d, v.cmd, 0) != hipSuccess ||
      hipHostMalloc((void **)&v.host, sizeof(SvcHost), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&v.host_d, v.host, 0) != hipSuccess ||
      hipExtMallocWithFlags((void **)&v.dev, sizeof(SvcDev), hipDeviceMallocUncached) != hipSuccess ||
      hipMemset(v.dev, 0, sizeof(SvcDev)) != hipSuccess ||
      hipStreamCreateWithPriority(&v.s, hipStreamNonBlocking, greatest) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  memset(v.cmd, 0, sizeof(SvcCmd));
  memset(v.host, 0, sizeof(SvcHost));
  atexit(svc_atexit);
  return 1;
}

// wait for host word *w >= target: ~2 ms of polling, then false
bool svc_poll(const uint64_t *w, uint64_t target, double us) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned k = 0;; k++) {
    if (__atomic_load_n(w, __ATOMIC_ACQUIRE) >= target) return true;
    if ((k & 255) == 255 &&
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > us)
      return false;
    __builtin_ia32_pause();
  }
}
}  // namespace

// 1: served (inout final); 0: not served (the caller launches); < 0 error.
// in2 != nullptr: the 3-buffer form, inout = in OP in2.
int svc_reduce(int op, int type, const void *in, const void *in2, void *inout, size_t count) {
  if (!svc_enabled()) return 0;
  const size_t es = mx_type_size(type);
  if (!es || count * es > kSvcMaxBytes || (((uintptr_t)in | (uintptr_t)in2 | (uintptr_t)inout) & 15)) return 0;
  SvcVisitor vis;
  const svc_launch_fn fn = dispatch(op, type, vis);
  if (!fn) return 0;
  Service &v = g_svc;
  std::lock_guard<std::mutex> lk(v.mu);
  if (v.state == 0) v.state = svc_setup(v);
  if (v.state != 1) return 0;
  if (v.live && (v.op != op || v.type != type)) svc_stop_locked(v);
  if (v.live && svc_left(v)) v.live = false;   // left while idle
  if (!v.live) {
    const uint64_t ep = ++v.epoch;
    fn(v.cmd_d, v.host_d, v.dev, v.seq, ep, v.idle_ticks, v.s);
    if (hipGetLastError() != hipSuccess) { v.state = -1; return 0; }
    if (!svc_poll(&v.host->running, ep, kSvcStartUs)) {
      // not running (its hardware queue is held): tell it to leave when it
      // starts, and launch per call from now on
      v.cmd->exit = 1;
      __atomic_store_n(&v.cmd->seq, ++v.seq, __ATOMIC_RELEASE);
      v.state = -1;
      return 0;
    }
    v.live = true;
    v.op = op;
    v.type = type;
  }
  v.cmd->in = (uint64_t)(uintptr_t)in;
  v.cmd->inout = (uint64_t)(uintptr_t)inout;
  v.cmd->count = count;
  v.cmd->in2 = (uint64_t)(uintptr_t)in2;
  v.cmd->exit = 0;
  const uint64_t q = ++v.seq;
  __atomic_store_n(&v.cmd->seq, q, __ATOMIC_RELEASE);
  for (;;) {
    if (svc_poll(&v.host->done, q, 200)) { v.served++; return 1; }
    if (svc_left(v)) {
      // it left before taking the command (idle exit): the command is not
      // taken -- run a new kernel from the one before
      if (__atomic_load_n(&v.host->done, __ATOMIC_ACQUIRE) >= q) { v.served++; return 1; }
      const uint64_t ep = ++v.epoch;
      fn(v.cmd_d, v.host_d, v.dev, q - 1, ep, v.idle_ticks, v.s);
      if (hipGetLastError() != hipSuccess) { v.live = false; v.state = -1; return MX_ERR_HIP; }
    }
  }
}

}  // namespace mx

extern "C" int mx_op_service_stats(unsigned long long *served, unsigned long long *launches) {
  mx::Service &v = mx::g_svc;
  std::lock_guard<std::mutex> lk(v.mu);
  if (served) *served = v.served;
  if (launches) *launches = v.epoch;
  return v.state;
}
