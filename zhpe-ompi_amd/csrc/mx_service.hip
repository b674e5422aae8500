// mx_service.hip -- a resident reduce service for the op component's
// synchronous calls (ompi_op_reduce on device buffers, ompi/op/op.h:547-610,
// op/mi355x's 2- and 3-buffer handlers; round 4).
//
// A blocking ompi_op_reduce of a few KiB costs ~7 us with a launch per call
// (profiles/r04/op_call_cost_r4_fused_default.txt): the host's launch, the
// packet processor's dispatch and the wake-up, not the ~0.5 us of work.  The
// service removes the launch and the dispatch: a grid of kSvcGrid workgroups
// stays resident on a non-blocking stream of its own, at the least priority,
// whose hardware queue nothing else of the process shares
// (svc_stream_create), and serves the calls of up to kSvcMaxBytes that the
// host writes into coherent mapped host memory.  Per call:
//   * the host fills the command (operands, count) and raises its sequence
//     number (a release store); workgroup 0 reads the 64-byte command line
//     over PCIe;
//   * up to kSvcSoloBytes workgroup 0 serves it alone: a system-scope
//     acquire (stale operand lines dropped: the service never passes a
//     kernel boundary), the op kernels' element functors, a wait for its
//     stores, a system-scope release and the done word in mapped host
//     memory, which the host polls -- mx_reduce2_sync's completion contract
//     (inout final for every agent on return);
//   * above, it broadcasts the command through device memory to the helper
//     workgroups, which sleep between polls; every workgroup takes a share
//     and raises its own flag after its release, and the host waits for all.
// One service per process, bound to one (op, type) at a time (a kernel per
// pair, like the op kernels); a call for another pair stops it and starts
// that pair's.  It leaves by itself after kSvcIdleS without a command, and
// between commands once kSvcLifeS old, so it holds its CUs only while calls
// keep coming and never holds its hardware queue for long.  The host
// relaunches it on demand, waits until it runs and only then posts -- a
// launched kernel takes only the commands after the last one posted, so a
// command never runs twice; one that does not start within kSvcStartUs (its
// queue held by a kernel that may wait for this very thread) is told to
// leave and the call launches instead, as do the calls after it until that
// kernel has left.  At exit the host stops the kernel (atexit), so the grid
// has drained before the process ends.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include "mx_dispatch.hpp"
#include "mx_internal.h"
#include "mx_mem.hpp"

namespace mx {

constexpr int kSvcB = 256;                 // lanes of the one resident workgroup (4 waves; 16 waves cost
                                           // ~1 us more per command, svc_pingpong_probe mode 9)
constexpr int kSvcU = 8;                   // 16-byte vectors in flight per lane and operand
constexpr size_t kSvcMaxBytes = 2 << 20;   // calls up to 2 MiB per buffer (larger: launches, faster from
                                           // ~3 MiB on: profiles/r04/svc_grid_ab.txt)
constexpr size_t kSvcSoloBytes = 64 << 10; // up to 64 KiB workgroup 0 alone; above, the whole grid
constexpr unsigned kSvcGridMax = 64;       // workgroups at most: 0 serves the host, the rest join large commands
constexpr unsigned kSvcGrid = 32;          // (default)
// MX_SVC_DIAG (measurement only, wrong results): bits above the helpers'
// sleep select (16) no acquire, (32) no release, (64) no reduce per command
constexpr int kSvcDiagNoAcq = 16, kSvcDiagNoRel = 32, kSvcDiagNoWork = 64;
constexpr double kSvcIdleS = 100e-6;      // leave after 100 us without a command
constexpr double kSvcLifeS = 1e-3;         // and between commands once 1 ms old (then relaunched)
constexpr double kSvcStartUs = 1000;       // a kernel not running 1 ms after its launch is held
constexpr double kSvcFirstStartUs = 50000; // (50 ms for a pair's first launch: its code object loads)

struct alignas(64) SvcCmd {                // coherent mapped host memory, written by the host
  uint64_t seq;                            // raised last (release): a new command
  uint64_t q;                              // = seq of the command the fields below belong to
  uint64_t in, inout, in2, count;          // in2 != 0: inout = in OP in2; else inout = inout OP in
  uint64_t exit;                           // leave
  uint64_t chk;                            // svc_chk of the words above seq: a torn read never matches
};
static_assert(sizeof(SvcCmd) == 64, "one line");
struct alignas(64) SvcBcast {              // device memory (uncached): workgroup 0 -> the helpers
  uint64_t tag;                            // (launch epoch << 32) | broadcast number, written last
  uint64_t q, in, inout, in2, count, exit, pad;
};
struct alignas(64) SvcHost {               // mapped host memory, written by the kernel
  uint64_t done;                           // last command completed
  uint64_t running;                        // launch epoch the kernel reported at start
  uint64_t left;                           // launch epoch that left idle (before leaving)
};

// The command line is read by one load instruction of wave 0 (lanes 0..7
// one 8-byte system-scope load each): one PCIe round trip.  Eight loads
// from one lane cost ~1.1 us more per command and plain or nontemporal
// loads may be served from the CU's vector cache and never see the host's
// store (tools/svc_pingpong_probe.hip modes 8, 6).  PCIe may serve the
// lanes' words at different times around the host's stores; seq is raised
// last, and a read whose fields are older than its seq would pair a new q
// with old operands, which the checksum over (q, operands) catches (a
// 64-bit mix: a stale set of operands that matches is the same set).  A
// mismatch is read again.
__host__ __device__ __forceinline__ uint64_t svc_mix(uint64_t h, uint64_t x) {
  h ^= x + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
  h ^= h >> 31;
  h *= 0xBF58476D1CE4E5B9ull;
  return h ^ (h >> 29);
}
__host__ __device__ __forceinline__ uint64_t svc_chk(const uint64_t w[8]) {
  uint64_t h = 0x6A09E667F3BCC909ull;
  for (int k = 1; k < 7; k++) h = svc_mix(h, w[k]);
  return h;
}

// wave 0, all lanes: w[] = the command line
__device__ __forceinline__ void svc_read_cmd(const SvcCmd *c, uint64_t w[8]) {
  const int lane = threadIdx.x & 63;
  const uint64_t x = lane < 8 ? __hip_atomic_load(reinterpret_cast<const uint64_t *>(c) + lane, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_SYSTEM)
                              : 0;
#pragma unroll
  for (int k = 0; k < 8; k++) w[k] = __shfl(x, k);
}

// workgroup w of nwg: its share of inout = inout OP in (2-buffer, the op
// kernels' K1) or out = in1 OP in2 (3-buffer, K2) -- 16-byte vectors
// w*kSvcB + t + j*nwg*kSvcB, kSvcU of them per operand in flight, then the
// elements past the last whole vector
template <class T, class OP, class OP3>
__device__ __forceinline__ void svc_work(uint64_t in, uint64_t inout, uint64_t in2, size_t n, unsigned w,
                                         unsigned nwg) {
  const T *a = reinterpret_cast<const T *>(in);
  T *b = reinterpret_cast<T *>(inout);
  constexpr size_t N = 16 / sizeof(T);
  struct alignas(16) V { T e[N]; };
  const size_t nvec = n / N;
  const size_t st = (size_t)nwg * kSvcB;
  const V *va = reinterpret_cast<const V *>(a);
  V *vb = reinterpret_cast<V *>(b);
  size_t i = (size_t)w * kSvcB + threadIdx.x;
  if (!in2) {
    OP op;
    for (; i + (kSvcU - 1) * st < nvec; i += kSvcU * st) {
      V x[kSvcU], y[kSvcU];
#pragma unroll
      for (int u = 0; u < kSvcU; u++) {
        ld16<false>(x[u], vb + i + u * st);
        ld16<false>(y[u], va + i + u * st);
      }
#pragma unroll
      for (int u = 0; u < kSvcU; u++) {
#pragma unroll
        for (size_t j = 0; j < N; j++) store_fields(&x[u].e[j], op(x[u].e[j], y[u].e[j]));
        st16<false>(vb + i + u * st, x[u]);
      }
    }
    for (; i < nvec; i += st) {
      V x, y;
      ld16<false>(x, vb + i);
      ld16<false>(y, va + i);
#pragma unroll
      for (size_t j = 0; j < N; j++) store_fields(&x.e[j], op(x.e[j], y.e[j]));
      st16<false>(vb + i, x);
    }
    for (size_t k = nvec * N + (size_t)w * kSvcB + threadIdx.x; k < n; k += st) store_fields(&b[k], op(b[k], a[k]));
  } else {
    OP3 op;
    const T *a2 = reinterpret_cast<const T *>(in2);
    const V *va2 = reinterpret_cast<const V *>(a2);
    for (; i + (kSvcU - 1) * st < nvec; i += kSvcU * st) {
      V x[kSvcU], y[kSvcU];
#pragma unroll
      for (int u = 0; u < kSvcU; u++) {
        ld16<false>(x[u], va + i + u * st);
        ld16<false>(y[u], va2 + i + u * st);
      }
#pragma unroll
      for (int u = 0; u < kSvcU; u++) {
#pragma unroll
        for (size_t j = 0; j < N; j++) x[u].e[j] = op(x[u].e[j], y[u].e[j]);
        st16<false>(vb + i + u * st, x[u]);
      }
    }
    for (; i < nvec; i += st) {
      V x, y;
      ld16<false>(x, va + i);
      ld16<false>(y, va2 + i);
#pragma unroll
      for (size_t j = 0; j < N; j++) x.e[j] = op(x.e[j], y.e[j]);
      st16<false>(vb + i, x);
    }
    for (size_t k = nvec * N + (size_t)w * kSvcB + threadIdx.x; k < n; k += st) b[k] = op(a[k], a2[k]);
  }
}

// The grid: workgroup 0 serves the host; the helpers 1..nwg-1 join the
// large commands.  Measured on the box (tools/svc_pingpong_probe,
// profiles/r04/svc_pingpong_*.txt): a host -> kernel -> host round trip with
// the service's fences and a 4 KiB reduce costs ~3.5 us; 63 more resident
// workgroups polling a device word between 64-clock sleeps add ~1.9 us to
// every command, with 127 x 64-clock sleeps nothing.  So a command up to
// solo_max bytes is workgroup 0's alone (one release, the host's `done`
// word); a larger one is broadcast through device memory and every
// workgroup takes a share and raises its own flag in mapped host memory
// (`flags[w] = (q << 12) | (nwg - 1)`, the launch marks' format).  Leaving
// (a host EXIT, idle, lifetime) is broadcast too, so the helpers never
// outlive workgroup 0's decision.
template <class T, class OP, class OP3>
__global__ void __launch_bounds__(kSvcB) k_svc(const SvcCmd *cmd, SvcHost *host, uint64_t *flags, SvcBcast *bc,
                                               uint64_t *acks, uint64_t *hrun, uint64_t last, uint64_t epoch,
                                               uint64_t idle_ticks, uint64_t life_ticks, uint64_t solo_max,
                                               int hsleep) {
  __shared__ uint64_t s_in, s_inout, s_count, s_q, s_in2;
  __shared__ int s_exit, s_bcast;
  const unsigned nwg = gridDim.x;
  if (blockIdx.x > 0) {                    // helper: the broadcasts of this launch, in order
    // resident: the host posts to this launch only once every helper says so
    // (a helper never dispatched -- its CUs held by other streams' waves --
    // would leave a broadcast command waiting for its flag)
    if (threadIdx.x == 0)
      __hip_atomic_store(hrun + blockIdx.x, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (uint64_t k = 1;; k++) {
      if (threadIdx.x == 0) {
        const uint64_t want = (epoch << 32) | k;
        // a relaxed poll: an acquire load is followed by an L2 invalidate
        // (buffer_inv sc1) on every iteration, and 31 helpers polling that
        // way dropped the lines of whatever else ran on their XCDs (a
        // concurrent copy lost 33 % at 1 MiB calls, tools/svc_interference.py,
        // profiles/r05/svc_interference_r5.txt).  One acquire once it matches.
        while (__hip_atomic_load(&bc->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
          switch (hsleep & 3) {                // s_sleep takes an immediate
            case 0: __builtin_amdgcn_s_sleep(8); break;
            case 1: __builtin_amdgcn_s_sleep(32); break;
            case 2: __builtin_amdgcn_s_sleep(64); break;
            default: __builtin_amdgcn_s_sleep(127); break;
          }
        }
        // system scope: the broadcast's fields below, and no stale operand line
        if (!(hsleep & kSvcDiagNoAcq)) __atomic_thread_fence(__ATOMIC_ACQUIRE);
        s_q = bc->q;
        s_in = bc->in;
        s_inout = bc->inout;
        s_in2 = bc->in2;
        s_count = bc->count;
        s_exit = bc->exit != 0;
      }
      __syncthreads();
      if (s_exit) return;
      if (!(hsleep & kSvcDiagNoWork)) svc_work<T, OP, OP3>(s_in, s_inout, s_in2, s_count, blockIdx.x, nwg);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores reached L2
      __syncthreads();
      if (threadIdx.x == 0) {
        // the ack first (workgroup 0 reads it before it may broadcast
        // again), then the release, then the host's flag
        __hip_atomic_store(acks + blockIdx.x, (epoch << 32) | k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // release only (system scope: this XCD's L2 written back); a seq_cst
        // __threadfence_system also invalidates the XCD's L2 per call
        if (!(hsleep & kSvcDiagNoRel)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(flags + blockIdx.x, (s_q << 12) | (uint64_t)(nwg - 1), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __syncthreads();                     // s_* are rewritten next round
    }
  }
  uint64_t seen = last;                    // command sequence number taken last (wave 0)
  uint64_t nb = 0;                         // broadcasts of this launch (wave 0)
  uint64_t kc = 0;                         // the last command broadcast's number (wave 0)
  const uint64_t born = wall_clock64();
  if (threadIdx.x == 0)
    __hip_atomic_store(&host->running, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    if (threadIdx.x < 64) {                // wave 0 polls
      const uint64_t t0 = wall_clock64();
      uint64_t w[8];
      int ex = 0;
      for (;;) {
        svc_read_cmd(cmd, w);
        if (w[0] > seen && w[1] == w[0] && w[7] == svc_chk(w)) break;   // a whole new command
        const uint64_t now = wall_clock64();
        if (now - t0 > idle_ticks || now - born > life_ticks) { ex = 1; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      if (!ex) seen = w[0];
      const bool exit_now = ex || w[6] != 0;
      const bool bc_now = !exit_now && nwg > 1 && w[5] * sizeof(T) > solo_max;
      if (nwg > 1 && ex && kc) {
        // no broadcast overwrites the last command's before every helper has
        // acknowledged it.  The host posts a command (or EXIT) only once
        // every flag of the last one is up, so only a leaving decision of
        // this workgroup's own (lifetime, idle) can come while a slow helper
        // has not even read it.
        const unsigned lane = threadIdx.x;
        for (;;) {
          const bool ok = lane == 0 || lane >= nwg ||
                          __hip_atomic_load(acks + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                              ((epoch << 32) | kc);
          if (__all(ok)) break;
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (bc_now) kc = nb + 1;
      if (nwg > 1 && (exit_now || bc_now)) nb++;
      if (threadIdx.x == 0) {
        s_exit = exit_now;
        if (!ex) {
          s_q = w[1];
          s_in = w[2];
          s_inout = w[3];
          s_in2 = w[4];
          s_count = w[5];
        }
        s_bcast = bc_now;
        if (nwg > 1 && (exit_now || bc_now)) {   // the helpers take part (or leave)
          bc->q = s_q;
          bc->in = s_in;
          bc->inout = s_inout;
          bc->in2 = s_in2;
          bc->count = s_count;
          bc->exit = exit_now;
          __hip_atomic_store(&bc->tag, (epoch << 32) | nb, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        // system-scope acquire: stale operand lines dropped from this CU's
        // caches and its XCD's L2 (the service never passes a kernel boundary)
        if (!s_exit && !(hsleep & kSvcDiagNoAcq)) __atomic_thread_fence(__ATOMIC_ACQUIRE);
      }
    }
    __syncthreads();
    if (s_exit) {
      if (threadIdx.x == 0)
        __hip_atomic_store(&host->left, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    const bool bcast = s_bcast;
    if (!(hsleep & kSvcDiagNoWork)) svc_work<T, OP, OP3>(s_in, s_inout, s_in2, s_count, 0, bcast ? nwg : 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores reached L2
    __syncthreads();
    if (threadIdx.x == 0) {
      if (!(hsleep & kSvcDiagNoRel)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // release (system)
      if (bcast)
        __hip_atomic_store(flags, (s_q << 12) | (uint64_t)(nwg - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      else
        __hip_atomic_store(&host->done, s_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();                       // s_* are rewritten next round
  }
}

typedef void (*svc_launch_fn)(const SvcCmd *, SvcHost *, uint64_t *, SvcBcast *, uint64_t *, uint64_t *, uint64_t,
                              uint64_t, uint64_t, uint64_t, uint64_t, int, unsigned, hipStream_t);

template <class T, class OP, class OP3>
static void svc_launch(const SvcCmd *c, SvcHost *h, uint64_t *f, SvcBcast *bc, uint64_t *acks, uint64_t *hrun,
                       uint64_t last, uint64_t epoch, uint64_t idle, uint64_t life, uint64_t solo, int hsleep,
                       unsigned grid, hipStream_t s) {
  hipLaunchKernelGGL((k_svc<T, OP, OP3>), dim3(grid), dim3(kSvcB), 0, s, c, h, f, bc, acks, hrun, last, epoch, idle,
                     life, solo, hsleep);
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
  hipStream_t s = nullptr;
  uint64_t *flags = nullptr, *flags_d = nullptr;   // per-workgroup flags (mapped host memory, kSvcGridMax)
  SvcBcast *bc = nullptr;                          // workgroup 0 -> helpers (device, uncached)
  uint64_t *acks = nullptr;                        // helpers -> workgroup 0 (device, uncached, kSvcGridMax)
  uint64_t *hrun = nullptr, *hrun_d = nullptr;     // helper w's launch epoch at start (mapped host memory)
  unsigned grid = kSvcGrid;
  uint64_t solo = kSvcSoloBytes;
  uint64_t maxb = kSvcMaxBytes;   // calls served up to this many bytes per buffer
  int hsleep = 2;         // helpers' sleep between polls: 8 / 32 / 64 / 127 x 64 clocks
  uint64_t seq = 0;       // commands posted
  uint64_t epoch = 0;     // launches
  bool live = false;      // a kernel is running and has not been seen to leave
  uint64_t pending = 0;   // epoch of a kernel launched but not seen running, told to leave
  int op = -1, type = -1;
  int device = -1;        // the device the service runs on (the caller's at setup)
  uint64_t idle_ticks = 0, life_ticks = 0;
  uint64_t served = 0;    // commands completed by the service
  uint64_t held = 0;      // launches that did not start within kSvcStartUs
  std::vector<svc_launch_fn> started;   // pairs whose kernel has run in this process
};
Service g_svc;

// MX_OP_SERVICE (default on); mx_op_service_set() overrides it at run time
std::atomic<int> g_svc_on{-1};
bool svc_enabled() {
  int on = g_svc_on.load(std::memory_order_relaxed);
  if (on < 0) {
    const char *e = getenv("MX_OP_SERVICE");
    int v = (e && *e == '0') ? 0 : 1;
    g_svc_on.compare_exchange_strong(on, v);
    on = g_svc_on.load(std::memory_order_relaxed);
  }
  return on != 0;
}

// the kernel launched as `ep` has left (it writes `left` after its last
// `done`, from the same thread: once `left` shows, `done` is final)
bool svc_gone(const Service &v, uint64_t ep) { return __atomic_load_n(&v.host->left, __ATOMIC_ACQUIRE) >= ep; }

// wait for host word *w >= target: `us` microseconds of polling, then false
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
// post the command in v.cmd's operand fields as number ++v.seq
uint64_t svc_post(Service &v) {
  const uint64_t q = ++v.seq;
  v.cmd->q = q;
  v.cmd->chk = svc_chk(reinterpret_cast<const uint64_t *>(v.cmd));
  __atomic_store_n(&v.cmd->seq, q, __ATOMIC_RELEASE);
  return q;
}

// stop a running kernel (rebinding to another pair, process exit)
void svc_stop_locked(Service &v) {
  if (!v.live) return;
  if (!svc_gone(v, v.epoch)) {
    // exit stays 1 in the line (the checksum covers it) until the next
    // command is filled in: clearing it right after the post would let the
    // kernel read seq new, exit 0 and a checksum made with exit 1 -- a line it
    // never takes, so it would leave only by its idle timeout
    v.cmd->exit = 1;
    svc_post(v);
    // a running kernel reads it within microseconds; a second of silence
    // means something else went wrong: wait for the stream instead
    if (!svc_poll(&v.host->left, v.epoch, 1e6)) (void)hipStreamSynchronize(v.s);
  }
  v.live = false;
}

void svc_atexit() {
  Service &v = g_svc;
  std::lock_guard<std::mutex> lk(v.mu);
  if (v.state == 1) svc_stop_locked(v);
}

// The service stream takes the LEAST priority: HIP keeps a pool of hardware
// queues per priority (range 1..-1 here: low, normal, high), and nothing
// else of the process runs at low priority, so the service gets a queue of
// its own -- not shared with the application's ordinary streams (whose
// kernels would wait behind a resident service) nor with a communicator's
// high-priority p2p channels (whose spinning receives would hold a
// relaunch).  tools/svc_queue_probe.py: every ordinary and high-priority
// queue held by spinning waves, 20 calls all served at low priority, held
// at normal or high (profiles/r04/svc_queue_probe.txt).
// MX_SVC_PRIORITY=normal|greatest: measurement switch.
hipError_t svc_stream_create(hipStream_t *s) {
  const char *e = getenv("MX_SVC_PRIORITY");
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = greatest = 0;
  if (e && !strcmp(e, "normal")) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  if (e && !strcmp(e, "greatest")) return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, least);
}

int svc_setup(Service &v) {
  if (hipGetDevice(&v.device) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  int rate_khz = 0;
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, v.device) != hipSuccess ||
      rate_khz <= 0)
    rate_khz = 100000;
  v.idle_ticks = (uint64_t)(kSvcIdleS * rate_khz * 1000.0);
  v.life_ticks = (uint64_t)(kSvcLifeS * rate_khz * 1000.0);
  if (hipHostMalloc((void **)&v.cmd, sizeof(SvcCmd), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&v.cmd_d, v.cmd, 0) != hipSuccess ||
      hipHostMalloc((void **)&v.host, sizeof(SvcHost), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&v.host_d, v.host, 0) != hipSuccess ||
      hipHostMalloc((void **)&v.flags, kSvcGridMax * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void **)&v.flags_d, v.flags, 0) != hipSuccess ||
      hipHostMalloc((void **)&v.hrun, kSvcGridMax * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void **)&v.hrun_d, v.hrun, 0) != hipSuccess ||
      hipExtMallocWithFlags((void **)&v.bc, sizeof(SvcBcast), hipDeviceMallocUncached) != hipSuccess ||
      hipExtMallocWithFlags((void **)&v.acks, kSvcGridMax * sizeof(uint64_t), hipDeviceMallocUncached) !=
          hipSuccess ||
      svc_stream_create(&v.s) != hipSuccess ||   // no device-wide sync: other streams may hold spinning kernels
      hipMemsetAsync(v.bc, 0, sizeof(SvcBcast), v.s) != hipSuccess ||
      hipMemsetAsync(v.acks, 0, kSvcGridMax * sizeof(uint64_t), v.s) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  memset(v.cmd, 0, sizeof(SvcCmd));
  memset(v.host, 0, sizeof(SvcHost));
  memset(v.flags, 0, kSvcGridMax * sizeof(uint64_t));
  memset(v.hrun, 0, kSvcGridMax * sizeof(uint64_t));
  // MX_SVC_GRID (1..kSvcGridMax workgroups), MX_SVC_SOLO (bytes workgroup 0
  // takes alone), MX_SVC_HSLEEP (0..3): measurement switches
  if (const char *e = getenv("MX_SVC_GRID")) {
    const long g = atol(e);
    v.grid = g < 1 ? 1 : g > (long)kSvcGridMax ? kSvcGridMax : (unsigned)g;
  }
  if (const char *e = getenv("MX_SVC_HSLEEP")) v.hsleep = atoi(e) & 3;
  if (const char *e = getenv("MX_SVC_DIAG")) {
    v.hsleep |= (atoi(e) & 7) << 4;
    if (v.hsleep >> 4)   // measurement only: served results are wrong
      fprintf(stderr, "mx: MX_SVC_DIAG=%d: the op service skips its acquire / release / reduce -- "
                      "interference measurements only, served results are NOT valid\n", (v.hsleep >> 4) & 7);
  }
  if (const char *e = getenv("MX_SVC_SOLO")) v.solo = (uint64_t)atoll(e);
  if (const char *e = getenv("MX_SVC_MAX")) v.maxb = std::min<uint64_t>((uint64_t)atoll(e), kSvcMaxBytes);
  atexit(svc_atexit);
  return 1;
}

}  // namespace

// `s` and the legacy default stream hold no pending work -- now or within a
// short spin: a launch of ours whose completion word was already seen
// retires in the runtime's books several microseconds later (without the
// spin, one launched call keeps every back-to-back call after it on the
// launch path: test_service_resumes_after_a_launch), and work the caller
// still has queued would hold a launch just as long.  Two queries, ~0.2 us
// when idle (tools/query_cost_probe.py).
static bool svc_streams_idle(hipStream_t s) {
  constexpr double kIdleSpinUs = 50;
  std::chrono::steady_clock::time_point t0;
  for (unsigned k = 0;; k++) {
    const hipError_t e1 = hipStreamQuery(s);
    const hipError_t e2 = e1 == hipSuccess ? hipStreamQuery(nullptr) : hipSuccess;
    if (e1 == hipSuccess && e2 == hipSuccess) return true;
    // any other status is the caller's fault (a failed kernel of theirs):
    // decline, leaving it pending for the launch path to report
    if ((e1 != hipSuccess && e1 != hipErrorNotReady) || (e2 != hipSuccess && e2 != hipErrorNotReady)) return false;
    (void)hipGetLastError();   // hipErrorNotReady is no error
    if (k == 0) t0 = std::chrono::steady_clock::now();
    else if (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > kIdleSpinUs)
      return false;
    __builtin_ia32_pause();
  }
}

// Launch a kernel that takes the commands after v.seq and wait until it
// runs.  A kernel that does not start within kSvcStartUs has its hardware
// queue held -- possibly by a kernel of another stream that waits for what
// this thread does after this call (a spinning wait on a host flag), so
// waiting longer could deadlock.  It is told to leave when it
// starts (an EXIT command it will read first) and calls launch until it has.
static bool svc_start(Service &v, svc_launch_fn fn) {
  const uint64_t ep = ++v.epoch;
  fn(v.cmd_d, v.host_d, v.flags_d, v.bc, v.acks, v.hrun_d, v.seq, ep, v.idle_ticks, v.life_ticks, v.solo, v.hsleep,
     v.grid, v.s);
  if (hipGetLastError() != hipSuccess) { v.state = -1; return false; }
  const bool first = std::find(v.started.begin(), v.started.end(), fn) == v.started.end();
  const auto t0 = std::chrono::steady_clock::now();
  const double budget = first ? kSvcFirstStartUs : kSvcStartUs;
  bool all = svc_poll(&v.host->running, ep, budget);
  // the whole grid must be resident: a broadcast command waits for every
  // helper's flag, and a helper that never dispatched would never raise it
  for (unsigned w = 1; all && w < v.grid; w++) {
    const double used = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    all = svc_poll(v.hrun + w, ep, std::max(0.0, budget - used));
  }
  if (all) {
    if (first) v.started.push_back(fn);
    v.live = true;
    return true;
  }
  // held (or only part of the grid dispatched): told to leave -- workgroup 0
  // broadcasts the EXIT, so helpers that start later leave at once
  v.cmd->exit = 1;
  svc_post(v);
  v.pending = ep;
  v.live = false;
  v.held++;
  return false;
}

// 1: served (inout final); 0: not served (the caller launches); < 0 error.
// in2 != nullptr: the 3-buffer form, inout = in OP in2.  A command is posted
// only to a kernel seen running that was launched after every earlier
// command, so no command runs twice and none waits on a held queue.
int svc_reduce(int op, int type, const void *in, const void *in2, void *inout, size_t count, hipStream_t stream) {
  if (!svc_enabled()) return 0;
  const size_t es = mx_type_size(type);
  if (!es || count * es > kSvcMaxBytes || (((uintptr_t)in | (uintptr_t)in2 | (uintptr_t)inout) & 15)) return 0;
  SvcVisitor vis;
  const svc_launch_fn fn = dispatch(op, type, vis);
  if (!fn) return 0;
  if (!svc_streams_idle(stream)) return 0;
  Service &v = g_svc;
  std::lock_guard<std::mutex> lk(v.mu);
  if (v.state == 0) v.state = svc_setup(v);
  if (v.state != 1 || count * es > v.maxb) return 0;
  int dev = -1;                               // a caller on another device launches there
  if (hipGetDevice(&dev) != hipSuccess || dev != v.device) return 0;
  if (v.pending) {
    if (!svc_gone(v, v.pending)) return 0;    // still held: launch
    v.pending = 0;
  }
  if (v.live && (v.op != op || v.type != type)) svc_stop_locked(v);
  if (v.live && svc_gone(v, v.epoch)) v.live = false;   // left (idle or lifetime)
  if (!v.live) {
    v.op = op;
    v.type = type;
    if (!svc_start(v, fn)) return 0;
  }
  v.cmd->in = (uint64_t)(uintptr_t)in;
  v.cmd->inout = (uint64_t)(uintptr_t)inout;
  v.cmd->count = count;
  v.cmd->in2 = (uint64_t)(uintptr_t)in2;
  v.cmd->exit = 0;
  // the kernel makes the same choice (count * sizeof(T) > solo): a large
  // command completes through every workgroup's flag, a small one through
  // workgroup 0's `done`
  const bool bcast = v.grid > 1 && count * es > v.solo;
  auto finished = [&](uint64_t q) {
    if (!bcast) return __atomic_load_n(&v.host->done, __ATOMIC_ACQUIRE) >= q;
    for (unsigned w = 0; w < v.grid; w++)
      if ((__atomic_load_n(v.flags + w, __ATOMIC_RELAXED) >> 12) < q) return false;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    return true;
  };
  uint64_t q = svc_post(v);
  for (unsigned k = 0;; k++) {
    if (finished(q)) { v.served++; return 1; }
    if ((k & 0xfffff) == 0xfffff) {
      // ~tens of ms without the word: a kernel that faulted or was killed
      // writes neither `done` nor `left` -- the runtime reports it
      const hipError_t e = hipStreamQuery(v.s);
      if (e != hipSuccess && e != hipErrorNotReady) {
        (void)hipGetLastError();
        v.live = false;
        v.state = -1;
        return MX_ERR_HIP;
      }
      if (e == hipSuccess && !finished(q) && !svc_gone(v, v.epoch)) {
        v.live = false;                        // gone without a word: inout unknown, no retry
        v.state = -1;
        return MX_ERR_HIP;
      }
    }
    if ((k & 15) == 15 && svc_gone(v, v.epoch)) {
      // it left: before taking q, or after (a helper may still be finishing
      // its share) -- once the grid has drained the words are final
      if (hipStreamSynchronize(v.s) != hipSuccess) {
        (void)hipGetLastError();
        v.live = false;
        v.state = -1;
        return MX_ERR_HIP;
      }
      if (finished(q)) { v.served++; return 1; }
      v.live = false;
      if (!svc_start(v, fn)) return 0;        // the new kernel starts after q: it never takes it
      q = svc_post(v);                         // the same operands, a new number
    }
    __builtin_ia32_pause();
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

extern "C" int mx_op_service_set(int on) {
  mx::Service &v = mx::g_svc;
  std::lock_guard<std::mutex> lk(v.mu);
  mx::g_svc_on.store(on ? 1 : 0, std::memory_order_relaxed);
  if (!on && v.state == 1) mx::svc_stop_locked(v);
  return MX_SUCCESS;
}

extern "C" int mx_op_service_held(unsigned long long *held) {
  mx::Service &v = mx::g_svc;
  std::lock_guard<std::mutex> lk(v.mu);
  if (held) *held = v.held;
  return v.pending ? 1 : 0;
}

// Test support: a kernel that holds its stream's hardware queue the way a
// p2p receive waiting for a peer does, to test that the
// service never waits on a held queue.  One wave spins on a mapped host
// word until mx_debug_release() raises it or timeout_ms of wall clock
// pass, so the grid always drains.
namespace {
uint64_t *g_hold_word = nullptr, *g_hold_word_d = nullptr;
uint64_t g_hold_gen = 0;
std::mutex g_hold_mu;
}  // namespace

__global__ void __launch_bounds__(64) k_debug_hold(const uint64_t *word, uint64_t gen, uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  if (threadIdx.x == 0)
    while (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < gen && wall_clock64() - t0 < ticks)
      __builtin_amdgcn_s_sleep(8);
}

extern "C" int mx_debug_hold(void *stream, unsigned timeout_ms) {
  if (int rc = mx_ensure_init()) return rc;
  std::lock_guard<std::mutex> lk(g_hold_mu);
  if (!g_hold_word) {
    if (hipHostMalloc((void **)&g_hold_word, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void **)&g_hold_word_d, g_hold_word, 0) != hipSuccess) {
      (void)hipGetLastError();
      g_hold_word = nullptr;
      return MX_ERR_HIP;
    }
    *g_hold_word = 0;
  }
  int rate_khz = 0;
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, mx::g_device < 0 ? 0 : mx::g_device) !=
          hipSuccess || rate_khz <= 0)
    rate_khz = 100000;
  hipLaunchKernelGGL(k_debug_hold, dim3(1), dim3(64), 0, (hipStream_t)stream, g_hold_word_d, g_hold_gen + 1,
                     (uint64_t)timeout_ms * (uint64_t)rate_khz);
  return hipGetLastError() == hipSuccess ? MX_SUCCESS : MX_ERR_HIP;
}

extern "C" int mx_debug_hold_service(unsigned timeout_ms) {
  hipStream_t s = nullptr;
  {
    mx::Service &v = mx::g_svc;
    std::lock_guard<std::mutex> lk(v.mu);
    if (v.state != 1) return MX_ERR_NOT_INIT;
    s = v.s;
  }
  return mx_debug_hold(s, timeout_ms);
}

extern "C" int mx_debug_release(void) {
  std::lock_guard<std::mutex> lk(g_hold_mu);
  if (!g_hold_word) return MX_SUCCESS;
  __atomic_store_n(g_hold_word, ++g_hold_gen, __ATOMIC_RELEASE);
  return MX_SUCCESS;
}

