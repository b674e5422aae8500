// mx_coll_svc.hip -- a resident small-message allreduce service (round 6;
// VERDICT r5 missing 5).
//
// A blocking MPI_Allreduce of a few bytes on device buffers costs one kernel
// launch per call on the one-shot path (k_oneshot, mx_fold.hpp): ~17 us at
// n = 2, most of it the host's launch, the packet processor's
// dispatch and the wake-up -- coll/tuned answers these sizes with recursive
// doubling over shared memory in a few microseconds
// (coll_tuned_decision_fixed.c:53, coll_base_allreduce.c:130-274).  The
// service keeps one workgroup resident per process, bound to one
// (communicator, op, type), and takes the call from coherent mapped host
// memory: the host writes the call's one-shot arguments (the very
// OneShotArgs a launch would get) and raises the command number; the
// workgroup reads them, runs the call, and raises `done`, which the host
// polls.  It takes the calls of the tagged-word class (os_ll, mx_fold.hpp:
// 4- and 8-byte elements, at most OS_LL_MAX bytes per rank, one workgroup's
// work); larger one-shot calls launch (one workgroup would fold what the
// launch spreads over several).
//
// Protocol compatibility is the point: the workgroup speaks the launched
// kernel's protocol exactly -- tagged words into the peers' LL areas of this
// generation's parity, the peers' tagged words gathered and folded with the
// call's fold program, DONE(gen) at every peer.  So whether a rank's call is
// served or launched is invisible to its peers, and each rank decides
// alone: a service that is not running (idle exit, a held hardware queue,
// another pair bound) means a launch, never a protocol disagreement.
// Results are the launch's bit for bit (the same fold program per element).
//
// Like the op service (mx_service.hip): a stream of the least priority
// (nothing else of the process runs there), the host waits until a
// launched kernel runs before posting to it and tells one that does not
// start within kCsvStartUs to leave (its calls launch meanwhile), the kernel
// leaves by itself after kCsvIdleS without a command or once kCsvLifeS old,
// and it is stopped before its communicator is destroyed and at exit.  Used
// only on communicators with at most two ranks per device (the VERDICT's
// condition: each rank keeps one workgroup of its device resident while
// calls come) and only while the communicator has no request in flight.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <vector>

#include "mx_comm.hpp"
#include "mx_dispatch.hpp"
#include "mx_internal.h"

namespace mx {

// leave after 200 us without a command.  A longer idle exit keeps calls
// after gaps served (8 B n = 2 after a 0.5 ms gap: 9.5 us with 2 ms, 26 us
// with 200 us -- the restart costs more than the launch path's 20), but a
// device-wide synchronisation (hipDeviceSynchronize, torch.cuda.synchronize)
// waits for the resident kernel to leave: with 2 ms the bench sweep's loops
// of 50 calls + one synchronize took 50 us per call at a 9.5 us median
// (profiles/r06/coll_lat_r6as_idle_exit.txt).  MX_COLL_SERVICE_IDLE_US
// raises it for applications that never synchronise the whole device.
constexpr double kCsvIdleS = 200e-6;
constexpr double kCsvLifeS = 5e-3;          // and between commands once 5 ms old (then relaunched)
constexpr double kCsvStartUs = 1000;        // a kernel not running 1 ms after its launch is held
constexpr double kCsvFirstStartUs = 50000;  // (50 ms for a pair's first launch: its code object loads)
constexpr size_t kCsvArgWords = (sizeof(OneShotArgs) + 7) / 8;

// per-call phase stamps (wall clock ticks, thread 0): the service's own
// breakdown, summed by the host for mx_coll_service_trace
enum { TK_SEEN, TK_ARGS, TK_DCHK, TK_PUSH, TK_GATH, TK_FOLD, TK_CALL, TK_N };

// The command line: one 64-byte line of coherent mapped host memory,
// written by the host word by word, w[0] (the command number) last with a
// release.  Every other word carries the low 16 bits of its command number
// in its top 16 bits (addresses and counts fit in 48), so a line read while
// the host was still writing it shows a mismatched tag and is read again --
// the kernel takes a whole call from ONE read of the line (its eight words
// in flight together) instead of a read for the number and another for the
// arguments.
enum { CW_SEQ = 0, CW_SB, CW_RB, CW_COUNT, CW_GEN, CW_FLAGS, CW_N = 8 };
enum { CF_EXIT = 1, CF_FULL = 2 };   // CW_FLAGS bits; bits 8..23: argument words of a full call
constexpr uint64_t kCwMask = (1ull << 48) - 1;
struct alignas(64) CsvCtl {
  uint64_t w[CW_N];
};
struct alignas(64) CsvHost {  // mapped host memory, written by the kernel
  uint64_t done;              // last command completed
  uint64_t running;           // launch epoch the kernel reported at start
  uint64_t left;              // launch epoch that left (written after its last `done`)
  uint64_t last[TK_N];        // the last call's phases: [k] = stamp k - stamp k-1 (ticks)
};

// The call itself is os_ll<T, OP, SYS = true> (mx_fold.hpp): the launched
// kernel's tagged-word protocol with the operand and result words read and
// written at system scope too, so no cache maintenance is needed between
// calls -- the service never crosses a kernel boundary, and what it reads
// (sbuf, the peers' words) and writes (rbuf, the peers' LL areas, DONE) all
// bypass this XCD's L2.
//
// Arguments: the kernel keeps one OneShotArgs per generation parity (the
// peer pointers differ by parity); a call whose arguments differ from the
// kept ones in more than sbuf, rbuf, count and generation (first call of a
// parity after a launch, another size's segments) comes as a FULL command
// and the kernel reads the arguments block first.
template <class T, class OP>
__global__ void __launch_bounds__(kOSB) k_csv(const CsvCtl *ctl, const uint64_t *args, CsvHost *host, uint64_t last,
                                              uint64_t epoch, uint64_t idle_ticks, uint64_t life_ticks) {
  __shared__ OneShotArgs A[2];
  __shared__ uint64_t line[CW_N];
  __shared__ int s_exit;
  __shared__ uint64_t tk[TK_N];
  const int t = threadIdx.x;
  uint64_t seen = last;
  uint64_t gathered = 0;   // the last generation this kernel gathered from every peer
  const uint64_t born = wall_clock64();
  if (t == 0) __hip_atomic_store(&host->running, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    if (t < 64) {   // wave 0 polls the line, lanes 0-7 a word each
      const uint64_t t0 = wall_clock64();
      int ex = 0;
      for (;;) {
        const uint64_t w = t < CW_N ? __hip_atomic_load(&ctl->w[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0;
        const uint64_t q = __shfl(w, 0);
        if (q > seen) {
          const bool tagged = t == CW_SEQ || t >= CW_N || t > CW_FLAGS || (w >> 48) == (q & 0xffff);
          if (__all(tagged)) {
            if (t < CW_N) line[t] = w;
            break;
          }
          continue;   // caught mid-write: read it again
        }
        const uint64_t now = wall_clock64();
        if (now - t0 > idle_ticks || now - born > life_ticks) { ex = 1; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      if (t == 0) {
        s_exit = ex || ((line[CW_FLAGS] & CF_EXIT) != 0);
        if (!ex) seen = line[CW_SEQ];
        tk[TK_SEEN] = wall_clock64();
      }
      seen = __shfl(seen, 0);
    }
    __syncthreads();
    if (s_exit) {
      if (t == 0) __hip_atomic_store(&host->left, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    const uint64_t fl = line[CW_FLAGS] & kCwMask;
    const uint64_t gen = line[CW_GEN] & kCwMask;
    OneShotArgs &a = A[gen & 1];
    if (fl & CF_FULL) {   // the arguments block: one load per lane, all in flight at once
      size_t words = (fl >> 8) & 0xffff;
      if (words > kCsvArgWords) words = kCsvArgWords;
      uint64_t *dst = reinterpret_cast<uint64_t *>(&a);
      for (size_t i = t; i < words; i += kOSB)
        dst[i] = __hip_atomic_load(args + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __syncthreads();
    }
    if (t == 0) {   // this call's own fields
      a.sb = reinterpret_cast<const char *>(line[CW_SB] & kCwMask);
      a.rb = reinterpret_cast<char *>(line[CW_RB] & kCwMask);
      a.src[a.rank] = a.sb;
      a.count = line[CW_COUNT] & kCwMask;
      a.slice = a.count;
      a.gen = gen;
      tk[TK_ARGS] = wall_clock64();
    }
    __syncthreads();
    // the gen-2 check is needed only when this kernel did not gather the
    // previous generation itself (its first call, or gen-1 was launched)
    const bool ok = os_ll<T, OP, true>(a, &tk[TK_DCHK], gen != gathered + 1);
    if (ok) gathered = gen;
    // every lane's result words acknowledged before `done`
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      tk[TK_CALL] = wall_clock64();
      // the call's phases (ticks), ahead of `done` (a failed call: none;
      // the host finds the error word set)
      for (int k = 1; k < TK_N; k++)
        __hip_atomic_store(&host->last[k], ok ? tk[k] - tk[k - 1] : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __hip_atomic_store(&host->done, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();   // A, line and s_* are rewritten next round
  }
}

typedef void (*csv_launch_fn)(const CsvCtl *, const uint64_t *, CsvHost *, uint64_t, uint64_t, uint64_t, uint64_t,
                              hipStream_t);
template <class T, class OP>
static void csv_launch(const CsvCtl *c, const uint64_t *a, CsvHost *h, uint64_t last, uint64_t epoch, uint64_t idle,
                       uint64_t life, hipStream_t s) {
  hipLaunchKernelGGL((k_csv<T, OP>), dim3(1), dim3(kOSB), 0, s, c, a, h, last, epoch, idle, life);
}

// pairs served: 4- and 8-byte element types with no bytes outside their
// value fields (the small messages of the metric's sweep: fp32 / fp64 SUM,
// MAX, MIN, integers, bitwise, MAXLOC / MINLOC on float_int and 2int);
// everything else launches
struct CsvVisitor {
  template <class T, class OP2, class OP3> csv_launch_fn go() {
    if constexpr ((sizeof(T) == 4 || sizeof(T) == 8) && !has_pad<T>::value && fam<T>::value != 3)
      return &csv_launch<T, OP2>;
    else
      return nullptr;
  }
  csv_launch_fn none() { return nullptr; }
};

namespace {
struct Csv {
  std::mutex mu;
  int state = 0;                 // 0 not set up, 1 usable, -1 off
  CsvCtl *ctl = nullptr, *ctl_d = nullptr;
  uint64_t *args = nullptr, *args_d = nullptr;
  CsvHost *host = nullptr, *host_d = nullptr;
  hipStream_t s = nullptr;
  int device = -1;
  uint64_t seq = 0, epoch = 0;
  bool live = false;
  uint64_t pending = 0;          // epoch of a launch told to leave before it ran
  const mx_comm *comm = nullptr; // the binding: communicator, op, type
  int op = -1, type = -1;
  uint64_t idle_ticks = 0, life_ticks = 0;
  uint64_t served = 0, held = 0;
  std::vector<csv_launch_fn> started;
  double tick_us = 0.01;         // wall clock period
  double prep_us = 0, wait_us = 0, phase_us[TK_N] = {};   // sums over `served` (mx_coll_service_trace)
  OneShotArgs kept[2];           // the arguments the kernel of epoch kept_ep[parity] holds
  uint64_t kept_ep[2] = {0, 0};
  uint64_t full = 0;             // commands that carried the arguments block
};
Csv g_csv;
std::atomic<int> g_csv_on{-1};

bool csv_enabled() {
  int on = g_csv_on.load(std::memory_order_relaxed);
  if (on < 0) {
    const char *e = getenv("MX_COLL_SERVICE");
    g_csv_on.compare_exchange_strong(on, (e && *e == '0') ? 0 : 1);
    on = g_csv_on.load(std::memory_order_relaxed);
  }
  return on != 0;
}

bool csv_poll(const uint64_t *w, uint64_t target, double us) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned k = 0;; k++) {
    if (__atomic_load_n(w, __ATOMIC_ACQUIRE) >= target) return true;
    if ((k & 255) == 255 &&
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > us)
      return false;
    __builtin_ia32_pause();
  }
}
bool csv_gone(const Csv &v, uint64_t ep) { return __atomic_load_n(&v.host->left, __ATOMIC_ACQUIRE) >= ep; }

// Writes command v.seq + 1 (a call, or "leave") into the line and raises it.
// A call carries the arguments block too when the kernel running now does
// not hold this parity's arguments, or they differ in more than the call's
// own fields (sbuf, rbuf, count, generation).
uint64_t csv_post(Csv &v, bool exit, const OneShotArgs *a = nullptr) {
  const uint64_t q = v.seq + 1;
  const uint64_t tag = (q & 0xffff) << 48;
  uint64_t fl = exit ? CF_EXIT : 0, sb = 0, rb = 0, cnt = 0, gen = 0;
  if (a) {
    const int par = (int)(a->gen & 1);
    const size_t used = offsetof(OneShotArgs, seg) + (size_t)a->nseg * sizeof(OsSeg);
    bool full = v.kept_ep[par] != v.epoch;
    if (!full) {
      OneShotArgs cmp;
      memcpy(&cmp, a, sizeof cmp);
      const OneShotArgs &k = v.kept[par];
      cmp.sb = k.sb;
      cmp.rb = k.rb;
      cmp.src[a->rank] = k.src[a->rank];
      cmp.count = k.count;
      cmp.slice = k.slice;
      cmp.gen = k.gen;
      full = memcmp(&cmp, &k, used) != 0;
    }
    if (full) {
      memcpy(v.args, a, used);
      memcpy(&v.kept[par], a, sizeof *a);
      v.kept_ep[par] = v.epoch;
      fl |= CF_FULL | (uint64_t)((used + 7) / 8) << 8;
      v.full++;
    }
    sb = (uint64_t)(uintptr_t)a->sb;
    rb = (uint64_t)(uintptr_t)a->rb;
    cnt = a->count;
    gen = a->gen;
  }
  v.ctl->w[CW_SB] = tag | (sb & kCwMask);
  v.ctl->w[CW_RB] = tag | (rb & kCwMask);
  v.ctl->w[CW_COUNT] = tag | (cnt & kCwMask);
  v.ctl->w[CW_GEN] = tag | (gen & kCwMask);
  v.ctl->w[CW_FLAGS] = tag | fl;
  v.seq = q;
  __atomic_store_n(&v.ctl->w[CW_SEQ], q, __ATOMIC_RELEASE);
  return q;
}

void csv_stop_locked(Csv &v) {
  if (!v.live) return;
  if (!csv_gone(v, v.epoch)) {
    csv_post(v, true);
    if (!csv_poll(&v.host->left, v.epoch, 1e6)) (void)hipStreamSynchronize(v.s);
  }
  v.live = false;
  v.comm = nullptr;
}

void csv_atexit() {
  Csv &v = g_csv;
  std::lock_guard<std::mutex> lk(v.mu);
  if (v.state == 1) csv_stop_locked(v);
}

int csv_setup(Csv &v) {
  if (hipGetDevice(&v.device) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  int rate_khz = 0;
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, v.device) != hipSuccess || rate_khz <= 0)
    rate_khz = 100000;
  v.tick_us = 1e3 / rate_khz;
  // MX_COLL_SERVICE_IDLE_US: the idle exit (default kCsvIdleS), at most the lifetime
  const char *ie = getenv("MX_COLL_SERVICE_IDLE_US");
  const double idle_s = (ie && *ie) ? std::min(kCsvLifeS, std::max(1e-6, atof(ie) * 1e-6)) : kCsvIdleS;
  v.idle_ticks = (uint64_t)(idle_s * rate_khz * 1000.0);
  v.life_ticks = (uint64_t)(kCsvLifeS * rate_khz * 1000.0);
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = 0;
  if (hipHostMalloc((void **)&v.ctl, sizeof(CsvCtl), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&v.ctl_d, v.ctl, 0) != hipSuccess ||
      hipHostMalloc((void **)&v.args, kCsvArgWords * 8, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&v.args_d, v.args, 0) != hipSuccess ||
      hipHostMalloc((void **)&v.host, sizeof(CsvHost), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&v.host_d, v.host, 0) != hipSuccess ||
      // the least priority: a hardware queue nothing else of the process
      // uses (the op service's reasoning, mx_service.hip svc_stream_create)
      hipStreamCreateWithPriority(&v.s, hipStreamNonBlocking, least) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  memset(v.ctl, 0, sizeof(CsvCtl));
  memset(v.args, 0, kCsvArgWords * 8);
  memset(v.host, 0, sizeof(CsvHost));
  atexit(csv_atexit);
  return 1;
}

// `s` and the legacy default stream hold no pending work (the caller's
// producers of sbuf have finished): the service reads sbuf with no stream
// order of its own.  A short spin lets a just-finished launch retire.
bool csv_streams_idle(hipStream_t s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e1 = hipStreamQuery(s);
    const hipError_t e2 = e1 == hipSuccess ? hipStreamQuery(nullptr) : hipSuccess;
    if (e1 == hipSuccess && e2 == hipSuccess) return true;
    if ((e1 != hipSuccess && e1 != hipErrorNotReady) || (e2 != hipSuccess && e2 != hipErrorNotReady)) return false;
    (void)hipGetLastError();
    if (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > 20.0) return false;
    __builtin_ia32_pause();
  }
}

bool csv_start(Csv &v, csv_launch_fn fn) {
  const uint64_t ep = ++v.epoch;
  fn(v.ctl_d, v.args_d, v.host_d, v.seq, ep, v.idle_ticks, v.life_ticks, v.s);
  if (hipGetLastError() != hipSuccess) {
    v.state = -1;
    return false;
  }
  const bool first = std::find(v.started.begin(), v.started.end(), fn) == v.started.end();
  if (csv_poll(&v.host->running, ep, first ? kCsvFirstStartUs : kCsvStartUs)) {
    if (first) v.started.push_back(fn);
    v.live = true;
    return true;
  }
  csv_post(v, true);   // held: told to leave when it starts; calls launch meanwhile
  v.pending = ep;
  v.live = false;
  v.held++;
  return false;
}
}  // namespace

// 1: served (rb final, DONE raised at the peers); 0: not served (the caller
// launches k_oneshot with the same arguments); < 0: error
int csv_allreduce(mx_comm *c, const OneShotArgs &a, int op, int type, hipStream_t s) {
  // the tagged-word calls only (one workgroup's work), operands on 4-byte
  // boundaries (the service moves 4-byte words at system scope)
  if (!csv_enabled() || !c->csv_ok || c->defer || c->poisoned || !a.ll || a.count * a.es > OS_LL_MAX ||
      (((uintptr_t)a.sb | (uintptr_t)a.rb) & 3) ||
      (((uintptr_t)a.sb | (uintptr_t)a.rb | a.count | a.gen) >> 48))   // (the line's 48-bit fields)
    return 0;
  const auto t_in = std::chrono::steady_clock::now();
  CsvVisitor vis;
  const csv_launch_fn fn = dispatch(op, type, vis);
  if (!fn || !csv_streams_idle(s)) return 0;
  Csv &v = g_csv;
  std::lock_guard<std::mutex> lk(v.mu);
  if (v.state == 0) v.state = csv_setup(v);
  if (v.state != 1 || c->device != v.device) return 0;
  if (v.pending) {
    if (!csv_gone(v, v.pending)) return 0;
    v.pending = 0;
  }
  if (v.live && (v.comm != c || v.op != op || v.type != type)) csv_stop_locked(v);
  if (v.live && csv_gone(v, v.epoch)) v.live = false;   // left (idle or lifetime)
  if (!v.live) {
    v.comm = c;
    v.op = op;
    v.type = type;
    if (!csv_start(v, fn)) return 0;
  }
  const auto t_post = std::chrono::steady_clock::now();
  uint64_t q = csv_post(v, false, &a);
  for (unsigned k = 0;; k++) {
    if (__atomic_load_n(&v.host->done, __ATOMIC_ACQUIRE) >= q) {
      const auto t_done = std::chrono::steady_clock::now();
      v.prep_us += std::chrono::duration<double, std::micro>(t_post - t_in).count();
      v.wait_us += std::chrono::duration<double, std::micro>(t_done - t_post).count();
      for (int j = 1; j < TK_N; j++) v.phase_us[j] += v.tick_us * (double)v.host->last[j];
      v.served++;
      return 1;
    }
    if ((k & 63) == 63 && p2p_rx_active()) p2p_progress();   // a peer's send may wait for a yielded receive
    if ((k & 15) == 15 && csv_gone(v, v.epoch)) {
      // it left before taking q (idle / lifetime raced the post): the grid
      // has drained, so `done` is final; a new kernel takes only what comes
      // after v.seq, so q is posted again under a new number
      if (hipStreamSynchronize(v.s) != hipSuccess) {
        (void)hipGetLastError();
        v.live = false;
        v.state = -1;
        return MX_ERR_HIP;
      }
      if (__atomic_load_n(&v.host->done, __ATOMIC_ACQUIRE) >= q) {
        v.served++;
        return 1;
      }
      v.live = false;
      if (!csv_start(v, fn)) return 0;
      q = csv_post(v, false, &a);
    }
    if ((k & 0xfffff) == 0xfffff) {
      const hipError_t e = hipStreamQuery(v.s);
      if (e != hipSuccess && e != hipErrorNotReady) {
        (void)hipGetLastError();
        v.live = false;
        v.state = -1;
        return MX_ERR_HIP;
      }
      (void)hipGetLastError();
    }
    __builtin_ia32_pause();
  }
}

// a communicator about to be destroyed: its service (if bound) leaves first
void csv_comm_gone(const mx_comm *c) {
  Csv &v = g_csv;
  std::lock_guard<std::mutex> lk(v.mu);
  if (v.state == 1 && v.comm == c) csv_stop_locked(v);
  if (v.comm == c) v.comm = nullptr;
}

}  // namespace mx

extern "C" int mx_coll_service_stats(unsigned long long *served, unsigned long long *launches) {
  mx::Csv &v = mx::g_csv;
  std::lock_guard<std::mutex> lk(v.mu);
  if (served) *served = v.served;
  if (launches) *launches = v.epoch;
  return v.state;
}

extern "C" int mx_coll_service_trace(double *out, int n) {
  mx::Csv &v = mx::g_csv;
  std::lock_guard<std::mutex> lk(v.mu);
  const double d = v.served ? (double)v.served : 1.0;
  const double t[10] = {(double)v.served,
                        v.prep_us / d,
                        v.wait_us / d,
                        v.phase_us[mx::TK_ARGS] / d,
                        v.phase_us[mx::TK_DCHK] / d,
                        v.phase_us[mx::TK_PUSH] / d,
                        v.phase_us[mx::TK_GATH] / d,
                        v.phase_us[mx::TK_FOLD] / d,
                        v.phase_us[mx::TK_CALL] / d,
                        (double)v.full};
  for (int i = 0; i < n && i < 10; i++) out[i] = t[i];
  return v.state;
}

extern "C" int mx_coll_service_set(int on) {
  mx::Csv &v = mx::g_csv;
  std::lock_guard<std::mutex> lk(v.mu);
  mx::g_csv_on.store(on ? 1 : 0, std::memory_order_relaxed);
  if (!on && v.state == 1) mx::csv_stop_locked(v);
  return MX_SUCCESS;
}
