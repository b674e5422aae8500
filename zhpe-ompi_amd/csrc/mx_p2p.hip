// mx_p2p.hip -- point-to-point transfers of device buffers between the
// ranks of a communicator.
//
// The reference moves intra-node CUDA buffers with btl/smcuda: the sender's
// buffer is registered and its IPC handle sent in the rendezvous, the
// receiver opens it and issues cuMemcpy from the peer buffer, completion by
// CUDA events polled from opal_progress (mca_common_cuda_memcpy,
// opal/mca/common/cuda/common_cuda.c:1008-1180); non-contiguous layouts go
// through the convertor's CUDA hooks, one copy per block
// (opal_datatype_cuda.c:44-140).
//
// MI355X design: no per-message IPC export (an export costs far more than a
// copy, and late exports are the operation this image has been seen to get
// wrong, see mx_coll.hip).  Instead every rank owns, next to its collective
// staging, one mailbox per source rank, mapped by every peer at
// communicator creation.  A message is a device-driven stream through that
// mailbox: the send kernel (one workgroup per lane) writes the envelope
// (bytes, tag) into the mailbox's header ring and each lane streams its
// stripe of the payload in P2P_C chunks through P2P_S slots, directly into
// the receiver's memory over xGMI; the receive kernel copies the chunks out
// as they land and hands the slots back.  Flow control is cumulative
// counters in the ranks' uncached flag arrays (system-scope atomics), so a
// message of any size streams with no host involvement, and with P2P_L
// lanes in flight per pair.  Sends and receives run on two internal
// streams, after the work the caller's stream had queued, so a send never
// waits behind a receive of its own process.
//
// Matching: messages of one (source, destination) pair match in order --
// the i-th receive from a source gets the i-th send to it (the envelope's
// tag is checked: a mismatch completes the receive with MX_ERR_TAG, tag < 0
// is MPI_ANY_TAG).  A receive from MX_ANY_SOURCE is preceded on the receive
// stream by a one-thread pick kernel that waits until some source has a
// posted envelope this process has not consumed yet (scanning from a
// rotating start, so no source starves) and records it in the request's
// status; the receive kernel then takes its mailbox and flags from that
// slot.  Receives run in issue order on one stream, so an ANY_SOURCE
// receive consumes exactly one message and later receives -- specific or
// not -- see the channel advanced (MPI only orders messages per pair); a
// receive still waiting when one queued behind it could progress yields
// and is launched again by the host's wait (round 5, rx_control /
// p2p_progress).  A message longer than the receive buffer delivers what
// fits and completes with MX_ERR_TRUNCATE (MPI_ERR_TRUNCATE); the status
// holds the delivered byte count.  Non-contiguous layouts are packed /
// unpacked by the device convertor (mx_convertor.h) around the stream.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <thread>

#include "mx_comm.hpp"
#include "../../include/mx_convertor.h"

namespace mx {

constexpr int kP2PThreads = 256;

// Memory ordering of the channel: a counter moves with a relaxed
// system-scope store after the data it covers was fenced (one system fence
// per chunk or envelope), and a wait spins with relaxed loads and takes one
// acquire fence when it succeeds.  Release / acquire atomics in the loops
// themselves cost an L2 write-back / invalidate per access on gfx950.
__device__ __forceinline__ bool p2p_wait_ge(const uint64_t *f, uint64_t v, uint64_t t0, uint64_t tmo, int *err) {
  while (__hip_atomic_load(gp(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < v) {
    __builtin_amdgcn_s_sleep(2);
    if (wall_clock64() - t0 > tmo) {
      __hip_atomic_store(err, MX_ERR_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  return true;
}

// len bytes: 16-byte vectors when both ends are aligned, 4-byte words when
// they are word aligned, bytes otherwise
__device__ __forceinline__ void p2p_copy(char *dst, const char *src, uint64_t len) {
  const int t = threadIdx.x;
  if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
    const uint64_t nv = len / 16;
    for (uint64_t i = t; i < nv; i += kP2PThreads)   // (global accesses, mx_mem.hpp gp)
      gp(reinterpret_cast<u32x4 *>(dst))[i] = gp(reinterpret_cast<const u32x4 *>(src))[i];
    for (uint64_t i = nv * 16 + t; i < len; i += kP2PThreads) dst[i] = src[i];
  } else if ((((uintptr_t)dst | (uintptr_t)src) & 3) == 0) {
    const uint64_t nw = len / 4;
    for (uint64_t i = t; i < nw; i += kP2PThreads)
      reinterpret_cast<uint32_t *>(dst)[i] = reinterpret_cast<const uint32_t *>(src)[i];
    for (uint64_t i = nw * 4 + t; i < len; i += kP2PThreads) dst[i] = src[i];
  } else {
    for (uint64_t i = t; i < len; i += kP2PThreads) dst[i] = src[i];
  }
}

// stripe of lane l among the nl lanes from `first` (eager: [0, P2P_LE), at
// most 32 KiB each; rendezvous: [P2P_LE, P2P_L)): 16-byte multiples of at least kMinStripe,
// the last lanes short or empty -- a small message moves in one or a few
// lanes (each lane with data pays a drained / filled handshake per chunk;
// 4 KiB spread over all 64 lanes cost 9 us more per hop than 8 B in one)
constexpr uint64_t kMinStripe = 16 << 10;
__device__ __forceinline__ void p2p_lane(uint64_t bytes, int l, int first, int nl, uint64_t *lo, uint64_t *hi) {
  const int j = l - first;
  if (j < 0 || j >= nl) {
    *lo = *hi = 0;
    return;
  }
  uint64_t stripe = ((bytes + nl - 1) / nl + 15) & ~(uint64_t)15;
  if (stripe < kMinStripe) stripe = kMinStripe;
  *lo = std::min<uint64_t>(bytes, (uint64_t)j * stripe);
  *hi = std::min<uint64_t>(bytes, *lo + stripe);
}
constexpr int P2P_LR = P2P_L - P2P_LE;   // rendezvous lanes

// Host-visible completion of a transfer kernel: every lane workgroup counts
// itself out on a device counter (kernels of one internal stream run one
// after another, so the counter reaches `target` exactly when this kernel's
// last lane is done, whatever path the lanes took), and that last lane
// raises `done` in the request's mapped status block.  mx_wait polls the
// word in host memory instead of querying a HIP event, which wakes tens of
// microseconds late.
struct P2PDone {
  uint64_t *lanes;       // device counter of finished lanes (per stream)
  uint64_t target;
  int64_t *done;         // mapped host word, or null
  uint64_t *hfin;        // mapped host word: `target` of the communicator's last finished kernel on this
                         // channel (what its destroy and quiet check wait for; no event per kernel)
  uint64_t *exits;       // receive launches with a control workgroup: device count of the launch's
  uint64_t xtarget;      // two exits (last lane, control); whichever makes it xtarget raises hfin
};

// the last lane's or the control workgroup's exit from a receive launch:
// hfin is raised once both have left, so a communicator seen idle has no
// workgroup of its own still reading its channel state (thread 0 only)
__device__ __forceinline__ void rx_exit(const P2PDone &f) {
  if (!f.hfin) return;
  if (f.exits) {
    const uint64_t old = __hip_atomic_fetch_add(f.exits, (uint64_t)1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 != f.xtarget) return;
  }
  __hip_atomic_store(f.hfin, f.target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// `wrote`: this lane stored user data without a fence after it (a receive
// lane with data): make it visible device-wide before counting out -- work
// the host launches once `done` is seen may run on any XCD.  Send lanes
// fenced every chunk already; lanes without data have nothing to publish.
// Returns whether this was the kernel's last lane.
__device__ __forceinline__ bool lane_finished(const P2PDone &f, bool wrote) {
  __syncthreads();
  bool last = false;
  if (threadIdx.x == 0) {
    if (wrote) __threadfence();
    const uint64_t old = __hip_atomic_fetch_add(f.lanes, (uint64_t)1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = old + 1 == f.target;
    if (last && f.done) __hip_atomic_store(f.done, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (last && f.hfin) __hip_atomic_store(f.hfin, f.target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return last;
}

// Push [lo, hi) of `src` through lane l's chunk slots of mailbox `box`.
__device__ __forceinline__ bool send_stream(int l, uint64_t lo, uint64_t hi, const char *src, char *box,
                                            uint64_t *filled, const uint64_t *drained, P2PSendState *st,
                                            uint64_t t0, uint64_t tmo, int *err) {
  __shared__ int ok;
  uint64_t k = st->lane_chunks[l];   // this lane's counter: read and written by this workgroup only
  for (uint64_t pos = lo; pos < hi; pos += P2P_C) {
    const uint64_t len = std::min<uint64_t>(P2P_C, hi - pos);
    k++;
    if (threadIdx.x == 0) ok = p2p_wait_ge(drained + l, k > P2P_S ? k - P2P_S : 0, t0, tmo, err);
    __syncthreads();
    if (!ok) return false;
    char *slot = box + 4096 + ((size_t)l * P2P_S + (size_t)((k - 1) % P2P_S)) * P2P_C;
    p2p_copy(slot, src + pos, len);
    __threadfence_system();   // my stores reach the peer before the counter moves
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(filled + l, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x == 0) st->lane_chunks[l] = k;
  return true;
}

struct P2PSendArgs {
  const char *buf;
  uint64_t bytes;
  int64_t tag;
  int rndv;                  // rendezvous: the envelope only (the data follows its CTS)
  int has_desc;              // rendezvous with a descriptor of `buf` (the receiver may pull it)
  P2PRgetDesc desc;
  char *box;                 // the receiver's mailbox for me
  uint64_t *posted;          // receiver's flags: posted[me]
  uint64_t *filled;          // receiver's flags: filled[me][lane]
  const uint64_t *seen;      // my flags: seen[dst][lane]
  const uint64_t *drained;   // my flags: drained[dst][lane]
  P2PSendState *st;
  uint64_t timeout_ticks;
  int *err;
  P2PDone fin;
};

// one workgroup per eager lane; lane 0 also writes the envelope
__global__ void __launch_bounds__(kP2PThreads) k_p2p_send(P2PSendArgs a) {
  const int l = blockIdx.x;
  const uint64_t t0 = wall_clock64();
  __shared__ int s_seen_bad;
  if (l == 0) {
    // envelope: the header slot is free once every lane of the receiver has
    // read the envelope P2P_H messages back -- one thread per lane counter
    // (a serial scan of 64 uncached words by one thread cost most of a
    // small message's latency)
    const uint64_t m = a.st->msgs;
    if (threadIdx.x == 0) s_seen_bad = 0;
    __syncthreads();
    if (threadIdx.x < P2P_L &&
        !p2p_wait_ge(a.seen + threadIdx.x, m + 1 > P2P_H ? m + 1 - P2P_H : 0, t0, a.timeout_ticks, a.err))
      s_seen_bad = 1;
    __syncthreads();
    if (threadIdx.x == 0 && !s_seen_bad) {
      volatile uint64_t *h = reinterpret_cast<volatile uint64_t *>(a.box + (m % P2P_H) * P2P_HDR);
      if (a.has_desc) {   // the descriptor slot of this envelope, before the envelope is posted
        volatile uint64_t *dd = reinterpret_cast<volatile uint64_t *>(a.box + P2P_DESC_OFF + (m % P2P_H) * P2P_DESC);
        const uint64_t *src = reinterpret_cast<const uint64_t *>(&a.desc);
        for (int w = 0; w < (int)(sizeof(P2PRgetDesc) / 8); w++) dd[w] = src[w];
      }
      h[0] = a.bytes;
      h[1] = (uint64_t)a.tag;
      h[2] = (uint64_t)a.rndv | (a.has_desc ? 2u : 0u);
      __threadfence_system();
      __hip_atomic_store(a.posted, m + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      a.st->msgs = m + 1;
    }
  }
  if (!a.rndv) {
    uint64_t lo, hi;
    p2p_lane(a.bytes, l, 0, P2P_LE, &lo, &hi);
    send_stream(l, lo, hi, a.buf, a.box, a.filled, a.drained, a.st, t0, a.timeout_ticks, a.err);
  }
  lane_finished(a.fin, false);
}

// ---- rendezvous sends ------------------------------------------------------
// Each rendezvous send enqueues one rendezvous kernel on the rendezvous
// stream.  Its workgroup 0 waits until some destination has cleared a
// message of this process (its CTS ticket moved past what was served) and
// publishes that message; every workgroup then streams its lane's stripe of
// it -- whichever message it is: receivers clear messages in their own
// matching order and the kernels are interchangeable, so no message waits
// behind another.  (Workgroup 0 is dispatched first, so the waiting
// workgroups never hold back the one they wait for.)
struct P2PRndvArgs {
  P2PRndvCur *cur;
  uint64_t gen;              // this kernel's publication number
  const uint64_t *cts0;      // my flags: cts[0][0] (the ring of destination d at + d * P2P_RNDV_Q)
  int n;
  const P2PRndvTable *tab;   // device address of the mapped table
  char *box[MAXR];           // box[d]: d's mailbox for me
  uint64_t *filled[MAXR];    // filled[d]: d's flags, filled[me][lane]
  const uint64_t *drained0;  // my flags: drained[0][lane]
  P2PSendState *st0;
  uint64_t timeout_ticks;
  int *err;
  P2PDone fin;
};

__device__ __forceinline__ void rndv_pick(const P2PRndvArgs &a) {
  __shared__ int s_dst, s_hit, s_fin;
  __shared__ uint64_t s_seq;
  const uint64_t t0 = wall_clock64();
  if (threadIdx.x == 0) {
    s_dst = -1;
    for (;;) {
      for (int d = 0; d < a.n && s_dst < 0; d++) {
        // d's next ring entry, taken once its stamp is the entry's index + 1
        const uint64_t k = a.st0[d].cts_served;
        const uint64_t w =
            __hip_atomic_load(a.cts0 + (size_t)d * P2P_RNDV_Q + k % P2P_RNDV_Q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((w >> 40) == ((k + 1) & 0xffffffull)) {
          __atomic_thread_fence(__ATOMIC_ACQUIRE);
          s_seq = w & ((1ull << 39) - 1);
          s_fin = (int)((w >> 39) & 1);
          a.st0[d].cts_served = k + 1;
          s_dst = d;
        }
      }
      if (s_dst >= 0) break;
      if (__hip_atomic_load(&a.tab->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
        s_dst = -2;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > a.timeout_ticks) {
        __hip_atomic_store(a.err, MX_ERR_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s_dst = -3;
        break;
      }
    }
    s_hit = -1;
  }
  __syncthreads();
  const int d = s_dst;
  if (d == -3) {   // timed out: release every pending send (they complete with the error)
    for (int i = threadIdx.x; i < P2P_RNDV_Q; i += blockDim.x)
      if (a.tab->e[i].valid)
        __hip_atomic_store(a.tab->e[i].done, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (d >= 0) {    // the table is in host memory: scan it with every thread
    for (int i = threadIdx.x; i < P2P_RNDV_Q; i += blockDim.x) {
      const P2PRndvEntry &e = a.tab->e[i];
      if (e.valid && e.dst == d && e.seq == s_seq) s_hit = i;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    P2PRndvCur &c = *a.cur;
    c.ok = 0;
    if (d >= 0 && s_hit >= 0) {
      const P2PRndvEntry &e = a.tab->e[s_hit];
      c.buf = e.buf;
      c.bytes = e.bytes;
      c.done = e.done;
      c.dst = d;
      c.ok = s_fin ? 2 : 1;   // 2: the receiver pulled the data (FIN): nothing to stream
    } else if (d >= 0) {   // a CTS for no pending send: the channel is corrupt
      __hip_atomic_store(a.err, MX_ERR_STATE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __threadfence();
    __hip_atomic_store(&c.gen, a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();   // the rest of this workgroup reads the pick too
  // aborted (communicator teardown) or a CTS for no pending send: release
  // every pending send as the timeout does, so no waiter sleeps forever on
  // a status word nobody will raise (their requests complete with err)
  if (d == -2 || (d >= 0 && s_hit < 0)) {
    for (int i = threadIdx.x; i < P2P_RNDV_Q; i += blockDim.x)
      if (a.tab->e[i].valid)
        __hip_atomic_store(a.tab->e[i].done, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// one workgroup per rendezvous lane (workgroup 0 also picks); the last lane
// out raises the send request's status word
__global__ void __launch_bounds__(kP2PThreads) k_p2p_rndv(P2PRndvArgs a) {
  const int l = P2P_LE + blockIdx.x;
  if (blockIdx.x == 0) {
    rndv_pick(a);
  } else {
    if (threadIdx.x == 0) {
      while (__hip_atomic_load(&a.cur->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.gen)
        __builtin_amdgcn_s_sleep(4);
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
    }
    __syncthreads();
  }
  const P2PRndvCur c = *a.cur;   // after the acquire fence (or written by this workgroup)
  if (c.ok == 1) {
    uint64_t lo, hi;
    p2p_lane(c.bytes, l, P2P_LE, P2P_LR, &lo, &hi);
    send_stream(l, lo, hi, c.buf, a.box[c.dst], a.filled[c.dst], a.drained0 + (size_t)c.dst * P2P_L,
                a.st0 + c.dst, wall_clock64(), a.timeout_ticks, a.err);
  }
  if (lane_finished(a.fin, false) && c.ok)
    __hip_atomic_store(c.done, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- receives --------------------------------------------------------------
struct P2PRecvArgs {
  char *buf;
  uint64_t cap;
  int64_t tag;               // < 0: any
  int64_t *status;           // mapped host: delivered bytes, tag, error, source
  uint64_t timeout_ticks;
  int *err;
  // the source's mailbox, flags and state, from these per-source bases; with
  // `any` (MX_ANY_SOURCE) the source is the one the pick kernel stored in
  // status[3]
  int src, any, me;
  const char *box0;          // my mailbox for source 0 (source p at + p * P2P_BOX)
  const uint64_t *flag0;     // my flag array
  uint64_t *peer_flags[MAXR];
  P2PRecvState *st0;
  char *stash0;              // stash payloads of source 0 (source p at + p * N * C)
  P2PDone fin;
  int rget_ok;               // a rendezvous envelope with a descriptor is left for the host to pull
  // yielding (round 5): this launch's number and the receive's
  // post number, the device's launch queue (mapped; null: never yield) and
  // decision ring, and this communicator's displaced receives
  uint64_t launch, post;
  const P2PRxQueue *rq;
  uint64_t *dec;
  P2PDisplaced *disp;
};

// A message of source p with `tag` is reserved when a displaced receive of
// the communicator posted before `post` matches it: that receive gets it
// when it runs again.  (The displaced set changes only at a receive
// kernel's end, so every lane of a kernel sees the same one.)
__device__ __forceinline__ bool reserved(const P2PDisplaced *d, uint64_t post, int p, int64_t tag) {
  if (!d) return false;
  const uint64_t n = d->n;
  for (uint64_t i = 0; i < n && i < P2P_DISP_N; i++) {
    const P2PDispEntry &e = d->d[i];
    if (e.post < post && (e.src < 0 || e.src == p) && (e.tag < 0 || e.tag == tag)) return true;
  }
  return false;
}

// oldest message set aside in `st` (source p; stashed eager payload or
// deferred rendezvous envelope) that a receive with `tag` (< 0: any) posted
// as `post` matches and no earlier displaced receive does: {kind 0 stash /
// 1 defer, slot}, or {-1, -1}
__device__ __forceinline__ int2 held_match(const P2PRecvState *st, int64_t tag, const P2PDisplaced *disp = nullptr,
                                           uint64_t post = 0, int p = 0) {
  int2 hit{-1, -1};
  if (!st->held) return hit;
  uint64_t best = ~(uint64_t)0;
  for (int k = 0; k < P2P_STASH_N; k++) {
    const P2PStashEntry &e = st->stash[k];
    if (e.valid && (tag < 0 || e.tag == tag) && e.seq < best && !reserved(disp, post, p, e.tag)) {
      best = e.seq;
      hit = int2{0, k};
    }
  }
  for (int k = 0; k < P2P_DEFER_N; k++) {
    const P2PStashEntry &e = st->defer[k];
    if (e.valid && (tag < 0 || e.tag == tag) && e.seq < best && !reserved(disp, post, p, e.tag)) {
      best = e.seq;
      hit = int2{1, k};
    }
  }
  return hit;
}

// Could a receive launched behind launch `me` take a message now?  For each
// queued launch (the device's launch queue, up to P2P_Q of them): a held
// message of one of its sources that it matches (and no earlier displaced
// receive reserves), or an envelope it matches that its source posted and
// no finished kernel consumed.  The running receive's own source p of its
// communicator is judged by what the running launch set aside (`aside`, the
// tags of the envelopes it took and did not keep), since its lanes consume
// that source's envelopes themselves.  One thread; reads mapped host memory
// (the queue) and, after an acquire, envelope headers.
__device__ bool rx_queued_can_progress(const P2PRxQueue *rq, uint64_t me, const P2PRecvState *my_st0, int my_p,
                                       const int64_t *aside, int naside) {
  const uint64_t enq = __hip_atomic_load(&rq->enq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  bool fenced = false;
  for (uint64_t L = me + 1; L <= enq && L <= me + P2P_Q; L++) {
    const P2PQEntry *e = &rq->e[L % P2P_Q];
    if (__hip_atomic_load(&e->launch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != L) continue;
    if (!fenced) {
      __atomic_thread_fence(__ATOMIC_ACQUIRE);   // the entries' fields, the envelopes
      fenced = true;
    }
    const int n = e->n, src = e->src;
    const int64_t tag = e->tag;
    for (int q = src < 0 ? 0 : src; q < (src < 0 ? n : src + 1); q++) {
      const P2PRecvState *s = e->st0 + q;
      const bool own = my_p >= 0 && s == my_st0 + my_p;
      if (own) {
        for (int i = 0; i < naside; i++)
          if ((tag < 0 || aside[i] == tag) && !reserved(e->disp, e->post, q, aside[i])) return true;
      }
      if (held_match(s, tag, e->disp, e->post, q).x >= 0) return true;
      if (own) continue;
      const uint64_t done = s->msgs_done;
      const uint64_t posted = __hip_atomic_load(e->flag0 + P2P_POSTED + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (posted <= done) continue;
      if (tag < 0) return true;
      __atomic_thread_fence(__ATOMIC_ACQUIRE);   // the envelopes before their `posted` count
      const char *box = e->box0 + (size_t)q * P2P_BOX;
      for (uint64_t m = done; m < posted && m < done + P2P_H; m++)
        if ((int64_t)reinterpret_cast<const volatile uint64_t *>(box + (m % P2P_H) * P2P_HDR)[1] == tag) return true;
    }
  }
  return false;
}

// may a receive posted as `post` yield (the displaced set has room for it,
// or holds it already from an earlier launch)?
__device__ __forceinline__ bool disp_room(const P2PDisplaced *d, uint64_t post) {
  if (!d) return false;
  const uint64_t n = d->n;
  for (uint64_t i = 0; i < n && i < P2P_DISP_N; i++)
    if (d->d[i].post == post) return true;
  return n < P2P_DISP_N;
}

// how often a blocked receive asks whether to yield (wall-clock ticks, 100 MHz)
constexpr uint64_t kYieldPollTicks = 500;

// MX_ANY_SOURCE: wait until some source p has a message this receive can
// take -- a matching held one, or, among the envelopes p has posted beyond
// what this process consumed from it (lane 0's message count), one whose tag
// matches (any, for MPI_ANY_TAG) -- and store p in status[3] (-1 after a
// timeout).  A source whose pending messages all carry other tags is not
// chosen: its messages stay in its mailbox for the receives that match them
// (pml/ob1 matches an ANY_SOURCE receive against every peer's queue).  The
// envelope ring slots read here cannot be rewritten meanwhile: a sender
// reuses slot m % P2P_H only after this process has consumed message m.
// Yielding (round 5): with a receive queued behind it that could take a
// message, the pick stores -2 (its receive kernel then yields too); with
// displaced receives in the communicator it reads envelope tags for
// MPI_ANY_TAG as well, and skips messages they reserve.
struct P2PPickArgs {
  const uint64_t *flag0;
  const P2PRecvState *st0;
  const char *box0;
  int n, start;
  int64_t tag;
  int64_t *status;
  uint64_t timeout_ticks;
  int *err;
  uint64_t launch, post;
  const P2PRxQueue *rq;
  const P2PDisplaced *disp;
};

__global__ void k_p2p_pick(P2PPickArgs a) {
  if (threadIdx.x != 0) return;
  const uint64_t *flag0 = a.flag0;
  const P2PRecvState *st0 = a.st0;
  const int n = a.n, start = a.start;
  const int64_t tag = a.tag;
  int64_t *status = a.status;
  const uint64_t t0 = wall_clock64();
  for (int i = 0; i < n; i++) {
    const int p = (start + i) % n;
    if (held_match(st0 + p, tag, a.disp, a.post, p).x >= 0) {
      __hip_atomic_store(&status[3], (int64_t)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
  const bool filter = a.disp && a.disp->n > 0;   // reserved messages: read every tag
  // envelopes of source p already read without a match (< 64 sources): the
  // acquire before a scan invalidates the XCD's L2, so a source whose pending
  // messages carry other tags is not rescanned on every pass
  __shared__ uint64_t s_scanned[64];
  for (int p = 0; p < n && p < 64; p++) s_scanned[p] = 0;
  uint64_t polled = t0;
  for (;;) {
    for (int i = 0; i < n; i++) {
      const int p = (start + i) % n;
      const uint64_t posted = __hip_atomic_load(flag0 + P2P_POSTED + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint64_t m0 = st0[p].lane_msgs[0];
      if (posted <= m0) continue;
      bool hit = tag < 0 && !filter;
      if (!hit) {
        if (p < 64 && posted <= s_scanned[p]) continue;
        if (p < 64) s_scanned[p] = posted;
        __atomic_thread_fence(__ATOMIC_ACQUIRE);   // the envelopes before their `posted` count
        const char *box = a.box0 + (size_t)p * P2P_BOX;
        for (uint64_t m = m0; !hit && m < posted && m < m0 + P2P_H; m++) {
          const int64_t et = (int64_t)reinterpret_cast<const volatile uint64_t *>(box + (m % P2P_H) * P2P_HDR)[1];
          hit = (tag < 0 || et == tag) && !reserved(a.disp, a.post, p, et);
        }
      }
      if (hit) {
        __hip_atomic_store(&status[3], (int64_t)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
    }
    __builtin_amdgcn_s_sleep(2);
    const uint64_t now = wall_clock64();
    if (a.rq && now - polled > kYieldPollTicks) {
      polled = now;
      if (disp_room(a.disp, a.post) && rx_queued_can_progress(a.rq, a.launch, st0, -1, nullptr, 0)) {
        __hip_atomic_store(&status[3], (int64_t)-2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
    }
    if (wall_clock64() - t0 > a.timeout_ticks) {
      __hip_atomic_store(&status[3], (int64_t)-1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(a.err, MX_ERR_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
}

// What a receive kernel decided, identically in every lane (each lane sees
// the same held tables -- they change only at a kernel's end -- and the same
// envelope sequence): the held message it took, and the messages it set
// aside.  In LDS, written by thread 0.
struct HoldPlan {
  int kind, hit;                   // held message delivered: kind 0 stash / 1 defer, or -1
  int n;                           // entries set aside by this kernel
  int defer[P2P_STASH_N + P2P_DEFER_N];
  int slot[P2P_STASH_N + P2P_DEFER_N];
  int64_t tag[P2P_STASH_N + P2P_DEFER_N];
  uint64_t bytes[P2P_STASH_N + P2P_DEFER_N], seq[P2P_STASH_N + P2P_DEFER_N];
};

// Copy one message of `bytes` through this lane's stripe (lanes [first,
// first + nl)): from the mailbox (chunk handshake) into dst (dst_cap bytes
// kept; the rest drained).
__device__ __forceinline__ bool recv_stream(int l, int first, int nl, uint64_t bytes, char *dst, uint64_t dst_cap,
                                            const char *box, const uint64_t *filled, uint64_t *drained,
                                            P2PRecvState *st, uint64_t t0, const P2PRecvArgs &a, bool *wrote) {
  __shared__ int ok;
  uint64_t lo, hi;
  p2p_lane(bytes, l, first, nl, &lo, &hi);
  uint64_t k = st->lane_chunks[l];
  for (uint64_t pos = lo; pos < hi; pos += P2P_C) {
    const uint64_t len = std::min<uint64_t>(P2P_C, hi - pos);
    k++;
    if (threadIdx.x == 0) ok = p2p_wait_ge(filled + l, k, t0, a.timeout_ticks, a.err);
    __syncthreads();
    if (!ok) return false;
    const char *slot = box + 4096 + ((size_t)l * P2P_S + (size_t)((k - 1) % P2P_S)) * P2P_C;
    if (pos < dst_cap) {
      p2p_copy(dst + pos, slot, std::min<uint64_t>(len, dst_cap - pos));
      *wrote = true;
    }
    __syncthreads();          // every load of the slot has returned
    if (threadIdx.x == 0) {
      __hip_atomic_store(drained + l, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      st->lane_chunks[l] = k;
    }
  }
  return true;
}

// first free slot of a held table (valid entries and this kernel's new ones taken), or -1
__device__ __forceinline__ int held_free(const P2PStashEntry *tab, int n, const HoldPlan &plan, int defer) {
  for (int k = 0; k < n; k++) {
    bool taken = tab[k].valid != 0;
    for (int j = 0; j < plan.n; j++) taken = taken || (plan.defer[j] == defer && plan.slot[j] == k);
    if (!taken) return k;
  }
  return -1;
}

// Envelope k of this launch (the pair's envelope m), thread 0 of a lane:
// 1 take it, 0 the launch stopped there (yield), -1 timed out.  The first
// lane to see the envelope posted claims "go" for it in the device's
// decision ring; the control workgroup claims "stop" for an envelope not
// posted yet when a receive queued behind could progress; whichever claim
// lands first holds for every lane.
constexpr uint64_t kDecGo = 1, kDecStop = 2;
__device__ __forceinline__ uint64_t dec_key(uint64_t launch, uint64_t k) {
  return ((launch & 0xffffffffull) << 30) | (k & 0x3fffffffull);
}
__device__ int gate_wait(const P2PRecvArgs &a, const uint64_t *posted, uint64_t m, uint64_t k, uint64_t t0) {
  uint64_t *w = a.dec + (k % P2P_DEC);
  const uint64_t key = dec_key(a.launch, k);
  for (;;) {
    uint64_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((v >> 2) == key) {
      if ((v & 3) != kDecGo) return 0;
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
      return 1;
    }
    if (__hip_atomic_load(posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) > m) {
      __hip_atomic_compare_exchange_strong(w, &v, (key << 2) | kDecGo, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      continue;   // re-read: this claim or the other one
    }
    __builtin_amdgcn_s_sleep(2);
    if (wall_clock64() - t0 > a.timeout_ticks) {
      __hip_atomic_store(a.err, MX_ERR_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return -1;
    }
  }
}

// one lane of a receive; returns whether this lane stored user data;
// *yielded: the launch stopped at an envelope boundary (nothing delivered)
__device__ __forceinline__ bool recv_body(const P2PRecvArgs &a, HoldPlan &plan, P2PRecvState **stp, bool *yielded,
                                          bool *rget) {
  const int l = blockIdx.x;
  const uint64_t t0 = wall_clock64();
  __shared__ int ok;
  __shared__ uint64_t s_bytes;
  __shared__ int64_t s_tag;
  __shared__ uint64_t s_seq;
  __shared__ int s_rndv, s_desc;
  int p = a.src;
  *yielded = false;
  *rget = false;
  if (a.any) {
    p = (int)__hip_atomic_load(&a.status[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (p == -2) *yielded = true;   // the pick yielded
    if (p < 0) return false;        // ... or timed out (error already raised)
  }
  const char *box = a.box0 + (size_t)p * P2P_BOX;
  const uint64_t *posted = a.flag0 + P2P_POSTED + p, *filled = a.flag0 + P2P_FILLED + (size_t)p * P2P_L;
  uint64_t *seen = a.peer_flags[p] + P2P_SEEN + (size_t)a.me * P2P_L;
  uint64_t *drained = a.peer_flags[p] + P2P_DRAINED + (size_t)a.me * P2P_L;
  uint64_t *cts = a.peer_flags[p] + P2P_CTS + (size_t)a.me * P2P_RNDV_Q;   // my ring at the sender
  P2PRecvState *st = a.st0 + p;
  char *stash = a.stash0 + (size_t)p * P2P_STASH_N * P2P_STASH_C;
  *stp = st;
  bool wrote = false;
  // clear rendezvous message `seq` with the sender, then take its data
  // through the rendezvous lanes
  auto rndv_take = [&](uint64_t seq, uint64_t bytes) -> bool {
    if (l == 0 && threadIdx.x == 0) {
      const uint64_t t = __hip_atomic_fetch_add(&st->cts_sent, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(cts + t % P2P_RNDV_Q, cts_word(t, false, seq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return recv_stream(l, P2P_LE, P2P_LR, bytes, a.buf, a.cap, box, filled, drained, st, t0, a, &wrote);
  };
  auto deliver_status = [&](uint64_t bytes, int64_t tag, int err) {
    if (l == 0 && threadIdx.x == 0) {
      a.status[0] = (int64_t)std::min<uint64_t>(bytes, a.cap);
      a.status[1] = tag;
      a.status[2] = err ? err : bytes > a.cap ? MX_ERR_TRUNCATE : 0;
      __threadfence_system();
    }
  };
  // (1) a held message this receive matches: deliver it, consume no envelope
  const int2 h = held_match(st, a.tag, a.disp, a.post, p);
  if (h.x >= 0) {
    if (threadIdx.x == 0) {
      plan.kind = h.x;
      plan.hit = h.y;
    }
    const P2PStashEntry e = h.x == 0 ? st->stash[h.y] : st->defer[h.y];
    if (h.x == 0) {
      uint64_t lo, hi;
      p2p_lane(e.bytes, l, 0, P2P_LE, &lo, &hi);
      if (lo < hi && lo < a.cap) {
        p2p_copy(a.buf + lo, stash + (size_t)h.y * P2P_STASH_C + lo, std::min(hi, a.cap) - lo);
        wrote = true;
      }
    } else if (!rndv_take(e.seq, e.bytes)) {
      return wrote;
    }
    deliver_status(e.bytes, e.tag, 0);
    return wrote;
  }
  // (2) envelopes in order: a mismatch (or a message an earlier displaced
  // receive reserves) is set aside (eager payload stashed, rendezvous
  // envelope deferred) while a slot is free
  const uint64_t m0 = st->msgs_done;
  for (;;) {
    if (threadIdx.x == 0) {
      const uint64_t m = st->lane_msgs[l];
      ok = a.rq ? gate_wait(a, posted, m, m - m0, t0) : p2p_wait_ge(posted, m + 1, t0, a.timeout_ticks, a.err);
      if (ok == 1) {
        const volatile uint64_t *hd = reinterpret_cast<const volatile uint64_t *>(box + (m % P2P_H) * P2P_HDR);
        s_bytes = hd[0];
        s_tag = (int64_t)hd[1];
        s_rndv = (int)(hd[2] & 1);
        s_desc = (int)((hd[2] >> 1) & 1);
        s_seq = m;
        if (l == 0 && s_desc && a.rget_ok) {   // the descriptor, before the slot is handed back (seen)
          const volatile uint64_t *dd =
              reinterpret_cast<const volatile uint64_t *>(box + P2P_DESC_OFF + (m % P2P_H) * P2P_DESC);
          for (int w = 0; w < (int)(sizeof(P2PRgetDesc) / 8); w++)
            __hip_atomic_store(&a.status[8 + w], (int64_t)dd[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __hip_atomic_store(seen + l, m + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        st->lane_msgs[l] = m + 1;
      }
    }
    __syncthreads();
    if (ok == 0 && a.rq) {    // stopped here: yield
      *yielded = true;
      return wrote;
    }
    if (ok != 1) return wrote;
    const uint64_t bytes = s_bytes;
    const int64_t tag = s_tag;
    const uint64_t seq = s_seq;
    const int rndv = s_rndv;
    const int desc = s_desc;
    __syncthreads();          // every thread has read the envelope before the next one
    int slot = -1;
    if ((a.tag >= 0 && tag != a.tag) || reserved(a.disp, a.post, p, tag)) {
      slot = rndv ? held_free(st->defer, P2P_DEFER_N, plan, 1)
                  : bytes <= P2P_STASH_C ? held_free(st->stash, P2P_STASH_N, plan, 0) : -1;
    }
    if (slot >= 0) {          // unexpected: keep it for a later receive
      if (!rndv) {
        bool stashed = false;
        if (!recv_stream(l, 0, P2P_LE, bytes, stash + (size_t)slot * P2P_STASH_C, bytes, box, filled, drained, st,
                         t0, a, &stashed))
          return wrote;
      }
      if (threadIdx.x == 0) {
        plan.defer[plan.n] = rndv;
        plan.slot[plan.n] = slot;
        plan.tag[plan.n] = tag;
        plan.bytes[plan.n] = bytes;
        plan.seq[plan.n] = seq;
        plan.n++;
      }
      __syncthreads();
      continue;
    }
    // this receive's message (or one that cannot be set aside: MX_ERR_TAG)
    if (rndv && desc && a.rget_ok) {
      // single copy: the host maps the sender's buffer and pulls the payload
      // (p2p_rget_launch); the status tells it which message
      *rget = true;
      if (l == 0 && threadIdx.x == 0) {
        __hip_atomic_store(&a.status[7], (int64_t)seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&a.status[3], (int64_t)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      deliver_status(bytes, tag, ((a.tag >= 0 && tag != a.tag) || reserved(a.disp, a.post, p, tag)) ? MX_ERR_TAG : 0);
      if (l == 0 && threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(&a.status[6], (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      return wrote;
    }
    if (rndv) {
      if (!rndv_take(seq, bytes)) return wrote;
    } else if (!recv_stream(l, 0, P2P_LE, bytes, a.buf, a.cap, box, filled, drained, st, t0, a, &wrote)) {
      return wrote;
    }
    deliver_status(bytes, tag, ((a.tag >= 0 && tag != a.tag) || reserved(a.disp, a.post, p, tag)) ? MX_ERR_TAG : 0);
    return wrote;
  }
}

// The control workgroup of a launch that may yield (the last workgroup, not
// a lane): follows the envelopes the lanes take, and while the next one is
// not posted asks every kYieldPollTicks whether a receive queued behind
// could progress -- if so it claims "stop" there.  Ends with the lanes.
__device__ void rx_control(const P2PRecvArgs &a) {
  if (threadIdx.x != 0) return;
  int p = a.src;
  if (a.any) p = (int)__hip_atomic_load(&a.status[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (p < 0) return;
  const P2PRecvState *st = a.st0 + p;
  const uint64_t *posted = a.flag0 + P2P_POSTED + p;
  const char *box = a.box0 + (size_t)p * P2P_BOX;
  const uint64_t m0 = st->msgs_done;
  constexpr int kAside = 32;   // tags of the envelopes set aside, the first 32 (a yield heuristic)
  int64_t aside[kAside];
  int naside = 0;
  uint64_t k = 0, polled = wall_clock64();
  for (;;) {
    if (__hip_atomic_load(a.fin.lanes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= a.fin.target) return;
    uint64_t *w = a.dec + (k % P2P_DEC);
    uint64_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t key = dec_key(a.launch, k);
    if ((v >> 2) == key) {
      if ((v & 3) != kDecGo) return;
      // taken and the lanes go on: it was not this receive's message
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
      if (naside < kAside)
        aside[naside++] = (int64_t)reinterpret_cast<const volatile uint64_t *>(box + ((m0 + k) % P2P_H) * P2P_HDR)[1];
      k++;
      continue;
    }
    __builtin_amdgcn_s_sleep(2);
    if (__hip_atomic_load(posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) > m0 + k) continue;   // lanes take it
    const uint64_t now = wall_clock64();
    if (now - polled < kYieldPollTicks) continue;
    polled = now;
    if (disp_room(a.disp, a.post) && rx_queued_can_progress(a.rq, a.launch, a.st0, p, aside, naside) &&
        __hip_atomic_compare_exchange_strong(w, &v, (key << 2) | kDecStop, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return;
  }
}

// workgroups [0, P2P_L) are the lanes; with a launch queue one more, the
// control workgroup (rx_control)
__global__ void __launch_bounds__(kP2PThreads) k_p2p_recv(P2PRecvArgs a) {
  if (blockIdx.x >= P2P_L) {
    if (threadIdx.x == 0) {
      rx_control(a);
      rx_exit(a.fin);
    }
    return;
  }
  __shared__ HoldPlan plan;
  if (threadIdx.x == 0) {
    plan.kind = plan.hit = -1;
    plan.n = 0;
  }
  __syncthreads();
  P2PRecvState *st = nullptr;
  bool yielded = false, rget = false;
  const bool wrote = recv_body(a, plan, &st, &yielded, &rget);
  // the last lane out commits the held-table changes (the tables are read by
  // every lane during the kernel, so they only change between kernels)
  __syncthreads();
  if (threadIdx.x == 0) {
    if (wrote) __threadfence();
    const uint64_t old = __hip_atomic_fetch_add(a.fin.lanes, (uint64_t)1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == a.fin.target) {
      if (st) {
        st->held += (uint64_t)plan.n - (plan.hit >= 0 ? 1 : 0);
        if (plan.hit >= 0) (plan.kind ? st->defer : st->stash)[plan.hit].valid = 0;
        for (int j = 0; j < plan.n; j++) {
          P2PStashEntry &e = (plan.defer[j] ? st->defer : st->stash)[plan.slot[j]];
          e.tag = plan.tag[j];
          e.bytes = plan.bytes[j];
          e.seq = plan.seq[j];
          e.valid = 1;
        }
        st->msgs_done = st->lane_msgs[blockIdx.x];
      }
      if (P2PDisplaced *d = a.disp) {   // join or leave the displaced receives
        const uint64_t n = d->n;
        uint64_t at = n;
        for (uint64_t i = 0; i < n; i++)
          if (d->d[i].post == a.post) at = i;
        if (yielded && at == n && n < P2P_DISP_N) {
          d->d[n].post = a.post;
          d->d[n].src = a.any ? -1 : a.src;
          d->d[n].tag = a.tag;
          d->n = n + 1;
        } else if (!yielded && at < n) {
          d->d[at] = d->d[n - 1];
          d->n = n - 1;
        }
      }
      __threadfence();
      if (yielded) {   // the host launches this receive again (p2p_progress)
        __hip_atomic_store(&a.status[5], (int64_t)a.launch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
        __hip_atomic_store(const_cast<uint64_t *>(&a.rq->yields), a.launch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      } else if (a.fin.done && !rget) {   // a pulled message completes after its pull (p2p_rget_launch)
        __hip_atomic_store(a.fin.done, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      rx_exit(a.fin);
    }
  }
}

// The end of a single-copy rendezvous receive (after its pull and, for a
// datatype, its unpack, on the pull stream): FIN into the sender's CTS ring
// -- its buffer is free, its send completes -- and the receive's status word.
struct P2PFinArgs {
  uint64_t *ring;      // the sender's ring of this pair
  uint64_t *alloc;     // my P2PRecvState.cts_sent of this pair
  uint64_t seq;
  int64_t *done;       // the receive's status[4] (mapped host)
};
__global__ void k_p2p_rget_fin(P2PFinArgs a) {
  if (threadIdx.x != 0) return;
  __threadfence_system();
  const uint64_t t = __hip_atomic_fetch_add(a.alloc, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(a.ring + t % P2P_RNDV_Q, cts_word(t, true, a.seq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(a.done, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The internal streams spin on the device (a receive waits for its message,
// a rendezvous pick for a CTS).  HIP multiplexes a process's streams onto
// GPU_MAX_HW_QUEUES hardware queues per priority, and a kernel spinning on
// a queue holds back every kernel queued behind it there, whatever its
// stream (tools/queue_probe.hip, profiles/r02/queue_probe.txt): created at
// the highest priority, the channel streams get queues the process's
// ordinary streams do not share.
// (MX_P2P_PRIORITY=0: ordinary priority, for measurements)
static hipError_t p2p_stream_create(hipStream_t *s) {
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
  const char *e = getenv("MX_P2P_PRIORITY");
  if (e && atoi(e) == 0) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
}

// The send and receive channel streams of a device are shared by all its
// communicators: HIP maps a process's streams onto 4
// hardware queues per priority, and a kernel spinning on a queue holds back
// every kernel behind it there, whatever its stream.  Three streams per
// communicator overran the 4 high-priority queues from the second
// communicator on, so two communicators' channels landed on one queue in an
// order nothing controlled.  Shared, sends and receives take 2 queues
// however many communicators exist, and the channel work of all
// communicators runs in post order per direction -- the order one
// communicator's work always had.  The rendezvous stream stays
// per communicator and is made at its first rendezvous send: its kernels
// wait for that communicator's CTS tickets only, so on a shared stream a
// send of one communicator would hold back a cleared send of another.
static std::mutex g_chan_mu;
static hipStream_t g_chan[64][2];

// Per device, like the receive stream the receive kernels share: the launch
// queue a blocked receive reads (mapped host), the decision ring (device),
// and the receive requests in flight in the order of their first launch
// (the host launches yielded ones again in that order, p2p_progress).
// MX_P2P_YIELD=0: receives never yield (each blocks the receive stream
// until its message comes -- the round-4 behaviour).
struct RxDev {
  P2PRxQueue *rq = nullptr, *rq_dev = nullptr;
  uint64_t *dec = nullptr;
  uint64_t launches = 0, seen = 0;
  std::vector<mx_request *> active;
  std::vector<mx_request *> rget;   // receives in flight that may be left a rendezvous to pull
  hipStream_t pull = nullptr;       // the pulls: an ordinary-priority stream (they never spin)
};
static RxDev g_rx[64];
static int g_rx_dev[64], g_rx_ndev;
// MX_P2P_RGET=0: rendezvous messages always stream through the mailbox
// (round 5's two-copy path); default: single copy from registered buffers
static bool rget_on() {
  static const bool on = [] {
    const char *e = getenv("MX_P2P_RGET");
    return !(e && *e == '0');
  }();
  return on;
}
// smallest rendezvous message sent with its descriptor (MX_P2P_RGET_MIN,
// bytes): below it the mailbox's two copies beat the pull's host round trip
// (one GPU, profiles/r06/p2p_lat_r6*.txt: 1 MiB 37 vs 52 us, 16 MiB 81 vs 58 us)
static size_t rget_min() {
  static const size_t m = [] {
    const char *e = getenv("MX_P2P_RGET_MIN");
    return e ? (size_t)strtoull(e, nullptr, 0) : (size_t)4 << 20;
  }();
  return m;
}
static void rx_dev_note(int dev) {   // caller holds g_chan_mu
  for (int i = 0; i < g_rx_ndev; i++)
    if (g_rx_dev[i] == dev) return;
  g_rx_dev[g_rx_ndev++] = dev;
}
static bool rx_yield_on() {
  static const bool on = [] {
    const char *e = getenv("MX_P2P_YIELD");
    return !(e && *e == '0');
  }();
  return on;
}
static int p2p_channels(hipStream_t out[3]) {
  int dev = g_device;
  if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return MX_ERR_HIP;
  if (dev < 0 || dev >= 64) return MX_ERR_HIP;
  std::lock_guard<std::mutex> lk(g_chan_mu);
  for (int i = 0; i < 2; i++) {
    if (!g_chan[dev][i] && p2p_stream_create(&g_chan[dev][i]) != hipSuccess) {
      g_chan[dev][i] = nullptr;
      (void)hipGetLastError();
      return MX_ERR_HIP;
    }
    out[i] = g_chan[dev][i];
  }
  return MX_SUCCESS;
}
static int p2p_rndv_stream(mx_comm *c) {
  if (c->p2p_stream[2]) return MX_SUCCESS;
  if (p2p_stream_create(&c->p2p_stream[2]) != hipSuccess) {
    c->p2p_stream[2] = nullptr;
    (void)hipGetLastError();
    return MX_ERR_HIP;
  }
  return MX_SUCCESS;
}

// this communicator's kernel just enqueued on channel i.  Its completion is
// the mapped word its last lane raises (P2PDone::hfin reaching p2p_ltot[i]):
// an event recorded after every kernel put a second packet behind each one
// on the channel's queue, and a kernel enqueued while the one before had not
// retired then waited ~27 us more to start -- the 8 B hop's slow mode
// (profiles/r05/p2p_latency_modes_r5ar.txt)
static int p2p_note(mx_comm *c, int i) {
  c->p2p_last_valid[i] = 1;
  return MX_SUCCESS;
}

// the communicator's kernels on channel i have all finished (the word their
// last lanes raise), or the channel's stream failed
static bool p2p_channel_idle(mx_comm *c, int i) {
  if (!c->p2p_last_valid[i] || !c->p2p_hfin) return true;
  // a datatype receive's unpack runs after the receive kernel raised the word
  if (i == 1 && c->p2p_unpack_pending) {
    if (hipEventQuery(c->p2p_unpack_ev) == hipErrorNotReady) {
      (void)hipGetLastError();   // NotReady is no error of a later launch
      return false;
    }
    (void)hipGetLastError();
    c->p2p_unpack_pending = 0;
  }
  if (i == 1 && c->p2p_pull_pending) {   // the host-launched pulls of this communicator
    if (hipEventQuery(c->p2p_pull_ev) == hipErrorNotReady) {
      (void)hipGetLastError();
      return false;
    }
    (void)hipGetLastError();
    c->p2p_pull_pending = 0;
  }
  if (__atomic_load_n(&c->p2p_hfin[i], __ATOMIC_ACQUIRE) >= c->p2p_ltot[i]) return true;
  // a drained stream ran every kernel of the channel (a failed stream never
  // raises the word either); the streams are shared, so idle is also idle
  // for this communicator
  const hipError_t e = c->p2p_stream[i] ? hipStreamQuery(c->p2p_stream[i]) : hipSuccess;
  (void)hipGetLastError();
  return e != hipErrorNotReady;
}

static void p2p_channel_wait(mx_comm *c, int i) {
  for (int k = 0; !p2p_channel_idle(c, i); k++)
    if (k > 1000) std::this_thread::sleep_for(std::chrono::microseconds(50));
}

// Setup makes no device-wide synchronisation: a receive of another
// communicator may be spinning for a message whose sender waits for this
// rank's first send here (example 3).  Buffers come from
// the process pools (hipMalloc / hipFree wait for the whole device on this
// runtime), the memsets run on the lifecycle stream.
static size_t p2p_stash_bytes(const mx_comm *c) { return (size_t)c->size * P2P_STASH_N * P2P_STASH_C; }

int p2p_setup(mx_comm *c) {
  if (c->p2p_send) return MX_SUCCESS;
  const size_t sb = sizeof(P2PSendState) * c->size, rb = sizeof(P2PRecvState) * c->size;
  hipStream_t ls = life_stream();
  if (!(c->p2p_send = (P2PSendState *)pool_dev_get(sb))) {
    c->p2p_send = nullptr;
    return MX_ERR_NOMEM;
  }
  const bool ok =
      (c->p2p_recv = (P2PRecvState *)pool_dev_get(rb)) != nullptr &&
      (c->p2p_lanes = (uint64_t *)pool_dev_get(4 * sizeof(uint64_t))) != nullptr &&
      (c->p2p_stash = (char *)pool_dev_get(p2p_stash_bytes(c))) != nullptr &&
      (c->p2p_rndv_cur = (P2PRndvCur *)pool_dev_get(sizeof(P2PRndvCur))) != nullptr &&
      (c->p2p_rndv = (P2PRndvTable *)pool_host_get(sizeof(P2PRndvTable))) != nullptr &&
      hipHostGetDevicePointer((void **)&c->p2p_rndv_dev, c->p2p_rndv, 0) == hipSuccess &&
      (c->p2p_disp = (P2PDisplaced *)pool_dev_get(sizeof(P2PDisplaced))) != nullptr &&
      (c->p2p_hfin = (uint64_t *)pool_host_get(3 * sizeof(uint64_t))) != nullptr &&
      hipHostGetDevicePointer((void **)&c->p2p_hfin_dev, c->p2p_hfin, 0) == hipSuccess;
  if (!ok) {
    p2p_release(c);
    return MX_ERR_NOMEM;
  }
  c->p2p_posts = 0;
  c->p2p_hfin[0] = c->p2p_hfin[1] = c->p2p_hfin[2] = 0;
  if (rx_yield_on() && c->device >= 0 && c->device < 64) {
    std::lock_guard<std::mutex> lk(g_chan_mu);
    RxDev &D = g_rx[c->device];
    if (!D.rq) {
      P2PRxQueue *rq = (P2PRxQueue *)pool_host_get(sizeof(P2PRxQueue));
      uint64_t *dec = (uint64_t *)pool_dev_get(P2P_DEC * sizeof(uint64_t));
      P2PRxQueue *rq_dev = nullptr;
      if (!rq || !dec || hipHostGetDevicePointer((void **)&rq_dev, rq, 0) != hipSuccess ||
          hipMemsetAsync(dec, 0, P2P_DEC * sizeof(uint64_t), ls) != hipSuccess) {
        if (rq) pool_host_put(rq, sizeof(P2PRxQueue));
        if (dec) pool_dev_put(dec, P2P_DEC * sizeof(uint64_t));
        p2p_release(c);
        return MX_ERR_NOMEM;
      }
      memset(rq, 0, sizeof(P2PRxQueue));
      D.rq = rq;
      D.rq_dev = rq_dev;
      D.dec = dec;
      rx_dev_note(c->device);
    }
  }
  if (rget_on() && c->device >= 0 && c->device < 64) {
    std::lock_guard<std::mutex> lk(g_chan_mu);
    RxDev &D = g_rx[c->device];
    if (!D.pull && hipStreamCreateWithFlags(&D.pull, hipStreamNonBlocking) != hipSuccess) {
      (void)hipGetLastError();
      D.pull = nullptr;
    }
    rx_dev_note(c->device);
  }
  memset(c->p2p_rndv, 0, sizeof(P2PRndvTable));
  c->p2p_rndv_gen = 0;
  c->p2p_rndv_free = new std::vector<int>();
  for (int i = P2P_RNDV_Q - 1; i >= 0; i--) c->p2p_rndv_free->push_back(i);
  c->p2p_ltot[0] = c->p2p_ltot[1] = c->p2p_ltot[2] = 0;
  c->p2p_xtot = 0;
  c->p2p_unpack_pending = 0;
  c->p2p_pull_pending = 0;
  for (int j = 0; j < MAXR; j++) c->p2p_host_msgs[j] = 0;
  if (hipMemsetAsync(c->p2p_send, 0, sb, ls) != hipSuccess || hipMemsetAsync(c->p2p_recv, 0, rb, ls) != hipSuccess ||
      hipMemsetAsync(c->p2p_lanes, 0, 4 * sizeof(uint64_t), ls) != hipSuccess ||
      hipMemsetAsync(c->p2p_rndv_cur, 0, sizeof(P2PRndvCur), ls) != hipSuccess ||
      hipMemsetAsync(c->p2p_disp, 0, sizeof(P2PDisplaced), ls) != hipSuccess ||
      p2p_channels(c->p2p_stream) != MX_SUCCESS ||
      hipEventCreateWithFlags(&c->p2p_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->p2p_unpack_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->p2p_pull_ev, hipEventDisableTiming) != hipSuccess ||
      hipStreamSynchronize(ls) != hipSuccess) {
    p2p_release(c);
    return MX_ERR_HIP;
  }
  return MX_SUCCESS;
}

void p2p_quiesce(mx_comm *c) {
  // this communicator's kernels only (the streams are shared)
  for (int i = 0; i < 2; i++) p2p_channel_wait(c, i);
  // rendezvous sends no receive ever cleared: their picks give up
  if (c->p2p_rndv) __atomic_store_n(&c->p2p_rndv->abort, 1, __ATOMIC_RELEASE);
  p2p_channel_wait(c, 2);
  c->p2p_last_valid[0] = c->p2p_last_valid[1] = c->p2p_last_valid[2] = 0;
}

bool p2p_pending(mx_comm *c) {
  for (int i = 0; i < 3; i++)
    if (!p2p_channel_idle(c, i)) return true;
  return false;
}

void p2p_release(mx_comm *c) {
  p2p_quiesce(c);
  // receives of this communicator still in flight (yielded, never launched
  // again) are launched by nobody from now on
  if (c->device >= 0 && c->device < 64) {
    std::vector<mx_request *> &v = g_rx[c->device].active;
    v.erase(std::remove_if(v.begin(), v.end(), [c](mx_request *q) { return q->c == c; }), v.end());
    std::vector<mx_request *> &w = g_rx[c->device].rget;
    w.erase(std::remove_if(w.begin(), w.end(), [c](mx_request *q) { return q->c == c; }), w.end());
  }
  pool_host_put(c->p2p_hfin, 3 * sizeof(uint64_t));
  c->p2p_hfin = c->p2p_hfin_dev = nullptr;
  if (c->p2p_stream[2]) (void)hipStreamDestroy(c->p2p_stream[2]);   // its own; [0], [1] are the device's
  if (c->p2p_ev) (void)hipEventDestroy(c->p2p_ev);
  if (c->p2p_unpack_ev) (void)hipEventDestroy(c->p2p_unpack_ev);
  c->p2p_unpack_ev = nullptr;
  c->p2p_unpack_pending = 0;
  if (c->p2p_pull_ev) (void)hipEventDestroy(c->p2p_pull_ev);
  c->p2p_pull_ev = nullptr;
  c->p2p_pull_pending = 0;
  const size_t sb = sizeof(P2PSendState) * c->size, rb = sizeof(P2PRecvState) * c->size;
  pool_dev_put(c->p2p_send, sb);
  pool_dev_put(c->p2p_recv, rb);
  pool_dev_put(c->p2p_lanes, 4 * sizeof(uint64_t));
  pool_dev_put(c->p2p_stash, p2p_stash_bytes(c));
  pool_dev_put(c->p2p_rndv_cur, sizeof(P2PRndvCur));
  pool_dev_put(c->p2p_disp, sizeof(P2PDisplaced));
  c->p2p_disp = nullptr;
  pool_host_put(c->p2p_rndv, sizeof(P2PRndvTable));
  delete c->p2p_rndv_free;
  c->p2p_rndv_free = nullptr;
  c->p2p_rndv = c->p2p_rndv_dev = nullptr;
  c->p2p_rndv_cur = nullptr;
  c->p2p_lanes = nullptr;
  c->p2p_stash = nullptr;
  c->p2p_stream[0] = c->p2p_stream[1] = c->p2p_stream[2] = nullptr;
  c->p2p_ev = nullptr;
  c->p2p_send = nullptr;
  c->p2p_recv = nullptr;
}

void p2p_finish(mx_request *q) {
  mx_comm *c = q->c;
  if (q->rndv && c->p2p_rndv) {
    c->p2p_rndv->e[q->rndv - 1].valid = 0;
    c->p2p_rndv_free->push_back(q->rndv - 1);
  }
  q->rndv = 0;
  const int ch = q->kind == RQ_RECV ? 1 : 2;
  if (q->tmp) (void)hipFreeAsync(q->tmp, c->p2p_stream[ch] ? c->p2p_stream[ch] : nullptr);
  q->tmp = nullptr;
  if (q->kind == RQ_RECV) {
    if (c->device >= 0 && c->device < 64) {
      std::vector<mx_request *> &v = g_rx[c->device].active;
      const auto it = std::find(v.begin(), v.end(), q);
      if (it != v.end()) v.erase(it);
      std::vector<mx_request *> &w = g_rx[c->device].rget;
      const auto jt = std::find(w.begin(), w.end(), q);
      if (jt != w.end()) w.erase(jt);
    }
    q->rget = 0;
    q->rget_t0 = 0;
    delete static_cast<P2PRecvArgs *>(q->rx);
    q->rx = nullptr;
    q->launch = 0;
  }
}

bool p2p_yielded(const mx_request *q) {
  return q->kind == RQ_RECV && q->status && q->launch &&
         __atomic_load_n(&q->status[5], __ATOMIC_ACQUIRE) == (int64_t)q->launch;
}

// not complete although its launch ended: the launch yielded (launched again
// by p2p_progress), or it left a rendezvous for the host to pull that
// p2p_progress has not launched yet
bool p2p_rx_waiting(const mx_request *q) {
  if (q->kind != RQ_RECV || !q->status) return false;
  if (!q->rget && __atomic_load_n(&q->status[6], __ATOMIC_ACQUIRE)) return true;
  return p2p_yielded(q);
}

namespace {
constexpr int kStatusPool = 4096;
std::mutex g_status_mu;
int64_t *g_status_pool;          // kStatusPool blocks of P2P_STATUS_WORDS x int64
int64_t *g_status_pool_dev;      // its device address
int g_status_free[kStatusPool];
int g_status_nfree = -1;         // -1: not allocated yet
}  // namespace

int64_t *p2p_status_get() {
  {
    std::lock_guard<std::mutex> lk(g_status_mu);
    if (g_status_nfree < 0) {
      g_status_nfree = 0;
      if (hipHostMalloc((void **)&g_status_pool, (size_t)kStatusPool * P2P_STATUS_WORDS * sizeof(int64_t),
                        hipHostMallocMapped) ==
          hipSuccess) {
        for (int i = 0; i < kStatusPool; i++) g_status_free[i] = kStatusPool - 1 - i;
        g_status_nfree = kStatusPool;
        if (hipHostGetDevicePointer((void **)&g_status_pool_dev, g_status_pool, 0) != hipSuccess)
          g_status_pool_dev = nullptr;
      } else {
        g_status_pool = nullptr;
      }
    }
    if (g_status_nfree > 0) return g_status_pool + (size_t)g_status_free[--g_status_nfree] * P2P_STATUS_WORDS;
  }
  int64_t *st = nullptr;
  if (hipHostMalloc((void **)&st, P2P_STATUS_WORDS * sizeof(int64_t), hipHostMallocMapped) != hipSuccess)
    return nullptr;
  return st;
}

// device address of a status block (pool blocks: no runtime call)
int64_t *p2p_status_dev(int64_t *st) {
  {
    std::lock_guard<std::mutex> lk(g_status_mu);
    if (g_status_pool && g_status_pool_dev && st >= g_status_pool &&
        st < g_status_pool + (size_t)kStatusPool * P2P_STATUS_WORDS)
      return g_status_pool_dev + (st - g_status_pool);
  }
  int64_t *d = nullptr;
  return hipHostGetDevicePointer((void **)&d, st, 0) == hipSuccess ? d : nullptr;
}

void p2p_status_put(int64_t *st) {
  if (!st) return;
  {
    std::lock_guard<std::mutex> lk(g_status_mu);
    if (g_status_pool && st >= g_status_pool && st < g_status_pool + (size_t)kStatusPool * P2P_STATUS_WORDS) {
      g_status_free[g_status_nfree++] = (int)((st - g_status_pool) / P2P_STATUS_WORDS);
      return;
    }
  }
  (void)hipHostFree(st);
}

int p2p_rx_launch(mx_request *q);

// Enqueue request q (RQ_SEND / RQ_RECV) on the internal stream, after the
// caller's stream; *done_stream receives the stream completion is on.
int p2p_enqueue(mx_request *q, hipStream_t *done_stream) {
  mx_comm *c = q->c;
  if (c->local || !(c->flags & MX_COMM_IPC) || !(c->flags & MX_COMM_P2P)) return MX_ERR_STATE;
  if (c->poisoned) return c->poisoned;
  int rc = p2p_setup(c);
  if (rc) return rc;
  const bool send = q->kind == RQ_SEND;
  const int dir = send ? 0 : 1;
  hipStream_t s = c->p2p_stream[dir];
  // after the work the caller's stream has queued -- none when it is idle
  // (the event pair costs as much as the transfer of a small message)
  const hipError_t qe = hipStreamQuery(q->s);
  if (qe != hipSuccess) {
    if (qe != hipErrorNotReady) return MX_ERR_HIP;
    if (hipEventRecord(c->p2p_ev, q->s) != hipSuccess || hipStreamWaitEvent(s, c->p2p_ev, 0) != hipSuccess)
      return MX_ERR_HIP;
  }
  *done_stream = s;
  if (!q->status && !(q->status = p2p_status_get())) return MX_ERR_NOMEM;
  memset(q->status, 0, P2P_STATUS_WORDS * sizeof(int64_t));
  int64_t *st_dev = p2p_status_dev(q->status);
  if (!st_dev) return MX_ERR_HIP;
  const int me = c->rank, p = q->peer;
  const size_t bytes = q->ddt ? q->count * mx_ddt_size(q->ddt) : q->count;
  const bool rndv = send && bytes > P2P_STASH_C;
  if (rndv && c->p2p_rndv_free->empty()) return MX_ERR_NOMEM;   // P2P_RNDV_Q rendezvous sends pending
  if (rndv && (rc = p2p_rndv_stream(c))) return rc;
  // completion through status[4] when the transfer kernel is the last one
  // (a send's pack runs before it on the same stream; a receive's unpack
  // after it); a rendezvous send completes only through status[4], raised
  // by whichever rendezvous kernel takes its CTS
  q->fast = rndv ? 2 : (send || !q->ddt) ? 1 : 0;
  const int nl = send ? P2P_LE : P2P_L;
  P2PDone fin;
  fin.lanes = c->p2p_lanes + dir;
  fin.target = c->p2p_ltot[dir] + nl;
  fin.done = q->fast == 1 ? st_dev + 4 : nullptr;
  fin.hfin = c->p2p_hfin_dev + dir;
  fin.exits = nullptr;
  fin.xtarget = 0;
  char *tmp = nullptr;
  if (q->ddt && bytes && hipMallocAsync((void **)&tmp, bytes, s) != hipSuccess) return MX_ERR_NOMEM;
  if (send) {
    if (tmp && (rc = mx_pack(q->ddt, q->count, q->sbuf, tmp, 0, bytes, s))) return rc;
    const char *src = tmp ? tmp : (const char *)q->sbuf;
    if (rndv) {
      const int slot = c->p2p_rndv_free->back();
      c->p2p_rndv_free->pop_back();
      P2PRndvEntry &e = c->p2p_rndv->e[slot];
      e.buf = src;
      e.bytes = bytes;
      e.seq = c->p2p_host_msgs[p];
      e.done = st_dev + 4;
      e.dst = p;
      __atomic_store_n(&e.valid, 1, __ATOMIC_RELEASE);
      q->rndv = slot + 1;
      q->tmp = tmp;
    }
    c->p2p_host_msgs[p]++;
    P2PSendArgs a;
    memset(&a, 0, sizeof a);
    a.buf = src;
    a.bytes = bytes;
    a.tag = q->tag;
    a.rndv = rndv;
    // single copy: a contiguous device buffer (one runtime allocation) goes
    // out with its descriptor, the receiver pulls it (btl_smcuda_get_cuda's
    // role, btl_smcuda.c:1077-1180); the mailbox stream stays the fallback
    // (a packed datatype lives in stream-ordered memory, which has no IPC
    // handle; a receiver that set the envelope aside clears it with a CTS)
    if (rndv && !tmp && rget_on() && bytes >= rget_min() && mx_rdma_register(src, bytes, &a.desc.h) == MX_SUCCESS) {
      a.desc.addr = (uint64_t)(uintptr_t)src;
      a.has_desc = 1;
    }
    a.box = c->peer_staging[p] + c->p2p_off + (size_t)me * P2P_BOX;
    a.posted = c->peer_flags[p] + P2P_POSTED + me;
    a.filled = c->peer_flags[p] + P2P_FILLED + (size_t)me * P2P_L;
    a.seen = c->flagmem + P2P_SEEN + (size_t)p * P2P_L;
    a.drained = c->flagmem + P2P_DRAINED + (size_t)p * P2P_L;
    a.st = c->p2p_send + p;
    a.timeout_ticks = c->timeout_ticks;
    a.err = c->err_dev;
    a.fin = fin;
    hipLaunchKernelGGL(k_p2p_send, dim3(P2P_LE), dim3(kP2PThreads), 0, s, a);
    if ((rc = mx_check_launch())) return rc;
    c->p2p_ltot[0] += nl;   // every launched transfer kernel counts its lanes, flagged or not
    p2p_note(c, 0);
    if (rndv) {
      // the rendezvous kernel needs no event: the CTS it waits for follows
      // the envelope, which follows the caller's stream and the pack
      P2PRndvArgs ra;
      memset(&ra, 0, sizeof ra);
      ra.cur = c->p2p_rndv_cur;
      ra.gen = ++c->p2p_rndv_gen;
      ra.cts0 = c->flagmem + P2P_CTS;
      ra.n = c->size;
      ra.tab = c->p2p_rndv_dev;
      for (int j = 0; j < c->size; j++) {
        ra.box[j] = c->peer_staging[j] + c->p2p_off + (size_t)me * P2P_BOX;
        ra.filled[j] = c->peer_flags[j] + P2P_FILLED + (size_t)me * P2P_L;
      }
      ra.drained0 = c->flagmem + P2P_DRAINED;
      ra.st0 = c->p2p_send;
      ra.timeout_ticks = c->timeout_ticks;
      ra.err = c->err_dev;
      ra.fin.lanes = c->p2p_lanes + 2;
      ra.fin.target = c->p2p_ltot[2] + P2P_LR;
      ra.fin.done = nullptr;
      ra.fin.hfin = c->p2p_hfin_dev + 2;
      ra.fin.exits = nullptr;
      ra.fin.xtarget = 0;
      hipLaunchKernelGGL(k_p2p_rndv, dim3(P2P_LR), dim3(kP2PThreads), 0, c->p2p_stream[2], ra);
      if ((rc = mx_check_launch())) return rc;
      c->p2p_ltot[2] += P2P_LR;
      p2p_note(c, 2);
      return MX_SUCCESS;   // tmp is freed when the request completes (p2p_finish)
    }
  } else {
    q->status[3] = p;
    P2PRecvArgs *ap = static_cast<P2PRecvArgs *>(q->rx);
    if (!ap && !(ap = new (std::nothrow) P2PRecvArgs())) {
      if (tmp) (void)hipFreeAsync(tmp, s);
      return MX_ERR_NOMEM;
    }
    q->rx = ap;
    P2PRecvArgs &a = *ap;
    memset(&a, 0, sizeof a);
    a.buf = tmp ? tmp : (char *)q->rbuf;
    a.cap = bytes;
    a.tag = q->tag;
    a.src = p;
    a.any = p < 0;
    a.me = me;
    a.box0 = c->staging + c->p2p_off;
    a.flag0 = c->flagmem;
    for (int j = 0; j < c->size; j++) a.peer_flags[j] = c->peer_flags[j];
    a.st0 = c->p2p_recv;
    a.stash0 = c->p2p_stash;
    a.status = st_dev;
    a.timeout_ticks = c->timeout_ticks;
    a.err = c->err_dev;
    a.rget_ok = rget_on() && g_rx[c->device].pull != nullptr;
    q->rget = 0;
    q->rget_t0 = 0;
    q->tmp = tmp;   // freed at completion: a receive that yields runs (and unpacks) again
    q->post = ++c->p2p_posts;
    if ((rc = p2p_rx_launch(q))) {
      p2p_finish(q);
      return rc;
    }
    if (g_rx[c->device].rq) g_rx[c->device].active.push_back(q);
    if (a.rget_ok) g_rx[c->device].rget.push_back(q);
    return MX_SUCCESS;
  }
  if (tmp) (void)hipFreeAsync(tmp, s);
  return MX_SUCCESS;
}

// One launch of receive q on the receive stream: the pick (MPI_ANY_SOURCE),
// the receive kernel, the unpack (a datatype).  With yielding on, the launch
// is first published in the device's launch queue, so a receive blocked
// ahead of it can see it; the kernel gets one workgroup more (rx_control).
int p2p_rx_launch(mx_request *q) {
  mx_comm *c = q->c;
  hipStream_t s = c->p2p_stream[1];
  P2PRecvArgs &a = *static_cast<P2PRecvArgs *>(q->rx);
  RxDev &D = g_rx[c->device];
  a.launch = a.post = 0;
  a.rq = nullptr;
  a.dec = nullptr;
  a.disp = nullptr;
  if (D.rq) {
    const uint64_t L = ++D.launches;
    P2PQEntry &e = D.rq->e[L % P2P_Q];
    __atomic_store_n(&e.launch, (uint64_t)0, __ATOMIC_RELAXED);
    e.post = q->post;
    e.flag0 = c->flagmem;
    e.st0 = c->p2p_recv;
    e.box0 = c->staging + c->p2p_off;
    e.disp = c->p2p_disp;
    e.n = c->size;
    e.src = a.src;
    e.tag = a.tag;
    __atomic_store_n(&e.launch, L, __ATOMIC_RELEASE);
    __atomic_store_n(&D.rq->enq, L, __ATOMIC_RELEASE);
    a.launch = L;
    a.post = q->post;
    a.rq = D.rq_dev;
    a.dec = D.dec;
    a.disp = c->p2p_disp;
  }
  q->launch = a.launch;
  a.fin.lanes = c->p2p_lanes + 1;
  a.fin.target = c->p2p_ltot[1] + P2P_L;
  a.fin.done = q->fast == 1 ? a.status + 4 : nullptr;
  a.fin.hfin = c->p2p_hfin_dev + 1;
  a.fin.exits = a.rq ? c->p2p_lanes + 3 : nullptr;
  a.fin.xtarget = c->p2p_xtot + 2;
  int rc;
  if (a.any) {
    P2PPickArgs pa;
    memset(&pa, 0, sizeof pa);
    pa.flag0 = c->flagmem;
    pa.st0 = c->p2p_recv;
    pa.box0 = c->staging + c->p2p_off;
    pa.n = c->size;
    pa.start = (int)(c->p2p_any_rr++ % (unsigned)c->size);
    pa.tag = a.tag;
    pa.status = a.status;
    pa.timeout_ticks = c->timeout_ticks;
    pa.err = c->err_dev;
    pa.launch = a.launch;
    pa.post = a.post;
    pa.rq = a.rq;
    pa.disp = a.disp;
    hipLaunchKernelGGL(k_p2p_pick, dim3(1), dim3(64), 0, s, pa);
    if ((rc = mx_check_launch())) return rc;
  }
  hipLaunchKernelGGL(k_p2p_recv, dim3(a.rq ? P2P_L + 1 : P2P_L), dim3(kP2PThreads), 0, s, a);
  if ((rc = mx_check_launch())) return rc;
  c->p2p_ltot[1] += P2P_L;   // counted once launched: a failed launch never raises the word
  if (a.rq) c->p2p_xtot += 2;
  p2p_note(c, 1);
  if (q->tmp) {   // the unpack reads tmp and writes the user buffer after the word is raised
    if ((rc = mx_unpack(q->ddt, q->count, q->rbuf, q->tmp, 0, a.cap, s))) return rc;
    if (hipEventRecord(c->p2p_unpack_ev, s) != hipSuccess) return MX_ERR_HIP;
    c->p2p_unpack_pending = 1;
  }
  return MX_SUCCESS;
}

bool p2p_rx_active() {
  for (int i = 0; i < g_rx_ndev; i++)
    if (!g_rx[g_rx_dev[i]].active.empty()) return true;
  return false;
}

// Launch again every receive whose last launch yielded, in the order of
// their first launches (the kernels record the latest yield in the queue,
// so nothing is scanned while no receive yielded).
// The pull of a single-copy rendezvous receive whose kernel noted the
// message (status[6]): map the sender's allocation (mx_rdma's import cache),
// one copy kernel from it into the receive buffer (the packed staging for a
// datatype, unpacked after), then FIN to the sender and the receive's status
// word -- all on the device's pull stream.  The request completes through the
// status word from then on (fast 2).  A mapping that cannot be made yet (a
// stale import still waiting for its close) is tried again at the next
// progress; a failed one completes the receive with the error, and FIN still
// releases the sender.
static void p2p_rget_launch(mx_request *q) {
  mx_comm *c = q->c;
  RxDev &D = g_rx[c->device];
  P2PRecvArgs &a = *static_cast<P2PRecvArgs *>(q->rx);
  const int p = (int)__atomic_load_n(&q->status[3], __ATOMIC_ACQUIRE);
  if (p < 0 || p >= c->size || !D.pull) return;
  P2PRgetDesc d;
  memcpy(&d, (const void *)&q->status[8], sizeof d);
  const uint64_t n = (uint64_t)q->status[0];
  int rc = n ? rdma_pull(a.buf, &d.h, d.addr, n, D.pull) : MX_SUCCESS;
  if (rc == MX_ERR_STATE) {   // retried at the next progress, for at most the communicator's timeout (or 60 s)
    const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now().time_since_epoch()).count();
    if (!q->rget_t0) q->rget_t0 = now;
    const double lim = c->timeout_s > 0 ? c->timeout_s : 60.0;
    if ((double)(now - q->rget_t0) * 1e-9 < lim) return;
    rc = MX_ERR_HIP;   // the sender's allocation could not be mapped: the receive fails, FIN still goes
  }
  if (!rc && q->tmp) rc = mx_unpack(q->ddt, q->count, q->rbuf, q->tmp, 0, a.cap, D.pull);
  if (rc && !q->status[2]) q->status[2] = rc;
  P2PFinArgs f;
  f.ring = c->peer_flags[p] + P2P_CTS + (size_t)c->rank * P2P_RNDV_Q;
  f.alloc = &c->p2p_recv[p].cts_sent;
  f.seq = (uint64_t)q->status[7];
  f.done = a.status + 4;
  hipLaunchKernelGGL(k_p2p_rget_fin, dim3(1), dim3(64), 0, D.pull, f);
  if (mx_check_launch() != MX_SUCCESS) return;
  if (hipEventRecord(c->p2p_pull_ev, D.pull) == hipSuccess) c->p2p_pull_pending = 1;
  c->p2p_last_valid[1] = 1;
  q->fast = 2;   // complete through status[4] only
  q->rget = 1;
  c->st.p2p_pulls++;
}

void p2p_progress() {
  for (int i = 0; i < g_rx_ndev; i++) {
    RxDev &D = g_rx[g_rx_dev[i]];
    for (size_t j = 0; j < D.rget.size(); j++) {
      mx_request *q = D.rget[j];
      if (q->active && !q->rget && q->status && __atomic_load_n(&q->status[6], __ATOMIC_ACQUIRE)) p2p_rget_launch(q);
    }
    if (!D.rq || D.active.empty()) continue;
    const uint64_t y = __atomic_load_n(&D.rq->yields, __ATOMIC_ACQUIRE);
    if (y == D.seen) continue;
    D.seen = y;
    for (size_t j = 0; j < D.active.size(); j++) {
      mx_request *q = D.active[j];
      if (!q->active || !p2p_yielded(q)) continue;
      if (p2p_rx_launch(q) == MX_SUCCESS) {
        (void)hipEventRecord(q->done, q->c->p2p_stream[1]);
        q->c->st.p2p_relaunches++;
      }
    }
  }
}

}  // namespace mx

using namespace mx;

namespace {

static int p2p_request(mx_comm_t *c, int kind, int persistent, const void *sbuf, void *rbuf, size_t count,
                       const mx_ddt_t *ddt, int peer, int tag, void *stream, mx_request_t **req) {
  if (!c || !req || peer >= c->size) return MX_ERR_ARG;
  if (peer < 0 && !(kind == RQ_RECV && peer == MX_ANY_SOURCE)) return MX_ERR_ARG;
  if (count && (kind == RQ_SEND ? !sbuf : !rbuf)) return MX_ERR_ARG;
  mx_request *q;
  int rc = req_create(c, kind, persistent, stream, &q);
  if (rc) return rc;
  q->sbuf = sbuf;
  q->rbuf = rbuf;
  q->count = count;
  q->ddt = ddt;
  q->peer = peer;
  q->tag = tag;
  return req_submit(q, req);
}

static int p2p_blocking(mx_comm_t *c, int kind, const void *sbuf, void *rbuf, size_t count, const mx_ddt_t *ddt,
                        int peer, int tag, void *stream, size_t *received) {
  mx_request_t *q = nullptr;
  int rc = p2p_request(c, kind, 0, sbuf, rbuf, count, ddt, peer, tag, stream, &q);
  if (rc) return rc;
  rc = mx_wait(q);
  if (received) *received = (kind == RQ_RECV && q->status) ? (size_t)q->status[0] : 0;
  const int frc = mx_request_free(q);
  return rc ? rc : frc;
}

}  // namespace

extern "C" int mx_isend(mx_comm_t *c, const void *buf, size_t bytes, int dst, int tag, void *stream,
                        mx_request_t **req) {
  return p2p_request(c, RQ_SEND, 0, buf, nullptr, bytes, nullptr, dst, tag, stream, req);
}
extern "C" int mx_irecv(mx_comm_t *c, void *buf, size_t bytes, int src, int tag, void *stream, mx_request_t **req) {
  return p2p_request(c, RQ_RECV, 0, nullptr, buf, bytes, nullptr, src, tag, stream, req);
}
extern "C" int mx_send_init(mx_comm_t *c, const void *buf, size_t bytes, int dst, int tag, void *stream,
                            mx_request_t **req) {
  return p2p_request(c, RQ_SEND, 1, buf, nullptr, bytes, nullptr, dst, tag, stream, req);
}
extern "C" int mx_recv_init(mx_comm_t *c, void *buf, size_t bytes, int src, int tag, void *stream,
                            mx_request_t **req) {
  return p2p_request(c, RQ_RECV, 1, nullptr, buf, bytes, nullptr, src, tag, stream, req);
}
extern "C" int mx_send(mx_comm_t *c, const void *buf, size_t bytes, int dst, int tag, void *stream) {
  return p2p_blocking(c, RQ_SEND, buf, nullptr, bytes, nullptr, dst, tag, stream, nullptr);
}
extern "C" int mx_recv(mx_comm_t *c, void *buf, size_t bytes, int src, int tag, void *stream, size_t *received) {
  return p2p_blocking(c, RQ_RECV, nullptr, buf, bytes, nullptr, src, tag, stream, received);
}
extern "C" int mx_isend_ddt(mx_comm_t *c, const void *buf, size_t count, const mx_ddt_t *ddt, int dst, int tag,
                            void *stream, mx_request_t **req) {
  if (!ddt) return MX_ERR_ARG;
  return p2p_request(c, RQ_SEND, 0, buf, nullptr, count, ddt, dst, tag, stream, req);
}
extern "C" int mx_irecv_ddt(mx_comm_t *c, void *buf, size_t count, const mx_ddt_t *ddt, int src, int tag,
                            void *stream, mx_request_t **req) {
  if (!ddt) return MX_ERR_ARG;
  return p2p_request(c, RQ_RECV, 0, nullptr, buf, count, ddt, src, tag, stream, req);
}

// MPI_Sendrecv: both directions in flight at once (send and receive streams)
extern "C" int mx_sendrecv(mx_comm_t *c, const void *sbuf, size_t sbytes, int dst, int stag, void *rbuf,
                           size_t rbytes, int src, int rtag, void *stream, size_t *received) {
  mx_request_t *rq = nullptr, *sq = nullptr;
  int rc = p2p_request(c, RQ_RECV, 0, nullptr, rbuf, rbytes, nullptr, src, rtag, stream, &rq);
  if (rc) return rc;
  rc = p2p_request(c, RQ_SEND, 0, sbuf, nullptr, sbytes, nullptr, dst, stag, stream, &sq);
  const int wrc = sq ? mx_wait(sq) : MX_SUCCESS;
  const int rrc = mx_wait(rq);
  if (received) *received = rq->status ? (size_t)rq->status[0] : 0;
  if (sq) mx_request_free(sq);
  mx_request_free(rq);
  return rc ? rc : wrc ? wrc : rrc;
}

// MPI_SOURCE of a completed receive request (the matched source for
// MX_ANY_SOURCE)
extern "C" int mx_request_source(const mx_request_t *q, int *source) {
  if (!q || q->kind != RQ_RECV || !q->status || !source) return MX_ERR_ARG;
  if (q->active) return MX_ERR_STATE;
  *source = (int)q->status[3];
  return MX_SUCCESS;
}

// status of a completed receive request (MPI_Get_count / MPI_TAG)
extern "C" int mx_request_status(const mx_request_t *q, size_t *bytes, int *tag) {
  if (!q || q->kind != RQ_RECV || !q->status) return MX_ERR_ARG;
  if (q->active) return MX_ERR_STATE;
  if (bytes) *bytes = (size_t)q->status[0];
  if (tag) *tag = (int)q->status[1];
  return MX_SUCCESS;
}
