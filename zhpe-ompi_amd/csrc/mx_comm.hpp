// mx_comm.hpp -- state shared by the collective (mx_coll.hip) and
// point-to-point (mx_p2p.hip) translation units: the communicator, its flag
// word layout, and requests.  Internal; the C-ABI is include/mx_coll.h.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <vector>

#include "mx_fold.hpp"
#include "mx_coll.h"
#include "mx_rdma.h"

namespace mx {

// ---- flag words (uncached, IPC-mapped; one array per rank) ---------------
// [NFLAGS x MAXR] generation flags READY / PUSHED / DONE per source rank;
// one-shot small-message allreduce: per (source rank, workgroup) READY
// flags, then one local completion counter; then 8 words of which the first
// two are the creation signatures read back through every mapping.
constexpr size_t OS_FLAG_BASE = NFLAGS * MAXR;
constexpr size_t OS_COUNTER = OS_FLAG_BASE + (size_t)MAXR * OSWG;
constexpr size_t FLAG_WORDS = OS_COUNTER + 8;

// ---- point-to-point channels (mx_p2p.hip) --------------------------------
// Every rank owns one mailbox per source rank after the collective staging:
// a header ring of P2P_H message envelopes and P2P_L lanes of P2P_S chunk
// slots of P2P_C bytes.  Lanes [0, P2P_LE) carry eager messages (at most
// P2P_STASH_C bytes, pushed as soon as they are sent); lanes [P2P_LE, P2P_L)
// carry rendezvous messages (larger ones), whose data moves only after the
// matching receive has cleared it (CTS), so a large message no receive wants
// yet never blocks the pair's later messages.  Counters (cumulative, per pair):
//   posted[src]          my flags: envelopes src has written into my mailbox
//   filled[src][lane]    my flags: chunks src has written into my lane
//   seen[dst][lane]      my flags (written by dst): envelopes dst has read
//   drained[dst][lane]   my flags (written by dst): chunks dst has consumed
//   cts[dst][P2P_RNDV_Q] my flags (written by dst): a ring of the rendezvous
//                        messages dst has cleared, one word each (cts_word):
//                        stream the data through the lanes (CTS), or dst
//                        already pulled it straight from my buffer (FIN)
// Rendezvous send with a descriptor (single copy, round 6): the envelope's
// mode word has bit 1 set and the sender's buffer descriptor (P2PRgetDesc:
// the allocation's IPC handle and the buffer address) sits in the mailbox's
// descriptor slot m % P2P_H; the receiver's host maps the allocation and
// one copy kernel pulls the payload, then FIN goes into the ring.
constexpr int P2P_RNDV_Q = 256;   // rendezvous sends pending per communicator (and CTS ring entries per pair)
constexpr int P2P_LE = 8;
constexpr int P2P_L = P2P_LE + 64;
constexpr int P2P_S = 4;
constexpr size_t P2P_C = 64 << 10;
constexpr int P2P_H = 8;
constexpr size_t P2P_HDR = 64;
constexpr size_t P2P_DESC_OFF = 512;   // descriptor slots after the header ring (P2P_H x P2P_HDR)
constexpr size_t P2P_DESC = 128;
constexpr size_t P2P_BOX = 4096 + (size_t)P2P_L * P2P_S * P2P_C;
constexpr size_t P2P_POSTED = FLAG_WORDS + 8;
constexpr size_t P2P_FILLED = P2P_POSTED + MAXR;
constexpr size_t P2P_SEEN = P2P_FILLED + (size_t)MAXR * P2P_L;
constexpr size_t P2P_DRAINED = P2P_SEEN + (size_t)MAXR * P2P_L;
constexpr size_t P2P_CTS = P2P_DRAINED + (size_t)MAXR * P2P_L;
// BYE[src]: written once by src in mx_comm_destroy, after its device was
// idle -- its last access to this rank's regions is over, so the regions may
// serve another communicator (mx_coll.hip, the IPC region pool)
constexpr size_t BYE_BASE = P2P_CTS + (size_t)MAXR * P2P_RNDV_Q;
constexpr size_t ALL_FLAG_WORDS = BYE_BASE + (size_t)MAXR;
constexpr uint64_t BYE_WORD = 0xB7EB7EB7EB7EB7EBull;

// Unexpected messages: a receive whose tag does not match the pair's next
// envelope sets that message aside and goes on to the next envelope; later
// receives match what was set aside first, oldest first (MPI's per-pair
// order among the messages a receive could match).  An eager message is
// drained into a stash slot (P2P_STASH_N per source, P2P_STASH_C bytes
// each); a rendezvous message only has its envelope recorded (P2P_DEFER_N
// per source) -- its data stays with the sender until a receive clears it.
constexpr int P2P_STASH_N = 16;
constexpr size_t P2P_STASH_C = 256 << 10;
constexpr int P2P_DEFER_N = 64;
struct P2PStashEntry { uint64_t valid; int64_t tag; uint64_t bytes; uint64_t seq; };

// device-local sequence state of the channels (not shared)
struct P2PSendState {
  uint64_t msgs;
  uint64_t lane_chunks[P2P_L];
  uint64_t cts_served;                 // entries of this destination's CTS ring taken
};
struct P2PRecvState {
  uint64_t lane_msgs[P2P_L];
  uint64_t lane_chunks[P2P_L];
  uint64_t cts_sent;                   // CTS ring entries issued to this source (atomic: receive kernels and pulls)
  uint64_t held;                       // valid entries in stash + defer (0: skip the scan)
  P2PStashEntry stash[P2P_STASH_N];    // written only by the last lane of a receive kernel
  P2PStashEntry defer[P2P_DEFER_N];    // likewise
  uint64_t msgs_done;                  // envelopes consumed by finished kernels (lane_msgs at their end)
};

// Receives that yield.  Receive kernels run one at a
// time on the device's receive stream; one that waits for its message while
// a receive queued behind it could take a message that has arrived (or that
// was set aside) stops at an envelope boundary instead of blocking the
// stream ("yields"), and the host launches it again behind the others.  A
// receive that yielded is "displaced": later receives of its communicator
// leave the messages it matches alone, so each message still goes to the
// earliest posted receive that matches it (pml/ob1's order).
constexpr int P2P_Q = 256;        // launches a blocked receive looks at behind it
constexpr int P2P_DISP_N = 32;    // displaced receives per communicator
struct P2PQEntry {                // one receive launch (mapped host, written before the launch)
  uint64_t launch;                // launch number (written last)
  uint64_t post;                  // its post number in its communicator
  const uint64_t *flag0;          // its communicator's flag array
  const P2PRecvState *st0;        // ... receive state per source
  const char *box0;               // ... mailboxes
  const struct P2PDisplaced *disp;
  int32_t n, src;                 // src < 0: MPI_ANY_SOURCE
  int64_t tag;                    // < 0: MPI_ANY_TAG
};
struct P2PRxQueue {               // one per device, mapped host memory
  uint64_t enq;                   // receive launches enqueued (host)
  uint64_t yields;                // launch number of the latest yield (device)
  P2PQEntry e[P2P_Q];             // launch L at e[L % P2P_Q]
};
struct P2PDispEntry { uint64_t post; int32_t src, pad; int64_t tag; };
struct P2PDisplaced {             // device memory, changed only by a receive kernel's last lane
  uint64_t n;
  P2PDispEntry d[P2P_DISP_N];
};
constexpr int P2P_DEC = 16;       // decision ring: envelope k of a launch taken or stopped at

// one CTS ring word: stamp (entry index + 1, 24 bits) | FIN | message seq
__host__ __device__ constexpr uint64_t cts_word(uint64_t ticket, bool fin, uint64_t seq) {
  return ((ticket + 1) & 0xffffffull) << 40 | (fin ? 1ull << 39 : 0) | (seq & ((1ull << 39) - 1));
}
// the sender's descriptor of a rendezvous buffer (13 words in the mailbox's
// descriptor slot, copied by the receive kernel into status[8..21))
struct P2PRgetDesc {
  mx_rdma_handle_t h;
  uint64_t addr;
};
static_assert(sizeof(P2PRgetDesc) == 13 * 8 && sizeof(P2PRgetDesc) <= P2P_DESC, "descriptor slot");

// Rendezvous sends waiting for their CTS (mapped host memory, written by the
// host when the send is posted, read by the rendezvous pick kernel)
struct P2PRndvEntry {
  const char *buf;
  uint64_t bytes, seq;
  int64_t *done;       // device address of the request's status[4]
  int32_t dst, valid;
};
struct P2PRndvTable {
  P2PRndvEntry e[P2P_RNDV_Q];
  int32_t abort;       // communicator teardown: pending picks give up
};
// the message the running rendezvous kernel's workgroup 0 picked (device
// memory, read by its other workgroups once `gen` moves)
struct P2PRndvCur {
  const char *buf;
  uint64_t bytes;
  int64_t *done;
  int32_t dst, ok;
  uint64_t gen;        // rendezvous kernels that have published a pick
};

}  // namespace mx

// a peer allocation mapped for zero-copy collectives.  Key: peer + the
// exporter's allocation base + its runtime buffer id (HIP_POINTER_ATTRIBUTE_
// BUFFER_ID): an allocation freed and re-made at the same address -- what a
// caching allocator does after empty_cache() -- can carry byte-identical IPC
// handles, so the handle alone does not tell a stale mapping from a live one.
struct mx_reg_import {
  int peer;
  uint64_t base, size, id;
  char *ptr;
  uint64_t used;
  unsigned char h[64];   // the handle it was opened from
};

// ---------------------------------------------------------------------------
// communicator
// ---------------------------------------------------------------------------
struct mx_comm {
  int rank, size, device, local;
  int flags;
  size_t staging_bytes;
  size_t staging_alloc;        // bytes of the staging allocation (+ mailboxes)
  size_t main_bytes;           // staging for the chunked paths: [0, main_bytes)
  size_t os_max, os_slot;      // one-shot: default max bytes per rank, slot stride
  size_t os_cap;               // one-shot: the most a slot holds (autotuning may pick it up to here)
  size_t os_ll;                // one-shot: the tagged-word (LL) protocol up to this many bytes per rank (<= OS_LL_CAP)
                               // (its area, 2 * os_ll, follows the raw os_cap + 256 in each slot)
  uint64_t os_count;           // one-shot workgroup completions so far
  char *staging;               // mine (uncached, IPC-exported)
  char *peer_staging[mx::MAXR];    // mapped views (peer_staging[rank] = staging)
  uint64_t *flagmem;           // mine: [NFLAGS][mx::MAXR]
  uint64_t *peer_flags[mx::MAXR];  // mapped views
  int *err_host, *err_dev;
  // poison word (device memory): set by the kernel whose peer wait timed
  // out; every later copy / fold / signal kernel of the communicator sees
  // it and does nothing, so no peer is handed stale staging data and no
  // staging a late peer still reads is overwritten.  `poisoned` is the
  // host's sticky copy: every later call fails with it.
  int *poison;
  int poisoned;
  uint64_t gen;
  // created on every rank (peers map this rank's regions): destroy says BYE
  int live;
  // fault injection for the regression tests only (MX_DEBUG_LAG_RANK /
  // MX_DEBUG_LAG_US): this rank starts every fold kernel lag_ticks late
  uint64_t lag_ticks;
  // staged allreduce data movement (MX_PROTO_*): PUSH writes each part to
  // its owner before the fold (two xGMI phases); PULL copies the input into
  // the rank's own staging and the owner's fold reads the parts over xGMI
  // while it writes results to the peers (one xGMI phase; the default).
  // `xdev`: some peer runs on another GPU (PCI bus ids differ).
  int proto, xdev;
  // user-buffer registration (zero-copy allreduce): a host
  // shared-memory page per communicator where every rank publishes the IPC
  // handles of its call's buffers; peers' allocations stay mapped in an LRU
  // cache.  reg_shm null: registration unavailable (every rank agrees).
  void *reg_shm;
  size_t reg_shm_bytes, reg_min;
  // zero-copy allreduce results written straight into the peers' registered
  // rbufs (no gather area, no gather copy; mx_comm_set_zc_direct)
  int zc_direct;
  uint64_t reg_seq, reg_tick;
  std::vector<struct mx_reg_import> *reg_imp;
  std::vector<mx::IpcGone> *reg_gone;   // the imports closed (ipc_open_checked)
  void *reg_fast;   // the last exchange's records and mappings (mx_coll.hip RegFast)
  // data-movement autotuning of blocking collectives: per
  // collective kind (TUNE_*) and power-of-two size class, the first call
  // warms up, the next ones time each candidate (allreduce from 64 KiB:
  // zero-copy / PULL / PUSH / one-shot; reduce_scatter, allgather from
  // 256 KiB: zero-copy / staged; bcast from 64 KiB: zero-copy / scatter /
  // direct; max over ranks, exchanged in the registration page; below 4 MiB
  // every candidate runs 3 times and its fastest run counts) and the fastest
  // is kept.  tune_best: choice + 1, 0 = not yet.
  int tune_on;
  uint8_t tune_calls[4][64];
  int8_t tune_best[4][64];
  double tune_t[4][64][4];
  uint64_t tune_seq;
  double timeout_s;
  uint64_t timeout_ticks;
  ncclComm_t nccl;
  // the host bootstrap exchange, kept for later collective setups
  // (symmetric heaps); ctx must outlive the communicator
  mx_allgather_fn ag;
  void *ag_ctx;
  // symmetric-heap region exported with the staging at creation
  // (mx_comm_create_ex heap_bytes): heaps are carved from it
  char *hregion;
  char *peer_hregion[mx::MAXR];
  size_t hregion_bytes, hregion_used;
  // profiling: event pairs recorded around kernels of the current call
  int prof;
  hipEvent_t ev[64];
  int nev;
  int ev_kind[32];   // 0 fold, 1 push, 2 gather
  double ev_bytes[32];
  mx_coll_stats_t st;
  // non-blocking / persistent requests: while `defer`
  // is set, finish() leaves the stream running; `tail` is an event after the
  // last deferred collective, which a collective enqueued on another stream
  // waits for (collectives of a communicator stay in issue order across
  // streams, as MPI orders them); `pending` counts active requests.
  int defer;
  int tail_valid;
  hipEvent_t tail;
  hipStream_t tail_stream;
  int pending;
  // point-to-point: mailboxes at staging + p2p_off (P2P_BOX per source),
  // device-local channel state, and the two streams sends and receives run
  // on (so a send never waits behind a receive of the same process)
  size_t p2p_off;
  mx::P2PSendState *p2p_send;   // [size]
  mx::P2PRecvState *p2p_recv;   // [size]
  char *p2p_stash;              // [size][P2P_STASH_N][P2P_STASH_C] unexpected-message payloads
  // streams: [0] sends (envelopes, eager data), [1] receives, [2] rendezvous
  // data; all three spin on the device, so they are created at the highest
  // priority, whose hardware queues the process's ordinary streams do not
  // share
  // the device's three channel streams (send, receive, rendezvous pick),
  // shared by every communicator of the process (p2p_setup): the spinning
  // channels hold 3 high-priority hardware queues per device, whatever the
  // number of communicators.  p2p_hfin[i] reaching p2p_ltot[i]: this
  // communicator's last kernel on channel i has finished (its own work, for
  // destroy and quiet checks; raised by that kernel's last lane).
  hipStream_t p2p_stream[3];
  int p2p_last_valid[3];             // work was enqueued on channel i since the last quiesce
  uint64_t *p2p_hfin, *p2p_hfin_dev; // mapped [3]: target of the last finished kernel per channel
  hipEvent_t p2p_ev;
  uint64_t *p2p_lanes;     // device: finished-lane counters of the three streams, [3] receive-launch exits
  uint64_t p2p_ltot[3];    // lanes (workgroups) of the transfer kernels enqueued per stream
  uint64_t p2p_xtot;       // exits of the receive launches with a control workgroup (p2p_lanes[3])
  hipEvent_t p2p_unpack_ev;          // after the last datatype receive's unpack
  int p2p_unpack_pending;            // ... which p2p_channel_idle has not yet seen complete
  hipEvent_t p2p_pull_ev;            // after the last single-copy pull (+ unpack + FIN) of this communicator
  int p2p_pull_pending;
  // small allreduces may be served by the resident service (mx_coll_svc.hip):
  // at most two ranks of the communicator per device (set at creation)
  int csv_ok;
  uint64_t p2p_host_msgs[mx::MAXR];   // envelopes enqueued per destination (the device's msgs)
  mx::P2PRndvTable *p2p_rndv;        // mapped host: pending rendezvous sends
  mx::P2PRndvTable *p2p_rndv_dev;    // its device address
  mx::P2PRndvCur *p2p_rndv_cur;      // device
  uint64_t p2p_rndv_gen;             // rendezvous kernels enqueued
  std::vector<int> *p2p_rndv_free;   // free table slots
  unsigned p2p_any_rr;   // MPI_ANY_SOURCE: source the next pick scans first
  mx::P2PDisplaced *p2p_disp;        // device: receives of this communicator that yielded
  uint64_t p2p_posts;                // receives posted (their post numbers)
};


enum { RQ_ALLREDUCE, RQ_REDUCE, RQ_REDUCE_SCATTER, RQ_REDUCE_SCATTER_BLOCK, RQ_SCAN, RQ_EXSCAN, RQ_ALLGATHER, RQ_BCAST,
       RQ_SEND, RQ_RECV };

struct mx_request {
  mx_comm *c;
  int kind, persistent, active;
  hipStream_t s;
  hipEvent_t done;
  const void *sbuf;
  void *rbuf;
  size_t count;   // elements (bytes for allgather / bcast)
  int type, op, alg, root;
  std::vector<size_t> rcounts;
  // point-to-point: peer, tag, and the status the receiving kernel writes
  // (mapped host memory: received bytes, envelope tag, error)
  int peer, tag;
  int64_t *status;   // [0] bytes [1] tag [2] error [3] source [4] done [5] yielded launch
                     // [6] rendezvous to pull [7] its seq [8..21) its P2PRgetDesc (P2P_STATUS_WORDS)
  int fast;          // completion by status[4]: 1 also by the event, 2 only by status[4]
                     // (a rendezvous send: its data moves on whichever kernel takes its CTS)
  int rndv;          // rendezvous send: table slot + 1, else 0
  void *tmp;         // packed staging freed at completion (a rendezvous send or a receive of a datatype)
  const struct mx_ddt *ddt;   // non-contiguous user layout (count instances), or null
  // a receive: its post number, its current launch (status[5] == launch: that
  // launch yielded) and its kernel arguments, kept for the next launch
  uint64_t post, launch;
  void *rx;
  int rget;          // the host launched this receive's pull (single-copy rendezvous)
  int64_t rget_t0;   // steady-clock ns of the pull's first refused mapping (0: none)
};

namespace mx {
// point-to-point (mx_p2p.hip): enqueue a send / receive request, completion
// recorded by the caller on *done_stream; release the channel state
int p2p_enqueue(mx_request *q, hipStream_t *done_stream);
// request plumbing of mx_coll.hip: create (inactive), submit (start unless
// persistent; frees on failure), discard (never submitted)
int req_create(mx_comm *c, int kind, int persistent, void *stream, mx_request **q);
int req_submit(mx_request *q, mx_request_t **out);
void req_discard(mx_request *q);
int p2p_setup(mx_comm *c);
// wait for the communicator's point-to-point channels (rendezvous sends no
// receive ever cleared give up first); no device-wide synchronisation
void p2p_quiesce(mx_comm *c);
bool p2p_pending(mx_comm *c);   // this communicator's channel kernels not yet done
void p2p_release(mx_comm *c);
// a point-to-point request completed: release its rendezvous slot / staging
void p2p_finish(mx_request *q);
// launch again the receives whose kernels yielded (from every wait / test)
void p2p_progress();
// a receive request's current launch yielded (it is not complete)
bool p2p_yielded(const mx_request *q);
// ... or it is a receive whose kernel ended without completing it (yielded,
// or a rendezvous left to pull): what the completion checks ask
bool p2p_rx_waiting(const mx_request *q);
// some receive of this process is in flight (its launches may yield)
bool p2p_rx_active();
// status blocks (P2P_STATUS_WORDS x int64, mapped host memory): from a process-wide
// pool allocated once (never released, so a request may outlive its
// communicator), else one hipHostMalloc each
constexpr int P2P_STATUS_WORDS = 24;
// the resident small-allreduce service (mx_coll_svc.hip): 1 served, 0 the
// caller launches the same one-shot arguments, < 0 error; csv_comm_gone
// stops a service bound to a communicator about to be destroyed
int csv_allreduce(mx_comm *c, const OneShotArgs &a, int op, int type, hipStream_t s);
void csv_comm_gone(const mx_comm *c);
int64_t *p2p_status_get();
void p2p_status_put(int64_t *st);
}  // namespace mx
