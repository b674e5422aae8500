// mx_comm.hpp -- state shared by the collective (mx_coll.hip) and
// point-to-point (mx_p2p.hip) translation units: the communicator, its flag
// word layout, and requests.  Internal; the C-ABI is include/mx_coll.h.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <vector>

#include "mx_fold.hpp"
#include "mx_coll.h"

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
// slots of P2P_C bytes.  Counters (cumulative, per pair):
//   posted[src]          my flags: envelopes src has written into my mailbox
//   filled[src][lane]    my flags: chunks src has written into my lane
//   seen[dst][lane]      my flags (written by dst): envelopes dst has read
//   drained[dst][lane]   my flags (written by dst): chunks dst has consumed
constexpr int P2P_L = 64;
constexpr int P2P_S = 4;
constexpr size_t P2P_C = 64 << 10;
constexpr int P2P_H = 8;
constexpr size_t P2P_HDR = 64;
constexpr size_t P2P_BOX = 4096 + (size_t)P2P_L * P2P_S * P2P_C;
constexpr size_t P2P_POSTED = FLAG_WORDS + 8;
constexpr size_t P2P_FILLED = P2P_POSTED + MAXR;
constexpr size_t P2P_SEEN = P2P_FILLED + (size_t)MAXR * P2P_L;
constexpr size_t P2P_DRAINED = P2P_SEEN + (size_t)MAXR * P2P_L;
constexpr size_t ALL_FLAG_WORDS = P2P_DRAINED + (size_t)MAXR * P2P_L;

// Unexpected messages: a receive whose tag does not match the pair's next
// envelope drains that message into a stash slot (up to P2P_STASH_N
// messages of at most P2P_STASH_C bytes per source) and goes on to the next
// envelope; later receives match the stash first, oldest first (MPI's
// per-pair order among the messages a receive could match).
constexpr int P2P_STASH_N = 8;
constexpr size_t P2P_STASH_C = 256 << 10;
struct P2PStashEntry { uint64_t valid; int64_t tag; uint64_t bytes; uint64_t seq; };

// device-local sequence state of the channels (not shared)
struct P2PSendState { uint64_t msgs; uint64_t lane_chunks[P2P_L]; };
struct P2PRecvState {
  uint64_t lane_msgs[P2P_L];
  uint64_t lane_chunks[P2P_L];
  P2PStashEntry stash[P2P_STASH_N];   // written only by the last lane of a receive kernel
};

}  // namespace mx

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
  hipStream_t p2p_stream[2];
  hipEvent_t p2p_ev;
  uint64_t *p2p_lanes;     // device: finished-lane counters of the two streams
  uint64_t p2p_kseq[2];    // transfer kernels enqueued per stream
  unsigned p2p_any_rr;   // MPI_ANY_SOURCE: source the next pick scans first
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
  int64_t *status;   // [0] bytes [1] tag [2] error [3] source [4] done (P2P_STATUS_WORDS)
  int fast;          // completion by status[4] (no unpack kernel after the transfer)
  const struct mx_ddt *ddt;   // non-contiguous user layout (count instances), or null
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
void p2p_release(mx_comm *c);
// status blocks (P2P_STATUS_WORDS x int64, mapped host memory): from a process-wide
// pool allocated once (never released, so a request may outlive its
// communicator), else one hipHostMalloc each
constexpr int P2P_STATUS_WORDS = 8;
int64_t *p2p_status_get();
void p2p_status_put(int64_t *st);
}  // namespace mx
