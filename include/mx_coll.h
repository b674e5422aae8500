/*
 * mx_coll.h -- C-ABI of the MI355X collective data path (libmx_kernels.so).
 *
 * Replaces, for device-resident buffers, the host algorithms behind the coll
 * module slots (ompi/mca/coll/coll.h:200-244):
 *   mx_allreduce       <- ompi_coll_base_allreduce_intra_{recursivedoubling,
 *                         ring, ring_segmented, redscat_allgather,
 *                         basic_linear} (ompi/mca/coll/base/
 *                         coll_base_allreduce.c:130-274, 341-536, 618-856,
 *                         970-1243, 881-912) as chosen by
 *                         ompi_coll_tuned_allreduce_intra_dec_fixed
 *                         (ompi/mca/coll/tuned/coll_tuned_decision_fixed.c:44-95)
 *   mx_reduce_scatter  <- ompi_coll_base_reduce_scatter_intra_{ring,
 *                         basic_recursivehalving} (coll_base_reduce_scatter.c:
 *                         456-623, 132-) + tuned rule (decision_fixed.c:466-512)
 *   mx_allgather       <- coll_base_allgather.c (pure data movement)
 *   mx_bcast           <- coll_base_bcast.c (pure data movement)
 *
 * Design (MI355X-first, not the reference's message pattern):
 *  * data moves ALL-PEER over xGMI in one step per phase (every GPU writes
 *    straight into the IPC-mapped staging of each of the other n-1 GPUs,
 *    so all 7 links of an MI355X carry traffic at once) instead of the
 *    reference's n-1 neighbour steps;
 *  * the local reduction is ONE fused HIP kernel per output part that
 *    reads the n contributions and evaluates, per element, exactly the
 *    reduction tree (operand order and roles) that the selected reference
 *    algorithm would have applied -- so results are bit-identical to
 *    coll/tuned's for every op, including FP SUM/PROD -- and writes the
 *    result to the local rbuf and to every peer's gather area;
 *  * cross-GPU ordering uses generation-tagged flags in uncached device
 *    memory written with system-scope atomics, waited on by device spins
 *    (optionally bounded: mx_comm_set_timeout).
 *
 * Ownership: the caller owns all buffers.  Calls are blocking with respect
 * to `stream` semantics: work is enqueued on `stream`, and the call returns
 * after the stream completed (MPI blocking-collective semantics); results
 * are in rbuf on return.  Collectives are issued in the same order on every
 * rank (MPI semantics); the non-blocking / persistent forms below return
 * before completion.
 */
#ifndef MX_COLL_H
#define MX_COLL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mx_comm mx_comm_t;
struct mx_ddt;   /* mx_convertor.h */

/* MPI_IN_PLACE as the reference defines it (mpi.h: (void *) 1). */
#define MX_IN_PLACE ((const void *)1)

/* Maximum ranks of the custom all-peer path (one MI355X node has 8). */
#define MX_MAX_RANKS 16

/* Host bootstrap all-gather supplied by the caller: gather `bytes` from each
 * rank into `recv` (rank-major).  In the coll component this is the host
 * allgather of the lower-priority module saved at module enable (the
 * coll/cuda stacking pattern, coll_cuda_module.c:120-155); in tests it is
 * torch.distributed over gloo.  Returns 0 on success. */
typedef int (*mx_allgather_fn)(const void *send, void *recv, size_t bytes, void *ctx);

/* comm flags */
#define MX_COMM_IPC   1   /* all-peer xGMI path over IPC-mapped staging  */
#define MX_COMM_RCCL  2   /* also create an RCCL communicator             */
#define MX_COMM_P2P   4   /* point-to-point mailboxes (size x 16 MiB of
                             device memory per rank; needs MX_COMM_IPC)   */

/* Multi-process communicator: one rank per process (per GPU). */
int mx_comm_create(int rank, int size, int device, size_t staging_bytes, int flags,
                   mx_allgather_fn allgather, void *ctx, mx_comm_t **comm);
/* As mx_comm_create, plus a symmetric-heap region of heap_bytes per rank,
 * exported and mapped (and verified) with the staging; mx_heap_create
 * carves heaps from it (see "device symmetric heap" below). */
int mx_comm_create_ex(int rank, int size, int device, size_t staging_bytes, size_t heap_bytes, int flags,
                      mx_allgather_fn allgather, void *ctx, mx_comm_t **comm);
/* `size` virtual ranks in ONE process on ONE device.  Same algorithms, same
 * kernels, same fold order; the data path reads/writes all ranks' buffers
 * directly (no staging, no flags).  Used by the parity tests on a single
 * GPU and as the intra-process path. */
int mx_comm_create_local(int size, int device, mx_comm_t **comm);
int mx_comm_destroy(mx_comm_t *comm);
int mx_comm_size(const mx_comm_t *comm);
int mx_comm_rank(const mx_comm_t *comm);
/* Timeout of the device-side peer waits (default 60 s; 0 = wait forever,
 * what an MPI communicator needs: a peer may legally arrive arbitrarily
 * late).  When a wait does time out the communicator is POISONED: every
 * copy / fold / signal kernel already queued behind the wait does nothing
 * (no peer is handed stale data, no staging a late peer still reads is
 * overwritten), the call returns MX_ERR_TIMEOUT, and every later call on
 * the communicator fails with it. */
int mx_comm_set_timeout(mx_comm_t *comm, double seconds);

/* Data movement of the staged (above the one-shot range) allreduce.  Results
 * are identical under every protocol (same fold programs); only the traffic
 * pattern differs (the link bytes are the same):
 *   PUSH  each rank writes part p of its input into rank p's staging, then
 *         rank p folds locally and writes the result to every peer (two
 *         xGMI phases with a flag round trip between them);
 *   PULL  each rank copies its input into its own staging (local HBM), then
 *         rank p's fold reads part p of every peer's staging over xGMI while
 *         it writes the result to every peer (one xGMI phase, remote reads).
 * AUTO (the default) is PULL (measured ahead of PUSH on one GPU at every size
 * from 2 MiB); env MX_ALLREDUCE_PROTO=push|pull overrides it at creation.  Every rank of a communicator must use the same protocol:
 * set it on all ranks between collectives.  Returns the protocol in force
 * (MX_PROTO_PUSH / MX_PROTO_PULL) or an error. */
enum { MX_PROTO_AUTO = 0, MX_PROTO_PUSH = 1, MX_PROTO_PULL = 2 };
int mx_comm_set_protocol(mx_comm_t *comm, int proto);
int mx_comm_get_protocol(const mx_comm_t *comm);

/* Zero-copy allreduce between user buffers (the device-buffer registration
 * of btl/smcuda + rcache/gpusm, done per call): a blocking mx_allreduce of at
 * least `min_bytes` per rank publishes the IPC handles of its sbuf / rbuf
 * allocations in a host shared-memory page of the communicator; every peer
 * maps them (cached, LRU) and rank p folds part p straight from every
 * rank's sbuf into every rank's rbuf -- no staging copies.  A call falls back
 * to the staged path on every rank when any rank's buffers cannot be
 * exported or mapped, or their misalignments mod 16 differ.  Default
 * 256 KiB (env MX_REG_MIN at creation; 0 = off).  Same value on every rank.
 * Returns MX_ERR_UNSUPPORTED when the communicator has no registration page
 * (single rank, local communicator, or /dev/shm unavailable on some rank). */
int mx_comm_set_reg_min(mx_comm_t *comm, size_t min_bytes);

/* Zero-copy allreduce results written straight into every peer's registered
 * rbuf by the rank that folds each part (1, the default; env MX_ZC_DIRECT=0
 * at creation switches it off), or through the peers' uncached gather areas
 * and a local gather copy (0).  Results are identical either way.  Direct
 * needs sbuf and rbuf at the same misalignment mod 16 (else the gather path
 * runs).  Same value on every rank. */
int mx_comm_set_zc_direct(mx_comm_t *comm, int on);

/* Lifecycle calls (communicator / heap create and destroy, first
 * point-to-point on a communicator, datatype destroy) never wait for the
 * whole device: another communicator's nonblocking work may be spinning on a
 * peer that waits for this rank.  The runtime calls that do wait for every
 * stream (hipFree, hipHostFree, hipIpcCloseMemHandle) are deferred while any
 * live communicator has device work pending and run at the next lifecycle
 * call that finds the process quiet.  Returns how many are still deferred
 * (test support). */
int mx_release_pending(void);

/* IPC regions of destroyed communicators waiting for every peer's BYE
 * before reuse, and groups given up on (a peer that never destroyed the
 * communicator: after 64 scans, or beyond 32 groups, a group stays allocated
 * and unused).  Test support. */
int mx_ipc_quarantine_stats(int *held, unsigned long long *abandoned);

/* One-shot allreduce (one kernel: push, flag, fold) up to `max_bytes` per
 * rank; clamped to the one-shot slot capacity reserved at creation (1 MiB or
 * staging / (8 n); MX_ONESHOT_MAX at creation sets both).  0 = off.  Same
 * value on every rank.  Returns the crossover in force (bytes). */
long long mx_comm_set_oneshot_max(mx_comm_t *comm, size_t max_bytes);

/* Autotuning of the data movement (default on when the registration page
 * exists and neither MX_ALLREDUCE_PROTO nor MX_REG_MIN forces a path;
 * MX_AUTOTUNE=0 switches it off).  Per collective and power-of-two size
 * class of blocking calls, the first call runs candidate 0 as a warm-up, the
 * next ones time each candidate (3 runs each below 4 MiB, the fastest
 * counts), on the host, with the maximum over ranks exchanged through the
 * registration page; the fastest candidate is kept for that class:
 *   allreduce, from 64 KiB per rank: 0 zero-copy, 1 staged PULL, 2 staged
 *     PUSH, 3 one-shot (size classes up to the one-shot slot capacity,
 *     1 MiB or staging / (8 n));
 *   reduce_scatter, allgather, from 256 KiB: 0 zero-copy, 1 staged;
 *   bcast (n > 2), from 64 KiB: 0 zero-copy, 1 scatter + allgather, 2 direct.
 * Results are identical on every path.  mx_comm_get_tuning_ex returns the
 * choice of collective `coll` (MX_TUNE_*) for a message size, or -1 while
 * untuned; mx_comm_get_tuning is the allreduce's.  Same setting on every
 * rank. */
enum { MX_TUNE_ALLREDUCE = 0, MX_TUNE_REDUCE_SCATTER = 1, MX_TUNE_ALLGATHER = 2, MX_TUNE_BCAST = 3 };
int mx_comm_set_autotune(mx_comm_t *comm, int on);
int mx_comm_get_tuning(const mx_comm_t *comm, size_t bytes);
int mx_comm_get_tuning_ex(const mx_comm_t *comm, int coll, size_t bytes);

/* Per-communicator kernel timing (HIP events on the collective's stream),
 * off by default.  Times are summed over calls since the last reset. */
typedef struct mx_coll_stats {
    uint64_t calls;            /* collective calls                          */
    uint64_t fold_launches;    /* fused fold kernels                        */
    double fold_ms;            /* device time of the fold kernels           */
    double fold_bytes;         /* algorithmic bytes: n reads + ndst writes  */
    double push_ms;            /* scatter-push copies to peers' staging     */
    double gather_ms;          /* gather-area -> rbuf copies                */
    double total_ms;           /* first -> last event of each call          */
    /* counted whether or not profiling is on: */
    uint64_t zero_copy_calls;  /* allreduces folded between registered user
                                  buffers (no staging copies)               */
    uint64_t staged_calls;     /* allreduces through the staging chunks     */
    uint64_t direct_calls;     /* zero-copy allreduces whose results went
                                  straight into the peers' rbufs            */
    uint64_t reg_fast_calls;   /* registration exchanges that found every
                                  rank's buffers as in the last one (one
                                  host round instead of two)                */
    uint64_t p2p_relaunches;   /* receive launches that yielded to receives
                                  posted after them and were launched again */
    uint64_t p2p_pulls;        /* rendezvous receives pulled straight from the
                                  sender's buffer (single copy)             */
    uint64_t service_calls;    /* small allreduces served by the resident
                                  service (no launch)                       */
    uint64_t reg_stale_refused; /* zero-copy imports refused: the runtime
                                  handed back the import of a peer's freed
                                  allocation (the call took the staged path) */
} mx_coll_stats_t;
/* The resident small-allreduce service (csrc/mx_coll_svc.hip): commands served
 * and kernel launches so far in this process; returns 1 usable, 0 before first
 * use, -1 off.  mx_coll_service_set turns it on or off at run time (overrides
 * MX_COLL_SERVICE; off stops a running service). */
int mx_coll_service_stats(unsigned long long *served, unsigned long long *launches);
int mx_coll_service_set(int on);
/* Where a served call's time goes, means over the served calls (microseconds):
 * out[0] calls, [1] host preparation, [2] host wait from the post to `done`,
 * and the kernel's phases [3] arguments (the command line, and the
 * arguments block when the call carried it), [4] the peers' gen-2 check,
 * [5] the push issued, [6] the gather of the peers' words, [7] the fold,
 * [8] DONE and the result words acknowledged; [9] commands that carried the
 * arguments block (a count).  Fills min(n, 10) entries. */
int mx_coll_service_trace(double *out, int n);
int mx_comm_set_profiling(mx_comm_t *comm, int on);
int mx_comm_get_stats(mx_comm_t *comm, mx_coll_stats_t *stats, int reset);

/* Algorithm words.  The low byte selects the algorithm.  The algorithms
 * built on a rooted reduce -- allreduce NONOVERLAPPING (reduce to 0 + bcast,
 * coll_base_allreduce.c:54-86), reduce_scatter NONOVERLAPPING (reduce to 0 +
 * scatterv, coll_base_reduce_scatter.c:47-110), reduce_scatter_block and the
 * rooted reduce itself -- take the reduce algorithm the communicator's
 * coll_reduce would run from bits 8-15 (MX_REDUCE_*, 0 = the tuned fixed
 * decision; for mx_reduce / mx_reduce_scatter_block it is the low byte) and
 * the fanout of the chain tree (MX_REDUCE_CHAIN) from bits 16-23 (0 = 4,
 * coll_tuned's default chain fanout, coll_tuned_component.c:56) -- what
 * coll_tuned_reduce_algorithm[_chain_fanout] choose in the reference. */
#define MX_ALG_WORD(alg, reduce_alg, chain_fanout) \
    ((int)(alg) | ((int)(reduce_alg) << 8) | ((int)(chain_fanout) << 16))

/* Allreduce algorithm ids == coll_tuned_allreduce_algorithm values
 * (ompi/mca/coll/tuned/coll_tuned_allreduce_decision.c:37-46). */
enum {
    MX_ALLREDUCE_AUTO = 0,           /* tuned fixed decision                 */
    MX_ALLREDUCE_BASIC_LINEAR = 1,
    MX_ALLREDUCE_NONOVERLAPPING = 2, /* rooted reduce to 0 + bcast           */
    MX_ALLREDUCE_RECURSIVE_DOUBLING = 3,
    MX_ALLREDUCE_RING = 4,
    MX_ALLREDUCE_SEGMENTED_RING = 5,
    MX_ALLREDUCE_RABENSEIFNER = 6,
    MX_ALLREDUCE_RCCL = 100          /* RCCL ncclAllReduce (order differs:
                                        FP results within tolerance only)  */
};
/* Reduce-scatter algorithm ids == coll_tuned_reduce_scatter_algorithm
 * (coll_tuned_reduce_scatter_decision.c:36-43). */
enum {
    MX_RS_AUTO = 0,
    MX_RS_NONOVERLAPPING = 1,        /* rooted reduce to 0 + scatterv        */
    MX_RS_RECURSIVE_HALVING = 2,
    MX_RS_RING = 3,
    MX_RS_BUTTERFLY = 4,             /* coll_base_reduce_scatter.c:691-880   */
    MX_RS_RCCL = 100
};

/* Rooted reduce algorithm ids == coll_tuned_reduce_algorithm values
 * (ompi/mca/coll/tuned/coll_tuned_reduce_decision.c:36-45). */
enum {
    MX_REDUCE_AUTO = 0,              /* tuned fixed decision (decision_fixed.c:354-429) */
    MX_REDUCE_LINEAR = 1,
    MX_REDUCE_CHAIN = 2,             /* fanout from bits 16-23 of the word, default
                                        MX_REDUCE_CHAIN_FANOUT (tuned's 4,
                                        coll_tuned_component.c:56) */
    MX_REDUCE_PIPELINE = 3,
    MX_REDUCE_BINARY = 4,
    MX_REDUCE_BINOMIAL = 5,
    MX_REDUCE_IN_ORDER_BINARY = 6,
    MX_REDUCE_RABENSEIFNER = 7       /* not provided: MX_ERR_UNSUPPORTED      */
};
#define MX_REDUCE_CHAIN_FANOUT 4
/* Scan / exscan algorithm ids == coll_tuned_{scan,exscan}_algorithm
 * (coll_tuned_scan_decision.c:29-33).  AUTO = linear: coll/tuned leaves
 * the scan slots empty (coll_tuned_module.c:106,112), so coll/basic's
 * linear scan / exscan run (coll_basic_scan.c:43-50, coll_basic_exscan.c:45-52). */
enum { MX_SCAN_AUTO = 0, MX_SCAN_LINEAR = 1, MX_SCAN_RECURSIVE_DOUBLING = 2 };

/* Returns the algorithm MX_ALLREDUCE_AUTO resolves to for this call shape
 * (the tuned fixed decision), for introspection and tests. */
int mx_allreduce_decision(int comm_size, size_t count, int type);
int mx_reduce_scatter_decision(int comm_size, size_t total_count, int type);
int mx_reduce_decision(int comm_size, size_t count, int type);

/* ---- multi-process (or local rank 0 of a local comm: use *_local) ------- */
int mx_allreduce(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t count,
                 int type, int op, int alg, void *stream);
int mx_reduce_scatter(mx_comm_t *comm, const void *sbuf, void *rbuf,
                      const size_t *rcounts, int type, int op, int alg, void *stream);
/* Contiguous byte allgather: rank r's `bytes` land at rbuf + r*bytes. */
int mx_allgather(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t bytes, void *stream);
int mx_bcast(mx_comm_t *comm, void *buf, size_t bytes, int root, void *stream);

/* Rooted reduce (coll slot `reduce`, coll.h:239-241): the result lands in
 * rbuf on `root` only (rbuf may be NULL elsewhere); sbuf MPI_IN_PLACE on
 * the root.  Bit-identical to the reference algorithm `alg` (the tree of
 * coll_base_topo.c, the operand roles of coll_base_reduce.c:143-240). */
int mx_reduce(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
              int root, int alg, void *stream);
/* Inclusive / exclusive prefix reductions (slots `scan`, `exscan`,
 * coll.h:228-230, 248-250).  exscan leaves rank 0's rbuf untouched. */
int mx_scan(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
            int alg, void *stream);
int mx_exscan(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
              int alg, void *stream);
/* MPI_Reduce_scatter_block (slot coll.h:245-247): rank r receives block r
 * (rcount elements) of the reduction, folded as coll/tuned's basic_linear
 * does it (reduce to rank 0 with the reduce algorithm `alg`, then scatter). */
int mx_reduce_scatter_block(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t rcount,
                            int type, int op, int alg, void *stream);

/* ---- non-blocking and persistent collectives ----------------------------
 * Replace, for device buffers, coll/libnbc's slots (coll.h:261-338 i<coll>,
 * :339-420 <coll>_init; ompi/mca/coll/libnbc/nbc_i*.c).  The collective is
 * enqueued on `stream` exactly like the blocking call but the call returns
 * at once: the GPU progresses every step itself (device-side flag waits),
 * nothing needs host progress calls.  A request completes when its last
 * kernel has run.  Collectives of one communicator execute in issue order
 * even across streams (MPI ordering); buffers must not be touched until
 * completion.  Reduction orders are libnbc's (its algorithm numbering and
 * default rule below), so results are bit-identical to MPI_I<coll> on the
 * reference.  Persistent requests (*_init, MPI-4) are created inactive and
 * run on every mx_start. */
typedef struct mx_request mx_request_t;
/* coll_libnbc_iallreduce_algorithm (coll_libnbc_component.c:58-64) */
enum {
    MX_IALLREDUCE_AUTO = 0,          /* libnbc rule (nbc_iallreduce.c:113-121)  */
    MX_IALLREDUCE_RING = 1,
    MX_IALLREDUCE_BINOMIAL = 2,
    MX_IALLREDUCE_RABENSEIFNER = 3,
    MX_IALLREDUCE_RECURSIVE_DOUBLING = 4
};
/* coll_libnbc_ireduce_algorithm (coll_libnbc_component.c:87-92) */
enum {
    MX_IREDUCE_AUTO = 0,             /* libnbc rule (nbc_ireduce.c:107-116)     */
    MX_IREDUCE_CHAIN = 1,
    MX_IREDUCE_BINOMIAL = 2,
    MX_IREDUCE_RABENSEIFNER = 3
};
/* iscan / iexscan: MX_SCAN_* (== coll_libnbc_i{scan,exscan}_algorithm:
 * 1 linear, 2 recursive doubling; AUTO = linear). */
int mx_iallreduce_decision(int comm_size, size_t count, int type, int inplace);
int mx_ireduce_decision(int comm_size, size_t count, int type);

int mx_iallreduce(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
                  int alg, void *stream, mx_request_t **req);
int mx_ireduce(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
               int root, int alg, void *stream, mx_request_t **req);
int mx_ireduce_scatter(mx_comm_t *comm, const void *sbuf, void *rbuf, const size_t *rcounts,
                       int type, int op, void *stream, mx_request_t **req);
int mx_ireduce_scatter_block(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t rcount,
                             int type, int op, void *stream, mx_request_t **req);
int mx_iscan(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
             int alg, void *stream, mx_request_t **req);
int mx_iexscan(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
               int alg, void *stream, mx_request_t **req);
int mx_iallgather(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t bytes, void *stream,
                  mx_request_t **req);
int mx_ibcast(mx_comm_t *comm, void *buf, size_t bytes, int root, void *stream, mx_request_t **req);

int mx_allreduce_init(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
                      int alg, void *stream, mx_request_t **req);
int mx_reduce_init(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
                   int root, int alg, void *stream, mx_request_t **req);
int mx_reduce_scatter_init(mx_comm_t *comm, const void *sbuf, void *rbuf, const size_t *rcounts,
                           int type, int op, void *stream, mx_request_t **req);
int mx_reduce_scatter_block_init(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t rcount,
                                 int type, int op, void *stream, mx_request_t **req);
int mx_scan_init(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
                 int alg, void *stream, mx_request_t **req);
int mx_exscan_init(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t count, int type, int op,
                   int alg, void *stream, mx_request_t **req);
int mx_allgather_init(mx_comm_t *comm, const void *sbuf, void *rbuf, size_t bytes, void *stream,
                      mx_request_t **req);
int mx_bcast_init(mx_comm_t *comm, void *buf, size_t bytes, int root, void *stream, mx_request_t **req);

/* MPI_Start / MPI_Startall (persistent requests only). */
int mx_start(mx_request_t *req);
int mx_startall(size_t n, mx_request_t *const *reqs);
/* MPI_Test / MPI_Wait: flag = 1 once complete (also for an inactive
 * persistent request); the return value is the operation's status. */
int mx_test(mx_request_t *req, int *flag);
int mx_wait(mx_request_t *req);
/* MPI_Waitall / MPI_Waitany / MPI_Testall / MPI_Testany over an array of
 * requests (ompi_request_default_wait_all / _wait_any, ompi/request/
 * req_wait.c:84-383; _test_any / _test_all, req_test.c:105-294).  Null and
 * inactive entries are skipped; completed requests become inactive (free them
 * with mx_request_free, as after mx_wait).  Waitall completes every request
 * and returns the first error among them.  Waitany / Testany: *index of the
 * request completed, MX_UNDEFINED when none is active (Testany: *flag = 1
 * then).  Testall completes the requests only when every one is complete
 * (*flag = 1); otherwise nothing changes.  Every pass progresses yielded
 * receives. */
#define MX_UNDEFINED (-32766)   /* MPI_UNDEFINED, mpi.h.in:488 */
int mx_waitall(size_t n, mx_request_t *const *reqs);
int mx_waitany(size_t n, mx_request_t *const *reqs, int *index);
int mx_testall(size_t n, mx_request_t *const *reqs, int *flag);
int mx_testany(size_t n, mx_request_t *const *reqs, int *index, int *flag);
/* Make `stream` wait for the request on the device, without a host wait. */
int mx_request_stream_wait(mx_request_t *req, void *stream);
int mx_request_is_active(const mx_request_t *req);
/* MPI_Request_free: an active request is completed first. */
int mx_request_free(mx_request_t *req);

/* ---- point-to-point on device buffers ------------------------------------
 * MPI_Send / MPI_Recv / MPI_Isend / MPI_Irecv / MPI_Sendrecv /
 * MPI_Send_init / MPI_Recv_init between ranks of a multi-process
 * communicator (the role btl/smcuda + common/cuda play for CUDA buffers:
 * opal/mca/btl/smcuda, common_cuda.c:1008-1180; non-contiguous layouts via
 * the device convertor, as the convertor CUDA hooks do,
 * opal_datatype_cuda.c:44-140).  Each message streams through a mailbox the
 * receiver owns (mapped at communicator creation) under device-side flow
 * control; no host progress, no per-message IPC.  Work starts after what
 * `stream` had queued; completion is through the request (blocking forms
 * return complete).  Matching is in order per (source, destination) pair;
 * the envelope tag is checked (MX_ERR_TAG on a mismatch, tag < 0 = any);
 * a longer message than the receive buffer delivers what fits and
 * completes with MX_ERR_TRUNCATE.  `received` / mx_request_status: bytes
 * delivered and the envelope tag.  A receive may name MX_ANY_SOURCE
 * (MPI_ANY_SOURCE): it matches the next unconsumed message of whichever
 * source has one (per-pair order is kept); mx_request_source gives the
 * matched source (MPI_SOURCE). */
#define MX_ANY_SOURCE (-1)
int mx_send(mx_comm_t *comm, const void *buf, size_t bytes, int dst, int tag, void *stream);
int mx_recv(mx_comm_t *comm, void *buf, size_t bytes, int src, int tag, void *stream, size_t *received);
int mx_isend(mx_comm_t *comm, const void *buf, size_t bytes, int dst, int tag, void *stream,
             mx_request_t **req);
int mx_irecv(mx_comm_t *comm, void *buf, size_t bytes, int src, int tag, void *stream, mx_request_t **req);
int mx_send_init(mx_comm_t *comm, const void *buf, size_t bytes, int dst, int tag, void *stream,
                 mx_request_t **req);
int mx_recv_init(mx_comm_t *comm, void *buf, size_t bytes, int src, int tag, void *stream,
                 mx_request_t **req);
int mx_sendrecv(mx_comm_t *comm, const void *sbuf, size_t sbytes, int dst, int stag, void *rbuf,
                size_t rbytes, int src, int rtag, void *stream, size_t *received);
/* `count` instances of a derived datatype (mx_convertor.h) at `buf`. */
int mx_isend_ddt(mx_comm_t *comm, const void *buf, size_t count, const struct mx_ddt *ddt, int dst,
                 int tag, void *stream, mx_request_t **req);
int mx_irecv_ddt(mx_comm_t *comm, void *buf, size_t count, const struct mx_ddt *ddt, int src,
                 int tag, void *stream, mx_request_t **req);
int mx_request_status(const mx_request_t *req, size_t *bytes, int *tag);
int mx_request_source(const mx_request_t *req, int *source);

/* ---- OpenSHMEM reductions (shmem_<type>_<op>_to_all) --------------------
 * The OSHMEM op/type numbering (oshmem/op/op.h: OSHMEM_OP_AND..PROD,
 * OSHMEM_OP_TYPE_SHORT..FREAL16).  mx_shmem_to_mpi restates scoll/mpi's
 * mapping onto an MPI op + datatype (oshmem/mca/scoll/mpi/
 * scoll_mpi_dtypes.h: shmem_dtype_to_ompi_dtype / shmem_op_to_ompi_op;
 * integer types map by dt_size: 8/16/32/64 bits), which then runs as a
 * coll allreduce (scoll_mpi_ops.c:212-275). */
enum { MX_SHMEM_AND, MX_SHMEM_OR, MX_SHMEM_XOR, MX_SHMEM_MAX, MX_SHMEM_MIN, MX_SHMEM_SUM, MX_SHMEM_PROD };
enum { MX_SHMEM_SHORT, MX_SHMEM_INT, MX_SHMEM_LONG, MX_SHMEM_LLONG, MX_SHMEM_INT16, MX_SHMEM_INT32,
       MX_SHMEM_INT64, MX_SHMEM_FLOAT, MX_SHMEM_DOUBLE, MX_SHMEM_LDOUBLE, MX_SHMEM_FCOMPLEX,
       MX_SHMEM_DCOMPLEX, MX_SHMEM_FINT2, MX_SHMEM_FINT4, MX_SHMEM_FINT8, MX_SHMEM_FREAL4,
       MX_SHMEM_FREAL8, MX_SHMEM_FREAL16 };
int mx_shmem_to_mpi(int shmem_op, int shmem_type, size_t dt_size, int *mx_op, int *mx_type);
/* target[i] = reduction over the active set of source[i], i < nreduce
 * (target may equal source).  Runs mx_allreduce with the tuned decision,
 * exactly what scoll/mpi asks of coll/tuned (mca_scoll_mpi_reduce,
 * scoll_mpi_ops.c:212-275); above INT_MAX elements scoll/mpi falls back to
 * the previous scoll module (:246-259), and so does this call:
 * mx_shmem_reduce_basic. */
int mx_shmem_reduce(mx_comm_t *comm, int shmem_op, int shmem_type, size_t dt_size, void *target,
                    const void *source, size_t nreduce, void *stream);
/* scoll/basic's reduce on the device, its default recursive-doubling order
 * (oshmem/mca/scoll/basic/scoll_basic_reduce.c:374-542): every PE folds the
 * partner's value into its own, so for MAX / MIN with NaNs or signed zeros
 * the PEs' results can differ, as they do in the reference.  FINT2 folds
 * 2-byte integers (the reference's scoll/basic applies integer4 functions
 * there and overruns its buffers, oshmem/op/op.c:195; not reproduced). */
int mx_shmem_reduce_basic(mx_comm_t *comm, int shmem_op, int shmem_type, size_t dt_size, void *target,
                          const void *source, size_t nreduce, void *stream);

/* ---- device symmetric heap (OpenSHMEM on device memory) ------------------
 * Replaces, for GPU-resident symmetric data, the host-only symmetric heap of
 * oshmem/mca/sshmem + oshmem/mca/memheap (device addresses fail
 * RUNTIME_CHECK_ADDR today, oshmem/runtime/runtime.h:205-210).  Collective
 * over `comm` (same `bytes` on every PE): each PE allocates its heap in
 * device memory and maps every peer's.  mx_shmalloc / mx_shfree are
 * collective too (same call sequence on every PE -> same offsets). */
typedef struct mx_heap mx_heap_t;
int mx_heap_create(mx_comm_t *comm, size_t bytes, mx_heap_t **heap);
int mx_heap_destroy(mx_heap_t *heap);
void *mx_heap_base(const mx_heap_t *heap);
void *mx_shmalloc(mx_heap_t *heap, size_t bytes);
int mx_shfree(mx_heap_t *heap, void *ptr);
/* shmem_ptr (oshmem/shmem/c/shmem_ptr.c:32-70): `addr` as PE `pe`'s array,
 * directly loadable/storable by kernels on this GPU; NULL if not symmetric. */
void *mx_shmem_ptr(const mx_heap_t *heap, const void *addr, int pe);
/* shmem_putmem / shmem_getmem (blocking; device copies over xGMI). */
int mx_shmem_putmem(mx_heap_t *heap, void *dest, const void *src, size_t bytes, int pe, void *stream);
int mx_shmem_getmem(mx_heap_t *heap, void *dest, const void *src, size_t bytes, int pe, void *stream);
int mx_shmem_barrier_all(mx_heap_t *heap, void *stream);
/* shmem_<type>_<op>_to_all (shmem_reduce.c:29-65) on symmetric target and
 * source over the active set (PE_start, logPE_stride, PE_size): every member
 * folds its element part straight from all members' sources into all
 * members' targets (no staging), in the order coll/tuned gives scoll/mpi's
 * allreduce on the active set, i.e. bit-identical to mx_shmem_reduce. */
int mx_shmem_reduce_heap(mx_heap_t *heap, int shmem_op, int shmem_type, size_t dt_size, void *target,
                         const void *source, size_t nreduce, int pe_start, int log_pe_stride,
                         int pe_size, void *stream);

/* ---- one-sided accumulate on the symmetric heap ---------------------------
 * MPI_Accumulate / MPI_Get_accumulate / MPI_Fetch_and_op /
 * MPI_Compare_and_swap (osc/rdma: osc_rdma_accumulate.c:121-251, 770-1100;
 * ompi_osc_base_sndrcv_op, osc_base_obj_convert.c:160-253) with the target
 * at the symmetric address `target` of PE `pe`: target = origin OP target
 * element-wise (ompi_op_reduce(op, origin, target)), op MX_OP_REPLACE /
 * MX_OP_NO_OP included.  Accumulates to one PE are serialised by an
 * exclusive device lock in that PE's heap (MPI's per-element atomicity);
 * get_accumulate / fetch_and_op return the value before the update in
 * `result` (local device memory).  Calls complete before returning. */
int mx_accumulate(mx_heap_t *heap, const void *origin, size_t count, int type, int op, int pe, void *target,
                  void *stream);
int mx_get_accumulate(mx_heap_t *heap, const void *origin, void *result, size_t count, int type, int op, int pe,
                      void *target, void *stream);
int mx_fetch_and_op(mx_heap_t *heap, const void *origin, void *result, int type, int op, int pe, void *target,
                    void *stream);
int mx_compare_and_swap(mx_heap_t *heap, const void *origin, const void *compare, void *result, int type, int pe,
                        void *target, void *stream);
/* Derived datatypes (mx_convertor.h) on either side, NULL = contiguous
 * elements of `type`; both sides hold the same number of `type` elements,
 * matched in type-map order. */
int mx_accumulate_ddt(mx_heap_t *heap, const void *origin, size_t origin_count, const struct mx_ddt *origin_ddt,
                      int type, int op, int pe, void *target, size_t target_count, const struct mx_ddt *target_ddt,
                      void *stream);

/* ---- local communicator: arrays of `size` buffers, one per rank --------- */
int mx_allreduce_local(mx_comm_t *comm, const void *const *sbufs, void *const *rbufs,
                       size_t count, int type, int op, int alg, void *stream);
int mx_reduce_scatter_local(mx_comm_t *comm, const void *const *sbufs, void *const *rbufs,
                            const size_t *rcounts, int type, int op, int alg, void *stream);
int mx_allgather_local(mx_comm_t *comm, const void *const *sbufs, void *const *rbufs,
                       size_t bytes, void *stream);
int mx_bcast_local(mx_comm_t *comm, void *const *bufs, size_t bytes, int root, void *stream);
int mx_reduce_local(mx_comm_t *comm, const void *const *sbufs, void *const *rbufs, size_t count,
                    int type, int op, int root, int alg, void *stream);
int mx_scan_local(mx_comm_t *comm, const void *const *sbufs, void *const *rbufs, size_t count,
                  int type, int op, int alg, void *stream);
int mx_exscan_local(mx_comm_t *comm, const void *const *sbufs, void *const *rbufs, size_t count,
                    int type, int op, int alg, void *stream);
int mx_reduce_scatter_block_local(mx_comm_t *comm, const void *const *sbufs, void *const *rbufs,
                                  size_t rcount, int type, int op, int alg, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* MX_COLL_H */
