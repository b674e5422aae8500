/*
 * coll_mi355x.c -- the `mi355x` component of Open MPI's `coll` framework.
 *
 * Takes the allreduce / reduce_scatter / allgather / bcast slots (plus
 * reduce / reduce_scatter_block / scan / exscan, their nonblocking and
 * persistent forms and, above coll/self's priority, reduce_local) of a
 * communicator and runs them on the MI355X all-peer path of
 * libmx_kernels.so (include/mx_coll.h).
 *
 * Follows the reference's stacking accelerator component, coll/cuda:
 *  - comm_query returns a module with only the slots we implement
 *    (coll_cuda_module.c:79-117); priority 80 by default (above tuned's 30
 *    and coll/cuda's 78, and above coll/self's 75 for reduce_local), MCA var
 *    coll_mi355x_priority;
 *  - module_enable saves and RETAINs the previous c_coll slot + module for
 *    delegation (CHECK_AND_RETAIN, coll_cuda_module.c:120-155) and fails with
 *    OMPI_ERR_NOT_FOUND if a needed lower slot is missing.
 *
 * Every rank of a communicator must run the same protocol, so whether a call
 * takes the device path depends only on what MPI requires to match across
 * ranks -- the op, the type signature, the counts, the root -- and on state
 * all ranks agreed on (the device communicator, created collectively at the
 * first eligible call).  Where the buffers live does NOT enter the decision:
 * coll/cuda makes the same point the other way round (every rank stages its
 * device buffers through the host and calls the same lower collective,
 * coll_cuda_allreduce.c:30-73).  Here a rank whose buffer is host memory (or
 * a non-contiguous layout) stages it through device scratch; device buffers
 * are used in place.
 *
 * Size split and order (round 3).  A call of at most coll_mi355x_host_max_kb
 * (default 64 KiB: count x type size, the same on every rank) runs on the
 * saved host module -- device buffers are copied to host memory around it,
 * coll/cuda's direction (coll_cuda_allreduce.c:30-73) -- so a host-only
 * program never touches the GPU and small device calls get the host's
 * latency.  Larger calls run on the device with the reduction order of the
 * module they replaced: coll/tuned's fixed decision, or its forced algorithm
 * / rules file when coll_tuned_use_dynamic_rules is set
 * (coll_mi355x_rules.c); coll/basic's compositions (allreduce = coll_reduce
 * to 0 + coll_bcast, coll_basic_allreduce.c:45-71; linear reduce up to
 * coll_basic_crossover ranks; recursive-halving reduce_scatter below 8 MiB,
 * coll_basic_reduce_scatter.c:107-108).  Whatever the device cannot
 * reproduce bit for bit (an unknown lower module, coll/basic's log-tree
 * reduce, tuned's redscat_gather reduce, RSB algorithms 2-4) runs on the
 * saved module the same way small calls do.  Intercommunicators are declined
 * at query (coll_tuned_module.c:66-69).
 *
 * Blocking collectives run on a stream the module owns, created blocking
 * (mx_stream_create_ordered): implicitly ordered with the legacy default
 * stream, with no event per call.  Nonblocking and persistent requests run
 * on a second, non-blocking high-priority stream (mx_stream_create), so a
 * request waiting for a late peer never stalls the default stream.
 * Peer waits are unbounded by default (a peer may legally arrive arbitrarily
 * late); coll_mi355x_wait_timeout bounds them, and a timeout poisons the
 * communicator (include/mx_coll.h).
 *
 * The nonblocking and persistent slots (iallreduce, ireduce, ireduce_scatter,
 * ireduce_scatter_block, iscan, iexscan, iallgather, ibcast and their
 * *_init forms) replace coll/libnbc's: the collective is enqueued on the GPU
 * and the request completes through a progress callback that polls its event
 * (libnbc's ompi_coll_libnbc_progress, coll_libnbc_component.c:426-482,
 * progresses the schedule on the host instead); reduction orders are
 * libnbc's, algorithm selection follows the coll_libnbc_<coll>_algorithm vars
 * (coll_mi355x_<coll>_algorithm wins).  The blocking algorithm is chosen with
 * coll/tuned's fixed decision (coll_tuned_decision_fixed.c:44-95, :466-512)
 * unless forced with coll_mi355x_allreduce_algorithm /
 * coll_mi355x_reduce_scatter_algorithm (coll_tuned_*_algorithm numbering), so
 * results match coll/tuned bit for bit.
 */
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mx_coll.h"
#include "mx_convertor.h"
#include "mx_kernels.h"
#include "mx_ompi_abi.h"
#include "coll_mi355x_rules.h"

/* device scratch a staged buffer lives in (grown on demand, kept); the
 * pinned host copies of device buffers for the saved module likewise */
typedef struct { void *p; size_t bytes; } mx_scratch_t;
enum { SCR_IN, SCR_OUT, SCR_N };

/* the module a saved slot came from: its reduction order */
enum { LOW_TUNED = 1, LOW_BASIC, LOW_LIBNBC, LOW_OTHER };

/* device convertor handles of the datatypes this communicator moved, keyed
 * by the datatype AND a copy of its committed records (a freed datatype's
 * address may come back as another type) */
typedef struct {
    struct ompi_datatype_t *dt;
    void *recs;
    size_t nrec, size;
    ptrdiff_t lb, ub;
    mx_ddt_t *h;
    unsigned long used;
} mx_ddt_slot_t;
#define MX_DDT_CACHE 4

typedef struct {
    mca_coll_base_module_t super;
    struct ompi_communicator_t *comm;
    mx_comm_t *mx;
    int mx_state;         /* 0 not created yet, 1 ready, -1 unavailable (agreed by all ranks) */
    void *stream;         /* blocking collectives: module-owned stream ordered with the default one */
    void *nb_stream;      /* nonblocking / persistent requests: non-blocking stream */
    mx_scratch_t scratch[SCR_N];
    mx_scratch_t hbuf[SCR_N];   /* pinned host copies for the saved module */
    /* order of the saved reduction slots, coll/tuned's configuration, the
     * size split */
    int low_allreduce, low_reduce_scatter, low_reduce, low_rsb, low_scan, low_exscan, low_nbc;
    int basic_crossover;
    size_t host_max;
    mx_tuned_cfg_t tuned;
    mx_ddt_slot_t ddt[MX_DDT_CACHE];
    unsigned long ddt_clock;
    /* delegation targets (the slots we replaced) */
    mca_coll_base_module_allreduce_fn_t prev_allreduce;
    mca_coll_base_module_t *prev_allreduce_module;
    mca_coll_base_module_reduce_scatter_fn_t prev_reduce_scatter;
    mca_coll_base_module_t *prev_reduce_scatter_module;
    mca_coll_base_module_allgather_fn_t prev_allgather;
    mca_coll_base_module_t *prev_allgather_module;
    mca_coll_base_module_bcast_fn_t prev_bcast;
    mca_coll_base_module_t *prev_bcast_module;
    mca_coll_base_module_reduce_local_fn_t prev_reduce_local;
    mca_coll_base_module_t *prev_reduce_local_module;
    mca_coll_base_module_reduce_fn_t prev_reduce;
    mca_coll_base_module_t *prev_reduce_module;
    mca_coll_base_module_reduce_scatter_block_fn_t prev_reduce_scatter_block;
    mca_coll_base_module_t *prev_reduce_scatter_block_module;
    mca_coll_base_module_scan_fn_t prev_scan;
    mca_coll_base_module_t *prev_scan_module;
    mca_coll_base_module_exscan_fn_t prev_exscan;
    mca_coll_base_module_t *prev_exscan_module;
    /* nonblocking / persistent delegation targets (coll/libnbc); a slot the
     * lower modules do not provide is left to them (not installed) */
#define MX_PREV_SLOT(T, name) T prev_##name; mca_coll_base_module_t *prev_##name##_module;
    MX_PREV_SLOT(mca_coll_base_module_iallreduce_fn_t, iallreduce)
    MX_PREV_SLOT(mca_coll_base_module_ireduce_fn_t, ireduce)
    MX_PREV_SLOT(mca_coll_base_module_ireduce_scatter_fn_t, ireduce_scatter)
    MX_PREV_SLOT(mca_coll_base_module_ireduce_scatter_block_fn_t, ireduce_scatter_block)
    MX_PREV_SLOT(mca_coll_base_module_iscan_fn_t, iscan)
    MX_PREV_SLOT(mca_coll_base_module_iexscan_fn_t, iexscan)
    MX_PREV_SLOT(mca_coll_base_module_iallgather_fn_t, iallgather)
    MX_PREV_SLOT(mca_coll_base_module_ibcast_fn_t, ibcast)
    MX_PREV_SLOT(mca_coll_base_module_allreduce_init_fn_t, allreduce_init)
    MX_PREV_SLOT(mca_coll_base_module_reduce_init_fn_t, reduce_init)
    MX_PREV_SLOT(mca_coll_base_module_reduce_scatter_init_fn_t, reduce_scatter_init)
    MX_PREV_SLOT(mca_coll_base_module_reduce_scatter_block_init_fn_t, reduce_scatter_block_init)
    MX_PREV_SLOT(mca_coll_base_module_scan_init_fn_t, scan_init)
    MX_PREV_SLOT(mca_coll_base_module_exscan_init_fn_t, exscan_init)
    MX_PREV_SLOT(mca_coll_base_module_allgather_init_fn_t, allgather_init)
    MX_PREV_SLOT(mca_coll_base_module_bcast_init_fn_t, bcast_init)
#undef MX_PREV_SLOT
} mx_coll_module_t;

#define MX_NB_SLOTS(X)                                                                                    \
    X(iallreduce) X(ireduce) X(ireduce_scatter) X(ireduce_scatter_block) X(iscan) X(iexscan) X(iallgather) \
    X(ibcast) X(allreduce_init) X(reduce_init) X(reduce_scatter_init) X(reduce_scatter_block_init)        \
    X(scan_init) X(exscan_init) X(allgather_init) X(bcast_init)

/* coll_mi355x_verbose > 0: device-path failures are reported on stderr */
static int g_verbose = -1;
static int map_rc(int rc)
{
    if (rc != MX_SUCCESS) {
        if (g_verbose < 0) g_verbose = mx_ompi_host ? mx_ompi_host->mca_int("coll_mi355x_verbose", 0) : 0;
        if (g_verbose > 0) fprintf(stderr, "coll/mi355x: %s (%d)\n", mx_strerror(rc), rc);
    }
    switch (rc) {
    case MX_SUCCESS: return OMPI_SUCCESS;
    case MX_ERR_NOMEM: return OMPI_ERR_OUT_OF_RESOURCE;
    case MX_ERR_UNSUPPORTED: return OMPI_ERR_NOT_SUPPORTED;
    default: return OMPI_ERROR;
    }
}

/* releases what the module holds; the object itself is freed by OBJ_RELEASE */
static void coll_module_destruct(mx_coll_module_t *m)
{
    if (m->mx) mx_comm_destroy(m->mx);
    for (int k = 0; k < SCR_N; k++) {
        mx_free(m->scratch[k].p);
        mx_host_free(m->hbuf[k].p);
    }
    for (int k = 0; k < MX_DDT_CACHE; k++) {
        if (m->ddt[k].h) mx_ddt_destroy(m->ddt[k].h);
        free(m->ddt[k].recs);
    }
    if (m->stream) mx_stream_destroy(m->stream);
    if (m->nb_stream) mx_stream_destroy(m->nb_stream);
    if (m->prev_allreduce_module) MX_OBJ_RELEASE(m->prev_allreduce_module);
    if (m->prev_reduce_scatter_module) MX_OBJ_RELEASE(m->prev_reduce_scatter_module);
    if (m->prev_allgather_module) MX_OBJ_RELEASE(m->prev_allgather_module);
    if (m->prev_bcast_module) MX_OBJ_RELEASE(m->prev_bcast_module);
    if (m->prev_reduce_local_module) MX_OBJ_RELEASE(m->prev_reduce_local_module);
    if (m->prev_reduce_module) MX_OBJ_RELEASE(m->prev_reduce_module);
    if (m->prev_reduce_scatter_block_module) MX_OBJ_RELEASE(m->prev_reduce_scatter_block_module);
    if (m->prev_scan_module) MX_OBJ_RELEASE(m->prev_scan_module);
    if (m->prev_exscan_module) MX_OBJ_RELEASE(m->prev_exscan_module);
#define MX_RELEASE_PREV(name) if (m->prev_##name##_module) MX_OBJ_RELEASE(m->prev_##name##_module);
    MX_NB_SLOTS(MX_RELEASE_PREV)
#undef MX_RELEASE_PREV
}

MX_MODULE_CLASS(mx_coll_module_t, mca_coll_base_module_t, coll_module_destruct);

/* Bootstrap exchange for mx_comm_create: the saved host allgather on
 * MPI_BYTE buffers (host memory, so it never recurses into us). */
static int bootstrap_allgather(const void *send, void *recv, size_t bytes, void *ctx)
{
    mx_coll_module_t *m = (mx_coll_module_t *)ctx;
    if (bytes > INT_MAX) return -1;
    return m->prev_allgather(send, (int)bytes, mx_ompi_host->byte_dtype, recv, (int)bytes,
                             mx_ompi_host->byte_dtype, m->comm, m->prev_allgather_module);
}

/* The device communicator, created at the first call every rank found
 * eligible (eligibility only uses arguments MPI requires to match, so all
 * ranks get here in the same call).  mx_comm_create is itself collective and
 * either succeeds on every rank or on none, so mx_state agrees everywhere. */
static int comm_ready(mx_coll_module_t *m)
{
    if (m->mx_state) return m->mx_state > 0;
    const int n = mx_ompi_host->comm_size(m->comm), rank = mx_ompi_host->comm_rank(m->comm);
    const size_t staging = (size_t)mx_ompi_host->mca_int("coll_mi355x_staging_mb", 256) << 20;
    int flags = MX_COMM_IPC;
    if (mx_ompi_host->mca_int("coll_mi355x_rccl", 0)) flags |= MX_COMM_RCCL;
    int rc = mx_comm_create(rank, n, -1, staging, flags, bootstrap_allgather, m, &m->mx);
    if (rc == MX_SUCCESS) {
        const int t = mx_ompi_host->mca_int("coll_mi355x_wait_timeout", 0);
        rc = mx_comm_set_timeout(m->mx, t > 0 ? (double)t : 0.0);
    }
    if (rc == MX_SUCCESS) {
        /* MCA vars are job-wide, so every rank sets the same data path:
         * zero-copy from coll_mi355x_reg_min_kb per rank (0 = off; the
         * communicator declines it collectively when /dev/shm is missing),
         * staged protocol 0 auto / 1 push / 2 pull */
        const int kb = mx_ompi_host->mca_int("coll_mi355x_reg_min_kb", -1);
        (void)mx_comm_set_reg_min(m->mx, kb > 0 ? (size_t)kb << 10 : kb < 0 ? (size_t)256 << 10 : 0);
        const int proto = mx_ompi_host->mca_int("coll_mi355x_protocol", MX_PROTO_AUTO);
        if (mx_comm_set_protocol(m->mx, proto) < 0) rc = MX_ERR_ARG;
        /* data-movement autotuning of large allreduces (on by default); a
         * data path forced through MCA (protocol, registration threshold)
         * switches it off, as the environment overrides do */
        if (!mx_ompi_host->mca_int("coll_mi355x_autotune", 1) || proto != MX_PROTO_AUTO || kb >= 0)
            (void)mx_comm_set_autotune(m->mx, 0);
    }
    /* the streams are process-local: a failure here is reported by the calls
     * (or falls back to the default stream), never turned into a different
     * protocol on this rank */
    if (rc == MX_SUCCESS && !m->stream && mx_stream_create_ordered(&m->stream) != MX_SUCCESS) m->stream = NULL;
    if (rc == MX_SUCCESS && !m->nb_stream && mx_stream_create(&m->nb_stream) != MX_SUCCESS) m->nb_stream = NULL;
    if (rc != MX_SUCCESS) {
        if (m->mx) mx_comm_destroy(m->mx);
        m->mx = NULL;
        m->mx_state = -1;
        return 0;
    }
    m->mx_state = 1;
    return 1;
}

/* Blocking waits of the component (staging copies, reduce_local): through the
 * marker kernel's mapped completion word unless coll_mi355x_fast_sync = 0 */
static int g_fast_sync = -1;
static int stream_wait(void *s)
{
    if (g_fast_sync < 0) g_fast_sync = mx_ompi_host->mca_int("coll_mi355x_fast_sync", 1) != 0;
    return g_fast_sync ? mx_stream_sync_fast(s) : mx_stream_sync(s);
}

/* ---- staging of host / non-contiguous buffers ---------------------------- */

static int scratch(mx_coll_module_t *m, int k, size_t bytes, void **p)
{
    mx_scratch_t *s = &m->scratch[k];
    if (s->bytes < bytes) {
        mx_free(s->p);
        s->p = NULL;
        s->bytes = 0;
        const size_t want = bytes < ((size_t)1 << 20) ? ((size_t)1 << 20) : bytes;
        if (mx_alloc(want, &s->p) != MX_SUCCESS) return MX_ERR_NOMEM;
        s->bytes = want;
    }
    *p = s->p;
    return MX_SUCCESS;
}

/* A caller buffer as the device path sees it (`count` elements of `dt`):
 *  dev      what to hand to mx_* (the buffer itself if it is contiguous
 *           device memory, else scratch k);
 *  user     the caller's buffer, for the copy back (NULL: nothing to copy). */
typedef struct {
    void *dev, *user;
    size_t bytes;
    struct ompi_datatype_t *dt;
    int count, contiguous;
} xbuf_t;

/* the device convertor for dt (mx_ddt_create from the committed records),
 * or NULL when the host cannot describe it */
static mx_ddt_t *ddt_for(mx_coll_module_t *m, struct ompi_datatype_t *dt)
{
    const void *recs;
    size_t nrec, size;
    ptrdiff_t lb, ub;
    if (!mx_ompi_host->dtype_desc || mx_ompi_host->dtype_desc(dt, &recs, &nrec, &size, &lb, &ub) != OMPI_SUCCESS ||
        !nrec)
        return NULL;
    int victim = 0;
    for (int k = 0; k < MX_DDT_CACHE; k++) {
        mx_ddt_slot_t *e = &m->ddt[k];
        if (e->h && e->dt == dt && e->nrec == nrec && e->size == size && e->lb == lb && e->ub == ub &&
            !memcmp(e->recs, recs, nrec * 32)) {
            e->used = ++m->ddt_clock;
            return e->h;
        }
        if (e->used < m->ddt[victim].used) victim = k;
    }
    mx_ddt_slot_t *e = &m->ddt[victim];
    if (e->h) mx_ddt_destroy(e->h);
    free(e->recs);
    memset(e, 0, sizeof *e);
    if (!(e->recs = malloc(nrec * 32))) return NULL;
    memcpy(e->recs, recs, nrec * 32);
    if (mx_ddt_create(recs, nrec, NULL, size, (int64_t)lb, (int64_t)ub, &e->h) != MX_SUCCESS) {
        free(e->recs);
        memset(e, 0, sizeof *e);
        return NULL;
    }
    e->dt = dt;
    e->nrec = nrec;
    e->size = size;
    e->lb = lb;
    e->ub = ub;
    e->used = ++m->ddt_clock;
    return e->h;
}

/* contiguous bytes [0, bytes) of a non-contiguous layout <-> packed: on the
 * device for a device buffer whose datatype the host describes (the reference
 * would walk it with one cuMemcpy per block, opal_datatype_cuda.c:121-140),
 * else through the host convertor */
static int xfer_packed(mx_coll_module_t *m, const xbuf_t *x, void *packed_dev, int to_device)
{
    ptrdiff_t lo = 0, hi = 0;
    const int on_dev = mx_is_device_ptr(x->user) == 1;
    /* the packed length follows x->count: a staged rbuf that held the whole
     * input vector (MPI_IN_PLACE reduce_scatter) is copied back as its own
     * block only */
    const size_t len = (size_t)x->count * mx_ompi_host->dtype_size(x->dt);
    if (on_dev) {
        mx_ddt_t *h = ddt_for(m, x->dt);
        if (h) {
            int rc = to_device ? mx_pack(h, (size_t)x->count, x->user, packed_dev, 0, len, m->stream)
                               : mx_unpack(h, (size_t)x->count, x->user, packed_dev, 0, len, m->stream);
            return rc ? rc : stream_wait(m->stream);
        }
    }
    if (!mx_ompi_host->dtype_pack || !mx_ompi_host->dtype_unpack || !mx_ompi_host->dtype_span ||
        mx_ompi_host->dtype_span(x->dt, x->count, &lo, &hi) != OMPI_SUCCESS || hi < lo)
        return MX_ERR_UNSUPPORTED;
    char *span = NULL, *packed = malloc(len ? len : 1);
    char *user = (char *)x->user;
    int rc = packed ? MX_SUCCESS : MX_ERR_NOMEM;
    if (!rc && on_dev) {   /* the convertor walks host memory: bring the span over */
        span = malloc((size_t)(hi - lo) ? (size_t)(hi - lo) : 1);
        if (!span) rc = MX_ERR_NOMEM;
        else if (!(rc = mx_memcpy(span, user + lo, (size_t)(hi - lo), m->stream))) rc = stream_wait(m->stream);
        user = span - lo;
    }
    if (!rc && to_device) {
        if (mx_ompi_host->dtype_pack(x->dt, x->count, user, packed) != OMPI_SUCCESS) rc = MX_ERR_ARG;
        if (!rc) rc = mx_memcpy(packed_dev, packed, len, m->stream);
        if (!rc) rc = stream_wait(m->stream);
    } else if (!rc) {
        if (!(rc = mx_memcpy(packed, packed_dev, len, m->stream))) rc = stream_wait(m->stream);
        if (!rc && mx_ompi_host->dtype_unpack(x->dt, x->count, packed, user) != OMPI_SUCCESS) rc = MX_ERR_ARG;
        if (!rc && on_dev && !(rc = mx_memcpy((char *)x->user + lo, span, (size_t)(hi - lo), m->stream)))
            rc = stream_wait(m->stream);
    }
    free(span);
    free(packed);
    return rc;
}

/* stage `count` x `dt` at `user`; copy_in: the call reads it */
static int xin(mx_coll_module_t *m, int k, const void *user, struct ompi_datatype_t *dt, size_t count, int copy_in,
               xbuf_t *x)
{
    memset(x, 0, sizeof *x);
    x->bytes = count * mx_ompi_host->dtype_size(dt);
    x->dt = dt;
    x->count = count > INT_MAX ? INT_MAX : (int)count;
    x->contiguous = mx_ompi_host->dtype_contiguous(dt, x->count);
    if (x->contiguous && (!x->bytes || mx_is_device_ptr(user) == 1)) {
        x->dev = (void *)user;   /* in place: nothing to copy back */
        return MX_SUCCESS;
    }
    int rc = scratch(m, k, x->bytes, &x->dev);
    if (rc) return rc;
    x->user = (void *)user;
    if (!copy_in) return MX_SUCCESS;
    if (!x->contiguous) return xfer_packed(m, x, x->dev, 1);
    return mx_memcpy(x->dev, user, x->bytes, m->stream);
}

/* copy the first `bytes` of a staged result back to the caller */
static int xout(mx_coll_module_t *m, xbuf_t *x, size_t bytes)
{
    if (!x->user || !bytes) return MX_SUCCESS;
    if (!x->contiguous) return xfer_packed(m, x, x->dev, 0);
    int rc = mx_memcpy(x->user, x->dev, bytes, m->stream);
    return rc ? rc : stream_wait(m->stream);
}

/* The device work of a call starts after what the legacy default stream
 * already holds (the caller's kernels filling the buffers).  Blocking
 * collectives run on a blocking stream, which is ordered with the default
 * one implicitly; requests run on a non-blocking stream (a collective waiting
 * for a late peer must not hold up the default stream -- a PML's device copy,
 * say -- while the request is outstanding) and take an explicit event order
 * (~11 us of host time per post, profiles/r02/stream_probe.txt). */
static int begin(mx_coll_module_t *m)
{
    (void)m;
    return MX_SUCCESS;
}
static int begin_nb(mx_coll_module_t *m)
{
    return m->nb_stream ? mx_stream_order(m->nb_stream, NULL) : MX_SUCCESS;
}

/* reduction eligibility: intrinsic op with a kernel for the (predefined)
 * type -- identical on every rank for a correct MPI program */
static int reducible(struct ompi_datatype_t *dtype, struct ompi_op_t *op, size_t count, int n, int *slot, int *opi)
{
    *slot = mx_ompi_host->dtype_slot(dtype);
    *opi = mx_ompi_host->op_index(op);
    return count > 0 && n <= MX_MAX_RANKS && *slot >= 0 && (mx_ompi_host->op_flags(op) & OMPI_OP_FLAGS_INTRINSIC) &&
           mx_op_supported(*opi, *slot, MX_TABLE_WITH_FORTRAN);
}

/* ---- the saved module on host copies (coll/cuda's direction) -----------
 * A call the device does not take runs on the saved lower module.  That
 * module walks host memory, so a device buffer is copied to a host buffer
 * over its whole span (coll_cuda_allreduce.c:41-61 does the same with
 * opal_datatype_span) and an output is copied back after the call. */
typedef struct {
    void *user;        /* the caller's device buffer (NULL: used directly) */
    char *copy;        /* host copy of its span                            */
    ptrdiff_t lo;      /* span start relative to the buffer                */
    size_t span;
    int owned;         /* malloc'd (requests) vs the module's pinned buffer */
} hview_t;

static int ensure_stream(mx_coll_module_t *m)
{
    if (!m->stream && mx_stream_create_ordered(&m->stream) != MX_SUCCESS) m->stream = NULL;
    return MX_SUCCESS;
}

static int hbuf(mx_coll_module_t *m, int k, size_t bytes, void **p)
{
    mx_scratch_t *s = &m->hbuf[k];
    if (s->bytes < bytes) {
        mx_host_free(s->p);
        s->p = NULL;
        s->bytes = 0;
        const size_t want = bytes < ((size_t)64 << 10) ? ((size_t)64 << 10) : bytes;
        if (mx_host_alloc(want, &s->p) != MX_SUCCESS) return MX_ERR_NOMEM;
        s->bytes = want;
    }
    *p = s->p;
    return MX_SUCCESS;
}

/* The buffer the saved module gets for `user` (count x dt): the buffer itself
 * when it is host memory (or MPI_IN_PLACE / NULL), else a host copy of its
 * span -- module pinned buffer k, or malloc'd when k < 0 (a request's own) --
 * filled from the device when copy_in. */
static int hview_in(mx_coll_module_t *m, int k, const void *user, struct ompi_datatype_t *dt, size_t count,
                    int copy_in, hview_t *v, void **out)
{
    ptrdiff_t lo = 0, hi = (ptrdiff_t)(count * mx_ompi_host->dtype_size(dt));
    memset(v, 0, sizeof *v);
    *out = (void *)user;
    if (!user || user == MPI_IN_PLACE || !count || mx_is_device_ptr(user) != 1) return MX_SUCCESS;
    if (mx_ompi_host->dtype_span && mx_ompi_host->dtype_span(dt, (int)count, &lo, &hi) != OMPI_SUCCESS)
        return MX_ERR_UNSUPPORTED;
    if (hi < lo) return MX_ERR_UNSUPPORTED;
    v->span = (size_t)(hi - lo);
    void *p = NULL;
    if (k >= 0) {
        if (hbuf(m, k, v->span ? v->span : 1, &p)) return MX_ERR_NOMEM;
    } else if (!(p = malloc(v->span ? v->span : 1))) {
        return MX_ERR_NOMEM;
    }
    v->copy = p;
    v->owned = k < 0;
    v->user = (void *)user;
    v->lo = lo;
    *out = v->copy - lo;
    if (!copy_in || !v->span) return MX_SUCCESS;
    ensure_stream(m);
    int rc = mx_memcpy(v->copy, (const char *)user + lo, v->span, m->stream);
    return rc ? rc : stream_wait(m->stream);
}

/* the host copy of an output back into the caller's device buffer */
static int hview_out(mx_coll_module_t *m, const hview_t *v)
{
    if (!v->user || !v->span) return MX_SUCCESS;
    ensure_stream(m);
    int rc = mx_memcpy((char *)v->user + v->lo, v->copy, v->span, m->stream);
    return rc ? rc : stream_wait(m->stream);
}

static void hview_release(hview_t *v)
{
    if (v->owned) free(v->copy);
    v->copy = NULL;
    v->user = NULL;
}

/* the output view: copied in when the call reads it (MPI_IN_PLACE) or when
 * the copy-back must keep the bytes between its elements */
static int hview_out_in(mx_coll_module_t *m, int k, void *user, struct ompi_datatype_t *dt, size_t count,
                        int reads, hview_t *v, void **out)
{
    const int keep = reads || !mx_ompi_host->dtype_contiguous(dt, count > INT_MAX ? INT_MAX : (int)count);
    return hview_in(m, k, user, dt, count, keep, v, out);
}

/* ---- which reduction order the device must reproduce ---------------------
 * Each saved reduction slot is classified by its module's OPAL class name
 * (opal_object_t.obj_class->cls_name, OBJ_CLASS_INSTANCE in
 * coll_tuned_component.c:291, coll_basic_component.c:109,
 * coll_libnbc_component.c:504). */
static int low_kind(mca_coll_base_module_t *pm)
{
    const opal_object_t *o = (const opal_object_t *)pm;
    const char *nm = (o && o->obj_class) ? o->obj_class->cls_name : NULL;
    if (!nm) return LOW_OTHER;
    if (!strcmp(nm, "mca_coll_tuned_module_t")) return LOW_TUNED;
    if (!strcmp(nm, "mca_coll_basic_module_t")) return LOW_BASIC;
    if (!strcmp(nm, "ompi_coll_libnbc_module_t")) return LOW_LIBNBC;
    return LOW_OTHER;
}

static int comm_n(mx_coll_module_t *m) { return mx_ompi_host->comm_size(m->comm); }

/* The reduce word (MX_ALG_WORD: algorithm | chain fanout << 16) that this
 * communicator's coll_reduce -- this module's own reduce slot, i.e. the
 * saved module's order -- runs for count x es bytes; -1 when the device
 * cannot reproduce it. */
static int reduce_rule(mx_coll_module_t *m, size_t count, size_t es)
{
    switch (m->low_reduce) {
    case LOW_TUNED: {
        int fan;
        const int a = mx_tuned_choice(&m->tuned, MX_CT_REDUCE, count * es, &fan);
        if (a < 0 || a > MX_REDUCE_IN_ORDER_BINARY) return -1;   /* 7 redscat_gather: saved module */
        return a | ((a == MX_REDUCE_CHAIN && fan > 0 && fan < 256) ? fan << 16 : 0);
    }
    case LOW_BASIC:
        /* coll_basic_module.c:92-128: linear reduce up to coll_basic_crossover
         * ranks, the log-tree reduce above (not on the device) */
        return comm_n(m) <= m->basic_crossover ? MX_REDUCE_LINEAR : -1;
    default:
        return -1;
    }
}

static int nonoverlapping_word(int alg, int rw)
{
    return rw < 0 ? -1 : MX_ALG_WORD(alg, rw & 0xff, (rw >> 16) & 0xff);
}

/* the allreduce algorithm word, -1 = the saved module */
static int allreduce_rule(mx_coll_module_t *m, size_t count, size_t es, int slot)
{
    const int forced = mx_ompi_host->mca_int("coll_mi355x_allreduce_algorithm", MX_ALLREDUCE_AUTO);
    if (forced) return forced;   /* an explicit device algorithm (not the lower module's) */
    switch (m->low_allreduce) {
    case LOW_TUNED: {
        int fan;
        int a = mx_tuned_choice(&m->tuned, MX_CT_ALLREDUCE, count * es, &fan);
        if (a == 0 && mx_allreduce_decision(comm_n(m), count, slot) == MX_ALLREDUCE_NONOVERLAPPING)
            a = MX_ALLREDUCE_NONOVERLAPPING;
        if (a == MX_ALLREDUCE_NONOVERLAPPING) return nonoverlapping_word(a, reduce_rule(m, count, es));
        return (a >= 0 && a <= MX_ALLREDUCE_RABENSEIFNER) ? a : -1;
    }
    case LOW_BASIC:   /* coll_reduce to 0 + coll_bcast (coll_basic_allreduce.c:45-71) */
        return nonoverlapping_word(MX_ALLREDUCE_NONOVERLAPPING, reduce_rule(m, count, es));
    default:
        return -1;
    }
}

/* the reduce_scatter algorithm word for `total` elements, -1 = saved module */
static int reduce_scatter_rule(mx_coll_module_t *m, size_t total, size_t es, int inplace)
{
    const int forced = mx_ompi_host->mca_int("coll_mi355x_reduce_scatter_algorithm", MX_RS_AUTO);
    if (forced) return forced;
    switch (m->low_reduce_scatter) {
    case LOW_TUNED: {
        int fan;
        const int a = mx_tuned_choice(&m->tuned, MX_CT_REDUCESCATTER, total * es, &fan);
        if (a == MX_RS_NONOVERLAPPING) return nonoverlapping_word(a, reduce_rule(m, total, es));
        return (a >= 0 && a <= MX_RS_BUTTERFLY) ? a : -1;
    }
    case LOW_BASIC:
        /* coll_basic_reduce_scatter.c:107-108: recursive halving below
         * COMMUTATIVE_LONG_MSG (8 MiB), else coll_reduce (sbuf = rbuf when in
         * place, so the root never reduces in place) + scatterv */
        if (total * es < ((size_t)8 << 20)) return MX_RS_RECURSIVE_HALVING;
        return inplace ? -1 : nonoverlapping_word(MX_RS_NONOVERLAPPING, reduce_rule(m, total, es));
    default:
        return -1;
    }
}

/* reduce_scatter_block: basic_linear (tuned fixed, coll_tuned_decision_fixed.c:
 * 522-532; coll/basic, coll_basic_reduce_scatter_block.c:60) = coll_reduce
 * to 0 + scatter; the reduce word, -1 = saved module */
static int rsb_rule(mx_coll_module_t *m, size_t total, size_t es)
{
    const int forced = mx_ompi_host->mca_int("coll_mi355x_reduce_algorithm", MX_REDUCE_AUTO);
    if (forced) return forced;
    switch (m->low_rsb) {
    case LOW_TUNED: {
        int fan;
        const int a = mx_tuned_choice(&m->tuned, MX_CT_REDUCESCATTERBLOCK, total * es, &fan);
        return (a == 0 || a == 1) ? reduce_rule(m, total, es) : -1;   /* 2-4: saved module */
    }
    case LOW_BASIC:
        return reduce_rule(m, total, es);
    default:
        return -1;
    }
}

/* scan / exscan: MX_SCAN_*, -1 = saved module.  coll/tuned owns these slots
 * only with dynamic rules that name them (coll_tuned_module.c:235-238);
 * coll/basic's are linear (coll_basic_scan.c:43-50, coll_basic_exscan.c:45-52). */
static int scan_rule(mx_coll_module_t *m, size_t es, int exclusive)
{
    const int forced = mx_ompi_host->mca_int(exclusive ? "coll_mi355x_exscan_algorithm" : "coll_mi355x_scan_algorithm",
                                             MX_SCAN_AUTO);
    if (forced) return forced;
    switch (exclusive ? m->low_exscan : m->low_scan) {
    case LOW_TUNED: {
        int fan;
        const int a = mx_tuned_choice(&m->tuned, exclusive ? MX_CT_EXSCAN : MX_CT_SCAN, es * comm_n(m), &fan);
        return (a == 0 || a == 1) ? MX_SCAN_LINEAR : a == 2 ? MX_SCAN_RECURSIVE_DOUBLING : -1;
    }
    case LOW_BASIC:
        return MX_SCAN_LINEAR;
    default:
        return -1;
    }
}

/* a call of `bytes` (the same on every rank) for the device */
static int big(mx_coll_module_t *m, size_t bytes) { return bytes > m->host_max; }

/* ---- blocking slots -------------------------------------------------------- */

/* Blocking calls on the saved module, device buffers through host copies
 * (pinned buffers SCR_IN / SCR_OUT of the module). */
static int host_allreduce(mx_coll_module_t *m, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt,
                          struct ompi_op_t *op)
{
    hview_t s, r;
    void *hs, *hr;
    int rc = hview_in(m, SCR_IN, sbuf, dt, (size_t)count, 1, &s, &hs);
    if (!rc) rc = hview_out_in(m, SCR_OUT, rbuf, dt, (size_t)count, sbuf == MPI_IN_PLACE, &r, &hr);
    if (rc) return map_rc(rc);
    int ret = m->prev_allreduce(hs, hr, count, dt, op, m->comm, m->prev_allreduce_module);
    if (ret == OMPI_SUCCESS) ret = map_rc(hview_out(m, &r));
    return ret;
}

static int mx_coll_allreduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                             struct ompi_op_t *op, struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const int n = mx_ompi_host->comm_size(comm);
    const size_t es = mx_ompi_host->dtype_size(dtype);
    int slot, opi, alg;
    if (reducible(dtype, op, (size_t)count, n, &slot, &opi) && big(m, (size_t)count * es) &&
        (alg = allreduce_rule(m, (size_t)count, es, slot)) >= 0 && comm_ready(m)) {
        const int inplace = sbuf == MPI_IN_PLACE;
        xbuf_t s, r;
        int rc = begin(m);
        if (!rc && !inplace) rc = xin(m, SCR_IN, sbuf, dtype, (size_t)count, 1, &s);
        if (!rc) rc = xin(m, SCR_OUT, rbuf, dtype, (size_t)count, inplace, &r);
        if (!rc) rc = mx_allreduce(m->mx, inplace ? MX_IN_PLACE : s.dev, r.dev, (size_t)count, slot, opi, alg, m->stream);
        if (!rc) rc = xout(m, &r, r.bytes);
        return map_rc(rc);
    }
    return host_allreduce(m, sbuf, rbuf, count, dtype, op);
}

static int host_reduce_scatter(mx_coll_module_t *m, const void *sbuf, void *rbuf, const int *rcounts, size_t total,
                               struct ompi_datatype_t *dt, struct ompi_op_t *op)
{
    const int rank = mx_ompi_host->comm_rank(m->comm);
    const int inplace = sbuf == MPI_IN_PLACE;
    hview_t s, r;
    void *hs, *hr;
    int rc = hview_in(m, SCR_IN, sbuf, dt, total, 1, &s, &hs);
    /* MPI_IN_PLACE: rbuf holds the whole input vector */
    if (!rc) rc = hview_out_in(m, SCR_OUT, rbuf, dt, inplace ? total : (size_t)rcounts[rank], inplace, &r, &hr);
    if (rc) return map_rc(rc);
    int ret = m->prev_reduce_scatter(hs, hr, rcounts, dt, op, m->comm, m->prev_reduce_scatter_module);
    if (ret == OMPI_SUCCESS) ret = map_rc(hview_out(m, &r));
    return ret;
}

static int mx_coll_reduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, struct ompi_datatype_t *dtype,
                                  struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                  mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const int n = mx_ompi_host->comm_size(comm), rank = mx_ompi_host->comm_rank(comm);
    const size_t es = mx_ompi_host->dtype_size(dtype);
    size_t rc64[MX_MAX_RANKS], total = 0;
    int slot, opi, alg;
    for (int i = 0; i < n; i++) {
        if (i < MX_MAX_RANKS) rc64[i] = (size_t)rcounts[i];
        total += (size_t)rcounts[i];
    }
    const int inplace = sbuf == MPI_IN_PLACE;
    if (reducible(dtype, op, total, n, &slot, &opi) && big(m, total * es) &&
        (alg = reduce_scatter_rule(m, total, es, inplace)) >= 0 && comm_ready(m)) {
        xbuf_t s, r;
        int rc = begin(m);
        if (!rc && !inplace) rc = xin(m, SCR_IN, sbuf, dtype, total, 1, &s);
        /* MPI_IN_PLACE: rbuf holds the whole input vector */
        if (!rc) rc = xin(m, SCR_OUT, rbuf, dtype, inplace ? total : rc64[rank], inplace, &r);
        if (!rc) rc = mx_reduce_scatter(m->mx, inplace ? MX_IN_PLACE : s.dev, r.dev, rc64, slot, opi, alg, m->stream);
        if (!rc) {
            r.count = rcounts[rank];
            r.bytes = rc64[rank] * es;
            rc = xout(m, &r, r.bytes);
        }
        return map_rc(rc);
    }
    return host_reduce_scatter(m, sbuf, rbuf, rcounts, total, dtype, op);
}

static int host_allgather(mx_coll_module_t *m, const void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                          void *rbuf, int rcount, struct ompi_datatype_t *rdtype)
{
    const int n = mx_ompi_host->comm_size(m->comm);
    hview_t s, r;
    void *hs, *hr;
    int rc = hview_in(m, SCR_IN, sbuf, sdtype, (size_t)scount, 1, &s, &hs);
    if (!rc) rc = hview_out_in(m, SCR_OUT, rbuf, rdtype, (size_t)rcount * n, sbuf == MPI_IN_PLACE, &r, &hr);
    if (rc) return map_rc(rc);
    int ret = m->prev_allgather(hs, scount, sdtype, hr, rcount, rdtype, m->comm, m->prev_allgather_module);
    if (ret == OMPI_SUCCESS) ret = map_rc(hview_out(m, &r));
    return ret;
}

static int mx_coll_allgather(const void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                             struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                             mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const size_t rbytes = (size_t)rcount * mx_ompi_host->dtype_size(rdtype);
    const int n = mx_ompi_host->comm_size(comm);
    /* (rcount, rdtype) is significant, and its signature equal, on every
     * rank; pure data movement: any lower module gives the same bytes */
    if (rbytes && n <= MX_MAX_RANKS && big(m, rbytes * n) && comm_ready(m)) {
        const int inplace = sbuf == MPI_IN_PLACE;
        xbuf_t s, r;
        int rc = begin(m);
        if (!rc && !inplace) rc = xin(m, SCR_IN, sbuf, sdtype, (size_t)scount, 1, &s);
        if (!rc && !inplace && s.bytes != rbytes) rc = MX_ERR_ARG;   /* type signatures differ */
        if (!rc) rc = xin(m, SCR_OUT, rbuf, rdtype, (size_t)rcount * n, inplace, &r);
        if (!rc)
            rc = mx_allgather(m->mx, inplace ? MX_IN_PLACE : s.dev, r.dev, rbytes, m->stream);
        if (!rc) rc = xout(m, &r, r.bytes);
        return map_rc(rc);
    }
    return host_allgather(m, sbuf, scount, sdtype, rbuf, rcount, rdtype);
}

static int mx_coll_bcast(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                         struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const size_t bytes = (size_t)count * mx_ompi_host->dtype_size(dtype);
    const int n = mx_ompi_host->comm_size(comm), rank = mx_ompi_host->comm_rank(comm);
    if (bytes && n <= MX_MAX_RANKS && big(m, bytes) && comm_ready(m)) {
        xbuf_t b;
        int rc = begin(m);
        if (!rc) rc = xin(m, SCR_OUT, buf, dtype, (size_t)count, rank == root, &b);
        if (!rc) rc = mx_bcast(m->mx, b.dev, bytes, root, m->stream);
        if (!rc && rank != root) rc = xout(m, &b, bytes);
        return map_rc(rc);
    }
    hview_t v;
    void *h;
    int rc = hview_out_in(m, SCR_OUT, buf, dtype, (size_t)count, rank == root, &v, &h);
    if (rc) return map_rc(rc);
    int ret = m->prev_bcast(h, count, dtype, root, comm, m->prev_bcast_module);
    if (ret == OMPI_SUCCESS && rank != root) ret = map_rc(hview_out(m, &v));
    return ret;
}

/* inout = inout OP in on device memory */
static int reduce_local_dev(mx_coll_module_t *m, int opi, int slot, const void *in, void *inout, size_t count)
{
    int rc = begin(m);
    if (g_fast_sync < 0) g_fast_sync = mx_ompi_host->mca_int("coll_mi355x_fast_sync", 1) != 0;
    if (!rc && g_fast_sync) {   /* completion word: from small reduce launches themselves, else a marker kernel */
        rc = mx_reduce2_sync(opi, slot, in, inout, count, m->stream);
    } else {
        if (!rc) rc = mx_reduce2(opi, slot, in, inout, count, m->stream);
        if (!rc) rc = stream_wait(m->stream);
    }
    return rc;
}

/* MPI_Reduce_local has no peers: the per-call buffer check is all it needs.
 * Operands in different memories (MPI_Reduce_local(device_in, host_inout) is
 * legal) are staged one by one, as coll/cuda checks each buffer
 * (coll_cuda_allreduce.c:44-62): a device inout gets a host `in` copied to
 * device scratch; a host inout gets the device `in` copied to host memory and
 * the saved slot runs when the call is at most coll_mi355x_mixed_host_max_kb
 * (default 64 KiB), else inout goes to device scratch and comes back. */
static int mx_coll_reduce_local(const void *inbuf, void *inoutbuf, int count, struct ompi_datatype_t *dtype,
                                struct ompi_op_t *op, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int slot, opi;
    const int din = mx_is_device_ptr(inbuf) == 1, dio = mx_is_device_ptr(inoutbuf) == 1;
    if ((din || dio) && reducible(dtype, op, (size_t)count, 1, &slot, &opi)) {
        ensure_stream(m);
        if (din && dio) return map_rc(reduce_local_dev(m, opi, slot, inbuf, inoutbuf, (size_t)count));
        const size_t bytes = (size_t)count * mx_type_size(slot);
        const int kb = mx_ompi_host->mca_int("coll_mi355x_mixed_host_max_kb", 64);
        void *a, *b;
        int rc;
        if (!dio && bytes <= (kb > 0 ? (size_t)kb << 10 : 0)) {   /* small, host result: `in` to the host */
            if ((rc = hbuf(m, SCR_IN, bytes, &a)) || (rc = mx_memcpy(a, inbuf, bytes, m->stream)) ||
                (rc = stream_wait(m->stream)))
                return map_rc(rc);
            return m->prev_reduce_local(a, inoutbuf, count, dtype, op, m->prev_reduce_local_module);
        }
        a = (void *)inbuf;
        b = inoutbuf;
        if (!din && ((rc = scratch(m, SCR_IN, bytes, &a)) || (rc = mx_memcpy(a, inbuf, bytes, m->stream))))
            return map_rc(rc);
        if (!dio && ((rc = scratch(m, SCR_OUT, bytes, &b)) || (rc = mx_memcpy(b, inoutbuf, bytes, m->stream))))
            return map_rc(rc);
        rc = reduce_local_dev(m, opi, slot, a, b, (size_t)count);
        if (!rc && b != inoutbuf && !(rc = mx_memcpy(inoutbuf, b, bytes, m->stream))) rc = stream_wait(m->stream);
        return map_rc(rc);
    }
    return m->prev_reduce_local(inbuf, inoutbuf, count, dtype, op, m->prev_reduce_local_module);
}

/* ---- size-1 communicators (MPI_COMM_SELF, a one-rank MPI_COMM_WORLD) -------
 * coll/self answers every collective of a size-1 communicator with a local
 * copy: ompi_datatype_copy_content_same_ddt for allreduce / reduce / scan /
 * reduce_scatter (coll_self_allreduce.c:41-44, coll_self_reduce.c,
 * coll_self_scan.c, coll_self_reduce_scatter.c:44), ompi_datatype_sndrcv for
 * allgather; exscan and bcast touch nothing.  Those walk host memory: without
 * the CUDA copy hooks (opal_datatype_copy.c:75-136, SET_CUDA_COPY_FCT) a
 * device buffer is read and written with host memcpy.  coll/cuda does not
 * exclude size 1 and stages every device buffer (coll_cuda_module.c:78-113,
 * coll_cuda_allreduce.c:44-72).  Here the copy runs on the device when either
 * buffer is device memory -- one K7 copy kernel (2 x bytes of HBM traffic)
 * for contiguous layouts, the device convertor for derived ones (packed
 * straight into a contiguous destination, unpacked straight from a contiguous
 * source) -- and host-only calls go to the saved slot. */
static int self_device(const void *sbuf, const void *rbuf)
{
    return (sbuf != MPI_IN_PLACE && mx_is_device_ptr(sbuf) == 1) || mx_is_device_ptr(rbuf) == 1;
}

/* scount x sdt at sbuf -> rcount x rdt at rbuf (equal type signatures) */
static int self_copy(mx_coll_module_t *m, const void *sbuf, struct ompi_datatype_t *sdt, size_t scount, void *rbuf,
                     struct ompi_datatype_t *rdt, size_t rcount)
{
    const size_t bytes = scount * mx_ompi_host->dtype_size(sdt);
    if (bytes != rcount * mx_ompi_host->dtype_size(rdt)) return MX_ERR_ARG;
    if (!bytes) return MX_SUCCESS;
    if (scount > INT_MAX || rcount > INT_MAX) return MX_ERR_UNSUPPORTED;
    ensure_stream(m);
    const int sc = mx_ompi_host->dtype_contiguous(sdt, (int)scount);
    const int rcn = mx_ompi_host->dtype_contiguous(rdt, (int)rcount);
    const int rdev = mx_is_device_ptr(rbuf) == 1;
    int rc;
    if (sc && rcn) {
        rc = (rdev && mx_is_device_ptr(sbuf) == 1) ? mx_copy(rbuf, sbuf, bytes, m->stream)
                                                   : mx_memcpy(rbuf, sbuf, bytes, m->stream);
    } else if (rcn && rdev) {   /* pack straight into the destination */
        xbuf_t s = {.user = (void *)sbuf, .bytes = bytes, .dt = sdt, .count = (int)scount, .contiguous = 0};
        rc = xfer_packed(m, &s, rbuf, 1);
    } else {                    /* the packed input on the device, unpacked into rbuf */
        xbuf_t s;
        rc = xin(m, SCR_IN, sbuf, sdt, scount, 1, &s);
        if (!rc && rcn) {
            rc = mx_memcpy(rbuf, s.dev, bytes, m->stream);
        } else if (!rc) {
            xbuf_t r = {.user = rbuf, .bytes = bytes, .dt = rdt, .count = (int)rcount, .contiguous = 0};
            rc = xfer_packed(m, &r, s.dev, 0);
        }
    }
    return rc ? rc : stream_wait(m->stream);
}

static int mx_self_allreduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                             struct ompi_op_t *op, struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    if (sbuf == MPI_IN_PLACE) return OMPI_SUCCESS;
    if (!self_device(sbuf, rbuf)) return m->prev_allreduce(sbuf, rbuf, count, dtype, op, comm, m->prev_allreduce_module);
    return map_rc(self_copy(m, sbuf, dtype, (size_t)count, rbuf, dtype, (size_t)count));
}

static int mx_self_reduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, struct ompi_datatype_t *dtype,
                                  struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                  mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    if (sbuf == MPI_IN_PLACE) return OMPI_SUCCESS;
    if (!self_device(sbuf, rbuf))
        return m->prev_reduce_scatter(sbuf, rbuf, rcounts, dtype, op, comm, m->prev_reduce_scatter_module);
    return map_rc(self_copy(m, sbuf, dtype, (size_t)rcounts[0], rbuf, dtype, (size_t)rcounts[0]));
}

static int mx_self_reduce_scatter_block(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dtype,
                                        struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                        mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    if (sbuf == MPI_IN_PLACE) return OMPI_SUCCESS;   /* the result is rbuf's first rcount elements already */
    if (!self_device(sbuf, rbuf))
        return m->prev_reduce_scatter_block(sbuf, rbuf, rcount, dtype, op, comm, m->prev_reduce_scatter_block_module);
    return map_rc(self_copy(m, sbuf, dtype, (size_t)rcount, rbuf, dtype, (size_t)rcount));
}

static int mx_self_allgather(const void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                             struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                             mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    if (sbuf == MPI_IN_PLACE) return OMPI_SUCCESS;
    if (!self_device(sbuf, rbuf))
        return m->prev_allgather(sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, m->prev_allgather_module);
    return map_rc(self_copy(m, sbuf, sdtype, (size_t)scount, rbuf, rdtype, (size_t)rcount));
}

static int mx_self_reduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                          int root, struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    if (sbuf == MPI_IN_PLACE) return OMPI_SUCCESS;
    if (!self_device(sbuf, rbuf))
        return m->prev_reduce(sbuf, rbuf, count, dtype, op, root, comm, m->prev_reduce_module);
    return map_rc(self_copy(m, sbuf, dtype, (size_t)count, rbuf, dtype, (size_t)count));
}

static int mx_self_scan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                        struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    if (sbuf == MPI_IN_PLACE) return OMPI_SUCCESS;
    if (!self_device(sbuf, rbuf)) return m->prev_scan(sbuf, rbuf, count, dtype, op, comm, m->prev_scan_module);
    return map_rc(self_copy(m, sbuf, dtype, (size_t)count, rbuf, dtype, (size_t)count));
}

/* rank 0's exscan result is undefined: nothing is read or written
 * (coll_self_exscan.c), whatever memory the buffers are in */
static int mx_self_exscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                          struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    (void)sbuf; (void)rbuf; (void)count; (void)dtype; (void)op; (void)comm; (void)module;
    return OMPI_SUCCESS;
}

/* Reduction slots beyond the four of the north star:
 * MPI_Reduce (coll.h:239-241), MPI_Reduce_scatter_block (:245-247),
 * MPI_Scan / MPI_Exscan (:248-250, :228-230).  Algorithms follow coll/tuned's
 * fixed decisions (reduce: coll_tuned_decision_fixed.c:354-429;
 * reduce_scatter_block: basic_linear, :522-532) and coll/basic's linear scan /
 * exscan (tuned leaves those slots empty, coll_tuned_module.c:106,112), or
 * the forced algorithm of coll_mi355x_{reduce,scan,exscan}_algorithm. */
static int mx_coll_reduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                          struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                          mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const int n = mx_ompi_host->comm_size(comm), rank = mx_ompi_host->comm_rank(comm);
    const size_t es = mx_ompi_host->dtype_size(dtype);
    const int inplace = sbuf == MPI_IN_PLACE && rank == root;   /* rbuf matters on the root only */
    int slot, opi, alg = -1;
    if (reducible(dtype, op, (size_t)count, n, &slot, &opi) && big(m, (size_t)count * es)) {
        alg = mx_ompi_host->mca_int("coll_mi355x_reduce_algorithm", MX_REDUCE_AUTO);
        if (!alg) alg = reduce_rule(m, (size_t)count, es);
    }
    if (alg >= 0 && comm_ready(m)) {
        xbuf_t s, r;
        memset(&r, 0, sizeof r);
        int rc = begin(m);
        if (!rc && !inplace) rc = xin(m, SCR_IN, sbuf, dtype, (size_t)count, 1, &s);
        if (!rc && rank == root) rc = xin(m, SCR_OUT, rbuf, dtype, (size_t)count, inplace, &r);
        if (!rc)
            rc = mx_reduce(m->mx, inplace ? MX_IN_PLACE : s.dev, rank == root ? r.dev : NULL, (size_t)count, slot, opi,
                           root, alg, m->stream);
        if (!rc && rank == root) rc = xout(m, &r, r.bytes);
        return map_rc(rc);
    }
    hview_t sv, rv;
    void *hs, *hr = rbuf;
    int rc = hview_in(m, SCR_IN, sbuf, dtype, (size_t)count, 1, &sv, &hs);
    memset(&rv, 0, sizeof rv);
    if (!rc && rank == root) rc = hview_out_in(m, SCR_OUT, rbuf, dtype, (size_t)count, inplace, &rv, &hr);
    if (rc) return map_rc(rc);
    int ret = m->prev_reduce(hs, hr, count, dtype, op, root, comm, m->prev_reduce_module);
    if (ret == OMPI_SUCCESS && rank == root) ret = map_rc(hview_out(m, &rv));
    return ret;
}

static int mx_coll_reduce_scatter_block(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dtype,
                                        struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                        mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const int n = mx_ompi_host->comm_size(comm);
    const size_t total = (size_t)rcount * (size_t)n, es = mx_ompi_host->dtype_size(dtype);
    const int inplace = sbuf == MPI_IN_PLACE;
    int slot, opi, alg;
    if (reducible(dtype, op, total, n, &slot, &opi) && big(m, total * es) && (alg = rsb_rule(m, total, es)) >= 0 &&
        comm_ready(m)) {
        xbuf_t s, r;
        int rc = begin(m);
        if (!rc && !inplace) rc = xin(m, SCR_IN, sbuf, dtype, total, 1, &s);
        if (!rc) rc = xin(m, SCR_OUT, rbuf, dtype, inplace ? total : (size_t)rcount, inplace, &r);
        if (!rc)
            rc = mx_reduce_scatter_block(m->mx, inplace ? MX_IN_PLACE : s.dev, r.dev, (size_t)rcount, slot, opi, alg,
                                         m->stream);
        if (!rc) {
            r.count = rcount;
            r.bytes = (size_t)rcount * es;
            rc = xout(m, &r, r.bytes);
        }
        return map_rc(rc);
    }
    hview_t sv, rv;
    void *hs, *hr;
    int rc = hview_in(m, SCR_IN, sbuf, dtype, total, 1, &sv, &hs);
    if (!rc) rc = hview_out_in(m, SCR_OUT, rbuf, dtype, inplace ? total : (size_t)rcount, inplace, &rv, &hr);
    if (rc) return map_rc(rc);
    int ret = m->prev_reduce_scatter_block(hs, hr, rcount, dtype, op, comm, m->prev_reduce_scatter_block_module);
    if (ret == OMPI_SUCCESS) ret = map_rc(hview_out(m, &rv));
    return ret;
}

/* returns 1 when the call should be delegated */
static int scan_common(mx_coll_module_t *m, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                       struct ompi_op_t *op, int exclusive, int *ret)
{
    const int n = mx_ompi_host->comm_size(m->comm);
    const size_t es = mx_ompi_host->dtype_size(dtype);
    int slot, opi, alg;
    if (!reducible(dtype, op, (size_t)count, n, &slot, &opi) || !big(m, (size_t)count * es) ||
        (alg = scan_rule(m, es, exclusive)) < 0 || !comm_ready(m))
        return 1;
    const int inplace = sbuf == MPI_IN_PLACE;
    xbuf_t s, r;
    int rc = begin(m);
    if (!rc && !inplace) rc = xin(m, SCR_IN, sbuf, dtype, (size_t)count, 1, &s);
    /* exscan leaves rank 0's rbuf untouched: stage it in so the copy back is a no-op */
    if (!rc) rc = xin(m, SCR_OUT, rbuf, dtype, (size_t)count, inplace || exclusive, &r);
    const void *sb = inplace ? MX_IN_PLACE : s.dev;
    if (!rc)
        rc = exclusive ? mx_exscan(m->mx, sb, r.dev, (size_t)count, slot, opi, alg, m->stream)
                       : mx_scan(m->mx, sb, r.dev, (size_t)count, slot, opi, alg, m->stream);
    if (!rc) rc = xout(m, &r, r.bytes);
    *ret = map_rc(rc);
    return 0;
}

static int host_scan(mx_coll_module_t *m, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                     struct ompi_op_t *op, int exclusive)
{
    hview_t sv, rv;
    void *hs, *hr;
    int rc = hview_in(m, SCR_IN, sbuf, dtype, (size_t)count, 1, &sv, &hs);
    /* exscan leaves rank 0's rbuf untouched: copy it in so the copy back keeps it */
    if (!rc) rc = hview_out_in(m, SCR_OUT, rbuf, dtype, (size_t)count, sbuf == MPI_IN_PLACE || exclusive, &rv, &hr);
    if (rc) return map_rc(rc);
    int ret = exclusive ? m->prev_exscan(hs, hr, count, dtype, op, m->comm, m->prev_exscan_module)
                        : m->prev_scan(hs, hr, count, dtype, op, m->comm, m->prev_scan_module);
    if (ret == OMPI_SUCCESS) ret = map_rc(hview_out(m, &rv));
    return ret;
}

static int mx_coll_scan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                        struct ompi_op_t *op, struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    (void)comm;
    if (!scan_common(m, sbuf, rbuf, count, dtype, op, 0, &ret)) return ret;
    return host_scan(m, sbuf, rbuf, count, dtype, op, 0);
}

static int mx_coll_exscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                          struct ompi_op_t *op, struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    (void)comm;
    if (!scan_common(m, sbuf, rbuf, count, dtype, op, 1, &ret)) return ret;
    return host_scan(m, sbuf, rbuf, count, dtype, op, 1);
}

/* ---- nonblocking and persistent slots ------------------
 * A device-path request is an mx_request_t (include/mx_coll.h) wrapped in a
 * host ompi_request_t; active ones sit on a list that the progress callback
 * (registered once, like libnbc's) polls with mx_test and completes.  The
 * GPU needs no host progress: polling only reports completion.  A staged
 * buffer belongs to its request (requests overlap): it is filled when the
 * operation starts and copied back when the progress callback sees the
 * device part complete. */
typedef struct mx_coll_req {
    struct ompi_request_t *req;
    mx_request_t *mx;
    mx_coll_module_t *m;
    struct mx_coll_req *next;
    int active;
    /* staged buffers: s (input, copied in at every start) and r (output,
     * copied in too when the operation reads it; copied back at completion) */
    xbuf_t s, r;
    int s_in, r_in;
    size_t r_back;   /* bytes of r copied back */
    /* a request of the saved module run on host copies of device buffers:
     * hv[0] input, hv[1] output (copied in at every start when hv_in) */
    struct ompi_request_t *inner;
    hview_t hv[2];
    int hv_in[2];
    int persistent;
} mx_coll_req_t;

static mx_coll_req_t *g_active;
static int g_progress_registered;

static void req_release_staging(mx_coll_req_t *r)
{
    if (r->s.user) mx_free(r->s.dev);
    if (r->r.user) mx_free(r->r.dev);
    r->s.user = r->r.user = NULL;
}

/* a request's own staging (not the module's scratch: requests overlap) */
static int req_stage(mx_coll_req_t *q, const void *user, struct ompi_datatype_t *dt, size_t count, int copy_in,
                     xbuf_t *x)
{
    memset(x, 0, sizeof *x);
    x->bytes = count * mx_ompi_host->dtype_size(dt);
    x->dt = dt;
    x->count = count > INT_MAX ? INT_MAX : (int)count;
    x->contiguous = mx_ompi_host->dtype_contiguous(dt, x->count);
    if (x->contiguous && (!x->bytes || mx_is_device_ptr(user) == 1)) {
        x->dev = (void *)user;
        return MX_SUCCESS;
    }
    if (mx_alloc(x->bytes, &x->dev) != MX_SUCCESS) return MX_ERR_NOMEM;
    x->user = (void *)user;
    (void)copy_in;   /* filled by req_fill at each start */
    return MX_SUCCESS;
}

static int req_fill(mx_coll_req_t *q)
{
    mx_coll_module_t *m = q->m;
    int rc = begin_nb(m);
    const xbuf_t *xs[2] = {&q->s, &q->r};
    const int in[2] = {q->s_in, q->r_in};
    for (int i = 0; i < 2 && !rc; i++) {
        const xbuf_t *x = xs[i];
        if (!x->user || !in[i]) continue;
        rc = x->contiguous ? mx_memcpy(x->dev, x->user, x->bytes, m->nb_stream) : xfer_packed(m, x, x->dev, 1);
    }
    return rc;
}

/* completion of a host-path request: the output back to the device */
static int hreq_complete(mx_coll_req_t *r, int status)
{
    if (status == OMPI_SUCCESS) status = map_rc(hview_out(r->m, &r->hv[1]));
    if (!r->persistent && r->inner) mx_ompi_host->request_free(&r->inner);
    return status;
}

static int g_in_progress;
static int mx_coll_progress(void)
{
    int completed = 0;
    /* testing the saved module's requests must not re-enter (a host's
     * request test may progress, and so call back here) */
    if (g_in_progress) return 0;
    g_in_progress = 1;
    mx_coll_req_t **pp = &g_active;
    while (*pp) {
        mx_coll_req_t *r = *pp;
        int flag = 0, status = OMPI_SUCCESS;
        if (r->inner) {
            const int rc = mx_ompi_host->request_test(r->inner, &flag, &status);
            if (rc != OMPI_SUCCESS) { flag = 1; status = rc; }
            if (flag) {
                *pp = r->next;
                r->active = 0;
                mx_ompi_host->request_complete(r->req, hreq_complete(r, status));
                completed++;
                continue;
            }
            pp = &r->next;
            continue;
        }
        int rc = mx_test(r->mx, &flag);
        if (flag || rc != MX_SUCCESS) {
            *pp = r->next;
            r->active = 0;
            if (rc == MX_SUCCESS && r->r.user) rc = xout(r->m, &r->r, r->r_back);
            mx_ompi_host->request_complete(r->req, map_rc(rc));
            completed++;
        } else {
            pp = &r->next;
        }
    }
    g_in_progress = 0;
    return completed;
}

static void activate(mx_coll_req_t *r)
{
    r->active = 1;
    r->next = g_active;
    g_active = r;
}

static void deactivate(mx_coll_req_t *r)
{
    for (mx_coll_req_t **pp = &g_active; *pp; pp = &(*pp)->next)
        if (*pp == r) { *pp = r->next; break; }
    r->active = 0;
}

static int req_start_cb(struct ompi_request_t *req)     /* MPI_Start */
{
    mx_coll_req_t *r = (mx_coll_req_t *)mx_ompi_host->request_ctx(req);
    if (r->inner) {   /* host path: refresh the host copies, start the saved module's request */
        int rc = MX_SUCCESS;
        for (int i = 0; i < 2 && !rc; i++)
            if (r->hv_in[i] && r->hv[i].user && r->hv[i].span) {
                ensure_stream(r->m);
                rc = mx_memcpy(r->hv[i].copy, (const char *)r->hv[i].user + r->hv[i].lo, r->hv[i].span,
                               r->m->stream);
                if (!rc) rc = stream_wait(r->m->stream);
            }
        if (rc) return map_rc(rc);
        const int ret = mx_ompi_host->request_start(r->inner);
        if (ret != OMPI_SUCCESS) return ret;
        mx_ompi_host->request_activate(req);
        activate(r);
        return OMPI_SUCCESS;
    }
    int rc = req_fill(r);
    if (!rc) rc = mx_start(r->mx);
    if (rc != MX_SUCCESS) return map_rc(rc);
    mx_ompi_host->request_activate(req);
    activate(r);
    return OMPI_SUCCESS;
}

static int req_free_cb(struct ompi_request_t *req)      /* MPI_Request_free */
{
    mx_coll_req_t *r = (mx_coll_req_t *)mx_ompi_host->request_ctx(req);
    if (r->active) deactivate(r);
    int rc = MX_SUCCESS;
    if (r->mx) rc = mx_request_free(r->mx);   /* lets an active operation finish */
    if (r->inner) mx_ompi_host->request_free(&r->inner);
    hview_release(&r->hv[0]);
    hview_release(&r->hv[1]);
    req_release_staging(r);
    free(r);
    return map_rc(rc);
}

/* ---- nonblocking calls on the saved module ---------------------------------
 * With host buffers the saved module's request is returned as is.  A device
 * buffer is copied to a host buffer owned by a wrapper request: the saved
 * module runs on the copy, the progress callback completes the wrapper
 * (output copied back) when the inner request completes.  Persistent forms
 * refresh the input copies at every MPI_Start. */
static mx_coll_req_t *hreq_new(mx_coll_module_t *m, const void *sbuf, struct ompi_datatype_t *sdt, size_t scount,
                               void *rbuf, struct ompi_datatype_t *rdt, size_t rcount, int r_reads, void **hs,
                               void **hr, int *ret)
{
    mx_coll_req_t *r = calloc(1, sizeof *r);
    int rc = r ? MX_SUCCESS : MX_ERR_NOMEM;
    *hs = (void *)sbuf;
    *hr = rbuf;
    if (!rc && sbuf) {
        rc = hview_in(m, -1, sbuf, sdt, scount, 1, &r->hv[0], hs);
        r->hv_in[0] = 1;
    }
    if (!rc && rbuf) {
        r->hv_in[1] = r_reads || !mx_ompi_host->dtype_contiguous(rdt, rcount > INT_MAX ? INT_MAX : (int)rcount);
        rc = hview_in(m, -1, rbuf, rdt, rcount, r->hv_in[1], &r->hv[1], hr);
    }
    if (rc || !r || (!r->hv[0].user && !r->hv[1].user)) {   /* error, or host memory only: no wrapper */
        if (r) { hview_release(&r->hv[0]); hview_release(&r->hv[1]); free(r); }
        *ret = map_rc(rc);
        return NULL;
    }
    r->m = m;
    return r;
}

/* wraps the saved module's request `inner` (posted with status ret) */
static int hreq_post(mx_coll_req_t *r, int ret, struct ompi_request_t *inner, int persistent,
                     struct ompi_request_t **request)
{
    if (ret != OMPI_SUCCESS) {
        hview_release(&r->hv[0]);
        hview_release(&r->hv[1]);
        free(r);
        return ret;
    }
    r->inner = inner;
    r->persistent = persistent;
    r->req = mx_ompi_host->request_create(persistent, req_start_cb, req_free_cb, r);
    if (!r->req) {
        mx_ompi_host->request_free(&r->inner);
        hview_release(&r->hv[0]);
        hview_release(&r->hv[1]);
        free(r);
        return OMPI_ERR_OUT_OF_RESOURCE;
    }
    if (!g_progress_registered) {
        mx_ompi_host->progress_register(mx_coll_progress);
        g_progress_registered = 1;
    }
    if (!persistent) activate(r);
    *request = r->req;
    return OMPI_SUCCESS;
}

/* Delegation of one nonblocking / persistent slot: HCALL(hs, hr, req) is the
 * saved module's call on the (possibly host-copied) buffers. */
#define MX_HOST_NB(m, sbuf, sdt, scount, rbuf, rdt, rcount, r_reads, persistent, request, HCALL)               \
    do {                                                                                                   \
        void *hs_, *hr_;                                                                                   \
        int ret_ = OMPI_SUCCESS;                                                                           \
        mx_coll_req_t *w_ = hreq_new((m), (sbuf), (sdt), (scount), (rbuf), (rdt), (rcount), (r_reads), &hs_, \
                                     &hr_, &ret_);                                                         \
        if (!w_) {                                                                                         \
            if (ret_ != OMPI_SUCCESS) return ret_;                                                         \
            struct ompi_request_t **rq_ = (request);                                                       \
            return HCALL(hs_, hr_, rq_);                                                                   \
        }                                                                                                  \
        struct ompi_request_t *in_ = NULL;                                                                 \
        ret_ = HCALL(hs_, hr_, &in_);                                                                      \
        return hreq_post(w_, ret_, in_, (persistent), (request));                                          \
    } while (0)

/* a request wrapper with its staged buffers (NULL on failure) */
static mx_coll_req_t *req_new(mx_coll_module_t *m)
{
    mx_coll_req_t *r = calloc(1, sizeof *r);
    if (r) r->m = m;
    return r;
}

/* wrap the mx request created with rc into *request */
static int post(mx_coll_req_t *r, int rc, mx_request_t *mxr, int persistent, struct ompi_request_t **request)
{
    if (rc != MX_SUCCESS) {
        req_release_staging(r);
        free(r);
        return map_rc(rc);
    }
    r->req = mx_ompi_host->request_create(persistent, req_start_cb, req_free_cb, r);
    if (!r->req) {
        mx_request_free(mxr);
        req_release_staging(r);
        free(r);
        return OMPI_ERR_OUT_OF_RESOURCE;
    }
    r->mx = mxr;
    if (!g_progress_registered) {
        mx_ompi_host->progress_register(mx_coll_progress);
        g_progress_registered = 1;
    }
    if (!persistent) activate(r);
    *request = r->req;
    return OMPI_SUCCESS;
}

/* coll_mi355x_<name>_algorithm, defaulting to coll_libnbc_<name>_algorithm */
static int nbc_alg(const char *name)
{
    char a[96], b[96];
    snprintf(a, sizeof a, "coll_mi355x_%s_algorithm", name);
    snprintf(b, sizeof b, "coll_libnbc_%s_algorithm", name);
    return mx_ompi_host->mca_int(a, mx_ompi_host->mca_int(b, 0));
}

/* Common set-up of a device-path request: staging of sbuf (count_s
 * elements, read) and rbuf (count_r elements, read when r_in, copied back
 * r_back bytes); a nonblocking request is filled here, a persistent one at
 * each start.  Returns the request or NULL (error in *ret). */
static mx_coll_req_t *req_setup(mx_coll_module_t *m, const void *sbuf, size_t count_s, struct ompi_datatype_t *sdt,
                                void *rbuf, size_t count_r, struct ompi_datatype_t *rdt, int r_in, size_t r_back,
                                int persistent, int *ret)
{
    mx_coll_req_t *r = req_new(m);
    int rc = r ? MX_SUCCESS : MX_ERR_NOMEM;
    if (!rc && sbuf && sbuf != MPI_IN_PLACE) {
        rc = req_stage(r, sbuf, sdt, count_s, 1, &r->s);
        r->s_in = 1;
    } else if (r) {
        r->s.dev = (void *)sbuf;
    }
    if (!rc && rbuf) {
        rc = req_stage(r, rbuf, rdt, count_r, r_in, &r->r);
        r->r_in = r_in;
        r->r_back = r_back;
        r->r.count = rdt && mx_ompi_host->dtype_size(rdt) ? (int)(r_back / mx_ompi_host->dtype_size(rdt)) : 0;
    }
    if (!rc && !persistent) rc = req_fill(r);
    if (rc) {
        if (r) { req_release_staging(r); free(r); }
        *ret = map_rc(rc);
        return NULL;
    }
    return r;
}
#define SB(r) ((r)->s.dev == MPI_IN_PLACE ? MX_IN_PLACE : (r)->s.dev)

/* A nonblocking call takes the device only on a communicator whose device
 * path already exists: creating it is a collective exchange, which a
 * nonblocking call must not wait for (MPI-3.1 5.12; e.g. rank 0
 * MPI_Iallreduce + MPI_Send while rank 1 MPI_Recv + MPI_Iallreduce).  It is
 * created by the first eligible blocking collective (every rank issues the
 * same collectives in the same order, so the state agrees on all ranks).
 * Reductions also need the saved slot to be coll/libnbc, whose orders the
 * device reproduces. */
static int nb_device(mx_coll_module_t *m, size_t bytes, int reduction)
{
    return m->mx_state == 1 && big(m, bytes) && (!reduction || m->low_nbc == LOW_LIBNBC);
}

/* returns 1 when the call should be delegated */
static int allreduce_like(mx_coll_module_t *m, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                          struct ompi_op_t *op, int persistent, struct ompi_request_t **request, int *ret)
{
    const int n = mx_ompi_host->comm_size(m->comm);
    int slot, opi;
    mx_request_t *q = NULL;
    const size_t bytes = (size_t)count * mx_ompi_host->dtype_size(dtype);
    if (!reducible(dtype, op, (size_t)count, n, &slot, &opi) || !nb_device(m, bytes, 1)) return 1;
    mx_coll_req_t *r = req_setup(m, sbuf, (size_t)count, dtype, rbuf, (size_t)count, dtype, sbuf == MPI_IN_PLACE,
                                 bytes, persistent, ret);
    if (!r) return 0;
    const int alg = nbc_alg("iallreduce");
    const int rc = persistent ? mx_allreduce_init(m->mx, SB(r), r->r.dev, (size_t)count, slot, opi, alg, m->nb_stream, &q)
                              : mx_iallreduce(m->mx, SB(r), r->r.dev, (size_t)count, slot, opi, alg, m->nb_stream, &q);
    *ret = post(r, rc, q, persistent, request);
    return 0;
}

static int mx_coll_iallreduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                              struct ompi_op_t *op, struct ompi_communicator_t *comm, struct ompi_request_t **request,
                              mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!allreduce_like(m, sbuf, rbuf, count, dtype, op, 0, request, &ret)) return ret;
#define H(hs, hr, rq) m->prev_iallreduce(hs, hr, count, dtype, op, comm, rq, m->prev_iallreduce_module)
    MX_HOST_NB(m, sbuf, dtype, (size_t)count, rbuf, dtype, (size_t)count, sbuf == MPI_IN_PLACE, 0, request, H);
#undef H
}

static int mx_coll_allreduce_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                                  struct ompi_op_t *op, struct ompi_communicator_t *comm, struct ompi_info_t *info,
                                  struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!allreduce_like(m, sbuf, rbuf, count, dtype, op, 1, request, &ret)) return ret;
#define H(hs, hr, rq) m->prev_allreduce_init(hs, hr, count, dtype, op, comm, info, rq, m->prev_allreduce_init_module)
    MX_HOST_NB(m, sbuf, dtype, (size_t)count, rbuf, dtype, (size_t)count, sbuf == MPI_IN_PLACE, 1, request, H);
#undef H
}

static int reduce_like(mx_coll_module_t *m, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                       struct ompi_op_t *op, int root, struct ompi_communicator_t *comm, int persistent,
                       struct ompi_request_t **request, int *ret)
{
    const int n = mx_ompi_host->comm_size(comm), rank = mx_ompi_host->comm_rank(comm);
    int slot, opi;
    mx_request_t *q = NULL;
    const size_t bytes = (size_t)count * mx_ompi_host->dtype_size(dtype);
    if (!reducible(dtype, op, (size_t)count, n, &slot, &opi) || !nb_device(m, bytes, 1)) return 1;
    const int inplace = sbuf == MPI_IN_PLACE && rank == root;
    mx_coll_req_t *r = req_setup(m, inplace ? MPI_IN_PLACE : sbuf, (size_t)count, dtype, rank == root ? rbuf : NULL,
                                 (size_t)count, dtype, inplace, bytes, persistent, ret);
    if (!r) return 0;
    void *rb = rank == root ? r->r.dev : NULL;
    const int alg = nbc_alg("ireduce");
    const int rc = persistent ? mx_reduce_init(m->mx, SB(r), rb, (size_t)count, slot, opi, root, alg, m->nb_stream, &q)
                              : mx_ireduce(m->mx, SB(r), rb, (size_t)count, slot, opi, root, alg, m->nb_stream, &q);
    *ret = post(r, rc, q, persistent, request);
    return 0;
}

static int mx_coll_ireduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                           int root, struct ompi_communicator_t *comm, struct ompi_request_t **request,
                           mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!reduce_like(m, sbuf, rbuf, count, dtype, op, root, comm, 0, request, &ret)) return ret;
    const int is_root = mx_ompi_host->comm_rank(comm) == root;
#define H(hs, hr, rq) m->prev_ireduce(hs, hr, count, dtype, op, root, comm, rq, m->prev_ireduce_module)
    MX_HOST_NB(m, sbuf, dtype, (size_t)count, is_root ? rbuf : NULL, dtype, (size_t)count, sbuf == MPI_IN_PLACE, 0,
               request, H);
#undef H
}

static int mx_coll_reduce_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                               struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                               struct ompi_info_t *info, struct ompi_request_t **request,
                               mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!reduce_like(m, sbuf, rbuf, count, dtype, op, root, comm, 1, request, &ret)) return ret;
    const int is_root = mx_ompi_host->comm_rank(comm) == root;
#define H(hs, hr, rq) m->prev_reduce_init(hs, hr, count, dtype, op, root, comm, info, rq, m->prev_reduce_init_module)
    MX_HOST_NB(m, sbuf, dtype, (size_t)count, is_root ? rbuf : NULL, dtype, (size_t)count, sbuf == MPI_IN_PLACE, 1,
               request, H);
#undef H
}

/* rcounts == NULL: the _block form with `rcount` per rank */
static int rs_like(mx_coll_module_t *m, const void *sbuf, void *rbuf, const int *rcounts, int rcount,
                   struct ompi_datatype_t *dtype, struct ompi_op_t *op, struct ompi_communicator_t *comm,
                   int persistent, struct ompi_request_t **request, int *ret)
{
    const int n = mx_ompi_host->comm_size(comm), rank = mx_ompi_host->comm_rank(comm);
    size_t rc64[MX_MAX_RANKS], total = 0;
    int slot, opi;
    mx_request_t *q = NULL;
    if (n > MX_MAX_RANKS) return 1;
    for (int i = 0; i < n; i++) { rc64[i] = (size_t)(rcounts ? rcounts[i] : rcount); total += rc64[i]; }
    const size_t es = mx_ompi_host->dtype_size(dtype);
    if (!reducible(dtype, op, total, n, &slot, &opi) || !nb_device(m, total * es, 1)) return 1;
    const int inplace = sbuf == MPI_IN_PLACE;
    mx_coll_req_t *r = req_setup(m, sbuf, total, dtype, rbuf, inplace ? total : rc64[rank], dtype, inplace,
                                 rc64[rank] * es, persistent, ret);
    if (!r) return 0;
    int rc;
    if (rcounts)
        rc = persistent ? mx_reduce_scatter_init(m->mx, SB(r), r->r.dev, rc64, slot, opi, m->nb_stream, &q)
                        : mx_ireduce_scatter(m->mx, SB(r), r->r.dev, rc64, slot, opi, m->nb_stream, &q);
    else
        rc = persistent ? mx_reduce_scatter_block_init(m->mx, SB(r), r->r.dev, (size_t)rcount, slot, opi, m->nb_stream, &q)
                        : mx_ireduce_scatter_block(m->mx, SB(r), r->r.dev, (size_t)rcount, slot, opi, m->nb_stream, &q);
    *ret = post(r, rc, q, persistent, request);
    return 0;
}

static int mx_coll_ireduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, struct ompi_datatype_t *dtype,
                                   struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                   struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!rs_like(m, sbuf, rbuf, rcounts, 0, dtype, op, comm, 0, request, &ret)) return ret;
    size_t total = 0;
    const int rank = mx_ompi_host->comm_rank(comm), inpl = sbuf == MPI_IN_PLACE;
    for (int i = 0; i < mx_ompi_host->comm_size(comm); i++) total += (size_t)rcounts[i];
#define H(hs, hr, rq) m->prev_ireduce_scatter(hs, hr, rcounts, dtype, op, comm, rq, m->prev_ireduce_scatter_module)
    MX_HOST_NB(m, sbuf, dtype, total, rbuf, dtype, inpl ? total : (size_t)rcounts[rank], inpl, 0, request, H);
#undef H
}

static int mx_coll_reduce_scatter_init(const void *sbuf, void *rbuf, const int *rcounts,
                                       struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                       struct ompi_communicator_t *comm, struct ompi_info_t *info,
                                       struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!rs_like(m, sbuf, rbuf, rcounts, 0, dtype, op, comm, 1, request, &ret)) return ret;
    size_t total = 0;
    const int rank = mx_ompi_host->comm_rank(comm), inpl = sbuf == MPI_IN_PLACE;
    for (int i = 0; i < mx_ompi_host->comm_size(comm); i++) total += (size_t)rcounts[i];
#define H(hs, hr, rq) \
    m->prev_reduce_scatter_init(hs, hr, rcounts, dtype, op, comm, info, rq, m->prev_reduce_scatter_init_module)
    MX_HOST_NB(m, sbuf, dtype, total, rbuf, dtype, inpl ? total : (size_t)rcounts[rank], inpl, 1, request, H);
#undef H
}

static int mx_coll_ireduce_scatter_block(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dtype,
                                         struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                         struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!rs_like(m, sbuf, rbuf, NULL, rcount, dtype, op, comm, 0, request, &ret)) return ret;
    const size_t total = (size_t)rcount * mx_ompi_host->comm_size(comm);
    const int inpl = sbuf == MPI_IN_PLACE;
#define H(hs, hr, rq) \
    m->prev_ireduce_scatter_block(hs, hr, rcount, dtype, op, comm, rq, m->prev_ireduce_scatter_block_module)
    MX_HOST_NB(m, sbuf, dtype, total, rbuf, dtype, inpl ? total : (size_t)rcount, inpl, 0, request, H);
#undef H
}

static int mx_coll_reduce_scatter_block_init(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dtype,
                                             struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                             struct ompi_info_t *info, struct ompi_request_t **request,
                                             mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!rs_like(m, sbuf, rbuf, NULL, rcount, dtype, op, comm, 1, request, &ret)) return ret;
    const size_t total = (size_t)rcount * mx_ompi_host->comm_size(comm);
    const int inpl = sbuf == MPI_IN_PLACE;
#define H(hs, hr, rq) m->prev_reduce_scatter_block_init(hs, hr, rcount, dtype, op, comm, info, rq, \
                                                         m->prev_reduce_scatter_block_init_module)
    MX_HOST_NB(m, sbuf, dtype, total, rbuf, dtype, inpl ? total : (size_t)rcount, inpl, 1, request, H);
#undef H
}

static int scan_like(mx_coll_module_t *m, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                     struct ompi_op_t *op, int exclusive, int persistent, struct ompi_request_t **request, int *ret)
{
    const int n = mx_ompi_host->comm_size(m->comm);
    int slot, opi, rc;
    mx_request_t *q = NULL;
    const size_t bytes = (size_t)count * mx_ompi_host->dtype_size(dtype);
    if (!reducible(dtype, op, (size_t)count, n, &slot, &opi) || !nb_device(m, bytes, 1)) return 1;
    mx_coll_req_t *r = req_setup(m, sbuf, (size_t)count, dtype, rbuf, (size_t)count, dtype,
                                 sbuf == MPI_IN_PLACE || exclusive, bytes, persistent, ret);
    if (!r) return 0;
    const int alg = nbc_alg(exclusive ? "iexscan" : "iscan");
    if (exclusive)
        rc = persistent ? mx_exscan_init(m->mx, SB(r), r->r.dev, (size_t)count, slot, opi, alg, m->nb_stream, &q)
                        : mx_iexscan(m->mx, SB(r), r->r.dev, (size_t)count, slot, opi, alg, m->nb_stream, &q);
    else
        rc = persistent ? mx_scan_init(m->mx, SB(r), r->r.dev, (size_t)count, slot, opi, alg, m->nb_stream, &q)
                        : mx_iscan(m->mx, SB(r), r->r.dev, (size_t)count, slot, opi, alg, m->nb_stream, &q);
    *ret = post(r, rc, q, persistent, request);
    return 0;
}

static int mx_coll_iscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                         struct ompi_communicator_t *comm, struct ompi_request_t **request,
                         mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!scan_like(m, sbuf, rbuf, count, dtype, op, 0, 0, request, &ret)) return ret;
#define H(hs, hr, rq) m->prev_iscan(hs, hr, count, dtype, op, comm, rq, m->prev_iscan_module)
    MX_HOST_NB(m, sbuf, dtype, (size_t)count, rbuf, dtype, (size_t)count, sbuf == MPI_IN_PLACE, 0, request, H);
#undef H
}

static int mx_coll_iexscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                           struct ompi_op_t *op, struct ompi_communicator_t *comm, struct ompi_request_t **request,
                           mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!scan_like(m, sbuf, rbuf, count, dtype, op, 1, 0, request, &ret)) return ret;
#define H(hs, hr, rq) m->prev_iexscan(hs, hr, count, dtype, op, comm, rq, m->prev_iexscan_module)
    MX_HOST_NB(m, sbuf, dtype, (size_t)count, rbuf, dtype, (size_t)count, 1, 0, request, H);
#undef H
}

static int mx_coll_scan_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                             struct ompi_op_t *op, struct ompi_communicator_t *comm, struct ompi_info_t *info,
                             struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!scan_like(m, sbuf, rbuf, count, dtype, op, 0, 1, request, &ret)) return ret;
#define H(hs, hr, rq) m->prev_scan_init(hs, hr, count, dtype, op, comm, info, rq, m->prev_scan_init_module)
    MX_HOST_NB(m, sbuf, dtype, (size_t)count, rbuf, dtype, (size_t)count, sbuf == MPI_IN_PLACE, 1, request, H);
#undef H
}

static int mx_coll_exscan_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                               struct ompi_op_t *op, struct ompi_communicator_t *comm, struct ompi_info_t *info,
                               struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!scan_like(m, sbuf, rbuf, count, dtype, op, 1, 1, request, &ret)) return ret;
#define H(hs, hr, rq) m->prev_exscan_init(hs, hr, count, dtype, op, comm, info, rq, m->prev_exscan_init_module)
    MX_HOST_NB(m, sbuf, dtype, (size_t)count, rbuf, dtype, (size_t)count, 1, 1, request, H);
#undef H
}

static int allgather_like(mx_coll_module_t *m, const void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                          void *rbuf, int rcount, struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                          int persistent, struct ompi_request_t **request, int *ret)
{
    const size_t rbytes = (size_t)rcount * mx_ompi_host->dtype_size(rdtype);
    const int n = mx_ompi_host->comm_size(comm);
    mx_request_t *q = NULL;
    if (!rbytes || n > MX_MAX_RANKS || !nb_device(m, rbytes * n, 0)) return 1;
    if (sbuf != MPI_IN_PLACE && (size_t)scount * mx_ompi_host->dtype_size(sdtype) != rbytes) {
        *ret = OMPI_ERROR;   /* type signatures differ: erroneous program */
        return 0;
    }
    mx_coll_req_t *r = req_setup(m, sbuf, (size_t)scount, sdtype, rbuf, (size_t)rcount * n, rdtype,
                                 sbuf == MPI_IN_PLACE, rbytes * n, persistent, ret);
    if (!r) return 0;
    const int rc = persistent ? mx_allgather_init(m->mx, SB(r), r->r.dev, rbytes, m->nb_stream, &q)
                              : mx_iallgather(m->mx, SB(r), r->r.dev, rbytes, m->nb_stream, &q);
    *ret = post(r, rc, q, persistent, request);
    return 0;
}

static int mx_coll_iallgather(const void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                              struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                              struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!allgather_like(m, sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, 0, request, &ret)) return ret;
    const size_t nr = (size_t)rcount * mx_ompi_host->comm_size(comm);
#define H(hs, hr, rq) m->prev_iallgather(hs, scount, sdtype, hr, rcount, rdtype, comm, rq, m->prev_iallgather_module)
    MX_HOST_NB(m, sbuf, sdtype, (size_t)scount, rbuf, rdtype, nr, sbuf == MPI_IN_PLACE, 0, request, H);
#undef H
}

static int mx_coll_allgather_init(const void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf,
                                  int rcount, struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                                  struct ompi_info_t *info, struct ompi_request_t **request,
                                  mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!allgather_like(m, sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, 1, request, &ret)) return ret;
    const size_t nr = (size_t)rcount * mx_ompi_host->comm_size(comm);
#define H(hs, hr, rq) m->prev_allgather_init(hs, scount, sdtype, hr, rcount, rdtype, comm, info, rq, \
                                             m->prev_allgather_init_module)
    MX_HOST_NB(m, sbuf, sdtype, (size_t)scount, rbuf, rdtype, nr, sbuf == MPI_IN_PLACE, 1, request, H);
#undef H
}

static int bcast_like(mx_coll_module_t *m, void *buf, int count, struct ompi_datatype_t *dtype, int root,
                      int persistent, struct ompi_request_t **request, int *ret)
{
    const size_t bytes = (size_t)count * mx_ompi_host->dtype_size(dtype);
    const int n = mx_ompi_host->comm_size(m->comm), rank = mx_ompi_host->comm_rank(m->comm);
    mx_request_t *q = NULL;
    if (!bytes || n > MX_MAX_RANKS || !nb_device(m, bytes, 0)) return 1;
    mx_coll_req_t *r = req_setup(m, NULL, 0, NULL, buf, (size_t)count, dtype, rank == root,
                                 rank == root ? 0 : bytes, persistent, ret);
    if (!r) return 0;
    const int rc = persistent ? mx_bcast_init(m->mx, r->r.dev, bytes, root, m->nb_stream, &q)
                              : mx_ibcast(m->mx, r->r.dev, bytes, root, m->nb_stream, &q);
    *ret = post(r, rc, q, persistent, request);
    return 0;
}

static int mx_coll_ibcast(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                          struct ompi_communicator_t *comm, struct ompi_request_t **request,
                          mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!bcast_like(m, buf, count, dtype, root, 0, request, &ret)) return ret;
    const int is_root = mx_ompi_host->comm_rank(comm) == root;
#define H(hs, hr, rq) ((void)(hs), m->prev_ibcast(hr, count, dtype, root, comm, rq, m->prev_ibcast_module))
    MX_HOST_NB(m, NULL, dtype, 0, buf, dtype, (size_t)count, is_root, 0, request, H);
#undef H
}

static int mx_coll_bcast_init(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                              struct ompi_communicator_t *comm, struct ompi_info_t *info,
                              struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!bcast_like(m, buf, count, dtype, root, 1, request, &ret)) return ret;
    const int is_root = mx_ompi_host->comm_rank(comm) == root;
#define H(hs, hr, rq) ((void)(hs), m->prev_bcast_init(hr, count, dtype, root, comm, info, rq, m->prev_bcast_init_module))
    MX_HOST_NB(m, NULL, dtype, 0, buf, dtype, (size_t)count, is_root, 1, request, H);
#undef H
}

/* ---- module enable / component query ------------------------------------ */

#define SAVE_PREV(m, comm, name, type)                                                              \
    do {                                                                                            \
        mca_coll_base_module_t *pm_ = NULL;                                                         \
        (m)->prev_##name = (type)mx_ompi_host->comm_coll_fn((comm), #name, &pm_);                   \
        (m)->prev_##name##_module = pm_;                                                            \
        if (!(m)->prev_##name || !pm_) return OMPI_ERR_NOT_FOUND;                                   \
        MX_OBJ_RETAIN(pm_);                                                                         \
    } while (0)

static int mx_coll_module_enable(mca_coll_base_module_t *module, struct ompi_communicator_t *comm)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const int n = mx_ompi_host->comm_size(comm);
    m->comm = comm;
    if (n == 1) {
        /* size 1: a slot whose lower module is missing is left to the
         * framework (cleared before mca_coll_base_comm_select copies it) */
#define SAVE_PREV_SELF(name)                                                                        \
    if (m->super.coll_##name) {                                                                     \
        mca_coll_base_module_t *pm_ = NULL;                                                         \
        m->prev_##name = (__typeof__(m->prev_##name))mx_ompi_host->comm_coll_fn(comm, #name, &pm_); \
        m->prev_##name##_module = pm_;                                                              \
        if (m->prev_##name && pm_) MX_OBJ_RETAIN(pm_);                                              \
        else { m->prev_##name = NULL; m->prev_##name##_module = NULL; m->super.coll_##name = NULL; } \
    }
        SAVE_PREV_SELF(allreduce) SAVE_PREV_SELF(reduce_scatter) SAVE_PREV_SELF(allgather) SAVE_PREV_SELF(reduce)
        SAVE_PREV_SELF(reduce_scatter_block) SAVE_PREV_SELF(scan)
#undef SAVE_PREV_SELF
        if (m->super.coll_reduce_local) SAVE_PREV(m, comm, reduce_local, mca_coll_base_module_reduce_local_fn_t);
        m->mx_state = -1;   /* no peers: no device communicator */
        return OMPI_SUCCESS;
    }
    if (m->super.coll_allreduce) {
        SAVE_PREV(m, comm, allreduce, mca_coll_base_module_allreduce_fn_t);
        SAVE_PREV(m, comm, reduce_scatter, mca_coll_base_module_reduce_scatter_fn_t);
        SAVE_PREV(m, comm, allgather, mca_coll_base_module_allgather_fn_t);
        SAVE_PREV(m, comm, bcast, mca_coll_base_module_bcast_fn_t);
        SAVE_PREV(m, comm, reduce, mca_coll_base_module_reduce_fn_t);
        SAVE_PREV(m, comm, reduce_scatter_block, mca_coll_base_module_reduce_scatter_block_fn_t);
        SAVE_PREV(m, comm, scan, mca_coll_base_module_scan_fn_t);
        SAVE_PREV(m, comm, exscan, mca_coll_base_module_exscan_fn_t);
    }
    if (m->super.coll_reduce_local) SAVE_PREV(m, comm, reduce_local, mca_coll_base_module_reduce_local_fn_t);
    /* nonblocking / persistent: take a slot only where a lower module
     * (coll/libnbc) provides it for delegation; mca_coll_base_comm_select
     * copies the slots after enable, so a cleared one stays theirs */
#define SAVE_PREV_OPT(name)                                                                         \
    if (m->super.coll_##name) {                                                                     \
        mca_coll_base_module_t *pm_ = NULL;                                                         \
        m->prev_##name = (__typeof__(m->prev_##name))mx_ompi_host->comm_coll_fn(comm, #name, &pm_); \
        m->prev_##name##_module = pm_;                                                              \
        if (m->prev_##name && pm_) MX_OBJ_RETAIN(pm_);                                              \
        else { m->prev_##name = NULL; m->prev_##name##_module = NULL; m->super.coll_##name = NULL; } \
    }
    MX_NB_SLOTS(SAVE_PREV_OPT)
#undef SAVE_PREV_OPT
    /* the reduction orders of the saved modules, coll/tuned's configuration
     * (read at enable, as ompi_coll_tuned_forced_getvalues does), the size
     * split (identical on every rank: MCA variables are job-wide) */
    m->low_allreduce = low_kind(m->prev_allreduce_module);
    m->low_reduce_scatter = low_kind(m->prev_reduce_scatter_module);
    m->low_reduce = low_kind(m->prev_reduce_module);
    m->low_rsb = low_kind(m->prev_reduce_scatter_block_module);
    m->low_scan = low_kind(m->prev_scan_module);
    m->low_exscan = low_kind(m->prev_exscan_module);
    m->low_nbc = low_kind(m->prev_iallreduce_module);
    m->basic_crossover = mx_ompi_host->mca_int("coll_basic_crossover", 4);   /* coll_basic_component.c:98-104 */
    {
        const int kb = mx_ompi_host->mca_int("coll_mi355x_host_max_kb", 64);
        m->host_max = kb > 0 ? (size_t)kb << 10 : 0;
    }
    (void)mx_tuned_cfg_load(&m->tuned, n);
    /* the device communicator (IPC staging, flags) is created at the first
     * eligible collective, so a communicator that never runs one on the
     * device -- an MPI_Comm_dup kept for a library, say -- costs no device
     * memory; communicators above the all-peer path's rank limit delegate */
    m->mx_state = (n > 1 && n <= MX_MAX_RANKS) ? 0 : -1;
    return OMPI_SUCCESS;
}

static int mx_coll_component_init_query(bool enable_progress_threads, bool enable_mpi_threads)
{
    (void)enable_progress_threads;
    (void)enable_mpi_threads;
    if (!mx_ompi_host) return OMPI_ERR_NOT_SUPPORTED;
    return mx_init(-1) == MX_SUCCESS ? OMPI_SUCCESS : OMPI_ERR_NOT_SUPPORTED;
}

static mca_coll_base_module_t *mx_coll_component_comm_query(struct ompi_communicator_t *comm, int *priority)
{
    mx_coll_module_t *m;
    const int n = mx_ompi_host->comm_size(comm);
    *priority = mx_ompi_host->mca_int("coll_mi355x_priority", 80);
    if (*priority < 0) return NULL;
    /* intra-communicator semantics only: the intercommunicator forms
     * (remote-group results, coll/inter and coll/basic's _inter functions)
     * stay with the components built for them, as coll/tuned
     * (coll_tuned_module.c:66-69) and coll/cuda (coll_cuda_module.c:141) do */
    if (mx_ompi_host->comm_is_inter && mx_ompi_host->comm_is_inter(comm)) {
        *priority = 0;
        return NULL;
    }
    m = MX_MODULE_NEW(mx_coll_module_t, super);
    if (!m) return NULL;
    m->super.coll_module_enable = mx_coll_module_enable;
    if (n > 1) {
        m->super.coll_allreduce = mx_coll_allreduce;
        m->super.coll_reduce_scatter = mx_coll_reduce_scatter;
        m->super.coll_allgather = mx_coll_allgather;
        m->super.coll_bcast = mx_coll_bcast;
        m->super.coll_reduce = mx_coll_reduce;
        m->super.coll_reduce_scatter_block = mx_coll_reduce_scatter_block;
        m->super.coll_scan = mx_coll_scan;
        m->super.coll_exscan = mx_coll_exscan;
#define SET_NB(name) m->super.coll_##name = mx_coll_##name;
        MX_NB_SLOTS(SET_NB)
#undef SET_NB
    } else {
        /* size-1 comms (MPI_COMM_SELF): coll/self's slots (priority 75,
         * coll_self_module.c:60-84) with device copies for device buffers;
         * MPI_Reduce_local lands here when our priority beats 75 */
        m->super.coll_allreduce = mx_self_allreduce;
        m->super.coll_reduce_scatter = mx_self_reduce_scatter;
        m->super.coll_allgather = mx_self_allgather;
        m->super.coll_reduce = mx_self_reduce;
        m->super.coll_reduce_scatter_block = mx_self_reduce_scatter_block;
        m->super.coll_scan = mx_self_scan;
        m->super.coll_exscan = mx_self_exscan;
    }
    if (*priority > 75) m->super.coll_reduce_local = mx_coll_reduce_local;
    return &m->super;
}

#ifdef MX_OMPI_REAL
int mx_ompi_host_real_register(void);
static int mx_coll_component_open(void) { return mx_ompi_host_real_register(); }
#endif

mca_coll_base_component_2_0_0_t mca_coll_mi355x_component = {
    .collm_version = {
        .mca_major_version = 2, .mca_minor_version = 1, .mca_release_version = 0,
        .mca_project_name = "ompi",
        .mca_type_name = "coll", .mca_type_major_version = 2,
        .mca_component_name = "mi355x", .mca_component_major_version = 1,
#ifdef MX_OMPI_REAL
        .mca_open_component = mx_coll_component_open,
#endif
    },
    .collm_init_query = mx_coll_component_init_query,
    .collm_comm_query = mx_coll_component_comm_query,
};
