/*
 * coll_mi355x.c -- the `mi355x` component of Open MPI's `coll` framework.
 *
 * Takes the allreduce / reduce_scatter / allgather / bcast slots (plus
 * reduce / reduce_scatter_block / scan / exscan and, above coll/self's
 * priority, reduce_local) of a communicator and runs them
 * on the MI355X all-peer path of libmx_kernels.so (include/mx_coll.h) when
 * the buffers are device memory; everything else is handed to the module
 * that owned the slot before us.
 *
 * Follows the reference's stacking accelerator component, coll/cuda:
 *  - comm_query returns a module with only the slots we implement
 *    (coll_cuda_module.c:79-117); priority 80 by default (above tuned's 30
 *    and coll/cuda's 78, below coll/self's 75 only for reduce_local unless
 *    raised), MCA var coll_mi355x_priority;
 *  - module_enable saves and RETAINs the previous c_coll slot + module for
 *    delegation (CHECK_AND_RETAIN, coll_cuda_module.c:120-155) and fails with
 *    OMPI_ERR_NOT_FOUND if a needed lower slot is missing;
 *  - the device/host decision is taken per call from the buffers
 *    (coll_cuda_allreduce.c:39-56) -- but instead of staging through host
 *    memory the device path runs the collective on the GPUs.
 * The nonblocking and persistent slots (iallreduce, ireduce, ireduce_scatter,
 * ireduce_scatter_block, iscan, iexscan, iallgather, ibcast and their
 * *_init forms) replace coll/libnbc's for device buffers: the collective is
 * enqueued on the GPU and the request completes through a progress
 * callback that polls its event (libnbc's ompi_coll_libnbc_progress,
 * coll_libnbc_component.c:426-482, progresses the schedule on the host
 * instead); reduction orders are libnbc's, algorithm selection follows the
 * coll_libnbc_<coll>_algorithm vars (coll_mi355x_<coll>_algorithm wins).
 * The algorithm is chosen with coll/tuned's fixed decision
 * (coll_tuned_decision_fixed.c:44-95, :466-512) unless forced with the MCA
 * vars coll_mi355x_allreduce_algorithm / coll_mi355x_reduce_scatter_algorithm
 * (same numbering as coll_tuned_*_algorithm), so results match coll/tuned
 * bit for bit.  The mx communicator is created at enable time with the
 * saved host allgather as the bootstrap exchange.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mx_coll.h"
#include "mx_kernels.h"
#include "mx_ompi_abi.h"

typedef struct {
    mca_coll_base_module_t super;
    struct ompi_communicator_t *comm;
    mx_comm_t *mx;
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

static int map_rc(int rc)
{
    switch (rc) {
    case MX_SUCCESS: return OMPI_SUCCESS;
    case MX_ERR_NOMEM: return OMPI_ERR_OUT_OF_RESOURCE;
    case MX_ERR_UNSUPPORTED: return OMPI_ERR_NOT_SUPPORTED;
    default: return OMPI_ERROR;
    }
}

static void coll_module_destruct(void *obj)
{
    mx_coll_module_t *m = (mx_coll_module_t *)obj;
    if (m->mx) mx_comm_destroy(m->mx);
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
    free(m);
}

static mx_obj_class_t mx_coll_module_class = {"mx_coll_module_t", coll_module_destruct};

static int on_device(const void *p) { return p != MPI_IN_PLACE && mx_is_device_ptr(p) == 1; }

/* Bootstrap exchange for mx_comm_create: the saved host allgather on
 * MPI_BYTE buffers (host memory, so it never recurses into us). */
static int bootstrap_allgather(const void *send, void *recv, size_t bytes, void *ctx)
{
    mx_coll_module_t *m = (mx_coll_module_t *)ctx;
    return m->prev_allgather(send, (int)bytes, mx_ompi_host->byte_dtype, recv, (int)bytes,
                             mx_ompi_host->byte_dtype, m->comm, m->prev_allgather_module);
}

/* ---- slots -------------------------------------------------------------- */

static int mx_coll_allreduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                             struct ompi_op_t *op, struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const int slot = mx_ompi_host->dtype_slot(dtype);
    const int opi = mx_ompi_host->op_index(op);
    const int sb_dev = (sbuf == MPI_IN_PLACE) ? 1 : on_device(sbuf);
    if (m->mx && count > 0 && slot >= 0 && (mx_ompi_host->op_flags(op) & OMPI_OP_FLAGS_INTRINSIC) &&
        mx_op_supported(opi, slot, MX_TABLE_WITH_FORTRAN) && mx_ompi_host->dtype_contiguous(dtype, count) &&
        sb_dev && on_device(rbuf)) {
        const int alg = mx_ompi_host->mca_int("coll_mi355x_allreduce_algorithm", MX_ALLREDUCE_AUTO);
        int rc = mx_allreduce(m->mx, sbuf == MPI_IN_PLACE ? MX_IN_PLACE : sbuf, rbuf, (size_t)count, slot, opi,
                              alg, NULL);
        if (rc != MX_ERR_UNSUPPORTED) return map_rc(rc);
    }
    return m->prev_allreduce(sbuf, rbuf, count, dtype, op, comm, m->prev_allreduce_module);
}

static int mx_coll_reduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, struct ompi_datatype_t *dtype,
                                  struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                  mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const int slot = mx_ompi_host->dtype_slot(dtype);
    const int opi = mx_ompi_host->op_index(op);
    const int n = mx_ompi_host->comm_size(comm);
    if (m->mx && slot >= 0 && (mx_ompi_host->op_flags(op) & OMPI_OP_FLAGS_INTRINSIC) &&
        mx_op_supported(opi, slot, MX_TABLE_WITH_FORTRAN) && n <= MX_MAX_RANKS &&
        (sbuf == MPI_IN_PLACE || on_device(sbuf)) && on_device(rbuf)) {
        size_t rc64[MX_MAX_RANKS];
        int total = 0;
        for (int i = 0; i < n; i++) { rc64[i] = (size_t)rcounts[i]; total += rcounts[i]; }
        if (mx_ompi_host->dtype_contiguous(dtype, total)) {
            const int alg = mx_ompi_host->mca_int("coll_mi355x_reduce_scatter_algorithm", MX_RS_AUTO);
            int rc = mx_reduce_scatter(m->mx, sbuf == MPI_IN_PLACE ? MX_IN_PLACE : sbuf, rbuf, rc64, slot, opi,
                                       alg, NULL);
            if (rc != MX_ERR_UNSUPPORTED && rc != MX_ERR_NOMEM) return map_rc(rc);
        }
    }
    return m->prev_reduce_scatter(sbuf, rbuf, rcounts, dtype, op, comm, m->prev_reduce_scatter_module);
}

static int mx_coll_allgather(const void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                             struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                             mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const size_t rbytes = (size_t)rcount * mx_ompi_host->dtype_size(rdtype);
    const int n = mx_ompi_host->comm_size(comm);
    if (m->mx && rbytes && on_device(rbuf) && mx_ompi_host->dtype_contiguous(rdtype, rcount * n) &&
        (sbuf == MPI_IN_PLACE ||
         (on_device(sbuf) && mx_ompi_host->dtype_contiguous(sdtype, scount) &&
          (size_t)scount * mx_ompi_host->dtype_size(sdtype) == rbytes))) {
        int rc = mx_allgather(m->mx, sbuf == MPI_IN_PLACE ? MX_IN_PLACE : sbuf, rbuf, rbytes, NULL);
        if (rc != MX_ERR_UNSUPPORTED) return map_rc(rc);
    }
    return m->prev_allgather(sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, m->prev_allgather_module);
}

static int mx_coll_bcast(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                         struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const size_t bytes = (size_t)count * mx_ompi_host->dtype_size(dtype);
    if (m->mx && bytes && on_device(buf) && mx_ompi_host->dtype_contiguous(dtype, count)) {
        int rc = mx_bcast(m->mx, buf, bytes, root, NULL);
        if (rc != MX_ERR_UNSUPPORTED) return map_rc(rc);
    }
    return m->prev_bcast(buf, count, dtype, root, comm, m->prev_bcast_module);
}

static int mx_coll_reduce_local(const void *inbuf, void *inoutbuf, int count, struct ompi_datatype_t *dtype,
                                struct ompi_op_t *op, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const int slot = mx_ompi_host->dtype_slot(dtype);
    const int opi = mx_ompi_host->op_index(op);
    if (count > 0 && slot >= 0 && (mx_ompi_host->op_flags(op) & OMPI_OP_FLAGS_INTRINSIC) &&
        mx_op_supported(opi, slot, MX_TABLE_WITH_FORTRAN) && on_device(inbuf) && on_device(inoutbuf)) {
        int rc = mx_reduce2(opi, slot, inbuf, inoutbuf, (size_t)count, NULL);
        if (rc == MX_SUCCESS) rc = mx_stream_sync(NULL);
        return map_rc(rc);
    }
    return m->prev_reduce_local(inbuf, inoutbuf, count, dtype, op, m->prev_reduce_local_module);
}

/* Reduction slots beyond the four of the north star:
 * MPI_Reduce (coll.h:239-241), MPI_Reduce_scatter_block (:245-247),
 * MPI_Scan / MPI_Exscan (:248-250, :228-230).  Same device / host split
 * and delegation; algorithms follow coll/tuned's fixed decisions (reduce:
 * coll_tuned_decision_fixed.c:354-429; reduce_scatter_block: basic_linear,
 * :522-532) and coll/basic's linear scan / exscan (tuned leaves those slots
 * empty, coll_tuned_module.c:106,112), or the forced algorithm of the MCA
 * vars coll_mi355x_{reduce,scan,exscan}_algorithm (tuned's numbering). */
static int reducible(mx_coll_module_t *m, struct ompi_datatype_t *dtype, struct ompi_op_t *op, int count, int *slot,
                     int *opi)
{
    *slot = mx_ompi_host->dtype_slot(dtype);
    *opi = mx_ompi_host->op_index(op);
    return m->mx && count > 0 && *slot >= 0 && (mx_ompi_host->op_flags(op) & OMPI_OP_FLAGS_INTRINSIC) &&
           mx_op_supported(*opi, *slot, MX_TABLE_WITH_FORTRAN) && mx_ompi_host->dtype_contiguous(dtype, count);
}

static int mx_coll_reduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                          struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                          mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const int rank = mx_ompi_host->comm_rank(comm);
    int slot, opi;
    /* rbuf matters on the root only (MPI-3.1 5.9.1) */
    if (reducible(m, dtype, op, count, &slot, &opi) && (sbuf == MPI_IN_PLACE ? rank == root : on_device(sbuf)) &&
        (rank != root || on_device(rbuf))) {
        const int alg = mx_ompi_host->mca_int("coll_mi355x_reduce_algorithm", MX_REDUCE_AUTO);
        int rc = mx_reduce(m->mx, sbuf == MPI_IN_PLACE ? MX_IN_PLACE : sbuf, rank == root ? rbuf : NULL,
                           (size_t)count, slot, opi, root, alg, NULL);
        if (rc != MX_ERR_UNSUPPORTED) return map_rc(rc);
    }
    return m->prev_reduce(sbuf, rbuf, count, dtype, op, root, comm, m->prev_reduce_module);
}

static int mx_coll_reduce_scatter_block(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dtype,
                                        struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                        mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    const int n = mx_ompi_host->comm_size(comm);
    int slot, opi;
    if (reducible(m, dtype, op, rcount * n, &slot, &opi) && (sbuf == MPI_IN_PLACE || on_device(sbuf)) &&
        on_device(rbuf)) {
        const int alg = mx_ompi_host->mca_int("coll_mi355x_reduce_algorithm", MX_REDUCE_AUTO);
        int rc = mx_reduce_scatter_block(m->mx, sbuf == MPI_IN_PLACE ? MX_IN_PLACE : sbuf, rbuf, (size_t)rcount,
                                         slot, opi, alg, NULL);
        if (rc != MX_ERR_UNSUPPORTED) return map_rc(rc);
    }
    return m->prev_reduce_scatter_block(sbuf, rbuf, rcount, dtype, op, comm, m->prev_reduce_scatter_block_module);
}

static int scan_common(mx_coll_module_t *m, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                       struct ompi_op_t *op, int exclusive)
{
    int slot, opi;
    if (reducible(m, dtype, op, count, &slot, &opi) && (sbuf == MPI_IN_PLACE || on_device(sbuf)) &&
        on_device(rbuf)) {
        const int alg = mx_ompi_host->mca_int(exclusive ? "coll_mi355x_exscan_algorithm"
                                                        : "coll_mi355x_scan_algorithm", MX_SCAN_AUTO);
        const void *sb = sbuf == MPI_IN_PLACE ? MX_IN_PLACE : sbuf;
        int rc = exclusive ? mx_exscan(m->mx, sb, rbuf, (size_t)count, slot, opi, alg, NULL)
                           : mx_scan(m->mx, sb, rbuf, (size_t)count, slot, opi, alg, NULL);
        if (rc != MX_ERR_UNSUPPORTED) return map_rc(rc);
    }
    return 1;   /* delegate */
}

static int mx_coll_scan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                        struct ompi_op_t *op, struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int rc = scan_common(m, sbuf, rbuf, count, dtype, op, 0);
    return rc != 1 ? rc : m->prev_scan(sbuf, rbuf, count, dtype, op, comm, m->prev_scan_module);
}

static int mx_coll_exscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                          struct ompi_op_t *op, struct ompi_communicator_t *comm, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int rc = scan_common(m, sbuf, rbuf, count, dtype, op, 1);
    return rc != 1 ? rc : m->prev_exscan(sbuf, rbuf, count, dtype, op, comm, m->prev_exscan_module);
}

/* ---- nonblocking and persistent slots ------------------
 * A device-path request is an mx_request_t (include/mx_coll.h) wrapped in a
 * host ompi_request_t; active ones sit on a list that the progress callback
 * (registered once, like libnbc's) polls with mx_test and completes.  The
 * GPU needs no host progress: polling only reports completion. */
typedef struct mx_coll_req {
    struct ompi_request_t *req;
    mx_request_t *mx;
    struct mx_coll_req *next;
    int active;
} mx_coll_req_t;

static mx_coll_req_t *g_active;
static int g_progress_registered;

static int mx_coll_progress(void)
{
    int completed = 0;
    mx_coll_req_t **pp = &g_active;
    while (*pp) {
        mx_coll_req_t *r = *pp;
        int flag = 0;
        const int rc = mx_test(r->mx, &flag);
        if (flag || rc != MX_SUCCESS) {
            *pp = r->next;
            r->active = 0;
            mx_ompi_host->request_complete(r->req, map_rc(rc));
            completed++;
        } else {
            pp = &r->next;
        }
    }
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
    const int rc = mx_start(r->mx);
    if (rc != MX_SUCCESS) return map_rc(rc);
    mx_ompi_host->request_activate(req);
    activate(r);
    return OMPI_SUCCESS;
}

static int req_free_cb(struct ompi_request_t *req)      /* MPI_Request_free */
{
    mx_coll_req_t *r = (mx_coll_req_t *)mx_ompi_host->request_ctx(req);
    if (r->active) deactivate(r);
    const int rc = mx_request_free(r->mx);   /* lets an active operation finish */
    free(r);
    return map_rc(rc);
}

/* wrap an mx request (rc from its creation) into *request; returns 1 when
 * the call should be delegated instead */
static int post(int rc, mx_request_t *mxr, int persistent, struct ompi_request_t **request, int *ret)
{
    if (rc == MX_ERR_UNSUPPORTED || rc == MX_ERR_NOMEM) return 1;
    if (rc != MX_SUCCESS) { *ret = map_rc(rc); return 0; }
    mx_coll_req_t *r = calloc(1, sizeof *r);
    if (r) r->req = mx_ompi_host->request_create(persistent, req_start_cb, req_free_cb, r);
    if (!r || !r->req) {
        mx_request_free(mxr);
        free(r);
        *ret = OMPI_ERR_OUT_OF_RESOURCE;
        return 0;
    }
    r->mx = mxr;
    if (!g_progress_registered) {
        mx_ompi_host->progress_register(mx_coll_progress);
        g_progress_registered = 1;
    }
    if (!persistent) activate(r);
    *request = r->req;
    *ret = OMPI_SUCCESS;
    return 0;
}

/* coll_mi355x_<name>_algorithm, defaulting to coll_libnbc_<name>_algorithm */
static int nbc_alg(const char *name)
{
    char a[96], b[96];
    snprintf(a, sizeof a, "coll_mi355x_%s_algorithm", name);
    snprintf(b, sizeof b, "coll_libnbc_%s_algorithm", name);
    return mx_ompi_host->mca_int(a, mx_ompi_host->mca_int(b, 0));
}

static int allreduce_like(mx_coll_module_t *m, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                          struct ompi_op_t *op, int persistent, struct ompi_request_t **request, int *ret)
{
    int slot, opi;
    mx_request_t *q = NULL;
    if (!reducible(m, dtype, op, count, &slot, &opi) || !(sbuf == MPI_IN_PLACE || on_device(sbuf)) ||
        !on_device(rbuf))
        return 1;
    const void *sb = sbuf == MPI_IN_PLACE ? MX_IN_PLACE : sbuf;
    const int alg = nbc_alg("iallreduce");
    const int rc = persistent ? mx_allreduce_init(m->mx, sb, rbuf, (size_t)count, slot, opi, alg, NULL, &q)
                              : mx_iallreduce(m->mx, sb, rbuf, (size_t)count, slot, opi, alg, NULL, &q);
    return post(rc, q, persistent, request, ret);
}

static int mx_coll_iallreduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                              struct ompi_op_t *op, struct ompi_communicator_t *comm, struct ompi_request_t **request,
                              mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!allreduce_like(m, sbuf, rbuf, count, dtype, op, 0, request, &ret)) return ret;
    return m->prev_iallreduce(sbuf, rbuf, count, dtype, op, comm, request, m->prev_iallreduce_module);
}

static int mx_coll_allreduce_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                                  struct ompi_op_t *op, struct ompi_communicator_t *comm, struct ompi_info_t *info,
                                  struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!allreduce_like(m, sbuf, rbuf, count, dtype, op, 1, request, &ret)) return ret;
    return m->prev_allreduce_init(sbuf, rbuf, count, dtype, op, comm, info, request,
                                  m->prev_allreduce_init_module);
}

static int reduce_like(mx_coll_module_t *m, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                       struct ompi_op_t *op, int root, struct ompi_communicator_t *comm, int persistent,
                       struct ompi_request_t **request, int *ret)
{
    const int rank = mx_ompi_host->comm_rank(comm);
    int slot, opi;
    mx_request_t *q = NULL;
    if (!reducible(m, dtype, op, count, &slot, &opi) || !(sbuf == MPI_IN_PLACE ? rank == root : on_device(sbuf)) ||
        (rank == root && !on_device(rbuf)))
        return 1;
    const void *sb = sbuf == MPI_IN_PLACE ? MX_IN_PLACE : sbuf;
    void *rb = rank == root ? rbuf : NULL;
    const int alg = nbc_alg("ireduce");
    const int rc = persistent ? mx_reduce_init(m->mx, sb, rb, (size_t)count, slot, opi, root, alg, NULL, &q)
                              : mx_ireduce(m->mx, sb, rb, (size_t)count, slot, opi, root, alg, NULL, &q);
    return post(rc, q, persistent, request, ret);
}

static int mx_coll_ireduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                           int root, struct ompi_communicator_t *comm, struct ompi_request_t **request,
                           mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!reduce_like(m, sbuf, rbuf, count, dtype, op, root, comm, 0, request, &ret)) return ret;
    return m->prev_ireduce(sbuf, rbuf, count, dtype, op, root, comm, request, m->prev_ireduce_module);
}

static int mx_coll_reduce_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                               struct ompi_op_t *op, int root, struct ompi_communicator_t *comm,
                               struct ompi_info_t *info, struct ompi_request_t **request,
                               mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!reduce_like(m, sbuf, rbuf, count, dtype, op, root, comm, 1, request, &ret)) return ret;
    return m->prev_reduce_init(sbuf, rbuf, count, dtype, op, root, comm, info, request, m->prev_reduce_init_module);
}

/* rcounts == NULL: the _block form with `rcount` per rank */
static int rs_like(mx_coll_module_t *m, const void *sbuf, void *rbuf, const int *rcounts, int rcount,
                   struct ompi_datatype_t *dtype, struct ompi_op_t *op, struct ompi_communicator_t *comm,
                   int persistent, struct ompi_request_t **request, int *ret)
{
    const int n = mx_ompi_host->comm_size(comm);
    size_t rc64[MX_MAX_RANKS];
    int total = 0, slot, opi;
    mx_request_t *q = NULL;
    if (n > MX_MAX_RANKS) return 1;
    for (int i = 0; i < n; i++) { rc64[i] = (size_t)(rcounts ? rcounts[i] : rcount); total += (int)rc64[i]; }
    if (!reducible(m, dtype, op, total, &slot, &opi) || !(sbuf == MPI_IN_PLACE || on_device(sbuf)) ||
        !on_device(rbuf))
        return 1;
    const void *sb = sbuf == MPI_IN_PLACE ? MX_IN_PLACE : sbuf;
    int rc;
    if (rcounts)
        rc = persistent ? mx_reduce_scatter_init(m->mx, sb, rbuf, rc64, slot, opi, NULL, &q)
                        : mx_ireduce_scatter(m->mx, sb, rbuf, rc64, slot, opi, NULL, &q);
    else
        rc = persistent ? mx_reduce_scatter_block_init(m->mx, sb, rbuf, (size_t)rcount, slot, opi, NULL, &q)
                        : mx_ireduce_scatter_block(m->mx, sb, rbuf, (size_t)rcount, slot, opi, NULL, &q);
    return post(rc, q, persistent, request, ret);
}

static int mx_coll_ireduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, struct ompi_datatype_t *dtype,
                                   struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                   struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!rs_like(m, sbuf, rbuf, rcounts, 0, dtype, op, comm, 0, request, &ret)) return ret;
    return m->prev_ireduce_scatter(sbuf, rbuf, rcounts, dtype, op, comm, request, m->prev_ireduce_scatter_module);
}

static int mx_coll_reduce_scatter_init(const void *sbuf, void *rbuf, const int *rcounts,
                                       struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                       struct ompi_communicator_t *comm, struct ompi_info_t *info,
                                       struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!rs_like(m, sbuf, rbuf, rcounts, 0, dtype, op, comm, 1, request, &ret)) return ret;
    return m->prev_reduce_scatter_init(sbuf, rbuf, rcounts, dtype, op, comm, info, request,
                                       m->prev_reduce_scatter_init_module);
}

static int mx_coll_ireduce_scatter_block(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dtype,
                                         struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                         struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!rs_like(m, sbuf, rbuf, NULL, rcount, dtype, op, comm, 0, request, &ret)) return ret;
    return m->prev_ireduce_scatter_block(sbuf, rbuf, rcount, dtype, op, comm, request,
                                         m->prev_ireduce_scatter_block_module);
}

static int mx_coll_reduce_scatter_block_init(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dtype,
                                             struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                             struct ompi_info_t *info, struct ompi_request_t **request,
                                             mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!rs_like(m, sbuf, rbuf, NULL, rcount, dtype, op, comm, 1, request, &ret)) return ret;
    return m->prev_reduce_scatter_block_init(sbuf, rbuf, rcount, dtype, op, comm, info, request,
                                             m->prev_reduce_scatter_block_init_module);
}

static int scan_like(mx_coll_module_t *m, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                     struct ompi_op_t *op, int exclusive, int persistent, struct ompi_request_t **request, int *ret)
{
    int slot, opi, rc;
    mx_request_t *q = NULL;
    if (!reducible(m, dtype, op, count, &slot, &opi) || !(sbuf == MPI_IN_PLACE || on_device(sbuf)) ||
        !on_device(rbuf))
        return 1;
    const void *sb = sbuf == MPI_IN_PLACE ? MX_IN_PLACE : sbuf;
    const int alg = nbc_alg(exclusive ? "iexscan" : "iscan");
    if (exclusive)
        rc = persistent ? mx_exscan_init(m->mx, sb, rbuf, (size_t)count, slot, opi, alg, NULL, &q)
                        : mx_iexscan(m->mx, sb, rbuf, (size_t)count, slot, opi, alg, NULL, &q);
    else
        rc = persistent ? mx_scan_init(m->mx, sb, rbuf, (size_t)count, slot, opi, alg, NULL, &q)
                        : mx_iscan(m->mx, sb, rbuf, (size_t)count, slot, opi, alg, NULL, &q);
    return post(rc, q, persistent, request, ret);
}

static int mx_coll_iscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                         struct ompi_communicator_t *comm, struct ompi_request_t **request,
                         mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!scan_like(m, sbuf, rbuf, count, dtype, op, 0, 0, request, &ret)) return ret;
    return m->prev_iscan(sbuf, rbuf, count, dtype, op, comm, request, m->prev_iscan_module);
}

static int mx_coll_iexscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                           struct ompi_op_t *op, struct ompi_communicator_t *comm, struct ompi_request_t **request,
                           mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!scan_like(m, sbuf, rbuf, count, dtype, op, 1, 0, request, &ret)) return ret;
    return m->prev_iexscan(sbuf, rbuf, count, dtype, op, comm, request, m->prev_iexscan_module);
}

static int mx_coll_scan_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                             struct ompi_op_t *op, struct ompi_communicator_t *comm, struct ompi_info_t *info,
                             struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!scan_like(m, sbuf, rbuf, count, dtype, op, 0, 1, request, &ret)) return ret;
    return m->prev_scan_init(sbuf, rbuf, count, dtype, op, comm, info, request, m->prev_scan_init_module);
}

static int mx_coll_exscan_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                               struct ompi_op_t *op, struct ompi_communicator_t *comm, struct ompi_info_t *info,
                               struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!scan_like(m, sbuf, rbuf, count, dtype, op, 1, 1, request, &ret)) return ret;
    return m->prev_exscan_init(sbuf, rbuf, count, dtype, op, comm, info, request, m->prev_exscan_init_module);
}

static int allgather_like(mx_coll_module_t *m, const void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                          void *rbuf, int rcount, struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                          int persistent, struct ompi_request_t **request, int *ret)
{
    const size_t rbytes = (size_t)rcount * mx_ompi_host->dtype_size(rdtype);
    const int n = mx_ompi_host->comm_size(comm);
    mx_request_t *q = NULL;
    if (!m->mx || !rbytes || !on_device(rbuf) || !mx_ompi_host->dtype_contiguous(rdtype, rcount * n) ||
        !(sbuf == MPI_IN_PLACE ||
          (on_device(sbuf) && mx_ompi_host->dtype_contiguous(sdtype, scount) &&
           (size_t)scount * mx_ompi_host->dtype_size(sdtype) == rbytes)))
        return 1;
    const void *sb = sbuf == MPI_IN_PLACE ? MX_IN_PLACE : sbuf;
    const int rc = persistent ? mx_allgather_init(m->mx, sb, rbuf, rbytes, NULL, &q)
                              : mx_iallgather(m->mx, sb, rbuf, rbytes, NULL, &q);
    return post(rc, q, persistent, request, ret);
}

static int mx_coll_iallgather(const void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                              struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                              struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!allgather_like(m, sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, 0, request, &ret)) return ret;
    return m->prev_iallgather(sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, request, m->prev_iallgather_module);
}

static int mx_coll_allgather_init(const void *sbuf, int scount, struct ompi_datatype_t *sdtype, void *rbuf,
                                  int rcount, struct ompi_datatype_t *rdtype, struct ompi_communicator_t *comm,
                                  struct ompi_info_t *info, struct ompi_request_t **request,
                                  mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!allgather_like(m, sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, 1, request, &ret)) return ret;
    return m->prev_allgather_init(sbuf, scount, sdtype, rbuf, rcount, rdtype, comm, info, request,
                                  m->prev_allgather_init_module);
}

static int bcast_like(mx_coll_module_t *m, void *buf, int count, struct ompi_datatype_t *dtype, int root,
                      int persistent, struct ompi_request_t **request, int *ret)
{
    const size_t bytes = (size_t)count * mx_ompi_host->dtype_size(dtype);
    mx_request_t *q = NULL;
    if (!m->mx || !bytes || !on_device(buf) || !mx_ompi_host->dtype_contiguous(dtype, count)) return 1;
    const int rc = persistent ? mx_bcast_init(m->mx, buf, bytes, root, NULL, &q)
                              : mx_ibcast(m->mx, buf, bytes, root, NULL, &q);
    return post(rc, q, persistent, request, ret);
}

static int mx_coll_ibcast(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                          struct ompi_communicator_t *comm, struct ompi_request_t **request,
                          mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!bcast_like(m, buf, count, dtype, root, 0, request, &ret)) return ret;
    return m->prev_ibcast(buf, count, dtype, root, comm, request, m->prev_ibcast_module);
}

static int mx_coll_bcast_init(void *buf, int count, struct ompi_datatype_t *dtype, int root,
                              struct ompi_communicator_t *comm, struct ompi_info_t *info,
                              struct ompi_request_t **request, mca_coll_base_module_t *module)
{
    mx_coll_module_t *m = (mx_coll_module_t *)module;
    int ret;
    if (!bcast_like(m, buf, count, dtype, root, 1, request, &ret)) return ret;
    return m->prev_bcast_init(buf, count, dtype, root, comm, info, request, m->prev_bcast_init_module);
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
    const int n = mx_ompi_host->comm_size(comm), rank = mx_ompi_host->comm_rank(comm);
    m->comm = comm;
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
    if (m->super.coll_allreduce && n > 1 && n <= MX_MAX_RANKS) {
        const size_t staging = (size_t)mx_ompi_host->mca_int("coll_mi355x_staging_mb", 1024) << 20;
        int flags = MX_COMM_IPC;
        if (mx_ompi_host->mca_int("coll_mi355x_rccl", 0)) flags |= MX_COMM_RCCL;
        int rc = mx_comm_create(rank, n, -1, staging, flags, bootstrap_allgather, m, &m->mx);
        if (rc != MX_SUCCESS) m->mx = NULL;   /* every call delegates */
    }
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
    m = calloc(1, sizeof *m);
    if (!m) return NULL;
    m->super.super.obj_class = &mx_coll_module_class;
    m->super.super.obj_reference_count = 1;
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
        /* size-1 comms (MPI_COMM_SELF): MPI_Reduce_local lands here when
         * our priority beats coll/self's 75 (coll_self_module.c:60,84) */
        m->super.coll_allreduce = NULL;
    }
    if (*priority > 75) m->super.coll_reduce_local = mx_coll_reduce_local;
    if (n == 1 && !m->super.coll_reduce_local) {
        free(m);
        return NULL;
    }
    return &m->super;
}

mca_coll_base_component_2_0_0_t mca_coll_mi355x_component = {
    .collm_version = {
        .mca_major_version = 2, .mca_minor_version = 1, .mca_release_version = 0,
        .mca_project_name = "ompi",
        .mca_type_name = "coll", .mca_type_major_version = 2,
        .mca_component_name = "mi355x", .mca_component_major_version = 1,
    },
    .collm_init_query = mx_coll_component_init_query,
    .collm_comm_query = mx_coll_component_comm_query,
};
