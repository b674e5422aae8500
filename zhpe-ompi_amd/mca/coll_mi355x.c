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
} mx_coll_module_t;

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
