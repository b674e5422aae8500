/*
 * op_mi355x.c -- the `mi355x` component of Open MPI's `op` framework.
 *
 * Plugs the HIP kernels of libmx_kernels.so into the per-(op, type) function
 * tables that ompi_op_base_op_select() builds for every intrinsic MPI_Op
 * (ompi/mca/op/base/op_base_op_select.c:88-204), so MPI_Reduce_local, every
 * coll/base algorithm's ompi_op_reduce() and the OpenSHMEM reductions run the
 * GPU kernel whenever both buffers are device memory.
 *
 * Follows the reference's accelerator template ompi/mca/op/example:
 *  - component struct + init_query + op_query (op_example_component.c:50-77,
 *    185-245, 251-311); priority 50 by default, MCA var op_mi355x_priority,
 *    clamped to 100 by the framework (op_base_op_select.c:279);
 *  - at query time the slots already on the op are cached as the fallback and
 *    RETAINed (op_example_module_max.c:203-258);
 *  - the hardware-or-fallback decision is taken per call from the buffer
 *    location (op_example_module_max.c:130-149).
 * Differences by design: one generic handler serves every slot (the module
 * remembers its op; the slot comes from the datatype), and every
 * (op, type) pair of the reference table is covered -- including long
 * double and its complex/pair types through the device x87 emulation.
 *
 * Synchronous ABI: the handler returns void and the caller immediately uses
 * `inout` (coll_base_allreduce.c:471-477), so each call completes its kernel
 * before returning (sync of the calling thread's stream).  Errors cannot be returned
 * (ompi/mca/op/op.h:258-273): a device failure aborts, like the CUDA path
 * does on copy failure (opal_datatype_cuda.c:121-140).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mx_kernels.h"
#include "mx_ompi_abi.h"

#ifndef MX_OMPI_WITH_FORTRAN
#define MX_OMPI_WITH_FORTRAN 1   /* table variant of the host Open MPI build */
#endif

#ifndef MX_OMPI_REAL
/* one library holds both components here; in an Open MPI tree each
 * component DSO gets its own copy from mx_ompi_host_real.c */
const mx_ompi_host_t *mx_ompi_host;

int mx_ompi_set_host(const mx_ompi_host_t *host)
{
    mx_ompi_host = host;
    return OMPI_SUCCESS;
}
#else
int mx_ompi_host_real_register(void);
static int mx_op_component_open(void) { return mx_ompi_host_real_register(); }
#endif

typedef struct {
    ompi_op_base_module_t super;
    int op_index;                                   /* OMPI_OP_BASE_FORTRAN_* */
    ompi_op_base_handler_fn_t fallback[OMPI_OP_BASE_TYPE_MAX];
    ompi_op_base_module_t *fallback_module[OMPI_OP_BASE_TYPE_MAX];
    ompi_op_base_3buff_handler_fn_t fallback3[OMPI_OP_BASE_TYPE_MAX];
    ompi_op_base_module_t *fallback3_module[OMPI_OP_BASE_TYPE_MAX];
} mx_op_module_t;

/* releases the cached fallbacks; the object itself is freed by OBJ_RELEASE */
static void op_module_destruct(mx_op_module_t *m)
{
    for (int i = 0; i < OMPI_OP_BASE_TYPE_MAX; i++) {
        if (m->fallback_module[i]) MX_OBJ_RELEASE(m->fallback_module[i]);
        if (m->fallback3_module[i]) MX_OBJ_RELEASE(m->fallback3_module[i]);
    }
}

MX_MODULE_CLASS(mx_op_module_t, ompi_op_base_module_t, op_module_destruct);

static int both_on_device(const void *a, const void *b)
{
    return mx_is_device_ptr(a) == 1 && mx_is_device_ptr(b) == 1;   /* range-cached: no runtime call */
}

/* The kernels run on a stream of the calling thread: one per thread, so
 * concurrent callers under MPI_THREAD_MULTIPLE neither share a stream nor
 * synchronise each other's work; a blocking stream, so it is implicitly
 * ordered after what the legacy default stream holds (the kernels that
 * produced the operands) at no per-call cost.  Measured per handler call
 * (profiles/r02/op_call_cost.txt, stream_probe.txt): a non-blocking stream
 * plus an explicit event order costs ~11 us more than this.
 * op_mi355x_stream = 0 selects the legacy default stream instead. */
static _Thread_local void *t_stream;
static _Thread_local int t_stream_tried;
static int g_use_stream = -1;   /* op_mi355x_stream, read once */

static void *op_stream(void)
{
    if (g_use_stream < 0) g_use_stream = mx_ompi_host->mca_int("op_mi355x_stream", 1) != 0;
    if (!g_use_stream) return NULL;
    if (!t_stream_tried) {
        t_stream_tried = 1;
        if (mx_stream_create_ordered(&t_stream) != MX_SUCCESS) t_stream = NULL;
    }
    return t_stream;
}

/* op_mi355x_fast_sync (default 1): wait through the marker kernel's mapped
 * completion word instead of hipStreamSynchronize (profiles/r02/op_call_cost.txt) */
static int g_fast_sync = -1;

static int run_sync(void *s, int rc)
{
    if (g_fast_sync < 0) g_fast_sync = mx_ompi_host->mca_int("op_mi355x_fast_sync", 1) != 0;
    if (rc == MX_SUCCESS) rc = g_fast_sync ? mx_stream_sync_fast(s) : mx_stream_sync(s);
    return rc;
}

static void die(const char *what, int rc)
{
    fprintf(stderr, "op/mi355x: %s failed: %s (%d)\n", what, mx_strerror(rc), rc);
    abort();
}

/* 2-buffer handler: inout = inout OP in (op.h:258-262) */
static void mx_op_2buff(void *in, void *inout, int *count, struct ompi_datatype_t **dtype,
                        ompi_op_base_module_t *module)
{
    mx_op_module_t *m = (mx_op_module_t *)module;
    const int slot = mx_ompi_host->dtype_slot(*dtype);
    if (slot < 0) die("datatype lookup", MX_ERR_ARG);
    if (*count > 0 && both_on_device(in, inout)) {
        void *s = op_stream();
        int rc;
        if (g_fast_sync < 0) g_fast_sync = mx_ompi_host->mca_int("op_mi355x_fast_sync", 1) != 0;
        if (g_fast_sync)   /* the resident service, or the launch marking itself (per-workgroup flags) */
            rc = mx_reduce2_sync(m->op_index, slot, in, inout, (size_t)*count, s);
        else
            rc = run_sync(s, mx_reduce2(m->op_index, slot, in, inout, (size_t)*count, s));
        if (rc != MX_SUCCESS) die("mx_reduce2", rc);
        return;
    }
    m->fallback[slot](in, inout, count, dtype, m->fallback_module[slot]);
}

/* 3-buffer handler: out = in1 OP in2 (op.h:267-273) */
static void mx_op_3buff(void *in1, void *in2, void *out, int *count, struct ompi_datatype_t **dtype,
                        ompi_op_base_module_t *module)
{
    mx_op_module_t *m = (mx_op_module_t *)module;
    const int slot = mx_ompi_host->dtype_slot(*dtype);
    if (slot < 0) die("datatype lookup", MX_ERR_ARG);
    if (*count > 0 && both_on_device(in1, in2) && mx_is_device_ptr(out) == 1) {
        void *s = op_stream();
        int rc;
        if (g_fast_sync < 0) g_fast_sync = mx_ompi_host->mca_int("op_mi355x_fast_sync", 1) != 0;
        if (g_fast_sync)   /* the resident service, or the launch + completion word */
            rc = mx_reduce3_sync(m->op_index, slot, in1, in2, out, (size_t)*count, s);
        else
            rc = run_sync(s, mx_reduce3(m->op_index, slot, in1, in2, out, (size_t)*count, s));
        if (rc != MX_SUCCESS) die("mx_reduce3", rc);
        return;
    }
    m->fallback3[slot](in1, in2, out, count, dtype, m->fallback3_module[slot]);
}

static int mx_op_component_init_query(bool enable_progress_threads, bool enable_mpi_threads)
{
    (void)enable_progress_threads;
    (void)enable_mpi_threads;  /* one stream per calling thread: safe under THREAD_MULTIPLE */
    if (!mx_ompi_host) return OMPI_ERR_NOT_SUPPORTED;
    return mx_init(-1) == MX_SUCCESS ? OMPI_SUCCESS : OMPI_ERR_NOT_SUPPORTED;
}

static ompi_op_base_module_t *mx_op_component_op_query(struct ompi_op_t *op, int *priority)
{
    const int idx = mx_ompi_host->op_index(op);
    ompi_op_base_op_fns_t *cur = mx_ompi_host->op_fns(op);
    ompi_op_base_op_3buff_fns_t *cur3 = mx_ompi_host->op_3buff_fns(op);
    mx_op_module_t *m;
    int any = 0;

    if (!(mx_ompi_host->op_flags(op) & OMPI_OP_FLAGS_INTRINSIC)) return NULL;
    if (idx <= 0 || idx >= MX_OP_REPLACE) return NULL;      /* MPI_OP_NULL, REPLACE, NO_OP */
    m = MX_MODULE_NEW(mx_op_module_t, super);
    if (!m) return NULL;
    m->super.opm_op = op;
    m->op_index = idx;
    for (int t = 0; t < OMPI_OP_BASE_TYPE_MAX; t++) {
        /* only slots that have a kernel AND are non-NULL on the op: the
         * framework requires the NULL pattern to stay identical
         * (op_base_op_select.c:185-201) */
        if (!mx_op_supported(idx, t, MX_OMPI_WITH_FORTRAN)) continue;
        if (cur->fns[t]) {
            m->super.opm_fns[t] = mx_op_2buff;
            m->fallback[t] = cur->fns[t];
            m->fallback_module[t] = cur->modules[t];
            if (cur->modules[t]) MX_OBJ_RETAIN(cur->modules[t]);
            any = 1;
        }
        if (cur3->fns[t]) {
            m->super.opm_3buff_fns[t] = mx_op_3buff;
            m->fallback3[t] = cur3->fns[t];
            m->fallback3_module[t] = cur3->modules[t];
            if (cur3->modules[t]) MX_OBJ_RETAIN(cur3->modules[t]);
            any = 1;
        }
    }
    if (!any) {
        MX_OBJ_RELEASE(m);
        return NULL;
    }
    *priority = mx_ompi_host->mca_int("op_mi355x_priority", 50);
    return &m->super;
}

/* MPI_Finalize closes the framework: the resident reduce service (if it
 * ran) is stopped here, so its grid has drained before the process ends */
static int mx_op_component_close(void)
{
    (void)mx_op_service_set(0);
    return OMPI_SUCCESS;
}

ompi_op_base_component_1_0_0_t mca_op_mi355x_component = {
    .opc_version = {
        .mca_major_version = 2, .mca_minor_version = 1, .mca_release_version = 0,
        .mca_project_name = "ompi",
        .mca_type_name = "op", .mca_type_major_version = 1,
        .mca_component_name = "mi355x", .mca_component_major_version = 1,
#ifdef MX_OMPI_REAL
        .mca_open_component = mx_op_component_open,
#endif
        .mca_close_component = mx_op_component_close,
    },
    .opc_init_query = mx_op_component_init_query,
    .opc_op_query = mx_op_component_op_query,
};
