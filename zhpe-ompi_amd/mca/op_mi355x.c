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

/* ---- operands in different memories ---------------------------------------
 * MPI_Reduce_local(device_in, host_inout), or any coll/base algorithm mixing a
 * device user buffer with its host temporaries, is legal MPI.  The reference's
 * accelerator path checks and stages each buffer on its own
 * (coll_cuda_allreduce.c:44-62, through opal_cuda_check_bufs,
 * opal_datatype_cuda.c:70).  Here the result is produced in the memory it
 * lives in:
 *  - result in device memory: each host operand is copied to device scratch
 *    (one copy per operand) and the kernel runs;
 *  - result in host memory, at most op_mi355x_mixed_host_max_kb (default
 *    64 KiB): each device operand is copied to host scratch and the host
 *    function the module replaced runs (no device round trip of the result);
 *  - result in host memory, larger: host operands go to device scratch, the
 *    kernel writes device scratch, the result is copied back.
 * Both routes are bit-exact with the base function (the kernels are).
 * Scratch belongs to the calling thread: device buffers for up to three
 * operands, pinned host buffers for two. */
typedef struct { void *p; size_t bytes; } mx_tscratch_t;
static _Thread_local mx_tscratch_t t_dev[3], t_host[2];
static size_t g_mixed_host_max = (size_t)-1;

static void *tscratch(mx_tscratch_t *s, size_t bytes, int host)
{
    if (s->bytes < bytes) {
        if (host) mx_host_free(s->p); else mx_free(s->p);
        s->p = NULL;
        s->bytes = 0;
        const size_t want = bytes < ((size_t)1 << 20) ? ((size_t)1 << 20) : bytes;
        if ((host ? mx_host_alloc(want, &s->p) : mx_alloc(want, &s->p)) != MX_SUCCESS) return NULL;
        s->bytes = want;
    }
    return s->p;
}

static size_t mixed_host_max(void)
{
    if (g_mixed_host_max == (size_t)-1) {
        const int kb = mx_ompi_host->mca_int("op_mi355x_mixed_host_max_kb", 64);
        g_mixed_host_max = kb > 0 ? (size_t)kb << 10 : 0;
    }
    return g_mixed_host_max;
}

/* `p` in the memory the call computes in: itself, or a copy in scratch k
 * (filled when `read`); NULL when the copy cannot be made */
static void *stage(void *p, int on_dev, int want_dev, size_t bytes, int k, int read, void *s)
{
    if (on_dev == want_dev) return p;
    void *q = tscratch(want_dev ? &t_dev[k] : &t_host[k], bytes, !want_dev);
    if (!q) die("scratch allocation", MX_ERR_NOMEM);
    if (read) {
        int rc = mx_memcpy(q, p, bytes, s);
        if (rc == MX_SUCCESS && !want_dev) rc = mx_stream_sync(s);   /* the host function reads it next */
        if (rc != MX_SUCCESS) die("operand staging", rc);
    }
    return q;
}

/* the kernel on device operands (every pointer device memory) */
static void run2(mx_op_module_t *m, int slot, void *in, void *inout, size_t count, void *s)
{
    int rc;
    if (g_fast_sync < 0) g_fast_sync = mx_ompi_host->mca_int("op_mi355x_fast_sync", 1) != 0;
    if (g_fast_sync)   /* the resident service, or the launch marking itself (per-workgroup flags) */
        rc = mx_reduce2_sync(m->op_index, slot, in, inout, count, s);
    else
        rc = run_sync(s, mx_reduce2(m->op_index, slot, in, inout, count, s));
    if (rc != MX_SUCCESS) die("mx_reduce2", rc);
}

static void run3(mx_op_module_t *m, int slot, void *in1, void *in2, void *out, size_t count, void *s)
{
    int rc;
    if (g_fast_sync < 0) g_fast_sync = mx_ompi_host->mca_int("op_mi355x_fast_sync", 1) != 0;
    if (g_fast_sync)   /* the resident service, or the launch + completion word */
        rc = mx_reduce3_sync(m->op_index, slot, in1, in2, out, count, s);
    else
        rc = run_sync(s, mx_reduce3(m->op_index, slot, in1, in2, out, count, s));
    if (rc != MX_SUCCESS) die("mx_reduce3", rc);
}

/* 2-buffer handler: inout = inout OP in (op.h:258-262) */
static void mx_op_2buff(void *in, void *inout, int *count, struct ompi_datatype_t **dtype,
                        ompi_op_base_module_t *module)
{
    mx_op_module_t *m = (mx_op_module_t *)module;
    const int slot = mx_ompi_host->dtype_slot(*dtype);
    if (slot < 0) die("datatype lookup", MX_ERR_ARG);
    const int din = *count > 0 && mx_is_device_ptr(in) == 1, dio = *count > 0 && mx_is_device_ptr(inout) == 1;
    if (*count <= 0 || (!din && !dio)) {
        m->fallback[slot](in, inout, count, dtype, m->fallback_module[slot]);
        return;
    }
    void *s = op_stream();
    if (din && dio) {
        run2(m, slot, in, inout, (size_t)*count, s);
        return;
    }
    const size_t bytes = (size_t)*count * mx_type_size(slot);
    if (dio || bytes > mixed_host_max()) {   /* compute on the device */
        void *din_p = stage(in, din, 1, bytes, 0, 1, s);
        void *dio_p = stage(inout, dio, 1, bytes, 1, 1, s);
        run2(m, slot, din_p, dio_p, (size_t)*count, s);
        if (dio_p != inout) {
            int rc = mx_memcpy(inout, dio_p, bytes, s);
            if (rc == MX_SUCCESS) rc = mx_stream_sync(s);
            if (rc != MX_SUCCESS) die("result copy", rc);
        }
        return;
    }
    /* small, result in host memory: the device operand comes to the host */
    void *hin = stage(in, 1, 0, bytes, 0, 1, s);
    m->fallback[slot](hin, inout, count, dtype, m->fallback_module[slot]);
}

/* 3-buffer handler: out = in1 OP in2 (op.h:267-273) */
static void mx_op_3buff(void *in1, void *in2, void *out, int *count, struct ompi_datatype_t **dtype,
                        ompi_op_base_module_t *module)
{
    mx_op_module_t *m = (mx_op_module_t *)module;
    const int slot = mx_ompi_host->dtype_slot(*dtype);
    if (slot < 0) die("datatype lookup", MX_ERR_ARG);
    const int pos = *count > 0;
    const int d1 = pos && mx_is_device_ptr(in1) == 1, d2 = pos && mx_is_device_ptr(in2) == 1;
    const int dout = pos && mx_is_device_ptr(out) == 1;
    if (!pos || (!d1 && !d2 && !dout)) {
        m->fallback3[slot](in1, in2, out, count, dtype, m->fallback3_module[slot]);
        return;
    }
    void *s = op_stream();
    if (d1 && d2 && dout) {
        run3(m, slot, in1, in2, out, (size_t)*count, s);
        return;
    }
    const size_t bytes = (size_t)*count * mx_type_size(slot);
    if (dout || bytes > mixed_host_max()) {   /* compute on the device */
        void *a = stage(in1, d1, 1, bytes, 0, 1, s);
        void *b = stage(in2, d2, 1, bytes, 1, 1, s);
        void *o = stage(out, dout, 1, bytes, 2, 0, s);
        run3(m, slot, a, b, o, (size_t)*count, s);
        if (o != out) {
            int rc = mx_memcpy(out, o, bytes, s);
            if (rc == MX_SUCCESS) rc = mx_stream_sync(s);
            if (rc != MX_SUCCESS) die("result copy", rc);
        }
        return;
    }
    void *a = stage(in1, d1, 0, bytes, 0, 1, s);
    void *b = stage(in2, d2, 0, bytes, 1, 1, s);
    m->fallback3[slot](a, b, out, count, dtype, m->fallback3_module[slot]);
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
