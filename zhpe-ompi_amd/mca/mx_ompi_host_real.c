/*
 * mx_ompi_host_real.c -- the mx_ompi_host_t table (mx_ompi_abi.h) filled
 * from a real Open MPI tree.  Compiled only inside one, next to the
 * components, with -DMX_OMPI_REAL; in this
 * repository the same table is filled by the mini-host harness
 * (mca/host/mx_host.c), which restates each of these internals.
 *
 * Each entry maps one-to-one onto an Open MPI internal:
 *   comm_rank / comm_size        ompi_comm_rank / ompi_comm_size
 *   dtype_slot                   ompi_op_ddt_map[dt->id] (ompi/op/op.c:131-229),
 *                                derived types through their single predefined
 *                                base (ompi_datatype_args.c:825-865)
 *   dtype_size / _contiguous     ompi_datatype_type_size,
 *                                ompi_datatype_is_contiguous_memory_layout
 *   dtype_pack / _unpack / _span opal_convertor_pack / _unpack on host memory
 *                                (opal_convertor.c:218-325), opal_datatype_span
 *   dtype_desc                   dt->super.opt_desc (or desc): the committed
 *                                records the device convertor is built from
 *   op_index / op_flags / fns    op->o_f_to_c_index, op->o_flags,
 *                                op->o_func.intrinsic, op->o_3buff_intrinsic
 *   comm_coll_fn                 comm->c_coll->coll_<slot> and its module
 *   obj_retain / obj_release     OBJ_RETAIN / OBJ_RELEASE
 *   mca_int / mca_string         mca_base_var_find + mca_base_var_get_value
 *                                (bool, int and string variables)
 *   comm_is_inter                OMPI_COMM_IS_INTER
 *   request_test/_start/_free    REQUEST_COMPLETE + req_status, req_start,
 *                                ompi_request_free (the saved module's
 *                                requests, driven by the component)
 *   requests                     an ompi_request_t subclass carrying the
 *                                component's context, like
 *                                ompi_coll_libnbc_request_t
 *                                (coll_libnbc_component.c:570-583)
 *   progress_register            opal_progress_register
 */
#include "ompi_config.h"

#include <string.h>

#include "mpi.h"
#include "ompi/communicator/communicator.h"
#include "ompi/datatype/ompi_datatype.h"
#include "ompi/op/op.h"
#include "ompi/request/request.h"
#include "opal/datatype/opal_convertor.h"
#include "opal/mca/base/mca_base_var.h"
#include "opal/runtime/opal_progress.h"

#include "mx_ompi_abi.h"

static int h_rank(struct ompi_communicator_t *c) { return ompi_comm_rank(c); }
static int h_size(struct ompi_communicator_t *c) { return ompi_comm_size(c); }

static int h_slot(struct ompi_datatype_t *dt)
{
    if (!ompi_datatype_is_predefined(dt)) {
        const ompi_datatype_t *p = ompi_datatype_get_single_predefined_type_from_args(dt);
        return p ? ompi_op_ddt_map[p->id] : -1;
    }
    return ompi_op_ddt_map[dt->id];
}

static size_t h_dsize(struct ompi_datatype_t *dt)
{
    size_t s = 0;
    ompi_datatype_type_size(dt, &s);
    return s;
}

static int h_contig(struct ompi_datatype_t *dt, int n)
{
    return ompi_datatype_is_contiguous_memory_layout(dt, n) ? 1 : 0;
}

/* one host-memory convertor pass over count elements */
static int h_convert(struct ompi_datatype_t *dt, int count, void *user, void *packed, int pack)
{
    size_t bytes = 0;
    ompi_datatype_type_size(dt, &bytes);
    bytes *= (size_t)count;
    opal_convertor_t *cv = opal_convertor_create(opal_local_arch, 0);
    if (!cv) return OMPI_ERR_OUT_OF_RESOURCE;
    int rc = pack ? opal_convertor_copy_and_prepare_for_send(ompi_mpi_local_convertor, &dt->super, count, user, 0, cv)
                  : opal_convertor_copy_and_prepare_for_recv(ompi_mpi_local_convertor, &dt->super, count, user, 0, cv);
    if (OPAL_SUCCESS == rc) {
        struct iovec iov = {.iov_base = packed, .iov_len = bytes};
        uint32_t n = 1;
        size_t max = bytes;
        rc = pack ? opal_convertor_pack(cv, &iov, &n, &max) : opal_convertor_unpack(cv, &iov, &n, &max);
        rc = (rc >= 0 && max == bytes) ? OMPI_SUCCESS : OMPI_ERROR;
    }
    OBJ_RELEASE(cv);
    return rc;
}
static int h_pack(struct ompi_datatype_t *dt, int count, const void *user, void *packed)
{
    return h_convert(dt, count, (void *)user, packed, 1);
}
static int h_unpack(struct ompi_datatype_t *dt, int count, const void *packed, void *user)
{
    return h_convert(dt, count, user, (void *)packed, 0);
}
static int h_span(struct ompi_datatype_t *dt, int count, ptrdiff_t *lo, ptrdiff_t *hi)
{
    ptrdiff_t gap = 0;
    const ptrdiff_t span = opal_datatype_span(&dt->super, count, &gap);
    *lo = gap;
    *hi = gap + span;
    return OMPI_SUCCESS;
}

/* the committed description (opal_datatype.h:126): the optimized records
 * when the datatype has them, else the plain ones, plus the closing END_LOOP */
static int h_desc(struct ompi_datatype_t *dt, const void **recs, size_t *nrec, size_t *size, ptrdiff_t *lb,
                  ptrdiff_t *ub)
{
    const opal_datatype_t *d = &dt->super;
    const dt_type_desc_t *td = d->opt_desc.used ? &d->opt_desc : &d->desc;
    if (!td->desc || !td->used) return OMPI_ERROR;
    *recs = td->desc;
    *nrec = (size_t)td->used + 1;
    *size = d->size;
    *lb = d->lb;
    *ub = d->ub;
    return OMPI_SUCCESS;
}

static int h_opidx(struct ompi_op_t *op) { return op->o_f_to_c_index; }
static uint32_t h_opflags(struct ompi_op_t *op) { return op->o_flags; }
static ompi_op_base_op_fns_t *h_fns(struct ompi_op_t *op) { return &op->o_func.intrinsic; }
static ompi_op_base_op_3buff_fns_t *h_fns3(struct ompi_op_t *op) { return &op->o_3buff_intrinsic; }

/* comm->c_coll->coll_<slot> / coll_<slot>_module (coll.h:622-) */
static void *h_coll(struct ompi_communicator_t *c, const char *slot, struct mca_coll_base_module_2_3_0_t **m)
{
#define MX_SLOT(name)                                                   \
    if (!strcmp(slot, #name)) {                                         \
        *m = c->c_coll->coll_##name##_module;                           \
        return (void *)c->c_coll->coll_##name;                          \
    }
    MX_SLOT(allreduce) MX_SLOT(reduce_scatter) MX_SLOT(allgather) MX_SLOT(bcast) MX_SLOT(reduce_local)
    MX_SLOT(reduce) MX_SLOT(reduce_scatter_block) MX_SLOT(scan) MX_SLOT(exscan)
    MX_SLOT(iallreduce) MX_SLOT(ireduce) MX_SLOT(ireduce_scatter) MX_SLOT(ireduce_scatter_block) MX_SLOT(iscan)
    MX_SLOT(iexscan) MX_SLOT(iallgather) MX_SLOT(ibcast)
    MX_SLOT(allreduce_init) MX_SLOT(reduce_init) MX_SLOT(reduce_scatter_init) MX_SLOT(reduce_scatter_block_init)
    MX_SLOT(scan_init) MX_SLOT(exscan_init) MX_SLOT(allgather_init) MX_SLOT(bcast_init)
#undef MX_SLOT
    *m = NULL;
    return NULL;
}

static void h_retain(opal_object_t *o) { OBJ_RETAIN(o); }
static void h_release(opal_object_t *o) { OBJ_RELEASE(o); }

/* "coll_mi355x_<var>" / "op_mi355x_<var>" / "coll_libnbc_<var>" /
 * "coll_tuned_<var>" / "coll_basic_<var>": framework, component, variable */
static int h_var(const char *name)
{
    char fw[16] = "", comp[16] = "";
    const char *u1 = strchr(name, '_'), *u2 = u1 ? strchr(u1 + 1, '_') : NULL;
    if (!u1 || !u2 || (size_t)(u1 - name) >= sizeof fw || (size_t)(u2 - u1 - 1) >= sizeof comp) return -1;
    memcpy(fw, name, (size_t)(u1 - name));
    memcpy(comp, u1 + 1, (size_t)(u2 - u1 - 1));
    return mca_base_var_find("ompi", fw, comp, u2 + 1);
}
static int h_mca_int(const char *name, int def)
{
    const int idx = h_var(name);
    const mca_base_var_t *var = NULL;
    const void *p = NULL;
    if (idx < 0 || OPAL_SUCCESS != mca_base_var_get(idx, &var) || !var ||
        OPAL_SUCCESS != mca_base_var_get_value(idx, &p, NULL, NULL) || !p)
        return def;
    switch (var->mbv_type) {   /* coll_tuned_use_dynamic_rules is a bool */
    case MCA_BASE_VAR_TYPE_BOOL: return *(const bool *)p ? 1 : 0;
    case MCA_BASE_VAR_TYPE_INT: case MCA_BASE_VAR_TYPE_UNSIGNED_INT: return *(const int *)p;
    default: return def;
    }
}
static const char *h_mca_string(const char *name)
{
    const int idx = h_var(name);
    const mca_base_var_t *var = NULL;
    const char *const *p = NULL;
    if (idx < 0 || OPAL_SUCCESS != mca_base_var_get(idx, &var) || !var || var->mbv_type != MCA_BASE_VAR_TYPE_STRING ||
        OPAL_SUCCESS != mca_base_var_get_value(idx, &p, NULL, NULL) || !p)
        return NULL;
    return *p;
}

static int h_is_inter(struct ompi_communicator_t *c) { return OMPI_COMM_IS_INTER(c) ? 1 : 0; }

/* the saved module's requests (the component polls them from its progress
 * callback, so no progress and no free here) */
static int h_inner_test(struct ompi_request_t *r, int *flag, int *status)
{
    *flag = REQUEST_COMPLETE(r) ? 1 : 0;
    *status = *flag ? r->req_status.MPI_ERROR : OMPI_SUCCESS;
    return OMPI_SUCCESS;
}
static int h_inner_start(struct ompi_request_t *r) { return r->req_start(1, &r); }
static int h_inner_free(struct ompi_request_t **r) { return ompi_request_free(r); }

/* requests of the nonblocking / persistent slots */
typedef struct {
    ompi_request_t super;
    void *ctx;
    int (*start)(struct ompi_request_t *);
    int (*free_fn)(struct ompi_request_t *);
} mx_real_request_t;
OBJ_CLASS_INSTANCE(mx_real_request_t, ompi_request_t, NULL, NULL);

static int h_req_start(size_t n, ompi_request_t **r)          /* req_start: MPI_Start / MPI_Startall */
{
    for (size_t i = 0; i < n; i++) {
        const int rc = ((mx_real_request_t *)r[i])->start(r[i]);
        if (OMPI_SUCCESS != rc) return rc;
    }
    return OMPI_SUCCESS;
}
static int h_req_free(ompi_request_t **r)                      /* req_free: MPI_Request_free */
{
    const int rc = ((mx_real_request_t *)*r)->free_fn(*r);
    OBJ_RELEASE(*r);
    *r = MPI_REQUEST_NULL;
    return rc;
}
static struct ompi_request_t *h_req_create(int persistent, int (*start)(struct ompi_request_t *),
                                           int (*free_fn)(struct ompi_request_t *), void *ctx)
{
    mx_real_request_t *q = OBJ_NEW(mx_real_request_t);
    if (!q) return NULL;
    OMPI_REQUEST_INIT(&q->super, persistent);
    q->super.req_type = OMPI_REQUEST_COLL;
    q->super.req_start = h_req_start;
    q->super.req_free = h_req_free;
    q->super.req_state = persistent ? OMPI_REQUEST_INACTIVE : OMPI_REQUEST_ACTIVE;
    q->ctx = ctx;
    q->start = start;
    q->free_fn = free_fn;
    return &q->super;
}
static void *h_req_ctx(struct ompi_request_t *r) { return ((mx_real_request_t *)r)->ctx; }
static void h_req_activate(struct ompi_request_t *r)
{
    r->req_state = OMPI_REQUEST_ACTIVE;
    r->req_complete = REQUEST_PENDING;
}
static void h_req_complete(struct ompi_request_t *r, int status)
{
    r->req_status.MPI_ERROR = status;
    ompi_request_complete(r, true);
}

static mx_ompi_host_t real_host;

/* this component DSO's view of the host (op_mi355x.c defines it for the
 * single-library build of this repository) */
const mx_ompi_host_t *mx_ompi_host;

int mx_ompi_set_host(const mx_ompi_host_t *host)
{
    mx_ompi_host = host;
    return OMPI_SUCCESS;
}

/* Called from each component's open function (mca_open_component) before
 * any query: fills the table from the real internals. */
int mx_ompi_host_real_register(void)
{
    real_host.comm_rank = h_rank;
    real_host.comm_size = h_size;
    real_host.dtype_slot = h_slot;
    real_host.dtype_size = h_dsize;
    real_host.dtype_contiguous = h_contig;
    real_host.op_index = h_opidx;
    real_host.op_flags = h_opflags;
    real_host.op_fns = h_fns;
    real_host.op_3buff_fns = h_fns3;
    real_host.comm_coll_fn = h_coll;
    real_host.obj_retain = h_retain;
    real_host.obj_release = h_release;
    real_host.mca_int = h_mca_int;
    real_host.byte_dtype = &ompi_mpi_byte.dt;
    real_host.request_create = h_req_create;
    real_host.request_ctx = h_req_ctx;
    real_host.request_activate = h_req_activate;
    real_host.request_complete = h_req_complete;
    real_host.progress_register = opal_progress_register;
    real_host.dtype_pack = h_pack;
    real_host.dtype_unpack = h_unpack;
    real_host.dtype_span = h_span;
    real_host.dtype_desc = h_desc;
    real_host.comm_is_inter = h_is_inter;
    real_host.mca_string = h_mca_string;
    real_host.request_test = h_inner_test;
    real_host.request_start = h_inner_start;
    real_host.request_free = h_inner_free;
    return mx_ompi_set_host(&real_host);
}
