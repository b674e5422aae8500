/*
 * mx_host.c -- TEST HARNESS ("mini-host") for the mi355x op/coll
 * components.  See mx_host.h for what it restates from Open MPI.  It is
 * not part of the product: the real host is Open MPI itself
 * (INTEGRATION.md).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>
#include <sys/uio.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../mx_ompi_abi.h"
#include "../mx_opal_convertor_abi.h"
#include "../mx_btl_abi.h"
#include "mx_host.h"

/* ---- objects -------------------------------------------------------------- */
static void obj_retain(opal_object_t *o)
{
    if (o) __atomic_add_fetch(&o->obj_reference_count, 1, __ATOMIC_RELAXED);
}
/* OBJ_RELEASE: at zero the class destructor runs and the object is freed
 * (objects of classes without a destructor are the harness's static ones) */
static void obj_release(opal_object_t *o)
{
    if (o && __atomic_sub_fetch(&o->obj_reference_count, 1, __ATOMIC_ACQ_REL) == 0 && o->obj_class &&
        o->obj_class->cls_destruct) {
        o->obj_class->cls_destruct(o);
        free(o);
    }
}

/* ---- datatypes (ompi/datatype/ompi_datatype_internal.h:37-200) ----------- */
struct ompi_datatype_t {
    const char *name;
    int id;          /* OMPI_DATATYPE_MPI_* */
    int slot;        /* ompi_op_ddt_map[id] (op.c:131-229) */
    size_t size;
    int predefined;
    struct ompi_datatype_t *base;   /* derived: base type */
    int base_count;
    /* MPI_Type_vector of the base type (vcount blocks of vblen, stride
     * vstride elements); vcount == 0: contiguous */
    int vcount, vblen, vstride;
    void *desc;      /* committed description records, built on first use */
};

#define DT(nm, id, slot, sz) {nm, id, slot, sz, 1, NULL, 0, 0, 0, 0, NULL}
static struct ompi_datatype_t g_dtypes[] = {
    DT("MPI_INT8_T", 0x01, 0, 1), DT("MPI_UINT8_T", 0x02, 1, 1), DT("MPI_INT16_T", 0x03, 2, 2),
    DT("MPI_UINT16_T", 0x04, 3, 2), DT("MPI_INT32_T", 0x05, 4, 4), DT("MPI_UINT32_T", 0x06, 5, 4),
    DT("MPI_INT64_T", 0x07, 6, 8), DT("MPI_UINT64_T", 0x08, 7, 8),
    /* C aliases (LP64) */
    DT("MPI_CHAR", 0x01, 0, 1), DT("MPI_SIGNED_CHAR", 0x01, 0, 1), DT("MPI_UNSIGNED_CHAR", 0x02, 1, 1),
    DT("MPI_BYTE", 0x02, 1, 1), DT("MPI_SHORT", 0x03, 2, 2), DT("MPI_UNSIGNED_SHORT", 0x04, 3, 2),
    DT("MPI_INT", 0x05, 4, 4), DT("MPI_UNSIGNED", 0x06, 5, 4), DT("MPI_LONG", 0x07, 6, 8),
    DT("MPI_UNSIGNED_LONG", 0x08, 7, 8), DT("MPI_LONG_LONG", 0x07, 6, 8),
    DT("MPI_UNSIGNED_LONG_LONG", 0x08, 7, 8),
    DT("MPI_FLOAT", 0x09, 15, 4), DT("MPI_DOUBLE", 0x0A, 16, 8), DT("MPI_LONG_DOUBLE", 0x0B, 23, 16),
    DT("MPI_WCHAR", 0x10, 40, 4), DT("MPI_CXX_BOOL", 0x12, 25, 1), DT("MPI_LOGICAL", 0x13, 24, 4),
    DT("MPI_CHARACTER", 0x14, 1, 1), DT("MPI_INTEGER", 0x15, 8, 4), DT("MPI_REAL", 0x16, 17, 4),
    DT("MPI_DOUBLE_PRECISION", 0x17, 22, 8), DT("MPI_LONG_DOUBLE_COMPLEX", 0x1A, 29, 32),
    DT("MPI_2INT", 0x1B, 37, 8), DT("MPI_2INTEGER", 0x1C, 33, 8), DT("MPI_2REAL", 0x1D, 31, 8),
    DT("MPI_2DOUBLE_PRECISION", 0x1E, 32, 16), DT("MPI_FLOAT_INT", 0x21, 34, 8),
    DT("MPI_DOUBLE_INT", 0x22, 35, 16), DT("MPI_LONG_DOUBLE_INT", 0x23, 39, 32),
    DT("MPI_LONG_INT", 0x24, 36, 16), DT("MPI_SHORT_INT", 0x25, 38, 8), DT("MPI_AINT", 0x26, 6, 8),
    DT("MPI_OFFSET", 0x27, 7, 8), DT("MPI_C_BOOL", 0x28, 25, 1), DT("MPI_C_COMPLEX", 0x29, 27, 8),
    DT("MPI_C_FLOAT_COMPLEX", 0x2A, 27, 8), DT("MPI_C_DOUBLE_COMPLEX", 0x2B, 28, 16),
    DT("MPI_C_LONG_DOUBLE_COMPLEX", 0x2C, 29, 32), DT("MPI_COUNT", 0x2F, 6, 8),
};
#define NDT (sizeof g_dtypes / sizeof g_dtypes[0])

void *mxh_dtype(const char *name)
{
    for (size_t i = 0; i < NDT; i++)
        if (!strcmp(g_dtypes[i].name, name)) return &g_dtypes[i];
    return NULL;
}

void *mxh_dtype_contiguous(int count, void *oldtype)
{
    struct ompi_datatype_t *o = oldtype, *d = calloc(1, sizeof *d);
    if (!d || !o || count < 0 || o->vcount) { free(d); return NULL; }   /* contiguous of predefined / contiguous */
    d->name = "";
    d->id = -1;
    d->predefined = 0;
    d->base = o->predefined ? o : o->base;
    d->base_count = count * (o->predefined ? 1 : o->base_count);
    d->size = o->size * (size_t)count;
    /* ompi_datatype_get_single_predefined_type_from_args (ompi_datatype_args.c:825-865) */
    d->slot = d->base ? d->base->slot : -1;
    return d;
}

/* MPI_Type_vector(count, blocklen, stride, oldtype) over a predefined type:
 * the non-contiguous layouts of the allgather / bcast tests */
void *mxh_dtype_vector(int count, int blocklen, int stride, void *oldtype)
{
    struct ompi_datatype_t *o = oldtype, *d;
    if (!o || !o->predefined || count < 1 || blocklen < 1 || stride < blocklen) return NULL;
    d = calloc(1, sizeof *d);
    if (!d) return NULL;
    d->name = "";
    d->id = -1;
    d->base = o;
    d->base_count = count * blocklen;
    d->size = o->size * (size_t)count * (size_t)blocklen;
    d->slot = -1;                 /* no reductions on derived types (ompi_op_is_valid) */
    d->vcount = count;
    d->vblen = blocklen;
    d->vstride = stride;
    return d;
}

static size_t dtype_extent(const struct ompi_datatype_t *d)
{
    if (!d->vcount) return d->size;
    return ((size_t)(d->vcount - 1) * (size_t)d->vstride + (size_t)d->vblen) * d->base->size;
}

/* ---- ops ------------------------------------------------------------------ */
struct ompi_op_t {
    opal_object_t super;
    char o_name[64];
    uint32_t o_flags;
    int o_f_to_c_index;
    ompi_op_base_op_fns_t intrinsic;
    ompi_op_base_op_3buff_fns_t o_3buff_intrinsic;
};

static const char *g_opnames[] = {"MPI_OP_NULL", "MPI_MAX", "MPI_MIN", "MPI_SUM", "MPI_PROD", "MPI_LAND",
                                  "MPI_BAND", "MPI_LOR", "MPI_BOR", "MPI_LXOR", "MPI_BXOR", "MPI_MAXLOC",
                                  "MPI_MINLOC", "MPI_REPLACE", "MPI_NO_OP"};
static struct ompi_op_t g_ops[OMPI_OP_BASE_FORTRAN_OP_MAX];

/* base module per op: carries the op index for the base trampolines */
typedef struct { ompi_op_base_module_t super; int op; } base_op_module_t;
static base_op_module_t g_base_mod[OMPI_OP_BASE_FORTRAN_OP_MAX];
static mx_obj_class_t g_static_class = {"static", NULL};

static mxh_reducer_t g_base;
static mxh_pattern_t g_pattern;

static void base_2buff(void *in, void *inout, int *count, struct ompi_datatype_t **dt, ompi_op_base_module_t *m)
{
    g_base(((base_op_module_t *)m)->op, (*dt)->slot, in, inout, (size_t)*count, 1);
}
static void base_3buff(void *in1, void *in2, void *out, int *count, struct ompi_datatype_t **dt,
                       ompi_op_base_module_t *m)
{
    /* the test reducers only expose 2-buffer form: out = in1; out op= in2 is
     * NOT the 3-buffer semantics for MAX/MIN roles, so route through a
     * dedicated 3-buffer reducer when the injected one provides it */
    memcpy(out, in1, (size_t)*count * (*dt)->size);
    g_base(((base_op_module_t *)m)->op, (*dt)->slot, in2, out, (size_t)*count, 1);
}

void *mxh_op(const char *name)
{
    for (int i = 0; i < OMPI_OP_BASE_FORTRAN_OP_MAX; i++)
        if (!strcmp(g_opnames[i], name)) return &g_ops[i];
    return NULL;
}

int mxh_op_slot_owner(void *opv, int t, int three)
{
    struct ompi_op_t *op = opv;
    ompi_op_base_module_t *m = three ? op->o_3buff_intrinsic.modules[t] : op->intrinsic.modules[t];
    if (!m) return -1;
    return (m == &g_base_mod[op->o_f_to_c_index].super) ? 0 : 1;
}

/* ---- MCA variables --------------------------------------------------------- */
#define NVARS 64
static struct { char name[96]; int value; int set; } g_vars[NVARS];
int mxh_set_mca(const char *name, int value)
{
    for (int i = 0; i < NVARS; i++) {
        if (!g_vars[i].set || !strcmp(g_vars[i].name, name)) {
            snprintf(g_vars[i].name, sizeof g_vars[i].name, "%s", name);
            g_vars[i].value = value;
            g_vars[i].set = 1;
            return 0;
        }
    }
    return -1;
}
static int mca_int(const char *name, int def)
{
    char env[160];
    const char *e;
    for (int i = 0; i < NVARS; i++)
        if (g_vars[i].set && !strcmp(g_vars[i].name, name)) return g_vars[i].value;
    snprintf(env, sizeof env, "OMPI_MCA_%s", name);   /* opal_set_mca_prefix.m4:26 */
    e = getenv(env);
    return e ? atoi(e) : def;
}

/* ---- communicators --------------------------------------------------------- */
#define NSLOTS 25
static const char *g_slot_names[NSLOTS] = {
    "allreduce", "reduce_scatter", "allgather", "bcast", "reduce_local", "reduce", "reduce_scatter_block", "scan",
    "exscan",
    /* nonblocking (coll.h:534-550) and persistent (:553-569) */
    "iallreduce", "ireduce", "ireduce_scatter", "ireduce_scatter_block", "iscan", "iexscan", "iallgather", "ibcast",
    "allreduce_init", "reduce_init", "reduce_scatter_init", "reduce_scatter_block_init", "scan_init", "exscan_init",
    "allgather_init", "bcast_init"};
enum { S_IALLREDUCE = 9, S_IREDUCE, S_IREDUCE_SCATTER, S_IREDUCE_SCATTER_BLOCK, S_ISCAN, S_IEXSCAN, S_IALLGATHER,
       S_IBCAST, S_PERSISTENT0 };

struct ompi_communicator_t {
    int rank, size;
    int inter;       /* an intercommunicator (OMPI_COMM_IS_INTER) */
    mxh_allgather_t ag;
    void *ag_ctx;
    /* c_coll: (fn, module, owner-name) per slot (coll.h:622-) */
    void *fn[NSLOTS];
    mca_coll_base_module_t *mod[NSLOTS];
    const char *owner[NSLOTS];
    mca_coll_base_module_t *modules[4];
    int nmodules;
};

static int slot_index(const char *s)
{
    for (int i = 0; i < NSLOTS; i++)
        if (!strcmp(g_slot_names[i], s)) return i;
    return -1;
}

static void *comm_coll_fn(struct ompi_communicator_t *c, const char *slot, mca_coll_base_module_t **module)
{
    int i = slot_index(slot);
    if (i < 0) return NULL;
    *module = c->mod[i];
    return c->fn[i];
}

static int dtype_slot(struct ompi_datatype_t *d) { return d ? d->slot : -1; }
static size_t dtype_size(struct ompi_datatype_t *d) { return d->size; }
static int dtype_contiguous(struct ompi_datatype_t *d, int count)
{
    (void)count;
    return !d->vcount || d->vblen == d->vstride || (d->vcount == 1);
}
/* opal_convertor_pack / _unpack over host memory (opal_convertor.c:218-325) */
static void vec_copy(struct ompi_datatype_t *d, int count, char *user, char *packed, int pack)
{
    const size_t bs = d->base->size, blk = (size_t)d->vblen * bs, ext = dtype_extent(d);
    for (int i = 0; i < count; i++)
        for (int b = 0; b < d->vcount; b++) {
            char *u = user + (size_t)i * ext + (size_t)b * (size_t)d->vstride * bs;
            if (pack) memcpy(packed, u, blk);
            else memcpy(u, packed, blk);
            packed += blk;
        }
}
static int dtype_pack(struct ompi_datatype_t *d, int count, const void *user, void *packed)
{
    if (!d->vcount) memcpy(packed, user, (size_t)count * d->size);
    else vec_copy(d, count, (char *)user, packed, 1);
    return OMPI_SUCCESS;
}
static int dtype_unpack(struct ompi_datatype_t *d, int count, const void *packed, void *user)
{
    if (!d->vcount) memcpy(user, packed, (size_t)count * d->size);
    else vec_copy(d, count, user, (char *)packed, 0);
    return OMPI_SUCCESS;
}
/* opal_datatype_span (opal_datatype.h:329-340), true lb = 0 here */
static int dtype_span(struct ompi_datatype_t *d, int count, ptrdiff_t *lo, ptrdiff_t *hi)
{
    *lo = 0;
    *hi = count > 0 ? (ptrdiff_t)((size_t)count * dtype_extent(d)) : 0;
    return OMPI_SUCCESS;
}
/* committed description of a mini-host datatype, in the reference's record
 * format (opal_datatype_internal.h:146-196): one ELEM of the raw bytes
 * (OPAL_UINT1 -- pack / unpack on a homogeneous node only move bytes) and
 * the closing END_LOOP.  Records live with the datatype. */
#define MXH_OPAL_UINT1 9
#define MXH_OPAL_END_LOOP 1
#define MXH_DT_DATA 0x0100
struct mxh_rec { uint16_t flags, type; uint32_t count; uint64_t blocklen; int64_t extent; int64_t disp; };
static int dtype_desc(struct ompi_datatype_t *d, const void **recs, size_t *nrec, size_t *size, ptrdiff_t *lb,
                      ptrdiff_t *ub)
{
    if (!d->desc) {
        struct mxh_rec *r = calloc(2, sizeof *r);
        if (!r) return OMPI_ERROR;
        const size_t bs = d->vcount ? d->base->size : d->size;
        r[0].flags = MXH_DT_DATA;
        r[0].type = MXH_OPAL_UINT1;
        r[0].count = d->vcount ? (uint32_t)d->vcount : 1;
        r[0].blocklen = d->vcount ? (uint64_t)d->vblen * bs : d->size;
        r[0].extent = d->vcount ? (int64_t)d->vstride * (int64_t)bs : (int64_t)d->size;
        r[1].type = MXH_OPAL_END_LOOP;
        r[1].count = 1;
        r[1].extent = (int64_t)d->size;
        d->desc = r;
    }
    *recs = d->desc;
    *nrec = 2;
    *size = d->size;
    *lb = 0;
    *ub = (ptrdiff_t)dtype_extent(d);
    return OMPI_SUCCESS;
}
static int comm_rank(struct ompi_communicator_t *c) { return c->rank; }
static int comm_is_inter(struct ompi_communicator_t *c) { return c->inter; }
static int comm_size(struct ompi_communicator_t *c) { return c->size; }
static int op_index(struct ompi_op_t *op) { return op->o_f_to_c_index; }
static uint32_t op_flags(struct ompi_op_t *op) { return op->o_flags; }
static ompi_op_base_op_fns_t *op_fns(struct ompi_op_t *op) { return &op->intrinsic; }
static ompi_op_base_op_3buff_fns_t *op_3fns(struct ompi_op_t *op) { return &op->o_3buff_intrinsic; }

static mx_ompi_host_t g_host;

/* ---- requests (ompi/request/request.h:125-139) and progress -------------- */
struct ompi_request_t {
    int persistent, active, complete, status;
    int (*start)(struct ompi_request_t *req);
    int (*free_fn)(struct ompi_request_t *req);
    void *ctx;
};

static struct ompi_request_t *request_create(int persistent, int (*start)(struct ompi_request_t *),
                                             int (*free_fn)(struct ompi_request_t *), void *ctx)
{
    struct ompi_request_t *r = calloc(1, sizeof *r);
    if (!r) return NULL;
    r->persistent = persistent;
    r->active = !persistent;          /* OMPI_REQUEST_INACTIVE until MPI_Start */
    r->complete = persistent;         /* an inactive request tests complete */
    r->start = start;
    r->free_fn = free_fn;
    r->ctx = ctx;
    return r;
}
static void *request_ctx(struct ompi_request_t *r) { return r->ctx; }
/* the host's side of a request a component drives itself (mx_ompi_abi.h) */
static int inner_test(struct ompi_request_t *r, int *flag, int *status)
{
    *flag = r->complete;
    *status = r->complete ? r->status : OMPI_SUCCESS;
    return OMPI_SUCCESS;
}
static int inner_start(struct ompi_request_t *r) { return r->start(r); }
static int inner_free(struct ompi_request_t **rp)
{
    struct ompi_request_t *r = *rp;
    if (!r) return OMPI_SUCCESS;
    const int rc = r->free_fn(r);
    free(r);
    *rp = NULL;
    return rc;
}
static void request_activate(struct ompi_request_t *r) { r->active = 1; r->complete = 0; r->status = 0; }
static void request_complete(struct ompi_request_t *r, int status) { r->status = status; r->complete = 1; }

#define MAXPROGRESS 8
static int (*g_progress[MAXPROGRESS])(void);
static int g_nprogress;
static int progress_register(int (*fn)(void))        /* opal_progress_register */
{
    for (int i = 0; i < g_nprogress; i++)
        if (g_progress[i] == fn) return 0;
    if (g_nprogress == MAXPROGRESS) return -1;
    g_progress[g_nprogress++] = fn;
    return 0;
}
static void opal_progress(void)
{
    for (int i = 0; i < g_nprogress; i++) g_progress[i]();
}

/* ompi_op_reduce (op.h:547-610) */
static void op_reduce(struct ompi_op_t *op, const void *source, void *target, int count, struct ompi_datatype_t *dt)
{
    struct ompi_datatype_t *d = dt;
    int cnt = count;
    op->intrinsic.fns[dt->slot]((void *)source, target, &cnt, &d, op->intrinsic.modules[dt->slot]);
}

/* ---- host coll modules ---------------------------------------------------
 * Stand-ins for the modules coll/mi355x stacks on, with the reference's
 * class names (coll/mi355x reads the order it must reproduce from them):
 *   tuned  (priority 30, "mca_coll_tuned_module_t"): coll/tuned's algorithms
 *          -- the fixed decision, or with coll_tuned_use_dynamic_rules the
 *          forced coll_tuned_<coll>_algorithm -- evaluated by the injected
 *          oracle restatement over every rank's inputs; its compositions
 *          (allreduce / reduce_scatter nonoverlapping, reduce_scatter_block
 *          basic_linear) call the communicator's current coll_reduce /
 *          coll_bcast like coll/base does (coll_base_allreduce.c:54-86);
 *   basic  (priority 10, "mca_coll_basic_module_t"): coll/basic's
 *          allreduce = coll_reduce to 0 + coll_bcast, linear reduce up to
 *          coll_basic_crossover ranks (its log-tree reduce above that is not
 *          restated: the call fails), recursive-halving reduce_scatter below
 *          8 MiB else coll_reduce + scatterv, linear scan / exscan;
 *   libnbc (priority 10, "ompi_coll_libnbc_module_t"): the nonblocking and
 *          persistent slots with libnbc's orders (oracle), complete at post /
 *          start.
 * `coll` (OMPI_MCA_coll / mxh_set_mca_str) "^tuned" excludes tuned as
 * --mca coll ^tuned does.  Host memory only: the harness transport is a
 * host allgather. */
static int dtype_pack(struct ompi_datatype_t *d, int count, const void *user, void *packed);
static int dtype_unpack(struct ompi_datatype_t *d, int count, const void *packed, void *user);

static mxh_coll_oracle_t g_or;
int mxh_set_coll_oracle(const mxh_coll_oracle_t *o)
{
    g_or = *o;
    return 0;
}

#define NSVARS 16
static struct { char name[96]; char value[512]; int set; } g_svars[NSVARS];
int mxh_set_mca_str(const char *name, const char *value)
{
    for (int i = 0; i < NSVARS; i++) {
        if (!g_svars[i].set || !strcmp(g_svars[i].name, name)) {
            snprintf(g_svars[i].name, sizeof g_svars[i].name, "%s", name);
            if (value) snprintf(g_svars[i].value, sizeof g_svars[i].value, "%s", value);
            g_svars[i].set = value != NULL;
            return 0;
        }
    }
    return -1;
}
static const char *mca_string(const char *name)
{
    char env[160];
    for (int i = 0; i < NSVARS; i++)
        if (g_svars[i].set && !strcmp(g_svars[i].name, name)) return g_svars[i].value;
    snprintf(env, sizeof env, "OMPI_MCA_%s", name);
    return getenv(env);
}

static int comm_is_inter(struct ompi_communicator_t *c);

/* every rank's `bytes` (rank-major) through the harness transport */
static char *gather(struct ompi_communicator_t *c, const void *mine, size_t bytes)
{
    char *all = malloc(bytes * (size_t)c->size + 1);
    if (all && c->ag(mine, all, bytes, c->ag_ctx)) {
        free(all);
        all = NULL;
    }
    return all;
}

/* the current (top) entry of a slot: what coll/base's compositions call */
#define TOP(c, name, T) ((T)(c)->fn[slot_index(#name)])
#define TOPMOD(c, name) ((c)->mod[slot_index(#name)])

/* coll/tuned's forced algorithm of a collective (dynamic rules only) */
static int tuned_forced(const char *coll, int *fanout)
{
    char v[96];
    *fanout = 0;
    if (!mca_int("coll_tuned_use_dynamic_rules", 0)) return 0;
    snprintf(v, sizeof v, "coll_tuned_%s_algorithm_chain_fanout", coll);
    *fanout = mca_int(v, 0);
    snprintf(v, sizeof v, "coll_tuned_%s_algorithm", coll);
    return mca_int(v, 0);
}

/* n-rank oracle allreduce on everyone's inputs, my result to rbuf */
static int oracle_allreduce(int alg, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt,
                            struct ompi_op_t *op, struct ompi_communicator_t *c, int nbc)
{
    const int n = c->size, inplace = sbuf == MPI_IN_PLACE;
    const size_t b = (size_t)count * dt->size;
    char *all = gather(c, inplace ? rbuf : sbuf, b), *outs = malloc(b * n + 1);
    const void *sp[256];
    void *rp[256];
    int rc = (all && outs && n <= 256) ? 0 : OMPI_ERR_OUT_OF_RESOURCE;
    for (int r = 0; !rc && r < n; r++) {
        sp[r] = all + (size_t)r * b;
        rp[r] = outs + (size_t)r * b;
        if (inplace) memcpy(rp[r], sp[r], b);
    }
    if (!rc) rc = nbc ? g_or.iallreduce(alg, op->o_f_to_c_index, dt->slot, n, (size_t)count, inplace ? NULL : sp, rp)
                      : g_or.allreduce(alg, op->o_f_to_c_index, dt->slot, n, (size_t)count, inplace ? NULL : sp, rp);
    if (!rc) memcpy(rbuf, outs + (size_t)c->rank * b, b);
    free(all);
    free(outs);
    return rc ? OMPI_ERROR : OMPI_SUCCESS;
}

/* n-rank oracle rooted reduce (root's result to rbuf); nbc: libnbc's */
static int oracle_reduce(int alg, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt,
                         struct ompi_op_t *op, int root, struct ompi_communicator_t *c, int nbc)
{
    const int n = c->size, inplace = sbuf == MPI_IN_PLACE && c->rank == root;
    const size_t b = (size_t)count * dt->size;
    /* rank order of inputs; the root's flag travels in one extra byte */
    char *mine = malloc(b + 1);
    if (!mine) return OMPI_ERR_OUT_OF_RESOURCE;
    memcpy(mine, inplace ? rbuf : sbuf, b);
    mine[b] = (char)inplace;
    char *all = gather(c, mine, b + 1);
    free(mine);
    if (!all) return OMPI_ERROR;
    int rc = 0;
    if (c->rank == root) {
        const void *sp[256];
        const int root_inplace = all[(size_t)root * (b + 1) + b];
        for (int r = 0; r < n; r++) sp[r] = all + (size_t)r * (b + 1);
        char *out = malloc(b + 1);
        if (root_inplace) {
            memcpy(out, sp[root], b);
            sp[root] = NULL;
        }
        rc = nbc ? g_or.ireduce(alg, op->o_f_to_c_index, dt->slot, n, (size_t)count, root, sp, out)
                 : g_or.reduce(alg, op->o_f_to_c_index, dt->slot, n, (size_t)count, root, sp, out);
        if (!rc) memcpy(rbuf, out, b);
        free(out);
    }
    free(all);
    return rc ? OMPI_ERROR : OMPI_SUCCESS;
}

/* n-rank oracle reduce_scatter (alg < 0: libnbc's ireduce_scatter) */
static int oracle_reduce_scatter(int alg, const void *sbuf, void *rbuf, const int *rcounts,
                                 struct ompi_datatype_t *dt, struct ompi_op_t *op, struct ompi_communicator_t *c)
{
    const int n = c->size, inplace = sbuf == MPI_IN_PLACE;
    size_t total = 0, rc64[256], disp = 0;
    if (n > 256) return OMPI_ERR_NOT_SUPPORTED;
    for (int r = 0; r < n; r++) {
        rc64[r] = (size_t)rcounts[r];
        if (r < c->rank) disp += rc64[r];
        total += rc64[r];
    }
    const size_t b = total * dt->size;
    char *all = gather(c, inplace ? rbuf : sbuf, b), *outs = malloc(b * n + 1);
    const void *sp[256];
    void *rp[256];
    int rc = (all && outs) ? 0 : OMPI_ERR_OUT_OF_RESOURCE;
    for (int r = 0; !rc && r < n; r++) {
        sp[r] = all + (size_t)r * b;
        rp[r] = outs + (size_t)r * b;
        if (inplace) memcpy(rp[r], sp[r], b);
    }
    if (!rc)
        rc = alg < 0 ? g_or.ireduce_scatter(op->o_f_to_c_index, dt->slot, n, rc64, inplace ? NULL : sp, rp)
                     : g_or.reduce_scatter(alg, op->o_f_to_c_index, dt->slot, n, rc64, inplace ? NULL : sp, rp);
    if (!rc) memcpy(rbuf, outs + (size_t)c->rank * b, rc64[c->rank] * dt->size);
    (void)disp;
    free(all);
    free(outs);
    return rc ? OMPI_ERROR : OMPI_SUCCESS;
}

static int oracle_scan(int alg, const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt,
                       struct ompi_op_t *op, struct ompi_communicator_t *c, int exclusive)
{
    const int n = c->size, inplace = sbuf == MPI_IN_PLACE;
    const size_t b = (size_t)count * dt->size;
    char *all = gather(c, inplace ? rbuf : sbuf, b), *outs = malloc(b * n + 1);
    const void *sp[256];
    void *rp[256];
    int rc = (all && outs && n <= 256) ? 0 : OMPI_ERR_OUT_OF_RESOURCE;
    for (int r = 0; !rc && r < n; r++) {
        sp[r] = all + (size_t)r * b;
        rp[r] = outs + (size_t)r * b;
    }
    if (!rc) rc = (exclusive ? g_or.exscan : g_or.scan)(alg, op->o_f_to_c_index, dt->slot, n, (size_t)count, sp, rp);
    if (!rc && !(exclusive && c->rank == 0)) memcpy(rbuf, outs + (size_t)c->rank * b, b);
    free(all);
    free(outs);
    return rc ? OMPI_ERROR : OMPI_SUCCESS;
}

/* scatterv of root 0's `full` vector (bytes) by rcounts: my block to rbuf */
static int scatter_from0(struct ompi_communicator_t *c, const char *full, size_t total, const int *rcounts,
                         struct ompi_datatype_t *dt, void *rbuf)
{
    const size_t b = total * dt->size;
    char *zero = calloc(1, b + 1);
    if (!zero) return OMPI_ERR_OUT_OF_RESOURCE;
    char *all = gather(c, c->rank == 0 ? full : zero, b);
    free(zero);
    if (!all) return OMPI_ERROR;
    size_t disp = 0;
    for (int r = 0; r < c->rank; r++) disp += (size_t)rcounts[r];
    memcpy(rbuf, all + disp * dt->size, (size_t)rcounts[c->rank] * dt->size);
    free(all);
    return OMPI_SUCCESS;
}

/* coll_reduce (the top entry) of `total` to root 0, then scatterv.  root_ip:
 * an MPI_IN_PLACE call reduces MPI_IN_PLACE on the root (coll/base's
 * nonoverlapping); else sbuf = rbuf (coll/basic, basic_linear) */
static int reduce_then_scatter(const void *sbuf, void *rbuf, const int *rcounts, size_t total,
                               struct ompi_datatype_t *dt, struct ompi_op_t *op, struct ompi_communicator_t *c,
                               int root_ip)
{
    const int inplace = sbuf == MPI_IN_PLACE;
    char *tmp = c->rank == 0 ? malloc(total * dt->size + 1) : NULL;
    int rc;
    if (c->rank == 0 && !tmp) return OMPI_ERR_OUT_OF_RESOURCE;
    if (inplace && root_ip) {
        if (c->rank == 0) memcpy(tmp, rbuf, total * dt->size);
        rc = TOP(c, reduce, mca_coll_base_module_reduce_fn_t)(c->rank == 0 ? MPI_IN_PLACE : rbuf, tmp, (int)total,
                                                              dt, op, 0, c, TOPMOD(c, reduce));
    } else {
        rc = TOP(c, reduce, mca_coll_base_module_reduce_fn_t)(inplace ? rbuf : sbuf, tmp, (int)total, dt, op, 0, c,
                                                              TOPMOD(c, reduce));
    }
    if (rc == OMPI_SUCCESS) rc = scatter_from0(c, tmp, total, rcounts, dt, rbuf);
    free(tmp);
    return rc;
}

/* coll_reduce to 0 + coll_bcast (coll_base_allreduce.c:54-86,
 * coll_basic_allreduce.c:45-71) */
static int reduce_then_bcast(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt,
                             struct ompi_op_t *op, struct ompi_communicator_t *c)
{
    int rc;
    if (sbuf == MPI_IN_PLACE)
        rc = TOP(c, reduce, mca_coll_base_module_reduce_fn_t)(c->rank == 0 ? MPI_IN_PLACE : rbuf,
                                                              c->rank == 0 ? rbuf : NULL, count, dt, op, 0, c,
                                                              TOPMOD(c, reduce));
    else
        rc = TOP(c, reduce, mca_coll_base_module_reduce_fn_t)(sbuf, rbuf, count, dt, op, 0, c, TOPMOD(c, reduce));
    if (rc != OMPI_SUCCESS) return rc;
    return TOP(c, bcast, mca_coll_base_module_bcast_fn_t)(rbuf, count, dt, 0, c, TOPMOD(c, bcast));
}

/* data movement (any module gives the same bytes) */
static int base_allgather(const void *sbuf, int scount, struct ompi_datatype_t *sdt, void *rbuf, int rcount,
                          struct ompi_datatype_t *rdt, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    const size_t rb = (size_t)rcount * rdt->size, rext = (size_t)rcount * dtype_extent(rdt);
    char *mine = malloc(rb + 1), *tmp;
    if (!mine) return OMPI_ERR_OUT_OF_RESOURCE;
    if (sbuf == MPI_IN_PLACE) dtype_pack(rdt, rcount, (char *)rbuf + (size_t)c->rank * rext, mine);
    else dtype_pack(sdt, scount, sbuf, mine);
    tmp = gather(c, mine, rb);
    free(mine);
    if (!tmp) return OMPI_ERROR;
    for (int p = 0; p < c->size; p++) dtype_unpack(rdt, rcount, tmp + (size_t)p * rb, (char *)rbuf + p * rext);
    free(tmp);
    return OMPI_SUCCESS;
}

static int base_bcast(void *buf, int count, struct ompi_datatype_t *dt, int root, struct ompi_communicator_t *c,
                      mca_coll_base_module_t *m)
{
    (void)m;
    const size_t b = (size_t)count * dt->size;
    char *mine = malloc(b + 1), *all;
    if (!mine) return OMPI_ERR_OUT_OF_RESOURCE;
    dtype_pack(dt, count, buf, mine);
    all = gather(c, mine, b);
    free(mine);
    if (!all) return OMPI_ERROR;
    dtype_unpack(dt, count, all + (size_t)root * b, buf);
    free(all);
    return OMPI_SUCCESS;
}

/* coll/self-like reduce_local: mca_coll_base_reduce_local (coll_base_reduce.c:42-49) */
static int base_reduce_local(const void *in, void *inout, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                             mca_coll_base_module_t *m)
{
    (void)m;
    op_reduce(op, in, inout, count, dt);
    return OMPI_SUCCESS;
}

/* ---- coll/self (priority 75, coll_self_module.c:60-84) on size-1
 * communicators: local copies over HOST memory (ompi_datatype_copy_content_
 * same_ddt, coll_self_allreduce.c:41-44; ompi_datatype_sndrcv for allgather),
 * in place a no-op; exscan and bcast touch nothing.  reduce_scatter_block is
 * coll/basic's on one rank (reduce to 0, then scatter): the same copy.
 * g_self_calls counts the calls that reached these functions, so a test sees
 * what was delegated to them. */
static int g_self_calls;
int mxh_self_calls(void) { return g_self_calls; }
static int self_copy(const void *s, struct ompi_datatype_t *sdt, int scount, void *r, struct ompi_datatype_t *rdt,
                     int rcount)
{
    g_self_calls++;
    if (s == MPI_IN_PLACE) return OMPI_SUCCESS;
    const size_t b = (size_t)scount * sdt->size;
    if (b != (size_t)rcount * rdt->size) return OMPI_ERROR;
    char *tmp = malloc(b + 1);
    if (!tmp) return OMPI_ERR_OUT_OF_RESOURCE;
    dtype_pack(sdt, scount, s, tmp);
    dtype_unpack(rdt, rcount, tmp, r);
    free(tmp);
    return OMPI_SUCCESS;
}
static int self_allreduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                          struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)op; (void)c; (void)m;
    return self_copy(sbuf, dt, count, rbuf, dt, count);
}
static int self_reduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, struct ompi_datatype_t *dt,
                               struct ompi_op_t *op, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)op; (void)c; (void)m;
    return self_copy(sbuf, dt, rcounts[0], rbuf, dt, rcounts[0]);
}
static int self_reduce_scatter_block(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dt,
                                     struct ompi_op_t *op, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)op; (void)c; (void)m;
    return self_copy(sbuf, dt, rcount, rbuf, dt, rcount);
}
static int self_allgather(const void *sbuf, int scount, struct ompi_datatype_t *sdt, void *rbuf, int rcount,
                          struct ompi_datatype_t *rdt, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)c; (void)m;
    return self_copy(sbuf, sdt, scount, rbuf, rdt, rcount);
}
static int self_bcast(void *buf, int count, struct ompi_datatype_t *dt, int root, struct ompi_communicator_t *c,
                      mca_coll_base_module_t *m)
{
    (void)buf; (void)count; (void)dt; (void)root; (void)c; (void)m;
    g_self_calls++;
    return OMPI_SUCCESS;
}
static int self_reduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                       int root, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)op; (void)root; (void)c; (void)m;
    return self_copy(sbuf, dt, count, rbuf, dt, count);
}
static int self_scan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                     struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)op; (void)c; (void)m;
    return self_copy(sbuf, dt, count, rbuf, dt, count);
}
static int self_exscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                       struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)sbuf; (void)rbuf; (void)count; (void)dt; (void)op; (void)c; (void)m;
    g_self_calls++;
    return OMPI_SUCCESS;
}

/* ---- tuned ---- */
static int tuned_allreduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                           struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    int fan;
    const int alg = tuned_forced("allreduce", &fan);
    (void)m;
    if (alg == 2) return reduce_then_bcast(sbuf, rbuf, count, dt, op, c);   /* nonoverlapping */
    return oracle_allreduce(alg, sbuf, rbuf, count, dt, op, c, 0);
}

static int tuned_reduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, struct ompi_datatype_t *dt,
                                struct ompi_op_t *op, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    int fan;
    const int alg = tuned_forced("reduce_scatter", &fan);
    size_t total = 0;
    (void)m;
    for (int r = 0; r < c->size; r++) total += (size_t)rcounts[r];
    if (alg == 1) return reduce_then_scatter(sbuf, rbuf, rcounts, total, dt, op, c, 1);   /* nonoverlapping */
    return oracle_reduce_scatter(alg, sbuf, rbuf, rcounts, dt, op, c);
}

static int tuned_reduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                        int root, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    int fan;
    const int alg = tuned_forced("reduce", &fan);
    (void)m;
    if (alg == 7) return OMPI_ERR_NOT_SUPPORTED;   /* redscat_gather: not restated */
    return oracle_reduce(alg | ((alg == 2 && fan > 0) ? fan << 16 : 0), sbuf, rbuf, count, dt, op, root, c, 0);
}

static int tuned_reduce_scatter_block(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dt,
                                      struct ompi_op_t *op, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    int fan, rcounts[256];
    const int alg = tuned_forced("reduce_scatter_block", &fan);
    (void)m;
    if ((alg != 0 && alg != 1) || c->size > 256) return OMPI_ERR_NOT_SUPPORTED;   /* 2-4: not restated */
    for (int r = 0; r < c->size; r++) rcounts[r] = rcount;
    return reduce_then_scatter(sbuf, rbuf, rcounts, (size_t)rcount * c->size, dt, op, c, 0);   /* basic_linear */
}

static int tuned_scan_common(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt,
                             struct ompi_op_t *op, struct ompi_communicator_t *c, int exclusive)
{
    int fan;
    const int alg = tuned_forced(exclusive ? "exscan" : "scan", &fan);
    return oracle_scan(alg == 2 ? 2 : 1, sbuf, rbuf, count, dt, op, c, exclusive);
}
static int tuned_scan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                      struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    return tuned_scan_common(sbuf, rbuf, count, dt, op, c, 0);
}
static int tuned_exscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                        struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    return tuned_scan_common(sbuf, rbuf, count, dt, op, c, 1);
}

/* ---- basic ---- */
static int basic_allreduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                           struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    return reduce_then_bcast(sbuf, rbuf, count, dt, op, c);
}

static int basic_reduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                        int root, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    if (c->size > mca_int("coll_basic_crossover", 4)) return OMPI_ERR_NOT_SUPPORTED;   /* log tree: not restated */
    return oracle_reduce(1, sbuf, rbuf, count, dt, op, root, c, 0);                      /* linear */
}

static int basic_reduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, struct ompi_datatype_t *dt,
                                struct ompi_op_t *op, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    size_t total = 0;
    (void)m;
    for (int r = 0; r < c->size; r++) total += (size_t)rcounts[r];
    if (total * dt->size < ((size_t)8 << 20)) return oracle_reduce_scatter(2, sbuf, rbuf, rcounts, dt, op, c);
    return reduce_then_scatter(sbuf, rbuf, rcounts, total, dt, op, c, 0);
}

static int basic_reduce_scatter_block(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dt,
                                      struct ompi_op_t *op, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    int rcounts[256];
    (void)m;
    if (c->size > 256) return OMPI_ERR_NOT_SUPPORTED;
    for (int r = 0; r < c->size; r++) rcounts[r] = rcount;
    return reduce_then_scatter(sbuf, rbuf, rcounts, (size_t)rcount * c->size, dt, op, c, 0);
}

static int basic_scan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                      struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    return oracle_scan(1, sbuf, rbuf, count, dt, op, c, 0);
}
static int basic_exscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                        struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    return oracle_scan(1, sbuf, rbuf, count, dt, op, c, 1);
}

/* ---- libnbc: nonblocking / persistent, complete at post (or MPI_Start) ---- */
typedef struct {
    int slot;
    const void *sbuf;
    void *rbuf;
    int count, scount, root;
    int *rcounts;
    struct ompi_datatype_t *dt, *rdt;
    struct ompi_op_t *op;
    struct ompi_communicator_t *c;
} base_nb_t;

static int base_nb_run(const base_nb_t *a)
{
    switch (a->slot) {
    case S_IALLREDUCE:
        return oracle_allreduce(mca_int("coll_libnbc_iallreduce_algorithm", 0), a->sbuf, a->rbuf, a->count, a->dt,
                                a->op, a->c, 1);
    case S_IREDUCE:
        return oracle_reduce(mca_int("coll_libnbc_ireduce_algorithm", 0), a->sbuf, a->rbuf, a->count, a->dt, a->op,
                             a->root, a->c, 1);
    case S_IREDUCE_SCATTER: return oracle_reduce_scatter(-1, a->sbuf, a->rbuf, a->rcounts, a->dt, a->op, a->c);
    case S_IREDUCE_SCATTER_BLOCK: return oracle_reduce_scatter(-1, a->sbuf, a->rbuf, a->rcounts, a->dt, a->op, a->c);
    case S_ISCAN: return oracle_scan(1, a->sbuf, a->rbuf, a->count, a->dt, a->op, a->c, 0);
    case S_IEXSCAN: return oracle_scan(1, a->sbuf, a->rbuf, a->count, a->dt, a->op, a->c, 1);
    case S_IALLGATHER: return base_allgather(a->sbuf, a->scount, a->dt, a->rbuf, a->count, a->rdt, a->c, NULL);
    case S_IBCAST: return base_bcast(a->rbuf, a->count, a->dt, a->root, a->c, NULL);
    }
    return OMPI_ERROR;
}
/* Like libnbc, a posted operation does not wait for the peers: it runs (a
 * blocking exchange over the harness transport) when the process next
 * progresses -- MPI_Test / MPI_Wait -- in posting order, which every rank
 * shares (collectives are issued in the same order everywhere). */
#define NB_PENDING 256
static struct ompi_request_t *g_nb_pending[NB_PENDING];
static int g_nb_head, g_nb_tail;
static int base_nb_progress(void)
{
    int done = 0;
    while (g_nb_head != g_nb_tail) {
        struct ompi_request_t *r = g_nb_pending[g_nb_head];
        g_nb_head = (g_nb_head + 1) % NB_PENDING;
        request_complete(r, base_nb_run(r->ctx));
        done++;
    }
    return done;
}
static int base_nb_enqueue(struct ompi_request_t *r)
{
    if ((g_nb_tail + 1) % NB_PENDING == g_nb_head) return OMPI_ERR_OUT_OF_RESOURCE;
    g_nb_pending[g_nb_tail] = r;
    g_nb_tail = (g_nb_tail + 1) % NB_PENDING;
    return OMPI_SUCCESS;
}
static int base_nb_start(struct ompi_request_t *r)
{
    request_activate(r);
    return base_nb_enqueue(r);
}
static int base_nb_free(struct ompi_request_t *r)
{
    base_nb_t *a = r->ctx;
    free(a->rcounts);
    free(a);
    return OMPI_SUCCESS;
}
static int base_nb_post(const base_nb_t *a, int persistent, struct ompi_request_t **request)
{
    base_nb_t *h = malloc(sizeof *h);
    if (!h) return OMPI_ERR_OUT_OF_RESOURCE;
    *h = *a;
    if (a->rcounts || a->slot == S_IREDUCE_SCATTER_BLOCK) {
        h->rcounts = malloc(sizeof(int) * (size_t)a->c->size);
        if (!h->rcounts) { free(h); return OMPI_ERR_OUT_OF_RESOURCE; }
        for (int r = 0; r < a->c->size; r++) h->rcounts[r] = a->rcounts ? a->rcounts[r] : a->count;
    }
    *request = request_create(persistent, base_nb_start, base_nb_free, h);
    if (!*request) { free(h->rcounts); free(h); return OMPI_ERR_OUT_OF_RESOURCE; }
    if (!persistent) return base_nb_enqueue(*request);
    return OMPI_SUCCESS;
}
#define NB(...) base_nb_t a_ = {__VA_ARGS__}
static int base_iallreduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                           struct ompi_communicator_t *c, struct ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m;
    NB(.slot = S_IALLREDUCE, .sbuf = sbuf, .rbuf = rbuf, .count = count, .dt = dt, .op = op, .c = c);
    return base_nb_post(&a_, 0, req);
}
static int base_allreduce_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt,
                               struct ompi_op_t *op, struct ompi_communicator_t *c, struct ompi_info_t *info,
                               struct ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m; (void)info;
    NB(.slot = S_IALLREDUCE, .sbuf = sbuf, .rbuf = rbuf, .count = count, .dt = dt, .op = op, .c = c);
    return base_nb_post(&a_, 1, req);
}
static int base_ireduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                        int root, struct ompi_communicator_t *c, struct ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m;
    NB(.slot = S_IREDUCE, .sbuf = sbuf, .rbuf = rbuf, .count = count, .dt = dt, .op = op, .root = root, .c = c);
    return base_nb_post(&a_, 0, req);
}
static int base_reduce_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                            int root, struct ompi_communicator_t *c, struct ompi_info_t *info,
                            struct ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m; (void)info;
    NB(.slot = S_IREDUCE, .sbuf = sbuf, .rbuf = rbuf, .count = count, .dt = dt, .op = op, .root = root, .c = c);
    return base_nb_post(&a_, 1, req);
}
static int base_ireduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, struct ompi_datatype_t *dt,
                                struct ompi_op_t *op, struct ompi_communicator_t *c, struct ompi_request_t **req,
                                mca_coll_base_module_t *m)
{
    (void)m;
    NB(.slot = S_IREDUCE_SCATTER, .sbuf = sbuf, .rbuf = rbuf, .rcounts = (int *)rcounts, .dt = dt, .op = op, .c = c);
    return base_nb_post(&a_, 0, req);
}
static int base_reduce_scatter_init(const void *sbuf, void *rbuf, const int *rcounts, struct ompi_datatype_t *dt,
                                    struct ompi_op_t *op, struct ompi_communicator_t *c, struct ompi_info_t *info,
                                    struct ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m; (void)info;
    NB(.slot = S_IREDUCE_SCATTER, .sbuf = sbuf, .rbuf = rbuf, .rcounts = (int *)rcounts, .dt = dt, .op = op, .c = c);
    return base_nb_post(&a_, 1, req);
}
static int base_ireduce_scatter_block(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dt,
                                      struct ompi_op_t *op, struct ompi_communicator_t *c, struct ompi_request_t **req,
                                      mca_coll_base_module_t *m)
{
    (void)m;
    NB(.slot = S_IREDUCE_SCATTER_BLOCK, .sbuf = sbuf, .rbuf = rbuf, .count = rcount, .dt = dt, .op = op, .c = c);
    return base_nb_post(&a_, 0, req);
}
static int base_reduce_scatter_block_init(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dt,
                                          struct ompi_op_t *op, struct ompi_communicator_t *c,
                                          struct ompi_info_t *info, struct ompi_request_t **req,
                                          mca_coll_base_module_t *m)
{
    (void)m; (void)info;
    NB(.slot = S_IREDUCE_SCATTER_BLOCK, .sbuf = sbuf, .rbuf = rbuf, .count = rcount, .dt = dt, .op = op, .c = c);
    return base_nb_post(&a_, 1, req);
}
#define BASE_SCAN_NB(fname, SLOT)                                                                               \
    static int base_i##fname(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt,               \
                             struct ompi_op_t *op, struct ompi_communicator_t *c, struct ompi_request_t **req,  \
                             mca_coll_base_module_t *m)                                                        \
    {                                                                                                           \
        (void)m;                                                                                                \
        NB(.slot = SLOT, .sbuf = sbuf, .rbuf = rbuf, .count = count, .dt = dt, .op = op, .c = c);             \
        return base_nb_post(&a_, 0, req);                                                                       \
    }                                                                                                           \
    static int base_##fname##_init(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt,         \
                                   struct ompi_op_t *op, struct ompi_communicator_t *c, struct ompi_info_t *info, \
                                   struct ompi_request_t **req, mca_coll_base_module_t *m)                     \
    {                                                                                                           \
        (void)m; (void)info;                                                                                    \
        NB(.slot = SLOT, .sbuf = sbuf, .rbuf = rbuf, .count = count, .dt = dt, .op = op, .c = c);             \
        return base_nb_post(&a_, 1, req);                                                                       \
    }
BASE_SCAN_NB(scan, S_ISCAN)
BASE_SCAN_NB(exscan, S_IEXSCAN)
static int base_iallgather(const void *sbuf, int scount, struct ompi_datatype_t *sdt, void *rbuf, int rcount,
                           struct ompi_datatype_t *rdt, struct ompi_communicator_t *c, struct ompi_request_t **req,
                           mca_coll_base_module_t *m)
{
    (void)m;
    NB(.slot = S_IALLGATHER, .sbuf = sbuf, .scount = scount, .dt = sdt, .rbuf = rbuf, .count = rcount, .rdt = rdt,
       .c = c);
    return base_nb_post(&a_, 0, req);
}
static int base_allgather_init(const void *sbuf, int scount, struct ompi_datatype_t *sdt, void *rbuf, int rcount,
                               struct ompi_datatype_t *rdt, struct ompi_communicator_t *c, struct ompi_info_t *info,
                               struct ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m; (void)info;
    NB(.slot = S_IALLGATHER, .sbuf = sbuf, .scount = scount, .dt = sdt, .rbuf = rbuf, .count = rcount, .rdt = rdt,
       .c = c);
    return base_nb_post(&a_, 1, req);
}
static int base_ibcast(void *buf, int count, struct ompi_datatype_t *dt, int root, struct ompi_communicator_t *c,
                       struct ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m;
    NB(.slot = S_IBCAST, .rbuf = buf, .count = count, .dt = dt, .root = root, .c = c);
    return base_nb_post(&a_, 0, req);
}
static int base_bcast_init(void *buf, int count, struct ompi_datatype_t *dt, int root, struct ompi_communicator_t *c,
                           struct ompi_info_t *info, struct ompi_request_t **req, mca_coll_base_module_t *m)
{
    (void)m; (void)info;
    NB(.slot = S_IBCAST, .rbuf = buf, .count = count, .dt = dt, .root = root, .c = c);
    return base_nb_post(&a_, 1, req);
}
#undef NB

/* modules: static, one of each (stateless), with the reference's class names */
static mx_obj_class_t g_tuned_class = {"mca_coll_tuned_module_t", NULL};
static mx_obj_class_t g_basic_class = {"mca_coll_basic_module_t", NULL};
static mx_obj_class_t g_libnbc_class = {"ompi_coll_libnbc_module_t", NULL};
static mca_coll_base_module_t g_tuned_coll, g_basic_coll, g_libnbc_coll;
static mca_coll_base_module_t g_self_coll;

static ompi_op_base_component_1_0_0_t *g_op_comp;
static mca_coll_base_component_2_0_0_t *g_coll_comp;
static void *g_dl;
static struct ompi_communicator_t g_self;

/* ompi_op_base_op_select (op_base_op_select.c:88-204) for one op */
static int op_select(struct ompi_op_t *op)
{
    base_op_module_t *bm = &g_base_mod[op->o_f_to_c_index];
    int prio = 0;
    ompi_op_base_module_t *m;
    bm->super.super.obj_class = &g_static_class;
    bm->super.super.obj_reference_count = 1;
    bm->op = op->o_f_to_c_index;
    for (int t = 0; t < OMPI_OP_BASE_TYPE_MAX; t++) {
        const int has = g_pattern(op->o_f_to_c_index, t, 1);
        op->intrinsic.fns[t] = has ? base_2buff : NULL;
        op->intrinsic.modules[t] = &bm->super;
        op->o_3buff_intrinsic.fns[t] = has ? base_3buff : NULL;
        op->o_3buff_intrinsic.modules[t] = &bm->super;
        obj_retain(&bm->super.super);
        obj_retain(&bm->super.super);
    }
    if (!g_op_comp || !(op->o_flags & OMPI_OP_FLAGS_INTRINSIC)) return 0;
    m = g_op_comp->opc_op_query(op, &prio);
    if (!m) return 0;
    if (prio > 100) prio = 100;          /* :279 */
    if (prio < 0) { obj_release(&m->super); return 0; }
    if (m->opm_enable && m->opm_enable(m, op) != OMPI_SUCCESS) { obj_release(&m->super); return 0; }
    for (int t = 0; t < OMPI_OP_BASE_TYPE_MAX; t++) {
        if (m->opm_fns[t]) {
            obj_release(&op->intrinsic.modules[t]->super);
            op->intrinsic.fns[t] = m->opm_fns[t];
            op->intrinsic.modules[t] = m;
            obj_retain(&m->super);
        }
        if (m->opm_3buff_fns[t]) {
            obj_release(&op->o_3buff_intrinsic.modules[t]->super);
            op->o_3buff_intrinsic.fns[t] = m->opm_3buff_fns[t];
            op->o_3buff_intrinsic.modules[t] = m;
            obj_retain(&m->super);
        }
    }
    obj_release(&m->super);
    /* NULL-pattern sanity check (:185-201) */
    for (int t = 0; t < OMPI_OP_BASE_TYPE_MAX; t++)
        if ((g_pattern(op->o_f_to_c_index, t, 1) != 0) != (op->intrinsic.fns[t] != NULL)) return OMPI_ERR_NOT_FOUND;
    return 0;
}

/* --mca coll ^a,b (mca_base_components_filter): excluded component names */
static int coll_excluded(const char *name)
{
    const char *v = mca_string("coll");
    if (!v || v[0] != '^') return 0;
    const size_t l = strlen(name);
    for (const char *p = v + 1; *p;) {
        const char *e = strchr(p, ',');
        const size_t k = e ? (size_t)(e - p) : strlen(p);
        if (k == l && !strncmp(p, name, l)) return 1;
        p += k + (e ? 1 : 0);
    }
    return 0;
}

static void static_module(mca_coll_base_module_t *b, mx_obj_class_t *cls)
{
    b->super.obj_class = cls;
    b->super.obj_reference_count = 1000000;
}

/* mca_coll_base_comm_select (coll_base_comm_select.c:108-309): modules
 * enabled lowest priority first, each non-NULL slot copied over */
static int comm_select(struct ompi_communicator_t *c, int is_self)
{
    memset(c->fn, 0, sizeof c->fn);
#define COPY(MOD, OWNER)                                                                             \
    do {                                                                                             \
        void *f_[NSLOTS] = {(void *)(MOD)->coll_allreduce, (void *)(MOD)->coll_reduce_scatter,       \
                            (void *)(MOD)->coll_allgather, (void *)(MOD)->coll_bcast,                \
                            (void *)(MOD)->coll_reduce_local, (void *)(MOD)->coll_reduce,            \
                            (void *)(MOD)->coll_reduce_scatter_block, (void *)(MOD)->coll_scan,      \
                            (void *)(MOD)->coll_exscan, (void *)(MOD)->coll_iallreduce,              \
                            (void *)(MOD)->coll_ireduce, (void *)(MOD)->coll_ireduce_scatter,        \
                            (void *)(MOD)->coll_ireduce_scatter_block, (void *)(MOD)->coll_iscan,    \
                            (void *)(MOD)->coll_iexscan, (void *)(MOD)->coll_iallgather,             \
                            (void *)(MOD)->coll_ibcast, (void *)(MOD)->coll_allreduce_init,          \
                            (void *)(MOD)->coll_reduce_init, (void *)(MOD)->coll_reduce_scatter_init, \
                            (void *)(MOD)->coll_reduce_scatter_block_init,                           \
                            (void *)(MOD)->coll_scan_init, (void *)(MOD)->coll_exscan_init,          \
                            (void *)(MOD)->coll_allgather_init, (void *)(MOD)->coll_bcast_init};     \
        for (int i_ = 0; i_ < NSLOTS; i_++)                                                          \
            if (f_[i_]) { c->fn[i_] = f_[i_]; c->mod[i_] = (MOD); c->owner[i_] = (OWNER); }          \
    } while (0)
    int base_prio = 30;
    if (is_self) {
        mca_coll_base_module_t *b = &g_self_coll;
        static_module(b, &g_static_class);
        b->coll_reduce_local = base_reduce_local;
        b->coll_allreduce = self_allreduce;
        b->coll_reduce_scatter = self_reduce_scatter;
        b->coll_allgather = self_allgather;
        b->coll_bcast = self_bcast;
        b->coll_reduce = self_reduce;
        b->coll_reduce_scatter_block = self_reduce_scatter_block;
        b->coll_scan = self_scan;
        b->coll_exscan = self_exscan;
        COPY(b, "self");
        base_prio = 75;
    } else {
        /* basic (10): every blocking slot (coll_basic_module.c:92-128) */
        mca_coll_base_module_t *b = &g_basic_coll;
        memset(b, 0, sizeof *b);
        static_module(b, &g_basic_class);
        b->coll_allreduce = basic_allreduce;
        b->coll_reduce_scatter = basic_reduce_scatter;
        b->coll_allgather = base_allgather;
        b->coll_bcast = base_bcast;
        b->coll_reduce_local = base_reduce_local;
        b->coll_reduce = basic_reduce;
        b->coll_reduce_scatter_block = basic_reduce_scatter_block;
        b->coll_scan = basic_scan;
        b->coll_exscan = basic_exscan;
        if (!coll_excluded("basic")) COPY(b, "basic");
        /* libnbc (10): the nonblocking and persistent slots */
        b = &g_libnbc_coll;
        memset(b, 0, sizeof *b);
        static_module(b, &g_libnbc_class);
#define SET_BASE_NB(name) b->coll_##name = base_##name;
        SET_BASE_NB(iallreduce) SET_BASE_NB(ireduce) SET_BASE_NB(ireduce_scatter) SET_BASE_NB(ireduce_scatter_block)
        SET_BASE_NB(iscan) SET_BASE_NB(iexscan) SET_BASE_NB(iallgather) SET_BASE_NB(ibcast)
        SET_BASE_NB(allreduce_init) SET_BASE_NB(reduce_init) SET_BASE_NB(reduce_scatter_init)
        SET_BASE_NB(reduce_scatter_block_init) SET_BASE_NB(scan_init) SET_BASE_NB(exscan_init)
        SET_BASE_NB(allgather_init) SET_BASE_NB(bcast_init)
#undef SET_BASE_NB
        if (!coll_excluded("libnbc")) COPY(b, "libnbc");
        /* tuned (30): intra-communicators only (coll_tuned_module.c:66-69);
         * scan / exscan only when dynamic rules force them (:235-238) */
        b = &g_tuned_coll;
        memset(b, 0, sizeof *b);
        static_module(b, &g_tuned_class);
        b->coll_allreduce = tuned_allreduce;
        b->coll_reduce_scatter = tuned_reduce_scatter;
        b->coll_allgather = base_allgather;
        b->coll_bcast = base_bcast;
        b->coll_reduce = tuned_reduce;
        b->coll_reduce_scatter_block = tuned_reduce_scatter_block;
        {
            int fan;
            if (tuned_forced("scan", &fan)) b->coll_scan = tuned_scan;
            if (tuned_forced("exscan", &fan)) b->coll_exscan = tuned_exscan;
        }
        if (!coll_excluded("tuned") && !comm_is_inter(c)) COPY(b, "tuned");
    }
    if (g_coll_comp && !coll_excluded("mi355x")) {
        int prio = 0;
        mca_coll_base_module_t *m = g_coll_comp->collm_comm_query(c, &prio);
        if (m) {
            if (prio > base_prio && (!m->coll_module_enable || m->coll_module_enable(m, c) == OMPI_SUCCESS)) {
                COPY(m, "mi355x");
                c->modules[c->nmodules++] = m;
            } else {
                obj_release(&m->super);
            }
        }
    }
#undef COPY
    return 0;
}

const char *mxh_comm_slot_owner(void *cv, const char *slot)
{
    struct ompi_communicator_t *c = cv;
    int i = slot_index(slot);
    return (i >= 0 && c->fn[i]) ? c->owner[i] : "";
}

static int self_ag(const void *s, void *r, size_t b, void *ctx)
{
    (void)ctx;
    memcpy(r, s, b);
    return 0;
}

int mxh_init(const char *component_lib, mxh_reducer_t base, mxh_pattern_t pattern)
{
    g_base = base;
    g_pattern = pattern;
    g_host = (mx_ompi_host_t){comm_rank, comm_size, dtype_slot, dtype_size, dtype_contiguous, op_index, op_flags,
                              op_fns, op_3fns, comm_coll_fn, obj_retain, obj_release, mca_int, NULL};
    g_host.byte_dtype = mxh_dtype("MPI_BYTE");
    g_host.request_create = request_create;
    g_host.request_ctx = request_ctx;
    g_host.request_activate = request_activate;
    g_host.request_complete = request_complete;
    g_host.progress_register = progress_register;
    g_host.dtype_pack = dtype_pack;
    g_host.dtype_unpack = dtype_unpack;
    g_host.dtype_span = dtype_span;
    g_host.dtype_desc = getenv("MXH_NO_DTYPE_DESC") ? NULL : dtype_desc;
    g_host.comm_is_inter = comm_is_inter;
    g_host.mca_string = mca_string;
    g_host.request_test = inner_test;
    g_host.request_start = inner_start;
    g_host.request_free = inner_free;
    g_nprogress = 0;
    g_nb_head = g_nb_tail = 0;
    progress_register(base_nb_progress);
    g_op_comp = NULL;
    g_coll_comp = NULL;
    if (component_lib && *component_lib) {
        int (*set_host)(const mx_ompi_host_t *);
        g_dl = dlopen(component_lib, RTLD_NOW | RTLD_GLOBAL);
        if (!g_dl) { fprintf(stderr, "mxh_init: %s\n", dlerror()); return -1; }
        /* mca_base_component_repository: mca_<type>_<name>_component */
        g_op_comp = dlsym(g_dl, "mca_op_mi355x_component");
        g_coll_comp = dlsym(g_dl, "mca_coll_mi355x_component");
        set_host = (int (*)(const mx_ompi_host_t *))dlsym(g_dl, "mx_ompi_set_host");
        if (!g_op_comp || !g_coll_comp || !set_host) return -2;
        set_host(&g_host);
        if (g_op_comp->opc_init_query(false, false) != OMPI_SUCCESS) g_op_comp = NULL;
        if (g_coll_comp->collm_init_query(false, false) != OMPI_SUCCESS) g_coll_comp = NULL;
    }
    for (int i = 0; i < OMPI_OP_BASE_FORTRAN_OP_MAX; i++) {
        struct ompi_op_t *op = &g_ops[i];
        memset(op, 0, sizeof *op);
        snprintf(op->o_name, sizeof op->o_name, "%s", g_opnames[i]);
        op->o_f_to_c_index = i;
        op->o_flags = OMPI_OP_FLAGS_INTRINSIC | OMPI_OP_FLAGS_COMMUTE;
        if (op_select(op)) return -3;
    }
    memset(&g_self, 0, sizeof g_self);
    g_self.rank = 0;
    g_self.size = 1;
    g_self.ag = self_ag;
    comm_select(&g_self, 1);
    return 0;
}

int mxh_finalize(void)
{
    return 0;
}

void *mxh_comm_create(int rank, int size, mxh_allgather_t ag, void *ctx)
{
    struct ompi_communicator_t *c = calloc(1, sizeof *c);
    if (!c) return NULL;
    c->rank = rank;
    c->size = size;
    c->ag = ag;
    c->ag_ctx = ctx;
    comm_select(c, size == 1);
    return c;
}

/* an intercommunicator (local group of `size`): only its selection is
 * modelled -- which components take it */
void *mxh_intercomm_create(int rank, int size, mxh_allgather_t ag, void *ctx)
{
    struct ompi_communicator_t *c = calloc(1, sizeof *c);
    if (!c) return NULL;
    c->rank = rank;
    c->size = size;
    c->inter = 1;
    c->ag = ag;
    c->ag_ctx = ctx;
    comm_select(c, 0);
    return c;
}

void *mxh_comm_self(void) { return &g_self; }

int mxh_comm_free(void *cv)
{
    struct ompi_communicator_t *c = cv;
    if (!c || c == &g_self) return 0;
    for (int i = 0; i < c->nmodules; i++) {
        mca_coll_base_module_t *m = c->modules[i];
        for (int s = 0; s < NSLOTS; s++) (void)s;
        obj_release(&m->super);
    }
    free(c);
    return 0;
}

/* ---- MPI entry points -------------------------------------------------- */
/* ompi_op_reduce(op, source, target, count, dtype) as the coll/base
 * algorithms call it (op.h:547-610) */
int mxh_op_reduce(void *opv, const void *source, void *target, int count, void *dt)
{
    struct ompi_op_t *op = opv;
    struct ompi_datatype_t *d = dt;
    if (!d || d->slot < 0 || !op->intrinsic.fns[d->slot]) return -1;
    op_reduce(op, source, target, count, d);
    return 0;
}

/* ompi_3buff_op_reduce(op, source1, source2, target, count, dtype) (op.h:618-660) */
int mxh_3buff_op_reduce(void *opv, const void *source1, const void *source2, void *target, int count, void *dt)
{
    struct ompi_op_t *op = opv;
    struct ompi_datatype_t *d = dt;
    int cnt = count;
    if (!d || d->slot < 0 || !op->o_3buff_intrinsic.fns[d->slot]) return -1;
    op->o_3buff_intrinsic.fns[d->slot]((void *)source1, (void *)source2, target, &cnt, &d,
                                       op->o_3buff_intrinsic.modules[d->slot]);
    return 0;
}

/* Cost of one ompi_op_reduce through the op table (the segmented ring's
 * per-segment call, coll_base_allreduce.c:782): average ns over `iters`
 * back-to-back calls, after one warm-up call. */
double mxh_time_op_reduce(void *opv, const void *source, void *target, int count, void *dt, int iters)
{
    struct ompi_op_t *op = opv;
    struct ompi_datatype_t *d = dt;
    struct timespec t0, t1;
    if (!d || d->slot < 0 || !op->intrinsic.fns[d->slot] || iters < 1) return -1.0;
    op_reduce(op, source, target, count, d);
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < iters; i++) op_reduce(op, source, target, count, d);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return ((double)(t1.tv_sec - t0.tv_sec) * 1e9 + (double)(t1.tv_nsec - t0.tv_nsec)) / iters;
}

int mxh_reduce_local(const void *in, void *inout, int count, void *dt, void *opv)
{
    struct ompi_op_t *op = opv;
    struct ompi_datatype_t *d = dt;
    /* ompi_op_is_valid (op.h:477-514) */
    if (!d || d->slot < 0 || !op->intrinsic.fns[d->slot]) return -1;
    return ((mca_coll_base_module_reduce_local_fn_t)g_self.fn[4])(in, inout, count, d, op, g_self.mod[4]);
}

int mxh_allreduce(const void *sbuf, void *rbuf, int count, void *dt, void *op, void *cv)
{
    struct ompi_communicator_t *c = cv;
    struct ompi_datatype_t *d = dt;
    if (!d || d->slot < 0 || !((struct ompi_op_t *)op)->intrinsic.fns[d->slot]) return -1;
    return ((mca_coll_base_module_allreduce_fn_t)c->fn[0])(sbuf, rbuf, count, d, op, c, c->mod[0]);
}

int mxh_reduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, void *dt, void *op, void *cv)
{
    struct ompi_communicator_t *c = cv;
    return ((mca_coll_base_module_reduce_scatter_fn_t)c->fn[1])(sbuf, rbuf, rcounts, dt, op, c, c->mod[1]);
}

int mxh_allgather(const void *sbuf, int scount, void *sdt, void *rbuf, int rcount, void *rdt, void *cv)
{
    struct ompi_communicator_t *c = cv;
    return ((mca_coll_base_module_allgather_fn_t)c->fn[2])(sbuf, scount, sdt, rbuf, rcount, rdt, c, c->mod[2]);
}

int mxh_bcast(void *buf, int count, void *dt, int root, void *cv)
{
    struct ompi_communicator_t *c = cv;
    return ((mca_coll_base_module_bcast_fn_t)c->fn[3])(buf, count, dt, root, c, c->mod[3]);
}

int mxh_reduce(const void *sbuf, void *rbuf, int count, void *dt, void *op, int root, void *cv)
{
    struct ompi_communicator_t *c = cv;
    struct ompi_datatype_t *d = dt;
    if (!d || d->slot < 0 || !((struct ompi_op_t *)op)->intrinsic.fns[d->slot]) return -1;
    if (root < 0 || root >= c->size) return -1;
    return ((mca_coll_base_module_reduce_fn_t)c->fn[5])(sbuf, rbuf, count, d, op, root, c, c->mod[5]);
}

int mxh_reduce_scatter_block(const void *sbuf, void *rbuf, int rcount, void *dt, void *op, void *cv)
{
    struct ompi_communicator_t *c = cv;
    return ((mca_coll_base_module_reduce_scatter_block_fn_t)c->fn[6])(sbuf, rbuf, rcount, dt, op, c, c->mod[6]);
}

int mxh_scan(const void *sbuf, void *rbuf, int count, void *dt, void *op, void *cv)
{
    struct ompi_communicator_t *c = cv;
    return ((mca_coll_base_module_scan_fn_t)c->fn[7])(sbuf, rbuf, count, dt, op, c, c->mod[7]);
}

int mxh_exscan(const void *sbuf, void *rbuf, int count, void *dt, void *op, void *cv)
{
    struct ompi_communicator_t *c = cv;
    return ((mca_coll_base_module_exscan_fn_t)c->fn[8])(sbuf, rbuf, count, dt, op, c, c->mod[8]);
}

/* ---- nonblocking / persistent entry points and request completion ------ */
int mxh_iallreduce(const void *sbuf, void *rbuf, int count, void *dt, void *op, void *cv, void **req)
{
    struct ompi_communicator_t *c = cv;
    struct ompi_datatype_t *d = dt;
    if (!d || d->slot < 0 || !((struct ompi_op_t *)op)->intrinsic.fns[d->slot]) return -1;
    return ((mca_coll_base_module_iallreduce_fn_t)c->fn[S_IALLREDUCE])(sbuf, rbuf, count, d, op, c,
                                                                        (struct ompi_request_t **)req,
                                                                        c->mod[S_IALLREDUCE]);
}
int mxh_allreduce_init(const void *sbuf, void *rbuf, int count, void *dt, void *op, void *cv, void **req)
{
    struct ompi_communicator_t *c = cv;
    const int k = slot_index("allreduce_init");
    return ((mca_coll_base_module_allreduce_init_fn_t)c->fn[k])(sbuf, rbuf, count, dt, op, c, NULL,
                                                                 (struct ompi_request_t **)req, c->mod[k]);
}
int mxh_ireduce(const void *sbuf, void *rbuf, int count, void *dt, void *op, int root, void *cv, void **req)
{
    struct ompi_communicator_t *c = cv;
    if (root < 0 || root >= c->size) return -1;
    return ((mca_coll_base_module_ireduce_fn_t)c->fn[S_IREDUCE])(sbuf, rbuf, count, dt, op, root, c,
                                                                  (struct ompi_request_t **)req, c->mod[S_IREDUCE]);
}
int mxh_reduce_init(const void *sbuf, void *rbuf, int count, void *dt, void *op, int root, void *cv, void **req)
{
    struct ompi_communicator_t *c = cv;
    const int k = slot_index("reduce_init");
    if (root < 0 || root >= c->size) return -1;
    return ((mca_coll_base_module_reduce_init_fn_t)c->fn[k])(sbuf, rbuf, count, dt, op, root, c, NULL,
                                                              (struct ompi_request_t **)req, c->mod[k]);
}
int mxh_ireduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, void *dt, void *op, void *cv, void **req)
{
    struct ompi_communicator_t *c = cv;
    return ((mca_coll_base_module_ireduce_scatter_fn_t)c->fn[S_IREDUCE_SCATTER])(
        sbuf, rbuf, rcounts, dt, op, c, (struct ompi_request_t **)req, c->mod[S_IREDUCE_SCATTER]);
}
int mxh_ireduce_scatter_block(const void *sbuf, void *rbuf, int rcount, void *dt, void *op, void *cv, void **req)
{
    struct ompi_communicator_t *c = cv;
    return ((mca_coll_base_module_ireduce_scatter_block_fn_t)c->fn[S_IREDUCE_SCATTER_BLOCK])(
        sbuf, rbuf, rcount, dt, op, c, (struct ompi_request_t **)req, c->mod[S_IREDUCE_SCATTER_BLOCK]);
}
int mxh_iscan(const void *sbuf, void *rbuf, int count, void *dt, void *op, void *cv, void **req)
{
    struct ompi_communicator_t *c = cv;
    return ((mca_coll_base_module_iscan_fn_t)c->fn[S_ISCAN])(sbuf, rbuf, count, dt, op, c,
                                                              (struct ompi_request_t **)req, c->mod[S_ISCAN]);
}
int mxh_iexscan(const void *sbuf, void *rbuf, int count, void *dt, void *op, void *cv, void **req)
{
    struct ompi_communicator_t *c = cv;
    return ((mca_coll_base_module_iexscan_fn_t)c->fn[S_IEXSCAN])(sbuf, rbuf, count, dt, op, c,
                                                                  (struct ompi_request_t **)req, c->mod[S_IEXSCAN]);
}
int mxh_iallgather(const void *sbuf, int scount, void *sdt, void *rbuf, int rcount, void *rdt, void *cv, void **req)
{
    struct ompi_communicator_t *c = cv;
    return ((mca_coll_base_module_iallgather_fn_t)c->fn[S_IALLGATHER])(
        sbuf, scount, sdt, rbuf, rcount, rdt, c, (struct ompi_request_t **)req, c->mod[S_IALLGATHER]);
}
int mxh_ibcast(void *buf, int count, void *dt, int root, void *cv, void **req)
{
    struct ompi_communicator_t *c = cv;
    return ((mca_coll_base_module_ibcast_fn_t)c->fn[S_IBCAST])(buf, count, dt, root, c,
                                                                (struct ompi_request_t **)req, c->mod[S_IBCAST]);
}

/* MPI_Start (ompi/mpi/c/start.c: req->req_start) */
int mxh_start(void *rv)
{
    struct ompi_request_t *r = rv;
    if (!r || !r->persistent || r->active) return -1;
    return r->start(r);
}

/* MPI_Test / MPI_Wait (ompi_request_default_test / _wait): drive
 * opal_progress until complete; a completed nonblocking request is freed
 * (set to MPI_REQUEST_NULL), a persistent one becomes inactive. */
static int finish_request(void **rp)
{
    struct ompi_request_t *r = *rp;
    const int st = r->status;
    if (r->persistent) {
        r->active = 0;
    } else {
        const int frc = r->free_fn(r);
        free(r);
        *rp = NULL;
        if (st == OMPI_SUCCESS && frc != OMPI_SUCCESS) return frc;
    }
    return st;
}
int mxh_test(void **rp, int *flag)
{
    struct ompi_request_t *r = *rp;
    *flag = 1;
    if (!r || (r->persistent && !r->active)) return 0;
    if (!r->complete) opal_progress();
    if (!r->complete) { *flag = 0; return 0; }
    return finish_request(rp);
}
int mxh_wait(void **rp)
{
    struct ompi_request_t *r = *rp;
    if (!r || (r->persistent && !r->active)) return 0;
    while (!r->complete) opal_progress();
    return finish_request(rp);
}
/* MPI_Request_free (ompi/mpi/c/request_free.c -> req_free) */
int mxh_request_free(void **rp)
{
    struct ompi_request_t *r = *rp;
    if (!r) return 0;
    const int rc = r->free_fn(r);
    free(r);
    *rp = NULL;
    return rc;
}

/* ---------------------------------------------------------------------------
 * The datatype engine around the mi355x convertor hook.  Restates what
 * opal_convertor_prepare_for_send / _for_recv leave in the convertor for a
 * homogeneous committed type (OPAL_CONVERTOR_PREPARE, opal_convertor.c:
 * 520-560: pDesc, use_desc = &opt_desc, count, pBaseBuf, local_size), where a
 * fragmenting sender / receiver starts (opal_convertor_set_position: the
 * packed byte `start`), calls the hook the maintainer adds after the loop
 * choice, then drives fAdvance the way
 * opal_convertor_pack / _unpack do (opal_convertor.c:218-330) with `niov`
 * iovecs of `frag` bytes per call, until the message is complete.
 * `packed` holds the stream bytes [start, local_size).  Returns 0, or < 0
 * (the hook declined: -10; an fAdvance error: -11; a contract violation:
 * -12).  *calls: fAdvance calls made.
 * ------------------------------------------------------------------------- */
int mxh_convertor_run(const void *desc, size_t nrec, size_t size, int64_t lb, int64_t ub, int64_t true_lb,
                      int64_t true_ub, size_t count, void *user, void *packed, size_t start, size_t frag,
                      int niov, int recv, int *calls)
{
    int (*prep)(opal_convertor_t *) = g_dl ? (int (*)(opal_convertor_t *))dlsym(g_dl, "mca_convertor_mi355x_prepare")
                                           : NULL;
    if (!prep || niov < 1 || niov > 8 || !frag) return -1;
    opal_datatype_t dt;
    memset(&dt, 0, sizeof dt);
    dt.size = size;
    dt.lb = lb;
    dt.ub = ub;
    dt.true_lb = true_lb;
    dt.true_ub = true_ub;
    dt.flags = 0x0004;                              /* OPAL_DATATYPE_FLAG_COMMITTED */
    dt.opt_desc.desc = (void *)desc;
    dt.opt_desc.used = nrec - 1;                    /* the closing END_LOOP is not counted */
    dt.opt_desc.length = nrec;
    dt.desc = dt.opt_desc;
    opal_convertor_t c;
    memset(&c, 0, sizeof c);
    c.flags = CONVERTOR_HOMOGENEOUS | (recv ? CONVERTOR_RECV : CONVERTOR_SEND);
    c.pDesc = &dt;
    c.use_desc = &dt.opt_desc;
    c.count = count;
    c.pBaseBuf = (unsigned char *)user;
    c.local_size = count * size;
    c.remote_size = c.local_size;
    c.pStack = c.static_stack;
    c.stack_size = DT_STATIC_STACK_SIZE;
    c.bConverted = start;
    if (!prep(&c) || !c.fAdvance) return -10;
    *calls = 0;
    char *p = (char *)packed;
    while (!(c.flags & CONVERTOR_COMPLETED)) {
        struct iovec iov[8];
        for (int i = 0; i < niov; i++) {
            iov[i].iov_base = p + (size_t)i * frag;
            iov[i].iov_len = frag;
        }
        uint32_t out = (uint32_t)niov;
        size_t max = (size_t)niov * frag;
        const size_t before = c.bConverted;
        const int32_t rc = c.fAdvance(&c, iov, &out, &max);
        (*calls)++;
        if (rc < 0) return -11;
        size_t sum = 0;
        for (uint32_t i = 0; i < out; i++) sum += iov[i].iov_len;
        /* the contract: max_data = the bytes moved = the iovecs' lengths,
         * bConverted advanced by them, 1 exactly at the end of the message */
        if (sum != max || c.bConverted != before + max || (rc == 1) != (c.bConverted == c.local_size) ||
            (!max && rc != 1))
            return -12;
        /* iovecs are filled in order: only the last one used may be short */
        for (uint32_t i = 0; i + 1 < out; i++)
            if (iov[i].iov_len != frag) return -12;
        p += max;
    }
    /* a completed convertor packs nothing more (OPAL_CONVERTOR_SET_STATUS_BEFORE_PACK_UNPACK) */
    struct iovec extra = {p, frag};
    uint32_t out = 1;
    size_t max = frag;
    if (c.fAdvance(&c, &extra, &out, &max) != 1 || out != 0 || max != 0) return -12;
    return 0;
}

/* ---------------------------------------------------------------------------
 * A host shared-memory BTL module (vader / smcuda stand-in: eager and send
 * limits only, no transport of its own) with the mi355x GPU RDMA slots
 * installed by the component's mca_btl_mi355x_install, the way smcuda's
 * component init installs its CUDA get (btl_smcuda_component.c:936), and
 * ob1's RGET / PUT steps on device buffers restated around it: the owner
 * registers its buffer (btl_register_mem) and ships the handle bytes
 * (btl_registration_handle_size of them, in the PML header); the peer calls
 * btl_get / btl_put with them and drives opal_progress -- here the
 * component's progress function -- until the completion callback runs.
 * ------------------------------------------------------------------------- */
static mca_btl_base_module_t g_btl;
static int (*g_btl_progress)(void);
static int g_btl_ready;

/* The stand-in's own host single-copy RDMA (vader's CMA / xpmem path,
 * btl_sm_component.c:487, btl_sm_xpmem.c:70): a registration is {pid, base,
 * size}; get / put copy with process_vm_readv / _writev (memcpy within the
 * process) and call back at once, as vader's CMA get does.  g_host_btl_calls
 * counts what reached these slots. */
typedef struct { uint64_t magic; int64_t pid; uint64_t base, size; } mxh_host_reg_t;
#define MXH_HOST_REG_MAGIC 0x484f5354524547ull
static int g_host_btl_calls;
int mxh_btl_host_calls(void) { return g_host_btl_calls; }
static struct mca_btl_base_registration_handle_t *host_btl_register(mca_btl_base_module_t *btl,
                                                                    struct mca_btl_base_endpoint_t *ep, void *base,
                                                                    size_t size, uint32_t flags)
{
    (void)btl; (void)ep; (void)flags;
    g_host_btl_calls++;
    mxh_host_reg_t *r = calloc(1, sizeof *r);
    if (!r) return NULL;
    *r = (mxh_host_reg_t){MXH_HOST_REG_MAGIC, (int64_t)getpid(), (uint64_t)(uintptr_t)base, size};
    return (struct mca_btl_base_registration_handle_t *)r;
}
static int host_btl_deregister(mca_btl_base_module_t *btl, struct mca_btl_base_registration_handle_t *h)
{
    (void)btl;
    g_host_btl_calls++;
    free(h);
    return OPAL_SUCCESS;
}
static int host_btl_rdma(int get, mca_btl_base_module_t *btl, struct mca_btl_base_endpoint_t *ep, void *local,
                         uint64_t raddr, struct mca_btl_base_registration_handle_t *rh, size_t size,
                         mca_btl_base_rdma_completion_fn_t cb, void *ctx, void *data)
{
    const mxh_host_reg_t *r = (const mxh_host_reg_t *)rh;
    g_host_btl_calls++;
    if (!r || r->magic != MXH_HOST_REG_MAGIC || raddr < r->base || raddr + size > r->base + r->size)
        return OPAL_ERR_BAD_PARAM;
    if (r->pid == (int64_t)getpid()) {
        if (get) memcpy(local, (void *)(uintptr_t)raddr, size);
        else memcpy((void *)(uintptr_t)raddr, local, size);
    } else {
        struct iovec l = {local, size}, rv = {(void *)(uintptr_t)raddr, size};
        const ssize_t n = get ? process_vm_readv((pid_t)r->pid, &l, 1, &rv, 1, 0)
                              : process_vm_writev((pid_t)r->pid, &l, 1, &rv, 1, 0);
        if (n != (ssize_t)size) return OPAL_ERROR;
    }
    if (cb) cb(btl, ep, local, NULL, ctx, data, OPAL_SUCCESS);
    return OPAL_SUCCESS;
}
static int host_btl_get(mca_btl_base_module_t *btl, struct mca_btl_base_endpoint_t *ep, void *local, uint64_t raddr,
                        struct mca_btl_base_registration_handle_t *lh, struct mca_btl_base_registration_handle_t *rh,
                        size_t size, int flags, int order, mca_btl_base_rdma_completion_fn_t cb, void *ctx, void *data)
{
    (void)lh; (void)flags; (void)order;
    return host_btl_rdma(1, btl, ep, local, raddr, rh, size, cb, ctx, data);
}
static int host_btl_put(mca_btl_base_module_t *btl, struct mca_btl_base_endpoint_t *ep, void *local, uint64_t raddr,
                        struct mca_btl_base_registration_handle_t *lh, struct mca_btl_base_registration_handle_t *rh,
                        size_t size, int flags, int order, mca_btl_base_rdma_completion_fn_t cb, void *ctx, void *data)
{
    (void)lh; (void)flags; (void)order;
    return host_btl_rdma(0, btl, ep, local, raddr, rh, size, cb, ctx, data);
}

int mxh_btl_init(uint32_t *flags, size_t *handle_bytes)
{
    int (*install)(mca_btl_base_module_t *) =
        g_dl ? (int (*)(mca_btl_base_module_t *))dlsym(g_dl, "mca_btl_mi355x_install") : NULL;
    g_btl_progress = g_dl ? (int (*)(void))dlsym(g_dl, "mca_btl_mi355x_progress") : NULL;
    if (!install || !g_btl_progress) return -1;
    memset(&g_btl, 0, sizeof g_btl);
    g_btl.btl_eager_limit = 4096;                 /* vader's defaults (btl_vader_component.c) */
    g_btl.btl_rndv_eager_limit = 32768;
    g_btl.btl_max_send_size = 32768;
    g_btl.btl_exclusivity = 65536;                /* MCA_BTL_EXCLUSIVITY_HIGH */
    g_btl.btl_flags = 0x0001;                     /* MCA_BTL_FLAGS_SEND */
    g_btl.btl_register_mem = host_btl_register;   /* the host single-copy slots install keeps */
    g_btl.btl_deregister_mem = host_btl_deregister;
    g_btl.btl_get = host_btl_get;
    g_btl.btl_put = host_btl_put;
    g_btl.btl_registration_handle_size = sizeof(mxh_host_reg_t);
    if (install(&g_btl) != OPAL_SUCCESS) return -2;
    *flags = g_btl.btl_flags;
    *handle_bytes = g_btl.btl_registration_handle_size;
    g_btl_ready = 1;
    return 0;
}

/* the owner: register [base, base + size) and copy the handle bytes out */
int mxh_btl_register(void *base, size_t size, void *handle_out, void **reg)
{
    if (!g_btl_ready) return -1;
    struct mca_btl_base_registration_handle_t *h = g_btl.btl_register_mem(&g_btl, NULL, base, size, 0);
    if (!h) return -2;
    memcpy(handle_out, h, g_btl.btl_registration_handle_size);
    *reg = h;
    return 0;
}

int mxh_btl_deregister(void *reg)
{
    return g_btl_ready ? g_btl.btl_deregister_mem(&g_btl, reg) : -1;
}

typedef struct { volatile int done; int status; void *local; void *ctx; void *data; } mxh_rdma_cb_t;

static void rdma_cb(mca_btl_base_module_t *module, struct mca_btl_base_endpoint_t *ep, void *local_address,
                    struct mca_btl_base_registration_handle_t *local_handle, void *context, void *cbdata, int status)
{
    (void)module; (void)ep; (void)local_handle;
    mxh_rdma_cb_t *cb = (mxh_rdma_cb_t *)cbdata;
    cb->status = status;
    cb->local = local_address;
    cb->ctx = context;
    cb->done = 1;
}

/* the peer: get (1) or put (0) `size` bytes between `local` and the owner's
 * remote_addr, then progress until the callback; returns the callback's
 * status, or < -100 (-101 the slot refused, -102 no callback within 30 s,
 * -103 a callback with other arguments than those given) */
int mxh_btl_rdma(int get, void *local, uint64_t remote_addr, const void *remote_handle, size_t size, int ntimes)
{
    if (!g_btl_ready) return -100;
    mxh_rdma_cb_t cbs[16];
    if (ntimes < 1 || ntimes > 16) return -100;
    void *lreg = NULL;
    struct mca_btl_base_registration_handle_t *lh = g_btl.btl_register_mem(&g_btl, NULL, local, size ? size : 1, 0);
    lreg = lh;
    /* several operations in flight before any progress call */
    for (int k = 0; k < ntimes; k++) {
        memset(&cbs[k], 0, sizeof cbs[k]);
        mca_btl_base_module_get_fn_t fn = get ? g_btl.btl_get : g_btl.btl_put;
        const int rc = fn(&g_btl, NULL, local, remote_addr, lh, (struct mca_btl_base_registration_handle_t *)remote_handle,
                          size, 0, 255, rdma_cb, (void *)(intptr_t)(k + 1), &cbs[k]);
        if (rc != OPAL_SUCCESS) return -101;
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int st = 0;
    for (int k = 0; k < ntimes; k++) {
        while (!cbs[k].done) {
            g_btl_progress();
            clock_gettime(CLOCK_MONOTONIC, &t1);
            if ((t1.tv_sec - t0.tv_sec) > 30) return -102;
        }
        if (cbs[k].local != local || cbs[k].ctx != (void *)(intptr_t)(k + 1)) return -103;
        if (cbs[k].status != OPAL_SUCCESS) st = cbs[k].status;
    }
    if (lreg) g_btl.btl_deregister_mem(&g_btl, lreg);
    return st;
}

/* queue `n` gets without progress, then btl_flush: every callback has run */
int mxh_btl_flush_gets(void *local, uint64_t remote_addr, const void *remote_handle, size_t size, int n)
{
    if (!g_btl_ready || n < 1 || n > 16) return -100;
    mxh_rdma_cb_t cbs[16];
    for (int k = 0; k < n; k++) {
        memset(&cbs[k], 0, sizeof cbs[k]);
        if (g_btl.btl_get(&g_btl, NULL, (char *)local + (size_t)k * size, remote_addr + (uint64_t)k * size, NULL,
                          (struct mca_btl_base_registration_handle_t *)remote_handle, size, 0, 255, rdma_cb, NULL,
                          &cbs[k]) != OPAL_SUCCESS)
            return -101;
    }
    if (g_btl.btl_flush(&g_btl, NULL) != OPAL_SUCCESS) return -104;
    for (int k = 0; k < n; k++)
        if (!cbs[k].done || cbs[k].status != OPAL_SUCCESS) return -102;
    return 0;
}
