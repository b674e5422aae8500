/*
 * mx_host.c -- TEST HARNESS ("mini-host") for the mi355x op/coll
 * components.  See mx_host.h for what it restates from Open MPI.  It is
 * not part of the product: the real host is Open MPI itself
 * (INTEGRATION.md).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../mx_ompi_abi.h"
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

/* ---- host base coll module (stands in for tuned/basic on host buffers) ---- */
static int dtype_pack(struct ompi_datatype_t *d, int count, const void *user, void *packed);
static int dtype_unpack(struct ompi_datatype_t *d, int count, const void *packed, void *user);

static int base_allgather(const void *sbuf, int scount, struct ompi_datatype_t *sdt, void *rbuf, int rcount,
                          struct ompi_datatype_t *rdt, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    const size_t rb = (size_t)rcount * rdt->size, rext = (size_t)rcount * dtype_extent(rdt);
    char *tmp = malloc(rb * c->size + 1), *mine = malloc(rb + 1);
    int rc;
    if (!tmp || !mine) { free(tmp); free(mine); return OMPI_ERR_OUT_OF_RESOURCE; }
    if (sbuf == MPI_IN_PLACE) dtype_pack(rdt, rcount, (char *)rbuf + (size_t)c->rank * rext, mine);
    else dtype_pack(sdt, scount, sbuf, mine);
    rc = c->ag(mine, tmp, rb, c->ag_ctx);
    for (int p = 0; p < c->size && !rc; p++) dtype_unpack(rdt, rcount, tmp + (size_t)p * rb, (char *)rbuf + p * rext);
    free(tmp);
    free(mine);
    return rc ? OMPI_ERROR : OMPI_SUCCESS;
}

static int base_allreduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                          struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    size_t b = (size_t)count * dt->size;
    char *all = malloc(b * c->size + 1);
    (void)m;
    if (!all) return OMPI_ERR_OUT_OF_RESOURCE;
    if (c->ag(sbuf == MPI_IN_PLACE ? rbuf : sbuf, all, b, c->ag_ctx)) { free(all); return OMPI_ERROR; }
    /* basic linear order (coll_base_reduce.c:627-720): x_{n-1} op x_{n-2} ... */
    memcpy(rbuf, all + (size_t)(c->size - 1) * b, b);
    for (int i = c->size - 2; i >= 0; i--) op_reduce(op, all + (size_t)i * b, rbuf, count, dt);
    free(all);
    return OMPI_SUCCESS;
}

static int base_reduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, struct ompi_datatype_t *dt,
                               struct ompi_op_t *op, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    int total = 0, disp = 0;
    char *full;
    for (int i = 0; i < c->size; i++) { if (i < c->rank) disp += rcounts[i]; total += rcounts[i]; }
    full = malloc((size_t)total * dt->size + 1);
    if (!full) return OMPI_ERR_OUT_OF_RESOURCE;
    int rc = base_allreduce(sbuf == MPI_IN_PLACE ? rbuf : sbuf, full, total, dt, op, c, m);
    if (!rc) memcpy(rbuf, full + (size_t)disp * dt->size, (size_t)rcounts[c->rank] * dt->size);
    free(full);
    return rc;
}

static int base_bcast(void *buf, int count, struct ompi_datatype_t *dt, int root, struct ompi_communicator_t *c,
                      mca_coll_base_module_t *m)
{
    size_t b = (size_t)count * dt->size;
    char *all = malloc(b * c->size + 1), *mine = malloc(b + 1);
    (void)m;
    if (!all || !mine) { free(all); free(mine); return OMPI_ERR_OUT_OF_RESOURCE; }
    dtype_pack(dt, count, buf, mine);
    if (c->ag(mine, all, b, c->ag_ctx)) { free(all); free(mine); return OMPI_ERROR; }
    dtype_unpack(dt, count, all + (size_t)root * b, buf);
    free(all);
    free(mine);
    return OMPI_SUCCESS;
}

/* rooted reduce, basic linear order (coll_base_reduce.c:626-735) */
static int base_reduce(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                       int root, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    size_t b = (size_t)count * dt->size;
    char *all = malloc(b * c->size + 1);
    (void)m;
    if (!all) return OMPI_ERR_OUT_OF_RESOURCE;
    if (c->ag(sbuf == MPI_IN_PLACE ? rbuf : sbuf, all, b, c->ag_ctx)) { free(all); return OMPI_ERROR; }
    if (c->rank == root) {
        memcpy(rbuf, all + (size_t)(c->size - 1) * b, b);
        for (int i = c->size - 2; i >= 0; i--) op_reduce(op, all + (size_t)i * b, rbuf, count, dt);
    }
    free(all);
    return OMPI_SUCCESS;
}

static int base_reduce_scatter_block(const void *sbuf, void *rbuf, int rcount, struct ompi_datatype_t *dt,
                                     struct ompi_op_t *op, struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    int rcounts[256];
    if (c->size > 256) return OMPI_ERR_NOT_SUPPORTED;
    for (int i = 0; i < c->size; i++) rcounts[i] = rcount;
    return base_reduce_scatter(sbuf, rbuf, rcounts, dt, op, c, m);
}

/* linear scan / exscan (coll_base_scan.c:35-122, coll_base_exscan.c:35-107) */
static int base_scan_common(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                            struct ompi_communicator_t *c, int exclusive)
{
    size_t b = (size_t)count * dt->size;
    char *all = malloc(b * c->size + 1), *acc = malloc(b + 1), *tmp = malloc(b + 1);
    int rc = OMPI_SUCCESS;
    if (!all || !acc || !tmp) { rc = OMPI_ERR_OUT_OF_RESOURCE; goto out; }
    if (c->ag(sbuf == MPI_IN_PLACE ? rbuf : sbuf, all, b, c->ag_ctx)) { rc = OMPI_ERROR; goto out; }
    memcpy(acc, all, b);
    for (int r = 1; r <= (exclusive ? c->rank - 1 : c->rank); r++) {
        memcpy(tmp, all + (size_t)r * b, b);                 /* own data is the target */
        op_reduce(op, acc, tmp, count, dt);
        memcpy(acc, tmp, b);
    }
    if (!exclusive || c->rank > 0) memcpy(rbuf, acc, b);
out:
    free(all); free(acc); free(tmp);
    return rc;
}
static int base_scan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                     struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    return base_scan_common(sbuf, rbuf, count, dt, op, c, 0);
}
static int base_exscan(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                       struct ompi_communicator_t *c, mca_coll_base_module_t *m)
{
    (void)m;
    return base_scan_common(sbuf, rbuf, count, dt, op, c, 1);
}

/* coll/self-like reduce_local: mca_coll_base_reduce_local (coll_base_reduce.c:42-49) */
static int base_reduce_local(const void *in, void *inout, int count, struct ompi_datatype_t *dt, struct ompi_op_t *op,
                             mca_coll_base_module_t *m)
{
    (void)m;
    op_reduce(op, in, inout, count, dt);
    return OMPI_SUCCESS;
}

/* nonblocking / persistent stand-ins for coll/libnbc on host buffers: the
 * blocking base algorithm runs at post (or MPI_Start) time and the request
 * is complete at once */
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
    case S_IALLREDUCE: return base_allreduce(a->sbuf, a->rbuf, a->count, a->dt, a->op, a->c, NULL);
    case S_IREDUCE: return base_reduce(a->sbuf, a->rbuf, a->count, a->dt, a->op, a->root, a->c, NULL);
    case S_IREDUCE_SCATTER: return base_reduce_scatter(a->sbuf, a->rbuf, a->rcounts, a->dt, a->op, a->c, NULL);
    case S_IREDUCE_SCATTER_BLOCK: return base_reduce_scatter_block(a->sbuf, a->rbuf, a->count, a->dt, a->op, a->c, NULL);
    case S_ISCAN: return base_scan(a->sbuf, a->rbuf, a->count, a->dt, a->op, a->c, NULL);
    case S_IEXSCAN: return base_exscan(a->sbuf, a->rbuf, a->count, a->dt, a->op, a->c, NULL);
    case S_IALLGATHER: return base_allgather(a->sbuf, a->scount, a->dt, a->rbuf, a->count, a->rdt, a->c, NULL);
    case S_IBCAST: return base_bcast(a->rbuf, a->count, a->dt, a->root, a->c, NULL);
    }
    return OMPI_ERROR;
}
static int base_nb_start(struct ompi_request_t *r)
{
    request_activate(r);
    request_complete(r, base_nb_run(r->ctx));
    return OMPI_SUCCESS;
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
    if (a->rcounts) {
        h->rcounts = malloc(sizeof(int) * (size_t)a->c->size);
        if (!h->rcounts) { free(h); return OMPI_ERR_OUT_OF_RESOURCE; }
        memcpy(h->rcounts, a->rcounts, sizeof(int) * (size_t)a->c->size);
    }
    *request = request_create(persistent, base_nb_start, base_nb_free, h);
    if (!*request) { free(h->rcounts); free(h); return OMPI_ERR_OUT_OF_RESOURCE; }
    if (!persistent) request_complete(*request, base_nb_run(h));
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

static mca_coll_base_module_t g_base_coll;   /* static, never freed */
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

/* mca_coll_base_comm_select (coll_base_comm_select.c:108-309) */
static int comm_select(struct ompi_communicator_t *c, int is_self)
{
    mca_coll_base_module_t *base = is_self ? &g_self_coll : &g_base_coll;
    memset(c->fn, 0, sizeof c->fn);
    base->super.obj_class = &g_static_class;
    base->super.obj_reference_count = 1000000;
    if (is_self) {
        base->coll_reduce_local = base_reduce_local;
    } else {
        base->coll_allreduce = base_allreduce;
        base->coll_reduce_scatter = base_reduce_scatter;
        base->coll_allgather = base_allgather;
        base->coll_bcast = base_bcast;
        base->coll_reduce_local = base_reduce_local;
        base->coll_reduce = base_reduce;
        base->coll_reduce_scatter_block = base_reduce_scatter_block;
        base->coll_scan = base_scan;
        base->coll_exscan = base_exscan;
#define SET_BASE_NB(name) base->coll_##name = base_##name;
        SET_BASE_NB(iallreduce) SET_BASE_NB(ireduce) SET_BASE_NB(ireduce_scatter) SET_BASE_NB(ireduce_scatter_block)
        SET_BASE_NB(iscan) SET_BASE_NB(iexscan) SET_BASE_NB(iallgather) SET_BASE_NB(ibcast)
        SET_BASE_NB(allreduce_init) SET_BASE_NB(reduce_init) SET_BASE_NB(reduce_scatter_init)
        SET_BASE_NB(reduce_scatter_block_init) SET_BASE_NB(scan_init) SET_BASE_NB(exscan_init)
        SET_BASE_NB(allgather_init) SET_BASE_NB(bcast_init)
#undef SET_BASE_NB
    }
    /* lowest priority first: the base module (30 / 75) */
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
    COPY(base, is_self ? "self" : "base");
    if (g_coll_comp) {
        int prio = 0;
        mca_coll_base_module_t *m = g_coll_comp->collm_comm_query(c, &prio);
        const int base_prio = is_self ? 75 : 30;
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
    g_nprogress = 0;
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
