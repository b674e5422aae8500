/* TEST INFRASTRUCTURE: a flat C API over the reference's datatype engine
 * (built into oracle/_ref/libref_ddt.so) so tests and bench.py's
 * cpu_baseline can build MPI-style types and pack/unpack with the
 * reference's own convertor. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "opal_config.h"
#include "opal/datatype/opal_convertor.h"
#include "opal/datatype/opal_datatype.h"
#include "opal/datatype/opal_datatype_internal.h"
#include "opal/runtime/opal.h"

static int inited;
static void init(void) { if (!inited) { opal_init_util(NULL, NULL); inited = 1; } }

static const opal_datatype_t *basic(int id) { init(); return opal_datatype_basicDatatypes[id]; }

void *refddt_vector(int count, int blen, int stride, int basic_id)
{
    const opal_datatype_t *old = basic(basic_id);
    const ptrdiff_t ext = old->ub - old->lb;
    opal_datatype_t *t = opal_datatype_create(8), *b = NULL;
    if (blen > 1) { b = opal_datatype_create(4); opal_datatype_add(b, old, blen, 0, ext); }
    opal_datatype_add(t, b ? b : old, count, 0, stride * ext);
    if (b) OBJ_RELEASE(b);
    opal_datatype_commit(t);
    return t;
}

void *refddt_indexed(int n, const int *blens, const int *disps, int basic_id)
{
    const opal_datatype_t *old = basic(basic_id);
    const ptrdiff_t ext = old->ub - old->lb;
    opal_datatype_t *t = opal_datatype_create(2 * n + 2);
    for (int i = 0; i < n; i++) opal_datatype_add(t, old, blens[i], disps[i] * ext, ext);
    opal_datatype_commit(t);
    return t;
}

/* {char, double[3], int} resized to `extent` */
void *refddt_struct_cdi(int extent)
{
    init();
    opal_datatype_t *s = opal_datatype_create(8), *r = opal_datatype_create(8);
    opal_datatype_add(s, &opal_datatype_int1, 1, 0, 1);
    opal_datatype_add(s, &opal_datatype_float8, 3, 8, 8);
    opal_datatype_add(s, &opal_datatype_int4, 1, 32, 4);
    opal_datatype_commit(s);
    opal_datatype_clone(s, r);
    opal_datatype_resize(r, 0, extent);
    opal_datatype_commit(r);
    OBJ_RELEASE(s);
    return r;
}

/* committed description + geometry */
int refddt_info(void *dtv, int64_t *size, int64_t *lb, int64_t *ub, int64_t *true_lb, int64_t *true_ub,
                const void **desc, int *nrec)
{
    opal_datatype_t *dt = dtv;
    const dt_type_desc_t *d = (dt->opt_desc.desc && dt->opt_desc.used) ? &dt->opt_desc : &dt->desc;
    *size = (int64_t)dt->size; *lb = dt->lb; *ub = dt->ub; *true_lb = dt->true_lb; *true_ub = dt->true_ub;
    *desc = d->desc;
    *nrec = (int)d->used + 1;
    return 0;
}

int refddt_pack(void *dtv, int count, const void *user, void *packed, int unpack)
{
    opal_datatype_t *dt = dtv;
    opal_convertor_t *c = opal_convertor_create(opal_local_arch, 0);
    struct iovec iov = {packed, dt->size * (size_t)count};
    uint32_t n = 1;
    size_t max = iov.iov_len;
    int rc = unpack ? opal_convertor_prepare_for_recv(c, dt, count, user)
                    : opal_convertor_prepare_for_send(c, dt, count, user);
    if (rc) return -1;
    rc = unpack ? opal_convertor_unpack(c, &iov, &n, &max) : opal_convertor_pack(c, &iov, &n, &max);
    OBJ_RELEASE(c);
    return rc < 0 ? -2 : 0;
}

void refddt_free(void *dtv) { opal_datatype_t *dt = dtv; OBJ_RELEASE(dt); }
