/*
 * convertor_mi355x.c -- the opal_convertor hook for device user buffers:
 * pack / unpack of derived datatypes on the GPU.
 *
 * Where it plugs in.  opal_convertor_prepare_for_send / _for_recv
 * (opal/datatype/opal_convertor.c:565-660) pick the convertor's loop,
 * `fAdvance`, after OPAL_CONVERTOR_PREPARE has filled the convertor
 * (pDesc, use_desc = the committed opt_desc, count, pBaseBuf, local_size):
 * opal_generic_simple_pack (:649) / opal_generic_simple_unpack (:601) for a
 * homogeneous non-contiguous type.  The CUDA build keeps those loops and
 * turns each contiguous block into a cuMemcpy (MEMCPY_CUDA,
 * opal_datatype_cuda.c:121-140; the function table of
 * opal_datatype_cuda.h:16-22).  Here the maintainer adds one call after
 * that choice:
 *
 *     mca_convertor_mi355x_prepare(convertor);
 *
 * which, for a device user buffer, replaces fAdvance with
 * mca_convertor_mi355x_pack / _unpack: one mx_pack / mx_unpack launch per
 * iovec (csrc/mx_convertor.hip, the kernels of DESIGN 4) instead of one
 * copy per block.  The packed stream position is `bConverted`, so a BTL that
 * fragments (opal_convertor_set_position, any byte) resumes where it left;
 * a fragment ends complete on return (the caller sends or reads it at
 * once), as after the reference's generic loop.
 *
 * The contract restated from opal_generic_simple_pack_function
 * (opal_datatype_pack.c:235-370) and opal_convertor_pack (opal_convertor.c:
 * 218-274): iovecs are filled in order up to their lengths; *out_size = the
 * iovecs used, *max_data = the bytes moved, bConverted advances by them;
 * at the end of the message CONVERTOR_COMPLETED is set and 1 returned, else
 * 0; -1 on an error.  Packed buffers may be device or host memory (host
 * fragments are staged through a device bounce buffer).
 *
 * Heterogeneous conversion, checksums and the NO_OP contiguous path stay on
 * the reference's loops (the hook declines them).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "mx_opal_convertor_abi.h"
#include "mx_convertor.h"
#include "mx_kernels.h"

#define MX_CONV_CACHE 64
#define MX_REC_BYTES 32                   /* sizeof(dt_elem_desc_t) */

/* Cached device handles, keyed by the datatype AND a copy of its committed
 * records, size and bounds: a datatype freed and re-created per iteration
 * (MPI_Type_vector with a new stride, say) often comes back at the same
 * addresses with the same record count.  g_mu is held from the lookup to the
 * end of the fragment's kernels, so an eviction never destroys a handle in
 * use. */
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static struct {
    const void *dt, *desc;
    size_t used, size;
    ptrdiff_t lb, ub;
    void *recs;
    mx_ddt_t *h;
    uint64_t tick;
} g_cache[MX_CONV_CACHE];
static uint64_t g_tick;
static void *g_stream;                    /* ordered with the legacy default stream */
static void *g_bounce;                    /* device staging for host fragments */
static size_t g_bounce_bytes;

/* the device representation of a committed datatype: its opt_desc records
 * verbatim (opal_datatype.h:126), built once per (datatype, description);
 * the caller holds g_mu */
static mx_ddt_t *ddt_for_locked(const opal_datatype_t *dt, const dt_type_desc_t *d)
{
    const size_t rb = ((size_t)d->used + 1) * MX_REC_BYTES;
    int victim = 0;
    for (int i = 0; i < MX_CONV_CACHE; i++) {
        if (g_cache[i].h && g_cache[i].dt == dt && g_cache[i].desc == d->desc && g_cache[i].used == d->used &&
            g_cache[i].size == dt->size && g_cache[i].lb == dt->lb && g_cache[i].ub == dt->ub &&
            !memcmp(g_cache[i].recs, d->desc, rb)) {
            g_cache[i].tick = ++g_tick;
            return g_cache[i].h;
        }
        if (g_cache[i].tick < g_cache[victim].tick) victim = i;
    }
    void *recs = malloc(rb);
    mx_ddt_t *h = NULL;
    if (!recs) return NULL;
    memcpy(recs, d->desc, rb);
    if (mx_ddt_create(d->desc, d->used + 1, NULL, dt->size, dt->lb, dt->ub, &h) != MX_SUCCESS) {
        free(recs);
        return NULL;
    }
    if (g_cache[victim].h) mx_ddt_destroy(g_cache[victim].h);
    free(g_cache[victim].recs);
    g_cache[victim].dt = dt;
    g_cache[victim].desc = d->desc;
    g_cache[victim].used = d->used;
    g_cache[victim].size = dt->size;
    g_cache[victim].lb = dt->lb;
    g_cache[victim].ub = dt->ub;
    g_cache[victim].recs = recs;
    g_cache[victim].h = h;
    g_cache[victim].tick = ++g_tick;
    if (!g_stream && mx_stream_create_ordered(&g_stream) != MX_SUCCESS) g_stream = NULL;
    return h;
}

/* a device buffer of at least `bytes` for host fragments (grown, kept) */
static void *bounce(size_t bytes)
{
    if (g_bounce_bytes >= bytes) return g_bounce;
    if (g_bounce) mx_free(g_bounce);
    g_bounce = NULL;
    g_bounce_bytes = 0;
    if (mx_alloc(bytes, &g_bounce) != MX_SUCCESS) return NULL;
    g_bounce_bytes = bytes;
    return g_bounce;
}

static int32_t advance(opal_convertor_t *c, struct iovec *iov, uint32_t *out_size, size_t *max_data, int pack)
{
    if (c->flags & CONVERTOR_COMPLETED) {   /* OPAL_CONVERTOR_SET_STATUS_BEFORE_PACK_UNPACK */
        iov[0].iov_len = 0;
        *out_size = 0;
        *max_data = 0;
        return 1;
    }
    pthread_mutex_lock(&g_mu);              /* the handle and the one bounce buffer */
    mx_ddt_t *h = ddt_for_locked(c->pDesc, c->use_desc);
    if (!h || !g_stream) {
        pthread_mutex_unlock(&g_mu);
        return -1;
    }
    size_t done = 0;
    uint32_t i = 0;
    int rc = MX_SUCCESS;
    for (; i < *out_size && c->bConverted + done < c->local_size && rc == MX_SUCCESS; i++) {
        size_t len = iov[i].iov_len;
        if (len > c->local_size - (c->bConverted + done)) len = c->local_size - (c->bConverted + done);
        if (!len || !iov[i].iov_base) {
            iov[i].iov_len = 0;
            continue;
        }
        const size_t off = c->bConverted + done;
        char *frag = (char *)iov[i].iov_base;
        if (mx_is_device_ptr(frag)) {
            rc = pack ? mx_pack(h, c->count, c->pBaseBuf, frag, off, len, g_stream)
                      : mx_unpack(h, c->count, c->pBaseBuf, frag, off, len, g_stream);
        } else {
            char *b = bounce(len);
            if (!b) { rc = MX_ERR_NOMEM; break; }
            if (pack) {
                rc = mx_pack(h, c->count, c->pBaseBuf, b, off, len, g_stream);
                if (rc == MX_SUCCESS) rc = mx_memcpy(frag, b, len, g_stream);
            } else {
                rc = mx_memcpy(b, frag, len, g_stream);
                if (rc == MX_SUCCESS) rc = mx_unpack(h, c->count, c->pBaseBuf, b, off, len, g_stream);
            }
            /* the bounce buffer is reused by the next fragment */
            if (rc == MX_SUCCESS) rc = mx_stream_sync(g_stream);
        }
        iov[i].iov_len = len;
        done += len;
    }
    if (rc == MX_SUCCESS) rc = mx_stream_sync_fast(g_stream);   /* fragments complete on return */
    pthread_mutex_unlock(&g_mu);
    if (rc != MX_SUCCESS) return -1;
    *max_data = done;
    *out_size = i;
    c->bConverted += done;
    if (c->bConverted == c->local_size) {
        c->flags |= CONVERTOR_COMPLETED;
        return 1;
    }
    return 0;
}

int32_t mca_convertor_mi355x_pack(opal_convertor_t *c, struct iovec *iov, uint32_t *out_size, size_t *max_data)
{
    return advance(c, iov, out_size, max_data, 1);
}

int32_t mca_convertor_mi355x_unpack(opal_convertor_t *c, struct iovec *iov, uint32_t *out_size, size_t *max_data)
{
    return advance(c, iov, out_size, max_data, 0);
}

/* 1: fAdvance now runs on the GPU; 0: the reference's loop stays */
int mca_convertor_mi355x_prepare(opal_convertor_t *c)
{
    if (!c || !c->pDesc || !c->use_desc || !c->count || !c->local_size) return 0;
    if ((c->flags & (CONVERTOR_NO_OP | CONVERTOR_WITH_CHECKSUM)) || !(c->flags & CONVERTOR_HOMOGENEOUS)) return 0;
    if (!(c->flags & (CONVERTOR_SEND | CONVERTOR_RECV))) return 0;
    if (!mx_is_device_ptr(c->pBaseBuf + c->pDesc->true_lb)) return 0;
    pthread_mutex_lock(&g_mu);
    const int ok = ddt_for_locked(c->pDesc, c->use_desc) && g_stream;
    pthread_mutex_unlock(&g_mu);
    if (!ok) return 0;
    c->fAdvance = (c->flags & CONVERTOR_SEND) ? mca_convertor_mi355x_pack : mca_convertor_mi355x_unpack;
    return 1;
}
