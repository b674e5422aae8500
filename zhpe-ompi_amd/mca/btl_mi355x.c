/*
 * btl_mi355x.c -- GPU RDMA for a shared-memory BTL on MI355X: the get / put /
 * register_mem / deregister_mem / flush slots of mca_btl_base_module_t
 * (opal/mca/btl/btl.h:1189-1261) for device buffers, and the progress
 * function that completes them.
 *
 * The reference's CUDA build gives btl/smcuda these roles: its component
 * init installs mca_btl_smcuda_get_cuda as the module's btl_get
 * (btl_smcuda_component.c:936), btl_register_mem exports a CUDA IPC handle
 * of the user buffer (btl_smcuda.c:1030-1062), and the get opens the peer's
 * handle through the rcache, copies with cuMemcpyAsync and completes the
 * descriptor from the component's progress (btl_smcuda.c:1077-1180,
 * common_cuda.c progress_one_cuda_dtoh_event).  ob1 then runs its RGET
 * protocol on device buffers unchanged (pml_ob1_recvreq.c: the receiver
 * calls btl_get with the sender's registration handle from the RGET header).
 *
 * Here mca_btl_mi355x_install(btl) sets the same slots on a host
 * shared-memory BTL module (vader or smcuda):
 *   btl_register_mem   the mx_rdma_handle_t of the allocation holding the
 *                      range (include/mx_rdma.h), btl_registration_handle_size
 *                      = its size (it travels in the PML header);
 *   btl_get / btl_put  mx_rdma_get / mx_rdma_put: the peer allocation mapped
 *                      once, one copy kernel; OPAL_SUCCESS = queued, the
 *                      completion callback runs from progress;
 *   btl_flush          every queued operation completed and called back;
 * and the flags MCA_BTL_FLAGS_GET | PUT | CUDA_GET | CUDA_PUT (ob1's test
 * for device-capable RDMA, pml_ob1.c).  mca_btl_mi355x_progress is what the
 * maintainer registers with opal_progress_register (int (*)(void), returns
 * the completions it made).
 *
 * Host memory stays the BTL's own (vader's CMA / xpmem / knem single copy,
 * btl_sm_component.c:487, btl_sm_xpmem.c:70): install keeps the module's
 * original slots and handle size, register_mem hands host ranges to the
 * original registration and tags every handle with where its memory is --
 * the tag travels in the PML header with the handle bytes -- and get / put /
 * deregister send host handles back to the original slots with the
 * original's own handle bytes.
 *
 * Return codes are OPAL's: OPAL_ERR_OUT_OF_RESOURCE tells the PML to try
 * again later (a stale mapping of a re-made peer allocation is still
 * waiting for its deferred close, include/mx_coll.h mx_release_pending).
 */
#include <pthread.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#include "mx_btl_abi.h"
#include "mx_kernels.h"
#include "mx_rdma.h"

/* What register_mem hands out.  The first btl_registration_handle_size
 * bytes are the public part the PML copies into its header: the location tag
 * and the payload (an mx_rdma_handle_t, or the original BTL's handle bytes).
 * `orig` (the original's registration, for its deregister) is private. */
enum { MX_REG_DEVICE = 0x4d58444556494345ull, MX_REG_HOST = 0x4d58484f53545f5full };
typedef struct mx_btl_reg {
    uint64_t kind;
    union {
        mx_rdma_handle_t h;
        unsigned char bytes[1];
    } u;
} mx_btl_reg_t;
#define MX_REG_PAYLOAD offsetof(mx_btl_reg_t, u)

/* the slots a module had before install (one entry per installed module) */
typedef struct {
    mca_btl_base_module_t *btl;
    mca_btl_base_module_get_fn_t get, put;
    mca_btl_base_module_register_mem_fn_t reg;
    mca_btl_base_module_deregister_mem_fn_t dereg;
    mca_btl_base_module_flush_fn_t flush;
    size_t handle_size;                  /* the original's public handle bytes */
    size_t public_size;                  /* ours: tag + max(original, mx handle) */
} mx_btl_orig_t;
#define MX_BTL_MAX_MODULES 16
static mx_btl_orig_t g_orig[MX_BTL_MAX_MODULES];
static int g_norig;

typedef struct mx_btl_pending {
    mx_rdma_op_t *op;
    mca_btl_base_module_t *btl;
    struct mca_btl_base_endpoint_t *ep;
    void *local_address;
    struct mca_btl_base_registration_handle_t *local_handle;
    mca_btl_base_rdma_completion_fn_t cbfunc;
    void *cbcontext, *cbdata;
} mx_btl_pending_t;

#define MX_BTL_MAX_PENDING 1024

static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static mx_btl_pending_t g_pending[MX_BTL_MAX_PENDING];
static int g_npending;

static int opal_rc(int mx)
{
    switch (mx) {
    case MX_SUCCESS: return OPAL_SUCCESS;
    case MX_ERR_ARG: return OPAL_ERR_BAD_PARAM;
    case MX_ERR_STATE:
    case MX_ERR_NOMEM: return OPAL_ERR_OUT_OF_RESOURCE;
    default: return OPAL_ERROR;
    }
}

static const mx_btl_orig_t *orig_of(const mca_btl_base_module_t *btl)
{
    for (int i = 0; i < g_norig; i++)
        if (g_orig[i].btl == btl) return &g_orig[i];
    return NULL;
}

static size_t public_size(const mx_btl_orig_t *o)
{
    return o ? o->public_size : MX_REG_PAYLOAD + sizeof(mx_rdma_handle_t);
}

/* the private pointer to the original's registration, after the public part */
static struct mca_btl_base_registration_handle_t **orig_slot(const mx_btl_orig_t *o, mx_btl_reg_t *r)
{
    return (struct mca_btl_base_registration_handle_t **)((char *)r + ((public_size(o) + 7) & ~(size_t)7));
}

struct mca_btl_base_registration_handle_t *mca_btl_mi355x_register_mem(mca_btl_base_module_t *btl,
                                                                       struct mca_btl_base_endpoint_t *endpoint,
                                                                       void *base, size_t size, uint32_t flags)
{
    const mx_btl_orig_t *o = orig_of(btl);
    const size_t alloc = ((public_size(o) + 7) & ~(size_t)7) + sizeof(void *);
    if (mx_is_device_ptr(base) != 1) {   /* host memory: the BTL's own registration, tagged */
        if (!o || !o->reg) return NULL;
        struct mca_btl_base_registration_handle_t *oh = o->reg(btl, endpoint, base, size, flags);
        if (!oh) return NULL;
        mx_btl_reg_t *r = (mx_btl_reg_t *)calloc(1, alloc);
        if (!r) {
            if (o->dereg) o->dereg(btl, oh);
            return NULL;
        }
        r->kind = MX_REG_HOST;
        memcpy(r->u.bytes, oh, o->handle_size);
        *orig_slot(o, r) = oh;
        return (struct mca_btl_base_registration_handle_t *)r;
    }
    mx_btl_reg_t *r = (mx_btl_reg_t *)calloc(1, alloc);
    if (!r) return NULL;
    r->kind = MX_REG_DEVICE;
    if (mx_rdma_register(base, size, &r->u.h) != MX_SUCCESS) {
        free(r);
        return NULL;
    }
    return (struct mca_btl_base_registration_handle_t *)r;
}

int mca_btl_mi355x_deregister_mem(mca_btl_base_module_t *btl, struct mca_btl_base_registration_handle_t *handle)
{
    if (!handle) return OPAL_SUCCESS;
    mx_btl_reg_t *r = (mx_btl_reg_t *)handle;
    int rc = OPAL_SUCCESS;
    if (r->kind == MX_REG_HOST) {
        const mx_btl_orig_t *o = orig_of(btl);
        struct mca_btl_base_registration_handle_t *oh = *orig_slot(o, r);
        if (o && o->dereg && oh) rc = o->dereg(btl, oh);
    }
    free(r);                             /* device exports stay cached by the library (one per allocation) */
    return rc;
}

static int queue(mx_rdma_op_t *op, mca_btl_base_module_t *btl, struct mca_btl_base_endpoint_t *ep,
                 void *local_address, struct mca_btl_base_registration_handle_t *local_handle,
                 mca_btl_base_rdma_completion_fn_t cbfunc, void *cbcontext, void *cbdata)
{
    pthread_mutex_lock(&g_mu);
    if (g_npending == MX_BTL_MAX_PENDING) {
        pthread_mutex_unlock(&g_mu);
        mx_rdma_wait(op);                /* full: complete this one in place */
        mx_rdma_op_free(op);
        if (cbfunc) cbfunc(btl, ep, local_address, local_handle, cbcontext, cbdata, OPAL_SUCCESS);
        return OPAL_SUCCESS;
    }
    g_pending[g_npending++] = (mx_btl_pending_t){op, btl, ep, local_address, local_handle, cbfunc, cbcontext, cbdata};
    pthread_mutex_unlock(&g_mu);
    return OPAL_SUCCESS;
}

static int rdma(int get, mca_btl_base_module_t *btl, struct mca_btl_base_endpoint_t *ep, void *local_address,
                uint64_t remote_address, struct mca_btl_base_registration_handle_t *local_handle,
                struct mca_btl_base_registration_handle_t *remote_handle, size_t size, int flags, int order,
                mca_btl_base_rdma_completion_fn_t cbfunc, void *cbcontext, void *cbdata)
{
    if (!local_address) return OPAL_ERR_BAD_PARAM;
    const mx_btl_reg_t *rr = (const mx_btl_reg_t *)remote_handle;
    if (!rr || rr->kind != MX_REG_DEVICE) {
        /* host memory (or no registration): the BTL's own single-copy path,
         * with the original's handle bytes on both sides */
        const mx_btl_orig_t *o = orig_of(btl);
        mca_btl_base_module_get_fn_t fn = o ? (get ? o->get : o->put) : NULL;
        if (!fn) return OPAL_ERR_NOT_AVAILABLE;
        const mx_btl_reg_t *lr = (const mx_btl_reg_t *)local_handle;
        struct mca_btl_base_registration_handle_t *lo =
            (lr && lr->kind == MX_REG_HOST) ? *orig_slot(o, (mx_btl_reg_t *)lr) : NULL;
        struct mca_btl_base_registration_handle_t *ro =
            rr ? (struct mca_btl_base_registration_handle_t *)(uintptr_t)rr->u.bytes : NULL;
        return fn(btl, ep, local_address, remote_address, lo, ro, size, flags, order, cbfunc, cbcontext, cbdata);
    }
    const mx_rdma_handle_t *rh = &rr->u.h;
    mx_rdma_op_t *op = NULL;
    const int rc = get ? mx_rdma_get(local_address, rh, remote_address, size, NULL, &op)
                       : mx_rdma_put(local_address, rh, remote_address, size, NULL, &op);
    if (rc != MX_SUCCESS) return opal_rc(rc);
    return queue(op, btl, ep, local_address, local_handle, cbfunc, cbcontext, cbdata);
}

int mca_btl_mi355x_get(mca_btl_base_module_t *btl, struct mca_btl_base_endpoint_t *ep, void *local_address,
                       uint64_t remote_address, struct mca_btl_base_registration_handle_t *local_handle,
                       struct mca_btl_base_registration_handle_t *remote_handle, size_t size, int flags, int order,
                       mca_btl_base_rdma_completion_fn_t cbfunc, void *cbcontext, void *cbdata)
{
    return rdma(1, btl, ep, local_address, remote_address, local_handle, remote_handle, size, flags, order, cbfunc,
                cbcontext, cbdata);
}

int mca_btl_mi355x_put(mca_btl_base_module_t *btl, struct mca_btl_base_endpoint_t *ep, void *local_address,
                       uint64_t remote_address, struct mca_btl_base_registration_handle_t *local_handle,
                       struct mca_btl_base_registration_handle_t *remote_handle, size_t size, int flags, int order,
                       mca_btl_base_rdma_completion_fn_t cbfunc, void *cbcontext, void *cbdata)
{
    return rdma(0, btl, ep, local_address, remote_address, local_handle, remote_handle, size, flags, order, cbfunc,
                cbcontext, cbdata);
}

/* complete what has finished (all of it with `wait`), callbacks outside the lock */
static int complete(int wait)
{
    mx_btl_pending_t done[64];
    int total = 0;
    for (;;) {
        int n = 0;
        pthread_mutex_lock(&g_mu);
        for (int i = 0; i < g_npending && n < 64;) {
            if (wait) mx_rdma_wait(g_pending[i].op);
            if (mx_rdma_test(g_pending[i].op) != 0) {
                done[n++] = g_pending[i];
                g_pending[i] = g_pending[--g_npending];
                continue;
            }
            i++;
        }
        pthread_mutex_unlock(&g_mu);
        for (int i = 0; i < n; i++) {
            const int st = mx_rdma_test(done[i].op) == 1 ? OPAL_SUCCESS : OPAL_ERROR;
            mx_rdma_op_free(done[i].op);
            if (done[i].cbfunc)
                done[i].cbfunc(done[i].btl, done[i].ep, done[i].local_address, done[i].local_handle,
                               done[i].cbcontext, done[i].cbdata, st);
        }
        total += n;
        if (n < 64) return total;
    }
}

int mca_btl_mi355x_progress(void)
{
    return complete(0);
}

int mca_btl_mi355x_flush(mca_btl_base_module_t *btl, struct mca_btl_base_endpoint_t *ep)
{
    complete(1);
    const mx_btl_orig_t *o = orig_of(btl);
    return (o && o->flush) ? o->flush(btl, ep) : OPAL_SUCCESS;
}

/* the smcuda pattern (btl_smcuda_component.c:936): device RDMA slots on a
 * host shared-memory BTL module; the maintainer also registers
 * mca_btl_mi355x_progress with opal_progress_register */
int mca_btl_mi355x_install(mca_btl_base_module_t *btl)
{
    if (!btl) return OPAL_ERR_BAD_PARAM;
    pthread_mutex_lock(&g_mu);
    mx_btl_orig_t *o = (mx_btl_orig_t *)orig_of(btl);
    if (!o) {
        if (g_norig == MX_BTL_MAX_MODULES) {
            pthread_mutex_unlock(&g_mu);
            return OPAL_ERR_OUT_OF_RESOURCE;
        }
        o = &g_orig[g_norig++];
    }
    if (btl->btl_get != mca_btl_mi355x_get) {   /* installing twice keeps the first originals */
        o->btl = btl;
        o->get = btl->btl_get;
        o->put = btl->btl_put;
        o->reg = btl->btl_register_mem;
        o->dereg = btl->btl_deregister_mem;
        o->flush = btl->btl_flush;
        o->handle_size = o->reg ? btl->btl_registration_handle_size : 0;
        const size_t payload = o->handle_size > sizeof(mx_rdma_handle_t) ? o->handle_size : sizeof(mx_rdma_handle_t);
        o->public_size = MX_REG_PAYLOAD + payload;
    }
    pthread_mutex_unlock(&g_mu);
    btl->btl_get = mca_btl_mi355x_get;
    btl->btl_put = mca_btl_mi355x_put;
    btl->btl_register_mem = mca_btl_mi355x_register_mem;
    btl->btl_deregister_mem = mca_btl_mi355x_deregister_mem;
    btl->btl_flush = mca_btl_mi355x_flush;
    btl->btl_registration_handle_size = o->public_size;
    btl->btl_flags |= MCA_BTL_FLAGS_GET | MCA_BTL_FLAGS_PUT | MCA_BTL_FLAGS_CUDA_GET | MCA_BTL_FLAGS_CUDA_PUT |
                      MCA_BTL_FLAGS_RDMA_FLUSH;
    btl->btl_get_limit = btl->btl_put_limit = SIZE_MAX;
    btl->btl_get_alignment = btl->btl_put_alignment = 0;
    return OPAL_SUCCESS;
}

int mca_btl_mi355x_pending(void)
{
    pthread_mutex_lock(&g_mu);
    const int n = g_npending;
    pthread_mutex_unlock(&g_mu);
    return n;
}
