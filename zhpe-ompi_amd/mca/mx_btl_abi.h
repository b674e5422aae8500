/*
 * mx_btl_abi.h -- layout mirror of the BTL module interface the mi355x GPU
 * RDMA extension installs into (mca/btl_mi355x.c).
 *
 * Mirrored (reference = HewlettPackard/zhpe-ompi, Open MPI 5.0.0a1, x86-64,
 * BTL_VERSION 310, OPAL_CUDA_SUPPORT = OPAL_CUDA_GDR_SUPPORT = 0 -- an MI355X
 * build has no CUDA):
 *   mca_btl_base_module_t                  opal/mca/btl/btl.h:1189-1261
 *   mca_btl_base_module_get_fn_t           :1017-1020
 *   mca_btl_base_module_put_fn_t           :980-984
 *   mca_btl_base_module_register_mem_fn_t  :861-863
 *   mca_btl_base_module_deregister_mem_fn_t :881-882
 *   mca_btl_base_module_flush_fn_t         :1187
 *   mca_btl_base_rdma_completion_fn_t      :401-408
 *   MCA_BTL_FLAGS_*                        :197-251
 *   OPAL_SUCCESS / OPAL_ERR_*              opal/include/opal/constants.h:29-46
 * btl.h needs configure-generated headers (the threads framework's
 * MCA_threads_mutex_base_include_HEADER), so tests/test_abi_layout.py
 * derives the reference offsets from the struct's text (every member a
 * size_t, uint32_t, pointer or the 256-byte padding) and compares them with
 * this mirror.
 */
#ifndef MX_BTL_ABI_H
#define MX_BTL_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct mca_btl_base_module_t;
struct mca_btl_base_endpoint_t;
struct mca_btl_base_registration_handle_t;
struct mca_btl_base_component_2_0_0_t;
struct mca_mpool_base_module_t;

typedef void (*mca_btl_base_rdma_completion_fn_t)(struct mca_btl_base_module_t *module,
                                                  struct mca_btl_base_endpoint_t *endpoint, void *local_address,
                                                  struct mca_btl_base_registration_handle_t *local_handle,
                                                  void *context, void *cbdata, int status);
typedef int (*mca_btl_base_module_get_fn_t)(struct mca_btl_base_module_t *btl, struct mca_btl_base_endpoint_t *endpoint,
                                            void *local_address, uint64_t remote_address,
                                            struct mca_btl_base_registration_handle_t *local_handle,
                                            struct mca_btl_base_registration_handle_t *remote_handle, size_t size,
                                            int flags, int order, mca_btl_base_rdma_completion_fn_t cbfunc,
                                            void *cbcontext, void *cbdata);
typedef mca_btl_base_module_get_fn_t mca_btl_base_module_put_fn_t;
typedef struct mca_btl_base_registration_handle_t *(*mca_btl_base_module_register_mem_fn_t)(
    struct mca_btl_base_module_t *btl, struct mca_btl_base_endpoint_t *endpoint, void *base, size_t size,
    uint32_t flags);
typedef int (*mca_btl_base_module_deregister_mem_fn_t)(struct mca_btl_base_module_t *btl,
                                                       struct mca_btl_base_registration_handle_t *handle);
typedef int (*mca_btl_base_module_flush_fn_t)(struct mca_btl_base_module_t *btl,
                                              struct mca_btl_base_endpoint_t *endpoint);
typedef void (*mx_btl_fn_t)(void);       /* slots this extension leaves alone */

typedef struct mca_btl_base_module_t {
    struct mca_btl_base_component_2_0_0_t *btl_component;
    size_t btl_eager_limit;
    size_t btl_rndv_eager_limit;
    size_t btl_max_send_size;
    size_t btl_rdma_pipeline_send_length;
    size_t btl_rdma_pipeline_frag_size;
    size_t btl_min_rdma_pipeline_size;
    uint32_t btl_exclusivity;
    uint32_t btl_latency;
    uint32_t btl_bandwidth;
    uint32_t btl_flags;
    uint32_t btl_atomic_flags;
    size_t btl_registration_handle_size;
    size_t btl_get_limit;
    size_t btl_get_alignment;
    size_t btl_put_limit;
    size_t btl_put_alignment;
    size_t btl_get_local_registration_threshold;
    size_t btl_put_local_registration_threshold;
    mx_btl_fn_t btl_add_procs;
    mx_btl_fn_t btl_del_procs;
    mx_btl_fn_t btl_register;
    mx_btl_fn_t btl_finalize;
    mx_btl_fn_t btl_alloc;
    mx_btl_fn_t btl_free;
    mx_btl_fn_t btl_prepare_src;
    mx_btl_fn_t btl_send;
    mx_btl_fn_t btl_sendi;
    mca_btl_base_module_put_fn_t btl_put;
    mca_btl_base_module_get_fn_t btl_get;
    mx_btl_fn_t btl_dump;
    mx_btl_fn_t btl_atomic_op;
    mx_btl_fn_t btl_atomic_fop;
    mx_btl_fn_t btl_atomic_cswap;
    mca_btl_base_module_register_mem_fn_t btl_register_mem;
    mca_btl_base_module_deregister_mem_fn_t btl_deregister_mem;
    struct mca_mpool_base_module_t *btl_mpool;
    mx_btl_fn_t btl_register_error;
    mx_btl_fn_t btl_ft_event;
    mca_btl_base_module_flush_fn_t btl_flush;
    unsigned char padding[256];
} mca_btl_base_module_t;

#define MCA_BTL_FLAGS_PUT        0x0002
#define MCA_BTL_FLAGS_GET        0x0004
#define MCA_BTL_FLAGS_CUDA_PUT   0x0400
#define MCA_BTL_FLAGS_CUDA_GET   0x0800
#define MCA_BTL_FLAGS_RDMA_FLUSH 0x80000

#define OPAL_SUCCESS              0
#define OPAL_ERROR                (-1)
#define OPAL_ERR_OUT_OF_RESOURCE  (-2)
#define OPAL_ERR_BAD_PARAM        (-5)
#define OPAL_ERR_NOT_AVAILABLE    (-16)

#ifdef __cplusplus
}
#endif

#endif /* MX_BTL_ABI_H */
