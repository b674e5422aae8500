/*
 * mx_ompi_abi.h -- layout mirror of the Open MPI plugin ABI used by the
 * mi355x `op` and `coll` components, plus the small set of accessors the
 * components need from the host MPI library.
 *
 * Mirrored layouts (reference = HewlettPackard/zhpe-ompi, Open MPI 5.0.0a1):
 *   opal_object_t                      opal/class/opal_object.h:194-206
 *                                      (OPAL_ENABLE_DEBUG = 0 layout)
 *   ompi_op_base_handler_fn_t          ompi/mca/op/op.h:258-262
 *   ompi_op_base_3buff_handler_fn_t    ompi/mca/op/op.h:267-273
 *   ompi_op_base_module_1_0_0_t        ompi/mca/op/op.h:362-378
 *   ompi_op_base_op_fns_1_0_0_t        ompi/mca/op/op.h:390-395
 *   ompi_op_base_component_1_0_0_t     ompi/mca/op/op.h:331-341
 *   mca_coll_base_module_2_3_0_t       ompi/mca/coll/coll.h:504-604
 *   mca_coll_base_component_2_0_0_t    ompi/mca/coll/coll.h:471-481
 *   slot typedefs                      ompi/mca/coll/coll.h:195-250, 261-420, 440-443
 *   request services                   ompi/request/request.h:125-139, 436-
 *
 * Building against a real Open MPI tree: compile the components with
 * -DMX_OMPI_REAL and the Open MPI include paths.  This header then includes
 * the real framework headers (ompi/mca/op/op.h, ompi/mca/coll/coll.h,
 * ompi/request/request.h) instead of the mirrors below, and module objects
 * are real OPAL classes (OBJ_CLASS_INSTANCE / OBJ_NEW).  The host services
 * stay behind the mx_ompi_host_t table, filled from the real internals by
 * mca/mx_ompi_host_real.c.  -DMX_OMPI_REAL_NO_COLL leaves
 * out the coll headers (the op component needs only op.h).
 * Without MX_OMPI_REAL (the default here) the mirrors are used and the
 * table is filled by the host that loads the component -- the mini-host
 * harness in mca/host/.  tests/test_abi_layout.py checks every mirrored
 * offset against the reference's own headers and compiles op_mi355x.c in
 * the real mode against them.
 */
#ifndef MX_OMPI_ABI_H
#define MX_OMPI_ABI_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifdef MX_OMPI_REAL
/* ---- real Open MPI headers -------------------------------------------- */
#include "ompi_config.h"
#include "ompi/constants.h"
#include "opal/class/opal_object.h"
#include "ompi/mca/op/op.h"
#ifndef MX_OMPI_REAL_NO_COLL
#include "mpi.h"
#include "ompi/mca/coll/coll.h"
#include "ompi/request/request.h"
#endif
#ifndef OMPI_OP_FLAGS_INTRINSIC          /* ompi/op/op.h:99-117 */
#define OMPI_OP_FLAGS_INTRINSIC 0x0001
#define OMPI_OP_FLAGS_COMMUTE 0x0040
#endif
struct mca_coll_base_module_2_3_0_t;
/* module classes: real OPAL classes derived from the framework's module
 * class; the destructor runs before OBJ_RELEASE frees the object */
#define MX_MODULE_CLASS(T, PARENT, DTOR) OBJ_CLASS_INSTANCE(T, PARENT, NULL, DTOR)
#define MX_MODULE_NEW(T, SUPER_FIELD)                                                          \
    ({                                                                                          \
        T *o_ = OBJ_NEW(T);                                                                     \
        if (o_) memset((char *)o_ + sizeof(o_->SUPER_FIELD), 0, sizeof(T) - sizeof(o_->SUPER_FIELD)); \
        o_;                                                                                     \
    })
#else /* !MX_OMPI_REAL */

#define OMPI_SUCCESS 0
#define OMPI_ERROR -1
#define OMPI_ERR_OUT_OF_RESOURCE -2
#define OMPI_ERR_NOT_SUPPORTED -8
#define OMPI_ERR_NOT_FOUND -13
#define MPI_IN_PLACE ((void *)1)

#define OMPI_OP_BASE_TYPE_MAX 41
#define OMPI_OP_BASE_FORTRAN_OP_MAX 15

#define OMPI_OP_FLAGS_INTRINSIC 0x0001
#define OMPI_OP_FLAGS_COMMUTE 0x0040

struct ompi_datatype_t;
struct ompi_op_t;
struct ompi_communicator_t;
struct ompi_request_t;
struct ompi_info_t;

/* ---- opal_object_t (non-debug) ------------------------------------------- */
typedef struct mx_obj_class {
    const char *cls_name;
    void (*cls_destruct)(void *obj);
} mx_obj_class_t;

typedef struct opal_object_t {
    mx_obj_class_t *obj_class;
    volatile int32_t obj_reference_count;
} opal_object_t;

/* opaque MCA base component blocks (mca_base_component_2_1_0_t is 0x300+
 * bytes of version/name strings and open/close/register hooks in the real
 * tree; only their presence matters to the selection logic) */
typedef struct mca_base_component_t {
    int mca_major_version, mca_minor_version, mca_release_version;
    char mca_project_name[16];
    int mca_project_major_version, mca_project_minor_version, mca_project_release_version;
    char mca_type_name[32];
    int mca_type_major_version, mca_type_minor_version, mca_type_release_version;
    char mca_component_name[64];
    int mca_component_major_version, mca_component_minor_version, mca_component_release_version;
    int (*mca_open_component)(void);
    int (*mca_close_component)(void);
    int (*mca_query_component)(void *, int *);
    int (*mca_register_component_params)(void);
    int32_t mca_component_flags;
    char reserved[28];
} mca_base_component_t;

typedef struct mca_base_component_data_t {
    uint32_t param_field;
    char reserved[32];
} mca_base_component_data_t;

/* ---- op framework (ompi/mca/op/op.h) ------------------------------------- */
struct ompi_op_base_module_1_0_0_t;
typedef void (*ompi_op_base_handler_fn_t)(void *, void *, int *, struct ompi_datatype_t **,
                                          struct ompi_op_base_module_1_0_0_t *);
typedef void (*ompi_op_base_3buff_handler_fn_t)(void *, void *, void *, int *, struct ompi_datatype_t **,
                                                struct ompi_op_base_module_1_0_0_t *);
typedef int (*ompi_op_base_component_init_query_fn_t)(bool enable_progress_threads, bool enable_mpi_threads);
typedef struct ompi_op_base_module_1_0_0_t *(*ompi_op_base_component_op_query_1_0_0_fn_t)(
    struct ompi_op_t *op, int *priority);
typedef int (*ompi_op_base_module_enable_1_0_0_fn_t)(struct ompi_op_base_module_1_0_0_t *module,
                                                      struct ompi_op_t *op);

typedef struct ompi_op_base_component_1_0_0_t {
    mca_base_component_t opc_version;
    mca_base_component_data_t opc_data;
    ompi_op_base_component_init_query_fn_t opc_init_query;
    ompi_op_base_component_op_query_1_0_0_fn_t opc_op_query;
} ompi_op_base_component_1_0_0_t;

typedef struct ompi_op_base_module_1_0_0_t {
    opal_object_t super;
    ompi_op_base_module_enable_1_0_0_fn_t opm_enable;
    struct ompi_op_t *opm_op;
    ompi_op_base_handler_fn_t opm_fns[OMPI_OP_BASE_TYPE_MAX];
    ompi_op_base_3buff_handler_fn_t opm_3buff_fns[OMPI_OP_BASE_TYPE_MAX];
} ompi_op_base_module_1_0_0_t;
typedef ompi_op_base_module_1_0_0_t ompi_op_base_module_t;

typedef struct ompi_op_base_op_fns_1_0_0_t {
    ompi_op_base_handler_fn_t fns[OMPI_OP_BASE_TYPE_MAX];
    ompi_op_base_module_t *modules[OMPI_OP_BASE_TYPE_MAX];
} ompi_op_base_op_fns_t;

typedef struct ompi_op_base_op_3buff_fns_1_0_0_t {
    ompi_op_base_3buff_handler_fn_t fns[OMPI_OP_BASE_TYPE_MAX];
    ompi_op_base_module_t *modules[OMPI_OP_BASE_TYPE_MAX];
} ompi_op_base_op_3buff_fns_t;

/* ---- coll framework (ompi/mca/coll/coll.h) ------------------------------- */
struct mca_coll_base_module_2_3_0_t;
typedef struct mca_coll_base_module_2_3_0_t mca_coll_base_module_t;
typedef int (*mca_coll_base_component_init_query_fn_t)(bool enable_progress_threads, bool enable_mpi_threads);
typedef mca_coll_base_module_t *(*mca_coll_base_component_comm_query_2_0_0_fn_t)(
    struct ompi_communicator_t *comm, int *priority);
typedef int (*mca_coll_base_module_enable_1_1_0_fn_t)(mca_coll_base_module_t *module,
                                                      struct ompi_communicator_t *comm);
typedef int (*mca_coll_base_module_disable_1_2_0_fn_t)(mca_coll_base_module_t *module,
                                                       struct ompi_communicator_t *comm);
typedef int (*mca_coll_base_module_allgather_fn_t)(const void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                                                   void *rbuf, int rcount, struct ompi_datatype_t *rdtype,
                                                   struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_allreduce_fn_t)(const void *sbuf, void *rbuf, int count,
                                                   struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                                   struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_bcast_fn_t)(void *buff, int count, struct ompi_datatype_t *datatype, int root,
                                               struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_reduce_scatter_fn_t)(const void *sbuf, void *rbuf, const int *rcounts,
                                                        struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                                        struct ompi_communicator_t *comm,
                                                        mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_reduce_local_fn_t)(const void *inbuf, void *inoutbuf, int count,
                                                      struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                                      mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_reduce_fn_t)(const void *sbuf, void *rbuf, int count,
                                                struct ompi_datatype_t *dtype, struct ompi_op_t *op, int root,
                                                struct ompi_communicator_t *comm, mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_reduce_scatter_block_fn_t)(const void *sbuf, void *rbuf, int rcount,
                                                              struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                                              struct ompi_communicator_t *comm,
                                                              mca_coll_base_module_t *module);
typedef int (*mca_coll_base_module_scan_fn_t)(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                                              struct ompi_op_t *op, struct ompi_communicator_t *comm,
                                              mca_coll_base_module_t *module);
typedef mca_coll_base_module_scan_fn_t mca_coll_base_module_exscan_fn_t;
/* nonblocking (coll.h:261-338) and persistent (:339-420: + MPI_Info) */
#define MX_NB_ARGS struct ompi_communicator_t *comm, struct ompi_request_t **request, mca_coll_base_module_t *module
#define MX_PI_ARGS struct ompi_communicator_t *comm, struct ompi_info_t *info, struct ompi_request_t **request, \
                   mca_coll_base_module_t *module
typedef int (*mca_coll_base_module_iallgather_fn_t)(const void *sbuf, int scount, struct ompi_datatype_t *sdtype,
                                                    void *rbuf, int rcount, struct ompi_datatype_t *rdtype,
                                                    MX_NB_ARGS);
typedef int (*mca_coll_base_module_iallreduce_fn_t)(const void *sbuf, void *rbuf, int count,
                                                    struct ompi_datatype_t *dtype, struct ompi_op_t *op, MX_NB_ARGS);
typedef int (*mca_coll_base_module_ibcast_fn_t)(void *buff, int count, struct ompi_datatype_t *datatype, int root,
                                                MX_NB_ARGS);
typedef int (*mca_coll_base_module_ireduce_fn_t)(const void *sbuf, void *rbuf, int count,
                                                 struct ompi_datatype_t *dtype, struct ompi_op_t *op, int root,
                                                 MX_NB_ARGS);
typedef int (*mca_coll_base_module_ireduce_scatter_fn_t)(const void *sbuf, void *rbuf, const int *rcounts,
                                                         struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                                         MX_NB_ARGS);
typedef int (*mca_coll_base_module_ireduce_scatter_block_fn_t)(const void *sbuf, void *rbuf, int rcount,
                                                               struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                                               MX_NB_ARGS);
typedef int (*mca_coll_base_module_iscan_fn_t)(const void *sbuf, void *rbuf, int count, struct ompi_datatype_t *dtype,
                                               struct ompi_op_t *op, MX_NB_ARGS);
typedef mca_coll_base_module_iscan_fn_t mca_coll_base_module_iexscan_fn_t;
typedef int (*mca_coll_base_module_allgather_init_fn_t)(const void *sbuf, int scount,
                                                        struct ompi_datatype_t *sdtype, void *rbuf, int rcount,
                                                        struct ompi_datatype_t *rdtype, MX_PI_ARGS);
typedef int (*mca_coll_base_module_allreduce_init_fn_t)(const void *sbuf, void *rbuf, int count,
                                                        struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                                        MX_PI_ARGS);
typedef int (*mca_coll_base_module_bcast_init_fn_t)(void *buff, int count, struct ompi_datatype_t *datatype,
                                                    int root, MX_PI_ARGS);
typedef int (*mca_coll_base_module_reduce_init_fn_t)(const void *sbuf, void *rbuf, int count,
                                                     struct ompi_datatype_t *dtype, struct ompi_op_t *op, int root,
                                                     MX_PI_ARGS);
typedef int (*mca_coll_base_module_reduce_scatter_init_fn_t)(const void *sbuf, void *rbuf, const int *rcounts,
                                                             struct ompi_datatype_t *dtype, struct ompi_op_t *op,
                                                             MX_PI_ARGS);
typedef int (*mca_coll_base_module_reduce_scatter_block_init_fn_t)(const void *sbuf, void *rbuf, int rcount,
                                                                   struct ompi_datatype_t *dtype,
                                                                   struct ompi_op_t *op, MX_PI_ARGS);
typedef int (*mca_coll_base_module_scan_init_fn_t)(const void *sbuf, void *rbuf, int count,
                                                   struct ompi_datatype_t *dtype, struct ompi_op_t *op, MX_PI_ARGS);
typedef mca_coll_base_module_scan_init_fn_t mca_coll_base_module_exscan_init_fn_t;
typedef int (*mca_coll_base_module_ft_event_fn_t)(int state);
typedef void *mx_coll_slot_unused_t;   /* slots this component never fills */

struct mca_coll_base_module_2_3_0_t {
    opal_object_t super;
    mca_coll_base_module_enable_1_1_0_fn_t coll_module_enable;
    /* blocking */
    mca_coll_base_module_allgather_fn_t coll_allgather;
    mx_coll_slot_unused_t coll_allgatherv;
    mca_coll_base_module_allreduce_fn_t coll_allreduce;
    mx_coll_slot_unused_t coll_alltoall, coll_alltoallv, coll_alltoallw, coll_barrier;
    mca_coll_base_module_bcast_fn_t coll_bcast;
    mca_coll_base_module_exscan_fn_t coll_exscan;
    mx_coll_slot_unused_t coll_gather, coll_gatherv;
    mca_coll_base_module_reduce_fn_t coll_reduce;
    mca_coll_base_module_reduce_scatter_fn_t coll_reduce_scatter;
    mca_coll_base_module_reduce_scatter_block_fn_t coll_reduce_scatter_block;
    mca_coll_base_module_scan_fn_t coll_scan;
    mx_coll_slot_unused_t coll_scatter, coll_scatterv;
    /* nonblocking (17) */
    mca_coll_base_module_iallgather_fn_t coll_iallgather;
    mx_coll_slot_unused_t coll_iallgatherv;
    mca_coll_base_module_iallreduce_fn_t coll_iallreduce;
    mx_coll_slot_unused_t coll_ialltoall, coll_ialltoallv, coll_ialltoallw, coll_ibarrier;
    mca_coll_base_module_ibcast_fn_t coll_ibcast;
    mca_coll_base_module_iexscan_fn_t coll_iexscan;
    mx_coll_slot_unused_t coll_igather, coll_igatherv;
    mca_coll_base_module_ireduce_fn_t coll_ireduce;
    mca_coll_base_module_ireduce_scatter_fn_t coll_ireduce_scatter;
    mca_coll_base_module_ireduce_scatter_block_fn_t coll_ireduce_scatter_block;
    mca_coll_base_module_iscan_fn_t coll_iscan;
    mx_coll_slot_unused_t coll_iscatter, coll_iscatterv;
    /* persistent (17) */
    mca_coll_base_module_allgather_init_fn_t coll_allgather_init;
    mx_coll_slot_unused_t coll_allgatherv_init;
    mca_coll_base_module_allreduce_init_fn_t coll_allreduce_init;
    mx_coll_slot_unused_t coll_alltoall_init, coll_alltoallv_init, coll_alltoallw_init, coll_barrier_init;
    mca_coll_base_module_bcast_init_fn_t coll_bcast_init;
    mca_coll_base_module_exscan_init_fn_t coll_exscan_init;
    mx_coll_slot_unused_t coll_gather_init, coll_gatherv_init;
    mca_coll_base_module_reduce_init_fn_t coll_reduce_init;
    mca_coll_base_module_reduce_scatter_init_fn_t coll_reduce_scatter_init;
    mca_coll_base_module_reduce_scatter_block_init_fn_t coll_reduce_scatter_block_init;
    mca_coll_base_module_scan_init_fn_t coll_scan_init;
    mx_coll_slot_unused_t coll_scatter_init, coll_scatterv_init;
    /* neighborhood (5 + 5 nonblocking + 5 persistent) */
    mx_coll_slot_unused_t coll_neighbor_allgather, coll_neighbor_allgatherv, coll_neighbor_alltoall,
        coll_neighbor_alltoallv, coll_neighbor_alltoallw;
    mx_coll_slot_unused_t coll_ineighbor_allgather, coll_ineighbor_allgatherv, coll_ineighbor_alltoall,
        coll_ineighbor_alltoallv, coll_ineighbor_alltoallw;
    mx_coll_slot_unused_t coll_neighbor_allgather_init, coll_neighbor_allgatherv_init,
        coll_neighbor_alltoall_init, coll_neighbor_alltoallv_init, coll_neighbor_alltoallw_init;
    mca_coll_base_module_ft_event_fn_t ft_event;
    mca_coll_base_module_disable_1_2_0_fn_t coll_module_disable;
    mca_coll_base_module_reduce_local_fn_t coll_reduce_local;
    struct mca_coll_base_comm_t *base_data;
};

typedef struct mca_coll_base_component_2_0_0_t {
    mca_base_component_t collm_version;
    mca_base_component_data_t collm_data;
    mca_coll_base_component_init_query_fn_t collm_init_query;
    mca_coll_base_component_comm_query_2_0_0_fn_t collm_comm_query;
} mca_coll_base_component_2_0_0_t;

/* module classes (mirror): the destructor runs, then the host frees the
 * object -- the OPAL OBJ_RELEASE semantics */
#define MX_MODULE_CLASS(T, PARENT, DTOR) static mx_obj_class_t T##_class = {#T, (void (*)(void *))(DTOR)}
#define MX_MODULE_NEW(T, SUPER_FIELD) ((T *)mx_obj_new(sizeof(T), &T##_class))
#include <stdlib.h>
static inline void *mx_obj_new(size_t bytes, mx_obj_class_t *cls)
{
    opal_object_t *o = (opal_object_t *)calloc(1, bytes);
    if (o) {
        o->obj_class = cls;
        o->obj_reference_count = 1;
    }
    return o;
}
#endif /* MX_OMPI_REAL */

/* ---- host services (Open MPI internals the components use) ---------------
 * In a real build these are ompi_comm_rank/size, ompi_op_ddt_map[dt->id] +
 * ompi_datatype_get_single_predefined_type_from_args, ompi_datatype_type_size,
 * ompi_datatype_is_contiguous_memory_layout, op->o_f_to_c_index / o_flags,
 * op->o_func.intrinsic, comm->c_coll, OBJ_RETAIN/OBJ_RELEASE and
 * mca_base_var lookups.  The mini-host harness supplies them through this
 * table before it queries the components. */
typedef struct mx_ompi_host {
    int (*comm_rank)(struct ompi_communicator_t *comm);
    int (*comm_size)(struct ompi_communicator_t *comm);
    /* reducible slot of a datatype (ompi_op_ddt_map, op.c:131-229), -1 if none */
    int (*dtype_slot)(struct ompi_datatype_t *dt);
    size_t (*dtype_size)(struct ompi_datatype_t *dt);
    /* 1 if count elements are one contiguous block of count*size bytes */
    int (*dtype_contiguous)(struct ompi_datatype_t *dt, int count);
    int (*op_index)(struct ompi_op_t *op);       /* o_f_to_c_index */
    uint32_t (*op_flags)(struct ompi_op_t *op);  /* o_flags */
    ompi_op_base_op_fns_t *(*op_fns)(struct ompi_op_t *op);              /* &op->o_func.intrinsic */
    ompi_op_base_op_3buff_fns_t *(*op_3buff_fns)(struct ompi_op_t *op);  /* &op->o_3buff_intrinsic */
    /* the communicator's current function table entry for a slot name
     * ("allreduce", "allgather", ...) and its module (comm->c_coll) */
    void *(*comm_coll_fn)(struct ompi_communicator_t *comm, const char *slot,
                          struct mca_coll_base_module_2_3_0_t **module);
    void (*obj_retain)(opal_object_t *obj);
    void (*obj_release)(opal_object_t *obj);
    /* integer MCA variable lookup (mca_base_var); returns def if unset */
    int (*mca_int)(const char *name, int def);
    /* the MPI_BYTE datatype handle (ompi_mpi_byte) for bootstrap exchanges */
    struct ompi_datatype_t *byte_dtype;
    /* ---- requests of the nonblocking / persistent slots ----
     * request_create: OBJ_NEW of the component's ompi_request_t subclass +
     *   OMPI_REQUEST_INIT(req, persistent) with req_type OMPI_REQUEST_COLL,
     *   req_start / req_free set to the given callbacks and `ctx` stored in
     *   the subclass (coll_libnbc_component.c:570-583 does the same);
     *   persistent requests start inactive (OMPI_REQUEST_INACTIVE), others
     *   active (OMPI_REQUEST_ACTIVE, REQUEST_PENDING);
     * request_ctx: the subclass field;
     * request_activate: MPI_Start's part of req_start -- req_state = ACTIVE,
     *   req_complete = REQUEST_PENDING;
     * request_complete: req_status.MPI_ERROR = status;
     *   ompi_request_complete(req, true) (request.h:436-);
     * progress_register: opal_progress_register (opal/runtime/opal_progress.h). */
    struct ompi_request_t *(*request_create)(int persistent, int (*start)(struct ompi_request_t *req),
                                             int (*free_fn)(struct ompi_request_t *req), void *ctx);
    void *(*request_ctx)(struct ompi_request_t *req);
    void (*request_activate)(struct ompi_request_t *req);
    void (*request_complete)(struct ompi_request_t *req, int status);
    int (*progress_register)(int (*fn)(void));
    /* ---- non-contiguous layouts (allgather / bcast may use any datatype;
     * the reductions only predefined ones, ompi_op_is_valid, op.h:477-514).
     * The layout of a datatype may differ between ranks as long as the type
     * signatures match, so the device-or-delegate choice cannot depend on
     * it: a non-contiguous buffer is packed into a contiguous one and back.
     * In a real build: opal_convertor_pack / _unpack over host memory
     * (opal_convertor.c:218-325) and opal_datatype_span (opal_datatype.h:
     * 329-340).  Host memory only; the component copies a device span to
     * the host first. */
    int (*dtype_pack)(struct ompi_datatype_t *dt, int count, const void *user, void *packed);
    int (*dtype_unpack)(struct ompi_datatype_t *dt, int count, const void *packed, void *user);
    /* bytes [*lo, *hi) relative to the buffer that count elements touch */
    int (*dtype_span)(struct ompi_datatype_t *dt, int count, ptrdiff_t *lo, ptrdiff_t *hi);
    /* the committed description of dt: the 32-byte dt_elem_desc records the
     * convertor walks (opal_datatype_t opt_desc.desc, used + 1 records with
     * the closing END_LOOP, opal_datatype.h:126 / opal_datatype_internal.h:
     * 146-196) with size, lb and ub -- the input of mx_ddt_create, so a
     * non-contiguous DEVICE buffer is packed / unpacked on the device.  NULL
     * (or an error return): device spans go through the host as above. */
    int (*dtype_desc)(struct ompi_datatype_t *dt, const void **recs, size_t *nrec, size_t *size, ptrdiff_t *lb,
                      ptrdiff_t *ub);
    /* ---- round 3 ----
     * comm_is_inter: OMPI_COMM_IS_INTER(comm) (communicator.h); every coll
     *   component on this path declines intercommunicators
     *   (coll_tuned_module.c:66-69, coll_cuda_module.c:141);
     * mca_string: string MCA variable (coll_tuned_dynamic_rules_filename),
     *   NULL if unset;
     * requests of the saved module, driven by the component when it runs a
     *   nonblocking collective on host copies of device buffers:
     *   request_test = REQUEST_COMPLETE(req) + req_status.MPI_ERROR, without
     *   progressing or freeing (the component polls from its own progress
     *   callback); request_start = req->req_start(1, &req) (MPI_Start);
     *   request_free = ompi_request_free(&req). */
    int (*comm_is_inter)(struct ompi_communicator_t *comm);
    const char *(*mca_string)(const char *name);
    int (*request_test)(struct ompi_request_t *req, int *flag, int *status);
    int (*request_start)(struct ompi_request_t *req);
    int (*request_free)(struct ompi_request_t **req);
} mx_ompi_host_t;

/* Set by the host before component queries. */
extern const mx_ompi_host_t *mx_ompi_host;

#define MX_OBJ_RETAIN(o) mx_ompi_host->obj_retain((opal_object_t *)(o))
#define MX_OBJ_RELEASE(o) mx_ompi_host->obj_release((opal_object_t *)(o))

/* Component symbols, looked up by name like mca_base_component_repository
 * does (mca_<type>_<name>_component, mca_base_component_repository.c:449-462). */
extern ompi_op_base_component_1_0_0_t mca_op_mi355x_component;
#if !defined(MX_OMPI_REAL) || !defined(MX_OMPI_REAL_NO_COLL)
extern mca_coll_base_component_2_0_0_t mca_coll_mi355x_component;
#endif
/* Host registration entry of the component library. */
int mx_ompi_set_host(const mx_ompi_host_t *host);

#ifdef __cplusplus
}
#endif

#endif /* MX_OMPI_ABI_H */
