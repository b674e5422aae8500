/*
 * mx_host.h -- TEST HARNESS ("mini-host"): just enough of Open MPI's
 * runtime to load and exercise the mi355x op and coll components without a
 * full Open MPI build.  It restates:
 *   - ompi_op_base_op_select (op_base_op_select.c:88-204): seed every slot
 *     with the base function, overlay component modules in ascending
 *     priority, check the NULL pattern;
 *   - mca_coll_base_comm_select (coll_base_comm_select.c:108-309): enable
 *     modules lowest -> highest priority, COPY each non-NULL slot;
 *   - the MPI entry points MPI_Reduce_local (reduce_local.c:46-91),
 *     MPI_Allreduce (allreduce.c:46-118), MPI_Reduce_scatter, MPI_Allgather,
 *     MPI_Bcast, MPI_Reduce, MPI_Reduce_scatter_block, MPI_Scan, MPI_Exscan
 *     and their nonblocking / persistent forms: parameter checks + dispatch
 *     through comm->c_coll;
 *   - requests (ompi/request/request.h:125-139), opal_progress_register and
 *     MPI_Start / MPI_Test / MPI_Wait / MPI_Request_free;
 *   - host coll modules standing in for coll/tuned (30), coll/basic (10) and
 *     coll/libnbc (10) on host buffers, under the reference's class names,
 *     their algorithms evaluated by the injected oracle restatement (and
 *     coll/base's compositions through the communicator's current slots),
 *     and a coll/self-like module (priority 75) for COMM_SELF;
 *   - --mca coll ^name exclusion, intercommunicator selection.
 * The base op functions, the collective oracle and the host transport are
 * injected by the test.
 */
#ifndef MX_HOST_H
#define MX_HOST_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* base op kernels injected by the test: the oracle restatement of
 * op_base_functions.c (oracle/mx_oracle_op.c) */
typedef int (*mxh_reducer_t)(int op, int type, const void *in, void *inout, size_t n, int fortran);
typedef int (*mxh_pattern_t)(int op, int type, int fortran);
/* host transport: allgather `bytes` per rank (rank-major) */
typedef int (*mxh_allgather_t)(const void *send, void *recv, size_t bytes, void *ctx);

/* the collective oracle (oracle/mx_oracle_coll.c entry points) the host
 * modules evaluate their algorithms with */
typedef struct {
    int (*allreduce)(int alg, int op, int type, int n, size_t count, const void *const *sbufs, void *const *rbufs);
    int (*reduce_scatter)(int alg, int op, int type, int n, const size_t *rcounts, const void *const *sbufs,
                          void *const *rbufs);
    int (*reduce)(int alg, int op, int type, int n, size_t count, int root, const void *const *sbufs, void *rbuf);
    int (*scan)(int alg, int op, int type, int n, size_t count, const void *const *sbufs, void *const *rbufs);
    int (*exscan)(int alg, int op, int type, int n, size_t count, const void *const *sbufs, void *const *rbufs);
    int (*iallreduce)(int alg, int op, int type, int n, size_t count, const void *const *sbufs, void *const *rbufs);
    int (*ireduce)(int alg, int op, int type, int n, size_t count, int root, const void *const *sbufs, void *rbuf);
    int (*ireduce_scatter)(int op, int type, int n, const size_t *rcounts, const void *const *sbufs,
                           void *const *rbufs);
} mxh_coll_oracle_t;
int mxh_set_coll_oracle(const mxh_coll_oracle_t *o);

int mxh_init(const char *component_lib, mxh_reducer_t base, mxh_pattern_t pattern);
int mxh_finalize(void);
/* MCA variable (OMPI_MCA_<name>), e.g. "coll_mi355x_priority" */
int mxh_set_mca(const char *name, int value);
/* string MCA variable (e.g. "coll" = "^tuned", coll_tuned_dynamic_rules_filename); NULL unsets */
int mxh_set_mca_str(const char *name, const char *value);

void *mxh_dtype(const char *mpi_name);   /* MPI_FLOAT, MPI_2INT, ...; NULL if unknown */
void *mxh_dtype_contiguous(int count, void *oldtype);  /* MPI_Type_contiguous */
void *mxh_dtype_vector(int count, int blocklen, int stride, void *oldtype);  /* MPI_Type_vector */
void *mxh_op(const char *mpi_name);      /* MPI_SUM, MPI_MAXLOC, ... */
/* which module owns slot t of op: 0 base, 1 mi355x */
int mxh_op_slot_owner(void *op, int type, int three_buffer);

void *mxh_comm_create(int rank, int size, mxh_allgather_t ag, void *ctx);
void *mxh_comm_self(void);
/* an intercommunicator whose local group has `size` ranks (selection only) */
void *mxh_intercomm_create(int rank, int size, mxh_allgather_t ag, void *ctx);
int mxh_comm_free(void *comm);
/* name of the component whose module owns a coll slot ("mi355x", "tuned",
 * "basic", "libnbc", "self") */
const char *mxh_comm_slot_owner(void *comm, const char *slot);

int mxh_op_reduce(void *op, const void *source, void *target, int count, void *dtype);
int mxh_3buff_op_reduce(void *op, const void *source1, const void *source2, void *target, int count, void *dtype);
/* calls that reached the coll/self stand-in's slots so far */
int mxh_self_calls(void);
/* average ns of one ompi_op_reduce through the op table over `iters` calls */
double mxh_time_op_reduce(void *op, const void *source, void *target, int count, void *dtype, int iters);
int mxh_reduce_local(const void *in, void *inout, int count, void *dtype, void *op);
int mxh_allreduce(const void *sbuf, void *rbuf, int count, void *dtype, void *op, void *comm);
int mxh_reduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, void *dtype, void *op, void *comm);
int mxh_allgather(const void *sbuf, int scount, void *sdtype, void *rbuf, int rcount, void *rdtype, void *comm);
int mxh_bcast(void *buf, int count, void *dtype, int root, void *comm);
int mxh_reduce(const void *sbuf, void *rbuf, int count, void *dtype, void *op, int root, void *comm);
int mxh_reduce_scatter_block(const void *sbuf, void *rbuf, int rcount, void *dtype, void *op, void *comm);
int mxh_scan(const void *sbuf, void *rbuf, int count, void *dtype, void *op, void *comm);
int mxh_exscan(const void *sbuf, void *rbuf, int count, void *dtype, void *op, void *comm);
/* nonblocking / persistent (MPI_I<coll>, MPI_<Coll>_init): *req receives
 * the request; MPI_Start / MPI_Test / MPI_Wait / MPI_Request_free */
int mxh_iallreduce(const void *sbuf, void *rbuf, int count, void *dtype, void *op, void *comm, void **req);
int mxh_allreduce_init(const void *sbuf, void *rbuf, int count, void *dtype, void *op, void *comm, void **req);
int mxh_ireduce(const void *sbuf, void *rbuf, int count, void *dtype, void *op, int root, void *comm, void **req);
int mxh_reduce_init(const void *sbuf, void *rbuf, int count, void *dtype, void *op, int root, void *comm, void **req);
int mxh_ireduce_scatter(const void *sbuf, void *rbuf, const int *rcounts, void *dtype, void *op, void *comm,
                        void **req);
int mxh_ireduce_scatter_block(const void *sbuf, void *rbuf, int rcount, void *dtype, void *op, void *comm,
                              void **req);
int mxh_iscan(const void *sbuf, void *rbuf, int count, void *dtype, void *op, void *comm, void **req);
int mxh_iexscan(const void *sbuf, void *rbuf, int count, void *dtype, void *op, void *comm, void **req);
int mxh_iallgather(const void *sbuf, int scount, void *sdtype, void *rbuf, int rcount, void *rdtype, void *comm,
                   void **req);
int mxh_ibcast(void *buf, int count, void *dtype, int root, void *comm, void **req);
int mxh_start(void *req);
int mxh_test(void **req, int *flag);
int mxh_wait(void **req);
int mxh_request_free(void **req);
#define MXH_IN_PLACE ((void *)1)

/* the datatype engine around the mi355x convertor hook (mca/convertor_mi355x.c) */
/* a host shared-memory BTL module with the mi355x GPU RDMA slots (mca/btl_mi355x.c) */
int mxh_btl_init(uint32_t *flags, size_t *handle_bytes);
int mxh_btl_register(void *base, size_t size, void *handle_out, void **reg);
int mxh_btl_deregister(void *reg);
/* calls that reached the stand-in BTL's own host RDMA slots (delegation from the installed ones) */
int mxh_btl_host_calls(void);
int mxh_btl_rdma(int get, void *local, uint64_t remote_addr, const void *remote_handle, size_t size, int ntimes);
int mxh_btl_flush_gets(void *local, uint64_t remote_addr, const void *remote_handle, size_t size, int n);
int mxh_convertor_run(const void *desc, size_t nrec, size_t size, int64_t lb, int64_t ub, int64_t true_lb,
                      int64_t true_ub, size_t count, void *user, void *packed, size_t start, size_t frag,
                      int niov, int recv, int *calls);

#ifdef __cplusplus
}
#endif
#endif
