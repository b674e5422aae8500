/*
 * mx_rdma.h -- one-sided copies between the device buffers of processes on
 * a node: what btl/smcuda's CUDA IPC path does for the PML's RDMA protocols
 * (the registration of opal/mca/btl/smcuda/btl_smcuda.c:1030-1075, the get
 * of :1077-1180, installed as the module's btl_get at
 * btl_smcuda_component.c:936), here for MI355X over xGMI / the device's HBM.
 *
 * The owner registers a device allocation range (mx_rdma_register: the IPC
 * handle of its allocation, exported once and cached); the handle travels to
 * a peer inside the PML's message (ob1's RGET / PUT headers); the peer moves
 * bytes between its own buffer and the owner's with mx_rdma_get /
 * mx_rdma_put, which map the owner's allocation once (process-wide cache,
 * keyed by the owner's pid, allocation base and runtime buffer id, so an
 * allocation freed and re-made at the same address is a new entry) and
 * launch a copy kernel.  Completion is asynchronous (mx_rdma_test).
 *
 * Data readiness follows the CUDA-aware MPI contract the reference's build
 * selects (OPAL_CUDA_SYNC_MEMOPS, opal/mca/common/cuda/common_cuda.c): the
 * owner's writes to its buffer are complete when it hands the handle over
 * (the application synchronised before MPI_Send / the window epoch).
 * Coherence: a get reads the owner's memory after a system-scope acquire on
 * every XCD of the reader (stale lines of an earlier get dropped); a put's
 * copy kernel ends with the runtime's end-of-kernel release, and the owner
 * consumes the bytes after the PML's completion message, in a later kernel
 * (DESIGN 7.1).
 *
 * Returns MX_SUCCESS (0) or a negative MX_ERR_* (include/mx_kernels.h).
 */
#ifndef MX_RDMA_H
#define MX_RDMA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mx_rdma_handle {
    unsigned char ipc[64];     /* IPC handle of the owner's allocation            */
    uint64_t base;             /* the allocation's base in the owner's address space */
    uint64_t size;             /* its bytes                                        */
    uint64_t id;               /* runtime buffer id of the allocation              */
    int32_t pid;               /* owner process                                    */
    int32_t device;            /* owner's device ordinal                           */
} mx_rdma_handle_t;

typedef struct mx_rdma_op mx_rdma_op_t;

/* Handle of the device allocation holding [ptr, ptr + bytes). */
int mx_rdma_register(const void *ptr, size_t bytes, mx_rdma_handle_t *handle);
/* local[0, bytes) <- the owner's [remote_addr, remote_addr + bytes), where
 * remote_addr is an address in the owner's space inside the registered
 * allocation.  stream: NULL = the library's RDMA stream.  *op: completion. */
int mx_rdma_get(void *local, const mx_rdma_handle_t *remote, uint64_t remote_addr, size_t bytes, void *stream,
                mx_rdma_op_t **op);
/* the owner's [remote_addr, ...) <- local[0, bytes). */
int mx_rdma_put(const void *local, const mx_rdma_handle_t *remote, uint64_t remote_addr, size_t bytes,
                void *stream, mx_rdma_op_t **op);
/* 1 complete, 0 not yet, < 0 error (the op stays valid until freed). */
int mx_rdma_test(mx_rdma_op_t *op);
int mx_rdma_wait(mx_rdma_op_t *op);
int mx_rdma_op_free(mx_rdma_op_t *op);
/* mapped peer allocations held by the process (test support) */
int mx_rdma_mapped(void);

#ifdef __cplusplus
}
#endif

#endif /* MX_RDMA_H */
