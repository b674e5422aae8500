/*
 * mx_kernels.h -- C-ABI boundary of the MI355X-native collective-reduction
 * hot path (libmx_kernels.so, built by hipcc for gfx950).
 *
 * Everything here is plain C: pointers, sizes, ints.  No HIP, torch or MPI
 * types cross this boundary (streams are passed as `void *` = hipStream_t).
 * All entry points return MX_SUCCESS (0) or a negative MX_ERR_* code.
 *
 * Which reference interface each group replaces (paths relative to the
 * reference checkout, HewlettPackard/zhpe-ompi = Open MPI 5.0.0a1):
 *
 *   mx_reduce2  <- ompi_op_base_handler_fn_t slots
 *                  ompi/mca/op/op.h:258-262, instantiated by the OP_FUNC /
 *                  FUNC_FUNC / LOC_FUNC macros of
 *                  ompi/mca/op/base/op_base_functions.c:40-104 and tabled at
 *                  :1485-1569 (ompi_op_base_functions[op][type]).
 *                  Semantics: inout[i] = inout[i] OP in[i].
 *   mx_reduce3  <- ompi_op_base_3buff_handler_fn_t slots
 *                  ompi/mca/op/op.h:267-273; op_base_functions.c:654-775,
 *                  table :1572-1655.  Semantics: out[i] = in1[i] OP in2[i].
 *   mx_op_supported <- the NULL / non-NULL pattern of those tables, which
 *                  ompi_op_base_op_select() checks
 *                  (ompi/mca/op/base/op_base_op_select.c:185-201).
 *   mx_is_device_ptr <- the per-call buffer probe of the accelerator
 *                  pattern (opal/datatype/opal_datatype_cuda.c:70-90,
 *                  opal/mca/common/cuda/common_cuda.c:1736-1857).
 *   mx_copy     <- opal_datatype_copy_content_same_ddt for contiguous
 *                  types (opal/datatype/opal_datatype_copy.c:99-141).
 *   mx_ddt_* / mx_pack / mx_unpack <- the convertor pack/unpack loops
 *                  opal_generic_simple_pack_function
 *                  (opal/datatype/opal_datatype_pack.c:235-370) and
 *                  opal_generic_simple_unpack_function
 *                  (opal/datatype/opal_datatype_unpack.c:245-427), see
 *                  mx_convertor.h.
 *   mx_comm_* / mx_allreduce / ... <- the coll module slots
 *                  ompi/mca/coll/coll.h:200-244 as implemented by
 *                  ompi/mca/coll/base/coll_base_allreduce.c et al., see
 *                  mx_coll.h.
 *
 * The op and type numbering is IDENTICAL to the reference's
 * OMPI_OP_BASE_FORTRAN_* (ompi/mca/op/op.h:206-240) and
 * OMPI_OP_BASE_TYPE_* (ompi/mca/op/op.h:104-199) enums, so an op component
 * passes op->o_f_to_c_index and ompi_op_ddt_map[dtype->id] straight through.
 */
#ifndef MX_KERNELS_H
#define MX_KERNELS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MX_ABI_VERSION 1

/* ---- return codes ---------------------------------------------------- */
#define MX_SUCCESS          0
#define MX_ERR_ARG         -1  /* bad argument (NULL, misaligned, size)     */
#define MX_ERR_UNSUPPORTED -2  /* (op,type) has no kernel: NULL table slot  */
#define MX_ERR_HIP         -3  /* HIP runtime error                          */
#define MX_ERR_NOMEM       -4  /* allocation failure                         */
#define MX_ERR_TIMEOUT     -5  /* a peer never arrived (bounded spin)        */
#define MX_ERR_RCCL        -6  /* RCCL error                                 */
#define MX_ERR_NOT_INIT    -7  /* mx_init not called / no device             */
#define MX_ERR_STATE       -8  /* object in the wrong state                  */
#define MX_ERR_TRUNCATE    -9  /* message longer than the receive buffer     */
#define MX_ERR_TAG        -10  /* in-order channel: envelope tag differs     */

/* ---- predefined reduction ops (== OMPI_OP_BASE_FORTRAN_*) ------------ */
enum {
    MX_OP_NULL = 0,
    MX_OP_MAX,
    MX_OP_MIN,
    MX_OP_SUM,
    MX_OP_PROD,
    MX_OP_LAND,
    MX_OP_BAND,
    MX_OP_LOR,
    MX_OP_BOR,
    MX_OP_LXOR,
    MX_OP_BXOR,
    MX_OP_MAXLOC,
    MX_OP_MINLOC,
    MX_OP_REPLACE,
    MX_OP_NO_OP,
    MX_OP_COUNT
};

/* ---- reducible type slots (== OMPI_OP_BASE_TYPE_*) ------------------- */
enum {
    MX_TYPE_INT8_T = 0,
    MX_TYPE_UINT8_T,
    MX_TYPE_INT16_T,
    MX_TYPE_UINT16_T,
    MX_TYPE_INT32_T,
    MX_TYPE_UINT32_T,
    MX_TYPE_INT64_T,
    MX_TYPE_UINT64_T,
    MX_TYPE_INTEGER,          /* Fortran INTEGER   (4 B)                  */
    MX_TYPE_INTEGER1,
    MX_TYPE_INTEGER2,
    MX_TYPE_INTEGER4,
    MX_TYPE_INTEGER8,
    MX_TYPE_INTEGER16,        /* never built by the reference (no kernel) */
    MX_TYPE_SHORT_FLOAT,      /* never built by the reference (no kernel) */
    MX_TYPE_FLOAT,
    MX_TYPE_DOUBLE,
    MX_TYPE_REAL,             /* Fortran REAL      (4 B)                  */
    MX_TYPE_REAL2,            /* never built                              */
    MX_TYPE_REAL4,
    MX_TYPE_REAL8,
    MX_TYPE_REAL16,           /* never built                              */
    MX_TYPE_DOUBLE_PRECISION,
    MX_TYPE_LONG_DOUBLE,      /* x87 80-bit in 16 B                       */
    MX_TYPE_LOGICAL,          /* Fortran LOGICAL   (4 B)                  */
    MX_TYPE_BOOL,
    MX_TYPE_C_SHORT_FLOAT_COMPLEX, /* never built                         */
    MX_TYPE_C_FLOAT_COMPLEX,
    MX_TYPE_C_DOUBLE_COMPLEX,
    MX_TYPE_C_LONG_DOUBLE_COMPLEX,
    MX_TYPE_BYTE,
    MX_TYPE_2REAL,
    MX_TYPE_2DOUBLE_PRECISION,
    MX_TYPE_2INTEGER,
    MX_TYPE_FLOAT_INT,
    MX_TYPE_DOUBLE_INT,
    MX_TYPE_LONG_INT,
    MX_TYPE_2INT,
    MX_TYPE_SHORT_INT,
    MX_TYPE_LONG_DOUBLE_INT,
    MX_TYPE_WCHAR,            /* mapped by ompi_op_ddt_map, every kernel NULL */
    MX_TYPE_COUNT
};

/* Table-shape variants: the reference builds its kernel tables either with
 * or without the Fortran types (OMPI_HAVE_FORTRAN_*).  C-only = 116 pairs,
 * with Fortran = 176 pairs. */
#define MX_TABLE_C_ONLY      0
#define MX_TABLE_WITH_FORTRAN 1

/* ---- runtime --------------------------------------------------------- */

/* Select the HIP device and allocate per-process state.  Idempotent. */
int mx_init(int device);
int mx_finalize(void);
/* 1 = device (or device-mapped) memory, 0 = host memory, <0 = error.
 * Device allocations are cached as address ranges (64 entries, LRU), so the
 * per-call probe of the accelerator pattern (common_cuda.c:1736-1857) costs
 * no runtime call for a known buffer. */
int mx_is_device_ptr(const void *p);
/* Drop cached ranges overlapping [p, p+bytes) (a caller freeing device
 * memory it did not get from mx_alloc). */
int mx_ptr_cache_forget(const void *p, size_t bytes);
/* Block until all work queued on `stream` (NULL = default) completed. */
int mx_stream_sync(void *stream);
/* As mx_stream_sync, through a completion word in mapped host memory that a
 * marker kernel raises last on the stream (the host sees it without the
 * runtime's wake-up latency); falls back to mx_stream_sync after ~2 ms. */
int mx_stream_sync_fast(void *stream);

/* ---- memory and streams for the host components ----------------------
 * The coll component stages host buffers through device scratch (every
 * rank of a communicator takes the same path whatever memory its buffers
 * are in) and runs its kernels on streams it owns. */
int mx_alloc(size_t bytes, void **p);      /* device memory                */
int mx_free(void *p);
/* Pinned host memory (hipHostMalloc): the coll component's host copies of
 * device buffers when a collective runs on the saved host module (the
 * coll/cuda staging direction, coll_cuda_allreduce.c:30-73). */
int mx_host_alloc(size_t bytes, void **p);
int mx_host_free(void *p);
/* Any direction (host pageable / pinned / device), ordered on `stream`. */
int mx_memcpy(void *dst, const void *src, size_t bytes, void *stream);
/* A non-blocking stream (does not synchronise with the legacy default one),
 * at the highest stream priority so the kernels that spin on it (request
 * collectives) never share a hardware queue with ordinary streams. */
int mx_stream_create(void **stream);
/* A blocking stream: ordered with the legacy default stream implicitly (no
 * per-call event; same host cost as the default stream). */
int mx_stream_create_ordered(void **stream);
int mx_stream_destroy(void *stream);
/* `stream` waits on the device for the work queued on `after` so far
 * (NULL = the legacy default stream). */
int mx_stream_order(void *stream, void *after);
const char *mx_strerror(int rc);
/* Library identification, e.g. "mx_kernels gfx950 abi 1". */
const char *mx_version(void);

/* ---- reduction kernels (K1-K4) --------------------------------------- */

/* Element size in bytes of a type slot (pair types include padding:
 * short_int 8, double_int 16, long_double_int 32 ...); 0 if none. */
size_t mx_type_size(int type);
/* 1 if (op,type) has a kernel in the given table variant, else 0.  The
 * pattern equals the reference table's non-NULL pattern exactly. */
int mx_op_supported(int op, int type, int table_variant);

/* inout[i] = inout[i] OP in[i], i < count.  Asynchronous on `stream`
 * (hipStream_t, NULL = default stream).  Both buffers must be
 * device-accessible.  count is size_t: no INT_MAX limit. */
int mx_reduce2(int op, int type, const void *in, void *inout,
               size_t count, void *stream);
/* As mx_reduce2, and returns when the result is complete: the blocking form
 * the op component's handler needs (ompi_op_reduce, ompi/op/op.h:547-610,
 * returns with `inout` final, for every agent).  Launches of <= 1024
 * workgroups (count <= 262128) mark themselves: every workgroup releases
 * its stores at system scope and writes its own flag in mapped host memory;
 * larger ones are followed by mx_stream_sync_fast's marker kernel
 * (MX_FUSED_MARK=0: always the marker).  The host polls the flags; after
 * ~2 ms the wait falls back to hipStreamSynchronize, which also reports
 * faults.  A peer process reading `inout` right after return is tested in
 * tests/test_op_consumer_gpu.py. */
int mx_reduce2_sync(int op, int type, const void *in, void *inout,
                    size_t count, void *stream);
/* mx_reduce2_sync on a non-NULL stream hands calls of <= 2 MiB per buffer
 * (16-byte aligned buffers, element types without padding or x87) to a
 * resident service kernel instead of launching (no launch and no dispatch
 * per call: 4 KiB 7 -> 4 us, 1 MiB 9.8 -> 7.5 us; it
 * leaves after 100 us without calls or, between calls, once 1 ms old, and
 * is relaunched on demand; MX_OP_SERVICE=0 switches it off).  A call is
 * served only when `stream` and the legacy default stream hold no pending
 * work, so it keeps the launch's stream order.
 * Commands served and service launches so far; returns 1 when the service
 * is usable, 0 before first use, -1 when off. */
int mx_op_service_stats(unsigned long long *served, unsigned long long *launches);
/* Turns the service on or off at run time (overrides MX_OP_SERVICE; off
 * stops a running service kernel). */
int mx_op_service_set(int on);
/* Service launches that did not start within 1 ms (their hardware queue
 * held by a kernel of another stream) so far; returns 1 while such
 * a kernel has not yet left (calls launch meanwhile), else 0. */
int mx_op_service_held(unsigned long long *held);
/* Test support: launch on `stream` one wave that spins on a mapped host
 * word, as a p2p receive waiting for its peer holds its hardware queue,
 * until mx_debug_release() or timeout_ms pass. */
int mx_debug_hold(void *stream, unsigned timeout_ms);
/* The same on the op service's own stream (MX_ERR_NOT_INIT before its
 * first use): its next relaunch finds its hardware queue held. */
int mx_debug_hold_service(unsigned timeout_ms);
int mx_debug_release(void);
/* out[i] = in1[i] OP in2[i].  out may alias neither input (restrict, as
 * in the reference's 3-buffer functions). */
int mx_reduce3(int op, int type, const void *in1, const void *in2,
               void *out, size_t count, void *stream);
/* As mx_reduce3, and returns when `out` is complete for every agent (the
 * op component's 3-buffer handler, ompi_3buff_op_reduce, op.h:618-660):
 * the resident service on a non-NULL stream, as mx_reduce2_sync, else the
 * launch followed by mx_stream_sync_fast's marker kernel. */
int mx_reduce3_sync(int op, int type, const void *in1, const void *in2,
                    void *out, size_t count, void *stream);

/* Contiguous device copy (K7), asynchronous on stream. */
int mx_copy(void *dst, const void *src, size_t bytes, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* MX_KERNELS_H */
