/*
 * mx_convertor.h -- C-ABI of the device datatype engine (libmx_kernels.so):
 * pack / unpack of non-contiguous derived datatypes on MI355X.
 *
 * Replaces, for device-resident user buffers, the convertor hot loops
 *   opal_generic_simple_pack_function   opal/datatype/opal_datatype_pack.c:235-370
 *   opal_generic_simple_unpack_function opal/datatype/opal_datatype_unpack.c:245-427
 *   opal_pack_homogeneous_contig[_with_gaps] opal_datatype_pack.c:60-222
 * which, on the CUDA path, issue one cuMemcpy per contiguous block
 * (opal_datatype_cuda.c:121-140).
 *
 * Input is the reference's own committed description: the array of 32-byte
 * dt_elem_desc records (ELEM / LOOP / END_LOOP, opal_datatype_internal.h:
 * 146-196) that opal_datatype_commit leaves in opt_desc, terminated by the
 * final END_LOOP, plus the datatype's size, lb and ub.  mx_ddt_create walks
 * it once on the host and uploads a flat table of strided runs (disp,
 * block bytes, two levels of count/stride, packed offset); the kernels map
 * every 16-byte granule of the packed stream to its user address with a
 * binary search over that table staged in LDS, so one launch moves the
 * whole message (no per-block copies).
 *
 * Positions are byte offsets into the packed stream of `count` instances,
 * so packing is resumable at any byte exactly like the convertor's
 * bConverted / opal_convertor_set_position (opal_datatype_position.c:154):
 * mx_pack(..., offset, len) produces bytes [offset, offset + len).
 * `user` is the buffer address passed to MPI (displacements are relative
 * to it and may be negative).  Homogeneous (same-architecture) data only.
 */
#ifndef MX_CONVERTOR_H
#define MX_CONVERTOR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mx_ddt mx_ddt_t;

/* Sizes of the OPAL basic types 0..25 (OPAL_DATATYPE_LOOP .. UNAVAILABLE)
 * the descriptions refer to (opal_datatype_internal.h:50-80), x86-64 LP64. */
#define MX_OPAL_NBASIC 26

/* desc: nrec 32-byte records (opt_desc incl. its terminating END_LOOP).
 * basic_sizes: MX_OPAL_NBASIC sizes, or NULL for the built-in LP64 table. */
int mx_ddt_create(const void *desc, size_t nrec, const uint64_t *basic_sizes, size_t size,
                  int64_t lb, int64_t ub, mx_ddt_t **ddt);
int mx_ddt_destroy(mx_ddt_t *ddt);
size_t mx_ddt_size(const mx_ddt_t *ddt);            /* packed bytes per instance */
int64_t mx_ddt_extent(const mx_ddt_t *ddt);         /* ub - lb                   */
size_t mx_ddt_runs(const mx_ddt_t *ddt);            /* flattened strided runs    */
/* [*lo, *hi): bytes relative to the user pointer that `count` instances
 * touch (true lb .. true ub of the whole message). */
int mx_ddt_span(const mx_ddt_t *ddt, size_t count, int64_t *lo, int64_t *hi);

/* Kernel family selection (tuning / tests; results are identical):
 * MX_DDT_PATH_AUTO picks per layout and call (the default); MX_DDT_PATH_BLOCK
 * sends every call the block table can take to the BLOCK kernels (one
 * 16-byte packed granule per lane, the instance tabled as its contiguous
 * user blocks).  Returns MX_ERR_UNSUPPORTED when the table cannot be built
 * (instances >= 2 GiB, > 4M blocks). */
#define MX_DDT_PATH_AUTO  0
#define MX_DDT_PATH_BLOCK 1
int mx_ddt_set_path(mx_ddt_t *ddt, int path);
/* The kernel family of the last mx_pack / mx_unpack on this datatype:
 * 1 copy (contiguous), 2 vector, 3 granule, 4 byte map, 5 piece,
 * 6 block, 7 tile / pipelined tile; 0 before the first call. */
int mx_ddt_last_path(const mx_ddt_t *ddt);

/* Pack bytes [offset, offset+len) of the packed stream of `count`
 * instances starting at `user` into `packed` (which receives exactly len
 * bytes).  Asynchronous on `stream`. */
int mx_pack(const mx_ddt_t *ddt, size_t count, const void *user, void *packed, size_t offset,
            size_t len, void *stream);
/* Inverse: scatter `len` packed bytes, which are bytes [offset, offset+len)
 * of the stream, into the user layout. */
int mx_unpack(const mx_ddt_t *ddt, size_t count, void *user, const void *packed, size_t offset,
              size_t len, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* MX_CONVERTOR_H */
