/*
 * mx_opal_convertor_abi.h -- layout mirror of the OPAL datatype engine
 * structures the mi355x convertor hook reads (mca/convertor_mi355x.c).
 *
 * Mirrored layouts (reference = HewlettPackard/zhpe-ompi, Open MPI 5.0.0a1,
 * x86-64, OPAL_ENABLE_DEBUG = 0, OPAL_CUDA_SUPPORT = 0 -- an MI355X build
 * has no CUDA):
 *   dt_type_desc_t              opal/datatype/opal_datatype.h:96-100
 *   opal_datatype_t             opal/datatype/opal_datatype.h:107-139
 *   dt_stack_t                  opal/datatype/opal_convertor.h:73-79
 *   opal_convertor_t            opal/datatype/opal_convertor.h:85-124
 *   convertor_advance_fct_t     opal/datatype/opal_convertor.h:63-66
 *   CONVERTOR_* flags           opal/datatype/opal_convertor.h:43-58
 *   OPAL_DATATYPE_FLAG_*        opal/datatype/opal_datatype.h:68-76
 * With -DMX_OMPI_REAL the real opal/datatype/opal_convertor.h is included
 * instead (tests/test_abi_layout.py compiles the hook that way against the
 * reference headers and checks every mirrored offset against them).
 */
#ifndef MX_OPAL_CONVERTOR_ABI_H
#define MX_OPAL_CONVERTOR_ABI_H

#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

#ifdef MX_OMPI_REAL
#include "opal_config.h"
#include "opal/datatype/opal_convertor.h"
#include "opal/datatype/opal_datatype.h"
#else

#include "mx_ompi_abi.h"   /* opal_object_t */

#define MX_OPAL_MAX_OBJECT_NAME 64             /* OPAL_MAX_OBJECT_NAME (opal_config.h) */

typedef size_t opal_datatype_count_t;           /* opal_datatype.h:92 */

typedef struct dt_type_desc_t {
    opal_datatype_count_t length;                /* records allocated */
    opal_datatype_count_t used;                  /* records used (without the closing END_LOOP) */
    void *desc;                                  /* dt_elem_desc_t[]: 32-byte records */
} dt_type_desc_t;

typedef struct opal_datatype_t {
    opal_object_t super;
    uint16_t flags;
    uint16_t id;
    uint32_t bdt_used;
    size_t size;
    ptrdiff_t true_lb;
    ptrdiff_t true_ub;
    ptrdiff_t lb;
    ptrdiff_t ub;
    size_t nbElems;
    uint32_t align;
    uint32_t loops;
    char name[MX_OPAL_MAX_OBJECT_NAME];
    dt_type_desc_t desc;
    dt_type_desc_t opt_desc;
    size_t *ptypes;
} opal_datatype_t;

typedef struct dt_stack_t {
    int32_t index;
    int16_t type;
    int16_t padding;
    size_t count;
    ptrdiff_t disp;
} dt_stack_t;

#define DT_STATIC_STACK_SIZE 5

typedef struct opal_convertor_t opal_convertor_t;
typedef int32_t (*convertor_advance_fct_t)(opal_convertor_t *pConvertor, struct iovec *iov, uint32_t *out_size,
                                           size_t *max_data);

struct opal_convertor_t {
    opal_object_t super;
    uint32_t remoteArch;
    uint32_t flags;
    size_t local_size;
    size_t remote_size;
    const opal_datatype_t *pDesc;
    const dt_type_desc_t *use_desc;
    opal_datatype_count_t count;
    uint32_t stack_size;
    unsigned char *pBaseBuf;
    dt_stack_t *pStack;
    convertor_advance_fct_t fAdvance;
    struct opal_convertor_master_t *master;
    uint32_t stack_pos;
    size_t partial_length;
    size_t bConverted;
    uint32_t checksum;
    uint32_t csum_ui1;
    size_t csum_ui2;
    dt_stack_t static_stack[DT_STATIC_STACK_SIZE];
};

#define CONVERTOR_SEND_CONVERSION  0x00010000
#define CONVERTOR_RECV             0x00020000
#define CONVERTOR_SEND             0x00040000
#define CONVERTOR_HOMOGENEOUS      0x00080000
#define CONVERTOR_NO_OP            0x00100000
#define CONVERTOR_WITH_CHECKSUM    0x00200000
#define CONVERTOR_COMPLETED        0x08000000

#define OPAL_DATATYPE_FLAG_CONTIGUOUS 0x0010
#define OPAL_DATATYPE_FLAG_NO_GAPS    0x0020

#endif /* MX_OMPI_REAL */

#endif /* MX_OPAL_CONVERTOR_ABI_H */
