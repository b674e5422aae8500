/* Test-infrastructure shim (NOT product code): the minimum autoconf-style
 * configuration needed to compile the reference's
 * ompi/mca/op/base/op_base_functions.c standalone with gcc, so the oracle
 * can be pinned against the reference's own kernels.  SURVEY.md Appendix A.1.
 * MX_WITH_FORTRAN selects the 176-entry (Fortran types present) table;
 * default is the 116-entry C-only table. */
#ifndef MX_SHIM_OMPI_CONFIG_H
#define MX_SHIM_OMPI_CONFIG_H
#include <stdint.h>
#include <stdbool.h>
#include <stddef.h>
#define BEGIN_C_DECLS
#define END_C_DECLS
#define OMPI_DECLSPEC
#define HAVE_SYS_TYPES_H 1
#ifndef MX_WITH_FORTRAN
#define MX_WITH_FORTRAN 0
#endif
#define OMPI_HAVE_FORTRAN_INTEGER MX_WITH_FORTRAN
#define OMPI_HAVE_FORTRAN_INTEGER1 MX_WITH_FORTRAN
#define OMPI_HAVE_FORTRAN_INTEGER2 MX_WITH_FORTRAN
#define OMPI_HAVE_FORTRAN_INTEGER4 MX_WITH_FORTRAN
#define OMPI_HAVE_FORTRAN_INTEGER8 MX_WITH_FORTRAN
#define OMPI_HAVE_FORTRAN_INTEGER16 0
#define OMPI_HAVE_FORTRAN_REAL MX_WITH_FORTRAN
#define OMPI_HAVE_FORTRAN_REAL2 0
#define OMPI_HAVE_FORTRAN_REAL4 MX_WITH_FORTRAN
#define OMPI_HAVE_FORTRAN_REAL8 MX_WITH_FORTRAN
#define OMPI_HAVE_FORTRAN_REAL16 0
#define OMPI_REAL16_MATCHES_C 0
#define OMPI_HAVE_FORTRAN_DOUBLE_PRECISION MX_WITH_FORTRAN
#define OMPI_HAVE_FORTRAN_LOGICAL MX_WITH_FORTRAN
typedef int32_t ompi_fortran_integer_t;
typedef int8_t ompi_fortran_integer1_t;
typedef int16_t ompi_fortran_integer2_t;
typedef int32_t ompi_fortran_integer4_t;
typedef int64_t ompi_fortran_integer8_t;
typedef float ompi_fortran_real_t;
typedef float ompi_fortran_real4_t;
typedef double ompi_fortran_real8_t;
typedef double ompi_fortran_double_precision_t;
typedef int32_t ompi_fortran_logical_t;
#endif
