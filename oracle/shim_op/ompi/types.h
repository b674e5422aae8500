/* Test-infrastructure shim: forward declarations only. */
#ifndef MX_SHIM_OMPI_TYPES_H
#define MX_SHIM_OMPI_TYPES_H
struct ompi_datatype_t;
struct ompi_op_t;
struct ompi_communicator_t;
#endif
