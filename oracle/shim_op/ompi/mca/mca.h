/* Test-infrastructure shim: opaque MCA base component types. */
#ifndef MX_SHIM_OMPI_MCA_H
#define MX_SHIM_OMPI_MCA_H
typedef struct { char opaque[256]; } mca_base_component_t;
typedef struct { char opaque[32]; } mca_base_component_data_t;
#define OMPI_MCA_BASE_VERSION_2_1_0(type, a, b, c) {{0}}
#endif
