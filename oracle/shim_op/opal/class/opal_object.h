/* Test-infrastructure shim: layout-only stand-in for opal_object_t (non-debug
 * build, opal/class/opal_object.h:194-206) so op.h compiles. */
#ifndef MX_SHIM_OPAL_OBJECT_H
#define MX_SHIM_OPAL_OBJECT_H
#include <stdint.h>
typedef struct { void *obj_class; volatile int32_t obj_reference_count; } opal_object_t;
#define OBJ_CLASS_DECLARATION(NAME) extern int NAME##_dummy
#endif
