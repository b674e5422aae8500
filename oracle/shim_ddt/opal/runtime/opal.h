/* Test-infrastructure shim: the datatype engine only needs the init hooks. */
#ifndef MX_SHIM_OPAL_RUNTIME_H
#define MX_SHIM_OPAL_RUNTIME_H
#include "opal_config.h"
#include <stdbool.h>
extern bool opal_uses_threads;
int opal_init_util(int *argc, char ***argv);
int opal_finalize_util(void);
typedef void (*opal_cleanup_fn_t)(void);
void opal_finalize_register_cleanup_arg(const char *name, void (*fn)(void *), void *arg);
#define opal_finalize_register_cleanup(fn) opal_finalize_register_cleanup_arg(#fn, (void (*)(void *))(fn), NULL)
#endif
