/* TEST INFRASTRUCTURE: link-time stand-ins for the few OPAL runtime
 * services the reference's opal/datatype engine calls (output, init/final
 * hooks, MCA var registration).  Only used to build oracle/_ref/. */
#include <stdarg.h>
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>

bool opal_uses_threads = false;
int opal_output_open(void *lds) { (void)lds; return 0; }
void opal_output_close(int id) { (void)id; }
void opal_output_set_verbosity(int id, int level) { (void)id; (void)level; }
void opal_output(int id, const char *fmt, ...)
{
    va_list ap;
    (void)id;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    fputc('\n', stderr);
}
void opal_output_verbose(int level, int id, const char *fmt, ...) { (void)level; (void)id; (void)fmt; }
void opal_output_vverbose(int level, int id, const char *fmt, va_list ap) { (void)level; (void)id; (void)fmt; (void)ap; }
int opal_output_get_verbosity(int id) { (void)id; return 0; }
void opal_finalize_register_cleanup_arg(const char *name, void (*fn)(void *), void *arg)
{
    (void)name; (void)fn; (void)arg;
}
int mca_base_var_register(const char *project, const char *framework, const char *component,
                          const char *name, const char *desc, int type, void *enumr, int bind, int flags,
                          int info, int scope, void *storage)
{
    (void)project; (void)framework; (void)component; (void)name; (void)desc; (void)type; (void)enumr;
    (void)bind; (void)flags; (void)info; (void)scope; (void)storage;
    return 0;
}
extern int opal_arch_init(void);
extern int opal_datatype_init(void);
int opal_init_util(int *argc, char ***argv)
{
    (void)argc; (void)argv;
    opal_arch_init();
    return opal_datatype_init();
}
int opal_finalize_util(void) { return 0; }
#undef snprintf
int opal_snprintf(char *str, size_t size, const char *fmt, ...)
{
    va_list ap;
    int n;
    va_start(ap, fmt);
    n = vsnprintf(str, size, fmt, ap);
    va_end(ap);
    return n;
}
