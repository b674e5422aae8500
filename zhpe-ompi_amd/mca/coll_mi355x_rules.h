/*
 * coll_mi355x_rules.h -- which algorithm coll/tuned would run for a call,
 * so coll/mi355x can run that algorithm's reduction order on the device.
 *
 * coll/tuned picks, per collective and communicator (coll_tuned_module.c:
 * 152-170, coll_tuned_decision_dynamic.c): with coll_tuned_use_dynamic_rules
 * set, a rule of the coll_tuned_dynamic_rules_filename file for the
 * communicator size and message size, else the forced algorithm of
 * coll_tuned_<coll>_algorithm (with its _chain_fanout / _segmentsize), else
 * the fixed decision (coll_tuned_decision_fixed.c).
 */
#ifndef COLL_MI355X_RULES_H
#define COLL_MI355X_RULES_H
#include <stddef.h>

/* COLLTYPE numbering of the rules file (coll_base_functions.h:44-68) */
enum {
    MX_CT_ALLREDUCE = 2,
    MX_CT_EXSCAN = 8,
    MX_CT_REDUCE = 11,
    MX_CT_REDUCESCATTER = 12,
    MX_CT_REDUCESCATTERBLOCK = 13,
    MX_CT_SCAN = 14,
    MX_CT_COUNT = 22
};

/* one message-size rule (ompi_coll_msg_rule_t) */
typedef struct { size_t msg_size; int alg, faninout; long segsize; } mx_msg_rule_t;
/* the message-size rules of one communicator size (ompi_coll_com_rule_t) */
typedef struct { int comsize, nmsg; mx_msg_rule_t *msg; } mx_com_rule_t;

/* What coll/tuned was configured with for one communicator, read at module
 * enable (ompi_coll_tuned_forced_getvalues, coll_tuned_module.c:181-208). */
typedef struct {
    int dynamic;                         /* coll_tuned_use_dynamic_rules       */
    int forced_alg[MX_CT_COUNT];         /* coll_tuned_<coll>_algorithm        */
    int forced_chain[MX_CT_COUNT];       /* ..._algorithm_chain_fanout         */
    int forced_tree[MX_CT_COUNT];        /* ..._algorithm_tree_fanout          */
    int forced_seg[MX_CT_COUNT];         /* ..._algorithm_segmentsize          */
    const mx_com_rule_t *com[MX_CT_COUNT];   /* file rule for this comm size   */
} mx_tuned_cfg_t;

/* Loads the configuration for a communicator of `comm_size` ranks.  Returns
 * 0, or -1 when the rules file is named but unreadable or malformed (the
 * reference then ignores the whole file: dynamic rules fall back to the
 * forced / fixed choices, coll_tuned_component.c:241-258). */
int mx_tuned_cfg_load(mx_tuned_cfg_t *cfg, int comm_size);

/* coll/tuned's algorithm for collective `coll` at `dsize` bytes (the
 * message size its dynamic decision computes for that collective); 0 = the
 * fixed decision.  *fanout: the chain fanout the algorithm would use (file
 * rule faninout, else the forced chain fanout, else 0 = default). */
int mx_tuned_choice(const mx_tuned_cfg_t *cfg, int coll, size_t dsize, int *fanout);

/* Parses a rules file (ompi_coll_tuned_read_rules_config_file,
 * coll_tuned_dynamic_file.c) into per-collective arrays of `ncoll` entries;
 * returns the number of collectives with rules, or -1 (nothing kept).
 * Exposed for the tests. */
int mx_tuned_rules_parse(const char *fname, int ncoll, int *ncs, mx_com_rule_t **coms);
void mx_tuned_rules_free(int ncoll, int *ncs, mx_com_rule_t **coms);

#endif
