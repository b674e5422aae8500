/*
 * coll_mi355x_rules.c -- coll/tuned's algorithm selection beyond the fixed
 * decision, restated for coll/mi355x (coll_mi355x_rules.h):
 *  - forced algorithms: ompi_coll_tuned_forced_getvalues
 *    (coll_tuned_module.c:181-208) reads coll_tuned_<coll>_algorithm and its
 *    _segmentsize / _tree_fanout / _chain_fanout when the module is enabled;
 *  - rules file: ompi_coll_tuned_read_rules_config_file
 *    (coll_tuned_dynamic_file.c:56-259) -- whitespace-separated integers,
 *    '#' starts a comment, anything else not a number is skipped:
 *      <#collectives> { <coll id> <#comm sizes> { <comm size> <#msg sizes>
 *        { <msg size> <alg> <faninout> <segsize> } } }
 *    the first message size of every communicator size must be 0; a bad
 *    file is dropped as a whole;
 *  - lookup: ompi_coll_tuned_get_com_rule_ptr (coll_tuned_dynamic_rules.c:
 *    300-340: the last communicator size <= the communicator's, the first
 *    one when none is) and ompi_coll_tuned_get_target_method_params
 *    (:343-391: the last message size <= the message's);
 *  - order: file rule (if its algorithm is not 0), else forced, else fixed
 *    (coll_tuned_decision_dynamic.c, e.g. :55-95).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "coll_mi355x_rules.h"
#include "mx_ompi_abi.h"

#define MYEOF (-999)

static void skip_to_newline(FILE *f)
{
    int c;
    do { c = fgetc(f); } while (c != EOF && c != '\n');
}

/* getnext (coll_tuned_dynamic_file.c:280-296) */
static long next_value(FILE *f)
{
    long v;
    for (;;) {
        const int rc = fscanf(f, "%li", &v);
        if (rc == EOF) return MYEOF;
        if (rc == 1) return v;
        const int c = fgetc(f);
        if (c == EOF) return MYEOF;
        if (c == '#') skip_to_newline(f);
    }
}

void mx_tuned_rules_free(int ncoll, int *ncs, mx_com_rule_t **coms)
{
    for (int c = 0; c < ncoll; c++) {
        for (int k = 0; coms[c] && k < ncs[c]; k++) free(coms[c][k].msg);
        free(coms[c]);
        coms[c] = NULL;
        ncs[c] = 0;
    }
}

int mx_tuned_rules_parse(const char *fname, int ncoll, int *ncs, mx_com_rule_t **coms)
{
    for (int c = 0; c < ncoll; c++) { ncs[c] = 0; coms[c] = NULL; }
    if (!fname || ncoll < 1) return -1;
    FILE *f = fopen(fname, "r");
    if (!f) return -1;
    int total = 0;
    const long X = next_value(f);
    if (X < 0 || X > ncoll) goto bad;
    for (long x = 0; x < X; x++) {
        const long CI = next_value(f);
        if (CI < 0 || CI >= ncoll) goto bad;
        const long NCS = next_value(f);
        if (NCS < 0) goto bad;
        /* a repeated collective id replaces the earlier rules */
        for (int k = 0; coms[CI] && k < ncs[CI]; k++) free(coms[CI][k].msg);
        free(coms[CI]);
        coms[CI] = calloc((size_t)NCS + 1, sizeof(mx_com_rule_t));
        ncs[CI] = 0;
        if (!coms[CI]) goto bad;
        for (long k = 0; k < NCS; k++) {
            mx_com_rule_t *cr = &coms[CI][k];
            const long CS = next_value(f);
            if (CS < 0) goto bad;
            const long NMS = next_value(f);
            if (NMS < 0) goto bad;
            cr->comsize = (int)CS;
            cr->msg = calloc((size_t)NMS + 1, sizeof(mx_msg_rule_t));
            if (!cr->msg) goto bad;
            ncs[CI] = (int)k + 1;
            for (long j = 0; j < NMS; j++) {
                const long MS = next_value(f), ALG = MS < 0 ? -1 : next_value(f);
                const long FAN = ALG < 0 ? -1 : next_value(f), SS = FAN < 0 ? -1 : next_value(f);
                if (MS < 0 || ALG < 0 || FAN < 0 || SS < 0) goto bad;
                if (j == 0 && MS != 0) goto bad;   /* rules start at message size 0 */
                cr->msg[j] = (mx_msg_rule_t){(size_t)MS, (int)ALG, (int)FAN, SS};
                cr->nmsg = (int)j + 1;
            }
        }
        total++;
    }
    fclose(f);
    return total;
bad:
    fclose(f);
    mx_tuned_rules_free(ncoll, ncs, coms);
    return -1;
}

/* the rules of this process, parsed once per file name (coll/tuned reads
 * its file once, at component open) */
static char *g_rules_file;
static int g_rules_ok;
static int g_ncs[MX_CT_COUNT];
static mx_com_rule_t *g_coms[MX_CT_COUNT];

static int rules_for(const char *fname)
{
    if (g_rules_file && !strcmp(g_rules_file, fname)) return g_rules_ok;
    mx_tuned_rules_free(MX_CT_COUNT, g_ncs, g_coms);
    free(g_rules_file);
    g_rules_file = strdup(fname);
    g_rules_ok = mx_tuned_rules_parse(fname, MX_CT_COUNT, g_ncs, g_coms) >= 0;
    return g_rules_ok;
}

static const char *const g_coll_names[MX_CT_COUNT] = {
    [MX_CT_ALLREDUCE] = "allreduce", [MX_CT_EXSCAN] = "exscan", [MX_CT_REDUCE] = "reduce",
    [MX_CT_REDUCESCATTER] = "reduce_scatter", [MX_CT_REDUCESCATTERBLOCK] = "reduce_scatter_block",
    [MX_CT_SCAN] = "scan"};

int mx_tuned_cfg_load(mx_tuned_cfg_t *cfg, int comm_size)
{
    int rc = 0;
    memset(cfg, 0, sizeof *cfg);
    cfg->dynamic = mx_ompi_host->mca_int("coll_tuned_use_dynamic_rules", 0) != 0;
    if (!cfg->dynamic) return 0;
    for (int c = 0; c < MX_CT_COUNT; c++) {
        char v[96];
        if (!g_coll_names[c]) continue;
        snprintf(v, sizeof v, "coll_tuned_%s_algorithm", g_coll_names[c]);
        cfg->forced_alg[c] = mx_ompi_host->mca_int(v, 0);
        snprintf(v, sizeof v, "coll_tuned_%s_algorithm_chain_fanout", g_coll_names[c]);
        cfg->forced_chain[c] = mx_ompi_host->mca_int(v, 0);
        snprintf(v, sizeof v, "coll_tuned_%s_algorithm_tree_fanout", g_coll_names[c]);
        cfg->forced_tree[c] = mx_ompi_host->mca_int(v, 0);
        snprintf(v, sizeof v, "coll_tuned_%s_algorithm_segmentsize", g_coll_names[c]);
        cfg->forced_seg[c] = mx_ompi_host->mca_int(v, 0);
    }
    const char *fname = mx_ompi_host->mca_string ? mx_ompi_host->mca_string("coll_tuned_dynamic_rules_filename")
                                                 : NULL;
    if (fname && *fname) {
        if (!rules_for(fname)) return -1;
        for (int c = 0; c < MX_CT_COUNT; c++) {
            if (!g_ncs[c]) continue;
            const mx_com_rule_t *best = &g_coms[c][0];     /* the first one even if larger */
            for (int k = 0; k < g_ncs[c] && g_coms[c][k].comsize <= comm_size; k++) best = &g_coms[c][k];
            cfg->com[c] = best;
        }
    }
    return rc;
}

int mx_tuned_choice(const mx_tuned_cfg_t *cfg, int coll, size_t dsize, int *fanout)
{
    *fanout = 0;
    if (!cfg->dynamic || coll < 0 || coll >= MX_CT_COUNT) return 0;
    const mx_com_rule_t *cr = cfg->com[coll];
    if (cr && cr->nmsg > 0) {
        const mx_msg_rule_t *best = &cr->msg[0];
        for (int j = 0; j < cr->nmsg && cr->msg[j].msg_size <= dsize; j++) best = &cr->msg[j];
        if (best->alg) {
            *fanout = best->faninout;
            return best->alg;
        }
    }
    if (cfg->forced_alg[coll]) {
        *fanout = cfg->forced_chain[coll];
        return cfg->forced_alg[coll];
    }
    return 0;
}
