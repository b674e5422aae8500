/*
 * mx_oracle_coll.c -- TEST INFRASTRUCTURE ONLY.
 *
 * In-process n-rank simulator of the reference's collective algorithms
 * (ompi/mca/coll/base/coll_base_allreduce.c, coll_base_reduce_scatter.c,
 * coll_base_reduce.c, coll/tuned/coll_tuned_decision_fixed.c), used as the
 * CPU checker of libmx_kernels.so's collectives.  The reference's coll/base
 * cannot be compiled standalone (it needs mpi.h, the PML, communicators;
 * SURVEY.md 8(c)), so this file restates each algorithm step by step:
 * every rank keeps the same buffers the reference keeps (rbuf, inbuf[2],
 * tmp_buf, accumbuf, result_buf, ...), point-to-point messages are modelled
 * in lockstep rounds (a message is a snapshot of the sender's buffer at the
 * moment of the send), and every local reduction is a call of the op oracle
 * (mxo_reduce2: target = target OP source, i.e. ompi_op_reduce(op, source,
 * target)).  Floating-point results therefore follow the reference's exact
 * operation order.
 *
 * Parity of this simulator is pinned by (a) the op oracle, itself pinned to
 * the reference's compiled op kernels, and (b) the step diagrams in the
 * reference's own comments (ring allreduce :298-330, ring reduce_scatter
 * coll_base_reduce_scatter.c:420-455), checked symbolically in
 * tests/test_coll_oracle.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mx_kernels.h"

extern int mxo_reduce2(int op, int t, const void *in, void *inout, size_t n, int fortran);
extern size_t mxo_type_size(int t);

#define MAXN 64

static int g_op, g_type;
static size_t g_es;

/* Symbolic mode (tests only): elements are int64 expression ids; a reduce
 * records node (target, source) instead of computing, so the test can print
 * the exact operation tree and compare it with the reference's diagrams. */
static int g_sym;
static int64_t *g_node_t, *g_node_s;
static size_t g_nnodes, g_cap;

void mxo_sym_reset(int on)
{
    g_sym = on;
    g_nnodes = 0;
}

/* returns -1 for a leaf, else fills target/source ids of node `id` */
int mxo_sym_node(int64_t id, int64_t *target, int64_t *source)
{
    if (id < 0 || (size_t)id >= g_nnodes) return -1;
    *target = g_node_t[id];
    *source = g_node_s[id];
    return 0;
}

/* ompi_op_reduce(op, source, target, count) */
static void red(const void *source, void *target, size_t count)
{
    if (!count) return;
    if (g_sym) {
        int64_t *t = (int64_t *)target;
        const int64_t *s = (const int64_t *)source;
        for (size_t i = 0; i < count; i++) {
            if (g_nnodes == g_cap) {
                g_cap = g_cap ? 2 * g_cap : 1024;
                g_node_t = realloc(g_node_t, g_cap * sizeof(int64_t));
                g_node_s = realloc(g_node_s, g_cap * sizeof(int64_t));
            }
            g_node_t[g_nnodes] = t[i];
            g_node_s[g_nnodes] = s[i];
            t[i] = (int64_t)g_nnodes++;
        }
        return;
    }
    mxo_reduce2(g_op, g_type, source, target, count, 1);
}

static void cp(void *d, const void *s, size_t count)
{
    if (count && d != s) memmove(d, s, count * g_es);
}

#define AT(buf, i) ((char *)(buf) + (size_t)(i) * g_es)

/* COLL_BASE_COMPUTE_BLOCKCOUNT (coll_base_functions.h:428-435) */
static void blockcount(size_t count, int nb, size_t *split, size_t *early, size_t *late)
{
    *early = *late = count / nb;
    *split = count % nb;
    if (*split) *early += 1;
}
static size_t boff(size_t b, size_t split, size_t early, size_t late)
{
    return b < split ? b * early : b * late + split;
}
static size_t bcnt(size_t b, size_t split, size_t early, size_t late)
{
    return b < split ? early : late;
}

static int next_pow2_le(int n) { int p = 1; while (p * 2 <= n) p *= 2; return p; }

/* ---- recursive doubling (coll_base_allreduce.c:130-274) -------------- */
static void ar_recursive_doubling(int n, size_t count, void **rbuf)
{
    char *inpl[MAXN], *tsend[MAXN], *trecv[MAXN], *msg[MAXN];
    int newrank[MAXN];
    const int adjsize = next_pow2_le(n), extra = n - adjsize;
    for (int r = 0; r < n; r++) {
        inpl[r] = malloc(count * g_es);
        msg[r] = malloc(count * g_es);
        cp(inpl[r], rbuf[r], count);       /* inplacebuf = sbuf (sbuf == rbuf here) */
        tsend[r] = inpl[r];
        trecv[r] = rbuf[r];
    }
    /* non-power-of-two: even r < 2*extra send to r+1; odd reduce */
    for (int r = 0; r < n; r++) {
        if (r < 2 * extra) {
            if (r % 2 == 0) newrank[r] = -1;
            else {
                cp(trecv[r], tsend[r - 1], count);
                red(trecv[r], tsend[r], count);   /* tmpsend = tmpsend OP tmprecv */
                newrank[r] = r >> 1;
            }
        } else newrank[r] = r - extra;
    }
    for (int d = 1; d < adjsize; d <<= 1) {
        int remote[MAXN];
        for (int r = 0; r < n; r++) {
            if (newrank[r] < 0) continue;
            const int nr = newrank[r] ^ d;
            remote[r] = nr < extra ? nr * 2 + 1 : nr + extra;
            cp(msg[r], tsend[r], count);          /* sendrecv: snapshot of tmpsend */
        }
        for (int r = 0; r < n; r++) {
            if (newrank[r] < 0) continue;
            cp(trecv[r], msg[remote[r]], count);
            if (r < remote[r]) {
                char *sw;
                red(tsend[r], trecv[r], count);   /* tmprecv = tmprecv OP tmpsend */
                sw = trecv[r]; trecv[r] = tsend[r]; tsend[r] = sw;
            } else {
                red(trecv[r], tsend[r], count);   /* tmpsend = tmpsend OP tmprecv */
            }
        }
    }
    for (int r = 0; r < n; r++) {
        if (r < 2 * extra && r % 2 == 0) {
            cp(rbuf[r], tsend[r + 1], count);
            tsend[r] = rbuf[r];
        }
    }
    for (int r = 0; r < n; r++)
        if (tsend[r] != (char *)rbuf[r]) cp(rbuf[r], tsend[r], count);
    for (int r = 0; r < n; r++) { free(inpl[r]); free(msg[r]); }
}

/* ---- ring (coll_base_allreduce.c:341-536) ----------------------------- */
static void ar_ring(int n, size_t count, void **rbuf)
{
    size_t split, early, late;
    char *inbuf[MAXN][2], *msg[MAXN];
    int inbi = 0;
    blockcount(count, n, &split, &early, &late);
    for (int r = 0; r < n; r++) {
        inbuf[r][0] = malloc(early * g_es + 1);
        inbuf[r][1] = malloc(early * g_es + 1);
        msg[r] = malloc(early * g_es + 1);
    }
    /* send my block to r+1 into its inbuf[0] */
    for (int r = 0; r < n; r++) cp(msg[r], AT(rbuf[r], boff(r, split, early, late)), bcnt(r, split, early, late));
    for (int r = 0; r < n; r++) {
        const int from = (r + n - 1) % n;
        cp(inbuf[r][0], msg[from], bcnt(from, split, early, late));
    }
    for (int k = 2; k < n; k++) {
        inbi ^= 1;
        for (int r = 0; r < n; r++) {
            const int pb = (r + n - k + 1) % n;
            const size_t bc = bcnt(pb, split, early, late);
            char *t = AT(rbuf[r], boff(pb, split, early, late));
            red(inbuf[r][inbi ^ 1], t, bc);
            cp(msg[r], t, bc);
        }
        for (int r = 0; r < n; r++) {
            const int from = (r + n - 1) % n;
            const int pb = (from + n - k + 1) % n;
            cp(inbuf[r][inbi], msg[from], bcnt(pb, split, early, late));
        }
    }
    for (int r = 0; r < n; r++) {
        const int b = (r + 1) % n;
        red(inbuf[r][inbi], AT(rbuf[r], boff(b, split, early, late)), bcnt(b, split, early, late));
    }
    /* ring allgather */
    for (int k = 0; k < n - 1; k++) {
        for (int r = 0; r < n; r++) {
            const int sd = (r + 1 + n - k) % n;
            cp(msg[r], AT(rbuf[r], boff(sd, split, early, late)), bcnt(sd, split, early, late));
        }
        for (int r = 0; r < n; r++) {
            const int rd = (r + n - k) % n;
            cp(AT(rbuf[r], boff(rd, split, early, late)), msg[(r + n - 1) % n], bcnt(rd, split, early, late));
        }
    }
    for (int r = 0; r < n; r++) { free(inbuf[r][0]); free(inbuf[r][1]); free(msg[r]); }
}

/* ---- segmented ring (coll_base_allreduce.c:618-856) ------------------- */
static void ar_ring_segmented(int n, size_t count, void **rbuf, size_t segsize)
{
    size_t segcount = count, split, early, late, nph;
    size_t typelng = g_es;
    /* COLL_BASE_COMPUTED_SEGCOUNT (coll_base_functions.h:407-415) */
    if (segsize >= typelng && segsize < typelng * segcount) {
        size_t residual;
        segcount = segsize / typelng;
        residual = segsize - segcount * typelng;
        if (residual > (typelng >> 1)) segcount++;
    }
    if (count < (size_t)n * segcount) { ar_ring(n, count, rbuf); return; }
    nph = count / ((size_t)n * segcount);
    if ((count % ((size_t)n * segcount) >= (size_t)n) && (count % ((size_t)n * segcount) > ((size_t)n * segcount) / 2))
        nph++;
    blockcount(count, n, &split, &early, &late);
    {
        size_t maxseg, s2, l2;
        char *inbuf[MAXN][2], *msg[MAXN];
        blockcount(early, nph, &s2, &maxseg, &l2);
        for (int r = 0; r < n; r++) {
            inbuf[r][0] = malloc(maxseg * g_es + 1);
            inbuf[r][1] = malloc(maxseg * g_es + 1);
            msg[r] = malloc(early * g_es + 1);
        }
#define PHASE(b, ph, OFF, CNT)                                                  \
        do { size_t bc_ = bcnt(b, split, early, late), sp_, e_, l_;             \
             blockcount(bc_, nph, &sp_, &e_, &l_);                              \
             CNT = (ph) < sp_ ? e_ : l_;                                        \
             OFF = boff(b, split, early, late) + ((ph) < sp_ ? (ph) * e_ : (ph) * l_ + sp_); \
             (void)OFF; } while (0)
        for (size_t ph = 0; ph < nph; ph++) {
            int inbi = 0;
            for (int r = 0; r < n; r++) {
                size_t o, c;
                PHASE(r, ph, o, c);
                cp(msg[r], AT(rbuf[r], o), c);
            }
            for (int r = 0; r < n; r++) {
                size_t o, c;
                const int from = (r + n - 1) % n;
                PHASE(from, ph, o, c);
                cp(inbuf[r][0], msg[from], c);
            }
            for (int k = 2; k < n; k++) {
                inbi ^= 1;
                for (int r = 0; r < n; r++) {
                    size_t o, c;
                    const int pb = (r + n - k + 1) % n;
                    PHASE(pb, ph, o, c);
                    red(inbuf[r][inbi ^ 1], AT(rbuf[r], o), c);
                    cp(msg[r], AT(rbuf[r], o), c);
                }
                for (int r = 0; r < n; r++) {
                    size_t o, c;
                    const int from = (r + n - 1) % n, pb = (from + n - k + 1) % n;
                    PHASE(pb, ph, o, c);
                    cp(inbuf[r][inbi], msg[from], c);
                }
            }
            for (int r = 0; r < n; r++) {
                size_t o, c;
                const int b = (r + 1) % n;
                PHASE(b, ph, o, c);
                red(inbuf[r][inbi], AT(rbuf[r], o), c);
            }
        }
#undef PHASE
        for (int k = 0; k < n - 1; k++) {
            for (int r = 0; r < n; r++) {
                const int sd = (r + 1 + n - k) % n;
                cp(msg[r], AT(rbuf[r], boff(sd, split, early, late)), bcnt(sd, split, early, late));
            }
            for (int r = 0; r < n; r++) {
                const int rd = (r + n - k) % n;
                cp(AT(rbuf[r], boff(rd, split, early, late)), msg[(r + n - 1) % n], bcnt(rd, split, early, late));
            }
        }
        for (int r = 0; r < n; r++) { free(inbuf[r][0]); free(inbuf[r][1]); free(msg[r]); }
    }
}

/* ---- basic linear (coll_base_allreduce.c:881-912 -> reduce basic linear
 *      coll_base_reduce.c:627-720 to root 0, then bcast) ------------------ */
static void ar_basic_linear(int n, size_t count, void **rbuf)
{
    char *acc = malloc(count * g_es + 1);
    cp(acc, rbuf[n - 1], count);                   /* rbuf(root) = x_{n-1} */
    for (int i = n - 2; i >= 0; --i) red(rbuf[i], acc, count);   /* rbuf = rbuf OP x_i */
    for (int r = 0; r < n; r++) cp(rbuf[r], acc, count);
    free(acc);
}

/* ---- Rabenseifner (coll_base_allreduce.c:970-1243) -------------------- */
static void ar_rabenseifner(int n, size_t count, void **rbuf)
{
    int nsteps = 0;
    while ((1 << (nsteps + 1)) <= n) nsteps++;
    const int p2 = 1 << nsteps, rem = n - p2;
    if (count < (size_t)p2) { ar_basic_linear(n, count, rbuf); return; }
    char *tmp[MAXN], *snap[MAXN];
    int vrank[MAXN];
    size_t rindex[MAXN][8], sindex[MAXN][8], rcount[MAXN][8], scount[MAXN][8];
    for (int r = 0; r < n; r++) { tmp[r] = malloc(count * g_es + 1); snap[r] = malloc(count * g_es + 1); }
    /* step 1: fold the extra ranks */
    {
        const size_t lh = count / 2, rh = count - lh;
        for (int r = 0; r < n; r++) cp(snap[r], rbuf[r], count);
        for (int r = 0; r < 2 * rem; r++) {
            if (r % 2) {   /* odd: recv even's right half into tmp[lh..], reduce into rbuf[lh..] */
                cp(AT(tmp[r], lh), AT(snap[r - 1], lh), rh);
                red(AT(tmp[r], lh), AT(rbuf[r], lh), rh);
                vrank[r] = -1;
            } else {       /* even: recv odd's left half into tmp[0..lh), reduce */
                cp(tmp[r], snap[r + 1], lh);
                red(tmp[r], rbuf[r], lh);
                vrank[r] = r / 2;
            }
        }
        for (int r = 0; r < 2 * rem; r += 2) cp(AT(rbuf[r], lh), AT(rbuf[r + 1], lh), rh);
        for (int r = 2 * rem; r < n; r++) vrank[r] = r - rem;
    }
    /* step 2: reduce-scatter by recursive halving */
    {
        size_t wsize[MAXN];
        for (int r = 0; r < n; r++) { wsize[r] = count; sindex[r][0] = rindex[r][0] = 0; }
        int step = 0;
        for (int mask = 1; mask < p2; mask <<= 1) {
            int dest[MAXN];
            for (int r = 0; r < n; r++) {
                if (vrank[r] < 0) continue;
                const int vd = vrank[r] ^ mask;
                dest[r] = vd < rem ? vd * 2 : vd + rem;
                if (r < dest[r]) {
                    rcount[r][step] = wsize[r] / 2;
                    scount[r][step] = wsize[r] - rcount[r][step];
                    sindex[r][step] = rindex[r][step] + rcount[r][step];
                } else {
                    scount[r][step] = wsize[r] / 2;
                    rcount[r][step] = wsize[r] - scount[r][step];
                    rindex[r][step] = sindex[r][step] + scount[r][step];
                }
            }
            for (int r = 0; r < n; r++)
                if (vrank[r] >= 0) cp(snap[r], rbuf[r], count);
            for (int r = 0; r < n; r++) {
                if (vrank[r] < 0) continue;
                const int d = dest[r];
                /* receive d's send part into tmp at my rindex */
                cp(AT(tmp[r], rindex[r][step]), AT(snap[d], sindex[d][step]), rcount[r][step]);
                red(AT(tmp[r], rindex[r][step]), AT(rbuf[r], rindex[r][step]), rcount[r][step]);
            }
            if (step + 1 < nsteps) {
                for (int r = 0; r < n; r++) {
                    if (vrank[r] < 0) continue;
                    rindex[r][step + 1] = rindex[r][step];
                    sindex[r][step + 1] = rindex[r][step];
                    wsize[r] = rcount[r][step];
                }
                step++;
            }
        }
        /* step 3: allgather by recursive doubling */
        step = nsteps - 1;
        for (int mask = p2 >> 1; mask > 0; mask >>= 1) {
            int dest[MAXN];
            for (int r = 0; r < n; r++) {
                if (vrank[r] < 0) continue;
                const int vd = vrank[r] ^ mask;
                dest[r] = vd < rem ? vd * 2 : vd + rem;
                cp(snap[r], rbuf[r], count);
            }
            for (int r = 0; r < n; r++) {
                if (vrank[r] < 0) continue;
                const int d = dest[r];
                cp(AT(rbuf[r], sindex[r][step]), AT(snap[d], rindex[d][step]), scount[r][step]);
            }
            step--;
        }
    }
    /* step 4: send result to the excluded odd ranks */
    for (int r = 1; r < 2 * rem; r += 2) cp(rbuf[r], rbuf[r - 1], count);
    for (int r = 0; r < n; r++) { free(tmp[r]); free(snap[r]); }
}

/* ---- tuned fixed decision (coll_tuned_decision_fixed.c:44-95) ---------- */
int mxo_allreduce_decision(int n, size_t count, size_t es)
{
    const size_t block_dsize = es * count;
    if (block_dsize < 10000) return 3;
    if (count > (size_t)n) return ((size_t)n * (1u << 20) >= block_dsize) ? 4 : 5;
    return 2;
}

/* Allreduce of `count` elements on n simulated ranks.  sbufs may be NULL
 * (MPI_IN_PLACE on every rank).  Returns 0, -1 bad args, -2 unsupported. */
int mxo_reduce(int alg, int op, int type, int n, size_t count, int root, const void *const *sbufs, void *rbuf);

/* ---- nonoverlapping (coll_base_allreduce.c:54-86): comm->c_coll->coll_reduce
 * to rank 0 -- with MPI_IN_PLACE rank 0 reduces in place and the others send
 * their rbuf -- then coll_bcast from 0.  `rword` is the reduce algorithm
 * word coll_reduce runs (0 = the tuned fixed decision). */
static int ar_nonoverlapping(int rword, int op, int type, int n, size_t count, const void *const *sbufs,
                             void *const *rbufs)
{
    const void *sb[MAXN];
    for (int r = 0; r < n; r++) sb[r] = sbufs ? sbufs[r] : (r == 0 ? NULL : rbufs[r]);
    int rc = mxo_reduce(rword, op, type, n, count, 0, sb, rbufs[0]);
    if (rc) return rc;
    for (int r = 1; r < n; r++) memcpy(rbufs[r], rbufs[0], count * mxo_type_size(type));
    return 0;
}

int mxo_allreduce(int alg, int op, int type, int n, size_t count, const void *const *sbufs, void *const *rbufs)
{
    void *rb[MAXN];
    if (n < 1 || n > MAXN) return -1;
    /* algorithm word (MX_ALG_WORD): low byte algorithm, bits 8-15 the reduce
     * algorithm of nonoverlapping, bits 16-23 its chain fanout */
    const int rword = ((alg >> 8) & 0xff) | (alg & 0xff0000);
    alg &= 0xff;
    if (alg == 2 && n > 1 && count > 0) return ar_nonoverlapping(rword, op, type, n, count, sbufs, rbufs);
    g_op = op; g_type = type; g_es = mxo_type_size(type);
    if (!g_es) return -1;
    for (int r = 0; r < n; r++) {
        rb[r] = rbufs[r];
        if (sbufs && sbufs[r]) cp(rb[r], sbufs[r], count);   /* copy_content_same_ddt */
    }
    if (n == 1 || count == 0) return 0;
    if (alg == 0) alg = mxo_allreduce_decision(n, count, g_es);
    switch (alg) {
    case 1: ar_basic_linear(n, count, rb); return 0;
    case 3: ar_recursive_doubling(n, count, rb); return 0;
    case 4:
        if (count < (size_t)n) ar_recursive_doubling(n, count, rb);
        else ar_ring(n, count, rb);
        return 0;
    case 5:
        if (count < (size_t)n) { ar_recursive_doubling(n, count, rb); return 0; }
        ar_ring_segmented(n, count, rb, 1u << 20);
        return 0;
    case 6: ar_rabenseifner(n, count, rb); return 0;
    default: return -2;
    }
}

/* segmented ring with an explicit segment size (tests exercise phases) */
int mxo_allreduce_segring(int op, int type, int n, size_t count, void *const *rbufs, size_t segsize)
{
    void *rb[MAXN];
    g_op = op; g_type = type; g_es = mxo_type_size(type);
    for (int r = 0; r < n; r++) rb[r] = rbufs[r];
    if (n == 1 || count == 0) return 0;
    if (count < (size_t)n) { ar_recursive_doubling(n, count, rb); return 0; }
    ar_ring_segmented(n, count, rb, segsize);
    return 0;
}

/* ---- reduce_scatter ---------------------------------------------------- */
/* ring (coll_base_reduce_scatter.c:456-623) */
static void rs_ring(int n, const size_t *rc, char **acc, void *const *rbufs)
{
    size_t displs[MAXN], maxb = 0, total = 0;
    char *inbuf[MAXN][2], *msg[MAXN];
    int inbi = 0;
    for (int i = 0; i < n; i++) { displs[i] = total; total += rc[i]; if (rc[i] > maxb) maxb = rc[i]; }
    for (int r = 0; r < n; r++) {
        inbuf[r][0] = malloc(maxb * g_es + 1); inbuf[r][1] = malloc(maxb * g_es + 1); msg[r] = malloc(maxb * g_es + 1);
    }
    for (int r = 0; r < n; r++) {
        const int from = (r + n - 1) % n;
        cp(msg[r], AT(acc[r], displs[from]), rc[from]);
    }
    for (int r = 0; r < n; r++) {
        const int from = (r + n - 1) % n, blk = (from + n - 1) % n;
        cp(inbuf[r][0], msg[from], rc[blk]);
    }
    for (int k = 2; k < n; k++) {
        inbi ^= 1;
        for (int r = 0; r < n; r++) {
            const int pb = (r + n - k) % n;
            red(inbuf[r][inbi ^ 1], AT(acc[r], displs[pb]), rc[pb]);
            cp(msg[r], AT(acc[r], displs[pb]), rc[pb]);
        }
        for (int r = 0; r < n; r++) {
            const int from = (r + n - 1) % n, pb = (from + n - k) % n;
            cp(inbuf[r][inbi], msg[from], rc[pb]);
        }
    }
    for (int r = 0; r < n; r++) {
        red(inbuf[r][inbi], AT(acc[r], displs[r]), rc[r]);
        cp(rbufs[r], AT(acc[r], displs[r]), rc[r]);
    }
    for (int r = 0; r < n; r++) { free(inbuf[r][0]); free(inbuf[r][1]); free(msg[r]); }
}

/* basic recursive halving (coll_base_reduce_scatter.c:132-455) */
static void rs_recursive_halving(int n, const size_t *rc, char **res, void *const *rbufs)
{
    size_t disps[MAXN], total = 0;
    int tmp_rank[MAXN];
    char *recv[MAXN], *snap[MAXN];
    for (int i = 0; i < n; i++) { disps[i] = total; total += rc[i]; }
    const int tsize = next_pow2_le(n), remain = n - tsize;
    for (int r = 0; r < n; r++) { recv[r] = malloc(total * g_es + 1); snap[r] = malloc(total * g_es + 1); }
    for (int r = 0; r < n; r++) {
        if (r < 2 * remain) {
            if ((r & 1) == 0) tmp_rank[r] = -1;
            else {
                cp(recv[r], res[r - 1], total);
                red(recv[r], res[r], total);
                tmp_rank[r] = r / 2;
            }
        } else tmp_rank[r] = r - remain;
    }
    {
        size_t trc[MAXN], td[MAXN];
        int send_index[MAXN], recv_index[MAXN], last_index[MAXN];
        for (int i = 0; i < tsize; i++) trc[i] = i < remain ? rc[2 * i + 1] + rc[2 * i] : rc[i + remain];
        td[0] = 0;
        for (int i = 0; i < tsize - 1; i++) td[i + 1] = td[i] + trc[i];
        for (int r = 0; r < n; r++) { send_index[r] = recv_index[r] = 0; last_index[r] = tsize; }
        for (int mask = tsize >> 1; mask > 0; mask >>= 1) {
            int peer[MAXN];
            size_t scnt[MAXN], rcnt[MAXN];
            for (int r = 0; r < n; r++) {
                if (tmp_rank[r] < 0) continue;
                const int tp = tmp_rank[r] ^ mask;
                peer[r] = tp < remain ? tp * 2 + 1 : tp + remain;
                scnt[r] = rcnt[r] = 0;
                if (tmp_rank[r] < tp) {
                    send_index[r] = recv_index[r] + mask;
                    for (int i = send_index[r]; i < last_index[r]; i++) scnt[r] += trc[i];
                    for (int i = recv_index[r]; i < send_index[r]; i++) rcnt[r] += trc[i];
                } else {
                    recv_index[r] = send_index[r] + mask;
                    for (int i = send_index[r]; i < recv_index[r]; i++) scnt[r] += trc[i];
                    for (int i = recv_index[r]; i < last_index[r]; i++) rcnt[r] += trc[i];
                }
            }
            for (int r = 0; r < n; r++) if (tmp_rank[r] >= 0) cp(snap[r], res[r], total);
            for (int r = 0; r < n; r++) {
                if (tmp_rank[r] < 0) continue;
                const int p = peer[r];
                if (rcnt[r] > 0) {
                    /* the peer sends from its send_index, which equals my recv_index */
                    cp(AT(recv[r], td[recv_index[r]]), AT(snap[p], td[send_index[p]]), rcnt[r]);
                    red(AT(recv[r], td[recv_index[r]]), AT(res[r], td[recv_index[r]]), rcnt[r]);
                }
            }
            for (int r = 0; r < n; r++) {
                if (tmp_rank[r] < 0) continue;
                send_index[r] = recv_index[r];
                last_index[r] = recv_index[r] + mask;
            }
        }
        for (int r = 0; r < n; r++)
            if (tmp_rank[r] >= 0 && rc[r]) cp(rbufs[r], AT(res[r], disps[r]), rc[r]);
    }
    for (int r = 0; r < 2 * remain; r += 2)
        if (rc[r]) cp(rbufs[r], AT(res[r + 1], disps[r]), rc[r]);
    for (int r = 0; r < n; r++) { free(recv[r]); free(snap[r]); }
}

int mxo_reduce_scatter_decision(int n, size_t total_count, size_t es)
{
    const double a = 0.0012, b = 8.0;
    const size_t total = total_count * es;
    int pow2 = 1;
    while (pow2 < n) pow2 <<= 1;
    if (total <= 12 * 1024 || (total <= 256 * 1024 && pow2 == n) || (double)n >= a * (double)total + b) return 2;
    return 3;
}

/* butterfly (coll_base_reduce_scatter.c:691-880), restated step by step over
 * the n simulated ranks: psend/precv double buffers per rank, the sendrecv
 * of every step snapshotted before any rank reduces. */
static unsigned mirror_perm(unsigned x, int nbits)                  /* coll_base_util.c:88-96 */
{
    unsigned r = 0;
    for (int i = 0; i < nbits; i++) if (x & (1u << i)) r |= 1u << (nbits - 1 - i);
    return r;
}
static size_t sum_counts(const size_t *rc, const size_t *displs, int rem, int lo, int hi)   /* :629-635 */
{
    lo = lo < rem ? lo * 2 : lo + rem;
    hi = hi < rem ? hi * 2 + 1 : hi + rem;
    return displs[hi] + rc[hi] - displs[lo];
}
static void rs_butterfly(int n, const size_t *rc, char **work, void *const *rbufs)
{
    size_t displs[MAXN], total = 0;
    for (int i = 0; i < n; i++) { displs[i] = total; total += rc[i]; }
    const int pof2 = next_pow2_le(n), rem = n - pof2;
    int log2 = 0;
    while ((1 << log2) < pof2) log2++;
    char *buf[MAXN][2];
    int cur[MAXN], vrank[MAXN], sidx[MAXN], ridx[MAXN];
    for (int r = 0; r < n; r++) {
        buf[r][0] = malloc(total * g_es + 1);
        buf[r][1] = malloc(total * g_es + 1);
        cp(buf[r][0], work[r], total);            /* psend = copy of sbuf */
        cur[r] = 0;
        sidx[r] = ridx[r] = 0;
    }
#define PSEND(r) buf[r][cur[r]]
#define PRECV(r) buf[r][cur[r] ^ 1]
    /* step 1: even r < 2 rem send the whole vector to r+1, which reduces
     * precv into psend (:764-776) */
    for (int r = 0; r < n; r++) {
        if (r < 2 * rem) {
            if (r % 2 == 0) vrank[r] = -1;
            else {
                cp(PRECV(r), PSEND(r - 1), total);
                red(PRECV(r), PSEND(r), total);
                vrank[r] = r / 2;
            }
        } else vrank[r] = r - rem;
    }
    int nblocks = pof2;
    for (int mask = 1; mask < pof2; mask <<= 1) {
        int peer[MAXN];
        size_t scnt[MAXN], sdsp[MAXN], rcnt[MAXN], rdsp[MAXN];
        nblocks /= 2;
        for (int r = 0; r < n; r++) {
            if (vrank[r] < 0) continue;
            const int vp = vrank[r] ^ mask;
            peer[r] = vp < rem ? vp * 2 + 1 : vp + rem;
            if ((vrank[r] & mask) == 0) sidx[r] += nblocks; else ridx[r] += nblocks;
            scnt[r] = sum_counts(rc, displs, rem, sidx[r], sidx[r] + nblocks - 1);
            int ix = sidx[r] < rem ? 2 * sidx[r] : rem + sidx[r];
            sdsp[r] = displs[ix];
            rcnt[r] = sum_counts(rc, displs, rem, ridx[r], ridx[r] + nblocks - 1);
            ix = ridx[r] < rem ? 2 * ridx[r] : rem + ridx[r];
            rdsp[r] = displs[ix];
        }
        /* sendrecv: every rank receives its peer's send part into precv at
         * its own rdispl (the peer's sdispl), before anyone reduces */
        for (int r = 0; r < n; r++) {
            if (vrank[r] < 0) continue;
            const int p = peer[r];
            if (scnt[p] != rcnt[r] || sdsp[p] != rdsp[r]) abort();   /* the peer sends what I receive */
            cp(AT(PRECV(r), rdsp[r]), AT(PSEND(p), sdsp[p]), rcnt[r]);
        }
        for (int r = 0; r < n; r++) {
            if (vrank[r] < 0) continue;
            const int vp = vrank[r] ^ mask;
            if (vrank[r] < vp) {                      /* precv = psend OP precv; swap */
                red(AT(PSEND(r), rdsp[r]), AT(PRECV(r), rdsp[r]), rcnt[r]);
                cur[r] ^= 1;
            } else {                                  /* psend = precv OP psend */
                red(AT(PRECV(r), rdsp[r]), AT(PSEND(r), rdsp[r]), rcnt[r]);
            }
            sidx[r] = ridx[r];
        }
    }
    /* mirror-permutation exchange of the result blocks (:846-887) */
    for (int r = 0; r < n; r++) {
        if (vrank[r] < 0) continue;
        const int vp = (int)mirror_perm((unsigned)vrank[r], log2);
        const int peer = vp < rem ? vp * 2 + 1 : vp + rem;
        int ix = sidx[r] < rem ? 2 * sidx[r] : rem + sidx[r];
        if (vp < rem) {                               /* first block to the excluded even rank */
            if (rc[peer - 1]) cp(rbufs[peer - 1], AT(PSEND(r), displs[ix]), rc[ix]);
            ix++;
        }
        if (rc[peer]) cp(rbufs[peer], AT(PSEND(r), displs[ix]), rc[ix]);
    }
#undef PSEND
#undef PRECV
    for (int r = 0; r < n; r++) { free(buf[r][0]); free(buf[r][1]); }
}

/* reduce_scatter NONOVERLAPPING (coll_base_reduce_scatter.c:47-110):
 * coll_reduce of the whole vector to rank 0 (MPI_IN_PLACE: the root reduces
 * in place), then scatterv */
static int rs_nonoverlapping(int rword, int op, int type, int n, const size_t *rc, const void *const *sbufs,
                             void *const *rbufs)
{
    size_t total = 0, es = mxo_type_size(type);
    for (int i = 0; i < n; i++) total += rc[i];
    const void *sb[MAXN];
    for (int r = 0; r < n; r++) sb[r] = sbufs ? sbufs[r] : (r == 0 ? NULL : rbufs[r]);
    char *full = malloc(total * es + 1);
    if (!sbufs) memcpy(full, rbufs[0], total * es);   /* the root's in-place data */
    int rc0 = mxo_reduce(rword, op, type, n, total, 0, sb, full);
    size_t d = 0;
    for (int r = 0; r < n && !rc0; r++) { memcpy(rbufs[r], full + d * es, rc[r] * es); d += rc[r]; }
    free(full);
    return rc0;
}

/* alg word: low byte 0 auto, 1 nonoverlapping (bits 8-23: its reduce word),
 * 2 recursive halving, 3 ring, 4 butterfly.  sbufs NULL = MPI_IN_PLACE
 * (rbufs hold the full vectors). */
int mxo_reduce_scatter(int alg, int op, int type, int n, const size_t *rcounts, const void *const *sbufs,
                       void *const *rbufs)
{
    size_t total = 0;
    char *work[MAXN];
    if (n < 1 || n > MAXN) return -1;
    const int rword = ((alg >> 8) & 0xff) | (alg & 0xff0000);
    alg &= 0xff;
    g_op = op; g_type = type; g_es = mxo_type_size(type);
    for (int i = 0; i < n; i++) total += rcounts[i];
    if (alg == 1 && n > 1) return rs_nonoverlapping(rword, op, type, n, rcounts, sbufs, rbufs);
    for (int r = 0; r < n; r++) {
        work[r] = malloc(total * g_es + 1);
        cp(work[r], sbufs ? sbufs[r] : rbufs[r], total);
    }
    if (n == 1) { cp(rbufs[0], work[0], total); free(work[0]); return 0; }
    if (alg == 0) alg = mxo_reduce_scatter_decision(n, total, g_es);
    if (alg == 3) rs_ring(n, rcounts, work, rbufs);
    else if (alg == 2) rs_recursive_halving(n, rcounts, work, rbufs);
    else if (alg == 4) rs_butterfly(n, rcounts, work, rbufs);
    else { for (int r = 0; r < n; r++) free(work[r]); return -2; }
    for (int r = 0; r < n; r++) free(work[r]);
    return 0;
}

/* ======================================================================
 * Rooted reduce, scan, exscan, reduce_scatter_block (TEST INFRASTRUCTURE)
 * ====================================================================== */

/* ---- topology (coll_base_topo.c), restated ------------------------------ */
typedef struct { int nnext; int next[MAXN]; } otree_t;

static int o_pown(int fanout, int num)                    /* :34-46 */
{
    int p = 1;
    if (num < 0) return 0;
    if (num == 1) return fanout;
    if (fanout == 2) return p << num;
    for (int j = 0; j < num; j++) p *= fanout;
    return p;
}
static int o_level(int fanout, int rank)                  /* :48-56 */
{
    int level, num;
    if (rank < 0) return -1;
    for (level = 0, num = 0; num <= rank; level++) num += o_pown(fanout, level);
    return level - 1;
}
static void o_tree(int fanout, int size, int root, int rank, otree_t *t)   /* build_tree :78-175 */
{
    int shiftedrank, level, delta;
    t->nnext = 0;
    if (size < 2) return;
    shiftedrank = rank - root;
    if (shiftedrank < 0) shiftedrank += size;
    level = o_level(fanout, shiftedrank);
    delta = o_pown(fanout, level);
    for (int i = 0; i < fanout; i++) {
        int schild = shiftedrank + delta * (i + 1);
        if (schild < size) t->next[t->nnext++] = (schild + root) % size;
        else break;
    }
}
static void o_in_order_bmtree(int size, int root, int rank, otree_t *t)   /* :403-458 */
{
    int vrank = (rank - root + size) % size, mask = 1;
    t->nnext = 0;
    while (mask < size) {
        int remote = vrank ^ mask;
        if (remote < vrank) break;
        else if (remote < size) t->next[t->nnext++] = (remote + root) % size;
        mask <<= 1;
    }
}
static void o_chain(int fanout, int size, int root, int rank, otree_t *t)  /* build_chain :531-673 */
{
    int maxchainlen, mark, head, len, srank;
    if (fanout < 1) fanout = 1;
    if (fanout > 32) fanout = 32;
    t->nnext = 0;
    if ((size - 1) < fanout) fanout = size - 1;
    srank = rank - root;
    if (srank < 0) srank += size;
    if (fanout == 1) {
        if (srank + 1 < size) t->next[t->nnext++] = (srank + 1 + root) % size;
        return;
    }
    if (size == 1 || fanout < 1) return;
    maxchainlen = (size - 1) / fanout;
    if ((size - 1) % fanout != 0) { maxchainlen++; mark = (size - 1) % fanout; }
    else mark = fanout + 1;
    if (srank != 0) {
        if (srank - 1 < mark * maxchainlen) {
            int column = (srank - 1) / maxchainlen;
            head = 1 + column * maxchainlen;
            len = maxchainlen;
        } else {
            int column = mark + (srank - 1 - mark * maxchainlen) / (maxchainlen - 1);
            head = mark * maxchainlen + 1 + (column - mark) * (maxchainlen - 1);
            len = maxchainlen - 1;
        }
        if (srank != head + len - 1 && srank + 1 < size) t->next[t->nnext++] = (srank + 1 + root) % size;
    } else {
        t->next[0] = (root + 1) % size;
        for (int i = 1; i < fanout; i++) {
            t->next[i] = t->next[i - 1] + maxchainlen;
            if (i > mark) t->next[i]--;
            t->next[i] %= size;
        }
        t->nnext = fanout;
    }
}
static void o_in_order_bintree(int size, int rank, otree_t *t)            /* :192-295 */
{
    int myrank = rank, parent = size - 1, delta = 0, rightsize, lchild, rchild;
    int n0 = -1, n1 = -1;
    while (1) {
        rightsize = size >> 1;
        lchild = -1;
        rchild = -1;
        if (size - 1 > 0) {
            lchild = parent - 1;
            if (lchild > 0) rchild = rightsize - 1;
        }
        if (myrank == parent) {
            if (lchild >= 0) n0 = lchild + delta;
            if (rchild >= 0) n1 = rchild + delta;
            break;
        }
        if (myrank > rchild) {
            size = size - rightsize - 1;
            delta = delta + rightsize;
            myrank = myrank - rightsize;
            parent = size - 1;
        } else {
            size = rightsize;
            parent = rchild;
        }
    }
    t->nnext = 0;
    if (n0 >= 0) t->next[t->nnext++] = n0;
    if (n1 >= 0) t->next[t->nnext++] = n1;
}

/* tuned fixed reduce decision (coll_tuned_decision_fixed.c:354-429) ->
 * algorithm id and segment size */
int mxo_reduce_decision(int n, size_t count, size_t es, int *segsize)
{
    const double a1 = 0.6016 / 1024.0, b1 = 1.3496, a2 = 0.0410 / 1024.0, b2 = 9.7128;
    const double a3 = 0.0422 / 1024.0, b3 = 1.1614, a4 = 0.0033 / 1024.0, b4 = 1.6761;
    const size_t message_size = es * count;
    int seg = 0, alg;
    if (n < 8 && message_size < 512) alg = 1;
    else if ((n < 8 && message_size < 20480) || message_size < 2048 || count <= 1) { alg = 5; seg = 0; }
    else if (n > a1 * (double)message_size + b1) { alg = 5; seg = 1024; }
    else if (n > a2 * (double)message_size + b2) { alg = 3; seg = 1024; }
    else if (n > a3 * (double)message_size + b3) { alg = 4; seg = 32 * 1024; }
    else { alg = 3; seg = (n > a4 * (double)message_size + b4) ? 32 * 1024 : 64 * 1024; }
    if (segsize) *segsize = seg;
    return alg;
}

/* ompi_coll_base_reduce_generic (coll_base_reduce.c:62-370), commutative
 * op, over the tree of `kind`.  Ranks are processed children-first; a
 * "message" from a child for segment s is the child's accumulator (or, for a
 * leaf, its sendbuf) for that segment after the child finished it. */
static int g_tree_kind, g_tree_fanout;
static void o_tree_of(int n, int root, int rank, otree_t *t)
{
    switch (g_tree_kind) {
    case 2: o_chain(g_tree_fanout, n, root, rank, t); break;
    case 3: o_chain(1, n, root, rank, t); break;
    case 4: o_tree(2, n, root, rank, t); break;
    case 5: o_in_order_bmtree(n, root, rank, t); break;
    case 6: o_in_order_bintree(n, rank, t); break;
    default: t->nnext = 0;
    }
}

static char *rg_out[MAXN];     /* what rank r sends to its parent */
static char *rg_free[MAXN];

static void rg_rank(int r, int n, int root, size_t count, size_t segcount, char *const *sendbuf, char *recvbuf,
                    int inplace_root)
{
    otree_t t;
    o_tree_of(n, root, r, &t);
    for (int i = 0; i < t.nnext; i++) rg_rank(t.next[i], n, root, count, segcount, sendbuf, recvbuf, inplace_root);
    if (t.nnext == 0) { rg_out[r] = sendbuf[r]; return; }     /* leaf: sends sendbuf segments */
    char *accum = (r == root && recvbuf) ? recvbuf : (rg_free[r] = malloc(count * g_es + 1));
    char *sendtmp = (r == root && inplace_root) ? recvbuf : sendbuf[r];
    const int role_inplace = (r == root && inplace_root);
    const size_t nseg = (count + segcount - 1) / segcount;
    for (size_t s = 0; s < nseg; s++) {
        const size_t o = s * segcount, cnt = (s == nseg - 1) ? count - o : segcount;
        if (!role_inplace) {
            cp(AT(accum, o), AT(rg_out[t.next[0]], o), cnt);          /* irecv child 0 into accumbuf */
            red(AT(sendtmp, o), AT(accum, o), cnt);                     /* own data onto it (:196-215) */
            for (int i = 1; i < t.nnext; i++) red(AT(rg_out[t.next[i]], o), AT(accum, o), cnt);
        } else {                                                        /* accumbuf = recvbuf = own data */
            for (int i = 0; i < t.nnext; i++) red(AT(rg_out[t.next[i]], o), AT(accum, o), cnt);
        }
    }
    rg_out[r] = accum;
}

/* reduce_intra_basic_linear (:626-735) */
static void reduce_linear(int n, size_t count, char *const *sendbuf, char *rbuf)
{
    cp(rbuf, sendbuf[n - 1], count);                                   /* from rank size-1 */
    for (int i = n - 2; i >= 0; --i) red(sendbuf[i], rbuf, count);
}

/* MPI_Reduce of `count` elements on n simulated ranks.  sbufs[r] may be NULL
 * only for r == root (MPI_IN_PLACE: the root's data is in rbuf).  alg ids:
 * 0 tuned decision, 1 linear, 2 chain (fanout 4 unless bits 16-23 give
 * another), 3 pipeline, 4 binary, 5 binomial, 6 in-order binary. */
int mxo_reduce(int alg, int op, int type, int n, size_t count, int root, const void *const *sbufs, void *rbuf)
{
    char *sb[MAXN];
    int segsize = 0, inplace;
    /* algorithm word (include/mx_coll.h MX_ALG_WORD): bits 16-23 carry the
     * chain fanout (coll_tuned_reduce_algorithm_chain_fanout), 0 = 4 */
    const int fanout = (alg >> 16) & 0xff;
    alg &= 0xff;
    if (n < 1 || n > MAXN || root < 0 || root >= n || !rbuf) return -1;
    g_op = op; g_type = type; g_es = mxo_type_size(type);
    if (!g_es) return -1;
    inplace = !sbufs[root];
    for (int r = 0; r < n; r++) sb[r] = (char *)(sbufs[r] ? sbufs[r] : rbuf);
    if (count == 0) return 0;
    if (n == 1) { if (!inplace) cp(rbuf, sb[0], count); return 0; }
    if (alg == 0) alg = mxo_reduce_decision(n, count, g_es, &segsize);
    else segsize = 0;
    size_t segcount = count;
    if ((size_t)segsize >= g_es && (size_t)segsize < g_es * segcount) {   /* COMPUTED_SEGCOUNT */
        segcount = segsize / g_es;
        if (segsize - segcount * g_es > (g_es >> 1)) segcount++;
    }
    if (alg == 1) {
        if (inplace) {                                                  /* rbuf = temp, copied back */
            char *tmp = malloc(count * g_es + 1);
            reduce_linear(n, count, sb, tmp);
            cp(rbuf, tmp, count);
            free(tmp);
        } else {
            reduce_linear(n, count, sb, rbuf);
        }
        return 0;
    }
    if (alg < 2 || alg > 6) return -2;
    g_tree_kind = alg;
    g_tree_fanout = fanout ? fanout : 4;                                /* ompi_coll_tuned_init_chain_fanout */
    memset(rg_free, 0, sizeof rg_free);
    if (alg == 6) {
        /* in-order binary (:509-605): generic rooted at io_root = n-1 */
        const int io_root = n - 1;
        char *tmp_send = NULL, *tmp_recv = NULL, *io_recv = (char *)rbuf;
        int io_inplace = inplace;
        if (io_root != root) {
            if (inplace) {                                              /* root: copy rbuf to a temp sendbuf */
                tmp_send = malloc(count * g_es + 1);
                cp(tmp_send, rbuf, count);
                sb[root] = tmp_send;
                io_inplace = 0;
            }
            tmp_recv = malloc(count * g_es + 1);                        /* io_root's temporary recvbuf */
            io_recv = tmp_recv;
        }
        rg_rank(io_root, n, io_root, count, segcount, sb, io_recv, io_inplace);
        if (io_root != root) cp(rbuf, io_recv, count);                  /* io_root sends the result to root */
        free(tmp_send);
        free(tmp_recv);
    } else {
        rg_rank(root, n, root, count, segcount, sb, (char *)rbuf, inplace);
    }
    for (int r = 0; r < n; r++) free(rg_free[r]);
    return 0;
}

/* scan / exscan (coll_base_scan.c, coll_base_exscan.c), alg 0/1 linear,
 * 2 recursive doubling.  sbufs NULL = MPI_IN_PLACE everywhere. */
static int scan_common(int alg, int op, int type, int n, size_t count, const void *const *sbufs, void *const *rbufs,
                       int exclusive)
{
    char *sb[MAXN];
    if (n < 1 || n > MAXN) return -1;
    g_op = op; g_type = type; g_es = mxo_type_size(type);
    if (!g_es) return -1;
    for (int r = 0; r < n; r++) sb[r] = (char *)((sbufs && sbufs[r]) ? sbufs[r] : rbufs[r]);
    if (count == 0) return 0;
    if (alg == 0 || alg == 1) {
        if (!exclusive) {
            /* rank 0 copies; rank r copies sbuf into rbuf, receives rank r-1's
             * rbuf and reduces it in (target = own rbuf) (:51-109) */
            for (int r = 0; r < n; r++) {
                if (sb[r] != (char *)rbufs[r]) cp(rbufs[r], sb[r], count);
                if (r > 0) red(rbufs[r - 1], rbufs[r], count);
            }
        } else {
            /* rank r receives rank r-1's reduce_buffer into rbuf; sends
             * reduce_buffer = sbuf op rbuf (target = own copy) (:57-100) */
            char *rb_prev = malloc(count * g_es + 1), *rbuf_tmp = malloc(count * g_es + 1);
            cp(rb_prev, sb[0], count);                                  /* rank 0 sends its sbuf */
            for (int r = 1; r < n; r++) {
                cp(rbuf_tmp, rb_prev, count);                           /* what rank r receives */
                if (r < n - 1) {
                    char *reduce_buffer = malloc(count * g_es + 1);
                    cp(reduce_buffer, sb[r], count);
                    red(rbuf_tmp, reduce_buffer, count);
                    cp(rb_prev, reduce_buffer, count);
                    free(reduce_buffer);
                }
                cp(rbufs[r], rbuf_tmp, count);
            }
            free(rb_prev);
            free(rbuf_tmp);
        }
        return 0;
    }
    if (alg != 2) return -2;
    {
        char *psend[MAXN], *precv[MAXN], *rb[MAXN];
        int first[MAXN];
        for (int r = 0; r < n; r++) {
            psend[r] = malloc(count * g_es + 1);
            precv[r] = malloc(count * g_es + 1);
            rb[r] = malloc(count * g_es + 1);
            cp(psend[r], sb[r], count);                                 /* exscan :169-175 / scan :173-191 */
            cp(rb[r], sb[r], count);
            first[r] = 1;
        }
        for (int mask = 1; mask < n; mask <<= 1) {
            for (int r = 0; r < n; r++) {                               /* sendrecv: snapshot */
                int remote = r ^ mask;
                if (remote < n) cp(precv[r], psend[remote], count);
            }
            for (int r = 0; r < n; r++) {
                int remote = r ^ mask;
                if (remote >= n) continue;
                if (r > remote) {
                    if (exclusive && first[r]) { cp(rb[r], precv[r], count); first[r] = 0; }
                    else red(precv[r], rb[r], count);                   /* recvbuf = precv op recvbuf */
                    red(precv[r], psend[r], count);
                } else {
                    red(precv[r], psend[r], count);                     /* commutative branch */
                }
            }
        }
        for (int r = exclusive ? 1 : 0; r < n; r++) cp(rbufs[r], rb[r], count);
        for (int r = 0; r < n; r++) { free(psend[r]); free(precv[r]); free(rb[r]); }
    }
    return 0;
}

int mxo_scan(int alg, int op, int type, int n, size_t count, const void *const *sbufs, void *const *rbufs)
{
    return scan_common(alg, op, type, n, count, sbufs, rbufs, 0);
}

int mxo_exscan(int alg, int op, int type, int n, size_t count, const void *const *sbufs, void *const *rbufs)
{
    return scan_common(alg, op, type, n, count, sbufs, rbufs, 1);
}

/* reduce_scatter_block basic_linear (coll_base_reduce_scatter_block.c:55-110):
 * coll_reduce to rank 0 (tuned reduce decision on rcount*n; `alg` forces the
 * reduce algorithm) then a linear scatter.  sbufs NULL = MPI_IN_PLACE. */
int mxo_reduce_scatter_block(int alg, int op, int type, int n, size_t rcount, const void *const *sbufs,
                             void *const *rbufs)
{
    const void *sb[MAXN];
    size_t es = mxo_type_size(type);
    if (n < 1 || n > MAXN || !es) return -1;
    if (rcount == 0) return 0;
    for (int r = 0; r < n; r++) sb[r] = (sbufs && sbufs[r]) ? sbufs[r] : rbufs[r];
    char *full = malloc(rcount * n * es + 1);
    int rc = mxo_reduce(alg, op, type, n, rcount * n, 0, sb, full);
    if (rc == 0)
        for (int r = 0; r < n; r++) memcpy(rbufs[r], full + (size_t)r * rcount * es, rcount * es);
    free(full);
    return rc;
}

/* children of `rank` in the tree of a reduce algorithm (tests print trees) */
int mxo_reduce_tree(int kind, int n, int root, int rank, int *children)
{
    otree_t t;
    g_tree_kind = kind;
    g_tree_fanout = 4;
    o_tree_of(n, root, rank, &t);
    for (int i = 0; i < t.nnext; i++) children[i] = t.next[i];
    return t.nnext;
}

/* ========================================================================
 * coll/libnbc schedules -- what MPI_I<coll> and MPI_<Coll>_init compute
 * (ompi/mca/coll/libnbc).  Same lockstep model; every NBC_Sched_op(buf1,
 * buf2) executes ompi_op_reduce(op, buf1, buf2) (nbc.c:523): buf2 is the
 * target.
 * ======================================================================== */
#include <math.h>
#define NBC_LOG2 0.69314718055994530941     /* nbc_internal.h:54 */

static int nbc_maxr(int p) { return (int)ceil(log((double)p) / NBC_LOG2); }
/* RANK2VRANK / VRANK2RANK (nbc_iallreduce.c:353-364): 0 <-> root */
static int nbc_swap(int v, int root) { return v == 0 ? root : (v == root ? 0 : v); }
static int nbc_pof2(int p) { int q = 1; while (q * 2 <= p) q *= 2; return q; }   /* opal_next_poweroftwo(p) >> 1 */

/* Reduction half of allred_sched_diss (nbc_iallreduce.c:365-424),
 * red_sched_binomial (nbc_ireduce.c:356-445) and ireduce_scatter(_block)
 * (nbc_ireduce_scatter.c:103-150): in round r a vrank with v % 2^r == 0
 * receives the partner's current buffer into rbuf and computes
 * rbuf = own OP rbuf (NBC_Sched_op(sendbuf|lbuf, rbuf)), then swaps lbuf and
 * rbuf; the other vranks send their current buffer and leave.  `x` is
 * indexed by real rank; the result is vrank 0's buffer. */
static void nbc_binomial(int n, int vroot, size_t count, char *const *x, char *out)
{
    char *cur[MAXN], *msg[MAXN];
    int left[MAXN];
    const int maxr = nbc_maxr(n);
    for (int v = 0; v < n; v++) {
        cur[v] = malloc(count * g_es + 1);
        msg[v] = malloc(count * g_es + 1);
        cp(cur[v], x[nbc_swap(v, vroot)], count);
        left[v] = 0;
    }
    for (int r = 1; r <= maxr; r++) {
        for (int v = 0; v < n; v++)                       /* this round's senders */
            if (!left[v] && v % (1 << r) != 0) { cp(msg[v], cur[v], count); left[v] = 1; }
        for (int v = 0; v < n; v++) {
            if (left[v] || v % (1 << r) != 0) continue;
            const int vp = v + (1 << (r - 1));
            if (nbc_swap(vp, vroot) >= n) continue;        /* peer < p (:393) */
            char *rb = msg[vp];
            red(cur[v], rb, count);                         /* rbuf = own OP rbuf */
            msg[vp] = cur[v];                               /* swap left and right buffers */
            cur[v] = rb;
        }
    }
    cp(out, cur[0], count);
    for (int v = 0; v < n; v++) { free(cur[v]); free(msg[v]); }
}

/* allred_sched_ring (nbc_iallreduce.c:629-860).  segsize = ceil(count/p);
 * rounds 0..p-2: rank r sends segment (r+1-round) (round 0 from sendbuf,
 * then from recvbuf) to r+1, receives segment (r-round) from r-1 into
 * recvbuf and reduces recvbuf = sendbuf OP recvbuf; rounds p-1..2p-3 pass
 * the finished segments on. */
static void nbc_ring(int p, size_t count, char *const *sbuf, void *const *rbuf)
{
    size_t segsize = (count + p - 1) / p, segsizes[MAXN], segoffsets[MAXN];
    char *msg[MAXN];
    long mycount = (long)count;
    segoffsets[0] = 0;
    for (int i = 0; i < p; i++) {
        mycount -= (long)segsize;
        segsizes[i] = segsize;
        if (mycount < 0) { segsizes[i] = (size_t)((long)segsize + mycount); mycount = 0; }
        if (i) segoffsets[i] = segoffsets[i - 1] + segsizes[i - 1];
    }
    for (int r = 0; r < p; r++) msg[r] = malloc(segsize * g_es + 1);
    for (int round = 0; round < 2 * p - 2; round++) {
        for (int r = 0; r < p; r++) {
            const int se = (r + 1 - round + 2 * p) % p;
            const char *from = round == 0 ? sbuf[r] : (const char *)rbuf[r];
            cp(msg[r], AT(from, segoffsets[se]), segsizes[se]);
        }
        for (int r = 0; r < p; r++) {
            const int re = (r - round + 2 * p) % p, from = (r - 1 + p) % p;
            cp(AT(rbuf[r], segoffsets[re]), msg[from], segsizes[re]);
            if (round < p - 1) red(AT(sbuf[r], segoffsets[re]), AT(rbuf[r], segoffsets[re]), segsizes[re]);
        }
    }
    for (int r = 0; r < p; r++) free(msg[r]);
}

/* libnbc default iallreduce rule (nbc_iallreduce.c:113-121), commutative ops */
int mxo_iallreduce_decision(int n, size_t count, size_t es, int inplace)
{
    if (n < 4 || es * count < 65536 || inplace) return 2;
    if (count >= (size_t)nbc_pof2(n)) return 3;
    return 1;
}

/* MPI_Iallreduce on n simulated ranks; sbufs NULL = MPI_IN_PLACE.  alg:
 * 0 libnbc rule, 1 ring, 2 binomial, 3 Rabenseifner, 4 recursive doubling.
 * allred_sched_redscat_allgather (:976-1180) and
 * allred_sched_recursivedoubling (:512-625) are step for step coll/base's
 * (coll_base_allreduce.c:970-1243, :130-274), simulated above.  libnbc's
 * ring is not in-place safe (round 0 receives over the input when
 * sendbuf == recvbuf); here in-place ring reads the input from a copy. */
int mxo_iallreduce(int alg, int op, int type, int n, size_t count, const void *const *sbufs, void *const *rbufs)
{
    void *rb[MAXN];
    char *sb[MAXN], *tmp[MAXN] = {0};
    const int inplace = !sbufs;
    if (n < 1 || n > MAXN) return -1;
    g_op = op; g_type = type; g_es = mxo_type_size(type);
    if (!g_es) return -1;
    for (int r = 0; r < n; r++) rb[r] = rbufs[r];
    if (count == 0) return 0;
    if (n == 1) { if (!inplace) cp(rb[0], sbufs[0], count); return 0; }
    if (alg == 0) alg = mxo_iallreduce_decision(n, count, g_es, inplace);
    if (alg == 3 && count < (size_t)nbc_pof2(n)) alg = 1;             /* :121-124 */
    if (alg < 1 || alg > 4) alg = 1;
    for (int r = 0; r < n; r++) {
        if (inplace) { tmp[r] = malloc(count * g_es + 1); cp(tmp[r], rb[r], count); sb[r] = tmp[r]; }
        else sb[r] = (char *)sbufs[r];
    }
    switch (alg) {
    case 1: nbc_ring(n, count, sb, rb); break;
    case 2: {
        char *out = malloc(count * g_es + 1);
        nbc_binomial(n, 0, count, sb, out);
        for (int r = 0; r < n; r++) cp(rb[r], out, count);             /* bcast half (:426-455) */
        free(out);
        break;
    }
    case 3:
        for (int r = 0; r < n; r++) cp(rb[r], sb[r], count);           /* NBC_Sched_copy(sbuf, rbuf) */
        ar_rabenseifner(n, count, rb);
        break;
    case 4:
        for (int r = 0; r < n; r++) cp(rb[r], sb[r], count);
        ar_recursive_doubling(n, count, rb);
        break;
    }
    for (int r = 0; r < n; r++) free(tmp[r]);
    return 0;
}

/* libnbc default ireduce rule (nbc_ireduce.c:107-116), commutative ops */
int mxo_ireduce_decision(int n, size_t count, size_t es)
{
    if (n > 2 && count >= (size_t)nbc_pof2(n)) return 3;
    if (n > 4 || es * count < 65536) return 2;
    return 1;
}

/* red_sched_chain (nbc_ireduce.c:461-536): vrank p-1 sends its sendbuf to
 * p-2; every vrank receives the partial result into tmp and computes
 * tmp = sendbuf OP tmp; the root (vrank 0) computes recvbuf = sendbuf OP
 * recvbuf, or -- MPI_IN_PLACE, sendbuf == recvbuf -- recvbuf = tmp OP recvbuf.
 * Fragmentation (:474-485) splits elements, not the per-element order. */
static void nbc_chain(int n, int root, size_t count, char *const *x, char *rbuf, int inplace)
{
    char *acc = malloc(count * g_es + 1), *tmp = malloc(count * g_es + 1);
    cp(acc, x[nbc_swap(n - 1, root)], count);
    for (int v = n - 2; v >= 1; v--) {
        cp(tmp, acc, count);                                         /* recv into tmp */
        red(x[nbc_swap(v, root)], tmp, count);
        cp(acc, tmp, count);
    }
    if (inplace) {
        red(acc, rbuf, count);                                       /* recvbuf = tmp OP recvbuf */
    } else {
        cp(rbuf, acc, count);
        red(x[root], rbuf, count);                                   /* recvbuf = sendbuf OP recvbuf */
    }
    free(acc);
    free(tmp);
}

/* MPI_Ireduce: sbufs[root] NULL = MPI_IN_PLACE on the root.  alg: 0 libnbc
 * rule, 1 chain, 2 binomial, 3 Rabenseifner (red_sched_redscat_gather
 * :649-: steps 1-2 are the allreduce's reduce-scatter, then a gather). */
int mxo_ireduce(int alg, int op, int type, int n, size_t count, int root, const void *const *sbufs, void *rbuf)
{
    char *sb[MAXN];
    if (n < 1 || n > MAXN || root < 0 || root >= n || !rbuf) return -1;
    g_op = op; g_type = type; g_es = mxo_type_size(type);
    if (!g_es) return -1;
    const int inplace = !sbufs[root];
    for (int r = 0; r < n; r++) sb[r] = (char *)(sbufs[r] ? sbufs[r] : rbuf);
    if (count == 0) return 0;
    if (n == 1) { if (!inplace) cp(rbuf, sb[0], count); return 0; }
    if (alg == 0) alg = mxo_ireduce_decision(n, count, g_es);
    else if (alg == 3 && !(n > 2 && count >= (size_t)nbc_pof2(n))) alg = 1;   /* :121-125 */
    else if (alg != 2 && alg != 3) alg = 1;
    if (alg == 1) {
        if (inplace) nbc_chain(n, root, count, sb, rbuf, 1);
        else nbc_chain(n, root, count, sb, rbuf, 0);
        return 0;
    }
    if (alg == 2) {
        char *in_copy = NULL;
        if (inplace) { in_copy = malloc(count * g_es + 1); cp(in_copy, rbuf, count); sb[root] = in_copy; }
        nbc_binomial(n, root, count, sb, rbuf);
        free(in_copy);
        return 0;
    }
    {
        void *rb[MAXN];
        char *all = malloc((size_t)n * count * g_es + 1);
        for (int r = 0; r < n; r++) { rb[r] = all + (size_t)r * count * g_es; cp(rb[r], sb[r], count); }
        ar_rabenseifner(n, count, rb);
        cp(rbuf, rb[root], count);
        free(all);
    }
    return 0;
}

/* MPI_Ireduce_scatter (nbc_ireduce_scatter.c:103-186) and
 * MPI_Ireduce_scatter_block: binomial reduction to rank 0, then rank 0
 * scatters the blocks.  sbufs NULL = MPI_IN_PLACE. */
int mxo_ireduce_scatter(int op, int type, int n, const size_t *rcounts, const void *const *sbufs, void *const *rbufs)
{
    char *sb[MAXN];
    size_t total = 0;
    if (n < 1 || n > MAXN) return -1;
    g_op = op; g_type = type; g_es = mxo_type_size(type);
    if (!g_es) return -1;
    for (int r = 0; r < n; r++) total += rcounts[r];
    if (total == 0) return 0;
    char *full = malloc(total * g_es + 1), *copies = malloc((size_t)n * total * g_es + 1);
    for (int r = 0; r < n; r++) {
        sb[r] = copies + (size_t)r * total * g_es;
        cp(sb[r], (sbufs && sbufs[r]) ? sbufs[r] : rbufs[r], total);
    }
    nbc_binomial(n, 0, total, sb, full);
    for (int r = 0, off = 0; r < n; off += (int)rcounts[r], r++) cp(rbufs[r], AT(full, off), rcounts[r]);
    free(full);
    free(copies);
    return 0;
}

/* ========================================================================
 * OpenSHMEM scoll/basic reduce, recursive doubling -- the module's default
 * (mca_scoll_basic_param_reduce_algorithm = SCOLL_ALG_REDUCE_RECURSIVE_
 * DOUBLING, scoll_basic_component.c:35), restated step by step from
 * _algorithm_recursive_doubling (scoll_basic_reduce.c:374-542):
 *   floor2_proc: :392-398;  target_cur = copy of source: :400-405;
 *   extra PE (my_id >= floor2) puts target_cur into its partner's target
 *   and waits: :413-440;  partner folds it: :441-465,
 *     op->o_func.c_fn(target, target_cur, n)  (in = received, out = own);
 *   pairwise rounds peer = my_id ^ (1 << round) while exit_flag
 *   (floor2 - 1 >> per round): :467-507, each PE folding the partner's
 *   target_cur (put into its target) into its own target_cur;
 *   memcpy(target, target_cur) and the extra gets the same: :509-528.
 * oshmem's c_fn is *out = calc(*out, *in) (oshmem/op/op.c:165-178), i.e.
 * ompi_op_reduce(op, source = received, target = own) -- the MPI op's
 * operand roles -- so red() evaluates it with the op restatement.  Rounds
 * exchange the values of the previous round (every put precedes its
 * partner's fold).  sbufs NULL: MPI-style in place (target holds the input).
 * ======================================================================== */
int mxo_shmem_basic_reduce(int op, int type, int n, size_t count, const void *const *sbufs, void *const *rbufs)
{
    if (n < 1 || n > MAXN) return -1;
    g_op = op; g_type = type; g_es = mxo_type_size(type);
    if (!g_es) return -1;
    if (count == 0) return 0;
    void *cur[MAXN], *prev[MAXN];
    int rc = 0;
    for (int r = 0; r < n; r++) {
        cur[r] = malloc(count * g_es);
        prev[r] = malloc(count * g_es);
        if (!cur[r] || !prev[r]) rc = -3;
        else cp(cur[r], (sbufs && sbufs[r]) ? sbufs[r] : rbufs[r], count);
    }
    if (rc == 0) {
        int floor2 = 1;
        for (int i = n >> 1; i; i >>= 1) floor2 <<= 1;
        for (int r = 0; r + floor2 < n; r++) red(cur[r + floor2], cur[r], count);   /* the extra's source */
        for (int round = 0, exit_flag = floor2 - 1; exit_flag; exit_flag >>= 1, round++) {
            for (int r = 0; r < floor2; r++) cp(prev[r], cur[r], count);
            for (int r = 0; r < floor2; r++) red(prev[r ^ (1 << round)], cur[r], count);
        }
        for (int r = 0; r < n; r++) cp(rbufs[r], cur[r < floor2 ? r : r - floor2], count);
    }
    for (int r = 0; r < n; r++) { free(cur[r]); free(prev[r]); }
    return rc;
}
