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
int mxo_allreduce(int alg, int op, int type, int n, size_t count, const void *const *sbufs, void *const *rbufs)
{
    void *rb[MAXN];
    if (n < 1 || n > MAXN) return -1;
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

/* alg: 0 auto, 2 recursive halving, 3 ring */
int mxo_reduce_scatter(int alg, int op, int type, int n, const size_t *rcounts, const void *const *sbufs,
                       void *const *rbufs)
{
    size_t total = 0;
    char *work[MAXN];
    if (n < 1 || n > MAXN) return -1;
    g_op = op; g_type = type; g_es = mxo_type_size(type);
    for (int i = 0; i < n; i++) total += rcounts[i];
    for (int r = 0; r < n; r++) {
        work[r] = malloc(total * g_es + 1);
        cp(work[r], sbufs[r], total);
    }
    if (n == 1) { cp(rbufs[0], work[0], total); free(work[0]); return 0; }
    if (alg == 0) alg = mxo_reduce_scatter_decision(n, total, g_es);
    if (alg == 3) rs_ring(n, rcounts, work, rbufs);
    else if (alg == 2) rs_recursive_halving(n, rcounts, work, rbufs);
    else { for (int r = 0; r < n; r++) free(work[r]); return -2; }
    for (int r = 0; r < n; r++) free(work[r]);
    return 0;
}
