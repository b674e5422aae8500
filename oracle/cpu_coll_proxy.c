/*
 * cpu_coll_proxy.c -- TEST INFRASTRUCTURE ONLY (CPU baseline, BASELINE.md 2
 * "Fallback"): the host MPI_Allreduce the reference would run with
 * coll/tuned + the vader (sm) BTL, restated as N forked processes over one
 * shared-memory segment, because no Open MPI install exists on the GPU box.
 *
 * Algorithms (coll/tuned's ids, coll_tuned_allreduce_decision.c:37-46):
 *  4 ring, ompi_coll_base_allreduce_intra_ring (coll_base_allreduce.c:
 *    341-536): rbuf = sbuf (copy_content_same_ddt, :408); reduce-scatter in
 *    n-1 steps, step k receiving block (r-k) mod n from the left neighbour
 *    and computing rbuf[b] = inbuf OP rbuf[b] (:470-477, :488-496);
 *    allgather in n-1 steps, step k receiving block (r-k) mod n (:500-530);
 *  5 segmented ring (:618-856), what the fixed decision picks for
 *    commutative ops above n x 1 MiB (coll_tuned_decision_fixed.c:72-82):
 *    the reduce-scatter runs num_phases times (phase rule :663-667), each
 *    time on one segment of every block, then one allgather of the blocks;
 *  6 Rabenseifner (:970-1243), power-of-two rank counts: recursive-halving
 *    reduce-scatter, recursive-doubling allgather.
 * Blocks follow COLL_BASE_COMPUTE_BLOCKCOUNT (coll_base_functions.h:
 * 428-435).  Transport is modelled as vader's single-copy path (CMA): the
 * receiver copies the part straight out of the sender's buffer.  Round 4:
 * a ring step waits only for its left neighbour to have finished the step
 * before (a per-rank step counter in shared memory: the pairwise
 * send/recv completion), not for every rank (round 3 put a process-shared
 * barrier around every copy, which held all ranks to the slowest); one
 * barrier separates the reduce-scatter from the allgather.  Ranks are
 * pinned one per core, spread over the L3 domains first (MX_PROXY_PLACEMENT=
 * packed: consecutive cores, round 3's placement): 8 ranks on one CCD share
 * that CCD's link to memory.
 * Every algorithm is timed; "value" is the fixed decision's.
 * The local reduction is a plain C loop of the OP_FUNC shape
 * (op_base_functions.c:40-51) ("port"); an optional shared library
 * exporting the reference's table may be named instead (not built here).
 *
 * usage: cpu_coll_proxy RANKS BYTES ITERS [lib exporting ompi_op_base_functions]
 * prints one JSON object: busBW GB/s = S/t * 2(n-1)/n, t = median, for the
 * fixed decision's algorithm, and every algorithm's busBW beside it.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

typedef void (*ref_fn)(void *in, void *inout, int *count, void *dtype, void *module);

static ref_fn g_ref;

static void reduce_sum_float(const float *in, float *inout, size_t n)
{
    if (g_ref) {
        /* the reference takes an int count; feed it in <= 2^30 pieces */
        while (n) {
            int c = n > (1u << 30) ? (1 << 30) : (int)n;
            g_ref((void *)in, inout, &c, NULL, NULL);
            in += c; inout += c; n -= (size_t)c;
        }
        return;
    }
    for (size_t i = 0; i < n; i++) inout[i] += in[i];   /* op_base_functions.c:312 */
}

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

struct shared {
    pthread_barrier_t bar;
    double times[8];          /* per algorithm id */
    int mismatch;
    volatile uint64_t done[64] __attribute__((aligned(64)));   /* last ring step each rank finished */
};

/* the left neighbour has finished step s (its send of this step is ready) */
static void wait_step(struct shared *sh, int p, uint64_t s)
{
    while (__atomic_load_n(&sh->done[p], __ATOMIC_ACQUIRE) < s) __builtin_ia32_pause();
}
static void post_step(struct shared *sh, int r, uint64_t s)
{
    __atomic_store_n(&sh->done[r], s, __ATOMIC_RELEASE);
}

static void blockcount(size_t count, int n, int b, size_t *off, size_t *len)
{
    const size_t late = count / n, split = count % n, early = late + (split ? 1 : 0);
    *off = (size_t)b < split ? b * early : b * late + split;
    *len = (size_t)b < split ? early : late;
}

/* order cpus[] round-robin over their L3 domains (first core of every
 * domain, then the second, ...); returns the number of domains */
static int spread_over_l3(int *cpus, int ncpu)
{
    char (*key)[128] = calloc((size_t)ncpu, 128);
    int *dom = calloc((size_t)ncpu, sizeof(int)), *out = calloc((size_t)ncpu, sizeof(int));
    int ndom = 0;
    if (!key || !dom || !out) { free(key); free(dom); free(out); return 1; }
    for (int i = 0; i < ncpu; i++) {
        char path[128];
        snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", cpus[i]);
        FILE *f = fopen(path, "r");
        if (!f || !fgets(key[i], 128, f)) snprintf(key[i], 128, "cpu%d", cpus[i] / 8);   /* unknown: groups of 8 */
        if (f) fclose(f);
        dom[i] = -1;
        for (int j = 0; j < i; j++)
            if (!strcmp(key[i], key[j])) { dom[i] = dom[j]; break; }
        if (dom[i] < 0) dom[i] = ndom++;
    }
    int k = 0;
    for (int round = 0; k < ncpu; round++)
        for (int d = 0; d < ndom; d++) {
            int seen = 0;
            for (int i = 0; i < ncpu; i++)
                if (dom[i] == d && seen++ == round) { out[k++] = cpus[i]; break; }
        }
    memcpy(cpus, out, sizeof(int) * (size_t)ncpu);
    free(key); free(dom); free(out);
    return ndom;
}

static int cmp_double(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

/* ring reduce-scatter over `nph` phases (1: the plain ring; the segmented
 * ring's phase p covers segment p of every block, COLL_BASE_COMPUTE_BLOCKCOUNT
 * of the block over the phases), then the ring allgather of whole blocks */
static void ring(struct shared *sh, int r, int n, size_t count, float *rbuf, float *inbuf, const float *lrbuf,
                 int nph, uint64_t *step)
{
    const int left = (r + n - 1) % n;
    for (int ph = 0; ph < nph; ph++) {
        for (int k = 1; k < n; k++) {
            const int b = (r - k + 2 * n) % n;
            size_t bo, bl, po, pl;
            blockcount(count, n, b, &bo, &bl);
            blockcount(bl, nph, ph, &po, &pl);
            wait_step(sh, left, *step);         /* left reduced this segment of block b one step ago */
            memcpy(inbuf, lrbuf + bo + po, pl * 4);
            reduce_sum_float(inbuf, rbuf + bo + po, pl);
            post_step(sh, r, ++*step);
        }
    }
    pthread_barrier_wait(&sh->bar);             /* every block final before any is overwritten */
    for (int k = 0; k < n - 1; k++) {
        const int b = (r - k + 2 * n) % n;
        size_t bo, bl;
        blockcount(count, n, b, &bo, &bl);
        if (k) wait_step(sh, left, *step);      /* left holds block b (final) since its step before */
        memcpy(rbuf + bo, lrbuf + bo, bl * 4);
        post_step(sh, r, ++*step);
    }
}

/* recursive halving reduce-scatter + recursive doubling allgather (power-of-
 * two n): at distance d the rank keeps the half of its current range on its
 * side of the partner r ^ d and folds the partner's copy of that half in */
static void rabenseifner(struct shared *sh, char *mem, size_t per_rank, int r, int n, size_t count, float *rbuf,
                         float *inbuf)
{
    size_t lo = 0, hi = count;
    size_t los[32], his[32];
    int steps = 0;
    for (int d = n / 2; d >= 1; d /= 2) {
        const int p = r ^ d;
        const float *prbuf = (const float *)(mem + per_rank * p) + count;
        const size_t mid = lo + (hi - lo + 1) / 2;
        los[steps] = lo; his[steps] = hi; steps++;
        if (r < p) hi = mid; else lo = mid;                  /* the half kept */
        pthread_barrier_wait(&sh->bar);
        memcpy(inbuf, prbuf + lo, (hi - lo) * 4);
        reduce_sum_float(inbuf, rbuf + lo, hi - lo);
    }
    for (int d = 1; d < n; d *= 2) {
        const int p = r ^ d;
        const float *prbuf = (const float *)(mem + per_rank * p) + count;
        steps--;
        const size_t plo = los[steps], phi = his[steps];     /* the range both held before the split */
        pthread_barrier_wait(&sh->bar);
        if (lo > plo) memcpy(rbuf + plo, prbuf + plo, (lo - plo) * 4);
        if (phi > hi) memcpy(rbuf + hi, prbuf + hi, (phi - hi) * 4);
        lo = plo; hi = phi;
    }
}

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s RANKS BYTES ITERS [libref_op.so]\n", argv[0]);
        return 2;
    }
    const int n = atoi(argv[1]);
    const size_t bytes = strtoull(argv[2], NULL, 0);
    const int iters = atoi(argv[3]);
    const char *kind = "port";
    if (argc > 4) {
        void *h = dlopen(argv[4], RTLD_NOW);
        if (h) {
            void **tab = (void **)dlsym(h, "ompi_op_base_functions");
            if (tab) {
                g_ref = (ref_fn)tab[3 * 41 + 15];   /* [MPI_SUM][OMPI_OP_BASE_TYPE_FLOAT] */
                kind = "reference";
            }
        }
    }
    if (n < 2 || n > 64 || iters < 1) return 2;
    const size_t count = bytes / 4;
    /* the fixed decision (coll_tuned_decision_fixed.c:64-85) and the phase
     * count of the segmented ring (coll_base_allreduce.c:652-667, 1 MiB) */
    const size_t segcount = (1u << 20) / 4;
    int decided = bytes < 10000 ? 3 : ((size_t)n * (1u << 20) >= bytes ? 4 : 5);
    int phases = (int)(count / ((size_t)n * segcount));
    if (count % ((size_t)n * segcount) >= (size_t)n && count % ((size_t)n * segcount) > ((size_t)n * segcount) / 2)
        phases++;
    if (phases < 1) { phases = 1; if (decided == 5) decided = 4; }
    int algs[3], nalg = 0;
    algs[nalg++] = 4;
    algs[nalg++] = 5;
    if ((n & (n - 1)) == 0) algs[nalg++] = 6;
    if (decided == 3) decided = 4;   /* recursive doubling below 10 kB: not a bandwidth case; ring stands in */
    size_t off, maxblk;
    blockcount(count, n, 0, &off, &maxblk);
    /* the receive buffer holds one ring block, or the first half a
     * Rabenseifner exchange moves */
    const size_t inmax = maxblk > count / 2 + 1 ? maxblk : count / 2 + 1;
    const size_t per_rank = 2 * count * 4 + inmax * 4 + 4096;
    struct shared *sh = mmap(NULL, sizeof *sh, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    char *mem = mmap(NULL, per_rank * n, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (sh == MAP_FAILED || mem == MAP_FAILED) { perror("mmap"); return 1; }
    pthread_barrierattr_t ba;
    pthread_barrierattr_init(&ba);
    pthread_barrierattr_setpshared(&ba, PTHREAD_PROCESS_SHARED);
    pthread_barrier_init(&sh->bar, &ba, n);
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    sched_getaffinity(0, sizeof allowed, &allowed);
    int cpus[1024], ncpu = 0;
    for (int i = 0; i < CPU_SETSIZE && ncpu < 1024; i++) if (CPU_ISSET(i, &allowed)) cpus[ncpu++] = i;
    const char *pl = getenv("MX_PROXY_PLACEMENT");
    const int spread = !(pl && !strcmp(pl, "packed"));
    int ndom = 1;
    if (spread && ncpu) ndom = spread_over_l3(cpus, ncpu);

    for (int r = 0; r < n; r++) {
        pid_t pid = fork();
        if (pid < 0) { perror("fork"); return 1; }
        if (pid > 0) continue;
        if (ncpu) {   /* --bind-to core */
            cpu_set_t one;
            CPU_ZERO(&one);
            CPU_SET(cpus[r % ncpu], &one);
            sched_setaffinity(0, sizeof one, &one);
        }
        float *sbuf = (float *)(mem + per_rank * r);
        float *rbuf = sbuf + count;
        float *inbuf = rbuf + count;
        uint64_t x = 0x5EED + (uint64_t)r;
        for (size_t i = 0; i < count; i++) {   /* xorshift64*, uniform [-1, 1) */
            x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
            sbuf[i] = (float)((double)((x * 0x2545F4914F6CDD1DULL) >> 11) * 0x1.0p-52 - 1.0);
        }
        const int left = (r + n - 1) % n;
        const float *lrbuf = (const float *)(mem + per_rank * left) + count;
        double *ts = malloc(sizeof(double) * (iters + 2));
        uint64_t step = 0;   /* ring steps done by this rank (the same count on every rank) */
        for (int ai = 0; ai < nalg; ai++) {
            const int alg = algs[ai];
            for (int it = 0; it < iters + 2; it++) {   /* 2 warmup iterations */
                pthread_barrier_wait(&sh->bar);
                const double t0 = now();
                memcpy(rbuf, sbuf, count * 4);
                if (alg == 6) rabenseifner(sh, mem, per_rank, r, n, count, rbuf, inbuf);
                else ring(sh, r, n, count, rbuf, inbuf, lrbuf, alg == 5 ? phases : 1, &step);
                pthread_barrier_wait(&sh->bar);
                ts[it] = now() - t0;
            }
            /* all ranks hold the same vector (each element is reduced by one rank and then copied) */
            if (r > 0 && memcmp(rbuf, (const float *)mem + count, count * 4) != 0) sh->mismatch = 1;
            if (r == 0) {
                qsort(ts + 2, iters, sizeof(double), cmp_double);
                sh->times[alg] = ts[2 + iters / 2];
            }
            pthread_barrier_wait(&sh->bar);
        }
        _exit(0);
    }
    int bad = 0;
    for (int r = 0; r < n; r++) {
        int st;
        wait(&st);
        if (!WIFEXITED(st) || WEXITSTATUS(st)) bad = 1;
    }
    if (bad || sh->mismatch) { fprintf(stderr, "cpu_coll_proxy: rank failure or mismatch\n"); return 1; }
    static const char *names[8] = {"", "", "", "", "ring", "segmented_ring", "rabenseifner", ""};
    const double t = sh->times[decided];
    const double algbw = (double)count * 4 / t / 1e9;
    printf("{\"value\": %.3f, \"unit\": \"GB/s\", \"cores\": %d, \"kind\": \"%s\", "
           "\"algorithm\": \"%s\", \"algbw_gbs\": %.3f, \"ms_per_call\": %.3f, \"algorithms_busbw_gbs\": {",
           algbw * 2.0 * (n - 1) / n, n, kind, names[decided], algbw, t * 1e3);
    for (int ai = 0; ai < nalg; ai++)
        printf("%s\"%s\": %.3f", ai ? ", " : "", names[algs[ai]],
               (double)count * 4 / sh->times[algs[ai]] / 1e9 * 2.0 * (n - 1) / n);
    printf("}, \"placement\": \"%s\", \"l3_domains\": %d, \"sample\": \"MPI_Allreduce fp32 SUM %zu B, %d ranks "
           "(processes pinned one per core, %s over %d L3 domains), coll/tuned's fixed decision (%s, %d phases of 1 MiB "
           "segments) over shared memory with single-copy transfers and pairwise step completion, median of %d "
           "calls; busBW = S/t*2(n-1)/n\"}\n",
           spread ? "spread" : "packed", ndom, count * 4, n, spread ? "spread" : "packed", ndom, names[decided],
           decided == 5 ? phases : 1, iters);
    return 0;
}
