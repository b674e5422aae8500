/*
 * gen_ddt_golden.c -- TEST INFRASTRUCTURE ONLY.  RETIRED: kept as the record
 * of how the committed tests/golden/ddt_vectors.bin was made in round 1; it
 * is no longer built.  It linked the reference's datatype engine compiled
 * through configuration stand-ins (oracle/shim_ddt, removed), a build that
 * pins nothing under the rules: the fixture's descriptions and
 * streams are checked against our own restatement (oracle/mx_oracle_ddt.c)
 * and, where the reference's own datatype tests state expected values,
 * against those (tests/test_convertor_pins.py).
 *
 * Golden vectors for the convertor (derived-datatype pack/unpack).  Links
 * the reference's OWN datatype engine (opal/datatype/*.c compiled unmodified
 * from /root/reference by oracle/Makefile) and the
 * reference's own test type library (test/datatype/opal_ddt_lib.c), builds
 * CFG-C-shaped types plus the reference test suite's types, and records:
 *   - the committed optimized description (opt_desc, the 32-byte
 *     dt_elem_desc records the convertor walks, opal_datatype_internal.h:
 *     146-196) with size / extent / lb / true bounds -- the input of the
 *     device convertor (mx_ddt_create);
 *   - a seeded user buffer, its packed stream produced by
 *     opal_convertor_pack (checked identical when packed in odd-size
 *     fragments, as opal_datatype_test.c does);
 *   - the result of opal_convertor_unpack of that stream into a prefilled
 *     buffer (gaps keep the prefill).
 *
 * Output: tests/golden/ddt_vectors.bin
 *   "MXDDT001" | u32 nrec | u32 nbasic | nbasic x u64 basic sizes |
 *   nrec x { char name[48], u32 count, u32 nelem (records incl. the final
 *   END_LOOP), i64 size, i64 lb, i64 ub, i64 true_lb, i64 true_ub,
 *   u64 span, nelem x 32 B desc, span B user, count*size B packed,
 *   span B prefill, span B unpacked }
 * `span` bytes start at the lowest touched address (buffer + true_lb).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "opal_config.h"
#include "opal/datatype/opal_convertor.h"
#include "opal/datatype/opal_datatype.h"
#include "opal/datatype/opal_datatype_internal.h"
#include "opal/runtime/opal.h"
#include "test/datatype/opal_ddt_lib.h"

static uint64_t rs = 0x5EEDC0DEULL;
static uint64_t rnd(void) { rs ^= rs >> 12; rs ^= rs << 25; rs ^= rs >> 27; return rs * 0x2545F4914F6CDD1DULL; }

/* MPI-style constructors restated on top of the public opal_datatype_add
 * (what ompi_datatype_create_{vector,indexed,struct} do). */
static opal_datatype_t *mk_contig(int n, const opal_datatype_t *old)
{
    opal_datatype_t *t = opal_datatype_create(old->desc.used + 2);
    opal_datatype_add(t, old, n, 0, old->ub - old->lb);
    return t;
}
static opal_datatype_t *mk_vector(int count, int blen, int stride, const opal_datatype_t *old)
{
    const ptrdiff_t ext = old->ub - old->lb;
    opal_datatype_t *t = opal_datatype_create(old->desc.used + 4);
    if (blen == 1) {
        opal_datatype_add(t, old, count, 0, stride * ext);
    } else {
        opal_datatype_t *b = mk_contig(blen, old);
        opal_datatype_add(t, b, count, 0, stride * ext);
        OBJ_RELEASE(b);
    }
    return t;
}
static opal_datatype_t *mk_indexed(int n, const int *blens, const int *disps, const opal_datatype_t *old)
{
    const ptrdiff_t ext = old->ub - old->lb;
    opal_datatype_t *t = opal_datatype_create(n * (old->desc.used + 2) + 2);
    for (int i = 0; i < n; i++) opal_datatype_add(t, old, blens[i], disps[i] * ext, ext);
    return t;
}
static opal_datatype_t *mk_struct(int n, const int *blens, const ptrdiff_t *disps, const opal_datatype_t **types)
{
    opal_datatype_t *t = opal_datatype_create(64);
    for (int i = 0; i < n; i++) opal_datatype_add(t, types[i], blens[i], disps[i], types[i]->ub - types[i]->lb);
    return t;
}

static FILE *g_out;
static uint32_t g_nrec;

static void put(const void *p, size_t n) { fwrite(p, 1, n, g_out); }
static void put32(uint32_t v) { put(&v, 4); }
static void put64(int64_t v) { put(&v, 8); }

static int pack_all(const opal_datatype_t *dt, int count, const char *base, char *out, size_t chunk)
{
    opal_convertor_t *c = opal_convertor_create(opal_local_arch, 0);
    size_t total = 0, want = dt->size * (size_t)count;
    if (opal_convertor_prepare_for_send(c, dt, count, base)) return -1;
    while (total < want) {
        struct iovec iov;
        uint32_t n = 1;
        size_t max = chunk;
        iov.iov_base = out + total;
        iov.iov_len = (want - total) < chunk ? (want - total) : chunk;
        max = iov.iov_len;
        if (opal_convertor_pack(c, &iov, &n, &max) < 0) return -2;
        if (max == 0) return -3;
        total += max;
    }
    OBJ_RELEASE(c);
    return 0;
}

static int unpack_all(const opal_datatype_t *dt, int count, char *base, const char *in, size_t chunk)
{
    opal_convertor_t *c = opal_convertor_create(opal_local_arch, 0);
    size_t total = 0, want = dt->size * (size_t)count;
    if (opal_convertor_prepare_for_recv(c, dt, count, base)) return -1;
    while (total < want) {
        struct iovec iov;
        uint32_t n = 1;
        size_t max;
        iov.iov_base = (char *)in + total;
        iov.iov_len = (want - total) < chunk ? (want - total) : chunk;
        max = iov.iov_len;
        if (opal_convertor_unpack(c, &iov, &n, &max) < 0) return -2;
        if (max == 0) return -3;
        total += max;
    }
    OBJ_RELEASE(c);
    return 0;
}

static void record(const char *name, opal_datatype_t *dt, int count)
{
    char nm[48] = {0};
    const ptrdiff_t ext = dt->ub - dt->lb;
    const ptrdiff_t tlb = dt->true_lb, tub = dt->true_ub;
    const size_t span = (size_t)(ext * (count - 1) + tub - tlb);
    const size_t psz = dt->size * (size_t)count;
    const dt_type_desc_t *d = &dt->opt_desc;
    char *user = malloc(span + 16), *packed = malloc(psz + 16), *packed2 = malloc(psz + 16);
    char *prefill = malloc(span + 16), *unpacked = malloc(span + 16);
    const size_t chunks[] = {11, 48, 956, 16384, (size_t)1 << 40};

    if (!d->desc || d->used == 0) d = &dt->desc;
    for (size_t i = 0; i < span; i++) { user[i] = (char)rnd(); prefill[i] = (char)rnd(); }
    if (pack_all(dt, count, user - tlb, packed, (size_t)1 << 40)) { fprintf(stderr, "%s: pack failed\n", name); exit(1); }
    for (int k = 0; k < 4; k++) {   /* resumable packing in odd fragments gives the same stream */
        memset(packed2, 0, psz);
        if (pack_all(dt, count, user - tlb, packed2, chunks[k]) || memcmp(packed, packed2, psz)) {
            fprintf(stderr, "%s: fragmented pack differs (chunk %zu)\n", name, chunks[k]);
            exit(1);
        }
    }
    memcpy(unpacked, prefill, span);
    if (unpack_all(dt, count, unpacked - tlb, packed, (size_t)1 << 40)) { fprintf(stderr, "%s: unpack failed\n", name); exit(1); }

    snprintf(nm, sizeof nm, "%s", name);
    put(nm, sizeof nm);
    put32((uint32_t)count);
    put32((uint32_t)(d->used + 1));
    put64((int64_t)dt->size);
    put64(dt->lb);
    put64(dt->ub);
    put64(tlb);
    put64(tub);
    put64((int64_t)span);
    put(d->desc, (d->used + 1) * sizeof(dt_elem_desc_t));
    put(user, span);
    put(packed, psz);
    put(prefill, span);
    put(unpacked, span);
    g_nrec++;
    free(user); free(packed); free(packed2); free(prefill); free(unpacked);
}

int main(int argc, char **argv)
{
    const char *path = argc > 1 ? argv[1] : "tests/golden/ddt_vectors.bin";
    opal_init_util(NULL, NULL);
    g_out = fopen(path, "wb");
    if (!g_out) { perror(path); return 1; }
    put("MXDDT001", 8);
    put32(0);
    put32(OPAL_DATATYPE_MAX_PREDEFINED);
    for (int i = 0; i < OPAL_DATATYPE_MAX_PREDEFINED; i++) put64((int64_t)opal_datatype_basicDatatypes[i]->size);

    /* CFG-C: MPI_Type_vector(count, blocklen in {1,4,16,64}, stride 2*blocklen, MPI_FLOAT) */
    const int blens[] = {1, 4, 16, 64};
    for (int b = 0; b < 4; b++) {
        char nm[64];
        opal_datatype_t *v = mk_vector(97, blens[b], 2 * blens[b], &opal_datatype_float4);
        opal_datatype_commit(v);
        snprintf(nm, sizeof nm, "vector_f32_b%d_s%d", blens[b], 2 * blens[b]);
        record(nm, v, 3);
        OBJ_RELEASE(v);
    }
    /* vector of doubles with a stride not multiple of 16 bytes */
    {
        opal_datatype_t *v = mk_vector(33, 3, 5, &opal_datatype_float8);
        opal_datatype_commit(v);
        record("vector_f64_b3_s5", v, 5);
        OBJ_RELEASE(v);
    }
    /* CFG-C: indexed with random 1..64-element blocks */
    {
        int bl[40], dp[40], pos = 0;
        for (int i = 0; i < 40; i++) { bl[i] = 1 + (int)(rnd() % 64); pos += (int)(rnd() % 17); dp[i] = pos; pos += bl[i]; }
        opal_datatype_t *t = mk_indexed(40, bl, dp, &opal_datatype_float4);
        opal_datatype_commit(t);
        record("indexed_f32_random", t, 4);
        OBJ_RELEASE(t);
    }
    /* CFG-C: struct {char, double[3], int} resized */
    {
        int bl[3] = {1, 3, 1};
        ptrdiff_t dp[3] = {0, 8, 32};
        const opal_datatype_t *ty[3] = {&opal_datatype_int1, &opal_datatype_float8, &opal_datatype_int4};
        opal_datatype_t *s = mk_struct(3, bl, dp, ty), *r;
        opal_datatype_commit(s);
        r = opal_datatype_create(s->desc.used + 2);
        opal_datatype_clone(s, r);
        opal_datatype_resize(r, 0, 48);
        opal_datatype_commit(r);
        record("struct_char_d3_int_resized48", r, 17);
        OBJ_RELEASE(s);
        OBJ_RELEASE(r);
    }
    /* types of the reference's own test suite (test/datatype/opal_ddt_lib.c) */
    {
        opal_datatype_t *t;
        t = create_vector_type(&opal_datatype_float8, 450, 10, 11); opal_datatype_commit(t);
        record("ref_vector_450x10_s11_f64", t, 2); OBJ_RELEASE(t);
        t = test_struct_char_double(); opal_datatype_commit(t);
        record("ref_struct_char_double", t, 50); OBJ_RELEASE(t);
        t = test_create_twice_two_doubles(); opal_datatype_commit(t);
        record("ref_twice_two_doubles", t, 20); OBJ_RELEASE(t);
        t = test_create_blacs_type(); opal_datatype_commit(t);
        record("ref_blacs_indexed", t, 3); OBJ_RELEASE(t);
        t = upper_matrix(60); opal_datatype_commit(t);
        record("ref_upper_matrix_60", t, 1); OBJ_RELEASE(t);
        t = lower_matrix(47); opal_datatype_commit(t);
        record("ref_lower_matrix_47", t, 2); OBJ_RELEASE(t);
        t = create_strange_dt(); opal_datatype_commit(t);
        record("ref_strange", t, 7); OBJ_RELEASE(t);
        t = test_struct(); opal_datatype_commit(t);
        record("ref_struct", t, 9); OBJ_RELEASE(t);
        t = test_matrix_borders(20, 3); opal_datatype_commit(t);
        record("ref_matrix_borders_20_3", t, 2); OBJ_RELEASE(t);
        t = create_struct_constant_gap_resized_ddt(&opal_datatype_float4); opal_datatype_commit(t);
        record("ref_struct_constant_gap_resized", t, 31); OBJ_RELEASE(t);
        t = create_contiguous_type(&opal_datatype_int2, 77); opal_datatype_commit(t);
        record("ref_contiguous_int2_77", t, 5); OBJ_RELEASE(t);
    }
    fseek(g_out, 8, SEEK_SET);
    put32(g_nrec);
    fclose(g_out);
    printf("wrote %u datatype records to %s\n", g_nrec, path);
    return 0;
}
