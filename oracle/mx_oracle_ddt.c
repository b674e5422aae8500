/*
 * mx_oracle_ddt.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the convertor's homogeneous pack/unpack
 * (opal_generic_simple_pack_function, opal/datatype/opal_datatype_pack.c:
 * 235-370, with pack_predefined_data / pack_contiguous_loop,
 * opal_datatype_pack.h:86-185; unpack opal_datatype_unpack.c:245-427) over
 * the committed description records (opal_datatype_internal.h:146-196):
 * the datatype-count loop repeats the description `count` times advancing by
 * the extent (ub - lb); an ELEM copies `count` blocks of `blocklen` basic
 * elements at disp + j*extent; a LOOP repeats its items `loops` times
 * advancing by the loop extent; END_LOOP closes it.  The packed stream is
 * the blocks' bytes in that order.  Pinned against the reference's own
 * engine through tests/golden/ddt_vectors.bin (tests/test_convertor.py).
 */
#include <stdint.h>
#include <string.h>

typedef struct { uint16_t flags, type; uint32_t count; uint64_t blocklen; int64_t extent; int64_t disp; } rec_elem;
typedef struct { uint16_t flags, type; uint32_t items; uint32_t loops; uint32_t pad; uint64_t unused; int64_t extent; } rec_loop;

#define T_LOOP 0
#define T_END_LOOP 1
#define F_DATA 0x0100

struct walk {
    const uint8_t *recs;
    const uint64_t *bs;
    char *user;
    char *packed;
    size_t pos;    /* bytes moved so far */
    int unpack;
};

static void move(struct walk *w, char *addr, size_t n)
{
    if (w->unpack) memcpy(addr, w->packed + w->pos, n);
    else memcpy(w->packed + w->pos, addr, n);
    w->pos += n;
}

/* walk records [lo, hi) at origin `base`; returns the index after the level */
static size_t walk_level(struct walk *w, size_t lo, size_t hi, char *base)
{
    size_t i = lo;
    while (i < hi) {
        rec_elem e;
        memcpy(&e, w->recs + 32 * i, 32);
        if (e.type == T_END_LOOP) return i + 1;
        if (e.type == T_LOOP) {
            rec_loop L;
            memcpy(&L, w->recs + 32 * i, 32);
            for (uint32_t l = 0; l < L.loops; l++) walk_level(w, i + 1, i + L.items, base + (int64_t)l * L.extent);
            i += L.items + 1;
            continue;
        }
        if (e.flags & F_DATA) {
            const size_t blk = e.blocklen * w->bs[e.type];
            for (uint32_t j = 0; j < e.count; j++) move(w, base + e.disp + (int64_t)j * e.extent, blk);
        }
        i++;
    }
    return i;
}

/* Pack `count` instances at `user` (the MPI buffer pointer) into packed. */
int mxo_ddt_convert(const void *desc, size_t nrec, const uint64_t *basic_sizes, int64_t lb, int64_t ub,
                    size_t count, void *user, void *packed, int unpack)
{
    struct walk w = {desc, basic_sizes, user, packed, 0, unpack};
    for (size_t i = 0; i < count; i++) walk_level(&w, 0, nrec, (char *)user + (int64_t)i * (ub - lb));
    return (int)(w.pos > 0x7fffffff ? 0x7fffffff : w.pos);
}
