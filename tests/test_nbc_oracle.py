"""CPU: the coll/libnbc restatements (oracle/mx_oracle_coll.c, "coll/libnbc
schedules") behind MPI_Iallreduce / MPI_Ireduce / MPI_Ireduce_scatter and
their persistent forms.

* libnbc's ring reduces in the order of the step diagram in its own comment
  (ompi/mca/coll/libnbc/nbc_iallreduce.c:710-770, p = 4), checked
  symbolically -- it is NOT coll/tuned's ring (other start rank, other
  operand roles), which is why the non-blocking path has its own trees;
* the binomial (allred_sched_diss / red_sched_binomial) and chain
  (red_sched_chain) trees, including the chain root's MPI_IN_PLACE operand
  swap, as derived from the schedule code;
* every algorithm delivers exact integer results on every rank for 1..12
  ranks, ragged counts, every root, in place or not;
* libnbc's default rules agree with the product library's decisions.
"""
import ctypes

import numpy as np
import pytest

import mxompi
import oracle_lib

vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
I64 = mxompi.TYPE["INT64_T"]
SUM = mxompi.OP["SUM"]


def _L():
    L = oracle_lib.oracle()
    L.mxo_iallreduce.argtypes = [i, i, i, i, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_ireduce.argtypes = [i, i, i, i, sz, i, ctypes.POINTER(vp), vp]
    L.mxo_ireduce_scatter.argtypes = [i, i, i, ctypes.POINTER(sz), ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_iallreduce_decision.argtypes = [i, sz, sz, i]
    L.mxo_ireduce_decision.argtypes = [i, sz, sz]
    L.mxo_sym_node.argtypes = [ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    return L


def _leaf(rank, elem):
    return -(rank * 1000 + elem + 1)


def _expr(L, v):
    """Diagram notation: the reducing rank's own operand (source) first."""
    if v < 0:
        k = -v - 1
        return f"{k // 1000}{k % 1000}"
    t, s = ctypes.c_int64(), ctypes.c_int64()
    assert L.mxo_sym_node(v, ctypes.byref(t), ctypes.byref(s)) == 0
    return _expr(L, s.value) + "+" + _expr(L, t.value)


def _sym_iallreduce(L, alg, n, count, inplace=False):
    xs = [np.array([_leaf(r, e) for e in range(count)], np.int64) for r in range(n)]
    rb = [x.copy() if inplace else np.zeros(count, np.int64) for x in xs]
    L.mxo_sym_reset(1)
    try:
        sp = None if inplace else (vp * n)(*[x.ctypes.data for x in xs])
        assert L.mxo_iallreduce(alg, SUM, I64, n, count, sp, (vp * n)(*[r.ctypes.data for r in rb])) == 0
        return [[_expr(L, int(rb[r][e])) for e in range(count)] for r in range(n)]
    finally:
        L.mxo_sym_reset(0)


def test_libnbc_ring_matches_its_diagram():
    # nbc_iallreduce.c:710-770 (p = 4): element 0 is started by node 3
    # ("00+30"), then reduced by 1 ("10+00/30") and 2; element 1 by 0, 1
    # ("11+01"), 2 ("21+11/01"), 3 ... -- own data first, "/" = earlier step.
    got = _sym_iallreduce(_L(), 1, 4, 4)
    for b in range(4):
        chain = [(b - 1 + k) % 4 for k in range(4)]          # b-1, b, b+1, b+2
        exp = "+".join(f"{r}{b}" for r in reversed(chain))
        assert all(got[r][b] == exp for r in range(4)), (b, got[0][b], exp)


def test_libnbc_binomial_tree():
    # allred_sched_diss, root 0: round 1 pairs (0,1) (2,3), round 2 (0,2),
    # round 3 (0,4); the receiver's own value is the source operand
    got = _sym_iallreduce(_L(), 2, 5, 1)
    assert all(g[0] == "00+10+20+30+40" for g in got)
    got = _sym_iallreduce(_L(), 2, 6, 1, inplace=True)      # in place: same roles
    assert all(g[0] == "00+10+20+30+40+50" for g in got)


def test_libnbc_recursive_doubling_and_rabenseifner_are_coll_base():
    # allred_sched_recursivedoubling / _redscat_allgather restate coll/base's
    # algorithms line for line; the symbolic trees must coincide.
    L = _L()
    L.mxo_allreduce.argtypes = [i, i, i, i, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    for n in (3, 5, 6, 8):
        count = 2 * n + 1
        for nbc_alg, tuned_alg in ((4, 3), (3, 6)):
            a = _sym_iallreduce(L, nbc_alg, n, count)
            xs = [np.array([_leaf(r, e) for e in range(count)], np.int64) for r in range(n)]
            rb = [np.zeros(count, np.int64) for _ in range(n)]
            L.mxo_sym_reset(1)
            try:
                assert L.mxo_allreduce(tuned_alg, SUM, I64, n, count, (vp * n)(*[x.ctypes.data for x in xs]),
                                       (vp * n)(*[r.ctypes.data for r in rb])) == 0
                b = [[_expr(L, int(rb[r][e])) for e in range(count)] for r in range(n)]
            finally:
                L.mxo_sym_reset(0)
            assert a == b, (n, nbc_alg)


def _sym_ireduce(L, alg, n, root, inplace):
    xs = [np.array([_leaf(r, 0)], np.int64) for r in range(n)]
    out = xs[root].copy() if inplace else np.zeros(1, np.int64)
    sp = [x.ctypes.data for x in xs]
    if inplace:
        sp[root] = None
    L.mxo_sym_reset(1)
    try:
        assert L.mxo_ireduce(alg, SUM, I64, n, 1, root, (vp * n)(*sp), out.ctypes.data) == 0
        return _expr(L, int(out[0]))
    finally:
        L.mxo_sym_reset(0)


def test_libnbc_chain_root_inplace_swaps_roles():
    L = _L()
    # vranks: 0 <-> root swapped; v = 3 starts, 2 and 1 add their own data
    # as the source; the root adds its own data as the source, or -- in
    # place -- keeps it as the target (nbc_ireduce.c:494-503)
    assert _sym_ireduce(L, 1, 4, 2, False) == "20+10+00+30"
    assert _sym_ireduce(L, 1, 4, 2, True) == "10+00+30+20"
    assert _sym_ireduce(L, 1, 4, 0, False) == "00+10+20+30"
    # binomial in virtual ranks (root 2: v0 = rank 2, v2 = rank 0)
    assert _sym_ireduce(L, 2, 4, 2, False) == "20+10+00+30"
    assert _sym_ireduce(L, 2, 4, 2, True) == "20+10+00+30"


@pytest.mark.parametrize("n", list(range(1, 13)))
@pytest.mark.parametrize("alg", [0, 1, 2, 3, 4])
def test_iallreduce_integer_exact(n, alg):
    L = _L()
    rng = np.random.default_rng(n * 7 + alg)
    for count in (1, 3, n, 97):
        for inplace in (False, True):
            xs = [rng.integers(-1000, 1000, count).astype(np.int64) for _ in range(n)]
            rb = [x.copy() if inplace else np.zeros(count, np.int64) for x in xs]
            sp = None if inplace else (vp * n)(*[x.ctypes.data for x in xs])
            assert L.mxo_iallreduce(alg, SUM, I64, n, count, sp, (vp * n)(*[r.ctypes.data for r in rb])) == 0
            total = np.sum(xs, axis=0)
            for r in range(n):
                np.testing.assert_array_equal(rb[r], total, err_msg=f"n={n} alg={alg} count={count} r={r}")


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8, 11])
@pytest.mark.parametrize("alg", [0, 1, 2, 3])
def test_ireduce_integer_exact(n, alg):
    L = _L()
    rng = np.random.default_rng(n * 5 + alg)
    for count in (1, 2 * n + 3, 64):
        for root in range(n):
            for inplace in (False, True):
                xs = [rng.integers(-1000, 1000, count).astype(np.int64) for _ in range(n)]
                out = xs[root].copy() if inplace else np.zeros(count, np.int64)
                sp = [x.ctypes.data for x in xs]
                if inplace:
                    sp[root] = None
                assert L.mxo_ireduce(alg, SUM, I64, n, count, root, (vp * n)(*sp), out.ctypes.data) == 0
                np.testing.assert_array_equal(out, np.sum(xs, axis=0))


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8])
def test_ireduce_scatter_integer_exact(n):
    L = _L()
    rng = np.random.default_rng(n)
    for rc in ([3] * n, [int(x) for x in rng.integers(0, 9, n)]):
        total = sum(rc)
        if total == 0:
            continue
        xs = [rng.integers(-1000, 1000, total).astype(np.int64) for _ in range(n)]
        rb = [np.zeros(max(1, c), np.int64) for c in rc]
        assert L.mxo_ireduce_scatter(SUM, I64, n, (sz * n)(*rc), (vp * n)(*[x.ctypes.data for x in xs]),
                                     (vp * n)(*[r.ctypes.data for r in rb])) == 0
        full = np.sum(xs, axis=0)
        off = np.cumsum([0] + rc)
        for r in range(n):
            np.testing.assert_array_equal(rb[r][: rc[r]], full[off[r]: off[r + 1]])


def test_libnbc_decisions_agree_with_product():
    L = _L()
    for n in (1, 2, 3, 4, 5, 7, 8, 16):
        for count in (1, 3, 7, 8, 15, 16, 1000, 16383, 16384, 16385, 1 << 20):
            for t in ("FLOAT", "DOUBLE", "INT8_T", "LONG_DOUBLE_INT"):
                es = mxompi.type_size(t)
                for inplace in (False, True):
                    assert mxompi.iallreduce_decision(n, count, t, inplace) == \
                        L.mxo_iallreduce_decision(n, count, es, 1 if inplace else 0), (n, count, t, inplace)
                assert mxompi.ireduce_decision(n, count, t) == L.mxo_ireduce_decision(n, count, es), (n, count, t)
