"""CPU: the collective simulator (oracle/mx_oracle_coll.c).

* the reduction trees it produces match the step diagrams in the
  reference's own comments (ring reduce_scatter,
  ompi/mca/coll/base/coll_base_reduce_scatter.c:420-455; ring allreduce
  ompi/mca/coll/base/coll_base_allreduce.c:298-330), checked symbolically;
* every algorithm delivers the exact integer result on every rank for
  ragged counts and 1..12 ranks (data movement is right);
* the tuned decision thresholds (coll_tuned_decision_fixed.c:44-95,
  :466-512) agree with the product library's mx_*_decision.
"""
import ctypes

import numpy as np
import pytest

import mxompi
import oracle_lib

vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int


def _L():
    L = oracle_lib.oracle()
    L.mxo_allreduce.argtypes = [i, i, i, i, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_reduce_scatter.argtypes = [i, i, i, i, ctypes.POINTER(sz), ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_sym_node.argtypes = [ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    L.mxo_allreduce_decision.argtypes = [i, sz, sz]
    L.mxo_reduce_scatter_decision.argtypes = [i, sz, sz]
    return L


def _leaf(rank, elem):
    return -(rank * 1000 + elem + 1)


def _expr(L, v):
    """Flatten to the diagrams' notation: source first, then target."""
    if v < 0:
        k = -v - 1
        return f"{k // 1000}{k % 1000}"
    t, s = ctypes.c_int64(), ctypes.c_int64()
    assert L.mxo_sym_node(v, ctypes.byref(t), ctypes.byref(s)) == 0
    return _expr(L, s.value) + "+" + _expr(L, t.value)


def test_ring_reduce_scatter_matches_reference_diagram():
    L = _L()
    n = 5
    L.mxo_sym_reset(1)
    try:
        xs = [np.array([_leaf(r, e) for e in range(n)], np.int64) for r in range(n)]
        rb = [np.zeros(1, np.int64) for _ in range(n)]
        rc = (sz * n)(*([1] * n))
        sp = (vp * n)(*[x.ctypes.data for x in xs])
        rp = (vp * n)(*[r.ctypes.data for r in rb])
        assert L.mxo_reduce_scatter(3, 3, mxompi.TYPE["INT64_T"], n, rc, sp, rp) == 0
        got = [_expr(L, int(rb[r][0])) for r in range(n)]
    finally:
        L.mxo_sym_reset(0)
    # "DONE" state of the diagram: rank r holds block r (digits: rank, block)
    assert got == ["10+20+30+40+00", "21+31+41+01+11", "32+42+02+12+22",
                   "43+03+13+23+33", "04+14+24+34+44"]


def test_ring_allreduce_fold_starts_at_block_owner():
    L = _L()
    n = 5
    L.mxo_sym_reset(1)
    try:
        xs = [np.array([_leaf(r, e) for e in range(n)], np.int64) for r in range(n)]
        rb = [np.zeros(n, np.int64) for _ in range(n)]
        sp = (vp * n)(*[x.ctypes.data for x in xs])
        rp = (vp * n)(*[r.ctypes.data for r in rb])
        assert L.mxo_allreduce(4, 3, mxompi.TYPE["INT64_T"], n, n, sp, rp) == 0
        got = [[_expr(L, int(rb[r][b])) for b in range(n)] for r in range(n)]
    finally:
        L.mxo_sym_reset(0)
    # diagram (coll_base_allreduce.c:298-330): block b is started by rank b
    # ("[00+10]", "[11+21]", ...) and completed on rank b-1; then copied.
    for b in range(n):
        exp = "+".join(f"{(b + j) % n}{b}" for j in range(n))
        for r in range(n):
            assert got[r][b] == exp


ALGS = [1, 2, 3, 4, 5, 6]


@pytest.mark.parametrize("alg", ALGS)
@pytest.mark.parametrize("n", list(range(1, 13)))
def test_allreduce_integer_exact(alg, n):
    L = _L()
    for count in (1, 2, 3, 5, 8, 31, 1001):
        rng = np.random.default_rng(count * 7 + n)
        xs = [rng.integers(-1000, 1000, count).astype(np.int64) for _ in range(n)]
        rb = [np.zeros(count, np.int64) for _ in range(n)]
        sp = (vp * n)(*[x.ctypes.data for x in xs])
        rp = (vp * n)(*[r.ctypes.data for r in rb])
        assert L.mxo_allreduce(alg, 3, mxompi.TYPE["INT64_T"], n, count, sp, rp) == 0
        for r in rb:
            np.testing.assert_array_equal(r, sum(xs))


@pytest.mark.parametrize("alg", [1, 2, 3, 4])
@pytest.mark.parametrize("n", list(range(1, 13)))
def test_reduce_scatter_integer_exact(alg, n):
    L = _L()
    rng = np.random.default_rng(n)
    rcounts = [int(x) for x in rng.integers(0, 9, n)]
    total = sum(rcounts)
    xs = [rng.integers(-1000, 1000, total).astype(np.int64) for _ in range(n)]
    rb = [np.zeros(max(1, c), np.int64) for c in rcounts]
    sp = (vp * n)(*[x.ctypes.data for x in xs])
    rp = (vp * n)(*[r.ctypes.data for r in rb])
    assert L.mxo_reduce_scatter(alg, 3, mxompi.TYPE["INT64_T"], n, (sz * n)(*rcounts), sp, rp) == 0
    full = sum(xs)
    off = 0
    for r in range(n):
        np.testing.assert_array_equal(rb[r][: rcounts[r]], full[off: off + rcounts[r]])
        off += rcounts[r]


def test_decisions_agree_with_product():
    L = _L()
    for n in (2, 3, 4, 5, 7, 8, 12, 16):
        for t in ("INT8_T", "FLOAT", "DOUBLE", "LONG_DOUBLE_INT"):
            es = mxompi.type_size(t)
            for count in (1, 7, 100, 1249, 1250, 2500, 9999, 10000, 1 << 18, (1 << 20) + 3, 1 << 26):
                mine = mxompi.allreduce_decision(n, count, t)
                ref = L.mxo_allreduce_decision(n, count, es)
                assert mine == ref, (n, t, count)
                assert mxompi.reduce_scatter_decision(n, count, t) == L.mxo_reduce_scatter_decision(n, count, es)


def _sym_tree(L, v):
    """Canonical nested form of a symbolic node: leaves as (rank, elem)."""
    if v < 0:
        k = -v - 1
        return (k // 1000, k % 1000)
    t, s_ = ctypes.c_int64(), ctypes.c_int64()
    assert L.mxo_sym_node(v, ctypes.byref(t), ctypes.byref(s_)) == 0
    return ("op", _sym_tree(L, t.value), _sym_tree(L, s_.value))    # (target, source)


def _sym_allreduce(L, alg, n, count, inplace=False):
    L.mxo_sym_reset(1)
    try:
        xs = [np.array([_leaf(r, e) for e in range(count)], np.int64) for r in range(n)]
        rb = [x.copy() if inplace else np.zeros(count, np.int64) for x in xs]
        sp = None if inplace else (vp * n)(*[x.ctypes.data for x in xs])
        rp = (vp * n)(*[r.ctypes.data for r in rb])
        assert L.mxo_allreduce(alg, 3, mxompi.TYPE["INT64_T"], n, count, sp, rp) == 0
        return [[_sym_tree(L, int(rb[r][e])) for e in range(count)] for r in range(n)]
    finally:
        L.mxo_sym_reset(0)


def _sym_reduce_scatter(L, alg, n, rcounts, inplace=False):
    total = sum(rcounts)
    L.mxo_sym_reset(1)
    try:
        xs = [np.array([_leaf(r, e) for e in range(total)], np.int64) for r in range(n)]
        rb = [x.copy() if inplace else np.zeros(max(1, c), np.int64) for x, c in zip(xs, rcounts)]
        sp = None if inplace else (vp * n)(*[x.ctypes.data for x in xs])
        rp = (vp * n)(*[r.ctypes.data for r in rb])
        assert L.mxo_reduce_scatter(alg, 3, mxompi.TYPE["INT64_T"], n, (sz * n)(*rcounts), sp, rp) == 0
        return [[_sym_tree(L, int(rb[r][e])) for e in range(rcounts[r])] for r in range(n)]
    finally:
        L.mxo_sym_reset(0)


@pytest.mark.parametrize("n", list(range(2, 17)))
def test_butterfly_reduce_scatter_is_the_recursive_doubling_tree(n):
    """coll_base_reduce_scatter.c:691-880 restated step by step (psend /
    precv swaps, mirror-permutation hand-off) gives every element the tree
    recursive doubling allreduce gives it (coll_base_allreduce.c:130-274):
    masks ascending, the higher virtual rank's partial the target, the odd
    rank the target of the non-power-of-two leaf.  This is the identity the
    device fold program relies on (mx_coll.hip reduce_scatter_segments)."""
    L = _L()
    rng = np.random.default_rng(n)
    rcounts = [int(x) for x in rng.integers(0, 4, n)]
    rcounts[0] += 1
    total = sum(rcounts)
    bf = _sym_reduce_scatter(L, 4, n, rcounts)
    rd = _sym_allreduce(L, 3, n, total)
    off = 0
    for r in range(n):
        for e in range(rcounts[r]):
            assert bf[r][e] == rd[0][off + e], (n, r, e)
        off += rcounts[r]


def _sym_reduce(L, alg, n, count, root, inplace):
    L.mxo_reduce.argtypes = [i, i, i, i, sz, i, ctypes.POINTER(vp), vp]
    L.mxo_sym_reset(1)
    try:
        xs = [np.array([_leaf(r, e) for e in range(count)], np.int64) for r in range(n)]
        out = xs[root].copy() if inplace else np.zeros(count, np.int64)
        ptrs = [None if (inplace and r == root) else x.ctypes.data for r, x in enumerate(xs)]
        assert L.mxo_reduce(alg, 3, mxompi.TYPE["INT64_T"], n, count, root, (vp * n)(*ptrs), out.ctypes.data) == 0
        return [_sym_tree(L, int(v)) for v in out]
    finally:
        L.mxo_sym_reset(0)


@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("ralg", [1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("n", [2, 3, 5, 8])
def test_nonoverlapping_is_the_rooted_reduce_tree(n, ralg, inplace):
    """allreduce alg 2 (coll_base_allreduce.c:54-86) and reduce_scatter alg 1
    (coll_base_reduce_scatter.c:47-110) are coll_reduce to rank 0 -- with the
    reduce algorithm the communicator's coll_reduce runs, carried in bits
    8-15 of the algorithm word -- then a bcast / scatterv.  MPI_IN_PLACE makes
    rank 0 reduce in place (its data becomes the accumulator)."""
    L = _L()
    count = 7
    red = _sym_reduce(L, ralg, n, count, 0, inplace)
    ar = _sym_allreduce(L, 2 | (ralg << 8), n, count, inplace)
    for r in range(n):
        assert ar[r] == red, (r, ralg)
    rcounts = [1 + (r % 3) for r in range(n)]
    red = _sym_reduce(L, ralg, n, sum(rcounts), 0, inplace)
    rs = _sym_reduce_scatter(L, 1 | (ralg << 8), n, rcounts, inplace)
    off = 0
    for r in range(n):
        assert rs[r] == red[off:off + rcounts[r]], (r, ralg)
        off += rcounts[r]


def test_chain_fanout_changes_the_chain_tree():
    """coll_tuned_reduce_algorithm_chain_fanout reaches the chain topology
    (coll_base_topo.c:393-506) through bits 16-23 of the algorithm word:
    0 means tuned's default 4, and distinct fanouts give distinct trees."""
    L = _L()
    n = 9
    trees = {f: _sym_reduce(L, 2 | (f << 16), n, 1, 0, False)[0] for f in (1, 2, 3, 4, 7)}
    assert trees[4] == _sym_reduce(L, 2, n, 1, 0, False)[0]
    assert len({repr(t) for t in trees.values()}) == len(trees)
