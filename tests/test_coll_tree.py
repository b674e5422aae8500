"""Rooted reduce, scan, exscan and reduce_scatter_block.

CPU (no GPU): the oracle restatements of coll_base_reduce.c /
coll_base_scan.c / coll_base_exscan.c / coll_base_reduce_scatter_block.c are
checked against exact integer arithmetic and against the topology diagrams
printed in the reference's own coll_base_topo.c comments; the product's
tuned reduce decision equals the oracle's restatement.

GPU: the VM fold (mx_fold.hpp k_vm) over n virtual ranks is bit-identical
to the oracle for every algorithm, root, MPI_IN_PLACE and the adversarial
inputs of test_coll_gpu (NaN / -0 for MAX/MIN, ties for MAXLOC, 16-decade
floating-point sums).
"""
import ctypes

import numpy as np
import pytest

import golden_io
import mxompi
import oracle_lib

vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int


def _oracle():
    L = oracle_lib.oracle()
    L.mxo_reduce.argtypes = [ci, ci, ci, ci, sz, ci, ctypes.POINTER(vp), vp]
    L.mxo_scan.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_exscan.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_reduce_scatter_block.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_reduce_decision.argtypes = [ci, sz, sz, ctypes.POINTER(ci)]
    L.mxo_reduce_tree.argtypes = [ci, ci, ci, ci, ctypes.POINTER(ci)]
    return L


def _children(kind, n, root, rank):
    out = (ci * 64)()
    k = _oracle().mxo_reduce_tree(kind, n, root, rank, out)
    return list(out[:k])


# ---------------------------------------------------------------------------
# CPU: oracle pinned to the reference's topology diagrams and to exact sums
# ---------------------------------------------------------------------------
def test_topology_matches_reference_diagrams():
    # coll_base_topo.c:65-75  fanout 2, size 7: 0 -> 1 2; 1 -> 3 5; 2 -> 4 6
    assert _children(4, 7, 0, 0) == [1, 2]
    assert _children(4, 7, 0, 1) == [3, 5]
    assert _children(4, 7, 0, 2) == [4, 6]
    assert all(_children(4, 7, 0, r) == [] for r in range(3, 7))
    # :388-401  in-order binomial, size 8: 0 -> 1 2 4; 2 -> 3; 4 -> 5 6; 6 -> 7
    assert _children(5, 8, 0, 0) == [1, 2, 4]
    assert _children(5, 8, 0, 2) == [3]
    assert _children(5, 8, 0, 4) == [5, 6]
    assert _children(5, 8, 0, 6) == [7]
    assert _children(5, 4, 0, 0) == [1, 2] and _children(5, 4, 0, 2) == [3]
    # :177-190  in-order binary tree, size 9: 8 -> 7 3; 7 -> 6 5; 5 -> 4; 3 -> 2 1; 1 -> 0
    assert _children(6, 9, 8, 8) == [7, 3]
    assert _children(6, 9, 8, 7) == [6, 5]
    assert _children(6, 9, 8, 5) == [4]
    assert _children(6, 9, 8, 6) == []
    assert _children(6, 9, 8, 3) == [2, 1]
    assert _children(6, 9, 8, 1) == [0]
    assert _children(6, 4, 3, 3) == [2, 1] and _children(6, 4, 3, 1) == [0]
    # pipeline = chain of fanout 1 from the root
    assert [_children(3, 5, 2, r) for r in range(5)] == [[1], [], [3], [4], [0]]
    # chain fanout 4 over 9 ranks: root -> 4 chains of 2
    assert _children(2, 9, 0, 0) == [1, 3, 5, 7]
    assert _children(2, 9, 0, 1) == [2] and _children(2, 9, 0, 2) == []


def _every_rank_once(kind, n, root):
    seen = []

    def walk(v):
        seen.append(v)
        for c in _children(kind, n, root, v):
            walk(c)
    walk(n - 1 if kind == 6 else root)
    return sorted(seen) == list(range(n))


@pytest.mark.parametrize("kind", [2, 3, 4, 5, 6])
@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 13, 16])
def test_trees_span_every_rank(kind, n):
    for root in {0, n // 2, n - 1}:
        assert _every_rank_once(kind, n, root)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 16])
@pytest.mark.parametrize("alg", [0, 1, 2, 3, 4, 5, 6])
def test_oracle_reduce_exact_int_sum(n, alg):
    L = _oracle()
    count = 1001
    rng = np.random.default_rng(n * 10 + alg)
    xs = [rng.integers(-1000, 1000, count).astype(np.int64) for _ in range(n)]
    for root in {0, n - 1, n // 2}:
        out = np.zeros(count, np.int64)
        sp = (vp * n)(*[x.ctypes.data for x in xs])
        assert L.mxo_reduce(alg, mxompi.OP["SUM"], mxompi.TYPE["INT64_T"], n, count, root, sp, out.ctypes.data) == 0
        np.testing.assert_array_equal(out, np.sum(xs, axis=0))


@pytest.mark.parametrize("n", [1, 2, 3, 6, 8])
@pytest.mark.parametrize("alg", [1, 2])
def test_oracle_scan_exscan_exact(n, alg):
    L = _oracle()
    count = 257
    rng = np.random.default_rng(n + 7 * alg)
    xs = [rng.integers(-50, 50, count).astype(np.int32) for _ in range(n)]
    pref = np.cumsum(xs, axis=0)
    out = [np.zeros(count, np.int32) for _ in range(n)]
    assert L.mxo_scan(alg, mxompi.OP["SUM"], mxompi.TYPE["INT32_T"], n, count,
                      (vp * n)(*[x.ctypes.data for x in xs]), (vp * n)(*[o.ctypes.data for o in out])) == 0
    for r in range(n):
        np.testing.assert_array_equal(out[r], pref[r])
    out = [np.full(count, 77, np.int32) for _ in range(n)]
    assert L.mxo_exscan(alg, mxompi.OP["SUM"], mxompi.TYPE["INT32_T"], n, count,
                        (vp * n)(*[x.ctypes.data for x in xs]), (vp * n)(*[o.ctypes.data for o in out])) == 0
    np.testing.assert_array_equal(out[0], 77)      # rank 0's rbuf is not written
    for r in range(1, n):
        np.testing.assert_array_equal(out[r], pref[r - 1])


def test_reduce_decision_matches_oracle():
    O = _oracle()
    seg = ci()
    for n in (2, 3, 4, 7, 8, 9, 12, 16, 64):
        for es in (1, 4, 8):
            for count in (0, 1, 2, 100, 511, 2047, 5000, 20000, 10 ** 5, 10 ** 6, 10 ** 7, 10 ** 8):
                exp = O.mxo_reduce_decision(n, count, es, ctypes.byref(seg))
                got = mxompi.lib().mx_reduce_decision(n, count, -es)
                assert got == exp, (n, es, count, got, exp)


# ---------------------------------------------------------------------------
# GPU: VM fold vs oracle
# ---------------------------------------------------------------------------
CASES = [("SUM", "FLOAT"), ("SUM", "DOUBLE"), ("MAX", "FLOAT"), ("MIN", "DOUBLE"), ("MAXLOC", "FLOAT_INT"),
         ("PROD", "C_FLOAT_COMPLEX"), ("SUM", "LONG_DOUBLE"), ("BXOR", "UINT16_T"), ("PROD", "INT8_T"),
         ("MINLOC", "SHORT_INT"), ("MAXLOC", "LONG_DOUBLE_INT"), ("LAND", "BOOL")]
RED_ALGS = ["auto", "linear", "chain", "pipeline", "binary", "binomial", "in_order_binary"]


def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    mxompi.init(0)
    return torch


def _gen(t, op, count, seed):
    from test_coll_gpu import gen
    return gen(t, op, count, seed)


@pytest.mark.gpu
@pytest.mark.parametrize("alg", RED_ALGS)
@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 16])
@pytest.mark.parametrize("op,t", CASES)
def test_reduce_local_bitexact(alg, n, op, t):
    torch = _gpu()
    L = _oracle()
    es = mxompi.type_size(t)
    comm = mxompi.Comm.local(n)
    st = torch.cuda.current_stream().cuda_stream
    for count in (1, 7, 1000, 4099):
        xs = [_gen(t, op, count, 300 * n + count + r) for r in range(n)]
        for root in sorted({0, n - 1, (n * 5) // 7}):
            for inplace in (False, True):
                exp = np.zeros(count * es, np.uint8)
                sp = [x.ctypes.data for x in xs]
                if inplace:
                    exp[:] = xs[root]
                    sp[root] = None
                assert L.mxo_reduce(mxompi.REDUCE[alg], mxompi.OP[op], mxompi.TYPE[t], n, count, root,
                                    (vp * n)(*sp), exp.ctypes.data) == 0
                S = [torch.from_numpy(x.copy()).cuda() for x in xs]
                R = torch.zeros(count * es, dtype=torch.uint8, device="cuda")
                rb = [0] * n
                if inplace:
                    sb = [s.data_ptr() for s in S]
                    sb[root] = mxompi.IN_PLACE
                    rb[root] = S[root].data_ptr()
                    out = S[root]
                else:
                    sb = [s.data_ptr() for s in S]
                    rb[root] = R.data_ptr()
                    out = R
                comm.reduce_local(sb, rb, count, t, op, root, alg, st)
                golden_io.assert_coll_equal(out.cpu().numpy(), exp, mxompi.OP[op], mxompi.TYPE[t],
                                            f"reduce {alg} n={n} count={count} root={root} inplace={inplace}")
    comm.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["scan", "exscan"])
@pytest.mark.parametrize("alg", ["auto", "recursive_doubling"])
@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 16])
@pytest.mark.parametrize("op,t", CASES)
def test_scan_local_bitexact(kind, alg, n, op, t):
    torch = _gpu()
    L = _oracle()
    es = mxompi.type_size(t)
    comm = mxompi.Comm.local(n)
    st = torch.cuda.current_stream().cuda_stream
    fn = L.mxo_scan if kind == "scan" else L.mxo_exscan
    for count in (1, 13, 3001):
        for inplace in (False, True):
            xs = [_gen(t, op, count, 900 * n + count + r) for r in range(n)]
            exp = [np.full(count * es, 0xA5, np.uint8) for _ in range(n)]
            assert fn(mxompi.SCAN[alg], mxompi.OP[op], mxompi.TYPE[t], n, count,
                      (vp * n)(*[x.ctypes.data for x in xs]), (vp * n)(*[e.ctypes.data for e in exp])) == 0
            S = [torch.from_numpy(x.copy()).cuda() for x in xs]
            if inplace:
                R = S
                for r in range(n):
                    if kind == "exscan" and r == 0:
                        exp[0] = xs[0].copy()          # untouched in place
                sb = None
            else:
                R = [torch.full((count * es,), 0xA5, dtype=torch.uint8, device="cuda") for _ in range(n)]
                sb = [s.data_ptr() for s in S]
            getattr(comm, kind + "_local")(sb, [r.data_ptr() for r in R], count, t, op, alg, st)
            for r in range(n):
                golden_io.assert_coll_equal(R[r].cpu().numpy(), exp[r], mxompi.OP[op], mxompi.TYPE[t],
                                            f"{kind} {alg} n={n} count={count} rank {r} inplace={inplace}")
    comm.close()


@pytest.mark.gpu
@pytest.mark.parametrize("alg", ["auto", "linear", "pipeline", "binary", "binomial"])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 7, 8])
@pytest.mark.parametrize("op,t", [("SUM", "FLOAT"), ("MAX", "DOUBLE"), ("MAXLOC", "FLOAT_INT"), ("SUM", "INT64_T")])
@pytest.mark.parametrize("inplace", [False, True])
def test_reduce_scatter_block_local_bitexact(alg, n, op, t, inplace):
    torch = _gpu()
    L = _oracle()
    es = mxompi.type_size(t)
    comm = mxompi.Comm.local(n)
    st = torch.cuda.current_stream().cuda_stream
    for rcount in (1, 5, 1000):
        xs = [_gen(t, op, rcount * n, 40 * n + rcount + r) for r in range(n)]
        exp = [np.zeros(rcount * es, np.uint8) for _ in range(n)]
        assert L.mxo_reduce_scatter_block(mxompi.REDUCE[alg], mxompi.OP[op], mxompi.TYPE[t], n, rcount,
                                          (vp * n)(*[x.ctypes.data for x in xs]),
                                          (vp * n)(*[e.ctypes.data for e in exp])) == 0
        S = [torch.from_numpy(x.copy()).cuda() for x in xs]
        if inplace:
            comm.reduce_scatter_block_local(None, [s.data_ptr() for s in S], rcount, t, op, alg, st)
            R = S
        else:
            R = [torch.zeros(rcount * es, dtype=torch.uint8, device="cuda") for _ in range(n)]
            comm.reduce_scatter_block_local([s.data_ptr() for s in S], [r.data_ptr() for r in R], rcount, t, op,
                                            alg, st)
        for r in range(n):
            golden_io.assert_coll_equal(R[r].cpu().numpy()[: rcount * es], exp[r], mxompi.OP[op], mxompi.TYPE[t],
                                        f"reduce_scatter_block {alg} n={n} rcount={rcount} rank {r}")
    comm.close()
