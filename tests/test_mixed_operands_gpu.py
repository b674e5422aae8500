"""Reduction operands in different memories.

MPI_Reduce_local(device_in, host_inout) -- and any coll/base algorithm that
mixes a device user buffer with host temporaries -- is legal MPI.  The
reference's accelerator path checks and stages each buffer on its own
(coll_cuda_allreduce.c:44-62, opal_cuda_check_bufs in
opal_datatype_cuda.c:70).  Both routes are covered:
  - coll/mi355x's reduce_local slot (MPI_Reduce_local on MPI_COMM_SELF);
  - op/mi355x's 2-buffer and 3-buffer slots (ompi_op_reduce /
    ompi_3buff_op_reduce, op.h:547-660, as every coll/base algorithm calls
    them).
The result is produced where it lives; a host result of at most 64 KiB runs
the saved host function on host copies, a larger one runs the kernel on device
copies (both sizes are tested).  Every location combination -- 4 for two
buffers, 8 for three -- is checked bit-exact against the oracle for fp32 SUM,
MAXLOC on MPI_FLOAT_INT (with ties) and x87 long double SUM."""
import itertools

import numpy as np
import pytest

import golden_io
import minihost
import mxompi
import oracle_lib

torch = pytest.importorskip("torch")

PAIRS = [("MPI_SUM", "MPI_FLOAT"), ("MPI_MAXLOC", "MPI_FLOAT_INT"), ("MPI_SUM", "MPI_LONG_DOUBLE")]
COUNTS = [1000, 100_003]     # host result: host function (<= 64 KiB) / device kernel


@pytest.fixture(scope="module")
def H():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    mxompi.init(0)
    return minihost.host(with_components=True)


def _operand(rng, dt, n):
    if dt == "MPI_FLOAT":
        return rng.uniform(-1, 1, n).astype(np.float32).view(np.uint8)
    if dt == "MPI_FLOAT_INT":
        p = np.zeros(n, dtype=[("v", "<f4"), ("k", "<i4")])
        p["v"] = rng.integers(0, 4, n)
        p["k"] = rng.integers(0, 100, n)
        return p.view(np.uint8).copy()
    return rng.uniform(-3, 3, n).astype(np.longdouble).view(np.uint8).copy()


def _place(buf, on_dev):
    """(pointer, keeper) with a copy of buf in device or host memory"""
    if on_dev:
        t = torch.from_numpy(buf.copy()).cuda()
        return t.data_ptr(), t
    h = buf.copy()
    return h.ctypes.data, h


def _read(keeper):
    return keeper.cpu().numpy() if isinstance(keeper, torch.Tensor) else keeper


@pytest.mark.gpu
@pytest.mark.parametrize("count", COUNTS)
@pytest.mark.parametrize("opname,dt", PAIRS)
@pytest.mark.parametrize("route", ["coll_reduce_local", "op_component"])
def test_two_buffers_every_location(H, route, opname, dt, count):
    O = oracle_lib.oracle()
    slot = mxompi.TYPE[mxompi.MPI_DTYPE_SLOT[dt]]
    opi = mxompi.OP[opname[4:]]
    rng = np.random.default_rng(opi * 1000 + slot + count)
    a, b = _operand(rng, dt, count), _operand(rng, dt, count)
    exp = b.copy()
    assert O.mxo_reduce2(opi, slot, a.ctypes.data, exp.ctypes.data, count, 1) == 0
    op, d = minihost.op(H, opname), minihost.dtype(H, dt)
    for din, dio in itertools.product([False, True], repeat=2):
        pa, ka = _place(a, din)
        pb, kb = _place(b, dio)
        torch.cuda.synchronize()
        if route == "coll_reduce_local":
            rc = H.mxh_reduce_local(pa, pb, count, d, op)
        else:
            rc = H.mxh_op_reduce(op, pa, pb, count, d)
        assert rc == 0
        got = _read(kb)
        golden_io.assert_coll_equal(got, exp, opi, slot, f"{route} {opname} {dt} n={count} in_dev={din} inout_dev={dio}")
        assert np.array_equal(_read(ka), a), "the input operand changed"


@pytest.mark.gpu
@pytest.mark.parametrize("count", COUNTS)
@pytest.mark.parametrize("opname,dt", PAIRS)
def test_three_buffers_every_location(H, opname, dt, count):
    O = oracle_lib.oracle()
    slot = mxompi.TYPE[mxompi.MPI_DTYPE_SLOT[dt]]
    opi = mxompi.OP[opname[4:]]
    rng = np.random.default_rng(opi * 1000 + slot + count + 7)
    a, b, o = _operand(rng, dt, count), _operand(rng, dt, count), _operand(rng, dt, count)
    exp = o.copy()
    assert O.mxo_reduce3(opi, slot, a.ctypes.data, b.ctypes.data, exp.ctypes.data, count, 1) == 0
    op, d = minihost.op(H, opname), minihost.dtype(H, dt)
    for d1, d2, do in itertools.product([False, True], repeat=3):
        p1, k1 = _place(a, d1)
        p2, k2 = _place(b, d2)
        po, ko = _place(o, do)
        torch.cuda.synchronize()
        assert H.mxh_3buff_op_reduce(op, p1, p2, po, count, d) == 0
        golden_io.assert_coll_equal(_read(ko), exp, opi, slot,
                                    f"3buff {opname} {dt} n={count} dev=({d1},{d2},{do})")
        assert np.array_equal(_read(k1), a) and np.array_equal(_read(k2), b), "an input operand changed"
