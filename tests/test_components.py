"""The drop-in boundary: the op/mi355x and coll/mi355x MCA components,
loaded by the mini-host harness exactly the way Open MPI selects them
(op_base_op_select.c:88-204, coll_base_comm_select.c:108-309), driven
through MPI_Reduce_local / MPI_Allreduce-shaped entry points.

CPU tests: ABI layout of the mirrored structs vs the reference's headers,
component libraries load, and without a GPU the components decline
(init_query) so every slot stays on the base functions.
GPU tests: device buffers run the HIP kernels through both routes
(coll/mi355x reduce_local above coll/self's priority 75, and op/mi355x
inside ompi_op_reduce below it), host buffers delegate to the cached base
functions, all bit-exact vs the oracle."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

import golden_io
import minihost
import mxompi
import oracle_lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


# the op / coll / mca_base layouts are checked member by member against the
# reference's headers in tests/test_abi_layout.py


def test_component_library_exports_component_structs():
    L = ctypes.CDLL(os.path.join(mxompi.LIB_DIR, "libmx_ompi.so"))
    for sym in ("mca_op_mi355x_component", "mca_coll_mi355x_component", "mx_ompi_set_host"):
        assert hasattr(L, sym), sym


def test_base_path_without_components_matches_oracle():
    """Host buffers through the harness's MPI_Reduce_local with only the
    base functions: exercises the selection logic and the dispatch."""
    H = minihost.host(with_components=False)
    O = oracle_lib.oracle()
    rng = np.random.default_rng(3)
    a = rng.uniform(-1, 1, 1000).astype(np.float32)
    b = rng.uniform(-1, 1, 1000).astype(np.float32)
    exp = b.copy()
    O.mxo_reduce2(3, 15, a.ctypes.data, exp.ctypes.data, 1000, 1)
    assert H.mxh_reduce_local(a.ctypes.data, b.ctypes.data, 1000, minihost.dtype(H, "MPI_FLOAT"),
                              minihost.op(H, "MPI_SUM")) == 0
    np.testing.assert_array_equal(b, exp)
    # an undefined (op, type) pair is rejected like ompi_op_is_valid does
    assert H.mxh_reduce_local(a.ctypes.data, b.ctypes.data, 10, minihost.dtype(H, "MPI_FLOAT"),
                              minihost.op(H, "MPI_BXOR")) == -1


def test_self_comm_host_buffers_run_coll_self():
    """MPI_COMM_SELF without the components (no GPU): every slot is the
    coll/self stand-in's local copy (coll_self_allreduce.c:41-44 ...), in
    place a no-op, exscan untouched."""
    H = minihost.host(with_components=False)
    c = H.mxh_comm_self()
    f32 = minihost.dtype(H, "MPI_FLOAT")
    SUM = minihost.op(H, "MPI_SUM")
    for s in ("allreduce", "reduce", "scan", "exscan", "reduce_scatter", "reduce_scatter_block", "allgather"):
        assert H.mxh_comm_slot_owner(c, s.encode()) == b"self", s
    src = np.arange(64, dtype=np.float32)
    for call in (lambda r: H.mxh_allreduce(src.ctypes.data, r.ctypes.data, 64, f32, SUM, c),
                 lambda r: H.mxh_reduce(src.ctypes.data, r.ctypes.data, 64, f32, SUM, 0, c),
                 lambda r: H.mxh_scan(src.ctypes.data, r.ctypes.data, 64, f32, SUM, c),
                 lambda r: H.mxh_reduce_scatter_block(src.ctypes.data, r.ctypes.data, 64, f32, SUM, c),
                 lambda r: H.mxh_allgather(src.ctypes.data, 64, f32, r.ctypes.data, 64, f32, c)):
        r = np.zeros(64, dtype=np.float32)
        before = H.mxh_self_calls()
        assert call(r) == 0
        assert H.mxh_self_calls() == before + 1
        np.testing.assert_array_equal(r, src)
    r = np.full(64, 7, dtype=np.float32)
    assert H.mxh_exscan(src.ctypes.data, r.ctypes.data, 64, f32, SUM, c) == 0
    np.testing.assert_array_equal(r, 7)
    assert H.mxh_allreduce(1, r.ctypes.data, 64, f32, SUM, c) == 0      # MPI_IN_PLACE
    np.testing.assert_array_equal(r, 7)


# ---------------------------------------------------------------------------
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu_host():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    mxompi.init(0)
    return minihost.host(with_components=True)


PAIRS = [("MPI_SUM", "MPI_FLOAT"), ("MPI_MAX", "MPI_DOUBLE"), ("MPI_MAXLOC", "MPI_2INT"), ("MPI_BXOR", "MPI_BYTE"),
         ("MPI_PROD", "MPI_C_DOUBLE_COMPLEX"), ("MPI_SUM", "MPI_LONG_DOUBLE"), ("MPI_LAND", "MPI_C_BOOL"),
         ("MPI_MINLOC", "MPI_LONG_DOUBLE_INT"), ("MPI_SUM", "MPI_INTEGER"), ("MPI_MIN", "MPI_REAL")]


@pytest.mark.gpu
def test_all_slots_selected_for_mi355x(gpu_host):
    """After selection every non-NULL slot of every intrinsic op is owned by
    the mi355x module (all 176 pairs, 2- and 3-buffer)."""
    H = gpu_host
    O = oracle_lib.oracle()
    n = 0
    for k, name in enumerate(mxompi.OPS):
        o = minihost.op(H, "MPI_" + name if name != "NULL" else "MPI_OP_NULL")
        for t in range(41):
            if O.mxo_supported(k, t, 1):
                assert H.mxh_op_slot_owner(o, t, 0) == 1, (name, mxompi.TYPES[t])
                assert H.mxh_op_slot_owner(o, t, 1) == 1, (name, mxompi.TYPES[t])
                n += 1
    assert n == 176


@pytest.mark.gpu
@pytest.mark.parametrize("route", ["coll_reduce_local", "op_component"])
@pytest.mark.parametrize("opname,dt", PAIRS)
def test_reduce_local_device_buffers(gpu_host, route, opname, dt):
    H = gpu_host
    O = oracle_lib.oracle()
    slot = mxompi.TYPE[mxompi.MPI_DTYPE_SLOT[dt]]
    opi = mxompi.OP[opname[4:]]
    es = mxompi.type_size(slot)
    n = 5003
    rng = np.random.default_rng(opi * 100 + slot)
    if "LONG_DOUBLE" in dt:
        vals = rng.uniform(-3, 3, (2, n * es // 16)).astype(np.longdouble)
        a, b = (v.view(np.uint8).copy() for v in vals)
        if dt == "MPI_LONG_DOUBLE_INT":  # zero the int halves' padding, small ints in k
            for x in (a, b):
                x.reshape(-1, 32)[:, 16:] = 0
                x.reshape(-1, 32)[:, 16] = rng.integers(0, 9, n)
    elif dt == "MPI_C_BOOL":
        a, b = rng.integers(0, 2, (2, n), dtype=np.uint8)
    else:
        a, b = rng.integers(0, 256, (2, n * es), dtype=np.uint8)
    exp = b.copy()
    assert O.mxo_reduce2(opi, slot, a.ctypes.data, exp.ctypes.data, n, 1) == 0
    # coll/mi355x owns MPI_COMM_SELF's reduce_local at priority 80 (> coll/self 75);
    # below 75 the call goes coll/self -> ompi_op_reduce -> op/mi355x's slot
    assert H.mxh_comm_slot_owner(H.mxh_comm_self(), b"reduce_local") == b"mi355x"
    A = torch.from_numpy(a).cuda()
    B = torch.from_numpy(b.copy()).cuda()
    torch.cuda.synchronize()
    if route == "coll_reduce_local":
        rc = H.mxh_reduce_local(A.data_ptr(), B.data_ptr(), n, minihost.dtype(H, dt), minihost.op(H, opname))
    else:
        # ompi_op_reduce through the op table, as coll/self and every
        # coll/base algorithm call it: the slot must be op/mi355x's
        assert H.mxh_op_slot_owner(minihost.op(H, opname), slot, 0) == 1
        rc = H.mxh_op_reduce(minihost.op(H, opname), A.data_ptr(), B.data_ptr(), n, minihost.dtype(H, dt))
    assert rc == 0
    golden_io.assert_op_equal(B.cpu().numpy(), exp, opi, slot, f"{opname} {dt} via {route}")


@pytest.mark.gpu
def test_reduce_local_host_buffers_delegate_to_base(gpu_host):
    H = gpu_host
    O = oracle_lib.oracle()
    a = np.arange(100, dtype=np.float64)
    b = np.ones(100, dtype=np.float64)
    exp = b.copy()
    O.mxo_reduce2(2, 16, a.ctypes.data, exp.ctypes.data, 100, 1)
    assert H.mxh_reduce_local(a.ctypes.data, b.ctypes.data, 100, minihost.dtype(H, "MPI_DOUBLE"),
                              minihost.op(H, "MPI_MIN")) == 0
    np.testing.assert_array_equal(b, exp)
