"""Size-1 communicators (MPI_COMM_SELF, a one-rank MPI_COMM_WORLD) on device
buffers.

coll/self answers every collective of a size-1 communicator with a local
copy over host memory (ompi_datatype_copy_content_same_ddt,
coll_self_allreduce.c:41-44, coll_self_reduce_scatter.c:44,
coll_self_reduce.c, coll_self_scan.c; ompi_datatype_sndrcv for allgather;
exscan touches nothing).  coll/mi355x takes those slots at priority 80 and
copies on the device when either buffer is device memory (one copy kernel for
contiguous layouts, the device convertor for derived ones); host-only calls
are delegated to the saved coll/self slot.  The mini-host's coll/self stand-in
copies with host memcpy, so a device buffer that reached it would fault the
test process -- and it counts its calls (mxh_self_calls), so delegation is
checked, not inferred.

MPI_Allreduce / MPI_Reduce reject derived datatypes with an intrinsic op
(ompi_op_is_valid, op.h:477-514; the harness's entry points check it too),
so vector layouts are driven through the slots whose entry points reach the
component with any datatype: reduce_scatter, reduce_scatter_block, scan and
allgather (sndrcv between different send and receive layouts)."""
import numpy as np
import pytest

import minihost
import mxompi

torch = pytest.importorskip("torch")

IN_PLACE = 1
N = 1 << 20          # contiguous floats per call (4 MiB)
VEC = (4, 3, 5)      # MPI_Type_vector(count, blocklen, stride) of MPI_FLOAT
NINST = 5003         # vector instances per call (ragged)


@pytest.fixture(scope="module")
def H():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    mxompi.init(0)
    return minihost.host(with_components=True)


def _call(H, slot, sb, rb, count, dt, sdt=None, scount=None):
    c = H.mxh_comm_self()
    SUM = minihost.op(H, "MPI_SUM")
    if slot == "allreduce":
        return H.mxh_allreduce(sb, rb, count, dt, SUM, c)
    if slot == "reduce":
        return H.mxh_reduce(sb, rb, count, dt, SUM, 0, c)
    if slot == "scan":
        return H.mxh_scan(sb, rb, count, dt, SUM, c)
    if slot == "exscan":
        return H.mxh_exscan(sb, rb, count, dt, SUM, c)
    if slot == "reduce_scatter":
        import ctypes
        rc = (ctypes.c_int * 1)(count)
        return H.mxh_reduce_scatter(sb, rb, rc, dt, SUM, c)
    if slot == "reduce_scatter_block":
        return H.mxh_reduce_scatter_block(sb, rb, count, dt, SUM, c)
    if slot == "allgather":
        return H.mxh_allgather(sb, scount if scount is not None else count, sdt or dt, rb, count, dt, c)
    raise AssertionError(slot)


SLOTS = ["allreduce", "reduce", "scan", "exscan", "reduce_scatter", "reduce_scatter_block", "allgather"]


@pytest.mark.gpu
def test_slots_owned_by_mi355x(H):
    c = H.mxh_comm_self()
    for s in SLOTS + ["reduce_local"]:
        assert H.mxh_comm_slot_owner(c, s.encode()) == b"mi355x", s
    assert H.mxh_comm_slot_owner(c, b"bcast") == b"self"     # nothing to copy: left to coll/self


@pytest.mark.gpu
@pytest.mark.parametrize("inplace", [False, True], ids=["copy", "in_place"])
def test_contiguous_device_buffers(H, inplace):
    f32 = minihost.dtype(H, "MPI_FLOAT")
    rng = np.random.default_rng(11)
    for slot in SLOTS:
        src = rng.standard_normal(N).astype(np.float32)
        old = rng.standard_normal(N).astype(np.float32)
        S = torch.from_numpy(src).cuda()
        R = torch.from_numpy(old if not inplace else src).clone().cuda()
        torch.cuda.synchronize()
        before = H.mxh_self_calls()
        rc = _call(H, slot, IN_PLACE if inplace else S.data_ptr(), R.data_ptr(), N, f32)
        assert rc == 0, slot
        assert H.mxh_self_calls() == before, f"{slot}: device call delegated to coll/self's host copy"
        got = R.cpu().numpy()
        # exscan on one rank leaves rbuf untouched (coll_self_exscan.c); in
        # place every slot's result is the input already there
        exp = old if (slot == "exscan" and not inplace) else src
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), slot


def _vec_mask(ninst):
    cnt, blen, stride = VEC
    ext = (cnt - 1) * stride + blen
    m = np.zeros(ninst * ext, dtype=bool)
    for i in range(ninst):
        for b in range(cnt):
            m[i * ext + b * stride: i * ext + b * stride + blen] = True
    return m


@pytest.mark.gpu
@pytest.mark.parametrize("slot", ["reduce_scatter", "reduce_scatter_block", "scan", "allgather"])
def test_vector_device_buffers_gaps_untouched(H, slot):
    f32 = minihost.dtype(H, "MPI_FLOAT")
    vec = H.mxh_dtype_vector(*VEC, f32)
    mask = _vec_mask(NINST)
    rng = np.random.default_rng(12)
    src = rng.standard_normal(mask.size).astype(np.float32)
    old = rng.standard_normal(mask.size).astype(np.float32)
    S = torch.from_numpy(src).cuda()
    R = torch.from_numpy(old).cuda()
    torch.cuda.synchronize()
    before = H.mxh_self_calls()
    assert _call(H, slot, S.data_ptr(), R.data_ptr(), NINST, vec) == 0
    assert H.mxh_self_calls() == before
    got = R.cpu().numpy()
    exp = np.where(mask, src, old)                    # data copied, gap bytes as they were
    assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), slot


@pytest.mark.gpu
@pytest.mark.parametrize("direction", ["contig_to_vector", "vector_to_contig"])
def test_allgather_sndrcv_between_layouts(H, direction):
    """ompi_datatype_sndrcv: the send layout packed, the receive layout unpacked."""
    f32 = minihost.dtype(H, "MPI_FLOAT")
    vec = H.mxh_dtype_vector(*VEC, f32)
    mask = _vec_mask(NINST)
    per = VEC[0] * VEC[1]
    rng = np.random.default_rng(13)
    if direction == "contig_to_vector":
        packed = rng.standard_normal(NINST * per).astype(np.float32)
        old = rng.standard_normal(mask.size).astype(np.float32)
        S, R = torch.from_numpy(packed).cuda(), torch.from_numpy(old).cuda()
        torch.cuda.synchronize()
        assert H.mxh_allgather(S.data_ptr(), NINST * per, f32, R.data_ptr(), NINST, vec, H.mxh_comm_self()) == 0
        exp = old.copy()
        exp[mask] = packed
    else:
        user = rng.standard_normal(mask.size).astype(np.float32)
        old = rng.standard_normal(NINST * per).astype(np.float32)
        S, R = torch.from_numpy(user).cuda(), torch.from_numpy(old).cuda()
        torch.cuda.synchronize()
        assert H.mxh_allgather(S.data_ptr(), NINST, vec, R.data_ptr(), NINST * per, f32, H.mxh_comm_self()) == 0
        exp = user[mask]
    assert np.array_equal(R.cpu().numpy().view(np.uint32), exp.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["host_to_device", "device_to_host"])
def test_mixed_locations(H, where):
    """One buffer in host memory, the other on the device: the component moves
    it (coll/self would host-memcpy the device side)."""
    f32 = minihost.dtype(H, "MPI_FLOAT")
    vec = H.mxh_dtype_vector(*VEC, f32)
    rng = np.random.default_rng(14)
    src = rng.standard_normal(N).astype(np.float32)
    old = rng.standard_normal(N).astype(np.float32)
    if where == "host_to_device":
        R = torch.from_numpy(old.copy()).cuda()
        torch.cuda.synchronize()
        assert _call(H, "allreduce", src.ctypes.data, R.data_ptr(), N, f32) == 0
        got = R.cpu().numpy()
    else:
        S = torch.from_numpy(src).cuda()
        got = old.copy()
        torch.cuda.synchronize()
        assert _call(H, "allreduce", S.data_ptr(), got.ctypes.data, N, f32) == 0
    assert np.array_equal(got.view(np.uint32), src.view(np.uint32))
    # a vector layout on each side
    mask = _vec_mask(NINST)
    vs = rng.standard_normal(mask.size).astype(np.float32)
    vo = rng.standard_normal(mask.size).astype(np.float32)
    if where == "host_to_device":
        R = torch.from_numpy(vo.copy()).cuda()
        torch.cuda.synchronize()
        assert _call(H, "scan", vs.ctypes.data, R.data_ptr(), NINST, vec) == 0
        got = R.cpu().numpy()
    else:
        S = torch.from_numpy(vs).cuda()
        got = vo.copy()
        torch.cuda.synchronize()
        assert _call(H, "scan", S.data_ptr(), got.ctypes.data, NINST, vec) == 0
    assert np.array_equal(got.view(np.uint32), np.where(mask, vs, vo).view(np.uint32))


@pytest.mark.gpu
def test_host_buffers_delegate_to_coll_self(H):
    f32 = minihost.dtype(H, "MPI_FLOAT")
    rng = np.random.default_rng(15)
    for slot in SLOTS:
        src = rng.standard_normal(4096).astype(np.float32)
        dst = np.zeros(4096, dtype=np.float32)
        before = H.mxh_self_calls()
        assert _call(H, slot, src.ctypes.data, dst.ctypes.data, 4096, f32) == 0
        # exscan never reaches coll/self: nothing to do on one rank, device or not
        assert H.mxh_self_calls() == before + (slot != "exscan"), slot
        if slot != "exscan":
            assert np.array_equal(dst, src), slot
