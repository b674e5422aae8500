"""The reference's own convertor tests, restated: their datatypes, inputs,
fragment schedules and EXPECTED VALUES are taken from the test sources and
run through the CPU oracle and the device convertor.  These are the known
answers the reference holds for this path, so they pin the
convertor independently of any golden file.

* test/datatype/position_noncontig.c:197-237 -- MPI_Type_vector(150, 1, 2,
  MPI_INT); the packed stream is cut into 113-byte segments (positions found
  with opal_convertor_set_position), the segment order is shuffled
  (shuffle_segments :86-98), every segment is packed and unpacked at its own
  position; expected: recv[i] = i for even i, 0xdeadbeef for odd i.
* test/datatype/unpack_ooo.c:157-296 -- struct {vector(2,1,2,INT) @0,
  vector(2,1,2,DOUBLE) @16} x 331, unpacked out of order from the packed
  image of `struct pfoo_t[331]` with the test's four fragment schedules
  (test1..test4, :199-247, fragments split basic elements); expected
  (:120-127): bar.i[0] = pbar.i[0], bar.i[1] = 0, bar.i[2] = pbar.i[1],
  bar.d[0] = pbar.d[0], bar.d[1] = 0, bar.d[2] = pbar.d[1].
* test/datatype/opal_datatype_test.c:64-132 + opal_ddt_lib.c:498-563
  (upper_matrix, init_random_upper_matrix, check_diag_matrix) -- the upper
  triangle of a 500x500 double matrix, unpacked in chunks of (N+1)*8 bytes
  into a zeroed matrix; expected: check_diag_matrix (every upper-triangle
  element equal), plus the lower triangle untouched.
* test/datatype/opal_datatype_test.c:377-456 (RESET_CONVERTORS) -- after
  each chunk the convertor is set back to position 0 and then forward to
  the bytes done so far, and must resume exactly there: here a fragment is
  re-converted from position 0 before every next one, and the stream must
  equal the one-shot conversion.

The descriptions are built by ddt_build below: MPI constructors restated as
description records (opal_datatype_internal.h:146-196 -- ELEM {flags, type,
count, blocklen, extent, disp}), the input of mx_ddt_create.
"""
import ctypes
import struct

import numpy as np
import pytest

import mxompi
import oracle_lib

vp, sz = ctypes.c_void_p, ctypes.c_size_t

# OPAL basic type ids (opal_datatype_internal.h:50-80) and LP64 sizes
INT4, FLOAT8 = 6, 16
BASIC = np.array([0, 0, 0, 0, 1, 2, 4, 8, 16, 1, 2, 4, 8, 16, 2, 4, 8, 16, 16, 4, 8, 16, 32, 1, 4, 0], np.uint64)
F_DATA = 0x0100
T_END_LOOP = 1


class Desc:
    """A committed-description stand-in: ELEM records + the datatype's size,
    lb and ub (the arguments of mx_ddt_create)."""

    def __init__(self, elems, size, lb, ub):
        recs = b"".join(struct.pack("<HHIQqq", F_DATA, t, cnt, blen, ext, disp)
                        for t, cnt, blen, ext, disp in elems)
        recs += struct.pack("<HHIQqq", 0, T_END_LOOP, len(elems), 0, size, 0)
        self.bytes = recs
        self.nrec = len(elems) + 1
        self.size, self.lb, self.ub = size, lb, ub


def vector(count, blocklen, stride, t, es):
    """MPI_Type_vector(count, blocklen, stride, t): extent (count-1)*stride + blocklen elements."""
    return Desc([(t, count, blocklen, stride * es, 0)], count * blocklen * es, 0,
                ((count - 1) * stride + blocklen) * es)


def struct_of(members, lb, ub):
    """MPI_Type_create_struct of (Desc, byte displacement) members (count 1 each)."""
    elems, size = [], 0
    for d, disp in members:
        for t, cnt, blen, ext, dd in _elems(d):
            elems.append((t, cnt, blen, ext, dd + disp))
        size += d.size
    return Desc(elems, size, lb, ub)


def indexed(blocklens, disps, t, es):
    """MPI_Type_indexed / opal_datatype_create_indexed (displacements in elements)."""
    elems = [(t, 1, b, b * es, d * es) for b, d in zip(blocklens, disps) if b]
    lo = min(d for b, d in zip(blocklens, disps) if b) * es
    hi = max((d + b) for b, d in zip(blocklens, disps) if b) * es
    return Desc(elems, sum(blocklens) * es, lo, hi)


def _elems(d):
    out = []
    for k in range(d.nrec - 1):
        _, t, cnt, blen, ext, disp = struct.unpack_from("<HHIQqq", d.bytes, 32 * k)
        out.append((t, cnt, blen, ext, disp))
    return out


# ---- the two convertor implementations under test ---------------------------
def cpu_convert(d, count, user, packed, unpack):
    """CPU oracle (oracle/mx_oracle_ddt.c): the whole stream at once."""
    O = oracle_lib.oracle()
    O.mxo_ddt_convert.argtypes = [vp, sz, vp, ctypes.c_int64, ctypes.c_int64, sz, vp, vp, ctypes.c_int]
    desc = np.frombuffer(d.bytes, np.uint8).copy()
    n = O.mxo_ddt_convert(desc.ctypes.data, d.nrec, BASIC.ctypes.data, d.lb, d.ub, count, user.ctypes.data,
                          packed.ctypes.data, 1 if unpack else 0)
    assert n == d.size * count


def cpu_fragment(d, count, user, packed, offset, length, unpack):
    """Fragment [offset, offset+length) of the stream through the oracle: the
    oracle converts whole streams, so a fragment is cut out of (pack) or
    merged into (unpack) a full conversion -- the byte semantics the device
    convertor must reproduce one fragment at a time."""
    total = d.size * count
    if not unpack:
        full = np.zeros(total, np.uint8)
        cpu_convert(d, count, user, full, False)
        packed[:] = full[offset:offset + length]
        return
    # unpack: pack what `user` holds now, splice the fragment in, unpack the whole
    full = np.zeros(total, np.uint8)
    cpu_convert(d, count, user, full, False)
    full[offset:offset + length] = packed[:length]
    cpu_convert(d, count, user, full, True)


class Device:
    def __init__(self, torch):
        self.torch = torch
        mxompi.init(0)
        self.s = torch.cuda.current_stream().cuda_stream

    def dt(self, d):
        return mxompi.Datatype(d.bytes, d.nrec, d.size, d.lb, d.ub)


# ---- position_noncontig.c --------------------------------------------------------
def _segments(total, seg):
    segs = [(p, min(seg, total - p)) for p in range(0, total, seg)]
    n = len(segs)
    for i in range(0, n // 2, 2):                       # shuffle_segments (position_noncontig.c:86-98)
        segs[i], segs[n - i - 1] = segs[n - i - 1], segs[i]
    return segs


def _position_noncontig_expected():
    NELT = 300
    return np.array([i if i % 2 == 0 else -559038737 for i in range(NELT)], np.int32)   # 0xdeadbeef


def test_position_noncontig_cpu():
    d = vector(150, 1, 2, INT4, 4)
    send = np.arange(300, dtype=np.int32)
    recv = np.full(300, -559038737, np.int32)
    segs = _segments(d.size, 113)
    bufs = {}
    for p, l in segs:                                    # pack every segment at its position
        buf = np.zeros(l, np.uint8)
        cpu_fragment(d, 1, send.view(np.uint8), buf, p, l, False)
        bufs[p] = buf
    for p, l in segs:                                    # unpack in the shuffled order
        cpu_fragment(d, 1, recv.view(np.uint8), bufs[p], p, l, True)
    np.testing.assert_array_equal(recv, _position_noncontig_expected())


# ---- unpack_ooo.c -------------------------------------------------------------------
N_OOO = 331
OOO_TESTS = {
    "test1": [(992, 0), (1325, 992), (992, 2317), (992, 3309), (992, 4301), (992, 5293), (992, 6285), (667, 7277)],
    "test2": [(992, 0), (992, 2317), (992, 3309), (992, 4301), (992, 5293), (992, 6285), (1325, 992), (667, 7277)],
    "test3": [(992, 0), (4960, 2317), (1325, 992), (667, 7277)],
    "test4": [(992, 0), (992, 2976), (992, 1984), (992, 992), (3976, 3968)],
}
FOO = np.dtype([("i", "<i4", 3), ("pad", "<i4"), ("d", "<f8", 3)])    # struct foo_t, 40 B
PFOO = np.dtype([("i", "<i4", 2), ("d", "<f8", 2)])                  # struct pfoo_t, 24 B


def _ooo_type():
    t1 = vector(2, 1, 2, INT4, 4)
    t2 = vector(2, 1, 2, FLOAT8, 8)
    return struct_of([(t1, 0), (t2, 16)], 0, 40)


def _ooo_buffers():
    j = np.arange(N_OOO)
    pbar = np.zeros(N_OOO, PFOO)
    pbar["i"][:, 0] = 123 + j
    pbar["i"][:, 1] = 789 + j
    pbar["d"][:, 0] = 123.456 + j
    pbar["d"][:, 1] = 789.123 + j
    bar = np.zeros(N_OOO, FOO)
    bar_bytes = bar.view(np.uint8).reshape(N_OOO, 40)
    bar_bytes[:, 0:4] = 0xFF          # i[0]
    bar_bytes[:, 8:12] = 0xFF         # i[2]
    bar_bytes[:, 16:24] = 0xFF        # d[0]
    bar_bytes[:, 32:40] = 0xFF        # d[2]
    return pbar, bar


def _ooo_check(bar, pbar, name):
    ok = ((bar["i"][:, 0] == pbar["i"][:, 0]) & (bar["i"][:, 1] == 0) & (bar["i"][:, 2] == pbar["i"][:, 1]) &
          (bar["d"][:, 0] == pbar["d"][:, 0]) & (bar["d"][:, 1] == 0.0) & (bar["d"][:, 2] == pbar["d"][:, 1]))
    bad = np.nonzero(~ok)[0]
    assert not len(bad), f"unpack_ooo {name}: {len(bad)} wrong elements, first at {bad[0]}"


def test_unpack_ooo_type_matches_the_test_structs():
    d = _ooo_type()
    assert d.size == PFOO.itemsize == 24 and d.ub - d.lb == FOO.itemsize == 40
    for segs in OOO_TESTS.values():                      # every schedule covers the stream exactly
        cover = np.zeros(d.size * N_OOO, np.int32)
        for l, p in segs:
            cover[p:p + l] += 1
        assert np.all(cover == 1)


@pytest.mark.parametrize("name", list(OOO_TESTS))
def test_unpack_ooo_cpu(name):
    d = _ooo_type()
    pbar, bar = _ooo_buffers()
    src = pbar.view(np.uint8)
    for l, p in OOO_TESTS[name]:
        cpu_fragment(d, N_OOO, bar.view(np.uint8), src[p:p + l].copy(), p, l, True)
    _ooo_check(bar, pbar, name)


# ---- opal_datatype_test.c test_upper ---------------------------------------------
UPPER_N = 500


def _upper():
    n = UPPER_N
    d = indexed([n - i for i in range(n)], [i * n + i for i in range(n)], FLOAT8, 8)   # opal_ddt_lib.c:534-563
    rng = np.random.default_rng(500)
    mat1 = np.zeros((n, n))
    iu = np.triu_indices(n)
    mat1[iu] = rng.integers(0, 2 ** 31, len(iu[0])).astype(np.float64)               # init_random_upper_matrix
    inbuf = mat1[iu].copy()                            # row-major upper triangle = the packed stream
    return d, mat1, inbuf


def check_diag_matrix(n, mat1, mat2):
    """opal_ddt_lib.c:513-531"""
    iu = np.triu_indices(n)
    return bool(np.array_equal(mat1[iu], mat2[iu]))


def test_upper_matrix_cpu():
    d, mat1, inbuf = _upper()
    n = UPPER_N
    assert d.size == n * (n + 1) // 2 * 8
    mat2 = np.zeros((n, n))
    src = inbuf.view(np.uint8)
    chunk = (n + 1) * 8                                   # split_chunk (opal_datatype_test.c:100)
    for p in range(0, len(src), chunk):
        l = min(chunk, len(src) - p)
        cpu_fragment(d, 1, mat2.view(np.uint8).reshape(-1), src[p:p + l].copy(), p, l, True)
    assert check_diag_matrix(n, mat1, mat2)
    assert not np.any(mat2[np.tril_indices(n, -1)])


# ---- device ------------------------------------------------------------------------
torch = pytest.importorskip("torch")


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()


@pytest.mark.gpu
def test_position_noncontig_device():
    dev = Device(torch)
    d = vector(150, 1, 2, INT4, 4)
    dt = dev.dt(d)
    send = _dev(np.arange(300, dtype=np.int32))
    recv = _dev(np.full(300, -559038737, np.int32))
    segs = _segments(d.size, 113)
    bufs = {p: torch.zeros(l, dtype=torch.uint8, device="cuda") for p, l in segs}
    for p, l in segs:
        dt.pack(1, send.data_ptr(), bufs[p].data_ptr(), offset=p, length=l, stream=dev.s)
    for p, l in segs:
        dt.unpack(1, recv.data_ptr(), bufs[p].data_ptr(), offset=p, length=l, stream=dev.s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(recv.cpu().numpy().view(np.int32), _position_noncontig_expected())
    dt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(OOO_TESTS))
def test_unpack_ooo_device(name):
    dev = Device(torch)
    d = _ooo_type()
    dt = dev.dt(d)
    pbar, bar = _ooo_buffers()
    B = _dev(bar)
    src = pbar.view(np.uint8)
    for l, p in OOO_TESTS[name]:
        # the fragment sits between 1 KiB of 0xAA garbage on each side (unpack_ooo.c:92-99)
        frag = np.full(l + 2048, 0xAA, np.uint8)
        frag[1024:1024 + l] = src[p:p + l]
        F = _dev(frag)
        dt.unpack(N_OOO, B.data_ptr(), F.data_ptr() + 1024, offset=p, length=l, stream=dev.s)
    torch.cuda.synchronize()
    got = B.cpu().numpy().view(FOO)
    _ooo_check(got, pbar, name)
    dt.close()


@pytest.mark.gpu
def test_upper_matrix_device():
    dev = Device(torch)
    d, mat1, inbuf = _upper()
    n = UPPER_N
    dt = dev.dt(d)
    M = _dev(np.zeros((n, n)))
    S = _dev(inbuf)
    chunk = (n + 1) * 8
    for p in range(0, d.size, chunk):
        l = min(chunk, d.size - p)
        dt.unpack(1, M.data_ptr(), S.data_ptr() + p, offset=p, length=l, stream=dev.s)
    torch.cuda.synchronize()
    mat2 = M.cpu().numpy().view(np.float64).reshape(n, n)
    assert check_diag_matrix(n, mat1, mat2)
    assert not np.any(mat2[np.tril_indices(n, -1)])
    dt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [11, 12, 48, 82, 956, 6000, 16384, 36000])
def test_reset_position_resumes_exactly_device(chunk):
    """RESET_CONVERTORS (opal_datatype_test.c:377-456): before every fragment
    the conversion is restarted from position 0 (fragment [0, done) again) and
    then resumed at `done`; the stream and the unpacked layout must equal the
    one-shot conversion.  Types: the unpack_ooo struct and the upper matrix,
    at the test suite's chunk sizes (opal_datatype_test.c:500-721)."""
    dev = Device(torch)
    for d, count, user in ((_ooo_type(), N_OOO, _ooo_buffers()[1].view(np.uint8)),
                           (_upper()[0], 1, _upper()[1].view(np.uint8).reshape(-1))):
        dt = dev.dt(d)
        total = d.size * count
        U = _dev(user)
        ref = torch.zeros(total, dtype=torch.uint8, device="cuda")
        dt.pack(count, U.data_ptr(), ref.data_ptr(), stream=dev.s)
        P = torch.zeros(total, dtype=torch.uint8, device="cuda")
        R = torch.zeros_like(U)
        done = 0
        while done < total:
            if done:
                dt.pack(count, U.data_ptr(), P.data_ptr(), offset=0, length=done, stream=dev.s)
                dt.unpack(count, R.data_ptr(), P.data_ptr(), offset=0, length=done, stream=dev.s)
            l = min(chunk, total - done)
            dt.pack(count, U.data_ptr(), P.data_ptr() + done, offset=done, length=l, stream=dev.s)
            dt.unpack(count, R.data_ptr(), P.data_ptr() + done, offset=done, length=l, stream=dev.s)
            done += l
        torch.cuda.synchronize()
        assert torch.equal(P, ref)
        full = torch.zeros_like(U)
        dt.unpack(count, full.data_ptr(), ref.data_ptr(), stream=dev.s)
        torch.cuda.synchronize()
        assert torch.equal(R, full)
        dt.close()
