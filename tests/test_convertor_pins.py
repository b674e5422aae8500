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


# ---- position.c (round 4) ----------------------------------------------------------
# test/datatype/position.c:220-275: MPI_LONG_DOUBLE_INT x 2048 (struct {long
# double ld; int i;}: ld at 0 with its 16-byte storage, i at 16, extent 32,
# size 20 -- DECLARE_MPI2_COMPOSED_STRUCT_DDT, ompi_datatype_module.c:404-434,
# 525), packed in 113-byte segments whose positions create_segments (:44-87)
# finds with opal_convertor_set_position, the segment order shuffled
# (shuffle_segments :89-101), every segment packed at its position
# (pack_segments :103-141) and unpacked at its position in the shuffled order
# (unpack_segments :143-180); expected (:254-268): recv[i].ld == send[i].ld and
# recv[i].i == send[i].i for every i.  send[i].ld = i + i / 100000.0, send[i].i = i.
# The reference starts recv as a copy of send (:236), which the positioned
# unpack must leave intact; the stronger variant starts recv filled with 0xEE:
# every packed byte must arrive and the 12 bytes of struct padding after `i`
# stay 0xEE (the convertor never writes outside the description).
FLOAT16 = 18                       # OPAL_DATATYPE_FLOAT16: long double on x86-64 (16-byte storage)
LDI = np.dtype([("ld", np.longdouble), ("i", "<i4"), ("pad", "<i4", 3)])   # 32 B
POS_COUNT, POS_FRAG = 2048, 113


def _long_double_int():
    return Desc([(FLOAT16, 1, 1, 16, 0), (INT4, 1, 1, 4, 16)], 20, 0, 32)


def _position_send():
    send = np.zeros(POS_COUNT, LDI)
    i = np.arange(POS_COUNT)
    send["ld"] = i.astype(np.longdouble) + i.astype(np.longdouble) / np.longdouble(100000.0)
    send["i"] = i
    return send


def _position_check(recv, send, strong):
    assert np.array_equal(recv["ld"], send["ld"]) and np.array_equal(recv["i"], send["i"]), \
        f"{int(np.sum((recv['ld'] != send['ld']) | (recv['i'] != send['i'])))} errors"
    if strong:
        rb, sb = recv.view(np.uint8).reshape(-1, 32), send.view(np.uint8).reshape(-1, 32)
        np.testing.assert_array_equal(rb[:, :20], sb[:, :20])       # every packed byte (incl. the x87 pad)
        assert np.all(rb[:, 20:] == 0xEE)                            # struct padding untouched


def test_position_long_double_int_segments_cover_the_stream():
    d = _long_double_int()
    assert d.size == 20 and d.ub - d.lb == LDI.itemsize == 32
    segs = _segments(d.size * POS_COUNT, POS_FRAG)
    assert len(segs) == -(-d.size * POS_COUNT // POS_FRAG)
    cover = np.zeros(d.size * POS_COUNT, np.int32)
    for p, l in segs:
        cover[p:p + l] += 1
    assert np.all(cover == 1)


@pytest.mark.parametrize("strong", [False, True], ids=["reference", "recv_filled"])
def test_position_long_double_int_cpu(strong):
    d = _long_double_int()
    send = _position_send()
    recv = send.copy()
    if strong:
        recv.view(np.uint8)[:] = 0xEE
    segs = _segments(d.size * POS_COUNT, POS_FRAG)
    bufs = {}
    for p, l in segs:
        buf = np.zeros(l, np.uint8)
        cpu_fragment(d, POS_COUNT, send.view(np.uint8), buf, p, l, False)
        bufs[p] = buf
    for p, l in segs:
        cpu_fragment(d, POS_COUNT, recv.view(np.uint8), bufs[p], p, l, True)
    _position_check(recv, send, strong)


@pytest.mark.gpu
@pytest.mark.parametrize("strong", [False, True], ids=["reference", "recv_filled"])
def test_position_long_double_int_device(strong):
    dev = Device(torch)
    d = _long_double_int()
    dt = dev.dt(d)
    send = _position_send()
    recv = send.copy()
    if strong:
        recv.view(np.uint8)[:] = 0xEE
    S, R = _dev(send), _dev(recv)
    segs = _segments(d.size * POS_COUNT, POS_FRAG)
    bufs = {p: torch.zeros(l, dtype=torch.uint8, device="cuda") for p, l in segs}
    for p, l in segs:                     # pack_segments: the shuffled order, each at its position
        dt.pack(POS_COUNT, S.data_ptr(), bufs[p].data_ptr(), offset=p, length=l, stream=dev.s)
    for p, l in segs:                     # unpack_segments
        dt.unpack(POS_COUNT, R.data_ptr(), bufs[p].data_ptr(), offset=p, length=l, stream=dev.s)
    torch.cuda.synchronize()
    got = np.frombuffer(R.cpu().numpy().tobytes(), LDI)
    _position_check(got, send, strong)
    dt.close()


# ---- large_data.c (round 4) --------------------------------------------------------
# test/datatype/large_data.c:87-174: types over 4 GB -- a contiguous of
# 20,000,000 floats indexed twice with blocks of 192 at displacements {576, 0}
# (sparse, 30.72 GB of data over a 61.44 GB span) and {192, 384} (adjacent
# blocks), a vector of INT_MAX/2 blocks of 4 floats at stride 4 (> 2^31
# elements), and contiguous(INT_MAX/2, contiguous(4, float)); expected: the
# bytes the convertor's raw walk covers (count_length_via_convertor_raw
# :34-85) == the type size.  Here that is mx_ddt_create's own check (the
# flattened walk's total must equal `size`, else MX_ERR_ARG), plus the span,
# plus pack / unpack windows at packed offsets above 4 GiB (and across the
# indexed type's block boundary) compared byte for byte with the user bytes
# they map to.
PER_TYPE, PER_PROC = 20_000_000, 192
CONTIG_BYTES = PER_TYPE * 4                         # ddt = contiguous(20M, MPI_FLOAT)
INT_MAX = 2 ** 31 - 1
FLOAT4 = 15


def _large_types():
    blk = PER_PROC * CONTIG_BYTES                   # one indexed block: 192 x 80 MB
    vcount = INT_MAX // 2
    return {
        # ompi_datatype_create_indexed(2, {192,192}, {576,0}, ddt)
        "1. INDEX": (Desc([(FLOAT4, 1, blk // 4, blk, 576 * CONTIG_BYTES), (FLOAT4, 1, blk // 4, blk, 0)],
                          2 * blk, 0, (576 + 192) * CONTIG_BYTES),
                     [(576 * CONTIG_BYTES, blk), (0, blk)]),
        # {192, 384}: adjacent blocks
        "2. INDEX": (Desc([(FLOAT4, 1, blk // 4, blk, 192 * CONTIG_BYTES), (FLOAT4, 1, blk // 4, blk, 384 * CONTIG_BYTES)],
                          2 * blk, 192 * CONTIG_BYTES, 576 * CONTIG_BYTES),
                     [(192 * CONTIG_BYTES, blk), (384 * CONTIG_BYTES, blk)]),
        # ompi_datatype_create_vector(INT_MAX/2, 4, 4, MPI_FLOAT)
        "3. VECTOR": (Desc([(FLOAT4, vcount, 4, 16, 0)], vcount * 16, 0, vcount * 16), [(0, vcount * 16)]),
        # contiguous(INT_MAX/2, contiguous(4, MPI_FLOAT))
        "4. CONTIG": (Desc([(FLOAT4, 1, vcount * 4, vcount * 16, 0)], vcount * 16, 0, vcount * 16),
                      [(0, vcount * 16)]),
    }


def _stream_to_user(blocks, off):
    """packed offset -> user byte offset (the blocks in packed order)"""
    for disp, n in blocks:
        if off < n:
            return disp + off
        off -= n
    raise ValueError(off)


def test_large_data_sizes_are_the_reference_formulas():
    T = _large_types()
    assert T["1. INDEX"][0].size == 2 * 192 * 20_000_000 * 4 == 30_720_000_000
    assert T["3. VECTOR"][0].size == (INT_MAX // 2) * 4 * 4 > 2 ** 32
    for name, (d, blocks) in T.items():
        assert sum(n for _, n in blocks) == d.size, name       # the raw walk's bytes == the type size


@pytest.mark.gpu
def test_large_data_device():
    dev = Device(torch)
    T = _large_types()
    for name, (d, blocks) in T.items():
        dt = dev.dt(d)                                          # raw length == size, checked at creation
        assert dt.size == d.size
        lo, hi = ctypes.c_int64(), ctypes.c_int64()
        assert mxompi.lib().mx_ddt_span(dt.h, 1, ctypes.byref(lo), ctypes.byref(hi)) == 0
        assert (lo.value, hi.value) == (min(b for b, _ in blocks), max(b + n for b, n in blocks)), name
        dt.close()
        with pytest.raises(mxompi.MxError):                    # a size the walk does not give is refused
            mxompi.Datatype(d.bytes, d.nrec, d.size + 4, d.lb, d.ub)
    # windows above 4 GiB: one user allocation covering the largest span (61.44 GB)
    span = max(max(b + n for b, n in bl) for _, bl in T.values())
    U = torch.empty(span, dtype=torch.uint8, device="cuda")
    gen = torch.Generator(device="cuda").manual_seed(4)
    W = (1 << 20) + 7
    cases = [("1. INDEX", (4 << 30) + 12345), ("1. INDEX", T["1. INDEX"][1][0][1] - 1000),   # across blocks
             ("1. INDEX", (20 << 30) + 3), ("3. VECTOR", (4 << 30) + 5), ("3. VECTOR", T["3. VECTOR"][0].size - W),
             ("4. CONTIG", (9 << 30) + 1)]
    for name, off in cases:
        d, blocks = T[name]
        dt = dev.dt(d)
        u0 = [_stream_to_user(blocks, off + k) for k in (0, W - 1)]
        pieces = []                                             # the user bytes of the window, in stream order
        k = 0
        while k < W:
            ua = _stream_to_user(blocks, off + k)
            run = W - k
            for disp, n in blocks:                              # stay inside one block
                if disp <= ua < disp + n:
                    run = min(run, disp + n - ua)
            pieces.append((ua, run))
            k += run
        for ua, n in pieces:
            U[ua:ua + n] = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=gen)
        exp = torch.cat([U[ua:ua + n] for ua, n in pieces])
        P = torch.zeros(W, dtype=torch.uint8, device="cuda")
        dt.pack(1, U.data_ptr(), P.data_ptr(), offset=off, length=W, stream=dev.s)
        torch.cuda.synchronize()
        assert torch.equal(P, exp), f"{name} pack window at {off} (user {u0})"
        # unpack the window back over zeroed user bytes
        for ua, n in pieces:
            U[ua:ua + n] = 0
        dt.unpack(1, U.data_ptr(), P.data_ptr(), offset=off, length=W, stream=dev.s)
        torch.cuda.synchronize()
        assert torch.equal(torch.cat([U[ua:ua + n] for ua, n in pieces]), exp), f"{name} unpack window at {off}"
        dt.close()
    del U
    torch.cuda.empty_cache()
