"""Derived-datatype pack/unpack (convertor).

CPU: the oracle restatement (oracle/mx_oracle_ddt.c) reproduces the
reference engine's packed streams and unpack results for every golden type
(tests/golden/ddt_vectors.bin, produced by the reference's own
opal_convertor from its committed descriptions, incl. the reference test
suite's types: BLACS indexed, triangular matrices, "strange", resized
structs ...).
GPU: the device convertor (mx_ddt_create + mx_pack/mx_unpack) built from
the same committed descriptions matches bit for bit -- whole-message and
resumed at odd fragment boundaries (the convertor's bConverted /
set_position semantics) -- and at CFG-C sizes against the oracle.
"""
import ctypes

import numpy as np
import pytest

import golden_io
import mxompi
import oracle_lib

BASIC, RECS = golden_io.ddt_records()
vp, sz = ctypes.c_void_p, ctypes.c_size_t


def _oracle():
    O = oracle_lib.oracle()
    O.mxo_ddt_convert.argtypes = [vp, sz, vp, ctypes.c_int64, ctypes.c_int64, sz, vp, vp, ctypes.c_int]
    return O


def _cpu(rec, unpack):
    O = _oracle()
    bs = np.ascontiguousarray(BASIC)
    if not unpack:
        user = rec["user"].copy()
        out = np.zeros(rec["size"] * rec["count"], np.uint8)
        O.mxo_ddt_convert(rec["desc"].ctypes.data, rec["nrec"], bs.ctypes.data, rec["lb"], rec["ub"],
                          rec["count"], user.ctypes.data - rec["true_lb"], out.ctypes.data, 0)
        return out
    user = rec["prefill"].copy()
    packed = rec["packed"].copy()
    O.mxo_ddt_convert(rec["desc"].ctypes.data, rec["nrec"], bs.ctypes.data, rec["lb"], rec["ub"], rec["count"],
                      user.ctypes.data - rec["true_lb"], packed.ctypes.data, 1)
    return user


def test_basic_type_sizes_match_builtin_table():
    # the device library's built-in LP64 table == the reference build's
    builtin = [0, 0, 0, 0, 1, 2, 4, 8, 16, 1, 2, 4, 8, 16, 2, 4, 8, 16, 16, 4, 8, 16, 32, 1, 4, 0]
    ref = [int(x) for x in BASIC]
    for i, (a, b) in enumerate(zip(builtin, ref)):
        if b:  # UNAVAILABLE/markers may be 0
            assert a == b, i


@pytest.mark.parametrize("rec", RECS, ids=lambda r: r["name"])
def test_oracle_pack_unpack_match_reference(rec):
    np.testing.assert_array_equal(_cpu(rec, False), rec["packed"])
    np.testing.assert_array_equal(_cpu(rec, True), rec["unpacked"])


torch = pytest.importorskip("torch")


def _dt(rec):
    return mxompi.Datatype(rec["desc"].tobytes(), rec["nrec"], rec["size"], rec["lb"], rec["ub"])


@pytest.mark.gpu
@pytest.mark.parametrize("rec", RECS, ids=lambda r: r["name"])
def test_device_pack_unpack_match_reference(rec):
    mxompi.init(0)
    dt = _dt(rec)
    total = rec["size"] * rec["count"]
    U = torch.from_numpy(rec["user"].copy()).cuda()
    P = torch.zeros(total, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    base = U.data_ptr() - rec["true_lb"]
    dt.pack(rec["count"], base, P.data_ptr(), stream=s)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(P.cpu().numpy(), rec["packed"], err_msg=rec["name"] + " pack")
    # resumable: odd fragments at odd offsets (opal_datatype_test.c chunk sizes)
    for chunk in (11, 48, 956, 6000):
        P2 = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
        off = 0
        while off < total:
            ln = min(chunk, total - off)
            dt.pack(rec["count"], base, P2.data_ptr() + off, offset=off, length=ln, stream=s)
            off += ln
        torch.cuda.synchronize()
        np.testing.assert_array_equal(P2.cpu().numpy()[:total], rec["packed"], err_msg=f"{rec['name']} chunk {chunk}")
    # unpack into the prefilled buffer (gaps keep the prefill), whole and fragmented
    for chunk in (None, 13, 1000):
        D = torch.from_numpy(rec["prefill"].copy()).cuda()
        Pk = torch.from_numpy(rec["packed"].copy()).cuda()
        dbase = D.data_ptr() - rec["true_lb"]
        if chunk is None:
            dt.unpack(rec["count"], dbase, Pk.data_ptr(), stream=s)
        else:
            off = 0
            while off < total:
                ln = min(chunk, total - off)
                dt.unpack(rec["count"], dbase, Pk.data_ptr() + off, offset=off, length=ln, stream=s)
                off += ln
        torch.cuda.synchronize()
        np.testing.assert_array_equal(D.cpu().numpy(), rec["unpacked"], err_msg=f"{rec['name']} unpack {chunk}")


@pytest.mark.gpu
@pytest.mark.parametrize("shift", [0, 3, 4, 8])
@pytest.mark.parametrize("name", ["vector_f32_b1_s2", "vector_f32_b4_s8", "vector_f32_b16_s32",
                                  "vector_f32_b64_s128", "indexed_f32_random", "struct_char_d3_int_resized48",
                                  "ref_lower_matrix_47", "ref_strange", "ref_blacs_indexed"])
def test_device_pack_large_cfg_c(name, shift):
    """The golden type description with a large instance count (16 MiB
    packed: thousands of tiles), user buffer aligned or shifted by 3, 4, 8
    bytes, checked against the oracle restatement."""
    mxompi.init(0)
    rec = next(r for r in RECS if r["name"] == name)
    dt = _dt(rec)
    count = max(1, (16 << 20) // rec["size"]) + 7      # thousands of tiles (below the 384 MiB nt threshold either way)
    ext = rec["ub"] - rec["lb"]
    span = ext * (count - 1) + rec["true_ub"] - rec["true_lb"]
    rng = np.random.default_rng(5)
    user = rng.integers(0, 256, span, dtype=np.uint8)
    exp = np.zeros(rec["size"] * count, np.uint8)
    O = _oracle()
    O.mxo_ddt_convert(rec["desc"].ctypes.data, rec["nrec"], np.ascontiguousarray(BASIC).ctypes.data, rec["lb"],
                      rec["ub"], count, user.ctypes.data - rec["true_lb"], exp.ctypes.data, 0)
    Ubuf = torch.zeros(span + 16, dtype=torch.uint8, device="cuda")
    Ubuf[shift:shift + span] = torch.from_numpy(user).cuda()
    P = torch.zeros(exp.size, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    dt.pack(count, Ubuf.data_ptr() + shift - rec["true_lb"], P.data_ptr(), stream=st)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(P.cpu().numpy(), exp)
    # fragments that straddle tiles, at odd offsets
    P2 = torch.zeros(exp.size + 16, dtype=torch.uint8, device="cuda")
    off = 0
    while off < exp.size:
        ln = min(100003, exp.size - off)
        dt.pack(count, Ubuf.data_ptr() + shift - rec["true_lb"], P2.data_ptr() + off, offset=off, length=ln, stream=st)
        off += ln
    torch.cuda.synchronize()
    np.testing.assert_array_equal(P2.cpu().numpy()[:exp.size], exp)
    # and back (whole, then fragmented into a second buffer)
    Dbuf = torch.zeros(span + 16, dtype=torch.uint8, device="cuda")
    dt.unpack(count, Dbuf.data_ptr() + shift - rec["true_lb"], P.data_ptr(), stream=st)
    D2 = torch.zeros(span + 16, dtype=torch.uint8, device="cuda")
    off = 0
    while off < exp.size:
        ln = min(77777, exp.size - off)
        dt.unpack(count, D2.data_ptr() + shift - rec["true_lb"], P.data_ptr() + off, offset=off, length=ln, stream=st)
        off += ln
    torch.cuda.synchronize()
    got = Dbuf.cpu().numpy()[shift:shift + span]
    np.testing.assert_array_equal(D2.cpu().numpy()[shift:shift + span], got)
    exp_u = np.zeros(span, np.uint8)
    O.mxo_ddt_convert(rec["desc"].ctypes.data, rec["nrec"], np.ascontiguousarray(BASIC).ctypes.data, rec["lb"],
                      rec["ub"], count, exp_u.ctypes.data - rec["true_lb"], exp.ctypes.data, 1)
    np.testing.assert_array_equal(got, exp_u)


# ---- BLOCK kernels (k_convert_blk): large instances, and every golden type forced --------
def _check_device_vs_oracle(d, dt, count, shift=0, pshift=0, chunks=(None,), rng_seed=11, expect_path="block",
                            expect_unpack="same"):
    """pack whole / in fragments and unpack into a prefilled buffer, each vs the
    oracle restatement; user buffer displaced by `shift` bytes, packed buffer
    by `pshift` bytes; asserts the kernel family that ran (None: any)."""
    if expect_unpack == "same":
        expect_unpack = expect_path
    O = _oracle()
    bs = np.ascontiguousarray(BASIC)
    ext = d.ub - d.lb
    # true span from the flattened records: [min disp, max disp + len) of instance 0 + (count-1) * ext
    tl, tu = d.true_lb, d.true_ub
    span = ext * (count - 1) + tu - tl
    rng = np.random.default_rng(rng_seed)
    user = rng.integers(0, 256, span, dtype=np.uint8)
    total = d.size * count
    exp = np.zeros(total, np.uint8)
    O.mxo_ddt_convert(d.desc.ctypes.data, d.nrec, bs.ctypes.data, d.lb, d.ub, count, user.ctypes.data - tl,
                      exp.ctypes.data, 0)
    st = torch.cuda.current_stream().cuda_stream
    U = torch.zeros(span + 32, dtype=torch.uint8, device="cuda")
    U[shift:shift + span] = torch.from_numpy(user).cuda()
    ubase = U.data_ptr() + shift - tl
    for chunk in chunks:
        P = torch.zeros(total + 32, dtype=torch.uint8, device="cuda")
        off = 0
        while off < total:
            ln = total - off if chunk is None else min(chunk, total - off)
            dt.pack(count, ubase, P.data_ptr() + pshift + off, offset=off, length=ln, stream=st)
            off += ln
        torch.cuda.synchronize()
        assert expect_path is None or dt.last_path == expect_path
        got = P.cpu().numpy()
        np.testing.assert_array_equal(got[pshift:pshift + total], exp, err_msg=f"pack chunk {chunk}")
        assert not got[:pshift].any() and not got[pshift + total:].any(), "pack wrote outside its window"
    pre = rng.integers(0, 256, span, dtype=np.uint8)
    exp_u = pre.copy()
    O.mxo_ddt_convert(d.desc.ctypes.data, d.nrec, bs.ctypes.data, d.lb, d.ub, count, exp_u.ctypes.data - tl,
                      exp.ctypes.data, 1)
    Pk = torch.zeros(total + 32, dtype=torch.uint8, device="cuda")
    Pk[pshift:pshift + total] = torch.from_numpy(exp).cuda()
    for chunk in chunks:
        D = torch.zeros(span + 32, dtype=torch.uint8, device="cuda")
        D[shift:shift + span] = torch.from_numpy(pre).cuda()
        dbase = D.data_ptr() + shift - tl
        off = 0
        while off < total:
            ln = total - off if chunk is None else min(chunk, total - off)
            dt.unpack(count, dbase, Pk.data_ptr() + pshift + off, offset=off, length=ln, stream=st)
            off += ln
        torch.cuda.synchronize()
        assert expect_unpack is None or dt.last_path == expect_unpack
        got = D.cpu().numpy()
        np.testing.assert_array_equal(got[shift:shift + span], exp_u, err_msg=f"unpack chunk {chunk}")
        assert not got[:shift].any() and not got[shift + span:].any(), "unpack wrote outside the span"


class _Big:
    """A synthetic committed description (ELEM records) with its true bounds."""

    def __init__(self, elems, size, lb, ub):
        import test_convertor_pins as P
        dd = P.Desc(elems, size, lb, ub)
        self.desc = np.frombuffer(dd.bytes, np.uint8).copy()
        self.nrec, self.size, self.lb, self.ub = dd.nrec, size, lb, ub
        self.true_lb = min(disp + min(0, (cnt - 1) * ext) for t, cnt, blen, ext, disp in elems)
        self.true_ub = max(disp + max(0, (cnt - 1) * ext) + blen * _ES[t] for t, cnt, blen, ext, disp in elems)

    def dt(self):
        return mxompi.Datatype(self.desc.tobytes(), self.nrec, self.size, self.lb, self.ub)


_ES = {4: 1, 6: 4, 15: 4, 16: 8}     # OPAL INT1, INT4, FLOAT4, FLOAT8


def _random_indexed(nb, seed, t=15, max_bl=64, max_gap=16, shuffle=False):
    """indexed_f32_random's recipe (oracle/gen_ddt_golden.c) at nb blocks:
    1..max_bl-element blocks, 0..max_gap-element gaps; `shuffle` permutes the
    blocks' order in the stream (a non-monotonic layout)."""
    es = _ES[t]
    rng = np.random.default_rng(seed)
    bl = rng.integers(1, max_bl + 1, nb)
    gaps = rng.integers(0, max_gap + 1, nb)
    dp = np.cumsum(gaps) + np.concatenate(([0], np.cumsum(bl)[:-1]))
    order = rng.permutation(nb) if shuffle else np.arange(nb)
    elems = [(t, 1, int(bl[i]), int(bl[i]) * es, int(dp[i]) * es) for i in order]
    lo = int(dp.min()) * es
    hi = int((dp + bl).max()) * es
    return _Big(elems, int(bl.sum()) * es, lo, hi)


def _upper_triangle(n):
    """upper triangle of an n x n double matrix (row i: n - i elements from (i, i))."""
    elems = [(16, 1, n - i, (n - i) * 8, (i * n + i) * 8) for i in range(n)]
    return _Big(elems, n * (n + 1) // 2 * 8, 0, n * n * 8)


@pytest.mark.gpu
@pytest.mark.parametrize("shift,pshift", [(0, 0), (3, 0), (8, 5), (1, 16)])
def test_block_kernels_indexed_1e5_random_blocks(shift, pshift):
    """An indexed type of 10^5 random blocks (a 13 MB instance: no byte map)
    takes the BLOCK kernels by default; bit-exact vs the oracle, whole and in
    odd fragments that cut blocks and granules, misaligned user and packed."""
    mxompi.init(0)
    d = _random_indexed(100000, 7)
    dt = d.dt()
    _check_device_vs_oracle(d, dt, 3, shift, pshift, chunks=(None, 1000003, 4099))
    dt.close()


@pytest.mark.gpu
def test_block_kernels_upper_triangle_500():
    """The 500 x 500 upper triangle (1 MB instances), 4 instances, fragments."""
    mxompi.init(0)
    d = _upper_triangle(500)
    dt = d.dt()
    _check_device_vs_oracle(d, dt, 4, 4, 0, chunks=(None, 65537))
    dt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("shuffle", [False, True])
def test_block_kernels_byte_blocks(shuffle):
    """1..3-byte blocks with 0..2-byte gaps (many parts per granule: the PACK
    kernel's multi-round part loop), in stream order and shuffled."""
    mxompi.init(0)
    d = _random_indexed(120000, 9, t=4, max_bl=3, max_gap=2, shuffle=shuffle)
    dt = d.dt()
    _check_device_vs_oracle(d, dt, 2, 5, 3, chunks=(None, 7777))
    dt.close()


# ---- periodic small-block PACK (k_pack_vec_span) ------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("t,blen,stride", [(15, 1, 8), (16, 1, 16), (15, 1, 16), (15, 2, 16)])
@pytest.mark.parametrize("layout", ["resized", "plain1", "plain3"])
@pytest.mark.parametrize("shift,pshift", [(0, 0), (0, 5), (3, 0), (16, 8)])
def test_vec_span_pack(t, blen, stride, layout, shift, pshift):
    """A vector of blen-element blocks every `stride` bytes: resized so
    instances continue the period (the span kernel over every instance), a
    plain MPI vector packed as one instance, and three plain instances (the
    span kernel only for fragments inside instance 0).  Aligned user buffers
    take the span kernel; shifted user / odd packed buffers the run-walking
    VEC kernel -- both bit-exact vs the oracle, whole and in odd fragments."""
    mxompi.init(0)
    es = _ES[t]
    cnt = 100003
    ub = cnt * stride if layout == "resized" else (cnt - 1) * stride + blen * es
    d = _Big([(t, cnt, blen, stride, 0)], cnt * blen * es, 0, ub)
    dt = d.dt()
    count = 1 if layout == "plain1" else 3
    span_ok = shift % 16 == 0 and pshift % 4 == 0 and layout != "plain3"
    _check_device_vs_oracle(d, dt, count, shift, pshift, chunks=(None, 4099, 65536, 1000003),
                            expect_path="vector" if span_ok else None, expect_unpack=None)
    dt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("rec", RECS, ids=lambda r: r["name"])
def test_block_kernels_forced_on_golden_types(rec):
    """MX_DDT_PATH_BLOCK on every golden type (small instances, many per tile):
    the reference's own packed streams and unpack results, whole and in odd
    fragments."""
    mxompi.init(0)
    dt = _dt(rec)
    dt.set_path("block")
    total = rec["size"] * rec["count"]
    contiguous = rec["size"] == rec["ub"] - rec["lb"] and dt.runs == 1
    want = "copy" if contiguous else "block"
    U = torch.from_numpy(rec["user"].copy()).cuda()
    s = torch.cuda.current_stream().cuda_stream
    base = U.data_ptr() - rec["true_lb"]
    for chunk in (None, 11, 956):
        P = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
        off = 0
        while off < total:
            ln = total - off if chunk is None else min(chunk, total - off)
            dt.pack(rec["count"], base, P.data_ptr() + off, offset=off, length=ln, stream=s)
            off += ln
        torch.cuda.synchronize()
        assert dt.last_path == want
        np.testing.assert_array_equal(P.cpu().numpy()[:total], rec["packed"], err_msg=f"{rec['name']} {chunk}")
    for chunk in (None, 13, 1000):
        D = torch.from_numpy(rec["prefill"].copy()).cuda()
        Pk = torch.from_numpy(rec["packed"].copy()).cuda()
        dbase = D.data_ptr() - rec["true_lb"]
        off = 0
        while off < total:
            ln = total - off if chunk is None else min(chunk, total - off)
            dt.unpack(rec["count"], dbase, Pk.data_ptr() + off, offset=off, length=ln, stream=s)
            off += ln
        torch.cuda.synchronize()
        assert dt.last_path == want
        np.testing.assert_array_equal(D.cpu().numpy(), rec["unpacked"], err_msg=f"{rec['name']} unpack {chunk}")
    dt.close()
