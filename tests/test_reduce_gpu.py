"""GPU parity: the HIP op kernels (K1-K4) vs the oracle restatement.

* every golden record (all 176 (op,type) pairs, 2- and 3-buffer;
  tests/golden/op_vectors.bin, written by oracle/gen_op_golden.c -- value
  parity with the reference is unpinned) through mx_reduce2/3;
* ragged counts and misaligned sub-buffers (the head/tail and element
  paths) vs the oracle restatement;
* full-size (1 GiB) fp32 SUM vs the oracle (CFG-B).
"""
import numpy as np
import pytest

import golden_io
import mxompi
import oracle_lib

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

RECS = golden_io.op_records()


def _dev(arr):
    a = np.ascontiguousarray(arr)
    if not a.flags.writeable:          # golden records are read-only views of the fixture file
        a = a.copy()
    return torch.from_numpy(a).to("cuda")


def _stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.fixture(scope="module", autouse=True)
def _init():
    assert torch.cuda.is_available()
    mxompi.init(0)


@pytest.mark.parametrize("rec", RECS, ids=lambda r: f"k{r['kind']}-{mxompi.OPS[r['op']]}-{mxompi.TYPES[r['type']]}")
def test_kernel_matches_reference_golden(rec):
    a = _dev(rec["a"])
    b = _dev(rec["b"])
    if rec["kind"] == 2:
        mxompi.reduce2(rec["op"], rec["type"], a.data_ptr(), b.data_ptr(), rec["n"], _stream())
        out = b
    else:
        out = torch.zeros_like(b)
        mxompi.reduce3(rec["op"], rec["type"], a.data_ptr(), b.data_ptr(), out.data_ptr(), rec["n"], _stream())
    torch.cuda.synchronize()
    golden_io.assert_op_equal(out.cpu().numpy(), rec["out"], rec["op"], rec["type"],
                              f"{mxompi.OPS[rec['op']]} {mxompi.TYPES[rec['type']]}")


CASES = [("SUM", "FLOAT"), ("MAX", "DOUBLE"), ("BXOR", "UINT8_T"), ("PROD", "INT16_T"),
         ("MINLOC", "SHORT_INT"), ("SUM", "C_FLOAT_COMPLEX"), ("LXOR", "BOOL"),
         ("SUM", "LONG_DOUBLE"), ("MAXLOC", "DOUBLE_INT"), ("BAND", "BYTE")]


@pytest.mark.parametrize("op,t", CASES)
@pytest.mark.parametrize("offs", [(0, 0, 0), (1, 1, 1), (3, 3, 3), (0, 1, 2), (5, 0, 7)])
@pytest.mark.parametrize("n", [1, 7, 64, 1000, 4099])
def test_ragged_and_misaligned(op, t, offs, n):
    O = oracle_lib.oracle()
    es = mxompi.type_size(t)
    rng = np.random.default_rng(n * 131 + offs[0] + 7 * offs[1])
    nb = es * n
    if t == "BOOL":
        raw = [rng.integers(0, 2, nb + 8 * es + 64, dtype=np.uint8) for _ in range(3)]
    else:
        raw = [rng.integers(0, 256, nb + 8 * es + 64, dtype=np.uint8) for _ in range(3)]
    if "LONG_DOUBLE" in t:  # keep only finite-ish x87 encodings: random doubles widened
        for r in raw:
            v = r[: len(r) // 16 * 16].reshape(-1, 16)
            d = rng.uniform(-4, 4, len(v)).astype(np.longdouble)
            v[:] = d.view(np.uint8).reshape(-1, 16)
    A = _dev(raw[0]); B = _dev(raw[1])
    ea = es * offs[0]; eb = es * offs[1]
    # 2-buffer with element offsets (same or different misalignment mod 16)
    mxompi.reduce2(op, t, A.data_ptr() + ea, B.data_ptr() + eb, n, _stream())
    torch.cuda.synchronize()
    exp_b = raw[1].copy()
    assert O.mxo_reduce2(mxompi.OP[op], mxompi.TYPE[t], raw[0][ea:].ctypes.data,
                         exp_b[eb:].ctypes.data, n, 1) == 0
    golden_io.assert_op_equal(B.cpu().numpy()[eb:eb + nb], exp_b[eb:eb + nb], mxompi.OP[op],
                              mxompi.TYPE[t], f"{op} {t} offs={offs} n={n}")
    # untouched bytes around the destination
    np.testing.assert_array_equal(B.cpu().numpy()[:eb], raw[1][:eb])
    np.testing.assert_array_equal(B.cpu().numpy()[eb + nb:], raw[1][eb + nb:])


@pytest.mark.parametrize("op,t", CASES)
@pytest.mark.parametrize("offs", [(0, 0, 0), (2, 2, 2), (1, 2, 3)])
def test_three_buffer_misaligned(op, t, offs):
    O = oracle_lib.oracle()
    n = 3001
    es = mxompi.type_size(t)
    rng = np.random.default_rng(99 + offs[2])
    raw = [rng.integers(0, 2 if t == "BOOL" else 256, es * n + 8 * es + 64, dtype=np.uint8) for _ in range(2)]
    if "LONG_DOUBLE" in t:
        for r in raw:
            v = r[: len(r) // 16 * 16].reshape(-1, 16)
            v[:] = rng.uniform(-4, 4, len(v)).astype(np.longdouble).view(np.uint8).reshape(-1, 16)
    A = _dev(raw[0]); B = _dev(raw[1])
    out = torch.zeros(es * n + 8 * es + 64, dtype=torch.uint8, device="cuda")
    e1, e2, eo = (es * o for o in offs)
    mxompi.reduce3(op, t, A.data_ptr() + e1, B.data_ptr() + e2, out.data_ptr() + eo, n, _stream())
    torch.cuda.synchronize()
    exp = np.zeros(es * n, np.uint8)
    assert O.mxo_reduce3(mxompi.OP[op], mxompi.TYPE[t], raw[0][e1:].ctypes.data,
                         raw[1][e2:].ctypes.data, exp.ctypes.data, n, 1) == 0
    golden_io.assert_op_equal(out.cpu().numpy()[eo:eo + es * n], exp, mxompi.OP[op], mxompi.TYPE[t])


def test_full_size_fp32_sum_1gib():
    """CFG-B at its full size: 2^28 fp32 elements (1 GiB per buffer)."""
    O = oracle_lib.oracle()
    n = 1 << 28
    rng = np.random.default_rng(0x5EEDC0DE)
    a = rng.uniform(-1, 1, n).astype(np.float32)
    b = rng.uniform(-1, 1, n).astype(np.float32)
    A = _dev(a); B = _dev(b)
    mxompi.reduce2("SUM", "FLOAT", A.data_ptr(), B.data_ptr(), n, _stream())
    torch.cuda.synchronize()
    got = B.cpu().numpy()
    assert O.mxo_reduce2(3, 15, a.ctypes.data, b.ctypes.data, n, 1) == 0
    np.testing.assert_array_equal(got.view(np.uint32), b.view(np.uint32))


# CFG-B at full size beyond fp32 SUM: one pair per kernel family x element
# size (arithmetic, MAX/MIN, bitwise, logical, complex, x87 soft-float, every
# LOC pair layout), 1 GiB per buffer (the non-temporal 128-lane instance),
# checked against the restatement element for element.  Inputs: full-range
# bytes for integer and bitwise ops, a small value range for MAX/MIN and the
# LOC ops (ties), [0.5, 2) for FP PROD.
_FULL = [("BAND", "UINT16_T"), ("PROD", "INT64_T"), ("MAX", "DOUBLE"), ("MAXLOC", "FLOAT_INT"),
         ("MINLOC", "DOUBLE_INT"), ("PROD", "C_FLOAT_COMPLEX"), ("LXOR", "INT8_T"), ("SUM", "LONG_DOUBLE"),
         # round 3: the rest of (family x element size)
         ("SUM", "INT8_T"), ("SUM", "INT16_T"), ("MIN", "INT32_T"), ("SUM", "UINT64_T"), ("MIN", "FLOAT"),
         ("PROD", "DOUBLE"), ("MAX", "UINT8_T"), ("SUM", "C_DOUBLE_COMPLEX"), ("PROD", "C_LONG_DOUBLE_COMPLEX"),
         ("MAX", "LONG_DOUBLE"), ("BOR", "INT32_T"), ("BXOR", "UINT64_T"), ("BAND", "INT8_T"), ("LAND", "INT16_T"),
         ("LOR", "UINT32_T"), ("MAXLOC", "2INT"), ("MINLOC", "SHORT_INT"), ("MAXLOC", "LONG_INT"),
         ("MINLOC", "LONG_DOUBLE_INT"), ("PROD", "FLOAT")]

# LOC pair layouts (value dtype, value offset, index offset) -- op.h pair structs, x86-64
_LOC = {"FLOAT_INT": ("<f4", 0, 4), "DOUBLE_INT": ("<f8", 0, 8), "LONG_INT": ("<i8", 0, 8), "2INT": ("<i4", 0, 4),
        "SHORT_INT": ("<i2", 0, 4), "LONG_DOUBLE_INT": (np.longdouble, 0, 16)}
_FP = {"FLOAT": np.float32, "DOUBLE": np.float64, "SHORT_FLOAT": np.float16, "C_FLOAT_COMPLEX": np.float32,
       "C_DOUBLE_COMPLEX": np.float64}


def _full_input(op, t, n, es, rng):
    # padding bytes stay random (raw generator words: 3x faster than integers() at 1 GiB)
    raw = [rng.bit_generator.random_raw((n * es + 7) // 8).view(np.uint8)[:n * es] for _ in range(2)]
    for r in raw:
        rows = r.reshape(n, es)
        if t in _LOC:
            vt, vo, io = _LOC[t]
            vs = np.dtype(vt).itemsize
            vals = rng.integers(0, 16, n).astype(vt)                    # ties
            vb = vals.view(np.uint8).reshape(n, -1)[:, :min(vs, 10 if vt is np.longdouble else vs)]
            rows[:, vo:vo + vb.shape[1]] = vb
            rows[:, io:io + 4] = rng.integers(-1000, 1000, n).astype("<i4").view(np.uint8).reshape(n, 4)
        elif t in ("LONG_DOUBLE", "C_LONG_DOUBLE_COMPLEX"):
            k = es // 16
            lo, hi = (0.5, 2.0) if op == "PROD" else (-4.0, 4.0)
            v = rng.uniform(lo, hi, n * k).astype(np.longdouble).view(np.uint8).reshape(n * k, 16)[:, :10]
            rows.reshape(n * k, 16)[:, :10] = v
        elif t in _FP:
            ft = _FP[t]
            k = es // np.dtype(ft).itemsize
            lo, hi = (0.5, 2.0) if op == "PROD" else ((0, 16) if op in ("MAX", "MIN") else (-1e3, 1e3))
            v = rng.uniform(lo, hi, n * k).astype(ft)
            if op in ("MAX", "MIN"):
                v = np.floor(v).astype(ft)
            rows[:] = v.view(np.uint8).reshape(n, es)
    return raw


# a period of the 1 GiB operands: prime, so a kernel that mixes up element
# indices (a wrong grid stride, a 32-bit offset overflow past 2^31 bytes, a
# vector tail) pairs operands the period did not pair
_PERIOD = 1_000_003


@pytest.mark.parametrize("op,t", _FULL, ids=[f"{o}-{t}" for o, t in _FULL])
def test_full_size_1gib_pairs(op, t):
    """One kernel launch over 1 GiB operands, every output element checked
    bit for bit.  The operands repeat a period of _PERIOD random elements
    (generated and reduced by the oracle once, then tiled on the device), so
    the expected 1 GiB is the oracle's period result tiled the same way --
    the whole check runs in a fraction of a second instead of generating and
    reducing 2 GiB on the host."""
    O = oracle_lib.oracle()
    es = mxompi.type_size(t)
    n = (1 << 30) // es
    rng = np.random.default_rng(0x5EEDC0DE + mxompi.TYPE[t])
    raw = _full_input(op, t, _PERIOD, es, rng)
    exp_p = raw[1].copy()
    assert O.mxo_reduce2(mxompi.OP[op], mxompi.TYPE[t], raw[0].ctypes.data, exp_p.ctypes.data, _PERIOD, 1) == 0
    reps = -(-n // _PERIOD)

    def tile(a):
        return _dev(a).repeat(reps)[: n * es].contiguous()
    A, B = tile(raw[0]), tile(raw[1])
    mxompi.reduce2(op, t, A.data_ptr(), B.data_ptr(), n, _stream())
    del A
    E = tile(exp_p)
    torch.cuda.synchronize()
    if not torch.equal(B, E):   # the first differing element, in the oracle's terms
        bad = int(torch.nonzero(B != E)[0, 0]) // es
        golden_io.assert_op_equal(B[bad * es:(bad + 1) * es].cpu().numpy(),
                                  E[bad * es:(bad + 1) * es].cpu().numpy(), mxompi.OP[op], mxompi.TYPE[t],
                                  f"element {bad} of {n}")
    del B, E
    torch.cuda.empty_cache()


@pytest.mark.parametrize("shift", [0, 1, 3])
def test_streaming_instance_ragged(shift):
    """The non-temporal, XCD-mapped K1 instance (>= 384 MiB footprint) on a
    count that leaves a partial grid tail and, shifted, a ragged head."""
    O = oracle_lib.oracle()
    n = 34_000_001
    rng = np.random.default_rng(11 + shift)
    a = rng.uniform(-1, 1, n + shift).astype(np.float32)
    b = rng.uniform(-1, 1, n + shift).astype(np.float32)
    A = _dev(a); B = _dev(b)
    mxompi.reduce2("SUM", "FLOAT", A.data_ptr() + 4 * shift, B.data_ptr() + 4 * shift, n, _stream())
    torch.cuda.synchronize()
    got = B.cpu().numpy()
    exp = b.copy()
    assert O.mxo_reduce2(3, 15, a[shift:].ctypes.data, exp[shift:].ctypes.data, n, 1) == 0
    np.testing.assert_array_equal(got.view(np.uint32), exp.view(np.uint32))


def test_count_zero_is_noop():
    B = torch.ones(16, device="cuda")
    mxompi.reduce2("SUM", "FLOAT", B.data_ptr(), B.data_ptr(), 0, _stream())
    torch.cuda.synchronize()
    assert float(B.sum()) == 16.0


# ---- mx_reduce2_sync: the kernel's own completion mark ---------------------
@pytest.mark.parametrize("op,t", CASES + [("PROD", "C_LONG_DOUBLE_COMPLEX"), ("MAXLOC", "LONG_DOUBLE_INT")])
@pytest.mark.parametrize("offs", [(0, 0), (1, 1), (0, 1)])
@pytest.mark.parametrize("n", [1, 1000, 16384, 16385, 300001])
def test_reduce2_sync_complete_on_return(op, t, offs, n):
    """mx_reduce2_sync on a side stream returns with the result complete:
    read back on the default stream with no synchronisation against the side
    stream, bit-exact vs the oracle.  Vector, per-element and 32-byte kernels
    (aligned / same / different misalignment), launches under and over the
    fused-mark cap (2^14 elements and 256 KiB: over it a marker kernel
    follows)."""
    O = oracle_lib.oracle()
    es = mxompi.type_size(t)
    rng = np.random.default_rng(n + 17 * offs[1])
    nb = es * n
    raw = [rng.integers(0, 2 if t == "BOOL" else 256, nb + 8 * es + 64, dtype=np.uint8) for _ in range(2)]
    if "LONG_DOUBLE" in t:
        for r in raw:
            v = r[: len(r) // 16 * 16].reshape(-1, 16)
            v[:] = rng.uniform(-4, 4, len(v)).astype(np.longdouble).view(np.uint8).reshape(-1, 16)
    A = _dev(raw[0]); B = _dev(raw[1])
    torch.cuda.synchronize()
    ea, eb = es * offs[0], es * offs[1]
    side = torch.cuda.Stream()
    mxompi.reduce2_sync(op, t, A.data_ptr() + ea, B.data_ptr() + eb, n, side.cuda_stream)
    got = B.cpu().numpy()                    # default stream: not ordered after `side`
    exp_b = raw[1].copy()
    assert O.mxo_reduce2(mxompi.OP[op], mxompi.TYPE[t], raw[0][ea:].ctypes.data,
                         exp_b[eb:].ctypes.data, n, 1) == 0
    golden_io.assert_op_equal(got[eb:eb + nb], exp_b[eb:eb + nb], mxompi.OP[op], mxompi.TYPE[t],
                              f"{op} {t} offs={offs} n={n}")
    np.testing.assert_array_equal(got[:eb], raw[1][:eb])
    np.testing.assert_array_equal(got[eb + nb:], raw[1][eb + nb:])


@pytest.mark.parametrize("n", [4099, 262144])
def test_reduce2_sync_chain_across_streams(n):
    """300 dependent calls alternating between two streams with no event
    between them: each call must see the previous one's result, so every
    return must mean complete and visible (the mark's counter is reused by
    every call of the thread)."""
    a = torch.ones(n, dtype=torch.int32, device="cuda")
    b = torch.zeros(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for i in range(300):
        mxompi.reduce2_sync("SUM", "INT32_T", a.data_ptr(), b.data_ptr(), n, (s1 if i % 2 else s2).cuda_stream)
    assert torch.equal(b.cpu(), torch.full((n,), 300, dtype=torch.int32))


# value bytes of the padded element types (the rest is padding the 3-buffer
# form must leave as the destination held it: LOC_FUNC_3BUF assigns members)
_VALUE_BYTES = {"SHORT_INT": [(0, 2), (4, 8)], "DOUBLE_INT": [(0, 12)], "LONG_DOUBLE": [(0, 10)],
                "LONG_DOUBLE_INT": [(0, 10), (16, 20)], "C_LONG_DOUBLE_COMPLEX": [(0, 10), (16, 26)]}


@pytest.mark.parametrize("op,t", [("MINLOC", "SHORT_INT"), ("MAXLOC", "DOUBLE_INT"), ("SUM", "LONG_DOUBLE"),
                                  ("MAXLOC", "LONG_DOUBLE_INT"), ("PROD", "C_LONG_DOUBLE_COMPLEX")])
@pytest.mark.parametrize("n,eo", [(100003, 0), (4099, 1), (2, 0)])
def test_three_buffer_keeps_destination_padding(op, t, n, eo):
    """The 3-buffer kernels of padded types merge the results' value fields
    into the destination's own bytes (whole-line writes): values bit-exact
    vs the oracle, every padding byte of `out` as it was."""
    O = oracle_lib.oracle()
    es = mxompi.type_size(t)
    rng = np.random.default_rng(n + es)
    raw = [rng.integers(0, 256, es * (n + eo) + 64, dtype=np.uint8) for _ in range(3)]
    if "LONG_DOUBLE" in t:
        for r in raw[:2]:
            v = r[: len(r) // 16 * 16].reshape(-1, 16)
            v[:] = rng.uniform(-4, 4, len(v)).astype(np.longdouble).view(np.uint8).reshape(-1, 16)
    A = _dev(raw[0]); B = _dev(raw[1]); OUT = _dev(raw[2])
    e = es * eo
    mxompi.reduce3(op, t, A.data_ptr() + e, B.data_ptr() + e, OUT.data_ptr() + e, n, _stream())
    torch.cuda.synchronize()
    got = OUT.cpu().numpy()
    exp = raw[2].copy()
    assert O.mxo_reduce3(mxompi.OP[op], mxompi.TYPE[t], raw[0][e:].ctypes.data, raw[1][e:].ctypes.data,
                         exp[e:].ctypes.data, n, 1) == 0
    golden_io.assert_op_equal(got[e:e + es * n], exp[e:e + es * n], mxompi.OP[op], mxompi.TYPE[t], f"{op} {t} n={n}")
    pad = np.ones(es, bool)
    for lo, hi in _VALUE_BYTES[t]:
        pad[lo:hi] = False
    padmask = np.tile(pad, n)
    np.testing.assert_array_equal(got[e:e + es * n][padmask], raw[2][e:e + es * n][padmask])
    np.testing.assert_array_equal(got[:e], raw[2][:e])
    np.testing.assert_array_equal(got[e + es * n:], raw[2][e + es * n:])
