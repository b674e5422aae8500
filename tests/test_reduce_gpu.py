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
    return torch.from_numpy(np.ascontiguousarray(arr)).to("cuda")


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


# CFG-B at full size beyond fp32 SUM: one pair per kernel family / operator
# class, 1 GiB per buffer (the non-temporal instance), checked against the
# restatement element for element.  Inputs: full-range bytes for integer and
# bitwise ops, ties-heavy pairs for the LOC ops, [0.5, 2) for FP PROD.
_FULL = [("BAND", "UINT16_T"), ("PROD", "INT64_T"), ("MAX", "DOUBLE"), ("MAXLOC", "FLOAT_INT"),
         ("MINLOC", "DOUBLE_INT"), ("PROD", "C_FLOAT_COMPLEX"), ("LXOR", "INT8_T"), ("SUM", "LONG_DOUBLE")]


@pytest.mark.parametrize("op,t", _FULL, ids=[f"{o}-{t}" for o, t in _FULL])
def test_full_size_1gib_pairs(op, t):
    O = oracle_lib.oracle()
    es = mxompi.type_size(t)
    n = (1 << 30) // es
    rng = np.random.default_rng(0x5EEDC0DE + mxompi.TYPE[t])
    if t == "FLOAT_INT":
        v = np.zeros((2, n), dtype=[("v", "<f4"), ("k", "<i4")])
        v["v"] = rng.integers(0, 16, (2, n))
        v["k"] = rng.integers(-1000, 1000, (2, n))
        raw = [v[0].view(np.uint8), v[1].view(np.uint8)]
    elif t == "DOUBLE_INT":
        v = np.zeros((2, n), dtype=[("v", "<f8"), ("k", "<i4"), ("pad", "<i4")])
        v["v"] = rng.integers(0, 16, (2, n))
        v["k"] = rng.integers(-1000, 1000, (2, n))
        v["pad"] = rng.integers(-1 << 31, 1 << 31, (2, n))
        raw = [v[0].view(np.uint8), v[1].view(np.uint8)]
    elif t == "C_FLOAT_COMPLEX":
        raw = [rng.uniform(0.5, 2.0, 2 * n).astype(np.float32).view(np.uint8) for _ in range(2)]
    elif t == "DOUBLE":
        raw = [rng.uniform(-1e6, 1e6, n).view(np.uint8) for _ in range(2)]
    elif t == "LONG_DOUBLE":
        raw = []
        for _ in range(2):
            r = rng.integers(0, 256, n * 16, dtype=np.uint8)
            r.reshape(-1, 16)[:] = rng.uniform(-4, 4, n).astype(np.longdouble).view(np.uint8).reshape(-1, 16)
            raw.append(r)
    else:
        raw = [rng.integers(0, 256, n * es, dtype=np.uint8) for _ in range(2)]
    A, B = _dev(raw[0]), _dev(raw[1])
    mxompi.reduce2(op, t, A.data_ptr(), B.data_ptr(), n, _stream())
    torch.cuda.synchronize()
    got = B.cpu().numpy()
    del A, B
    torch.cuda.empty_cache()
    exp = raw[1].copy()
    assert O.mxo_reduce2(mxompi.OP[op], mxompi.TYPE[t], raw[0].ctypes.data, exp.ctypes.data, n, 1) == 0
    golden_io.assert_op_equal(got, exp, mxompi.OP[op], mxompi.TYPE[t])


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
