"""Readers for the committed golden fixtures in tests/golden/.

op_vectors.bin is produced by oracle/gen_op_golden.c from the reference's
own op_base_functions.c (see that file for the record layout).
"""
import os
import struct

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def op_records(path=None):
    path = path or os.path.join(GOLDEN, "op_vectors.bin")
    with open(path, "rb") as f:
        data = f.read()
    assert data[:8] == b"MXGOLD01", "bad golden magic"
    (nrec,) = struct.unpack_from("<I", data, 8)
    off = 12
    recs = []
    for _ in range(nrec):
        kind, op, t, es, n = struct.unpack_from("<5I", data, off)
        off += 20
        nb = es * n
        a = np.frombuffer(data, np.uint8, nb, off); off += nb
        b = np.frombuffer(data, np.uint8, nb, off); off += nb
        o = np.frombuffer(data, np.uint8, nb, off); off += nb
        recs.append(dict(kind=kind, op=op, type=t, es=es, n=n, a=a, b=b, out=o))
    return recs


# Floating-point slots and their component layout: (component dtype, bytes
# per component, components per element).  x87 long double = 16-byte
# components whose first 10 bytes carry the value.
_F4 = {15, 17, 19}            # FLOAT, REAL, REAL4
_F8 = {16, 20, 22}            # DOUBLE, REAL8, DOUBLE_PRECISION
_LD = {23}                    # LONG_DOUBLE
_CF4, _CF8, _CLD = 27, 28, 29  # complex float/double/long double
SUM, PROD = 3, 4


def _components(buf, t):
    """View a byte buffer of slot t as (values-as-bytes, isnan mask) per FP
    component, or None for non floating-point slots."""
    if t in _F4 or t == _CF4:
        v = buf.view(np.uint32)
        return v, np.isnan(buf.view(np.float32))
    if t in _F8 or t == _CF8:
        v = buf.view(np.uint64)
        return v, np.isnan(buf.view(np.float64))
    if t in _LD or t == _CLD:
        c = buf.reshape(-1, 16)
        m = c[:, 0:8].copy().view(np.uint64).ravel()
        se = c[:, 8:10].copy().view(np.uint16).ravel()
        nan = ((se & 0x7FFF) == 0x7FFF) & ((m << np.uint64(1)) != 0)
        key = np.concatenate([c[:, :10]], axis=1)   # value bytes only
        return key, nan
    return None


# Bytes of an element that carry MPI data, for types whose storage has
# other bytes: struct gaps of the pair datatypes (size < extent -- the
# convertor never moves them) and the 6 pad bytes of an x87 long double.
# Collective results are compared on these bytes only.
_DATA_BYTES = {
    38: (8, [0, 1, 4, 5, 6, 7]),                       # SHORT_INT
    35: (16, list(range(12))),                          # DOUBLE_INT
    36: (16, list(range(12))),                          # LONG_INT
    39: (32, list(range(10)) + [16, 17, 18, 19]),       # LONG_DOUBLE_INT
    23: (16, list(range(10))),                          # LONG_DOUBLE
    29: (32, list(range(10)) + list(range(16, 26))),    # C_LONG_DOUBLE_COMPLEX
}


def data_bytes(buf, t):
    """Drop the non-data bytes of slot-t elements (no-op for other types)."""
    buf = np.ascontiguousarray(buf).view(np.uint8).ravel()
    if t not in _DATA_BYTES:
        return buf
    es, keep = _DATA_BYTES[t]
    return buf.reshape(-1, es)[:, keep].ravel()


def assert_coll_equal(out, expected, op, t, what=""):
    """assert_op_equal on the data bytes only (collective results)."""
    if t in _DATA_BYTES and not (op in (SUM, PROD) and t in (23, 29)):
        out, expected = data_bytes(out, t), data_bytes(expected, t)
    assert_op_equal(out, expected, op, t, what)


def assert_op_equal(out, expected, op, t, what=""):
    """Bit-exact comparison, except that for floating-point SUM/PROD a NaN
    result only has to be a NaN: which NaN payload/sign survives a
    NaN (op) NaN depends on the host compiler's operand order (SSE/x87
    return one of the operands), not on the MPI_Op semantics.  MAX/MIN and
    MAXLOC/MINLOC select an operand, so they stay bit-exact incl. NaNs."""
    out = np.ascontiguousarray(out).view(np.uint8).ravel()
    expected = np.ascontiguousarray(expected).view(np.uint8).ravel()
    comp = _components(out, t) if op in (SUM, PROD) else None
    if comp is None:
        np.testing.assert_array_equal(out, expected, err_msg=what)
        return
    vo, no = comp
    ve, ne = _components(expected, t)
    np.testing.assert_array_equal(no, ne, err_msg=f"{what}: NaN positions differ")
    keep = ~no
    np.testing.assert_array_equal(vo[keep], ve[keep], err_msg=what)


def ddt_records(path=None):
    """tests/golden/ddt_vectors.bin (oracle/gen_ddt_golden.c layout)."""
    path = path or os.path.join(GOLDEN, "ddt_vectors.bin")
    with open(path, "rb") as f:
        data = f.read()
    assert data[:8] == b"MXDDT001", "bad ddt golden magic"
    nrec, nbasic = struct.unpack_from("<II", data, 8)
    off = 16
    basic = np.frombuffer(data, np.uint64, nbasic, off).copy()
    off += 8 * nbasic
    recs = []
    for _ in range(nrec):
        name = data[off: off + 48].split(b"\0")[0].decode()
        off += 48
        count, nelem = struct.unpack_from("<II", data, off)
        off += 8
        size, lb, ub, tlb, tub, span = struct.unpack_from("<6q", data, off)
        off += 48

        def take(nb):
            nonlocal off
            a = np.frombuffer(data, np.uint8, nb, off).copy()
            off += nb
            return a
        desc = take(32 * nelem)
        user = take(span)
        packed = take(size * count)
        prefill = take(span)
        unpacked = take(span)
        recs.append(dict(name=name, count=count, nrec=nelem, size=size, lb=lb, ub=ub, true_lb=tlb,
                         true_ub=tub, span=span, desc=desc, user=user, packed=packed, prefill=prefill,
                         unpacked=unpacked))
    return basic, recs
