"""The opal_convertor hook for device user buffers (mca/convertor_mi355x.c;
VERDICT r4 missing 4), driven the way Open MPI's datatype engine drives it.

The mini-host restates what opal_convertor_prepare_for_send / _for_recv
leave in the convertor (OPAL_CONVERTOR_PREPARE, opal_convertor.c:520-560),
calls mca_convertor_mi355x_prepare (the one call a maintainer adds after the
loop choice), then loops fAdvance like opal_convertor_pack
/ _unpack (opal_convertor.c:218-330) with fragments of a fixed size, as a
fragmenting BTL does -- from the start of the message or from a position set
in the middle of it (opal_convertor_set_position).  Every call's contract is
checked by the harness (max_data = the iovec lengths, bConverted advanced by
them, 1 exactly at the end, nothing more once complete).

Bytes are pinned by the reference test suite's own types and the fixtures
made from the oracle's restated convertor walk (tests/golden/ddt_vectors.bin,
oracle/mx_oracle_ddt.c of opal_datatype_pack.c:235-370 /
opal_datatype_unpack.c:245-427); larger counts against the oracle itself.
Packed fragments in device memory and in host memory (staged).
"""
import ctypes

import numpy as np
import pytest

import golden_io
import minihost
import mxompi
import oracle_lib

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

vp, sz, ci, i64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int64
TYPES = ["struct_char_d3_int_resized48", "indexed_f32_random", "vector_f32_b4_s8", "ref_blacs_indexed",
         "ref_struct", "ref_strange", "ref_upper_matrix_60", "ref_matrix_borders_20_3", "vector_f64_b3_s5"]


def _host():
    H = minihost.host(with_components=True)
    H.mxh_convertor_run.argtypes = [vp, sz, sz, i64, i64, i64, i64, sz, vp, vp, sz, sz, ci, ci,
                                    ctypes.POINTER(ci)]
    return H


def _rec(name):
    _, recs = golden_io.ddt_records()
    return next(r for r in recs if r["name"] == name)


def _oracle_pack(rec, count, user, unpack=False, packed=None):
    basic, _ = golden_io.ddt_records()
    B = np.ascontiguousarray(basic)
    O = oracle_lib.oracle()
    O.mxo_ddt_convert.argtypes = [vp, sz, vp, i64, i64, sz, vp, vp, ci]
    if packed is None:
        packed = np.zeros(count * rec["size"], np.uint8)
    assert O.mxo_ddt_convert(rec["desc"].ctypes.data, rec["nrec"], B.ctypes.data, rec["lb"], rec["ub"], count,
                             user.ctypes.data - rec["true_lb"], packed.ctypes.data,
                             1 if unpack else 0) == count * rec["size"]          # bytes converted
    return packed


def _run(H, rec, count, ubase, packed_ptr, start, frag, niov, recv):
    calls = ci(0)
    rc = H.mxh_convertor_run(rec["desc"].ctypes.data, rec["nrec"], rec["size"], rec["lb"], rec["ub"],
                             rec["true_lb"], rec["true_ub"], count, ubase, packed_ptr, start, frag, niov,
                             1 if recv else 0, ctypes.byref(calls))
    assert rc == 0, rc
    return calls.value


@pytest.mark.parametrize("name", TYPES)
def test_hook_pack_unpack_golden(name):
    """The fixture's own count, one-fragment and 113-byte fragments."""
    H = _host()
    rec = _rec(name)
    count, nb = rec["count"], rec["count"] * rec["size"]
    U = torch.from_numpy(rec["user"].copy()).cuda()
    ubase = U.data_ptr() - rec["true_lb"]
    for frag, niov in ((nb, 1), (113, 1), (113, 3)):
        P = torch.zeros(nb, dtype=torch.uint8, device="cuda")
        _run(H, rec, count, ubase, P.data_ptr(), 0, frag, niov, False)
        assert np.array_equal(P.cpu().numpy(), rec["packed"]), (name, frag, niov)
        # unpack into the fixture's pre-filled buffer: gaps keep their bytes
        R = torch.from_numpy(rec["prefill"].copy()).cuda()
        Pk = torch.from_numpy(rec["packed"].copy()).cuda()
        _run(H, rec, count, R.data_ptr() - rec["true_lb"], Pk.data_ptr(), 0, frag, niov, True)
        assert np.array_equal(R.cpu().numpy(), rec["unpacked"]), (name, frag, niov)


@pytest.mark.parametrize("name", ["struct_char_d3_int_resized48", "indexed_f32_random", "ref_blacs_indexed"])
@pytest.mark.parametrize("where", ["device", "host"])
def test_hook_large_fragmented_from_a_position(name, where):
    """~8 MiB packed, 64 KiB + 7 fragments, started at a position in the
    middle of an element (set_position); packed fragments in device or host
    memory.  Against the oracle's walk."""
    H = _host()
    rec = _rec(name)
    count = (8 << 20) // rec["size"] + 3
    nb = count * rec["size"]
    ext = rec["ub"] - rec["lb"]
    span = ext * (count - 1) + rec["true_ub"] - rec["true_lb"]
    rng = np.random.default_rng(5)
    user = rng.integers(0, 256, span, dtype=np.uint8)
    exp = _oracle_pack(rec, count, user)
    start = nb // 3 + 5
    U = torch.from_numpy(user).cuda()
    ubase = U.data_ptr() - rec["true_lb"]
    frag = (64 << 10) + 7
    if where == "device":
        P = torch.zeros(nb - start, dtype=torch.uint8, device="cuda")
        pptr = P.data_ptr()
    else:
        Ph = np.zeros(nb - start, np.uint8)
        pptr = Ph.ctypes.data
    calls = _run(H, rec, count, ubase, pptr, start, frag, 2, False)
    assert calls == -(-(nb - start) // (2 * frag))
    got = P.cpu().numpy() if where == "device" else Ph
    assert np.array_equal(got, exp[start:]), name
    # unpack the same stream tail into a pre-filled buffer: only the bytes of
    # elements from `start` on change, gap bytes never
    pre = rng.integers(0, 256, span, dtype=np.uint8)
    want = pre.copy()
    full = exp.copy()
    tmp = _oracle_pack(rec, count, pre)          # the prefill's own stream
    full[:start] = tmp[:start]                   # bytes before `start` rewritten with themselves
    _oracle_pack(rec, count, want, unpack=True, packed=full)
    R = torch.from_numpy(pre.copy()).cuda()
    if where == "device":
        Pk = torch.from_numpy(exp[start:].copy()).cuda()
        kptr = Pk.data_ptr()
    else:
        Pkh = exp[start:].copy()
        kptr = Pkh.ctypes.data
    _run(H, rec, count, R.data_ptr() - rec["true_lb"], kptr, start, frag, 2, True)
    assert np.array_equal(R.cpu().numpy(), want), name


def test_hook_declines_host_user_buffers():
    """A host user buffer keeps the reference's loop (the hook returns 0)."""
    H = _host()
    rec = _rec("struct_char_d3_int_resized48")
    user = rec["user"].copy()
    packed = np.zeros(rec["count"] * rec["size"], np.uint8)
    calls = ci(0)
    rc = H.mxh_convertor_run(rec["desc"].ctypes.data, rec["nrec"], rec["size"], rec["lb"], rec["ub"],
                             rec["true_lb"], rec["true_ub"], rec["count"], user.ctypes.data - rec["true_lb"],
                             packed.ctypes.data, 0, 4096, 1, 0, ctypes.byref(calls))
    assert rc == -10


def test_hook_recreated_datatype_at_the_same_address():
    """A datatype freed and re-created with another stride often comes back
    at the same addresses with the same record count: the hook's
    handle cache keys on the records' contents too, so each layout packs its
    own bytes.  The harness's datatype lives at one stack address; the records
    are rewritten in place between calls."""
    H = _host()
    recs = np.zeros(2, dtype=[("flags", "<u2"), ("type", "<u2"), ("count", "<u4"), ("blocklen", "<u8"),
                              ("extent", "<i8"), ("disp", "<i8")])
    count, ext, size = 4099, 32, 16          # 4 blocks of 4 bytes in a 32-byte extent
    rng = np.random.default_rng(9)
    user = rng.integers(0, 256, count * ext, dtype=np.uint8)
    U = torch.from_numpy(user).cuda()
    for stride in (8, 6, 8, 4):
        recs[0] = (0x0100, 9, 4, 4, stride, 0)   # DATA | OPAL_UINT1, 4 blocks of 4 bytes every `stride`
        recs[1] = (0, 1, 1, 0, size, 0)          # END_LOOP
        P = torch.zeros(count * size, dtype=torch.uint8, device="cuda")
        calls = ci(0)
        rc = H.mxh_convertor_run(recs.ctypes.data, 2, size, 0, ext, 0, 3 * stride + 4, count, U.data_ptr(),
                                 P.data_ptr(), 0, count * size, 1, 0, ctypes.byref(calls))
        assert rc == 0, rc
        idx = (np.arange(count)[:, None, None] * ext + np.arange(4)[None, :, None] * stride
               + np.arange(4)[None, None, :]).ravel()
        assert np.array_equal(P.cpu().numpy(), user[idx]), f"stride {stride}"
