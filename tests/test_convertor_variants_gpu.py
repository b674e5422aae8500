"""The PACK kernels' shapes other than each type's default
(csrc/mx_convertor.hip k_pack_bmap): every A/B switch selects
a different kernel or a different gather inside it, and each must give the
reference walk's bytes (opal_datatype_pack.c:235-370, restated by the
oracle).  One child process per switch (the switches are read once per
process); in each, the struct / indexed / BLACS / "strange" types at ~4 MiB
packed, user pointer aligned and shifted by 3 bytes, whole and as a window
starting inside an element, and the unpack of the stream into a pre-filled
buffer (gap bytes keep theirs)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1] + "/zhpe-ompi_amd"); sys.path.insert(0, sys.argv[1] + "/tests")
import ctypes, golden_io, mxompi, oracle_lib
vp, sz, ci, i64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int64
basic, recs = golden_io.ddt_records()
B = np.ascontiguousarray(basic)
O = oracle_lib.oracle()
O.mxo_ddt_convert.argtypes = [vp, sz, vp, i64, i64, sz, vp, vp, ci]
mxompi.init(0)
bad = []
for name in sys.argv[2].split(","):
    rec = next(r for r in recs if r["name"] == name)
    dt = mxompi.Datatype(rec["desc"].tobytes(), rec["nrec"], rec["size"], rec["lb"], rec["ub"])
    count = (4 << 20) // rec["size"] + 7
    nb = count * rec["size"]
    ext = rec["ub"] - rec["lb"]
    span = ext * (count - 1) + rec["true_ub"] - rec["true_lb"]
    user = np.random.default_rng(11).integers(0, 256, span, dtype=np.uint8)
    exp = np.zeros(nb, np.uint8)
    O.mxo_ddt_convert(rec["desc"].ctypes.data, rec["nrec"], B.ctypes.data, rec["lb"], rec["ub"], count,
                      user.ctypes.data - rec["true_lb"], exp.ctypes.data, 0)
    st = torch.cuda.current_stream().cuda_stream
    for shift in (0, 3):
        U = torch.zeros(span + 16, dtype=torch.uint8, device="cuda")
        U[shift:shift + span] = torch.from_numpy(user).cuda()
        base = U.data_ptr() + shift - rec["true_lb"]
        P = torch.zeros(nb, dtype=torch.uint8, device="cuda")
        dt.pack(count, base, P.data_ptr(), stream=st)
        # a window starting inside an element, its bytes at their stream
        # positions (packed - offset 16-aligned: the byte-map kernel's case)
        off, ln = nb // 3 + 5, nb // 2 + 3
        W = torch.zeros(nb, dtype=torch.uint8, device="cuda")
        dt.pack(count, base, W.data_ptr() + off, offset=off, length=ln, stream=st)
        torch.cuda.synchronize()
        if not np.array_equal(P.cpu().numpy(), exp):
            bad.append((name, shift, "whole"))
        w = W.cpu().numpy()
        if not (np.array_equal(w[off:off + ln], exp[off:off + ln]) and not w[:off].any() and not w[off + ln:].any()):
            bad.append((name, shift, "window"))
        # unpack the stream into a pre-filled buffer: gap bytes keep theirs
        pre = np.random.default_rng(12).integers(0, 256, span, dtype=np.uint8)
        want = pre.copy()
        O.mxo_ddt_convert(rec["desc"].ctypes.data, rec["nrec"], B.ctypes.data, rec["lb"], rec["ub"], count,
                          want.ctypes.data - rec["true_lb"], exp.ctypes.data, 1)
        R = torch.zeros(span + 16, dtype=torch.uint8, device="cuda")
        R[shift:shift + span] = torch.from_numpy(pre).cuda()
        dt.unpack(count, R.data_ptr() + shift - rec["true_lb"], P.data_ptr(), stream=st)
        torch.cuda.synchronize()
        if not np.array_equal(R[shift:shift + span].cpu().numpy(), want):
            bad.append((name, shift, "unpack"))
print("BAD", bad)
sys.exit(1 if bad else 0)
"""


BMAP_TYPES = "struct_char_d3_int_resized48,indexed_f32_random,ref_blacs_indexed,ref_strange"
VEC_TYPES = "vector_f32_b1_s2,vector_f64_b3_s5,vector_f32_b4_s8"


def _env(env):
    e = dict(os.environ)
    for kv in env.split():
        k, v = kv.split("=")
        e[k] = v
    return e


def _run_all(cases):
    """Every (env, types) case in its own child process, all at once (the
    switches are read once per process; a child's run is mostly its own
    start-up, so they overlap it): each must exit 0."""
    procs = [(env, subprocess.Popen([sys.executable, "-c", CHILD, ROOT, types], stdout=subprocess.PIPE,
                                    stderr=subprocess.PIPE, text=True, env=_env(env))) for env, types in cases]
    failed = []
    for env, p in procs:
        try:
            out, err = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            out, err = p.communicate()
        if p.returncode != 0:
            failed.append((env, p.returncode, out[-2000:], err[-3000:]))
    assert not failed, failed


BMAP_SWITCHES = ["MX_CONV_BMAP_SPAN=12288", "MX_CONV_BMAP_SPAN=24576", "MX_CONV_BMAP_UNROLL=0", "MX_CONV_BMAP_QUAD=0",
                 "MX_CONV_BMAP_WORD=1", "MX_CONV_BMAP_NT=0", "MX_CONV_BMAP_DW=0", "MX_CONV_BMAP_CW=0",
                 "MX_NT_MIN_BYTES=0 MX_CONV_UNPACK_NTLD=1", "MX_CONV_BMAP_INST=0",
                 # the piece unpack forms (by default measured per datatype: staged or one piece per lane)
                 "MX_CONV_UNPACK_DIRECT=0", "MX_CONV_UNPACK_DIRECT=1", "MX_CONV_UNPACK_DIRECT=0 MX_CONV_UNPACK_U32=0",
                 "MX_CONV_UNPACK_DIRECT=0 MX_NT_MIN_BYTES=0 MX_CONV_UNPACK_NTLD=1"]


def test_byte_map_pack_switches():
    """Every byte-map switch, each in its own process, run concurrently."""
    _run_all([(env, BMAP_TYPES) for env in BMAP_SWITCHES])


def test_vec_pack_nontemporal():
    """The VEC and VEC-span PACK kernels' non-temporal instances (taken from
    MX_NT_MIN_BYTES of span + stream on; forced here at 4 MiB) and their
    ordinary ones."""
    _run_all([(env, VEC_TYPES) for env in ("MX_NT_MIN_BYTES=0", "MX_CONV_VEC_NT=0 MX_NT_MIN_BYTES=0")])
