"""Loader for the CPU oracle (TEST INFRASTRUCTURE).

oracle/build/libmx_oracle.so is our plain-C restatement of the reference's
op kernels, coll/base + libnbc algorithms and convertor walk.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline may use this module.
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
_cache = {}


def oracle():
    if "o" in _cache:
        return _cache["o"]
    path = os.path.join(ORACLE, "build", "libmx_oracle.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", ORACLE, "build/libmx_oracle.so"], check=True)
    L = ctypes.CDLL(path)
    vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L.mxo_reduce2.argtypes = [i, i, vp, vp, sz, i]
    L.mxo_reduce3.argtypes = [i, i, vp, vp, vp, sz, i]
    L.mxo_supported.argtypes = [i, i, i]
    L.mxo_type_size.restype = sz
    L.mxo_type_size.argtypes = [i]
    _cache["o"] = L
    return L
