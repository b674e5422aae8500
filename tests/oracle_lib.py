"""Loader for the CPU oracle (TEST INFRASTRUCTURE).

oracle/build/libmx_oracle.so is our plain-C restatement; oracle/_ref/*.so
are the reference's own kernels compiled from /root/reference (present only
when they were built in the development container; they travel to the GPU
box as prebuilt files).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline may use this module.
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


def ref_op(fortran=True):
    """The reference's compiled op_base_functions.c, or None if not built."""
    name = "libref_op_f.so" if fortran else "libref_op.so"
    path = os.path.join(ORACLE, "_ref", name)
    if not os.path.exists(path):
        return None
    key = "ref" + name
    if key not in _cache:
        _cache[key] = ctypes.CDLL(path)
    return _cache[key]


def ref_table(lib, three=False):
    """Read ompi_op_base_[3buff_]functions[15][41] as a 15x41 list of ints."""
    sym = "ompi_op_base_3buff_functions" if three else "ompi_op_base_functions"
    arr = (ctypes.c_void_p * (15 * 41)).in_dll(lib, sym)
    return [[arr[o * 41 + t] or 0 for t in range(41)] for o in range(15)]
