"""CPU: the C-ABI library loads and exports every symbol include/*.h
declares; its (op,type) pattern and sizes equal the oracle's (which is
pinned to the reference tables).  No compute calls: no GPU here."""
import ctypes
import os
import re

import pytest

import mxompi
import oracle_lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DECL = re.compile(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*(mx[a-z]*_[A-Za-z0-9_]+)\s*\(", re.M)


def _declared(header):
    with open(os.path.join(ROOT, "include", header)) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(DECL.findall(text)))


def _headers():
    return sorted(h for h in os.listdir(os.path.join(ROOT, "include")) if h.endswith(".h"))


@pytest.mark.parametrize("header", _headers())
def test_all_declared_symbols_exported(header):
    names = _declared(header)
    assert names, header
    libs = [mxompi.lib()]
    if os.path.exists(os.path.join(mxompi.LIB_DIR, "libmx_ompi.so")):
        libs.append(mxompi._load("libmx_ompi.so"))
    missing = [n for n in names if not any(hasattr(L, n) for L in libs)]
    assert not missing, f"{header}: not exported: {missing}"


@pytest.mark.parametrize("table", [mxompi.TABLE_C_ONLY, mxompi.TABLE_WITH_FORTRAN])
def test_kernel_pattern_equals_reference_pattern(table):
    O = oracle_lib.oracle()
    L = mxompi.lib()
    for op in range(15):
        for t in range(41):
            assert bool(L.mx_op_supported(op, t, table)) == bool(O.mxo_supported(op, t, table)), \
                (mxompi.OPS[op], mxompi.TYPES[t])


def test_type_sizes():
    O = oracle_lib.oracle()
    for t in range(41):
        assert mxompi.type_size(t) == O.mxo_type_size(t), mxompi.TYPES[t]


def test_unsupported_pair_is_rejected_without_device():
    L = mxompi.lib()
    # MPI_LAND on MPI_FLOAT has a NULL slot in the reference table
    assert L.mx_reduce2(mxompi.OP["LAND"], mxompi.TYPE["FLOAT"], None, None, 4, None) == -2
    assert L.mx_reduce2(99, 0, None, None, 4, None) == -1
    assert L.mx_strerror(-2) == b"operation not defined for this datatype"


def test_request_array_helpers_on_null_and_inactive_entries():
    """mx_waitall / mx_waitany / mx_testall / mx_testany over arrays whose
    entries are all null (MPI_REQUEST_NULL): ompi_request_default_wait_any /
    test_any give MPI_UNDEFINED and, for Testany, flag = true
    (req_wait.c:84-125, req_test.c:172-185); Waitall / Testall complete at
    once.  No request is active, so no GPU call is made."""
    assert mxompi.UNDEFINED == -32766            # MPI_UNDEFINED, mpi.h.in:488
    mxompi.waitall([None, None])
    assert mxompi.waitany([None, None, None]) == mxompi.UNDEFINED
    assert mxompi.testany([None]) == (True, mxompi.UNDEFINED)
    assert mxompi.testall([None, None]) is True
    mxompi.waitall([])
    assert mxompi.waitany([]) == mxompi.UNDEFINED
    L = mxompi._coll_lib()
    idx, flag = ctypes.c_int(0), ctypes.c_int(0)
    assert L.mx_waitany(1, None, ctypes.byref(idx)) == -1           # MX_ERR_ARG: n > 0, no array
    assert L.mx_testany(0, None, None, ctypes.byref(flag)) == -1    # no index
