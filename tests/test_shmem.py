"""OpenSHMEM reductions (shmem_<type>_<op>_to_all -> scoll/mpi ->
coll allreduce, oshmem/mca/scoll/mpi/scoll_mpi_ops.c:212-275).

The (op, type) -> MPI mapping restates scoll_mpi_dtypes.h; every
shmem_*_to_all entry of oshmem/shmem/c/shmem_reduce.c must land on an
(op, type) pair the reference op table defines (except REAL16, for which the
reference has no kernel either)."""
import pytest

import mxompi

# (op, type, C type size) for every SHMEM_TYPE_REDUCE_OP instantiation in
# oshmem/shmem/c/shmem_reduce.c
ENTRIES = []
for op in ("AND", "OR", "XOR"):
    ENTRIES += [(op, "SHORT", 2), (op, "INT", 4), (op, "LONG", 8), (op, "LLONG", 8), (op, "INT16", 2),
                (op, "INT32", 4), (op, "INT64", 8)]
for op in ("MAX", "MIN"):
    ENTRIES += [(op, "SHORT", 2), (op, "INT", 4), (op, "LONG", 8), (op, "LLONG", 8), (op, "FLOAT", 4),
                (op, "DOUBLE", 8), (op, "LDOUBLE", 16), (op, "INT16", 2), (op, "INT32", 4), (op, "INT64", 8)]
for op in ("SUM", "PROD"):
    ENTRIES += [(op, "SHORT", 2), (op, "INT", 4), (op, "LONG", 8), (op, "LLONG", 8), (op, "FLOAT", 4),
                (op, "DOUBLE", 8), (op, "LDOUBLE", 16), (op, "FCOMPLEX", 8), (op, "DCOMPLEX", 16),
                (op, "INT16", 2), (op, "INT32", 4), (op, "INT64", 8)]
SOPS = ["AND", "OR", "XOR", "MAX", "MIN", "SUM", "PROD"]
STYPES = ["SHORT", "INT", "LONG", "LLONG", "INT16", "INT32", "INT64", "FLOAT", "DOUBLE", "LDOUBLE", "FCOMPLEX",
          "DCOMPLEX", "FINT2", "FINT4", "FINT8", "FREAL4", "FREAL8", "FREAL16"]
EXPECT_OP = {"AND": "BAND", "OR": "BOR", "XOR": "BXOR", "MAX": "MAX", "MIN": "MIN", "SUM": "SUM", "PROD": "PROD"}


def _map(op, t, size):
    import ctypes
    L = mxompi.lib()
    mo, mt = ctypes.c_int(), ctypes.c_int()
    rc = L.mx_shmem_to_mpi(SOPS.index(op), STYPES.index(t), ctypes.c_size_t(size), ctypes.byref(mo), ctypes.byref(mt))
    return rc, mo.value, mt.value


@pytest.mark.parametrize("op,t,size", ENTRIES)
def test_every_c_entry_maps_to_a_defined_pair(op, t, size):
    rc, mo, mt = _map(op, t, size)
    assert rc == 0
    assert mxompi.OPS[mo] == EXPECT_OP[op]
    fp = {"FLOAT": "FLOAT", "DOUBLE": "DOUBLE", "LDOUBLE": "LONG_DOUBLE", "FCOMPLEX": "C_FLOAT_COMPLEX",
          "DCOMPLEX": "C_DOUBLE_COMPLEX"}
    exp_t = fp[t] if t in fp else {2: "INT16_T", 4: "INT32_T", 8: "INT64_T"}[size]
    assert mxompi.TYPES[mt] == exp_t
    assert mxompi.op_supported(mo, mt)


def test_fortran_types_and_real16():
    assert _map("SUM", "FINT4", 4)[2] == mxompi.TYPE["INTEGER4"]
    assert _map("PROD", "FREAL8", 8)[2] == mxompi.TYPE["REAL8"]
    assert _map("OR", "FINT2", 2)[2] == mxompi.TYPE["INT16_T"]     # by size (default branch)
    rc, mo, mt = _map("SUM", "FREAL16", 16)
    assert mt == mxompi.TYPE["REAL16"] and not mxompi.op_supported(mo, mt)
