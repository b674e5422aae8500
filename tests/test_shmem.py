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


# ---- scoll/basic recursive doubling (round 4): the oracle restatement -------------
def _basic(op, t, n, xs):
    import ctypes
    import numpy as np
    import oracle_lib
    vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L = oracle_lib.oracle()
    L.mxo_shmem_basic_reduce.argtypes = [ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    outs = [np.zeros_like(xs[0]) for _ in range(n)]
    assert L.mxo_shmem_basic_reduce(mxompi.OP[op], mxompi.TYPE[t], n, len(xs[0]),
                                    (vp * n)(*[x.ctypes.data for x in xs]),
                                    (vp * n)(*[o.ctypes.data for o in outs])) == 0
    return outs


@pytest.mark.parametrize("n", range(1, 17))
def test_scoll_basic_oracle_gives_the_examples_answer(n):
    """examples/oshmem_max_reduction.c:36-46 (N = 3): src[i] = my_pe + i,
    shmem_long_max_to_all -> dst[i] = npes - 1 + i on every PE, for every PE
    count (extras when n is not a power of two)."""
    import numpy as np
    outs = _basic("MAX", "INT64_T", n, [np.array([r + i for i in range(3)], np.int64) for r in range(n)])
    for o in outs:
        assert o.tolist() == [n - 1 + i for i in range(3)]


def test_scoll_basic_oracle_keeps_each_pes_own_operand_roles():
    """Each PE folds the partner's value into its own (c_fn(in = received,
    out = own), scoll_basic_reduce.c:502-504): with MAX = (own > received ?
    own : received) a NaN on one side of a pair stays with that side only,
    so the two PEs of a pair end with different values (n = 2: PE 0 holds
    NaN, PE 1 holds 1.0 -> PE 0: NaN > 1 false -> 1.0; PE 1: 1 > NaN false ->
    NaN)."""
    import numpy as np
    outs = _basic("MAX", "DOUBLE", 2, [np.array([np.nan]), np.array([1.0])])
    assert outs[0][0] == 1.0 and np.isnan(outs[1][0])
