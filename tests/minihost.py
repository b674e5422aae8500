"""ctypes view of the mini-host harness (zhpe-ompi_amd/lib/libmx_host.so),
which loads the mi355x components from lib/libmx_ompi.so the way Open MPI's
MCA repository would and restates op/coll selection and the MPI entry
points.  TEST INFRASTRUCTURE: the base op functions it seeds the tables
with, and the algorithms of its host coll modules, are the oracle
restatements (oracle/mx_oracle_op.c, oracle/mx_oracle_coll.c)."""
import ctypes
import os

import mxompi
import oracle_lib

vp, ci, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
AG = ctypes.CFUNCTYPE(ci, vp, vp, sz, vp)
REDUCER = ctypes.CFUNCTYPE(ci, ci, ci, vp, vp, sz, ci)
PATTERN = ctypes.CFUNCTYPE(ci, ci, ci, ci)
_state = {}


def host(with_components=True):
    """The harness, initialised with (or without) the components.  One
    library serves both modes, so switching re-runs mxh_init: a test that
    asked for the base functions only must not leave the next test's op
    tables and communicators without the components."""
    key = ("h", with_components)
    if key in _state:
        H = _state[key]
        if _state.get("mode") != with_components:
            comp = os.path.join(mxompi.LIB_DIR, "libmx_ompi.so").encode() if with_components else b""
            O = oracle_lib.oracle()
            rc = H.mxh_init(comp, ctypes.cast(O.mxo_reduce2, vp), ctypes.cast(O.mxo_supported, vp))
            assert rc == 0, rc
            _state["mode"] = with_components
        return H
    H = ctypes.CDLL(os.path.join(mxompi.LIB_DIR, "libmx_host.so"), mode=ctypes.RTLD_GLOBAL)
    H.mxh_init.argtypes = [ctypes.c_char_p, vp, vp]
    H.mxh_dtype.restype = vp
    H.mxh_dtype.argtypes = [ctypes.c_char_p]
    H.mxh_dtype_contiguous.restype = vp
    H.mxh_dtype_contiguous.argtypes = [ci, vp]
    H.mxh_dtype_vector.restype = vp
    H.mxh_dtype_vector.argtypes = [ci, ci, ci, vp]
    H.mxh_op.restype = vp
    H.mxh_op.argtypes = [ctypes.c_char_p]
    H.mxh_op_slot_owner.argtypes = [vp, ci, ci]
    H.mxh_set_mca.argtypes = [ctypes.c_char_p, ci]
    H.mxh_set_mca_str.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    H.mxh_intercomm_create.restype = vp
    H.mxh_intercomm_create.argtypes = [ci, ci, AG, vp]
    H.mxh_set_coll_oracle.argtypes = [vp]
    H.mxh_comm_create.restype = vp
    H.mxh_comm_create.argtypes = [ci, ci, AG, vp]
    H.mxh_comm_self.restype = vp
    H.mxh_comm_free.argtypes = [vp]
    H.mxh_comm_slot_owner.restype = ctypes.c_char_p
    H.mxh_comm_slot_owner.argtypes = [vp, ctypes.c_char_p]
    H.mxh_reduce_local.argtypes = [vp, vp, ci, vp, vp]
    H.mxh_op_reduce.argtypes = [vp, vp, vp, ci, vp]
    H.mxh_3buff_op_reduce.argtypes = [vp, vp, vp, vp, ci, vp]
    H.mxh_self_calls.argtypes = []
    H.mxh_allreduce.argtypes = [vp, vp, ci, vp, vp, vp]
    H.mxh_reduce_scatter.argtypes = [vp, vp, ctypes.POINTER(ci), vp, vp, vp]
    H.mxh_allgather.argtypes = [vp, ci, vp, vp, ci, vp, vp]
    H.mxh_bcast.argtypes = [vp, ci, vp, ci, vp]
    H.mxh_reduce.argtypes = [vp, vp, ci, vp, vp, ci, vp]
    H.mxh_reduce_scatter_block.argtypes = [vp, vp, ci, vp, vp, vp]
    H.mxh_scan.argtypes = [vp, vp, ci, vp, vp, vp]
    H.mxh_exscan.argtypes = [vp, vp, ci, vp, vp, vp]
    rq = ctypes.POINTER(vp)
    for name in ("mxh_iallreduce", "mxh_allreduce_init", "mxh_iscan", "mxh_iexscan"):
        getattr(H, name).argtypes = [vp, vp, ci, vp, vp, vp, rq]
    H.mxh_ireduce.argtypes = [vp, vp, ci, vp, vp, ci, vp, rq]
    H.mxh_reduce_init.argtypes = [vp, vp, ci, vp, vp, ci, vp, rq]
    H.mxh_ireduce_scatter.argtypes = [vp, vp, ctypes.POINTER(ci), vp, vp, vp, rq]
    H.mxh_ireduce_scatter_block.argtypes = [vp, vp, ci, vp, vp, vp, rq]
    H.mxh_iallgather.argtypes = [vp, ci, vp, vp, ci, vp, vp, rq]
    H.mxh_ibcast.argtypes = [vp, ci, vp, ci, vp, rq]
    H.mxh_start.argtypes = [vp]
    H.mxh_test.argtypes = [rq, ctypes.POINTER(ci)]
    H.mxh_wait.argtypes = [rq]
    H.mxh_request_free.argtypes = [rq]
    O = oracle_lib.oracle()
    base = ctypes.cast(O.mxo_reduce2, vp)
    pat = ctypes.cast(O.mxo_supported, vp)
    # the host coll modules evaluate coll/tuned, coll/basic and coll/libnbc
    # algorithms with the oracle restatement (mx_host.h mxh_coll_oracle_t)
    fns = [ctypes.cast(getattr(O, f), vp).value for f in
           ("mxo_allreduce", "mxo_reduce_scatter", "mxo_reduce", "mxo_scan", "mxo_exscan", "mxo_iallreduce",
            "mxo_ireduce", "mxo_ireduce_scatter")]
    table = (vp * len(fns))(*fns)
    _state[("oracle_table",)] = table
    H.mxh_set_coll_oracle(ctypes.cast(table, vp))
    comp = os.path.join(mxompi.LIB_DIR, "libmx_ompi.so").encode() if with_components else b""
    rc = H.mxh_init(comp, base, pat)
    assert rc == 0, rc
    _state[key] = H
    _state["mode"] = with_components
    return H


def dtype(H, name):
    return H.mxh_dtype(name.encode())


def op(H, name):
    return H.mxh_op(name.encode())
