"""mxompi -- Python view of the MI355X collective-reduction hot path.

Thin ctypes binding of the C-ABI libraries built in-tree by
``zhpe-ompi_amd/Makefile``:

* ``lib/libmx_kernels.so`` -- HIP kernels for gfx950 behind
  ``include/mx_kernels.h`` (op kernels), ``include/mx_convertor.h``
  (datatype pack/unpack) and ``include/mx_coll.h`` (collectives);
* ``lib/libmx_ompi.so`` -- the host C MCA components (``op/mi355x``,
  ``coll/mi355x``) plus the mini-host harness that mimics Open MPI's
  selection logic.

Python is used by the tests and by ``bench.py`` only (device memory comes
from torch tensors); the product path is C/HIP.  There is no CPU fallback:
if the HIP library is missing, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_DIR = os.path.join(PKG_ROOT, "lib")

# ---- op / type numbering == OMPI_OP_BASE_FORTRAN_* / OMPI_OP_BASE_TYPE_* ----
OPS = ["NULL", "MAX", "MIN", "SUM", "PROD", "LAND", "BAND", "LOR", "BOR",
       "LXOR", "BXOR", "MAXLOC", "MINLOC", "REPLACE", "NO_OP"]
OP = {name: i for i, name in enumerate(OPS)}

TYPES = ["INT8_T", "UINT8_T", "INT16_T", "UINT16_T", "INT32_T", "UINT32_T",
         "INT64_T", "UINT64_T", "INTEGER", "INTEGER1", "INTEGER2", "INTEGER4",
         "INTEGER8", "INTEGER16", "SHORT_FLOAT", "FLOAT", "DOUBLE", "REAL",
         "REAL2", "REAL4", "REAL8", "REAL16", "DOUBLE_PRECISION", "LONG_DOUBLE",
         "LOGICAL", "BOOL", "C_SHORT_FLOAT_COMPLEX", "C_FLOAT_COMPLEX",
         "C_DOUBLE_COMPLEX", "C_LONG_DOUBLE_COMPLEX", "BYTE", "2REAL",
         "2DOUBLE_PRECISION", "2INTEGER", "FLOAT_INT", "DOUBLE_INT", "LONG_INT",
         "2INT", "SHORT_INT", "LONG_DOUBLE_INT", "WCHAR"]
TYPE = {name: i for i, name in enumerate(TYPES)}

TABLE_C_ONLY = 0
TABLE_WITH_FORTRAN = 1

# MPI predefined datatype -> op type slot (restates ompi/op/op.c:131-229 with
# the C aliases of ompi/datatype/ompi_datatype_internal.h:130-200 for LP64).
MPI_DTYPE_SLOT = {
    "MPI_INT8_T": "INT8_T", "MPI_UINT8_T": "UINT8_T", "MPI_INT16_T": "INT16_T",
    "MPI_UINT16_T": "UINT16_T", "MPI_INT32_T": "INT32_T", "MPI_UINT32_T": "UINT32_T",
    "MPI_INT64_T": "INT64_T", "MPI_UINT64_T": "UINT64_T",
    "MPI_CHAR": "INT8_T", "MPI_SIGNED_CHAR": "INT8_T", "MPI_UNSIGNED_CHAR": "UINT8_T",
    "MPI_BYTE": "UINT8_T", "MPI_SHORT": "INT16_T", "MPI_UNSIGNED_SHORT": "UINT16_T",
    "MPI_INT": "INT32_T", "MPI_UNSIGNED": "UINT32_T", "MPI_LONG": "INT64_T",
    "MPI_UNSIGNED_LONG": "UINT64_T", "MPI_LONG_LONG_INT": "INT64_T",
    "MPI_LONG_LONG": "INT64_T", "MPI_UNSIGNED_LONG_LONG": "UINT64_T",
    "MPI_FLOAT": "FLOAT", "MPI_DOUBLE": "DOUBLE", "MPI_LONG_DOUBLE": "LONG_DOUBLE",
    "MPI_WCHAR": "WCHAR", "MPI_CXX_BOOL": "BOOL", "MPI_LOGICAL": "LOGICAL",
    "MPI_CHARACTER": "UINT8_T", "MPI_INTEGER": "INTEGER", "MPI_REAL": "REAL",
    "MPI_DOUBLE_PRECISION": "DOUBLE_PRECISION",
    "MPI_LONG_DOUBLE_COMPLEX": "C_LONG_DOUBLE_COMPLEX",
    "MPI_2INT": "2INT", "MPI_2INTEGER": "2INTEGER", "MPI_2REAL": "2REAL",
    "MPI_2DOUBLE_PRECISION": "2DOUBLE_PRECISION", "MPI_FLOAT_INT": "FLOAT_INT",
    "MPI_DOUBLE_INT": "DOUBLE_INT", "MPI_LONG_DOUBLE_INT": "LONG_DOUBLE_INT",
    "MPI_LONG_INT": "LONG_INT", "MPI_SHORT_INT": "SHORT_INT",
    "MPI_AINT": "INT64_T", "MPI_OFFSET": "UINT64_T", "MPI_C_BOOL": "BOOL",
    "MPI_C_COMPLEX": "C_FLOAT_COMPLEX", "MPI_C_FLOAT_COMPLEX": "C_FLOAT_COMPLEX",
    "MPI_C_DOUBLE_COMPLEX": "C_DOUBLE_COMPLEX",
    "MPI_C_LONG_DOUBLE_COMPLEX": "C_LONG_DOUBLE_COMPLEX", "MPI_COUNT": "INT64_T",
}

ERRORS = {0: "MX_SUCCESS", -1: "MX_ERR_ARG", -2: "MX_ERR_UNSUPPORTED", -3: "MX_ERR_HIP",
          -4: "MX_ERR_NOMEM", -5: "MX_ERR_TIMEOUT", -6: "MX_ERR_RCCL",
          -7: "MX_ERR_NOT_INIT", -8: "MX_ERR_STATE", -9: "MX_ERR_TRUNCATE", -10: "MX_ERR_TAG"}


class MxError(RuntimeError):
    def __init__(self, rc: int, what: str = ""):
        super().__init__(f"{what}: {ERRORS.get(rc, rc)} ({rc})")
        self.rc = rc


_libs: dict = {}


def _load(name: str) -> ctypes.CDLL:
    if name in _libs:
        return _libs[name]
    path = os.path.join(LIB_DIR, name)
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} is missing: the HIP product library was not built "
            "(run `make -C zhpe-ompi_amd` or __graft_entry__.build()); "
            "there is no CPU fallback")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    _libs[name] = lib
    return lib


def lib() -> ctypes.CDLL:
    """The HIP kernel library (C-ABI of include/mx_kernels.h)."""
    L = _load("libmx_kernels.so")
    if not getattr(L, "_mx_typed", False):
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.mx_init.argtypes = [i]
        L.mx_is_device_ptr.argtypes = [vp]
        L.mx_stream_sync.argtypes = [vp]
        L.mx_strerror.restype = ctypes.c_char_p
        L.mx_strerror.argtypes = [i]
        L.mx_version.restype = ctypes.c_char_p
        L.mx_type_size.restype = sz
        L.mx_type_size.argtypes = [i]
        L.mx_op_supported.argtypes = [i, i, i]
        L.mx_reduce2.argtypes = [i, i, vp, vp, sz, vp]
        L.mx_reduce2_sync.argtypes = [i, i, vp, vp, sz, vp]
        L.mx_reduce3.argtypes = [i, i, vp, vp, vp, sz, vp]
        L.mx_reduce3_sync.argtypes = [i, i, vp, vp, vp, sz, vp]
        L.mx_copy.argtypes = [vp, vp, sz, vp]
        L.mx_shmem_to_mpi.argtypes = [i, i, sz, ctypes.POINTER(i), ctypes.POINTER(i)]
        L.mx_op_service_stats.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong)]
        L.mx_op_service_held.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
        L.mx_op_service_set.argtypes = [ctypes.c_int]
        L.mx_debug_hold.argtypes = [vp, ctypes.c_uint]
        L.mx_debug_hold_service.argtypes = [ctypes.c_uint]
        L._mx_typed = True
    return L


def check(rc: int, what: str = "mx call") -> int:
    if rc < 0:
        raise MxError(rc, what)
    return rc


def _slot(v) -> int:
    """Type slot from a slot name ("FLOAT"), an MPI datatype name ("MPI_FLOAT") or an int."""
    if isinstance(v, str):
        return TYPE[MPI_DTYPE_SLOT[v]] if v.startswith("MPI_") else TYPE[v]
    return int(v)


def _op(v) -> int:
    """Op index from "SUM", "MPI_SUM" or an int."""
    if isinstance(v, str):
        return OP[v[4:] if v.startswith("MPI_") else v]
    return int(v)


def type_size(t) -> int:
    return int(lib().mx_type_size(_slot(t)))


def op_supported(op, t, table=TABLE_WITH_FORTRAN) -> bool:
    return bool(lib().mx_op_supported(_op(op), _slot(t), table))


def reduce2(op, t, in_ptr: int, inout_ptr: int, count: int, stream: int = 0) -> None:
    """inout = inout OP in on the device (asynchronous on `stream`)."""
    check(lib().mx_reduce2(_op(op), _slot(t), in_ptr, inout_ptr, count, stream or None),
          f"mx_reduce2({op},{t})")


def reduce2_sync(op, t, in_ptr: int, inout_ptr: int, count: int, stream: int = 0) -> None:
    """inout = inout OP in on the device; returns with the result complete
    (mx_reduce2_sync: a completion word raised by the kernel's last workgroup
    for launches of <= 64 workgroups, else by a marker kernel)."""
    check(lib().mx_reduce2_sync(_op(op), _slot(t), in_ptr, inout_ptr, count, stream or None),
          f"mx_reduce2_sync({op},{t})")


def reduce3(op, t, in1_ptr: int, in2_ptr: int, out_ptr: int, count: int, stream: int = 0) -> None:
    """out = in1 OP in2 on the device (asynchronous on `stream`)."""
    check(lib().mx_reduce3(_op(op), _slot(t), in1_ptr, in2_ptr, out_ptr, count, stream or None),
          f"mx_reduce3({op},{t})")


def reduce3_sync(op, t, in1_ptr: int, in2_ptr: int, out_ptr: int, count: int, stream: int = 0) -> None:
    """out = in1 OP in2, returning with `out` complete (mx_reduce3_sync)."""
    check(lib().mx_reduce3_sync(_op(op), _slot(t), in1_ptr, in2_ptr, out_ptr, count, stream or None),
          f"mx_reduce3_sync({op},{t})")


def op_service_stats():
    """(state, commands served, service launches) of the resident reduce
    service behind mx_reduce2_sync (include/mx_kernels.h)."""
    a, b = ctypes.c_ulonglong(), ctypes.c_ulonglong()
    st = lib().mx_op_service_stats(ctypes.byref(a), ctypes.byref(b))
    return st, a.value, b.value


def op_service_set(on: bool) -> None:
    """Turn the resident reduce service on or off (overrides MX_OP_SERVICE)."""
    check(lib().mx_op_service_set(1 if on else 0), "mx_op_service_set")


def op_service_held():
    """(a held kernel has not yet left, launches held so far): service
    launches that did not start within 1 ms (include/mx_kernels.h)."""
    a = ctypes.c_ulonglong()
    st = lib().mx_op_service_held(ctypes.byref(a))
    return bool(st), a.value


def debug_hold(stream: int, timeout_ms: int = 5000) -> None:
    """Test support: hold `stream`'s hardware queue with a spinning wave
    until debug_release() or timeout_ms."""
    check(lib().mx_debug_hold(stream, timeout_ms), "mx_debug_hold")


def debug_hold_service(timeout_ms: int = 5000) -> None:
    """Test support: hold the op service's own stream the same way."""
    check(lib().mx_debug_hold_service(timeout_ms), "mx_debug_hold_service")


def debug_release() -> None:
    check(lib().mx_debug_release(), "mx_debug_release")


def init(device: int = 0) -> None:
    check(lib().mx_init(device), "mx_init")


def sync(stream: int = 0) -> None:
    check(lib().mx_stream_sync(stream or None), "mx_stream_sync")


# ---------------------------------------------------------------------------
# collectives (include/mx_coll.h)
# ---------------------------------------------------------------------------
IN_PLACE = 1                       # MX_IN_PLACE
ANY_SOURCE = -1                    # MX_ANY_SOURCE (MPI_ANY_SOURCE)
COMM_IPC, COMM_RCCL, COMM_P2P = 1, 2, 4
ALLREDUCE = {"auto": 0, "basic_linear": 1, "nonoverlapping": 2, "recursive_doubling": 3,
             "ring": 4, "segmented_ring": 5, "rabenseifner": 6, "rccl": 100}
REDUCE_SCATTER = {"auto": 0, "nonoverlapping": 1, "recursive_halving": 2, "ring": 3, "butterfly": 4, "rccl": 100}
REDUCE = {"auto": 0, "linear": 1, "chain": 2, "pipeline": 3, "binary": 4, "binomial": 5,
          "in_order_binary": 6, "rabenseifner": 7}
SCAN = {"auto": 0, "linear": 1, "recursive_doubling": 2}


def alg_word(alg, reduce_alg=0, chain_fanout=0):
    """MX_ALG_WORD (include/mx_coll.h): an algorithm id plus, for the
    algorithms built on a rooted reduce, the reduce algorithm coll_reduce
    runs (bits 8-15) and the chain fanout (bits 16-23)."""
    if isinstance(reduce_alg, str):
        reduce_alg = REDUCE[reduce_alg]
    return int(alg) | (int(reduce_alg) << 8) | (int(chain_fanout) << 16)
# libnbc numbering (coll_libnbc_component.c:58-92)
IALLREDUCE = {"auto": 0, "ring": 1, "binomial": 2, "rabenseifner": 3, "recursive_doubling": 4}
IREDUCE = {"auto": 0, "chain": 1, "binomial": 2, "rabenseifner": 3}

class CollStats(ctypes.Structure):
    _fields_ = [("calls", ctypes.c_uint64), ("fold_launches", ctypes.c_uint64), ("fold_ms", ctypes.c_double),
                ("fold_bytes", ctypes.c_double), ("push_ms", ctypes.c_double), ("gather_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double), ("zero_copy_calls", ctypes.c_uint64),
                ("staged_calls", ctypes.c_uint64), ("direct_calls", ctypes.c_uint64),
                ("reg_fast_calls", ctypes.c_uint64), ("p2p_relaunches", ctypes.c_uint64),
                ("p2p_pulls", ctypes.c_uint64), ("service_calls", ctypes.c_uint64),
                ("reg_stale_refused", ctypes.c_uint64)]


_AG_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


def _coll_lib():
    L = lib()
    if not getattr(L, "_mx_coll_typed", False):
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        pp = ctypes.POINTER(ctypes.c_void_p)
        L.mx_comm_create.argtypes = [i, i, i, sz, i, _AG_FN, vp, ctypes.POINTER(vp)]
        L.mx_comm_create_ex.argtypes = [i, i, i, sz, sz, i, _AG_FN, vp, ctypes.POINTER(vp)]
        L.mx_comm_create_local.argtypes = [i, i, ctypes.POINTER(vp)]
        L.mx_comm_destroy.argtypes = [vp]
        L.mx_comm_set_timeout.argtypes = [vp, ctypes.c_double]
        L.mx_comm_set_protocol.argtypes = [vp, i]
        L.mx_comm_get_protocol.argtypes = [vp]
        L.mx_comm_set_reg_min.argtypes = [vp, sz]
        L.mx_comm_set_zc_direct.argtypes = [vp, i]
        L.mx_comm_set_oneshot_max.argtypes = [vp, sz]
        L.mx_comm_set_oneshot_max.restype = ctypes.c_longlong
        L.mx_comm_set_autotune.argtypes = [vp, i]
        L.mx_comm_get_tuning.argtypes = [vp, sz]
        L.mx_comm_get_tuning_ex.argtypes = [vp, i, sz]
        L.mx_allreduce.argtypes = [vp, vp, vp, sz, i, i, i, vp]
        L.mx_allreduce_local.argtypes = [vp, pp, pp, sz, i, i, i, vp]
        L.mx_reduce_scatter.argtypes = [vp, vp, vp, ctypes.POINTER(sz), i, i, i, vp]
        L.mx_reduce_scatter_local.argtypes = [vp, pp, pp, ctypes.POINTER(sz), i, i, i, vp]
        L.mx_allgather.argtypes = [vp, vp, vp, sz, vp]
        L.mx_allgather_local.argtypes = [vp, pp, pp, sz, vp]
        L.mx_bcast.argtypes = [vp, vp, sz, i, vp]
        L.mx_bcast_local.argtypes = [vp, pp, sz, i, vp]
        L.mx_allreduce_decision.argtypes = [i, sz, i]
        L.mx_comm_set_profiling.argtypes = [vp, i]
        L.mx_shmem_reduce.argtypes = [vp, i, i, sz, vp, vp, sz, vp]
        L.mx_shmem_reduce_basic.argtypes = [vp, i, i, sz, vp, vp, sz, vp]
        L.mx_comm_get_stats.argtypes = [vp, ctypes.POINTER(CollStats), i]
        L.mx_reduce_scatter_decision.argtypes = [i, sz, i]
        L.mx_reduce_decision.argtypes = [i, sz, i]
        L.mx_reduce.argtypes = [vp, vp, vp, sz, i, i, i, i, vp]
        L.mx_reduce_local.argtypes = [vp, pp, pp, sz, i, i, i, i, vp]
        for name in ("mx_scan", "mx_exscan", "mx_reduce_scatter_block"):
            getattr(L, name).argtypes = [vp, vp, vp, sz, i, i, i, vp]
            getattr(L, name + "_local").argtypes = [vp, pp, pp, sz, i, i, i, vp]
        # non-blocking / persistent
        rq = ctypes.POINTER(vp)
        for name in ("mx_iallreduce", "mx_allreduce_init", "mx_iscan", "mx_scan_init", "mx_iexscan",
                     "mx_exscan_init"):
            getattr(L, name).argtypes = [vp, vp, vp, sz, i, i, i, vp, rq]
        for name in ("mx_ireduce", "mx_reduce_init"):
            getattr(L, name).argtypes = [vp, vp, vp, sz, i, i, i, i, vp, rq]
        for name in ("mx_ireduce_scatter", "mx_reduce_scatter_init"):
            getattr(L, name).argtypes = [vp, vp, vp, ctypes.POINTER(sz), i, i, vp, rq]
        for name in ("mx_ireduce_scatter_block", "mx_reduce_scatter_block_init"):
            getattr(L, name).argtypes = [vp, vp, vp, sz, i, i, vp, rq]
        for name in ("mx_iallgather", "mx_allgather_init"):
            getattr(L, name).argtypes = [vp, vp, vp, sz, vp, rq]
        for name in ("mx_ibcast", "mx_bcast_init"):
            getattr(L, name).argtypes = [vp, vp, sz, i, vp, rq]
        L.mx_start.argtypes = [vp]
        L.mx_startall.argtypes = [sz, pp]
        L.mx_waitall.argtypes = [sz, pp]
        L.mx_waitany.argtypes = [sz, pp, ctypes.POINTER(i)]
        L.mx_testall.argtypes = [sz, pp, ctypes.POINTER(i)]
        L.mx_testany.argtypes = [sz, pp, ctypes.POINTER(i), ctypes.POINTER(i)]
        L.mx_test.argtypes = [vp, ctypes.POINTER(i)]
        L.mx_wait.argtypes = [vp]
        L.mx_request_stream_wait.argtypes = [vp, vp]
        L.mx_request_is_active.argtypes = [vp]
        L.mx_request_free.argtypes = [vp]
        L.mx_iallreduce_decision.argtypes = [i, sz, i, i]
        # point-to-point
        L.mx_send.argtypes = [vp, vp, sz, i, i, vp]
        L.mx_recv.argtypes = [vp, vp, sz, i, i, vp, ctypes.POINTER(sz)]
        for name in ("mx_isend", "mx_irecv", "mx_send_init", "mx_recv_init"):
            getattr(L, name).argtypes = [vp, vp, sz, i, i, vp, rq]
        for name in ("mx_isend_ddt", "mx_irecv_ddt"):
            getattr(L, name).argtypes = [vp, vp, sz, vp, i, i, vp, rq]
        L.mx_sendrecv.argtypes = [vp, vp, sz, i, i, vp, sz, i, i, vp, ctypes.POINTER(sz)]
        L.mx_request_status.argtypes = [vp, ctypes.POINTER(sz), ctypes.POINTER(i)]
        L.mx_request_source.argtypes = [vp, ctypes.POINTER(i)]
        L.mx_ireduce_decision.argtypes = [i, sz, i]
        L._mx_coll_typed = True
    return L


def _ptrs(seq):
    arr = (ctypes.c_void_p * len(seq))()
    for k, p in enumerate(seq):
        arr[k] = p
    return arr


def _alg(table, a):
    return table[a] if isinstance(a, str) else int(a)


class Request:
    """A non-blocking or persistent collective (include/mx_coll.h requests):
    MPI_Test / MPI_Wait / MPI_Start / MPI_Request_free."""

    def __init__(self, handle, persistent, keep=()):
        self.h = handle
        self.persistent = persistent
        self._keep = keep          # ctypes arrays the request reads at start

    def start(self):
        check(_coll_lib().mx_start(self.h), "mx_start")

    def test(self) -> bool:
        flag = ctypes.c_int(0)
        check(_coll_lib().mx_test(self.h, ctypes.byref(flag)), "mx_test")
        return bool(flag.value)

    def wait(self):
        check(_coll_lib().mx_wait(self.h), "mx_wait")

    def stream_wait(self, stream=0):
        check(_coll_lib().mx_request_stream_wait(self.h, stream or None), "mx_request_stream_wait")

    @property
    def active(self) -> bool:
        return bool(_coll_lib().mx_request_is_active(self.h))

    def status(self):
        """(bytes delivered, envelope tag) of a completed receive."""
        nb, tag = ctypes.c_size_t(), ctypes.c_int()
        check(_coll_lib().mx_request_status(self.h, ctypes.byref(nb), ctypes.byref(tag)), "mx_request_status")
        return nb.value, tag.value

    def source(self):
        """MPI_SOURCE of a completed receive (the matched rank for ANY_SOURCE)."""
        src = ctypes.c_int()
        check(_coll_lib().mx_request_source(self.h, ctypes.byref(src)), "mx_request_source")
        return src.value

    def free(self):
        if getattr(self, "h", None):
            h, self.h = self.h, None
            check(_coll_lib().mx_request_free(h), "mx_request_free")

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001
            pass


def startall(reqs):
    arr = _ptrs([r.h for r in reqs])
    check(_coll_lib().mx_startall(len(reqs), arr), "mx_startall")


UNDEFINED = -32766   # MX_UNDEFINED (MPI_UNDEFINED)


def _hs(reqs):
    return _ptrs([r.h if r is not None else None for r in reqs])


def waitall(reqs):
    """MPI_Waitall: complete every request (None entries skipped)."""
    check(_coll_lib().mx_waitall(len(reqs), _hs(reqs)), "mx_waitall")


def waitany(reqs):
    """MPI_Waitany: index of the request completed, UNDEFINED if none is active."""
    idx = ctypes.c_int(0)
    check(_coll_lib().mx_waitany(len(reqs), _hs(reqs), ctypes.byref(idx)), "mx_waitany")
    return idx.value


def testall(reqs):
    """MPI_Testall: True (and all completed) once every request is complete."""
    flag = ctypes.c_int(0)
    check(_coll_lib().mx_testall(len(reqs), _hs(reqs), ctypes.byref(flag)), "mx_testall")
    return bool(flag.value)


def testany(reqs):
    """MPI_Testany: (flag, index)."""
    idx, flag = ctypes.c_int(0), ctypes.c_int(0)
    check(_coll_lib().mx_testany(len(reqs), _hs(reqs), ctypes.byref(idx), ctypes.byref(flag)), "mx_testany")
    return bool(flag.value), idx.value


def iallreduce_decision(n, count, t, inplace=False):
    return _coll_lib().mx_iallreduce_decision(n, count, _slot(t), 1 if inplace else 0)


def ireduce_decision(n, count, t):
    return _coll_lib().mx_ireduce_decision(n, count, _slot(t))


class Comm:
    """A communicator of the MI355X collective path.

    Comm.local(size): `size` virtual ranks in this process (one device).
    Comm(rank, size, allgather): one rank per process; `allgather(bytes) ->
    list[bytes]` is the host bootstrap exchange (e.g. torch.distributed)."""

    def __init__(self, rank=0, size=1, allgather=None, device=0, staging_bytes=64 << 20,
                 flags=COMM_IPC | COMM_P2P, heap_bytes=0, _handle=None):
        L = _coll_lib()
        self.size = size
        self.rank = rank
        self._cb = None
        if _handle is not None:
            self.h = _handle
            return
        if allgather is None:
            raise ValueError("a host allgather is required for a multi-process communicator")

        def _ag(send, recv, nbytes, ctx):
            try:
                parts = allgather(ctypes.string_at(send, nbytes))
                blob = b"".join(parts)
                ctypes.memmove(recv, blob, len(blob))
                return 0
            except Exception:  # noqa: BLE001 - reported as a C error code
                import traceback
                traceback.print_exc()
                return -1

        self._cb = _AG_FN(_ag)
        h = ctypes.c_void_p()
        check(L.mx_comm_create_ex(rank, size, device, staging_bytes, heap_bytes, flags, self._cb, None,
                                  ctypes.byref(h)), "mx_comm_create")
        self.h = h

    @classmethod
    def local(cls, size, device=0):
        h = ctypes.c_void_p()
        check(_coll_lib().mx_comm_create_local(size, device, ctypes.byref(h)), "mx_comm_create_local")
        return cls(0, size, _handle=h)

    def set_profiling(self, on=True):
        check(_coll_lib().mx_comm_set_profiling(self.h, 1 if on else 0), "mx_comm_set_profiling")

    def stats(self, reset=False):
        st = CollStats()
        check(_coll_lib().mx_comm_get_stats(self.h, ctypes.byref(st), 1 if reset else 0), "mx_comm_get_stats")
        return {k: getattr(st, k) for k, _ in CollStats._fields_}

    def set_timeout(self, seconds):
        check(_coll_lib().mx_comm_set_timeout(self.h, seconds), "mx_comm_set_timeout")

    PROTO = {"auto": 0, "push": 1, "pull": 2}

    def set_protocol(self, proto):
        """Staged allreduce data movement ("auto" | "push" | "pull", mx_comm_set_protocol);
        every rank must set the same one.  Returns the protocol in force."""
        rc = _coll_lib().mx_comm_set_protocol(self.h, self.PROTO[proto])
        check(min(rc, 0), "mx_comm_set_protocol")
        return {1: "push", 2: "pull"}[rc]

    def protocol(self):
        return {1: "push", 2: "pull"}.get(_coll_lib().mx_comm_get_protocol(self.h), "none")

    def set_autotune(self, on):
        """Data-movement autotuning of large blocking allreduces (mx_comm_set_autotune)."""
        check(_coll_lib().mx_comm_set_autotune(self.h, 1 if on else 0), "mx_comm_set_autotune")

    _TUNE = {"allreduce": (0, {0: "zero_copy", 1: "pull", 2: "push", 3: "one_shot"}),
             "reduce_scatter": (1, {0: "zero_copy", 1: "staged"}),
             "allgather": (2, {0: "zero_copy", 1: "staged"}),
             "bcast": (3, {0: "zero_copy", 1: "scatter", 2: "direct"})}

    def tuning(self, nbytes, coll="allreduce"):
        """The data movement autotuning kept for `coll` calls of nbytes per rank
        (mx_comm_get_tuning_ex), or None while untuned."""
        k, names = self._TUNE[coll]
        return names.get(_coll_lib().mx_comm_get_tuning_ex(self.h, k, nbytes))

    def set_reg_min(self, min_bytes):
        """Zero-copy (registered user buffers) allreduce from min_bytes per rank; 0 = off
        (mx_comm_set_reg_min).  Every rank must set the same value."""
        check(_coll_lib().mx_comm_set_reg_min(self.h, min_bytes), "mx_comm_set_reg_min")

    def set_zc_direct(self, on):
        """Zero-copy allreduce results straight into the peers' rbufs (True, the default) or
        through the gather areas (mx_comm_set_zc_direct).  Every rank must set the same value."""
        check(_coll_lib().mx_comm_set_zc_direct(self.h, 1 if on else 0), "mx_comm_set_zc_direct")

    def set_oneshot_max(self, max_bytes):
        """One-shot allreduce up to max_bytes per rank, clamped to the slot
        capacity (mx_comm_set_oneshot_max); 0 = off.  Every rank must set the
        same value.  Returns the crossover in force."""
        rc = _coll_lib().mx_comm_set_oneshot_max(self.h, max_bytes)
        check(min(rc, 0), "mx_comm_set_oneshot_max")
        return rc

    def close(self):
        if getattr(self, "h", None):
            _coll_lib().mx_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    # -- multi-process -----------------------------------------------------
    def allreduce(self, sbuf, rbuf, count, t, op, alg="auto", stream=0):
        check(_coll_lib().mx_allreduce(self.h, sbuf, rbuf, count, _slot(t), _op(op),
                                       _alg(ALLREDUCE, alg), stream or None), "mx_allreduce")

    def reduce_scatter(self, sbuf, rbuf, rcounts, t, op, alg="auto", stream=0):
        rc = (ctypes.c_size_t * len(rcounts))(*rcounts)
        check(_coll_lib().mx_reduce_scatter(self.h, sbuf, rbuf, rc, _slot(t), _op(op),
                                            _alg(REDUCE_SCATTER, alg), stream or None), "mx_reduce_scatter")

    def allgather(self, sbuf, rbuf, nbytes, stream=0):
        check(_coll_lib().mx_allgather(self.h, sbuf, rbuf, nbytes, stream or None), "mx_allgather")

    def shmem_reduce(self, op, t, dt_size, target, source, nreduce, stream=0):
        """shmem_<t>_<op>_to_all over this communicator's ranks (scoll/mpi path)."""
        sops = ["AND", "OR", "XOR", "MAX", "MIN", "SUM", "PROD"]
        sts = ["SHORT", "INT", "LONG", "LLONG", "INT16", "INT32", "INT64", "FLOAT", "DOUBLE", "LDOUBLE",
               "FCOMPLEX", "DCOMPLEX", "FINT2", "FINT4", "FINT8", "FREAL4", "FREAL8", "FREAL16"]
        check(_coll_lib().mx_shmem_reduce(self.h, sops.index(op), sts.index(t), dt_size, target, source, nreduce,
                                          stream or None), "mx_shmem_reduce")

    def shmem_reduce_basic(self, op, t, dt_size, target, source, nreduce, stream=0):
        """scoll/basic's recursive-doubling shmem_<t>_<op>_to_all (mx_shmem_reduce_basic)."""
        check(_coll_lib().mx_shmem_reduce_basic(self.h, SHMEM_OPS.index(op), SHMEM_TYPES.index(t), dt_size, target,
                                                source, nreduce, stream or None), "mx_shmem_reduce_basic")

    def bcast(self, buf, nbytes, root, stream=0):
        check(_coll_lib().mx_bcast(self.h, buf, nbytes, root, stream or None), "mx_bcast")

    def reduce(self, sbuf, rbuf, count, t, op, root, alg="auto", stream=0):
        check(_coll_lib().mx_reduce(self.h, sbuf, rbuf or None, count, _slot(t), _op(op), root,
                                    _alg(REDUCE, alg), stream or None), "mx_reduce")

    def scan(self, sbuf, rbuf, count, t, op, alg="auto", stream=0):
        check(_coll_lib().mx_scan(self.h, sbuf, rbuf, count, _slot(t), _op(op), _alg(SCAN, alg),
                                  stream or None), "mx_scan")

    def exscan(self, sbuf, rbuf, count, t, op, alg="auto", stream=0):
        check(_coll_lib().mx_exscan(self.h, sbuf, rbuf, count, _slot(t), _op(op), _alg(SCAN, alg),
                                    stream or None), "mx_exscan")

    def reduce_scatter_block(self, sbuf, rbuf, rcount, t, op, alg="auto", stream=0):
        check(_coll_lib().mx_reduce_scatter_block(self.h, sbuf, rbuf, rcount, _slot(t), _op(op),
                                                  _alg(REDUCE, alg), stream or None), "mx_reduce_scatter_block")

    # -- non-blocking (persistent=True: MPI-4 *_init, started with .start()) --
    def _req(self, name, persistent, *args, keep=()):
        h = ctypes.c_void_p()
        check(getattr(_coll_lib(), name)(self.h, *args, ctypes.byref(h)), name)
        return Request(h, persistent, keep)

    def iallreduce(self, sbuf, rbuf, count, t, op, alg="auto", stream=0, persistent=False):
        return self._req("mx_allreduce_init" if persistent else "mx_iallreduce", persistent, sbuf, rbuf, count,
                         _slot(t), _op(op), _alg(IALLREDUCE, alg), stream or None)

    def ireduce(self, sbuf, rbuf, count, t, op, root, alg="auto", stream=0, persistent=False):
        return self._req("mx_reduce_init" if persistent else "mx_ireduce", persistent, sbuf, rbuf or None, count,
                         _slot(t), _op(op), root, _alg(IREDUCE, alg), stream or None)

    def iscan(self, sbuf, rbuf, count, t, op, alg="auto", stream=0, persistent=False):
        return self._req("mx_scan_init" if persistent else "mx_iscan", persistent, sbuf, rbuf, count, _slot(t),
                         _op(op), _alg(SCAN, alg), stream or None)

    def iexscan(self, sbuf, rbuf, count, t, op, alg="auto", stream=0, persistent=False):
        return self._req("mx_exscan_init" if persistent else "mx_iexscan", persistent, sbuf, rbuf, count,
                         _slot(t), _op(op), _alg(SCAN, alg), stream or None)

    def ireduce_scatter(self, sbuf, rbuf, rcounts, t, op, stream=0, persistent=False):
        rc = (ctypes.c_size_t * len(rcounts))(*rcounts)
        return self._req("mx_reduce_scatter_init" if persistent else "mx_ireduce_scatter", persistent, sbuf, rbuf,
                         rc, _slot(t), _op(op), stream or None, keep=(rc,))

    def ireduce_scatter_block(self, sbuf, rbuf, rcount, t, op, stream=0, persistent=False):
        return self._req("mx_reduce_scatter_block_init" if persistent else "mx_ireduce_scatter_block", persistent,
                         sbuf, rbuf, rcount, _slot(t), _op(op), stream or None)

    def iallgather(self, sbuf, rbuf, nbytes, stream=0, persistent=False):
        return self._req("mx_allgather_init" if persistent else "mx_iallgather", persistent, sbuf, rbuf, nbytes,
                         stream or None)

    def ibcast(self, buf, nbytes, root, stream=0, persistent=False):
        return self._req("mx_bcast_init" if persistent else "mx_ibcast", persistent, buf, nbytes, root,
                         stream or None)

    # -- point-to-point on device buffers -------------------------------------
    def send(self, buf, nbytes, dst, tag=0, stream=0):
        check(_coll_lib().mx_send(self.h, buf, nbytes, dst, tag, stream or None), "mx_send")

    def recv(self, buf, nbytes, src, tag=-1, stream=0):
        got = ctypes.c_size_t()
        check(_coll_lib().mx_recv(self.h, buf, nbytes, src, tag, stream or None, ctypes.byref(got)), "mx_recv")
        return got.value

    def sendrecv(self, sbuf, sbytes, dst, rbuf, rbytes, src, stag=0, rtag=-1, stream=0):
        got = ctypes.c_size_t()
        check(_coll_lib().mx_sendrecv(self.h, sbuf, sbytes, dst, stag, rbuf, rbytes, src, rtag, stream or None,
                                      ctypes.byref(got)), "mx_sendrecv")
        return got.value

    def isend(self, buf, nbytes, dst, tag=0, stream=0, persistent=False):
        return self._req("mx_send_init" if persistent else "mx_isend", persistent, buf, nbytes, dst, tag,
                         stream or None)

    def irecv(self, buf, nbytes, src, tag=-1, stream=0, persistent=False):
        return self._req("mx_recv_init" if persistent else "mx_irecv", persistent, buf, nbytes, src, tag,
                         stream or None)

    def isend_ddt(self, buf, count, dt, dst, tag=0, stream=0):
        return self._req("mx_isend_ddt", False, buf, count, dt.h, dst, tag, stream or None, keep=(dt,))

    def irecv_ddt(self, buf, count, dt, src, tag=-1, stream=0):
        return self._req("mx_irecv_ddt", False, buf, count, dt.h, src, tag, stream or None, keep=(dt,))

    # -- local (all ranks in this process) ---------------------------------
    def allreduce_local(self, sbufs, rbufs, count, t, op, alg="auto", stream=0):
        sp = _ptrs(sbufs) if sbufs is not None else None
        check(_coll_lib().mx_allreduce_local(self.h, sp, _ptrs(rbufs), count, _slot(t), _op(op),
                                             _alg(ALLREDUCE, alg), stream or None), "mx_allreduce_local")

    def reduce_scatter_local(self, sbufs, rbufs, rcounts, t, op, alg="auto", stream=0):
        rc = (ctypes.c_size_t * len(rcounts))(*rcounts)
        sp = _ptrs(sbufs) if sbufs is not None else None
        check(_coll_lib().mx_reduce_scatter_local(self.h, sp, _ptrs(rbufs), rc, _slot(t), _op(op),
                                                  _alg(REDUCE_SCATTER, alg), stream or None),
              "mx_reduce_scatter_local")

    def allgather_local(self, sbufs, rbufs, nbytes, stream=0):
        sp = _ptrs(sbufs) if sbufs is not None else None
        check(_coll_lib().mx_allgather_local(self.h, sp, _ptrs(rbufs), nbytes, stream or None),
              "mx_allgather_local")

    def bcast_local(self, bufs, nbytes, root, stream=0):
        check(_coll_lib().mx_bcast_local(self.h, _ptrs(bufs), nbytes, root, stream or None), "mx_bcast_local")

    def reduce_local(self, sbufs, rbufs, count, t, op, root, alg="auto", stream=0):
        sp = _ptrs(sbufs) if sbufs is not None else None
        check(_coll_lib().mx_reduce_local(self.h, sp, _ptrs(rbufs), count, _slot(t), _op(op), root,
                                          _alg(REDUCE, alg), stream or None), "mx_reduce_local")

    def _local3(self, name, table, sbufs, rbufs, count, t, op, alg, stream):
        sp = _ptrs(sbufs) if sbufs is not None else None
        check(getattr(_coll_lib(), name)(self.h, sp, _ptrs(rbufs), count, _slot(t), _op(op), _alg(table, alg),
                                         stream or None), name)

    def scan_local(self, sbufs, rbufs, count, t, op, alg="auto", stream=0):
        self._local3("mx_scan_local", SCAN, sbufs, rbufs, count, t, op, alg, stream)

    def exscan_local(self, sbufs, rbufs, count, t, op, alg="auto", stream=0):
        self._local3("mx_exscan_local", SCAN, sbufs, rbufs, count, t, op, alg, stream)

    def reduce_scatter_block_local(self, sbufs, rbufs, rcount, t, op, alg="auto", stream=0):
        self._local3("mx_reduce_scatter_block_local", REDUCE, sbufs, rbufs, rcount, t, op, alg, stream)


SHMEM_OPS = ["AND", "OR", "XOR", "MAX", "MIN", "SUM", "PROD"]
SHMEM_TYPES = ["SHORT", "INT", "LONG", "LLONG", "INT16", "INT32", "INT64", "FLOAT", "DOUBLE", "LDOUBLE",
               "FCOMPLEX", "DCOMPLEX", "FINT2", "FINT4", "FINT8", "FREAL4", "FREAL8", "FREAL16"]


def _heap_lib():
    L = _coll_lib()
    if not getattr(L, "_mx_heap_typed", False):
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.mx_heap_create.argtypes = [vp, sz, ctypes.POINTER(vp)]
        L.mx_heap_destroy.argtypes = [vp]
        L.mx_heap_base.restype = vp
        L.mx_heap_base.argtypes = [vp]
        L.mx_shmalloc.restype = vp
        L.mx_shmalloc.argtypes = [vp, sz]
        L.mx_shfree.argtypes = [vp, vp]
        L.mx_shmem_ptr.restype = vp
        L.mx_shmem_ptr.argtypes = [vp, vp, i]
        L.mx_shmem_putmem.argtypes = [vp, vp, vp, sz, i, vp]
        L.mx_shmem_getmem.argtypes = [vp, vp, vp, sz, i, vp]
        L.mx_shmem_barrier_all.argtypes = [vp, vp]
        L.mx_shmem_reduce_heap.argtypes = [vp, i, i, sz, vp, vp, sz, i, i, i, vp]
        L.mx_accumulate.argtypes = [vp, vp, sz, i, i, i, vp, vp]
        L.mx_get_accumulate.argtypes = [vp, vp, vp, sz, i, i, i, vp, vp]
        L.mx_fetch_and_op.argtypes = [vp, vp, vp, i, i, i, vp, vp]
        L.mx_compare_and_swap.argtypes = [vp, vp, vp, vp, i, i, vp, vp]
        L.mx_accumulate_ddt.argtypes = [vp, vp, sz, vp, i, i, i, vp, sz, vp, vp]
        L._mx_heap_typed = True
    return L


class Heap:
    """Device symmetric heap over a multi-process Comm (collective calls)."""

    def __init__(self, comm, nbytes):
        L = _heap_lib()
        h = ctypes.c_void_p()
        check(L.mx_heap_create(comm.h, nbytes, ctypes.byref(h)), "mx_heap_create")
        self.h, self.comm = h, comm

    def alloc(self, nbytes):
        p = _heap_lib().mx_shmalloc(self.h, nbytes)
        if not p:
            raise MxError(-4, "mx_shmalloc")
        return p

    def free(self, p):
        check(_heap_lib().mx_shfree(self.h, p), "mx_shfree")

    def ptr(self, addr, pe):
        return _heap_lib().mx_shmem_ptr(self.h, addr, pe)

    def put(self, dest, src, nbytes, pe, stream=0):
        check(_heap_lib().mx_shmem_putmem(self.h, dest, src, nbytes, pe, stream or None), "mx_shmem_putmem")

    def get(self, dest, src, nbytes, pe, stream=0):
        check(_heap_lib().mx_shmem_getmem(self.h, dest, src, nbytes, pe, stream or None), "mx_shmem_getmem")

    def barrier_all(self, stream=0):
        check(_heap_lib().mx_shmem_barrier_all(self.h, stream or None), "mx_shmem_barrier_all")

    def reduce(self, op, t, dt_size, target, source, nreduce, pe_start=0, log_pe_stride=0, pe_size=None,
               stream=0):
        """shmem_<t>_<op>_to_all on symmetric arrays (active set defaults to all PEs)."""
        pe_size = self.comm.size if pe_size is None else pe_size
        check(_heap_lib().mx_shmem_reduce_heap(self.h, SHMEM_OPS.index(op), SHMEM_TYPES.index(t), dt_size, target,
                                               source, nreduce, pe_start, log_pe_stride, pe_size, stream or None),
              "mx_shmem_reduce_heap")

    # -- one-sided accumulate (MPI_Accumulate & co. on symmetric memory) ----
    def accumulate(self, origin, count, t, op, pe, target, stream=0):
        check(_heap_lib().mx_accumulate(self.h, origin or None, count, _slot(t), _op(op), pe, target,
                                        stream or None), "mx_accumulate")

    def get_accumulate(self, origin, result, count, t, op, pe, target, stream=0):
        check(_heap_lib().mx_get_accumulate(self.h, origin or None, result, count, _slot(t), _op(op), pe, target,
                                            stream or None), "mx_get_accumulate")

    def fetch_and_op(self, origin, result, t, op, pe, target, stream=0):
        check(_heap_lib().mx_fetch_and_op(self.h, origin or None, result, _slot(t), _op(op), pe, target,
                                          stream or None), "mx_fetch_and_op")

    def compare_and_swap(self, origin, compare, result, t, pe, target, stream=0):
        check(_heap_lib().mx_compare_and_swap(self.h, origin, compare, result, _slot(t), pe, target,
                                              stream or None), "mx_compare_and_swap")

    def accumulate_ddt(self, origin, origin_count, origin_dt, t, op, pe, target, target_count, target_dt,
                       stream=0):
        """origin_dt / target_dt: Datatype or None (contiguous elements of t)."""
        check(_heap_lib().mx_accumulate_ddt(self.h, origin, origin_count, origin_dt.h if origin_dt else None,
                                            _slot(t), _op(op), pe, target, target_count,
                                            target_dt.h if target_dt else None, stream or None),
              "mx_accumulate_ddt")

    def close(self):
        if getattr(self, "h", None):
            _heap_lib().mx_heap_destroy(self.h)
            self.h = None


def allreduce_decision(n, count, t):
    return int(_coll_lib().mx_allreduce_decision(n, count, _slot(t)))


def reduce_scatter_decision(n, total, t):
    return int(_coll_lib().mx_reduce_scatter_decision(n, total, _slot(t)))


def reduce_decision(n, count, t):
    return int(_coll_lib().mx_reduce_decision(n, count, _slot(t)))


# ---------------------------------------------------------------------------
# device convertor (include/mx_convertor.h)
# ---------------------------------------------------------------------------
def _ddt_lib():
    L = lib()
    if not getattr(L, "_mx_ddt_typed", False):
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.mx_ddt_create.argtypes = [vp, sz, vp, sz, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(vp)]
        L.mx_ddt_destroy.argtypes = [vp]
        L.mx_ddt_size.restype = sz
        L.mx_ddt_size.argtypes = [vp]
        L.mx_ddt_extent.restype = ctypes.c_int64
        L.mx_ddt_extent.argtypes = [vp]
        L.mx_ddt_runs.restype = sz
        L.mx_ddt_runs.argtypes = [vp]
        L.mx_pack.argtypes = [vp, sz, vp, vp, sz, sz, vp]
        L.mx_unpack.argtypes = [vp, sz, vp, vp, sz, sz, vp]
        L.mx_ddt_set_path.argtypes = [vp, ctypes.c_int]
        L.mx_ddt_last_path.argtypes = [vp]
        L._mx_ddt_typed = True
    return L


class Datatype:
    """A committed derived datatype on the device, built from the
    reference's committed description records (opt_desc)."""

    def __init__(self, desc: bytes, nrec: int, size: int, lb: int, ub: int, basic_sizes=None):
        L = _ddt_lib()
        h = ctypes.c_void_p()
        self._desc = ctypes.create_string_buffer(bytes(desc), len(desc))
        bs = None
        if basic_sizes is not None:
            self._bs = (ctypes.c_uint64 * len(basic_sizes))(*[int(x) for x in basic_sizes])
            bs = ctypes.cast(self._bs, ctypes.c_void_p)
        check(L.mx_ddt_create(ctypes.cast(self._desc, ctypes.c_void_p), nrec, bs, size, lb, ub, ctypes.byref(h)),
              "mx_ddt_create")
        self.h = h
        self.size, self.lb, self.ub = size, lb, ub

    @property
    def extent(self):
        return self.ub - self.lb

    @property
    def runs(self):
        return int(_ddt_lib().mx_ddt_runs(self.h))

    # kernel families (include/mx_convertor.h, mx_ddt_last_path)
    PATHS = {0: None, 1: "copy", 2: "vector", 3: "granule", 4: "bytemap", 5: "piece", 6: "block", 7: "tile"}

    def set_path(self, path):
        """'auto' or 'block' (mx_ddt_set_path)."""
        check(_ddt_lib().mx_ddt_set_path(self.h, {"auto": 0, "block": 1}[path]), "mx_ddt_set_path")

    @property
    def last_path(self):
        """Kernel family of the last pack / unpack (mx_ddt_last_path)."""
        return self.PATHS[int(_ddt_lib().mx_ddt_last_path(self.h))]

    def pack(self, count, user, packed, offset=0, length=None, stream=0):
        length = self.size * count - offset if length is None else length
        check(_ddt_lib().mx_pack(self.h, count, user, packed, offset, length, stream or None), "mx_pack")

    def unpack(self, count, user, packed, offset=0, length=None, stream=0):
        length = self.size * count - offset if length is None else length
        check(_ddt_lib().mx_unpack(self.h, count, user, packed, offset, length, stream or None), "mx_unpack")

    def close(self):
        if getattr(self, "h", None):
            _ddt_lib().mx_ddt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
