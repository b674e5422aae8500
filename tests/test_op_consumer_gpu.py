"""op/mi355x's completion contract, read from another process (round 4).

`ompi_op_reduce` on device buffers must leave `inout` complete on return
(ompi/mca/op/op.h:258-273): coll/base's recursive doubling hands the result
of one step straight to the next step's sendrecv (coll_base_allreduce.c:
218-236), and on device buffers the peer's transport reads it through an IPC
mapping.  Here 8 processes run that algorithm with the mini-host's op table
(op/mi355x's handler -> mx_reduce2_sync) on hipMalloc'ed device buffers, and
the "sendrecv" is the peer copying this rank's buffer through its IPC
mapping with a kernel on its own stream, started within microseconds of
this rank's handler returning (a shared-memory flag, no GPU sync between).
Nothing orders the peer's copy after the reduce kernel except the handler's
return -- so a result published early (a completion word raised before the
stores are visible to another agent) shows up as a wrong part.

Every completion path: the resident service (calls <= 128 KiB on the
handler's stream), the launch marking itself (every workgroup writes its
own flag after its system-scope release; MX_OP_SERVICE=0) and the marker
kernel (MX_OP_SERVICE=0 MX_FUSED_MARK=0).  Every rank's result bit-exact vs the recursive-doubling oracle
(mxo_allreduce alg 3, coll_base_allreduce.c:130-274) -- 32 allreduces of
4 KiB - 1 MiB with fresh inputs each.
"""
import ctypes
import os
import socket
import time

import numpy as np
import pytest

import golden_io
import mxompi
import oracle_lib

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

vp, ci, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
N = 8
STEPS = 3                                        # log2(N)
SIZES = [1000, 16384, 65536, 262144, 300000]     # floats: 4 KiB (1 wg) .. 1 MiB (256 wgs) .. 1.14 MiB (marker)
ITERS = 8


class _IpcHandle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_ubyte * 64)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gen(count, seed):
    rng = np.random.default_rng(seed)
    return (rng.uniform(-1, 1, count) * 10.0 ** rng.uniform(-7, 7, count)).astype(np.float32)


def _spin(arr, idx, timeout=60.0):
    t0 = time.monotonic()
    while arr[idx] == 0:
        if time.monotonic() - t0 > timeout:
            raise TimeoutError(f"flag {idx}")
    return arr[idx]


def _worker(rank, port, env, flags, q):
    try:
        os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
        os.environ.update(env)
        import torch.distributed as dist
        import minihost
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=N)
        torch.cuda.set_device(0)
        mxompi.init(0)
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
        hip.hipFree.argtypes = [vp]
        hip.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(_IpcHandle), vp]
        hip.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(vp), _IpcHandle, ctypes.c_uint]
        hip.hipIpcCloseMemHandle.argtypes = [vp]
        hip.hipMemcpy.argtypes = [vp, vp, sz, ci]
        H = minihost.host(with_components=True)
        f32, SUM = minihost.dtype(H, "MPI_FLOAT"), minihost.op(H, "MPI_SUM")
        assert H.mxh_op_slot_owner(SUM, mxompi.TYPE["FLOAT"], 0) == 1, "op/mi355x does not own MPI_SUM/FLOAT"
        nb_max = max(SIZES) * 4
        bufs, handles = [], []
        for _ in range(2):
            p = vp()
            assert hip.hipMalloc(ctypes.byref(p), nb_max) == 0
            h = _IpcHandle()
            assert hip.hipIpcGetMemHandle(ctypes.byref(h), p) == 0
            bufs.append(p.value)
            handles.append(bytes(bytearray(h.reserved)))
        allh = [None] * N
        dist.all_gather_object(allh, handles)
        peer = {}
        for p in range(N):
            if p == rank:
                continue
            for b in range(2):
                m = vp()
                h = _IpcHandle()
                h.reserved[:] = allh[p][b]
                assert hip.hipIpcOpenMemHandle(ctypes.byref(m), h, 1) == 0
                peer[(p, b)] = m.value
        dist.barrier()
        out = []
        sid = 0
        for count in SIZES:
            nb = count * 4
            for it in range(ITERS):
                x = _gen(count, 1000 * count + 10 * it + rank)
                assert hip.hipMemcpy(bufs[0], x.ctypes.data, nb, 1) == 0     # H2D (synchronous)
                tsend, trecv = 0, 1
                for k in range(STEPS):
                    remote = rank ^ (1 << k)
                    flags[(rank * 2) * 4096 + sid] = tsend + 1                # my tmpsend is complete
                    pb = _spin(flags, (remote * 2) * 4096 + sid) - 1
                    mxompi.lib().mx_copy(bufs[trecv], peer[(remote, pb)], nb, None)   # the peer's "send"
                    mxompi.sync(0)
                    flags[(rank * 2 + 1) * 4096 + sid] = 1                    # done reading the peer's buffer
                    _spin(flags, (remote * 2 + 1) * 4096 + sid)               # the peer is done reading mine
                    if rank < remote:      # tmprecv = tmpsend (op) tmprecv
                        assert H.mxh_op_reduce(SUM, bufs[tsend], bufs[trecv], count, f32) == 0
                        tsend, trecv = trecv, tsend
                    else:                  # tmpsend = tmprecv (op) tmpsend
                        assert H.mxh_op_reduce(SUM, bufs[trecv], bufs[tsend], count, f32) == 0
                    sid += 1
                res = np.empty(count, np.float32)
                assert hip.hipMemcpy(res.ctypes.data, bufs[tsend], nb, 2) == 0  # D2H
                out.append(res.tobytes())
        dist.barrier()
        for m in peer.values():
            hip.hipIpcCloseMemHandle(m)
        for b in bufs:
            hip.hipFree(b)
        dist.destroy_process_group()
        q.put((rank, "ok", out))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))


@pytest.mark.parametrize("env", [{"MX_OP_SERVICE": "1"}, {"MX_OP_SERVICE": "0", "MX_FUSED_MARK": "1"},
                                 {"MX_OP_SERVICE": "0", "MX_FUSED_MARK": "0"}],
                         ids=["service", "fused_mark", "marker_kernel"])
def test_op_reduce_result_read_by_peer_process_recursive_doubling(env):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    flags = ctx.Array("q", N * 2 * 4096, lock=False)
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, env, flags, q)) for r in range(N)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(N):
            rank, status, payload = q.get(timeout=300)
            assert status == "ok", payload
            got[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=60 if len(got) == N else 5)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    L = oracle_lib.oracle()
    L.mxo_allreduce.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    j = 0
    for count in SIZES:
        for it in range(ITERS):
            xs = [_gen(count, 1000 * count + 10 * it + r) for r in range(N)]
            exp = [np.zeros(count, np.float32) for _ in range(N)]
            assert L.mxo_allreduce(3, mxompi.OP["SUM"], mxompi.TYPE["FLOAT"], N, count,
                                   (vp * N)(*[x.ctypes.data for x in xs]),
                                   (vp * N)(*[e.ctypes.data for e in exp])) == 0
            for r in range(N):
                golden_io.assert_coll_equal(np.frombuffer(got[r][j], np.uint8), exp[r].view(np.uint8),
                                            mxompi.OP["SUM"], mxompi.TYPE["FLOAT"],
                                            f"{env} count {count} iter {it} rank {r}")
            j += 1
