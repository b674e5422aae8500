"""GPU RDMA through the BTL module interface (mca/btl_mi355x.c; VERDICT r4
missing 3): the btl_get / btl_put / btl_register_mem / btl_deregister_mem /
btl_flush slots of mca_btl_base_module_t (opal/mca/btl/btl.h:1189-1261) on
device buffers, installed on a host shared-memory BTL module the way
btl/smcuda's component installs mca_btl_smcuda_get_cuda
(btl_smcuda_component.c:936).

Two processes on the box's GPU.  The mini-host restates ob1's RGET and PUT
steps: the owner registers its device buffer and ships the handle bytes
(btl_registration_handle_size of them, the PML header's payload); the peer
calls the slot with them and drives progress until the completion callback.
Payload-exact at 0 B, 1 B, an odd size at an odd offset inside the
allocation, 64 MiB, several operations in flight before any progress, a
flush; an allocation freed and re-made by the owner (a new runtime buffer id
at possibly the same address) is read fresh, never through the stale
mapping; a process's own registration works too.
"""
import ctypes
import os
import socket

import numpy as np
import pytest

import minihost
import mxompi

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

vp, sz, ci, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _host():
    H = minihost.host(with_components=True)
    H.mxh_btl_init.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(sz)]
    H.mxh_btl_register.argtypes = [vp, sz, vp, ctypes.POINTER(vp)]
    H.mxh_btl_deregister.argtypes = [vp]
    H.mxh_btl_rdma.argtypes = [ci, vp, u64, vp, sz, ci]
    H.mxh_btl_flush_gets.argtypes = [vp, u64, vp, sz, ci]
    return H


def _data(seed, n):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


def _worker(rank, port, q):
    import torch.distributed as dist
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
        torch.cuda.set_device(0)
        mxompi.init(0)
        H = _host()
        flags, hb = ctypes.c_uint32(), sz()
        assert H.mxh_btl_init(ctypes.byref(flags), ctypes.byref(hb)) == 0
        res = {"flags": flags.value, "handle_bytes": hb.value}

        def exchange(obj):
            out = [None, None]
            dist.all_gather_object(out, obj)
            return out[1 - rank]

        def register(t):
            hbuf = ctypes.create_string_buffer(hb.value)
            reg = vp()
            assert H.mxh_btl_register(t.data_ptr(), t.numel(), hbuf, ctypes.byref(reg)) == 0
            return hbuf.raw, reg

        L = mxompi.lib()
        big = 64 << 20
        # --- RGET: rank 1 owns, rank 0 gets -------------------------------
        own = torch.from_numpy(_data(10 + rank, big)).cuda()
        torch.cuda.synchronize()
        handle, reg = register(own)
        peer_handle, peer_addr = exchange((handle, own.data_ptr()))
        got = {}
        if rank == 0:
            for nbytes, off in ((0, 0), (1, 0), (4099, 1237), (big, 0)):
                dst = torch.zeros(max(nbytes, 1), dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                hbuf = ctypes.create_string_buffer(peer_handle, len(peer_handle))
                rc = H.mxh_btl_rdma(1, dst.data_ptr(), peer_addr + off, hbuf, nbytes, 3)
                assert rc == 0, (nbytes, rc)
                got[f"get{nbytes}"] = dst[:nbytes].cpu().numpy().tobytes()
            # a flush completes gets queued with no progress call
            dst = torch.zeros(8 * 4096, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            hbuf = ctypes.create_string_buffer(peer_handle, len(peer_handle))
            assert H.mxh_btl_flush_gets(dst.data_ptr(), peer_addr, hbuf, 4096, 8) == 0
            got["flush"] = dst.cpu().numpy().tobytes()
            # this process's own registration (the PML's self path)
            mine = torch.zeros(4099, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            hself = ctypes.create_string_buffer(handle, len(handle))
            assert H.mxh_btl_rdma(1, mine.data_ptr(), own.data_ptr() + 77, hself, 4099, 1) == 0
            got["self"] = mine.cpu().numpy().tobytes()
        dist.barrier()
        # --- PUT: rank 0 writes into rank 1's buffer at an odd offset -------
        if rank == 0:
            src = torch.from_numpy(_data(50, 1 << 20)).cuda()
            torch.cuda.synchronize()
            hbuf = ctypes.create_string_buffer(peer_handle, len(peer_handle))
            assert H.mxh_btl_rdma(0, src.data_ptr(), peer_addr + 3, hbuf, 1 << 20, 1) == 0
        dist.barrier()                            # ob1's FIN: the owner reads after it
        if rank == 1:
            torch.cuda.synchronize()
            got["put"] = own[3:3 + (1 << 20)].cpu().numpy().tobytes()
            got["put_edges"] = (int(own[2].item()), int(own[3 + (1 << 20)].item()))
        H.mxh_btl_deregister(reg)
        # --- an allocation freed and re-made by the owner ---------------------
        for cycle in range(3):
            p = vp()
            if rank == 1:
                assert L.mx_alloc(sz(1 << 20), ctypes.byref(p)) == 0
                data = _data(100 + cycle, 1 << 20)
                assert L.mx_memcpy(p, vp(data.ctypes.data), sz(1 << 20), None) == 0
                torch.cuda.synchronize()
                hbuf = ctypes.create_string_buffer(hb.value)
                r2 = vp()
                # refused for an allocation re-made at an address exported
                # before: ob1 then moves the message by copy
                rc = H.mxh_btl_register(p, 1 << 20, hbuf, ctypes.byref(r2))
                exchange((rc, hbuf.raw, p.value))
                dist.barrier()                    # the peer has read it
                if rc == 0:
                    H.mxh_btl_deregister(r2)
                assert L.mx_free(p) == 0
            else:
                rc, ph, pa = exchange(None)
                got[f"remade{cycle}_rc"] = rc
                if rc == 0:
                    dst = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
                    torch.cuda.synchronize()
                    hbuf = ctypes.create_string_buffer(ph, len(ph))
                    assert H.mxh_btl_rdma(1, dst.data_ptr(), pa, hbuf, 1 << 20, 1) == 0
                    got[f"remade{cycle}"] = dst.cpu().numpy().tobytes()
                got[f"remade{cycle}_addr"] = pa
                dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok", {**res, **got}))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))


def test_btl_rdma_get_put_between_processes():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(2):
            rank, status, payload = q.get(timeout=240)
            assert status == "ok", payload
            out[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=60 if len(out) == 2 else 5)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    big = 64 << 20
    owner = _data(11, big)                       # rank 1's buffer
    r0, r1 = out[0], out[1]
    assert r0["flags"] & 0x0004 and r0["flags"] & 0x0800      # MCA_BTL_FLAGS_GET | CUDA_GET
    assert r0["flags"] & 0x0002 and r0["flags"] & 0x0400      # PUT | CUDA_PUT
    assert r0["handle_bytes"] >= 64
    for nbytes, off in ((0, 0), (1, 0), (4099, 1237), (big, 0)):
        assert r0[f"get{nbytes}"] == owner[off:off + nbytes].tobytes(), nbytes
    assert r0["flush"] == owner[:8 * 4096].tobytes()
    assert r0["self"] == _data(10, big)[77:77 + 4099].tobytes()
    assert r1["put"] == _data(50, 1 << 20).tobytes()
    assert r1["put_edges"] == (int(owner[2]), int(owner[3 + (1 << 20)]))
    for cycle in range(3):
        if r0[f"remade{cycle}_rc"] == 0:       # registered: the get reads the new allocation's bytes
            assert r0[f"remade{cycle}"] == _data(100 + cycle, 1 << 20).tobytes(), cycle
        else:                                    # refused only for a re-made allocation
            assert cycle > 0, cycle
