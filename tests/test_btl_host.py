"""The BTL extension leaves host memory to the BTL it is installed on
(ADVICE r5): mca_btl_mi355x_install keeps the module's original get / put /
register_mem / deregister_mem / flush and handle size; a host range is
registered by the original, its handle bytes travel tagged inside the
extension's handle, and get / put / deregister on it reach the original slots
with the original's own handle bytes -- vader's CMA / xpmem single copy
(btl_sm_component.c:487, btl_sm_xpmem.c:70) stays in charge of host memory.
The mini-host's stand-in BTL has such host slots (memcpy within a process)
and counts the calls that reach them.  No GPU needed: host memory only."""
import ctypes

import numpy as np

import minihost

vp, sz, ci, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64


def _host():
    H = minihost.host(with_components=True)
    H.mxh_btl_init.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(sz)]
    H.mxh_btl_register.argtypes = [vp, sz, vp, ctypes.POINTER(vp)]
    H.mxh_btl_deregister.argtypes = [vp]
    H.mxh_btl_rdma.argtypes = [ci, vp, u64, vp, sz, ci]
    H.mxh_btl_flush_gets.argtypes = [vp, u64, vp, sz, ci]
    H.mxh_btl_host_calls.argtypes = []
    return H


def test_host_rget_and_put_reach_the_original_slots():
    H = _host()
    flags, hb = ctypes.c_uint32(), sz()
    assert H.mxh_btl_init(ctypes.byref(flags), ctypes.byref(hb)) == 0
    assert flags.value & 0x0004 and flags.value & 0x0800          # GET | CUDA_GET
    assert hb.value >= 8 + 32                                       # tag + the original's 32 bytes
    rng = np.random.default_rng(4)
    own = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    hbuf = ctypes.create_string_buffer(hb.value)
    reg = vp()
    c0 = H.mxh_btl_host_calls()
    assert H.mxh_btl_register(own.ctypes.data, own.size, hbuf, ctypes.byref(reg)) == 0
    assert H.mxh_btl_host_calls() == c0 + 1                         # the original registered it
    # RGET of the owner's host buffer (ob1: the receiver's btl_get with the
    # handle bytes from the RGET header), three in flight
    dst = np.zeros(4099, dtype=np.uint8)
    c1 = H.mxh_btl_host_calls()
    peer = ctypes.create_string_buffer(hbuf.raw, hb.value)
    assert H.mxh_btl_rdma(1, dst.ctypes.data, own.ctypes.data + 1237, peer, 4099, 3) == 0
    assert np.array_equal(dst, own[1237:1237 + 4099])
    # local register + 3 gets + local deregister, all in the original
    assert H.mxh_btl_host_calls() == c1 + 5
    # PUT into the owner's buffer at an odd offset; flush queues nothing of ours
    src = rng.integers(0, 256, 777, dtype=np.uint8)
    assert H.mxh_btl_rdma(0, src.ctypes.data, own.ctypes.data + 3, peer, 777, 1) == 0
    assert np.array_equal(own[3:780], src)
    dst2 = np.zeros(4 * 512, dtype=np.uint8)
    assert H.mxh_btl_flush_gets(dst2.ctypes.data, own.ctypes.data, peer, 512, 4) == 0
    assert np.array_equal(dst2, own[:2048])
    c2 = H.mxh_btl_host_calls()
    assert H.mxh_btl_deregister(reg) == 0
    assert H.mxh_btl_host_calls() == c2 + 1                         # the original deregistered it
