"""Which hipMalloc'ed buffers can a peer process open through IPC? (probe)"""
import ctypes
import sys
import torch
import torch.multiprocessing as mp

vp, sz = ctypes.c_void_p, ctypes.c_size_t


class H(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_ubyte * 64)]


def hip():
    h = ctypes.CDLL("libamdhip64.so")
    h.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
    h.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
    h.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(H), vp]
    h.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(vp), H, ctypes.c_uint]
    return h


def child(q, handles):
    torch.cuda.set_device(0)
    h = hip()
    out = []
    for name, hb in handles:
        x = H()
        x.reserved[:] = hb
        m = vp()
        rc = h.hipIpcOpenMemHandle(ctypes.byref(m), x, 1)
        out.append((name, rc, m.value))
    q.put(out)


if __name__ == "__main__":
    torch.cuda.set_device(0)
    h = hip()
    handles = []
    for name, nb, ext in [("malloc_1M", 1 << 20, None), ("malloc_4M", 4 << 20, None), ("malloc_64M", 64 << 20, None),
                          ("ext_default_1M", 1 << 20, 0), ("ext_uncached_1M", 1 << 20, 3)]:
        p = vp()
        rc = h.hipMalloc(ctypes.byref(p), nb) if ext is None else h.hipExtMallocWithFlags(ctypes.byref(p), nb, ext)
        x = H()
        rc2 = h.hipIpcGetMemHandle(ctypes.byref(x), p)
        print(name, "alloc", rc, "export", rc2, hex(p.value or 0))
        handles.append((name, bytes(bytearray(x.reserved))))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=child, args=(q, handles))
    pr.start()
    print(q.get(timeout=120))
    pr.join()
