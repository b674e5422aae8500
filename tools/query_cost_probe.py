"""Diagnostic (not product): the host cost of hipStreamQuery on an idle
stream (legacy null stream and a non-blocking stream), of hipEventRecord +
hipStreamWaitEvent, measured in a C-speed loop via ctypes batches."""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
torch.cuda.init()
torch.zeros(1, device="cuda")
torch.cuda.synchronize()
s = ctypes.c_void_p()
hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)
s2 = ctypes.c_void_p()
hip.hipStreamCreateWithFlags(ctypes.byref(s2), 1)
ev = ctypes.c_void_p()
hip.hipEventCreateWithFlags(ctypes.byref(ev), 2)
N = 20000
for name, fn in [("query null", lambda: hip.hipStreamQuery(None)),
                 ("query nonblocking", lambda: hip.hipStreamQuery(s)),
                 ("ctypes no-op (hipGetLastError)", lambda: hip.hipGetLastError()),
                 ("record+wait", lambda: (hip.hipEventRecord(ev, s), hip.hipStreamWaitEvent(s2, ev, 0)))]:
    for _ in range(100):
        fn()
    t0 = time.perf_counter()
    for _ in range(N):
        fn()
    dt = (time.perf_counter() - t0) / N * 1e6
    print(f"{name:32s} {dt:6.2f} us per call (incl. ~0.1-0.3 us ctypes)", flush=True)
hip.hipStreamSynchronize(s2)

# a stream whose kernel is still running (a spinning wave, released after)
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zhpe-ompi_amd"))
import mxompi  # noqa: E402
mxompi.init(0)
mxompi.debug_hold(s.value, 3000)
time.sleep(0.01)
for name, fn in [("query busy nonblocking", lambda: hip.hipStreamQuery(s)),
                 ("query null while another busy", lambda: hip.hipStreamQuery(None))]:
    t0 = time.perf_counter()
    for _ in range(2000):
        fn()
    print(f"{name:32s} {(time.perf_counter() - t0) / 2000 * 1e6:6.2f} us per call", flush=True)
mxompi.debug_release()
hip.hipStreamSynchronize(s)
