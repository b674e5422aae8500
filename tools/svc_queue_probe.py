"""Diagnostic (not product): which hardware-queue pool the op service's
stream lands in.  Holds every ordinary and every high-priority queue with
spinning waves (8 streams each), then makes 20 service calls: a service
with a queue of its own serves them all; one sharing a held queue is held
(and its calls launch -- on a held queue too, so they wait for the holders'
5 s timeout).  usage: MX_SVC_PRIORITY=least|normal|greatest python tools/svc_queue_probe.py"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))
import torch  # noqa: E402
import mxompi  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
lo, hi = ctypes.c_int(), ctypes.c_int()
hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi))
print(f"priority range: least {lo.value} greatest {hi.value}; MX_SVC_PRIORITY={os.environ.get('MX_SVC_PRIORITY')}")
mxompi.init(0)
L = mxompi.lib()
n = 1000
a = torch.ones(n, dtype=torch.int64, device="cuda")
b = torch.zeros(n, dtype=torch.int64, device="cuda")
sp = ctypes.c_void_p()
mxompi.check(L.mx_stream_create(ctypes.byref(sp)), "mx_stream_create")
torch.cuda.synchronize()
mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), n, sp.value)   # service set up
time.sleep(0.01)
normal = [torch.cuda.Stream() for _ in range(8)]
high = []
for _ in range(8):
    p = ctypes.c_void_p()
    mxompi.check(L.mx_stream_create(ctypes.byref(p)), "mx_stream_create")
    high.append(p)
for st in normal:
    mxompi.debug_hold(st.cuda_stream, 5000)
for p in high:
    mxompi.debug_hold(p.value, 5000)
h0 = mxompi.op_service_held()[1]
s0 = mxompi.op_service_stats()[1]
t0 = time.time()
for _ in range(20):
    mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), n, sp.value)
dt = time.time() - t0
print(f"20 calls with every ordinary and high-priority queue held: {dt * 1e3:.1f} ms, "
      f"served {mxompi.op_service_stats()[1] - s0}, launches held {mxompi.op_service_held()[1] - h0}", flush=True)
mxompi.debug_release()
torch.cuda.synchronize()
print("b ok" if torch.all(b == 21).item() else f"b wrong {b[:4]}")
