#!/usr/bin/env python3
"""Cost of one ompi_op_reduce call through op/mi355x (the coll/base segmented
ring calls it once per 1 MiB segment, coll_base_allreduce.c:782), measured
through the mini-host's op table on device buffers, fp32 SUM, at 4 KiB
to 4 MiB.  One process per configuration (the pointer-cache switch
is read once per process):

  round1   MX_PTR_CACHE=0, op_mi355x_stream=0: hipPointerGetAttributes x2 per
           call, launch + synchronise on the legacy default stream
  cache    pointer-range cache, legacy default stream
  stream   pointer-range cache, the calling thread's own stream, hipStreamSynchronize
  marker   as stream, completion through a marker kernel's mapped word
           (MX_FUSED_MARK=0; the round-2 default)
  fastsync as stream, the reduce kernel's last workgroup raises the word
           itself (MX_FUSED_MARK=1, MX_OP_SERVICE=0)
  service  the resident reduce service (MX_OP_SERVICE=1, round 4's
           default): no launch per call

Prints one JSON line per configuration and size: avg us per call and the
kernel-only time (HIP events around 200 mx_reduce2 launches) for reference.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = {"round1": {"MX_PTR_CACHE": "0", "OMPI_MCA_op_mi355x_stream": "0"},
           "cache": {"MX_PTR_CACHE": "1", "OMPI_MCA_op_mi355x_stream": "0"},
           "stream": {"MX_PTR_CACHE": "1", "OMPI_MCA_op_mi355x_stream": "1", "OMPI_MCA_op_mi355x_fast_sync": "0"},
           "marker": {"MX_PTR_CACHE": "1", "OMPI_MCA_op_mi355x_stream": "1", "OMPI_MCA_op_mi355x_fast_sync": "1",
                      "MX_FUSED_MARK": "0", "MX_OP_SERVICE": "0"},
           "fastsync": {"MX_PTR_CACHE": "1", "OMPI_MCA_op_mi355x_stream": "1", "OMPI_MCA_op_mi355x_fast_sync": "1",
                        "MX_FUSED_MARK": "1", "MX_OP_SERVICE": "0"},
           "service": {"MX_PTR_CACHE": "1", "OMPI_MCA_op_mi355x_stream": "1", "OMPI_MCA_op_mi355x_fast_sync": "1",
                       "MX_FUSED_MARK": "1", "MX_OP_SERVICE": "1"}}
SIZES = [4 << 10, 16 << 10, 64 << 10, 128 << 10, 256 << 10, 1 << 20, 2 << 20, 4 << 20]


def child(cfg):
    sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes
    import torch
    import minihost
    import mxompi
    torch.cuda.set_device(0)
    mxompi.init(0)
    H = minihost.host(with_components=True)
    H.mxh_time_op_reduce.restype = ctypes.c_double
    H.mxh_time_op_reduce.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    f32, SUM = minihost.dtype(H, "MPI_FLOAT"), minihost.op(H, "MPI_SUM")
    assert H.mxh_op_slot_owner(SUM, mxompi.TYPE["FLOAT"], 0) == 1, "op/mi355x does not own MPI_SUM/FLOAT"
    for nbytes in SIZES:
        n = nbytes // 4
        a = torch.rand(n, device="cuda")
        b = torch.rand(n, device="cuda")
        torch.cuda.synchronize()
        iters = 2000 if nbytes <= (64 << 10) else 500
        ns = H.mxh_time_op_reduce(SUM, a.data_ptr(), b.data_ptr(), n, f32, iters)
        # kernel-only: back-to-back launches on one stream, HIP events
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(200):
            mxompi.reduce2("SUM", "FLOAT", a.data_ptr(), b.data_ptr(), n, s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        print(json.dumps({"config": cfg, "bytes": nbytes, "us_per_call": round(ns / 1e3, 2),
                          "kernel_us": round(e0.elapsed_time(e1) * 1e3 / 200, 2)}), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    order = sys.argv[1:] or list(CONFIGS)     # e.g. `marker fastsync marker fastsync` (interleaved A/B)
    for cfg in order:
        e = dict(os.environ, **CONFIGS[cfg])
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", cfg], env=e, timeout=300)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
