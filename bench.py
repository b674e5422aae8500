#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X collective-reduction path.

Metric (BASELINE.json): "MPI_Allreduce busBW GB/s (256 MiB fp32 SUM,
1/2/4/8 GPU); Reduce_local HBM GB/s".

* N = 1 (one process): the workload is BASELINE configs[1],
  MPI_Reduce_local on 1 GiB device buffers, fp32 SUM (the K1 kernel behind
  the op component's 2-buffer slot).  One step = one mx_reduce2 over the
  whole 1 GiB batch.  value = HBM GB/s with 3*N*4 algorithmic bytes
  (read in, read inout, write inout) per step.
* N > 1 (torchrun, one rank per GPU): the workload is configs[3]'s
  headline point, MPI_Allreduce of 256 MiB fp32 SUM per rank through the
  coll component's allreduce (all-peer xGMI reduce-scatter + allgather),
  value = busBW = (S / t) * 2(n-1)/n, t = max over ranks.  If the
  collective library is not available the N>1 run reports independent
  Reduce_local replicas instead and says so in config.workload.

The JSON line also carries `roofline` (the dominant kernel's achieved
bytes/launch / its HIP-event-timed average duration vs the 8 TB/s HBM
peak) and `cpu_baseline` (the reference's own op_base_functions.c compiled
from source -- oracle/_ref -- or our C restatement, timed on the host on a
bounded sample).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 153.0       # per xGMI link
METRIC = "MPI_Allreduce busBW GB/s (256 MiB fp32 SUM, 1/2/4/8 GPU); Reduce_local HBM GB/s"


def _env_int(k, d):
    try:
        return int(os.environ.get(k, d))
    except ValueError:
        return d


def load_traffic(kernel_key):
    """Per-launch HBM bytes for `kernel_key` from the committed PMC summary
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE
    doubled per the gfx950 correction).  None if absent."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(kernel_key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline_reduce_local(seconds=10.0):
    """Time the reference's own 2-buffer fp32 SUM (op_base_functions.c:312,
    compiled from source into oracle/_ref/libref_op.so) on one host core,
    on a bounded sample: 2 x 256 MiB host buffers, repeated ~`seconds`."""
    import numpy as np
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_op.so")
    n = 1 << 26
    a = np.random.default_rng(1).uniform(-1, 1, n).astype(np.float32)
    b = np.random.default_rng(2).uniform(-1, 1, n).astype(np.float32)
    if os.path.exists(ref):
        L = ctypes.CDLL(ref)
        tab = (ctypes.c_void_p * (15 * 41)).in_dll(L, "ompi_op_base_functions")
        FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.POINTER(ctypes.c_int), ctypes.c_void_p, ctypes.c_void_p)
        fn = FN(tab[3 * 41 + 15])          # [MPI_SUM][OMPI_OP_BASE_TYPE_FLOAT]
        cnt = ctypes.c_int(n)
        call = lambda: fn(a.ctypes.data, b.ctypes.data, ctypes.byref(cnt), None, None)
        kind = "reference"
    else:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        O = oracle_lib.oracle()
        call = lambda: O.mxo_reduce2(3, 15, a.ctypes.data, b.ctypes.data, n, 1)
        kind = "port"
    call()
    iters, t0 = 0, time.perf_counter()
    while True:
        call()
        iters += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    gbs = 3.0 * n * 4 * iters / el / 1e9
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": 1, "kind": kind,
            "sample": f"fp32 SUM 2-buffer, 2 x 256 MiB host buffers, {iters} calls in {el:.1f} s "
                      f"(1 pinned host thread; algorithmic 3*N*4 B per call)"}


def bench_reduce_local(torch, mx, steps, warmup, nbytes=1 << 30):
    n = nbytes // 4
    g = torch.Generator(device="cuda").manual_seed(0x5EEDC0DE)
    a = torch.rand(n, device="cuda", generator=g) * 2 - 1
    b0 = torch.rand(n, device="cuda", generator=g) * 2 - 1
    b = b0.clone()
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    for _ in range(warmup):
        mx.reduce2("SUM", "FLOAT", a.data_ptr(), b.data_ptr(), n, sp)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    t0 = time.perf_counter()
    for s, e in evs:
        s.record(stream)
        mx.reduce2("SUM", "FLOAT", a.data_ptr(), b.data_ptr(), n, sp)
        e.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kms = [s.elapsed_time(e) for s, e in evs]
    return wall, kms, 3.0 * n * 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import mxompi as mx

    world = _env_int("WORLD_SIZE", 1)
    rank = _env_int("RANK", 0)
    local_rank = _env_int("LOCAL_RANK", 0)
    torch.cuda.set_device(local_rank)
    mx.init(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    result = {"metric": METRIC, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
              "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
              "dtype": "f32", "data": "synthetic"}

    barrier()
    wall, kms, algo_bytes = bench_reduce_local(torch, mx, args.steps, args.warmup)
    barrier()
    t_max = wall
    if dist is not None:
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_max = float(t[0])
    ms_step = t_max / args.steps * 1e3
    value = algo_bytes * world / (t_max / args.steps) / 1e9
    avg_kernel_ms = sum(kms) / len(kms)
    achieved = algo_bytes / (avg_kernel_ms * 1e-3) / 1e9
    result.update({
        "value": round(value, 2), "unit": "GB/s", "ms_per_step": round(ms_step, 4),
        "config": {"workload": "MPI_Reduce_local fp32 SUM, 1 GiB device buffers"
                               + ("" if world == 1 else f" x {world} independent replicas"),
                   "count": algo_bytes // 12, "bytes_per_buffer": algo_bytes // 3,
                   "parallelism": "replicas" if world > 1 else "single-gpu"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": load_traffic("k_reduce2<float,OpSum>"),
                     "kernel": "k_reduce2<float, mx::OpSum>",
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "avg_kernel_ms": round(avg_kernel_ms, 4)},
    })
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_reduce_local(args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
