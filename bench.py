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
peak) and `cpu_baseline` (the CPU oracle's restatement of the reference's
fp32 SUM loop, timed on one host core on a bounded sample).
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


def _oracle_bench():
    """The CPU oracle built with the reference's default optimisation flags
    (oracle/Makefile build/libmx_oracle_bench.so: -O3 -finline-functions
    -fno-strict-aliasing, config/opal_setup_cc.m4:351-365, 481-493)."""
    import subprocess
    path = os.path.join(ROOT, "oracle", "build", "libmx_oracle_bench.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "build/libmx_oracle_bench.so"], check=True)
    L = ctypes.CDLL(path)
    vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L.mxo_reduce2.argtypes = [i, i, vp, vp, sz, i]
    L.mxo_ddt_convert.argtypes = [vp, sz, vp, ctypes.c_int64, ctypes.c_int64, sz, vp, vp, ctypes.c_int]
    return L


def cpu_baseline_reduce_local(seconds=10.0):
    """Time the 2-buffer fp32 SUM of the CPU oracle -- oracle/mx_oracle_op.c,
    the restatement of op_base_functions.c:40-51 (OP_FUNC, instantiated for
    float at :312), compiled with the reference's default flags (-O3
    -finline-functions, x86-64 baseline ISA) -- on one host core, on a
    bounded sample: 2 x 256 MiB host buffers, repeated ~`seconds`."""
    import numpy as np
    n = 1 << 26
    a = np.random.default_rng(1).uniform(-1, 1, n).astype(np.float32)
    b = np.random.default_rng(2).uniform(-1, 1, n).astype(np.float32)
    O = _oracle_bench()
    call = lambda: O.mxo_reduce2(3, 15, a.ctypes.data, b.ctypes.data, n, 1)   # [MPI_SUM][FLOAT]
    call()
    iters, t0 = 0, time.perf_counter()
    while True:
        call()
        iters += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    gbs = 3.0 * n * 4 * iters / el / 1e9
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": 1, "kind": "port", "host_cpu": _cpu_model(),
            "sample": f"fp32 SUM 2-buffer, 2 x 256 MiB host buffers, {iters} calls in {el:.1f} s "
                      f"(1 host thread; algorithmic 3*N*4 B per call; -O3 -finline-functions)"}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# CFG-C (BASELINE configs[2]): derived-datatype pack / unpack, one type of
# each constructor, 256 MiB packed per call
PACK_BENCH_TYPES = ["vector_f32_b4_s8", "indexed_f32_random", "struct_char_d3_int_resized48"]


def op_reduce_call_cost(torch, mx, sizes=(4 << 10, 64 << 10, 1 << 20)):
    """One blocking ompi_op_reduce on device buffers (fp32 SUM) through
    op/mi355x as Open MPI's op framework calls it (the mini-host's op table,
    ompi/op/op.h:547-610), microseconds per call measured in C: the resident
    service (default) and the launch marking itself (service off), A/B
    interleaved twice (tools/op_call_cost.py is the same loop)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import minihost
    H = minihost.host(with_components=True)
    H.mxh_time_op_reduce.restype = ctypes.c_double
    H.mxh_time_op_reduce.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    f32, SUM = minihost.dtype(H, "MPI_FLOAT"), minihost.op(H, "MPI_SUM")
    out = {"what": "ompi_op_reduce fp32 SUM, device buffers, op/mi355x via the mini-host op table",
           "service": {}, "launch": {}}
    for nbytes in sizes:
        n = nbytes // 4
        a = torch.rand(n, device="cuda")
        b = torch.rand(n, device="cuda")
        torch.cuda.synchronize()
        iters = 2000 if nbytes <= (64 << 10) else 500
        for rnd in range(2):
            for mode in ("service", "launch"):
                mx.op_service_set(mode == "service")
                ns = H.mxh_time_op_reduce(SUM, a.data_ptr(), b.data_ptr(), n, f32, iters)
                out[mode].setdefault(str(nbytes), []).append(round(ns / 1e3, 2))
    mx.op_service_set(True)
    return out


def allreduce_n1(torch, mx, nbytes=256 << 20, iters=20):
    """The 1-GPU point of the metric's "MPI_Allreduce ... 1/2/4/8 GPU": a
    size-1 communicator (MPI_COMM_SELF, a one-rank MPI_COMM_WORLD), 256 MiB
    fp32 SUM, sbuf -> rbuf.  coll/self would copy it with host memcpy
    (coll_self_allreduce.c:41-44); coll/mi355x's size-1 slot runs one device
    copy kernel.  Called as Open MPI calls it: the communicator's allreduce
    slot through the mini-host's MPI_Allreduce entry (the oracle is only the
    harness's base op table, never called here).  GB/s = 2 x S (read sbuf,
    write rbuf) / the blocking call's wall time; bit-exact copy
    checked after the timed calls."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import minihost
    H = minihost.host(with_components=True)
    H.mxh_self_calls.argtypes = []
    f32, SUM, self_comm = minihost.dtype(H, "MPI_FLOAT"), minihost.op(H, "MPI_SUM"), H.mxh_comm_self()
    owner = H.mxh_comm_slot_owner(self_comm, b"allreduce").decode()
    count = nbytes // 4
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    s_buf = torch.empty(count, device="cuda")
    r_buf = torch.empty(count, device="cuda")
    s_buf.uniform_(-1, 1, generator=g)
    r_buf.zero_()
    torch.cuda.synchronize()
    calls0 = H.mxh_self_calls()
    for _ in range(3):
        assert H.mxh_allreduce(s_buf.data_ptr(), r_buf.data_ptr(), count, f32, SUM, self_comm) == 0
    t0 = time.perf_counter()
    for _ in range(iters):
        H.mxh_allreduce(s_buf.data_ptr(), r_buf.data_ptr(), count, f32, SUM, self_comm)
    per = (time.perf_counter() - t0) / iters
    torch.cuda.synchronize()
    same = bool(torch.equal(s_buf.view(torch.int32), r_buf.view(torch.int32)))
    gbs = 2.0 * nbytes / per / 1e9
    return {"what": "MPI_Allreduce fp32 SUM 256 MiB on a size-1 communicator (MPI_COMM_SELF), device buffers, "
                    "through the communicator's allreduce slot (coll/mi355x size-1 path: one k_copy kernel)",
            "slot_owner": owner, "bytes": nbytes, "ms": round(per * 1e3, 4), "hbm_gbs": round(gbs, 1),
            "hbm_frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes": 2 * nbytes,
            "busbw_gbs": 0.0, "busbw_note": "busBW = algbw*2(n-1)/n is 0 at n = 1: nothing crosses a link",
            "delegated_to_coll_self": H.mxh_self_calls() - calls0,
            "parity": "ok" if same else "MISMATCH: rbuf differs from sbuf"}


def pack_side_by_side(torch, mx, cpu=True, packed_bytes=256 << 20, cpu_seconds=1.5):
    """MPI_Pack / MPI_Unpack of the CFG-C types on the device (mx_pack /
    mx_unpack, HIP events on the launch stream, median of 5 batches) and --
    `cpu` -- the convertor walk on one host core beside it (the oracle's
    restatement of opal_generic_simple_pack_function, opal_datatype_pack.c:
    235-370, and opal_datatype_unpack.c:245-427, -O3 build, kind "port").
    GB/s = 2 x packed bytes / time."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import golden_io
    basic, recs = golden_io.ddt_records()
    BASIC = np.ascontiguousarray(basic)
    O = _oracle_bench() if cpu else None
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    rows = []
    for name in PACK_BENCH_TYPES:
        rec = next(r for r in recs if r["name"] == name)
        ext = rec["ub"] - rec["lb"]
        count = packed_bytes // rec["size"]
        nbp = count * rec["size"]
        span = ext * (count - 1) + rec["true_ub"] - rec["true_lb"]
        row = {"type": name, "count": count, "packed_bytes": nbp}
        dt = mx.Datatype(rec["desc"].tobytes(), rec["nrec"], rec["size"], rec["lb"], rec["ub"])
        U = torch.randint(0, 256, (span,), dtype=torch.uint8, device="cuda")
        P = torch.empty(nbp, dtype=torch.uint8, device="cuda")
        ubase = U.data_ptr() - rec["true_lb"]
        for direction in ("pack", "unpack"):
            fn = (lambda: dt.pack(count, ubase, P.data_ptr(), stream=sp)) if direction == "pack" else \
                 (lambda: dt.unpack(count, ubase, P.data_ptr(), stream=sp))
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(4):
                    fn()
                e1.record(stream)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 4)
            ms = sorted(ts)[2]
            row[f"gpu_{direction}_gbs"] = round(2.0 * nbp / (ms * 1e-3) / 1e9, 1)
        del U, P
        dt.close()
        torch.cuda.empty_cache()
        if O is not None:
            user = np.random.default_rng(1).integers(0, 256, span, dtype=np.uint8)
            packed = np.zeros(nbp, np.uint8)
            for direction, unpack in (("pack", 0), ("unpack", 1)):
                call = lambda: O.mxo_ddt_convert(rec["desc"].ctypes.data, rec["nrec"], BASIC.ctypes.data, rec["lb"],
                                                 rec["ub"], count, user.ctypes.data - rec["true_lb"],
                                                 packed.ctypes.data, unpack)
                call()
                k, t0 = 0, time.perf_counter()
                while True:
                    call()
                    k += 1
                    el = time.perf_counter() - t0
                    if el >= cpu_seconds:
                        break
                row[f"cpu_{direction}_gbs"] = round(2.0 * nbp * k / el / 1e9, 3)
            del user, packed
            for d in ("pack", "unpack"):
                row[f"gpu_over_cpu_{d}"] = round(row[f"gpu_{d}_gbs"] / row[f"cpu_{d}_gbs"], 1)
        rows.append(row)
    out = {"unit": "GB/s", "types": rows,
           "gpu": "mx_pack / mx_unpack on one MI355X, HIP events, median of 5 x 4 calls"}
    if cpu:
        out["cpu"] = {"cores": 1, "kind": "port", "host_cpu": _cpu_model(),
                      "sample": f"the convertor walk restated (oracle/mx_oracle_ddt.c, -O3), one host thread, "
                                f"{packed_bytes >> 20} MiB packed per call, >= {cpu_seconds} s per type and direction"}
    return out


def cpu_baseline_allreduce(ranks=8, nbytes=256 << 20, iters=10):
    """The host MPI_Allreduce the reference runs with coll/tuned + vader,
    restated as `ranks` pinned processes over shared memory (single-copy;
    oracle/cpu_coll_proxy.c, BASELINE.md 2 "Fallback": no Open MPI on the
    box): coll/tuned's fixed decision (the 1 MiB segmented ring at 256 MiB)
    as `value`, the ring and Rabenseifner (coll_tuned_allreduce_algorithm
    4 / 6) beside it; fp32 SUM through a plain C loop of the
    reference's OP_FUNC shape (kind "port": the reference's loop cannot be
    built here)."""
    import subprocess
    exe = os.path.join(ROOT, "oracle", "build", "cpu_coll_proxy")
    if not os.path.exists(exe):
        return {"error": "oracle/build/cpu_coll_proxy not built"}
    cmd = [exe, str(ranks), str(nbytes), str(iters)]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        d = json.loads(p.stdout.strip().splitlines()[-1])
        d["sample"] = "proxy of coll/tuned + vader (no Open MPI on the box): " + d["sample"]
        return d
    except Exception as e:  # noqa: BLE001 - reported in the JSON line
        return {"error": repr(e)}


def bench_reduce_local(torch, mx, steps, warmup, nbytes=1 << 30):
    n = nbytes // 4
    g = torch.Generator(device="cuda").manual_seed(0x5EEDC0DE)
    # the three 1 GiB buffers are allocated first, as whole fresh segments,
    # and filled in place: temporaries of an out-of-place fill (rand * 2 - 1)
    # would leave the timed buffers in recycled, fragmented allocator blocks
    a = torch.empty(n, device="cuda")
    b0 = torch.empty(n, device="cuda")
    b = torch.empty(n, device="cuda")
    a.uniform_(-1, 1, generator=g)
    b0.uniform_(-1, 1, generator=g)
    b.copy_(b0)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    for _ in range(warmup):
        mx.reduce2("SUM", "FLOAT", a.data_ptr(), b.data_ptr(), n, sp)
    torch.cuda.synchronize()
    # one HIP event pair around the whole timed region (on the launch
    # stream): per-step event records would put 2 * steps marker packets
    # between the kernels and slow the very thing being timed
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        mx.reduce2("SUM", "FLOAT", a.data_ptr(), b.data_ptr(), n, sp)
    e1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kms = [e0.elapsed_time(e1) / steps] * steps      # average launch duration incl. the kernel boundaries
    # parity, outside the timed region: one more call on a fresh copy of b0
    # against the same IEEE fp32 sum computed by a torch kernel (a 2-operand
    # fp32 add has one correctly rounded result, so the check is bit-exact)
    c = b0.clone()
    mx.reduce2("SUM", "FLOAT", a.data_ptr(), c.data_ptr(), n, sp)
    ref = a + b0
    torch.cuda.synchronize()
    diff = (c.view(torch.int32) != ref.view(torch.int32))
    nbad = int(diff.sum().item())
    parity = "ok" if nbad == 0 else f"MISMATCH: {nbad} of {n} elements, first at {int(diff.nonzero()[0, 0])}"
    return wall, kms, 3.0 * n * 4, parity


def bench_allreduce(torch, mx, dist, rank, world, dev, steps, warmup, nbytes=256 << 20, extras=True):
    """MPI_Allreduce 256 MiB fp32 SUM per rank through the all-peer path
    (coll/tuned's fixed decision -> segmented-ring fold order).  Returns
    the result dict fields, or raises if the path is unavailable."""
    count = nbytes // 4

    def ag(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out

    ndev = torch.cuda.device_count()
    # RCCL runs on a communicator of its own after everything else (rccl_leg)
    flags = mx.COMM_IPC | mx.COMM_P2P
    comm = mx.Comm(rank, world, ag, device=dev, staging_bytes=2 * nbytes + (64 << 20), flags=flags,
                   heap_bytes=2 * nbytes + (4 << 20))
    x = _bench_input(torch, rank, count)
    out = torch.empty_like(x)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream

    def timed(alg, k):
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(k):
            comm.allreduce(x.data_ptr(), out.data_ptr(), count, "FLOAT", "SUM", alg, sp)
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    # the autotuner's trial calls for this size class run before the warmup
    # (untimed; a few calls: warm-up + one per candidate)
    tune_calls = 0
    while comm.tuning(nbytes) is None and tune_calls < 16 and world > 1:
        comm.allreduce(x.data_ptr(), out.data_ptr(), count, "FLOAT", "SUM", "auto", sp)
        tune_calls += 1
    for _ in range(warmup):
        comm.allreduce(x.data_ptr(), out.data_ptr(), count, "FLOAT", "SUM", "auto", sp)
    t_max = timed("auto", steps)
    algbw = nbytes / (t_max / steps) / 1e9
    busbw = algbw * 2 * (world - 1) / world
    # profiled pass: per-kernel device time of the fused fold (dominant kernel)
    comm.set_profiling(True)
    comm.stats(reset=True)
    for _ in range(3):
        comm.allreduce(x.data_ptr(), out.data_ptr(), count, "FLOAT", "SUM", "auto", sp)
    st = comm.stats(reset=True)
    comm.set_profiling(False)
    par = allreduce_parity(torch, mx, dist, rank, world, x, out, count)
    exp_sha = par.pop("_expected_sha", None)
    rccl_ref = (par.pop("_oracle_out", None), par.pop("_abs_sum", None))
    # data-movement A/B at the headline size (results are identical under
    # all three): zero-copy between registered user buffers (the default above
    # 256 KiB per rank), and the staged path under PUSH and PULL (the staged
    # default: PULL)
    proto_default = comm.protocol()
    proto_ab = {"staged_protocol": proto_default, "autotuned": comm.tuning(nbytes),
                "timed_path_last_calls": "zero_copy" if st["zero_copy_calls"] else "staged"}
    try:
        comm.set_autotune(False)   # the A/B below forces each path
    except mx.MxError:
        pass
    # zero_copy: results stored straight into the peers' rbufs (the default);
    # zero_copy_gather: through the peers' gather areas + a local copy (round 4)
    for name, reg, proto, direct in (("staged_push", 0, "push", True), ("staged_pull", 0, "pull", True),
                                     ("zero_copy_gather", 256 << 10, None, False), ("zero_copy", 256 << 10, None, True)):
        try:
            comm.set_reg_min(reg)
        except mx.MxError:
            if reg:
                proto_ab[name] = {"error": "registration unavailable"}
                continue
        comm.set_zc_direct(direct)
        comm.set_protocol(proto or proto_default)
        for _ in range(2):
            comm.allreduce(x.data_ptr(), out.data_ptr(), count, "FLOAT", "SUM", "auto", sp)
        k = max(3, steps // 2)
        zc0 = comm.stats()["zero_copy_calls"]
        tp = timed("auto", k)
        proto_ab[name] = {"busbw_gbs": round(nbytes / (tp / k) / 1e9 * 2 * (world - 1) / world, 2),
                          "ms": round(tp / k * 1e3, 4), "zero_copy_calls": comm.stats()["zero_copy_calls"] - zc0}
        # every data movement must give the same bytes as the checked call
        hs = [None] * world
        dist.all_gather_object(hs, _sha(torch, out))
        if rank == 0 and exp_sha is not None:
            proto_ab[name]["parity"] = "ok" if all(h == exp_sha for h in hs) else \
                f"MISMATCH on ranks {[r for r in range(world) if hs[r] != exp_sha]}"
    comm.set_protocol(proto_default)
    try:   # the sweep and CFG-E run with the defaults: autotuning on, zero-copy from 256 KiB
        comm.set_reg_min(256 << 10)
        comm.set_autotune(True)
    except mx.MxError:
        pass
    sweep = allreduce_sweep(torch, mx, dist, comm, world, x, out, sp, flags) if extras else "skipped (--no-sweep)"
    cfge = cfg_e(torch, mx, dist, comm, world, rank, sp) if extras else "skipped (--no-sweep)"
    # the data paths the autotuner kept per size class: where the
    # one-shot / zero-copy / staged crossovers fell on this machine
    tuned = {coll: {str(b): comm.tuning(b, coll) for b in (64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20,
                                                           256 << 20)}
             for coll in ("allreduce", "reduce_scatter", "allgather", "bcast")}
    tuned = {coll: {b: v for b, v in d.items() if v is not None} for coll, d in tuned.items()}
    extra = {}
    comm.close()
    fold_ms = st["fold_ms"] / max(1, st["fold_launches"])
    fold_bytes = st["fold_bytes"] / max(1, st["fold_launches"])
    shared_gpu = ndev < world
    peak_links = (world - 1) * XGMI_LINK_GBS
    fold_gbs = fold_bytes / (fold_ms * 1e-3) / 1e9 if fold_ms else None
    fold_bytes_call = st["fold_bytes"] / max(1, st["calls"])   # every chunk's fold of one call
    return {
        **par,
        "value": round(busbw, 2), "unit": "GB/s", "ms_per_step": round(t_max / steps * 1e3, 4),
        "config": {"workload": "MPI_Allreduce fp32 SUM 256 MiB per rank (coll/tuned fixed decision: "
                               "segmented-ring fold order), all-peer xGMI",
                   "count": count, "bytes": nbytes, "algorithm": "auto",
                   "parallelism": f"allreduce-{world}", "algbw_gbs": round(algbw, 2),
                   "data_path_ab": proto_ab,
                   "autotune_calls_before_warmup": tune_calls, "autotuned_paths": tuned,
                   "busbw_formula": "algbw*2(n-1)/n", **extra},
        # N>1 is bound by the xGMI links, not HBM: the all-peer exchange puts
        # 2S/n on each of a rank's n-1 links, so the busBW ceiling is
        # (n-1) x 153 GB/s (7 x 153 on a full node); the fold kernel's own
        # HBM fraction is reported beside it.  With the ranks sharing one GPU
        # (no link involved) the bound is that GPU's HBM: every rank's fold
        # bytes per call over the call's wall time (max over ranks) -- a lower
        # bound on the rate the GPU sustained, since the folds overlap for only
        # part of the call; summing the ranks' per-kernel rates instead assumes
        # they overlap completely (reported beside it: at n=8 it exceeds the
        # HBM peak, so they do not)
        "roofline": ({"bound": "xgmi", "achieved": round(busbw, 2), "peak": round(peak_links, 1), "unit": "GB/s",
                      "frac": round(busbw / peak_links, 4), "traffic": None,
                      "metric": "busBW = algbw*2(n-1)/n vs (n-1) links x 153 GB/s"} if not shared_gpu or not fold_gbs else
                     {"bound": "hbm", "achieved": round(world * fold_bytes_call / (t_max / steps) / 1e9, 1),
                      "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(world * fold_bytes_call / (t_max / steps) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                      "metric": "ranks sharing one GPU: all ranks' fold bytes per call / the call's wall time "
                                "(max over ranks) vs the GPU's HBM (no xGMI link involved); busBW in value",
                      "sum_of_rank_fold_rates_gbs": round(world * fold_gbs, 1),
                      "busbw_vs_links_if_separate_gpus": round(busbw / peak_links, 4)}) | {
                     "peak_all_links": 7 * XGMI_LINK_GBS, "frac_all_links": round(busbw / (7 * XGMI_LINK_GBS), 4),
                     "shared_gpu": shared_gpu,
                     "fold_kernel": {"kernel": "k_fold<float, mx::OpSum> (n reads + n writes, n-1 of them remote)",
                                     "algorithmic_bytes_per_launch": fold_bytes, "avg_kernel_ms": round(fold_ms, 4),
                                     "achieved_gbs": round(fold_gbs, 1) if fold_gbs else None,
                                     "hbm_peak_gbs": HBM_PEAK_GBS,
                                     "hbm_frac": round(fold_gbs / HBM_PEAK_GBS, 4) if fold_gbs else None},
                     "phase_ms_per_call": {k: round(st[k] / max(1, st["calls"]), 4)
                                           for k in ("fold_ms", "push_ms", "gather_ms", "total_ms")}},
        "sweep": sweep,
        "cfg_e": cfge,
        "_rccl_ref": rccl_ref,
    }


U_FP32 = 2.0 ** -24   # unit roundoff of IEEE binary32


def order_bound_check(got, ref, abs_sum, n):
    """Tolerance of an fp32 SUM over n ranks computed in another reduction
    order (BASELINE north_star: "within a stated relative tolerance
    (reduction-order bounded, scaled by rank count)").  Any order of the n-1
    additions rounds to within gamma_{n-1} * sum_i |x_i| of the exact sum
    (gamma_k = k u / (1 - k u), u = 2^-24, Higham 4.2), so two orders differ
    elementwise by at most 2 gamma_{n-1} sum_i |x_i|.  Returns (ok, worst
    |got - ref| / bound, index of the worst element); NaN / Inf positions must
    agree exactly."""
    import numpy as np
    got = np.asarray(got, np.float32)
    ref = np.asarray(ref, np.float32)
    k = max(1, n - 1)
    gamma = k * U_FP32 / (1.0 - k * U_FP32)
    bound = 2.0 * gamma * np.asarray(abs_sum, np.float64)
    fin = np.isfinite(ref)
    if not np.array_equal(fin, np.isfinite(got)):
        return False, float("inf"), int(np.nonzero(fin != np.isfinite(got))[0][0])
    diff = np.abs(got[fin].astype(np.float64) - ref[fin].astype(np.float64))
    b = bound[fin]
    over = np.where(b > 0, diff / np.where(b > 0, b, 1.0), np.where(diff > 0, np.inf, 0.0))
    if over.size == 0:
        return True, 0.0, -1
    i = int(np.argmax(over))
    return bool(over[i] <= 1.0), float(over[i]), int(np.nonzero(fin)[0][i])


def rccl_leg(torch, mx, dist, rank, world, dev, steps, rccl_ref, nbytes=256 << 20):
    """ncclAllReduce (RCCL over xGMI) on the headline buffers, on its own
    communicator, after every other measurement -- only when each rank has a
    GPU of its own (RCCL refuses two ranks on one device).  Timed like the
    headline (barrier + synchronize, max over ranks); its result is checked
    against the oracle's coll/tuned order (coll_base_allreduce.c:618-856) with
    order_bound_check: rank 0 against the bound, every other rank equal to
    rank 0 (SHA-256).  Returns the fields for the JSON line."""
    count = nbytes // 4

    def ag(b):
        out = [None] * world
        dist.all_gather_object(out, b)
        return out
    comm = mx.Comm(rank, world, ag, device=dev, staging_bytes=64 << 20, flags=mx.COMM_IPC | mx.COMM_RCCL)
    x = _bench_input(torch, rank, count)
    out = torch.empty_like(x)
    sp = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        comm.allreduce(x.data_ptr(), out.data_ptr(), count, "FLOAT", "SUM", "rccl", sp)
    k = max(3, steps // 2)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(k):
        comm.allreduce(x.data_ptr(), out.data_ptr(), count, "FLOAT", "SUM", "rccl", sp)
    torch.cuda.synchronize()
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    per = float(t[0]) / k
    hs = [None] * world
    dist.all_gather_object(hs, _sha(torch, out))
    res = {"rccl_busbw_gbs": round(nbytes / per / 1e9 * 2 * (world - 1) / world, 2),
           "rccl_ms": round(per * 1e3, 4)}
    if rank == 0:
        ref, abs_sum = rccl_ref
        if ref is None:
            res["rccl_parity"] = "unchecked: no oracle result"
        else:
            ok, worst, at = order_bound_check(out.cpu().numpy(), ref, abs_sum, world)
            same = all(h == hs[0] for h in hs)
            res["rccl_parity"] = ("ok" if ok and same else
                                  f"MISMATCH: worst |rccl - oracle| / bound = {worst:.3g} at element {at}"
                                  + ("" if same else "; ranks' results differ"))
            res["rccl_parity_check"] = {
                "what": "ncclAllReduce fp32 SUM vs the oracle's coll/tuned order, elementwise |d| <= "
                        "2 gamma_{n-1} sum_i |x_i| (gamma_k = k u / (1 - k u), u = 2^-24); every rank's result "
                        "equal to rank 0's", "worst_fraction_of_bound": round(worst, 4)}
    comm.close()
    return res


def _sha(torch, t):
    import hashlib
    return hashlib.sha256(t.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()


def _bench_input(torch, rank, count):
    """The bench's seeded input of `rank` (Philox on the device: any MI355X
    regenerates the same bytes from the seed)."""
    g = torch.Generator(device="cuda").manual_seed(0x5EED + rank)
    return torch.rand(count, device="cuda", generator=g) * 2 - 1


def allreduce_parity(torch, mx, dist, rank, world, x, out, count):
    """Bit-exact check of the timed allreduce (outside the timed region):
    every rank hashes its input and its result; rank 0 regenerates every
    rank's seeded input, confirms it against the rank's own input hash, runs
    the oracle restatement (oracle/mx_oracle_coll.c mxo_allreduce with the
    tuned fixed decision, coll_tuned_decision_fixed.c:44-95 ->
    coll_base_allreduce.c) over the n inputs and compares its result with
    every rank's.  Returns {"parity": "ok" | description, ...} on rank 0."""
    import numpy as np
    torch.cuda.synchronize()
    mine = (_sha(torch, x), _sha(torch, out))
    allh = [None] * world
    dist.all_gather_object(allh, mine)
    if rank != 0:
        return {}
    t0 = time.perf_counter()
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L = oracle_lib.oracle()
    L.mxo_allreduce.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    xs = []
    for r in range(world):
        xr = _bench_input(torch, r, count).cpu().numpy()
        import hashlib
        if hashlib.sha256(xr.view(np.uint8).tobytes()).hexdigest() != allh[r][0]:
            return {"parity": f"unchecked: rank {r}'s input did not regenerate from its seed on rank 0"}
        xs.append(xr)
    outs = [np.empty(count, np.float32) for _ in range(world)]
    rc = L.mxo_allreduce(0, mx.OP["SUM"], mx.TYPE["FLOAT"], world, count,
                         (vp * world)(*[a.ctypes.data for a in xs]), (vp * world)(*[o.ctypes.data for o in outs]))
    if rc != 0:
        return {"parity": f"unchecked: oracle rc {rc}"}
    import hashlib
    exp = hashlib.sha256(outs[0].view(np.uint8).tobytes()).hexdigest()
    bad = [r for r in range(world) if allh[r][1] != exp]
    res = {"parity_check": {"what": f"MPI_Allreduce fp32 SUM {count * 4} B per rank, tuned fixed decision, "
                                    "every rank's result vs oracle/mx_oracle_coll.c (SHA-256)",
                            "ranks_checked": world, "oracle_s": round(time.perf_counter() - t0, 2),
                            "result_sha256": exp[:16]}}
    if not bad:
        res["parity"] = "ok"
    else:
        where = ""
        if 0 in bad:
            got = out.cpu().numpy()
            d = np.nonzero(got.view(np.uint32) != outs[0].view(np.uint32))[0]
            where = f", rank 0 first differing byte offset {int(d[0]) * 4}" if len(d) else ""
        res["parity"] = f"MISMATCH on ranks {bad}{where}"
    res["_expected_sha"] = exp
    res["_oracle_out"] = outs[0]
    abs_sum = np.zeros(count, np.float64)
    for xr in xs:
        abs_sum += np.abs(xr.astype(np.float64))
    res["_abs_sum"] = abs_sum
    return res


def allreduce_sweep(torch, mx, dist, comm, world, x, out, sp, flags, budget_s=45.0):
    """CFG-D sweep (BASELINE configs[3]): MPI_Allreduce busBW / latency from
    8 B to 4 GiB per rank (x4 steps) for fp32 SUM under the tuned decision,
    the forced ring and Rabenseifner fold orders and RCCL, plus uint16 BAND
    (bf16-as-uint16); max over ranks, bounded to ~budget_s seconds."""
    rows = []
    algs = ["auto", "ring", "rabenseifner"] + (["rccl"] if flags & mx.COMM_RCCL else [])
    t_start = time.perf_counter()
    big = None
    sizes = [8 << (2 * k) for k in range(15)] + [4 << 30]       # 8 B, 32 B, ..., 2 GiB, 4 GiB
    for nbytes in sizes:
        if nbytes > x.numel() * 4:
            if big is None:   # one pair of buffers for every size above the headline's, sized for the largest
                try:
                    big = (torch.empty(sizes[-1] // 4, device="cuda").uniform_(-1, 1),
                           torch.empty(sizes[-1] // 4, device="cuda"))
                except RuntimeError:
                    rows.append({"bytes": nbytes, "error": "out of device memory"})
                    break
            bx, bo = big
        else:
            bx, bo = x, out
        assert bx.numel() * 4 >= nbytes and bo.numel() * 4 >= nbytes, "sweep buffer smaller than the message"
        for t, op in (("FLOAT", "SUM"), ("UINT16_T", "BAND")):
            if t == "UINT16_T" and nbytes not in (8, 64 << 10, 16 << 20, 256 << 20, 4 << 30):
                continue
            count = max(1, nbytes // (4 if t == "FLOAT" else 2))
            iters = 50 if nbytes <= (64 << 10) else (20 if nbytes <= (4 << 20) else (8 if nbytes <= (64 << 20)
                                                                                      else 3))
            for alg in algs:
                if alg == "rccl" and t == "UINT16_T":
                    continue
                ok = torch.tensor([1.0])
                # warm-up; the first call of a size class also runs the
                # autotuner's trials (13 calls below 4 MiB, 4 above, from 64 KiB)
                warm = 2 + ((13 if nbytes < (4 << 20) else 4) if nbytes >= (64 << 10) and alg == algs[0] else 0)
                try:
                    for _ in range(warm):
                        comm.allreduce(bx.data_ptr(), bo.data_ptr(), count, t, op, alg, sp)
                    torch.cuda.synchronize()
                except mx.MxError:
                    ok[0] = 0.0
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                if ok[0] == 0.0:
                    rows.append({"bytes": nbytes, "type": t, "op": op, "alg": alg, "error": "unsupported"})
                    continue
                dist.barrier()
                sv0 = comm.stats()["service_calls"]
                small = nbytes <= (64 << 10)   # blocking calls: each one's own time too (median)
                ts = []
                t0 = time.perf_counter()
                for _ in range(iters):
                    t1 = time.perf_counter() if small else 0.0
                    comm.allreduce(bx.data_ptr(), bo.data_ptr(), count, t, op, alg, sp)
                    if small:
                        ts.append(time.perf_counter() - t1)
                torch.cuda.synchronize()
                el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
                served = comm.stats()["service_calls"] - sv0
                med = None
                if small:
                    mt = torch.tensor([sorted(ts)[len(ts) // 2]], dtype=torch.float64)
                    dist.all_reduce(mt, op=dist.ReduceOp.MAX)
                    med = round(float(mt[0]) * 1e6, 2)
                dist.all_reduce(el, op=dist.ReduceOp.MAX)
                per = float(el[0]) / iters
                algbw = count * (4 if t == "FLOAT" else 2) / per / 1e9
                rows.append({"bytes": nbytes, "type": t, "op": op, "alg": alg, "us": round(per * 1e6, 2),
                             "algbw_gbs": round(algbw, 2), "busbw_gbs": round(algbw * 2 * (world - 1) / world, 2),
                             **({"us_median": med} if med is not None else {}),
                             **({"served": served} if served else {})})
        done = torch.tensor([1.0 if time.perf_counter() - t_start > budget_s else 0.0])
        dist.all_reduce(done, op=dist.ReduceOp.MAX)
        if done[0] > 0:
            rows.append({"note": f"sweep stopped after {nbytes} B (time budget {budget_s} s)"})
            break
    del big
    torch.cuda.empty_cache()
    return rows


def cfg_e(torch, mx, dist, comm, world, rank, sp, nbytes=256 << 20, iters=5):
    """CFG-E (BASELINE configs[4]) at 256 MiB: MPI_Reduce_scatter and
    MPI_Allgather (busBW = algBW*(n-1)/n, algBW over the full vector),
    MAXLOC float_int allreduce, OpenSHMEM float max_to_all and the other
    reduction slots (rooted reduce, reduce_scatter_block, scan), each with the
    coll/tuned (or coll/basic) fold order; then MPI_Accumulate on the symmetric
    heap, MPI_Iallreduce (libnbc orders) and an MPI_Sendrecv ring shift; max
    over ranks."""
    res = {}
    count = nbytes // 4
    g = torch.Generator(device="cuda").manual_seed(0x5EED + 101 * rank)
    x = torch.rand(count, device="cuda", generator=g)
    y = torch.empty_like(x)

    def timed(name, fn, algbw_bytes, factor):
        try:
            for _ in range(4):   # warm-up + the autotuner's trials of this size class
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize()
            el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            per = float(el[0]) / iters
            res[name] = {"ms": round(per * 1e3, 4), "algbw_gbs": round(algbw_bytes / per / 1e9, 2),
                         "busbw_gbs": round(algbw_bytes / per / 1e9 * factor, 2)}
        except mx.MxError as e:
            res[name] = {"error": str(e)}

    f_ring = (world - 1) / world
    rc = [count // world] * world
    timed("reduce_scatter_fp32_sum", lambda: comm.reduce_scatter(x.data_ptr(), y.data_ptr(), rc, "FLOAT", "SUM",
                                                                "auto", sp), nbytes, f_ring)
    per_rank = nbytes // world
    timed("allgather", lambda: comm.allgather(x.data_ptr(), y.data_ptr(), per_rank, sp), nbytes, f_ring)
    timed("bcast", lambda: comm.bcast(x.data_ptr(), nbytes, 0, sp), nbytes, 1.0)
    # MPI_FLOAT_INT pairs: 8 B per element, value ties and random indices
    timed("allreduce_maxloc_float_int", lambda: comm.allreduce(x.data_ptr(), y.data_ptr(), count // 2, "FLOAT_INT",
                                                               "MAXLOC", "auto", sp), nbytes, 2 * f_ring)
    timed("shmem_float_max_to_all", lambda: comm.shmem_reduce("MAX", "FLOAT", 4, y.data_ptr(), x.data_ptr(), count,
                                                              sp), nbytes, 2 * f_ring)
    timed("reduce_fp32_sum_root0", lambda: comm.reduce(x.data_ptr(), y.data_ptr(), count, "FLOAT", "SUM", 0,
                                                       "auto", sp), nbytes, 1.0)
    timed("reduce_scatter_block_fp32_sum", lambda: comm.reduce_scatter_block(x.data_ptr(), y.data_ptr(),
                                                                             count // world, "FLOAT", "SUM",
                                                                             "auto", sp), nbytes, f_ring)
    timed("scan_fp32_sum", lambda: comm.scan(x.data_ptr(), y.data_ptr(), count, "FLOAT", "SUM", "auto", sp),
          nbytes, 1.0)
    # OpenSHMEM max_to_all on the device symmetric heap: every PE folds its
    # part straight from all sources into all targets (no staging copies)
    try:
        heap = mx.Heap(comm, 2 * nbytes + (1 << 20))
        src, tgt = heap.alloc(nbytes), heap.alloc(nbytes)
        mx.lib().mx_copy(src, x.data_ptr(), nbytes, None)
        mx.sync()
        heap.barrier_all()
        timed("shmem_float_max_to_all_symheap", lambda: heap.reduce("MAX", "FLOAT", 4, tgt, src, count, stream=sp),
              nbytes, 2 * f_ring)
        # MPI_Accumulate(SUM) of a quarter of the buffer into the right
        # neighbour's window (lock, op kernel over xGMI, unlock); GB/s per rank
        acc = count // 4
        timed("accumulate_fp32_sum_to_right", lambda: heap.accumulate(src, acc, "FLOAT", "SUM", (rank + 1) % world,
                                                                      tgt, stream=sp), acc * 4, 1.0)
        heap.close()
    except mx.MxError as e:
        res["shmem_float_max_to_all_symheap"] = {"error": str(e)}
    # MPI_Iallreduce: eight slices posted back to back, then waited (libnbc's
    # orders); busBW over the whole vector
    k = 8

    def iar():
        sl = count // k
        reqs = [comm.iallreduce(x.data_ptr() + i * sl * 4, y.data_ptr() + i * sl * 4, sl, "FLOAT", "SUM", "auto", sp)
                for i in range(k)]
        for r in reqs:
            r.wait()
            r.free()
    timed("iallreduce_fp32_sum_8x", iar, (count // k) * k * 4, 2 * f_ring)
    # MPI_Sendrecv ring shift of the whole buffer (GB/s per rank per direction)
    timed("sendrecv_ring_shift", lambda: comm.sendrecv(x.data_ptr(), nbytes, (rank + 1) % world, y.data_ptr(),
                                                       nbytes, (rank - 1) % world, 0, 0, sp), nbytes, 1.0)
    del x, y
    torch.cuda.empty_cache()
    return res


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """`bench.py --gpus N` started without a launcher: form the N ranks here,
    one process per GPU, through torch.distributed.run as a child process
    (this process has not touched the GPU -- torch is not even imported yet
    -- and it never execs), relay rank 0's JSON line and return the launcher's
    exit code.  Ranks inherit the environment (HSA_ENABLE_IPC_MODE_LEGACY=0
    included) and rendezvous on 127.0.0.1."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env["MX_BENCH_SPAWNED"] = "1"
    env.setdefault("OMP_NUM_THREADS", "4")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    line = None
    for out in p.stdout:            # ranks' other stdout passes through
        if out.lstrip().startswith("{") and '"metric"' in out:
            line = out.strip()
        else:
            sys.stdout.write(out)
            sys.stdout.flush()
    rc = p.wait()
    if line is not None:
        print(line, flush=True)
    elif rc == 0:
        print(json.dumps({"metric": METRIC, "error": f"{n} ranks exited 0 without a result line"}), flush=True)
        rc = 1
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sweep", action="store_true",
                    help="N>1: skip the CFG-D size sweep and the CFG-E lines (the headline allreduce, its parity "
                         "check and the data-path A/B still run)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    launched = "WORLD_SIZE" in os.environ
    if not launched and args.gpus > 1:
        # the driver's `python3 bench.py --gpus N`: form the N ranks ourselves
        return spawn_ranks(args.gpus, sys.argv[1:])
    world = _env_int("WORLD_SIZE", 1)
    if launched and world != args.gpus:
        print(json.dumps({"metric": METRIC, "error": f"--gpus {args.gpus} but the launcher formed WORLD_SIZE={world} "
                                                     "ranks"}), flush=True)
        return 2

    import torch
    import mxompi as mx

    rank = _env_int("RANK", 0)
    local_rank = _env_int("LOCAL_RANK", 0)
    dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    mx.init(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)

    result = {"metric": METRIC, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
              "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
              "dtype": "f32", "data": "synthetic"}

    done = False
    if world > 1:
        try:
            result.update(bench_allreduce(torch, mx, dist, rank, world, dev, args.steps, args.warmup,
                                          extras=not args.no_sweep))
            done = True
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            result["allreduce_error"] = repr(e)
        rccl_ref = result.pop("_rccl_ref", (None, None))
        if done and torch.cuda.device_count() >= world and os.environ.get("MX_BENCH_RCCL", "1") != "0":
            # RCCL over xGMI beside the default path.  A watchdog ends the
            # ranks with the line printed if RCCL's bootstrap or a collective
            # never returns, so the headline is not lost with it.
            import threading

            def _expire():
                if rank == 0:
                    result["rccl_error"] = "timed out after 150 s"
                    print(json.dumps(result), flush=True)
                os._exit(0)
            wd = threading.Timer(150.0, _expire)
            wd.daemon = True
            wd.start()
            try:
                result.update(rccl_leg(torch, mx, dist, rank, world, dev, args.steps, rccl_ref))
            except Exception as e:  # noqa: BLE001 - reported in the JSON line
                result["rccl_error"] = repr(e)
            wd.cancel()
        elif done:
            result["rccl_busbw_gbs"] = None
            result["rccl_parity"] = f"not run: {torch.cuda.device_count()} GPU(s) for {world} ranks " \
                                    "(RCCL needs one GPU per rank)"
    if not done:
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        wall, kms, algo_bytes, parity = bench_reduce_local(torch, mx, args.steps, args.warmup)
        torch.cuda.synchronize()
        t_max = wall
        if dist is not None:
            dist.barrier()
            t = torch.tensor([wall], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t_max = float(t[0])
        avg_kernel_ms = sum(kms) / len(kms)
        achieved = algo_bytes / (avg_kernel_ms * 1e-3) / 1e9
        result.update({
            "value": round(algo_bytes * world / (t_max / args.steps) / 1e9, 2), "unit": "GB/s",
            "ms_per_step": round(t_max / args.steps * 1e3, 4),
            "config": {"workload": "MPI_Reduce_local fp32 SUM, 1 GiB device buffers"
                                   + ("" if world == 1 else f" x {world} independent replicas"),
                       "count": algo_bytes // 12, "bytes_per_buffer": algo_bytes // 3,
                       "parallelism": "replicas" if world > 1 else "single-gpu"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic("k_reduce2<float,OpSum>"),
                         "kernel": "k_reduce2<float, mx::OpSum, true> (non-temporal instance at >= 384 MiB footprint)",
                         "algorithmic_bytes_per_launch": algo_bytes,
                         "avg_kernel_ms": round(avg_kernel_ms, 4)},
            "parity": parity,
            "parity_check": {"what": "one more mx_reduce2 fp32 SUM of the 1 GiB inputs after the timed region, "
                                     "bit-compared with the same sum by a torch kernel (IEEE fp32 add)"},
        })
    if rank == 0 and world == 1:
        try:
            result["allreduce_n1"] = allreduce_n1(torch, mx)
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            result["allreduce_n1"] = {"error": repr(e)}
        # CFG-C beside the headline: device pack / unpack (+ the CPU walk)
        try:
            result["pack_unpack"] = pack_side_by_side(torch, mx, cpu=not args.no_cpu_baseline)
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            result["pack_unpack"] = {"error": repr(e)}
        try:
            result["op_reduce_call_us"] = op_reduce_call_cost(torch, mx)
        except Exception as e:  # noqa: BLE001 - reported in the JSON line
            result["op_reduce_call_us"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_reduce_local(args.cpu_seconds)
        result["cpu_baseline_pack"] = {k: result["pack_unpack"].get(k) for k in ("cpu", "types")} \
            if "types" in result.get("pack_unpack", {}) else result.get("pack_unpack")
        result["cpu_baseline_allreduce"] = cpu_baseline_allreduce()
    elif world > 1 and done and not args.no_cpu_baseline:
        # the host allreduce of the same shape (world ranks, 256 MiB fp32
        # SUM) on the box's own cores, beside the GPU number
        if rank == 0:
            result["cpu_baseline"] = cpu_baseline_allreduce(ranks=world, iters=5)
        dist.barrier()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
