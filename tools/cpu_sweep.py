#!/usr/bin/env python3
"""cpu_sweep.py -- the CPU baseline beside the GPU sweeps.

  pairs : MPI_Reduce_local on the host, every (op, type) pair of the C-only
          op table (116; op_base_functions.c:1485-1569 without the Fortran
          slots), 2-buffer, one host thread, bounded sample (2 x 64 MiB
          buffers; per pair the median of >= 20 calls, each from pristine
          operands; SURVEY 8(d) value distributions, seed 0x5EEDC0DE).
  pack  : MPI_Pack / MPI_Unpack of the CFG-C derived types (the pack sweep's
          types, tools/sweep.py PACK_TYPES) through the convertor walk, one
          host thread, 256 MiB packed per call, ~0.5 s per type and direction.

The loops timed are the oracle's restatements (oracle/mx_oracle_op.c of
op_base_functions.c:40-104 and the x87 / complex variants; oracle/
mx_oracle_ddt.c of opal_generic_simple_pack_function, opal_datatype_pack.c:
235-370, and its unpack twin opal_datatype_unpack.c:245-427) -- kind "port":
the reference itself cannot be built here -- compiled with the
reference's default flags (-O3 -finline-functions -fno-strict-aliasing,
config/opal_setup_cc.m4:351-365, 481-493; oracle/Makefile
build/libmx_oracle_bench.so).

`--merge-gpu A.json[,B.json]` puts the GPU sweep's rows (tools/sweep.py
output) beside each CPU row: GPU GB/s, CPU GB/s, ratio.  Algorithmic bytes as
the GPU sweep: reduce 3*count*sizeof(T), pack/unpack 2*packed bytes.
TEST/MEASUREMENT INFRASTRUCTURE: loads the oracle, never the product.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

PACK_TYPES = ["vector_f32_b1_s2", "vector_f64_b3_s5", "vector_f32_b4_s8", "vector_f32_b16_s32", "vector_f32_b64_s128",
              "indexed_f32_random", "struct_char_d3_int_resized48"]


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def bench_lib():
    path = os.path.join(ROOT, "oracle", "build", "libmx_oracle_bench.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "build/libmx_oracle_bench.so"], check=True)
    L = ctypes.CDLL(path)
    vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L.mxo_reduce2.argtypes = [i, i, vp, vp, sz, i]
    L.mxo_supported.argtypes = [i, i, i]
    L.mxo_type_size.restype = sz
    L.mxo_type_size.argtypes = [i]
    L.mxo_ddt_convert.argtypes = [vp, sz, vp, ctypes.c_int64, ctypes.c_int64, sz, vp, vp, ctypes.c_int]
    return L


def _timed(fn, min_s):
    fn()                                   # warm: pages touched, caches in their steady state
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        el = time.perf_counter() - t0
        if el >= min_s:
            return el / n, n


# SURVEY 8(d)'s value distributions, per (op, type): integers full-range
# uniform; FP (and complex parts, and x87 values) uniform [-1, 1) for SUM and
# MAX / MIN, [0.5, 2) for PROD; the LOC pairs' values drawn from 16 distinct
# values (ties) with random int indices.  tools/sweep.py fill() makes the same
# distributions on the device.
_LOC = {"FLOAT_INT": (np.float32, 8), "DOUBLE_INT": (np.float64, 16), "LONG_INT": (np.int64, 16),
        "2INT": (np.int32, 8), "SHORT_INT": (np.int16, 8), "LONG_DOUBLE_INT": (np.longdouble, 32),
        "2REAL": (np.float32, 8), "2DOUBLE_PRECISION": (np.float64, 16), "2INTEGER": (np.int32, 8)}
_F32 = {"FLOAT", "REAL", "REAL4", "C_FLOAT_COMPLEX"}
_F64 = {"DOUBLE", "REAL8", "DOUBLE_PRECISION", "C_DOUBLE_COMPLEX"}
_X87 = {"LONG_DOUBLE", "C_LONG_DOUBLE_COMPLEX"}


def fill(buf, tname, opname, rng):
    buf[:] = rng.bit_generator.random_raw((buf.size + 7) // 8).view(np.uint8)[:buf.size]
    lo, hi = (0.5, 2.0) if opname == "PROD" else (-1.0, 1.0)
    if tname in _F32:
        buf.view(np.float32)[:] = rng.uniform(lo, hi, buf.size // 4)
    elif tname in _F64:
        buf.view(np.float64)[:] = rng.uniform(lo, hi, buf.size // 8)
    elif tname in _X87:
        v = buf.view(np.longdouble)
        v[:] = rng.uniform(lo, hi, v.size).astype(np.longdouble)
    elif tname in _LOC:
        vt, es = _LOC[tname]
        n = buf.size // es
        rows = buf[:n * es].reshape(n, es)
        vals = rng.integers(0, 16, n).astype(vt)                     # 16 distinct values: ties
        vs = 10 if vt is np.longdouble else np.dtype(vt).itemsize
        rows[:, :vs] = vals.view(np.uint8).reshape(n, -1)[:, :vs]
        io = 16 if vt is np.longdouble else np.dtype(vt).itemsize
        io = 4 if tname == "SHORT_INT" else io                       # {short; int} at offset 4
        rows[:, io:io + 4] = rng.integers(-(1 << 31), 1 << 31, n, dtype=np.int64).astype("<i4").view(
            np.uint8).reshape(n, 4)


def sweep_pairs(L, nbytes, min_s, reps_min=20):
    """Every timed call starts from pristine operands: `inout` is restored
    from its untouched copy before each call, outside the timed region
    (a sweep that ran every op in place over the same
    buffer measured MINLOC on data converged to all ties).  Median of at
    least `reps_min` calls and `min_s` seconds of calls."""
    import mxompi as mx
    rng = np.random.default_rng(0x5EEDC0DE)
    a = np.empty(nbytes, np.uint8)
    b0 = np.empty(nbytes, np.uint8)
    b = np.empty(nbytes, np.uint8)
    rows = []
    for t, tname in enumerate(mx.TYPES):
        ops = [o for o in range(1, 13) if L.mxo_supported(o, t, 0)]   # the C-only table
        if not ops:
            continue
        es = L.mxo_type_size(t)
        count = nbytes // es
        for o in ops:
            fill(a, tname, mx.OPS[o], rng)
            fill(b0, tname, mx.OPS[o], rng)
            ts = []
            spent = 0.0
            for k in range(reps_min + 2):
                np.copyto(b, b0)                      # pristine inout, untimed
                t0 = time.perf_counter()
                L.mxo_reduce2(o, t, a.ctypes.data, b.ctypes.data, count, 0)
                dt = time.perf_counter() - t0
                if k >= 2:                            # two warm calls
                    ts.append(dt)
                    spent += dt
                if k >= reps_min + 1 and spent >= min_s:
                    break
            while spent < min_s:
                np.copyto(b, b0)
                t0 = time.perf_counter()
                L.mxo_reduce2(o, t, a.ctypes.data, b.ctypes.data, count, 0)
                dt = time.perf_counter() - t0
                ts.append(dt)
                spent += dt
            sec = float(np.median(ts))
            gbs = 3.0 * count * es / sec / 1e9
            rows.append({"op": mx.OPS[o], "type": tname, "elem_bytes": es, "count": count, "calls": len(ts),
                         "ms": round(sec * 1e3, 3), "gbs": round(gbs, 2)})
            print(f"cpu pair {mx.OPS[o]:>6} {tname:<22} {sec * 1e3:9.2f} ms {gbs:8.2f} GB/s", flush=True)
    return rows


def sweep_pack(L, packed_bytes, min_s):
    import golden_io
    basic, recs = golden_io.ddt_records()
    BASIC = np.ascontiguousarray(basic)
    rows = []
    for name in PACK_TYPES:
        rec = next(r for r in recs if r["name"] == name)
        ext = rec["ub"] - rec["lb"]
        count = max(1, packed_bytes // rec["size"])
        span = ext * (count - 1) + rec["true_ub"] - rec["true_lb"]
        user = np.random.default_rng(1).integers(0, 256, span, dtype=np.uint8)
        packed = np.zeros(count * rec["size"], np.uint8)
        ubase = user.ctypes.data - rec["true_lb"]
        for direction, unpack in (("pack", 0), ("unpack", 1)):
            sec, n = _timed(lambda: L.mxo_ddt_convert(rec["desc"].ctypes.data, rec["nrec"], BASIC.ctypes.data,
                                                      rec["lb"], rec["ub"], count, ubase, packed.ctypes.data,
                                                      unpack), min_s)
            gbs = 2.0 * packed.size / sec / 1e9
            rows.append({"type": name, "dir": direction, "count": count, "packed_bytes": int(packed.size),
                         "calls": n, "ms": round(sec * 1e3, 3), "gbs": round(gbs, 2)})
            print(f"cpu {direction:>6} {name:<30} {packed.size:>11} B {sec * 1e3:9.2f} ms {gbs:8.2f} GB/s",
                  flush=True)
    return rows


def merge(doc, gpu_paths):
    gpu_pairs, gpu_pack = {}, {}
    for p in gpu_paths:
        with open(p) as f:
            g = json.load(f)
        for r in g.get("pairs", []):
            gpu_pairs[(r["op"], r["type"])] = r
        for r in g.get("pack", []):
            k = (r["type"], r["dir"])
            if k not in gpu_pack or r["packed_bytes"] > gpu_pack[k]["packed_bytes"]:
                gpu_pack[k] = r                      # the largest size the GPU sweep ran
    side = []
    for r in doc.get("pairs", []):
        g = gpu_pairs.get((r["op"], r["type"]))
        if g:
            side.append({"op": r["op"], "type": r["type"], "gpu_gbs": g["gbs"], "gpu_bytes_per_buffer": g["count"] *
                         g["elem_bytes"], "cpu_gbs": r["gbs"], "cpu_bytes_per_buffer": r["count"] * r["elem_bytes"],
                         "gpu_over_cpu": round(g["gbs"] / r["gbs"], 1)})
    side = [dict(x, cpu_gbs=x.pop("cpu_gbs")) for x in side]
    doc["pairs_side_by_side"] = side
    sidep = []
    for r in doc.get("pack", []):
        g = gpu_pack.get((r["type"], r["dir"]))
        if g:
            sidep.append({"type": r["type"], "dir": r["dir"], "gpu_gbs": g["gbs"], "gpu_packed_bytes": g["packed_bytes"],
                          "cpu_gbs": r["gbs"], "cpu_packed_bytes": r["packed_bytes"],
                          "gpu_over_cpu": round(g["gbs"] / r["gbs"], 1)})
    doc["pack_side_by_side"] = sidep
    doc["gpu_sources"] = gpu_paths


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="pairs,pack")
    ap.add_argument("--out", default="gpurun_out/cpu_sweep.json")
    ap.add_argument("--pair-bytes", type=int, default=64 << 20)
    ap.add_argument("--pack-bytes", type=int, default=256 << 20)
    ap.add_argument("--min-s", type=float, default=0.2)
    ap.add_argument("--merge-gpu", default="", help="comma-separated tools/sweep.py JSON files")
    ap.add_argument("--from-json", default="", help="merge into an existing cpu_sweep JSON instead of measuring")
    args = ap.parse_args()
    if args.from_json:
        with open(args.from_json) as f:
            doc = json.load(f)
    else:
        L = bench_lib()
        doc = {"host_cpu": cpu_model(), "cores": 1, "kind": "port",
               "build": "oracle/build/libmx_oracle_bench.so: -O3 -finline-functions -fno-strict-aliasing (the "
                        "reference's default optimisation flags, config/opal_setup_cc.m4), x86-64 baseline ISA",
               "sample": f"pairs: 2 x {args.pair_bytes >> 20} MiB host buffers, per pair the median of >= 20 calls "
                         f"(>= {args.min_s} s of calls), every call from pristine operands (inout restored outside the "
                         "timed region), SURVEY 8(d) distributions (seed 0x5EEDC0DE: integers full range, FP SUM/MAX/MIN "
                         "uniform [-1,1), PROD [0.5,2), LOC 16 distinct values); pack: "
                         f"{args.pack_bytes >> 20} MiB packed per call, >= {2.5 * args.min_s} s per direction; "
                         "1 host thread",
               "when": time.strftime("%F %T"), "source_run": os.environ.get("MX_SWEEP_RUN", "")}
        what = args.what.split(",")
        if "pairs" in what:
            doc["pairs"] = sweep_pairs(L, args.pair_bytes, args.min_s)
        if "pack" in what:
            doc["pack"] = sweep_pack(L, args.pack_bytes, 2.5 * args.min_s)
    if args.merge_gpu:
        merge(doc, [p for p in args.merge_gpu.split(",") if p])
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(doc, f, indent=1)
    if doc.get("pairs_side_by_side") or doc.get("pack_side_by_side"):
        with open(os.path.splitext(args.out)[0] + ".txt", "w") as f:
            f.write(f"# CPU ({doc.get('host_cpu')}, {doc.get('cores')} core, {doc.get('kind')}; {doc.get('build')})\n"
                    f"# vs GPU ({', '.join(doc.get('gpu_sources', []))}); GB/s algorithmic\n"
                    f"# source run: {doc.get('source_run') or '(unnamed)'}, CPU column at {doc.get('when')}; the GPU "
                    f"and CPU columns come from this one run on one box\n"
                    f"# sample: {doc.get('sample')}\n")
            f.write(f"{'op':>7} {'type':<24} {'GPU GB/s':>10} {'CPU GB/s':>10} {'GPU/CPU':>8}\n")
            for r in doc.get("pairs_side_by_side", []):
                f.write(f"{r['op']:>7} {r['type']:<24} {r['gpu_gbs']:10.1f} {r['cpu_gbs']:10.2f} {r['gpu_over_cpu']:8.1f}\n")
            f.write(f"\n{'dir':>7} {'type':<30} {'GPU GB/s':>10} {'(packed B)':>12} {'CPU GB/s':>10} {'(packed B)':>12} "
                    f"{'GPU/CPU':>8}\n")
            for r in doc.get("pack_side_by_side", []):
                f.write(f"{r['dir']:>7} {r['type']:<30} {r['gpu_gbs']:10.1f} {r['gpu_packed_bytes']:12d} "
                        f"{r['cpu_gbs']:10.2f} {r['cpu_packed_bytes']:12d} {r['gpu_over_cpu']:8.1f}\n")


if __name__ == "__main__":
    main()
