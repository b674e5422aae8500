#!/usr/bin/env python3
"""sweep.py -- throughput sweeps of the device path on one MI355X.

  pairs : MPI_Reduce_local, every (op, type) pair of the with-Fortran table
          (176), 2-buffer, 1 GiB device buffers (CFG-B).
  sizes : fp32 SUM and uint16 BAND Reduce_local, 8 B .. 4 GiB per buffer.
  pack  : pack / unpack of the CFG-C derived types (vector b1/b4/16/64,
          indexed, struct-resized; descriptions from tests/golden) at packed
          sizes 8 B .. 4 GiB.

Algorithmic bytes: reduce 3*count*sizeof(T); pack/unpack 2*packed bytes.
Times are HIP events on the launch stream (median of `--iters` batches).
Writes one JSON document (``--out``).  GPU only; uses no oracle code.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0

F32 = {"FLOAT", "REAL", "REAL4", "C_FLOAT_COMPLEX", "2REAL"}
F64 = {"DOUBLE", "REAL8", "DOUBLE_PRECISION", "C_DOUBLE_COMPLEX", "2DOUBLE_PRECISION"}
X87 = {"LONG_DOUBLE", "C_LONG_DOUBLE_COMPLEX"}


LOC = {"FLOAT_INT": ("f4", 8, 4), "DOUBLE_INT": ("f8", 16, 8), "LONG_INT": ("i8", 16, 8), "2INT": ("i4", 8, 4),
       "SHORT_INT": ("i2", 8, 4), "2REAL": ("f4", 8, 4), "2DOUBLE_PRECISION": ("f8", 16, 8), "2INTEGER": ("i4", 8, 4)}


def fill(torch, buf, tname, gen, opname=None):
    """Overwrite a uint8 device buffer with values of type `tname` drawn from
    SURVEY 8(d)'s distributions (tools/cpu_sweep.py fill() is the host twin):
    integers full-range uniform; FP SUM / MAX / MIN uniform [-1, 1), PROD
    [0.5, 2) (complex parts alike); x87 values of magnitude ~1 (random sign
    and mantissa, exponent 16382..16383); LOC pairs' values from 16 distinct
    values (ties) with random int indices."""
    nb = buf.numel()
    buf.copy_(torch.randint(0, 256, (nb,), dtype=torch.uint8, device=buf.device, generator=gen))
    lo, hi = (0.5, 2.0) if opname == "PROD" else (-1.0, 1.0)
    if tname in F32:
        buf.view(torch.float32).uniform_(lo, hi, generator=gen)
    elif tname in F64:
        buf.view(torch.float64).uniform_(lo, hi, generator=gen)
    elif tname in X87 or tname == "LONG_DOUBLE_INT":
        stride = 4 if tname == "LONG_DOUBLE_INT" else 2   # int64 words per element
        w = buf.view(torch.int64).view(-1, stride)
        w[:, 0] |= torch.iinfo(torch.int64).min             # explicit integer bit
        sign = (torch.randint(0, 2, (w.shape[0],), device=buf.device, generator=gen) << 15) if opname != "PROD" else 0
        w[:, 1] = (16382 + torch.randint(0, 2, (w.shape[0],), device=buf.device, generator=gen)) | sign
        if tname == "LONG_DOUBLE_INT":                       # 16 distinct values (ties)
            w[:, 0] = torch.iinfo(torch.int64).min | (torch.randint(0, 16, (w.shape[0],), device=buf.device,
                                                                    generator=gen) << 59)
    elif tname in LOC:
        vt, es, io = LOC[tname]
        rows = buf.view(-1, es)
        n = rows.shape[0]
        tv = {"f4": torch.float32, "f8": torch.float64, "i8": torch.int64, "i4": torch.int32, "i2": torch.int16}[vt]
        vals = torch.randint(0, 16, (n,), device=buf.device, generator=gen).to(tv)
        vs = vals.element_size()
        rows[:, :vs] = vals.view(torch.uint8).view(n, vs)


def time_launches(torch, fn, iters, reps, prep=None):
    """median over `iters` batches of `reps` back-to-back launches, ms per
    launch; `prep` runs before each batch, outside the timed region (restores
    the in-place operand, so every batch starts from pristine data)"""
    stream = torch.cuda.current_stream()
    if prep:
        prep()
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(iters):
        if prep:
            prep()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        for _ in range(reps):
            fn()
        e.record(stream)
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / reps)
    out.sort()
    return out[len(out) // 2]


def sweep_pairs(torch, mx, nbytes, iters, only=None):
    sp = torch.cuda.current_stream().cuda_stream
    gen = torch.Generator(device="cuda").manual_seed(0x5EEDC0DE)
    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    b0 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    rows = []
    for t, tname in enumerate(mx.TYPES):
        if only and tname not in only:
            continue
        ops = [o for o in range(1, 13) if mx.op_supported(o, t)]
        if not ops:
            continue
        es = mx.type_size(t)
        count = nbytes // es
        for o in ops:
            fill(torch, a, tname, gen, mx.OPS[o])
            fill(torch, b0, tname, gen, mx.OPS[o])
            # every timed launch starts from pristine inout (b restored from b0)
            ms = time_launches(torch, lambda: mx.reduce2(o, t, a.data_ptr(), b.data_ptr(), count, sp), iters, 1,
                               prep=lambda: b.copy_(b0))
            gbs = 3.0 * count * es / (ms * 1e-3) / 1e9
            rows.append({"op": mx.OPS[o], "type": tname, "elem_bytes": es, "count": count,
                         "ms": round(ms, 4), "gbs": round(gbs, 1), "frac_hbm": round(gbs / HBM_PEAK_GBS, 4)})
            print(f"pair {mx.OPS[o]:>6} {tname:<22} {ms:8.3f} ms {gbs:8.1f} GB/s", flush=True)
    return rows


def sweep_sizes(torch, mx, max_bytes, iters):
    sp = torch.cuda.current_stream().cuda_stream
    gen = torch.Generator(device="cuda").manual_seed(7)
    a = torch.empty(max_bytes, dtype=torch.uint8, device="cuda")
    b = torch.empty(max_bytes, dtype=torch.uint8, device="cuda")
    rows = []
    for op, tname in (("SUM", "FLOAT"), ("BAND", "UINT16_T")):
        fill(torch, a, tname, gen)
        fill(torch, b, tname, gen)
        es = mx.type_size(tname)
        nb = 8
        while nb <= max_bytes:
            count = nb // es
            reps = 200 if nb <= (1 << 20) else (20 if nb <= (64 << 20) else 3)
            ms = time_launches(torch, lambda: mx.reduce2(op, tname, a.data_ptr(), b.data_ptr(), count, sp),
                               iters, reps)
            gbs = 3.0 * count * es / (ms * 1e-3) / 1e9
            rows.append({"op": op, "type": tname, "bytes_per_buffer": nb, "us": round(ms * 1e3, 2),
                         "gbs": round(gbs, 1), "frac_hbm": round(gbs / HBM_PEAK_GBS, 4)})
            print(f"size {op} {tname} {nb:>12} B {ms * 1e3:10.2f} us {gbs:8.1f} GB/s", flush=True)
            nb *= 4 if nb < (1 << 30) else 2
    return rows


PACK_TYPES = ["vector_f32_b1_s2", "vector_f64_b3_s5", "vector_f32_b4_s8", "vector_f32_b16_s32", "vector_f32_b64_s128",
              "indexed_f32_random", "struct_char_d3_int_resized48"]


def sweep_pack(torch, mx, max_packed, iters, types=None, min_packed=8):
    import golden_io
    _, recs = golden_io.ddt_records()
    sp = torch.cuda.current_stream().cuda_stream
    rows = []
    for name in (types or PACK_TYPES):
        rec = next(r for r in recs if r["name"] == name)
        dt = mx.Datatype(rec["desc"].tobytes(), rec["nrec"], rec["size"], rec["lb"], rec["ub"])
        ext = rec["ub"] - rec["lb"]
        top = max_packed // rec["size"]
        span = ext * (top - 1) + rec["true_ub"] - rec["true_lb"]
        U = torch.randint(0, 256, (span,), dtype=torch.uint8, device="cuda")
        P = torch.empty(top * rec["size"], dtype=torch.uint8, device="cuda")
        ubase = U.data_ptr() - rec["true_lb"]
        packed = 8
        while packed < min_packed:
            packed *= 8 if packed < (1 << 29) else 2
        while packed <= max_packed:
            count = packed // rec["size"]
            if count >= 1:
                nbp = count * rec["size"]
                reps = 100 if nbp <= (1 << 20) else (10 if nbp <= (64 << 20) else 2)
                for direction in ("pack", "unpack"):
                    if direction == "pack":
                        fn = lambda: dt.pack(count, ubase, P.data_ptr(), stream=sp)
                    else:
                        fn = lambda: dt.unpack(count, ubase, P.data_ptr(), stream=sp)
                    ms = time_launches(torch, fn, iters, reps)
                    gbs = 2.0 * nbp / (ms * 1e-3) / 1e9
                    rows.append({"type": name, "dir": direction, "runs": dt.runs, "count": count,
                                 "packed_bytes": nbp, "us": round(ms * 1e3, 2), "gbs": round(gbs, 1),
                                 "frac_hbm": round(gbs / HBM_PEAK_GBS, 4)})
                    print(f"{direction:>6} {name:<30} {nbp:>12} B {ms * 1e3:10.2f} us {gbs:8.1f} GB/s",
                          flush=True)
            packed *= 8 if packed < (1 << 29) else 2
        del U, P
        dt.close()
        torch.cuda.empty_cache()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="pairs,sizes,pack")
    ap.add_argument("--out", default="gpurun_out/sweep.json")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--pair-bytes", type=int, default=1 << 30)
    ap.add_argument("--max-bytes", type=int, default=4 << 30)
    ap.add_argument("--min-bytes", type=int, default=8)
    ap.add_argument("--types", default="", help="comma-separated golden type names for the pack sweep")
    ap.add_argument("--pair-types", default="", help="comma-separated MPI type names for the pairs sweep")
    args = ap.parse_args()
    import torch
    import mxompi as mx
    mx.init(0)
    doc = {"device": torch.cuda.get_device_name(0), "hbm_peak_gbs": HBM_PEAK_GBS,
           "timing": "HIP events on the launch stream, median of batches", "when": time.strftime("%F %T")}
    what = args.what.split(",")
    if "pairs" in what:
        doc["pairs"] = sweep_pairs(torch, mx, args.pair_bytes, args.iters,
                                   {t for t in args.pair_types.split(",") if t} or None)
        torch.cuda.empty_cache()
    if "sizes" in what:
        doc["sizes"] = sweep_sizes(torch, mx, args.max_bytes, args.iters)
        torch.cuda.empty_cache()
    if "pack" in what:
        doc["pack"] = sweep_pack(torch, mx, args.max_bytes, args.iters,
                                 [t for t in args.types.split(",") if t] or None, args.min_bytes)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
