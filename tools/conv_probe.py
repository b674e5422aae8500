#!/usr/bin/env python3
"""conv_probe.py -- time device pack / unpack of one or more datatypes at a
given packed size (HIP events, median of batches), for A/B runs of the
convertor kernels (environment switches MX_CONV_*) and as the driver of
rocprofv3 --pmc passes.

Types: golden names (tests/golden/ddt_vectors.bin), or
  vec:<f32|f64>:<blocklen>:<stride>   MPI_Type_vector(n, blocklen, stride)
  tri:<n>                              upper triangle of an n x n double matrix (row i: n - i
                                       elements from (i, i); ref_upper_matrix_60 at size n)
  idx:<nblocks>:<seed>                 MPI_Type_indexed of f32, nblocks random blocks of 1..64
                                       elements with 0..16-element gaps (the indexed_f32_random
                                       recipe of oracle/gen_ddt_golden.c at large block counts)
usage: conv_probe.py [--bytes N] [--dirs pack,unpack] [--reps R] TYPE [TYPE ...]
Algorithmic bytes: 2 x packed bytes.  Prints one line per (type, direction).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def make_type(mx, name):
    """(Datatype, size, extent, true_lb, true_ub)"""
    if name.startswith("vec:"):
        import test_convertor_pins as P
        _, t, blen, stride = name.split(":")
        tid, es = (15, 4) if t == "f32" else (16, 8)          # OPAL FLOAT4 / FLOAT8
        # one block per instance, resized to the stride: instances repeat every
        # `stride` elements (== MPI_Type_vector(n, blocklen, stride) as a whole)
        d = P.Desc([(tid, 1, int(blen), int(blen) * es, 0)], int(blen) * es, 0, int(stride) * es)
        return mx.Datatype(d.bytes, d.nrec, d.size, d.lb, d.ub), d.size, d.ub - d.lb, 0, int(blen) * es
    if name.startswith("tri:"):
        import test_convertor_pins as P
        n = int(name.split(":")[1])
        d = P.indexed([n - i for i in range(n)], [i * n + i for i in range(n)], 16, 8)
        return mx.Datatype(d.bytes, d.nrec, d.size, d.lb, d.ub), d.size, d.ub - d.lb, d.lb, d.ub
    if name.startswith("idx:"):
        import numpy as np
        import test_convertor_pins as P
        _, nb, seed = name.split(":")
        rng = np.random.default_rng(int(seed))
        bl = rng.integers(1, 65, int(nb))
        gaps = rng.integers(0, 17, int(nb))
        dp = np.cumsum(gaps) + np.concatenate(([0], np.cumsum(bl)[:-1]))
        d = P.indexed([int(x) for x in bl], [int(x) for x in dp], 15, 4)
        return mx.Datatype(d.bytes, d.nrec, d.size, d.lb, d.ub), d.size, d.ub - d.lb, d.lb, d.ub
    import golden_io
    _, recs = golden_io.ddt_records()
    r = next(x for x in recs if x["name"] == name)
    dt = mx.Datatype(r["desc"].tobytes(), r["nrec"], r["size"], r["lb"], r["ub"])
    return dt, r["size"], r["ub"] - r["lb"], r["true_lb"], r["true_ub"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--dirs", default="pack,unpack")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("types", nargs="+")
    args = ap.parse_args()
    import torch
    import mxompi as mx
    mx.init(0)
    s = torch.cuda.current_stream()
    for name in args.types:
        dt, size, ext, tlb, tub = make_type(mx, name)
        count = args.bytes // size
        span = ext * (count - 1) + tub - tlb
        U = torch.randint(0, 256, (span,), dtype=torch.uint8, device="cuda")
        P = torch.empty(count * size, dtype=torch.uint8, device="cuda")
        base = U.data_ptr() - tlb
        for d in args.dirs.split(","):
            fn = (lambda: dt.pack(count, base, P.data_ptr(), stream=s.cuda_stream)) if d == "pack" else \
                 (lambda: dt.unpack(count, base, P.data_ptr(), stream=s.cuda_stream))
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                fn()
                e1.record(s)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = sorted(ts)[len(ts) // 2]
            nb = count * size
            print(f"{d:>6} {name:<30} {nb:>11} B  runs {dt.runs:>3}  {ms * 1e3:9.1f} us  "
                  f"{2 * nb / (ms * 1e-3) / 1e9:8.1f} GB/s", flush=True)
        del U, P
        dt.close()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
