"""Small-allreduce latency, resident service vs launch (VERDICT r5 missing 5).

usage: python tools/coll_lat.py [N] [sizes]   (N processes sharing GPU 0,
default 2; sizes a comma list of bytes, default 8,1024,32768)

Per size and mode: the median of 1000 blocking fp32 SUM allreduces timed one
by one from Python through the Comm wrapper, and (`*_abi`) of 1000 more
through the bare C-ABI entry point mx_allreduce (ctypes, arguments converted
once), the maximum over ranks; the Python + ctypes cost of one two-argument
library call (mx_coll_service_stats, no GPU work) is printed beside it.  With the service on, rank 0 also prints
mx_coll_service_trace: where a served call's time goes (host preparation,
host wait from post to `done`, and the kernel's argument read and the call
itself)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zhpe-ompi_amd"))

ITERS = 1000


def worker(rank, n, port, q, sizes):
    import torch
    import torch.distributed as dist
    import mxompi
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n)
    torch.cuda.set_device(0)
    mxompi.init(0)

    def ag(b):
        out = [None] * n
        dist.all_gather_object(out, b)
        return out
    comm = mxompi.Comm(rank, n, ag, device=0, staging_bytes=16 << 20)
    comm.set_timeout(30.0)
    L = mxompi.lib()
    st = torch.cuda.current_stream().cuda_stream
    a, b = ctypes.c_ulonglong(), ctypes.c_ulonglong()
    t0 = time.perf_counter()
    for _ in range(ITERS):
        L.mx_coll_service_stats(ctypes.byref(a), ctypes.byref(b))
    ffi_us = (time.perf_counter() - t0) / ITERS * 1e6
    rows = []
    for nb in sizes:
        cnt = max(1, nb // 4)
        x = torch.rand(cnt, device="cuda")
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        row = {"bytes": nb}
        for mode in ("service", "launch"):
            L.mx_coll_service_set(1 if mode == "service" else 0)
            for _ in range(50):
                comm.allreduce(x.data_ptr(), y.data_ptr(), cnt, "FLOAT", "SUM", "auto", st)
            dist.barrier()
            tr0 = (ctypes.c_double * 10)()
            L.mx_coll_service_trace(tr0, 10)
            ts = []
            for _ in range(ITERS):
                t0 = time.perf_counter()
                comm.allreduce(x.data_ptr(), y.data_ptr(), cnt, "FLOAT", "SUM", "auto", st)
                ts.append(time.perf_counter() - t0)
            # the C-ABI call itself: mx_allreduce through ctypes with its
            # arguments converted once (no wrapper, no name lookups)
            fn = mxompi._coll_lib().mx_allreduce
            args = (comm.h, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), ctypes.c_size_t(cnt),
                    mxompi._slot("FLOAT"), mxompi._op("SUM"), mxompi._alg(mxompi.ALLREDUCE, "auto"),
                    ctypes.c_void_p(st) if st else None)
            ta = []
            for _ in range(ITERS):
                t0 = time.perf_counter()
                rc = fn(*args)
                ta.append(time.perf_counter() - t0)
                assert rc == 0, rc
            tr1 = (ctypes.c_double * 10)()
            L.mx_coll_service_trace(tr1, 10)
            med = torch.tensor([sorted(ts)[len(ts) // 2] * 1e6, sorted(ta)[len(ta) // 2] * 1e6])
            dist.all_reduce(med, op=dist.ReduceOp.MAX)
            row[mode] = round(float(med[0]), 2)
            row[mode + "_abi"] = round(float(med[1]), 2)
            if mode == "service":
                # means over this size's served calls only
                k = tr1[0] - tr0[0]
                row["served"] = int(k)
                if k > 0:
                    names = ("prep", "wait", "k_args", "k_dchk", "k_push", "k_gather", "k_fold", "k_ack")
                    row["trace_us"] = {nm: round((tr1[i + 1] * tr1[0] - tr0[i + 1] * tr0[0]) / k, 2)
                                       for i, nm in enumerate(names)}
                    row["full_commands"] = int(tr1[9] - tr0[9])
        if nb == sizes[0]:
            # calls after an idle gap (the service leaves after 200 us idle):
            # each call alone, the ranks aligned by a barrier, then the gap
            for mode, gap in (("service", 0.0005), ("service", 0.002), ("launch", 0.0005), ("launch", 0.002)):
                L.mx_coll_service_set(1 if mode == "service" else 0)
                ts = []
                for _ in range(60):
                    dist.barrier()
                    time.sleep(gap)
                    t0 = time.perf_counter()
                    comm.allreduce(x.data_ptr(), y.data_ptr(), cnt, "FLOAT", "SUM", "auto", st)
                    ts.append(time.perf_counter() - t0)
                ts = ts[10:]
                agg = torch.tensor([sorted(ts)[len(ts) // 2] * 1e6, sum(ts) / len(ts) * 1e6])
                dist.all_reduce(agg, op=dist.ReduceOp.MAX)
                row[f"{mode}_after_gap_{int(gap * 1e6)}us"] = {"median": round(float(agg[0]), 2),
                                                                "mean": round(float(agg[1]), 2)}
            L.mx_coll_service_set(1)
        rows.append(row)
        if rank == 0:
            print(f"n={n}", row, flush=True)
    L.mx_coll_service_set(1)
    comm.close()
    dist.destroy_process_group()
    q.put((rank, {"ffi_us": round(ffi_us, 2), "rows": rows}))


if __name__ == "__main__":
    import socket
    import torch.multiprocessing as mp
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    sizes = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [8, 1024, 32768]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, n, port, q, sizes)) for r in range(n)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(n))
    for p in ps:
        p.join(timeout=60)
    print(f"n={n} python+ctypes per call (us):", [res[r]["ffi_us"] for r in range(n)], flush=True)
    print(f"n={n} rank 0:", res[0]["rows"], flush=True)
