#!/usr/bin/env python3
"""Where does the 8-process one-GPU MPI_Sendrecv ring shift spend its time?
(diagnostic for VERDICT r2 item 9; not product)

usage (on the GPU box):
  python tools/sendrecv_trace.py launch [N] [MiB] [outdir]
      starts N rank processes, each as `rocprofv3 --kernel-trace -- python3
      tools/sendrecv_trace.py rank ...` (the launcher itself never touches the
      GPU, and the profiler's child is python3 itself), then merges the per-rank
      kernel traces with the per-rank host timestamps into outdir/summary.txt
  python tools/sendrecv_trace.py rank R N PORT MiB OUTDIR      (one rank)
  python tools/sendrecv_trace.py analyse OUTDIR N

Each rank runs the bench's ring shift (bench.py cfg_e, `sendrecv_ring_shift`):
4 warm-up and 5 timed MPI_Sendrecv of the whole buffer to rank+1 / from
rank-1, host timestamps (CLOCK_MONOTONIC ns, the clock rocprofv3 stamps
kernels with) around every call.  The analysis lists, per timed call and
rank, the kernels the call launched: when each was dispatched relative to
the call's start (queue wait) and how long it ran (spin / copy).
"""
import csv
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def launch(n, mib, out):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.makedirs(out, exist_ok=True)
    procs = []
    noprof = os.environ.get("SR_NOPROF") == "1"
    for r in range(n):
        cmd = ["python3", os.path.abspath(__file__), "rank", str(r), str(n), str(port), str(mib), out]
        if not noprof:
            cmd = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", os.path.join(out, f"r{r}"),
                   "-o", "run", "--"] + cmd
        procs.append(subprocess.Popen(cmd, stdout=open(os.path.join(out, f"r{r}.log"), "w"),
                                      stderr=subprocess.STDOUT))
    rc = 0
    for p in procs:
        rc |= p.wait(timeout=600)
    if rc:
        print("a rank failed; see", out, flush=True)
        return rc
    analyse(out, n)
    return 0


def rank_main(r, n, port, mib, out):
    sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))
    import torch
    import torch.distributed as dist
    import mxompi as mx
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=r, world_size=n)
    torch.cuda.set_device(0)
    mx.init(0)

    def ag(b):
        o = [None] * n
        dist.all_gather_object(o, b)
        return o
    nbytes = mib << 20
    comm = mx.Comm(r, n, ag, device=0, staging_bytes=64 << 20, flags=mx.COMM_IPC | mx.COMM_P2P)
    x = torch.full((nbytes,), r, dtype=torch.uint8, device="cuda")
    y = torch.empty_like(x)
    sp = torch.cuda.current_stream().cuda_stream
    rows = []
    for it in range(9):
        dist.barrier()
        t0 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
        comm.sendrecv(x.data_ptr(), nbytes, (r + 1) % n, y.data_ptr(), nbytes, (r - 1) % n, 0, 0, sp)
        t1 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
        torch.cuda.synchronize()
        t2 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
        rows.append({"it": it, "t0": t0, "t_ret": t1, "t_sync": t2})
    ok = bool((y[:4096] == (r - 1) % n).all().item())
    comm.close()
    dist.destroy_process_group()
    with open(os.path.join(out, f"host_r{r}.json"), "w") as f:
        json.dump({"rank": r, "ok": ok, "rows": rows}, f)


def analyse(out, n):
    lines = []
    for r in range(n):
        host = json.load(open(os.path.join(out, f"host_r{r}.json")))
        ks = []
        for path in glob.glob(os.path.join(out, f"r{r}", "**", "*kernel_trace.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    ks.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row["Kernel_Name"][:40]))
        ks.sort()
        for row in host["rows"][4:]:
            t0, t2 = row["t0"], row["t_sync"]
            mine = [k for k in ks if k[0] >= t0 - 1000 and k[0] <= t2]
            desc = "; ".join(f"{k[2].split('(')[0]} +{(k[0] - t0) / 1e6:.3f}ms run {(k[1] - k[0]) / 1e6:.3f}ms"
                             for k in mine)
            lines.append(f"r{r} it{row['it']} call {(t2 - t0) / 1e6:8.3f} ms (returned {(row['t_ret'] - t0) / 1e6:.3f})"
                         f" ok={host['ok']} | {desc}")
    with open(os.path.join(out, "summary.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines), flush=True)


if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "launch":
        n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
        mib = int(sys.argv[3]) if len(sys.argv) > 3 else 256
        out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "gpurun_out", "sendrecv_trace")
        sys.exit(launch(n, mib, out))
    elif mode == "rank":
        rank_main(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6])
    else:
        analyse(sys.argv[2], int(sys.argv[3]))
