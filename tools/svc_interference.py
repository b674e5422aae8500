#!/usr/bin/env python3
"""svc_interference.py -- what the resident op service costs the application
(VERDICT r4 next 7).

The application: a 1 GiB device copy (read 1 GiB + write 1 GiB) launched
back to back on an ordinary stream, timed with HIP events on that stream.
Beside it, a host thread makes blocking ompi_op_reduce-shaped calls
(mx_reduce2_sync, fp32 SUM, on a third, idle stream -- the op component's
handler) of 64 KiB or 1 MiB in a loop:
  alone     the copy with nothing beside it
  service   the calls served by the resident kernel (MX_OP_SERVICE default)
  launch    the same calls launched per call (service off)
Each configuration runs twice, interleaved.  Prints GB/s of the copy, its
slowdown against `alone`, and the calls made meanwhile.
usage: svc_interference.py [--reps 40] [--sizes 65536,1048576]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--sizes", default="65536,1048576")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    import mxompi as mx
    mx.init(0)
    n = 1 << 28                                        # 1 GiB of fp32
    a = torch.rand(n, device="cuda")
    b = torch.empty_like(a)
    app = torch.cuda.Stream()
    caller = torch.cuda.Stream()
    torch.cuda.synchronize()

    def run_app():
        with torch.cuda.stream(app):
            b.copy_(a)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(app)
            for _ in range(args.reps):
                b.copy_(a)
            e1.record(app)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        return 2.0 * n * 4 / (ms * 1e-3) / 1e9

    def calls_beside(nbytes, served):
        mx.op_service_set(served)
        cnt = nbytes // 4
        x = torch.rand(cnt, device="cuda")
        y = torch.rand(cnt, device="cuda")
        torch.cuda.synchronize()
        stop = threading.Event()
        made = [0]

        def loop():
            sp = caller.cuda_stream
            while not stop.is_set():
                mx.reduce2_sync("SUM", "FLOAT", x.data_ptr(), y.data_ptr(), cnt, sp)
                made[0] += 1

        th = threading.Thread(target=loop)
        th.start()
        time.sleep(0.02)
        t0 = time.perf_counter()
        gbs = run_app()
        el = time.perf_counter() - t0
        stop.set()
        th.join()
        st = mx.op_service_stats()
        mx.op_service_set(True)
        return gbs, made[0], el, st

    rows = []
    for rnd in range(2):
        alone = run_app()
        rows.append({"round": rnd, "config": "alone", "copy_gbs": round(alone, 1)})
        print(f"round {rnd} alone                 copy {alone:8.1f} GB/s", flush=True)
        for nbytes in [int(s) for s in args.sizes.split(",")]:
            for served in (True, False):
                gbs, made, el, st = calls_beside(nbytes, served)
                name = "service" if served else "launch"
                row = {"round": rnd, "config": name, "call_bytes": nbytes, "copy_gbs": round(gbs, 1),
                       "slowdown_pct": round(100.0 * (alone / gbs - 1.0), 2), "calls": made,
                       "calls_per_s": round(made / el, 0), "service_state_served_launches": st,
                       # application time lost per call: the copy's wall time times the share it lost
                       "app_us_lost_per_call": round(1e6 * el * (1.0 - gbs / alone) / max(1, made), 3)}
                rows.append(row)
                print(f"round {rnd} {name:7s} {nbytes:>8} B  copy {gbs:8.1f} GB/s  slowdown {row['slowdown_pct']:6.2f} %"
                      f"  calls {made} ({row['calls_per_s']:.0f}/s)  app lost {row['app_us_lost_per_call']:.2f} us/call",
                      flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"what": __doc__.strip().splitlines()[0], "reps": args.reps, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
