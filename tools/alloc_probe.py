"""alloc_probe.py -- does the headline kernel's speed depend on where its
1 GiB buffers land?  Times mx.reduce2 fp32 SUM (K1, non-temporal instance)
over buffers placed several ways in ONE process: three separate 1 GiB
allocations (bench.py's layout), one 3 GiB allocation carved in thirds,
and the same after freeing and re-allocating.  HIP events on the launch
stream, 20 launches per measurement, best / median of 5.
usage: python tools/alloc_probe.py"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))

import torch  # noqa: E402
import mxompi as mx  # noqa: E402

N = (1 << 30) // 4


def time_k1(a, b, reps=5, iters=20):
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    for _ in range(3):
        mx.reduce2("SUM", "FLOAT", a.data_ptr(), b.data_ptr(), N, sp)
    out = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(iters):
            mx.reduce2("SUM", "FLOAT", a.data_ptr(), b.data_ptr(), N, sp)
        e1.record(s)
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / iters)
    return min(out), statistics.median(out)


def report(name, a, b):
    best, med = time_k1(a, b)
    print(f"{name:44s} best {best:.4f} ms ({3 * N * 4 / best / 1e6:.0f} GB/s)  median {med:.4f} ms  "
          f"a%2M={a.data_ptr() % (2 << 20)} b%2M={b.data_ptr() % (2 << 20)}", flush=True)


def main():
    mx.init(0)
    a = torch.empty(N, device="cuda").uniform_(-1, 1)
    b0 = torch.empty(N, device="cuda").uniform_(-1, 1)
    b = torch.empty(N, device="cuda")
    b.copy_(b0)
    report("three 1 GiB allocations (bench.py)", a, b)
    report("  a, b0 (the second pair)", a, b0)
    big = torch.empty(3 * N, device="cuda")
    big[:N].copy_(a)
    big[N:2 * N].copy_(b0)
    report("one 3 GiB allocation, thirds 0 / 1", big[:N], big[N:2 * N])
    report("  thirds 0 / 2", big[:N], big[2 * N:])
    del a, b0, b
    torch.cuda.empty_cache()
    a2 = torch.empty(N, device="cuda").uniform_(-1, 1)
    b2 = torch.empty(N, device="cuda").uniform_(-1, 1)
    report("re-allocated after empty_cache", a2, b2)
    report("one 3 GiB allocation, thirds 0 / 1, again", big[:N], big[N:2 * N])


if __name__ == "__main__":
    main()
