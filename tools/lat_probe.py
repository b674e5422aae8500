"""Allreduce latency per size on n processes sharing the GPU (diagnostic).
usage: python tools/lat_probe.py N [modes]  (MX_ONESHOT_MAX in the environment)
modes: comma list of default | zc (registered user buffers) | push | pull
(staged path, registration off); default "default"."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zhpe-ompi_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def worker(rank, n, port, q, modes):
    import torch
    import torch.distributed as dist
    import mxompi
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n)
    torch.cuda.set_device(0)
    mxompi.init(0)

    def ag(b):
        out = [None] * n
        dist.all_gather_object(out, b)
        return out
    comm = mxompi.Comm(rank, n, ag, device=0, staging_bytes=256 << 20)
    big = 256 << 20 if "zc" in modes or "pull" in modes else 64 << 20
    x = torch.rand(big // 4, device="cuda")
    y = torch.empty_like(x)
    st = torch.cuda.current_stream().cuda_stream
    proto0 = comm.protocol()
    rows = []
    for nb in [4 << 10, 16 << 10, 64 << 10, 128 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20,
               16 << 20, 32 << 20, 64 << 20, 128 << 20, 256 << 20]:
        if nb > big:
            break
        cnt = nb // 4
        row = {"bytes": nb}
        for mode in modes:
            if mode == "default":          # the library defaults: zero-copy from 256 KiB, auto protocol
                comm.set_reg_min(256 << 10)
                comm.set_protocol("auto")
            elif mode == "zc":
                comm.set_reg_min(1)
            elif mode in ("push", "pull"):
                comm.set_reg_min(0)
                comm.set_protocol(mode)
            for _ in range(5):
                comm.allreduce(x.data_ptr(), y.data_ptr(), cnt, "FLOAT", "SUM", "auto", st)
            torch.cuda.synchronize()
            dist.barrier()
            it = 50 if nb <= (16 << 20) else 10
            t0 = time.perf_counter()
            for _ in range(it):
                comm.allreduce(x.data_ptr(), y.data_ptr(), cnt, "FLOAT", "SUM", "auto", st)
            torch.cuda.synchronize()
            el = torch.tensor([(time.perf_counter() - t0) / it])
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            row[mode] = round(float(el[0]) * 1e6, 1)
            comm.set_protocol(proto0)
        rows.append(row)
        if rank == 0:
            print(f"n={n}", row, flush=True)
    comm.close()
    dist.destroy_process_group()
    q.put((rank, rows))


if __name__ == "__main__":
    import socket
    import torch.multiprocessing as mp
    n = int(sys.argv[1])
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["default"]
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, n, port, q, modes)) for r in range(n)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(n))
    for p in ps:
        p.join(timeout=60)
    print(f"n={n} oneshot_max={os.environ.get('MX_ONESHOT_MAX', 'default')}:", res[0], flush=True)
