"""MPI_Send/MPI_Recv ping-pong latency between 2 processes sharing the GPU
(diagnostic): half round trip per size, blocking and Isend/Irecv forms.
usage: python tools/p2p_lat.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zhpe-ompi_amd"))


def worker(rank, n, port, q):
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
    comm = mxompi.Comm(rank, n, ag, device=0, staging_bytes=64 << 20)
    peer = 1 - rank
    rows = []
    sizes = [8, 4096, 65536, 256 << 10, (256 << 10) + 16, 1 << 20, 4 << 20, 8 << 20, 16 << 20, 64 << 20, 256 << 20]
    if os.environ.get("P2P_LAT_SIZES"):          # e.g. "8,4096" (diagnostics)
        sizes = [int(v) for v in os.environ["P2P_LAT_SIZES"].split(",")]
    # one buffer that holds the largest message (a send or receive past its
    # end reads / writes outside the allocation)
    x = torch.zeros(max(sizes), dtype=torch.uint8, device="cuda")
    assert x.numel() >= max(sizes)
    dist_out = {}
    for nb in sizes:
        for form in ("blocking", "nonblocking"):
            def one():
                if form == "blocking":
                    if rank == 0:
                        comm.send(x.data_ptr(), nb, peer, tag=1)
                        comm.recv(x.data_ptr(), nb, peer, tag=1)
                    else:
                        comm.recv(x.data_ptr(), nb, peer, tag=1)
                        comm.send(x.data_ptr(), nb, peer, tag=1)
                else:
                    if rank == 0:
                        s = comm.isend(x.data_ptr(), nb, peer, tag=1); s.wait(); s.free()
                        r = comm.irecv(x.data_ptr(), nb, peer, tag=1); r.wait(); r.free()
                    else:
                        r = comm.irecv(x.data_ptr(), nb, peer, tag=1); r.wait(); r.free()
                        s = comm.isend(x.data_ptr(), nb, peer, tag=1); s.wait(); s.free()
            for _ in range(10):
                one()
            dist.barrier()
            it = int(os.environ.get("P2P_LAT_ITERS", 100 if nb <= (1 << 20) else 20))
            ts = []
            for _ in range(it):
                t0 = time.perf_counter()
                one()
                ts.append(time.perf_counter() - t0)
            if os.environ.get("P2P_LAT_DIST"):     # the first 40 half round trips in order + percentiles
                dist_out[(nb, form)] = ([round(t / 2 * 1e6, 1) for t in ts[:40]],
                                        [round(sorted(ts)[int(q * (len(ts) - 1))] / 2 * 1e6, 1)
                                         for q in (0.1, 0.25, 0.5, 0.75, 0.9)])
            ts.sort()
            us = ts[len(ts) // 2] / 2 * 1e6      # median round trip (the mean is at the box's mercy)
            rows.append((nb, form, round(us, 1), round(nb / us / 1e3, 2)))
    comm.close()
    dist.destroy_process_group()
    q.put((rank, (rows, dist_out)))


if __name__ == "__main__":
    import socket
    import torch.multiprocessing as mp
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    for k, v in res[0][1].items():
        print("rank 0", k, "first 40:", v[0], "p10/25/50/75/90:", v[1], flush=True)
    print("p2p half-round-trip (bytes, form, us, GB/s):", res[0][0], flush=True)
