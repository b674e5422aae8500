"""Diagnostic (not product): two ranks on one GPU, Irecv; op service calls;
Isend; Wait -- with timestamps around each step and a traceback dump of a
rank stuck for 15 s.  usage: python tools/svc_p2p_debug.py [MX_ENV=VAL ...]"""
import faulthandler
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))


def worker(rank, port, env):
    import torch
    import torch.distributed as dist
    os.environ.update(env)
    faulthandler.dump_traceback_later(15, exit=True)
    import mxompi
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    torch.cuda.set_device(0)
    mxompi.init(0)

    def ag(b):
        out = [None] * 2
        dist.all_gather_object(out, b)
        return out

    def log(msg):
        print(f"[{time.time() % 1000:8.3f}] rank {rank}: {msg}", flush=True)

    comm = mxompi.Comm(rank, 2, ag, device=0, staging_bytes=1 << 20)
    comm.set_timeout(12.0)
    s = torch.cuda.Stream()
    a = torch.ones(4096, dtype=torch.int64, device="cuda")
    b = torch.zeros(4096, dtype=torch.int64, device="cuda")
    x = torch.full((4096,), rank, dtype=torch.uint8, device="cuda")
    y = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    mode = os.environ.get("DBG_MODE", "reduce_first")
    if mode == "reduce_first":   # the service starts before the receive spins
        mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), 4096, s.cuda_stream)
        log(f"warm reduce done {mxompi.op_service_stats()}")
    r = comm.irecv(y.data_ptr(), 4096, 1 - rank, tag=7)
    log("irecv posted")
    dist.barrier()
    for i in range(3):
        time.sleep(0.001)
        mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), 4096, s.cuda_stream)
        log(f"reduce {i} done {mxompi.op_service_stats()} held {mxompi.op_service_held()}")
    sq = comm.isend(x.data_ptr(), 4096, 1 - rank, tag=7)
    log("isend posted")
    sq.wait()
    log("send done")
    r.wait()
    log(f"recv done {int(y[0].item())}")
    comm.close()
    dist.destroy_process_group()


def main():
    env = dict(kv.split("=", 1) for kv in sys.argv[1:])
    import torch.multiprocessing as mp
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=worker, args=(r, port, env)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(60)
        if p.is_alive():
            p.terminate()
    print("exit codes", [p.exitcode for p in ps], flush=True)


if __name__ == "__main__":
    main()
