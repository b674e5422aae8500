"""Zero-copy allreduce into receive buffers freed and re-made at the same
address (the intermittent test_registration_fast_path_reused_and_remade_buffers
failure: a whole peer part of a re-made rbuf stays zero).

usage: python tools/reg_remade_probe.py [cycles]
Three processes share GPU 0.  Per cycle every rank allocates a new rbuf
(mx_alloc), runs two zero-copy int32 SUM allreduces of 1 Mi elements into it
(new inputs each), checks both results itself, and frees it.  Prints, per
rank, the wrong results per call of a cycle, the zero-copy call count and
the imports refused because the runtime handed back the import of the
peer's freed allocation (reg_stale_refused; the call then ran staged).

Round 6 (profiles/r06/reg_remade_probe_r6k.txt), before the check existed:
closing the stale import and then opening the new handle gave 8 of 30 cycles
wrong on two ranks (both calls: the cached mapping reached the freed
memory); opening the new handle while the stale import was still open
returned the stale mapping's address every time."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zhpe-ompi_amd"))

N = 3
COUNT = 1 << 20


def _x(rank, cyc, rep):
    import numpy as np
    return np.random.default_rng(7000 + 1000 * cyc + 10 * rep + rank).integers(
        -(1 << 31), 1 << 31, COUNT, dtype=np.int64).astype(np.int32)


def worker(rank, port, q, cycles):
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    import numpy as np
    import torch
    import torch.distributed as dist
    import mxompi
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=N)
    torch.cuda.set_device(0)
    mxompi.init(0)

    def ag(b):
        out = [None] * N
        dist.all_gather_object(out, b)
        return out
    comm = mxompi.Comm(rank, N, ag, device=0, staging_bytes=16 << 20)
    comm.set_timeout(30.0)
    comm.set_autotune(False)
    comm.set_reg_min(1)
    st = torch.cuda.current_stream().cuda_stream
    L = mxompi.lib()
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    X = torch.empty(COUNT, dtype=torch.int32, device="cuda")
    bad = [0, 0]
    fails = []
    st0 = comm.stats()
    for cyc in range(cycles):
        p = vp()
        assert L.mx_alloc(sz(4 * COUNT), ctypes.byref(p)) == 0
        for rep in range(2):
            X.copy_(torch.from_numpy(_x(rank, cyc, rep)).cuda())
            torch.cuda.synchronize()
            comm.allreduce(X.data_ptr(), p.value, COUNT, "INT32_T", "SUM", "auto", st)
            host = np.empty(COUNT, np.int32)
            assert L.mx_memcpy(vp(host.ctypes.data), p, sz(4 * COUNT), None) == 0
            want = sum(_x(r, cyc, rep).astype(np.int64) for r in range(N)).astype(np.int32)
            if not np.array_equal(host, want):
                bad[rep] += 1
                wrong = np.nonzero(host != want)[0]
                fails.append((cyc, rep, int(wrong[0]), len(wrong), hex(p.value)))
        torch.cuda.synchronize()
        assert L.mx_free(p) == 0
    st1 = comm.stats()
    comm.close()
    dist.destroy_process_group()
    q.put((rank, {"bad": bad, "fails": fails, "zc": st1["zero_copy_calls"] - st0["zero_copy_calls"],
                  "refused": st1["reg_stale_refused"] - st0["reg_stale_refused"]}))


if __name__ == "__main__":
    import socket
    import torch.multiprocessing as mp
    cycles = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, port, q, cycles)) for r in range(N)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(N))
    for p in ps:
        p.join(timeout=60)
    print(f"cycles {cycles}, per rank (wrong results of call 1, call 2; zero-copy calls; refused imports):",
          [(res[r]["bad"], res[r]["zc"], res[r]["refused"]) for r in range(N)], flush=True)
    for r in range(N):
        print(f"rank {r} wrong (cycle, call, first wrong element, wrong elements, rbuf):", res[r]["fails"][:12], flush=True)
