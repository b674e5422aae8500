"""Device waits under hardware-queue pressure.

Every collective wait is a device-side spin that needs the peers' kernels
resident.  Several ranks per GPU is a legal MPI deployment, and a process
that holds more streams than the runlist maps can starve its group: round 5
saw two timeouts of 8 processes on one GPU while a private lifecycle stream
added one hardware queue per process.

Here 8 processes share the one GPU and each holds, besides the streams the
library uses, two application streams with work queued on them (element-wise
passes over 64 MiB, not waited for) and an MPI_Iallreduce pending on a second
communicator (on a stream of its own), while the first communicator runs the
headline 256 MiB fp32 SUM allreduce three ways: staged PUSH, staged PULL and
zero-copy.  Every result is compared with the oracle's coll/tuned order
(oracle/mx_oracle_coll.c) through a SHA-256 digest, and so is the
Iallreduce's (libnbc's order)."""
import ctypes
import os

import numpy as np
import pytest

import mxompi
import oracle_lib
from test_coll_headline_gpu import C256, STAGING_ONE_CHUNK, digest, gen_big, _free_port

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
N = 8
NB = 1 << 20           # the pending Iallreduce: 1 Mi floats
PATHS = ("push", "pull", "zero_copy")


def _worker(rank, n, port, q):
    import torch.distributed as dist
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n)
        torch.cuda.set_device(0)
        mxompi.init(0)

        def ag(b):
            out = [None] * n
            dist.all_gather_object(out, b)
            return out
        A = mxompi.Comm(rank, n, ag, device=0, staging_bytes=STAGING_ONE_CHUNK)
        B = mxompi.Comm(rank, n, ag, device=0, staging_bytes=16 << 20)
        for c in (A, B):
            c.set_timeout(60.0)
        A.set_autotune(False)
        st = torch.cuda.current_stream().cuda_stream
        # two application streams with work queued (never waited for here)
        busy = []
        for k in range(2):
            s = torch.cuda.Stream()
            t = torch.ones(16 << 20, device="cuda")
            with torch.cuda.stream(s):
                for _ in range(200):
                    t.mul_(1.0000001)
            busy.append((s, t))
        # an Iallreduce pending on B, on a high-priority stream of its own
        sb_stream = torch.cuda.Stream(priority=-1)
        xb = torch.from_numpy(gen_big("FLOAT", "SUM", NB, 777 + rank)).to("cuda")
        yb = torch.empty_like(xb)
        torch.cuda.synchronize()
        req = B.iallreduce(xb.data_ptr(), yb.data_ptr(), NB, "FLOAT", "SUM", "auto", sb_stream.cuda_stream)
        res = {}
        x = torch.from_numpy(gen_big("FLOAT", "SUM", C256, 1000 + rank)).to("cuda")
        out = torch.empty_like(x)
        for path in PATHS:
            if path == "zero_copy":
                A.set_reg_min(256 << 10)
                A.set_protocol("auto")
            else:
                A.set_reg_min(0)
                A.set_protocol(path)
            before = A.stats()
            A.allreduce(x.data_ptr(), out.data_ptr(), C256, "FLOAT", "SUM", "auto", st)
            torch.cuda.synchronize()
            after = A.stats()
            res[path] = (digest(out.cpu().numpy()), after["zero_copy_calls"] - before["zero_copy_calls"],
                         after["staged_calls"] - before["staged_calls"])
        req.wait()
        req.free()
        res["iallreduce"] = digest(yb.cpu().numpy())
        for s, _ in busy:
            s.synchronize()
        A.close()
        B.close()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc() + str(e)))


def _expected_allreduce(seed0, count, alg, nb=False):
    L = oracle_lib.oracle()
    fn = L.mxo_iallreduce if nb else L.mxo_allreduce
    fn.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    xs = [gen_big("FLOAT", "SUM", count, seed0 + r) for r in range(N)]
    outs = [np.empty(count * 4, np.uint8) for _ in range(N)]
    assert fn(alg, mxompi.OP["SUM"], mxompi.TYPE["FLOAT"], N, count, (vp * N)(*[x.ctypes.data for x in xs]),
              (vp * N)(*[o.ctypes.data for o in outs])) == 0
    return [digest(o)[0] for o in outs]


def test_staged_and_zero_copy_waits_with_extra_streams_and_a_pending_iallreduce():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, N, port, q)) for r in range(N)]
    for p in procs:
        p.start()
    got = {}
    try:
        exp = _expected_allreduce(1000, C256, 0)
        exp_nb = _expected_allreduce(777, NB, 0, nb=True)
        for _ in range(N):
            rank, status, payload = q.get(timeout=280)
            assert status == "ok", payload
            got[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=60 if len(got) == N else 5)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    for r in range(N):
        for path in PATHS:
            (h, _), zc, staged = got[r][path]
            assert h == exp[r], (r, path)
            assert (zc, staged) == ((1, 0) if path == "zero_copy" else (0, 1)), (r, path, zc, staged)
        assert got[r]["iallreduce"][0] == exp_nb[r], r
