"""The resident reduce service behind mx_reduce2_sync (round 4,
csrc/mx_service.hip): calls of <= 2 MiB on an idle non-default stream are served
by a kernel that stays resident instead of a launch per call -- workgroup 0
alone up to 64 KiB, the whole grid above.

Bit-exact vs the op oracle (op_base_functions.c restated; op values
parity-unpinned) for every element family the service takes, at
ragged sizes up to its 2 MiB cap and either side of the 64 KiB solo bound; pairs interleaved (the service is rebound
to each pair), pauses longer than its 100 us idle exit (relaunch), a call over
the cap and a misaligned call (launch path), and the per-call counters show
which calls the service took; a relaunch behind a held hardware queue
launches instead of waiting."""
import time

import numpy as np
import pytest

import golden_io
import mxompi
import oracle_lib

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

PAIRS = [("SUM", "FLOAT"), ("MAX", "DOUBLE"), ("BXOR", "UINT16_T"), ("MAXLOC", "FLOAT_INT"),
         ("PROD", "C_FLOAT_COMPLEX"), ("LAND", "BOOL"), ("MIN", "INT8_T"), ("SUM", "INT64_T")]
SVC_MAX = 2 << 20            # kSvcMaxBytes
SVC_SOLO = 64 << 10          # kSvcSoloBytes: above, the whole grid takes the command


def _gen(op, t, count, seed):
    rng = np.random.default_rng(seed)
    es = mxompi.type_size(t)
    if t in ("FLOAT", "DOUBLE"):
        v = (rng.uniform(-1, 1, count) * 10.0 ** rng.uniform(-6, 6, count)).astype(np.float32 if t == "FLOAT"
                                                                                     else np.float64)
        v[rng.integers(0, count, max(1, count // 50))] = np.nan
        return v.view(np.uint8)
    if t == "C_FLOAT_COMPLEX":
        return rng.uniform(0.5, 1.5, 2 * count).astype(np.float32).view(np.uint8)
    if t == "FLOAT_INT":
        p = np.zeros(count, dtype=[("v", "<f4"), ("k", "<i4")])
        p["v"] = rng.integers(0, 4, count)
        p["k"] = rng.integers(-9, 9, count)
        return p.view(np.uint8)
    if t == "BOOL":
        return rng.integers(0, 2, count, dtype=np.uint8)
    return rng.integers(0, 256, count * es, dtype=np.uint8)


def _check(op, t, count, seed, stream, off=0):
    O = oracle_lib.oracle()
    es = mxompi.type_size(t)
    a, b = _gen(op, t, count, seed), _gen(op, t, count, seed + 1)
    A = torch.zeros(count * es + 16, dtype=torch.uint8, device="cuda")
    B = torch.zeros(count * es + 16, dtype=torch.uint8, device="cuda")
    A[off:off + count * es] = torch.from_numpy(a).cuda()
    B[off:off + count * es] = torch.from_numpy(b).cuda()
    torch.cuda.synchronize()
    mxompi.reduce2_sync(op, t, A.data_ptr() + off, B.data_ptr() + off, count, stream.cuda_stream)
    got = B[off:off + count * es].cpu().numpy()       # read back with no further sync
    exp = b.copy()
    assert O.mxo_reduce2(mxompi.OP[op], mxompi.TYPE[t], a.ctypes.data, exp.ctypes.data, count, 1) == 0
    golden_io.assert_op_equal(got, exp, mxompi.OP[op], mxompi.TYPE[t], f"service {op} {t} count {count}")


def test_service_serves_and_matches_the_oracle():
    mxompi.init(0)
    s = torch.cuda.Stream()
    st0, served0, launches0 = mxompi.op_service_stats()
    calls = 0
    for rnd in range(2):
        for op, t in PAIRS:
            es = mxompi.type_size(t)
            for count in (1, 17, 1000, 4099, SVC_SOLO // es, SVC_SOLO // es + 1, (256 << 10) // es + 3,
                          SVC_MAX // es):
                _check(op, t, count, 100 * rnd + count, s)
                calls += 1
        time.sleep(0.01)                               # > the 100 us idle exit: the next call relaunches
    st, served, launches = mxompi.op_service_stats()
    assert st == 1, "service unusable on this box"
    assert served - served0 == calls, (served - served0, calls)
    assert launches - launches0 >= 2 * len(PAIRS)      # rebound to every pair, every round
    # not served: over the cap, misaligned buffers
    _check("SUM", "FLOAT", SVC_MAX // 4 + 4, 7, s)
    _check("SUM", "FLOAT", (8 << 20) // 4, 9, s)
    _check("SUM", "FLOAT", 5000, 8, s, off=4)
    O = oracle_lib.oracle()
    assert mxompi.op_service_stats()[1] == served
    del O


@pytest.mark.parametrize("n", [4096, 16384, 262144], ids=["32KiB_solo", "128KiB_grid", "2MiB_grid"])
def test_service_back_to_back_same_buffers(n):
    """A segmented-ring-like sequence: 500 calls on the same buffers, each
    folding the previous result -- every call must see the last one's result
    (the service's acquire after a command, its release before done), by
    workgroup 0 alone and by the whole grid."""
    mxompi.init(0)
    s = torch.cuda.Stream()
    a = torch.ones(n, dtype=torch.int64, device="cuda")
    b = torch.zeros(n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    served0 = mxompi.op_service_stats()[1]
    for i in range(500):
        mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), n, s.cuda_stream)
        if i % 100 == 99:      # the host reads the result straight after the call
            assert int(b[n - 1].item()) == i + 1 and int(b[0].item()) == i + 1
    assert torch.all(b == 500).item()
    assert mxompi.op_service_stats()[1] - served0 == 500


def test_service_three_buffer_form():
    """mx_reduce3_sync (the op component's 3-buffer handler): out = in1 OP in2
    through the service (aligned, <= 2 MiB) and through the launch (misaligned
    or larger),
    bit-exact vs the oracle's 3-buffer functions, out read straight after."""
    mxompi.init(0)
    s = torch.cuda.Stream()
    O = oracle_lib.oracle()
    served0 = mxompi.op_service_stats()[1]
    served_calls = 0
    for op, t in PAIRS:
        es = mxompi.type_size(t)
        for count, off in ((1000, 0), (SVC_MAX // es, 0), (SVC_MAX // es + 1, 0), (3001, 4)):
            a, b = _gen(op, t, count, 5 + count), _gen(op, t, count, 6 + count)
            A = torch.zeros(count * es + 16, dtype=torch.uint8, device="cuda")
            B = torch.zeros(count * es + 16, dtype=torch.uint8, device="cuda")
            C = torch.full((count * es + 16,), 0x5A, dtype=torch.uint8, device="cuda")
            A[off:off + count * es] = torch.from_numpy(a).cuda()
            B[off:off + count * es] = torch.from_numpy(b).cuda()
            torch.cuda.synchronize()
            mxompi.reduce3_sync(op, t, A.data_ptr() + off, B.data_ptr() + off, C.data_ptr() + off, count,
                                s.cuda_stream)
            got = C[off:off + count * es].cpu().numpy()
            exp = np.zeros(count * es, np.uint8)
            assert O.mxo_reduce3(mxompi.OP[op], mxompi.TYPE[t], a.ctypes.data, b.ctypes.data, exp.ctypes.data,
                                 count, 1) == 0
            golden_io.assert_op_equal(got, exp, mxompi.OP[op], mxompi.TYPE[t], f"3-buffer {op} {t} {count}+{off}")
            served_calls += off == 0 and count * es <= SVC_MAX   # else a launch
    assert mxompi.op_service_stats()[1] - served0 == served_calls


def test_service_never_waits_on_a_held_queue():
    """A relaunch (after the idle exit) whose hardware queue is held -- here
    by a wave spinning on the service's own stream until released, as a
    kernel waiting for this very thread would hold it -- must not wait: the
    call launches instead, bit-exact, and the service serves again once the
    queue is free."""
    import ctypes
    mxompi.init(0)
    # the calls' own stream at the highest priority: a launch on it is not
    # queued behind the held ordinary-priority queue of the service
    L = mxompi.lib()
    hp = ctypes.c_void_p()
    mxompi.check(L.mx_stream_create(ctypes.byref(hp)), "mx_stream_create")
    sp = hp.value
    n = 1000
    a = torch.ones(n, dtype=torch.int64, device="cuda")
    b = torch.zeros(n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), n, sp)
    time.sleep(0.01)                                   # past the idle exit: the next call relaunches
    held0 = mxompi.op_service_held()[1]
    try:
        mxompi.debug_hold_service(20000)
        t0 = time.time()
        for _ in range(20):
            mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), n, sp)
        dt = time.time() - t0
        held = mxompi.op_service_held()[1] - held0
        print(f"20 calls with the service's queue held: {dt * 1e3:.1f} ms, launches held {held}")
        assert dt < 5.0, dt                            # the holder waits 20 s
        assert held >= 1                               # the relaunch did meet the held queue
        assert mxompi.op_service_held()[0]             # that kernel is still queued
        mxompi.check(L.mx_stream_sync(hp), "mx_stream_sync")
        assert torch.all(b == 21).item()
    finally:
        mxompi.debug_release()
    torch.cuda.synchronize()                           # the holder, then the held kernel (EXIT first)
    served0 = mxompi.op_service_stats()[1]
    for _ in range(3):                                 # served again
        mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), n, sp)
    assert torch.all(b == 24).item()
    assert mxompi.op_service_stats()[1] - served0 == 3
    assert not mxompi.op_service_held()[0]
    mxompi.check(L.mx_stream_destroy(hp), "mx_stream_destroy")


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _irecv_reduce_send_worker(rank, n, port, q, env):
    """Irecv; Reduce_local x k (relaunching the service between them); Send;
    Wait -- on both ranks.  The receive spins on a channel stream at the
    highest priority, the queues the service also uses; a
    service that waited for a queue held by that receive would never get to
    the Send, and neither rank would finish."""
    import os
    import torch.distributed as dist
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    os.environ.update(env)
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n)
        torch.cuda.set_device(0)
        mxompi.init(0)

        def ag(b):
            out = [None] * n
            dist.all_gather_object(out, b)
            return out

        comm = mxompi.Comm(rank, n, ag, device=0, staging_bytes=1 << 20)
        comm.set_timeout(20.0)
        s = torch.cuda.Stream()
        peer = 1 - rank
        m = 4096
        a = torch.ones(m, dtype=torch.int64, device="cuda")
        b = torch.zeros(m, dtype=torch.int64, device="cuda")
        t0 = time.time()
        out = []
        for it in range(6):
            nb = 4096 if it % 2 == 0 else 3 << 20          # eager, rendezvous
            x = torch.full((nb,), (rank + 3 * it) & 0xff, dtype=torch.uint8, device="cuda")
            y = torch.zeros(nb, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            r = comm.irecv(y.data_ptr(), nb, peer, tag=it)
            dist.barrier()                                  # both receives are spinning
            for _ in range(5):
                time.sleep(0.001)                           # past the idle exit: each call relaunches
                mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), m, s.cuda_stream)
            sreq = comm.isend(x.data_ptr(), nb, peer, tag=it)
            r.wait(); sreq.wait(); r.free(); sreq.free()
            out.append(int(y[0].item()) == ((peer + 3 * it) & 0xff) and bool(torch.all(y == y[0]).item()))
        res = {"seconds": time.time() - t0, "ok": out, "b": int(b[0].item()), "b_all": bool(torch.all(b == b[0]).item()),
               "held": mxompi.op_service_held()[1], "stats": mxompi.op_service_stats()}
        comm.close()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc() + str(e)))


@pytest.mark.parametrize("env", [{"MX_OP_SERVICE": "1"}, {"MX_OP_SERVICE": "0"}], ids=["served", "launched"])
def test_service_irecv_reduce_send_does_not_deadlock(env):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_irecv_reduce_send_worker, args=(r, 2, port, q, env)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(2):
            rank, status, payload = q.get(timeout=120)
            assert status == "ok", payload
            got[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=30 if len(got) == 2 else 5)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    for r in range(2):
        print(f"rank {r}: {got[r]['seconds']:.2f} s, launches held {got[r]['held']}, service {got[r]['stats']}")
        assert got[r]["ok"] == [True] * 6
        assert got[r]["b"] == 30 and got[r]["b_all"]
        assert got[r]["seconds"] < 15.0, got[r]["seconds"]
        if env["MX_OP_SERVICE"] == "1":
            assert got[r]["stats"][1] > 0                  # the service took calls


def test_service_concurrent_threads():
    """MPI_THREAD_MULTIPLE: four threads, each with its own stream and pair,
    call the blocking reduce 150 times on their own buffers -- the service
    is rebound between pairs as calls interleave; every result exact."""
    import threading
    mxompi.init(0)
    jobs = [("SUM", "INT64_T", 3000), ("BXOR", "UINT32_T", 70000), ("MAX", "INT32_T", 300000), ("SUM", "INT32_T", 17)]
    errs = []

    def run(op, t, n, seed):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            dt = {"INT64_T": torch.int64, "UINT32_T": torch.int32, "INT32_T": torch.int32}[t]
            g = torch.Generator(device="cpu").manual_seed(seed)
            a = torch.randint(-1000, 1000, (n,), generator=g, dtype=dt).cuda()
            b = torch.zeros(n, dtype=dt, device="cuda")
            ref = b.clone()
            torch.cuda.synchronize()
            for i in range(150):
                mxompi.reduce2_sync(op, t, a.data_ptr(), b.data_ptr(), n, s.cuda_stream)
                if op == "SUM":
                    ref += a
                elif op == "BXOR":
                    ref ^= a
                else:
                    ref = torch.maximum(ref, a)
            torch.cuda.synchronize()
            if not torch.equal(b, ref):
                errs.append(f"{op} {t} {n}: mismatch")
        except Exception as e:  # noqa: BLE001
            errs.append(f"{op} {t} {n}: {e!r}")

    served0 = mxompi.op_service_stats()[1]
    th = [threading.Thread(target=run, args=(op, t, n, 10 + i)) for i, (op, t, n) in enumerate(jobs)]
    for x in th:
        x.start()
    for x in th:
        x.join(120)
    assert not errs, errs
    print(f"served {mxompi.op_service_stats()[1] - served0} of {150 * len(jobs)}")


def test_service_keeps_stream_order():
    """Work still queued on the caller's stream when the call is made (here a
    wave holding the stream for 20 ms, then a fill of `in`): the call is not
    served -- the launch runs after that work, as on any stream -- and the
    result sees the fill.  On an idle stream the next call is served."""
    mxompi.init(0)
    s = torch.cuda.Stream()
    n = 5000
    a = torch.ones(n, dtype=torch.int64, device="cuda")
    b = torch.zeros(n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), n, s.cuda_stream)   # served: b = 1
    served0 = mxompi.op_service_stats()[1]
    mxompi.debug_hold(s.cuda_stream, 20)           # leaves by itself after 20 ms
    with torch.cuda.stream(s):
        a.fill_(5)
    mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), n, s.cuda_stream)   # launched after the fill
    assert torch.all(b == 6).item()
    assert mxompi.op_service_stats()[1] == served0
    mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), n, s.cuda_stream)   # idle again: served
    assert torch.all(b == 11).item()
    assert mxompi.op_service_stats()[1] == served0 + 1


def test_service_resumes_after_a_launch():
    """A call over the cap launches on the caller's stream; the small calls
    straight after it must be served again (the launched kernel's stream
    turns idle a little after its completion word -- the idleness check
    waits that out instead of launching every call that follows)."""
    mxompi.init(0)
    s = torch.cuda.Stream()
    big = torch.ones((8 << 20) // 8, dtype=torch.int64, device="cuda")
    bigo = torch.zeros_like(big)
    a = torch.ones(1000, dtype=torch.int64, device="cuda")
    b = torch.zeros(1000, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    for rnd in range(3):
        mxompi.reduce2_sync("SUM", "INT64_T", big.data_ptr(), bigo.data_ptr(), big.numel(), s.cuda_stream)
        served0 = mxompi.op_service_stats()[1]
        for _ in range(20):
            mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), 1000, s.cuda_stream)
        assert mxompi.op_service_stats()[1] - served0 == 20, rnd
    assert torch.all(b == 60).item() and torch.all(bigo == 3).item()


_NT_MARK_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import mxompi, oracle_lib
mxompi.init(0)
O = oracle_lib.oracle()
side = torch.cuda.Stream()
bad = []
# kFusedMarkMax = 1024 * 256 - 16 elements: with every launch forced onto the
# 64-lane non-temporal instances the grid is up to 4x kMarkFlags workgroups
for op, t, count in (("SUM", "FLOAT", 1024 * 256 - 16), ("SUM", "FLOAT", 1024 * 64 + 5), ("MAX", "DOUBLE", 1024 * 256 - 17),
                     ("MAXLOC", "LONG_DOUBLE_INT", 1024 * 256 - 16), ("BXOR", "UINT8_T", 1024 * 256 - 16)):
    es = mxompi.type_size(t)
    rng = np.random.default_rng(count)
    a = rng.integers(0, 7, count * es, dtype=np.uint8)
    b = rng.integers(0, 7, count * es, dtype=np.uint8)
    if t in ("FLOAT", "DOUBLE"):
        a = rng.uniform(-1, 1, count).astype(np.float32 if t == "FLOAT" else np.float64).view(np.uint8)
        b = rng.uniform(-1, 1, count).astype(np.float32 if t == "FLOAT" else np.float64).view(np.uint8)
    for rep in range(20):
        A = torch.from_numpy(a).cuda(); B = torch.from_numpy(b).cuda()
        torch.cuda.synchronize()
        # the call returns with inout final for every agent: read it at once
        # through a copy on another (non-blocking) stream, which is not ordered
        # after the launch on the default stream
        mxompi.reduce2_sync(op, t, A.data_ptr(), B.data_ptr(), count, 0)
        with torch.cuda.stream(side):
            got = B.cpu().numpy()
        exp = b.copy()
        assert O.mxo_reduce2(mxompi.OP[op], mxompi.TYPE[t], a.ctypes.data, exp.ctypes.data, count, 1) == 0
        if not np.array_equal(got, exp):
            bad.append((op, t, count, rep)); break
print("BAD", bad)
sys.exit(1 if bad else 0)
"""


def test_fused_mark_with_nt_forced_everywhere():
    """with MX_NT_MIN_BYTES=0 every launch takes the 64-lane
    non-temporal instances, whose grids near kFusedMarkMax exceed the
    kMarkFlags per-workgroup flags.  The mark must not ride on such a grid
    (mark_fit drops it and the call waits through the marker kernel): every
    result bit-exact vs the oracle."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MX_NT_MIN_BYTES="0", MX_OP_SERVICE="0")
    p = subprocess.run([sys.executable, "-c", _NT_MARK_CHILD, os.path.join(root, "zhpe-ompi_amd"),
                        os.path.join(root, "tests")], capture_output=True, text=True, env=env, timeout=200)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
