"""GPU: point-to-point transfers of device buffers (SURVEY 8(f) row 1:
MPI_Send / MPI_Recv / MPI_Isend / MPI_Irecv / MPI_Sendrecv / persistent
MPI_Send_init / MPI_Recv_init, derived datatypes through the device
convertor).

n processes share the one GPU.  Payload bytes must arrive unchanged for
every size (0 bytes, sub-vector tails, several times the mailbox), every
alignment (user pointers offset by 1..15 bytes), many messages in flight
per pair (more than the envelope ring), a ring shift, an all-to-all, and
sends to self; truncation completes with MPI's error and leaves the channel
usable; tags match out of order within a pair (unexpected eager messages
stashed on the device, unexpected rendezvous messages deferred with their
data left at the sender until a receive clears them); derived datatypes on either side match the
reference convertor's packed stream (golden vectors).
"""
import os

import numpy as np
import pytest

import golden_io
import mxompi
from test_coll_gpu import _dev, _free_port

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

BASIC, RECS = golden_io.ddt_records()
REC = {r["name"]: r for r in RECS}
SIZES = [0, 1, 15, 16, 17, 4097, 65536, 3 * (1 << 20) + 7]
SHIFT = 10 * (1 << 20) + 13


def _data(seed, nbytes):
    return np.random.default_rng(seed).integers(0, 256, nbytes, dtype=np.uint8)


def _p2p_worker(rank, n, port, q):
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

        comm = mxompi.Comm(rank, n, ag, device=0, staging_bytes=1 << 20)
        comm.set_timeout(30.0)
        res = {}
        right, left = (rank + 1) % n, (rank - 1) % n

        # (1) ring shift with MPI_Sendrecv, 5x the mailbox
        x = _dev(_data(rank, SHIFT))
        y = torch.zeros(SHIFT, dtype=torch.uint8, device="cuda")
        got = comm.sendrecv(x.data_ptr(), SHIFT, right, y.data_ptr(), SHIFT, left, 7, 7)
        res["shift"] = (got, y.cpu().numpy().tobytes())

        # (2) sizes x misalignment, 0 -> 1 (blocking on both sides)
        if rank == 0:
            for k, nb in enumerate(SIZES):
                src = _dev(_data(100 + k, nb + 32))
                comm.send(src.data_ptr() + (k * 3) % 16, nb, 1, tag=k)
        elif rank == 1:
            outs = []
            for k, nb in enumerate(SIZES):
                dst = torch.zeros(nb + 64, dtype=torch.uint8, device="cuda")
                off = (k * 5) % 16
                got = comm.recv(dst.data_ptr() + off, nb + 16, 0, tag=k)
                outs.append((got, dst.cpu().numpy()[off: off + nb].tobytes()))
            res["sizes"] = outs

        # (3) many in flight on one pair: 20 x 300 KB, posted before any wait
        M, MB = 20, 300 * 1024 + 3
        if rank == 0:
            bufs = [_dev(_data(200 + k, MB)) for k in range(M)]
            reqs = [comm.isend(b.data_ptr(), MB, 1, tag=k) for k, b in enumerate(bufs)]
            for r in reqs:
                r.wait()
                r.free()
        elif rank == 1:
            bufs = [torch.zeros(MB, dtype=torch.uint8, device="cuda") for _ in range(M)]
            reqs = [comm.irecv(b.data_ptr(), MB, 0, tag=k) for k, b in enumerate(bufs)]
            st = []
            for r in reqs:
                r.wait()
                st.append(r.status())
                r.free()
            res["inflight"] = (st, [b.cpu().numpy().tobytes() for b in bufs])

        # (4) truncation completes with MPI_ERR_TRUNCATE; tags match out of
        # order within the pair (pml/ob1's matching): a receive whose tag is
        # not the next message's stashes that message on the device and a
        # later receive takes it, oldest first
        if rank == 0:
            comm.send(_dev(_data(300, 1000)).data_ptr(), 1000, 1, tag=5)
            comm.send(_dev(_data(301, 1000)).data_ptr(), 1000, 1, tag=9)
            comm.send(_dev(_data(302, 1000)).data_ptr(), 1000, 1, tag=5)
            comm.send(_dev(_data(303, 2000)).data_ptr(), 2000, 1, tag=7)
            comm.send(_dev(_data(304, 700)).data_ptr(), 700, 1, tag=8)
            big = _dev(_data(305, 300 << 10))      # rendezvous: moves once a receive clears it
            rb = comm.isend(big.data_ptr(), 300 << 10, 1, tag=3)
            comm.send(_dev(_data(306, 64)).data_ptr(), 64, 1, tag=4)
            rb.wait()
            rb.free()
        elif rank == 1:
            d = torch.zeros(2000, dtype=torch.uint8, device="cuda")
            errs, data = [], []
            try:
                comm.recv(d.data_ptr(), 600, 0, tag=5)
            except mxompi.MxError as e:
                errs.append(e.rc)
            data.append(d.cpu().numpy()[:600].tobytes())
            for tag in (7, 5, -1, 8):          # 7 stashes the 9 and the second 5
                r = comm.irecv(d.data_ptr(), 2000, 0, tag=tag)
                r.wait()
                st = r.status()
                r.free()
                errs.append(st)
                data.append(d.cpu().numpy()[:st[0]].tobytes())
            # tag 4 defers the 300 KiB tag-3 rendezvous envelope (its data
            # stays with the sender) and takes the 64 B behind it; tag 3 then
            # clears the deferred message
            r = comm.irecv(d.data_ptr(), 64, 0, tag=4)
            r.wait()
            errs.append(r.status())
            data.append(d.cpu().numpy()[:64].tobytes())
            r.free()
            big = torch.zeros(300 << 10, dtype=torch.uint8, device="cuda")
            r = comm.irecv(big.data_ptr(), 300 << 10, 0, tag=3)
            r.wait()
            errs.append(r.status())
            data.append(big.cpu().numpy().tobytes())
            r.free()
            res["errs"] = errs
            res["tagdata"] = data

        # (5) persistent pair started three times on fresh data
        P = 1 << 20
        pb = torch.zeros(P, dtype=torch.uint8, device="cuda")
        if rank == 0:
            req = comm.isend(pb.data_ptr(), P, 1, tag=1, persistent=True)
        elif rank == 1:
            req = comm.irecv(pb.data_ptr(), P, 0, tag=1, persistent=True)
        reps = []
        for it in range(3):
            if rank == 0:
                pb.copy_(_dev(_data(400 + it, P)))
                torch.cuda.synchronize()
            if rank in (0, 1):
                req.start()
                req.wait()
                if rank == 1:
                    reps.append(pb.cpu().numpy().tobytes())
        if rank in (0, 1):
            req.free()
        res["persistent"] = reps

        # (6) derived datatypes on either side (golden reference types)
        tv = REC["vector_f64_b3_s5"]
        dt = mxompi.Datatype(tv["desc"].tobytes(), tv["nrec"], tv["size"], tv["lb"], tv["ub"])
        nbp = tv["size"] * tv["count"]
        if rank == 0:
            user = _dev(tv["user"])
            r1 = comm.isend_ddt(user.data_ptr() - tv["true_lb"], tv["count"], dt, 1, tag=2)
            pk = _dev(tv["packed"])
            r2 = comm.isend(pk.data_ptr(), nbp, 1, tag=3)
            r1.wait(); r2.wait(); r1.free(); r2.free()
        elif rank == 1:
            got = torch.zeros(nbp, dtype=torch.uint8, device="cuda")
            r1 = comm.irecv(got.data_ptr(), nbp, 0, tag=2)
            ub = _dev(tv["prefill"])
            r2 = comm.irecv_ddt(ub.data_ptr() - tv["true_lb"], tv["count"], dt, 0, tag=3)
            r1.wait(); r2.wait(); r1.free(); r2.free()
            res["ddt"] = (got.cpu().numpy().tobytes(), ub.cpu().numpy().tobytes())
        dt.close()

        # (7) all-to-all of isend / irecv, sends to self included
        A = 77777
        sb = [_dev(_data(1000 * rank + p, A)) for p in range(n)]
        rb = [torch.zeros(A, dtype=torch.uint8, device="cuda") for _ in range(n)]
        reqs = [comm.irecv(rb[p].data_ptr(), A, p, tag=11) for p in range(n)]
        reqs += [comm.isend(sb[p].data_ptr(), A, p, tag=11) for p in range(n)]
        for r in reqs:
            r.wait()
            r.free()
        res["a2a"] = [b.cpu().numpy().tobytes() for b in rb]

        # (7b) the same with rendezvous-sized messages: every rank's pick
        # kernels serve the CTS of several destinations in whatever order
        # they arrive (receives posted in descending source order)
        A2 = 300001
        sb = [_dev(_data(2000 * rank + p, A2)) for p in range(n)]
        rb = [torch.zeros(A2, dtype=torch.uint8, device="cuda") for _ in range(n)]
        reqs = [comm.isend(sb[p].data_ptr(), A2, p, tag=12) for p in range(n)]
        reqs += [comm.irecv(rb[p].data_ptr(), A2, p, tag=12) for p in reversed(range(n))]
        for r in reqs:
            r.wait()
            r.free()
        res["a2a_rndv"] = [b.cpu().numpy().tobytes() for b in rb]

        # (7c) rendezvous messages matched out of order within a pair: 0 -> 1
        # sends R1 (tag 31), R2 (tag 32), an eager E (tag 33), R3 (tag 31);
        # 1 takes 33 (deferring R1 and R2), 32, ANY_TAG (the oldest held:
        # R1), then 31 (R3, from the envelope ring) into a short buffer
        sizes = {31: (1 << 20) + 5, 32: 600 << 10, 33: 5000}
        if rank == 0:
            msgs = [(31, 401, sizes[31]), (32, 402, sizes[32]), (33, 403, sizes[33]), (31, 404, 2 << 20)]
            bufs = [_dev(_data(seed, nb)) for _, seed, nb in msgs]
            reqs = [comm.isend(b.data_ptr(), nb, 1, tag=t) for b, (t, _, nb) in zip(bufs, msgs)]
            for r in reqs:
                r.wait()
                r.free()
        elif rank == 1:
            out = []
            for tag, cap in ((33, 8000), (32, 700 << 10), (-1, 2 << 20), (31, (1 << 20) + 3)):
                b = torch.zeros(cap, dtype=torch.uint8, device="cuda")
                r = comm.irecv(b.data_ptr(), cap, 0, tag=tag)
                try:
                    r.wait()
                    st = r.status()
                except mxompi.MxError as e:
                    st = (e.rc, r.status())
                r.free()
                nb = st[0] if isinstance(st[0], int) and st[0] >= 0 else st[1][0]
                out.append((st, b.cpu().numpy()[:nb].tobytes()))
            res["rndv_order"] = out

        # (7d) rendezvous to self, receive posted after the send
        S = (1 << 20) + 17
        x = _dev(_data(7000 + rank, S))
        y = torch.zeros(S, dtype=torch.uint8, device="cuda")
        rs = comm.isend(x.data_ptr(), S, rank, tag=41)
        rr = comm.irecv(y.data_ptr(), S, rank, tag=41)
        rr.wait(); rs.wait(); rr.free(); rs.free()
        res["self_rndv"] = y.cpu().numpy().tobytes()

        # (8) MPI_ANY_SOURCE: every other rank sends two messages to rank 0,
        # which takes all but one with non-blocking ANY_SOURCE receives
        # posted at once and the last with a blocking one; after a barrier a
        # specific-source receive still finds the next message of its pair
        B = 50001
        if rank == 0:
            M = 2 * (n - 1)
            rbs = [torch.zeros(B, dtype=torch.uint8, device="cuda") for _ in range(M)]
            reqs = [comm.irecv(b.data_ptr(), B, mxompi.ANY_SOURCE, tag=-1) for b in rbs[:M - 1]]
            got = []
            for r, b in zip(reqs, rbs):
                r.wait()
                got.append((r.source(), r.status(), b.cpu().numpy().tobytes()))
                r.free()
            nb = comm.recv(rbs[M - 1].data_ptr(), B, mxompi.ANY_SOURCE, tag=-1)
            res["any"] = (got, nb, rbs[M - 1].cpu().numpy().tobytes())
        else:
            for k in range(2):
                m = _dev(_data(5000 + 10 * rank + k, B))
                comm.send(m.data_ptr(), B, 0, tag=20 + k)
        dist.barrier()
        if rank == n - 1:
            m = _dev(_data(6000, B))
            comm.send(m.data_ptr(), B, 0, tag=22)
        elif rank == 0:
            d = torch.zeros(B, dtype=torch.uint8, device="cuda")
            comm.recv(d.data_ptr(), B, n - 1, tag=22)
            res["any_specific"] = d.cpu().numpy().tobytes()

        # (9) MPI_ANY_SOURCE with a specific tag: rank 1's message (tag 50)
        # is already in rank 0's mailbox when rank 0 posts ANY_SOURCE / tag 51,
        # which only rank 2 sends, later -- the receive must take rank 2's
        # message, and the next ANY_SOURCE / tag 50 receive rank 1's
        if n >= 3:
            C = 3001
            if rank == 1:
                m = _dev(_data(8100, C))
                comm.send(m.data_ptr(), C, 0, tag=50)
            dist.barrier()
            if rank == 0:
                b51 = torch.zeros(C, dtype=torch.uint8, device="cuda")
                r51 = comm.irecv(b51.data_ptr(), C, mxompi.ANY_SOURCE, tag=51)
            dist.barrier()
            if rank == 2:
                m = _dev(_data(8200, C))
                comm.send(m.data_ptr(), C, 0, tag=51)
            if rank == 0:
                r51.wait()
                first = (r51.source(), r51.status(), b51.cpu().numpy().tobytes())
                r51.free()
                b50 = torch.zeros(C, dtype=torch.uint8, device="cuda")
                r50 = comm.irecv(b50.data_ptr(), C, mxompi.ANY_SOURCE, tag=50)
                r50.wait()
                res["any_tag"] = [first, (r50.source(), r50.status(), b50.cpu().numpy().tobytes())]
                r50.free()
            dist.barrier()

        comm.close()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc() + str(e)))


def _run(n):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_p2p_worker, args=(r, n, port, q)) for r in range(n)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(n):
            rank, status, payload = q.get(timeout=300)
            assert status == "ok", payload
            out[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=60 if len(out) == n else 5)
            if p.is_alive():      # a failed rank leaves its peers waiting: end them
                p.terminate()
                p.join(timeout=10)
    return out


@pytest.mark.parametrize("n", [2, 3, 4])
def test_point_to_point(n):
    got = _run(n)
    for r in range(n):
        nb, data = got[r]["shift"]
        assert nb == SHIFT
        assert data == _data((r - 1) % n, SHIFT).tobytes(), f"shift rank {r}"
    for k, (nb, data) in enumerate(got[1]["sizes"]):
        exp = _data(100 + k, SIZES[k] + 32)[(k * 3) % 16: (k * 3) % 16 + SIZES[k]]
        assert nb == SIZES[k] and data == exp.tobytes(), f"size {SIZES[k]}"
    st, bufs = got[1]["inflight"]
    assert st == [(300 * 1024 + 3, k) for k in range(20)]
    for k, b in enumerate(bufs):
        assert b == _data(200 + k, 300 * 1024 + 3).tobytes(), f"in-flight message {k}"
    # MX_ERR_TRUNCATE; then tag 7 (stashing 9 and 5), the stashed 5, the
    # stashed 9 for MPI_ANY_TAG (oldest), 8; tag 4 past the deferred 300 KiB
    # rendezvous message, which tag 3 then takes
    assert got[1]["errs"] == [-9, (2000, 7), (1000, 5), (1000, 9), (700, 8), (64, 4), (300 << 10, 3)], \
        got[1]["errs"]
    want = [_data(300, 1000)[:600], _data(303, 2000), _data(302, 1000), _data(301, 1000), _data(304, 700),
            _data(306, 64), _data(305, 300 << 10)]
    assert got[1]["tagdata"] == [w.tobytes() for w in want]
    for r in range(n):
        for p in range(n):
            assert got[r]["a2a_rndv"][p] == _data(2000 * p + r, 300001).tobytes(), f"rendezvous a2a {p} -> {r}"
        assert got[r]["self_rndv"] == _data(7000 + r, (1 << 20) + 17).tobytes(), f"rendezvous to self {r}"
    order = got[1]["rndv_order"]
    assert [o[0] for o in order] == [(5000, 33), (600 << 10, 32), ((1 << 20) + 5, 31),
                                     (-9, ((1 << 20) + 3, 31))], [o[0] for o in order]
    assert order[0][1] == _data(403, 5000).tobytes()
    assert order[1][1] == _data(402, 600 << 10).tobytes()
    assert order[2][1] == _data(401, (1 << 20) + 5).tobytes()
    assert order[3][1] == _data(404, 2 << 20)[:(1 << 20) + 3].tobytes()
    for it, b in enumerate(got[1]["persistent"]):
        assert b == _data(400 + it, 1 << 20).tobytes(), f"persistent start {it}"
    tv = REC["vector_f64_b3_s5"]
    packed, unpacked = got[1]["ddt"]
    np.testing.assert_array_equal(np.frombuffer(packed, np.uint8), tv["packed"])
    np.testing.assert_array_equal(np.frombuffer(unpacked, np.uint8), tv["unpacked"])
    for r in range(n):
        for p in range(n):
            assert got[r]["a2a"][p] == _data(1000 * p + r, 77777).tobytes(), f"a2a {p} -> {r}"
    if n >= 3:
        (s51, st51, d51), (s50, st50, d50) = got[0]["any_tag"]
        assert (s51, tuple(st51)[:2]) == (2, (3001, 51)) and d51 == _data(8200, 3001).tobytes(), (s51, st51)
        assert (s50, tuple(st50)[:2]) == (1, (3001, 50)) and d50 == _data(8100, 3001).tobytes(), (s50, st50)
    got0, nb_last, last = got[0]["any"]
    expect = {(p, k): _data(5000 + 10 * p + k, 50001).tobytes() for p in range(1, n) for k in range(2)}
    seen = {p: 0 for p in range(1, n)}
    payloads = []
    for src, (nb, tag), data in got0:
        assert 1 <= src < n, src
        k = seen[src]                                   # per-pair order holds under ANY_SOURCE
        assert (nb, tag) == (50001, 20 + k) and data == expect[(src, k)], f"ANY_SOURCE message {k} of {src}"
        seen[src] += 1
        payloads.append(data)
    assert nb_last == 50001
    payloads.append(last)
    assert sorted(payloads) == sorted(expect.values())
    assert got[0]["any_specific"] == _data(6000, 50001).tobytes()


def _busy_worker(rank, n, port, q):
    """A receive posted first spins on the device until its message comes;
    the peer only sends after work on each of 8 ordinary streams of its own
    (more than there are hardware queues, so they share every ordinary
    queue) has finished.  The channel streams run at the highest priority,
    on queues no ordinary stream shares, so that work is never queued behind
    the spinning receive."""
    import time
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

        comm = mxompi.Comm(rank, n, ag, device=0, staging_bytes=1 << 20)
        comm.set_timeout(20.0)
        busy = [torch.cuda.Stream() for _ in range(8)]
        Z = [torch.zeros(1024, device="cuda") for _ in busy]
        peer = 1 - rank
        t0 = time.time()
        out = {}
        for nb in (4096, 3 << 20):            # eager, rendezvous
            x = _dev(_data(900 + rank, nb))
            y = torch.zeros(nb, dtype=torch.uint8, device="cuda")
            r = comm.irecv(y.data_ptr(), nb, peer, tag=nb & 0xffff)
            dist.barrier()                    # both receives are spinning now
            for s_, z in zip(busy, Z):
                with torch.cuda.stream(s_):
                    z.add_(1.0)
                s_.synchronize()
            s = comm.isend(x.data_ptr(), nb, peer, tag=nb & 0xffff)
            r.wait(); s.wait(); r.free(); s.free()
            out[nb] = y.cpu().numpy().tobytes()
        res = {"seconds": time.time() - t0, "out": out, "z": [float(z[0]) for z in Z]}
        comm.close()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc() + str(e)))


def test_channel_streams_do_not_block_ordinary_streams():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_busy_worker, args=(r, 2, port, q)) for r in range(2)]
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
        assert got[r]["seconds"] < 10.0, got[r]["seconds"]
        assert got[r]["z"] == [2.0] * 8
        for nb in (4096, 3 << 20):
            assert got[r]["out"][nb] == _data(900 + (1 - r), nb).tobytes(), (r, nb)


# ---------------------------------------------------------------------------
# round 5: the hardware-queue budget is per device, not
# per communicator.  The send and receive channel streams are the device's,
# shared by every communicator; the rendezvous stream is made only by a
# communicator that sends one.  Two p2p communicators with crossing
# Irecv / Send pairs in opposite posting orders on the two ranks, an
# Iallreduce in flight on a request stream beside them, and 8 ordinary
# streams busy meanwhile -- within the pool's 4 queues per priority.
def _two_comm_worker(rank, n, port, q):
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

        comms = []
        for _ in range(2):
            c = mxompi.Comm(rank, n, ag, device=0, staging_bytes=8 << 20)
            c.set_timeout(30.0)
            comms.append(c)
        A, B = comms
        peer = 1 - rank
        side = torch.cuda.Stream()
        nb = 64 << 10                                   # eager
        res = {}
        for it in range(3):
            bufs = {k: torch.zeros(nb, dtype=torch.uint8, device="cuda") for k in ("a", "b")}
            msgs = {k: _dev(_data(1000 * it + 10 * rank + (k == "b"), nb)) for k in ("a", "b")}
            x = _dev(_data(700 + 10 * it + rank, 1 << 20)).view(torch.int32)
            y = torch.zeros_like(x)
            torch.cuda.synchronize()
            # rank 0 posts A's receive first, rank 1 B's; each sends in the other order
            order = ("a", "b") if rank == 0 else ("b", "a")
            reqs = [(A if k == "a" else B).irecv(bufs[k].data_ptr(), nb, peer, 5 if k == "a" else 6) for k in order]
            ia = A.iallreduce(x.data_ptr(), y.data_ptr(), x.numel(), "INT32_T", "SUM", "auto", side.cuda_stream)
            busy = [torch.cuda.Stream() for _ in range(8)]
            zs = []
            for s in busy:
                with torch.cuda.stream(s):
                    z = torch.ones(1 << 20, device="cuda")
                    zs.append((z * 2).sum())
            for k in reversed(order):
                (A if k == "a" else B).send(msgs[k].data_ptr(), nb, peer, 5 if k == "a" else 6)
            for r in reqs:
                r.wait()
                r.free()
            ia.wait()
            ia.free()
            torch.cuda.synchronize()
            res[it] = {k: bufs[k].cpu().numpy().tobytes() for k in bufs}
            res[it]["sum"] = y.cpu().numpy().tobytes()
            res[it]["z"] = [float(z) for z in zs]
        B.close()
        A.close()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc() + str(e)))


def test_two_p2p_communicators_crossing_with_an_iallreduce():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_two_comm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(2):
            rank, status, payload = q.get(timeout=200)
            assert status == "ok", payload
            got[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=30 if len(got) == 2 else 5)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    nb = 64 << 10
    for it in range(3):
        xs = [_data(700 + 10 * it + r, 1 << 20).view(np.int32).astype(np.int64) for r in range(2)]
        s = (xs[0] + xs[1]).astype(np.int32).tobytes()
        for r in range(2):
            p = 1 - r
            assert got[r][it]["a"] == _data(1000 * it + 10 * p, nb).tobytes(), (it, r, "a")
            assert got[r][it]["b"] == _data(1000 * it + 10 * p + 1, nb).tobytes(), (it, r, "b")
            assert got[r][it]["sum"] == s, (it, r)
            assert got[r][it]["z"] == [float(2 << 20)] * 8


# ---------------------------------------------------------------------------
# round 5: receives that yield.  Receive kernels share one
# receive stream per device; a receive waiting for its message used to hold
# back every receive posted after it, so a blocking rendezvous send whose
# receive was posted second could never be cleared -- legal MPI programs
# deadlocked.  Each case below did; each must now finish with every payload
# exact, and messages must still go to the earliest posted receive that
# matches them (pml/ob1's order) when a displaced receive runs again.
BIG = (1 << 20) + 5        # rendezvous


def _yield_worker(rank, n, port, q):
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

        A = mxompi.Comm(rank, n, ag, device=0, staging_bytes=1 << 20)
        B = mxompi.Comm(rank, n, ag, device=0, staging_bytes=1 << 20)
        for c in (A, B):
            c.set_timeout(30.0)
        right, left = (rank + 1) % n, (rank - 1) % n
        res = {}

        def buf():
            return torch.zeros(BIG, dtype=torch.uint8, device="cuda")

        # (1) halo: both receives posted, then blocking sends leftwards first
        for it in range(3):
            fl, fr = buf(), buf()
            r1 = A.irecv(fl.data_ptr(), BIG, left, tag=1)
            r2 = A.irecv(fr.data_ptr(), BIG, right, tag=2)
            A.send(_dev(_data(10 * it + 100 * rank + 2, BIG)).data_ptr(), BIG, left, tag=2)
            A.send(_dev(_data(10 * it + 100 * rank + 1, BIG)).data_ptr(), BIG, right, tag=1)
            for r in (r1, r2):
                r.wait()
                r.free()
            res[("halo", it)] = (fl.cpu().numpy().tobytes(), fr.cpu().numpy().tobytes())
        res["relaunch_halo"] = A.stats(reset=True)["p2p_relaunches"]
        dist.barrier()

        # (2) one source, tags crossed: the second-posted receive's message comes first
        if rank == 0:
            ba, bb = buf(), buf()
            ra = A.irecv(ba.data_ptr(), BIG, 1, tag=10)
            rb = A.irecv(bb.data_ptr(), BIG, 1, tag=11)
            ra.wait(); rb.wait(); ra.free(); rb.free()
            res["cross"] = (ba.cpu().numpy().tobytes(), bb.cpu().numpy().tobytes())
            res["relaunch_cross"] = A.stats(reset=True)["p2p_relaunches"]
        elif rank == 1:
            A.send(_dev(_data(511, BIG)).data_ptr(), BIG, 0, tag=11)
            A.send(_dev(_data(510, BIG)).data_ptr(), BIG, 0, tag=10)
        dist.barrier()

        # (3) two communicators, the receive of the second-posted one first
        if rank == 0:
            ba, bb = buf(), buf()
            ra = A.irecv(ba.data_ptr(), BIG, 1, tag=5)
            rb = B.irecv(bb.data_ptr(), BIG, 1, tag=6)
            rb.wait(); ra.wait(); ra.free(); rb.free()
            res["comms"] = (ba.cpu().numpy().tobytes(), bb.cpu().numpy().tobytes())
            res["relaunch_comms"] = A.stats(reset=True)["p2p_relaunches"] + B.stats(reset=True)["p2p_relaunches"]
        elif rank == 1:
            B.send(_dev(_data(606, BIG)).data_ptr(), BIG, 0, tag=6)
            A.send(_dev(_data(605, BIG)).data_ptr(), BIG, 0, tag=5)
        dist.barrier()

        # (4) order after a yield: R1 (source 1, tag 7) yields to R2 (source
        # 2); R3 (source 1, tag 7, posted after R1) runs while R1 is
        # displaced and must leave source 1's first tag-7 message to R1
        if rank == 0:
            b1, b2, b3 = buf(), buf(), buf()
            r1 = A.irecv(b1.data_ptr(), BIG, 1, tag=7)
            r2 = A.irecv(b2.data_ptr(), BIG, 2, tag=8)
            r3 = A.irecv(b3.data_ptr(), BIG, 1, tag=7)
            r2.wait()
            r1.wait()
            r3.wait()
            st = [r.status() for r in (r1, r2, r3)]
            for r in (r1, r2, r3):
                r.free()
            res["order"] = (st, [b.cpu().numpy().tobytes() for b in (b1, b2, b3)])
            res["relaunch_order"] = A.stats(reset=True)["p2p_relaunches"]
        elif rank == 2:
            A.send(_dev(_data(708, BIG)).data_ptr(), BIG, 0, tag=8)
            dist.send(torch.ones(1), dst=1)          # R1 has yielded by now
        elif rank == 1:
            dist.recv(torch.zeros(1), src=2)
            A.send(_dev(_data(701, BIG)).data_ptr(), BIG, 0, tag=7)
            A.send(_dev(_data(702, BIG)).data_ptr(), BIG, 0, tag=7)
        dist.barrier()

        # (5) MPI_ANY_SOURCE posted first, a specific receive behind it whose
        # blocking sender comes first
        if rank == 0:
            ba, bb = buf(), buf()
            ra = A.irecv(ba.data_ptr(), BIG, -1, tag=20)
            rb = A.irecv(bb.data_ptr(), BIG, 2, tag=21)
            rb.wait(); ra.wait()
            res["any"] = (ra.source(), ba.cpu().numpy().tobytes(), bb.cpu().numpy().tobytes())
            res["relaunch_any"] = A.stats(reset=True)["p2p_relaunches"]
            ra.free(); rb.free()
        elif rank == 2:
            A.send(_dev(_data(821, BIG)).data_ptr(), BIG, 0, tag=21)
            dist.send(torch.ones(1), dst=1)
        elif rank == 1:
            dist.recv(torch.zeros(1), src=2)
            A.send(_dev(_data(820, BIG)).data_ptr(), BIG, 0, tag=20)
        dist.barrier()

        # (6) a blocking collective progresses a yielded receive: rank 0
        # enters an allreduce with R1 yielded; rank 1 joins it only after its
        # blocking send to R1 completed
        x = torch.full((1024,), rank + 1, dtype=torch.int32, device="cuda")
        y = torch.zeros_like(x)
        if rank == 0:
            ba, bb = buf(), buf()
            ra = A.irecv(ba.data_ptr(), BIG, 1, tag=60)
            rb = A.irecv(bb.data_ptr(), BIG, 2, tag=61)
            B.allreduce(x.data_ptr(), y.data_ptr(), 1024, "INT32_T", "SUM")
            ra.wait(); rb.wait()
            res["coll"] = (ba.cpu().numpy().tobytes(), bb.cpu().numpy().tobytes(), int(y[0]),
                           A.stats(reset=True)["p2p_relaunches"])
            ra.free(); rb.free()
        else:
            if rank == 2:
                A.send(_dev(_data(861, BIG)).data_ptr(), BIG, 0, tag=61)
                dist.send(torch.ones(1), dst=1)
            else:
                dist.recv(torch.zeros(1), src=2)
                A.send(_dev(_data(860, BIG)).data_ptr(), BIG, 0, tag=60)
            B.allreduce(x.data_ptr(), y.data_ptr(), 1024, "INT32_T", "SUM")
        dist.barrier()
        B.close()
        A.close()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc() + str(e)))


def test_receives_yield_to_receives_posted_after_them():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n = 3
    procs = [ctx.Process(target=_yield_worker, args=(r, n, port, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(n):
            rank, status, payload = q.get(timeout=200)
            assert status == "ok", payload
            got[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=30 if len(got) == n else 5)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    for r in range(n):
        left, right = (r - 1) % n, (r + 1) % n
        for it in range(3):
            fl, fr = got[r][("halo", it)]
            assert fl == _data(10 * it + 100 * left + 1, BIG).tobytes(), ("halo from left", r, it)
            assert fr == _data(10 * it + 100 * right + 2, BIG).tobytes(), ("halo from right", r, it)
    assert got[0]["cross"] == (_data(510, BIG).tobytes(), _data(511, BIG).tobytes())
    assert got[0]["comms"] == (_data(605, BIG).tobytes(), _data(606, BIG).tobytes())
    st, data = got[0]["order"]
    assert [tuple(s)[:2] for s in st] == [(BIG, 7), (BIG, 8), (BIG, 7)], st
    assert data == [_data(701, BIG).tobytes(), _data(708, BIG).tobytes(), _data(702, BIG).tobytes()]
    src, da, db = got[0]["any"]
    assert src == 1 and da == _data(820, BIG).tobytes() and db == _data(821, BIG).tobytes()
    # the yields happened: a receive launched again in every case (the halo
    # on some rank: whose receive waits first depends on timing)
    assert sum(got[r]["relaunch_halo"] for r in range(n)) >= 1
    for case in ("cross", "comms", "order", "any"):
        assert got[0]["relaunch_" + case] >= 1, (case, got[0]["relaunch_" + case])
    assert got[0]["relaunch_order"] >= 2      # R1, then R3 behind R1's second launch
    ca, cb, total, relaunched = got[0]["coll"]
    assert ca == _data(860, BIG).tobytes() and cb == _data(861, BIG).tobytes() and total == 6
    assert relaunched >= 1


def _yield_worker2(rank, n, port, q):
    """A datatype receive, a persistent receive and mx_test-driven progress
    across a yield, and the order rule with eager messages (set aside in the
    device stash rather than deferred)."""
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

        A = mxompi.Comm(rank, n, ag, device=0, staging_bytes=1 << 20)
        A.set_timeout(30.0)
        res = {}

        def buf(nb=BIG):
            return torch.zeros(nb, dtype=torch.uint8, device="cuda")

        def first_from_2_then_1(tag2, tag1, nb1, payload1):
            """rank 2 sends (blocking) first; rank 1 sends only after it"""
            if rank == 2:
                A.send(_dev(_data(900 + tag2, BIG)).data_ptr(), BIG, 0, tag=tag2)
                dist.send(torch.ones(1), dst=1)
            elif rank == 1:
                dist.recv(torch.zeros(1), src=2)
                A.send(_dev(payload1).data_ptr(), nb1, 0, tag=tag1)

        # (1) a datatype receive yields, runs again, unpacks once more
        tv = REC["vector_f64_b3_s5"]
        dt = mxompi.Datatype(tv["desc"].tobytes(), tv["nrec"], tv["size"], tv["lb"], tv["ub"])
        nbp = tv["size"] * tv["count"]
        if rank == 0:
            ub = _dev(tv["prefill"])
            r1 = A.irecv_ddt(ub.data_ptr() - tv["true_lb"], tv["count"], dt, 1, tag=30)
            b2 = buf()
            r2 = A.irecv(b2.data_ptr(), BIG, 2, tag=31)
            r2.wait(); r1.wait(); r1.free(); r2.free()
            res["ddt"] = (ub.cpu().numpy().tobytes(), b2.cpu().numpy().tobytes())
            res["relaunch_ddt"] = A.stats(reset=True)["p2p_relaunches"]
        first_from_2_then_1(31, 30, nbp, tv["packed"])
        dist.barrier()

        # (2) progress from mx_test only
        if rank == 0:
            b1, b2 = buf(), buf()
            r1 = A.irecv(b1.data_ptr(), BIG, 1, tag=40)
            r2 = A.irecv(b2.data_ptr(), BIG, 2, tag=41)
            import time
            t0 = time.time()
            while not (r1.test() and r2.test()):
                assert time.time() - t0 < 60
            r1.free(); r2.free()
            res["test"] = (b1.cpu().numpy().tobytes(), b2.cpu().numpy().tobytes())
            res["relaunch_test"] = A.stats(reset=True)["p2p_relaunches"]
        first_from_2_then_1(41, 40, BIG, _data(940, BIG))
        dist.barrier()

        # (3) a persistent receive yields on each of its starts
        pb = buf()
        if rank == 0:
            pr = A.irecv(pb.data_ptr(), BIG, 1, tag=50, persistent=True)
        reps = []
        for it in range(2):
            if rank == 0:
                pr.start()
                b2 = buf()
                r2 = A.irecv(b2.data_ptr(), BIG, 2, tag=51)
                r2.wait(); pr.wait(); r2.free()
                reps.append(pb.cpu().numpy().tobytes())
            first_from_2_then_1(51, 50, BIG, _data(950 + it, BIG))
            dist.barrier()
        if rank == 0:
            pr.free()
            res["persistent"] = reps
            res["relaunch_persistent"] = A.stats(reset=True)["p2p_relaunches"]

        # (4) the order rule with eager messages: both of source 1's tag-7
        # messages land in the stash while R1 is displaced
        E = 64 << 10
        if rank == 0:
            b1, b2, b3 = buf(E), buf(), buf(E)
            r1 = A.irecv(b1.data_ptr(), E, 1, tag=7)
            r2 = A.irecv(b2.data_ptr(), BIG, 2, tag=8)
            r3 = A.irecv(b3.data_ptr(), E, 1, tag=7)
            r2.wait(); r1.wait(); r3.wait()
            res["order"] = [b.cpu().numpy().tobytes() for b in (b1, b3)]
            res["relaunch_order"] = A.stats(reset=True)["p2p_relaunches"]
            for r in (r1, r2, r3):
                r.free()
        elif rank == 2:
            A.send(_dev(_data(908, BIG)).data_ptr(), BIG, 0, tag=8)
            dist.send(torch.ones(1), dst=1)
        elif rank == 1:
            dist.recv(torch.zeros(1), src=2)
            A.send(_dev(_data(971, E)).data_ptr(), E, 0, tag=7)
            A.send(_dev(_data(972, E)).data_ptr(), E, 0, tag=7)
        dist.barrier()

        # (4b) mx_request_stream_wait on a receive that yields: the host waits
        # (progressing the yield) and work on the stream sees the payload
        if rank == 0:
            b1, b2 = buf(), buf()
            r1 = A.irecv(b1.data_ptr(), BIG, 1, tag=80)
            r2 = A.irecv(b2.data_ptr(), BIG, 2, tag=81)
            side = torch.cuda.Stream()
            r1.stream_wait(side.cuda_stream)
            with torch.cuda.stream(side):
                c1 = b1.clone()
            side.synchronize()
            r1.wait(); r2.wait(); r1.free(); r2.free()
            res["stream_wait"] = (c1.cpu().numpy().tobytes(), b2.cpu().numpy().tobytes())
        first_from_2_then_1(81, 80, BIG, _data(980, BIG))
        dist.barrier()

        # (5) MPI_Waitall / Waitany / Testall / Testany over receives that
        # yield (ompi/request/req_wait.c, req_test.c semantics)
        if rank == 0:
            b1, b2 = buf(), buf()
            r1 = A.irecv(b1.data_ptr(), BIG, 1, tag=60)
            r2 = A.irecv(b2.data_ptr(), BIG, 2, tag=61)
            flag0 = mxompi.testall([r1, None, r2])        # nothing sent yet: no change
            first = mxompi.waitany([None, r1, r2])       # rank 2's comes first
            second = mxompi.waitany([None, r1, r2])
            none_left = mxompi.waitany([None, r1, r2])
            any_done = mxompi.testany([r1, r2])
            r1.free(); r2.free()
            res["any_all"] = (flag0, first, second, none_left, any_done, b1.cpu().numpy().tobytes(),
                              b2.cpu().numpy().tobytes())
        first_from_2_then_1(61, 60, BIG, _data(960, BIG))
        dist.barrier()
        right, left = (rank + 1) % n, (rank - 1) % n
        fl, fr = buf(), buf()
        reqs = [A.irecv(fl.data_ptr(), BIG, left, tag=1), A.irecv(fr.data_ptr(), BIG, right, tag=2)]
        A.send(_dev(_data(1100 + rank, BIG)).data_ptr(), BIG, left, tag=2)
        reqs.append(A.isend(_dev(_data(1200 + rank, BIG)).data_ptr(), BIG, right, tag=1))
        mxompi.waitall(reqs)
        done = mxompi.testall(reqs)                     # inactive: true
        for r in reqs:
            r.free()
        res["waitall"] = (done, fl.cpu().numpy().tobytes(), fr.cpu().numpy().tobytes())
        dist.barrier()
        dt.close()
        A.close()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc() + str(e)))


def test_yield_with_datatypes_test_polling_and_persistent():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n = 3
    procs = [ctx.Process(target=_yield_worker2, args=(r, n, port, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(n):
            rank, status, payload = q.get(timeout=200)
            assert status == "ok", payload
            got[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=30 if len(got) == n else 5)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    tv = REC["vector_f64_b3_s5"]
    ub, b2 = got[0]["ddt"]
    np.testing.assert_array_equal(np.frombuffer(ub, np.uint8), tv["unpacked"])
    assert b2 == _data(931, BIG).tobytes()
    assert got[0]["test"] == (_data(940, BIG).tobytes(), _data(941, BIG).tobytes())
    assert got[0]["persistent"] == [_data(950, BIG).tobytes(), _data(951, BIG).tobytes()]
    assert got[0]["order"] == [_data(971, 64 << 10).tobytes(), _data(972, 64 << 10).tobytes()]
    for case, least in (("ddt", 1), ("test", 1), ("persistent", 2), ("order", 2)):
        assert got[0]["relaunch_" + case] >= least, (case, got[0]["relaunch_" + case])
    assert got[0]["stream_wait"] == (_data(980, BIG).tobytes(), _data(981, BIG).tobytes())
    flag0, first, second, none_left, any_done, b1, b2 = got[0]["any_all"]
    assert (flag0, first, second, none_left, any_done) == (False, 2, 1, mxompi.UNDEFINED, (True, mxompi.UNDEFINED))
    assert b1 == _data(960, BIG).tobytes() and b2 == _data(961, BIG).tobytes()
    for r in range(n):
        done, fl, fr = got[r]["waitall"]
        assert done and fl == _data(1200 + (r - 1) % n, BIG).tobytes() and fr == _data(1100 + (r + 1) % n, BIG).tobytes()


def _tables_worker(rank, n, port, q):
    """16 unexpected eager messages wait in the device stash and 64
    unexpected rendezvous messages as deferred envelopes (their data stays
    with the sender); the receive that meets one unexpected message more than
    the stash holds completes with MX_ERR_TAG (the documented bound) and the
    channel stays usable."""
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

        A = mxompi.Comm(rank, n, ag, device=0, staging_bytes=1 << 20)
        A.set_timeout(30.0)
        res = {}
        E, R = 1000, 300 << 10
        if rank == 0:
            keep = []
            reqs = []
            for t in range(200, 217):                   # 17 eager: one more than the stash
                b = _dev(_data(t, E)); keep.append(b)
                reqs.append(A.isend(b.data_ptr(), E, 1, tag=t))
            b = _dev(_data(299, E)); keep.append(b)
            reqs.append(A.isend(b.data_ptr(), E, 1, tag=299))
            for t in range(400, 464):                   # 64 rendezvous: the deferred table
                b = _dev(_data(t, R)); keep.append(b)
                reqs.append(A.isend(b.data_ptr(), R, 1, tag=t))
            b = _dev(_data(499, E)); keep.append(b)
            reqs.append(A.isend(b.data_ptr(), E, 1, tag=499))
            mxompi.waitall(reqs)
            for r in reqs:
                r.free()
        else:
            d = torch.zeros(R, dtype=torch.uint8, device="cuda")
            r = A.irecv(d.data_ptr(), E, 0, tag=299)    # stashes 200..215, then meets 216
            try:
                r.wait()
                res["overflow"] = ("no error", r.status())
            except mxompi.MxError as e:
                res["overflow"] = (e.rc, tuple(r.status())[:2], d[:E].cpu().numpy().tobytes())
            r.free()
            res["299"] = (A.recv(d.data_ptr(), E, 0, tag=299), d[:E].cpu().numpy().tobytes())
            res["499"] = (A.recv(d.data_ptr(), E, 0, tag=499), d[:E].cpu().numpy().tobytes())   # defers 400..463
            got = {}
            for t in list(range(215, 199, -1)) + list(range(463, 399, -1)):
                nb = E if t < 300 else R
                got[t] = (A.recv(d.data_ptr(), nb, 0, tag=t), d[:nb].cpu().numpy().tobytes())
            res["held"] = got
        dist.barrier()
        A.close()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc() + str(e)))


def test_unexpected_message_tables_and_their_bound():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tables_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(2):
            rank, status, payload = q.get(timeout=200)
            assert status == "ok", payload
            got[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=30 if len(got) == 2 else 5)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    E, R = 1000, 300 << 10
    res = got[1]
    rc, st, data = res["overflow"]
    assert rc == -10 and st == (E, 216) and data == _data(216, E).tobytes(), (rc, st)   # MX_ERR_TAG
    assert res["299"] == (E, _data(299, E).tobytes())
    assert res["499"] == (E, _data(499, E).tobytes())
    for t, (nb, data) in res["held"].items():
        want = _data(t, E if t < 300 else R)
        assert nb == len(want) and data == want.tobytes(), t


def _plan(seed, n, per_rank=12):
    """Every rank's sends (destination, tag, size, payload seed) in send
    order, and every rank's receive posting order: a list of (source, tag)."""
    import random
    rng = random.Random(seed)
    sends = {r: [] for r in range(n)}
    for r in range(n):
        for k in range(per_rank):
            dst = rng.choice([d for d in range(n) if d != r])
            tag = rng.randrange(3)
            size = rng.choice([2048 + rng.randrange(64), (300 << 10) + rng.randrange(64)])
            sends[r].append((dst, tag, size, 10000 * seed + 100 * r + k))
    posts = {}
    for d in range(n):
        incoming = [(s, t) for s in range(n) for (dst, t, _, _) in sends[s] if dst == d]
        rng.shuffle(incoming)
        posts[d] = incoming
    return sends, posts


def _random_worker(rank, n, port, q, seed):
    import torch.distributed as dist
    import random
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n)
        torch.cuda.set_device(0)
        mxompi.init(0)

        def ag(b):
            out = [None] * n
            dist.all_gather_object(out, b)
            return out

        A = mxompi.Comm(rank, n, ag, device=0, staging_bytes=1 << 20)
        A.set_timeout(30.0)
        sends, posts = _plan(seed, n)
        cap = (300 << 10) + 64
        bufs, reqs = [], []
        for (src, tag) in posts[rank]:                   # every receive posted before any send
            b = torch.zeros(cap, dtype=torch.uint8, device="cuda")
            bufs.append(b)
            reqs.append(A.irecv(b.data_ptr(), cap, src, tag=tag))
        dist.barrier()
        order = list(range(len(sends[rank])))
        random.Random(seed * 7 + rank).shuffle(order)    # blocking sends in a random order...
        per_pair = {}
        for k in order:                                  # ...but each (dst, tag) stream in plan order
            dst, tag, _, _ = sends[rank][k]
            per_pair.setdefault((dst, tag), []).append(k)
        for key in per_pair:
            per_pair[key].sort()
        for k in order:
            dst, tag, _, _ = sends[rank][k]
            kk = per_pair[(dst, tag)].pop(0)
            _, _, size, ps = sends[rank][kk]
            x = _dev(_data(ps, size))
            A.send(x.data_ptr(), size, dst, tag=tag)
        mxompi.waitall(reqs)
        got = [(tuple(r.status())[:2], b[: r.status()[0]].cpu().numpy().tobytes()) for r, b in zip(reqs, bufs)]
        for r in reqs:
            r.free()
        relaunched = A.stats(reset=True)["p2p_relaunches"]
        dist.barrier()
        A.close()
        dist.destroy_process_group()
        q.put((rank, "ok", {"got": got, "relaunched": relaunched}))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc() + str(e)))


@pytest.mark.parametrize("n,seed", [(3, 1), (3, 2), (3, 3), (4, 4), (4, 5)])
def test_randomised_posting_orders_complete_in_match_order(n, seed):
    """A safe program (every receive posted before any send) with receives
    posted in a random order and blocking sends in a random order: it must
    complete, and the k-th receive posted for (source, tag) must get the k-th
    message sent on (source, tag) (MPI's non-overtaking rule)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_random_worker, args=(r, n, port, q, seed)) for r in range(n)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(n):
            rank, status, payload = q.get(timeout=200)
            assert status == "ok", payload
            got[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=30 if len(got) == n else 5)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    sends, posts = _plan(seed, n)
    for d in range(n):
        streams = {}
        for s in range(n):
            for (dst, tag, size, ps) in sends[s]:
                if dst == d:
                    streams.setdefault((s, tag), []).append((size, ps))
        for i, (src, tag) in enumerate(posts[d]):
            size, ps = streams[(src, tag)].pop(0)
            (nb, t), data = got[d]["got"][i]
            assert (nb, t) == (size, tag) and data == _data(ps, size).tobytes(), (d, i, src, tag)
    print(f"seed {seed}: receive launches that yielded per rank",
          [got[r]["relaunched"] for r in range(n)])          # (-s / the log shows how much yielding ran)


def _wild_plan(seed, n, per_rank=12):
    """Like _plan, with each rank's blocking-send sequence fixed here and part
    of each destination's receives made wildcards.  Specific receives take the
    first messages of their (source, tag) stream and are posted first (random
    order); per destination the remaining messages are covered by (source,
    MPI_ANY_TAG) receives, then by (MPI_ANY_SOURCE, MPI_ANY_TAG) ones, posted
    in that order -- whatever the arrival order, every receive then has a
    message (a safe program)."""
    import random
    rng = random.Random(seed)
    sends, _ = _plan(seed, n, per_rank)
    seqs = {}
    for r in range(n):                                   # the blocking-send sequence of rank r
        order = list(range(per_rank))
        rng.shuffle(order)
        per = {}
        for k in range(per_rank):
            dst, tag, _, _ = sends[r][k]
            per.setdefault((dst, tag), []).append(k)
        seqs[r] = [per[(sends[r][k][0], sends[r][k][1])].pop(0) for k in order]
    posts = {}
    for d in range(n):
        streams = {}
        for s in range(n):
            for k in seqs[s]:
                dst, tag, _, _ = sends[s][k]
                if dst == d:
                    streams.setdefault((s, tag), []).append(k)
        specific, by_src, anyany = [], [], []
        for (s, t), ks in streams.items():
            keep = rng.randrange(len(ks) + 1)
            specific += [(s, t)] * keep
            for _ in ks[keep:]:
                (by_src if rng.random() < 0.5 else anyany).append((s, -1))
        rng.shuffle(specific)
        rng.shuffle(by_src)
        posts[d] = specific + by_src + [(-1, -1)] * len(anyany)
    return sends, seqs, posts


def _wild_worker(rank, n, port, q, seed):
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

        A = mxompi.Comm(rank, n, ag, device=0, staging_bytes=1 << 20)
        A.set_timeout(30.0)
        sends, seqs, posts = _wild_plan(seed, n)
        cap = (300 << 10) + 64
        bufs, reqs = [], []
        for (src, tag) in posts[rank]:
            b = torch.zeros(cap, dtype=torch.uint8, device="cuda")
            bufs.append(b)
            reqs.append(A.irecv(b.data_ptr(), cap, src, tag=tag))
        dist.barrier()
        for k in seqs[rank]:
            dst, tag, size, ps = sends[rank][k]
            A.send(_dev(_data(ps, size)).data_ptr(), size, dst, tag=tag)
        mxompi.waitall(reqs)
        got = [(r.source(), tuple(r.status())[:2], b[: r.status()[0]].cpu().numpy().tobytes())
               for r, b in zip(reqs, bufs)]
        for r in reqs:
            r.free()
        relaunched = A.stats(reset=True)["p2p_relaunches"]
        dist.barrier()
        A.close()
        dist.destroy_process_group()
        q.put((rank, "ok", {"got": got, "relaunched": relaunched}))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc() + str(e)))


@pytest.mark.parametrize("n,seed", [(3, 11), (3, 12), (4, 13)])
def test_randomised_wildcard_receives_keep_non_overtaking(n, seed):
    """Every message is delivered once, to a receive whose pattern matches it;
    specific receives get their streams' messages in order; and for two
    receives that both got messages from one source and could each have taken
    the other's, the earlier-posted one got the earlier-sent message (MPI's
    non-overtaking rule, which ob1's matching keeps)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_wild_worker, args=(r, n, port, q, seed)) for r in range(n)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(n):
            rank, status, payload = q.get(timeout=200)
            assert status == "ok", payload
            got[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=30 if len(got) == n else 5)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    sends, seqs, posts = _wild_plan(seed, n)
    for d in range(n):
        # every message to d by payload: (source, tag, position in the source's send sequence)
        msgs = {}
        for s in range(n):
            pos = 0
            for k in seqs[s]:
                dst, tag, size, ps = sends[s][k]
                if dst == d:
                    msgs[_data(ps, size).tobytes()] = (s, tag, pos)
                    pos += 1
        seen = []
        for i, (src_pat, tag_pat) in enumerate(posts[d]):
            source, (nb, tag), data = got[d]["got"][i]
            assert data in msgs, (d, i)
            s, t, pos = msgs.pop(data)
            assert (source, tag, nb) == (s, t, len(data)), (d, i)
            assert src_pat in (-1, s) and tag_pat in (-1, t), (d, i, src_pat, tag_pat, s, t)
            seen.append((src_pat, tag_pat, s, t, pos))
        assert not msgs, f"undelivered at {d}"
        for i in range(len(seen)):
            for j in range(i + 1, len(seen)):
                pi, ti, si, tgi, posi = seen[i]
                pj, tj, sj, tgj, posj = seen[j]
                both = (si == sj and pi in (-1, sj) and ti in (-1, tgj) and pj in (-1, si) and tj in (-1, tgi))
                assert not both or posi < posj, ("overtaken", d, i, j, seen[i], seen[j])
    print(f"seed {seed}: receive launches that yielded per rank", [got[r]["relaunched"] for r in range(n)])
