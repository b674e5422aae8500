"""Multi-rank communicators through the MCA components and the mini-host.

* CPU (gloo, world_size 2 and 3): host buffers.  The harness's MPI entry
  points dispatch through comm->c_coll; on a machine without a GPU the
  coll/mi355x component declines at init_query (no device), every slot stays
  with the host stand-ins of coll/tuned, coll/basic and coll/libnbc, and the
  results equal the oracle's orders for them.  Covers the bootstrap exchange
  (a host allgather over torch.distributed/gloo, the role the saved lower
  allgather plays inside Open MPI) and the N>1 host logic without a GPU.
* GPU (n processes sharing the one GPU): device buffers go through
  coll/mi355x -- on the device above coll_mi355x_host_max_kb, on the saved
  host module through host copies at or below it -- and must be
  bit-identical to the coll/tuned algorithm the oracle restates either way.
* Nonblocking and persistent forms (MPI_Iallreduce, MPI_Ireduce, MPI_Iscan,
  MPI_Iexscan, MPI_Ireduce_scatter_block posted together, then MPI_Test /
  MPI_Wait; MPI_Allreduce_init + MPI_Start twice) must match coll/libnbc's
  orders on either path.
"""
import ctypes
import os
import socket

import numpy as np
import pytest

vp, ci, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gen(kind, count, rank):
    rng = np.random.default_rng(1234 + 17 * rank + count)
    if kind == "int":
        return rng.integers(-1000, 1000, count).astype(np.int32)
    v = (rng.uniform(-1, 1, count) * 10.0 ** rng.uniform(-6, 6, count)).astype(np.float32)
    v[rng.integers(0, count, max(1, count // 50))] = np.nan
    return v


def _worker(rank, n, port, use_gpu, q):
    try:
        import torch
        import torch.distributed as dist
        import minihost
        import mxompi
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n)

        @minihost.AG
        def ag(send, recv, nbytes, ctx):
            out = [None] * n
            dist.all_gather_object(out, ctypes.string_at(send, nbytes))
            blob = b"".join(out)
            ctypes.memmove(recv, blob, len(blob))
            return 0

        if use_gpu:
            torch.cuda.set_device(0)
            mxompi.init(0)
        H = minihost.host(with_components=True)
        comm = H.mxh_comm_create(rank, n, ag, None)
        owners = {s: H.mxh_comm_slot_owner(comm, s.encode()).decode()
                  for s in ("allreduce", "reduce", "scan", "exscan", "reduce_scatter_block", "reduce_scatter",
                            "allgather", "bcast", "iallreduce", "ireduce", "iscan", "iexscan",
                            "ireduce_scatter_block", "allreduce_init")}
        f32, i32 = minihost.dtype(H, "MPI_FLOAT"), minihost.dtype(H, "MPI_INT")
        SUM, MAX = minihost.op(H, "MPI_SUM"), minihost.op(H, "MPI_MAX")
        res = {"owners": owners}
        count = 5003

        def buf(a):
            if use_gpu:
                return torch.from_numpy(a.copy()).cuda()
            return torch.from_numpy(a.copy())

        def out_like(a, nel=None):
            t = torch.zeros(nel if nel is not None else a.size, dtype=torch.float32 if a.dtype == np.float32
                            else torch.int32)
            return t.cuda() if use_gpu else t

        for kind, dt, op in (("int", i32, SUM), ("flt", f32, SUM), ("flt", f32, MAX)):
            x = _gen(kind, count, rank)
            X = buf(x)
            R = out_like(x)
            assert H.mxh_allreduce(X.data_ptr(), R.data_ptr(), count, dt, op, comm) == 0
            res[("allreduce", kind, op == MAX)] = R.cpu().numpy().tobytes()
            R = out_like(x)
            assert H.mxh_reduce(X.data_ptr(), R.data_ptr(), count, dt, op, n - 1, comm) == 0
            res[("reduce", kind, op == MAX)] = R.cpu().numpy().tobytes()
            R = out_like(x)
            assert H.mxh_scan(X.data_ptr(), R.data_ptr(), count, dt, op, comm) == 0
            res[("scan", kind, op == MAX)] = R.cpu().numpy().tobytes()
            R = out_like(x)
            assert H.mxh_exscan(X.data_ptr(), R.data_ptr(), count, dt, op, comm) == 0
            res[("exscan", kind, op == MAX)] = R.cpu().numpy().tobytes()
            xb = _gen(kind, 300 * n, rank)
            XB = buf(xb)
            R = out_like(xb, 300)
            assert H.mxh_reduce_scatter_block(XB.data_ptr(), R.data_ptr(), 300, dt, op, comm) == 0
            res[("rsb", kind, op == MAX)] = R.cpu().numpy().tobytes()
            # nonblocking: post five, then complete them (one by MPI_Test polling)
            outs, reqs = {}, []
            for what in ("allreduce", "reduce", "scan", "exscan", "rsb"):
                R = out_like(xb, 300) if what == "rsb" else out_like(x)
                r = vp()
                if what == "allreduce":
                    rc = H.mxh_iallreduce(X.data_ptr(), R.data_ptr(), count, dt, op, comm, ctypes.byref(r))
                elif what == "reduce":
                    rc = H.mxh_ireduce(X.data_ptr(), R.data_ptr(), count, dt, op, n - 1, comm, ctypes.byref(r))
                elif what == "rsb":
                    rc = H.mxh_ireduce_scatter_block(XB.data_ptr(), R.data_ptr(), 300, dt, op, comm, ctypes.byref(r))
                else:
                    fn = H.mxh_iscan if what == "scan" else H.mxh_iexscan
                    rc = fn(X.data_ptr(), R.data_ptr(), count, dt, op, comm, ctypes.byref(r))
                assert rc == 0, (what, rc)
                outs[what] = R
                reqs.append(r)
            flag = ci(0)
            while not flag.value:
                assert H.mxh_test(ctypes.byref(reqs[0]), ctypes.byref(flag)) == 0
            assert reqs[0].value is None                      # MPI_REQUEST_NULL after completion
            for r in reqs[1:]:
                assert H.mxh_wait(ctypes.byref(r)) == 0
                assert r.value is None
            for what, R in outs.items():
                res[("i" + what, kind, op == MAX)] = R.cpu().numpy().tobytes()
            # persistent: MPI_Allreduce_init, started twice
            P, R = vp(), out_like(x)
            assert H.mxh_allreduce_init(X.data_ptr(), R.data_ptr(), count, dt, op, comm, ctypes.byref(P)) == 0
            flag = ci(0)
            assert H.mxh_test(ctypes.byref(P), ctypes.byref(flag)) == 0 and flag.value   # inactive
            for _ in range(2):
                R.zero_()
                assert H.mxh_start(P) == 0
                assert H.mxh_wait(ctypes.byref(P)) == 0
                assert P.value is not None                    # persistent requests survive MPI_Wait
            res[("pallreduce", kind, op == MAX)] = R.cpu().numpy().tobytes()
            assert H.mxh_request_free(ctypes.byref(P)) == 0
        if use_gpu:
            torch.cuda.synchronize()
        H.mxh_comm_free(comm)
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))


def _run(n, use_gpu):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, n, port, use_gpu, q)) for r in range(n)]
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


def _expected(n, kind, is_max, what, alg_of):
    """Oracle results for the algorithm the owning module runs."""
    import mxompi
    import test_coll_tree
    import test_coll_gpu
    L = test_coll_gpu._oracle()
    T = test_coll_tree._oracle()
    t = "INT32_T" if kind == "int" else "FLOAT"
    op = mxompi.OP["MAX" if is_max else "SUM"]
    ty = mxompi.TYPE[t]
    count = 5003 if what != "rsb" else 300 * n
    xs = [_gen(kind, count, r) for r in range(n)]
    sp = (vp * n)(*[x.ctypes.data for x in xs])
    if what == "allreduce":
        exp = [np.zeros_like(xs[0]) for _ in range(n)]
        assert L.mxo_allreduce(alg_of("allreduce"), op, ty, n, count, sp, (vp * n)(*[e.ctypes.data for e in exp])) == 0
        return exp
    if what == "reduce":
        e = np.zeros_like(xs[0])
        assert T.mxo_reduce(alg_of("reduce"), op, ty, n, count, n - 1, sp, e.ctypes.data) == 0
        return {n - 1: e}
    if what in ("scan", "exscan"):
        exp = [np.zeros_like(xs[0]) for _ in range(n)]
        fn = T.mxo_scan if what == "scan" else T.mxo_exscan
        assert fn(1, op, ty, n, count, sp, (vp * n)(*[e.ctypes.data for e in exp])) == 0
        return {r: exp[r] for r in range(1 if what == "exscan" else 0, n)}
    exp = [np.zeros(300, xs[0].dtype) for _ in range(n)]
    assert T.mxo_reduce_scatter_block(alg_of("rsb"), op, ty, n, 300, sp,
                                      (vp * n)(*[e.ctypes.data for e in exp])) == 0
    return exp


def _expected_nbc(n, kind, is_max, what):
    """coll/libnbc's orders (oracle restatement) for the nonblocking forms."""
    import mxompi
    import test_nbc_oracle
    L = test_nbc_oracle._L()
    t = "INT32_T" if kind == "int" else "FLOAT"
    op = mxompi.OP["MAX" if is_max else "SUM"]
    ty = mxompi.TYPE[t]
    count = 5003 if what != "rsb" else 300 * n
    xs = [_gen(kind, count, r) for r in range(n)]
    sp = (vp * n)(*[x.ctypes.data for x in xs])
    if what == "allreduce":
        exp = [np.zeros_like(xs[0]) for _ in range(n)]
        assert L.mxo_iallreduce(0, op, ty, n, count, sp, (vp * n)(*[e.ctypes.data for e in exp])) == 0
        return exp
    if what == "reduce":
        e = np.zeros_like(xs[0])
        assert L.mxo_ireduce(0, op, ty, n, count, n - 1, sp, e.ctypes.data) == 0
        return {n - 1: e}
    if what == "rsb":
        exp = [np.zeros(300, xs[0].dtype) for _ in range(n)]
        assert L.mxo_ireduce_scatter(op, ty, n, (sz * n)(*([300] * n)), sp,
                                     (vp * n)(*[e.ctypes.data for e in exp])) == 0
        return exp
    return _expected(n, kind, is_max, what, lambda w: 1)     # libnbc scan / exscan: linear == coll/basic


def _check_nb(n, got):
    import golden_io
    import mxompi
    for kind in ("int", "flt"):
        for is_max in ((False,) if kind == "int" else (False, True)):
            for what in ("allreduce", "reduce", "scan", "exscan", "rsb", "pallreduce"):
                base = "allreduce" if what == "pallreduce" else what
                exp = _expected_nbc(n, kind, is_max, base)
                key = (what if what == "pallreduce" else "i" + what, kind, is_max)
                items = exp.items() if isinstance(exp, dict) else enumerate(exp)
                for r, e in items:
                    g = np.frombuffer(got[r][key], e.dtype)
                    golden_io.assert_coll_equal(g.view(np.uint8), e.view(np.uint8),
                                                mxompi.OP["MAX" if is_max else "SUM"],
                                                mxompi.TYPE["INT32_T" if kind == "int" else "FLOAT"],
                                                f"{key} rank {r}")


def _check(n, got, alg_of, bitexact_fp):
    import golden_io
    import mxompi
    for kind in ("int", "flt"):
        for is_max in ((False,) if kind == "int" else (False, True)):
            for what in ("allreduce", "reduce", "scan", "exscan", "rsb"):
                exp = _expected(n, kind, is_max, what, alg_of)
                items = exp.items() if isinstance(exp, dict) else enumerate(exp)
                for r, e in items:
                    g = np.frombuffer(got[r][(what, kind, is_max)], e.dtype)
                    t = mxompi.TYPE["INT32_T" if kind == "int" else "FLOAT"]
                    o = mxompi.OP["MAX" if is_max else "SUM"]
                    if kind == "int" or bitexact_fp or is_max:
                        golden_io.assert_coll_equal(g.view(np.uint8), e.view(np.uint8), o, t,
                                                    f"{what} {kind} max={is_max} rank {r}")
                    else:
                        np.testing.assert_allclose(g, e, rtol=1e-5 * n, atol=1e-30,
                                                   err_msg=f"{what} {kind} rank {r}")


@pytest.mark.parametrize("n", [2, 3])
def test_multirank_host_buffers_gloo_cpu(n):
    got = _run(n, use_gpu=False)
    import torch
    if not torch.cuda.is_available():
        assert set(got[0]["owners"].values()) == {"tuned", "basic", "libnbc"}, got[0]["owners"]
        assert got[0]["owners"]["allreduce"] == "tuned" and got[0]["owners"]["scan"] == "basic"
    # coll/tuned's fixed decisions (allreduce, reduce, RSB = coll_reduce +
    # scatter), coll/basic's linear scan / exscan, coll/libnbc's orders for
    # the nonblocking forms: bit-identical to the oracle
    _check(n, got, lambda w: 0, bitexact_fp=True)
    _check_nb(n, got)


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["host_copies", "device", "zero_copy"])
@pytest.mark.parametrize("n", [2, 3])
def test_multirank_device_buffers_through_components(n, path, monkeypatch):
    """Every slot through coll/mi355x on device buffers.  `host_copies`: the
    job's 20 KB calls are at or below coll_mi355x_host_max_kb (64), so they
    run on the saved host modules through host copies of the device buffers
    (coll/cuda's direction); `device` sets the threshold to 0, so they run on
    the device; `zero_copy` also lowers coll_mi355x_reg_min_kb to 1 KiB so the
    blocking reductions, allgather and bcast run between the ranks'
    registered buffers.  Same results on every path."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    if path != "host_copies":
        monkeypatch.setenv("OMPI_MCA_coll_mi355x_host_max_kb", "0")
    if path == "zero_copy":
        monkeypatch.setenv("OMPI_MCA_coll_mi355x_reg_min_kb", "1")
    got = _run(n, use_gpu=True)
    assert all(v == "mi355x" for v in got[0]["owners"].values()), got[0]["owners"]

    def alg_of(what):
        return 0       # coll/tuned fixed decisions (the oracle's alg 0)
    _check(n, got, alg_of, bitexact_fp=True)
    _check_nb(n, got)


# ---------------------------------------------------------------------------
# every rank takes the same protocol whatever memory its buffers are in
# ---------------------------------------------------------------------------
def _mixed_worker(rank, n, port, q):
    """Rank 0 passes HOST buffers (and, for allgather / bcast, a
    non-contiguous MPI_Type_vector layout of the same type signature); the
    other ranks pass contiguous device buffers.  MPI allows both, so the
    component must not let rank 0 delegate to the host module while the
    others run the device protocol (that would deadlock): all ranks run the
    device path, rank 0 staged through device scratch."""
    try:
        import torch
        import torch.distributed as dist
        import minihost
        import mxompi
        os.environ["OMPI_MCA_coll_mi355x_wait_timeout"] = "60"
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n)

        @minihost.AG
        def ag(send, recv, nbytes, ctx):
            out = [None] * n
            dist.all_gather_object(out, ctypes.string_at(send, nbytes))
            blob = b"".join(out)
            ctypes.memmove(recv, blob, len(blob))
            return 0

        torch.cuda.set_device(0)
        mxompi.init(0)
        H = minihost.host(with_components=True)
        comm = H.mxh_comm_create(rank, n, ag, None)
        f32, i32 = minihost.dtype(H, "MPI_FLOAT"), minihost.dtype(H, "MPI_INT")
        SUM = minihost.op(H, "MPI_SUM")
        host = rank == 0
        res = {}

        def buf(a):
            t = torch.from_numpy(np.ascontiguousarray(a).copy())
            return t if host else t.cuda()

        count = 5003
        x = _gen("flt", count, rank)
        X, R = buf(x), buf(np.zeros(count, np.float32))
        assert H.mxh_allreduce(X.data_ptr(), R.data_ptr(), count, f32, SUM, comm) == 0
        res["allreduce"] = R.cpu().numpy().tobytes()
        R = buf(x)
        assert H.mxh_allreduce(1, R.data_ptr(), count, f32, SUM, comm) == 0     # MPI_IN_PLACE
        res["allreduce_inplace"] = R.cpu().numpy().tobytes()
        R = buf(np.zeros(count, np.float32))
        assert H.mxh_reduce(X.data_ptr(), R.data_ptr(), count, f32, SUM, n - 1, comm) == 0
        res["reduce"] = R.cpu().numpy().tobytes()
        R = buf(np.zeros(count, np.float32))
        assert H.mxh_scan(X.data_ptr(), R.data_ptr(), count, f32, SUM, comm) == 0
        res["scan"] = R.cpu().numpy().tobytes()
        xb = _gen("int", 300 * n, rank)
        XB, RB = buf(xb), buf(np.zeros(300, np.int32))
        assert H.mxh_reduce_scatter_block(XB.data_ptr(), RB.data_ptr(), 300, i32, SUM, comm) == 0
        res["rsb"] = RB.cpu().numpy().tobytes()
        rc = (ctypes.c_int * n)(*[100 + 7 * r for r in range(n)])
        XR, RR = buf(_gen("int", sum(rc), rank)), buf(np.zeros(rc[rank], np.int32))
        assert H.mxh_reduce_scatter(XR.data_ptr(), RR.data_ptr(), rc, i32, SUM, comm) == 0
        res["reduce_scatter"] = RR.cpu().numpy().tobytes()
        # nonblocking + persistent with host buffers on rank 0
        R = buf(np.zeros(count, np.float32))
        r = vp()
        assert H.mxh_iallreduce(X.data_ptr(), R.data_ptr(), count, f32, SUM, comm, ctypes.byref(r)) == 0
        assert H.mxh_wait(ctypes.byref(r)) == 0
        res["iallreduce"] = R.cpu().numpy().tobytes()
        P, R = vp(), buf(np.zeros(count, np.float32))
        assert H.mxh_allreduce_init(X.data_ptr(), R.data_ptr(), count, f32, SUM, comm, ctypes.byref(P)) == 0
        for _ in range(2):
            R.zero_()
            assert H.mxh_start(P) == 0
            assert H.mxh_wait(ctypes.byref(P)) == 0
        assert H.mxh_request_free(ctypes.byref(P)) == 0
        res["pallreduce"] = R.cpu().numpy().tobytes()
        # allgather / bcast: rank 0 uses vector(4 blocks of 3 ints, stride 5)
        # x 10 elements, the others 120 contiguous ints: same signature
        vec = H.mxh_dtype_vector(4, 3, 5, i32)
        assert vec
        mine = np.arange(120, dtype=np.int32) + 1000 * rank
        # MPI_Type_vector(4, 3, 5): extent 18 ints, element i at 18 i
        pos = (np.arange(10)[:, None, None] * 18 + np.arange(4)[None, :, None] * 5
               + np.arange(3)[None, None, :]).reshape(-1)
        if host:
            lay = np.full(180, -1, np.int32)
            lay[pos] = mine
            S = buf(lay)
            sdt, scnt = vec, 10
        else:
            S, sdt, scnt = buf(mine), i32, 120
        G = buf(np.full(120 * n, -7, np.int32))
        assert H.mxh_allgather(S.data_ptr(), scnt, sdt, G.data_ptr(), 120, i32, comm) == 0
        res["allgather"] = G.cpu().numpy().tobytes()
        if host:
            lay = np.full(180, -1, np.int32)
            lay[pos] = mine
            B = buf(lay)
            assert H.mxh_bcast(B.data_ptr(), 10, vec, n - 1, comm) == 0
            got = B.cpu().numpy()
            res["bcast"] = got[pos].tobytes()
            gaps = np.ones(180, bool)
            gaps[pos] = False
            res["bcast_gaps"] = bool(np.all(got[gaps] == -1))
        else:
            B = buf(mine)
            assert H.mxh_bcast(B.data_ptr(), 120, i32, n - 1, comm) == 0
            res["bcast"] = B.cpu().numpy().tobytes()
        owners = {s: H.mxh_comm_slot_owner(comm, s.encode()).decode() for s in ("allreduce", "allgather", "bcast")}
        res["owners"] = owners
        torch.cuda.synchronize()
        H.mxh_comm_free(comm)
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))


def _run_fn(fn, n):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, n, port, q)) for r in range(n)]
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
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["host_copies", "device"])
@pytest.mark.parametrize("n", [2, 3])
def test_mixed_host_and_device_buffers_take_one_protocol(n, path, monkeypatch):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    if path == "device":
        monkeypatch.setenv("OMPI_MCA_coll_mi355x_host_max_kb", "0")
    got = _run_fn(_mixed_worker, n)
    assert got[0]["owners"] == {"allreduce": "mi355x", "allgather": "mi355x", "bcast": "mi355x"}
    import golden_io
    import mxompi
    FLT, INT, SUM = mxompi.TYPE["FLOAT"], mxompi.TYPE["INT32_T"], mxompi.OP["SUM"]
    # device-path orders: coll/tuned fixed decisions / libnbc for the i-forms
    ar = _expected(n, "flt", False, "allreduce", lambda w: 0)
    nb = _expected_nbc(n, "flt", False, "allreduce")
    red = _expected(n, "flt", False, "reduce", lambda w: 0)
    scan = _expected(n, "flt", False, "scan", lambda w: 1)
    rsb = _expected(n, "int", False, "rsb", lambda w: 0)
    for r in range(n):
        for key, exp in (("allreduce", ar[r]), ("allreduce_inplace", ar[r]), ("scan", scan[r]),
                         ("iallreduce", nb[r]), ("pallreduce", nb[r])):
            golden_io.assert_coll_equal(np.frombuffer(got[r][key], np.uint8), exp.view(np.uint8), SUM, FLT,
                                        f"{key} rank {r} (rank 0 host buffers)")
        np.testing.assert_array_equal(np.frombuffer(got[r]["rsb"], np.int32), rsb[r])
    golden_io.assert_coll_equal(np.frombuffer(got[n - 1]["reduce"], np.uint8), red[n - 1].view(np.uint8), SUM, FLT,
                                "reduce root")
    rc = [100 + 7 * r for r in range(n)]
    xs = [_gen("int", sum(rc), r).astype(np.int64) for r in range(n)]
    tot = np.sum(xs, axis=0).astype(np.int32)
    for r in range(n):
        lo = sum(rc[:r])
        np.testing.assert_array_equal(np.frombuffer(got[r]["reduce_scatter"], np.int32), tot[lo:lo + rc[r]])
    full = np.concatenate([np.arange(120, dtype=np.int32) + 1000 * p for p in range(n)])
    for r in range(n):
        np.testing.assert_array_equal(np.frombuffer(got[r]["allgather"], np.int32), full)
        np.testing.assert_array_equal(np.frombuffer(got[r]["bcast"], np.int32),
                                      np.arange(120, dtype=np.int32) + 1000 * (n - 1))
    assert got[0]["bcast_gaps"], "bcast into a vector layout wrote into its gaps"


# ---------------------------------------------------------------------------
# non-contiguous DEVICE buffers: the device convertor, not a host round trip
# ---------------------------------------------------------------------------
def _vec_positions(nelem):
    """element positions (in ints) of MPI_Type_vector(4, 3, 5, MPI_INT) x nelem"""
    return (np.arange(nelem)[:, None, None] * 18 + np.arange(4)[None, :, None] * 5
            + np.arange(3)[None, None, :]).reshape(-1)


def _noncontig_worker(rank, n, port, q):
    """Every rank passes DEVICE buffers laid out as MPI_Type_vector(4, 3, 5,
    MPI_INT) for allgather (send and receive side) and bcast.  coll/mi355x
    packs / unpacks them with the device convertor built from the datatype's
    committed description (host table dtype_desc) -- or, with
    MXH_NO_DTYPE_DESC set, through the host convertor: both must give the
    same bytes and leave the gaps alone."""
    try:
        import torch
        import torch.distributed as dist
        import minihost
        import mxompi
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n)

        @minihost.AG
        def ag(send, recv, nbytes, ctx):
            out = [None] * n
            dist.all_gather_object(out, ctypes.string_at(send, nbytes))
            blob = b"".join(out)
            ctypes.memmove(recv, blob, len(blob))
            return 0

        torch.cuda.set_device(0)
        mxompi.init(0)
        H = minihost.host(with_components=True)
        comm = H.mxh_comm_create(rank, n, ag, None)
        i32 = minihost.dtype(H, "MPI_INT")
        vec = H.mxh_dtype_vector(4, 3, 5, i32)
        assert vec
        res = {}
        pos = _vec_positions(10)
        mine = np.arange(120, dtype=np.int32) + 1000 * rank
        lay = np.full(180, -1, np.int32)
        lay[pos] = mine
        S = torch.from_numpy(lay).cuda()
        G = torch.full((180 * n,), -7, dtype=torch.int32, device="cuda")
        assert H.mxh_allgather(S.data_ptr(), 10, vec, G.data_ptr(), 10, vec, comm) == 0
        res["allgather"] = G.cpu().numpy().tobytes()
        B = torch.from_numpy(lay).cuda() if rank == n - 1 else torch.full((180,), -1, dtype=torch.int32,
                                                                            device="cuda")
        assert H.mxh_bcast(B.data_ptr(), 10, vec, n - 1, comm) == 0
        res["bcast"] = B.cpu().numpy().tobytes()
        res["owners"] = {s: H.mxh_comm_slot_owner(comm, s.encode()).decode() for s in ("allgather", "bcast")}
        torch.cuda.synchronize()
        H.mxh_comm_free(comm)
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.parametrize("desc", [True, False, None], ids=["device_convertor", "host_convertor", "host_copies"])
def test_noncontiguous_device_buffers(desc, monkeypatch):
    """device_convertor / host_convertor: the device path (threshold 0) with
    the layouts packed on the device or through the host convertor;
    host_copies: the saved host module on host copies of the spans."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    if desc is not None:
        monkeypatch.setenv("OMPI_MCA_coll_mi355x_host_max_kb", "0")
    desc = bool(desc)
    if desc:
        os.environ.pop("MXH_NO_DTYPE_DESC", None)
    else:
        os.environ["MXH_NO_DTYPE_DESC"] = "1"
    try:
        n = 2
        got = _run_fn(_noncontig_worker, n)
    finally:
        os.environ.pop("MXH_NO_DTYPE_DESC", None)
    pos = _vec_positions(10)
    for r in range(n):
        assert got[r]["owners"] == {"allgather": "mi355x", "bcast": "mi355x"}
        g = np.frombuffer(got[r]["allgather"], np.int32)
        exp = np.full(180 * n, -7, np.int32)
        for p in range(n):
            exp[180 * p + pos] = np.arange(120, dtype=np.int32) + 1000 * p
        np.testing.assert_array_equal(g, exp)              # data in place, gaps untouched
        b = np.frombuffer(got[r]["bcast"], np.int32)
        expb = np.full(180, -1, np.int32)
        expb[pos] = np.arange(120, dtype=np.int32) + 1000 * (n - 1)
        np.testing.assert_array_equal(b, expb)


def _overlap_worker(rank, n, port, q):
    """MPI-legal ordering that a collective spinning on the legacy default
    stream would deadlock: rank 0 posts MPI_Iallreduce and then needs a
    device copy on the default stream (what a PML's device-buffer transfer
    does) before the host handshake that lets rank 1 post its MPI_Iallreduce.
    The component's requests run on its own non-blocking stream, so the copy
    completes while the collective waits for rank 1."""
    try:
        import time
        import torch
        import torch.distributed as dist
        import minihost
        import mxompi
        os.environ["OMPI_MCA_coll_mi355x_wait_timeout"] = "20"
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n)

        @minihost.AG
        def ag(send, recv, nbytes, ctx):
            out = [None] * n
            dist.all_gather_object(out, ctypes.string_at(send, nbytes))
            blob = b"".join(out)
            ctypes.memmove(recv, blob, len(blob))
            return 0

        torch.cuda.set_device(0)
        mxompi.init(0)
        H = minihost.host(with_components=True)
        comm = H.mxh_comm_create(rank, n, ag, None)
        f32, SUM = minihost.dtype(H, "MPI_FLOAT"), minihost.op(H, "MPI_SUM")
        count = 100003
        x = _gen("flt", count, rank)
        X, R = torch.from_numpy(x.copy()).cuda(), torch.zeros(count, device="cuda")
        # warm up: the device communicator is created at the first eligible call
        assert H.mxh_allreduce(X.data_ptr(), R.data_ptr(), count, f32, SUM, comm) == 0
        Y = torch.arange(1 << 20, dtype=torch.float32, device="cuda")
        # ordinary streams in use (MX_TEST_BUSY_STREAMS): more than there are
        # hardware queues, so every ordinary queue is shared -- a kernel on
        # any of them would wait behind a collective spinning on that queue
        busy = [torch.cuda.Stream() for _ in range(int(os.environ.get("MX_TEST_BUSY_STREAMS", "0")))]
        Z = [torch.zeros(1024, device="cuda") for _ in busy]
        for s_, z in zip(busy, Z):
            with torch.cuda.stream(s_):
                z.add_(1.0)
        torch.cuda.synchronize()
        t0 = time.time()
        r = vp()
        if rank == 0:
            assert H.mxh_iallreduce(X.data_ptr(), R.data_ptr(), count, f32, SUM, comm, ctypes.byref(r)) == 0
            y = Y.cpu()                      # default-stream device copy while rank 1 is not in the collective
            assert float(y[-1]) == float((1 << 20) - 1)
            for s_, z in zip(busy, Z):       # and work on every ordinary stream
                with torch.cuda.stream(s_):
                    z.add_(1.0)
                s_.synchronize()
                assert float(z[0]) == 2.0
            dist.barrier()
        else:
            dist.barrier()
            assert H.mxh_iallreduce(X.data_ptr(), R.data_ptr(), count, f32, SUM, comm, ctypes.byref(r)) == 0
        rc = H.mxh_wait(ctypes.byref(r))
        el = time.time() - t0
        torch.cuda.synchronize()
        H.mxh_comm_free(comm)
        dist.destroy_process_group()
        q.put((rank, "ok", {"rc": rc, "seconds": el, "out": R.cpu().numpy().tobytes()}))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.parametrize("busy_streams", [0, 8])
def test_iallreduce_does_not_block_the_default_stream(busy_streams, monkeypatch):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    monkeypatch.setenv("MX_TEST_BUSY_STREAMS", str(busy_streams))
    got = _run_fn(_overlap_worker, 2)
    for r in range(2):
        assert got[r]["rc"] == 0, got[r]
        assert got[r]["seconds"] < 10.0, got[r]["seconds"]
    import golden_io
    import mxompi
    import test_nbc_oracle
    L = test_nbc_oracle._L()
    xs = [_gen("flt", 100003, r) for r in range(2)]
    exp = [np.zeros(100003, np.float32) for _ in range(2)]
    assert L.mxo_iallreduce(0, mxompi.OP["SUM"], mxompi.TYPE["FLOAT"], 2, 100003,
                            (vp * 2)(*[x.ctypes.data for x in xs]), (vp * 2)(*[e.ctypes.data for e in exp])) == 0
    for r in range(2):
        golden_io.assert_coll_equal(np.frombuffer(got[r]["out"], np.uint8), exp[r].view(np.uint8),
                                    mxompi.OP["SUM"], mxompi.TYPE["FLOAT"], f"iallreduce rank {r}")


def _dup_worker(rank, n, port, q):
    """8 communicators over the same ranks (MPI_Comm_dup x 8): the device
    communicator is created at each one's first eligible collective, so idle
    duplicates cost no device memory, and a used one costs its staging
    (coll_mi355x_staging_mb, default 256 MiB) plus ~1 KiB of flags -- no
    point-to-point mailboxes (the coll component never uses them)."""
    try:
        import torch
        import torch.distributed as dist
        import minihost
        import mxompi
        os.environ["OMPI_MCA_coll_mi355x_wait_timeout"] = "60"
        os.environ["OMPI_MCA_coll_mi355x_staging_mb"] = "64"
        os.environ["OMPI_MCA_coll_mi355x_host_max_kb"] = "0"     # the 4 KB calls on the device
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n)

        @minihost.AG
        def ag(send, recv, nbytes, ctx):
            out = [None] * n
            dist.all_gather_object(out, ctypes.string_at(send, nbytes))
            blob = b"".join(out)
            ctypes.memmove(recv, blob, len(blob))
            return 0

        torch.cuda.set_device(0)
        mxompi.init(0)
        H = minihost.host(with_components=True)
        f32, SUM = minihost.dtype(H, "MPI_FLOAT"), minihost.op(H, "MPI_SUM")
        X = torch.ones(1000, device="cuda")
        R = torch.zeros(1000, device="cuda")
        torch.cuda.synchronize()
        dist.barrier()     # the GPU is shared: measure while no rank allocates
        free0 = torch.cuda.mem_get_info()[0]
        dist.barrier()
        comms = [H.mxh_comm_create(rank, n, ag, None) for _ in range(8)]
        torch.cuda.synchronize()
        dist.barrier()
        free1 = torch.cuda.mem_get_info()[0]
        dist.barrier()
        sums = []
        for c in comms:
            R.zero_()
            assert H.mxh_allreduce(X.data_ptr(), R.data_ptr(), 1000, f32, SUM, c) == 0
            sums.append(float(R[0]))
        torch.cuda.synchronize()
        dist.barrier()
        free2 = torch.cuda.mem_get_info()[0]
        dist.barrier()
        for c in comms:
            H.mxh_comm_free(c)
        dist.destroy_process_group()
        q.put((rank, "ok", {"idle_bytes": free0 - free1, "used_bytes": free1 - free2, "sums": sums}))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))


@pytest.mark.gpu
def test_dup_communicators_bounded_device_memory():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    n = 2
    got = _run_fn(_dup_worker, n)
    MiB = 1 << 20
    for r in range(n):
        g = got[r]
        assert g["sums"] == [float(n)] * 8
        # mem_get_info is device-wide (both ranks share the GPU): budgets are per process x n
        assert g["idle_bytes"] < n * 8 * MiB, g
        assert g["used_bytes"] < n * 8 * (64 + 8) * MiB, g
