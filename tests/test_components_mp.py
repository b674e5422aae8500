"""Multi-rank communicators through the MCA components and the mini-host.

* CPU (gloo, world_size 2 and 3): host buffers.  The harness's MPI entry
  points dispatch through comm->c_coll; on a machine without a GPU the
  coll/mi355x component declines at init_query (no device), every slot stays
  with the host base module, and the results equal the oracle's linear
  orders.  Covers the bootstrap exchange (a host allgather over
  torch.distributed/gloo, the role the saved lower allgather plays inside
  Open MPI) and the N>1 host logic without a GPU.
* GPU (n processes sharing the one GPU): device buffers go through
  coll/mi355x -> mx_* all-peer path and must be bit-identical to the
  coll/tuned algorithm the oracle restates.
* Nonblocking and persistent forms (MPI_Iallreduce, MPI_Ireduce, MPI_Iscan,
  MPI_Iexscan, MPI_Ireduce_scatter_block posted together, then MPI_Test /
  MPI_Wait; MPI_Allreduce_init + MPI_Start twice): host buffers stay with
  the host base module (libnbc's role), device buffers go through
  coll/mi355x's requests and must match coll/libnbc's orders.
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


def _check_nb(n, got, gpu):
    import golden_io
    import mxompi
    for kind in ("int", "flt"):
        for is_max in ((False,) if kind == "int" else (False, True)):
            for what in ("allreduce", "reduce", "scan", "exscan", "rsb", "pallreduce"):
                base = "allreduce" if what == "pallreduce" else what
                exp = _expected_nbc(n, kind, is_max, base) if gpu else _expected(n, kind, is_max, base, lambda w: 1)
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
        assert set(got[0]["owners"].values()) == {"base"}, got[0]["owners"]
    # the host base module runs the linear orders: allreduce / reduce basic
    # linear (rbuf = x_{n-1}; op= x_i), linear scan / exscan, RSB = linear
    # reduce + scatter: bit-identical to the oracle's linear algorithms
    _check(n, got, lambda w: 1, bitexact_fp=True)
    _check_nb(n, got, gpu=False)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3])
def test_multirank_device_buffers_through_components(n):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    got = _run(n, use_gpu=True)
    assert all(v == "mi355x" for v in got[0]["owners"].values()), got[0]["owners"]
    import mxompi

    def alg_of(what):
        return 0       # coll/tuned fixed decisions (the oracle's alg 0)
    _check(n, got, alg_of, bitexact_fp=True)
    _check_nb(n, got, gpu=True)
