"""GPU parity of the non-blocking and persistent collectives (SURVEY 8(f)
row 2) vs coll/libnbc's schedules restated in the oracle.

n processes share the one GPU (IPC-mapped staging, cross-process flags,
torch.distributed/gloo bootstrap).  Each worker posts requests and only
then waits, so several collectives of one communicator are in flight on the
GPU at once; persistent requests are started repeatedly on fresh data; one
request runs on a side stream while a blocking collective follows on the
current stream (the communicator keeps them in issue order).  Every result
must be bit-identical to what libnbc computes for the same inputs.
"""
import ctypes
import os

import numpy as np
import pytest

import golden_io
import mxompi
import oracle_lib
from test_coll_gpu import _dev, _free_port, gen

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int


def _oracle():
    L = oracle_lib.oracle()
    L.mxo_iallreduce.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_ireduce.argtypes = [ci, ci, ci, ci, sz, ci, ctypes.POINTER(vp), vp]
    L.mxo_ireduce_scatter.argtypes = [ci, ci, ci, ctypes.POINTER(sz), ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_scan.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_exscan.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    return L


# (kind, count, op, type, alg, extra); data seed = 9000 + 97 * job + rank (+ 7 * rep)
JOBS = [
    ("iallreduce", 100003, "SUM", "FLOAT", "auto", False),            # Rabenseifner (n >= 4) / binomial
    ("iallreduce", 100003, "SUM", "FLOAT", "auto", True),             # in place -> binomial
    ("iallreduce", 3001, "SUM", "DOUBLE", "ring", False),
    ("iallreduce", 5, "SUM", "FLOAT", "ring", False),                  # empty ring segments
    ("iallreduce", 4099, "MAX", "FLOAT", "binomial", False),
    ("iallreduce", 777, "MAXLOC", "FLOAT_INT", "rabenseifner", False),
    ("iallreduce", 2500, "SUM", "DOUBLE", "recursive_doubling", True),
    ("iallreduce", 333, "PROD", "LONG_DOUBLE", "binomial", False),
    ("iallreduce", 20001, "PROD", "C_FLOAT_COMPLEX", "auto", False),
    ("ireduce", 100003, "SUM", "FLOAT", "auto", "root_last"),
    ("ireduce", 3001, "SUM", "DOUBLE", "chain", "root_inplace"),
    ("ireduce", 3001, "SUM", "DOUBLE", "chain", "root_last"),
    ("ireduce", 999, "MIN", "FLOAT", "binomial", "root_inplace"),
    ("ireduce", 5000, "SUM", "FLOAT", "rabenseifner", "root_last"),
    ("ireduce_scatter", 1000, "SUM", "FLOAT", "auto", False),
    ("ireduce_scatter", 70001, "SUM", "DOUBLE", "auto", True),       # in place, blocks > staging
    ("ireduce_scatter_block", 3000, "SUM", "DOUBLE", "auto", True),
    ("iscan", 20001, "SUM", "FLOAT", "auto", False),
    ("iexscan", 4097, "SUM", "DOUBLE", "recursive_doubling", False),
    ("iallgather", 300001, "BAND", "UINT8_T", "auto", False),
    ("ibcast", 200003, "BAND", "UINT8_T", "auto", False),
    ("persistent_allreduce", 50001, "SUM", "FLOAT", "auto", 3),
    ("persistent_reduce", 4001, "SUM", "DOUBLE", "chain", 2),
    ("xstream", 70001, "SUM", "FLOAT", "auto", False),
]


def _seed(j, rank, rep=0):
    return 9000 + 97 * j + rank + 7 * rep


def _root(extra, n):
    return 0 if extra == "root_inplace" else n - 1


def _nb_worker(rank, n, port, q):
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
        st = torch.cuda.current_stream().cuda_stream
        side = torch.cuda.Stream()
        posted, results = [], {}
        for j, (kind, count, op, t, alg, extra) in enumerate(JOBS):
            es = mxompi.type_size(t)
            if kind == "iallreduce":
                x = _dev(gen(t, op, count, _seed(j, rank)))
                if extra:
                    r = comm.iallreduce(mxompi.IN_PLACE, x.data_ptr(), count, t, op, alg, st)
                    posted.append((j, r, x, None))
                else:
                    out = torch.zeros(count * es, dtype=torch.uint8, device="cuda")
                    posted.append((j, comm.iallreduce(x.data_ptr(), out.data_ptr(), count, t, op, alg, st), out, x))
            elif kind == "ireduce":
                root = _root(extra, n)
                x = _dev(gen(t, op, count, _seed(j, rank)))
                if extra == "root_inplace" and rank == root:
                    r = comm.ireduce(mxompi.IN_PLACE, x.data_ptr(), count, t, op, root, alg, st)
                    posted.append((j, r, x, None))
                else:
                    out = torch.zeros(count * es, dtype=torch.uint8, device="cuda")
                    r = comm.ireduce(x.data_ptr(), out.data_ptr() if rank == root else 0, count, t, op, root, alg,
                                     st)
                    posted.append((j, r, out if rank == root else None, x))
            elif kind == "ireduce_scatter":
                rc = [count + 3 * p for p in range(n)]
                x = _dev(gen(t, op, sum(rc), _seed(j, rank)))
                if extra:
                    posted.append((j, comm.ireduce_scatter(mxompi.IN_PLACE, x.data_ptr(), rc, t, op, st), x, None))
                else:
                    out = torch.zeros(rc[rank] * es, dtype=torch.uint8, device="cuda")
                    posted.append((j, comm.ireduce_scatter(x.data_ptr(), out.data_ptr(), rc, t, op, st), out, x))
            elif kind == "ireduce_scatter_block":
                x = _dev(gen(t, op, count * n, _seed(j, rank)))
                r = comm.ireduce_scatter_block(mxompi.IN_PLACE, x.data_ptr(), count, t, op, st)
                posted.append((j, r, x, None))
            elif kind in ("iscan", "iexscan"):
                x = _dev(gen(t, op, count, _seed(j, rank)))
                out = torch.zeros(count * es, dtype=torch.uint8, device="cuda")
                r = getattr(comm, kind)(x.data_ptr(), out.data_ptr(), count, t, op, alg, st)
                posted.append((j, r, out, x))
            elif kind == "iallgather":
                x = _dev(gen(t, op, count, _seed(j, rank)))
                out = torch.zeros(n * count, dtype=torch.uint8, device="cuda")
                posted.append((j, comm.iallgather(x.data_ptr(), out.data_ptr(), count, st), out, x))
            elif kind == "ibcast":
                x = _dev(gen(t, op, count, _seed(j, rank)))
                posted.append((j, comm.ibcast(x.data_ptr(), count, 1 % n, st), x, None))
            elif kind.startswith("persistent"):
                # drain what is in flight, then reuse one request on fresh data
                for jj, r, out, keep in posted:
                    r.wait()
                    results[jj] = out.cpu().numpy().tobytes() if out is not None else b""
                    r.free()
                posted = []
                x = torch.zeros(count * es, dtype=torch.uint8, device="cuda")
                out = torch.zeros(count * es, dtype=torch.uint8, device="cuda")
                if kind == "persistent_allreduce":
                    req = comm.iallreduce(x.data_ptr(), out.data_ptr(), count, t, op, alg, st, persistent=True)
                else:
                    req = comm.ireduce(x.data_ptr(), out.data_ptr() if rank == n - 1 else 0, count, t, op, n - 1,
                                       alg, st, persistent=True)
                assert not req.active and req.test()      # inactive: MPI_Test gives true
                reps = []
                for rep in range(extra):
                    x.copy_(_dev(gen(t, op, count, _seed(j, rank, rep))))
                    req.start()
                    req.wait()
                    reps.append(out.cpu().numpy().tobytes())
                req.free()
                results[j] = reps
            elif kind == "xstream":
                # a request on a side stream, then a blocking allreduce on the
                # current stream: the communicator orders them
                x = _dev(gen(t, op, count, _seed(j, rank)))
                y = _dev(gen(t, op, count, _seed(j, rank, 1)))
                out = torch.zeros(count * es, dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                r = comm.iallreduce(x.data_ptr(), out.data_ptr(), count, t, op, "auto", side.cuda_stream)
                comm.allreduce(mxompi.IN_PLACE, y.data_ptr(), count, t, op, "auto", st)
                flag_polls = 0
                while not r.test():
                    flag_polls += 1
                r.free()
                results[j] = (out.cpu().numpy().tobytes(), y.cpu().numpy().tobytes())
        for jj, r, out, keep in posted:
            r.wait()
            results[jj] = out.cpu().numpy().tobytes() if out is not None else b""
            r.free()
        comm.close()
        dist.destroy_process_group()
        q.put((rank, "ok", results))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc() + str(e)))


def _run(n):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_nb_worker, args=(r, n, port, q)) for r in range(n)]
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


NBC_IAR = {"auto": 0, "ring": 1, "binomial": 2, "rabenseifner": 3, "recursive_doubling": 4}
NBC_IRED = {"auto": 0, "chain": 1, "binomial": 2, "rabenseifner": 3}


def _exp_iallreduce(L, n, alg, count, op, t, xs, inplace):
    es = mxompi.type_size(t)
    exp = [x.copy() if inplace else np.zeros(count * es, np.uint8) for x in xs]
    sp = None if inplace else (vp * n)(*[x.ctypes.data for x in xs])
    assert L.mxo_iallreduce(NBC_IAR[alg], mxompi.OP[op], mxompi.TYPE[t], n, count, sp,
                            (vp * n)(*[e.ctypes.data for e in exp])) == 0
    return exp


def _exp_ireduce(L, n, alg, count, op, t, xs, root, inplace):
    es = mxompi.type_size(t)
    exp = xs[root].copy() if inplace else np.zeros(count * es, np.uint8)
    sp = [x.ctypes.data for x in xs]
    if inplace:
        sp[root] = None
    assert L.mxo_ireduce(NBC_IRED[alg], mxompi.OP[op], mxompi.TYPE[t], n, count, root, (vp * n)(*sp),
                         exp.ctypes.data) == 0
    return exp


@pytest.mark.parametrize("n", [2, 3, 4])
def test_nonblocking_and_persistent_bitexact(n):
    L = _oracle()
    got = _run(n)

    def check(a, b, op, t, what):
        golden_io.assert_coll_equal(np.frombuffer(a, np.uint8), b, mxompi.OP[op], mxompi.TYPE[t], what)

    for j, (kind, count, op, t, alg, extra) in enumerate(JOBS):
        es = mxompi.type_size(t)
        what = f"{kind} {alg} {op} {t} n={n}"
        if kind == "iallreduce":
            xs = [gen(t, op, count, _seed(j, r)) for r in range(n)]
            exp = _exp_iallreduce(L, n, alg, count, op, t, xs, extra)
            for r in range(n):
                check(got[r][j], exp[r], op, t, f"{what} rank {r}")
        elif kind == "ireduce":
            root = _root(extra, n)
            xs = [gen(t, op, count, _seed(j, r)) for r in range(n)]
            exp = _exp_ireduce(L, n, alg, count, op, t, xs, root, extra == "root_inplace")
            check(got[root][j], exp, op, t, f"{what} root {root}")
        elif kind in ("ireduce_scatter", "ireduce_scatter_block"):
            rc = [count + 3 * p for p in range(n)] if kind == "ireduce_scatter" else [count] * n
            xs = [gen(t, op, sum(rc), _seed(j, r)) for r in range(n)]
            exp = [np.zeros(c * es, np.uint8) for c in rc]
            assert L.mxo_ireduce_scatter(mxompi.OP[op], mxompi.TYPE[t], n, (sz * n)(*rc),
                                         (vp * n)(*[x.ctypes.data for x in xs]),
                                         (vp * n)(*[e.ctypes.data for e in exp])) == 0
            for r in range(n):
                check(got[r][j][: rc[r] * es], exp[r], op, t, f"{what} rank {r}")
        elif kind in ("iscan", "iexscan"):
            xs = [gen(t, op, count, _seed(j, r)) for r in range(n)]
            exp = [np.zeros(count * es, np.uint8) for _ in range(n)]
            fn = L.mxo_scan if kind == "iscan" else L.mxo_exscan
            assert fn(mxompi.SCAN[alg], mxompi.OP[op], mxompi.TYPE[t], n, count,
                      (vp * n)(*[x.ctypes.data for x in xs]), (vp * n)(*[e.ctypes.data for e in exp])) == 0
            for r in range(1 if kind == "iexscan" else 0, n):
                check(got[r][j], exp[r], op, t, f"{what} rank {r}")
        elif kind == "iallgather":
            full = np.concatenate([gen(t, op, count, _seed(j, r)) for r in range(n)])
            for r in range(n):
                np.testing.assert_array_equal(np.frombuffer(got[r][j], np.uint8), full)
        elif kind == "ibcast":
            root = gen(t, op, count, _seed(j, 1 % n))
            for r in range(n):
                np.testing.assert_array_equal(np.frombuffer(got[r][j], np.uint8), root)
        elif kind == "persistent_allreduce":
            for rep in range(extra):
                xs = [gen(t, op, count, _seed(j, r, rep)) for r in range(n)]
                exp = _exp_iallreduce(L, n, alg, count, op, t, xs, False)
                for r in range(n):
                    check(got[r][j][rep], exp[r], op, t, f"{what} start {rep} rank {r}")
        elif kind == "persistent_reduce":
            for rep in range(extra):
                xs = [gen(t, op, count, _seed(j, r, rep)) for r in range(n)]
                exp = _exp_ireduce(L, n, alg, count, op, t, xs, n - 1, False)
                check(got[n - 1][j][rep], exp, op, t, f"{what} start {rep}")
        elif kind == "xstream":
            xs = [gen(t, op, count, _seed(j, r)) for r in range(n)]
            ys = [gen(t, op, count, _seed(j, r, 1)) for r in range(n)]
            exp_i = _exp_iallreduce(L, n, alg, count, op, t, xs, False)
            L.mxo_allreduce.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
            exp_b = [y.copy() for y in ys]
            assert L.mxo_allreduce(0, mxompi.OP[op], mxompi.TYPE[t], n, count, None,
                                   (vp * n)(*[e.ctypes.data for e in exp_b])) == 0
            for r in range(n):
                check(got[r][j][0], exp_i[r], op, t, f"xstream iallreduce rank {r}")
                check(got[r][j][1], exp_b[r], op, t, f"xstream blocking allreduce rank {r}")
