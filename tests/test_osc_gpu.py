"""GPU: one-sided accumulate on the device symmetric heap (SURVEY 8(f) row 4:
MPI_Accumulate / MPI_Get_accumulate / MPI_Fetch_and_op / MPI_Compare_and_swap,
osc/rdma's get-op-put under the target's accumulate lock).

n processes share the one GPU.  Checked:
* a single origin's accumulate is bit-identical to ompi_op_reduce(op,
  origin, target) (the op oracle), FP SUM with operands spanning 16 decades
  included, REPLACE / NO_OP too;
* concurrent accumulates from every PE into one target are atomic: integer
  sums are exact, every fetch_and_op ticket is handed out exactly once,
  exactly one compare_and_swap wins;
* get_accumulate returns the target as it was before the update;
* derived datatypes on either side (golden reference types: vector of
  doubles on the target, vector of floats on the origin) combine element for
  element in type-map order, like ompi_osc_base_sndrcv_op.
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
BASIC, RECS = golden_io.ddt_records()
REC = {r["name"]: r for r in RECS}
N_ACC, REPS, N_FOP = 4099, 5, 10


def _dt(rec):
    return mxompi.Datatype(rec["desc"].tobytes(), rec["nrec"], rec["size"], rec["lb"], rec["ub"])


def _i64(seed, count):
    return np.random.default_rng(seed).integers(-10**6, 10**6, count).astype(np.int64)


def _osc_worker(rank, n, port, q):
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

        comm = mxompi.Comm(rank, n, ag, device=0, staging_bytes=1 << 20, heap_bytes=64 << 20)
        comm.set_timeout(30.0)
        heap = mxompi.Heap(comm, 32 << 20)
        res = {}

        def to_heap(addr, arr):
            t = _dev(arr.view(np.uint8))
            torch.cuda.synchronize()
            mxompi.lib().mx_copy(addr, t.data_ptr(), t.numel(), None)
            mxompi.sync()

        def from_heap(addr, nbytes):
            t = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
            mxompi.lib().mx_copy(t.data_ptr(), addr, nbytes, None)
            mxompi.sync()
            return t.cpu().numpy().tobytes()

        # (1) single-origin accumulates into PE n-1, one (op, type) per PE
        cases = [("SUM", "FLOAT"), ("MAX", "DOUBLE"), ("PROD", "C_FLOAT_COMPLEX"), ("REPLACE", "INT32_T")]
        wins = []
        for k, (op, t) in enumerate(cases):
            es = mxompi.type_size(t)
            w = heap.alloc(N_ACC * es)
            to_heap(w, gen(t, "SUM" if op == "REPLACE" else op, N_ACC, 500 + 10 * k + rank))
            wins.append(w)
        heap.barrier_all()
        for k, (op, t) in enumerate(cases):
            if k % n == rank:
                o = _dev(gen(t, "SUM" if op == "REPLACE" else op, N_ACC, 900 + k))
                heap.accumulate(o.data_ptr(), N_ACC, t, op, n - 1, wins[k])
        heap.barrier_all()
        if rank == n - 1:
            res["single"] = [from_heap(wins[k], N_ACC * mxompi.type_size(t)) for k, (op, t) in enumerate(cases)]

        # (2) concurrent integer SUM accumulates into PE 0, REPS times each
        acc = heap.alloc(N_ACC * 8)
        to_heap(acc, _i64(11, N_ACC))
        heap.barrier_all()
        v = _dev(_i64(100 + rank, N_ACC).view(np.uint8))
        for _ in range(REPS):
            heap.accumulate(v.data_ptr(), N_ACC, "INT64_T", "SUM", 0, acc)
        heap.barrier_all()
        if rank == 0:
            res["concurrent"] = from_heap(acc, N_ACC * 8)

        # (3) fetch_and_op tickets on PE 0's counter; one compare_and_swap winner
        ctr = heap.alloc(16)
        to_heap(ctr, np.array([1000, -1], np.int64))
        heap.barrier_all()
        one = _dev(np.array([1], np.int64).view(np.uint8))
        got = torch.zeros(8, dtype=torch.uint8, device="cuda")
        tickets = []
        for _ in range(N_FOP):
            heap.fetch_and_op(one.data_ptr(), got.data_ptr(), "INT64_T", "SUM", 0, ctr)
            tickets.append(int(got.cpu().numpy().view(np.int64)[0]))
        mine = _dev(np.array([rank + 100], np.int64).view(np.uint8))
        cmp_ = _dev(np.array([-1], np.int64).view(np.uint8))
        heap.compare_and_swap(mine.data_ptr(), cmp_.data_ptr(), got.data_ptr(), "INT64_T", 0, ctr + 8)
        res["cas"] = int(got.cpu().numpy().view(np.int64)[0])
        res["tickets"] = tickets
        heap.barrier_all()
        if rank == 0:
            res["ctr"] = from_heap(ctr, 16)

        # (4) get_accumulate: PE 1 % n takes MIN on PE 0's region, returns the old values
        ga = heap.alloc(N_ACC * 4)
        to_heap(ga, gen("FLOAT", "MIN", N_ACC, 7))
        heap.barrier_all()
        if rank == 1 % n:
            o = _dev(gen("FLOAT", "MIN", N_ACC, 8))
            r = torch.zeros(N_ACC * 4, dtype=torch.uint8, device="cuda")
            heap.get_accumulate(o.data_ptr(), r.data_ptr(), N_ACC, "FLOAT", "MIN", 0, ga)
            res["ga_old"] = r.cpu().numpy().tobytes()
            r2 = torch.zeros(N_ACC * 4, dtype=torch.uint8, device="cuda")
            heap.get_accumulate(0, r2.data_ptr(), N_ACC, "FLOAT", "NO_OP", 0, ga)     # atomic get
            res["ga_new"] = r2.cpu().numpy().tobytes()
        heap.barrier_all()

        # (5) derived datatypes: target = vector of doubles (golden
        # vector_f64_b3_s5), origin contiguous; origin = vector of floats
        # (vector_f32_b1_s2), target contiguous
        tv, ov = REC["vector_f64_b3_s5"], REC["vector_f32_b1_s2"]
        tdt, odt = _dt(tv), _dt(ov)
        tbuf = heap.alloc(tv["span"])
        to_heap(tbuf, gen("DOUBLE", "SUM", tv["span"] // 8, 300 + rank))
        nel_t = tv["size"] * tv["count"] // 8
        cbuf = heap.alloc(ov["size"] * ov["count"])
        to_heap(cbuf, gen("FLOAT", "SUM", ov["size"] * ov["count"] // 4, 400 + rank))
        heap.barrier_all()
        if rank == 0:
            o = _dev(gen("DOUBLE", "SUM", nel_t, 301))
            heap.accumulate_ddt(o.data_ptr(), nel_t, None, "DOUBLE", "SUM", n - 1, tbuf - tv["true_lb"],
                                tv["count"], tdt)
            ouser = _dev(gen("FLOAT", "SUM", ov["span"] // 4, 401))
            heap.accumulate_ddt(ouser.data_ptr() - ov["true_lb"], ov["count"], odt, "FLOAT", "SUM", n - 1, cbuf,
                                ov["size"] * ov["count"] // 4, None)
        heap.barrier_all()
        if rank == n - 1:
            res["ddt_target"] = from_heap(tbuf, tv["span"])
            res["ddt_origin"] = from_heap(cbuf, ov["size"] * ov["count"])
        heap.barrier_all()
        tdt.close()
        odt.close()
        heap.close()
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
    procs = [ctx.Process(target=_osc_worker, args=(r, n, port, q)) for r in range(n)]
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


def _reduce2(op, t, origin, target):
    O = oracle_lib.oracle()
    exp = target.copy()
    if op == "REPLACE":
        return origin.copy()
    assert O.mxo_reduce2(mxompi.OP[op], mxompi.TYPE[t], origin.ctypes.data, exp.ctypes.data,
                         len(origin) // mxompi.type_size(t), 1) == 0
    return exp


def _ddt_convert(rec, user, packed, unpack):
    O = oracle_lib.oracle()
    O.mxo_ddt_convert.argtypes = [vp, sz, vp, ctypes.c_int64, ctypes.c_int64, sz, vp, vp, ci]
    O.mxo_ddt_convert(rec["desc"].ctypes.data, rec["nrec"], np.ascontiguousarray(BASIC).ctypes.data, rec["lb"],
                      rec["ub"], rec["count"], user.ctypes.data - rec["true_lb"], packed.ctypes.data,
                      1 if unpack else 0)


@pytest.mark.parametrize("n", [2, 3, 4])
def test_one_sided_accumulate(n):
    got = _run(n)
    # (1) single origin: ompi_op_reduce(op, origin, target)
    cases = [("SUM", "FLOAT"), ("MAX", "DOUBLE"), ("PROD", "C_FLOAT_COMPLEX"), ("REPLACE", "INT32_T")]
    for k, (op, t) in enumerate(cases):
        gop = "SUM" if op == "REPLACE" else op
        exp = _reduce2(op, t, gen(t, gop, N_ACC, 900 + k), gen(t, gop, N_ACC, 500 + 10 * k + n - 1))
        golden_io.assert_op_equal(np.frombuffer(got[n - 1]["single"][k], np.uint8), exp, mxompi.OP[gop],
                                  mxompi.TYPE[t], f"accumulate {op} {t}")
    # (2) atomic concurrent integer accumulates
    exp = _i64(11, N_ACC) + REPS * sum(_i64(100 + r, N_ACC) for r in range(n))
    np.testing.assert_array_equal(np.frombuffer(got[0]["concurrent"], np.int64), exp)
    # (3) every ticket once; one CAS winner
    tickets = sorted(t for r in range(n) for t in got[r]["tickets"])
    assert tickets == list(range(1000, 1000 + n * N_FOP))
    ctr = np.frombuffer(got[0]["ctr"], np.int64)
    assert ctr[0] == 1000 + n * N_FOP
    cas = [got[r]["cas"] for r in range(n)]
    winners = [r for r in range(n) if cas[r] == -1]
    assert len(winners) == 1 and ctr[1] == winners[0] + 100, (cas, ctr)
    assert all(c == ctr[1] for r, c in enumerate(cas) if r not in winners)
    # (4) get_accumulate: old values, then the MIN
    old = gen("FLOAT", "MIN", N_ACC, 7)
    g = got[1 % n]
    np.testing.assert_array_equal(np.frombuffer(g["ga_old"], np.uint8), old)
    golden_io.assert_op_equal(np.frombuffer(g["ga_new"], np.uint8),
                              _reduce2("MIN", "FLOAT", gen("FLOAT", "MIN", N_ACC, 8), old), mxompi.OP["MIN"],
                              mxompi.TYPE["FLOAT"], "get_accumulate MIN")
    # (5) derived datatypes, type-map order
    tv, ov = REC["vector_f64_b3_s5"], REC["vector_f32_b1_s2"]
    user = gen("DOUBLE", "SUM", tv["span"] // 8, 300 + n - 1).copy()
    packed = np.zeros(tv["size"] * tv["count"], np.uint8)
    _ddt_convert(tv, user, packed, False)
    nel_t = tv["size"] * tv["count"] // 8
    packed = _reduce2("SUM", "DOUBLE", gen("DOUBLE", "SUM", nel_t, 301), packed)
    _ddt_convert(tv, user, packed, True)
    np.testing.assert_array_equal(np.frombuffer(got[n - 1]["ddt_target"], np.uint8), user)
    ouser = gen("FLOAT", "SUM", ov["span"] // 4, 401).copy()
    opacked = np.zeros(ov["size"] * ov["count"], np.uint8)
    _ddt_convert(ov, ouser, opacked, False)
    exp = _reduce2("SUM", "FLOAT", opacked, gen("FLOAT", "SUM", ov["size"] * ov["count"] // 4, 400 + n - 1))
    np.testing.assert_array_equal(np.frombuffer(got[n - 1]["ddt_origin"], np.uint8), exp)
