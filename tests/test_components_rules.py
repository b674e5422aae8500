"""Which reduction order coll/mi355x runs, and where (round 3).

coll/mi355x must give the bytes the module it displaced would give:

* coll/tuned with coll_tuned_use_dynamic_rules: the forced
  coll_tuned_<coll>_algorithm (+ _chain_fanout), or a rules file
  (coll_tuned_dynamic_rules_filename), instead of the fixed decision
  (coll_tuned_decision_dynamic.c, coll_tuned_module.c:152-238);
* coll/basic when coll/tuned is excluded (--mca coll ^tuned): allreduce =
  coll_reduce to 0 + coll_bcast, linear reduce up to coll_basic_crossover,
  recursive-halving reduce_scatter below 8 MiB;
* intercommunicators are declined (coll_tuned_module.c:66-69);
* calls at or below coll_mi355x_host_max_kb run on the saved host module
  through host copies of device buffers, and a host-only program allocates
  no device memory;
* a nonblocking collective never waits for peers: before the device path
  exists it runs on the saved module (MPI-3.1 5.12), so rank 0 MPI_Iallreduce
  + MPI_Send / rank 1 MPI_Recv + MPI_Iallreduce completes.

Every GPU result is checked bit for bit against the oracle restatement with
the algorithm the reference would have run.  CPU: the rules-file parser.
"""
import ctypes
import os
import socket
import tempfile

import numpy as np
import pytest

import mxompi

vp, ci, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t


# ---------------------------------------------------------------------------
# CPU: the rules file, parsed like ompi_coll_tuned_read_rules_config_file
# ---------------------------------------------------------------------------
class MsgRule(ctypes.Structure):
    _fields_ = [("msg_size", sz), ("alg", ci), ("faninout", ci), ("segsize", ctypes.c_long)]


class ComRule(ctypes.Structure):
    _fields_ = [("comsize", ci), ("nmsg", ci), ("msg", ctypes.POINTER(MsgRule))]


def _parse(text):
    L = ctypes.CDLL(os.path.join(mxompi.LIB_DIR, "libmx_ompi.so"))
    L.mx_tuned_rules_parse.argtypes = [ctypes.c_char_p, ci, ctypes.POINTER(ci), ctypes.POINTER(ctypes.POINTER(ComRule))]
    L.mx_tuned_rules_free.argtypes = [ci, ctypes.POINTER(ci), ctypes.POINTER(ctypes.POINTER(ComRule))]
    with tempfile.NamedTemporaryFile("w", suffix=".rules", delete=False) as f:
        f.write(text)
        path = f.name
    try:
        ncs = (ci * 22)()
        coms = (ctypes.POINTER(ComRule) * 22)()
        n = L.mx_tuned_rules_parse(path.encode(), 22, ncs, coms)
        out = {}
        for c in range(22):
            if ncs[c]:
                out[c] = [(coms[c][k].comsize, [(coms[c][k].msg[j].msg_size, coms[c][k].msg[j].alg,
                                                  coms[c][k].msg[j].faninout, coms[c][k].msg[j].segsize)
                                                 for j in range(coms[c][k].nmsg)]) for k in range(ncs[c])]
        L.mx_tuned_rules_free(22, ncs, coms)
        return n, out
    finally:
        os.unlink(path)


RULES = """# two collectives
2
2        # allreduce
2        # two communicator sizes
1 2      # comm size 1: two message sizes
0 4 0 0
65536 6 0 0
8 1
0 3 0 0
11       # reduce
1
1 1
0 2 3 0
"""


def test_rules_file_parsed_like_the_reference():
    n, out = _parse(RULES)
    assert n == 2
    assert out[2] == [(1, [(0, 4, 0, 0), (65536, 6, 0, 0)]), (8, [(0, 3, 0, 0)])]
    assert out[11] == [(1, [(0, 2, 3, 0)])]


@pytest.mark.parametrize("bad", ["3\n2 1 1 1 0 4 0 0\n",            # more collectives announced than given
                                 "1\n2 1 1 1 5 4 0 0\n",             # first message size must be 0
                                 "1\n40 1 1 1 0 4 0 0\n",            # collective id out of range
                                 "1\n2 1 1 1 0 -4 0 0\n"])           # negative algorithm
def test_bad_rules_file_is_dropped_whole(bad):
    n, out = _parse(bad)
    assert n == -1 and out == {}


# ---------------------------------------------------------------------------
# GPU: n processes on the one GPU through the mini-host
# ---------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gen(t, count, seed):
    rng = np.random.default_rng(seed)
    if t == "FLOAT":
        return (rng.uniform(-1, 1, count) * 10.0 ** rng.uniform(-7, 7, count)).astype(np.float32)
    v = (rng.uniform(-1, 1, count) * 10.0 ** rng.uniform(-7, 7, count)).astype(np.float64)
    v[rng.integers(0, count, max(1, count // 20))] = np.nan
    return v


# jobs: (kind, type, op, count or rcounts, root)
def _jobs(n):
    rc_small = [1000 + 37 * r for r in range(n)]
    rc_big = [20000 + 37 * r for r in range(n)]
    return [("allreduce", "FLOAT", "SUM", 3001, None), ("allreduce", "FLOAT", "SUM", 40001, None),
            ("allreduce", "DOUBLE", "MAX", 20001, None),
            ("reduce_scatter", "FLOAT", "SUM", rc_small, None), ("reduce_scatter", "FLOAT", "SUM", rc_big, None),
            ("reduce", "FLOAT", "SUM", 30001, n - 1)]


def _rules_file(tmpdir):
    path = os.path.join(tmpdir, "mx_test.rules")
    with open(path, "w") as f:
        # allreduce: ring below 64 KiB, Rabenseifner from there; reduce_scatter: butterfly
        f.write("2\n2 1\n1 2\n0 4 0 0\n65536 6 0 0\n12 1\n1 1\n0 4 0 0\n")
    return path


def _configs(tmpdir, host_max=0):
    """(name, env, expected algorithm word per job kind and size).  The
    mini-host's tuned stand-in honours forced algorithms but reads no rules
    file, so the rules-file configuration runs with every call on the device
    only."""
    dyn = {"coll_tuned_use_dynamic_rules": "1"}
    cfgs = []
    for k in range(1, 7):
        cfgs.append((f"allreduce_alg{k}", {**dyn, "coll_tuned_allreduce_algorithm": str(k)},
                     {"allreduce": k if k != 2 else mxompi.alg_word(2, 0)}))
    for k in range(1, 5):
        cfgs.append((f"reduce_scatter_alg{k}", {**dyn, "coll_tuned_reduce_scatter_algorithm": str(k)},
                     {"reduce_scatter": k if k != 1 else mxompi.alg_word(1, 0)}))
    cfgs.append(("reduce_chain3_composed", {**dyn, "coll_tuned_reduce_algorithm": "2",
                                            "coll_tuned_reduce_algorithm_chain_fanout": "3",
                                            "coll_tuned_allreduce_algorithm": "2",
                                            "coll_tuned_reduce_scatter_algorithm": "1"},
                 {"allreduce": mxompi.alg_word(2, 2, 3), "reduce_scatter": mxompi.alg_word(1, 2, 3),
                  "reduce": mxompi.alg_word(2, 0, 3)}))
    if host_max == 0:
        cfgs.append(("rules_file", {**dyn, "coll_tuned_dynamic_rules_filename": _rules_file(tmpdir)},
                     {"allreduce": lambda bytes_: 4 if bytes_ < 65536 else 6, "reduce_scatter": 4}))
    cfgs.append(("no_tuned_basic", {"coll": "^tuned", "coll_basic_crossover": "16"},
                 {"allreduce": mxompi.alg_word(2, 1), "reduce": 1,
                  "reduce_scatter": 2}))
    return cfgs


def _worker(rank, n, port, host_max, tmpdir, q):
    try:
        import torch
        import torch.distributed as dist
        import minihost
        os.environ["OMPI_MCA_coll_mi355x_wait_timeout"] = "60"
        os.environ["OMPI_MCA_coll_mi355x_host_max_kb"] = str(host_max)
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
        res = {}
        for name, env, _ in _configs(tmpdir, host_max):
            for k, v in env.items():
                os.environ["OMPI_MCA_" + k] = v
            try:
                comm = H.mxh_comm_create(rank, n, ag, None)
                res[(name, "owner")] = H.mxh_comm_slot_owner(comm, b"allreduce").decode()
                for j, (kind, t, op, cnt, root) in enumerate(_jobs(n)):
                    dt = minihost.dtype(H, "MPI_" + t)
                    o = minihost.op(H, "MPI_" + op)
                    npdt = np.float32 if t == "FLOAT" else np.float64
                    total = sum(cnt) if isinstance(cnt, list) else cnt
                    X = torch.from_numpy(_gen(t, total, 1000 * j + rank)).cuda()
                    if kind == "allreduce":
                        R = torch.zeros(total, dtype=X.dtype, device="cuda")
                        rc = H.mxh_allreduce(X.data_ptr(), R.data_ptr(), total, dt, o, comm)
                    elif kind == "reduce_scatter":
                        R = torch.zeros(cnt[rank], dtype=X.dtype, device="cuda")
                        rc = H.mxh_reduce_scatter(X.data_ptr(), R.data_ptr(), (ci * n)(*cnt), dt, o, comm)
                    else:
                        R = torch.zeros(total, dtype=X.dtype, device="cuda")
                        rc = H.mxh_reduce(X.data_ptr(), R.data_ptr(), total, dt, o, root, comm)
                    assert rc == 0, (name, kind, rc)
                    torch.cuda.synchronize()
                    res[(name, j)] = R.cpu().numpy().astype(npdt).tobytes()
                H.mxh_comm_free(comm)
            finally:
                for k in env:
                    os.environ.pop("OMPI_MCA_" + k, None)
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))


def _run_fn(fn, n, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, n, port, *args, q)) for r in range(n)]
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


def _expected(n, kind, t, op, cnt, root, word, j):
    import oracle_lib
    L = oracle_lib.oracle()
    L.mxo_allreduce.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_reduce_scatter.argtypes = [ci, ci, ci, ci, ctypes.POINTER(sz), ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_reduce.argtypes = [ci, ci, ci, ci, sz, ci, ctypes.POINTER(vp), vp]
    total = sum(cnt) if isinstance(cnt, list) else cnt
    xs = [_gen(t, total, 1000 * j + r) for r in range(n)]
    sp = (vp * n)(*[x.ctypes.data for x in xs])
    o, ty = mxompi.OP[op], mxompi.TYPE[t]
    if kind == "allreduce":
        outs = [np.zeros_like(xs[0]) for _ in range(n)]
        assert L.mxo_allreduce(word, o, ty, n, total, sp, (vp * n)(*[e.ctypes.data for e in outs])) == 0
        return {r: outs[r] for r in range(n)}
    if kind == "reduce_scatter":
        outs = [np.zeros(c, xs[0].dtype) for c in cnt]
        assert L.mxo_reduce_scatter(word, o, ty, n, (sz * n)(*cnt), sp, (vp * n)(*[e.ctypes.data for e in outs])) == 0
        return {r: outs[r] for r in range(n)}
    out = np.zeros_like(xs[0])
    assert L.mxo_reduce(word, o, ty, n, total, root, sp, out.ctypes.data) == 0
    return {root: out}


@pytest.mark.gpu
@pytest.mark.parametrize("host_max", [0, 64], ids=["device", "host_small"])
@pytest.mark.parametrize("n", [2, 3, 8])
def test_tuned_forced_rules_and_basic_orders(n, host_max, tmp_path):
    """Every configuration above at n = 2, 3, 8; `device`: every call on the
    GPU (coll_mi355x_host_max_kb = 0); `host_small`: the calls of at most
    64 KiB on the saved host module through host copies, the larger ones on
    the GPU -- the same bytes either way."""
    import golden_io
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    tmpdir = str(tmp_path)
    got = _run_fn(_worker, n, host_max, tmpdir)
    es = {"FLOAT": 4, "DOUBLE": 8}
    for name, env, words in _configs(tmpdir, host_max):
        assert got[0][(name, "owner")] == "mi355x", name
        for j, (kind, t, op, cnt, root) in enumerate(_jobs(n)):
            w = words.get(kind, 0)
            total = sum(cnt) if isinstance(cnt, list) else cnt
            if callable(w):
                w = w(total * es[t])
            exp = _expected(n, kind, t, op, cnt, root, w, j)
            for r, e in exp.items():
                g = np.frombuffer(got[r][(name, j)], e.dtype)
                golden_io.assert_coll_equal(g.view(np.uint8), e.view(np.uint8), mxompi.OP[op], mxompi.TYPE[t],
                                            f"{name} {kind} {t} {op} n={n} word={w:#x} rank {r}")


# ---------------------------------------------------------------------------
def _inter_worker(rank, n, port, q):
    try:
        import torch
        import torch.distributed as dist
        import minihost
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
        intra = H.mxh_comm_create(rank, n, ag, None)
        inter = H.mxh_intercomm_create(rank, n, ag, None)
        slots = ("allreduce", "reduce_scatter", "allgather", "bcast", "reduce", "iallreduce")
        res = {"intra": {s: H.mxh_comm_slot_owner(intra, s.encode()).decode() for s in slots},
               "inter": {s: H.mxh_comm_slot_owner(inter, s.encode()).decode() for s in slots}}
        H.mxh_comm_free(inter)
        H.mxh_comm_free(intra)
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))


@pytest.mark.gpu
def test_intercommunicator_declined():
    """comm_query returns no module for an intercommunicator (so neither
    tuned nor mi355x takes its slots; coll/basic's remain), while an
    intracommunicator of the same size gets coll/mi355x."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    got = _run_fn(_inter_worker, 2)
    for r in range(2):
        assert set(got[r]["intra"].values()) == {"mi355x"}, got[r]
        assert "mi355x" not in got[r]["inter"].values() and "tuned" not in got[r]["inter"].values(), got[r]


# ---------------------------------------------------------------------------
def _nb_first_worker(rank, n, port, q):
    """The ADVICE r2 ordering: rank 0 MPI_Iallreduce then MPI_Send, rank 1
    MPI_Recv then MPI_Iallreduce, on a communicator that never ran a device
    collective (device buffers, 400 KB: above the host threshold).  Then a
    blocking allreduce creates the device path, and the same pattern runs on
    the device."""
    try:
        import time
        import torch
        import torch.distributed as dist
        import minihost
        os.environ["OMPI_MCA_coll_mi355x_wait_timeout"] = "30"
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
        X = torch.from_numpy(_gen("FLOAT", count, 77 + rank)).cuda()
        res = {}
        for phase in ("before_device_path", "after_device_path"):
            R = torch.zeros(count, device="cuda")
            r = vp()
            msg = torch.zeros(4)
            t0 = time.time()
            if rank == 0:
                assert H.mxh_iallreduce(X.data_ptr(), R.data_ptr(), count, f32, SUM, comm, ctypes.byref(r)) == 0
                dist.send(torch.ones(4), dst=1)
            else:
                dist.recv(msg, src=0)
                assert H.mxh_iallreduce(X.data_ptr(), R.data_ptr(), count, f32, SUM, comm, ctypes.byref(r)) == 0
            assert H.mxh_wait(ctypes.byref(r)) == 0
            torch.cuda.synchronize()
            res[phase] = (R.cpu().numpy().tobytes(), time.time() - t0)
            if phase == "before_device_path":   # a blocking call creates the device path
                B = torch.zeros(count, device="cuda")
                assert H.mxh_allreduce(X.data_ptr(), B.data_ptr(), count, f32, SUM, comm) == 0
        H.mxh_comm_free(comm)
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))


@pytest.mark.gpu
def test_nonblocking_collective_never_waits_for_device_path_creation():
    import golden_io
    import oracle_lib
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    got = _run_fn(_nb_first_worker, 2)
    L = oracle_lib.oracle()
    L.mxo_iallreduce.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    count = 100003
    xs = [_gen("FLOAT", count, 77 + r) for r in range(2)]
    exp = [np.zeros(count, np.float32) for _ in range(2)]
    assert L.mxo_iallreduce(0, mxompi.OP["SUM"], mxompi.TYPE["FLOAT"], 2, count,
                            (vp * 2)(*[x.ctypes.data for x in xs]), (vp * 2)(*[e.ctypes.data for e in exp])) == 0
    for r in range(2):
        for phase in ("before_device_path", "after_device_path"):
            data, secs = got[r][phase]
            assert secs < 20, (phase, secs)
            golden_io.assert_coll_equal(np.frombuffer(data, np.uint8), exp[r].view(np.uint8), mxompi.OP["SUM"],
                                        mxompi.TYPE["FLOAT"], f"iallreduce {phase} rank {r} (libnbc order)")


# ---------------------------------------------------------------------------
def _host_only_worker(rank, n, port, q):
    """Host buffers only, 8 B .. 64 KiB: the calls run on the saved host
    module; the device path is never created, so no device memory is
    allocated (mem_get_info is device-wide: measured between barriers)."""
    try:
        import time
        import torch
        import torch.distributed as dist
        import minihost
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
        torch.cuda.synchronize()
        dist.barrier()
        free0 = torch.cuda.mem_get_info()[0]
        dist.barrier()
        comm = H.mxh_comm_create(rank, n, ag, None)
        lat = {}
        for nbytes in (8, 1024, 16 << 10, 64 << 10):
            cnt = nbytes // 4
            x = np.full(cnt, rank + 1, np.float32)
            y = np.zeros(cnt, np.float32)
            t0 = time.perf_counter()
            for _ in range(5):
                assert H.mxh_allreduce(x.ctypes.data, y.ctypes.data, cnt, f32, SUM, comm) == 0
            lat[nbytes] = (time.perf_counter() - t0) / 5
            assert np.all(y == n * (n + 1) / 2)
        dist.barrier()
        free1 = torch.cuda.mem_get_info()[0]
        dist.barrier()
        owner = H.mxh_comm_slot_owner(comm, b"allreduce").decode()
        H.mxh_comm_free(comm)
        dist.destroy_process_group()
        q.put((rank, "ok", {"delta": free0 - free1, "owner": owner, "lat": lat}))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))


@pytest.mark.gpu
def test_host_only_small_allreduce_allocates_no_device_memory():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    got = _run_fn(_host_only_worker, 2)
    for r in range(2):
        assert got[r]["owner"] == "mi355x"
        assert got[r]["delta"] == 0, got[r]


# ---------------------------------------------------------------------------
_STALE_ITERS = 12


def _stale_worker(rank, n, port, q):
    """The zero-copy paths read the peers' registered buffers.  The same
    sbuf / rbuf allocations are rewritten with new data before every call:
    a reader that kept a peer's old line (or a writer whose data was not yet
    visible) gives a stale result, which the oracle comparison catches."""
    try:
        import torch
        import torch.distributed as dist
        import minihost
        os.environ["OMPI_MCA_coll_mi355x_wait_timeout"] = "60"
        os.environ["OMPI_MCA_coll_mi355x_host_max_kb"] = "0"
        os.environ["OMPI_MCA_coll_mi355x_reg_min_kb"] = "1"
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
        count = 65537
        X = torch.empty(count, device="cuda")
        R = torch.empty(count, device="cuda")
        G = torch.empty(count * n, device="cuda")
        T = torch.empty(count, device="cuda")
        res = {}
        for it in range(_STALE_ITERS):
            # new data written into the same allocation by a kernel on the
            # caller's stream right before the call (through this GPU's L2s)
            T.copy_(torch.from_numpy(_gen("FLOAT", count, 5000 + 10 * it + rank)))
            X.copy_(T)
            # R's lines are in this GPU's L2s (written by the fill kernel); the
            # zero-copy allreduce's peers write their parts straight into R, and a
            # kernel reads R right after the call returns (the clone): a line the
            # call's final acquire left stale would show the NaNs
            R.fill_(float("nan"))
            assert H.mxh_allreduce(X.data_ptr(), R.data_ptr(), count, f32, SUM, comm) == 0
            res[("allreduce", it)] = R.clone().cpu().numpy().tobytes()
            assert H.mxh_allgather(X.data_ptr(), count, f32, G.data_ptr(), count, f32, comm) == 0
            res[("allgather", it)] = G.cpu().numpy().tobytes()
        H.mxh_comm_free(comm)
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc()))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 8])
def test_zero_copy_reused_buffers_never_read_stale_data(n):
    import golden_io
    import oracle_lib
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    got = _run_fn(_stale_worker, n)
    L = oracle_lib.oracle()
    L.mxo_allreduce.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    count = 65537
    for it in range(_STALE_ITERS):
        xs = [_gen("FLOAT", count, 5000 + 10 * it + r) for r in range(n)]
        exp = [np.zeros(count, np.float32) for _ in range(n)]
        assert L.mxo_allreduce(0, mxompi.OP["SUM"], mxompi.TYPE["FLOAT"], n, count,
                               (vp * n)(*[x.ctypes.data for x in xs]), (vp * n)(*[e.ctypes.data for e in exp])) == 0
        full = np.concatenate(xs)
        for r in range(n):
            golden_io.assert_coll_equal(np.frombuffer(got[r][("allreduce", it)], np.uint8), exp[r].view(np.uint8),
                                        mxompi.OP["SUM"], mxompi.TYPE["FLOAT"], f"allreduce call {it} rank {r}")
            np.testing.assert_array_equal(np.frombuffer(got[r][("allgather", it)], np.float32), full,
                                          err_msg=f"allgather call {it} rank {r}")
