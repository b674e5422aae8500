"""Headline-size parity of the multi-process collectives (BASELINE configs[3]/[4]).

8 processes share the one GPU of the box (IPC-mapped staging, cross-process
flags -- the same code the driver's 8-GPU run takes over xGMI) and run the
metric's own shapes:

* MPI_Allreduce of 256 MiB fp32 SUM per rank under coll/tuned's fixed
  decision (segmented ring, 32 phases at n = 8, coll_base_allreduce.c:618-856),
  the forced ring (:341-536) and Rabenseifner (:970-1243);
* bf16-as-uint16 BAND allreduce at 256 MiB and at a ragged count;
* MPI_Reduce_scatter (ring, coll_base_reduce_scatter.c:456-623), MPI_Allgather
  and MAXLOC float_int allreduce at >= 64 MiB;
* the same allreduces with a staging area far smaller than the message, so the
  chunked path runs (every chunk re-derives the fold partition from the full
  count);
* the top of CFG-D's range at 2 processes: 1 GiB and 4 GiB fp32 SUM per rank
  (the bench sweep's largest sizes), zero-copy and chunked staged.

Each rank returns a SHA-256 of its result plus a strided sample; the parent
runs the oracle restatement (oracle/mx_oracle_coll.c, step by step over n
simulated ranks) on the same seeded inputs and compares bit for bit.
"""
import ctypes
import hashlib
import os
import socket

import numpy as np
import pytest

import mxompi
import oracle_lib

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
N = 8
MiB = 1 << 20
ALG_ID = {"auto": 0, "ring": 4, "segmented_ring": 5, "rabenseifner": 6}
SAMPLE_STRIDE = 1 << 20   # bytes between sampled 16-byte windows


def gen_big(t, op, count, seed):
    """Seeded inputs for one rank, fast at 10^8 elements.  fp32: uniform
    mantissas scaled over 2^-24..2^24, so the reduction order decides the
    rounding of almost every element; uint16: full-range random bits (BAND of
    8 such words keeps ~1/256 of the bits set); MAXLOC float_int: a handful of
    distinct values (ties everywhere) and random indices."""
    rng = np.random.default_rng(seed)
    if t == "FLOAT":
        u = rng.random(count, dtype=np.float32) * 2 - 1
        return np.ldexp(u, rng.integers(-24, 25, count, dtype=np.int8)).astype(np.float32).view(np.uint8)
    if t == "UINT16_T":
        # bias towards set bits so the 8-way AND is not all zeros
        a = rng.integers(0, 1 << 16, count, dtype=np.uint16)
        b = rng.integers(0, 1 << 16, count, dtype=np.uint16)
        return (a | b | rng.integers(0, 1 << 16, count, dtype=np.uint16)).view(np.uint8)
    if t == "FLOAT_INT":
        p = np.empty(count, dtype=[("v", "<f4"), ("k", "<i4")])
        p["v"] = rng.integers(0, 4, count).astype(np.float32)
        p["k"] = rng.integers(-1000, 1000, count, dtype=np.int32)
        return p.view(np.uint8)
    raise ValueError(t)


def digest(b: np.ndarray):
    b = np.ascontiguousarray(b).view(np.uint8)
    idx = np.arange(0, max(0, b.size - 16), SAMPLE_STRIDE)
    sample = np.stack([b[i:i + 16] for i in idx]) if len(idx) else np.zeros((0, 16), np.uint8)
    return hashlib.sha256(b.data).hexdigest(), sample   # no copy of a multi-GiB result


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rcounts(count, n):
    return [count + 3 * r for r in range(n)]


def _worker(rank, n, port, staging, jobs, q, env=None):
    import torch.distributed as dist
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    os.environ.update(env or {})
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=n)
        torch.cuda.set_device(0)
        mxompi.init(0)

        def ag(b):
            out = [None] * n
            dist.all_gather_object(out, b)
            return out

        comm = mxompi.Comm(rank, n, ag, device=0, staging_bytes=staging)
        comm.set_timeout(60.0)
        st = torch.cuda.current_stream().cuda_stream
        res = []
        for j, (kind, count, op, t, alg) in enumerate(jobs):
            es = mxompi.type_size(t)
            seed = 1000 * j + rank
            if kind == "allreduce":
                x = torch.from_numpy(gen_big(t, op, count, seed)).to("cuda")
                out = torch.empty(count * es, dtype=torch.uint8, device="cuda")
                comm.allreduce(x.data_ptr(), out.data_ptr(), count, t, op, alg, st)
            elif kind == "reduce_scatter":
                rc = _rcounts(count, n)
                x = torch.from_numpy(gen_big(t, op, sum(rc), seed)).to("cuda")
                out = torch.empty(rc[rank] * es, dtype=torch.uint8, device="cuda")
                comm.reduce_scatter(x.data_ptr(), out.data_ptr(), rc, t, op, alg, st)
            elif kind == "allgather":
                x = torch.from_numpy(gen_big(t, op, count, seed)).to("cuda")
                out = torch.empty(n * count * es, dtype=torch.uint8, device="cuda")
                comm.allgather(x.data_ptr(), out.data_ptr(), count * es, st)
            else:
                raise ValueError(kind)
            torch.cuda.synchronize()
            res.append(digest(out.cpu().numpy()))
            del x, out
            torch.cuda.empty_cache()
        comm.close()
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "err", traceback.format_exc() + str(e)))


def _run(jobs, staging, n=N, env=None):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, n, port, staging, jobs, q, env)) for r in range(n)]
    for p in procs:
        p.start()
    out = {}
    try:
        # the oracle runs here while the ranks generate, copy and reduce
        exp = [_expected(job, j, n) for j, job in enumerate(jobs)]
        for _ in range(n):
            rank, status, payload = q.get(timeout=240)
            assert status == "ok", payload
            out[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=60 if len(out) == n else 5)
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
    return out, exp


def _expected(job, j, n=N):
    """Per-rank expected digests from the oracle restatement."""
    kind, count, op, t, alg = job
    L = oracle_lib.oracle()
    L.mxo_allreduce.argtypes = [ci, ci, ci, ci, sz, ctypes.POINTER(vp), ctypes.POINTER(vp)]
    L.mxo_reduce_scatter.argtypes = [ci, ci, ci, ci, ctypes.POINTER(sz), ctypes.POINTER(vp), ctypes.POINTER(vp)]
    es = mxompi.type_size(t)
    if kind == "allreduce":
        xs = [gen_big(t, op, count, 1000 * j + r) for r in range(n)]
        outs = [np.empty(count * es, np.uint8) for _ in range(n)]
        assert L.mxo_allreduce(ALG_ID[alg], mxompi.OP[op], mxompi.TYPE[t], n, count,
                               (vp * n)(*[x.ctypes.data for x in xs]), (vp * n)(*[o.ctypes.data for o in outs])) == 0
        d = digest(outs[0])
        for o in outs[1:]:     # the allgather phase hands every rank the same bytes
            assert np.array_equal(o, outs[0])
        return [d] * n
    if kind == "reduce_scatter":
        rc = _rcounts(count, n)
        xs = [gen_big(t, op, sum(rc), 1000 * j + r) for r in range(n)]
        outs = [np.empty(c * es, np.uint8) for c in rc]
        assert L.mxo_reduce_scatter({"ring": 3, "recursive_halving": 2, "auto": 0}[alg], mxompi.OP[op],
                                    mxompi.TYPE[t], n, (sz * n)(*rc), (vp * n)(*[x.ctypes.data for x in xs]),
                                    (vp * n)(*[o.ctypes.data for o in outs])) == 0
        return [digest(o) for o in outs]
    if kind == "allgather":
        full = np.concatenate([gen_big(t, op, count, 1000 * j + r) for r in range(n)])
        return [digest(full)] * n
    raise ValueError(kind)


def _check(jobs, run, n=N):
    got, expected = run
    for j, job in enumerate(jobs):
        exp = expected[j]
        for r in range(n):
            h, sample = got[r][j]
            eh, esample = exp[r]
            if h != eh:
                bad = np.nonzero(np.any(sample != esample, axis=1))[0]
                where = f"first differing sampled window at byte {int(bad[0]) * SAMPLE_STRIDE}" if len(bad) else \
                    "no sampled window differs"
                pytest.fail(f"{job} rank {r}: result differs from the oracle ({where})")


# 256 MiB fp32 per rank: 2^26 elements.  One-chunk staging = n slots of
# ceil(C/n) elements + a gather area of C elements, plus the one-shot region.
C256 = (256 * MiB) // 4
STAGING_ONE_CHUNK = 2 * 256 * MiB + 96 * MiB
STAGING_CHUNKED = 48 * MiB


def test_allreduce_fp32_sum_256mib_8_ranks():
    """The metric's allreduce at its own size: tuned decision (segmented ring,
    32 phases of 1 MiB at n = 8), forced ring and forced Rabenseifner.  By
    default these run zero-copy between the ranks' registered buffers; the
    chunked test below takes the staged path under both protocols."""
    assert mxompi.allreduce_decision(N, C256, "FLOAT") == 5
    jobs = [("allreduce", C256, "SUM", "FLOAT", "auto"),
            ("allreduce", C256, "SUM", "FLOAT", "ring"),
            ("allreduce", C256, "SUM", "FLOAT", "rabenseifner")]
    _check(jobs, _run(jobs, STAGING_ONE_CHUNK))


def test_allreduce_uint16_band_8_ranks():
    """bf16-as-uint16 BAND (CFG-D): 256 MiB, and a ragged count whose blocks
    differ in size and whose byte offsets are not 16-byte aligned."""
    jobs = [("allreduce", (256 * MiB) // 2, "BAND", "UINT16_T", "auto"),
            ("allreduce", 100_000_007, "BAND", "UINT16_T", "auto"),
            ("allreduce", 33_554_437, "BAND", "UINT16_T", "rabenseifner")]
    _check(jobs, _run(jobs, STAGING_ONE_CHUNK))


def test_reduce_scatter_allgather_maxloc_64mib_8_ranks():
    """CFG-E at >= 64 MiB: ring reduce_scatter with ragged rcounts (64 MiB
    vector), allgather of 8 MiB per rank (64 MiB gathered), MAXLOC float_int
    allreduce of 8 Mi pairs (64 MiB) with ties."""
    jobs = [("reduce_scatter", (64 * MiB) // 4 // N, "SUM", "FLOAT", "ring"),
            ("reduce_scatter", (64 * MiB) // 4 // N + 5, "SUM", "FLOAT", "auto"),
            ("allgather", (8 * MiB) // 2, "BAND", "UINT16_T", "auto"),
            ("allreduce", (64 * MiB) // 8, "MAXLOC", "FLOAT_INT", "auto")]
    _check(jobs, _run(jobs, STAGING_ONE_CHUNK))


@pytest.mark.parametrize("proto", ["push", "pull"])
def test_allreduce_256mib_chunked_8_ranks(proto):
    """The same headline allreduces through a 48 MiB staging area (no
    registration): the message runs in ~12 chunks, each with its own work
    partition but the fold partition of the full count, so results must not
    change -- under both staged data movements."""
    jobs = [("allreduce", C256, "SUM", "FLOAT", "auto"),
            ("allreduce", C256 - 12345, "SUM", "FLOAT", "rabenseifner"),
            ("allreduce", 100_000_007, "BAND", "UINT16_T", "ring"),
            ("reduce_scatter", (64 * MiB) // 4 // N + 7, "SUM", "FLOAT", "ring")]
    _check(jobs, _run(jobs, STAGING_CHUNKED, env={"MX_REG_MIN": "0", "MX_ALLREDUCE_PROTO": proto}))


# CFG-D's range goes to 4 GiB per rank (BASELINE configs[3]; bench.py's
# sweep): 2 processes, so the inputs, results and the oracle's copies fit
# the box's host memory
def test_allreduce_fp32_sum_1gib_per_rank_2_ranks():
    """1 GiB fp32 SUM per rank: tuned decision (zero-copy between the
    registered buffers, chunked by the staging size), forced Rabenseifner,
    and the staged PULL path through a 48 MiB staging area (~40 chunks)."""
    c = (1 << 30) // 4
    jobs = [("allreduce", c, "SUM", "FLOAT", "auto"), ("allreduce", c - 7, "SUM", "FLOAT", "rabenseifner")]
    _check(jobs, _run(jobs, STAGING_ONE_CHUNK, n=2), n=2)
    jobs = [("allreduce", c + 3, "SUM", "FLOAT", "auto")]
    _check(jobs, _run(jobs, STAGING_CHUNKED, n=2, env={"MX_REG_MIN": "0", "MX_ALLREDUCE_PROTO": "pull"}), n=2)


def test_allreduce_fp32_sum_4gib_per_rank_2_ranks():
    """4 GiB fp32 SUM per rank (2^30 elements: byte offsets past 2^32 in every
    kernel's addressing), tuned decision."""
    jobs = [("allreduce", (4 << 30) // 4, "SUM", "FLOAT", "auto")]
    _check(jobs, _run(jobs, STAGING_ONE_CHUNK, n=2), n=2)
