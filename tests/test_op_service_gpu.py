"""The resident reduce service behind mx_reduce2_sync (round 4,
csrc/mx_service.hip): calls of <= 128 KiB on a non-default stream are
served by a one-workgroup kernel that stays resident instead of a launch per
call.

Bit-exact vs the op oracle (op_base_functions.c restated; op values
parity-unpinned) for every element family the service takes, at
ragged sizes up to its 128 KiB cap; pairs interleaved (the service is rebound
to each pair), pauses longer than its 200 us idle exit (relaunch), a call over
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
SVC_MAX = 128 << 10          # kSvcMaxBytes


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
            for count in (1, 17, 1000, 4099, (64 << 10) // es + 3, SVC_MAX // es):
                _check(op, t, count, 100 * rnd + count, s)
                calls += 1
        time.sleep(0.01)                               # > the 200 us idle exit: the next call relaunches
    st, served, launches = mxompi.op_service_stats()
    assert st == 1, "service unusable on this box"
    assert served - served0 == calls, (served - served0, calls)
    assert launches - launches0 >= 2 * len(PAIRS)      # rebound to every pair, every round
    # not served: over the cap, misaligned buffers
    _check("SUM", "FLOAT", SVC_MAX // 4 + 4, 7, s)
    _check("SUM", "FLOAT", (1 << 20) // 4, 9, s)
    _check("SUM", "FLOAT", 5000, 8, s, off=4)
    O = oracle_lib.oracle()
    assert mxompi.op_service_stats()[1] == served
    del O


def test_service_back_to_back_same_buffers():
    """A segmented-ring-like sequence: 500 calls on the same buffers, each
    folding the previous result -- every call must see the last one's result
    (the service's acquire after a command, its release before done)."""
    mxompi.init(0)
    s = torch.cuda.Stream()
    n = 16384              # 128 KiB: the service cap
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
    through the service (aligned, <= 128 KiB) and through the launch (misaligned
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
    """A relaunch (after the idle exit) whose hardware queue is held by a
    spinning kernel of another high-priority stream -- as a p2p receive
    waiting for its peer holds it -- must not wait for that
    kernel, which may be waiting for this very thread: the call launches
    instead, bit-exact, and the service serves again once the queue is free."""
    import ctypes
    mxompi.init(0)
    L = mxompi.lib()
    s = torch.cuda.Stream()
    n = 1000
    a = torch.ones(n, dtype=torch.int64, device="cuda")
    b = torch.zeros(n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), n, s.cuda_stream)
    time.sleep(0.01)                                   # past the idle exit: the next call relaunches
    held0 = mxompi.op_service_held()[1]
    holders = []
    try:
        for _ in range(8):                             # more than the 4 hardware queues per priority
            p = ctypes.c_void_p()
            mxompi.check(L.mx_stream_create(ctypes.byref(p)), "mx_stream_create")
            holders.append(p)
            mxompi.debug_hold(p.value, 20000)
        t0 = time.time()
        for _ in range(20):
            mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), n, s.cuda_stream)
        dt = time.time() - t0
        assert torch.all(b == 21).item()
        held = mxompi.op_service_held()[1] - held0
        print(f"20 calls with every high-priority queue held: {dt * 1e3:.1f} ms, launches held {held}")
        assert dt < 5.0, dt                            # the holders wait 20 s
        assert held >= 1                               # the relaunch did meet a held queue
    finally:
        mxompi.debug_release()
        for p in holders:
            mxompi.check(L.mx_stream_sync(p), "mx_stream_sync")
            mxompi.check(L.mx_stream_destroy(p), "mx_stream_destroy")
    torch.cuda.synchronize()
    served0 = mxompi.op_service_stats()[1]
    for _ in range(3):                                 # the held kernel left on release: served again
        mxompi.reduce2_sync("SUM", "INT64_T", a.data_ptr(), b.data_ptr(), n, s.cuda_stream)
    assert torch.all(b == 24).item()
    assert mxompi.op_service_stats()[1] - served0 == 3
    assert not mxompi.op_service_held()[0]
