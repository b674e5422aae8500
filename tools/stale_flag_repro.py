"""Regression demonstration for the round-3 8-rank wrong part.

Runs the communicator-recycling job list of
tests/test_coll_gpu.py::test_communicator_recycling_with_a_late_peer_8_ranks
twice at 8 processes on the one GPU -- with round 3's immediate reuse of a
freed communicator's IPC regions (MX_IPC_QUARANTINE=0) and with the
quarantine (default) -- and prints, per allreduce and rank, how many
elements differ from the oracle and which 1/8 parts they fall in.

    python tools/stale_flag_repro.py > profiles/r04/stale_flag_repro.txt
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "zhpe-ompi_amd"))

import mxompi  # noqa: E402
import test_coll_gpu as T  # noqa: E402


def _blocks(count, n):
    late, split = divmod(count, n)
    early = late + (1 if split else 0)
    return [(b * early, early) if b < split else (b * late + split, late) for b in range(n)]


def run(quarantine):
    n = 8
    env = {"MX_AUTOTUNE": "0", "MX_DEBUG_LAG_RANK": "3", "MX_DEBUG_LAG_US": "50000",
           "MX_IPC_QUARANTINE": "1" if quarantine else "0"}
    got = T._run_mp(n, T._JOBS_RECYCLE, staging=64 << 20, env=env)
    L = T._oracle()
    bad = 0
    for j, (kind, count, op, t, alg) in enumerate(T._JOBS_RECYCLE):
        if kind != "allreduce":
            continue
        xs = [T.gen(t, op, count, 7000 + r) for r in range(n)]
        exp = [np.zeros(count * 4, np.uint8) for _ in range(n)]
        assert L.mxo_allreduce(T.ALG_ID[alg], mxompi.OP[op], mxompi.TYPE[t], n, count,
                               (T.vp * n)(*[x.ctypes.data for x in xs]),
                               (T.vp * n)(*[e.ctypes.data for e in exp])) == 0
        for r in range(n):
            g = np.frombuffer(got[r][j], np.uint32)
            e = exp[r].view(np.uint32)
            wrong = np.nonzero(g != e)[0]
            if len(wrong):
                bad += 1
                parts = sorted({b for b, (o, ln) in enumerate(_blocks(count, n)) for w in wrong[:1] if o <= w < o + ln})
                print(f"  job {j:2d} allreduce {count} {alg}: rank {r}: {len(wrong)} wrong elements, "
                      f"first in part {parts}")
    return bad


if __name__ == "__main__":
    import torch
    assert torch.cuda.is_available()
    for q in (False, True):
        print(f"MX_IPC_QUARANTINE={int(q)}:", flush=True)
        b = run(q)
        print(f"  -> {b} wrong (allreduce, rank) results", flush=True)
