"""bench.py's contract at N > 1 without a launcher.

The driver runs `python3 bench.py --gpus N`: bench.py must form the N ranks
itself (one process per GPU; here two processes share the box's one GPU),
run the 256 MiB fp32 SUM allreduce of the metric
(coll_base_allreduce.c:618-856 under coll/tuned's fixed decision) and print
one JSON line from rank 0 with n_gpus = the ranks formed and parity checked
bit-exact against the oracle (bench.py allreduce_parity).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_gpus_2_without_launcher_runs_the_allreduce():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup",
                        "1", "--no-sweep", "--no-cpu-baseline"], capture_output=True, text=True, env=env,
                       timeout=280, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert "MPI_Allreduce fp32 SUM 256 MiB" in d["config"]["workload"], d.get("allreduce_error")
    assert d["parity"] == "ok", d.get("parity")
    assert d["value"] > 0 and d["unit"] == "GB/s"
    for name in ("staged_push", "staged_pull", "zero_copy_gather", "zero_copy"):
        ab = d["config"]["data_path_ab"][name]
        assert ab.get("parity") == "ok", (name, ab)


def test_bench_rejects_a_launcher_that_formed_other_ranks():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, env=env, timeout=60, cwd=ROOT)
    assert p.returncode == 2
    assert "WORLD_SIZE=2" in p.stdout
