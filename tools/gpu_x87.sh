#!/bin/bash
# GPU-box helper: x87 parity + throughput + one PMC pass
set -o pipefail
mkdir -p gpurun_out/x87
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_reduce_gpu.py -k "x87 or LONG_DOUBLE or long_double" > gpurun_out/x87/pytest.log 2>&1 || { tail -20 gpurun_out/x87/pytest.log; exit 1; }
tail -2 gpurun_out/x87/pytest.log
timeout -k 10 300 python -u tools/sweep.py --what pairs --pair-types C_LONG_DOUBLE_COMPLEX,LONG_DOUBLE --iters 5 --out gpurun_out/x87/sweep_x87.json > gpurun_out/x87/sweep.log 2>&1 || { tail -20 gpurun_out/x87/sweep.log; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/x87/sweep_x87.json"))
for p in d["pairs"]:
    print(p["op"], p["type"], p["gbs"], p["frac_hbm"])
PY
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/x87/pmc -o pmc -- python3 tools/sweep.py --what pairs --pair-types C_LONG_DOUBLE_COMPLEX,LONG_DOUBLE --iters 1 --out gpurun_out/x87/sweep_pmc.json > gpurun_out/x87/pmc.log 2>&1 || { tail -20 gpurun_out/x87/pmc.log; exit 1; }
find gpurun_out/x87/pmc -name "*.csv" | head
