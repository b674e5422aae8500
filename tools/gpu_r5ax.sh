#!/bin/bash
# randomised posting / sending orders (3 seeds) over yielding receives
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread "tests/test_p2p_gpu.py::test_randomised_posting_orders_complete_in_match_order" > gpurun_out/r5ax_random.txt 2>&1 || { echo FAILED; tail -80 gpurun_out/r5ax_random.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed|seed" gpurun_out/r5ax_random.txt
