#!/bin/bash
# randomised orders at 3 and 4 ranks; negative control: one seed with MX_P2P_YIELD=0 (must time out)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread "tests/test_p2p_gpu.py::test_randomised_posting_orders_complete_in_match_order" > gpurun_out/r5ay_random.txt 2>&1 || { echo FAILED; tail -80 gpurun_out/r5ay_random.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed|seed" gpurun_out/r5ay_random.txt
MX_P2P_YIELD=0 timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread "tests/test_p2p_gpu.py::test_randomised_posting_orders_complete_in_match_order[3-1]" > gpurun_out/r5ay_noyield.txt 2>&1
echo "noyield rc=$?"
grep -E "MX_ERR|passed|failed" gpurun_out/r5ay_noyield.txt | tail -3
