#!/bin/bash
# negative control (MX_P2P_YIELD=0 must time out on the yield test), then the other suites that use p2p
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MX_P2P_YIELD=0 timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  "tests/test_p2p_gpu.py::test_receives_yield_to_receives_posted_after_them" > gpurun_out/r5ai_noyield.txt 2>&1
echo "noyield rc=$?"
grep -E "MX_ERR|Timeout|timeout|passed|failed" gpurun_out/r5ai_noyield.txt | tail -5
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_btl_gpu.py tests/test_lifecycle_gpu.py tests/test_op_service_gpu.py tests/test_components_rules.py -m gpu > gpurun_out/r5ai_suites.txt 2>&1 || { echo SUITES_FAILED; tail -60 gpurun_out/r5ai_suites.txt; exit 1; }
tail -3 gpurun_out/r5ai_suites.txt
