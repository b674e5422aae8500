#!/bin/bash
# receives that yield: new test, the p2p suite, latency A/B (MX_P2P_YIELD=0 = round-4 behaviour)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  "tests/test_p2p_gpu.py::test_receives_yield_to_receives_posted_after_them" > gpurun_out/r5ah_yield.txt 2>&1 || { echo YIELD_TEST_FAILED; tail -60 gpurun_out/r5ah_yield.txt; exit 1; }
tail -3 gpurun_out/r5ah_yield.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_p2p_gpu.py > gpurun_out/r5ah_p2p.txt 2>&1 || { echo P2P_FAILED; tail -60 gpurun_out/r5ah_p2p.txt; exit 1; }
tail -3 gpurun_out/r5ah_p2p.txt
timeout -k 10 200 python -u tools/p2p_lat.py > gpurun_out/r5ah_lat_yield.txt 2>&1 && tail -2 gpurun_out/r5ah_lat_yield.txt
MX_P2P_YIELD=0 timeout -k 10 200 python -u tools/p2p_lat.py > gpurun_out/r5ah_lat_noyield.txt 2>&1 && tail -2 gpurun_out/r5ah_lat_noyield.txt
