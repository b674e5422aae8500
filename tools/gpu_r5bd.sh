#!/bin/bash
# channel completion through mapped words instead of a per-kernel event: p2p / lifecycle / btl suites, latency
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_p2p_gpu.py tests/test_lifecycle_gpu.py tests/test_btl_gpu.py > gpurun_out/r5bd_tests.txt 2>&1 || { echo FAILED; tail -60 gpurun_out/r5bd_tests.txt; exit 1; }
tail -1 gpurun_out/r5bd_tests.txt
for k in 1 2; do
  P2P_LAT_DIST=1 P2P_LAT_ITERS=300 timeout -k 10 200 python -u tools/p2p_lat.py > gpurun_out/r5bd_lat_$k.txt 2>&1 || exit 1
  grep -E "p10/25" gpurun_out/r5bd_lat_$k.txt | sed 's/first 40:.*p10/p10/' | head -4
  tail -1 gpurun_out/r5bd_lat_$k.txt
done
