#!/bin/bash
# yield tests with relaunch counts, then p2p latency A/B (median round trip), yielding on / off, twice
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  "tests/test_p2p_gpu.py::test_yield_with_datatypes_test_polling_and_persistent" \
  "tests/test_p2p_gpu.py::test_receives_yield_to_receives_posted_after_them" > gpurun_out/r5ak_yield.txt 2>&1 || { echo FAILED; tail -80 gpurun_out/r5ak_yield.txt; exit 1; }
tail -4 gpurun_out/r5ak_yield.txt
for k in 1 2; do
  timeout -k 10 200 python -u tools/p2p_lat.py > gpurun_out/r5ak_lat_on_$k.txt 2>&1 || exit 1
  MX_P2P_YIELD=0 timeout -k 10 200 python -u tools/p2p_lat.py > gpurun_out/r5ak_lat_off_$k.txt 2>&1 || exit 1
  echo "on  $k: $(tail -1 gpurun_out/r5ak_lat_on_$k.txt)"
  echo "off $k: $(tail -1 gpurun_out/r5ak_lat_off_$k.txt)"
done
