#!/bin/bash
# yield tests with relaunch counts, then p2p latency A/B (median round trip), yielding on / off, twice
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  "tests/test_p2p_gpu.py::test_yield_with_datatypes_test_polling_and_persistent" \
  "tests/test_p2p_gpu.py::test_receives_yield_to_receives_posted_after_them" > gpurun_out/r5ba_yield.txt 2>&1 || { echo FAILED; tail -80 gpurun_out/r5ba_yield.txt; exit 1; }
tail -4 gpurun_out/r5ba_yield.txt
