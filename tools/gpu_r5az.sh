#!/bin/bash
# randomised wildcard receives (ANY_SOURCE / ANY_TAG) with yielding: delivery, patterns, non-overtaking
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread "tests/test_p2p_gpu.py::test_randomised_wildcard_receives_keep_non_overtaking" > gpurun_out/r5az_wild.txt 2>&1 || { echo FAILED; tail -80 gpurun_out/r5az_wild.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed|seed" gpurun_out/r5az_wild.txt
