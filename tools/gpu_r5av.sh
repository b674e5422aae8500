#!/bin/bash
# larger unexpected-message tables (stash 16, deferred 64): the bound test and the whole p2p file
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_p2p_gpu.py > gpurun_out/r5av_p2p.txt 2>&1 || { echo FAILED; tail -80 gpurun_out/r5av_p2p.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r5av_p2p.txt
