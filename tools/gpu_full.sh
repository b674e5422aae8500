#!/bin/bash
# GPU-box helper: the whole GPU test suite + smoke, output under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 240 --timeout-method thread > gpurun_out/full_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/full_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
