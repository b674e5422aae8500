#!/bin/bash
# GPU-box helper: the round-3 parity tests (forced algorithms, component order/paths)
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 400 $T tests/test_coll_gpu.py -k "nonoverlapping_local or forced_local" > gpurun_out/r3a_local.log 2>&1 || { tail -30 gpurun_out/r3a_local.log; exit 1; }
tail -2 gpurun_out/r3a_local.log
timeout -k 10 600 $T tests/test_components_rules.py > gpurun_out/r3a_rules.log 2>&1 || { tail -40 gpurun_out/r3a_rules.log; exit 1; }
tail -2 gpurun_out/r3a_rules.log
timeout -k 10 500 $T tests/test_components_mp.py tests/test_components.py > gpurun_out/r3a_comp.log 2>&1 || { tail -40 gpurun_out/r3a_comp.log; exit 1; }
tail -2 gpurun_out/r3a_comp.log
