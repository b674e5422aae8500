#!/bin/bash
# the driver's scaling-command form at N=8 on the final tree (8 processes share the one GPU here)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python bench.py --gpus 8 > gpurun_out/bench_r5an_n8.txt 2>&1 || { echo BENCH8_FAILED; tail -40 gpurun_out/bench_r5an_n8.txt; exit 1; }
grep '^{"metric"' gpurun_out/bench_r5an_n8.txt | cut -c1-600
