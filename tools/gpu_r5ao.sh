#!/bin/bash
# shared-GPU roofline on the call's wall time: N=2 and N=8 in the driver's command form
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 8; do
  timeout -k 10 500 python bench.py --gpus $n > gpurun_out/bench_r5ao_n$n.txt 2>&1 || { echo BENCH_FAILED $n; tail -40 gpurun_out/bench_r5ao_n$n.txt; exit 1; }
  grep '^{"metric"' gpurun_out/bench_r5ao_n$n.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['value'], d['ms_per_step'], d['parity'], {k: d['roofline'][k] for k in ('achieved','frac','sum_of_rank_fold_rates_gbs')})"
done
