#!/bin/bash
# GPU-box helper: N=1 bench, then the N=2 bench path (2 ranks on the one GPU).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || exit $?
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err
