#!/bin/bash
# GPU-box helper, round 3 close: whole GPU suite + smoke, the N=1 bench line,
# a rocprofv3 kernel-stats pass of the same command, the 176-pair sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=${O:-gpurun_out/final_r3}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 240 --timeout-method thread > $O/full_gpu.log 2>&1 || { tail -20 $O/full_gpu.log; exit 1; }
tail -1 $O/full_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/prof.log 2>&1 || exit 1
[ "${SWEEP:-1}" = 0 ] || timeout -k 10 600 python tools/sweep.py --what pairs --out $O/sweep_pairs.json > $O/sweep_pairs.txt 2>&1 || exit 1
echo done
