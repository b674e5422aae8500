# round 5 (x): the N>1 bench lines with the CFG-D sweep and CFG-E (ranks sharing the box's GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_r5x_n2.txt 2>&1 || exit $?
grep '^{"metric"' $O/bench_r5x_n2.txt > $O/bench_r5x_n2.json
timeout -k 10 500 python bench.py --gpus 4 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_r5x_n4.txt 2>&1 || exit $?
grep '^{"metric"' $O/bench_r5x_n4.txt > $O/bench_r5x_n4.json
ls -la $O/bench_r5x*
