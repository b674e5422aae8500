# round 5 (s): smoke, N=1 bench, rocprof stats, PMC traffic; N=2 bench (two ranks on the box's GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
TAG=r5 STAGES="smoke bench prof pmc" bash tools/gpu_run.sh || exit $?
cat $O/r5_bench.txt | grep '^{"metric"' > $O/bench_r5_n1.json
timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --no-sweep --no-cpu-baseline > $O/bench_r5_n2.txt 2>&1 || exit $?
grep '^{"metric"' $O/bench_r5_n2.txt > $O/bench_r5_n2.json
cat $O/r5_log.txt
