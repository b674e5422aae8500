# round 5 (z): kernel trace of the N=2 allreduce bench (two ranks on the box's GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r5z_prof -o run -- python3 bench.py --gpus 2 --steps 20 --warmup 3 --no-sweep --no-cpu-baseline > $O/r5z_bench.txt 2>&1 || exit $?
grep '^{"metric"' $O/r5z_bench.txt | cut -c1-400
find $O/r5z_prof -name "*kernel_stats.csv" | head
