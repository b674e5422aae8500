# round 5 (ad): bench N=2 line with the shared-GPU HBM roofline; the bench test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=300 bash tools/gpu_pytest.sh r5ad "tests/test_bench_gpu.py -m gpu" || exit $?
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-sweep --no-cpu-baseline > $O/bench_r5ad_n2.txt 2>&1 || exit $?
grep '^{"metric"' $O/bench_r5ad_n2.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['roofline'])[:600])"
