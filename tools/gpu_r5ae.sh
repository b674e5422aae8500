# round 5 (ae): registration fast path -- the new test, the collective suites, N=2 bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=700 bash tools/gpu_pytest.sh r5ae "tests/test_coll_gpu.py tests/test_components_rules.py tests/test_components_mp.py tests/test_coll_headline_gpu.py tests/test_lifecycle_gpu.py -m gpu --durations=8" || exit $?
for rep in 1 2; do
for v in "" "MX_REG_FAST=0"; do
  env $v timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 3 --no-sweep --no-cpu-baseline > $O/bench_r5ae.txt 2>&1 || exit $?
  echo "== $v (rep $rep) $(grep '^{"metric"' $O/bench_r5ae.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O/reg_fast_ab_r5ae.txt
done
done
cat $O/reg_fast_ab_r5ae.txt
