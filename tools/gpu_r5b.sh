# round 5 (b): lifecycle probe, direct zero-copy results, service / mark fixes, N=2 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
timeout -k 10 120 ./tools/lifecycle_sync_probe > $O/lifecycle_sync_probe.txt 2>&1 || exit $?
STEP_TIMEOUT=400 bash tools/gpu_pytest.sh r5b "tests/test_coll_gpu.py -k 'zero_copy or path_switching'" \
  "tests/test_components_rules.py -k stale" "tests/test_op_service_gpu.py" || exit $?
for d in 1 0 1 0; do
  MX_ZC_DIRECT=$d timeout -k 10 200 python bench.py --gpus 2 --steps 20 --warmup 5 --no-sweep --no-cpu-baseline \
     > $O/bench_n2_direct$d.json 2> $O/bench_n2_direct$d.err || exit $?
  tail -c 600 $O/bench_n2_direct$d.json | head -c 300; echo
done
