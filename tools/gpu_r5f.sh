# round 5 (f): repeat the 8-rank zero-copy test (direct / gather) to separate a direct-write race from
# 8-processes-on-one-GPU scheduling; then the rest of the suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
for i in 1 2 3; do
  for v in 8-direct 8-gather; do
    timeout -k 10 150 python -u -m pytest -q --timeout 120 --timeout-method thread "tests/test_coll_gpu.py::test_multiprocess_allreduce_zero_copy[$v]" > $O/r5f_zc_${v}_$i.txt 2>&1
    echo "$v $i rc=$?" | tee -a $O/r5f_zc_summary.txt
  done
done
STEP_TIMEOUT=850 bash tools/gpu_pytest.sh r5f_full "tests -m gpu --durations=40 --deselect 'tests/test_coll_gpu.py::test_multiprocess_allreduce_zero_copy'" || exit $?
