# round 5 (ag): the reduce / convertor / collective suites with non-temporal accesses forced everywhere
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
MX_NT_MIN_BYTES=0 STEP_TIMEOUT=700 bash tools/gpu_pytest.sh r5ag_nt "tests/test_reduce_gpu.py tests/test_convertor.py tests/test_coll_gpu.py tests/test_op_service_gpu.py -m gpu -q" || exit $?
