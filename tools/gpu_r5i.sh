# round 5 (i): the GPU test files from test_convertor_hook_gpu on (r5h stopped there on a test bug), then r5g
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
F="tests/test_convertor_hook_gpu.py tests/test_convertor_pins.py tests/test_lifecycle_gpu.py tests/test_nbc_gpu.py tests/test_nbc_oracle.py tests/test_op_consumer_gpu.py tests/test_op_service_gpu.py tests/test_oracle_golden.py tests/test_osc_gpu.py tests/test_p2p_gpu.py tests/test_rccl_gpu.py tests/test_reduce_gpu.py tests/test_shmem.py tests/test_x87_host.py"
STEP_TIMEOUT=700 bash tools/gpu_pytest.sh r5i_rest "$F -m gpu --durations=30" || exit $?
bash tools/gpu_r5g.sh
