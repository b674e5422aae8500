# round 5 (u): p2p pick kernel (scanned-envelope cache), stale IPC imports kept until closed
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
STEP_TIMEOUT=600 bash tools/gpu_pytest.sh r5u "tests/test_p2p_gpu.py tests/test_btl_gpu.py tests/test_lifecycle_gpu.py tests/test_coll_gpu.py tests/test_components_mp.py -m gpu --durations=10" || exit $?
