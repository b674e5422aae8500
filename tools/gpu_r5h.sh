# round 5 (h): the full GPU suite with lifecycle work on the legacy default stream
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
STEP_TIMEOUT=1000 bash tools/gpu_pytest.sh r5h_full "tests -m gpu --durations=40" || exit $?
