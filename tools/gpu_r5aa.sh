# round 5 (aa): the full GPU suite on the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
STEP_TIMEOUT=1000 bash tools/gpu_pytest.sh r5aa_full "tests -m gpu --durations=15" || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
