# round 5 (be): final tree (channel completion words instead of per-kernel events) --: the full GPU suite on the final tree, then smoke and the N=1 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=1000 bash tools/gpu_pytest.sh r5be_full "tests -m gpu --durations=15" || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
timeout -k 10 400 python bench.py > $O/bench_r5be_n1.txt 2>&1 || exit $?
grep '^{"metric"' $O/bench_r5be_n1.txt | cut -c1-300
