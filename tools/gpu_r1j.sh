set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
MX_DEBUG_IPC=1 timeout -k 10 400 python -u -m pytest tests/test_coll_gpu.py -x -q -s -m gpu -k "multiprocess or multirank" --timeout 300 --timeout-method thread > $O/r1j_pytest.txt 2>&1
rc=$?
grep -E "symheap|mx_heap|mx ipc|passed|failed|Error" $O/r1j_pytest.txt | head -40
exit $rc
