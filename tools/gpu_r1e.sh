set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_coll_tree.py tests/test_coll_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/r1e_pytest.txt 2>&1
rc=$?
tail -30 $O/r1e_pytest.txt
exit $rc
