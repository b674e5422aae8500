set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_coll_gpu.py -x -v -m gpu -k multiprocess --timeout 400 --timeout-method thread > $O/r1am_pytest.txt 2>&1 || { tail -60 $O/r1am_pytest.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/r1am_pytest.txt | tail -6
