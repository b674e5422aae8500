set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/r1f_pytest.txt 2>&1
rc=$?
tail -15 $O/r1f_pytest.txt
exit $rc
