set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_p2p_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/r1ad_p2p.txt 2>&1 || { tail -60 $O/r1ad_p2p.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/r1ad_p2p.txt | tail -5
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/r1ad_pytest.txt 2>&1 || { tail -40 $O/r1ad_pytest.txt; exit 1; }
tail -1 $O/r1ad_pytest.txt
