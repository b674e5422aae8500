set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/r1m_pytest.txt 2>&1 || { tail -80 $O/r1m_pytest.txt; exit 1; }
tail -3 $O/r1m_pytest.txt
