set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/r1t_pytest.txt 2>&1 || { tail -40 $O/r1t_pytest.txt; exit 1; }
tail -2 $O/r1t_pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r1t_smoke.txt 2>&1 || { tail -20 $O/r1t_smoke.txt; exit 1; }
tail -2 $O/r1t_smoke.txt
