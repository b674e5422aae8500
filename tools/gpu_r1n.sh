set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_osc_gpu.py -x -v --timeout 300 --timeout-method thread > $O/r1n_osc.txt 2>&1 || { tail -60 $O/r1n_osc.txt; exit 1; }
tail -5 $O/r1n_osc.txt
