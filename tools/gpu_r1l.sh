set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_nbc_gpu.py -x -v --timeout 300 --timeout-method thread > $O/r1l_nbc.txt 2>&1 || { tail -60 $O/r1l_nbc.txt; exit 1; }
tail -5 $O/r1l_nbc.txt
timeout -k 10 600 python -u -m pytest tests/test_coll_gpu.py -x -q -k "multiprocess" --timeout 300 --timeout-method thread > $O/r1l_mp.txt 2>&1 || { tail -60 $O/r1l_mp.txt; exit 1; }
tail -3 $O/r1l_mp.txt
