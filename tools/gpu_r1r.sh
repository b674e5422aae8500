set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_coll_gpu.py tests/test_nbc_gpu.py -x -q -k "nonblocking" --timeout 300 --timeout-method thread > $O/r1r_rs.txt 2>&1 || { tail -60 $O/r1r_rs.txt; exit 1; }
tail -3 $O/r1r_rs.txt
