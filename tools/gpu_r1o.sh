set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_p2p_gpu.py -x -v --timeout 300 --timeout-method thread > $O/r1o_p2p.txt 2>&1 || { tail -80 $O/r1o_p2p.txt; exit 1; }
tail -5 $O/r1o_p2p.txt
timeout -k 10 600 python -u -m pytest tests/test_nbc_gpu.py tests/test_osc_gpu.py tests/test_coll_gpu.py -x -q -k "multiprocess or nonblocking or one_sided" --timeout 300 --timeout-method thread > $O/r1o_mp.txt 2>&1 || { tail -60 $O/r1o_mp.txt; exit 1; }
tail -3 $O/r1o_mp.txt
