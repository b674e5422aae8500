# p2p channel ordering relaxed: parity + latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_p2p_gpu.py tests/test_components_mp.py > $O/r2o_p2p.txt 2>&1 || { tail -40 $O/r2o_p2p.txt; exit 1; }
tail -2 $O/r2o_p2p.txt
timeout -k 10 300 python -u tools/p2p_lat.py 2>&1 | grep "half" > $O/r2o_p2plat.txt || exit 1
cat $O/r2o_p2plat.txt
echo ok
