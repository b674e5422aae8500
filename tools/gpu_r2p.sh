# collectives with relaxed flag stores after explicit fences: parity + latency
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_coll_gpu.py tests/test_nbc_gpu.py tests/test_osc_gpu.py tests/test_coll_tree.py > $O/r2p_coll.txt 2>&1 || { tail -40 $O/r2p_coll.txt; exit 1; }
tail -2 $O/r2p_coll.txt
for n in 2 4; do
  timeout -k 10 300 python -u tools/lat_probe.py $n 2>&1 | grep "^n=" >> $O/r2p_lat.txt || exit 1
done
cat $O/r2p_lat.txt
echo ok
