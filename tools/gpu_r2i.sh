# two-shot with one vector per lane: parity + latency A/B at n = 2 and 4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_coll_gpu.py -k "multiprocess" > $O/r2i_pytest.txt 2>&1 || { tail -40 $O/r2i_pytest.txt; exit 1; }
tail -2 $O/r2i_pytest.txt
for n in 2 4; do
for t in 0 default; do
  if [ $t = 0 ]; then export MX_TWOSHOT_MAX=0; else unset MX_TWOSHOT_MAX; fi
  timeout -k 10 300 python -u tools/lat_probe.py $n 2>&1 | grep "^n=" >> $O/r2i_lat.txt || exit 1
done
done
cat $O/r2i_lat.txt
echo ok
