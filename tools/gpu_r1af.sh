set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
for n in 2 4; do
  timeout -k 10 150 python -u tools/lat_probe.py $n > $O/r1af_lat_n$n.txt 2>&1 || { tail -20 $O/r1af_lat_n$n.txt; exit 1; }
  MX_ONESHOT_MAX=262144 timeout -k 10 150 python -u tools/lat_probe.py $n > $O/r1af_lat256k_n$n.txt 2>&1 || { tail -20 $O/r1af_lat256k_n$n.txt; exit 1; }
done
grep "n=" $O/r1af_lat_*.txt
timeout -k 10 400 python -u -m pytest tests/test_coll_gpu.py tests/test_nbc_gpu.py tests/test_components_mp.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/r1af_pytest.txt 2>&1 || { tail -40 $O/r1af_pytest.txt; exit 1; }
tail -1 $O/r1af_pytest.txt
