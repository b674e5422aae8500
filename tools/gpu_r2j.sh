# two-shot workgroup-count sweep; p2p completion word
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_p2p_gpu.py > $O/r2j_p2p.txt 2>&1 || { tail -40 $O/r2j_p2p.txt; exit 1; }
tail -2 $O/r2j_p2p.txt
timeout -k 10 300 python -u tools/p2p_lat.py 2>&1 | grep "half" > $O/r2j_p2plat.txt || exit 1
cat $O/r2j_p2plat.txt
for w in 8 32 128; do
  echo "WG=$w" >> $O/r2j_lat.txt
  MX_TWOSHOT_WG=$w timeout -k 10 300 python -u tools/lat_probe.py 2 2>&1 | grep "^n=" >> $O/r2j_lat.txt || exit 1
done
cat $O/r2j_lat.txt
echo ok
