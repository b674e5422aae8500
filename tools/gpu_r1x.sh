set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_convertor.py tests/test_p2p_gpu.py tests/test_osc_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/r1x_pytest.txt 2>&1 || { tail -40 $O/r1x_pytest.txt; exit 1; }
tail -1 $O/r1x_pytest.txt
timeout -k 10 300 python -u tools/sweep.py --what pack --max-bytes 1073741824 --out $O/r1x_sweep_vec.json > $O/r1x_sweep_vec.txt 2>&1 || { tail -20 $O/r1x_sweep_vec.txt; exit 1; }
MX_CONV_VEC=0 timeout -k 10 300 python -u tools/sweep.py --what pack --max-bytes 1073741824 --out $O/r1x_sweep_tile.json > $O/r1x_sweep_tile.txt 2>&1 || { tail -20 $O/r1x_sweep_tile.txt; exit 1; }
grep 1073 $O/r1x_sweep_vec.txt; grep 1073 $O/r1x_sweep_tile.txt
