set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
# p2p latency A/B: previous build (per-receive pinned status allocation) vs the status pool
L=zhpe-ompi_amd/lib/libmx_kernels.so
cp $L /tmp/libmx_new.so
cp tools/libmx_kernels_prev.so $L
timeout -k 10 150 python -u tools/p2p_lat.py > $O/r1ah_p2p_prev.txt 2>&1 || { cp /tmp/libmx_new.so $L; tail -20 $O/r1ah_p2p_prev.txt; exit 1; }
cp /tmp/libmx_new.so $L
timeout -k 10 150 python -u tools/p2p_lat.py > $O/r1ah_p2p_new.txt 2>&1 || { tail -20 $O/r1ah_p2p_new.txt; exit 1; }
echo prev; tail -1 $O/r1ah_p2p_prev.txt; echo new; tail -1 $O/r1ah_p2p_new.txt
timeout -k 10 400 python -u -m pytest tests/test_p2p_gpu.py tests/test_nbc_gpu.py tests/test_osc_gpu.py tests/test_components_mp.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/r1ah_pytest.txt 2>&1 || { tail -40 $O/r1ah_pytest.txt; exit 1; }
tail -1 $O/r1ah_pytest.txt
