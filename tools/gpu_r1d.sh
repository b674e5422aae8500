set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/r1d_pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/r1d_pytest.txt; exit 1; }
tail -1 $O/r1d_pytest.txt
timeout -k 10 300 python bench.py > $O/r1d_bench.txt 2>&1 || exit 1
tail -1 $O/r1d_bench.txt
timeout -k 10 300 python tools/sweep.py --what sizes --out $O/r1d_sweep_nt.json > /dev/null 2>&1 || exit 1
MX_NT_MIN_BYTES=-1 timeout -k 10 300 python tools/sweep.py --what sizes --out $O/r1d_sweep_nont.json > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r1d_prof -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/r1d_prof.txt 2>&1 || exit 1
echo done
