set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/r1h_pmc_fetch -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/r1h_pmc_fetch.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/r1h_pmc_write -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 > $O/r1h_pmc_write.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r1h_prof -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $O/r1h_prof.txt 2>&1 || exit 1
ls -R $O/r1h_pmc_fetch | head
