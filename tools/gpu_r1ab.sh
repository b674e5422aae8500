set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_reduce_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/r1ab_pytest.txt 2>&1 || { tail -40 $O/r1ab_pytest.txt; exit 1; }
tail -1 $O/r1ab_pytest.txt
for r in 1 2 3; do
  for x in 1 0; do
    MX_K1_XCD=$x timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --warmup 5 > $O/r1ab_b$x$r.txt 2>&1 || { tail -20 $O/r1ab_b$x$r.txt; exit 1; }
    tail -1 $O/r1ab_b$x$r.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('xcd=$x', d['value'], d['roofline']['achieved'], d['roofline']['avg_kernel_ms'])"
  done
done
