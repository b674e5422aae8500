set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/r1v_pytest.txt 2>&1 || { tail -40 $O/r1v_pytest.txt; exit 1; }
tail -1 $O/r1v_pytest.txt
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $O/r1v_bench_n2.txt 2>&1 || { tail -30 $O/r1v_bench_n2.txt; exit 1; }
tail -1 $O/r1v_bench_n2.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['phase_ms_per_call'])"
