set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
# scatter + allgather bcast: collective parity (2-4 processes) and the CFG-E bcast line at N=4 on one GPU
timeout -k 10 500 python -u -m pytest tests/test_coll_gpu.py tests/test_components_mp.py tests/test_nbc_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/r1aj_pytest.txt 2>&1 || { tail -40 $O/r1aj_pytest.txt; exit 1; }
tail -1 $O/r1aj_pytest.txt
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 4 --steps 3 --warmup 1 > $O/r1aj_bench_n4.txt 2>&1 || { tail -30 $O/r1aj_bench_n4.txt; exit 1; }
tail -1 $O/r1aj_bench_n4.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['cfg_e'].get('bcast'))"
