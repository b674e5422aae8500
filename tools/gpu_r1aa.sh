set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
# N=8 / N=4 rehearsal of the driver's scaling command with every rank on the one GPU of this box
# (plumbing only: no xGMI here, ranks share one HBM)
for n in 8 4; do
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2952$n bench.py --gpus $n --steps 3 --warmup 1 > $O/r1aa_bench_n$n.txt 2>&1 || { tail -30 $O/r1aa_bench_n$n.txt; exit 1; }
tail -1 $O/r1aa_bench_n$n.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['value'], d.get('allreduce_error'), d['roofline']['phase_ms_per_call'], len(d.get('sweep',[])), [ (k, v.get('busbw_gbs', v.get('error'))) for k,v in (d.get('cfg_e') or {}).items() if isinstance(v, dict)])"
done
