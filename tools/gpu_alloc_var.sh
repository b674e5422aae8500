#!/bin/bash
# GPU-box helper, round 3: run-to-run spread of the N=1 headline -- three
# bench.py processes, two with the expandable-segments allocator, the
# in-process placement probe twice, and the raw-hipMalloc K1 shape probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/allocvar
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 180 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/bench$i.json 2> /dev/null || exit 1
done
for i in 1 2; do
  PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 180 python -u bench.py --no-cpu-baseline \
      --steps 20 --warmup 5 > $O/bench_exp$i.json 2> /dev/null || exit 1
done
for i in 1 2; do
  timeout -k 10 180 python -u tools/alloc_probe.py > $O/alloc$i.txt 2>&1 || exit 1
done
timeout -k 10 180 ./tools/bw_probe5 > $O/bw_probe5.txt 2>&1 || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/allocvar/bench*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["roofline"]["avg_kernel_ms"])
PY
cat $O/alloc1.txt $O/alloc2.txt
