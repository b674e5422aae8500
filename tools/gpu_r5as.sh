#!/bin/bash
# p2p small-message latency modes: host spin-loop pauses A/B (MX_WAIT_PAUSE), 400 iterations
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for pz in 0 8 0 8; do
  MX_WAIT_PAUSE=$pz P2P_LAT_SIZES=8,4096 P2P_LAT_ITERS=400 P2P_LAT_DIST=1 timeout -k 10 200 python -u tools/p2p_lat.py > gpurun_out/r5as_p$pz.txt 2>&1 || exit 1
  echo "pause=$pz: $(grep 'p10/25' gpurun_out/r5as_p$pz.txt | sed 's/first 40:.*p10/p10/' | tr '\n' ' ')"
done
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; taskset -p $$ 2>/dev/null
