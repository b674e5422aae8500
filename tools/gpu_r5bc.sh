#!/bin/bash
# p2p latency modes: is the per-kernel p2p_last event record (an extra packet per kernel) behind the slow mode?
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for note in 1 0 1 0; do
  MX_P2P_NOTE=$note P2P_LAT_SIZES=8,4096 P2P_LAT_ITERS=400 P2P_LAT_DIST=1 timeout -k 10 200 python -u tools/p2p_lat.py > gpurun_out/r5bc_n$note.txt 2>&1 || exit 1
  echo "note=$note: $(grep 'p10/25' gpurun_out/r5bc_n$note.txt | sed 's/first 40:.*p10/p10/' | tr '\n' ' ')"
done
