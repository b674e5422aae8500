#!/bin/bash
# p2p small-message latency: distribution within a run (default, then channel streams at ordinary priority)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
P2P_LAT_SIZES=8,4096 P2P_LAT_ITERS=400 P2P_LAT_DIST=1 timeout -k 10 200 python -u tools/p2p_lat.py > gpurun_out/r5ar_dist.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5ar_dist.txt
P2P_LAT_SIZES=8,4096 P2P_LAT_ITERS=400 P2P_LAT_DIST=1 MX_P2P_PRIORITY=0 timeout -k 10 200 python -u tools/p2p_lat.py > gpurun_out/r5ar_dist_prio0.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5ar_dist_prio0.txt
