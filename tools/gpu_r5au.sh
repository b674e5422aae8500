#!/bin/bash
# p2p small-message latency: kernel + HIP API trace of the 2-process ping-pong (8 B, 300 iterations)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
P2P_LAT_SIZES=8 P2P_LAT_ITERS=300 P2P_LAT_DIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/r5au_trace -o run -- python3 tools/p2p_lat.py > gpurun_out/r5au_lat.txt 2>&1 || exit 1
grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/r5au_lat.txt | tail -3
find gpurun_out/r5au_trace -name "*.csv" | head -20
