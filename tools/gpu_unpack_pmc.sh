#!/bin/bash
# Unpack kernels against their floors on ONE box (round 4): product unpack times (conv_probe),
# the pattern-specific store / read+store floors (pattern_floor_probe), and per-kernel PMC
# FETCH_SIZE / WRITE_SIZE (separate passes) of pack + unpack at 1 GiB packed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${TAG:-unpack_pmc}
mkdir -p $O
TYPES=${TYPES:-"ref_blacs_indexed struct_char_d3_int_resized48 idx:100000:1 ref_struct vector_f32_b4_s8"}
timeout -k 10 300 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack,unpack $TYPES > $O/times.txt 2>&1 || exit 1
for t in blacs struct48; do timeout -k 10 100 ./tools/pattern_floor_probe $t >> $O/floors.txt 2>&1 || exit 1; done
timeout -k 10 300 python tools/conv_probe.py --bytes $((1<<30)) --dirs unpack $TYPES >> $O/times.txt 2>&1 || exit 1
i=0
for t in $TYPES; do
  i=$((i+1))
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${i}_$c -o run -- python3 tools/pmc_unpack.py $t 2 > $O/pmc_${i}_$c.log 2>&1 || exit 1
  done
  echo "$i $t" >> $O/pmc_index.txt
done
python tools/pmc_kernel_summary.py $O/pmc_* > $O/pmc_summary.jsonl
echo done
