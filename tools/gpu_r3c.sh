#!/bin/bash
# GPU-box helper, round 3: the partial-line write floor (sector_probe with
# prefetch variants), the convertor types VERDICT r2 names at 1 GiB, and
# single-counter PMC passes for BLACS / matrix-borders pack + unpack.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3c
mkdir -p $O
STAGES=${STAGES:-"sector conv pmc"}
CONV_TYPES=${CONV_TYPES:-"ref_blacs_indexed ref_matrix_borders_20_3 indexed_f32_random struct_char_d3_int_resized48 idx:100000:1"}
for s in $STAGES; do
  echo "[$(date +%T)] $s"
  case $s in
    sector)
      timeout -k 10 120 ./tools/sector_probe > $O/sector.txt 2>&1 || exit 1 ;;
    sectorbig)
      timeout -k 10 120 ./tools/sector_probe big > $O/sector_big.txt 2>&1 || exit 1 ;;
    blktest)
      timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_convertor.py \
          -k "block_kernels" > $O/blktest.log 2>&1 || { tail -30 $O/blktest.log; exit 1; } ;;
    convtest)   # every convertor test on the device
      timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convertor.py \
          tests/test_convertor_pins.py -m gpu > $O/convtest.log 2>&1 || { tail -30 $O/convtest.log; exit 1; } ;;
    convall)    # every golden type + the large-instance types at 1 GiB
      TYPES=$(python -c "
import sys; sys.path.insert(0, 'tests'); import golden_io
print(' '.join(r['name'] for r in golden_io.ddt_records()[1]))")
      timeout -k 10 600 python -u tools/conv_probe.py $TYPES idx:100000:1 idx:20000:2 tri:500 tri:2000 \
          2>&1 | grep -v amdgpu.ids > $O/conv_all.txt || exit 1 ;;
    convab)   # default dispatch vs the BLOCK kernels forced on every golden type
      for b in 1 2; do
        echo "MX_CONV_BLK=$b" >> $O/conv_ab.txt
        MX_CONV_BLK=$b timeout -k 10 400 python -u tools/conv_probe.py $CONV_TYPES >> $O/conv_ab.txt 2>&1 || exit 1
      done ;;
    blkab)    # BLOCK kernel geometry on the large-instance types
      IFS='|' read -ra CFGS <<< "${BLK_CFGS:-NG=0 W4=1 SPAN=1}"
      for cfg in "${CFGS[@]}"; do
        echo "$cfg" >> $O/blk_ab.txt
        env $(for kv in $cfg; do echo MX_CONV_BLK_$kv; done) timeout -k 10 200 python -u tools/conv_probe.py \
            ${BLK_TYPES:-idx:100000:1 idx:20000:2 tri:500 tri:2000} 2>&1 | grep -v amdgpu.ids >> $O/blk_ab.txt || exit 1
      done ;;
    conv)
      timeout -k 10 400 python -u tools/conv_probe.py $CONV_TYPES > $O/conv.txt 2>&1 || exit 1 ;;
    pmc)
      for t in ${PMC_TYPES:-ref_blacs_indexed ref_matrix_borders_20_3}; do
        for c in FETCH_SIZE WRITE_SIZE; do
          d=$(echo $t | tr ':' '_')
          timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${d}_$c -o run -- \
              python3 tools/pmc_unpack.py $t 2 > $O/pmc_${d}_$c.log 2>&1 || exit 1
        done
      done ;;
  esac
done
echo done
