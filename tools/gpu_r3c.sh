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
    convab)   # default dispatch vs the BLOCK kernels forced on every golden type
      for b in 1 2; do
        echo "MX_CONV_BLK=$b" >> $O/conv_ab.txt
        MX_CONV_BLK=$b timeout -k 10 400 python -u tools/conv_probe.py $CONV_TYPES >> $O/conv_ab.txt 2>&1 || exit 1
      done ;;
    blkab)    # BLOCK kernel geometry on the large-instance types
      for cfg in ${BLK_CFGS:-"NG=0 W4=1 SPAN=1"}; do
        set -- $cfg
        echo "$cfg" >> $O/blk_ab.txt
        env MX_CONV_BLK_${1} MX_CONV_BLK_${2} MX_CONV_BLK_${3} timeout -k 10 200 python -u tools/conv_probe.py \
            ${BLK_TYPES:-idx:100000:1 idx:20000:2 tri:500 tri:2000} 2>&1 | grep -v amdgpu.ids >> $O/blk_ab.txt || exit 1
      done ;;
    conv)
      timeout -k 10 400 python -u tools/conv_probe.py $CONV_TYPES > $O/conv.txt 2>&1 || exit 1 ;;
    pmc)
      for t in ref_blacs_indexed ref_matrix_borders_20_3; do
        for c in FETCH_SIZE WRITE_SIZE; do
          timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${t}_$c -o run -- \
              python3 tools/pmc_unpack.py $t 2 > $O/pmc_${t}_$c.log 2>&1 || exit 1
        done
      done ;;
  esac
done
echo done
