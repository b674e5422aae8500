# round 5 (j): byte-map PACK with a 32-bit tile loop and the wrapped map; parity, A/B, floors, PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=400 bash tools/gpu_pytest.sh r5j_conv "tests/test_convertor.py tests/test_convertor_pins.py tests/test_convertor_hook_gpu.py -m gpu" || exit $?
A256=$(python tools/pack_floor_args.py $((256<<20)))
A1G=$(python tools/pack_floor_args.py $((1<<30)))
for sh in 0 16; do
  echo "== PFP_SHIFT=$sh" >> $O/pack_floor_r5j.txt
  PFP_SHIFT=$sh timeout -k 10 120 ./tools/pack_floor_probe $A256 >> $O/pack_floor_r5j.txt 2>&1 || exit $?
  PFP_SHIFT=$sh timeout -k 10 120 ./tools/pack_floor_probe $A1G >> $O/pack_floor_r5j.txt 2>&1 || exit $?
done
T="struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed ref_struct ref_strange"
for rep in 1 2; do
for v in "" "MX_CONV_BMAP_ALIGN=16" "MX_CONV_BMAP_DW=0"; do
  echo "== $v (rep $rep)" >> $O/conv_ab_r5j.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack $T >> $O/conv_ab_r5j.txt 2>&1 || exit $?
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack $T >> $O/conv_ab_r5j.txt 2>&1 || exit $?
done
done
grep -v amdgpu.ids $O/conv_ab_r5j.txt
P=$O/pmc_pack_r5j
mkdir -p $P
i=0
for t in struct_char_d3_int_resized48 indexed_f32_random; do
  i=$((i+1))
  for c in FETCH_SIZE "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"; do
    n=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $P/pmc_${i}_$n -o run -- python3 tools/pmc_unpack.py $t 2 > $P/pmc_${i}_$n.log 2>&1 || exit 1
  done
  echo "$i $t" >> $P/pmc_index.txt
done
python tools/pmc_kernel_summary.py $P/pmc_* > $P/pmc_summary.jsonl
grep -i "k_pack_bmap" $P/pmc_summary.jsonl || true
