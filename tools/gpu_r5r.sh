# round 5 (r): byte-map PACK defaults (24 / 12 KiB span by map size, 4-dword gather, nt, word maps): parity,
# every CFG-C type's pack against its floor on one box, PMC of the byte-map kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=500 bash tools/gpu_pytest.sh r5r_conv "tests/test_convertor.py tests/test_convertor_pins.py tests/test_convertor_hook_gpu.py tests/test_convertor_variants_gpu.py -m gpu --durations=10" || exit $?
T="vector_f32_b1_s2 vector_f32_b4_s8 vector_f64_b3_s5 vector_f32_b16_s32 vector_f32_b64_s128 indexed_f32_random struct_char_d3_int_resized48 ref_blacs_indexed ref_struct ref_strange"
for rep in 1 2; do
  echo "== default (rep $rep)" >> $O/conv_r5r.txt
  timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack $T >> $O/conv_r5r.txt 2>&1 || exit $?
  timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack $T >> $O/conv_r5r.txt 2>&1 || exit $?
  echo "== MX_CONV_BMAP_WORD=0 (rep $rep)" >> $O/conv_r5r.txt
  MX_CONV_BMAP_WORD=0 timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack indexed_f32_random ref_blacs_indexed >> $O/conv_r5r.txt 2>&1 || exit $?
  MX_CONV_BMAP_WORD=0 timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack indexed_f32_random ref_blacs_indexed >> $O/conv_r5r.txt 2>&1 || exit $?
  timeout -k 10 120 ./tools/pack_floor_probe $(python tools/pack_floor_args.py $((256<<20))) >> $O/pack_floor_r5r.txt 2>&1 || exit $?
  timeout -k 10 120 ./tools/pack_floor_probe $(python tools/pack_floor_args.py $((1<<30))) >> $O/pack_floor_r5r.txt 2>&1 || exit $?
done
grep -v amdgpu.ids $O/conv_r5r.txt | grep -v "^$"
P=$O/pmc_pack_r5r
mkdir -p $P
i=0
for t in struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed; do
  i=$((i+1))
  for c in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
    n=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $P/pmc_${i}_$n -o run -- python3 tools/pmc_unpack.py $t 2 > $P/pmc_${i}_$n.log 2>&1 || exit 1
  done
  echo "$i $t" >> $P/pmc_index.txt
done
python tools/pmc_kernel_summary.py $P/pmc_* > $P/pmc_summary.jsonl
grep -i "k_pack_bmap" $P/pmc_summary.jsonl || true
