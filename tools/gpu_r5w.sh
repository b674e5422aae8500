# round 5 (w): piece UNPACK with a 32-bit store loop -- parity, A/B, SQ counters (old and new)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=400 bash tools/gpu_pytest.sh r5w_conv "tests/test_convertor.py tests/test_convertor_pins.py tests/test_convertor_hook_gpu.py -m gpu" || exit $?
T="struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed ref_struct ref_strange vector_f32_b4_s8"
for rep in 1 2; do
for v in "" "MX_CONV_UNPACK_U32=0"; do
  echo "== $v (rep $rep)" >> $O/conv_ab_r5w.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs unpack $T >> $O/conv_ab_r5w.txt 2>&1 || exit $?
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs unpack $T >> $O/conv_ab_r5w.txt 2>&1 || exit $?
done
done
grep -v amdgpu.ids $O/conv_ab_r5w.txt | grep -v "^$"
P=$O/pmc_unpack_r5w
mkdir -p $P
i=0
for v in "MX_CONV_UNPACK_U32=1" "MX_CONV_UNPACK_U32=0"; do
for t in struct_char_d3_int_resized48 ref_blacs_indexed; do
  i=$((i+1))
  c="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
  env $v timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $P/pmc_${i}_sq -o run -- python3 tools/pmc_unpack.py $t 2 > $P/pmc_${i}.log 2>&1 || exit 1
  echo "$i $t $v" >> $P/pmc_index.txt
done
done
python tools/pmc_kernel_summary.py $P/pmc_* > $P/pmc_summary.jsonl
grep -v "k_pack" $P/pmc_summary.jsonl || true
