# round 5 (m): byte-map PACK contiguous-word path; op-service interference by fence (diagnostic switches)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=400 bash tools/gpu_pytest.sh r5m_conv "tests/test_convertor.py tests/test_convertor_pins.py tests/test_convertor_hook_gpu.py -m gpu" || exit $?
T="struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed ref_struct ref_strange"
for rep in 1 2; do
for v in "" "MX_CONV_BMAP_CW=0"; do
  echo "== $v (rep $rep)" >> $O/conv_ab_r5m.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack $T >> $O/conv_ab_r5m.txt 2>&1 || exit $?
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack $T >> $O/conv_ab_r5m.txt 2>&1 || exit $?
done
done
grep -v amdgpu.ids $O/conv_ab_r5m.txt
for d in 0 1 2 3 4 7; do
  echo "== MX_SVC_DIAG=$d" >> $O/svc_diag_r5m.txt
  MX_SVC_DIAG=$d timeout -k 10 200 python tools/svc_interference.py --sizes 65536 --reps 30 >> $O/svc_diag_r5m.txt 2>&1 || exit $?
done
grep -v amdgpu.ids $O/svc_diag_r5m.txt
P=$O/pmc_pack_r5m
mkdir -p $P
i=0
for t in struct_char_d3_int_resized48 ref_blacs_indexed; do
  i=$((i+1))
  for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" FETCH_SIZE; do
    n=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $P/pmc_${i}_$n -o run -- python3 tools/pmc_unpack.py $t 2 > $P/pmc_${i}_$n.log 2>&1 || exit 1
  done
  echo "$i $t" >> $P/pmc_index.txt
done
python tools/pmc_kernel_summary.py $P/pmc_* > $P/pmc_summary.jsonl
grep -i "k_pack_bmap" $P/pmc_summary.jsonl || true
