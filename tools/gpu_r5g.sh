# round 5 (g): pack floors + convertor A/B, op-service interference, GPU + CPU sweeps in one run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
T="struct_char_d3_int_resized48 indexed_f32_random vector_f32_b4_s8 ref_blacs_indexed ref_struct"
for B in $((256<<20)) $((1<<30)); do
  timeout -k 10 120 ./tools/pack_floor_probe $(python tools/pack_floor_args.py $B) >> $O/pack_floor_r5.txt 2>&1 || exit $?
done
for v in "" "MX_CONV_BLK=2" "MX_CONV_BMAP_DW=0" "MX_CONV_BMAP_PIPE=0"; do
  echo "== $v" >> $O/conv_ab_r5.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack $T >> $O/conv_ab_r5.txt 2>&1 || exit $?
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack $T >> $O/conv_ab_r5.txt 2>&1 || exit $?
done
cat $O/conv_ab_r5.txt
timeout -k 10 300 python tools/svc_interference.py --out $O/svc_interference_r5.json > $O/svc_interference_r5.txt 2>&1 || exit $?
cat $O/svc_interference_r5.txt
export MX_SWEEP_RUN="gpu_r5g $(date +%F_%T) $(hostname)"
timeout -k 10 500 python tools/sweep.py --what pairs --out $O/sweep_pairs_r5.json > $O/sweep_pairs_r5.log 2>&1 || exit $?
timeout -k 10 300 python tools/sweep.py --what pack --min-bytes $((128<<20)) --max-bytes $((1<<30)) --out $O/sweep_pack_r5.json > $O/sweep_pack_r5.log 2>&1 || exit $?
timeout -k 10 400 python tools/cpu_sweep.py --what pairs,pack --merge-gpu $O/sweep_pairs_r5.json,$O/sweep_pack_r5.json --out $O/cpu_sweep_r5.json > $O/cpu_sweep_r5.log 2>&1 || exit $?
head -5 $O/cpu_sweep_r5.txt
# per-kernel PMC of the pack kernels (separate passes: FETCH_SIZE, WRITE_SIZE, SQ LDS counters)
P=$O/pmc_pack_r5
mkdir -p $P
i=0
for t in struct_char_d3_int_resized48 indexed_f32_random vector_f32_b4_s8; do
  i=$((i+1))
  for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES"; do
    n=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $P/pmc_${i}_$n -o run -- python3 tools/pmc_unpack.py $t 2 > $P/pmc_${i}_$n.log 2>&1 || exit 1
  done
  echo "$i $t" >> $P/pmc_index.txt
done
python tools/pmc_kernel_summary.py $P/pmc_* > $P/pmc_summary.jsonl
grep -i "pack" $P/pmc_summary.jsonl | head -40 || true
