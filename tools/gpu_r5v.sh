# round 5 (v): what bounds the unpack kernels -- SQ counters per kernel (struct / BLACS / vector)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
P=$O/pmc_unpack_r5v
mkdir -p $P
i=0
for t in struct_char_d3_int_resized48 ref_blacs_indexed vector_f32_b4_s8; do
  i=$((i+1))
  for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" WRITE_SIZE; do
    n=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $P/pmc_${i}_$n -o run -- python3 tools/pmc_unpack.py $t 2 > $P/pmc_${i}_$n.log 2>&1 || exit 1
  done
  echo "$i $t" >> $P/pmc_index.txt
done
python tools/pmc_kernel_summary.py $P/pmc_* > $P/pmc_summary.jsonl
grep -v "k_pack" $P/pmc_summary.jsonl || true
