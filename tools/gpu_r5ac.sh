# round 5 (ac): FETCH / WRITE per pack kernel for the remaining CFG-C types (1 GiB packed)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
P=$O/pmc_pack_r5ac
mkdir -p $P
i=0
for t in vector_f32_b1_s2 vector_f64_b3_s5 vector_f32_b4_s8 vector_f32_b64_s128 ref_struct ref_strange; do
  i=$((i+1))
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $P/pmc_${i}_$c -o run -- python3 tools/pmc_unpack.py $t 2 > $P/pmc_${i}_$c.log 2>&1 || exit 1
  done
  echo "$i $t $(grep path $P/pmc_${i}_FETCH_SIZE.log | tail -1)" >> $P/pmc_index.txt
done
python tools/pmc_kernel_summary.py $P/pmc_* | grep -v -e copyBuffer -e distribution_elementwise > $P/pmc_summary.jsonl
cat $P/pmc_index.txt
cat $P/pmc_summary.jsonl
