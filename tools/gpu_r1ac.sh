set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
for t in vector_f32_b4_s8 vector_f32_b1_s2; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/r1ac_f_$t -o run -- python3 tools/pmc_unpack.py $t 3 > $O/r1ac_f_$t.txt 2>&1 || { tail -20 $O/r1ac_f_$t.txt; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/r1ac_w_$t -o run -- python3 tools/pmc_unpack.py $t 3 > $O/r1ac_w_$t.txt 2>&1 || { tail -20 $O/r1ac_w_$t.txt; exit 1; }
done
ls -R $O | grep counter_collection | head
