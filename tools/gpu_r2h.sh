# two-shot allreduce parity + latency; byte-map pack lane layout A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_coll_gpu.py -k "multiprocess or late" > $O/r2h_pytest.txt 2>&1 || { tail -40 $O/r2h_pytest.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/r2h_pytest.txt | tail -8
for t in 0 default; do
  if [ $t = 0 ]; then export MX_TWOSHOT_MAX=0; else unset MX_TWOSHOT_MAX; fi
  timeout -k 10 300 python -u tools/lat_probe.py 2 >> $O/r2h_lat.txt 2>&1 || exit 1
done
unset MX_TWOSHOT_MAX
timeout -k 10 300 python -u tools/lat_probe.py 4 >> $O/r2h_lat.txt 2>&1 || exit 1
cat $O/r2h_lat.txt | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_convertor.py > $O/r2h_conv.txt 2>&1 || { tail -30 $O/r2h_conv.txt; exit 1; }
tail -2 $O/r2h_conv.txt
T="struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed ref_lower_matrix_47 ref_upper_matrix_60 ref_matrix_borders_20_3 ref_struct"
for dw in 0 1; do
  echo "DW=$dw" >> $O/r2h_ab.txt
  MX_CONV_BMAP_DW=$dw timeout -k 10 240 python -u tools/conv_probe.py --dirs pack $T >> $O/r2h_ab.txt 2>&1 || exit 1
done
cat $O/r2h_ab.txt | grep -v amdgpu.ids
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/r2h_sq -o run -- python3 tools/conv_probe.py --reps 1 --dirs pack struct_char_d3_int_resized48 > $O/r2h_sq.log 2>&1 || exit 1
echo ok
