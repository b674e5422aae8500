# byte-map pack (16/32-bit maps, monotonic spans) / piece unpack: parity, A/B, PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_convertor.py tests/test_convertor_pins.py > $O/r2g_pytest.txt 2>&1 || { tail -30 $O/r2g_pytest.txt; exit 1; }
tail -3 $O/r2g_pytest.txt
T="struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed ref_lower_matrix_47 ref_upper_matrix_60 ref_strange ref_struct_char_double ref_struct ref_twice_two_doubles ref_matrix_borders_20_3 ref_struct_constant_gap_resized vector_f64_b3_s5 ref_vector_450x10_s11_f64"
for b in 0 1; do
  echo "BMAP=$b" >> $O/r2g_ab.txt
  MX_CONV_BMAP=$b timeout -k 10 240 python -u tools/conv_probe.py $T >> $O/r2g_ab.txt 2>&1 || exit 1
done
cat $O/r2g_ab.txt
for b in 0 1; do
  MX_CONV_BMAP=$b timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/r2g_pmc_w$b -o run -- python3 tools/conv_probe.py --reps 1 --dirs unpack struct_char_d3_int_resized48 ref_lower_matrix_47 > $O/r2g_pmc_w$b.log 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/r2g_pmc_f -o run -- python3 tools/conv_probe.py --reps 1 struct_char_d3_int_resized48 ref_lower_matrix_47 > $O/r2g_pmc_f.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/r2g_sq -o run -- python3 tools/conv_probe.py --reps 1 struct_char_d3_int_resized48 > $O/r2g_sq.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/r2g_kt -o run -- python3 tools/conv_probe.py --reps 3 struct_char_d3_int_resized48 vector_f32_b4_s8 > $O/r2g_kt.log 2>&1 || exit 1
echo ok
