# byte-map pack / piece unpack: parity, then A/B against the run-walking kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_convertor.py tests/test_convertor_pins.py > $O/r2f_pytest.txt 2>&1 || { tail -30 $O/r2f_pytest.txt; exit 1; }
tail -3 $O/r2f_pytest.txt
T="struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed ref_lower_matrix_47 ref_strange ref_struct_char_double ref_struct vector_f32_b4_s8"
for b in 0 1; do
  echo "BMAP=$b" >> $O/r2f_ab.txt
  MX_CONV_BMAP=$b timeout -k 10 180 python -u tools/conv_probe.py $T >> $O/r2f_ab.txt 2>&1 || exit 1
done
cat $O/r2f_ab.txt
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/r2f_pmc_w -o run -- python3 tools/conv_probe.py --reps 1 struct_char_d3_int_resized48 > $O/r2f_pmc_w.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/r2f_pmc_f -o run -- python3 tools/conv_probe.py --reps 1 struct_char_d3_int_resized48 > $O/r2f_pmc_f.log 2>&1 || exit 1
echo ok
