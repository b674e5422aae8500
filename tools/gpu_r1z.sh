set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_convertor.py tests/test_p2p_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/r1z_pytest.txt 2>&1 || { tail -40 $O/r1z_pytest.txt; exit 1; }
tail -1 $O/r1z_pytest.txt
T=indexed_f32_random,struct_char_d3_int_resized48,ref_blacs_indexed,ref_lower_matrix_47
for tp in ${TPS:-8192 4096 2048}; do
  MX_CONV_TP=$tp timeout -k 10 200 python -u tools/sweep.py --what pack --types $T --min-bytes 100000000 --max-bytes 1073741824 --out $O/r1z_tp$tp.json > $O/r1z_tp$tp.txt 2>&1 || { tail -20 $O/r1z_tp$tp.txt; exit 1; }
  echo "TP=$tp"; grep -E " (1[0-9]{9}|[0-9]{9}) B" $O/r1z_tp$tp.txt
done
