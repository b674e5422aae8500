set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
# pipelined PACK tile kernel: parity (convertor + p2p ddt) and A/B against the one-tile kernel
timeout -k 10 300 python -u -m pytest tests/test_convertor.py tests/test_p2p_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/r1al_pytest.txt 2>&1 || { tail -40 $O/r1al_pytest.txt; exit 1; }
tail -1 $O/r1al_pytest.txt
T=indexed_f32_random,struct_char_d3_int_resized48,ref_blacs_indexed,ref_lower_matrix_47
for pipe in 1 0; do
  MX_CONV_PIPE=$pipe timeout -k 10 200 python -u tools/sweep.py --what pack --types $T --min-bytes 100000000 --max-bytes 1073741824 --out $O/r1al_pipe$pipe.json > $O/r1al_pipe$pipe.txt 2>&1 || { tail -20 $O/r1al_pipe$pipe.txt; exit 1; }
  echo "PIPE=$pipe"; grep -E "  pack .* (1[0-9]{9}|[0-9]{9}) B" $O/r1al_pipe$pipe.txt
done
