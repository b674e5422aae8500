# non-contiguous device buffers in coll; piece pack: parity + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_components_mp.py tests/test_convertor.py tests/test_convertor_pins.py tests/test_p2p_gpu.py > $O/r2r_pytest.txt 2>&1 || { tail -40 $O/r2r_pytest.txt; exit 1; }
tail -2 $O/r2r_pytest.txt
T="ref_upper_matrix_60 ref_matrix_borders_20_3 ref_lower_matrix_47 indexed_f32_random ref_blacs_indexed vector_f32_b64_s128"
for b in 0 1; do
  echo "PPACK=$b" >> $O/r2r_ab.txt
  MX_CONV_PPACK=$b timeout -k 10 240 python -u tools/conv_probe.py --dirs pack $T >> $O/r2r_ab.txt 2>&1 || exit 1
done
grep -v amdgpu $O/r2r_ab.txt
echo ok
