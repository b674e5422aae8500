# round 5 (y): UNPACK with non-temporal packed reads at streaming sizes -- parity (every switch), A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=500 bash tools/gpu_pytest.sh r5y_conv "tests/test_convertor.py tests/test_convertor_pins.py tests/test_convertor_hook_gpu.py tests/test_convertor_variants_gpu.py -m gpu --durations=5" || exit $?
T="struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed ref_struct ref_strange vector_f32_b4_s8 vector_f32_b1_s2"
for rep in 1 2; do
for v in "" "MX_CONV_UNPACK_NTLD=0"; do
  echo "== $v (rep $rep)" >> $O/conv_ab_r5y.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs unpack $T >> $O/conv_ab_r5y.txt 2>&1 || exit $?
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs unpack $T >> $O/conv_ab_r5y.txt 2>&1 || exit $?
done
done
grep -v amdgpu.ids $O/conv_ab_r5y.txt | grep -v "^$"
