# round 5 (p): byte-map PACK 48 KiB span where the map is small + 4-dword unrolled gather: parity, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=400 bash tools/gpu_pytest.sh r5p_conv "tests/test_convertor.py tests/test_convertor_pins.py tests/test_convertor_hook_gpu.py -m gpu" || exit $?
MX_CONV_BMAP_SPAN=24576 STEP_TIMEOUT=300 bash tools/gpu_pytest.sh r5p_conv24 "tests/test_convertor.py -m gpu" || exit $?
T="struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed ref_struct ref_strange"
for rep in 1 2; do
for v in "" "MX_CONV_BMAP_UNROLL=0" "MX_CONV_BMAP_DW=0"; do
  echo "== $v (rep $rep)" >> $O/conv_ab_r5p.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack $T >> $O/conv_ab_r5p.txt 2>&1 || exit $?
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack $T >> $O/conv_ab_r5p.txt 2>&1 || exit $?
done
done
grep -v amdgpu.ids $O/conv_ab_r5p.txt
