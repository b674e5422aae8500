# round 5 (o): byte-map PACK span size A/B (12 / 24 / 48 KiB staged per tile), parity under each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=300 bash tools/gpu_pytest.sh r5o_conv "tests/test_convertor.py -m gpu" || exit $?
MX_CONV_BMAP_SPAN=12288 STEP_TIMEOUT=300 bash tools/gpu_pytest.sh r5o_conv12 "tests/test_convertor.py -m gpu" || exit $?
MX_CONV_BMAP_SPAN=49152 STEP_TIMEOUT=300 bash tools/gpu_pytest.sh r5o_conv48 "tests/test_convertor.py -m gpu" || exit $?
T="struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed ref_struct ref_strange"
for rep in 1 2; do
for v in "" "MX_CONV_BMAP_SPAN=12288" "MX_CONV_BMAP_SPAN=49152"; do
  echo "== $v (rep $rep)" >> $O/conv_ab_r5o.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack $T >> $O/conv_ab_r5o.txt 2>&1 || exit $?
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack $T >> $O/conv_ab_r5o.txt 2>&1 || exit $?
done
done
grep -v amdgpu.ids $O/conv_ab_r5o.txt
