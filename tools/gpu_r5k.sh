# round 5 (k): byte-map PACK quads; op service relaxed helper polls -- parity, A/B, interference
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=400 bash tools/gpu_pytest.sh r5k_conv "tests/test_convertor.py tests/test_convertor_pins.py tests/test_convertor_hook_gpu.py tests/test_op_service_gpu.py -m gpu" || exit $?
T="struct_char_d3_int_resized48 indexed_f32_random ref_blacs_indexed ref_struct ref_strange"
for rep in 1 2; do
for v in "" "MX_CONV_BMAP_QUAD=0" "MX_CONV_BMAP_DW=0"; do
  echo "== $v (rep $rep)" >> $O/conv_ab_r5k.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack $T >> $O/conv_ab_r5k.txt 2>&1 || exit $?
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack $T >> $O/conv_ab_r5k.txt 2>&1 || exit $?
done
done
grep -v amdgpu.ids $O/conv_ab_r5k.txt
timeout -k 10 300 python tools/svc_interference.py --out $O/svc_interference_r5k.json > $O/svc_interference_r5k.txt 2>&1 || exit $?
MX_SVC_GRID=8 timeout -k 10 300 python tools/svc_interference.py --out $O/svc_interference_r5k_g8.json > $O/svc_interference_r5k_g8.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/svc_interference_r5k.txt $O/svc_interference_r5k_g8.txt
