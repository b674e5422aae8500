# round 5 (c): lifecycle test, full GPU suite, pack floors + convertor A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=300 bash tools/gpu_pytest.sh r5c "tests/test_lifecycle_gpu.py" || exit $?
STEP_TIMEOUT=800 bash tools/gpu_pytest.sh r5c_full "tests -m gpu --durations=30" || exit $?
T="struct_char_d3_int_resized48 indexed_f32_random vector_f32_b4_s8"
for B in $((256<<20)) $((1<<30)); do
  timeout -k 10 120 ./tools/pack_floor_probe $(python tools/pack_floor_args.py $B) >> $O/pack_floor_r5.txt 2>&1 || exit $?
done
for v in "" "MX_CONV_BLK=2" "MX_CONV_BMAP_DW=0" "MX_CONV_BMAP_PIPE=0"; do
  echo "== $v" >> $O/conv_ab_r5.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack $T >> $O/conv_ab_r5.txt 2>&1 || exit $?
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack $T >> $O/conv_ab_r5.txt 2>&1 || exit $?
done
cat $O/conv_ab_r5.txt
