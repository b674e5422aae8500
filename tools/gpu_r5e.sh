# round 5 (e): zero-copy tests (reproduction check), the rest of the suite, pack floors + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_coll_gpu.py -k "zero_copy" > $O/r5e_zc.txt 2>&1
echo "zc rc=$?"; tail -8 $O/r5e_zc.txt
STEP_TIMEOUT=850 bash tools/gpu_pytest.sh r5e_full "tests -m gpu --durations=40 --deselect 'tests/test_coll_gpu.py::test_multiprocess_allreduce_zero_copy'" || exit $?
T="struct_char_d3_int_resized48 indexed_f32_random vector_f32_b4_s8"
for B in $((256<<20)) $((1<<30)); do
  timeout -k 10 120 ./tools/pack_floor_probe $(python tools/pack_floor_args.py $B) >> $O/pack_floor_r5.txt 2>&1 || exit $?
done
for v in "" "MX_CONV_BLK=2" "MX_CONV_BMAP_DW=0"; do
  echo "== $v" >> $O/conv_ab_r5.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack $T >> $O/conv_ab_r5.txt 2>&1 || exit $?
done
cat $O/conv_ab_r5.txt
