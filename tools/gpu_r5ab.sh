# round 5 (ab): instance-aligned byte-map tiles for non-monotonic layouts (A/B), then the full GPU suite + smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
for rep in 1 2; do
for v in "" "MX_CONV_BMAP_INST=0"; do
  echo "== $v (rep $rep)" >> $O/conv_ab_r5ab.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack indexed_f32_random >> $O/conv_ab_r5ab.txt 2>&1 || exit $?
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack indexed_f32_random >> $O/conv_ab_r5ab.txt 2>&1 || exit $?
done
done
grep -v amdgpu.ids $O/conv_ab_r5ab.txt | grep -v "^$"
STEP_TIMEOUT=1000 bash tools/gpu_pytest.sh r5ab_full "tests -m gpu --durations=15" || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
