# round 5 (t): VEC pack kernels non-temporal -- parity, A/B against ordinary accesses, then the full GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
T="vector_f32_b1_s2 vector_f32_b4_s8 vector_f64_b3_s5 vector_f32_b16_s32 vector_f32_b64_s128"
for rep in 1 2; do
for v in "" "MX_CONV_VEC_NT=0"; do
  echo "== $v (rep $rep)" >> $O/conv_ab_r5t.txt
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((256<<20)) --dirs pack $T >> $O/conv_ab_r5t.txt 2>&1 || exit $?
  env $v timeout -k 10 200 python tools/conv_probe.py --bytes $((1<<30)) --dirs pack $T >> $O/conv_ab_r5t.txt 2>&1 || exit $?
done
done
grep -v amdgpu.ids $O/conv_ab_r5t.txt | grep -v "^$"
STEP_TIMEOUT=1000 bash tools/gpu_pytest.sh r5t_full "tests -m gpu --durations=25" || exit $?
