# round 5 (d): op-service interference, GPU + CPU sweeps in one run, two-comm p2p test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=400 bash tools/gpu_pytest.sh r5d "tests/test_p2p_gpu.py tests/test_lifecycle_gpu.py" || exit $?
timeout -k 10 300 python tools/svc_interference.py --out $O/svc_interference_r5.json > $O/svc_interference_r5.txt 2>&1 || exit $?
cat $O/svc_interference_r5.txt
export MX_SWEEP_RUN="gpu_r5d $(date +%F_%T) $(hostname)"
timeout -k 10 400 python tools/sweep.py --what pairs --out $O/sweep_pairs_r5.json > $O/sweep_pairs_r5.log 2>&1 || exit $?
timeout -k 10 300 python tools/sweep.py --what pack --min-bytes $((128<<20)) --max-bytes $((1<<30)) --out $O/sweep_pack_r5.json > $O/sweep_pack_r5.log 2>&1 || exit $?
timeout -k 10 400 python tools/cpu_sweep.py --what pairs,pack --merge-gpu $O/sweep_pairs_r5.json,$O/sweep_pack_r5.json --out $O/cpu_sweep_r5.json > $O/cpu_sweep_r5.log 2>&1 || exit $?
head -5 $O/cpu_sweep_r5.txt
