# round 5 (l): op service with release-only fences -- call cost per grid, interference per grid
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STEP_TIMEOUT=300 bash tools/gpu_pytest.sh r5l_svc "tests/test_op_service_gpu.py -m gpu" || exit $?
TAG=svc_tune_r5l CFGS="fastsync_-_- service_32_2 service_16_2 service_8_2" bash -c '
set -o pipefail
O=gpurun_out/$TAG; mkdir -p $O
for round in 1 2; do for cfg in $CFGS; do set -- ${cfg//_/ }
  echo "# round $round $1 grid $2 hsleep $3" >> $O/tune.txt
  if [ "$1" = fastsync ]; then timeout -k 10 120 python tools/op_call_cost.py fastsync >> $O/tune.txt 2>&1 || exit 1
  else MX_SVC_GRID=$2 MX_SVC_HSLEEP=$3 timeout -k 10 120 python tools/op_call_cost.py service >> $O/tune.txt 2>&1 || exit 1; fi
done; done' || exit $?
grep -v amdgpu.ids $O/svc_tune_r5l/tune.txt
for g in 32 16 8; do
  MX_SVC_GRID=$g timeout -k 10 300 python tools/svc_interference.py --out $O/svc_interference_r5l_g$g.json > $O/svc_interference_r5l_g$g.txt 2>&1 || exit $?
  grep -v amdgpu.ids $O/svc_interference_r5l_g$g.txt
done
