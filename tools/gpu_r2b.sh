set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out; mkdir -p $O
STEP_TIMEOUT=1000 TEST_TIMEOUT=300 bash tools/gpu_r2.sh r2b 'tests -m gpu' || exit 1
timeout -k 10 200 python -u tools/op_call_cost.py > $O/r2b_op_call_cost.txt 2>&1 || { tail -20 $O/r2b_op_call_cost.txt; exit 1; }
cat $O/r2b_op_call_cost.txt
timeout -k 10 60 ./tools/ipc_handle_probe > $O/r2b_ipc_handle_probe.txt 2>&1; echo probe rc=$?
tail -30 $O/r2b_ipc_handle_probe.txt
