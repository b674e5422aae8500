# full GPU suite after the convertor / p2p / stream changes, then latency and call-cost probes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out; mkdir -p $O
STEP_TIMEOUT=1000 TEST_TIMEOUT=300 bash tools/gpu_r2.sh r2l 'tests -m gpu' || exit 1
timeout -k 10 300 python -u tools/p2p_lat.py 2>&1 | grep "half" > $O/r2l_p2plat.txt || exit 1
cat $O/r2l_p2plat.txt
timeout -k 10 200 python -u tools/op_call_cost.py > $O/r2l_op_call_cost.txt 2>&1 || { tail -20 $O/r2l_op_call_cost.txt; exit 1; }
grep -v amdgpu.ids $O/r2l_op_call_cost.txt
echo ok
