# GPU pytest runner. usage on the box: bash tools/gpu_pytest.sh TAG "pytest args" [more pytest arg sets...]
# (each set is eval'd: quote a -k expression inside it, e.g. "t.py -k 'a or b'")
# Each argument set runs as one pytest process under its own time limit;
# the first failure ends the script (nothing more runs on the GPU after it).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; shift
O=gpurun_out
mkdir -p $O
i=0
for args in "$@"; do
  i=$((i+1))
  echo "[$(date +%T)] pytest $args" | tee -a $O/${T}_log.txt
  eval timeout -k 10 ${STEP_TIMEOUT:-900} python -u -m pytest -x -v --timeout ${TEST_TIMEOUT:-300} --timeout-method thread $args \
      > $O/${T}_pytest$i.txt 2>&1
  rc=$?
  echo "[$(date +%T)] rc=$rc" | tee -a $O/${T}_log.txt
  tail -3 $O/${T}_pytest$i.txt
  [ $rc -eq 0 ] || exit $rc
done
