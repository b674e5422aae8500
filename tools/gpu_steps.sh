# GPU-box step runner (replaces the per-session one-off scripts of rounds 3-5).
# usage on the box:  bash tools/gpu_steps.sh TAG 'name|seconds|command' ['name|seconds|command' ...]
# Each step runs under its own `timeout -k 10 seconds`, its output goes to
# gpurun_out/TAG_name.txt, and the first failing step ends the script (nothing
# more runs on the GPU after a failure, a fault or a time limit).
#   bash tools/gpu_steps.sh r6a \
#     'suite|900|python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu' \
#     'smoke|300|python -c "import __graft_entry__ as g; g.smoke()"' \
#     'bench|400|python bench.py'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
T=$1; shift
O=gpurun_out
mkdir -p $O
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}
  to=${rest%%|*}; cmd=${rest#*|}
  echo "[$(date +%T)] $name ($to s): $cmd" | tee -a $O/${T}_log.txt
  timeout -k 10 "$to" bash -c "$cmd" > $O/${T}_$name.txt 2>&1
  rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $O/${T}_log.txt
  tail -5 $O/${T}_$name.txt
  [ $rc -eq 0 ] || exit $rc
done
echo "all steps ok" | tee -a $O/${T}_log.txt
