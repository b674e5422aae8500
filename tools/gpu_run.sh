# GPU session script: tests -> smoke -> bench -> rocprof (stats + PMC passes).
# usage on the box: TAG=rN STAGES="test smoke bench prof pmc" bash tools/gpu_run.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${TAG:-r1}
O=gpurun_out
STAGES=${STAGES:-"test smoke bench prof pmc"}
mkdir -p $O
run() { # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] $name: $*" >> $O/${T}_log.txt
  timeout -k 10 $to "$@" > $O/${T}_$name.txt 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $O/${T}_log.txt
  return $rc
}
for s in $STAGES; do
  case $s in
    test)  run pytest 600 python -m pytest tests -x -q -m gpu ${PYTEST_ARGS:-} || exit 1 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench) run bench 400 python bench.py ${BENCH_ARGS:-} || exit 1 ;;
    prof)  run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- \
               python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 || exit 1 ;;
    pmc)   run pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${T}_pmc_fetch -o run -- \
               python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 || exit 1
           run pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${T}_pmc_write -o run -- \
               python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 || exit 1 ;;
    sweep) run sweep 900 python tools/sweep.py --out $O/${T}_sweep.json ${SWEEP_ARGS:-} || exit 1 ;;
    extra) run extra 900 bash -c "${EXTRA_CMD}" || exit 1 ;;
  esac
done
echo "all stages ok" >> $O/${T}_log.txt
