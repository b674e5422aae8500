set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 1000 python -u tools/sweep.py --out $O/r1ae_sweep.json > $O/r1ae_sweep.txt 2>&1 || { tail -20 $O/r1ae_sweep.txt; exit 1; }
tail -3 $O/r1ae_sweep.txt
