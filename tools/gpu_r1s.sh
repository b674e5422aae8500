set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
for n in 2 4; do for m in 262144 1048576; do
  MX_ONESHOT_MAX=$m timeout -k 10 120 python -u tools/lat_probe.py $n >> $O/r1s2_lat.txt 2>&1 || exit 1
done; done
grep "n=" $O/r1s2_lat.txt
