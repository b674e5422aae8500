set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
# blocking-call completion A/B: previous build (hipStreamSynchronize) vs spin-then-block stream_sync
L=zhpe-ompi_amd/lib/libmx_kernels.so
cp $L /tmp/libmx_new.so
cp tools/libmx_kernels_prev.so $L
for n in 2 4; do
  timeout -k 10 150 python -u tools/lat_probe.py $n > $O/r1ai_lat_prev_n$n.txt 2>&1 || { cp /tmp/libmx_new.so $L; tail -20 $O/r1ai_lat_prev_n$n.txt; exit 1; }
done
cp /tmp/libmx_new.so $L
for n in 2 4; do
  timeout -k 10 150 python -u tools/lat_probe.py $n > $O/r1ai_lat_new_n$n.txt 2>&1 || { tail -20 $O/r1ai_lat_new_n$n.txt; exit 1; }
done
grep -h "n=" $O/r1ai_lat_prev_n2.txt $O/r1ai_lat_new_n2.txt $O/r1ai_lat_prev_n4.txt $O/r1ai_lat_new_n4.txt
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/r1ai_pytest.txt 2>&1 || { tail -40 $O/r1ai_pytest.txt; exit 1; }
tail -1 $O/r1ai_pytest.txt
timeout -k 10 200 python bench.py > $O/r1ai_bench.txt 2>&1 || { tail -20 $O/r1ai_bench.txt; exit 1; }
tail -1 $O/r1ai_bench.txt | cut -c1-400
