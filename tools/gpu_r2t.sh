# convertor final A/B: current kernels vs the run-walking ones, every golden type at 1 GiB
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_convertor.py tests/test_convertor_pins.py > $O/r2t_pytest.txt 2>&1 || { tail -40 $O/r2t_pytest.txt; exit 1; }
tail -2 $O/r2t_pytest.txt
T=$(python -c "
import sys; sys.path.insert(0,'tests'); import golden_io
print(' '.join(r['name'] for r in golden_io.ddt_records()[1]))")
for b in 1 0; do
  echo "BMAP=$b (1: byte-map / piece kernels, 0: run-walking VEC / tile / pipe kernels)" >> $O/r2t_ab.txt
  MX_CONV_BMAP=$b timeout -k 10 400 python -u tools/conv_probe.py $T >> $O/r2t_ab.txt 2>&1 || exit 1
done
grep -v amdgpu $O/r2t_ab.txt
echo ok
