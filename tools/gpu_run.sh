set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
python -c "import torch;print(torch.cuda.get_device_name(0))" > gpurun_out/${TAG:-r1}_env.txt 2>&1
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/${TAG:-r1}_pytest.txt 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG:-r1}_smoke.txt 2>&1 && \
timeout -k 10 200 python bench.py --cpu-seconds 10 > gpurun_out/${TAG:-r1}_bench.txt 2>&1
echo "exit: $?"
