# Round-2 measurement stages (the records under profiles/r02/).  On the box:
#   STAGES="convertor latency p2p" bash tools/gpu_probes.sh
# Each stage runs under its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out
mkdir -p $O
STAGES=${STAGES:-"convertor sector latency p2p ipc stream opcost datapath"}
TYPES=$(python -c "
import sys; sys.path.insert(0, 'tests'); import golden_io
print(' '.join(r['name'] for r in golden_io.ddt_records()[1]))")
for s in $STAGES; do
  echo "[$(date +%T)] $s"
  case $s in
    convertor)   # byte-map / piece kernels vs the run-walking ones, every golden type at 1 GiB
      for b in 1 0; do
        echo "MX_CONV_BMAP=$b" >> $O/probe_convertor.txt
        MX_CONV_BMAP=$b timeout -k 10 400 python -u tools/conv_probe.py $TYPES >> $O/probe_convertor.txt 2>&1 || exit 1
      done ;;
    sector)      # write cost of gapped store patterns, time and WRITE_SIZE
      hipcc --offload-arch=gfx950 -O3 -w -o /tmp/sector_probe tools/sector_probe.hip || exit 1
      timeout -k 10 60 /tmp/sector_probe > $O/probe_sector.txt 2>&1 || exit 1
      timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/probe_sector_pmc -o run -- \
          /tmp/sector_probe > $O/probe_sector_pmc.log 2>&1 || exit 1 ;;
    latency)     # allreduce latency per size, 2 and 4 processes on the GPU
      for n in 2 4; do
        timeout -k 10 300 python -u tools/lat_probe.py $n 2>&1 | grep "^n=" >> $O/probe_latency.txt || exit 1
      done ;;
    p2p)         # send/recv ping-pong half round trip
      timeout -k 10 300 python -u tools/p2p_lat.py 2>&1 | grep half >> $O/probe_p2p.txt || exit 1 ;;
    ipc)         # IPC handle contents, same-VA imports (2-3 processes), imports across a re-allocation
      timeout -k 10 60 ./tools/ipc_handle_probe > $O/probe_ipc_handle.txt 2>&1 || exit 1
      timeout -k 10 60 ./tools/ipc_alias_probe > $O/probe_ipc_alias.txt 2>&1 || exit 1
      hipcc --offload-arch=gfx950 -O2 -o /tmp/ipc_realloc_probe tools/ipc_realloc_probe.cpp || exit 1
      timeout -k 10 60 /tmp/ipc_realloc_probe > $O/probe_ipc_realloc.txt 2>&1 || exit 1 ;;
    datapath)    # allreduce latency per size and data movement (zero-copy / push / pull), 2 and 4 processes
      for n in 2 4; do
        timeout -k 10 300 python -u tools/lat_probe.py $n zc,push,pull 2>&1 | grep "^n=. {" >> $O/probe_datapath.txt || exit 1
      done ;;
    stream)      # host cost of launch / sync disciplines
      timeout -k 10 60 ./tools/stream_probe > $O/probe_stream.txt 2>&1 || exit 1 ;;
    opcost)      # ompi_op_reduce through op/mi355x
      timeout -k 10 200 python -u tools/op_call_cost.py > $O/probe_opcost.txt 2>&1 || exit 1 ;;
  esac
done
echo "all stages ok"
