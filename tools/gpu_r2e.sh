# gapped-store write traffic, independent of the convertor
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -w -o /tmp/sector_probe tools/sector_probe.hip || exit 1
timeout -k 10 60 /tmp/sector_probe > $O/r2e_sector.txt 2>&1 || exit 1
cat $O/r2e_sector.txt
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/r2e_pmc_w -o run -- /tmp/sector_probe > $O/r2e_pmc_w.log 2>&1 || exit 1
echo ok
