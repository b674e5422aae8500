#!/bin/bash
# PMC FETCH_SIZE / WRITE_SIZE of the 32-byte element reduce kernels, per-element
# form (MX_REDUCE_W32T=0) vs through LDS (1); separate passes per counter.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-w32t_pmc}
mkdir -p $O
for v in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    MX_REDUCE_W32T=$v timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/w${v}_$c -o run -- \
      python3 tools/sweep.py --what pairs --pair-types C_LONG_DOUBLE_COMPLEX --iters 2 --out $O/w${v}_$c.json > $O/w${v}_$c.log 2>&1 || exit 1
  done
done
