#!/bin/bash
# A/B of the op service's grid (MX_SVC_GRID workgroups, MX_SVC_HSLEEP helper
# sleep) against the launch path, interleaved, one box (tools/op_call_cost.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-svc_tune}
mkdir -p $O
for round in 1 2; do
  for cfg in ${CFGS:-"fastsync - -" "service 1 1" "service 32 1" "service 32 2"}; do
    set -- $cfg
    echo "# round $round $1 grid $2 hsleep $3" >> $O/tune.txt
    if [ "$1" = fastsync ]; then
      timeout -k 10 120 python tools/op_call_cost.py fastsync >> $O/tune.txt 2>&1 || exit 1
    else
      MX_SVC_GRID=$2 MX_SVC_HSLEEP=$3 timeout -k 10 120 python tools/op_call_cost.py service >> $O/tune.txt 2>&1 || exit 1
    fi
  done
done
