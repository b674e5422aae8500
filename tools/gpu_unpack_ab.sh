#!/bin/bash
# A/B of the piece UNPACK kernel's register prefetch (MX_CONV_UNPACK_PIPE), interleaved,
# then the convertor GPU tests on the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${TAG:-unpack_ab}
mkdir -p $O
TYPES=${TYPES:-"ref_blacs_indexed struct_char_d3_int_resized48 ref_struct ref_strange ref_struct_char_double ref_lower_matrix_47 ref_upper_matrix_60 ref_struct_constant_gap_resized"}
for round in 1 2; do
  for pipe in 0 1; do
    echo "# round $round MX_CONV_UNPACK_PIPE=$pipe" >> $O/ab.txt
    MX_CONV_UNPACK_PIPE=$pipe timeout -k 10 300 python tools/conv_probe.py --bytes $((1<<30)) --dirs unpack $TYPES >> $O/ab.txt 2>&1 || exit 1
  done
done
[ "${TESTS:-1}" = 0 ] || timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convertor.py tests/test_convertor_pins.py -m gpu > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
