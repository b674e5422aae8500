#!/bin/bash
# GPU-box helper: round-3 new tests (RCCL path, CFG-D 1/4 GiB, stale lines, crossover autotuning)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread \
  tests/test_rccl_gpu.py \
  "tests/test_components_rules.py::test_zero_copy_reused_buffers_never_read_stale_data" \
  "tests/test_coll_gpu.py::test_multiprocess_autotune_crossovers" \
  "tests/test_coll_headline_gpu.py::test_allreduce_fp32_sum_1gib_per_rank_2_ranks" \
  "tests/test_coll_headline_gpu.py::test_allreduce_fp32_sum_4gib_per_rank_2_ranks" > gpurun_out/r3b.log 2>&1
rc=$?
tail -25 gpurun_out/r3b.log
exit $rc
