#!/bin/bash
# One GPU call for several checks (GPU slots are scarce): the tests touched by the
# current change, the whole suite and the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_steps.sh \
  "new:200:python -u -m pytest tests/test_gpu_table_scan.py tests/test_gpu_lz4.py tests/test_gpu_materialize.py tests/test_gpu_large_blocks.py -x -q --timeout 120 --timeout-method thread" \
  "tests:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ab:200:python -u scripts/ab_large.py --which 256KiB,1MiB,4MiB" \
  "bench:400:python -u bench.py > gpurun_out/bench_line.json"
