#!/bin/bash
# One GPU call for several checks (GPU slots are scarce).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_steps.sh \
  "t:300:python -u -m pytest tests/test_gpu_large_blocks.py tests/test_gpu_encode_args.py -x -q --timeout 120 --timeout-method thread" \
  "ab:300:for r in 1 2; do python -u scripts/ab_large.py --which 256KiB,1MiB,4MiB || exit 1; done"
