#!/bin/bash
# One GPU call for several checks (GPU slots are scarce).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_steps.sh \
  "t:300:python -u -m pytest tests/test_gpu_large_blocks.py tests/test_gpu_encode_args.py -q --timeout 120 --timeout-method thread"
