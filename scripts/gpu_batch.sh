#!/bin/bash
# One GPU call for several checks (GPU slots are scarce).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_steps.sh \
  "all:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ab:200:python -u scripts/ab_large.py --which 256KiB,1MiB,4MiB" \
  "kt:200:bash scripts/prof_steps.sh large 'rocprofv3 --kernel-trace --stats -d gpurun_out/kt_large -o run --output-format csv -- python3 scripts/ab_large.py --which 1MiB,4MiB --steps 2'"
