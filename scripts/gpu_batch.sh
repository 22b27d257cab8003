#!/bin/bash
# One GPU call for several checks (GPU slots are scarce).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=lsm-tree_amd/.variants
bash scripts/gpu_steps.sh \
  "new:300:python -u -m pytest tests/test_gpu_large_blocks.py tests/test_gpu_parity.py tests/test_gpu_config5.py tests/test_gpu_file_checksum.py tests/test_gpu_encode_args.py -x -q --timeout 120 --timeout-method thread" \
  "rph:120:LSMGPU_LIB=$V/libdiag.so python -u scripts/rec_phases.py" \
  "ab:200:python -u scripts/ab_large.py --which 256KiB,1MiB,4MiB"
