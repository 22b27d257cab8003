#!/bin/bash
# One GPU call for several checks (GPU slots are scarce).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=lsm-tree_amd/.variants
bash scripts/gpu_steps.sh \
  "t:300:LSMGPU_LIB=$V/libs16.so python -u -m pytest tests/test_gpu_large_blocks.py tests/test_gpu_parity.py tests/test_gpu_materialize.py tests/test_gpu_lz4.py -x -q --timeout 120 --timeout-method thread" \
  "ab:300:for r in 1 2; do for L in lsm-tree_amd/liblsmgpu.so $V/libs16.so; do echo == \$L; LSMGPU_LIB=\$L python -u scripts/ab_large.py --which 1MiB,4MiB || exit 1; done; done" \
  "ae:300:python -u scripts/ab_encode.py lsm-tree_amd/liblsmgpu.so $V/libs16.so --rounds 2 2>&1 | tail -6"
