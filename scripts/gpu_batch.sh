#!/bin/bash
# One GPU call for several checks (GPU slots are scarce).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=lsm-tree_amd/.variants
bash scripts/gpu_steps.sh \
  "new:300:python -u -m pytest tests/test_gpu_large_blocks.py tests/test_gpu_parity.py tests/test_gpu_config5.py tests/test_gpu_file_checksum.py -x -q --timeout 120 --timeout-method thread" \
  "ab:300:for L in lsm-tree_amd/liblsmgpu.so $V/libb1.so $V/libns.so $V/libold.so $V/libb8.so; do echo == \$L; LSMGPU_LIB=\$L python -u scripts/ab_large.py --which 1MiB,4MiB || exit 1; done" \
  "abd:300:python -u scripts/ab_decode.py lsm-tree_amd/liblsmgpu.so $V/libold.so --rounds 2 --which k64c,k64r --modes full"
