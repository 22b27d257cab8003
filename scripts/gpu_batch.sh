#!/bin/bash
# One GPU call for several checks (GPU slots are scarce).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=lsm-tree_amd/.variants
bash scripts/gpu_steps.sh \
  "ab:300:for r in 1 2; do for L in lsm-tree_amd/liblsmgpu.so $V/libi256.so $V/libi512.so; do echo == \$L; LSMGPU_LIB=\$L python -u scripts/ab_large.py --which 256KiB,1MiB,4MiB || exit 1; done; done"
