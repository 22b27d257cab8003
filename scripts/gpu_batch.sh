#!/bin/bash
# One GPU call for several checks (GPU slots are scarce).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=lsm-tree_amd/.variants
bash scripts/gpu_steps.sh \
  "new:240:python -u -m pytest tests/test_gpu_large_blocks.py tests/test_gpu_encode_args.py tests/test_gpu_parity.py tests/test_gpu_file_checksum.py -x -q --timeout 120 --timeout-method thread" \
  "ab:200:python -u scripts/ab_large.py --which 256KiB,1MiB,4MiB && LSMGPU_LIB=$V/libwpe3.so python -u scripts/ab_large.py --which 1MiB,4MiB && LSMGPU_LIB=$V/libwpe2.so python -u scripts/ab_large.py --which 1MiB,4MiB" \
  "kt:200:bash scripts/prof_steps.sh large 'rocprofv3 --kernel-trace --stats -d gpurun_out/kt_large -o run --output-format csv -- python3 scripts/ab_large.py --which 1MiB,4MiB --steps 2'"
