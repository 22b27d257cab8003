#!/bin/bash
# Large-block round: parity tests, A/B timing and a kernel trace (GPU box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/kt_large gpurun_out/ab.log
bash scripts/gpu_steps.sh "large:200:python -u -m pytest tests/test_gpu_large_blocks.py tests/test_gpu_encode_args.py tests/test_gpu_parity.py tests/test_gpu_config5.py -x -q --timeout 120 --timeout-method thread" "ab:200:python -u scripts/ab_large.py --which 256KiB,1MiB,4MiB" "kt:200:bash scripts/prof_steps.sh large 'rocprofv3 --kernel-trace --stats -d gpurun_out/kt_large -o run --output-format csv -- python3 scripts/ab_large.py --which 256KiB,1MiB,4MiB --steps 2'"
