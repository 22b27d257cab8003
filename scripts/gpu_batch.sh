#!/bin/bash
# One GPU call for several checks (GPU slots are scarce): the tests touched by the
# current change, the large-block A/B, a decode library A/B, the whole suite, a
# kernel trace of the large-block legs, PMC instruction mixes and a PC-sampling try.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/kt_large gpurun_out/pcs
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
bash scripts/gpu_steps.sh \
  "new:200:python -u -m pytest tests/test_gpu_table_scan.py tests/test_gpu_lz4.py tests/test_gpu_materialize.py tests/test_gpu_encode_args.py tests/test_gpu_large_blocks.py -x -q --timeout 120 --timeout-method thread" \
  "ab:200:python -u scripts/ab_large.py --which 256KiB,1MiB,4MiB" \
  "abd:200:python -u scripts/ab_decode.py lsm-tree_amd/.variants/libbase.so lsm-tree_amd/.variants/libpb32.so --rounds 2 --which c1,c3,k16c --modes full" \
  "tests:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "kt:200:bash scripts/prof_steps.sh large 'rocprofv3 --kernel-trace --stats -d gpurun_out/kt_large -o run --output-format csv -- python3 scripts/ab_large.py --which 256KiB,1MiB,4MiB --steps 2'" \
  "pmc:300:bash scripts/pmc_steps.sh mixe '$C' '@PMC@ python3 scripts/ab_encode.py --child 2 c1' mixd '$C' '@PMC@ python3 scripts/prof_decode.py --variants full --reps 2 --blocks 1048576'" \
  "pcs:200:rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d gpurun_out/pcs -o pcs --output-format csv -- python3 scripts/prof_decode.py --variants full --reps 4 --blocks 1048576"
