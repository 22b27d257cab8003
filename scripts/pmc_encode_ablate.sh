#!/bin/bash
# LDS / instruction counters of the encode group kernel with one phase ablated
# (diagnostic build, lsm_block_params.reserved bits; outputs invalid).
set -e
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"
mkdir -p gpurun_out/pabl
for bits in 0 1 2 4 8; do
  LSMGPU_LIB=lsm-tree_amd/.variants/libdiag.so timeout -k 10 120 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pabl/b$bits -o pmc -- python3 scripts/prof_encode.py --reps 1 --diag-bits $bits > gpurun_out/pabl/b$bits.log 2>&1 || true
  echo "== bits $bits" >> gpurun_out/pabl/summary.txt
  python3 scripts/pmc_kernel.py gpurun_out/pabl/b$bits encode_group_kernel 1048576 >> gpurun_out/pabl/summary.txt
done
cat gpurun_out/pabl/summary.txt
