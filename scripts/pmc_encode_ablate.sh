#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"
for bits in 0 1 2 8; do
  timeout -k 10 120 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pabl/b$bits -o pmc -- python scripts/prof_encode.py --reps 1 --diag-bits $bits > gpurun_out/pabl/b$bits.log 2>&1
done
