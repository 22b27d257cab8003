#!/bin/bash
# Instruction / LDS counters of decode_blocks_kernel with one phase ablated
# (diagnostic build, lsm_decode_tuning.flags bits; outputs invalid), one
# rocprofv3 run per variant.  usage: scripts/pmc_decode_ablate.sh OUTDIR
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"
mkdir -p $OUT
for v in ${VARIANTS:-full no-hash no-parse phaseA-only stage-only}; do
  LSMGPU_LIB=${DIAG_LIB:-lsm-tree_amd/.variants/libdiag.so} timeout -k 10 120 rocprofv3 --pmc $P1 --output-format csv -d $OUT/$v -o pmc -- python3 scripts/prof_decode.py --variants $v --reps 1 --blocks 1048576 > $OUT/$v.log 2>&1
  echo "== $v" >> $OUT/summary.txt
  python3 scripts/pmc_kernel.py $OUT/$v decode_blocks_kernel 1048576 >> $OUT/summary.txt
done
cat $OUT/summary.txt
