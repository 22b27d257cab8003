#!/bin/bash
# Instruction-mix PMC passes (diagnostic) for the encode and decode kernels on
# the configs[1] batch, one rocprofv3 run per pass.  usage: scripts/pmc_mix.sh OUTDIR
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1
mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD"
P3="GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d $OUT/e$i -o pmc -- python3 scripts/prof_encode.py --reps 2 > $OUT/e$i.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d $OUT/d$i -o pmc -- python3 scripts/prof_decode.py --variants full --reps 2 --blocks 1048576 > $OUT/d$i.log 2>&1
done
for k in encode_group_kernel encode_plan; do echo "== $k"; python3 scripts/pmc_kernel.py $OUT/ $k 1048576 | grep -v "^$"; done > $OUT/summary.txt
echo "== decode_blocks_kernel" >> $OUT/summary.txt
for i in 1 2 3; do python3 scripts/pmc_kernel.py $OUT/d$i decode_blocks_kernel 1048576; done >> $OUT/summary.txt
cat $OUT/summary.txt
