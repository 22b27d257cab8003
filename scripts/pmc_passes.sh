#!/bin/bash
# PMC passes over a profiling driver (diagnostic); one rocprofv3 run per pass.
# usage: scripts/pmc_passes.sh OUTDIR DRIVER.py [driver args...]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
P5="GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_IFETCH"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o pmc -- python "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -20 $OUT/p$i.log; exit 3; }
done
