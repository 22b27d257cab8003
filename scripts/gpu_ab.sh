#!/bin/bash
# A/B timing calls on the GPU box: each step under its own time limit, stopping at the first failure.
# usage: scripts/gpu_ab.sh OUT "step1 args" ["step2 args" ...]; a step is "enc|dec LIB... -- OPTIONS"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; shift
mkdir -p gpurun_out
i=0
for step in "$@"; do
  i=$((i+1))
  kind=${step%% *}; rest=${step#* }
  timeout -k 10 420 python3 -u scripts/ab_${kind}code.py $rest > gpurun_out/${OUT}_$i.log 2>&1 || { echo "step $i rc=$?"; tail -5 gpurun_out/${OUT}_$i.log; exit 1; }
  grep -A20 "^median" gpurun_out/${OUT}_$i.log
done
