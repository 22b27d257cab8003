#!/bin/bash
# rocprofv3 PMC passes (one counter set per run, no tracing domains), each under its
# own time limit; stops at the first failure.  usage (GPU box):
#   scripts/pmc_steps.sh NAME "COUNTERS" "ENV=.. python3 script args" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
while [ $# -ge 3 ]; do
  name=$1; ctr=$2; cmd=$3; shift 3
  out=gpurun_out/pmc_$name
  rm -rf $out
  echo "== [$name] $ctr"
  timeout -s KILL 120 bash -c "${cmd/@PMC@/rocprofv3 --pmc $ctr --output-format csv -d $out -o pmc --}" > $out.log 2>&1 || { echo "STOP: $name rc=$?"; tail -5 $out.log; exit 1; }
  f=$(find $out -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && cp "$f" $out.csv
done
