#!/bin/bash
# rocprofv3 kernel-trace summaries of short runs (one profile per step, each under
# its own time limit; stops at the first failure).  usage (GPU box):
#   scripts/prof_steps.sh NAME "ENV=.. python3 script args" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  name=$1; cmd=$2; shift 2
  out=gpurun_out/kt_$name
  rm -rf $out
  echo "== [$name] $cmd"
  timeout -k 10 240 bash -c "$cmd" > gpurun_out/kt_$name.log 2>&1 || { echo "STOP: $name rc=$?"; tail -5 gpurun_out/kt_$name.log; exit 1; }
  f=$(find $out -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" gpurun_out/kt_$name.csv && head -14 gpurun_out/kt_$name.csv | cut -d, -f1-4
done
