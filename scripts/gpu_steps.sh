#!/bin/bash
# Run GPU steps in sequence, each under its own time limit; stop at the first
# step that ends like a fault/abort/timeout (anything but 0 or an ordinary
# failure code 1 / pytest 5), so nothing else touches the GPU after it.
# usage: scripts/gpu_steps.sh "name:seconds:command" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "== [$name] (${secs}s) $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 8 "gpurun_out/$name.log"
  case $rc in
    0|1|5) ;;
    *) echo "STOP: step $name ended with rc=$rc"; exit $rc ;;
  esac
done
