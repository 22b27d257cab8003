#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of the encode
# bench loop for several library variants.  usage: scripts/kprof_libs.sh WHICH LIB...
# (on the GPU box; WHICH = c1 | c3 | c1,c3)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
which=$1; shift
for lib in "$@"; do
  name=$(basename "$lib" .so)
  out=gpurun_out/kp_${name}_${which//,/_}
  rm -rf "$out"
  LSMGPU_LIB=$(realpath "$lib") timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out" -o k --output-format csv -- \
    python3 scripts/ab_encode.py --child 10 "$which" > "$out.log" 2>&1
  echo "== $name"; tail -1 "$out.log"
  python3 scripts/kstats.py "$out" | grep -v "^=="
done
