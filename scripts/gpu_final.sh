#!/bin/bash
# Round-end measurement: the GPU tests, the default bench line, then the round profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_final.log 2>&1 || { echo "tests rc=$?"; tail -20 gpurun_out/tests_final.log; exit 1; }
tail -1 gpurun_out/tests_final.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | cut -c1-300
timeout -k 10 1100 bash scripts/profile_round.sh ${ROUND:-r05} > gpurun_out/prof_${ROUND:-r05}.log 2>&1 || { echo "prof rc=$?"; tail -20 gpurun_out/prof_${ROUND:-r05}.log; exit 1; }
tail -5 gpurun_out/prof_${ROUND:-r05}.log
