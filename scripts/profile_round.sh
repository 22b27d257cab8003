#!/bin/bash
# Round profile: rocprofv3 kernel-trace stats of a short bench run, and the
# two PMC passes (separate runs, no tracing domains) for HBM traffic.
# Usage (on the GPU box): scripts/profile_round.sh rNN
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${1:-r01}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o bench --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extra --no-host > $OUT/bench_kt.log 2>&1
NB=1048576
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o pmc -- \
  python3 scripts/prof_decode.py --variants full --reps 4 --blocks $NB > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o pmc -- \
  python3 scripts/prof_decode.py --variants full --reps 4 --blocks $NB > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/efetch -o pmc -- \
  python3 scripts/prof_encode.py --reps 4 --blocks $NB > $OUT/efetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/ewrite -o pmc -- \
  python3 scripts/prof_encode.py --reps 4 --blocks $NB > $OUT/ewrite.log 2>&1
line=$(grep "^variants:" $OUT/fetch.log)
BYTES=$(echo "$line" | sed 's/.* bytes \([0-9]*\) items.*/\1/')
ITEMS=$(echo "$line" | sed 's/.* items \([0-9]*\).*/\1/')
EALG=$(grep "alg_bytes" $OUT/efetch.log | sed 's/.*alg_bytes \([0-9]*\).*/\1/')
EITEMS=$(grep "alg_bytes" $OUT/efetch.log | sed 's/.*blocks \([0-9]*\) items.*/\1/')
# (the counter workload: 16 B keys, 64 B values; u32 offsets, as bench.py's timed encode)
python3 scripts/traffic_summary.py $OUT/fetch $OUT/write $NB $BYTES $ITEMS $OUT/efetch $OUT/ewrite $EALG \
  $EITEMS $((16 * EITEMS)) $((64 * EITEMS)) 4 > $OUT/traffic.json
cat $OUT/traffic.json
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 scripts/trace_by_grid.py $(find $OUT/kt -name "*kernel_trace.csv" | head -1) > $OUT/kernels_by_grid.csv
# the library build the trace belongs to: bench.py uses a committed trace only for this same build
python3 -c "import hashlib, json, sys; print(json.dumps({'lib_sha256': hashlib.sha256(open('lsm-tree_amd/liblsmgpu.so', 'rb').read()).hexdigest()}))" > $OUT/kernels_by_grid.lib.json
head -20 $OUT/kernel_stats.csv
