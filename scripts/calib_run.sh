#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (scripts/fetch_calib.py) and the encode
# kernels' per-kernel counters on configs[1] (scripts/prof_encode.py), one
# rocprofv3 pass per counter.  Output under gpurun_out/calib/.
set -e
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/calib
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $P --output-format csv -d $O/fc_$P -o pmc -- python3 scripts/fetch_calib.py run > $O/fc_$P.log 2>&1
done
python3 scripts/fetch_calib.py summary $O/fc_FETCH_SIZE $O/fc_WRITE_SIZE > $O/fetch_calib.json
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $P --output-format csv -d $O/ep_$P -o pmc -- python3 scripts/prof_encode.py --reps 2 > $O/ep_$P.log 2>&1
  for K in encode_plan_wave_kernel encode_group_kernel scan_; do
    echo "== $P $K" >> $O/encode_kernels.txt
    python3 scripts/pmc_kernel.py $O/ep_$P $K 1048576 >> $O/encode_kernels.txt
  done
done
