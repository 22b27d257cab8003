# diagnostic: decode kernel time on the configs[1] batch (item_start precomputed) for variant builds
for v in base $VARIANTS; do
  if [ $v = base ]; then L=lsm-tree_amd/liblsmgpu.so; else L=lsm-tree_amd/.variants/lib$v.so; fi
  echo "== $v"; LSMGPU_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/dk/$v -o d --output-format csv -- python3 scripts/prof_decode.py --variants full --reps 10 --blocks 1048576 > gpurun_out/dk/$v.log 2>&1 || exit 3
  python3 scripts/kstats.py gpurun_out/dk/$v | grep decode_blocks
done
