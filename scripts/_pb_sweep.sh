# diagnostic: kernel times of encode variant builds (lsm-tree_amd/.variants)
export TMPDIR=/tmp
O=gpurun_out/pb3
mkdir -p $O
for v in base $VARIANTS; do
  if [ $v = base ]; then L=lsm-tree_amd/liblsmgpu.so; else L=lsm-tree_amd/.variants/lib$v.so; fi
  LSMGPU_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o e --output-format csv -- python3 scripts/prof_encode.py --reps 10 > $O/$v.log 2>&1 || exit 3
done
python3 scripts/kstats.py $O/* | grep -E "==|plan|group"
