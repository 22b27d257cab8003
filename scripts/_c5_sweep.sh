# diagnostic: configs[4] per-segment decode rates for variant builds
for v in base $VARIANTS; do
  if [ $v = base ]; then L=lsm-tree_amd/liblsmgpu.so; else L=lsm-tree_amd/.variants/lib$v.so; fi
  echo "== $v"; LSMGPU_LIB=$L timeout -k 10 200 python3 -u scripts/config5_breakdown.py 2>&1 | grep -E "kernels|Error" || exit 3
done
