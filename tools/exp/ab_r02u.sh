# A/B of HIP runtime settings on C3 (100 steps): kernel arguments in device memory (HIP_FORCE_DEV_KERNARG) on/off.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in 1 2 3; do for v in "HIP_FORCE_DEV_KERNARG=0" "HIP_FORCE_DEV_KERNARG=1" "NR_NONE=0"; do
  env $v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/abv.json 2>&1 || exit 1
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abv.json) $(grep -o '"tile_raster": [0-9.]*' gpurun_out/abv.json)"
done; done
