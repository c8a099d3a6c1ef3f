# A/B of runtime knobs under the 3-wave k_vis (HEAD): slice target (NR_SLICE_TARGET) and binning sets (NR_BIN_SETS), C3.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in 1 2; do
  for v in "NR_SLICE_TARGET=512" "NR_SLICE_TARGET=384" "NR_SLICE_TARGET=768" "NR_SLICE_TARGET=1024" "NR_BIN_SETS=2"; do
    env $v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/abv.json 2>&1 || exit 1
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abv.json) $(grep -o '"tile_raster": [0-9.]*' gpurun_out/abv.json)"
  done
done
