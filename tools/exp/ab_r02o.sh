# A/B: k_vis at 3 waves/SIMD for large batches (HEAD default) vs 4 everywhere (NR_VIS_WPE3=0), same library;
# then the GPU suite at the default.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
ab() {  # bench args, reps
  for r in $(seq $2); do
    for v in 0 1; do
      NR_VIS_WPE3=$v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 $1 > gpurun_out/abv.json 2>&1 || exit 1
      echo "wpe3=$v $1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abv.json) $(grep -o '"tile_raster": [0-9.]*' gpurun_out/abv.json)"
    done
  done
}
ab "" 3 && ab "--steps 20 --warmup 5" 2 && ab "--emulate-shards 2" 2 && ab "--emulate-shards 4" 2 && ab "--emulate-shards 8" 1 && ab "--config c3_1080p" 1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_wpe3.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_wpe3.log
