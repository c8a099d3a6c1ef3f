# A/B: a TriangleBuffer batch issued to an idle main stream bins in line there (wide plan, no cross-queue wait;
# HEAD default) vs always on the binning stream (NR_BIN_IDLE_INLINE=0), same library; then the GPU suite.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
ab() {  # bench args, reps
  for r in $(seq $2); do
    for v in 0 1; do
      NR_BIN_IDLE_INLINE=$v timeout -k 10 120 python bench.py --no-cpu-baseline $1 > gpurun_out/abv.json 2>&1 || exit 1
      echo "inline=$v $1 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abv.json) $(grep -o '"tile_raster": [0-9.]*' gpurun_out/abv.json)"
    done
  done
}
ab "--steps 20 --warmup 5" 4 && ab "--steps 100" 2 && ab "--steps 20 --warmup 5 --config c2" 2 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_inline.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_inline.log
