# A/B of tools/exp/head.so vs tools/exp/new.so: GPU tests with new, then bench lines per config
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
cp tools/exp/new.so libnativecpurenderer_amd/libNativeCPURenderer.so
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_hn_tests.log 2>&1 || { tail -30 gpurun_out/r02_hn_tests.log; exit 1; }
tail -1 gpurun_out/r02_hn_tests.log
for a in "$@"; do
  for r in 1 2; do
    for v in head new; do
      cp tools/exp/$v.so libnativecpurenderer_amd/libNativeCPURenderer.so
      timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 $a > gpurun_out/abv.json 2>&1 || exit 1
      echo "$v $a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abv.json) $(grep -o '"tile_raster": [0-9.]*' gpurun_out/abv.json)"
    done
  done
done
cp tools/exp/new.so libnativecpurenderer_amd/libNativeCPURenderer.so
