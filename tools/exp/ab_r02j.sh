# A/B: CU partition between the raster and binning streams (NR_BIN_CUS), after the GPU parity suite.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for rep in 1 2; do
for a in "" "--emulate-shards 8" "--config c2"; do
  for k in 0 8 16 32; do
    NR_BIN_CUS=$k timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 $a > gpurun_out/ab.json 2>&1 || { tail -5 gpurun_out/ab.json; exit 1; }
    echo "bincus=$k $a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json) $(grep -o '"tile_raster": [0-9.]*' gpurun_out/ab.json)"
  done
done
done
