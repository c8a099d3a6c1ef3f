# A/B: wave-aggregated binning (NR_BIN_WAGG=1) vs LDS-histogram binning, after the GPU parity suite under WAGG.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
NR_BIN_WAGG=1 timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for rep in 1 2 3; do
for a in "" "--emulate-shards 8" "--emulate-shards 4" "--config c2"; do
  for w in 0 1; do
    NR_BIN_WAGG=$w timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 $a > gpurun_out/ab.json 2>&1 || { tail -5 gpurun_out/ab.json; exit 1; }
    echo "wagg=$w $a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json) $(grep -o '"kernel_us": {[^}]*}' gpurun_out/ab.json)"
  done
done
done
