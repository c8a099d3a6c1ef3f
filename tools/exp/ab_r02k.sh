# A/B: binning grid size (NR_BIN_GRID: persistent binning workgroups) x stream priority (NR_STREAM_PRIO 0: raster above binning, 1: binning above raster).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do
for a in "" "--emulate-shards 8"; do
  for pr in 0 1; do
  for g in 0 64 128 256; do
    NR_STREAM_PRIO=$pr NR_BIN_GRID=$g timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 $a > gpurun_out/ab.json 2>&1 || { tail -5 gpurun_out/ab.json; exit 1; }
    echo "prio=$pr grid=$g $a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json) $(grep -o '"kernel_us": {[^}]*}' gpurun_out/ab.json)"
  done
  done
done
done
