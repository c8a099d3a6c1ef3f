cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for cfg in "NR_SLICE_TARGET=512" "NR_SLICE_TARGET=256" "NR_SLICE_TARGET=1024" "NR_SLICE_TARGET=2048" "NR_WIDE_HEAVY=0" "NR_WIDE_HEAVY=4096"; do
  for extra in "--emulate-shards 8" "--emulate-shards 4"; do
    env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$cfg $extra: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log) $(grep -o '"kernel_us": [0-9.]*' gpurun_out/ab.log | head -1)"
  done
done
done
