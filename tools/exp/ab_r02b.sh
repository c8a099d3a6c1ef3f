# A/B: stream priorities x shard counts (bench ms/frame), after the register plan kernel
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for a in "" "--emulate-shards 8" "--config c2"; do
  for pr in 0 1 2; do
    NR_STREAM_PRIO=$pr timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 $a > gpurun_out/ab.json 2>&1 || exit 1
    echo "prio=$pr $a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json) $(grep -o '"kernel_us": {[^}]*}' gpurun_out/ab.json)"
  done
done
