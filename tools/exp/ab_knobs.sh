cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "NR_BIN_SETS=3" "NR_BIN_SETS=2" "NR_STREAM_PRIO=1" "NR_STREAM_PRIO=2" "NR_BIN_SETS=3" "NR_PLAN_SMALL=1"; do
  for extra in "" "--emulate-shards 8" "--emulate-shards 4"; do
    env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$cfg $extra: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
  done
done
