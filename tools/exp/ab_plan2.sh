cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for extra in "" "--config c2" "--config c5" "--emulate-shards 8"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  echo "$extra: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
done
