cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for rep in 1 2; do
  for extra in "" "--config c2" "--emulate-shards 2" "--emulate-shards 4" "--emulate-shards 8"; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 $extra > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$extra: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.log)"
  done
done
