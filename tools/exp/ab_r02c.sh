cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_t6.log 2>&1 || { tail -30 gpurun_out/r02_t6.log; exit 1; }
tail -2 gpurun_out/r02_t6.log
timeout -k 5 120 python tools/exp/host_cost.py 8 || exit 1
for a in "" "--emulate-shards 2" "--emulate-shards 4" "--emulate-shards 8" "--config c2"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 $a > gpurun_out/ab.json 2>&1 || exit 1
  echo "$a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json) $(grep -o '"kernel_us": {[^}]*}' gpurun_out/ab.json)"
done
