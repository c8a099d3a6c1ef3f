mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_t4.log 2>&1 || exit 1
for a in "" "--emulate-shards 2" "--emulate-shards 4" "--emulate-shards 8" "--config c2"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 $a > gpurun_out/r02_b4.json 2>&1 || exit 1
  echo "NEW $a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r02_b4.json) $(grep -o '"kernel_us": {[^}]*}' gpurun_out/r02_b4.json)"
  NR_PLAN_REG=0 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 $a > gpurun_out/r02_b4.json 2>&1 || exit 1
  echo "OLD $a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r02_b4.json) $(grep -o '"kernel_us": {[^}]*}' gpurun_out/r02_b4.json)"
done
