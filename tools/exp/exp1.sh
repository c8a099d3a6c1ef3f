cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/exp/run.sh times base s512 s256 || exit 1
for c in c2 c5 c3_1080p; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail gpurun_out/bench_$c.log; exit 1; }
  echo "$c $(grep -o '"value": [0-9.]*' gpurun_out/bench_$c.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$c.log) $(grep -o '"kernel_us": {[^}]*}' gpurun_out/bench_$c.log)"
done
