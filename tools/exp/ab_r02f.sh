cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_t9.log 2>&1 || { tail -30 gpurun_out/r02_t9.log; exit 1; }
tail -1 gpurun_out/r02_t9.log
for rep in 1 2; do
for a in "" "--emulate-shards 8" "--emulate-shards 4" "--config c2"; do
  for k in 1 0; do
    NR_KNOWN_SIZES=$k timeout -k 10 120 python bench.py --no-cpu-baseline --no-kernel-timing --steps 200 $a > gpurun_out/ab.json 2>&1 || exit 1
    echo "known=$k $a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab.json)"
  done
done
done
